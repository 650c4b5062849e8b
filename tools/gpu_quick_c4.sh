cd /root/repo
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_ft.log 2>&1 || { tail -30 gpurun_out/pt_ft.log; exit 1; }
tail -2 gpurun_out/pt_ft.log
timeout -k 10 120 python tools/c4_time.py
