"""CPU: the code path a driver `python bench.py --gpus N` run takes (BASELINE configs[3], [4];
SURVEY §8e).  bench.py starts the N ranks itself (no torchrun), they rendezvous on 127.0.0.1
(gloo here: fewer GPUs than ranks), time the barrier-bracketed steps, reduce max(time) and
sum(features) over the ranks, run the C5 cross-camera exchange, and rank 0 prints one line with
n_gpus = N.  The GPU legs are replaced by tests/bench_stub.py (--stub-gpu)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run_bench(n, extra=()):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
                        "GROUP_RANK", "ORBGPU_BENCH_BACKEND")}
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--stub-gpu", "--steps", "3",
           "--warmup", "1", "--pairs", "4", "--unique-pairs", "2", "--width", "320", "--height", "240", "--nlevels", "4",
           "--no-stereo", "--no-grid", "--no-wire", "--no-sbp", "--no-configs", "--no-cpu-baseline"] + list(extra)
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.strip()]
    # rank 0 alone prints, and only the JSON line (gloo's connection messages go to stderr)
    assert len(lines) == 1 and lines[0].startswith("{"), out.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [2, 3])
def test_bench_gpus_n_spawns_ranks(n):
    line = _run_bench(n)
    assert line["n_gpus"] == n and line["scaling"] == "weak"
    assert line["backend"] == "gloo"
    ranks = line["ranks"]
    assert sorted(r["rank"] for r in ranks) == list(range(n))
    assert len({r["pid"] for r in ranks}) == n  # one process per rank
    # weak scaling: every rank extracts its own pairs; the features of all ranks are summed
    feats = line["features_per_step_per_gpu"]
    assert line["value"] > 0 and feats > 0
    cross = line["cross_camera"]
    assert cross and "error" not in cross, cross
    assert cross["cameras"] == n and cross["exchange"].startswith("all_gather (gloo")
    assert "1920x1080, 12 levels, 5000" in cross["workload"]  # the C5 camera, not a C2 eye
    ing = line["ingest_c4"]
    assert ing and "error" not in ing, ing
    assert ing["ranks"] == n and ing["exchange"].startswith("scatter of frames + gather of results (gloo")
    assert ing["rank0_results_equal_local"] is True and ing["mfeatures_s"] > 0
    assert line["data"].startswith("stub")


def test_bench_single_rank_no_spawn():
    line = _run_bench(1)
    assert line["n_gpus"] == 1 and line["backend"] is None and len(line["ranks"]) == 1
    assert line["cross_camera"] is None
