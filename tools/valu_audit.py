"""VALU issue-cost audit of a kernel's hot loops, weighted by measured per-opcode rates.

usage: python tools/valu_audit.py listing.s KERNEL_SUBSTRING profiles/r06/valu_rates.json [min_valu]

listing.s: `hipcc --offload-arch=gfx950 -O3 ... --cuda-device-only -S` of the kernel's TU.  Every
basic block of the kernel with at least min_valu (default 20) VALU instructions is reported with
its VALU count, the ns it costs one SIMD per wave pass at the measured rates (tools/valu_rates.hip,
8 waves per SIMD, independent chains), and the split into the fast class (~1.1 ns: v_add/sub_u32,
v_and/or/xor, v_bitop3, v_lshrrev, v_mov, v_max_u16, f32 add/mul/fma) and the rest (~1.75 ns).
Opcodes the rate table lacks are priced at the slow rate and listed.
"""
import collections
import json
import re
import sys


def load_rates(path):
    rows = json.load(open(path))["rows"]
    rates = {}
    for r in rows:
        op = r["op"].split()[0]
        rates.setdefault(op, r["ns_per_wave_instr_per_simd"])
    return rates


def base_op(op):
    return re.sub(r"_(e32|e64|sdwa|dpp)$", "", op)


def blocks_of(listing, want):
    s = open(listing).read()
    start = None
    for m in re.finditer(r"^(_Z[A-Za-z0-9_]*):", s, re.M):
        if want in m.group(1):
            start = m.start()
            name = m.group(1)
            break
    if start is None:
        raise SystemExit("kernel %r not in %s" % (want, listing))
    body = s[start:s.index(".Lfunc_end", start)].split("\n")
    blocks, cur = [], ["entry", []]
    for ln in body:
        m = re.match(r"^(\.LBB[0-9_]+):", ln)
        if m:
            blocks.append(cur)
            cur = [m.group(1), []]
            continue
        m = re.match(r"^\s+([a-z_0-9]+)", ln)
        if m and not ln.strip().startswith((";", ".")):
            cur[1].append(m.group(1))
    blocks.append(cur)
    return name, blocks


def main():
    listing, want, rates_path = sys.argv[1:4]
    min_valu = int(sys.argv[4]) if len(sys.argv) > 4 else 20
    rates = load_rates(rates_path)
    slow = max(v for v in rates.values() if v < 5)  # the ~1.75 ns class (v_cndmask's 9.5 is a probe artifact)
    fast_cut = 1.3
    name, blocks = blocks_of(listing, want)
    print(name)
    unknown = collections.Counter()
    for label, ops in blocks:
        valu = [base_op(o) for o in ops if o.startswith("v_")]
        if len(valu) < min_valu:
            continue
        ns, nfast, nslow = 0.0, 0, 0
        per = collections.Counter(valu)
        for op, n in per.items():
            r = rates.get(op)
            if r is None or r > 5:
                unknown[op] += n
                r = slow
            ns += n * r
            if r < fast_cut:
                nfast += n
            else:
                nslow += n
        lds = sum(1 for o in ops if o.startswith("ds_"))
        print("  %-10s VALU %3d (fast %2d, slow %2d)  %6.1f ns/wave-pass  LDS %2d  | %s" % (
            label, len(valu), nfast, nslow, ns, lds, " ".join("%s:%d" % kv for kv in per.most_common(12))))
    if unknown:
        print("  priced at the slow rate (not in the table):", " ".join("%s:%d" % kv for kv in unknown.most_common()))


if __name__ == "__main__":
    main()
