#!/usr/bin/env python3
"""Exhaustive checks of orb_math.h libm_atanf / libm_tanf / libm_atan2f against the host libm
(the oracle's atan2f / tanf, KannalaBrandt8.cpp:61-78, 110-137): atanf on every positive float,
tanf on every float of [-2.35, 2.35], atan2f on 4e8 random pairs.  ~2 minutes on one core.
Run from the repo root: python3 tools/libm_fisheye_exhaustive.py"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from tests.conftest import build_harness  # noqa: E402

lib = C.CDLL(build_harness())
f = lib.harness_libm_atanf_tanf_mismatches
f.restype = C.c_longlong
f.argtypes = [C.c_float, C.c_float, C.c_int, C.c_int, C.POINTER(C.c_longlong)]
g = lib.harness_libm_atan2f_random
g.restype = C.c_longlong
g.argtypes = [C.c_longlong, C.c_ulonglong]
n = C.c_longlong(0)
res = {}
res["atanf [0, inf)"] = (f(0.0, float("inf"), 1, 0, C.byref(n)), n.value)
res["tanf [0, 2.35)"] = (f(0.0, 2.35, 1, 1, C.byref(n)), n.value)
res["tanf (-2.35, -0]"] = (f(-0.0, -2.35, 1, 1, C.byref(n)), n.value)
res["atan2f random pairs"] = (g(400_000_000, 88172645463325252), 400_000_000)
for k, (bad, cnt) in res.items():
    print("%-22s checked %11d mismatches %d" % (k, cnt, bad))
sys.exit(1 if any(b for b, _ in res.values()) else 0)
