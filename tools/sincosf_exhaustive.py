#!/usr/bin/env python3
"""Exhaustive check of orb_math.h libm_sincosf against the host libm cosf / sinf on every float of
[0, 6.2832) (the descriptor's angle domain, ORBextractor_old.cc:114-115).  ~1 minute on one core.
Run from the repo root: python3 tools/sincosf_exhaustive.py"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from tests.conftest import HARNESS_LIB  # noqa: E402

lib = C.CDLL(HARNESS_LIB)
f = lib.harness_libm_sincosf_mismatches
f.restype = C.c_longlong
f.argtypes = [C.c_float, C.c_float, C.c_int, C.POINTER(C.c_longlong)]
n = C.c_longlong(0)
bad = f(0.0, 6.2832, 1, C.byref(n))
print("floats checked %d, mismatches %d" % (n.value, bad))
sys.exit(1 if bad else 0)
