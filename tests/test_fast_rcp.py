"""CPU: the FAST cell kernel's item decode divides by the row's dword-group count ng with
v_rcp_f32 (1 ulp) instead of an IEEE division (orb_fast_cell.h fast_cell_detect): every quotient
it floors is (k + 0.5) / ng with k < 1500 and ng <= 20, at least 0.5 / ng from an integer, so any
reciprocal within a few ulps gives the same floor.  Checked exhaustively in float32 arithmetic with
the reciprocal perturbed by up to 4 ulps either way."""
import numpy as np


def test_rcp_floor_exact():
    k = np.arange(0, 1500, dtype=np.float32) + np.float32(0.5)
    for ng in range(1, 21):
        exact = np.floor((np.arange(0, 1500) + 0.5) / ng).astype(np.int64)
        r0 = np.float32(1.0) / np.float32(ng)
        for d in range(-4, 5):
            r = np.nextafter(r0, np.float32(np.inf if d > 0 else -np.inf), dtype=np.float32) if d else r0
            for _ in range(abs(d) - 1 if d else 0):
                r = np.nextafter(r, np.float32(np.inf if d > 0 else -np.inf), dtype=np.float32)
            got = np.floor((k * r).astype(np.float32)).astype(np.int64)
            np.testing.assert_array_equal(got, exact, err_msg="ng=%d ulps=%d" % (ng, d))
