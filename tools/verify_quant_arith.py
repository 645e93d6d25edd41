#!/usr/bin/env python3
"""Exhaustive CPU proof of the two arithmetic shortcuts in the lanes quantizer (csrc/qg_quantize.hip):

  div127(m) = fma(fma(-q0, 127, m), R, q0), q0 = RN(m * R), R = RN(1/127)   ==  RN(m / 127)
      for every finite float m >= 0 (2,139,095,040 values);
  roundf_small(y) = trunc(RN(y + 0.49999997f))                            ==  roundf(y)
      for every float 0 <= y <= 2^23 (above it every float is an integer and 0.49999997 < ulp / 2, so the
      add returns y; negative y mirror it through copysign; NaN and overflow convert alike).

fma is emulated exactly: the products are exact in float64, the residual m - 127 q0 is exact (Sterbenz), and
the correction's float64 sum is re-done in rationals whenever it lands on a float32 rounding midpoint (the
only case where rounding through float64 can differ from one rounding). Takes about 100 s.
  python tools/verify_quant_arith.py   ->  "div127: 0 mismatches ... roundf_small: 0 mismatches"
"""
import sys
import time
from fractions import Fraction

import numpy as np

R = np.float32(1.0) / np.float32(127.0)
HALF = np.float32(0.49999997)


def _rne32(ex: Fraction) -> np.float32:
    g = np.float32(float(ex))
    cand = [np.nextafter(g, np.float32(-np.inf)), g, np.nextafter(g, np.float32(np.inf))]
    return min(cand, key=lambda c: (abs(Fraction(float(c)) - ex), int(c.view(np.uint32)) & 1))


def div127_f32(m: np.ndarray):
    """(result, midpoint mask) of the fma sequence on float32 m, exact except where mask is set."""
    q0 = m * R
    r = (m.astype(np.float64) - q0.astype(np.float64) * 127.0).astype(np.float32)
    s64 = q0.astype(np.float64) + r.astype(np.float64) * np.float64(R)
    mid = (s64.view(np.uint64) & np.uint64((1 << 29) - 1)) == np.uint64(1 << 28)
    return s64.astype(np.float32), mid, q0, r


def check_div127(lo: int, hi: int, stride: int = 1) -> int:
    bad = 0
    step = 1 << 25
    for s in range(lo, hi, step * stride):
        m = np.arange(s, min(s + step * stride, hi), stride, dtype=np.uint32).view(np.float32)
        want = m / np.float32(127.0)
        got, mid, q0, r = div127_f32(m)
        for i in np.flatnonzero((got.view(np.uint32) != want.view(np.uint32)) | mid):
            ex = Fraction(float(q0[i])) + Fraction(float(r[i])) * Fraction(float(R))
            bad += int(_rne32(ex).view(np.uint32) != want[i].view(np.uint32))
    return bad


def check_round(hi_val: float = 8388608.0) -> int:
    hi = int(np.float32(hi_val).view(np.uint32))
    bad = 0
    for s in range(0, hi + 1, 1 << 25):
        y = np.arange(s, min(s + (1 << 25), hi + 1), dtype=np.uint32).view(np.float32)
        bad += int(np.count_nonzero(np.trunc(y + HALF).astype(np.float64) != np.floor(y.astype(np.float64) + 0.5)))
    return bad


def main() -> int:
    assert R.view(np.uint32) == 0x3C010204
    t = time.time()
    top = int(np.float32(np.inf).view(np.uint32))
    b1 = check_div127(0, top)
    print(f"div127: {b1} mismatches over {top} finite non-negative floats ({time.time() - t:.0f} s)")
    t = time.time()
    b2 = check_round()
    print(f"roundf_small: {b2} mismatches over every float in [0, 2^23] ({time.time() - t:.0f} s)")
    return 1 if b1 or b2 else 0


if __name__ == "__main__":
    sys.exit(main())
