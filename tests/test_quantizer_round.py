"""The lanes quantizer's two arithmetic shortcuts (csrc/qg_quantize.hip), checked on CPU.

* roundf_small(y) = (int)(y + copysign(0.49999997f, y)) replaces roundf (round half away from zero,
  include/quantize.h:165-193): an fp32 add (round to nearest even) and a truncating conversion, three
  instructions instead of seven. Checked here exhaustively over every float in [0, 2^23] (above it every
  float is an integer and the add returns y); negative y mirror it exactly through copysign.
* div127(m) = fma(fma(-q0, 127, m), R, q0), q0 = RN(m R), R = RN(1/127), replaces the IEEE division
  m / 127 (d = amax / 127). tools/verify_quant_arith.py checks every finite m >= 0 (0 mismatches,
  profiles/r05_tuning/quant/verify_quant_arith.txt, ~75 s); here: every subnormal and a strided sample of
  the normal range (m = +inf is passed through by the kernel, m is never NaN: fmaxf drops NaN).
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import verify_quant_arith as V  # noqa: E402


def test_constants():
    assert V.HALF == np.float32(0.5) - np.float32(2.0 ** -25)
    assert V.HALF.view(np.uint32) == 0x3EFFFFFF
    assert V.R.view(np.uint32) == 0x3C010204


def test_roundf_small_exhaustive_up_to_2_23():
    assert V.check_round() == 0


def test_div127_subnormals_exhaustive():
    assert V.check_div127(0, 1 << 23) == 0


def test_div127_normal_range_strided():
    top = int(np.float32(np.inf).view(np.uint32))
    assert V.check_div127(1 << 23, top, stride=251) == 0
