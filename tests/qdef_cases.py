"""Inputs for the quantization-definition parity tests (quantize_q8_1 / quantize_q4_0 Solutions).

x[num_elements] f32 with the block families the two quantizer semantics (include/quantize.h vs the
definitions, oracle.quantize_definition) can disagree on, plus bulk random blocks:
  * 2048 step4 U[-1, 1] blocks (the measurement recipe) and 1024 blocks of wide dynamic range;
  * all-zero blocks (the definitions store d = 1.0, quantize.h d = 0);
  * exact round-half ties (amax = 127 * 2^e or 7 * 2^e, the other elements at (j + 1/2) * 2^e):
    ties-to-even (torch.round) vs half-away (roundf);
  (no block can make f32-then-f16 rounding of amax / 127 or amax / 7 differ from one rounding of the
  exact quotient: an f32 amax one step off div * mid puts the quotient more than half an f32 step
  from the f16 midpoint mid — the oracle test checks the single rounding with exact rationals.)
Deterministic (numpy default_rng); about 3.1k blocks.
"""
import numpy as np


def definition_inputs(seed: int = 2026) -> np.ndarray:
    import oracle as O
    rng = np.random.default_rng(seed)
    a, _ = O.fill_uniform_step4(2048, 0, 32, 42)
    blocks = [a]
    wide = rng.standard_normal((1024, 32)) * np.exp2(rng.integers(-30, 30, (1024, 1)))
    blocks.append(wide.astype(np.float32))
    blocks.append(np.zeros((8, 32), np.float32))
    ties = []
    for div in (127, 7):
        for e in range(-6, 7):
            t = (rng.integers(-div, div, 32) + 0.5) * 2.0 ** e
            t[rng.integers(0, 32)] = div * 2.0 ** e * rng.choice([-1, 1])
            ties.append(t)
    blocks.append(np.array(ties, np.float32))
    return np.concatenate(blocks).astype(np.float32).ravel()
