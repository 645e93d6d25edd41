"""CPU check of the integer identities the GPU kernels rely on (no GPU needed).

1. The GEMV's nibble-plane dot (llama.cpp-quant-gemm_amd/csrc/qg_gemv_kernel.hpp): for a Q4 block
   (qs bytes: low nibble = element j, high nibble = element j+16) and a Q8_1 block (32 int8), each
   activation byte a = 16*h + l with h = a >> 4 (signed 4-bit) and l = a & 15; plane dword i holds
   the (l or h) nibbles of elements (4i+k, 16+4i+k) at nibbles (2k, 2k+1), i.e. the nibble order
   of raw weight dword i. Then, emulating v_dot8_u32_u4 / v_dot8_i32_i4 exactly,
       sumi = sum_i udot8(q_i, l_i) + 16 * sum_i sdot8(q_i ^ 0x88888888, h_i) + 128 * sum(h)
   equals the reference's sum_k qa[k] * lo(qw[k]) + qa[k+16] * hi(qw[k])
   (include/gemm_reference.h:205-212).
2. The biased accumulator (GEMV and MFMA epilogues): bits(1.5*2^23) + sumi read as f32 is
   1.5*2^23 + sumi for |sumi| < 2^22, and fma(d_a, cf, -1.5*2^23*d_a) == round(d_a * sumi).
"""
import numpy as np


def nibbles(x: int, signed: bool):
    out = [(x >> (4 * i)) & 0xF for i in range(8)]
    return [v - 16 if signed and v >= 8 else v for v in out]


def udot8(a: int, b: int, c: int) -> int:
    return (c + sum(x * y for x, y in zip(nibbles(a, False), nibbles(b, False)))) & 0xFFFFFFFF


def sdot8(a: int, b: int, c: int) -> int:
    return c + sum(x * y for x, y in zip(nibbles(a, True), nibbles(b, True)))


def planes(qa: np.ndarray):
    """(l[4], h[4], sum_h) of one Q8_1 block's 32 int8 values, as the LDS record stores them."""
    u = qa.astype(np.int64) & 0xFF
    l, h = [], []
    for i in range(4):
        a0 = int.from_bytes(bytes(u[4 * i:4 * i + 4].tolist()), "little")
        a1 = int.from_bytes(bytes(u[16 + 4 * i:16 + 4 * i + 4].tolist()), "little")
        l.append((a0 & 0x0F0F0F0F) | ((a1 << 4) & 0xF0F0F0F0))
        h.append(((a0 >> 4) & 0x0F0F0F0F) | (a1 & 0xF0F0F0F0))
    sh = sum(sdot8(x, 0x11111111, 0) for x in h)
    return l, h, sh


def test_nibble_plane_dot_matches_reference_sumi():
    rng = np.random.default_rng(0)
    cases = [rng.integers(-128, 128, 32), np.full(32, -128), np.full(32, 127), np.zeros(32, np.int64)]
    for qa in cases:
        for qs in [rng.integers(0, 256, 16), np.zeros(16, np.int64), np.full(16, 255)]:
            ref = sum(int(qa[k]) * (int(qs[k]) & 15) + int(qa[k + 16]) * (int(qs[k]) >> 4) for k in range(16))
            l, h, sh = planes(qa)
            L, H = 0, 0
            for i in range(4):
                q = int.from_bytes(bytes(qs[4 * i:4 * i + 4].astype(np.uint8).tolist()), "little")
                L = udot8(q, l[i], L)
                H = sdot8(q ^ 0x88888888, h[i], H)
            got = L + 16 * H + 128 * sh
            assert got == ref, (got, ref)


def test_biased_accumulator_is_exact():
    rng = np.random.default_rng(1)
    bias_bits = np.uint32(0x4B400000)
    bias = np.float32(12582912.0)
    sumi = np.concatenate([rng.integers(-(1 << 22) + 1, 1 << 22, 20000), [0, 1, -1, 60960, -60960, 524288]])
    cf = (bias_bits.astype(np.int64) + sumi).astype(np.uint32).view(np.float32)
    assert np.array_equal(cf.astype(np.float64) - 12582912.0, sumi.astype(np.float64))
    da = rng.uniform(1e-4, 2.0, sumi.size).astype(np.float16).astype(np.float32)
    nda = (-(da.astype(np.float64) * 12582912.0)).astype(np.float32)
    assert np.array_equal(nda.astype(np.float64), -(da.astype(np.float64) * 12582912.0))  # exact
    # fma(da, cf, nda) computed exactly in float64 (products of f32 fit), then rounded once to f32
    fused = (da.astype(np.float64) * cf.astype(np.float64) + nda.astype(np.float64)).astype(np.float32)
    ref = (da * sumi.astype(np.float32)).astype(np.float32)
    assert np.array_equal(fused, ref)
