"""GPU parity: the HIP kernels (through the C-ABI, via quant_gemm) vs the pinned CPU oracle.

Bars:
  * quantizer / dequantizer bytes: bit-exact;
  * per-block int32 sumi: bit-exact, computed by the very kernel instantiation the product
    dispatch launches for the shape (qg_debug_config asserts the match; test_gpu_product.py);
  * fp32 outputs: per-block terms are computed in the reference's operation order without
    contraction, so the only admissible difference is fp32 summation order:
    |C_gpu - C_ref| <= 2 * nb * 2^-24 * sum_b |term_b|   (oracle.summation_tol);
  * vs FP32 (gemm_fp32_reference): NMSE <= 5e-3 for Q4_0 x Q8_1 on the step4 U[-1,1] recipe
    (BASELINE.json north_star), per-format bounds for the all-quants config.
"""
import ctypes
import glob
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
WTYPES = [2, 3, 6, 7, 8]  # Q4_0, Q4_1, Q5_0, Q5_1, Q8_0 (W8A8)
ALGOS = {"gemv": 1, "mfma": 2, "generic": 3}


def dev(x):
    import torch
    return torch.from_numpy(np.ascontiguousarray(x)).cuda()


def host(t):
    import torch
    torch.cuda.synchronize()
    return t.cpu().numpy()


def make_case(O, m, n, k, t, seed=42):
    a, b = O.fill_uniform_step4(m, n, k, seed)
    return a, b, O.quantize(a, O.Q8_1), O.quantize(b, t)


def assert_close_to_oracle(O, c_gpu, aq, bq, t, mfma=None):
    """mfma: the output came from the MFMA prefill (None: whichever family the auto dispatch picks
    for the shape), whose EPI2 epilogue rounds each block term's two parts separately
    (oracle.reassoc_tol); every other family's terms are bit-identical to the oracle's and only the
    summation order differs (oracle.summation_tol)."""
    c_ref, s = O.gemm_w4a8(aq, bq, t, want_sumi=True)
    if mfma is None:  # auto dispatch: the family the product picks for this shape
        import quant_gemm
        mfma = quant_gemm.select_algo(aq.shape[0], bq.shape[0], 32 * aq.shape[1], t) == 2
    tol = O.reassoc_tol(aq, bq, s, t) if mfma else O.summation_tol(aq, bq, s, t)
    err = np.abs(c_gpu.astype(np.float64) - c_ref)
    assert (err <= tol).all(), f"max err {err.max()} vs tol {tol[err > tol].min()}"
    return c_ref


# ------------------------------------------------------------------------------- quantizers
def edge_rows():
    rng = np.random.default_rng(1)
    rows = [np.zeros(64, np.float32),                                  # amax = 0 -> d = 0, id = 0
            np.full(64, -3.0, np.float32),
            (np.arange(64, dtype=np.float32) - 31.5) / 8.0,             # exact ties for Q4_0 / Q8_1
            rng.standard_normal(64).astype(np.float32) * 1e-6,
            rng.standard_normal(64).astype(np.float32) * 1e3,
            np.where(np.arange(64) % 2 == 0, 1.0, -1.0).astype(np.float32)]
    # s = sum(x) lands exactly on an f16 tie after fp32 rounding (1 + 2^-11) while the exact sum
    # is just above it: catches a fused add->f16 conversion (single rounding) in the quantizer
    tie = np.zeros(64, np.float32)
    tie[0] = 1.0
    tie[31] = np.float32(2.0 ** -11 + 2.0 ** -30)
    tie[32:] = np.linspace(-0.7, 0.9, 32, dtype=np.float32)
    rows.append(tie)
    return np.stack(rows)


@pytest.mark.parametrize("t,variant", [(9, 0), (9, 1), (2, 0), (8, 0), (3, 0), (6, 0), (7, 0)])
def test_quantizer_bytes_bit_exact(O, qg, t, variant):
    a, b = O.fill_uniform_step4(64, 64, 4096)
    for x in (a, b, edge_rows()):
        got = host(qg.quantize(dev(x), t, variant))
        want = O.quantize(x, t, variant)
        assert np.array_equal(got, want)


def test_q8_1_quantizer_extreme_scales(O, qg):
    """Q8_1 blocks whose d = amax / 127 is subnormal (amax in 5e-37 .. 1.5e-36: d keeps 21-23 significant bits)
    or whose amax is near the float maximum, both quantizer variants:
    bytes identical to the oracle (the lanes quantizer's fma-corrected division and 3-instruction roundf,
    csrc/qg_quant_block.hpp, against the reference's IEEE division and roundf). Blocks whose 1 / d overflows
    (amax below ~3.7e-37) are left out: there the reference converts inf / NaN to int, which C leaves undefined."""
    rng = np.random.default_rng(11)
    rows = [rng.uniform(-1.0, 1.0, 256).astype(np.float32) * np.float32(s) for s in (5e-37, 8e-37, 1.4e-36)]
    rows.append(rng.uniform(-1.0, 1.0, 256).astype(np.float32) * np.float32(3.0e38))
    x = np.stack(rows)
    amax = np.abs(x.reshape(-1, 32)).max(axis=1)
    assert ((amax > 3.7e-37) | (amax == 0)).all()
    for variant in (0, 1):
        got = host(qg.quantize(dev(x), 9, variant))
        want = O.quantize(x, 9, variant)
        assert np.array_equal(got, want), variant


def test_quantize_reference_names(O, qg):
    a, b = O.fill_uniform_step4(3, 5, 1024)
    assert np.array_equal(host(qg.quantize_q8_1(dev(a))), O.quantize(a, O.Q8_1))
    assert np.array_equal(host(qg.quantize_q4_0(dev(b))), O.quantize(b, O.Q4_0))
    x3 = b.reshape(5, 4, 256)  # leading dims preserved: [..., K] -> [..., K/32, 18]
    assert host(qg.quantize_q4_0(dev(x3))).shape == (5, 4, 8, 18)


@pytest.mark.parametrize("t", [2, 3, 6, 7, 8, 9])
def test_dequantize_bit_exact(O, qg, t):
    _, b = O.fill_uniform_step4(1, 16, 2048)
    q = O.quantize(b, t)
    assert np.array_equal(host(qg.dequantize(dev(q), t)), O.dequantize(q, t))
    if t == 2:
        assert np.array_equal(host(qg.dequantize_q4_0(dev(q), 2048)), O.dequantize(q, t))


# ------------------------------------------------------------------------------- sumi (integer path)
@pytest.mark.parametrize("t", WTYPES)
@pytest.mark.parametrize("algo", ["gemv", "mfma", "generic"])
@pytest.mark.parametrize("m,n,k", [(1, 64, 4096), (3, 37, 2048), (8, 16, 4096), (2, 5, 16384), (40, 70, 1024)])
def test_sumi_bit_exact(O, qg, t, algo, m, n, k):
    if algo == "gemv" and m > 8:
        pytest.skip("GEMV path is M <= 8")
    _, _, aq, bq = make_case(O, m, n, k, t)
    got = host(qg.debug_sumi(dev(aq), dev(bq), m, n, k, t, ALGOS[algo]))
    _, want = O.gemm_w4a8(aq, bq, t, want_sumi=True)
    assert np.array_equal(got, want)


def random_byte_case(m, n, k, t, seed=7):
    """Raw random blocks: every weight nibble / byte value and every activation byte including
    -128 (which no quantizer emits), with finite f16 scales — the integer paths' full input range."""
    rng = np.random.default_rng(seed)
    nb, bb = k // 32, {2: 18, 3: 20, 6: 22, 7: 24, 8: 34}[t]
    aq = rng.integers(0, 256, (m, nb, 36), dtype=np.uint8)
    bq = rng.integers(0, 256, (n, nb, bb), dtype=np.uint8)
    f16 = lambda lo, hi, shape: rng.uniform(lo, hi, shape).astype(np.float16).view(np.uint8).reshape(shape + (2,))
    aq[..., 0:2] = f16(1e-3, 2e-2, (m, nb))
    aq[..., 2:4] = f16(-5.0, 5.0, (m, nb))
    bq[..., 0:2] = f16(-0.1, 0.1, (n, nb))
    if t in (3, 7):
        bq[..., 2:4] = f16(-0.5, 0.5, (n, nb))
    aq[0, 0, 4:36] = 0x80            # a whole block of -128
    bq[0, 0, bb - 16:] = 0x00 if t != 8 else 0x80   # nibbles 0 (q - 8 = -8) / bytes -128
    return aq, bq


@pytest.mark.parametrize("t", WTYPES)
@pytest.mark.parametrize("algo", ["gemv", "mfma", "generic"])
@pytest.mark.parametrize("m,n,k", [(1, 96, 4096), (4, 33, 1024), (24, 48, 2048)])
def test_random_bytes_bit_exact(O, qg, t, algo, m, n, k):
    if algo == "gemv" and m > 8:
        pytest.skip("GEMV path is M <= 8")
    aq, bq = random_byte_case(m, n, k, t)
    got = host(qg.debug_sumi(dev(aq), dev(bq), m, n, k, t, ALGOS[algo]))
    _, want = O.gemm_w4a8(aq, bq, t, want_sumi=True)
    assert np.array_equal(got, want)
    c = host(qg.gemm_w4a8(dev(aq), dev(bq), m, n, k, t, algo=ALGOS[algo]))
    assert_close_to_oracle(O, c, aq, bq, t, mfma=algo == "mfma")


@pytest.mark.parametrize("t", [2, 3, 6, 8])
@pytest.mark.parametrize("m,n,k", [(1, 70, 14336), (2, 33, 8192), (4, 40, 12288), (3, 17, 6144)])
def test_gemv_long_rows(O, qg, t, m, n, k):
    """GEMV shapes whose lanes own several units (the unit loop with preloaded records), incl. a
    partial last round of units (K = 14336: 224 two-block units over 64 lanes)."""
    _, _, aq, bq = make_case(O, m, n, k, t)
    c = host(qg.gemm_w4a8(dev(aq), dev(bq), m, n, k, t, algo=ALGOS["gemv"]))
    assert_close_to_oracle(O, c, aq, bq, t)
    aq2, bq2 = random_byte_case(m, n, k, t)
    c2 = host(qg.gemm_w4a8(dev(aq2), dev(bq2), m, n, k, t, algo=ALGOS["gemv"]))
    assert_close_to_oracle(O, c2, aq2, bq2, t)


@pytest.mark.parametrize("n,k,nu", [(70, 8192, 2), (33, 11008, 4), (4096, 14336, 4), (17, 12288, 4)])
def test_gemv_multi_unit_sumi_and_output(O, qg, n, k, nu):
    """The loop-free multi-unit GEMV (Q4_0, M = 1, K > 4096: every unit of a lane loaded before the staging,
    qg_gemv_kernel.hpp ONEU = 2 / 4; round 5): the parity hook runs that exact instantiation and its int32
    block dots equal the reference's inner loop (include/gemm_reference.h:202-212) bit for bit, incl. lanes
    whose last unit is past the row (K = 11008: 172 units over 64 lanes) and the published 4096 x 1 x 14336."""
    t, m = 2, 1
    cfg = qg.debug_config(m, n, k, t)
    assert f"ONEU={nu} SIG=m1" in cfg and cfg == qg.debug_config(m, n, k, t, sumi=True), cfg
    _, _, aq, bq = make_case(O, m, n, k, t, seed=k)
    _, want = O.gemm_w4a8(aq, bq, t, want_sumi=True)
    assert np.array_equal(host(qg.debug_sumi(dev(aq), dev(bq), m, n, k, t)), want)
    c = host(qg.gemm_w4a8(dev(aq), dev(bq), m, n, k, t))
    assert_close_to_oracle(O, c, aq, bq, t)


# ------------------------------------------------------------------------------- outputs
@pytest.mark.parametrize("t", WTYPES)
@pytest.mark.parametrize("m", [1, 2, 3, 4, 5, 8])
def test_gemv_matches_oracle(O, qg, t, m):
    n, k = 300, 4096
    _, _, aq, bq = make_case(O, m, n, k, t, seed=m)
    c = host(qg.gemm_w4a8(dev(aq), dev(bq), m, n, k, t, algo=1))
    assert_close_to_oracle(O, c, aq, bq, t)


@pytest.mark.parametrize("t", WTYPES)
@pytest.mark.parametrize("m", [9, 16, 32, 33, 100])
def test_mfma_matches_oracle(O, qg, t, m):
    n, k = 96, 2048
    _, _, aq, bq = make_case(O, m, n, k, t, seed=m)
    assert qg.select_algo(m, n, k, t) == 2
    c = host(qg.gemm_w4a8(dev(aq), dev(bq), m, n, k, t, algo=2))
    assert_close_to_oracle(O, c, aq, bq, t, mfma=True)


@pytest.mark.parametrize("t", WTYPES)
@pytest.mark.parametrize("m,n,k", [(12, 33, 512), (64, 4096, 256), (32, 65, 8192), (10, 40, 384), (33, 20, 640)])
def test_mfma_ragged(O, qg, t, m, n, k):
    """Ragged tiles; K % 256 == 128 takes the 4-byte weight-DMA variant, K % 256 == 0 the 16-byte one."""
    _, _, aq, bq = make_case(O, m, n, k, t)
    c = host(qg.gemm_w4a8(dev(aq), dev(bq), m, n, k, t, algo=2))
    assert_close_to_oracle(O, c, aq, bq, t, mfma=True)


@pytest.mark.parametrize("t", WTYPES)
def test_mfma_weights_4byte_aligned(O, qg, t):
    """Weights only 4-B aligned: the 16-byte DMA variant is not legal, the 4-byte one runs."""
    import torch
    m, n, k = 20, 48, 1024
    _, _, aq, bq = make_case(O, m, n, k, t)
    raw = torch.zeros(bq.size + 4, dtype=torch.uint8, device="cuda")
    raw[4:] = dev(bq.ravel())
    w = raw[4:]
    assert w.data_ptr() % 16 == 4
    c = host(qg.gemm_w4a8(dev(aq), w, m, n, k, t, algo=2))
    assert_close_to_oracle(O, c, aq, bq, t, mfma=True)


@pytest.mark.parametrize("m,t", [(1, 2), (3, 6), (12, 2)])
def test_strided_batched(O, qg, m, t):
    """One launch over independent products (GEMV path) == per-item oracle results."""
    nbatch, n, k = 5, 130, 1024
    items = [make_case(O, m, n, k, t, seed=100 + i) for i in range(nbatch)]
    a = np.stack([it[2] for it in items])
    b = np.stack([it[3] for it in items])
    out = host(qg.gemm_w4a8_batched(dev(a), dev(b), m, n, k, t))
    for i in range(nbatch):
        assert_close_to_oracle(O, out[i], a[i], b[i], t)


@pytest.mark.parametrize("m,n,k,t", [(1, 4096, 4096, 2), (2, 1000, 1024, 2), (4, 4096, 2048, 2), (1, 4096, 4096, 8),
                                     (1, 17, 4096, 6), (3, 8200, 4096, 2)])
def test_strided_batched_bit_identical(O, qg, m, n, k, t):
    """The strided batch (half-size workgroups where N fits one round, qg_gemv_kernel.hpp QG_GEMVB_WDIV;
    full-size beyond) is bit-identical, item by item, to the single launch."""
    nbatch = 3
    items = [make_case(O, m, n, k, t, seed=200 + i) for i in range(nbatch)]
    a = np.stack([it[2] for it in items])
    b = np.stack([it[3] for it in items])
    out = host(qg.gemm_w4a8_batched(dev(a), dev(b), m, n, k, t))
    for i in range(nbatch):
        single = host(qg.gemm_w4a8(dev(a[i]), dev(b[i]), m, n, k, t))
        assert np.array_equal(out[i].view(np.uint32), single.view(np.uint32)), f"item {i}"
    assert_close_to_oracle(O, out[-1], a[-1], b[-1], t)


@pytest.mark.parametrize("m,n,k", [(1, 1, 32), (1, 3, 96), (2, 7, 288), (4, 65, 4128), (1, 4097, 256),
                                   (9, 33, 512), (16, 64, 1024), (1, 5, 14336), (3, 17, 8192)])
def test_auto_dispatch_shapes(O, qg, m, n, k):
    """Ragged N, K not a multiple of 256, tiny and large K, M across the GEMV/prefill split."""
    _, _, aq, bq = make_case(O, m, n, k, 2)
    c = host(qg.gemm_w4a8(dev(aq), dev(bq), m, n, k, 2))
    assert_close_to_oracle(O, c, aq, bq, 2)


def test_empty_is_noop(qg):
    import torch
    u8 = dict(dtype=torch.uint8, device="cuda")
    assert qg.gemm_w4a8(torch.zeros(0, **u8), torch.zeros(8 * 2 * 18, **u8), 0, 8, 64).shape == (0, 8)
    assert qg.gemm_w4a8(torch.zeros(2 * 36, **u8), torch.zeros(0, **u8), 1, 0, 64).shape == (1, 0)
    assert qg.quantize_q8_1(torch.zeros((0, 64), device="cuda")).shape == (0, 2, 36)


def test_misaligned_weights_take_generic_path(O, qg):
    import torch
    m, n, k = 1, 40, 1024
    _, _, aq, bq = make_case(O, m, n, k, 2)
    raw = torch.zeros(bq.size + 2, dtype=torch.uint8, device="cuda")
    raw[2:] = dev(bq.ravel())
    w = raw[2:]  # 2-byte aligned only: the 16-B GEMV loads are not legal
    assert w.data_ptr() % 16 != 0
    c = torch.empty((m, n), dtype=torch.float32, device="cuda")
    lib = qg._lib.load()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    assert lib.qg_gemm_w4a8_ex(ctypes.c_void_p(dev(aq).data_ptr()), ctypes.c_void_p(w.data_ptr()),
                               ctypes.c_void_p(c.data_ptr()), m, n, k, 2, 1, st) == -3  # GEMV refuses
    a_t = dev(aq)
    assert lib.qg_gemm_w4a8(ctypes.c_void_p(a_t.data_ptr()), ctypes.c_void_p(w.data_ptr()),
                            ctypes.c_void_p(c.data_ptr()), m, n, k, 2, st) == 0
    assert_close_to_oracle(O, host(c), aq, bq, 2)


@pytest.mark.parametrize("t,sym", [(2, "gemm_q4_0_q8_1"), (3, "gemm_q4_1_q8_1"), (6, "gemm_q5_0_q8_1"),
                                   (7, "gemm_q5_1_q8_1"), (8, "gemm_q8_0_q8_1")])
@pytest.mark.parametrize("ntok", [1, 2, 6])
def test_weight_major_api(O, qg, t, sym, ntok):
    """python/quant_gemm convention: out[M_w, N_tok] = W @ A^T (kernels/gemm/gemm_quant_formats.cuh:312)."""
    mw, k = 130, 4096
    _, _, aq, wq = make_case(O, ntok, mw, k, t)
    out = host(getattr(qg, sym)(dev(wq), dev(aq), mw, ntok, k))
    assert out.shape == (mw, ntok)
    assert_close_to_oracle(O, np.ascontiguousarray(out.T), aq, wq, t)


@pytest.mark.parametrize("m,n,k", [(1, 4096, 4096), (3, 100, 1024), (32, 256, 2048), (5, 64, 96)])
def test_w8a8_matches_gemm_w8a8_reference(O, qg, m, n, k):
    """W8A8 (include/gemm_reference.h:233-267) through qg_gemm_w8a8, every dispatch branch."""
    a, b, aq, bq = make_case(O, m, n, k, O.Q8_0)
    c = host(qg.gemm_w8a8(dev(aq), dev(bq), m, n, k))
    c_ref = assert_close_to_oracle(O, c, aq, bq, O.Q8_0)
    assert np.array_equal(c_ref, O.gemm_w8a8(aq, bq))
    assert O.nmse(c, O.gemm_fp32(a, b)) <= 1e-4


def test_reference_harness_convention(O, qg):
    """python/test_operator.py:236-240: kernel(weight_q, activation_q, N, M, K).T == C[M, N]."""
    m, n, k = 4, 96, 1024
    a, b, aq, bq = make_case(O, m, n, k, 2)
    out = host(qg.gemm_q4_0_q8_1(dev(bq), dev(aq), n, m, k)).T
    assert_close_to_oracle(O, np.ascontiguousarray(out), aq, bq, 2)


def test_ggml_view_adapter(O, qg):
    import torch
    m, n, k = 2, 48, 512
    _, _, aq, bq = make_case(O, m, n, k, 2)
    a_t, b_t = dev(aq), dev(bq)
    c = torch.empty((m, n), dtype=torch.float32, device="cuda")

    class View(ctypes.Structure):
        _fields_ = [("data", ctypes.c_void_p), ("type", ctypes.c_int), ("ne", ctypes.c_int64 * 4),
                    ("nb", ctypes.c_size_t * 4)]

    def view(ptr, t, ne0, ne1, row):
        v = View()
        v.data, v.type = ptr, t
        v.ne[:] = [ne0, ne1, 1, 1]
        v.nb[:] = [0, row, row * ne1, row * ne1]
        return v

    act = view(a_t.data_ptr(), 9, k, m, (k // 32) * 36)
    w = view(b_t.data_ptr(), 2, k, n, (k // 32) * 18)
    out = view(c.data_ptr(), 0, n, m, n * 4)
    out.nb[0] = 4
    lib = qg._lib.load()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    assert lib.qg_gemm_w4a8_from_view(ctypes.byref(act), ctypes.byref(w), ctypes.byref(out), b"dp4a", st) == 0
    assert_close_to_oracle(O, host(c), aq, bq, 2)


@pytest.mark.parametrize("t", WTYPES)
def test_batched_equals_single_full_size(qg, t):
    """A strided batch of 6 full-size GEMVs (M=1, N=K=4096) equals six single launches bit for bit."""
    import torch
    gen = torch.Generator(device="cuda")
    gen.manual_seed(12 + t)
    k, n, B = 4096, 4096, 6
    aq = torch.stack([qg.quantize_q8_1(torch.rand((1, k), generator=gen, device="cuda") * 2 - 1) for _ in range(B)])
    bq = torch.stack([qg.quantize(torch.rand((n, k), generator=gen, device="cuda") * 2 - 1, t) for _ in range(B)])
    cb = qg.gemm_w4a8_batched(aq, bq, 1, n, k, t)
    for i in range(B):
        assert torch.equal(cb[i], qg.gemm_w4a8(aq[i], bq[i], 1, n, k, t))


def test_weight_major_is_transpose_full_size(qg):
    """BASELINE configs[2] (M=32 prefill): the reference's weight-major entry (gemm_q4_0_q8_1,
    out[Mw][Ntok]) is the activation-major product transposed, bit for bit."""
    import torch
    gen = torch.Generator(device="cuda")
    gen.manual_seed(13)
    m, n, k = 32, 4096, 4096
    aq = qg.quantize_q8_1(torch.rand((m, k), generator=gen, device="cuda") * 2 - 1)
    bq = qg.quantize_q4_0(torch.rand((n, k), generator=gen, device="cuda") * 2 - 1)
    c = qg.gemm_w4a8(aq, bq, m, n, k)
    w = qg.gemm_q4_0_q8_1(bq, aq, n, m, k)
    assert torch.equal(w.T, c)
