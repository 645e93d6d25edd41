#!/usr/bin/env python3
"""Debug aid (not product): DBG=4 builds output sum_b sumi, DBG=8 builds sum_b d_w d_a; checked here."""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "llama.cpp-quant-gemm_amd")); sys.path.insert(0, os.path.join(REPO, "tests"))
import torch
import quant_gemm as qg
mode = int(sys.argv[2])
qg._lib.LIB_PATH = os.path.abspath(sys.argv[1]); qg._lib._lib = None
from test_gpu_product import dev, host, random_blocks
for (m, n, k, t) in [(7, 32000, 1024, 2), (7, 32000, 4096, 2), (3, 32000, 1024, 2), (7, 32000, 1024, 8)]:
    aq, bq = random_blocks(np.random.default_rng(m * 13 + n + k + t), m, n, k, t)
    a, b = dev(aq), dev(bq)
    bt = qg.tile_weights(b, n, k, t)
    c = host(qg.gemm_w4a8_tiled(a, bt, m, n, k, t))
    if mode == 4:
        s = host(qg.debug_sumi_tiled(a, bt, m, n, k, t)).astype(np.float64).sum(-1)
    elif mode == 64:
        sa = aq[..., 2:4].copy().view(np.float16)[..., 0].astype(np.float64)
        dw = bq[..., 0:2].copy().view(np.float16)[..., 0].astype(np.float64)
        s = sa @ dw.T
    else:
        da = aq[..., 0:2].copy().view(np.float16)[..., 0].astype(np.float64)  # [m, nb]
        dw = bq[..., 0:2].copy().view(np.float16)[..., 0].astype(np.float64)  # [n, nb]
        s = da @ dw.T
    bad = ~(np.abs(c - s) <= 1e-3 * (np.abs(s) + 1))
    print(mode, m, n, k, t, "bad", bad.sum(), "of", bad.size)
    if bad.any():
        ii, jj = np.nonzero(bad)
        print("  tokens", np.unique(ii), "rows", jj.min(), jj.max(), "sample", [(int(i), int(j), c[i, j], s[i, j]) for i, j in list(zip(ii, jj))[:4]])
