#!/usr/bin/env python3
"""Debug aid (not product): gemvm outputs vs the reference-row entry on one shape, sentinel-filled output."""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "llama.cpp-quant-gemm_amd")); sys.path.insert(0, os.path.join(REPO, "tests"))
import torch
import quant_gemm as qg
if len(sys.argv) > 1:
    qg._lib.LIB_PATH = os.path.abspath(sys.argv[1]); qg._lib._lib = None
print("lib", qg._lib.LIB_PATH)
from test_gpu_product import dev, host, random_blocks
for (m, n, k, t) in [(7, 32000, 1024, 8), (3, 32000, 1024, 8), (16, 32000, 1024, 8), (7, 8192, 1024, 8), (7, 8224, 1024, 8),
                     (7, 32000, 1024, 2), (7, 32000, 2048, 8), (2, 32000, 1024, 8), (7, 16384, 4096, 8), (7, 32000, 4096, 2)]:
    aq, bq = random_blocks(np.random.default_rng(m * 13 + n + k + t), m, n, k, t)
    a, b = dev(aq), dev(bq)
    bt = qg.tile_weights(b, n, k, t)
    out = torch.full((m, n), 1234.5, dtype=torch.float32, device="cuda")
    qg.gemm_w4a8_tiled(a, bt, m, n, k, t, out=out)
    torch.cuda.synchronize()
    c = host(out)
    r = host(qg.gemm_w4a8(a, b, m, n, k, t))
    bad = ~(np.abs(c - r) <= 1e-3 * (np.abs(r) + 1))
    print(m, n, k, t, qg.debug_config_tiled(m, n, k, t), "bad", bad.sum(), "sentinel", (c == 1234.5).sum(), "inf", np.isinf(c).sum(), "nan", np.isnan(c).sum())
    if bad.any():
        ii, jj = np.nonzero(bad)
        print("  tokens", np.unique(ii), "rows", jj.min(), jj.max(), len(np.unique(jj)), "sample", c[ii[0], jj[0]], r[ii[0], jj[0]])
