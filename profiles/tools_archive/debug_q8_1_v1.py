import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import __graft_entry__ as g
g._paths()
import numpy as np, torch
import oracle as O, quant_gemm as qg
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
from test_gpu_parity import edge_rows
a, b = O.fill_uniform_step4(64, 64, 4096)
for name, x in (("a", a), ("b", b), ("edge", edge_rows())):
    got = qg.quantize(torch.from_numpy(x).cuda(), 9, 1).cpu().numpy()
    want = O.quantize(x, 9, 1)
    bad = np.argwhere((got != want).any(-1))
    print(name, "bad blocks", len(bad))
    for r, blk in bad[:3]:
        print(" row", r, "blk", blk, "got", got[r, blk, :8].tolist(), "want", want[r, blk, :8].tolist())
        xb = x[r, blk * 32:(blk + 1) * 32]
        print("  x", xb[:8], "amax", np.abs(xb).max())
