"""bench.py's compact summary (the bench line's LAST key): built from every kind of row the
line carries, short enough to survive the driver's tail of stdout. CPU only (no GPU, no measurement)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def test_compact_summary_rows_and_size():
    import bench
    side = []
    for (w, m, n, k, forms) in [("q4_0", 32, 4096, 4096, ("single", "tiled", "tiled_act")), ("q4_1", 1, 4096, 4096, ("single",)),
                                ("q5_0", 1, 4096, 4096, ("single",)), ("q5_1", 1, 4096, 4096, ("single",)),
                                ("q4_0", 1, 32000, 4096, ("single", "batched")), ("q4_0", 1, 4096, 14336, ("single", "tiled")),
                                ("q4_0", 2, 4096, 14336, ("single", "tiled")), ("q4_0", 3, 4096, 14336, ("single", "tiled")),
                                ("q4_0", 4, 4096, 14336, ("single", "tiled")), ("q4_0", 512, 4096, 4096, ("single", "tiled", "tiled_act")),
                                ("q4_0", 32, 4096, 4128, ("prepacked", "padded", "tiled", "tiled_act"))]:
        for f in forms:
            side.append({"wtype": w, "M": m, "N": n, "K": k, "form": f,
                         ("us_per_gemv" if f == "batched" else "us_per_launch"): 12.345, "frac_hbm": 0.1234})
    out = {"roofline": {"us_per_launch": 3.25, "frac": 0.3639, "floor_us": 2.78, "floor": {"units_read_store_us": 3.13}},
           "batched": {"us_per_gemv": 1.385, "frac": 0.854}, "grouped": {"us_per_gemv": 1.505, "frac": 0.786},
           "cpu_baseline": {"ms_per_gemv": 8.95}, "cpu_baseline_mt": [{"cores": 16, "ms_per_gemv": 0.5}],
           "side_configs": side}
    sm = bench.compact_summary(out)
    assert len(sm["side"]) == len(side)
    assert "1x32000x4096:b=12.345" in sm["side"] and "q5_1:1x4096x4096:s=12.345" in sm["side"]
    assert sm["batched_us"] == 1.385 and sm["grouped_us"] == 1.505 and sm["cpu_16t_ms"] == 0.5
    # the driver keeps about 2 KB of the tail: the summary with its key must fit in well under that
    assert len(json.dumps({"summary": sm})) < 1400
