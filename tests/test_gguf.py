"""GGUF reader (qg_gguf.hip via quant_gemm.ggml.GGUFFile) — host-side, no GPU needed.

Fixtures are written by tests/gguf_writer.py (an independent writer of the published layout) with
the oracle's quantizers. No GGUF file from llama.cpp is available offline: parity with llama.cpp's
own files stays unpinned beyond the layout and the block bytes (identical to qg/blocks.h).
"""
import numpy as np
import pytest

from gguf_writer import ARR, BOOL, F32, I32, STR, U32, U64, as_bytes, write_gguf


@pytest.fixture(scope="module")
def G():
    from quant_gemm import ggml
    return ggml


def make_model(O, path, alignment=32):
    rng = np.random.default_rng(0)
    _, b = O.fill_uniform_step4(1, 8, 256, seed=1)
    q40 = O.quantize(b, O.Q4_0)
    q80 = O.quantize(b, O.Q8_0)
    q41 = O.quantize(rng.standard_normal((2, 3, 64)).astype(np.float32), O.Q4_1)
    f32 = rng.standard_normal((3, 64)).astype(np.float32)
    f16 = rng.standard_normal((5, 32)).astype(np.float16)
    kvs = [("general.architecture", STR, "llama"), ("general.alignment", U32, alignment),
           ("llama.block_count", U32, 2), ("llama.rope.freq_base", F32, 10000.0), ("x.flag", BOOL, True),
           ("x.neg", I32, -7), ("x.big", U64, 1 << 40),
           ("tokenizer.ggml.tokens", ARR, (STR, ["<s>", "</s>", "hello"]))]
    tensors = [("blk.0.attn_q.weight", O.Q4_0, [256, 8], as_bytes(q40)),
               ("blk.0.attn_k.weight", O.Q8_0, [256, 8], as_bytes(q80)),
               ("blk.0.ffn.weight", O.Q4_1, [64, 3, 2], as_bytes(q41)),
               ("norm.weight", 0, [64, 3], as_bytes(f32)),
               ("emb.weight", 1, [32, 5], as_bytes(f16))]
    write_gguf(path, kvs, tensors, alignment=alignment)
    return dict(q40=q40, q80=q80, q41=q41, f32=f32, f16=f16)


@pytest.mark.parametrize("alignment", [32, 64])
def test_gguf_directory_and_bytes(O, G, tmp_path, alignment):
    p = tmp_path / "m.gguf"
    want = make_model(O, p, alignment)
    with G.GGUFFile(p) as f:
        assert f.version == 3 and f.alignment == alignment
        md = f.metadata
        assert md["general.architecture"] == "llama" and md["llama.block_count"] == 2
        assert md["llama.rope.freq_base"] == 10000.0 and md["x.flag"] is True and md["x.neg"] == -7
        assert md["x.big"] == 1 << 40 and md["tokenizer.ggml.tokens"] == ("array", STR, 3)
        t = f.tensors
        assert [t[n].type for n in t] == [2, 8, 3, 0, 1]
        assert t["blk.0.attn_q.weight"].shape == (8, 8, 18)
        assert t["blk.0.ffn.weight"].ne == [64, 3, 2] and t["blk.0.ffn.weight"].shape == (2, 3, 2, 20)
        assert np.array_equal(f.host_bytes("blk.0.attn_q.weight"), want["q40"])
        assert np.array_equal(f.host_bytes("blk.0.attn_k.weight"), want["q80"])
        assert np.array_equal(f.host_bytes("blk.0.ffn.weight"), want["q41"])
        assert np.array_equal(f.host_bytes("norm.weight"), want["f32"])
        assert np.array_equal(f.host_bytes("emb.weight"), want["f16"])
        v = f.view("blk.0.attn_q.weight", _FakeDev(1234))
        assert v.data == 1234 and v.type == 2 and list(v.ne) == [256, 8, 1, 1]
        assert list(v.nb)[:2] == [18, 8 * 18]
        with pytest.raises(KeyError):
            f.host_bytes("nope")


class _FakeDev:
    def __init__(self, ptr):
        self.ptr = ptr

    def data_ptr(self):
        return self.ptr


def test_gguf_rejects_corrupt_files(O, G, tmp_path):
    _, b = O.fill_uniform_step4(1, 4, 64, seed=2)
    q = as_bytes(O.quantize(b, O.Q4_0))
    good = tmp_path / "g.gguf"
    write_gguf(good, [], [("w", O.Q4_0, [64, 4], q)])
    G.GGUFFile(good).close()
    raw = good.read_bytes()
    cases = {
        "magic": b"GGUX" + raw[4:],
        "truncated_data": raw[:-10],
        "truncated_header": raw[:30],
        "version": raw[:4] + (9).to_bytes(4, "little") + raw[8:],
    }
    for name, data in cases.items():
        p = tmp_path / f"{name}.gguf"
        p.write_bytes(data)
        with pytest.raises(RuntimeError):
            G.GGUFFile(p)
    # the tensor's u64 data offset: after magic/version/counts (24), name (8 + 1), n_dims (4),
    # ne (2 x 8) and type (4)
    at = 24 + 9 + 4 + 16 + 4
    assert int.from_bytes(raw[at:at + 8], "little") == 0
    for name, off in (("past", 1 << 20), ("misaligned", 8), ("overlap_end", 32)):
        p = tmp_path / f"{name}.gguf"
        p.write_bytes(raw[:at] + off.to_bytes(8, "little") + raw[at + 8:])
        with pytest.raises(RuntimeError):
            G.GGUFFile(p)
    with pytest.raises(RuntimeError):
        G.GGUFFile(tmp_path / "missing.gguf")


def test_gguf_unsupported_tensor_type_listed_not_readable(G, tmp_path):
    p = tmp_path / "u.gguf"
    write_gguf(p, [], [("q6k", 14, [256, 2], b"\0" * 420)])  # Q6_K: listed, no kernel reads it
    with G.GGUFFile(p) as f:
        assert f.tensors["q6k"].nbytes == 0
        with pytest.raises(RuntimeError):
            f.host_bytes("q6k")
