"""Minimal GGUF v3 writer for test fixtures (test infrastructure; the product only reads GGUF).

Written from the published GGUF layout, independently of the library's reader (qg_gguf.hip):
magic "GGUF", u32 version, u64 tensor count, u64 kv count, key/value pairs, tensor infos
(name, u32 n_dims, u64 ne[], u32 ggml type, u64 offset), zero padding to the alignment, data.
"""
from __future__ import annotations

import struct

import numpy as np

U8, I8, U16, I16, U32, I32, F32, BOOL, STR, ARR, U64, I64, F64 = range(13)
_FMT = {U8: "<B", I8: "<b", U16: "<H", I16: "<h", U32: "<I", I32: "<i", F32: "<f", BOOL: "<?", U64: "<Q",
        I64: "<q", F64: "<d"}


def _str(s: str) -> bytes:
    b = s.encode()
    return struct.pack("<Q", len(b)) + b


def _value(t: int, v) -> bytes:
    if t == STR:
        return _str(v)
    if t == ARR:
        et, items = v
        return struct.pack("<IQ", et, len(items)) + b"".join(_value(et, x) for x in items)
    return struct.pack(_FMT[t], v)


def write_gguf(path, kvs: list[tuple[str, int, object]], tensors: list[tuple[str, int, list[int], bytes]],
               alignment: int = 32, version: int = 3, offsets: list[int] | None = None) -> None:
    """kvs: (key, gguf type, value); tensors: (name, ggml type, ne (ne[0] innermost), data bytes).
    ``offsets`` overrides the computed data offsets (to build corrupt files)."""
    head = b"GGUF" + struct.pack("<IQQ", version, len(tensors), len(kvs))
    head += b"".join(_str(k) + struct.pack("<I", t) + _value(t, v) for k, t, v in kvs)
    offs, pos = [], 0
    for _, _, _, data in tensors:
        pos = (pos + alignment - 1) // alignment * alignment
        offs.append(pos)
        pos += len(data)
    if offsets is not None:
        offs = offsets
    for (name, t, ne, _), off in zip(tensors, offs):
        head += _str(name) + struct.pack("<I", len(ne)) + b"".join(struct.pack("<Q", d) for d in ne)
        head += struct.pack("<IQ", t, off)
    head += b"\0" * ((-len(head)) % alignment)
    body = bytearray()
    for (_, _, _, data), off in zip(tensors, offs):
        if off > len(body):
            body += b"\0" * (off - len(body))
        body[off:off + len(data)] = data
    with open(path, "wb") as f:
        f.write(head + bytes(body))


def as_bytes(a: np.ndarray) -> bytes:
    return np.ascontiguousarray(a).tobytes()
