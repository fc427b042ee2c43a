"""Flat, self-describing binary form of a `CompiledModel` (what `dx_model_load` reads).

Layout (little endian):
    char[8]  magic  "DXMBLOB1"
    int64    count
    count x { char[48] name; int32 dtype (0=int32, 1=float64); int32 pad;
              int64 n_elems; int64 byte_offset }
    payload, every array 8-byte aligned.

The same blob feeds the HIP library (`include/dx.h`) and the CPU oracle
(`oracle/dx_oracle.h`); both look arrays up by name.
"""

from __future__ import annotations

import struct
from typing import Dict

import numpy as np

MAGIC = b"DXMBLOB1"
_NAME = 48


def pack(arrays: Dict[str, np.ndarray]) -> bytes:
    items = []
    for name, a in sorted(arrays.items()):
        a = np.asarray(a)
        if a.dtype.kind in "iub":
            items.append((name, 0, np.ascontiguousarray(a, dtype="<i4").ravel()))
        elif a.dtype.kind == "f":
            items.append((name, 1, np.ascontiguousarray(a, dtype="<f8").ravel()))
        else:
            raise TypeError(f"array {name} has unsupported dtype {a.dtype}")
    header = 8 + 8 + len(items) * (_NAME + 4 + 4 + 8 + 8)
    offset = (header + 7) & ~7
    table = bytearray()
    payload = bytearray()
    for name, code, a in items:
        if len(name) >= _NAME:
            raise ValueError(f"array name too long: {name}")
        table += name.encode().ljust(_NAME, b"\0")
        table += struct.pack("<iiqq", code, 0, a.size, offset + len(payload))
        payload += a.tobytes()
        payload += b"\0" * ((-len(payload)) % 8)
    out = bytearray(MAGIC)
    out += struct.pack("<q", len(items))
    out += table
    out += b"\0" * (offset - len(out))
    out += payload
    return bytes(out)


def unpack(blob: bytes) -> Dict[str, np.ndarray]:
    if blob[:8] != MAGIC:
        raise ValueError("not a DX model blob")
    (count,) = struct.unpack_from("<q", blob, 8)
    out = {}
    pos = 16
    for _ in range(count):
        name = blob[pos : pos + _NAME].rstrip(b"\0").decode()
        code, _, n, off = struct.unpack_from("<iiqq", blob, pos + _NAME)
        dt = "<i4" if code == 0 else "<f8"
        out[name] = np.frombuffer(blob, dtype=dt, count=n, offset=off)
        pos += _NAME + 24
    return out
