"""Minimal PLY reader/writer for Gaussian point clouds.

The reference writes and reads models with the third-party ``plyfile`` package
(scene/gaussian_model.py:7,180-246), which is not available here.  This module produces the same
files — ``binary_little_endian 1.0``, one ``vertex`` element, one ``property float <name>`` per
column in the reference's order (construct_list_of_attributes, gaussian_model.py:167-178) — and
reads binary (either endianness) and ASCII PLY with any scalar property types, so models move
between the reference and this repository in both directions.
"""
from __future__ import annotations

import os

import numpy as np

_TYPES = {  # PLY scalar type names -> numpy
    "char": "i1", "int8": "i1", "uchar": "u1", "uint8": "u1", "short": "i2", "int16": "i2",
    "ushort": "u2", "uint16": "u2", "int": "i4", "int32": "i4", "uint": "u4", "uint32": "u4",
    "float": "f4", "float32": "f4", "double": "f8", "float64": "f8",
}


def write_vertices(path: str, columns: dict[str, np.ndarray]) -> None:
    """Write one `vertex` element with float properties in the given (ordered) column order."""
    names = list(columns)
    n = len(next(iter(columns.values()))) if names else 0
    arr = np.empty(n, dtype=[(k, "<f4") for k in names])
    for k in names:
        col = np.asarray(columns[k], dtype=np.float32).reshape(-1)
        if col.shape[0] != n:
            raise ValueError(f"column {k} has {col.shape[0]} rows, expected {n}")
        arr[k] = col
    head = ["ply", "format binary_little_endian 1.0", f"element vertex {n}"]
    head += [f"property float {k}" for k in names]
    head.append("end_header")
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    with open(path, "wb") as f:
        f.write(("\n".join(head) + "\n").encode("ascii"))
        f.write(arr.tobytes())


def read_elements(path: str) -> dict[str, np.ndarray]:
    """Read every element of a PLY file: {element name: structured array}.  List properties are
    not supported (Gaussian PLYs have none)."""
    with open(path, "rb") as f:
        data = f.read()
    end = data.find(b"end_header")
    if not data.startswith(b"ply") or end < 0:
        raise ValueError(f"{path}: not a PLY file")
    nl = data.find(b"\n", end)
    header = data[:end].decode("ascii").splitlines()
    body = data[nl + 1:]
    fmt = None
    elements = []  # (name, count, [(prop, dtype)])
    for line in header[1:]:
        tok = line.split()
        if not tok or tok[0] in ("comment", "obj_info"):
            continue
        if tok[0] == "format":
            fmt = tok[1]
        elif tok[0] == "element":
            elements.append((tok[1], int(tok[2]), []))
        elif tok[0] == "property":
            if tok[1] == "list":
                raise ValueError(f"{path}: list properties are not supported")
            if tok[1] not in _TYPES:
                raise ValueError(f"{path}: unknown property type {tok[1]}")
            elements[-1][2].append((tok[2], _TYPES[tok[1]]))
    out = {}
    if fmt in ("binary_little_endian", "binary_big_endian"):
        e = "<" if fmt == "binary_little_endian" else ">"
        off = 0
        for name, count, props in elements:
            dt = np.dtype([(p, e + t) for p, t in props])
            arr = np.frombuffer(body, dtype=dt, count=count, offset=off)
            off += count * dt.itemsize
            out[name] = arr
    elif fmt == "ascii":
        lines = body.decode("ascii").split("\n")
        li = 0
        for name, count, props in elements:
            dt = np.dtype([(p, t) for p, t in props])
            arr = np.empty(count, dtype=dt)
            for i in range(count):
                vals = lines[li].split()
                li += 1
                arr[i] = tuple(vals[j] for j in range(len(props)))
            out[name] = arr
    else:
        raise ValueError(f"{path}: unsupported PLY format {fmt}")
    return out
