"""Decode the reference's committed ``Tuning_Parameters`` MAT files into JSON fixtures.

This script is run by hand in the build container (where ``/root/reference`` exists); its
outputs ``tests/golden/*_mat.json`` are committed and are what the tests read.  It never
executes anything from the MAT files: ``scipy.io.loadmat`` parses MAT v5 data only, and the
embedded MPC-Toolbox object (an MCOS opaque blob stored in ``__function_workspace__``) is walked
here with a 60-line MAT v5 element reader that only interprets numeric arrays, structs and
cells.

What is extracted (reference file:line of the writer in brackets):
  * ``Tuning_Parameters.{N,Nu,delta,lambda,scale.{L,R,Ru,Rv}}``  [MPCTuning.m:374-381]
  * from the embedded ``mpcobj`` (the toolbox object after MPCTuning scaled it):
      - the scaled discrete plant ``Pze = L*Pz*R`` numerators/denominators, z-domain, as
        ``tfdata`` returns them, row-major (i, j)                [MPCTuning.m:162,168-169]
      - its ``iodelay`` matrix                                   [Shell3x3.m:65 c2d]
      - MV bounds scaled by R (Min/Max/RateMin/RateMax/ScaleFactor) [MPCTuning.m:170-178]
      - OV bounds scaled by L, ECRs, ScaleFactors                [MPCTuning.m:179-185]
      - Weights (MV, MVRate, OV, ECR)                            [MPCTuning.m:351-354]
      - PredictionHorizon / ControlHorizon / Ts

Usage:  python tests/golden/make_mat_fixtures.py   (writes next to this file)
"""
from __future__ import annotations

import json
import os
import struct
import sys

import numpy as np
import scipy.io as sio

REF = "/root/reference/MPC-Tuning"
HERE = os.path.dirname(os.path.abspath(__file__))

_NUM = {1: "i1", 2: "u1", 3: "<i2", 4: "<u2", 5: "<i4", 6: "<u4", 7: "<f4", 9: "<f8", 12: "<i8", 13: "<u8"}


class Node:
    def __init__(self, kind, name, dims, value=None, children=None, fields=None):
        self.kind, self.name, self.dims = kind, name, dims
        self.value, self.children, self.fields = value, children or [], fields

    def walk(self):
        yield self
        for c in self.children:
            yield from c.walk()


def _tag(buf, p):
    t, n = struct.unpack_from("<II", buf, p)
    if t >> 16:  # small data element: 4-byte tag, <=4 bytes payload
        return t & 0xFFFF, t >> 16, p + 4, p + 8
    return t, n, p + 8, p + 8 + ((n + 7) // 8) * 8


def _elements(buf, p, end):
    out = []
    while p + 8 <= end:
        t, n, dp, nxt = _tag(buf, p)
        if t == 14:
            node = _matrix(buf, dp, dp + n)
            if node is not None:
                out.append(node)
        p = nxt
    return out


def _matrix(buf, p, end):
    if end - p < 16:
        return None
    _, n, dp, p2 = _tag(buf, p)
    cls = struct.unpack_from("<I", buf, dp)[0] & 0xFF
    _, n, dp, p3 = _tag(buf, p2)
    dims = [int(x) for x in np.frombuffer(buf[dp:dp + n], "<i4")]
    _, n, dp, p4 = _tag(buf, p3)
    name = buf[dp:dp + n].decode("latin1")
    if cls == 1:  # cell
        return Node("cell", name, dims, children=_elements(buf, p4, end))
    if cls == 2:  # struct
        _, n, dp, p5 = _tag(buf, p4)
        fl = struct.unpack_from("<i", buf, dp)[0]
        _, n, dp, p6 = _tag(buf, p5)
        names = [buf[dp + i * fl: dp + (i + 1) * fl].split(b"\0")[0].decode() for i in range(n // fl)]
        return Node("struct", name, dims, children=_elements(buf, p6, end), fields=names)
    if cls in (3, 16, 17):  # object / opaque
        return Node("object", name, dims, children=_elements(buf, p4, end))
    t, n, dp, _ = _tag(buf, p4)
    if t in _NUM:
        a = np.frombuffer(buf[dp:dp + n], _NUM[t]).astype(float)
        if cls == 4:  # char
            return Node("char", name, dims, value="".join(chr(int(c)) for c in a))
        return Node("num", name, dims, value=a.reshape(dims, order="F") if len(dims) == 2 and a.size == np.prod(dims) else a)
    return Node("other", name, dims)


def _struct_rows(node):
    """Return a list (struct array elements) of dicts field->Node."""
    nf = len(node.fields)
    kids = node.children
    return [dict(zip(node.fields, kids[k * nf:(k + 1) * nf])) for k in range(len(kids) // nf)]


def _num(x):
    v = np.asarray(x.value, dtype=float)
    return [None if not np.isfinite(e) else float(e) for e in v.ravel(order="F")] if v.size != 1 else (
        float(v.ravel()[0]) if np.isfinite(v.ravel()[0]) else ("inf" if v.ravel()[0] > 0 else "-inf"))


def _jsonable(v):
    if isinstance(v, np.ndarray):
        return [_jsonable(x) for x in v.tolist()]
    if isinstance(v, list):
        return [_jsonable(x) for x in v]
    if isinstance(v, float):
        if np.isfinite(v):
            return v
        return "inf" if v > 0 else "-inf"
    return v


def decode(fname: str) -> dict:
    d = sio.loadmat(os.path.join(REF, fname))
    tp = d["Tuning_Parameters"]
    out = {"source": f"MPC-Tuning/{fname}"}
    for key in ("N", "Nu", "delta", "lambda"):
        out[key] = np.asarray(tp[key][0, 0], dtype=float).ravel().tolist()
    sc = tp["scale"][0, 0]
    if sc.size and sc.dtype.names:
        out["scale"] = {k: np.diag(np.atleast_2d(np.asarray(sc[k][0, 0], dtype=float))).tolist() for k in sc.dtype.names}
    ws = d["__function_workspace__"].tobytes()
    root = _elements(ws, 8, len(ws))
    nodes = [n for r in root for n in r.walk()]
    # --- the scaled discrete plant: two cells of my*(nu+nd) 1x2.. double rows (num, den) ---
    cells = [n for n in nodes if n.kind == "cell" and n.children and all(c.kind == "num" for c in n.children)
             and len(n.children) > 1]
    plant = None
    iod = None
    for n in nodes:
        if n.kind == "struct" and n.fields == ["Input", "Output", "IO"]:
            iod = np.asarray(n.children[2].value, dtype=float)
            break
    if iod is not None and len(cells) >= 2:
        my, nin = iod.shape
        numc = [c for c in cells if len(c.children) == my * nin]
        if len(numc) >= 2:
            num, den = numc[0], numc[1]
            plant = {
                "my": my, "nin": nin,
                # MAT cells are column-major; re-index to row-major (i, j)
                "num": [[num.children[j * my + i].value.ravel().tolist() for j in range(nin)] for i in range(my)],
                "den": [[den.children[j * my + i].value.ravel().tolist() for j in range(nin)] for i in range(my)],
                "iodelay": iod.astype(int).tolist(),
            }
    if plant is not None:
        out["plant_scaled_discrete"] = plant
    # --- MV / OV bound struct arrays and weights ---
    for n in nodes:
        if n.kind != "struct" or not n.fields:
            continue
        if n.fields[:6] == ["Min", "Max", "MinECR", "MaxECR", "RateMin", "RateMax"]:
            rows = _struct_rows(n)
            out["MV"] = [{k: _jsonable(float(np.asarray(r[k].value).ravel()[0])) for k in
                          ("Min", "Max", "MinECR", "MaxECR", "RateMin", "RateMax", "RateMinECR", "RateMaxECR",
                           "ScaleFactor") if r[k].kind == "num" and np.asarray(r[k].value).size == 1} for r in rows]
        elif n.fields[:4] == ["Min", "Max", "MinECR", "MaxECR"] and "ScaleFactor" in n.fields and "RateMin" not in n.fields:
            rows = _struct_rows(n)
            key = "OV" if "OV" not in out else "DV"
            out[key] = [{k: _jsonable(float(np.asarray(r[k].value).ravel()[0])) for k in
                         ("Min", "Max", "MinECR", "MaxECR", "ScaleFactor") if k in r and r[k].kind == "num"
                         and np.asarray(r[k].value).size == 1} for r in rows]
        elif n.fields == ["ManipulatedVariables", "ManipulatedVariablesRate", "OutputVariables", "ECR"]:
            w = dict(zip(n.fields, n.children))
            out["Weights"] = {k: _jsonable(np.asarray(v.value, dtype=float).ravel().tolist()) for k, v in w.items()}
    return out


def main():
    files = {
        "shell3x3_25jul2023": "Shell3x3_Tuning_25Jul2023_12_06.mat",
        "shell3x3_caso2": "Shell3x3_Tuning_Caso2.mat",
        "shell7x5_25jul2023": "Shell7x5_Tuning_25Jul2023_12_18.mat",
        "shell7x5_14sep2024": "Shell7x5_Tuning_14Sep2024_14_22.mat",
        "vandevusse_25jul2023": "VanDeVusse_NMPC_Tuning_25Jul2023_11_04.mat",
        "vandevusse_06dec2023": "VanDeVusse_NMPC_Tuning_06Dec2023_09_50.mat",
    }
    allfx = {}
    for key, fn in files.items():
        if not os.path.exists(os.path.join(REF, fn)):
            print("missing", fn, file=sys.stderr)
            continue
        allfx[key] = decode(fn)
    with open(os.path.join(HERE, "tuning_parameters_mat.json"), "w") as f:
        json.dump(allfx, f, indent=1)
    print("wrote", len(allfx), "fixtures")


if __name__ == "__main__":
    main()
