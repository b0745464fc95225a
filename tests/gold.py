"""Fixture helpers: golden JSON records <-> HostBatch (test infrastructure)."""
import json
import os

import numpy as np

from oncrpc4j_amd import abi
from oncrpc4j_amd.columns import NP_DTYPE, HostBatch, parents

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

_FLOAT_BITS = {abi.T_FLOAT: np.uint32, abi.T_DOUBLE: np.uint64}


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def _arr(t, vals):
    if t in _FLOAT_BITS:
        return np.array(vals, dtype=_FLOAT_BITS[t]).view(NP_DTYPE[t])
    return np.array(vals, dtype=NP_DTYPE[t])


def batch_from_records(fields, records):
    """records[i][k] -> HostBatch (floats given as bit patterns, bytes as hex).
    A repeated group's slot holds its elements (each a list of member values)
    and its members' slots are None (tests/golden/make_golden.py)."""
    fields = [tuple(f) for f in fields]
    n = len(records)
    par = parents(fields)
    rowvals = {}   # field k -> its value at every row of its array

    def rows_of(k):
        if k not in rowvals:
            g = par[k]
            if g < 0:
                rowvals[k] = [r[k] for r in records]
            else:   # member of group g (an inner group's slot holds its elements): a row per element
                rowvals[k] = [e[k - g - 1] for els in rows_of(g) for e in els]
        return rowvals[k]

    arrays = []
    for k, f in enumerate(fields):
        t, kind, c = f[0], f[1], f[2]
        col = rows_of(k)
        if t == abi.T_GROUP:
            if kind == abi.K_FIXED:
                arrays.append(None)
            else:
                offs = np.zeros(len(col) + 1, dtype=np.uint64)
                np.cumsum(np.array([len(v) for v in col], dtype=np.uint64), out=offs[1:])
                arrays.append(offs)
            continue
        arrays.append(_column(t, kind, c, col, len(col)))
    return HostBatch(fields, n, arrays)


def _column(t, kind, c, col, n):
    """One field's array from its n row values."""
    if t in (abi.T_OPAQUE, abi.T_STRING):
        bs = [bytes.fromhex(v) for v in col]
        if kind == abi.K_FIXED:
            return np.frombuffer(b"".join(bs), dtype=np.uint8).reshape(n, c).copy()
        vals = np.frombuffer(b"".join(bs), dtype=np.uint8).copy()
        lens = [len(b) for b in bs]
    elif kind == abi.K_SCALAR:
        return _arr(t, col)
    elif kind == abi.K_FIXED:
        return _arr(t, col).reshape(n, c) if n else np.zeros((0, c), NP_DTYPE[t])
    else:
        vals = _arr(t, [x for v in col for x in v])
        lens = [len(v) for v in col]
    offs = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(np.array(lens, dtype=np.uint64), out=offs[1:])
    return (vals, offs)
