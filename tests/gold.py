"""Fixture helpers: golden JSON records <-> HostBatch (test infrastructure)."""
import json
import os

import numpy as np

from oncrpc4j_amd import abi
from oncrpc4j_amd.columns import NP_DTYPE, HostBatch

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
    """records[i][k] -> HostBatch (floats given as bit patterns, bytes as hex)."""
    fields = [tuple(f) for f in fields]
    n = len(records)
    arrays = []
    for k, (t, kind, c) in enumerate(fields):
        col = [r[k] for r in records]
        if t in (abi.T_OPAQUE, abi.T_STRING):
            bs = [bytes.fromhex(v) for v in col]
            if kind == abi.K_FIXED:
                arrays.append(np.frombuffer(b"".join(bs), dtype=np.uint8).reshape(n, c).copy())
                continue
            vals = np.frombuffer(b"".join(bs), dtype=np.uint8).copy()
            lens = [len(b) for b in bs]
        elif kind == abi.K_SCALAR:
            arrays.append(_arr(t, col))
            continue
        elif kind == abi.K_FIXED:
            arrays.append(_arr(t, col).reshape(n, c) if n else np.zeros((0, c), NP_DTYPE[t]))
            continue
        else:
            vals = _arr(t, [x for v in col for x in v])
            lens = [len(v) for v in col]
        offs = np.zeros(n + 1, dtype=np.uint64)
        np.cumsum(np.array(lens, dtype=np.uint64), out=offs[1:])
        arrays.append((vals, offs))
    return HostBatch(fields, n, arrays)
