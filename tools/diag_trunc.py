"""Truncated streams (the last record cut by 3 bytes, or half the stream) under
every record-path decode (group, staged + derived counts, one pass, exact
walk, lane per record) against the oracle: first bad record and code.  The
record-mark check once lost FRAME errors here."""
import sys, numpy as np, torch
import os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import oracle
from oncrpc4j_amd import abi, engine
from oncrpc4j_amd.columns import random_batch
from test_gpu_parity import gpu_decode, oracle_decode, SCHEMAS
ctx = engine.Context(0); ctx.set_stream(torch.cuda.current_stream())
for name, framed in (("cfg2_8xint", True), ("cfg4_int_string_intvec", True), ("cfg4_int_string_intvec", False)):
    fields = SCHEMAS[name]; n = 3000
    hb = random_batch(fields, n, seed=11, dyn_len=(0, 20))
    rc, xdr, offs = oracle.encode_batch(fields, hb.columns(), n, hb.xdr_total(framed), framed=framed)
    caps = hb.dyn_caps()
    for cut in (3, len(xdr) // 2):
        bad = xdr[:len(xdr) - cut]
        o = oracle_decode(fields, bad, n, offs, caps, framed)
        res = []
        for tunes in (((9, 0),), ((9, 4),), ((9, 4), (31, 2)), ((9, 4), (31, 1)), ((9, 4), (31, 0))):
            for k, v in tunes: ctx.tune(k, v)
            g = gpu_decode(ctx, fields, bad, n, offs, caps, framed)
            ctx.tune(0)
            res.append((tunes, g[:3]))
        print(name, framed, cut, "oracle", o[:3], res, flush=True)
