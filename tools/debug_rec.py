"""Debug: one small record-path round trip with XDRG_DEBUG kernel prints."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
os.environ["XDRG_DEBUG"] = "1"
import numpy as np
import torch
import oracle
from oncrpc4j_amd import abi, engine
from oncrpc4j_amd.columns import DeviceBatch, HostBatch, random_batch

ctx = engine.Context(0)
for fields in ([(abi.T_INT, abi.K_SCALAR, 0)] * 2 + [(abi.T_STRING, abi.K_DYNAMIC, 0)],
               [(abi.T_INT, abi.K_SCALAR, 0)] * 8):
    n = 9
    hb = random_batch(fields, n, seed=1, dyn_len=(1, 9))
    total = hb.xdr_total()
    rc, want, offs = oracle.encode_batch(fields, hb.columns(), n, total)
    sch = engine.Schema(fields)
    db = DeviceBatch.from_host(hb)
    out = torch.zeros(total, dtype=torch.uint8, device="cuda")
    o = torch.zeros(n + 1, dtype=torch.int64, device="cuda")
    ln = ctx.encode(sch, db.columns(), n, out, total, rec_offsets=o)
    print("encode ok:", out.cpu().numpy().tobytes() == want, "offs", o.cpu().tolist())
    back = DeviceBatch.empty(fields, n, hb.dyn_caps())
    r = ctx.decode(sch, out, ln, n, back.columns(), rec_offsets=o, raise_on_error=False)
    torch.cuda.synchronize()
    print("decode ->", r, flush=True)
