"""READDIR-shaped decode timing only (experiment builds: XDRG_LIBRARY)."""
import os, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from tools.group_bench import timed
from oncrpc4j_amd import abi, engine, rpcgen
from oncrpc4j_amd.columns import DeviceBatch, random_batch
s = rpcgen.parse_file(os.path.join(ROOT, "tests", "golden", "rpcgen", "list_types.x"))
fields = s.args_fields(400124, 1, 16)
n = 2 << 20
ctx = engine.Context(0); ctx.set_stream(torch.cuda.current_stream())
hb = random_batch(fields, n, seed=1, dyn_len=(8, 40), group_len=(0, 31), special_floats=False)
sch = engine.Schema(fields); db = DeviceBatch.from_host(hb)
total = hb.xdr_total(); out = torch.zeros(total, dtype=torch.uint8, device="cuda")
ro = torch.zeros(n + 1, dtype=torch.int64, device="cuda")
ctx.encode(sch, db.columns(), n, out, total, rec_offsets=ro)
back = DeviceBatch.empty(fields, n, hb.dyn_caps()); bc = back.columns()
print(json.dumps({"lib": os.environ.get("XDRG_LIBRARY", "tree"), "decode_ms": round(timed(lambda: ctx.decode(sch, out, total, n, bc, rec_offsets=ro, raise_on_error=False)), 3)}))
