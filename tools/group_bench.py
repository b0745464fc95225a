"""Throughput of the repeated-group path (arrays of structs, recursive lists;
oncrpc4j_amd/csrc/kernels_group.hip) on two reply shapes built from
tests/golden/rpcgen/list_types.x:

* DUMP: portmapper mapping lists (pmaplist), 4 Mi records of 0..15 entries;
* READDIR: dir_list of {fileid, name<>, cookie} entries, 2 Mi records of
  0..31 entries with 8..40-byte names.

Device-resident, HIP-event timed encode and decode (median of reps); bytes =
native + XDR per direction, as bench.py counts them."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oncrpc4j_amd import abi, engine, rpcgen  # noqa: E402
from oncrpc4j_amd.columns import DeviceBatch, random_batch  # noqa: E402


def timed(fn, reps=7):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return sorted(ts)[len(ts) // 2]


def run(name, fields, n, group_len, dyn_len):
    ctx = engine.Context(0)
    ctx.apply_tuning(os.environ.get("XDRG_TUNE"))   # measurement runs only
    ctx.set_stream(torch.cuda.current_stream())
    hb = random_batch(fields, n, seed=1, dyn_len=dyn_len, group_len=group_len, special_floats=False)
    for k, f in enumerate(fields):
        if f[0] == abi.T_BOOL:
            hb.arrays[k] = (hb.arrays[k] != 0).astype(np.uint8)
    sch = engine.Schema(fields)
    db = DeviceBatch.from_host(hb)
    total = hb.xdr_total()
    out = torch.zeros(total, dtype=torch.uint8, device="cuda")
    ro = torch.zeros(n + 1, dtype=torch.int64, device="cuda")
    cols = db.columns()
    t_enc = timed(lambda: ctx.encode(sch, cols, n, out, total, rec_offsets=ro))
    back = DeviceBatch.empty(fields, n, hb.dyn_caps())
    bcols = back.columns()
    t_dec = timed(lambda: ctx.decode(sch, out, total, n, bcols, rec_offsets=ro))
    if not os.environ.get("GB_NOCHECK"):   # (experiment builds that skip work write wrong output)
        assert back.to_host().equal(hb), "round trip differs"
    nat = hb.native_bytes()
    per_dir = nat + total
    elems = hb.dyn_caps()[0]
    return {"shape": name, "records": n, "elements": elems, "xdr_bytes": total, "native_bytes": nat,
            "encode_ms": round(t_enc, 3), "decode_ms": round(t_dec, 3),
            "encode_GBps": round(per_dir / t_enc / 1e6, 1), "decode_GBps": round(per_dir / t_dec / 1e6, 1),
            "Mrec_s": round(2 * n / (t_enc + t_dec) / 1e3, 1)}


def main(which=("dump", "readdir")):
    s = rpcgen.parse_file(os.path.join(ROOT, "tests", "golden", "rpcgen", "list_types.x"))
    if "dump" in which:
        print(json.dumps(run("DUMP mapping lists", s.result_fields(400124, 1, 4), 4 << 20, (0, 15), (0, 0))))
    if "readdir" in which:
        print(json.dumps(run("READDIR dir_list", s.args_fields(400124, 1, 16), 2 << 20, (0, 31), (8, 40))))


if __name__ == "__main__":
    main(sys.argv[1:] or ("dump", "readdir"))
