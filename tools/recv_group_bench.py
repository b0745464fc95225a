"""Host-memory receive of READDIR-shaped replies:
xdrg_receive_batch with XDRG_HOST_PTRS on a record-marked stream of
dir_list replies (tests/golden/rpcgen/list_types.x: a list of {fileid,
name<>, cookie} entries), the socket buffer in pageable or registered host
memory, the columns in the same kind of memory.  --schema volume_index runs
the nested-group replies of tests/golden/rpcgen/volume_index.x instead (lists
inside list elements, an optional and a union inside them).

Two staged forms (tuning key 42): 1 = the staging windows carry each
message's element rows (every stream byte crosses PCIe once), 0 = the
staged walk, deframe and body decode (three crossings).  One JSON line per
(memory, form): median wall time of the synchronous call, GB/s of stream +
native bytes; each form's columns are checked equal to the other's."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oncrpc4j_amd import abi, engine, rpcgen  # noqa: E402
from oncrpc4j_amd.columns import DeviceBatch, HostBatch, random_batch  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--replies", type=int, default=256 << 10)
    p.add_argument("--reps", type=int, default=5)
    p.add_argument("--slot-mib", type=int, default=64)
    p.add_argument("--schema", choices=["dir_list", "volume_index"], default="dir_list")
    p.add_argument("--forms", default="1,0", help="tuning key 42 values to run (1 windows, 0 three passes)")
    p.add_argument("--mems", default="pageable,registered")
    a = p.parse_args()
    from hostmem import Pageable, Registered, moved
    assert torch.cuda.is_available()
    n = a.replies
    conds = None
    if a.schema == "dir_list":
        s = rpcgen.parse_file(os.path.join(ROOT, "tests", "golden", "rpcgen", "list_types.x"))
        fields = s.args_fields(400124, 1, 16)
        hb = random_batch(fields, n, seed=1, dyn_len=(8, 40), group_len=(0, 31), special_floats=False)
        for k, f in enumerate(fields):
            if f[0] == abi.T_BOOL:
                hb.arrays[k] = (hb.arrays[k] != 0).astype(np.uint8)
    else:
        import test_volume_index as vol
        fields, conds = vol.FIELDS, vol.CONDS
        hb = vol._random(n, 1)
    ctx = engine.Context(0)
    ctx.set_stream(torch.cuda.current_stream())
    ctx.host_staging(a.slot_mib << 20, 4)
    sch = engine.Schema(fields, conds)
    # the framed stream, encoded on the device (one mark per reply: GrizzlyRpcTransport:103-110)
    db = DeviceBatch.from_host(hb)
    total = hb.xdr_total(True)
    out = torch.zeros(total, dtype=torch.uint8, device="cuda")
    ln = ctx.encode(sch, db.columns(), n, out, total, framed=True)
    stream = out[:ln].cpu().numpy()
    nat = hb.native_bytes()
    caps = hb.dyn_caps()
    # what the replies decode to (absent arms read as 0): the device receive
    rb = DeviceBatch.empty(fields, n, caps)
    ro = torch.zeros(n + 1, dtype=torch.int64, device="cuda")
    assert ctx.receive(sch, out, ln, n, rb.columns(), msg_offsets=ro)[:3] == (0, n, ln)
    ref = rb.to_host()
    results = {}
    for mem_name, Mem in (("pageable", Pageable), ("registered", Registered)):
        if mem_name not in a.mems.split(","):
            continue
        mem = Mem()
        try:
            data = mem.array(stream)
            for win in [int(v) for v in a.forms.split(",")]:
                ctx.tune(42, win)
                cols = moved(HostBatch.empty(fields, n, caps), mem)
                offs = mem.array(np.zeros(n + 1, np.uint64))
                ts = []
                for _ in range(a.reps):
                    t0 = time.perf_counter()
                    rc, nm, used, fb, err = ctx.receive(sch, data, ln, n, cols.columns(), msg_offsets=offs, host=True)
                    ts.append(time.perf_counter() - t0)
                    assert (rc, nm, used) == (0, n, ln), (rc, nm, used, fb, err)
                assert cols.equal(ref), "host receive differs from the device receive"
                ms = sorted(ts)[len(ts) // 2] * 1e3
                results[(mem_name, win)] = ms
                print(json.dumps({"schema": a.schema, "memory": mem_name, "form": "windows" if win else "three_pass",
                                  "replies": n,
                                  "entries": int(caps[min(k for k, f in enumerate(fields) if f[0] == abi.T_GROUP)]), "stream_bytes": int(ln), "native_bytes": int(nat),
                                  "ms": round(ms, 2), "GBps": round((ln + nat) / ms / 1e6, 2)}), flush=True)
            ctx.tune(0)
        finally:
            mem.close()
    for mem_name in ("pageable", "registered"):
        if (mem_name, 0) not in results or (mem_name, 1) not in results:
            continue
        print(json.dumps({"schema": a.schema, "memory": mem_name,
                          "speedup_windows_vs_three_pass": round(results[(mem_name, 0)] / results[(mem_name, 1)], 2)}))


if __name__ == "__main__":
    main()
