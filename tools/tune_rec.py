"""Interleaved sweep of the record-path copy unroll (encode / decode place
kernels) on BASELINE configs 3 and 4 (bench.py workloads), one process."""
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from oncrpc4j_amd import abi, engine  # noqa: E402


def main():
    cfgs = [int(c) for c in os.environ.get("CONFIGS", "4,3").split(",")]
    rounds = int(os.environ.get("ROUNDS", 5))
    L = engine.lib()
    L.xdrg_internal_tune.argtypes = [ctypes.c_int, ctypes.c_longlong]
    for cfg in cfgs:
        n = {3: 16 << 20, 4: 32 << 20}[cfg]
        wl = bench.Workload(cfg, n, False, 0)
        ctx = engine.Context(0, timing=True)
        ctx.set_stream(torch.cuda.current_stream())
        wl.step(ctx)
        torch.cuda.synchronize()
        wl.check()
        res = {}
        # (kernel, chunks per record, records per lane, lane bytes, tile bytes):
        # kernel 4 = staged sub-batches, 0 = group per record, 3 = lane per record
        if os.environ.get("QUICK"):
            variants = [(4, 2, 1, 32, 16384), (0, 2, 1, 32, 16384)]
        else:
            variants = [(4, 2, 1, lb, tb) for lb in (32, 64) for tb in (16384, 32768)] + \
                       [(0, 2, 1, 32, 16384)]
        for r in range(rounds):
            for kern, u, rr, g, tb in variants:
                assert L.xdrg_internal_tune(12, tb) == 0
                assert L.xdrg_internal_tune(9, kern) == 0
                assert L.xdrg_internal_tune(4, u) == 0
                assert L.xdrg_internal_tune(5, u) == 0
                assert L.xdrg_internal_tune(10, rr) == 0
                assert L.xdrg_internal_tune(11, rr) == 0
                assert L.xdrg_internal_tune(7, g) == 0
                assert L.xdrg_internal_tune(8, g) == 0
                if r == 0:   # every variant must round-trip on its own writes
                    wl.clear_outputs()
                ctx.reset_stats()
                wl.step(ctx)
                torch.cuda.synchronize()
                if r == 0:
                    wl.check()
                for kid, name in ((abi.KERNEL_VAR_SIZE, "sizes"), (abi.KERNEL_VAR_SCAN, "scan"),
                                  (abi.KERNEL_VAR_ENCODE, "enc_place"), (abi.KERNEL_VAR_DECODE, "dec_place")):
                    c, ms = ctx.kernel_stats(kid)
                    res.setdefault((kern, u, rr, g, tb, name), []).append(ms)
        L.xdrg_internal_tune(9, engine.DEFAULT_REC_KERNEL)   # defaults (kernels_rec.hip)
        L.xdrg_internal_tune(4, 2)
        L.xdrg_internal_tune(5, 2)
        L.xdrg_internal_tune(10, 1)
        L.xdrg_internal_tune(11, 1)
        L.xdrg_internal_tune(7, 32)
        L.xdrg_internal_tune(8, 32)
        L.xdrg_internal_tune(12, 16384)
        wl.step(ctx)
        torch.cuda.synchronize()
        wl.check()
        per_launch = wl.native_bytes + wl.xlen
        for (kern, u, rr, g, tb, name), t in sorted(res.items()):
            med = statistics.median(t)
            d = {"config": cfg, "impl": {0: "group", 3: "lane", 4: "staged"}[kern], "unroll": u, "recs": rr,
                 "lane_bytes": g, "tile": tb,
                 "kernel": name, "median_ms": round(med, 4)}
            if name.endswith("place"):
                d["GBps"] = round(per_launch / med / 1e6, 1)
            print(json.dumps(d), flush=True)
        ctx.close()
        del wl
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
