"""Interleaved A/B of one per-context kernel choice (xdrg_internal.h Tuning)
on a bench.py workload, one process: every variant first round-trips on its
own writes, then ROUNDS interleaved encode+decode steps; one JSON line per
variant with the median ms of each kernel class (HIP events, same stream).

  python tools/ab_knob.py --config 3 --key 18 --values 1,2 --rounds 7
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from oncrpc4j_amd import abi, engine  # noqa: E402

KERNELS = ((abi.KERNEL_FIXED_ENCODE, "fixed_enc"), (abi.KERNEL_FIXED_DECODE, "fixed_dec"),
           (abi.KERNEL_VAR_SIZE, "sizes"), (abi.KERNEL_VAR_SCAN, "scan"),
           (abi.KERNEL_VAR_ENCODE, "enc_place"), (abi.KERNEL_VAR_DECODE, "dec_place"))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--config", type=int, default=3)
    p.add_argument("--framed", action="store_true")
    p.add_argument("--records", type=int, default=0)
    p.add_argument("--key", type=int, required=True)
    p.add_argument("--values", required=True)
    p.add_argument("--rounds", type=int, default=7)
    p.add_argument("--base", default="", help="key=value,... applied before each variant")
    a = p.parse_args()
    values = [int(v) for v in a.values.split(",")]
    basek = [tuple(int(x) for x in kv.split("=")) for kv in a.base.split(",") if kv]
    ctx = engine.Context(0, timing=True)
    ctx.apply_tuning(os.environ.get("XDRG_TUNE"))   # measurement runs only
    ctx.set_stream(torch.cuda.current_stream())
    n = a.records or bench.SIZES[a.config]
    wl = bench.Workload(ctx, a.config, n, a.framed)
    res = {}
    for v in values:   # correctness of every variant on its own writes
        ctx.tune(0)
        for k, x in basek:
            ctx.tune(k, x)
        ctx.tune(a.key, v)
        wl.clear_outputs()
        wl.step()
        torch.cuda.synchronize()
        wl.check()
    for _ in range(a.rounds):
        for v in values:
            ctx.tune(0)
            for k, x in basek:
                ctx.tune(k, x)
            ctx.tune(a.key, v)
            ctx.reset_stats()
            wl.step()
            torch.cuda.synchronize()
            for kid, name in KERNELS:
                c, ms = ctx.kernel_stats(kid)
                if c:
                    res.setdefault((v, name), []).append(ms)
    ctx.tune(0)
    for (v, name), t in sorted(res.items()):
        print(json.dumps({"config": a.config, "framed": a.framed, "base": a.base, "key": a.key, "value": v, "kernel": name,
                          "median_ms": round(statistics.median(t), 4), "min_ms": round(min(t), 4)}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
