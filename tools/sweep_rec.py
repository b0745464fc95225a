"""Interleaved sweep of record-path knobs on BASELINE configs 3 and 4 (the
bench.py workloads, one process, every variant round-tripped on its own
writes first): loads in flight per lane (U chunks x R records, tuning keys
4/5 and 10/11) for the group kernels that take config 3's large records,
LDS tile bytes (key 12) and target payload bytes per lane (keys 7/8, the
lanes-per-record choice) for the staged kernels that take config 4.  One JSON
line per variant and kernel class: median ms over rounds.

  CONFIGS=3,4 ROUNDS=5 python tools/sweep_rec.py
"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from oncrpc4j_amd import abi, engine  # noqa: E402


VARIANTS = {
    3: [(f"u{u}r{r}", {4: u, 5: u, 10: r, 11: r}) for u in (1, 2, 4) for r in (1, 2)],
    4: [(f"tile{t}", {12: t}) for t in (int(x) for x in os.environ.get(
        "TILES", "4096,8192,12288,16384,24576").split(","))] +
       ([] if os.environ.get("TILES") else [(f"lanebytes{b}", {7: b, 8: b}) for b in (16, 64, 128, 256)]),
}


def run(cfg, variants, rounds):
    n = {3: 16 << 20, 4: 32 << 20}[cfg]
    ctx = engine.Context(0, timing=True)
    ctx.apply_tuning(os.environ.get("XDRG_TUNE"))   # measurement runs only
    ctx.set_stream(torch.cuda.current_stream())
    wl = bench.Workload(ctx, cfg, n, False)
    res = {}
    try:
        for r in range(rounds):
            for name, knobs in variants:
                ctx.tune(0)   # the defaults (xdrg_internal.h Tuning), then this variant's knobs
                for k, v in knobs.items():
                    ctx.tune(k, v)
                if r == 0:
                    wl.clear_outputs()
                ctx.reset_stats()
                wl.step()
                torch.cuda.synchronize()
                if r == 0:
                    wl.check()
                for kid, kn in ((abi.KERNEL_VAR_SIZE, "sizes"), (abi.KERNEL_VAR_ENCODE, "enc_place"),
                                (abi.KERNEL_VAR_DECODE, "dec_place")):
                    c, ms = ctx.kernel_stats(kid)
                    res.setdefault((name, kn), []).append(ms)
    finally:
        ctx.tune(0)
    per_launch = wl.native_bytes + wl.xlen
    for (name, kn), t in sorted(res.items()):
        med = statistics.median(t)
        d = {"config": cfg, "variant": name, "kernel": kn, "median_ms": round(med, 4)}
        if kn.endswith("place"):
            d["GBps"] = round(per_launch / med / 1e6, 1)
        print(json.dumps(d), flush=True)
    ctx.close()
    del wl
    torch.cuda.empty_cache()


def main():
    rounds = int(os.environ.get("ROUNDS", 5))
    for cfg in [int(c) for c in os.environ.get("CONFIGS", "3,4").split(",")]:
        run(cfg, VARIANTS[cfg], rounds)


if __name__ == "__main__":
    main()
