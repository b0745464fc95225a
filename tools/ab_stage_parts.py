"""Attribute config 4's staged-kernel time (k_enc_stage / k_dec_stage) by
timing encode and decode of bench.py's config-4 shard with the library named
by XDRG_LIBRARY (experiment builds that drop one part of the staged kernels).
No round-trip check: a variant that skips work writes wrong bytes on purpose.

  XDRG_LIBRARY=exp/lib_NOBYTES.so python tools/ab_stage_parts.py [records]

XDRG_TUNE="20=0,21=1" applies per-context kernel choices (xdrg_internal.h
Tuning keys) first; XDRG_PARTS=encode times only the encode (a build that
drops encode work leaves a stream the decode need not walk).
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from oncrpc4j_amd import abi, engine  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 32 << 20
    ctx = engine.Context(0, timing=True)
    ctx.set_stream(torch.cuda.current_stream())
    tune = os.environ.get("XDRG_TUNE", "")
    for kv in filter(None, tune.split(",")):
        k, v = kv.split("=")
        ctx.tune(int(k), int(v))
    cfg = int(os.environ.get("XDRG_CONFIG", "4"))
    wl = bench.Workload(ctx, cfg, n, False)
    out = {"lib": os.path.basename(os.environ.get("XDRG_LIBRARY", "libxdrgpu.so")), "tune": tune, "records": n}
    parts = os.environ.get("XDRG_PARTS", "encode,decode").split(",")   # encode probes: encode only
    if "encode" not in parts:
        wl.encode()   # the stream the decode reads (untimed)
    for name, fn in (("encode", wl.encode), ("decode", wl.decode)):
        if name not in parts:
            continue
        fn()
        torch.cuda.synchronize()
        ctx.reset_stats()
        reps = 10
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        b.synchronize()
        out[name + "_ms"] = round(a.elapsed_time(b) / reps, 3)
        for kid, kn in ((abi.KERNEL_VAR_SIZE, "size"), (abi.KERNEL_VAR_SCAN, "scan"),
                        (abi.KERNEL_VAR_ENCODE, "enc"), (abi.KERNEL_VAR_DECODE, "dec")):
            c, ms = ctx.kernel_stats(kid)
            if c:
                out[f"{name}_{kn}_ms"] = round(ms / reps, 3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
