"""Probe: time the staged record kernels of config 4 with parts switched off
(tuning key 17: bit0 dynamic scatter, bit1 fixed scatter, bit2 stage loads,
bit3 everything after the prologue).  Outputs are wrong under a mask; the
workload is re-encoded and checked at the end.  One process, interleaved."""
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
    cfg = int(os.environ.get("CONFIG", 4))
    n = {3: 16 << 20, 4: 32 << 20}[cfg]
    L = engine.lib()
    L.xdrg_internal_tune.argtypes = [ctypes.c_int, ctypes.c_longlong]
    wl = bench.Workload(cfg, n, False, 0)
    ctx = engine.Context(0, timing=True)
    ctx.set_stream(torch.cuda.current_stream())
    wl.step(ctx)
    torch.cuda.synchronize()
    wl.check()
    masks = [int(m) for m in os.environ.get("MASKS", "0,1,2,3,4,5,8").split(",")]
    res = {}
    for r in range(5):
        for m in masks:
            assert L.xdrg_internal_tune(17, m) == 0
            ctx.reset_stats()
            wl.step(ctx)
            torch.cuda.synchronize()
            for kid, name in ((abi.KERNEL_VAR_ENCODE, "enc_place"), (abi.KERNEL_VAR_DECODE, "dec_place")):
                c, ms = ctx.kernel_stats(kid)
                res.setdefault((m, name), []).append(ms)
    assert L.xdrg_internal_tune(17, 0) == 0
    wl.clear_outputs()
    wl.step(ctx)
    torch.cuda.synchronize()
    wl.check()
    for (m, name), t in sorted(res.items()):
        print(json.dumps({"config": cfg, "skip_mask": m, "kernel": name, "median_ms": round(statistics.median(t), 4)}))
    ctx.close()


if __name__ == "__main__":
    main()
