"""A/B of the record-marked streaming kernels (tuning key 14: 0 = direct
4-aligned windows, 1 = wave-local LDS transpose, 2 = lean) on the framed config-2
workload, interleaved rounds in one process; one JSON line per variant and
direction (median kernel ms over rounds, GB/s of algorithmic bytes)."""
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import Workload  # noqa: E402
from oncrpc4j_amd import abi, engine  # noqa: E402


def main():
    n = int(os.environ.get("RECORDS", 64 << 20))
    rounds = int(os.environ.get("ROUNDS", 7))
    reps = 5
    L = engine.lib()
    L.xdrg_internal_tune.restype = ctypes.c_int
    L.xdrg_internal_tune.argtypes = [ctypes.c_int, ctypes.c_longlong]
    wl = Workload(2, n, True, 0)
    ctx = engine.Context(0, timing=True)
    ctx.set_stream(torch.cuda.current_stream())
    times = {(v, k): [] for v in (0, 1, 2) for k in ("enc", "dec")}
    for _ in range(rounds):
        for v in (0, 1, 2):
            assert L.xdrg_internal_tune(14, v) == 0
            wl.clear_outputs()
            wl.step(ctx)
            torch.cuda.synchronize()
            wl.check()
            ctx.reset_stats()
            for _ in range(reps):
                wl.step(ctx)
            torch.cuda.synchronize()
            for kid, k in ((abi.KERNEL_FIXED_ENCODE, "enc"), (abi.KERNEL_FIXED_DECODE, "dec")):
                c, ms = ctx.kernel_stats(kid)
                times[(v, k)].append(ms / c)
    per_launch = wl.native_bytes + wl.xlen
    for (v, k), t in sorted(times.items()):
        med = statistics.median(t)
        print(json.dumps({"variant": v, "kernel": k, "median_ms": round(med, 4),
                          "GBps": round(per_launch / med / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
