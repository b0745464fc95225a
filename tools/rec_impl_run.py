"""Runs the cfg4 (or $CONFIG) record-path workload under each record-kernel
implementation in turn ($IMPLS, kernels_rec.hip launch_rec_phase ids), for
rocprofv3 counter collection: every kernel launch is then attributable to one
implementation by its name."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from oncrpc4j_amd import engine  # noqa: E402


def main():
    cfg = int(os.environ.get("CONFIG", 4))
    impls = [int(x) for x in os.environ.get("IMPLS", "0,3").split(",")]
    reps = int(os.environ.get("REPS", 2))
    n = {3: 16 << 20, 4: 32 << 20}[cfg]
    L = engine.lib()
    L.xdrg_internal_tune.argtypes = [ctypes.c_int, ctypes.c_longlong]
    wl = bench.Workload(cfg, n, False, 0)
    ctx = engine.Context(0)
    ctx.set_stream(torch.cuda.current_stream())
    for impl in impls:
        assert L.xdrg_internal_tune(9, impl) == 0
        for _ in range(reps):
            wl.step(ctx)
        torch.cuda.synchronize()
        wl.check()
        print("impl", impl, "ok", flush=True)
    L.xdrg_internal_tune(9, engine.DEFAULT_REC_KERNEL)


if __name__ == "__main__":
    main()
