"""A/B of the payload kernels on config 3 (tuning key 18: 0 = group kernels
copy the payload, 1 = a wave per record, 2 = a block per record), one
process, interleaved rounds; every variant round-trips on its own writes."""
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
    L = engine.lib()
    L.xdrg_internal_tune.argtypes = [ctypes.c_int, ctypes.c_longlong]
    wl = bench.Workload(3, 16 << 20, False, 0)
    ctx = engine.Context(0, timing=True)
    ctx.set_stream(torch.cuda.current_stream())
    res = {}
    for r in range(int(os.environ.get("ROUNDS", 4))):
        for v in (0, 1, 2, 3):
            assert L.xdrg_internal_tune(18, v) == 0
            if r == 0:
                wl.clear_outputs()
            ctx.reset_stats()
            wl.step(ctx)
            torch.cuda.synchronize()
            if r == 0:
                wl.check()
            for kid, name in ((abi.KERNEL_VAR_ENCODE, "enc_place"), (abi.KERNEL_VAR_DECODE, "dec_place")):
                res.setdefault((v, name), []).append(ctx.kernel_stats(kid)[1])
    L.xdrg_internal_tune(18, 3)
    for (v, name), t in sorted(res.items()):
        print(json.dumps({"config": 3, "payload": {0: "off (group kernels)", 1: "wave per record",
                                                    2: "block per record", 3: "wave per record, nontemporal"}[v],
                          "kernel": name, "median_ms": round(statistics.median(t), 3)}))
    ctx.close()


if __name__ == "__main__":
    main()
