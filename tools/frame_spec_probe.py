"""The record-mark walk alone on the bench's framed streams (configs[1] and
configs[3] record-marked, bench.py Workload): xdrg_frame_scan per call (HIP
events around the C-ABI call, host round trip included, as bench.py's
receive leg reports it), the speculative walk's counters (calls, give-ups,
re-walks) and the exact kernels (tuning key 47 = 0) beside it.

  python tools/frame_spec_probe.py [reps] [configs...]   -> one JSON line per config"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from oncrpc4j_amd import abi, engine  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    cfgs = [int(c) for c in sys.argv[2:]] or [2, 4]
    ctx = engine.Context(0, timing=True)
    ctx.apply_tuning(os.environ.get("XDRG_TUNE"))
    ctx.set_stream(torch.cuda.current_stream())
    for cfg in cfgs:
        wl = bench.Workload(ctx, cfg, bench.SIZES[cfg], True, shards=(0,))
        wl.encode()
        torch.cuda.synchronize()
        want = wl.rec_offsets if wl.rec_offsets is not None else \
            torch.arange(wl.n + 1, dtype=torch.int64, device="cuda") * (wl.xlen // wl.n)
        offs = torch.empty(wl.n + 1, dtype=torch.int64, device="cuda")
        res = {"config": f"{cfg} framed", "messages": wl.n, "stream_bytes": wl.xlen}
        for mode in (1, 0):
            ctx.tune(47, mode)
            s0 = [ctx.internal_stat(k) for k in (1, 2, 3)]
            assert ctx.frame_scan(wl.xdr, wl.xlen, offs, wl.n) == wl.n
            assert torch.equal(offs, want)
            ctx.reset_stats()
            for _ in range(reps):
                ctx.frame_scan(wl.xdr, wl.xlen, offs, wl.n)
            torch.cuda.synchronize()
            n, ms = ctx.kernel_stats(abi.KERNEL_FRAME_SCAN)
            s1 = [ctx.internal_stat(k) for k in (1, 2, 3)]
            walk_bytes = wl.xlen + 8 * (wl.n + 1)
            res["spec" if mode else "exact"] = {
                "frame_scan_ms": round(ms / n, 4),
                "frac_of_8TBps": round(walk_bytes / (ms / n * 1e-3) / 8e12, 4),
                "spec_calls": s1[0] - s0[0], "gave_up": s1[1] - s0[1], "rewalks": s1[2] - s0[2]}
        ctx.tune(0)
        print(json.dumps(res), flush=True)
        del wl, offs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
