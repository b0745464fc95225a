"""Config 2 (64 Mi records of 8 x int32) with struct-of-arrays native columns
— one column per field, the layout a Java BatchXdrEncoder fills (one direct
ByteBuffer per field) — against the array-of-structs
layout bench.py uses.  SoA records take the word-map kernels.  Kernel ms by
HIP events; one JSON line.

  python tools/soa_bench.py [--records N] [--reps R] [--framed]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=64 << 20)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--framed", action="store_true")
    ap.add_argument("--lane-kernel", type=int, default=None, help="tuning key 16 (0 word-map, 1 lane, 2 LDS-staged lane)")
    args = ap.parse_args()
    import torch
    from oncrpc4j_amd import abi, engine

    n = args.records
    fields = [(abi.T_INT, abi.K_SCALAR, 0)] * 8
    sch = engine.Schema(fields)
    rec = 36 if args.framed else 32
    cols_in = torch.randint(-2**31, 2**31 - 1, (8, n), dtype=torch.int32, device="cuda")
    cols_out = torch.empty_like(cols_in)
    xdr = torch.empty(n * rec, dtype=torch.uint8, device="cuda")

    def cols(t):
        arr = (abi.Column * 8)()
        for k in range(8):
            arr[k].data = t[k].data_ptr()
            arr[k].stride = 4
        return arr

    cin, cout = cols(cols_in), cols(cols_out)
    ctx = engine.Context(0, timing=True)
    if args.lane_kernel is not None:
        ctx.tune(16, args.lane_kernel)
    ctx.set_stream(torch.cuda.current_stream())
    ctx.encode(sch, cin, n, xdr, xdr.numel(), framed=args.framed, async_=True)
    ctx.decode(sch, xdr, xdr.numel(), n, cout, framed=args.framed, async_=True)
    torch.cuda.synchronize()
    assert torch.equal(cols_out, cols_in), "SoA round trip differs"
    if not args.framed:   # byte-exact against the AoS streaming path
        aos = cols_in.t().contiguous()
        x2 = torch.empty_like(xdr)
        from oncrpc4j_amd.columns import aos_columns
        ctx.encode(sch, aos_columns(fields, aos.data_ptr(), 32, [4 * k for k in range(8)]), n, x2,
                   x2.numel())
        assert torch.equal(x2, xdr), "SoA and AoS encodings differ"
    ctx.reset_stats()
    for _ in range(args.reps):
        ctx.encode(sch, cin, n, xdr, xdr.numel(), framed=args.framed, async_=True)
        ctx.decode(sch, xdr, xdr.numel(), n, cout, framed=args.framed, async_=True)
    torch.cuda.synchronize()
    _, enc = ctx.kernel_stats(abi.KERNEL_FIXED_ENCODE)
    _, dec = ctx.kernel_stats(abi.KERNEL_FIXED_DECODE)
    enc, dec = enc / args.reps, dec / args.reps
    per_launch = n * (32 + rec)
    print(json.dumps({"workload": f"{n} x 8 int32, struct-of-arrays columns" + (", framed" if args.framed else ""),
                      "lane_kernel": args.lane_kernel,
                      "encode_ms": round(enc, 4), "decode_ms": round(dec, 4),
                      "encode_GBps": round(per_launch / enc / 1e6, 1),
                      "decode_GBps": round(per_launch / dec / 1e6, 1)}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
