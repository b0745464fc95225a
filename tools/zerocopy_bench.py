"""Zero-copy payload paths on config 3 (16 Mi NFS-WRITE-shaped records,
6 x int32 + opaque<4096>): copy encode/decode vs by-reference encode
(xdrg_encode_batch_shallow) and view decode (xdrg_decode_batch_view), device
resident, HIP-event kernel times; plus the host-inclusive NFS-READ-reply
shape (headers from pinned host memory, payload left in host memory, only
the message heads cross PCIe) against the copy path that moves every
payload byte H2D and back.

  python tools/zerocopy_bench.py [--records N] [--reps R]  -> one JSON line
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=16 << 20)
    ap.add_argument("--payload", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch
    from oncrpc4j_amd import abi, engine

    n, L = args.records, args.payload
    I, O, SC, DY = abi.T_INT, abi.T_OPAQUE, abi.K_SCALAR, abi.K_DYNAMIC
    fields = [(I, SC, 0)] * 6 + [(O, DY, 0)]
    sch = engine.Schema(fields)
    g = torch.Generator(device="cuda").manual_seed(3)
    hdr = torch.randint(-2**31, 2**31 - 1, (n, 6), dtype=torch.int32, device="cuda", generator=g)
    offs = torch.arange(0, (n + 1) * L, L, dtype=torch.int64, device="cuda")
    vals = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device="cuda", generator=g)
    rec = 24 + 4 + L
    xdr = torch.empty(n * rec, dtype=torch.uint8, device="cuda")
    ro = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    head = torch.empty(n * 28, dtype=torch.uint8, device="cuda")
    hro = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    splice = torch.empty(n, dtype=torch.int64, device="cuda")
    pos = torch.empty(n, dtype=torch.int64, device="cuda")
    hdr_b = torch.empty_like(hdr)
    offs_b = torch.empty_like(offs)
    vals_b = torch.empty_like(vals)

    def cols(h, o, v):
        arr = (abi.Column * 7)()
        for k in range(6):
            arr[k].data = h.data_ptr() + 4 * k
            arr[k].stride = 24
        arr[6].data = v.data_ptr() if v is not None else None
        arr[6].offsets = o.data_ptr()
        arr[6].cap = v.numel() if v is not None else 0
        return arr

    cin, cout, cview = cols(hdr, offs, vals), cols(hdr_b, offs_b, vals_b), cols(hdr_b, offs_b, None)
    ctx = engine.Context(0, timing=True)
    ctx.set_stream(torch.cuda.current_stream())

    def timed(fn, kids):
        fn()
        torch.cuda.synchronize()
        ctx.reset_stats()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            fn()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / args.reps * 1e3
        ker = {k: round(ctx.kernel_stats(k)[1] / args.reps, 4) for k in kids}
        return round(wall, 4), ker

    VK = (abi.KERNEL_VAR_SIZE, abi.KERNEL_VAR_SCAN, abi.KERNEL_VAR_ENCODE, abi.KERNEL_VAR_DECODE)
    enc_ms, enc_k = timed(lambda: ctx.encode(sch, cin, n, xdr, xdr.numel(), rec_offsets=ro, async_=True), VK)
    dec_ms, dec_k = timed(lambda: ctx.decode(sch, xdr, xdr.numel(), n, cout, rec_offsets=ro, async_=True), VK)
    assert torch.equal(hdr_b, hdr) and torch.equal(vals_b, vals)
    sh_ms, sh_k = timed(lambda: ctx.encode_shallow(sch, cols(hdr, offs, None), n, head, head.numel(), 6,
                                                   splice, rec_offsets=hro), VK)
    # the heads are the stream minus the payloads: every record's first 28 bytes
    assert torch.equal(head.view(n, 28), xdr.view(n, rec)[:, :28])
    assert torch.equal(splice, torch.arange(n, device="cuda", dtype=torch.int64) * 28 + 28)
    hdr_b.zero_()
    vw_ms, vw_k = timed(lambda: ctx.decode_view(sch, xdr, xdr.numel(), n, cview, 6, pos, rec_offsets=ro), VK)
    assert torch.equal(hdr_b, hdr) and torch.equal(offs_b, offs)
    assert torch.equal(pos, torch.arange(n, device="cuda", dtype=torch.int64) * rec + 28)

    # host-inclusive reply send (NFS READ-like): headers + offsets in pinned
    # host memory, payload stays on the host; copy path: everything crosses
    m = min(n, 2 << 20)
    hdr_h = hdr[:m].cpu().pin_memory()
    offs_h = offs[:m + 1].cpu().pin_memory()
    vals_h = vals[:m * L].cpu().pin_memory()
    out_h = torch.empty(m * rec, dtype=torch.uint8).pin_memory()
    head_h = torch.empty(m * 28, dtype=torch.uint8).pin_memory()
    spl_h = torch.empty(m, dtype=torch.int64).pin_memory()

    def send_copy():
        hdr[:m].copy_(hdr_h, non_blocking=True)
        offs[:m + 1].copy_(offs_h, non_blocking=True)
        vals[:m * L].copy_(vals_h, non_blocking=True)
        ctx.encode(sch, cin, m, xdr, m * rec, async_=True)
        out_h.copy_(xdr[:m * rec], non_blocking=True)

    def send_shallow():
        hdr[:m].copy_(hdr_h, non_blocking=True)
        offs[:m + 1].copy_(offs_h, non_blocking=True)
        ctx.encode_shallow(sch, cols(hdr, offs, None), m, head, m * 28, 6, splice)
        head_h.copy_(head[:m * 28], non_blocking=True)
        spl_h.copy_(splice[:m], non_blocking=True)

    hc_ms, _ = timed(send_copy, ())
    hs_ms, _ = timed(send_shallow, ())
    ctx.close()
    gib = float(1 << 30)
    msg_bytes = m * rec
    print(json.dumps({
        "workload": f"{n} records of 6 x int32 + opaque<{L}> (config 3)",
        "device_resident_ms": {
            "encode_copy": enc_ms, "encode_copy_kernels": enc_k,
            "encode_by_reference": sh_ms, "encode_by_reference_kernels": sh_k,
            "decode_copy": dec_ms, "decode_copy_kernels": dec_k,
            "decode_view": vw_ms, "decode_view_kernels": vw_k},
        "algorithmic_bytes": {"encode_copy": n * (24 + L + 8 + rec), "encode_by_reference": n * (24 + 16 + 28 + 8),
                              "decode_copy": n * (rec + 24 + L + 8), "decode_view": n * (28 + 24 + 16)},
        "host_inclusive_send": {
            "records": m, "message_bytes": msg_bytes,
            "copy_ms": hc_ms, "copy_msgs_GiBps": round(msg_bytes / hc_ms * 1e3 / gib, 2),
            "by_reference_ms": hs_ms, "by_reference_msgs_GiBps": round(msg_bytes / hs_ms * 1e3 / gib, 2),
            "pcie_bytes_copy": m * (24 + 8 + L) + msg_bytes, "pcie_bytes_by_reference": m * (24 + 8 + 28 + 8)},
    }), flush=True)


if __name__ == "__main__":
    main()
