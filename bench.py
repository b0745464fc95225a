"""bench.py — XDR encode+decode throughput on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1]): per GPU, 64 Mi records of 8 x int32
(32 B native, 32 B XDR), seeded synthetic values, native records as an
array of structs resident in HBM.  One step = xdrg_encode_batch of the whole
batch (native -> XDR stream) + xdrg_decode_batch of that stream (XDR ->
native), both through the C-ABI of libxdrgpu.so.  Weak scaling: every rank
owns its own 64 Mi-record shard (records are independent, no data-path
collective); with --gpus > 1 the RCCL all-gather that reassembles one
contiguous stream (configs[4]) is timed separately and reported beside.

value = algorithmic bytes of all ranks / max-over-ranks wall time, GiB/s:
per record encode reads 32 B + writes 32 B, decode reads 32 + writes 32 B
= 128 B.  roofline: the dominant kernel's launches timed by
HIP events on the stream the engine launches on (xdrg_ctx_kernel_stats).
cpu_baseline: the oracle (C restatement of the reference Xdr, "port") on a
bounded sample on rank 0's host cores.
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

GIB = float(1 << 30)
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md, chip table)
HBM_COPY_GBS = 6290.0          # measured float4 copy ceiling (same table)
BYTES_PER_RECORD = 128         # encode 32+32, decode 32+32


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--records", type=int, default=64 << 20, help="records per GPU")
    p.add_argument("--framed", action="store_true", help="record-marked variant (36 B records)")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="cpu_baseline budget (0 = skip)")
    p.add_argument("--no-host-inclusive", action="store_true")
    return p.parse_args()


def dist_setup(args):
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return world, rank, local


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def max_over_ranks(x, world):
    if world == 1:
        return x
    import torch
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def cpu_baseline(budget_s):
    """Oracle (port of the reference Xdr semantics) on the host cores: encode +
    decode of a bounded sample of the same workload, all threads of the box's
    share (<= 16), repeated until the budget is spent."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    from oncrpc4j_amd import abi
    from oncrpc4j_amd.columns import HostBatch
    L = oracle.lib()
    threads = max(1, min(16, os.cpu_count() or 1))
    n = 8 << 20
    fields = [(abi.T_INT, abi.K_SCALAR, 0)] * 8
    fa = oracle.fields_array(fields)
    rng = np.random.default_rng(0x0DCAC4E5 + 2)
    nat = rng.integers(-2**31, 2**31 - 1, size=(n, 8), dtype=np.int32)
    back = np.zeros_like(nat)
    xdr = np.zeros(n * 32, dtype=np.uint8)

    def cols(a):
        arr = (abi.Column * 8)()
        for k in range(8):
            arr[k].data = a.ctypes.data + 4 * k
            arr[k].stride = 32
        return arr
    cin, cout = cols(nat), cols(back)
    out_len = ctypes.c_uint64()
    fb, err = ctypes.c_uint64(), ctypes.c_int()
    t0 = time.perf_counter()
    rounds = 0
    while True:
        rc = L.xo_encode_batch_mt(fa, 8, ctypes.addressof(cin), n, xdr.ctypes.data, xdr.size, 0,
                                  ctypes.byref(out_len), threads)
        rc |= L.xo_decode_batch_mt(fa, 8, xdr.ctypes.data, xdr.size, n, ctypes.addressof(cout), 0,
                                   ctypes.byref(fb), ctypes.byref(err), threads)
        assert rc == 0
        rounds += 1
        if time.perf_counter() - t0 >= budget_s:
            break
    dt = time.perf_counter() - t0
    assert np.array_equal(back, nat)
    return {"value": round(rounds * n * BYTES_PER_RECORD / dt / GIB, 3), "unit": "GiB/s",
            "cores": threads, "kind": "port",
            "mrecords_per_s": round(rounds * n / dt / 1e6, 2),
            "sample": f"{rounds} x (encode+decode of 8 Mi 8xint32 records), oracle/xdr_oracle.c "
                      f"xo_*_batch_mt on {threads} threads, {dt:.1f} s"}


def load_traffic(kernel, records):
    """HBM bytes per launch from the committed rocprofv3 --pmc summary
    (profiles/pmc_traffic.json, collected with separate FETCH_SIZE and
    WRITE_SIZE passes, FETCH doubled per the gfx950 correction)."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            d = json.load(f)
        e = d["kernels"][kernel]
        if e.get("records") == records:
            return e["bytes_per_launch"]
    except (OSError, KeyError, ValueError):
        pass
    return None


def host_inclusive(ctx, sch, cols_fn, n, rec_bytes):
    """H2D + encode + D2H, then H2D + decode + D2H, from pinned host buffers,
    pipelined in chunks over two streams (the path starts and ends in host
    NIO buffers)."""
    import torch
    from oncrpc4j_amd.columns import aos_columns
    nat_h = torch.randint(-2**31, 2**31 - 1, (n, 8), dtype=torch.int32).pin_memory()
    xdr_h = torch.empty(n * rec_bytes, dtype=torch.uint8).pin_memory()
    back_h = torch.empty_like(nat_h).pin_memory()
    chunk = 4 << 20
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    bufs = [(torch.empty((chunk, 8), dtype=torch.int32, device="cuda"),
             torch.empty(chunk * rec_bytes, dtype=torch.uint8, device="cuda")) for _ in streams]
    fields = sch.fields
    offs = [4 * k for k in range(8)]

    def run():
        for i, lo in enumerate(range(0, n, chunk)):
            m = min(chunk, n - lo)
            s = streams[i & 1]
            dn, dx = bufs[i & 1]
            with torch.cuda.stream(s):
                dn[:m].copy_(nat_h[lo:lo + m], non_blocking=True)
                ctx.set_stream(s)
                ctx.encode(sch, aos_columns(fields, dn.data_ptr(), 32, offs), m, dx, m * rec_bytes,
                           async_=True)
                xdr_h[lo * rec_bytes:(lo + m) * rec_bytes].copy_(dx[:m * rec_bytes], non_blocking=True)
        for i, lo in enumerate(range(0, n, chunk)):
            m = min(chunk, n - lo)
            s = streams[i & 1]
            dn, dx = bufs[i & 1]
            with torch.cuda.stream(s):
                dx[:m * rec_bytes].copy_(xdr_h[lo * rec_bytes:(lo + m) * rec_bytes], non_blocking=True)
                ctx.set_stream(s)
                ctx.decode(sch, dx, m * rec_bytes, m, aos_columns(fields, dn.data_ptr(), 32, offs),
                           async_=True)
                back_h[lo:lo + m].copy_(dn[:m], non_blocking=True)
        torch.cuda.synchronize()
    run()
    t0 = time.perf_counter()
    run()
    dt = time.perf_counter() - t0
    ok = torch.equal(back_h, nat_h)
    ctx.set_stream(torch.cuda.current_stream())
    return {"value": round(n * BYTES_PER_RECORD / dt / GIB, 3), "unit": "GiB/s",
            "ms": round(dt * 1e3, 3), "records": n, "pcie_bytes": 4 * n * 32, "roundtrip_ok": ok,
            "method": "pinned host, 4 Mi-record chunks, 2 streams, H2D/encode/D2H then H2D/decode/D2H"}


def main():
    args = parse()
    import torch
    from oncrpc4j_amd import abi, engine
    from oncrpc4j_amd.columns import aos_columns

    world, rank, local = dist_setup(args)
    n = args.records
    rec_bytes = 36 if args.framed else 32
    fields = [(abi.T_INT, abi.K_SCALAR, 0)] * 8
    offs = [4 * k for k in range(8)]
    sch = engine.Schema(fields)
    ctx = engine.Context(local, timing=True)
    stream = torch.cuda.current_stream()
    ctx.set_stream(stream)

    g = torch.Generator(device="cuda").manual_seed(0x0DCAC4E5 + 2 + rank)
    nat = torch.randint(-2**31, 2**31 - 1, (n, 8), dtype=torch.int32, device="cuda", generator=g)
    back = torch.empty_like(nat)
    xdr = torch.empty(n * rec_bytes, dtype=torch.uint8, device="cuda")
    cin = aos_columns(fields, nat.data_ptr(), 32, offs)
    cout = aos_columns(fields, back.data_ptr(), 32, offs)
    xlen = n * rec_bytes

    def step():
        ctx.encode(sch, cin, n, xdr, xlen, framed=args.framed, async_=True)
        ctx.decode(sch, xdr, xlen, n, cout, framed=args.framed, async_=True)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # correctness of the measured path (outside the timed region)
    assert torch.equal(back, nat), "decode(encode(x)) != x"
    if not args.framed:
        assert torch.equal(xdr.view(-1, 4)[:1 << 20], nat.view(torch.uint8).view(-1, 4)[:1 << 20].flip(1))
    ctx.reset_stats()

    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    barrier(world)
    dt = max_over_ranks(time.perf_counter() - t0, world)

    # per-kernel HIP-event durations (same stream, same timed region)
    ne, ms_e = ctx.kernel_stats(abi.KERNEL_FIXED_ENCODE)
    nd, ms_d = ctx.kernel_stats(abi.KERNEL_FIXED_DECODE)
    kernel = "k_wordmap_encode" if args.framed else "k_stream_bswap"
    launches = ne + nd
    avg_ms = (ms_e + ms_d) / max(launches, 1)
    per_launch_bytes = n * (rec_bytes + 32)       # read one side + write the other
    achieved = per_launch_bytes / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0

    total_records = n * world * args.steps
    value = total_records * (BYTES_PER_RECORD + (2 * 4 if args.framed else 0)) / dt / GIB

    gather = None
    if world > 1:
        import torch.distributed as dist
        full = torch.empty(world * xlen, dtype=torch.uint8, device="cuda")
        dist.all_gather_into_tensor(full, xdr)
        torch.cuda.synchronize()
        barrier(world)
        t1 = time.perf_counter()
        reps = 3
        for _ in range(reps):
            dist.all_gather_into_tensor(full, xdr)
        torch.cuda.synchronize()
        barrier(world)
        gdt = max_over_ranks((time.perf_counter() - t1) / reps, world)
        ok = torch.equal(full[rank * xlen:(rank + 1) * xlen], xdr)
        gather = {"ms": round(gdt * 1e3, 3), "bytes_in_per_gpu": (world - 1) * xlen,
                  "GBps_in_per_gpu": round((world - 1) * xlen / gdt / 1e9, 2),
                  "stream_bytes": world * xlen, "own_shard_ok": bool(ok),
                  "collective": "RCCL all_gather_into_tensor (torch.distributed nccl)"}
        del full

    cpu = None
    hinc = None
    if rank == 0 and world == 1:
        if not args.no_host_inclusive:
            hinc = host_inclusive(ctx, sch, None, min(n, 64 << 20), rec_bytes)
        if args.cpu_seconds > 0:
            cpu = cpu_baseline(args.cpu_seconds)

    if rank == 0:
        line = {
            "metric": "XDR encode+decode GiB/s (device-resident)",
            "value": round(value, 3), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int32",
            "data": "synthetic (seeded uniform int32)",
            "config": {"workload": "configs[1]: 64 Mi fixed-schema records of 8 x int32 (32 B), "
                                   "encode+decode round trip, array-of-structs native records"
                       if not args.framed else
                       "configs[1] record-marked variant (36 B XDR records)",
                       "records_per_gpu": n, "record_bytes_native": 32, "record_bytes_xdr": rec_bytes,
                       "bytes_per_record": BYTES_PER_RECORD + (8 if args.framed else 0),
                       "parallelism": f"records sharded {world} ways" if world > 1 else "single GPU"},
            "mrecords_per_s": round(total_records / dt / 1e6, 2),
            "roofline": {"bound": "hbm", "kernel": kernel, "achieved": round(achieved, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "frac_of_measured_copy": round(achieved / HBM_COPY_GBS, 4),
                         "traffic": load_traffic(kernel, n),
                         "launches": launches, "avg_launch_ms": round(avg_ms, 4),
                         "bytes_per_launch": per_launch_bytes},
            "cpu_baseline": cpu,
            "host_inclusive": hinc,
            "gather": gather,
        }
        print(json.dumps(line), flush=True)
    ctx.close()
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
