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
    p.add_argument("--config", type=int, default=2, choices=[2, 3, 4],
                   help="BASELINE config: 2 = 8 x int32 (the metric's workload), 3 = 6 x int32 + "
                        "opaque<4096>, 4 = int32 + string(8..256) + int32<0..16>")
    p.add_argument("--records", type=int, default=0, help="records per GPU (0 = the config's size)")
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


class Workload:
    """One BASELINE config made concrete: device-resident native columns, the
    XDR stream, decode targets, and one step = encode batch + decode batch."""

    def __init__(self, cfg, n, framed, rank):
        import torch
        from oncrpc4j_amd import abi, engine
        from oncrpc4j_amd.columns import aos_columns
        self.cfg, self.n, self.framed = cfg, n, framed
        I, SC, DY = abi.T_INT, abi.K_SCALAR, abi.K_DYNAMIC
        g = torch.Generator(device="cuda").manual_seed(0x0DCAC4E5 + cfg + 1000 * rank)
        dev = "cuda"
        if cfg == 2:
            self.fields = [(I, SC, 0)] * 8
            rec = 36 if framed else 32
            self.nat = torch.randint(-2**31, 2**31 - 1, (n, 8), dtype=torch.int32, device=dev, generator=g)
            self.back = torch.empty_like(self.nat)
            offs = [4 * k for k in range(8)]
            self.cin = aos_columns(self.fields, self.nat.data_ptr(), 32, offs)
            self.cout = aos_columns(self.fields, self.back.data_ptr(), 32, offs)
            self.xlen = n * rec
            self.native_bytes = n * 32
            self.rec_offsets = None
            self.kernels = ("k_stream_framed_enc/dec" if framed else "k_stream_bswap",
                            abi.KERNEL_FIXED_ENCODE, abi.KERNEL_FIXED_DECODE)
            self.desc = ("configs[1]: 64 Mi fixed-schema records of 8 x int32 (32 B), encode+decode "
                         "round trip, array-of-structs native records" if not framed else
                         "configs[1] record-marked variant (36 B XDR records)")
        else:
            if cfg == 3:   # 6 x int32 header (AoS) + opaque<> of 4096 B
                self.fields = [(I, SC, 0)] * 6 + [(abi.T_OPAQUE, DY, 0)]
                nh = 6
                lens = torch.full((n,), 4096, dtype=torch.int64, device=dev)
            else:          # int32 + string(8..256) + int32<0..16>
                self.fields = [(I, SC, 0), (abi.T_STRING, DY, 0), (I, DY, 0)]
                nh = 1
                lens = torch.randint(8, 257, (n,), dtype=torch.int64, device=dev, generator=g)
            self.hdr = torch.randint(-2**31, 2**31 - 1, (n, nh), dtype=torch.int32, device=dev, generator=g)
            self.hdr_back = torch.empty_like(self.hdr)
            self.dyn = []       # (values, offsets, values_back, offsets_back) per dynamic field
            offs = torch.zeros(n + 1, dtype=torch.int64, device=dev)
            torch.cumsum(lens, 0, out=offs[1:])
            total = int(offs[-1])
            if cfg == 3:
                vals = torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev, generator=g)
            else:
                vals = torch.randint(97, 123, (total,), dtype=torch.uint8, device=dev, generator=g)
            self.dyn.append((vals, offs, torch.empty_like(vals), torch.empty_like(offs)))
            if cfg == 4:
                k = torch.randint(0, 17, (n,), dtype=torch.int64, device=dev, generator=g)
                o2 = torch.zeros(n + 1, dtype=torch.int64, device=dev)
                torch.cumsum(k, 0, out=o2[1:])
                v2 = torch.randint(-2**31, 2**31 - 1, (int(o2[-1]),), dtype=torch.int32, device=dev,
                                   generator=g)
                self.dyn.append((v2, o2, torch.empty_like(v2), torch.empty_like(o2)))
            self.cin = self._cols(self.hdr, [(d[0], d[1]) for d in self.dyn], nh)
            self.cout = self._cols(self.hdr_back, [(d[2], d[3]) for d in self.dyn], nh)
            # XDR sizes: fixed part + per dynamic field 4 + payload (+pad)
            size = torch.full((n,), 4 * nh + (4 if framed else 0), dtype=torch.int64, device=dev)
            for (t, kd, _), d in zip([f for f in self.fields if f[1] == DY], self.dyn):
                cnt = d[1][1:] - d[1][:-1]
                size += 4 + (cnt + ((4 - (cnt & 3)) & 3) if t in (abi.T_OPAQUE, abi.T_STRING) else 4 * cnt)
            self.xlen = int(size.sum())
            self.rec_offsets = torch.zeros(n + 1, dtype=torch.int64, device=dev)
            self.native_bytes = n * 4 * nh + sum(d[0].numel() * d[0].element_size() for d in self.dyn)
            self.kernels = ("k_enc_place/k_dec_place", abi.KERNEL_VAR_ENCODE, abi.KERNEL_VAR_DECODE)
            self.desc = ("configs[2]: 16 Mi NFS-WRITE-shaped records, 6 x int32 + opaque<4096>"
                         if cfg == 3 else
                         "configs[3]: 32 Mi records int32 + string(8..256) + int32<0..16>")
        self.xdr = torch.empty(self.xlen, dtype=torch.uint8, device=dev)
        self.sch = engine.Schema(self.fields)
        # per-record algorithmic bytes: encode reads native + writes XDR, decode the reverse
        self.bytes_per_step = 2 * (self.native_bytes + self.xlen)

    def _cols(self, hdr, dyn, nh):
        from oncrpc4j_amd import abi
        arr = (abi.Column * len(self.fields))()
        for k in range(nh):
            arr[k].data = hdr.data_ptr() + 4 * k
            arr[k].stride = 4 * nh
        for j, (v, o) in enumerate(dyn):
            arr[nh + j].data = v.data_ptr()
            arr[nh + j].offsets = o.data_ptr()
            arr[nh + j].cap = v.numel()
        arr._keep = (hdr, dyn)
        return arr

    def step(self, ctx):
        ctx.encode(self.sch, self.cin, self.n, self.xdr, self.xlen, rec_offsets=self.rec_offsets,
                   framed=self.framed, async_=True)
        ctx.decode(self.sch, self.xdr, self.xlen, self.n, self.cout, rec_offsets=self.rec_offsets,
                   framed=self.framed, async_=True)

    def clear_outputs(self):
        """Zero the XDR stream and every decode target (tools/tune_*.py: each
        kernel variant must round-trip on its own writes)."""
        self.xdr.zero_()
        if self.cfg == 2:
            self.back.zero_()
            return
        self.hdr_back.zero_()
        for _, _, vb, ob in self.dyn:
            vb.zero_()
            ob.zero_()

    def check(self):
        import torch
        if self.cfg == 2:
            assert torch.equal(self.back, self.nat), "decode(encode(x)) != x"
            if not self.framed:
                m = min(self.n, 1 << 20) * 8
                assert torch.equal(self.xdr.view(-1, 4)[:m], self.nat.view(torch.uint8).view(-1, 4)[:m].flip(1))
            return
        assert torch.equal(self.hdr_back, self.hdr), "header columns differ"
        for v, o, vb, ob in self.dyn:
            assert torch.equal(ob, o), "offsets differ"
            assert torch.equal(vb, v), "values differ"


def main():
    args = parse()
    import torch
    from oncrpc4j_amd import engine

    world, rank, local = dist_setup(args)
    n = args.records if args.records else {2: 64 << 20, 3: 16 << 20, 4: 32 << 20}[args.config]
    wl = Workload(args.config, n, args.framed, rank)
    ctx = engine.Context(local, timing=True)
    ctx.set_stream(torch.cuda.current_stream())

    for _ in range(args.warmup):
        wl.step(ctx)
    torch.cuda.synchronize()
    wl.check()   # correctness of the measured path, outside the timed region
    ctx.reset_stats()

    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        wl.step(ctx)
    torch.cuda.synchronize()
    barrier(world)
    dt = max_over_ranks(time.perf_counter() - t0, world)

    # dominant kernel(s): per-launch HIP-event durations, same stream, same region
    kname, kid_e, kid_d = wl.kernels
    ne, ms_e = ctx.kernel_stats(kid_e)
    nd, ms_d = ctx.kernel_stats(kid_d)
    launches = ne + nd
    avg_ms = (ms_e + ms_d) / max(launches, 1)
    per_launch_bytes = wl.native_bytes + wl.xlen   # one side read, the other written
    achieved = per_launch_bytes / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    step_kernel_ms = {}
    for kid, name in ((0, "fixed_encode"), (1, "fixed_decode"), (2, "var_size"), (3, "var_scan"),
                      (4, "var_encode"), (5, "var_decode")):
        c, ms = ctx.kernel_stats(kid)
        if c:
            step_kernel_ms[name] = round(ms / args.steps, 4)

    total_records = n * world * args.steps
    value = wl.bytes_per_step * world * args.steps / dt / GIB

    gather = None
    if world > 1:
        import torch.distributed as dist
        xlen = wl.xlen
        full = torch.empty(world * xlen, dtype=torch.uint8, device="cuda")
        dist.all_gather_into_tensor(full, wl.xdr)
        torch.cuda.synchronize()
        barrier(world)
        t1 = time.perf_counter()
        reps = 3
        for _ in range(reps):
            dist.all_gather_into_tensor(full, wl.xdr)
        torch.cuda.synchronize()
        barrier(world)
        gdt = max_over_ranks((time.perf_counter() - t1) / reps, world)
        ok = torch.equal(full[rank * xlen:(rank + 1) * xlen], wl.xdr)
        gather = {"ms": round(gdt * 1e3, 3), "bytes_in_per_gpu": (world - 1) * xlen,
                  "GBps_in_per_gpu": round((world - 1) * xlen / gdt / 1e9, 2),
                  "stream_bytes": world * xlen, "own_shard_ok": bool(ok),
                  "collective": "RCCL all_gather_into_tensor (torch.distributed nccl)"}
        del full

    cpu = None
    hinc = None
    if rank == 0 and world == 1 and args.config == 2 and not args.framed:
        if not args.no_host_inclusive:
            hinc = host_inclusive(ctx, wl.sch, None, min(n, 64 << 20), 32)
        if args.cpu_seconds > 0:
            cpu = cpu_baseline(args.cpu_seconds)

    if rank == 0:
        line = {
            "metric": "XDR encode+decode GiB/s (device-resident)",
            "value": round(value, 3), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int32",
            "data": "synthetic (seeded uniform int32 / random bytes / [a-z] strings)",
            "config": {"workload": wl.desc, "records_per_gpu": n, "xdr_bytes_per_gpu": wl.xlen,
                       "native_bytes_per_gpu": wl.native_bytes, "bytes_per_step_per_gpu": wl.bytes_per_step,
                       "framed": bool(args.framed),
                       "parallelism": f"records sharded {world} ways" if world > 1 else "single GPU"},
            "mrecords_per_s": round(total_records / dt / 1e6, 2),
            "roofline": {"bound": "hbm", "kernel": kname, "achieved": round(achieved, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "frac_of_measured_copy": round(achieved / HBM_COPY_GBS, 4),
                         "traffic": load_traffic(kname, n),
                         "launches": launches, "avg_launch_ms": round(avg_ms, 4),
                         "bytes_per_launch": per_launch_bytes},
            "kernel_ms_per_step": step_kernel_ms,
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
