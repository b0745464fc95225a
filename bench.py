"""bench.py — XDR encode+decode throughput on MI355X (BASELINE.json metric).

Headline workload (BASELINE.json configs[1]): per GPU, 64 Mi records of
8 x int32 (32 B native, 32 B XDR), seeded synthetic values, native records as
an array of structs resident in HBM.  One step = xdrg_encode_batch of the
whole batch (native -> XDR stream) + xdrg_decode_batch of that stream
(XDR -> native), both through the C-ABI of libxdrgpu.so.

value = algorithmic bytes of all ranks / max-over-ranks wall time, GiB/s:
per record encode reads 32 B + writes 32 B, decode reads 32 + writes 32 B
= 128 B.  Weak scaling: every rank owns its own 64 Mi-record
shard (records are independent, no data-path collective).

`--gpus N` runs N ranks, one process per GPU: launched by torch.distributed.run
(WORLD_SIZE set, must equal N), or, when WORLD_SIZE is unset, by this script
itself, which spawns the N rank processes before anything touches a GPU.
With N > 1 the line also carries encode-only and decode-only rates and the
reassembly of one contiguous stream (configs[4]): RCCL all-gather for
fixed-size records, size exchange + grouped send/recv for variable-size ones
(oncrpc4j_amd/parallel.py), timed alone and together with the encode, and
checked byte for byte against a 1-rank encode of all ranks' records.

`extra_configs` (default run): configs[2] (6 x int32 + opaque<4096>),
configs[3] (int32 + string<8..256> + int32<0..16>) and the record-marked
configs[1], each with its own timing, dominant kernel and roofline fraction.

roofline: the dominant kernel's launches timed by HIP events on the stream the
engine launches on (xdrg_ctx_kernel_stats).  cpu_baseline: the oracle (C
restatement of the reference Xdr, "port") on bounded samples on rank 0's host
cores: configs[1] on all threads of the box's share and on one thread, and
configs[0] (int, int, string[16]) on one thread.
"""
import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

GIB = float(1 << 30)
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md, chip table)
HBM_COPY_GBS = 6290.0          # measured float4 copy ceiling (same table)
SIZES = {2: 64 << 20, 3: 16 << 20, 4: 32 << 20}
GATHER_MAX_BYTES = 80e9        # reassembled stream + its 1-rank reference must fit one GPU


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--config", type=int, default=2, choices=[2, 3, 4],
                   help="BASELINE config: 2 = 8 x int32 (the metric's workload), 3 = 6 x int32 + "
                        "opaque<4096>, 4 = int32 + string(8..256) + int32<0..16>")
    p.add_argument("--records", type=int, default=0, help="records per GPU (0 = the config's size)")
    p.add_argument("--framed", action="store_true", help="record-marked variant (36 B records)")
    p.add_argument("--extra", type=int, default=-1,
                   help="1 = also run the other BASELINE configs (default: on for the plain headline run)")
    p.add_argument("--extra-steps", type=int, default=5)
    p.add_argument("--gather-reps", type=int, default=3)
    p.add_argument("--cpu-seconds", type=float, default=15.0, help="cpu_baseline budget (0 = skip)")
    p.add_argument("--no-host-inclusive", action="store_true")
    p.add_argument("--no-check", action="store_true",
                   help="skip the round-trip checks (timing probe builds whose output is wrong by design; "
                        "never a bench line)")
    p.add_argument("--backend", default="nccl", choices=["nccl", "gloo"])
    p.add_argument("--test-codec", default="",
                   help="tests only: module providing make_workload() (CPU launcher test, gloo)")
    a = p.parse_args(argv)
    if a.extra < 0:
        a.extra = int(a.config == 2 and not a.framed and not a.records and not a.test_codec)
    return a


# ---------------------------------------------------------------------------
# launcher: one process per GPU
# ---------------------------------------------------------------------------
def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch(args, argv):
    """Spawn args.gpus rank processes of this script (RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_* set) and return the first non-zero exit status.
    Nothing in this process touches a GPU."""
    port = _free_port()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    # poll every rank: the first one that fails ends the job, so survivors
    # blocked in a rendezvous or a collective never hang the launcher
    rc = 0
    live = list(procs)
    while live and not rc:
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c:
                rc = c
                break
        if live and not rc:
            time.sleep(0.05)
    for p in live:
        if p.poll() is None:
            p.kill()
    for p in live:
        p.wait()
    return rc


class Rank:
    """This process's place in the job: world size, rank, collectives."""

    def __init__(self, args):
        import torch
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.cuda = not args.test_codec
        if self.cuda:
            torch.cuda.set_device(self.local)
            self.device = torch.device("cuda", self.local)
        else:
            self.device = torch.device("cpu")
        if self.world > 1:
            import torch.distributed as dist
            if args.backend == "nccl":
                dist.init_process_group("nccl", device_id=self.device)
            else:
                dist.init_process_group("gloo")

    def sync(self):
        if self.cuda:
            import torch
            torch.cuda.synchronize()

    def barrier(self):
        if self.world > 1:
            import torch.distributed as dist
            dist.barrier()

    def max(self, x):
        if self.world == 1:
            return x
        import torch
        import torch.distributed as dist
        t = torch.tensor([x], dtype=torch.float64, device=self.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def timed(self, fn):
        """Wall time of fn() bracketed by barrier + synchronize on both sides,
        max over ranks."""
        self.barrier()
        self.sync()
        t0 = time.perf_counter()
        fn()
        self.sync()
        self.barrier()
        return self.max(time.perf_counter() - t0)

    def close(self):
        if self.world > 1:
            import torch.distributed as dist
            dist.destroy_process_group()


# ---------------------------------------------------------------------------
# GPU workloads (one BASELINE config made concrete)
# ---------------------------------------------------------------------------
def _gen_shard(cfg, n, shard, dev):
    """Seeded synthetic records of one shard (seed 0x0DCAC4E5 + cfg + 1000 x shard)."""
    import torch
    g = torch.Generator(device=dev).manual_seed(0x0DCAC4E5 + cfg + 1000 * shard)
    I32 = dict(dtype=torch.int32, device=dev, generator=g)
    if cfg == 2:
        return {"nat": torch.randint(-2**31, 2**31 - 1, (n, 8), **I32)}
    if cfg == 3:
        lens = torch.full((n,), 4096, dtype=torch.int64, device=dev)
        hdr = torch.randint(-2**31, 2**31 - 1, (n, 6), **I32)
        vals = torch.randint(0, 256, (n * 4096,), dtype=torch.uint8, device=dev, generator=g)
        return {"hdr": hdr, "dyn": [(lens, vals)]}
    lens = torch.randint(8, 257, (n,), dtype=torch.int64, device=dev, generator=g)
    hdr = torch.randint(-2**31, 2**31 - 1, (n, 1), **I32)
    vals = torch.randint(97, 123, (int(lens.sum()),), dtype=torch.uint8, device=dev, generator=g)
    k = torch.randint(0, 17, (n,), dtype=torch.int64, device=dev, generator=g)
    v2 = torch.randint(-2**31, 2**31 - 1, (int(k.sum()),), **I32)
    return {"hdr": hdr, "dyn": [(lens, vals), (k, v2)]}


def _cat_shards(cfg, n, shards, dev):
    """The records of several shards back to back (a 1-rank batch of them)."""
    import torch
    parts = [_gen_shard(cfg, n, s, dev) for s in shards]
    if len(parts) == 1:
        return parts[0]
    if cfg == 2:
        return {"nat": torch.cat([p["nat"] for p in parts])}
    out = {"hdr": torch.cat([p["hdr"] for p in parts]), "dyn": []}
    for j in range(len(parts[0]["dyn"])):
        out["dyn"].append((torch.cat([p["dyn"][j][0] for p in parts]),
                           torch.cat([p["dyn"][j][1] for p in parts])))
    return out


class Workload:
    """Device-resident native columns, the XDR stream, decode targets; one step
    = encode batch + decode batch through the C-ABI."""

    def __init__(self, ctx, cfg, n, framed, shards=(0,), decode_targets=True):
        import torch
        from oncrpc4j_amd import abi, engine
        from oncrpc4j_amd.columns import aos_columns
        self.ctx, self.cfg, self.framed = ctx, cfg, framed
        self.n = n * len(shards)
        n = self.n
        I, SC, DY = abi.T_INT, abi.K_SCALAR, abi.K_DYNAMIC
        dev = torch.device("cuda", torch.cuda.current_device())
        d = _cat_shards(cfg, n // len(shards), list(shards), dev)
        if cfg == 2:
            self.fields = [(I, SC, 0)] * 8
            rec = 36 if framed else 32
            self.nat = d["nat"]
            self.back = torch.empty_like(self.nat) if decode_targets else None
            offs = [4 * k for k in range(8)]
            self.cin = aos_columns(self.fields, self.nat.data_ptr(), 32, offs)
            self.cout = aos_columns(self.fields, self.back.data_ptr(), 32, offs) if decode_targets else None
            self.xlen = n * rec
            self.native_bytes = n * 32
            self.rec_offsets = None
            self.kernels = ("k_stream_framed_enc/dec_lean" if framed else "k_stream_bswap",
                            abi.KERNEL_FIXED_ENCODE, abi.KERNEL_FIXED_DECODE)
            self.desc = ("configs[1]: 64 Mi fixed-schema records of 8 x int32 (32 B), encode+decode "
                         "round trip, array-of-structs native records" if not framed else
                         "configs[1] record-marked variant (36 B XDR records, one mark per record)")
        else:
            nh = 6 if cfg == 3 else 1
            self.fields = ([(I, SC, 0)] * 6 + [(abi.T_OPAQUE, DY, 0)] if cfg == 3 else
                           [(I, SC, 0), (abi.T_STRING, DY, 0), (I, DY, 0)])
            self.hdr = d["hdr"]
            self.hdr_back = torch.empty_like(self.hdr) if decode_targets else None
            self.dyn = []       # (values, offsets, values_back, offsets_back) per dynamic field
            for cnt, vals in d["dyn"]:
                o = torch.zeros(n + 1, dtype=torch.int64, device=dev)
                torch.cumsum(cnt, 0, out=o[1:])
                self.dyn.append((vals, o, torch.empty_like(vals) if decode_targets else None,
                                 torch.empty_like(o) if decode_targets else None))
            self.cin = self._cols(self.hdr, [(x[0], x[1]) for x in self.dyn], nh)
            self.cout = self._cols(self.hdr_back, [(x[2], x[3]) for x in self.dyn], nh) \
                if decode_targets else None
            # XDR sizes: fixed part + per dynamic field 4 + payload (+pad)
            size = torch.full((n,), 4 * nh + (4 if framed else 0), dtype=torch.int64, device=dev)
            for (t, _, _), x in zip([f for f in self.fields if f[1] == DY], self.dyn):
                cnt = x[1][1:] - x[1][:-1]
                size += 4 + (cnt + ((4 - (cnt & 3)) & 3) if t in (abi.T_OPAQUE, abi.T_STRING) else 4 * cnt)
            self.xlen = int(size.sum())
            del size
            self.rec_offsets = torch.zeros(n + 1, dtype=torch.int64, device=dev)
            self.native_bytes = n * 4 * nh + sum(x[0].numel() * x[0].element_size() for x in self.dyn)
            self.kernels = ("k_enc_place/k_dec_place (+payload)" if cfg == 3 else "k_enc_stage_rm/k_dec_sweep",
                            abi.KERNEL_VAR_ENCODE, abi.KERNEL_VAR_DECODE)
            self.desc = ("configs[2]: 16 Mi NFS-WRITE-shaped records, 6 x int32 + opaque<4096>"
                         if cfg == 3 else
                         "configs[3]: 32 Mi records int32 + string(8..256) + int32<0..16>")
        self.xdr = torch.empty(self.xlen, dtype=torch.uint8, device=dev)
        self.sch = engine.Schema(self.fields)
        # receive side of a record-marked stream: the mark walk's message offsets
        self.scan_offs = torch.empty(n + 1, dtype=torch.int64, device=dev) if framed and decode_targets else None
        # encode reads native + writes XDR, decode the reverse
        self.enc_bytes = self.native_bytes + self.xlen
        self.bytes_per_step = 2 * self.enc_bytes

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

    def encode(self):
        self.ctx.encode(self.sch, self.cin, self.n, self.xdr, self.xlen, rec_offsets=self.rec_offsets,
                        framed=self.framed, async_=True)

    def decode(self):
        self.ctx.decode(self.sch, self.xdr, self.xlen, self.n, self.cout, rec_offsets=self.rec_offsets,
                        framed=self.framed, async_=True)

    def step(self):
        self.encode()
        self.decode()

    def receive(self):
        """The receive pipeline of a record-marked stream (RpcMessageParserTCP
        -> RpcProtocolFilter) in one C-ABI call, xdrg_receive_batch on device
        memory: the mark walk, then the decode of every message at the offsets
        the walk found (never the encoder's), in place with its mark checked.
        Fixed-size messages: the engine checks the offsets for the fixed
        stride and takes the stride kernels (tuning key 29)."""
        rc, m, used, _, _ = self.ctx.receive(self.sch, self.xdr, self.xlen, self.n, self.cout,
                                             msg_offsets=self.scan_offs)
        assert (rc, m, used) == (0, self.n, self.xlen), f"receive: {rc}, {m} of {self.n} messages, {used} bytes"

    def clear_outputs(self):
        """Zero the XDR stream and every decode target (tools/sweep_rec.py:
        each kernel variant must round-trip on its own writes)."""
        self.xdr.zero_()
        if self.cfg == 2:
            self.back.zero_()
            return
        self.hdr_back.zero_()
        for _, _, vb, ob in self.dyn:
            vb.zero_()
            ob.zero_()

    def xdr_view(self):
        return self.xdr

    def offsets_view(self):
        return self.rec_offsets

    def check_receive(self):
        import torch
        want = self.rec_offsets if self.rec_offsets is not None else \
            torch.arange(self.n + 1, dtype=torch.int64, device=self.xdr.device) * (self.xlen // self.n)
        assert torch.equal(self.scan_offs, want), "frame scan offsets differ from the stream's records"
        self.check()

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

    def reset_stats(self):
        self.ctx.reset_stats()

    def roofline(self, steps):
        """Dominant kernel's average launch (HIP events, same stream) -> roofline dict."""
        kname, kid_e, kid_d = self.kernels
        ne, ms_e = self.ctx.kernel_stats(kid_e)
        nd, ms_d = self.ctx.kernel_stats(kid_d)
        launches = ne + nd
        avg_ms = (ms_e + ms_d) / max(launches, 1)
        per_launch = self.enc_bytes   # one side read, the other written
        achieved = per_launch / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
        step_ms = {}
        for kid, name in ((0, "fixed_encode"), (1, "fixed_decode"), (2, "var_size"), (3, "var_scan"),
                          (4, "var_encode"), (5, "var_decode")):
            c, ms = self.ctx.kernel_stats(kid)
            if c:
                step_ms[name] = round(ms / steps, 4)
        traffic, traffic_src = load_traffic(self.cfg, self.framed, self.n)
        roof = {"bound": "hbm", "kernel": kname, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                "frac_of_measured_copy": round(achieved / HBM_COPY_GBS, 4),
                "traffic": traffic, "traffic_source": traffic_src,
                "launches": launches, "avg_launch_ms": round(avg_ms, 4), "bytes_per_launch": per_launch}
        return roof, step_ms

    def gatherable(self, world):
        return world * self.xlen <= GATHER_MAX_BYTES

    def reference(self, world, n_per_rank):
        """A 1-rank workload holding every rank's records (encode only)."""
        return Workload(self.ctx, self.cfg, n_per_rank, self.framed, shards=range(world),
                        decode_targets=False)


def load_traffic(cfg, framed, records):
    """(HBM bytes per launch of the dominant kernel(s), their source) from the
    committed rocprofv3 --pmc summary (profiles/pmc_traffic.json,
    tools/pmc_summary.py: separate FETCH_SIZE and WRITE_SIZE passes over
    bench.py, FETCH doubled per the gfx950 correction; record configs average
    their encode and decode place kernels, as `achieved` does), or (None,
    reason) when the summary was taken on another record count.  The traffic
    is not measured in this run: PMC counters need their own rocprofv3 pass."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    key = f"{cfg}{'f' if framed else ''}"
    try:
        with open(p) as f:
            d = json.load(f)
        e = d["configs"][key]
        src = {"file": "profiles/pmc_traffic.json", "config_key": key, "tag": e.get("tag"),
               "records": e.get("records"), "kernels": {"encode": e.get("encode"), "decode": e.get("decode")},
               "measured_in_this_run": False}
        if e.get("records") == records:
            return e["bytes_per_launch"], src
        return None, dict(src, note="profiled on another record count")
    except (OSError, KeyError, ValueError):
        return None, {"file": "profiles/pmc_traffic.json", "config_key": key, "note": "no entry"}


# ---------------------------------------------------------------------------
# measurement legs
# ---------------------------------------------------------------------------
def gather_leg(R, wl, n_per_rank, reps):
    """Reassemble one contiguous stream from every rank's shard (exact-size
    exchange, parallel.py): timed alone and with the encode, checked against
    a 1-rank encode of all ranks' records and by a checksum every rank agrees on."""
    import torch
    from oncrpc4j_amd import parallel
    local, loffs = wl.xdr_view(), wl.offsets_view()
    sizes = parallel.all_gather_ints(local.numel())
    total = sum(sizes)
    out = torch.empty(total, dtype=torch.uint8, device=local.device)
    out_offs = torch.empty(wl.n * R.world + 1, dtype=torch.int64, device=local.device) \
        if loffs is not None else None

    def gather():
        parallel.gather_stream(local, loffs, out=out, out_offsets=out_offs)

    gather()
    t_g = R.timed(lambda: [gather() for _ in range(reps)]) / reps

    def enc_gather():
        for _ in range(reps):
            wl.encode()
            gather()
    t_eg = R.timed(enc_gather) / reps
    h = parallel.stream_hash(out)
    hashes = parallel.all_gather_ints(h)
    equal = None
    if R.rank == 0:
        ref = wl.reference(R.world, n_per_rank)
        ref.encode()
        R.sync()
        equal = bool(torch.equal(out, ref.xdr_view()))
        if loffs is not None:
            equal = equal and bool(torch.equal(out_offs, ref.offsets_view()))
        del ref
    R.barrier()
    fixed = len(set(sizes)) == 1 and out.is_cuda
    enc_all = wl.enc_bytes * R.world
    res = {"ms": round(t_g * 1e3, 3), "encode_plus_gather_ms": round(t_eg * 1e3, 3),
           "stream_bytes": total, "bytes_in_per_gpu": total - sizes[R.rank],
           "GBps_in_per_gpu": round((total - sizes[R.rank]) / t_g / 1e9, 2),
           "gather_inclusive_GiB_s": round(enc_all / t_eg / GIB, 3),
           "gather_inclusive_stream_GiB_s": round(total / t_eg / GIB, 3),
           "gather_inclusive_Mrec_s": round(wl.n * R.world / t_eg / 1e6, 2),
           "collective": ("RCCL all_gather_into_tensor (equal shard sizes)" if fixed else
                          "size all-gather + grouped send/recv (batch_isend_irecv), exact shard bytes"),
           "check": {"equal_to_1rank_encode": equal, "checksum_ranks_agree": len(set(hashes)) == 1}}
    del out, out_offs
    return res


def measure(R, args, make, cfg, framed, n, steps, warmup, with_gather):
    """One config: encode+decode steps (the value), encode-only and decode-only
    steps, the dominant kernel's roofline, and (N > 1) the stream reassembly."""
    wl = make(cfg, n, framed)
    for _ in range(warmup):
        wl.step()
    R.sync()
    if not args.no_check:
        wl.check()   # correctness of the measured path, outside the timed region
    wl.reset_stats()
    dt = R.timed(lambda: [wl.step() for _ in range(steps)])
    roof, step_ms = wl.roofline(steps)
    t_enc = R.timed(lambda: [wl.encode() for _ in range(steps)])
    t_dec = R.timed(lambda: [wl.decode() for _ in range(steps)])
    R.sync()
    if not args.no_check:
        wl.check()
    recs = wl.n * R.world * steps
    e = {"config": cfg, "framed": bool(framed), "workload": wl.desc, "records_per_gpu": wl.n,
         "xdr_bytes_per_gpu": wl.xlen, "native_bytes_per_gpu": wl.native_bytes,
         "bytes_per_step_per_gpu": wl.bytes_per_step, "steps": steps,
         "ms_per_step": round(dt / steps * 1e3, 4),
         "GiB_s": round(wl.bytes_per_step * R.world * steps / dt / GIB, 3),
         "Mrec_s": round(recs / dt / 1e6, 2),
         "encode_only": {"ms_per_step": round(t_enc / steps * 1e3, 4),
                         "GiB_s": round(wl.enc_bytes * R.world * steps / t_enc / GIB, 3),
                         "Mrec_s": round(recs / t_enc / 1e6, 2)},
         "decode_only": {"ms_per_step": round(t_dec / steps * 1e3, 4),
                         "GiB_s": round(wl.enc_bytes * R.world * steps / t_dec / GIB, 3),
                         "Mrec_s": round(recs / t_dec / 1e6, 2)},
         "roofline": roof, "kernel_ms_per_step": step_ms, "gather": None}
    if framed and hasattr(wl, "receive") and wl.scan_offs is not None:
        e["receive"] = receive_leg(R, wl, steps)
    if R.world > 1 and with_gather:
        if wl.gatherable(R.world):
            e["gather"] = gather_leg(R, wl, n, args.gather_reps)
        else:
            e["gather"] = {"skipped": f"{R.world} x {wl.xlen} stream bytes do not fit one GPU "
                                      "next to their 1-rank reference"}
    return e, wl


def receive_leg(R, wl, steps):
    """Receive pipeline on the bench clock: frame scan of the record-marked
    stream, then the decode at the scan's offsets (RpcMessageParserTCP.java:
    44-140 -> RpcProtocolFilter).  Bytes = the decode direction's (stream read,
    native written); the walk's roofline = stream bytes read + 8 B of offsets
    per message, over its average call (host round trips included)."""
    from oncrpc4j_amd import abi
    wl.receive()
    R.sync()
    wl.check_receive()
    wl.reset_stats()
    dt = R.timed(lambda: [wl.receive() for _ in range(steps)])
    R.sync()
    wl.check_receive()
    ns, ms_s = wl.ctx.kernel_stats(abi.KERNEL_FRAME_SCAN)
    walk_ms = ms_s / max(ns, 1)
    walk_bytes = wl.xlen + 8 * (wl.n + 1)
    walk_gbs = walk_bytes / (walk_ms * 1e-3) / 1e9 if walk_ms > 0 else 0.0
    step_ms = {}
    for kid, name in ((0, "fixed_encode"), (1, "fixed_decode"), (2, "var_size"), (3, "var_scan"),
                      (4, "var_encode"), (5, "var_decode"), (6, "frame_scan")):
        c, ms = wl.ctx.kernel_stats(kid)
        if c:
            step_ms[name] = round(ms / steps, 4)
    return {"ms_per_step": round(dt / steps * 1e3, 4),
            "GiB_s": round(wl.enc_bytes * R.world * steps / dt / GIB, 3),
            "Mrec_s": round(wl.n * R.world * steps / dt / 1e6, 2),
            "kernel_ms_per_step": step_ms,
            "frame_scan": {"calls": ns, "avg_ms": round(walk_ms, 4), "bytes_per_call": walk_bytes,
                           "achieved_GBps": round(walk_gbs, 1), "peak": HBM_PEAK_GBS,
                           "frac": round(walk_gbs / HBM_PEAK_GBS, 4)},
            "offsets": "the frame scan's (checked equal to the stream's record offsets)"}


# ---------------------------------------------------------------------------
# CPU baseline (oracle, rank 0, N = 1 only)
# ---------------------------------------------------------------------------
def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_threads():
    """Threads of this process's CPU share: the affinity mask, capped by the
    box's per-GPU share (OMP_NUM_THREADS is set to it on the GPU box)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    share = int(os.environ.get("OMP_NUM_THREADS") or aff)
    return max(1, min(aff, share)), aff


def cpu_baseline(budget_s):
    """Oracle (C restatement of the reference Xdr semantics) on the host
    cores, bounded samples of the same workloads (oracle/xdr_oracle.c;
    the reference's own harness is oncrpc4j-benchmark XdrBenchmark.java:17-59):
    configs[1] on every thread of the share and on one thread, configs[0]
    (int, int, string[16]) on one thread."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    from oncrpc4j_amd import abi
    L = oracle.lib()
    threads, aff = _cpu_threads()
    leg_s = budget_s / 3.0

    def rounds_for(fn, seconds):
        t0 = time.perf_counter()
        r = 0
        while True:
            fn()
            r += 1
            if time.perf_counter() - t0 >= seconds:
                return r, time.perf_counter() - t0

    # configs[1]: 8 x int32 AoS, 128 B per record round trip
    n2 = 8 << 20
    f2 = [(abi.T_INT, abi.K_SCALAR, 0)] * 8
    fa2 = oracle.fields_array(f2)
    rng = np.random.default_rng(0x0DCAC4E5 + 2)
    nat = rng.integers(-2**31, 2**31 - 1, size=(n2, 8), dtype=np.int32)
    back = np.zeros_like(nat)
    xdr = np.zeros(n2 * 32, dtype=np.uint8)

    def cols(a):
        arr = (abi.Column * 8)()
        for k in range(8):
            arr[k].data = a.ctypes.data + 4 * k
            arr[k].stride = 32
        return arr
    cin, cout = cols(nat), cols(back)
    out_len = ctypes.c_uint64()
    fb, err = ctypes.c_uint64(), ctypes.c_int()

    def cfg2(th):
        def run():
            rc = L.xo_encode_batch_mt(fa2, 8, ctypes.addressof(cin), n2, xdr.ctypes.data, xdr.size, 0,
                                      ctypes.byref(out_len), th)
            rc |= L.xo_decode_batch_mt(fa2, 8, xdr.ctypes.data, xdr.size, n2, ctypes.addressof(cout), 0,
                                       ctypes.byref(fb), ctypes.byref(err), th)
            assert rc == 0
        r, dt = rounds_for(run, leg_s)
        assert np.array_equal(back, nat)
        back[:] = 0
        return {"GiB_s": round(r * n2 * 128 / dt / GIB, 3), "Mrec_s": round(r * n2 / dt / 1e6, 2),
                "threads": th, "sample": f"{r} x encode+decode of 8 Mi 8xint32 records, {dt:.1f} s"}

    all_cores = cfg2(threads)
    single = cfg2(1)

    # configs[0]: (int a, int b, string s) with s 16 ASCII bytes, one thread;
    # 104 B per record round trip (2 x (native 24 + XDR 28))
    n1 = 1 << 20
    f1 = [(abi.T_INT, abi.K_SCALAR, 0), (abi.T_INT, abi.K_SCALAR, 0), (abi.T_STRING, abi.K_DYNAMIC, 0)]
    rng1 = np.random.default_rng(0x0DCAC4E5 + 1)
    a1 = rng1.integers(-2**31, 2**31 - 1, size=n1, dtype=np.int32)
    b1 = rng1.integers(-2**31, 2**31 - 1, size=n1, dtype=np.int32)
    s1 = rng1.integers(97, 123, size=16 * n1, dtype=np.uint8)
    o1 = np.arange(0, 16 * (n1 + 1), 16, dtype=np.uint64)
    ab, bb, sb, ob = np.zeros_like(a1), np.zeros_like(b1), np.zeros_like(s1), np.zeros_like(o1)

    def cols1(a, b, s, o):
        arr = (abi.Column * 3)()
        arr[0].data, arr[1].data = a.ctypes.data, b.ctypes.data
        arr[2].data, arr[2].offsets, arr[2].cap = s.ctypes.data, o.ctypes.data, s.size
        return arr
    c1in, c1out = cols1(a1, b1, s1, o1), cols1(ab, bb, sb, ob)
    fa1 = oracle.fields_array(f1)
    x1 = np.zeros(28 * n1, dtype=np.uint8)
    ro1 = np.zeros(n1 + 1, dtype=np.uint64)

    def run1():
        rc = L.xo_encode_batch(fa1, 3, ctypes.addressof(c1in), n1, x1.ctypes.data, x1.size, ro1.ctypes.data, 0,
                               ctypes.byref(out_len))
        rc |= L.xo_decode_batch(fa1, 3, x1.ctypes.data, x1.size, ro1.ctypes.data, n1, ctypes.addressof(c1out), 0,
                                ctypes.byref(fb), ctypes.byref(err))
        assert rc == 0
    r1, dt1 = rounds_for(run1, leg_s)
    assert np.array_equal(ab, a1) and np.array_equal(bb, b1) and np.array_equal(sb, s1)
    cfg1 = {"GiB_s": round(r1 * n1 * 104 / dt1 / GIB, 3), "Mrec_s": round(r1 * n1 / dt1 / 1e6, 2),
            "threads": 1, "sample": f"{r1} x encode+decode of 1 Mi (int, int, string[16]) records, {dt1:.1f} s"}

    return {"value": all_cores["GiB_s"], "unit": "GiB/s", "cores": threads, "kind": "port",
            "mrecords_per_s": all_cores["Mrec_s"],
            "sample": f"configs[1] {all_cores['sample']} on {threads} threads (oracle/xdr_oracle.c "
                      f"xo_*_batch_mt)",
            "cfg2_all_cores": all_cores, "cfg2_single_thread": single, "cfg1_single_thread": cfg1,
            "nproc": os.cpu_count(), "affinity_cpus": aff, "threads_used": threads,
            "cpu_model": _cpu_model(),
            "note": "threads_used = the CPU share of one GPU on the box (OMP_NUM_THREADS); nproc counts "
                    "the whole host"}


def cpu_var_baseline(cfg, seconds):
    """Oracle (oracle/xdr_oracle.c xo_encode_batch / xo_decode_batch, the
    reference Xdr semantics) on a bounded sample of configs[2] / configs[3]:
    one Python thread per core of the share, each encoding and decoding its
    own slice of records of the config's shape (ctypes drops the GIL), GiB/s
    of native + XDR bytes both ways, as the GPU line counts them."""
    import threading
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    from oncrpc4j_amd import abi
    L = oracle.lib()
    threads, _ = _cpu_threads()
    n = 2048 if cfg == 3 else 65536
    I, SC, DY = abi.T_INT, abi.K_SCALAR, abi.K_DYNAMIC
    fields = [(I, SC, 0)] * 6 + [(abi.T_OPAQUE, DY, 0)] if cfg == 3 else \
        [(I, SC, 0), (abi.T_STRING, DY, 0), (I, DY, 0)]
    fa = oracle.fields_array(fields)

    def make(seed):
        rng = np.random.default_rng(0x0DCAC4E5 + 100 * cfg + seed)
        if cfg == 3:
            hdr = rng.integers(-2**31, 2**31 - 1, (n, 6), dtype=np.int32)
            vals = rng.integers(0, 256, n * 4096, dtype=np.uint8)
            offs = np.arange(0, 4096 * (n + 1), 4096, dtype=np.uint64)
            dyn = [(vals, offs)]
        else:
            hdr = rng.integers(-2**31, 2**31 - 1, (n, 1), dtype=np.int32)
            lens = rng.integers(8, 257, n)
            so = np.zeros(n + 1, np.uint64)
            np.cumsum(lens, out=so[1:])
            sv = rng.integers(97, 123, int(so[-1]), dtype=np.uint8)
            k = rng.integers(0, 17, n)
            io = np.zeros(n + 1, np.uint64)
            np.cumsum(k, out=io[1:])
            iv = rng.integers(-2**31, 2**31 - 1, int(io[-1]), dtype=np.int32)
            dyn = [(sv, so), (iv, io)]
        nh = hdr.shape[1]

        def cols(h, d):
            arr = (abi.Column * len(fields))()
            for j in range(nh):
                arr[j].data = h.ctypes.data + 4 * j
                arr[j].stride = 4 * nh
            for j, (v, o) in enumerate(d):
                arr[nh + j].data, arr[nh + j].offsets, arr[nh + j].cap = v.ctypes.data, o.ctypes.data, v.size
            arr._keep = (h, d)
            return arr
        hb = np.zeros_like(hdr)
        db = [(np.zeros_like(v), np.zeros_like(o)) for v, o in dyn]
        native = hdr.nbytes + sum(int(o[-1]) * v.itemsize for v, o in dyn)
        xcap = 2 * native + 16 * n + 4096   # >= every record's XDR bytes (pads included)
        return cols(hdr, dyn), cols(hb, db), native, np.zeros(xcap, np.uint8), \
            np.zeros(n + 1, np.uint64), (hdr, dyn, hb, db)

    work = [make(t) for t in range(threads)]
    done = [0] * threads
    xbytes = [0] * threads

    def run(t):
        cin, cout, native, x, ro, _ = work[t]
        ol = ctypes.c_uint64()
        fb, er = ctypes.c_uint64(), ctypes.c_int()
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            rc = L.xo_encode_batch(fa, len(fields), ctypes.addressof(cin), n, x.ctypes.data, x.size, ro.ctypes.data,
                                   0, ctypes.byref(ol))
            rc |= L.xo_decode_batch(fa, len(fields), x.ctypes.data, ol.value, ro.ctypes.data, n,
                                    ctypes.addressof(cout), 0, ctypes.byref(fb), ctypes.byref(er))
            assert rc == 0
            done[t] += 1
            xbytes[t] = ol.value
    ths = [threading.Thread(target=run, args=(t,)) for t in range(threads)]
    t0 = time.perf_counter()
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    dt = time.perf_counter() - t0
    assert np.array_equal(work[0][5][0], work[0][5][2]), "oracle round trip"
    tot = sum(done[t] * 2 * (work[t][2] + xbytes[t]) for t in range(threads))
    recs = sum(done) * n
    return {"value": round(tot / dt / GIB, 3), "unit": "GiB/s", "cores": threads, "kind": "port",
            "mrecords_per_s": round(recs / dt / 1e6, 3),
            "sample": f"{sum(done)} x encode+decode of {n} configs[{cfg - 1}] records ({threads} threads, one "
                      f"record slice each, oracle/xdr_oracle.c), {dt:.1f} s"}


def _host_buffer(nbytes, register):
    """Page-aligned host buffer (anonymous mapping), optionally pinned with
    xdrg_host_register the way a JNI caller pins its pooled direct buffers."""
    import mmap
    import numpy as np
    from oncrpc4j_amd import engine
    m = mmap.mmap(-1, nbytes)
    a = np.frombuffer(m, dtype=np.uint8)
    ptr = ctypes.addressof(ctypes.c_char.from_buffer(m))
    if register:
        engine.host_register(ptr, nbytes)
    return m, a, ptr


def host_inclusive(device, sch, n, reps=3, slot_bytes=64 << 20, slots=4,
                   legs=("staged", "staged_dma", "mapped", "staged_pageable")):
    """Host-resident batches through the C-ABI (XDRG_HOST_PTRS), configs[1]:
    a server's two directions at once, one context per thread (Xdr's single
    owner, Xdr.java:56,71) — replies encode native records from host memory
    into a host XDR stream, requests decode a received host stream into host
    records.  Legs: `staged` (the context's staging ring: chunked H2D /
    kernels / D2H on its own streams, the copies by copy kernels),
    `staged_dma` (the same with the copies on the DMA engines) and `mapped` (XDRG_HOST_MAPPED: the
    kernels read and write the host buffers in place over PCIe), both on
    buffers pinned with xdrg_host_register; `staged_pageable` the same ring on
    unregistered memory (pinned bounce copies), on a quarter of the records.
    value = the best leg whose round trip is exact; rate = 128 B per record
    (both directions' native + XDR bytes) / wall time of the pair."""
    import threading
    import numpy as np
    from oncrpc4j_amd import engine
    from oncrpc4j_amd.columns import aos_columns
    offs = [4 * k for k in range(8)]
    fields = sch.fields
    rng = np.random.default_rng(0x0DCAC4E5 + 2)

    def leg(m, register, mode):
        bufs = [_host_buffer(m * 32, register) for _ in range(4)]
        (_, nat, p_nat), (_, xdr, p_xdr), (_, req, p_req), (_, back, p_back) = bufs
        nat.view(np.int32)[:] = rng.integers(-2**31, 2**31 - 1, m * 8, dtype=np.int32)
        ce, cd = engine.Context(device), engine.Context(device)
        for c_ in (ce, cd):
            c_.apply_tuning(os.environ.get("XDRG_TUNE"))   # measurement runs only
        for c in (ce, cd):
            c.host_staging(slot_bytes, slots)
            if mode == "staged_dma":   # the ring's copies on the DMA engines instead of copy kernels
                c.tune(26, 0)
        kw = {"mapped": True} if mode == "mapped" else {"host": True}
        # the request stream a peer sent: these records' encoding
        ce.encode(sch, aos_columns(fields, p_nat, 32, offs), m, p_req, m * 32, host=True)

        def enc():
            for _ in range(reps):
                ce.encode(sch, aos_columns(fields, p_nat, 32, offs), m, p_xdr, m * 32, **kw)

        def dec():
            for _ in range(reps):
                cd.decode(sch, p_req, m * 32, m, aos_columns(fields, p_back, 32, offs), **kw)

        enc()   # warm: rings, bounce buffers
        dec()
        xdr[:] = 0
        back[:] = 0
        ts = [threading.Thread(target=enc), threading.Thread(target=dec)]
        t0 = time.perf_counter()
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        dt = (time.perf_counter() - t0) / reps
        ok = bool(np.array_equal(back, nat)) and bool(np.array_equal(xdr, req))
        for c in (ce, cd):
            c.close()
        for mm, _, ptr in bufs:
            if register:
                engine.host_unregister(ptr)
        del nat, xdr, req, back, bufs   # the mappings go with their last reference
        return {"GiB_s": round(m * 128 / dt / GIB, 3), "ms": round(dt * 1e3, 3), "records": m,
                "pcie_GBps": round(4 * m * 32 / dt / 1e9, 2), "roundtrip_ok": ok}

    res = {}
    for name in legs:
        res[name] = leg(max(n // 4, 1), False, "staged") if name == "staged_pageable" else \
            leg(n, True, name)   # staged, staged_dma, mapped
    best = max((k for k in ("staged", "staged_dma", "mapped") if k in res and res[k]["roundtrip_ok"]),
               key=lambda k: res[k]["GiB_s"],
               default="staged")
    return {"value": res[best]["GiB_s"], "unit": "GiB/s", "ms": res[best]["ms"], "records": n,
            "pcie_bytes": 4 * n * 32, "pcie_GBps": res[best]["pcie_GBps"],
            "roundtrip_ok": all(r["roundtrip_ok"] for r in res.values()), "best": best, "legs": res,
            "slots": [slots, slot_bytes],
            "method": "C-ABI xdrg_encode_batch / xdrg_decode_batch with XDRG_HOST_PTRS, replies and requests at "
                      "once on two contexts (two threads); staged = the context's staging ring (slots x bytes "
                      "above, chunked H2D / kernels / D2H on the context's copy and compute streams), mapped = "
                      "XDRG_HOST_MAPPED (kernels on the registered host buffers over PCIe); buffers pinned with "
                      "xdrg_host_register, staged_pageable on unregistered memory (bounce copies)"}


def _host_cols4(n, nchars, nints, mk):
    """configs[3] columns (n records, nchars string bytes, nints vector
    elements) in host memory made by mk(nbytes) -> numpy uint8 array:
    (ctypes columns, (hdr, string bytes, string offsets, ints, int offsets))."""
    import numpy as np
    from oncrpc4j_amd import abi
    a_hdr = mk(4 * n).view(np.int32)
    a_sv = mk(max(nchars, 1))
    a_so = mk(8 * (n + 1)).view(np.uint64)
    a_iv = mk(4 * max(nints, 1)).view(np.int32)
    a_io = mk(8 * (n + 1)).view(np.uint64)
    arr = (abi.Column * 3)()
    arr[0].data, arr[0].stride = a_hdr.ctypes.data, 4
    arr[1].data, arr[1].offsets, arr[1].cap = a_sv.ctypes.data, a_so.ctypes.data, nchars
    arr[2].data, arr[2].offsets, arr[2].cap = a_iv.ctypes.data, a_io.ctypes.data, nints
    return arr, (a_hdr, a_sv, a_so, a_iv, a_io)


def host_inclusive_var(device, n, reps=2, slot_bytes=64 << 20, slots=4):
    """configs[3] (int32 + string<8..256> + int32<0..16>) on host memory
    through the C-ABI, the variable-size counterpart of host_inclusive: replies
    encode host columns into a host stream while requests decode a host
    stream into host columns (two contexts, two threads), and the receive
    side of a record-marked stream: xdrg_receive_batch walks the marks of a
    host socket buffer and decodes every message into host columns
    (RpcMessageParserTCP.handleRead + the per-message decode).  Legs: staged
    (the staging ring, registered buffers), staged_pageable (unregistered,
    bounce copies) and mapped (XDRG_HOST_MAPPED).  GiB/s = native + XDR bytes
    of the direction(s) / wall time; every leg checked against the original
    columns."""
    import threading
    import numpy as np
    import torch
    from oncrpc4j_amd import abi, engine
    dev = torch.device("cuda", device)
    d = _gen_shard(4, n, 0, dev)
    hdr = d["hdr"].reshape(-1).cpu().numpy()
    (lens, sv), (kk, iv) = d["dyn"]
    so = np.zeros(n + 1, np.uint64)
    io = np.zeros(n + 1, np.uint64)
    np.cumsum(lens.cpu().numpy(), out=so[1:])
    np.cumsum(kk.cpu().numpy(), out=io[1:])
    sv = sv.cpu().numpy()
    iv = iv.cpu().numpy()
    del d, lens, kk
    torch.cuda.empty_cache()
    fields = [(abi.T_INT, abi.K_SCALAR, 0), (abi.T_STRING, abi.K_DYNAMIC, 0), (abi.T_INT, abi.K_DYNAMIC, 0)]
    sch = engine.Schema(fields)
    # the XDR streams (raw and record-marked) by one device encode each
    sizes = 12 + (lens_np := np.diff(so)) + ((4 - (lens_np & 3)) & 3) + 4 * np.diff(io)
    xlen = int(sizes.sum())
    xlen_rm = xlen + 4 * n
    native = 4 * n + sv.size + 4 * iv.size
    ctx0 = engine.Context(device)
    ctx0.set_stream(torch.cuda.current_stream())
    streams = {}
    for framed, ln in ((False, xlen), (True, xlen_rm)):
        t = [torch.from_numpy(x).to(dev) for x in (hdr, sv, so.view(np.int64), iv, io.view(np.int64))]
        arr = (abi.Column * 3)()
        arr[0].data, arr[0].stride = t[0].data_ptr(), 4
        arr[1].data, arr[1].offsets, arr[1].cap = t[1].data_ptr(), t[2].data_ptr(), sv.size
        arr[2].data, arr[2].offsets, arr[2].cap = t[3].data_ptr(), t[4].data_ptr(), iv.size
        out = torch.empty(ln, dtype=torch.uint8, device=dev)
        assert ctx0.encode(sch, arr, n, out, ln, framed=framed) == ln
        streams[framed] = out.cpu().numpy()
        del t, out
        torch.cuda.empty_cache()
    ctx0.close()
    regs = []

    def mk_reg(nbytes):
        m_, a_, p_ = _host_buffer(max(nbytes, 1), True)
        regs.append((m_, p_))
        return a_[:nbytes] if nbytes else a_

    def mk_page(nbytes):
        return np.zeros(max(nbytes, 1), np.uint8)[:max(nbytes, 1)]

    def ok_cols(arrs, upto=n):
        a_hdr, a_sv, a_so, a_iv, a_io = arrs
        return (np.array_equal(a_hdr[:upto], hdr[:upto]) and np.array_equal(a_so, so)
                and np.array_equal(a_io, io) and np.array_equal(a_sv[:sv.size], sv)
                and np.array_equal(a_iv[:iv.size], iv))

    def leg(mode):
        mk = mk_page if mode == "staged_pageable" else mk_reg
        kw = {"mapped": True} if mode == "mapped" else {"host": True}
        src_cols, src = _host_cols4(n, sv.size, iv.size, mk)
        for a_, b_ in zip(src, (hdr, sv, so, iv, io)):
            a_[:b_.size] = b_
        out_cols, outs = _host_cols4(n, sv.size, iv.size, mk)
        back_cols, backs = _host_cols4(n, sv.size, iv.size, mk)
        req = mk(xlen)
        req[:] = streams[False]
        xdr = mk(xlen)
        ro = mk(8 * (n + 1)).view(np.uint64)
        ce, cd = engine.Context(device), engine.Context(device)
        for c in (ce, cd):
            c.apply_tuning(os.environ.get("XDRG_TUNE"))   # measurement runs only
            c.host_staging(slot_bytes, slots)
        res = {}
        # encode + decode at once (a server's replies and requests)
        ce.encode(sch, src_cols, n, xdr, xlen, rec_offsets=ro, **kw)   # warm
        cd.decode(sch, req, xlen, n, back_cols, rec_offsets=ro, **kw)

        def enc():
            for _ in range(reps):
                ce.encode(sch, src_cols, n, xdr, xlen, rec_offsets=ro, **kw)

        def dec():
            for _ in range(reps):
                cd.decode(sch, req, xlen, n, back_cols, rec_offsets=ro, **kw)

        xdr[:] = 0
        ts = [threading.Thread(target=enc), threading.Thread(target=dec)]
        t0 = time.perf_counter()
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        dt = (time.perf_counter() - t0) / reps
        ok = bool(np.array_equal(xdr, streams[False])) and ok_cols(backs)
        res["encode_decode"] = {"GiB_s": round(2 * (native + xlen) / dt / GIB, 3), "ms": round(dt * 1e3, 3),
                                "ok": ok}
        # receive: the record-marked socket buffer -> host columns
        sock = mk(xlen_rm)
        sock[:] = streams[True]
        rc, m, used, _, _ = cd.receive(sch, sock, xlen_rm, n, out_cols, **kw)   # warm
        for a_ in outs:
            a_[:] = 0
        t0 = time.perf_counter()
        for _ in range(reps):
            rc, m, used, _, _ = cd.receive(sch, sock, xlen_rm, n, out_cols, **kw)
        dt = (time.perf_counter() - t0) / reps
        ok = (rc, m, used) == (0, n, xlen_rm) and ok_cols(outs)
        res["receive"] = {"GiB_s": round((native + xlen_rm) / dt / GIB, 3), "ms": round(dt * 1e3, 3), "ok": ok}
        for c in (ce, cd):
            c.close()
        for _, p_ in regs:
            engine.host_unregister(p_)
        regs.clear()
        return res

    legs = {mode: leg(mode) for mode in ("staged", "mapped", "staged_pageable")}
    best = {k: max(legs, key=lambda m: legs[m][k]["GiB_s"] if legs[m][k]["ok"] else -1) for k in
            ("encode_decode", "receive")}
    return {"config": 4, "records": n, "native_bytes": native, "xdr_bytes": xlen, "xdr_bytes_framed": xlen_rm,
            "encode_decode": {"GiB_s": legs[best["encode_decode"]]["encode_decode"]["GiB_s"],
                              "best": best["encode_decode"]},
            "receive": {"GiB_s": legs[best["receive"]]["receive"]["GiB_s"], "best": best["receive"]},
            "legs": legs, "slots": [slots, slot_bytes],
            "ok": all(v["ok"] for l_ in legs.values() for v in l_.values()),
            "method": "C-ABI on host memory: encode_decode = xdrg_encode_batch + xdrg_decode_batch at once on two "
                      "contexts (replies / requests), GiB/s of both directions' native + XDR bytes; receive = "
                      "xdrg_receive_batch on a record-marked host socket buffer (mark walk + decode of every "
                      "message into host columns), GiB/s of stream + native bytes; staged = XDRG_HOST_PTRS "
                      "(staging ring, registered buffers), mapped = XDRG_HOST_MAPPED, staged_pageable = "
                      "unregistered memory (bounce copies)"}


def host_inclusive_byref(device, n=512 << 10, reps=3, slot_bytes=64 << 20, slots=4):
    """configs[2]-shaped replies (6 x int32 + a 4 KiB opaque, NFS WRITE / READ
    data) sent by reference from host memory: xdrg_encode_batch_shallow with
    XDRG_HOST_PTRS, the payload column NULL (the FileChunk / shallow
    ByteBuffer of Xdr.java:839-866, 978-988 stays where it is; only the
    heads are produced and cross PCIe), record-marked as sendRawTCP marks
    all parts (GrizzlyRpcTransport.java:130-168).  Legs: byref_staged (the
    staging ring, registered buffers), byref_mapped (XDRG_HOST_MAPPED), and
    copy_staged, the same replies encoded whole from a host payload column
    (every payload byte across PCIe twice).  wire_GiB_s = the messages' bytes
    on the wire (head + payload) / wall time; pcie_bytes = what the call
    moves.  Heads checked against their closed form (marks, big-endian
    ints, length words, splice positions)."""
    import numpy as np
    from oncrpc4j_amd import abi, engine
    P = 4096
    fields = [(abi.T_INT, abi.K_SCALAR, 0)] * 6 + [(abi.T_OPAQUE, abi.K_DYNAMIC, 0)]
    sch = engine.Schema(fields)
    rng = np.random.default_rng(0x0DCAC4E5 + 3)
    regs = []

    def mk(nbytes):
        m_, a_, p_ = _host_buffer(max(nbytes, 1), True)
        regs.append(p_)
        return a_[:nbytes]

    hdr = mk(24 * n).view(np.int32).reshape(n, 6)
    hdr[:] = rng.integers(-2**31, 2**31 - 1, (n, 6), dtype=np.int32)
    poffs = mk(8 * (n + 1)).view(np.uint64)
    poffs[:] = np.arange(n + 1, dtype=np.uint64) * P
    head = 4 + 24 + 4   # mark, six ints, length word
    out = mk(head * n)
    ro = mk(8 * (n + 1)).view(np.uint64)
    spl = mk(8 * n).view(np.uint64)
    want = np.empty((n, head // 4), ">u4")
    want[:, 0] = 0x80000000 | (head - 4 + P)
    want[:, 1:7] = hdr.view(np.uint32)
    want[:, 7] = P
    want = want.view(np.uint8).reshape(-1)

    def cols(payload):
        arr = (abi.Column * 7)()
        for k in range(6):
            arr[k].data, arr[k].stride = hdr.ctypes.data + 4 * k, 24
        arr[6].data = payload.ctypes.data if payload is not None else None
        arr[6].offsets, arr[6].cap = poffs.ctypes.data, n * P if payload is not None else 0
        return arr

    res = {}
    ctx = engine.Context(device)
    ctx.apply_tuning(os.environ.get("XDRG_TUNE"))   # measurement runs only
    ctx.host_staging(slot_bytes, slots)
    for mode in ("byref_staged", "byref_mapped"):
        kw = {"mapped": True} if mode == "byref_mapped" else {"host": True}
        c = cols(None)
        ctx.encode_shallow(sch, c, n, out, head * n, 6, spl, rec_offsets=ro, framed=True, **kw)   # warm
        out[:] = 0
        t0 = time.perf_counter()
        for _ in range(reps):
            ln = ctx.encode_shallow(sch, c, n, out, head * n, 6, spl, rec_offsets=ro, framed=True, **kw)
        dt = (time.perf_counter() - t0) / reps
        ok = ln == head * n and bool(np.array_equal(out, want)) and \
            bool(np.array_equal(spl, np.arange(n, dtype=np.uint64) * head + head)) and \
            bool(np.array_equal(ro, np.arange(n + 1, dtype=np.uint64) * head))
        res[mode] = {"ms": round(dt * 1e3, 3), "wire_GiB_s": round(n * (head + P) / dt / GIB, 2),
                     "Mmsg_s": round(n / dt / 1e6, 2), "pcie_bytes": n * (24 + 8 + head + 8 + 8), "ok": ok}
    # the copy form: the same replies with the payload column in host memory
    payload = mk(n * P)
    payload[:] = 7
    full = mk((head + P) * n)
    c = cols(payload)
    ctx.encode(sch, c, n, full, (head + P) * n, rec_offsets=ro, framed=True, host=True)   # warm
    t0 = time.perf_counter()
    for _ in range(reps):
        ln = ctx.encode(sch, c, n, full, (head + P) * n, rec_offsets=ro, framed=True, host=True)
    dt = (time.perf_counter() - t0) / reps
    f2 = full.reshape(n, head + P)
    ok = ln == (head + P) * n and bool(np.array_equal(f2[:, :head].reshape(-1), want)) and bool((f2[:, head:] == 7).all())
    res["copy_staged"] = {"ms": round(dt * 1e3, 3), "wire_GiB_s": round(n * (head + P) / dt / GIB, 2),
                          "Mmsg_s": round(n / dt / 1e6, 2), "pcie_bytes": n * (24 + 8 + 2 * P + head + 8), "ok": ok}
    ctx.close()
    for p_ in regs:
        engine.host_unregister(p_)
    del hdr, poffs, out, ro, spl, payload, full, f2
    return {"config": 3, "records": n, "payload_bytes": P, "legs": res,
            "ok": all(v["ok"] for v in res.values()),
            "method": "C-ABI xdrg_encode_batch_shallow (XDRG_HOST_PTRS / XDRG_HOST_MAPPED, payload column NULL) "
                      "vs xdrg_encode_batch of the same record-marked replies from a host payload column; host "
                      "buffers pinned with xdrg_host_register; wire_GiB_s counts head + payload bytes per message"}


# ---------------------------------------------------------------------------
def run_rank(args):
    import torch
    R = Rank(args)
    if args.test_codec:
        import importlib
        codec = importlib.import_module(args.test_codec)
        ctx = None

        def make(cfg, n, framed):
            return codec.make_workload(cfg, n, framed, R.rank)
    else:
        from oncrpc4j_amd import engine
        ctx = engine.Context(R.local, timing=True)
        ctx.apply_tuning(os.environ.get("XDRG_TUNE"))   # measurement runs only
        ctx.set_stream(torch.cuda.current_stream())

        def make(cfg, n, framed):
            return Workload(ctx, cfg, n, framed, shards=(R.rank,))

    n = args.records if args.records else SIZES[args.config]
    head, wl = measure(R, args, make, args.config, args.framed, n, args.steps, args.warmup, with_gather=True)
    hinc = None
    if R.rank == 0 and R.world == 1 and args.config == 2 and not args.framed and not args.no_host_inclusive \
            and ctx is not None:
        hinc = host_inclusive(R.local, wl.sch, min(n, 64 << 20))
    del wl
    hvar = hbyref = None
    if hinc is not None and args.extra:
        if R.cuda:
            torch.cuda.empty_cache()
        hvar = host_inclusive_var(R.local, SIZES[4])
        hbyref = host_inclusive_byref(R.local)
    if R.cuda:
        torch.cuda.empty_cache()

    extra = []
    if args.extra:
        for cfg, framed in ((2, True), (3, False), (4, False), (4, True)):
            if (cfg, framed) == (args.config, bool(args.framed)):
                continue
            e, w = measure(R, args, make, cfg, framed, SIZES[cfg], args.extra_steps, 2,
                           with_gather=(cfg == 4))
            del w
            if R.rank == 0 and R.world == 1 and cfg in (3, 4) and not framed and args.cpu_seconds > 0 \
                    and not args.test_codec:
                e["cpu_baseline"] = cpu_var_baseline(cfg, min(args.cpu_seconds / 3.0, 6.0))
            if R.cuda:
                torch.cuda.empty_cache()
            extra.append(e)

    cpu = None
    if R.rank == 0 and R.world == 1 and args.cpu_seconds > 0 and not args.test_codec:
        cpu = cpu_baseline(args.cpu_seconds)

    if R.rank == 0:
        line = {
            "metric": "XDR encode+decode GiB/s (device-resident)",
            "value": head["GiB_s"], "unit": "GiB/s", "n_gpus": R.world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": head["ms_per_step"],
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int32",
            "data": "synthetic (seeded uniform int32 / random bytes / [a-z] strings)",
            "config": {"workload": head["workload"], "records_per_gpu": head["records_per_gpu"],
                       "xdr_bytes_per_gpu": head["xdr_bytes_per_gpu"],
                       "native_bytes_per_gpu": head["native_bytes_per_gpu"],
                       "bytes_per_step_per_gpu": head["bytes_per_step_per_gpu"],
                       "framed": head["framed"],
                       "parallelism": f"records sharded {R.world} ways, one process per GPU"
                       if R.world > 1 else "single GPU"},
            "mrecords_per_s": head["Mrec_s"],
            "roofline": head["roofline"],
            "kernel_ms_per_step": head["kernel_ms_per_step"],
            "encode_only": head["encode_only"],
            "decode_only": head["decode_only"],
            "gather": head["gather"],
            "receive": head.get("receive"),
            "cpu_baseline": cpu,
            "host_inclusive": hinc,
            "host_inclusive_var": hvar,
            "host_inclusive_byref": hbyref,
            "extra_configs": extra,
        }
        if args.no_check:
            line["unchecked"] = True   # a probe build's timing, not a measurement of the product
        print(json.dumps(line), flush=True)
    if ctx is not None:
        ctx.close()
    R.close()


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None:
        if args.gpus > 1:
            sys.exit(launch(args, argv))
    elif int(env_world) != args.gpus:
        print(f"bench.py: WORLD_SIZE={env_world} but --gpus {args.gpus}", file=sys.stderr)
        sys.exit(2)
    run_rank(args)


if __name__ == "__main__":
    main()
