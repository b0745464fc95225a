"""Throughput of the parallel record-mark walk (xdrg_frame_scan / xdrg_deframe)
on a record-marked configs[1] stream (64 Mi x 36-byte messages, 2.25 GiB) and
on a mixed stream (re-fragmented messages of 0..4 KiB), against the serial
oracle walk (one host thread, oracle/xdr_oracle.c) on a bounded sample."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle  # noqa: E402
from oncrpc4j_amd import abi, engine  # noqa: E402


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return sorted(ts)[len(ts) // 2]


def main():
    ctx = engine.Context(0, timing=True)
    ctx.apply_tuning(os.environ.get("XDRG_TUNE"))   # measurement runs only
    ctx.set_stream(torch.cuda.current_stream())
    out = []
    # 1. framed configs[1] stream
    n = int(os.environ.get("N", 64 << 20))
    words = torch.randint(0, 2**31, (n, 9), dtype=torch.int32, device="cuda")
    words[:, 0] = int(np.uint32(0x80000020).byteswap().view(np.int32))
    stream = words.view(torch.uint8).reshape(-1)
    offs = torch.zeros(n + 1, dtype=torch.int64, device="cuda")
    t = timed(lambda: ctx.frame_scan(stream, 36 * n, offs, n))
    assert torch.equal(offs[:5].cpu(), torch.arange(0, 180, 36))
    payload = torch.empty(32 * n, dtype=torch.uint8, device="cuda")
    moffs = torch.zeros(n + 1, dtype=torch.int64, device="cuda")
    t2 = timed(lambda: ctx.deframe(stream, 36 * n, payload, payload.numel(), moffs, n))
    out.append({"stream": "configs[1] record-marked, 36-byte messages", "messages": n, "bytes": 36 * n,
                "frame_scan_ms": round(t * 1e3, 3), "frame_scan_GBps": round(36 * n / t / 1e9, 1),
                "deframe_ms": round(t2 * 1e3, 3), "deframe_GBps": round(36 * n / t2 / 1e9, 1)})
    # CPU serial walk on a bounded sample (the reference's per-buffer loop)
    m = 1 << 22
    host = stream[:36 * m].cpu().numpy().tobytes()
    t0 = time.perf_counter()
    rc, o = oracle.frame_scan(host, m)
    tc = time.perf_counter() - t0
    out[-1]["cpu_serial_walk_GBps"] = round(36 * m / tc / 1e9, 2)
    out[-1]["cpu_sample"] = f"{m} messages, oracle xo_frame_scan, 1 thread"
    del words, stream, payload, moffs, offs
    # 2. mixed stream
    rng = np.random.default_rng(3)
    parts = []
    for i in range(200000):
        body = rng.integers(0, 256, int(rng.integers(0, 1024)) * 4, dtype=np.uint8).tobytes()
        parts.append(oracle.fragment(body, int(rng.choice([64, 512, 4096]))))
    s = b"".join(parts)
    dev = torch.from_numpy(np.frombuffer(s, dtype=np.uint8).copy()).cuda()
    offs = torch.zeros(200001, dtype=torch.int64, device="cuda")
    payload = torch.empty(len(s), dtype=torch.uint8, device="cuda")
    t = timed(lambda: ctx.frame_scan(dev, len(s), offs, 200000))
    t2 = timed(lambda: ctx.deframe(dev, len(s), payload, payload.numel(), offs, 200000))
    t0 = time.perf_counter()
    oracle.frame_scan(s, 200000)
    tc = time.perf_counter() - t0
    out.append({"stream": "200k messages 0..4 KiB, fragments of 64/512/4096 B", "bytes": len(s),
                "frame_scan_ms": round(t * 1e3, 3), "frame_scan_GBps": round(len(s) / t / 1e9, 1),
                "deframe_ms": round(t2 * 1e3, 3), "deframe_GBps": round(len(s) / t2 / 1e9, 1),
                "cpu_serial_walk_GBps": round(len(s) / tc / 1e9, 2)})
    del dev, offs, payload
    # 3. the serial cliff: one fragment whose size is not a multiple of 4 on
    # the chain (a peer's odd-sized opaque body) sends the whole walk to the
    # one-lane k_fr_serial kernel (same results, measured bound)
    parts = [oracle.fragment(b"abc", 4096)]
    for i in range(20000):
        body = rng.integers(0, 256, int(rng.integers(0, 1024)) * 4, dtype=np.uint8).tobytes()
        parts.append(oracle.fragment(body, int(rng.choice([64, 512, 4096]))))
    s = b"".join(parts)
    dev = torch.from_numpy(np.frombuffer(s, dtype=np.uint8).copy()).cuda()
    offs = torch.zeros(20002, dtype=torch.int64, device="cuda")
    t = timed(lambda: ctx.frame_scan(dev, len(s), offs, 20001), reps=3)
    assert ctx.frame_scan(dev, len(s), offs, 20001) == 20001
    rc, want = oracle.frame_scan(s, 20001)
    assert offs.cpu().numpy().astype(np.uint64)[:20002].tolist() == list(want)[:20002]
    # the serial walk, for comparison: the same stream one byte off 4-byte alignment
    sh = torch.zeros(len(s) + 16, dtype=torch.uint8, device="cuda")
    sh[1:1 + len(s)] = dev
    ts = timed(lambda: ctx.frame_scan(sh.data_ptr() + 1, len(s), offs, 20001), reps=2)
    want_sh = [int(x) for x in list(want)[:20002]]
    assert offs.cpu().numpy().astype(np.uint64)[:20002].tolist() == want_sh
    del sh
    t0 = time.perf_counter()
    oracle.frame_scan(s, 20001)
    tc = time.perf_counter() - t0
    out.append({"stream": "20k messages 0..4 KiB after one 3-byte fragment (every later mark at 3 mod 4)",
                "bytes": len(s), "frame_scan_ms": round(t * 1e3, 3),
                "frame_scan_GBps": round(len(s) / t / 1e9, 3), "cpu_serial_walk_GBps": round(len(s) / tc / 1e9, 2),
                "serial_walk_ms": round(ts * 1e3, 3),
                "note": "word walk meets the odd size (kFUnal), then the byte-position walk; "
                        "serial_walk_ms = k_fr_serial, one lane hopping mark to mark (the stream 1 byte off alignment)"})
    for o in out:
        print(json.dumps(o))


if __name__ == "__main__":
    main()
