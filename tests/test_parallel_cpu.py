"""World-size-2 gloo tests of the record-sharded path (oncrpc4j_amd.parallel)
on CPU.  The per-shard codec is the oracle here (test infrastructure); on
MI355X it is the HIP engine (bench.py / tests/test_gpu_parity.py)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oncrpc4j_amd import abi, parallel
from oncrpc4j_amd.columns import HostBatch, random_batch

SCHEMAS = {
    "cfg2": [(abi.T_INT, abi.K_SCALAR, 0)] * 8,
    "cfg4": [(abi.T_INT, abi.K_SCALAR, 0), (abi.T_STRING, abi.K_DYNAMIC, 0), (abi.T_INT, abi.K_DYNAMIC, 0)],
}


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, name, n, framed, q):
    import oracle
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        fields = SCHEMAS[name]
        hb = random_batch(fields, n, seed=99, dyn_len=(0, 30))   # same batch on every rank

        def enc(lo, hi):
            sub = hb.slice(lo, hi)
            rc, xdr, offs = oracle.encode_batch(fields, sub.columns(), hi - lo, sub.xdr_total(framed),
                                                framed=framed)
            assert rc == 0
            return (torch.from_numpy(np.frombuffer(xdr, dtype=np.uint8).copy()),
                    torch.from_numpy(offs.astype(np.int64)))

        stream, offs = parallel.encode_sharded(enc, n)
        rc, want, want_offs = oracle.encode_batch(fields, hb.columns(), n, hb.xdr_total(framed),
                                                  framed=framed)
        ok_stream = stream.numpy().tobytes() == want
        ok_offs = np.array_equal(offs.numpy().astype(np.uint64), want_offs)

        # sharded decode of the reassembled stream, with one corrupted record
        # owned by the second rank: the global first error must be reported
        bad = bytearray(want)
        r_bad = (3 * n) // 4
        if name == "cfg4":
            p = int(want_offs[r_bad]) + (4 if framed else 0) + 4   # string length word
            bad[p:p + 4] = (0xfffffff0).to_bytes(4, "big")         # negative -> corrupted
        else:
            bad = bad[:int(want_offs[r_bad]) + 6]                  # truncated -> too short
        bad = bytes(bad)

        def dec(lo, hi):
            sub = HostBatch.empty(fields, hi - lo, {k: 64 * (hi - lo) for k in range(len(fields))})
            ro = want_offs[lo:hi + 1]
            rc, fb, err = oracle.decode_batch(fields, bad, ro, hi - lo, sub.columns(), framed=framed)
            return rc, (fb + lo if rc else hi), err

        st, fb, err = parallel.decode_sharded(dec, n)
        exp = oracle.decode_batch(fields, bad, want_offs, n,
                                  HostBatch.empty(fields, n, {k: 64 * n for k in range(len(fields))}).columns(),
                                  framed=framed)
        q.put((rank, ok_stream, ok_offs, (st, fb, err), exp))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("framed", [False, True], ids=["raw", "rm"])
@pytest.mark.parametrize("name", sorted(SCHEMAS))
def test_sharded_encode_decode_gloo(name, framed):
    world, n = 2, 1001
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, name, n, framed, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok_stream, ok_offs, got, exp in res:
        assert ok_stream, f"rank {rank}: reassembled stream differs from the 1-process encode"
        assert ok_offs, f"rank {rank}: rebased record offsets differ"
        assert got == exp, f"rank {rank}: sharded decode error {got} != sequential {exp}"


def test_shard_ranges_cover():
    for n in (0, 1, 7, 1000, 2**20 + 3):
        for world in (1, 2, 3, 8):
            rs = [parallel.shard_range(n, world, r) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
