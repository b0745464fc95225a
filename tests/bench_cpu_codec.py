"""TEST INFRASTRUCTURE: a CPU per-shard codec for bench.py's launcher test.

`bench.py --gpus 2 --backend gloo --test-codec bench_cpu_codec` runs the
bench's own launcher, rank setup, timed legs and stream reassembly
(oncrpc4j_amd/parallel.py) on CPU, with the oracle (oracle/xdr_oracle.c) as
the per-shard encoder/decoder in place of the HIP engine.  Only the launcher
test (tests/test_bench_launcher.py) loads this module.
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

import oracle  # noqa: E402
from oncrpc4j_amd import abi  # noqa: E402
from oncrpc4j_amd.columns import HostBatch, random_batch  # noqa: E402

SCHEMAS = {
    2: [(abi.T_INT, abi.K_SCALAR, 0)] * 8,
    3: [(abi.T_INT, abi.K_SCALAR, 0)] * 6 + [(abi.T_OPAQUE, abi.K_DYNAMIC, 0)],
    4: [(abi.T_INT, abi.K_SCALAR, 0), (abi.T_STRING, abi.K_DYNAMIC, 0), (abi.T_INT, abi.K_DYNAMIC, 0)],
}


def _concat(batches):
    fields = batches[0].fields
    arrays = []
    for k, f in enumerate(fields):
        if f[1] == abi.K_DYNAMIC:
            vals = np.concatenate([b.arrays[k][0] for b in batches])
            cnt = np.concatenate([np.diff(b.arrays[k][1]) for b in batches]).astype(np.uint64)
            offs = np.zeros(len(cnt) + 1, dtype=np.uint64)
            np.cumsum(cnt, out=offs[1:])
            arrays.append((vals, offs))
        else:
            arrays.append(np.concatenate([b.arrays[k] for b in batches]))
    return HostBatch(fields, sum(b.n for b in batches), arrays)


class OracleWorkload:
    def __init__(self, cfg, n, framed, shards):
        self.cfg, self.framed = cfg, framed
        self.fields = SCHEMAS[cfg]
        self.hb = _concat([random_batch(self.fields, n, seed=1000 * s + cfg, dyn_len=(0, 30))
                           for s in shards])
        self.n = self.hb.n
        self.desc = f"oracle codec, configs[{cfg - 1}] schema"
        self.xlen = self.hb.xdr_total(framed)
        self.native_bytes = self.hb.native_bytes()
        self.enc_bytes = self.native_bytes + self.xlen
        self.bytes_per_step = 2 * self.enc_bytes
        self.xdr = torch.zeros(self.xlen, dtype=torch.uint8)
        self.offs = torch.zeros(self.n + 1, dtype=torch.int64)
        self.back = None

    def encode(self):
        rc, xdr, offs = oracle.encode_batch(self.fields, self.hb.columns(), self.n, self.xlen,
                                            framed=self.framed)
        assert rc == 0
        self.xdr.copy_(torch.from_numpy(np.frombuffer(xdr, dtype=np.uint8).copy()))
        self.offs.copy_(torch.from_numpy(offs.astype(np.int64)))

    def decode(self):
        self.back = HostBatch.empty(self.fields, self.n, self.hb.dyn_caps())
        rc, fb, err = oracle.decode_batch(self.fields, self.xdr.numpy().tobytes(),
                                          self.offs.numpy().astype(np.uint64), self.n,
                                          self.back.columns(), framed=self.framed)
        assert rc == 0, (rc, fb, err)

    def step(self):
        self.encode()
        self.decode()

    def check(self):
        assert self.back is not None and self.back.equal(self.hb), "decode(encode(x)) != x"

    def xdr_view(self):
        return self.xdr

    def offsets_view(self):
        return None if self.cfg == 2 else self.offs

    def reset_stats(self):
        pass

    def roofline(self, steps):
        return None, {}

    def gatherable(self, world):
        return True

    def reference(self, world, n_per_rank):
        return OracleWorkload(self.cfg, n_per_rank, self.framed, range(world))


def make_workload(cfg, n, framed, rank):
    return OracleWorkload(cfg, n, framed, (rank,))
