"""GPU parity at the exact shapes of BASELINE.json's configs,
with the native layouts bench.py measures:

* configs[2]: 6 x int32 header (array of structs, 24-byte stride) + opaque<>
  of exactly 4096 random bytes — 4124-byte records, so every payload sits 12
  bytes off 16-byte alignment in the stream (Xdr.java:797-800);
* configs[3]: int32 + string of U[8, 256] bytes over [a-z] + int32<> of
  U[0, 16] elements (Xdr.java:760-763, :607-613).

At oracle-checkable sizes (>= 32 K / 128 K records) every byte and value is
compared with the oracle, raw and record-marked, plus error parity on a cut
and a corrupted stream.  At the full BASELINE sizes (16 Mi / 32 Mi records)
the checks are size-independent: the round trip, the record offsets against
the per-record sizes, and the oracle encode of a few thousand records
sampled across the batch against their slices of the GPU stream."""
import numpy as np
import pytest

import oracle
from oncrpc4j_amd import abi, engine
from oncrpc4j_amd.columns import HostBatch

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

I, O, STR, SC, DY = abi.T_INT, abi.T_OPAQUE, abi.T_STRING, abi.K_SCALAR, abi.K_DYNAMIC
CFG3 = [(I, SC, 0)] * 6 + [(O, DY, 0)]
CFG4 = [(I, SC, 0), (STR, DY, 0), (I, DY, 0)]


class Shape:
    """One BASELINE config's records in HBM, in bench.py's layout."""

    def __init__(self, cfg, n, seed):
        g = torch.Generator(device="cuda").manual_seed(seed)
        self.cfg, self.n = cfg, n
        self.fields = CFG3 if cfg == 3 else CFG4
        self.nh = 6 if cfg == 3 else 1
        self.hdr = torch.randint(-2**31, 2**31 - 1, (n, self.nh), dtype=torch.int32, device="cuda", generator=g)
        self.dyn = []
        if cfg == 3:
            cnt = torch.full((n,), 4096, dtype=torch.int64, device="cuda")
            vals = torch.randint(0, 256, (n * 4096,), dtype=torch.uint8, device="cuda", generator=g)
            self.dyn.append((vals, self._offs(cnt)))
        else:
            cnt = torch.randint(8, 257, (n,), dtype=torch.int64, device="cuda", generator=g)
            vals = torch.randint(97, 123, (int(cnt.sum()),), dtype=torch.uint8, device="cuda", generator=g)
            self.dyn.append((vals, self._offs(cnt)))
            k = torch.randint(0, 17, (n,), dtype=torch.int64, device="cuda", generator=g)
            v2 = torch.randint(-2**31, 2**31 - 1, (int(k.sum()),), dtype=torch.int32, device="cuda", generator=g)
            self.dyn.append((v2, self._offs(k)))
        self.sch = engine.Schema(self.fields)

    @staticmethod
    def _offs(cnt):
        o = torch.zeros(cnt.numel() + 1, dtype=torch.int64, device="cuda")
        torch.cumsum(cnt, 0, out=o[1:])
        return o

    def columns(self, hdr, dyn):
        arr = (abi.Column * len(self.fields))()
        for k in range(self.nh):
            arr[k].data = hdr.data_ptr() + 4 * k
            arr[k].stride = 4 * self.nh
        for j, (v, o) in enumerate(dyn):
            arr[self.nh + j].data = v.data_ptr()
            arr[self.nh + j].offsets = o.data_ptr()
            arr[self.nh + j].cap = v.numel()
        arr._keep = (hdr, dyn)
        return arr

    def sizes(self, framed):
        s = torch.full((self.n,), 4 * self.nh + (4 if framed else 0), dtype=torch.int64, device="cuda")
        for (t, _, _), (v, o) in zip(self.fields[self.nh:], self.dyn):
            c = o[1:] - o[:-1]
            s += 4 + ((c + 3) & ~3 if t in (O, STR) else 4 * c)
        return s

    def host_records(self, idx):
        """The records idx (numpy) as a HostBatch, for the oracle."""
        ti = torch.from_numpy(idx).cuda()
        arrays = [a for a in self.hdr[ti].cpu().numpy().T.copy()]
        for (t, _, _), (v, o) in zip(self.fields[self.nh:], self.dyn):
            oh = o.cpu().numpy()
            a, b = oh[idx], oh[idx + 1]
            cnt = (b - a).astype(np.uint64)
            offs = np.zeros(len(idx) + 1, dtype=np.uint64)
            np.cumsum(cnt, out=offs[1:])
            vh = v.cpu().numpy()
            vals = np.concatenate([vh[x:y] for x, y in zip(a, b)]) if len(idx) else vh[:0]
            arrays.append((vals, offs))
        return HostBatch(self.fields, len(idx), [np.ascontiguousarray(x) if not isinstance(x, tuple) else x
                                                 for x in arrays])


def _encode(ctx, sh, framed):
    total = int(sh.sizes(framed).sum())
    out = torch.zeros(total + 64, dtype=torch.uint8, device="cuda")
    ro = torch.zeros(sh.n + 1, dtype=torch.int64, device="cuda")
    ln = ctx.encode(sh.sch, sh.columns(sh.hdr, [(v, o) for v, o in sh.dyn]), sh.n, out, total,
                    rec_offsets=ro, framed=framed)
    assert ln == total
    assert not out[total:].any(), "engine wrote past the stream end"
    return out, ro, total


def _decode(ctx, sh, out, total, ro, framed):
    hb = torch.empty_like(sh.hdr)
    dyn = [(torch.empty_like(v), torch.empty_like(o)) for v, o in sh.dyn]
    rc, fb, err = ctx.decode(sh.sch, out, total, sh.n, sh.columns(hb, dyn), rec_offsets=ro, framed=framed,
                             raise_on_error=False)
    return (rc, fb, err), hb, dyn


@pytest.mark.parametrize("framed", [False, True], ids=["raw", "rm"])
@pytest.mark.parametrize("cfg,n", [(3, 32 << 10), (4, 128 << 10)], ids=["cfg3", "cfg4"])
def test_exact_shape_vs_oracle(gpu_ctx, cfg, n, framed):
    sh = Shape(cfg, n, seed=0x0DCAC4E5 + cfg)
    out, ro, total = _encode(gpu_ctx, sh, framed)
    hbatch = sh.host_records(np.arange(n))
    rc, want, want_offs = oracle.encode_batch(sh.fields, hbatch.columns(), n, total, framed=framed)
    assert rc == 0
    got = out[:total].cpu().numpy().tobytes()
    assert got == want, "XDR stream differs from the oracle"
    assert np.array_equal(ro.cpu().numpy().view(np.uint64), want_offs)
    st, hb, dyn = _decode(gpu_ctx, sh, out, total, ro, framed)
    assert st == (0, n, 0)
    assert torch.equal(hb, sh.hdr)
    for (v, o), (vb, ob) in zip(sh.dyn, dyn):
        assert torch.equal(ob, o) and torch.equal(vb, v)
    # error parity on a cut stream and a negative length in a late record
    caps = hbatch.dyn_caps()
    bad = bytearray(want)
    r = (7 * n) // 9
    p = int(want_offs[r]) + (4 if framed else 0) + 4 * sh.nh
    bad[p:p + 4] = (0xfffffff8).to_bytes(4, "big")
    for desc, stream in (("cut", want[:len(want) - 6]), ("negative length", bytes(bad))):
        o_ref = HostBatch.empty(sh.fields, n, caps)
        exp = oracle.decode_batch(sh.fields, stream, want_offs, n, o_ref.columns(), framed=framed)
        dev = torch.from_numpy(np.frombuffer(stream, dtype=np.uint8).copy()).cuda()
        st, _, _ = _decode(gpu_ctx, sh, dev, len(stream), ro, framed)
        assert exp[0] != 0 and st == exp, desc


@pytest.mark.slow
@pytest.mark.parametrize("framed", [False, True], ids=["raw", "rm"])
@pytest.mark.parametrize("cfg", [3, 4])
def test_full_size_properties(gpu_ctx, cfg, framed):
    """16 Mi configs[2] records / 32 Mi configs[3] records, device resident,
    raw and record-marked: decode(encode(x)) == x, offsets == exclusive sum
    of the per-record sizes, and 4096 sampled records (first, last, random)
    byte-equal to the oracle's encode of the same records.  Record-marked
    (config 4: a walk takes up to 16 GiB of stream): the frame scan of the
    whole stream (the receive side, RpcMessageParserTCP.java:63-140) finds
    exactly the encode's offsets."""
    n = 16 << 20 if cfg == 3 else 32 << 20
    sh = Shape(cfg, n, seed=0x0DCAC4E5 + 100 + cfg)
    out, ro, total = _encode(gpu_ctx, sh, framed)
    sizes = sh.sizes(framed)
    assert int(ro[0]) == 0 and torch.equal(ro[1:], torch.cumsum(sizes, 0))
    if framed and total < 16 << 30:   # (one frame walk takes up to 16 GiB: config 4's stream, not config 3's)
        offs = torch.empty(n + 1, dtype=torch.int64, device="cuda")
        assert gpu_ctx.frame_scan(out, total, offs, n) == n
        assert torch.equal(offs, ro)
        del offs
    st, hb, dyn = _decode(gpu_ctx, sh, out, total, ro, framed)
    assert st == (0, n, 0)
    assert torch.equal(hb, sh.hdr)
    for (v, o), (vb, ob) in zip(sh.dyn, dyn):
        assert torch.equal(ob, o) and torch.equal(vb, v)
    del hb, dyn
    rng = np.random.default_rng(cfg)
    idx = np.unique(np.concatenate([[0, 1, n - 2, n - 1], rng.integers(0, n, 4092)])).astype(np.int64)
    sub = sh.host_records(idx)
    rc, want, want_offs = oracle.encode_batch(sh.fields, sub.columns(), len(idx), sub.xdr_total(framed), framed=framed)
    assert rc == 0
    roh = ro.cpu().numpy()
    ti = torch.from_numpy(idx).cuda()
    starts, ends = ro[ti], ro[ti + 1]
    got = b"".join(out[int(a):int(b)].cpu().numpy().tobytes() for a, b in zip(starts.tolist(), ends.tolist()))
    assert got == want, "sampled records differ from the oracle"
    assert np.array_equal(np.diff(want_offs), (roh[idx + 1] - roh[idx]).astype(np.uint64))
