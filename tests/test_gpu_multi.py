"""xdrg_encode_batch_multi / xdrg_decode_batch_multi (include/xdrg.h; SURVEY.md
§8b, §8e): one process driving several contexts, record shards in context
order, full-mesh gather of the encoded shards.  The box has one GPU, so the
contexts share device 0 with separate output buffers: the gather then copies
device-locally through the same kernel the peer (xGMI) case uses.  Parity:
every context's stream and offsets equal a one-context oracle encode; the
sharded decode equals the oracle per shard and reports the batch's first
error."""
import zlib

import numpy as np
import pytest

import oracle
from oncrpc4j_amd import abi, engine, parallel
from oncrpc4j_amd.columns import DeviceBatch, HostBatch, random_batch

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

I, STR, O, H = abi.T_INT, abi.T_STRING, abi.T_OPAQUE, abi.T_HYPER
SC, FX, DY = abi.K_SCALAR, abi.K_FIXED, abi.K_DYNAMIC
SCHEMAS = {
    "cfg2_8xint": [(I, SC, 0)] * 8,
    "cfg4_int_string_intvec": [(I, SC, 0), (STR, DY, 0), (I, DY, 0)],
    "mixed": [(H, SC, 0), (O, FX, 5), (O, DY, 0), (I, SC, 0)],
}


@pytest.fixture(scope="module")
def ctxs():
    cs = [engine.Context(0) for _ in range(3)]
    for c in cs:
        c.set_stream(torch.cuda.current_stream())
    yield cs
    for c in cs:
        c.close()


def _shards(n, k):
    return [parallel.shard_range(n, k, r) for r in range(k)]


@pytest.mark.parametrize("framed", [False, True], ids=["raw", "rm"])
@pytest.mark.parametrize("k", [1, 2, 3])
@pytest.mark.parametrize("name", sorted(SCHEMAS))
def test_encode_decode_multi(ctxs, name, k, framed):
    fields = SCHEMAS[name]
    n = 10007
    hb = random_batch(fields, n, seed=zlib.crc32(f"{name}{k}{framed}".encode()), dyn_len=(0, 50))
    rc, want, want_offs = oracle.encode_batch(fields, hb.columns(), n, hb.xdr_total(framed) + 8, framed=framed)
    assert rc == 0
    sch = engine.Schema(fields)
    parts = _shards(n, k)
    dbs = [DeviceBatch.from_host(hb.slice(lo, hi)) for lo, hi in parts]
    cap = len(want) + 64
    outs = [torch.zeros(cap, dtype=torch.uint8, device="cuda") for _ in range(k)]
    offs = [torch.zeros(n + 1, dtype=torch.int64, device="cuda") for _ in range(k)]
    ln = engine.encode_multi(ctxs[:k], sch, [db.columns() for db in dbs], [hi - lo for lo, hi in parts],
                             outs, cap, rec_offsets=offs, framed=framed)
    assert ln == len(want)
    for i in range(k):
        assert outs[i][:ln].cpu().numpy().tobytes() == want, f"context {i} stream"
        assert not outs[i][ln:].any()
        assert np.array_equal(offs[i].cpu().numpy().view(np.uint64), want_offs), f"context {i} offsets"
    # sharded decode, each context from its own copy of the stream
    caps = [hb.slice(lo, hi).dyn_caps() for lo, hi in parts]
    outs_b = [DeviceBatch.empty(fields, hi - lo, c) for (lo, hi), c in zip(parts, caps)]
    ro = offs if any(f[1] == DY for f in fields) else None
    st = engine.decode_multi(ctxs[:k], sch, outs, ln, [hi - lo for lo, hi in parts],
                             [b.columns() for b in outs_b], rec_offsets=ro, framed=framed)
    assert st == (0, n, 0)
    for (lo, hi), b in zip(parts, outs_b):
        assert b.to_host().equal(hb.slice(lo, hi))


@pytest.mark.parametrize("name", ["cfg4_int_string_intvec", "cfg2_8xint"])
def test_decode_multi_first_error(ctxs, name):
    """Two defects in different shards: the batch reports the earlier one
    (a sequential reference decode throws there first, Xdr.java:1028-1037)."""
    fields = SCHEMAS[name]
    n, k = 6000, 3
    hb = random_batch(fields, n, seed=5, dyn_len=(1, 20))
    rc, xdr, offs = oracle.encode_batch(fields, hb.columns(), n, hb.xdr_total())
    bad = bytearray(xdr)
    r1, r2 = 4500, 2500   # shard 2 and shard 1
    if name.startswith("cfg4"):
        for r in (r1, r2):
            p = int(offs[r]) + 4
            bad[p:p + 4] = (0xfffffff0).to_bytes(4, "big")   # negative length -> corrupted
        ro_host = offs
    else:
        bad = bad[:int(offs[r2]) + 8]                         # truncated inside record r2
        ro_host = None
    bad = bytes(bad)
    exp = oracle.decode_batch(fields, bad, ro_host, n,
                              HostBatch.empty(fields, n, {d: 64 * n for d in range(len(fields))}).columns())
    assert exp[0] != 0 and exp[1] == r2
    sch = engine.Schema(fields)
    parts = _shards(n, k)
    dev = torch.from_numpy(np.frombuffer(bad, dtype=np.uint8).copy()).cuda()
    ro = None
    if ro_host is not None:
        ro = [torch.from_numpy(offs.view(np.int64).copy()).cuda() for _ in range(k)]
    outs_b = [DeviceBatch.empty(fields, hi - lo, {d: 64 * (hi - lo) for d in range(len(fields))}) for lo, hi in parts]
    st = engine.decode_multi(ctxs[:k], sch, [dev] * k, len(bad), [hi - lo for lo, hi in parts],
                             [b.columns() for b in outs_b], rec_offsets=ro, raise_on_error=False)
    assert st == exp
    lo, hi = parts[0]
    assert outs_b[0].to_host().equal(hb.slice(lo, hi))   # shard 0 is wholly before the error


def test_encode_multi_shared_output(ctxs):
    """Contexts writing into one shared buffer: shards land in place, no copy."""
    fields = SCHEMAS["cfg4_int_string_intvec"]
    n, k = 5000, 3
    hb = random_batch(fields, n, seed=9, dyn_len=(0, 40))
    rc, want, want_offs = oracle.encode_batch(fields, hb.columns(), n, hb.xdr_total())
    parts = _shards(n, k)
    dbs = [DeviceBatch.from_host(hb.slice(lo, hi)) for lo, hi in parts]
    out = torch.zeros(len(want) + 16, dtype=torch.uint8, device="cuda")
    ro = torch.zeros(n + 1, dtype=torch.int64, device="cuda")
    ln = engine.encode_multi(ctxs[:k], engine.Schema(fields), [db.columns() for db in dbs],
                             [hi - lo for lo, hi in parts], [out] * k, out.numel(), rec_offsets=[ro] * k)
    assert out[:ln].cpu().numpy().tobytes() == want
    assert np.array_equal(ro.cpu().numpy().view(np.uint64), want_offs)


@pytest.mark.parametrize("name", ["cfg4_int_string_intvec", "cfg2_8xint"])
def test_encode_multi_shared_output_own_streams(name):
    """Shared output and shared offsets array, every context on its own
    stream: the shards' boundary offsets entries are written by two
    contexts, so they must be stores of one value, never read-modify-writes."""
    fields = SCHEMAS[name]
    k = 4
    streams = [torch.cuda.Stream() for _ in range(k)]
    cs = [engine.Context(0) for _ in range(k)]
    try:
        for c, s in zip(cs, streams):
            c.set_stream(s)
        for rep, n in enumerate((4001, 20011, 7)):
            hb = random_batch(fields, n, seed=100 + rep, dyn_len=(0, 60))
            rc, want, want_offs = oracle.encode_batch(fields, hb.columns(), n, hb.xdr_total())
            parts = _shards(n, k)
            dbs = [DeviceBatch.from_host(hb.slice(lo, hi)) for lo, hi in parts]
            out = torch.zeros(len(want) + 16, dtype=torch.uint8, device="cuda")
            ro = torch.full((n + 1,), -1, dtype=torch.int64, device="cuda")
            torch.cuda.synchronize()
            ln = engine.encode_multi(cs, engine.Schema(fields), [db.columns() for db in dbs],
                                     [hi - lo for lo, hi in parts], [out] * k, out.numel(), rec_offsets=[ro] * k)
            torch.cuda.synchronize()
            assert ln == len(want)
            assert out[:ln].cpu().numpy().tobytes() == want
            assert np.array_equal(ro.cpu().numpy().view(np.uint64), want_offs), f"n={n}"
    finally:
        for c in cs:
            c.close()


def test_ctx_keeps_callers_device():
    """Every entry point restores the caller thread's current device."""
    if torch.cuda.device_count() < 2:
        pytest.skip("needs two devices to observe a device switch")
    torch.cuda.set_device(1)
    c = engine.Context(0)
    assert torch.cuda.current_device() == 1
    c.reset_stats()
    assert torch.cuda.current_device() == 1
    c.close()
    assert torch.cuda.current_device() == 1
    torch.cuda.set_device(0)


def test_encode_multi_capacity(ctxs):
    fields = SCHEMAS["cfg2_8xint"]
    hb = random_batch(fields, 100, seed=1)
    parts = _shards(100, 2)
    dbs = [DeviceBatch.from_host(hb.slice(lo, hi)) for lo, hi in parts]
    outs = [torch.zeros(3200, dtype=torch.uint8, device="cuda") for _ in range(2)]
    with pytest.raises(engine.CapacityError):
        engine.encode_multi(ctxs[:2], engine.Schema(fields), [db.columns() for db in dbs], [50, 50], outs, 3196)
    assert not any(o.any() for o in outs)


# ---- repeated groups (arrays of structs, lists, inner groups, unions) --------
def _group_cases():
    """(id, fields, conds, HostBatch, stream, offsets, framed) from the
    xdrlib-packed fixtures: READDIR / DUMP / RPCBPROC_DUMP lists, arrays of
    structs, two groups (group_vectors.json), chunk_map (conditional members
    inside elements) and volume_index (lists inside list elements)."""
    import gold
    out = []
    gv = gold.load("group_vectors.json")
    for b in gv["batches"]:
        fields = [tuple(f) for f in b["fields"]]
        out.append((f"{b['name']}-{'rm' if b['framed'] else 'raw'}", fields, None,
                    gold.batch_from_records(fields, b["records"]), bytes.fromhex(b["xdr"]),
                    np.asarray(b["rec_offsets"], np.uint64), b["framed"]))
    for fn in ("chunk_map_vectors.json", "volume_index_vectors.json", "group_cond_vectors.json"):
        d = gold.load(fn)
        fields = [tuple(f) for f in d["fields"]]
        conds = [(f, dd, bool(n_), list(v)) for f, dd, n_, v in d["conds"]]
        for b in d["batches"]:
            out.append((f"{fn.split('_vectors')[0]}-{'rm' if b['framed'] else 'raw'}", fields, conds,
                        gold.batch_from_records(fields, b["records"]), bytes.fromhex(b["xdr"]),
                        np.asarray(b["rec_offsets"], np.uint64), b["framed"]))
    return out


GROUP_CASES = _group_cases()


@pytest.mark.parametrize("k", [1, 2, 3])
@pytest.mark.parametrize("case", GROUP_CASES, ids=[c[0] for c in GROUP_CASES])
def test_group_schemas_multi(ctxs, case, k):
    """Group schemas shard by record: each context encodes its records' shard
    (element rows and member offsets counted from its first record) at the
    shard's stream offset and the gather reassembles the fixture's stream;
    the sharded decode returns every shard's records (XdrAble.java:40,49;
    jrpcgen.java:856-906)."""
    _, fields, conds, hb, want, want_offs, framed = case
    n = hb.n
    sch = engine.Schema(fields, conds)
    parts = _shards(n, k)
    dbs = [DeviceBatch.from_host(hb.slice(lo, hi)) for lo, hi in parts]
    cap = len(want) + 64
    outs = [torch.zeros(cap, dtype=torch.uint8, device="cuda") for _ in range(k)]
    offs = [torch.zeros(n + 1, dtype=torch.int64, device="cuda") for _ in range(k)]
    ln = engine.encode_multi(ctxs[:k], sch, [db.columns() for db in dbs], [hi - lo for lo, hi in parts],
                             outs, cap, rec_offsets=offs, framed=framed)
    assert ln == len(want)
    for i in range(k):
        assert outs[i][:ln].cpu().numpy().tobytes() == want, f"context {i} stream"
        assert np.array_equal(offs[i].cpu().numpy().view(np.uint64), want_offs), f"context {i} offsets"
    caps = [hb.slice(lo, hi).dyn_caps() for lo, hi in parts]
    outs_b = [DeviceBatch.empty(fields, hi - lo, c) for (lo, hi), c in zip(parts, caps)]
    st = engine.decode_multi(ctxs[:k], sch, outs, ln, [hi - lo for lo, hi in parts],
                             [b.columns() for b in outs_b], rec_offsets=offs, framed=framed)
    assert st == (0, n, 0)
    for (lo, hi), b in zip(parts, outs_b):
        assert b.to_host().equal(hb.slice(lo, hi))


@pytest.mark.parametrize("case", [c for c in GROUP_CASES if c[0] in ("dirlist-raw", "volume_index-raw")],
                         ids=lambda c: c[0])
def test_group_multi_first_error(ctxs, case):
    """A stream cut inside a late record: the shard holding it reports it,
    the batch's first bad record is the oracle's (Xdr.java:1028-1031)."""
    _, fields, conds, hb, want, want_offs, framed = case
    n, k = hb.n, 3
    cut = int(want_offs[n - 3]) + 6
    bad = want[:cut]
    caps = {d: 64 * n for d in range(len(fields))}
    exp = oracle.decode_batch(fields, bad, want_offs, n, HostBatch.empty(fields, n, caps).columns(), framed=framed,
                              conds=conds)
    assert exp[0] != 0
    sch = engine.Schema(fields, conds)
    parts = _shards(n, k)
    dev = torch.from_numpy(np.frombuffer(bad + bytes(8), dtype=np.uint8).copy()).cuda()
    ro = [torch.from_numpy(want_offs.view(np.int64).copy()).cuda() for _ in range(k)]
    outs_b = [DeviceBatch.empty(fields, hi - lo, {d: 64 * (hi - lo) for d in range(len(fields))})
              for lo, hi in parts]
    st = engine.decode_multi(ctxs[:k], sch, [dev] * k, len(bad), [hi - lo for lo, hi in parts],
                             [b.columns() for b in outs_b], rec_offsets=ro, framed=framed, raise_on_error=False)
    assert st == exp
    lo, hi = parts[0]
    assert outs_b[0].to_host().equal(hb.slice(lo, hi))
