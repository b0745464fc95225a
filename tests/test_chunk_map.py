"""A fixed array of structs inside list elements:
tests/golden/rpcgen/chunk_map.x `chunk_map` — every element of the
`chunk_ent *next` list holds `replica copies[2]`, and every replica an
optional checksum.

jrpcgen encodes a fixed array as its elements one after another with no
count word (jrpcgen.java:856-906) and a list as TRUE + element ... FALSE
(jrpcgen.java:835-851).  The tape (oncrpc4j_amd.rpcgen) unrolls the fixed
array into the element's members (two copies of the replica's fields, each
with its own optional-checksum condition, evaluated per element).  The
fixtures (tests/golden/chunk_map_vectors.json) were packed by CPython's
stdlib xdrlib from the declarations, not from the tape; the oracle is
checked against them on the CPU, the HIP engine against them and against the
oracle on the GPU, with first-bad errors inside elements."""
import os

import numpy as np
import pytest

import gold
import oracle
from oncrpc4j_amd import abi, rpcgen
from oncrpc4j_amd.columns import HostBatch

FIX = gold.load("chunk_map_vectors.json")
FIELDS = [tuple(f) for f in FIX["fields"]]
CONDS = [(f, d, bool(n), list(v)) for f, d, n, v in FIX["conds"]]
SPEC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "rpcgen", "chunk_map.x")


def _ids(b):
    return "rm" if b["framed"] else "raw"


def _batch(b):
    hb = gold.batch_from_records(FIELDS, b["records"])
    return hb, bytes.fromhex(b["xdr"]), np.asarray(b["rec_offsets"], np.uint64)


def test_chunk_map_tape():
    f, c = rpcgen.parse_file(SPEC).tape("chunk_map")
    assert [tuple(x) for x in f] == FIELDS
    assert [(a, b, bool(n), list(v)) for a, b, n, v in c] == CONDS
    assert FIELDS[1] == (abi.T_GROUP, abi.K_LIST, 0, 12)   # chunk_id, 2 x 5 replica members, sealed
    assert FIELDS[3:8] == FIELDS[8:13]                      # the two unrolled replicas
    assert CONDS == [(7, 6, True, [0]), (12, 11, True, [0])]


def test_unroll_limits():
    big = """struct r { int a; };
             struct e { r xs[17]; e *next; };
             struct top { e *l; };"""
    with pytest.raises(rpcgen.NotBatchable):
        rpcgen.parse(big).tape("top")
    var = """struct r { int a; };
             struct e { r xs<4>; e *next; };
             struct top { e *l; };"""
    f, c = rpcgen.parse(var).tape("top")   # an inner group: list element -> counted array
    assert f == [(abi.T_GROUP, abi.K_LIST, 0, 2), (abi.T_GROUP, abi.K_DYNAMIC, 0, 1), (abi.T_INT, abi.K_SCALAR, 0)]
    deep = """struct q { int a; };
              struct r { q qs<>; };
              struct e { r xs<4>; e *next; };
              struct top { e *l; };"""
    f, c = rpcgen.parse(deep).tape("top")   # three levels: list -> counted array -> counted array
    assert f == [(abi.T_GROUP, abi.K_LIST, 0, 3), (abi.T_GROUP, abi.K_DYNAMIC, 0, 2),
                 (abi.T_GROUP, abi.K_DYNAMIC, 0, 1), (abi.T_INT, abi.K_SCALAR, 0)] and not c
    deeper = """struct z { int a; };
                struct y { z zs<>; };
                struct x { y ys<>; };
                struct q { x xs<>; };
                struct r { q qs<>; };
                struct top { r rs<>; };"""
    with pytest.raises(rpcgen.NotBatchable):   # five levels (rpcgen.GROUP_LEVELS = 4)
        rpcgen.parse(deeper).tape("top")
    ok = """struct r { int a; hyper b; };
            struct e { r xs[3]; };
            struct top { e l<>; };"""
    f, c = rpcgen.parse(ok).tape("top")
    assert f[0] == (abi.T_GROUP, abi.K_DYNAMIC, 0, 6) and not c


@pytest.mark.parametrize("b", FIX["batches"], ids=_ids)
def test_oracle_chunk_map_fixture(b):
    hb, want, offs = _batch(b)
    rc, xdr, ro = oracle.encode_batch(FIELDS, hb.columns(), hb.n, len(want) + 64, framed=b["framed"], conds=CONDS)
    assert rc == 0
    assert xdr == want, "oracle encode differs from xdrlib"
    assert ro.tolist() == b["rec_offsets"]
    out = HostBatch.empty(FIELDS, hb.n, hb.dyn_caps())
    assert oracle.decode_batch(FIELDS, want, offs, hb.n, out.columns(), framed=b["framed"],
                               conds=CONDS) == (0, hb.n, 0)
    assert out.equal(hb)


def _mutations(want, offs, n, rng):
    """(name, stream, in_len) variants with an error inside an element."""
    out = []
    r = int(rng.integers(n // 2, n))
    a, e = int(offs[r]), int(offs[r + 1])
    y = bytearray(want)
    y[e - 12:e - 8] = b"\x00\x00\x00\x01"   # the list's closing FALSE turned into TRUE: an element past the record
    out.append(("element_past_record", bytes(y), len(y)))
    out.append(("truncated", bytes(want), a + (e - a) // 2 // 4 * 4))
    y = bytearray(want)
    y[a + 4:a + 8] = b"\x00\x00\x00\x09"    # the list's first bool word turned into another value
    out.append(("bool_changed", bytes(y), len(y)))
    return out


@pytest.fixture(params=[(8, 32768, 1024, 16384, 0, 1), (8, 32768, 1024, 16384, 0, 0), (8, 32768, 0, 0, 0, 1),
                        (64, 0, 0, 0, 0, 1), (4, 1024, 0, 4096, 1, 1), (8, 16384, 256, 32768, 2, 1)],
                ids=lambda p: f"enc{p[0]}-dtile{p[1]}-el{p[2]}-img{p[3]}-split{p[4]}-map{p[5]}")
def enc_lanes(request, gpu_ctx):
    """Group kernels under each production choice (tuning keys 32 / 33, as
    tests/test_group_cond.py)."""
    gpu_ctx.tune(32, request.param[0])
    gpu_ctx.tune(33, request.param[1])
    gpu_ctx.tune(38, request.param[2])   # element-parallel place (one top-level group)
    gpu_ctx.tune(41, request.param[3])   # element-parallel encode (key 41; 0: lanes per record)
    gpu_ctx.tune(43, request.param[4])   # element-parallel encode blocks per scan block (0: by batch size)
    gpu_ctx.tune(44, request.param[5])   # element-parallel decode from the walk's element-start map (0: record walk)
    yield request.param
    gpu_ctx.tune(0)


@pytest.mark.gpu
@pytest.mark.parametrize("b", FIX["batches"], ids=_ids)
def test_gpu_chunk_map_fixture(gpu_ctx, enc_lanes, b):
    import torch
    from oncrpc4j_amd import engine
    from oncrpc4j_amd.columns import DeviceBatch
    hb, want, offs = _batch(b)
    sch = engine.Schema(FIELDS, CONDS)
    db = DeviceBatch.from_host(hb)
    out = torch.zeros(len(want) + 64, dtype=torch.uint8, device="cuda")
    ro = torch.zeros(hb.n + 1, dtype=torch.int64, device="cuda")
    ln = gpu_ctx.encode(sch, db.columns(), hb.n, out, len(want) + 64, rec_offsets=ro, framed=b["framed"])
    assert out[:ln].cpu().numpy().tobytes() == want, "GPU encode differs from xdrlib"
    assert ro.cpu().numpy().astype(np.uint64).tolist() == b["rec_offsets"]
    back = DeviceBatch.empty(FIELDS, hb.n, hb.dyn_caps())
    assert gpu_ctx.decode(sch, out, ln, hb.n, back.columns(), rec_offsets=ro, framed=b["framed"]) == (0, hb.n, 0)
    assert back.to_host().equal(hb)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_gpu_chunk_map_errors_vs_oracle(gpu_ctx, enc_lanes, seed):
    """Streams with errors inside list elements: the engine's first bad
    record, code and the records before it equal the oracle's."""
    import torch
    from oncrpc4j_amd import engine
    from oncrpc4j_amd.columns import DeviceBatch
    b = FIX["batches"][0]
    hb, want, offs = _batch(b)
    sch = engine.Schema(FIELDS, CONDS)
    rng = np.random.default_rng(seed)
    for name, x, in_len in _mutations(want, offs, hb.n, rng):
        dev = torch.from_numpy(np.frombuffer(x, np.uint8).copy()).cuda()
        ro = torch.from_numpy(offs.astype(np.int64)).cuda()
        caps = hb.dyn_caps()
        back = DeviceBatch.empty(FIELDS, hb.n, caps)
        st = gpu_ctx.decode(sch, dev, in_len, hb.n, back.columns(), rec_offsets=ro, raise_on_error=False)
        ref = HostBatch.empty(FIELDS, hb.n, caps)
        rst = oracle.decode_batch(FIELDS, x[:in_len], offs, hb.n, ref.columns(), conds=CONDS)
        assert st == rst, (name, st, rst)
        assert back.to_host().equal(ref, upto=st[1]), name


@pytest.mark.gpu
def test_gpu_chunk_map_random_vs_oracle(gpu_ctx, enc_lanes):
    """A larger random batch of the same tape (long lists, every optional
    mix) through the engine and the oracle."""
    import torch
    from oncrpc4j_amd import engine
    from oncrpc4j_amd.columns import DeviceBatch, random_batch
    n = 3000
    hb = random_batch(FIELDS, n, seed=91, dyn_len=(0, 16), group_len=(0, 12))
    rng = np.random.default_rng(91)
    for k in (6, 11):   # per-replica checksum bools
        hb.arrays[k][:] = rng.integers(0, 2, hb.arrays[k].shape[0], dtype=np.uint8)
    rc, want, offs = oracle.encode_batch(FIELDS, hb.columns(), n, hb.xdr_total() + 64, conds=CONDS)
    assert rc == 0
    sch = engine.Schema(FIELDS, CONDS)
    db = DeviceBatch.from_host(hb)
    out = torch.zeros(len(want) + 64, dtype=torch.uint8, device="cuda")
    ro = torch.zeros(n + 1, dtype=torch.int64, device="cuda")
    ln = gpu_ctx.encode(sch, db.columns(), n, out, len(want) + 64, rec_offsets=ro)
    assert out[:ln].cpu().numpy().tobytes() == want
    back = DeviceBatch.empty(FIELDS, n, hb.dyn_caps())
    assert gpu_ctx.decode(sch, out, ln, n, back.columns(), rec_offsets=ro) == (0, n, 0)
    ref = HostBatch.empty(FIELDS, n, hb.dyn_caps())
    assert oracle.decode_batch(FIELDS, want, offs, n, ref.columns(), conds=CONDS) == (0, n, 0)
    assert back.to_host().equal(ref)


NESTED = """
const NB = 2;
struct span { unsigned int off; unsigned int len; };
union loc switch (int kind) {
    case 1: span spans[NB];
    case 2: opaque blob<8>;
    default: void;
};
struct part { hyper id; loc where; };
struct seg { part parts[2]; bool last; seg *next; };
struct seg_list { unsigned int n; seg *segs; };
"""


def test_nested_unroll_tape():
    """Fixed arrays of structs nested inside an unrolled copy, and inside a
    union arm inside it: every copy carries its own conditions."""
    f, c = rpcgen.parse(NESTED).tape("seg_list")
    assert f[1][:2] == (abi.T_GROUP, abi.K_LIST)
    m = f[1][3]
    assert len(f) == 2 + m
    # part = id, kind, 2 x (off, len), blob -> 7 fields; two parts + last
    assert m == 2 * 7 + 1
    # each part's span words hang off its own kind, the blob too
    kinds = [k for k, x in enumerate(f) if k >= 2 and any(d == k for _, d, _, _ in c)]
    assert len(kinds) == 2
    for kd in kinds:
        deps = sorted(k for k, d, _, _ in c if d == kd)
        assert deps == [kd + 1, kd + 2, kd + 3, kd + 4, kd + 5]


@pytest.mark.gpu
def test_gpu_nested_unroll_random_vs_oracle(gpu_ctx):
    import torch
    from oncrpc4j_amd import engine
    from oncrpc4j_amd.columns import DeviceBatch, random_batch
    fields, conds = rpcgen.parse(NESTED).tape("seg_list")
    n = 2000
    hb = random_batch(fields, n, seed=5, dyn_len=(0, 8), group_len=(0, 6))
    rng = np.random.default_rng(5)
    for kd in sorted({d for _, d, _, _ in conds}):
        hb.arrays[kd][:] = rng.choice(np.array([0, 1, 2], np.int32), hb.arrays[kd].shape[0])
    rc, want, offs = oracle.encode_batch(fields, hb.columns(), n, hb.xdr_total() + 64, conds=conds)
    assert rc == 0
    sch = engine.Schema(fields, conds)
    db = DeviceBatch.from_host(hb)
    out = torch.zeros(len(want) + 64, dtype=torch.uint8, device="cuda")
    ro = torch.zeros(n + 1, dtype=torch.int64, device="cuda")
    ln = gpu_ctx.encode(sch, db.columns(), n, out, len(want) + 64, rec_offsets=ro)
    assert out[:ln].cpu().numpy().tobytes() == want
    back = DeviceBatch.empty(fields, n, hb.dyn_caps())
    assert gpu_ctx.decode(sch, out, ln, n, back.columns(), rec_offsets=ro) == (0, n, 0)
    ref = HostBatch.empty(fields, n, hb.dyn_caps())
    assert oracle.decode_batch(fields, want, offs, n, ref.columns(), conds=conds) == (0, n, 0)
    assert back.to_host().equal(ref)
