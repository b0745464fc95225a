"""Unions inside list elements and a list inside a union arm (SURVEY.md §8f
row 2): READDIRPLUS-like replies, tests/golden/rpcgen/plus_types.x
`plus_res` — the reply union's OK arm holds optional directory attributes, a
verifier and a `plus_entry *next` list whose every element carries an
optional attribute union and an optional handle union; the default arm holds
only the directory attributes.

jrpcgen encodes the union's discriminant and then the matching arm
(jrpcgen.java:1240-1340) and a list as TRUE + element ... FALSE
(jrpcgen.java:835-851).  The tape (oncrpc4j_amd.rpcgen) makes the list a
repeated group under the status condition and the element unions conditions
between members of the group, evaluated per element.  The fixtures
(tests/golden/group_cond_vectors.json) were packed by CPython's stdlib xdrlib
from the declarations, not from the tape; the oracle is checked against them
on the CPU, the HIP engine against them and against the oracle on the GPU,
with first-bad errors inside elements."""
import os

import numpy as np
import pytest

import gold
import oracle
from oncrpc4j_amd import abi, rpcgen
from oncrpc4j_amd.columns import HostBatch

FIX = gold.load("group_cond_vectors.json")
FIELDS = [tuple(f) for f in FIX["fields"]]
CONDS = [(f, d, bool(n), list(v)) for f, d, n, v in FIX["conds"]]
SPEC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "rpcgen", "plus_types.x")


def _ids(b):
    return "rm" if b["framed"] else "raw"


def _batch(b):
    hb = gold.batch_from_records(FIELDS, b["records"])
    return hb, bytes.fromhex(b["xdr"]), np.asarray(b["rec_offsets"], np.uint64)


def test_plus_res_tape():
    f, c = rpcgen.parse_file(SPEC).tape("plus_res")
    assert [tuple(x) for x in f] == FIELDS
    assert [(a, b, bool(n), list(v)) for a, b, n, v in c] == CONDS
    assert FIELDS[7] == (abi.T_GROUP, abi.K_LIST, 0, 10)       # the entry list, in the OK arm
    assert (7, 0, False, [0]) in CONDS
    assert (12, 11, False, [1]) in CONDS and (17, 16, False, [1]) in CONDS   # element unions
    with pytest.raises(rpcgen.NotBatchable):
        rpcgen.parse_file(SPEC).fields("plus_res")


@pytest.mark.parametrize("b", FIX["batches"], ids=_ids)
def test_oracle_plus_res_fixture(b):
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
    x = bytearray(want)
    # a handle length word past the record (SHORT): the last 4-byte-aligned word that holds 0..64
    # inside some record's list is hard to find by offset, so corrupt records whole instead
    r = int(rng.integers(n // 2, n))
    a, e = int(offs[r]), int(offs[r + 1])
    y = bytearray(x)
    y[e - 8:e] = b"\x00\x00\x00\x01" + b"\x7f\xff\xff\x00"   # the list's FALSE / eof turned into TRUE + a bogus element
    out.append(("element_past_record", bytes(y), len(y)))
    out.append(("truncated", bytes(x), int(offs[r]) + (e - a) // 2 // 4 * 4))
    y = bytearray(x)
    y[a + 4:a + 8] = b"\x00\x00\x00\x07"   # status / attribute bool words turned into other values
    out.append(("disc_changed", bytes(y), len(y)))
    return out


@pytest.fixture(params=[(8, 32768, 1024, 16384, 0, 1), (8, 32768, 1024, 16384, 0, 0), (8, 32768, 0, 0, 0, 1),
                        (64, 0, 0, 0, 0, 1), (4, 1024, 0, 4096, 1, 1), (8, 16384, 256, 32768, 2, 1)],
                ids=lambda p: f"enc{p[0]}-dtile{p[1]}-el{p[2]}-img{p[3]}-split{p[4]}-map{p[5]}")
def enc_lanes(request, gpu_ctx):
    """Group kernels under each production choice: encode place lanes per
    record (tuning key 32; 8 the default, 64 a wave per record) and decode
    place LDS tile (key 33; 32 KiB the default, 0 records read from HBM,
    1 KiB: most records larger than the tile take the HBM path)."""
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
def test_gpu_plus_res_fixture(gpu_ctx, enc_lanes, b):
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
def test_gpu_plus_res_errors_vs_oracle(gpu_ctx, enc_lanes, seed):
    """Streams with errors inside list elements and changed discriminants:
    the engine's first bad record, code and the records before it equal the
    oracle's."""
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
def test_gpu_plus_res_random_vs_oracle(gpu_ctx, enc_lanes):
    """A larger random batch of the same tape (shapes the fixture does not
    hold: long lists, every arm mix) through the engine and the oracle."""
    import torch
    from oncrpc4j_amd import engine
    from oncrpc4j_amd.columns import DeviceBatch, random_batch
    n = 3000
    hb = random_batch(FIELDS, n, seed=77, dyn_len=(0, 40), group_len=(0, 12))
    rng = np.random.default_rng(77)
    hb.arrays[0][:] = rng.choice(np.array([0, 0, 0, 2, 5], np.int32), n)
    for k in (1, 19):
        hb.arrays[k][:] = rng.integers(0, 2, n, dtype=np.uint8)
    for k in (11, 16):   # element bools
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
