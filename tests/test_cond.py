"""Conditional fields: rpcgen unions and optional data (include/xdrg.h
xdrg_cond).

A union encodes its discriminant and then the matching arm, the default arm
or nothing (jrpcgen.java:1240-1340); optional data `T *x` encodes a bool and
then T when it is true.  The fixtures (tests/golden/cond_vectors.json) were
packed by CPython's stdlib xdrlib in that order; the oracle is checked
against them on the CPU, the HIP engine against them and against the oracle
on the GPU.  Absent fields decode to zero / empty (a fresh rpcgen object's
defaults)."""
import zlib

import numpy as np
import pytest

import gold
import oracle
from oncrpc4j_amd import abi
from oncrpc4j_amd.columns import HostBatch, random_batch

I, U, E, B, H = abi.T_INT, abi.T_UINT, abi.T_ENUM, abi.T_BOOL, abi.T_HYPER
O, STR = abi.T_OPAQUE, abi.T_STRING
SC, FX, DY = abi.K_SCALAR, abi.K_FIXED, abi.K_DYNAMIC

BATCHES = gold.load("cond_vectors.json")["batches"]


def _ids(b):
    return f'{b["name"]}-{"rm" if b["framed"] else "raw"}'


def _conds(b):
    return [(f, d, n, list(v)) for f, d, n, v in b["conds"]]


def _absent_value(field):
    t, k, c = field
    if t in (O, STR):
        return "00" * c if k == FX else ""
    if k == SC:
        return 0
    return [0] * c if k == FX else []


def expected_decode(b):
    """Fixture records with absent fields at their defaults."""
    fields = [tuple(f) for f in b["fields"]]
    recs = [[v if p else _absent_value(f) for f, v, p in zip(fields, r, pres)]
            for r, pres in zip(b["records"], b["present"])]
    return gold.batch_from_records(fields, recs)


def oracle_roundtrip(fields, conds, hb, framed):
    cap = hb.xdr_total(framed)           # all fields present: an upper bound
    rc, xdr, offs = oracle.encode_batch(fields, hb.columns(), hb.n, cap, framed=framed, conds=conds)
    return rc, xdr, offs


# ---- oracle vs the xdrlib fixtures (CPU) ---------------------------------------------
@pytest.mark.parametrize("b", BATCHES, ids=_ids)
def test_oracle_cond_fixture(b):
    fields = [tuple(f) for f in b["fields"]]
    conds = _conds(b)
    hb = gold.batch_from_records(fields, b["records"])
    rc, xdr, offs = oracle_roundtrip(fields, conds, hb, b["framed"])
    assert rc == 0
    assert xdr.hex() == b["xdr"]
    assert offs.tolist() == b["rec_offsets"]
    want = expected_decode(b)
    out = HostBatch.empty(fields, hb.n, hb.dyn_caps())
    rc, fb, err = oracle.decode_batch(fields, xdr, offs, hb.n, out.columns(), framed=b["framed"],
                                      conds=conds)
    assert (rc, fb, err) == (0, hb.n, 0)
    assert out.equal(want)


def test_oracle_bool_discriminant_any_nonzero():
    """Xdr.java:404-407: a bool decodes true for any non-zero word, so the
    optional value follows a discriminant word of 5."""
    fields = [(I, SC, 0), (B, SC, 0), (U, SC, 0)]
    conds = [(2, 1, True, [0])]
    xdr = bytes.fromhex("00000007" "00000005" "0000002a")
    out = HostBatch.empty(fields, 1)
    rc, fb, err = oracle.decode_batch(fields, xdr, np.array([0, 12], np.uint64), 1, out.columns(),
                                      conds=conds)
    assert (rc, fb, err) == (0, 1, 0)
    assert out.arrays[1][0] == 1 and out.arrays[2][0] == 42


@pytest.mark.parametrize("conds", [
    [(0, 0, False, [1])],            # a field conditional on itself
    [(1, 2, False, [1])],            # discriminant after the field
    [(2, 1, False, [1])],            # discriminant is a string
    [(1, 0, False, [1]), (1, 0, False, [2])],   # two conditions on one field
])
def test_oracle_cond_invalid(conds):
    fields = [(I, SC, 0), (STR, DY, 0), (I, SC, 0)]
    hb = random_batch(fields, 4, seed=1)
    rc, _, _ = oracle_roundtrip(fields, conds, hb, False)
    assert rc == oracle.E_INVAL


# ---- the HIP engine (GPU) -------------------------------------------------------------
def _engine():
    torch = pytest.importorskip("torch")
    from oncrpc4j_amd import engine
    from oncrpc4j_amd.columns import DeviceBatch
    return torch, engine, DeviceBatch


def gpu_encode(ctx, fields, conds, hb, framed):
    torch, engine, DeviceBatch = _engine()
    sch = engine.Schema(fields, conds)
    assert sch.fixed_size == 0 and not sch.is_fixed
    db = DeviceBatch.from_host(hb)
    cap = hb.xdr_total(framed)
    out = torch.zeros(cap + 64, dtype=torch.uint8, device="cuda")
    offs = torch.zeros(hb.n + 1, dtype=torch.int64, device="cuda")
    ln = ctx.encode(sch, db.columns(), hb.n, out, cap, rec_offsets=offs, framed=framed)
    assert not out[ln:].any(), "engine wrote past the stream end"
    return out[:ln].cpu().numpy().tobytes(), offs.cpu().numpy().view(np.uint64)


def gpu_decode(ctx, fields, conds, xdr, n, offs, caps, framed):
    torch, engine, DeviceBatch = _engine()
    sch = engine.Schema(fields, conds)
    db = DeviceBatch.empty(fields, n, caps)
    # poison the fixed outputs: absent fields must be written as zero, not left alone
    for (t, k, c), x in zip(fields, db.tensors):
        if k != DY:
            x.view(torch.uint8).fill_(0xA5)
    buf = torch.from_numpy(np.frombuffer(xdr, dtype=np.uint8).copy()).cuda() if xdr else \
        torch.zeros(4, dtype=torch.uint8, device="cuda")
    ro = torch.from_numpy(np.asarray(offs, dtype=np.uint64).view(np.int64)).cuda()
    rc, fb, err = ctx.decode(sch, buf, len(xdr), n, db.columns(), rec_offsets=ro, framed=framed,
                             raise_on_error=False)
    return rc, fb, err, db.to_host()


@pytest.mark.gpu
@pytest.mark.parametrize("b", BATCHES, ids=_ids)
def test_gpu_cond_fixture(gpu_ctx, b):
    fields = [tuple(f) for f in b["fields"]]
    conds = _conds(b)
    hb = gold.batch_from_records(fields, b["records"])
    xdr, offs = gpu_encode(gpu_ctx, fields, conds, hb, b["framed"])
    assert xdr.hex() == b["xdr"]
    assert offs.tolist() == b["rec_offsets"]
    rc, fb, err, out = gpu_decode(gpu_ctx, fields, conds, xdr, hb.n, offs, hb.dyn_caps(), b["framed"])
    assert (rc, fb, err) == (0, hb.n, 0)
    assert out.equal(expected_decode(b))


def _random_cond_batch(fields, conds, n, seed):
    hb = random_batch(fields, n, seed=seed, dyn_len=(0, 40))
    rng = np.random.default_rng(seed)
    cases = sorted({v for _, _, _, vals in conds for v in vals})
    for _, d, _, _ in conds:
        if fields[d][0] == B:
            hb.arrays[d][:] = rng.integers(0, 2, n, dtype=np.uint8)
        else:
            pool = np.array(cases + [cases[-1] + 1, -7, 1 << 30], dtype=np.int64)
            hb.arrays[d][:] = pool[rng.integers(0, pool.size, n)].astype(hb.arrays[d].dtype)
    return hb


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted({b["name"] for b in BATCHES}))
@pytest.mark.parametrize("framed", [False, True], ids=["raw", "rm"])
def test_gpu_cond_random_vs_oracle(gpu_ctx, name, framed):
    b = next(x for x in BATCHES if x["name"] == name)
    fields = [tuple(f) for f in b["fields"]]
    conds = _conds(b)
    n = 20011
    hb = _random_cond_batch(fields, conds, n, seed=zlib.crc32(name.encode()) & 0xffff)
    rc, want, want_offs = oracle_roundtrip(fields, conds, hb, framed)
    assert rc == 0
    xdr, offs = gpu_encode(gpu_ctx, fields, conds, hb, framed)
    assert xdr == want
    assert np.array_equal(offs, want_offs)
    ref = HostBatch.empty(fields, n, hb.dyn_caps())
    rc, fb, err = oracle.decode_batch(fields, want, want_offs, n, ref.columns(), framed=framed,
                                      conds=conds)
    assert (rc, fb, err) == (0, n, 0)
    rc, fb, err, out = gpu_decode(gpu_ctx, fields, conds, xdr, n, offs, hb.dyn_caps(), framed)
    assert (rc, fb, err) == (0, n, 0)
    assert out.equal(ref)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["result_union", "nested", "bool_union"])
def test_gpu_cond_errors_vs_oracle(gpu_ctx, name):
    """Truncations and negative lengths inside arms: the engine reports the
    first failing record and the code a sequential decode throws."""
    b = next(x for x in BATCHES if x["name"] == name)
    fields = [tuple(f) for f in b["fields"]]
    conds = _conds(b)
    n = 3001
    hb = _random_cond_batch(fields, conds, n, seed=7)
    rc, xdr, offs = oracle_roundtrip(fields, conds, hb, False)
    assert rc == 0
    rng = np.random.default_rng(11)
    for trial in range(6):
        buf = bytearray(xdr)
        o = offs.copy()
        r = int(rng.integers(n // 4, n))
        if trial % 2 == 0:      # cut record r short by 4 bytes (if it can be)
            if o[r + 1] - o[r] >= 8:
                cut = bytearray(buf[:int(o[r + 1]) - 4]) + buf[int(o[r + 1]):]
                o[r + 1:] -= 4
                buf = cut
        else:                   # a negative length word at the end of record r
            if o[r + 1] - o[r] >= 4:
                buf[int(o[r + 1]) - 4:int(o[r + 1])] = b"\xff\xff\xff\xfe"
        data = bytes(buf)
        ref = HostBatch.empty(fields, n, hb.dyn_caps())
        want = oracle.decode_batch(fields, data, o, n, ref.columns(), conds=conds)
        rc, fb, err, _ = gpu_decode(gpu_ctx, fields, conds, data, n, o, hb.dyn_caps(), False)
        assert (rc, fb, err) == want, f"trial {trial}: record {r}"


@pytest.mark.gpu
def test_gpu_bool_discriminant_any_nonzero(gpu_ctx):
    fields = [(I, SC, 0), (B, SC, 0), (U, SC, 0)]
    conds = [(2, 1, True, [0])]
    xdr = bytes.fromhex("00000007" "00000005" "0000002a" "00000008" "00000000")
    rc, fb, err, out = gpu_decode(gpu_ctx, fields, conds, xdr, 2, [0, 12, 20], {}, False)
    assert (rc, fb, err) == (0, 2, 0)
    assert out.arrays[1].tolist() == [1, 0] and out.arrays[2].tolist() == [42, 0]


# ---- the engine's schema compiler (host only, CPU) ---------------------------------------
@pytest.mark.parametrize("conds", [
    [(0, 0, False, [1])],
    [(1, 2, False, [1])],
    [(2, 1, False, [1])],
    [(1, 0, False, [1]), (1, 0, False, [2])],
    [(1, 0, 2, [1])],                                   # negate is 0 or 1
    [(1, 0, False, list(range(abi.MAX_CASES + 1)))],    # too many case values
    [(9, 0, False, [1])],                               # no such field
])
def test_engine_schema_rejects_bad_conds(conds):
    from oncrpc4j_amd import engine
    fields = [(I, SC, 0), (STR, DY, 0), (I, SC, 0)]
    with pytest.raises(engine.XdrgError) as ei:
        engine.Schema(fields, conds)
    assert ei.value.code == abi.E_INVAL


def test_engine_schema_cond_is_variable_size():
    from oncrpc4j_amd import engine
    fields = [(I, SC, 0), (I, FX, 3), (abi.T_SHORT, SC, 0)]
    assert engine.Schema(fields).fixed_size == 20
    s = engine.Schema(fields, [(1, 0, False, [5]), (2, 0, True, [5])])
    assert s.fixed_size == 0 and not s.is_fixed


def test_engine_schema_disc_slots():
    """At most XDRG_MAX_DISC distinct discriminant fields."""
    from oncrpc4j_amd import engine
    m = abi.MAX_DISC
    fields = [(I, SC, 0)] * (2 * m + 2)
    ok = [(m + 1 + i, i, False, [i]) for i in range(m)]
    engine.Schema(fields, ok)
    bad = [(m + 1 + i, i, False, [i]) for i in range(m + 1)]
    with pytest.raises(engine.XdrgError):
        engine.Schema(fields, bad)


WIDE = ([(I, SC, 0), (STR, DY, 0), (I, DY, 0), (O, DY, 0), (B, SC, 0), (STR, DY, 0), (H, DY, 0),
         (O, DY, 0), (I, SC, 0)],
        [(2, 0, False, [1, 2]), (3, 0, True, [1, 2]), (5, 4, True, [0]), (6, 4, True, [0]),
         (8, 0, False, [2])])


@pytest.mark.gpu
@pytest.mark.parametrize("framed", [False, True], ids=["raw", "rm"])
def test_gpu_cond_wide_schema_vs_oracle(gpu_ctx, framed):
    """More dynamic fields than the lane kernels stage (wave-per-record path)."""
    fields, conds = WIDE
    n = 5003
    hb = _random_cond_batch(fields, conds, n, seed=99)
    rc, want, want_offs = oracle_roundtrip(fields, conds, hb, framed)
    assert rc == 0
    xdr, offs = gpu_encode(gpu_ctx, fields, conds, hb, framed)
    assert xdr == want and np.array_equal(offs, want_offs)
    ref = HostBatch.empty(fields, n, hb.dyn_caps())
    assert oracle.decode_batch(fields, want, want_offs, n, ref.columns(), framed=framed,
                               conds=conds) == (0, n, 0)
    rc, fb, err, out = gpu_decode(gpu_ctx, fields, conds, xdr, n, offs, hb.dyn_caps(), framed)
    assert (rc, fb, err) == (0, n, 0)
    assert out.equal(ref)
