"""Repeated groups: arrays of structs and recursive lists (include/xdrg.h
"Repeated groups").

rpcgen encodes `T x<>` of a struct T as the element count and then every
element's fields, `T x[N]` without the count (jrpcgen.java:856-906), and a
recursive optional list `T *x` (struct T { ...; T *next; }) as TRUE +
element for each element, then FALSE (INDIRECTION, jrpcgen.java:835-851) —
the bytes oncrpc4j's own portmap/pmaplist.java:63-70 and rpcb_list.java
write.  Decoding a negative count is `new T[-2]`: NegativeArraySizeException
(XDRG_E_NEG_SIZE).  The fixtures (tests/golden/group_vectors.json) were
packed by CPython's stdlib xdrlib; the oracle is checked against them on the
CPU, the HIP engine against them and against the oracle on the GPU."""
import numpy as np
import pytest

import gold
import oracle
from oncrpc4j_amd import abi
from oncrpc4j_amd.columns import HostBatch, random_batch

I, U, B, H, F = abi.T_INT, abi.T_UINT, abi.T_BOOL, abi.T_HYPER, abi.T_FLOAT
O, STR, G = abi.T_OPAQUE, abi.T_STRING, abi.T_GROUP
SC, FX, DY, LS = abi.K_SCALAR, abi.K_FIXED, abi.K_DYNAMIC, abi.K_LIST

BATCHES = gold.load("group_vectors.json")["batches"]


def _ids(b):
    return f'{b["name"]}-{"rm" if b["framed"] else "raw"}'


def _fields(b):
    return [tuple(f) for f in b["fields"]]


def _offs(v):
    return np.asarray(v, dtype=np.uint64)


# ---- oracle vs the xdrlib fixtures (CPU) ---------------------------------------------
@pytest.mark.parametrize("b", BATCHES, ids=_ids)
def test_oracle_group_fixture(b):
    fields = _fields(b)
    hb = gold.batch_from_records(fields, b["records"])
    assert hb.xdr_sizes(b["framed"]).tolist() == np.diff(b["rec_offsets"]).tolist()
    rc, xdr, offs = oracle.encode_batch(fields, hb.columns(), hb.n, hb.xdr_total(b["framed"]),
                                        framed=b["framed"])
    assert rc == 0
    assert xdr.hex() == b["xdr"]
    assert offs.tolist() == b["rec_offsets"]
    out = HostBatch.empty(fields, hb.n, hb.dyn_caps())
    rc, fb, err = oracle.decode_batch(fields, xdr, offs, hb.n, out.columns(), framed=b["framed"])
    assert (rc, fb, err) == (0, hb.n, 0)
    assert out.equal(hb)


PMAP = [(G, LS, 0, 4), (I, SC, 0), (I, SC, 0), (I, SC, 0), (I, SC, 0)]
ITEMS = [(I, SC, 0), (G, DY, 0, 2), (I, SC, 0), (STR, DY, 0), (I, SC, 0)]


def _decode(fields, xdr, n=1, caps=None):
    out = HostBatch.empty(fields, n, caps or {k: 64 for k in range(len(fields))})
    offs = _offs([0, len(xdr)]) if n == 1 else None
    return oracle.decode_batch(fields, xdr, offs, n, out.columns()), out


ERROR_CASES = [
    # count -2: new item[-2] -> NegativeArraySizeException (jrpcgen.java:886-906)
    ("negative_count", ITEMS, "00000001" "fffffffe", abi.E_NEG_SIZE),
    # count 2, one element present -> the second element's int is short
    ("short_element", ITEMS, "00000001" "00000002" "00000007" "00000001" "61000000", abi.E_SHORT),
    # element string length -1 -> checkArraySize (Xdr.java:1034-1037)
    ("corrupt_member", ITEMS, "00000001" "00000001" "00000007" "ffffffff", abi.E_CORRUPT),
    # a list whose closing bool is missing
    ("list_unterminated", PMAP, "00000001" "00000001" "00000002" "00000003" "00000004", abi.E_SHORT),
    # the count word itself missing
    ("missing_count", ITEMS, "00000001", abi.E_SHORT),
]


@pytest.mark.parametrize("name,fields,hexs,code", ERROR_CASES, ids=[c[0] for c in ERROR_CASES])
def test_oracle_group_errors(name, fields, hexs, code):
    (rc, fb, err), _ = _decode(fields, bytes.fromhex(hexs))
    assert (rc, fb, err) == (code, 0, code)


def test_oracle_list_bool_any_nonzero():
    """xdrDecodeBoolean: any non-zero word continues the list (Xdr.java:404-407)."""
    xdr = bytes.fromhex("00000007" "00000001" "00000002" "00000003" "00000004" "00000000")
    (rc, fb, err), out = _decode(PMAP, xdr)
    assert (rc, fb, err) == (0, 1, 0)
    assert out.arrays[0].tolist() == [0, 1] and out.arrays[4][0] == 4


def test_oracle_group_capacity_after_walk():
    """Capacity is reported only when the group's walk succeeds: a SHORT
    element wins over too few element slots."""
    xdr = bytes.fromhex("00000001" "00000003" + "00000007" "00000000" * 2)   # 3rd element short
    (rc, _, _), _ = _decode(ITEMS, xdr, caps={1: 1, 3: 8})
    assert rc == abi.E_SHORT
    xdr = bytes.fromhex("00000001" "00000002" + "00000007" "00000000" * 2 + "00000009")
    (rc, _, _), _ = _decode(ITEMS, xdr, caps={1: 1, 3: 8})
    assert rc == abi.E_CAPACITY


@pytest.mark.parametrize("fields", [
    [(G, DY, 0, 0), (I, SC, 0)],               # no members
    [(G, DY, 0, 3), (I, SC, 0)],               # members past the tape
    [(G, LS, 2, 1), (I, SC, 0)],               # a list has no count
    [(G, DY, 0, 5), (G, DY, 0, 4), (G, DY, 0, 3), (G, DY, 0, 2), (G, DY, 0, 1), (I, SC, 0)],   # five levels
    [(G, DY, 0, 2), (I, SC, 0), (G, DY, 0, 1), (I, SC, 0)],      # an inner group past its parent's span
    [(G, DY, 0, 2), (G, FX, 2, 1), (I, FX, 0)],                  # inner elements of no bytes
    [(G, FX, 4, 1), (I, FX, 0)],               # elements of no bytes
])
def test_oracle_group_invalid(fields):
    hb = HostBatch.empty([(I, SC, 0)], 1)
    flat = [tuple(f) for f in fields]
    arr = oracle.fields_array(flat)
    cols = (oracle.Column * len(flat))()
    out = np.zeros(64, np.uint8)
    L = oracle.lib()
    rc = L.xo_encode_batch(arr, len(flat), __import__("ctypes").addressof(cols), 0, out.ctypes.data, 64,
                           None, 0, None)
    assert rc == abi.E_INVAL
    del hb


def test_oracle_group_random_roundtrip():
    fields = [(H, SC, 0), (G, DY, 0, 3), (U, SC, 0), (STR, DY, 0), (I, FX, 2),
              (G, LS, 0, 2), (B, SC, 0), (O, DY, 0), (I, DY, 0)]
    hb = random_batch(fields, 300, seed=11, dyn_len=(0, 9), group_len=(0, 6), special_floats=False)
    for framed in (False, True):
        rc, xdr, offs = oracle.encode_batch(fields, hb.columns(), hb.n, hb.xdr_total(framed), framed=framed)
        assert rc == 0 and len(xdr) == hb.xdr_total(framed)
        out = HostBatch.empty(fields, hb.n, hb.dyn_caps())
        rc, fb, err = oracle.decode_batch(fields, xdr, offs, hb.n, out.columns(), framed=framed)
        assert (rc, fb, err) == (0, hb.n, 0)
        # bools decode as 0/1 (Xdr.java:404-407)
        want = hb.arrays[6].copy()
        hb2 = HostBatch(hb.fields, hb.n, list(hb.arrays))
        hb2.arrays[6] = (want != 0).astype(np.uint8)
        assert out.equal(hb2)


# ---- the HIP engine (GPU) -------------------------------------------------------------
def _engine():
    torch = pytest.importorskip("torch")
    from oncrpc4j_amd import engine
    from oncrpc4j_amd.columns import DeviceBatch
    return torch, engine, DeviceBatch


def gpu_encode(ctx, fields, hb, framed):
    torch, engine, DeviceBatch = _engine()
    sch = engine.Schema(fields)
    assert sch.fixed_size == 0 and not sch.is_fixed
    db = DeviceBatch.from_host(hb)
    cap = hb.xdr_total(framed)
    out = torch.zeros(cap + 64, dtype=torch.uint8, device="cuda")
    offs = torch.zeros(hb.n + 1, dtype=torch.int64, device="cuda")
    ln = ctx.encode(sch, db.columns(), hb.n, out, cap, rec_offsets=offs, framed=framed)
    assert not out[ln:].any(), "engine wrote past the stream end"
    return out[:ln].cpu().numpy().tobytes(), offs.cpu().numpy().view(np.uint64)


def gpu_decode(ctx, fields, xdr, n, offs, caps, framed):
    torch, engine, DeviceBatch = _engine()
    sch = engine.Schema(fields)
    db = DeviceBatch.empty(fields, n, caps)
    buf = torch.from_numpy(np.frombuffer(xdr, dtype=np.uint8).copy()).cuda() if xdr else \
        torch.zeros(4, dtype=torch.uint8, device="cuda")
    ro = torch.from_numpy(np.asarray(offs, dtype=np.uint64).view(np.int64)).cuda()
    rc, fb, err = ctx.decode(sch, buf, len(xdr), n, db.columns(), rec_offsets=ro, framed=framed,
                             raise_on_error=False)
    return rc, fb, err, db.to_host()


@pytest.mark.gpu
@pytest.mark.parametrize("b", BATCHES, ids=_ids)
def test_gpu_group_fixture(gpu_ctx, enc_lanes, b):
    fields = _fields(b)
    hb = gold.batch_from_records(fields, b["records"])
    xdr, offs = gpu_encode(gpu_ctx, fields, hb, b["framed"])
    assert xdr.hex() == b["xdr"]
    assert offs.tolist() == b["rec_offsets"]
    rc, fb, err, out = gpu_decode(gpu_ctx, fields, xdr, hb.n, offs, hb.dyn_caps(), b["framed"])
    assert (rc, fb, err) == (0, hb.n, 0)
    assert out.equal(hb)


SHAPES = {
    "pmaplist": PMAP,
    "items": ITEMS,
    "dirlist": [(G, LS, 0, 3), (H, SC, 0), (STR, DY, 0), (H, SC, 0), (B, SC, 0)],
    "fixed_pairs": [(I, SC, 0), (G, FX, 3, 2), (abi.T_SHORT, SC, 0), (I, DY, 0), (H, SC, 0)],
    "two_groups": [(G, DY, 0, 2), (U, SC, 0), (STR, DY, 0), (G, LS, 0, 3), (B, SC, 0),
                   (abi.T_DOUBLE, SC, 0), (O, FX, 5), (O, DY, 0)],
    "fixed_members_only": [(O, DY, 0), (G, DY, 0, 3), (I, SC, 0), (abi.T_BYTE, FX, 3), (H, SC, 0)],
}


def _sane(hb):
    """Values the codec maps one to one: bools 0/1, no NaN payloads."""
    for k, f in enumerate(hb.fields):
        if f[0] == B:
            hb.arrays[k] = (hb.arrays[k] != 0).astype(np.uint8)
        if f[0] in (F, abi.T_DOUBLE) and f[1] != DY:
            a = hb.arrays[k]
            a[np.isnan(a)] = 0
    return hb


@pytest.fixture(params=[(8, 32768, 1024, 32768, 0, 1), (8, 32768, 1024, 32768, 0, 0), (8, 32768, 0, 0, 0, 1),
                        (64, 0, 0, 0, 0, 1), (4, 1024, 0, 4096, 1, 1), (8, 16384, 256, 16384, 2, 1)],
                ids=lambda p: f"enc{p[0]}-dtile{p[1]}-el{p[2]}-img{p[3]}-split{p[4]}-map{p[5]}")
def enc_lanes(request, gpu_ctx):
    """Group kernels under each production choice: encode place lanes per
    record (tuning key 32; 8 the default, 64 a wave per record) and decode
    place LDS tile (key 33; 32 KiB the default, 0 records read from HBM,
    1 KiB: most records larger than the tile take the HBM path); the
    element-parallel places (key 38 decode, key 41 encode image: 4 KiB sends
    the large-element records through the lane path)."""
    gpu_ctx.tune(32, request.param[0])
    gpu_ctx.tune(33, request.param[1])
    gpu_ctx.tune(38, request.param[2])   # element-parallel place (one top-level group)
    gpu_ctx.tune(41, request.param[3])   # element-parallel encode (one top-level group without inner groups)
    gpu_ctx.tune(43, request.param[4])   # element-parallel encode blocks per scan block (0: by batch size)
    gpu_ctx.tune(44, request.param[5])   # element-parallel decode from the walk's element-start map (0: record walk)
    yield request.param
    gpu_ctx.tune(0)


@pytest.mark.gpu
@pytest.mark.parametrize("framed", [False, True], ids=["raw", "rm"])
@pytest.mark.parametrize("shape", list(SHAPES), ids=list(SHAPES))
def test_gpu_group_vs_oracle(gpu_ctx, enc_lanes, shape, framed):
    fields = SHAPES[shape]
    for n, glen in ((1, (0, 3)), (3000, (0, 9)), (20000, (0, 3)), (900, (60, 140))):
        hb = _sane(random_batch(fields, n, seed=n + len(shape), dyn_len=(0, 21), group_len=glen))
        rc, want, woffs = oracle.encode_batch(fields, hb.columns(), n, hb.xdr_total(framed), framed=framed)
        assert rc == 0
        xdr, offs = gpu_encode(gpu_ctx, fields, hb, framed)
        assert xdr == want, f"n={n}: encode differs from the oracle"
        assert offs.tolist() == woffs.tolist()
        rc, fb, err, out = gpu_decode(gpu_ctx, fields, xdr, n, offs, hb.dyn_caps(), framed)
        assert (rc, fb, err) == (0, n, 0)
        assert out.equal(hb)


def _corrupt_cases():
    """(name, fields, record index, how to break its bytes)"""
    return [
        ("neg_count", ITEMS, lambda b: b[:4] + bytes.fromhex("fffffffe") + b[8:]),
        ("short_tail", ITEMS, lambda b: b[:-4]),
        ("corrupt_string", [(G, DY, 0, 1), (STR, DY, 0)],
         lambda b: b[:4] + bytes.fromhex("80000000") + b[8:] if len(b) > 8 else b[:-4]),
        ("list_cut", PMAP, lambda b: b[:-4]),
        ("list_bool_nonzero", PMAP, lambda b: bytes.fromhex("00000009") + b[4:]),
    ]


@pytest.mark.gpu
@pytest.mark.parametrize("case", _corrupt_cases(), ids=lambda c: c[0])
def test_gpu_group_errors_first_bad(gpu_ctx, enc_lanes, case):
    """Every record is its own message; one broken record in the middle: the
    engine reports the oracle's (first_bad, code) and decodes every record
    before it."""
    name, fields, brk = case
    hb = _sane(random_batch(fields, 4000, seed=7, dyn_len=(1, 9), group_len=(1, 5)))
    rc, xdr, offs = oracle.encode_batch(fields, hb.columns(), hb.n, hb.xdr_total(False))
    assert rc == 0
    recs = [xdr[int(offs[i]):int(offs[i + 1])] for i in range(hb.n)]
    bad = 2345
    recs[bad] = brk(recs[bad])
    stream = b"".join(recs)
    o = np.zeros(hb.n + 1, np.uint64)
    np.cumsum([len(r) for r in recs], out=o[1:])
    want = HostBatch.empty(fields, hb.n, hb.dyn_caps())
    wrc, wfb, werr = oracle.decode_batch(fields, stream, o, hb.n, want.columns())
    rc, fb, err, out = gpu_decode(gpu_ctx, fields, stream, hb.n, o, hb.dyn_caps(), False)
    assert (rc, fb, err) == (wrc, wfb, werr)
    if wrc:
        assert wfb == bad
        assert out.equal(want, upto=bad)


@pytest.mark.gpu
def test_gpu_group_capacity(gpu_ctx, enc_lanes):
    fields = ITEMS
    hb = random_batch(fields, 500, seed=3, dyn_len=(0, 9), group_len=(0, 5))
    rc, xdr, offs = oracle.encode_batch(fields, hb.columns(), hb.n, hb.xdr_total(False))
    caps = hb.dyn_caps()
    for k in (1, 3):   # too few element slots / too few string bytes
        small = dict(caps)
        small[k] = caps[k] // 2
        want = HostBatch.empty(fields, hb.n, small)
        wrc, wfb, werr = oracle.decode_batch(fields, xdr, offs, hb.n, want.columns())
        rc, fb, err, out = gpu_decode(gpu_ctx, fields, xdr, hb.n, offs, small, False)
        assert (rc, fb, err) == (wrc, wfb, werr) and wrc == abi.E_CAPACITY
        assert out.equal(want, upto=wfb)


@pytest.mark.gpu
def test_gpu_group_encode_capacity(gpu_ctx):
    torch, engine, DeviceBatch = _engine()
    hb = random_batch(PMAP, 100, seed=5)
    sch = engine.Schema(PMAP)
    db = DeviceBatch.from_host(hb)
    need = hb.xdr_total(False)
    out = torch.zeros(need, dtype=torch.uint8, device="cuda")
    with pytest.raises(engine.CapacityError):
        gpu_ctx.encode(sch, db.columns(), hb.n, out, need - 4)
    assert not out.any()


@pytest.mark.gpu
@pytest.mark.parametrize("framed", [False, True], ids=["raw", "rm"])
def test_gpu_group_extent_past_stream(gpu_ctx, enc_lanes, framed):
    """rec_offsets[n] beyond in_len while the last record still parses (its
    extent claims bytes the stream does not hold): decode reads nothing past
    in_len, and the staged decode's tile is clamped the same way
    (kernels_group.hip k_grp_dec_place_lds)."""
    fields = SHAPES["dirlist"]
    hb = _sane(random_batch(fields, 3000, seed=17, dyn_len=(0, 21), group_len=(0, 6)))
    rc, xdr, offs = oracle.encode_batch(fields, hb.columns(), hb.n, hb.xdr_total(framed), framed=framed)
    assert rc == 0
    ro = offs.astype(np.uint64).copy()
    ro[-1] += 4096   # the last extent runs 4 KiB past the stream
    want = HostBatch.empty(fields, hb.n, hb.dyn_caps())
    wrc, wfb, werr = oracle.decode_batch(fields, xdr, ro, hb.n, want.columns(), framed=framed)
    rc, fb, err, out = gpu_decode(gpu_ctx, fields, xdr, hb.n, ro, hb.dyn_caps(), framed)
    assert (rc, fb, err) == (wrc, wfb, werr)
    assert out.equal(want, upto=wfb)
