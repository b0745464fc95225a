"""Groups inside group elements (one level down):
tests/golden/rpcgen/volume_index.x `volume_index` — every element of the
`volume *next` list holds an `extent *next` list (each extent with an
optional checksum) and, behind a bool union, a counted `ace entries<8>`
array (each entry with a string).

jrpcgen writes an array of structs inside a struct as its count and then each
element's xdrEncode (jrpcgen.java:856-906), a list as TRUE + element ...
FALSE (jrpcgen.java:835-851), recursively, so the inner arrays are ordinary
generated code.  The tape (oncrpc4j_amd.rpcgen) keeps them as inner groups:
the inner group's column is indexed by the outer element (offsets per outer
element), its members by inner element; each level's counted columns get
their own per-record counts on the device.  The fixtures
(tests/golden/volume_index_vectors.json) were packed by CPython's stdlib
xdrlib from the declarations; the oracle is checked against them on the
CPU, the HIP engine against them and against the oracle on the GPU, with
first-bad errors inside inner elements (negative inner count, cut streams,
list bools, string lengths) and capacities of every inner column."""
import os

import numpy as np
import pytest

import gold
import oracle
from oncrpc4j_amd import abi, rpcgen
from oncrpc4j_amd.columns import HostBatch, random_batch

FIX = gold.load("volume_index_vectors.json")
FIELDS = [tuple(f) for f in FIX["fields"]]
CONDS = [(f, d, bool(n), list(v)) for f, d, n, v in FIX["conds"]]
SPEC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "rpcgen", "volume_index.x")
EXT, ACL, WHO, LABEL = 4, 10, 13, 3   # inner list, inner array, its string, the outer string


def _ids(b):
    return "rm" if b["framed"] else "raw"


def _batch(b):
    hb = gold.batch_from_records(FIELDS, b["records"])
    return hb, bytes.fromhex(b["xdr"]), np.asarray(b["rec_offsets"], np.uint64)


def test_volume_index_tape():
    f, c = rpcgen.parse_file(SPEC).tape("volume_index")
    assert [tuple(x) for x in f] == FIELDS
    assert [(a, b, bool(n), list(v)) for a, b, n, v in c] == CONDS
    assert FIELDS[1] == (abi.T_GROUP, abi.K_LIST, 0, 13)     # the volume list spans both inner groups
    assert FIELDS[EXT] == (abi.T_GROUP, abi.K_LIST, 0, 4)    # extent list inside a volume
    assert FIELDS[ACL] == (abi.T_GROUP, abi.K_DYNAMIC, 0, 3)  # ace entries<> inside a volume
    assert CONDS == [(8, 7, True, [0]), (ACL, 9, False, [1])]


def test_batch_layout():
    hb, want, offs = _batch(FIX["batches"][0])
    vols = hb.elems(1)
    assert hb.rows(EXT) == vols and hb.rows(ACL) == vols   # inner groups: a row per volume
    assert hb.arrays[EXT].shape == (vols + 1,)
    assert hb.rows(EXT + 1) == hb.elems(EXT) > 0            # extent members: a row per extent
    assert hb.rows(WHO) == hb.elems(ACL) > 0
    s = hb.slice(5, 30)   # records 5..29 with their volumes, extents and entries rebased
    rc, xdr, _ = oracle.encode_batch(FIELDS, s.columns(), s.n, len(want), conds=CONDS)
    assert rc == 0 and xdr == want[int(offs[5]):int(offs[30])]


@pytest.mark.parametrize("b", FIX["batches"], ids=_ids)
def test_oracle_volume_index_fixture(b):
    hb, want, offs = _batch(b)
    rc, xdr, ro = oracle.encode_batch(FIELDS, hb.columns(), hb.n, len(want) + 64, framed=b["framed"], conds=CONDS)
    assert rc == 0
    assert xdr == want, "oracle encode differs from xdrlib"
    assert ro.tolist() == b["rec_offsets"]
    out = HostBatch.empty(FIELDS, hb.n, hb.dyn_caps())
    assert oracle.decode_batch(FIELDS, want, offs, hb.n, out.columns(), framed=b["framed"],
                               conds=CONDS) == (0, hb.n, 0)
    assert out.equal(hb)


def _probe(b, kind, nth=0):
    ps = [p for p in b["probes"] if p[1] == kind]
    return ps[nth]


def _mutations(b, want, offs, rng):
    """(name, stream, in_len, code) variants with an error inside an inner element."""
    out = []
    r, _, at = _probe(b, "acl_count", int(rng.integers(0, 4)))
    y = bytearray(want)
    y[at:at + 4] = b"\xff\xff\xff\xf0"          # `new ace[-16]`: NegativeArraySizeException
    out.append(("negative_inner_count", bytes(y), len(y), abi.E_NEG_SIZE))
    r, _, at = _probe(b, "who_len", int(rng.integers(0, 6)))
    y = bytearray(want)
    y[at:at + 4] = b"\x80\x00\x00\x01"          # a negative string length: checkArraySize
    out.append(("inner_string_corrupt", bytes(y), len(y), abi.E_CORRUPT))
    r, _, at = _probe(b, "ext_bool", int(rng.integers(0, 10)))
    y = bytearray(want)
    y[at:at + 4] = b"\x00\x00\x00\x00"          # an extent list ends early: later bytes misparse
    out.append(("inner_list_cut", bytes(y), len(y), None))
    y = bytearray(want)
    y[at:at + 4] = b"\x00\x00\x01\x00"          # any non-zero bool continues the list
    out.append(("inner_bool_value", bytes(y), len(y), 0))
    r, _, at = _probe(b, "ext_bool", int(rng.integers(10, 20)))
    out.append(("truncated_in_inner", bytes(want), at + 6, None))
    return out


@pytest.mark.parametrize("b", FIX["batches"], ids=_ids)
def test_oracle_volume_index_errors(b):
    """The oracle's first bad record and code on each mutation (the codes
    the declarations imply where they are fixed)."""
    hb, want, offs = _batch(b)
    if b["framed"]:
        pytest.skip("mutations are placed for raw streams")
    for name, x, in_len, code in _mutations(b, want, offs, np.random.default_rng(3)):
        ref = HostBatch.empty(FIELDS, hb.n, hb.dyn_caps())
        rc, fb, err = oracle.decode_batch(FIELDS, x[:in_len], offs, hb.n, ref.columns(), conds=CONDS)
        if code is not None:
            assert err == code, (name, rc, fb, err)
        assert ref.equal(hb, upto=fb), name


def _caps_variants(hb):
    """Decode capacities one short on each inner column (and the outer list)."""
    caps = hb.dyn_caps()
    out = []
    for k in (1, LABEL, EXT, ACL, WHO):
        c = dict(caps)
        c[k] = max(caps[k] - 1, 0)
        out.append((f"cap{k}", c))
    return out


def test_oracle_volume_index_capacity():
    hb, want, offs = _batch(FIX["batches"][0])
    for name, caps in _caps_variants(hb):
        ref = HostBatch.empty(FIELDS, hb.n, caps)
        rc, fb, err = oracle.decode_batch(FIELDS, want, offs, hb.n, ref.columns(), conds=CONDS)
        assert err == abi.E_CAPACITY, name
        assert ref.equal(hb, upto=fb), name


def _random(n, seed):
    hb = random_batch(FIELDS, n, seed=seed, dyn_len=(0, 24), group_len=(0, 5), inner_len=(0, 6))
    rng = np.random.default_rng(seed)
    for k in (7, 9, 14):   # the crc bool (inner), the acl union's bool and online (outer)
        hb.arrays[k][:] = rng.integers(0, 2, hb.arrays[k].shape[0], dtype=np.uint8)
    # an absent acl arm has no entries on the wire: make the native rows agree
    present = hb.arrays[9].astype(bool)
    cnt = np.diff(hb.arrays[ACL].astype(np.int64))
    keep = np.where(present, cnt, 0)
    # rebuild the acl group and its members from the kept counts
    old = hb.arrays[ACL].astype(np.int64)
    rows = np.concatenate([np.arange(old[i], old[i] + keep[i]) for i in range(len(keep))]).astype(np.int64) \
        if keep.sum() else np.zeros(0, np.int64)
    offs = np.zeros(len(keep) + 1, np.uint64)
    np.cumsum(keep.astype(np.uint64), out=offs[1:])
    hb.arrays[ACL] = offs
    for k in (ACL + 1, ACL + 2):
        hb.arrays[k] = hb.arrays[k][rows] if len(rows) else hb.arrays[k][:1]
    vals, voffs = hb.arrays[WHO]
    lens = np.diff(voffs.astype(np.int64))[rows] if len(rows) else np.zeros(0, np.int64)
    starts = voffs.astype(np.int64)[rows] if len(rows) else np.zeros(0, np.int64)
    nv = np.concatenate([vals[s:s + l] for s, l in zip(starts, lens)]) if len(rows) else vals[:0]
    no = np.zeros(len(rows) + 1, np.uint64)
    np.cumsum(lens.astype(np.uint64), out=no[1:])
    hb.arrays[WHO] = (nv if nv.size else np.zeros(1, np.uint8), no)
    return hb


def test_oracle_random_roundtrip():
    hb = _random(400, 11)
    crc_present = hb.arrays[7].astype(bool)
    hb.arrays[8][~crc_present] = 0   # an absent crc decodes to 0
    rc, want, offs = oracle.encode_batch(FIELDS, hb.columns(), hb.n, hb.xdr_total() + 64, conds=CONDS)
    assert rc == 0
    out = HostBatch.empty(FIELDS, hb.n, hb.dyn_caps())
    assert oracle.decode_batch(FIELDS, want, offs, hb.n, out.columns(), conds=CONDS) == (0, hb.n, 0)
    assert out.equal(hb)


@pytest.fixture(params=[(8, 32768, 1024, 16384), (8, 32768, 0, 0), (64, 0, 0, 4096), (4, 1024, 0, 0),
                        (8, 16384, 256, 32768), (8, 65536, 0, 0)],
                ids=lambda p: f"enc{p[0]}-dtile{p[1]}-el{p[2]}-img{p[3]}")
def grp_tune(request, gpu_ctx):
    """Group kernels under each production choice (tuning keys 32 / 33)."""
    gpu_ctx.tune(32, request.param[0])
    gpu_ctx.tune(33, request.param[1])
    gpu_ctx.tune(38, request.param[2])   # element-parallel place (one top-level group)
    gpu_ctx.tune(41, request.param[3])   # element-parallel encode image (0: lanes per record)
    yield request.param
    gpu_ctx.tune(0)


def _gpu_roundtrip(gpu_ctx, hb, want, offs, framed, ref=None):
    """Engine encode == want, engine decode == ref (default: hb itself)."""
    import torch
    from oncrpc4j_amd import engine
    from oncrpc4j_amd.columns import DeviceBatch
    sch = engine.Schema(FIELDS, CONDS)
    db = DeviceBatch.from_host(hb)
    out = torch.zeros(len(want) + 64, dtype=torch.uint8, device="cuda")
    ro = torch.zeros(hb.n + 1, dtype=torch.int64, device="cuda")
    ln = gpu_ctx.encode(sch, db.columns(), hb.n, out, len(want) + 64, rec_offsets=ro, framed=framed)
    assert out[:ln].cpu().numpy().tobytes() == want, "GPU encode differs"
    assert ro.cpu().numpy().astype(np.uint64).tolist() == offs.tolist()
    back = DeviceBatch.empty(FIELDS, hb.n, hb.dyn_caps())
    assert gpu_ctx.decode(sch, out, ln, hb.n, back.columns(), rec_offsets=ro, framed=framed) == (0, hb.n, 0)
    assert back.to_host().equal(hb if ref is None else ref)


@pytest.mark.gpu
@pytest.mark.parametrize("b", FIX["batches"], ids=_ids)
def test_gpu_volume_index_fixture(gpu_ctx, grp_tune, b):
    hb, want, offs = _batch(b)
    _gpu_roundtrip(gpu_ctx, hb, want, offs, b["framed"])


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2])
def test_gpu_volume_index_errors_vs_oracle(gpu_ctx, grp_tune, seed):
    """Errors inside inner elements: the engine's first bad record, code and
    the records before it equal the oracle's."""
    import torch
    from oncrpc4j_amd import engine
    from oncrpc4j_amd.columns import DeviceBatch
    b = FIX["batches"][0]
    hb, want, offs = _batch(b)
    sch = engine.Schema(FIELDS, CONDS)
    for name, x, in_len, _ in _mutations(b, want, offs, np.random.default_rng(seed)):
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
def test_gpu_volume_index_capacity_vs_oracle(gpu_ctx, grp_tune):
    import torch
    from oncrpc4j_amd import engine
    from oncrpc4j_amd.columns import DeviceBatch
    hb, want, offs = _batch(FIX["batches"][0])
    sch = engine.Schema(FIELDS, CONDS)
    dev = torch.from_numpy(np.frombuffer(want, np.uint8).copy()).cuda()
    ro = torch.from_numpy(offs.astype(np.int64)).cuda()
    for name, caps in _caps_variants(hb):
        back = DeviceBatch.empty(FIELDS, hb.n, caps)
        st = gpu_ctx.decode(sch, dev, len(want), hb.n, back.columns(), rec_offsets=ro, raise_on_error=False)
        ref = HostBatch.empty(FIELDS, hb.n, caps)
        rst = oracle.decode_batch(FIELDS, want, offs, hb.n, ref.columns(), conds=CONDS)
        assert st == rst, (name, st, rst)
        assert back.to_host().equal(ref, upto=st[1]), name


@pytest.mark.gpu
@pytest.mark.parametrize("framed", [False, True], ids=["raw", "rm"])
def test_gpu_volume_index_random_vs_oracle(gpu_ctx, grp_tune, framed):
    """A larger random batch (long inner lists, every optional / union mix)."""
    hb = _random(3000, 23)
    rc, want, offs = oracle.encode_batch(FIELDS, hb.columns(), hb.n, hb.xdr_total(framed) + 64, framed=framed,
                                         conds=CONDS)
    assert rc == 0
    ref = HostBatch.empty(FIELDS, hb.n, hb.dyn_caps())   # absent crc values decode to 0
    assert oracle.decode_batch(FIELDS, want, offs, hb.n, ref.columns(), framed=framed, conds=CONDS) == (0, hb.n, 0)
    _gpu_roundtrip(gpu_ctx, hb, want, offs, framed, ref)


@pytest.mark.gpu
def test_gpu_volume_index_mapped_host():
    """XDRG_HOST_MAPPED: the kernels read and write registered host columns
    of the nested schema in place."""
    import torch
    from oncrpc4j_amd import engine
    from hostmem import Registered, moved
    assert torch.cuda.is_available()
    hb0, want, offs = _batch(FIX["batches"][0])
    n = hb0.n
    c = engine.Context(0)
    mem = Registered()
    try:
        hb = moved(hb0, mem)
        sch = engine.Schema(FIELDS, CONDS)
        out = mem.array(np.zeros(len(want) + 64, np.uint8))
        ro = mem.array(np.zeros(n + 1, np.uint64))
        ln = c.encode(sch, hb.columns(), n, out, len(want) + 64, rec_offsets=ro, mapped=True)
        assert out[:ln].tobytes() == want and np.array_equal(ro, offs)
        back = moved(HostBatch.empty(FIELDS, n, hb0.dyn_caps()), mem)
        assert c.decode(sch, out, ln, n, back.columns(), rec_offsets=ro, mapped=True) == (0, n, 0)
        assert back.equal(hb0)
    finally:
        mem.close()
        c.close()


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["pageable", "registered"])
def test_gpu_volume_index_host_ptrs(kind):
    """XDRG_HOST_PTRS on the nested schema: the staging ring moves every
    level's element rows with their records (test_nested_host_stream.py has
    the many-chunk batches).  Encode == the xdrlib fixture,
    decode == the batch, and a broken stream's status and the records before
    its first bad one == the oracle's."""
    import torch
    from oncrpc4j_amd import engine
    from hostmem import Pageable, Registered, moved
    assert torch.cuda.is_available()
    b = FIX["batches"][0]
    hb0, want, offs = _batch(b)
    n = hb0.n
    c = engine.Context(0)
    mem = Registered() if kind == "registered" else Pageable()
    try:
        hb = moved(hb0, mem)
        sch = engine.Schema(FIELDS, CONDS)
        out = mem.array(np.zeros(len(want) + 64, np.uint8))
        ro = mem.array(np.zeros(n + 1, np.uint64))
        ln = c.encode(sch, hb.columns(), n, out, len(want) + 64, rec_offsets=ro, host=True)
        assert out[:ln].tobytes() == want and np.array_equal(ro, offs)
        back = moved(HostBatch.empty(FIELDS, n, hb0.dyn_caps()), mem)
        assert c.decode(sch, out, ln, n, back.columns(), rec_offsets=ro, host=True) == (0, n, 0)
        assert back.equal(hb0)
        for name, x, in_len, _ in _mutations(b, want, offs, np.random.default_rng(5)):
            xin = mem.array(np.frombuffer(x, np.uint8).copy())
            got = moved(HostBatch.empty(FIELDS, n, hb0.dyn_caps()), mem)
            st = c.decode(sch, xin, in_len, n, got.columns(), rec_offsets=ro, host=True, raise_on_error=False)
            ref = HostBatch.empty(FIELDS, n, hb0.dyn_caps())
            rst = oracle.decode_batch(FIELDS, x[:in_len], offs, n, ref.columns(), conds=CONDS)
            assert st == rst, (name, st, rst)
            assert got.equal(ref, upto=st[1]), name
    finally:
        mem.close()
        c.close()


def _empty_members_batches():
    """Batches whose inner columns hold nothing: every inner string / label
    empty, volumes without extents or entries, and no records at all."""
    rng = np.random.default_rng(31)
    out = []
    hb = _random(300, 41)   # every string empty (offsets all 0)
    for k in (WHO, LABEL):
        vals, offs = hb.arrays[k]
        hb.arrays[k] = (np.zeros(0, np.uint8), np.zeros_like(offs))
    out.append(("empty_strings", hb))
    hb = random_batch(FIELDS, 200, seed=43, dyn_len=(0, 24), group_len=(1, 4), inner_len=(0, 0))
    hb.arrays[9][:] = rng.integers(0, 2, hb.arrays[9].shape[0], dtype=np.uint8)
    hb.arrays[14][:] = rng.integers(0, 2, hb.arrays[14].shape[0], dtype=np.uint8)
    for k in range(len(FIELDS)):   # the inner groups' member columns: zero rows, zero-length arrays
        if hb.rows(k) == 0 and FIELDS[k][0] != abi.T_GROUP:
            a = hb.arrays[k]
            hb.arrays[k] = ((a[0][:0], a[1][:1]) if FIELDS[k][1] == abi.K_DYNAMIC else a[:0])
    out.append(("no_inner_elements", hb))
    out.append(("no_records", random_batch(FIELDS, 0, seed=44)))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["pageable", "registered", "mapped"])
def test_gpu_volume_index_host_empty_members(kind):
    """Nested schema on host memory with columns that hold no bytes (ADVICE
    r4: the bounce path mapped zero-byte spans to nothing and copied a fixed
    member's row out of a zero-row column): encode == oracle, decode == the
    batch, into zero-length member arrays."""
    import torch
    from oncrpc4j_amd import engine
    from hostmem import Pageable, Registered, moved
    assert torch.cuda.is_available()
    c = engine.Context(0)
    mem = Pageable() if kind == "pageable" else Registered()
    host, mapped = kind != "mapped", kind == "mapped"
    try:
        for name, hb0 in _empty_members_batches():
            n = hb0.n
            rc, want, offs = oracle.encode_batch(FIELDS, hb0.columns(), n, hb0.xdr_total() + 64, conds=CONDS)
            assert rc == 0, name
            ref = HostBatch.empty(FIELDS, n, hb0.dyn_caps())
            assert oracle.decode_batch(FIELDS, want, offs, n, ref.columns(), conds=CONDS) == (0, n, 0), name
            hb = moved(hb0, mem)
            sch = engine.Schema(FIELDS, CONDS)
            out = mem.array(np.zeros(len(want) + 64, np.uint8))
            ro = mem.array(np.zeros(n + 1, np.uint64))
            ln = c.encode(sch, hb.columns(), n, out, len(want) + 64, rec_offsets=ro, host=host, mapped=mapped)
            assert out[:ln].tobytes() == want and np.array_equal(ro, offs), name
            back0 = HostBatch.empty(FIELDS, n, hb0.dyn_caps())
            for k in range(len(FIELDS)):   # zero-row member columns (rows of the batch) as zero-length arrays
                if FIELDS[k][0] != abi.T_GROUP and hb0.rows(k) == 0 and n:
                    a = back0.arrays[k]
                    back0.arrays[k] = (a[0][:0], a[1][:1]) if FIELDS[k][1] == abi.K_DYNAMIC else a[:0]
            back = moved(back0, mem)
            assert c.decode(sch, out, ln, n, back.columns(), rec_offsets=ro, host=host, mapped=mapped) == (0, n, 0), name
            assert back.equal(ref), name
    finally:
        mem.close()
        c.close()
