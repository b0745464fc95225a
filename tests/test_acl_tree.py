"""Four group levels (jrpcgen recurses through arrays of
structs and lists at any depth, jrpcgen.java:835-906):
tests/golden/rpcgen/acl_tree.x `tree_res` — the `tree_entry *next` list, a
`tree_ace *next` list inside every entry, a counted `tree_principal who<8>`
inside every access entry (each principal with optional data) and a counted
`tree_tag tags<>` inside every principal.

The tape (oncrpc4j_amd.rpcgen) nests the groups: each level's column is
indexed by the elements of the level above, each level's counted columns get
their own per-record counts on the device.  The fixtures
(tests/golden/acl_tree_vectors.json) were packed by CPython's stdlib xdrlib
from the declarations; the oracle is checked against them on the CPU, the HIP
engine against them and against the oracle on the GPU, with first-bad errors
at every level (negative counts, corrupt lengths, list bools, cut streams)
and capacities of every nested column."""
import os

import numpy as np
import pytest

import gold
import oracle
from oncrpc4j_amd import abi, rpcgen
from oncrpc4j_amd.columns import HostBatch, random_batch

FIX = gold.load("acl_tree_vectors.json")
FIELDS = [tuple(f) for f in FIX["fields"]]
CONDS = [(f, d, bool(n), list(v)) for f, d, n, v in FIX["conds"]]
SPEC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "rpcgen", "acl_tree.x")
ENT, NAME, ACL, WHO, REALM, GIDB, GID, TAGS, VALUE, EOF = 1, 3, 4, 6, 8, 9, 10, 11, 13, 14


def _ids(b):
    return "rm" if b["framed"] else "raw"


def _batch(b):
    hb = gold.batch_from_records(FIELDS, b["records"])
    return hb, bytes.fromhex(b["xdr"]), np.asarray(b["rec_offsets"], np.uint64)


def test_acl_tree_tape():
    f, c = rpcgen.parse_file(SPEC).tape("tree_res")
    assert [tuple(x) for x in f] == FIELDS
    assert [(a, b, bool(n), list(v)) for a, b, n, v in c] == CONDS
    assert FIELDS[ENT] == (abi.T_GROUP, abi.K_LIST, 0, 12)      # level 0 spans everything below
    assert FIELDS[ACL] == (abi.T_GROUP, abi.K_LIST, 0, 9)       # level 1: a list inside an entry
    assert FIELDS[WHO] == (abi.T_GROUP, abi.K_DYNAMIC, 0, 7)    # level 2: a counted array
    assert FIELDS[TAGS] == (abi.T_GROUP, abi.K_DYNAMIC, 0, 2)   # level 3: a counted array
    assert CONDS == [(GID, GIDB, True, [0])]                    # the optional gid at level 2


def test_batch_layout():
    hb, want, offs = _batch(FIX["batches"][0])
    assert hb.rows(ACL) == hb.elems(ENT)           # a level's column: a row per element above
    assert hb.rows(WHO) == hb.elems(ACL) > 0
    assert hb.rows(TAGS) == hb.elems(WHO) > 0
    assert hb.rows(VALUE) == hb.elems(TAGS) > 0
    s = hb.slice(5, 30)   # records 5..29 with every level rebased
    rc, xdr, _ = oracle.encode_batch(FIELDS, s.columns(), s.n, len(want), conds=CONDS)
    assert rc == 0 and xdr == want[int(offs[5]):int(offs[30])]


@pytest.mark.parametrize("b", FIX["batches"], ids=_ids)
def test_oracle_acl_tree_fixture(b):
    hb, want, offs = _batch(b)
    rc, xdr, ro = oracle.encode_batch(FIELDS, hb.columns(), hb.n, len(want) + 64, framed=b["framed"], conds=CONDS)
    assert rc == 0
    assert xdr == want, "oracle encode differs from xdrlib"
    assert ro.tolist() == b["rec_offsets"]
    out = HostBatch.empty(FIELDS, hb.n, hb.dyn_caps())
    assert oracle.decode_batch(FIELDS, want, offs, hb.n, out.columns(), framed=b["framed"],
                               conds=CONDS) == (0, hb.n, 0)
    assert out.equal(hb)


def test_five_levels_refused():
    """One level past the engine's four: the oracle and the schema refuse it."""
    G, DY, I, SC = abi.T_GROUP, abi.K_DYNAMIC, abi.T_INT, abi.K_SCALAR
    flat = [(G, DY, 0, 5), (G, DY, 0, 4), (G, DY, 0, 3), (G, DY, 0, 2), (G, DY, 0, 1), (I, SC, 0)]
    arr = oracle.fields_array(flat)
    cols = (oracle.Column * len(flat))()
    out = np.zeros(64, np.uint8)
    rc = oracle.lib().xo_encode_batch(arr, len(flat), __import__("ctypes").addressof(cols), 0,
                                      out.ctypes.data, 64, None, 0, None)
    assert rc == abi.E_INVAL
    four = flat[1:]
    arr4 = oracle.fields_array(four)
    cols4 = (oracle.Column * len(four))()
    rc4 = oracle.lib().xo_encode_batch(arr4, len(four), __import__("ctypes").addressof(cols4), 0,
                                       out.ctypes.data, 64, None, 0, None)
    assert rc4 == abi.OK


def _probe(b, kind, nth=0):
    ps = [p for p in b["probes"] if p[1] == kind]
    return ps[nth % len(ps)]


def _mutations(b, want, offs, rng):
    """(name, stream, in_len, code, record) variants with an error at each
    level, in record `record` (a cut list may still parse, into other values)."""
    out = []
    r, _, at = _probe(b, "tags_count", int(rng.integers(0, 30)))
    y = bytearray(want)
    y[at:at + 4] = b"\xff\xff\xff\xf0"          # level 3 `new tree_tag[-16]`: NegativeArraySizeException
    out.append(("negative_level3_count", bytes(y), len(y), abi.E_NEG_SIZE, r))
    r, _, at = _probe(b, "who_count", int(rng.integers(0, 20)))
    y = bytearray(want)
    y[at:at + 4] = b"\xff\xff\xff\xfe"          # level 2 count
    out.append(("negative_level2_count", bytes(y), len(y), abi.E_NEG_SIZE, r))
    r, _, at = _probe(b, "value_len", int(rng.integers(0, 30)))
    y = bytearray(want)
    y[at:at + 4] = b"\x80\x00\x00\x05"          # a negative opaque length at level 3: checkArraySize
    out.append(("level3_opaque_corrupt", bytes(y), len(y), abi.E_CORRUPT, r))
    r, _, at = _probe(b, "realm_len", int(rng.integers(0, 30)))
    y = bytearray(want)
    y[at:at + 4] = b"\x80\x00\x00\x01"          # a negative string length at level 2
    out.append(("level2_string_corrupt", bytes(y), len(y), abi.E_CORRUPT, r))
    r, _, at = _probe(b, "ace_bool", int(rng.integers(0, 20)))
    y = bytearray(want)
    y[at:at + 4] = b"\x00\x00\x00\x00"          # a level-1 list ends early: later bytes misparse
    out.append(("level1_list_cut", bytes(y), len(y), None, r))
    y = bytearray(want)
    y[at:at + 4] = b"\x00\x00\x02\x00"          # any non-zero bool continues the list
    out.append(("level1_bool_value", bytes(y), len(y), 0, r))
    r, _, at = _probe(b, "tags_count", int(rng.integers(30, 60)))
    out.append(("truncated_in_level3", bytes(want), at + 2, None, r))
    return out


@pytest.mark.parametrize("b", FIX["batches"], ids=_ids)
def test_oracle_acl_tree_errors(b):
    """The oracle's first bad record and code on each mutation (the codes the
    declarations imply where they are fixed)."""
    hb, want, offs = _batch(b)
    if b["framed"]:
        pytest.skip("mutations are placed for raw streams")
    for name, x, in_len, code, r in _mutations(b, want, offs, np.random.default_rng(3)):
        ref = HostBatch.empty(FIELDS, hb.n, hb.dyn_caps())
        rc, fb, err = oracle.decode_batch(FIELDS, x[:in_len], offs, hb.n, ref.columns(), conds=CONDS)
        if code is not None:
            assert err == code, (name, rc, fb, err)
        assert fb <= r or (code is None and err == 0) or code == 0, (name, fb, r)
        assert ref.equal(hb, upto=min(fb, r)), name


def _caps_variants(hb):
    """Decode capacities one short on every counted column at every level."""
    caps = hb.dyn_caps()
    out = []
    for k in (ENT, NAME, ACL, WHO, REALM, TAGS, VALUE):
        c = dict(caps)
        c[k] = max(caps[k] - 1, 0)
        out.append((f"cap{k}", c))
    return out


def test_oracle_acl_tree_capacity():
    hb, want, offs = _batch(FIX["batches"][0])
    for name, caps in _caps_variants(hb):
        ref = HostBatch.empty(FIELDS, hb.n, caps)
        rc, fb, err = oracle.decode_batch(FIELDS, want, offs, hb.n, ref.columns(), conds=CONDS)
        assert err == abi.E_CAPACITY, name
        assert ref.equal(hb, upto=fb), name


def _random(n, seed):
    hb = random_batch(FIELDS, n, seed=seed, dyn_len=(0, 20), group_len=(0, 4), inner_len=(0, 3))
    rng = np.random.default_rng(seed)
    hb.arrays[GIDB][:] = rng.integers(0, 2, hb.arrays[GIDB].shape[0], dtype=np.uint8)
    hb.arrays[EOF][:] = rng.integers(0, 2, hb.arrays[EOF].shape[0], dtype=np.uint8)
    return hb


def _decoded(hb):
    """What a decode of hb's encoding holds: an absent gid as 0."""
    out = HostBatch(hb.fields, hb.n, [a.copy() if isinstance(a, np.ndarray) else
                                      (tuple(x.copy() for x in a) if isinstance(a, tuple) else a)
                                      for a in hb.arrays])
    out.arrays[GID][~hb.arrays[GIDB].astype(bool)] = 0
    return out


def test_oracle_random_roundtrip():
    hb = _random(300, 11)
    rc, want, offs = oracle.encode_batch(FIELDS, hb.columns(), hb.n, hb.xdr_total() + 64, conds=CONDS)
    assert rc == 0
    out = HostBatch.empty(FIELDS, hb.n, hb.dyn_caps())
    assert oracle.decode_batch(FIELDS, want, offs, hb.n, out.columns(), conds=CONDS) == (0, hb.n, 0)
    assert out.equal(_decoded(hb))


# ---- GPU ---------------------------------------------------------------------
@pytest.fixture(params=[(8, 32768, 16384), (8, 0, 0), (64, 0, 4096), (4, 1024, 0)],
                ids=lambda p: f"enc{p[0]}-dtile{p[1]}-img{p[2]}")
def grp_tune(request, gpu_ctx):
    """Group kernels under each production choice (tuning keys 32 / 33 / 41)."""
    gpu_ctx.tune(32, request.param[0])
    gpu_ctx.tune(33, request.param[1])
    gpu_ctx.tune(41, request.param[2])   # element-parallel encode image (0: lanes per record)
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
    assert not out[ln:].any(), "engine wrote past the stream end"
    assert ro.cpu().numpy().astype(np.uint64).tolist() == offs.tolist()
    back = DeviceBatch.empty(FIELDS, hb.n, hb.dyn_caps())
    assert gpu_ctx.decode(sch, out, ln, hb.n, back.columns(), rec_offsets=ro, framed=framed) == (0, hb.n, 0)
    assert back.to_host().equal(hb if ref is None else ref)


@pytest.mark.gpu
@pytest.mark.parametrize("b", FIX["batches"], ids=_ids)
def test_gpu_acl_tree_fixture(gpu_ctx, grp_tune, b):
    hb, want, offs = _batch(b)
    _gpu_roundtrip(gpu_ctx, hb, want, offs, b["framed"])


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2])
def test_gpu_acl_tree_errors_vs_oracle(gpu_ctx, grp_tune, seed):
    """Errors at every level: the engine's first bad record, code and the
    records before it equal the oracle's."""
    import torch
    from oncrpc4j_amd import engine
    from oncrpc4j_amd.columns import DeviceBatch
    b = FIX["batches"][0]
    hb, want, offs = _batch(b)
    sch = engine.Schema(FIELDS, CONDS)
    for name, x, in_len, _, _ in _mutations(b, want, offs, np.random.default_rng(seed)):
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
def test_gpu_acl_tree_capacity_vs_oracle(gpu_ctx, grp_tune):
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
def test_gpu_acl_tree_random_vs_oracle(gpu_ctx, grp_tune, framed):
    """A larger random batch (every level's counts, every optional mix)."""
    hb = _random(2000, 23)
    rc, want, offs = oracle.encode_batch(FIELDS, hb.columns(), hb.n, hb.xdr_total(framed) + 64, framed=framed,
                                         conds=CONDS)
    assert rc == 0
    ref = HostBatch.empty(FIELDS, hb.n, hb.dyn_caps())
    assert oracle.decode_batch(FIELDS, want, offs, hb.n, ref.columns(), framed=framed, conds=CONDS) == (0, hb.n, 0)
    _gpu_roundtrip(gpu_ctx, hb, want, offs, framed, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["pageable", "registered"])
def test_gpu_acl_tree_host_ptrs(kind):
    """XDRG_HOST_PTRS on the four-level schema (streamed through the staging
    ring, every level's element rows with their records): encode == the
    fixture, decode == the batch."""
    import torch
    from oncrpc4j_amd import engine
    from hostmem import Pageable, Registered, moved
    assert torch.cuda.is_available()
    b = FIX["batches"][1]
    hb0, want, offs = _batch(b)
    n = hb0.n
    c = engine.Context(0)
    mem = Registered() if kind == "registered" else Pageable()
    try:
        hb = moved(hb0, mem)
        sch = engine.Schema(FIELDS, CONDS)
        out = mem.array(np.zeros(len(want) + 64, np.uint8))
        ro = mem.array(np.zeros(n + 1, np.uint64))
        ln = c.encode(sch, hb.columns(), n, out, len(want) + 64, rec_offsets=ro, framed=True, host=True)
        assert out[:ln].tobytes() == want and np.array_equal(ro, offs)
        back = moved(HostBatch.empty(FIELDS, n, hb0.dyn_caps()), mem)
        assert c.decode(sch, out, ln, n, back.columns(), rec_offsets=ro, framed=True, host=True) == (0, n, 0)
        assert back.equal(hb0)
    finally:
        mem.close()
        c.close()
