"""rpcgen .x -> engine field tapes (oncrpc4j_amd/rpcgen.py).

Fixtures: builder-designed .x inputs under tests/golden/rpcgen/:
sensor_feed.x (constants in every literal form jrpcgen reads, an enum, a
mixed-type struct, procedures with one / three / no arguments),
lease_cache.x (an int-discriminated union with a multi-label arm and a void
default as a procedure argument), batch_types.x and list_types.x.  The tape order is checked against an
independent per-declaration xdrlib packer that walks the parsed structs the
way jrpcgen's generated xdrEncode does (jrpcgen.java:758-913: one call per
declaration, nested structs through their own xdrEncode)."""
import os
import warnings

import numpy as np
import pytest

import oracle
from oncrpc4j_amd import abi, rpcgen
from oncrpc4j_amd.columns import random_batch

with warnings.catch_warnings():
    warnings.simplefilter("ignore", DeprecationWarning)
    import xdrlib

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "rpcgen")
I, U, E, B, H, UH = abi.T_INT, abi.T_UINT, abi.T_ENUM, abi.T_BOOL, abi.T_HYPER, abi.T_UHYPER
F, D, S, BY, O, STR = abi.T_FLOAT, abi.T_DOUBLE, abi.T_SHORT, abi.T_BYTE, abi.T_OPAQUE, abi.T_STRING
SC, FX, DY = abi.K_SCALAR, abi.K_FIXED, abi.K_DYNAMIC
G, LS = abi.T_GROUP, abi.K_LIST


def spec(name):
    return rpcgen.parse_file(os.path.join(HERE, name))


FEED = 0x2000F33D
LEASE = 0x2000F33E


def test_feed_consts_and_tapes():
    s = spec("sensor_feed.x")
    assert s.value("FEED_SLOTS") == 48 and s.value("FLAG_STALE") == 0x40
    assert s.value("MODE_BITS") == 0o644
    assert s.value("EPOCH_2023_NS") == 1672531200000000000
    assert s.value("SEED_64") == 0x9E3779B97F4A7C15
    assert s.value("TAG_80") == 0x7E57AB1E00000000000F
    assert s.value("LIMIT_OCT_32") == s.value("LIMIT_HEX_32") == 2**31 - 1
    assert s.types["unit_kind"].values == {"CELSIUS": 1, "PASCAL": 2, "VOLT": 3}
    assert s.fields("reading") == [(U, SC, 0), (E, SC, 0), (H, SC, 0), (D, SC, 0), (F, FX, 2)]
    procs = s.procedures()
    assert {k: p.name for k, p in procs.items()} == {(FEED, 3, 1): "LATEST", (FEED, 3, 2): "WINDOW",
                                                     (FEED, 3, 3): "FLUSH"}
    assert s.args_fields(FEED, 3, 1) == [(U, SC, 0)]
    assert s.result_fields(FEED, 3, 1) == s.fields("reading")
    assert s.args_fields(FEED, 3, 2) == [(U, SC, 0), (H, SC, 0), (H, SC, 0)]   # WINDOW(unsigned, hyper, hyper)
    assert s.result_fields(FEED, 3, 2) == [(H, SC, 0)]
    assert s.args_fields(FEED, 3, 3) == [] and s.result_fields(FEED, 3, 3) == []   # void FLUSH(void)


def test_lease_union_is_not_one_tape():
    s = spec("lease_cache.x")
    assert s.fields("lease_key") == [(UH, SC, 0), (STR, DY, 0)]
    assert s.args_fields(LEASE, 1, 1) == [(UH, SC, 0), (STR, DY, 0), (U, SC, 0)]   # ACQUIRE(lease_key, unsigned)
    with pytest.raises(rpcgen.NotBatchable, match="union lease_state"):
        s.fields("lease_state")
    with pytest.raises(rpcgen.NotBatchable):
        s.args_fields(LEASE, 1, 2)                                 # RELEASE(lease_key, lease_state)
    with pytest.raises(rpcgen.NotBatchable):
        s.result_fields(LEASE, 1, 1)                               # lease_state ACQUIRE
    u = s.types["lease_state"]
    assert u.disc.name == "code" and u.disc.type == "int"
    assert [(v, d.kind, d.type) for v, d in u.arms] == [([0], "dynamic", "opaque"),
                                                        ([1, 70], "scalar", ("unsigned", U))]
    assert u.default.kind == "void"
    assert s.result_fields(LEASE, 1, 2) == []                       # void RELEASE


FATTR = [(E, SC, 0), (U, SC, 0), (U, SC, 0), (H, SC, 0), (UH, SC, 0), (U, SC, 0), (U, SC, 0),
         (U, SC, 0), (U, SC, 0), (B, SC, 0)]
DIROP = [(O, FX, 32), (STR, DY, 0), (U, DY, 0), (BY, FX, 3), (S, DY, 0), (F, FX, 2), (D, SC, 0), (O, DY, 0)]


def test_batch_types_tapes():
    s = spec("batch_types.x")
    assert s.fields("fattr") == FATTR
    assert s.fields("dirop_args") == DIROP
    assert s.args_fields(400123, 1, 0) == [] and s.result_fields(400123, 1, 0) == []
    assert s.args_fields(400123, 1, 1) == [(O, FX, 32)]
    assert s.result_fields(400123, 1, 4) == FATTR
    assert s.args_fields(400123, 1, 5) == [(O, FX, 32), (U, SC, 0)]
    assert s.result_fields(400123, 1, 5) == [(STR, DY, 0)]
    # a list node (last declaration `optional_next *next`) and an array of
    # structs are repeated groups (include/xdrg.h)
    assert s.fields("optional_next") == [(I, SC, 0), (G, LS, 0, 1), (I, SC, 0)]
    assert s.fields("with_array_of_structs") == [(G, DY, 0, 2), (U, SC, 0), (U, SC, 0)]


def test_syntax_errors():
    with pytest.raises(rpcgen.XdrSyntaxError):
        rpcgen.parse("struct x { int a }")
    with pytest.raises(rpcgen.XdrSyntaxError):
        rpcgen.parse("struct x { undefined_t a; };").fields("x")


# ---- tape order == jrpcgen's per-declaration encode order --------------------------
def _pack_decl(s, p, decl, vals):
    """Pack one declaration the way its generated xdrEncode call would."""
    t, kind = decl.type, decl.kind
    if t == "opaque":
        v = vals.pop(0)
        (p.pack_fopaque(len(v), v) if kind == rpcgen.FIXED else p.pack_opaque(v))
        return
    if t == "string":
        p.pack_string(vals.pop(0))
        return
    base = None
    if isinstance(t, tuple):
        base = t[1]
    elif t in rpcgen.BASE:
        base = rpcgen.BASE[t]
    elif isinstance(s.types.get(t), rpcgen.Enum):
        base = E
    if base is None:
        d = s.types[t]
        if isinstance(d, rpcgen.Struct):
            for sub in d.decls:
                _pack_decl(s, p, sub, vals)
            return
        if kind == rpcgen.SCALAR:    # typedef
            _pack_decl(s, p, rpcgen.Decl(decl.name, d.type, d.kind, d.size), vals)
            return
        base = s._elem(t, "test")
    one = {I: p.pack_int, E: p.pack_int, B: p.pack_int, S: p.pack_int, BY: p.pack_int, U: p.pack_uint,
           H: p.pack_hyper, UH: p.pack_uhyper, F: p.pack_float, D: p.pack_double}[base]
    v = vals.pop(0)
    if kind == rpcgen.SCALAR:
        one(v)
    elif kind == rpcgen.FIXED:
        for x in v:
            one(x)
    else:
        p.pack_array(list(v), one)


def _record_values(fields, hb, i):
    vals = []
    for k, (t, kind, c) in enumerate(fields):
        v = hb.record(i, k)
        if t in (O, STR):
            vals.append(bytes(np.asarray(v, dtype=np.uint8)))
        elif kind == SC:
            vals.append(float(v) if t in (F, D) else int(v))
        else:
            vals.append([float(x) if t in (F, D) else int(x) for x in v])
    return vals


@pytest.mark.parametrize("type_name", ["fattr", "dirop_args"])
def test_tape_matches_declaration_order(type_name):
    s = spec("batch_types.x")
    fields = s.fields(type_name)
    n = 64
    hb = random_batch(fields, n, seed=3, dyn_len=(0, 9), special_floats=False)
    if type_name == "fattr":   # bool / enum fields take valid values
        hb.arrays[9][:] = hb.arrays[9] & 1
    rc, xdr, offs = oracle.encode_batch(fields, hb.columns(), n, hb.xdr_total() + 8)
    assert rc == 0
    for i in range(n):
        p = xdrlib.Packer()
        vals = _record_values(fields, hb, i)
        for decl in s.types[type_name].decls:
            _pack_decl(s, p, decl, vals)
        assert not vals
        assert xdr[offs[i]:offs[i + 1]] == p.get_buffer(), f"record {i}"


# ---- GPU: a call batch decoded with the tape of its procedure ----------------------
@pytest.mark.gpu
def test_feed_calls_decode_with_generated_tape(gpu_ctx):
    import torch
    from oncrpc4j_amd import rpc
    s = spec("sensor_feed.x")
    rng = np.random.default_rng(117)
    n = 4000
    sensor = rng.integers(0, 2**32, n, dtype=np.uint32)
    a = rng.integers(-2**63, 2**63, n, dtype=np.int64)
    b = rng.integers(-2**63, 2**63, n, dtype=np.int64)
    stream, offs = b"", [0]
    for i in range(n):
        p = xdrlib.Packer()
        for v in (i, rpc.CALL, rpc.RPCVERS):
            p.pack_int(v)
        for v in (FEED, 3, 2):
            p.pack_uint(v)
        p.pack_int(rpc.AUTH_NONE)
        p.pack_opaque(b"")
        p.pack_int(rpc.AUTH_NONE)
        p.pack_opaque(b"")
        p.pack_uint(int(sensor[i]))
        p.pack_hyper(int(a[i]))
        p.pack_hyper(int(b[i]))
        m = p.get_buffer()
        stream += (len(m) | 0x80000000).to_bytes(4, "big") + m
        offs.append(len(stream))
    dev = torch.from_numpy(np.frombuffer(stream, dtype=np.uint8).copy()).cuda()
    ro = torch.tensor(offs, dtype=torch.int64, device="cuda")
    dec = rpc.CallDecoder(gpu_ctx)
    hdr, st = dec.decode_headers(dev, len(stream), n, ro)
    assert st == (0, n, 0)
    (key, idx), = rpc.CallDecoder.group_by_procedure(hdr).items()
    assert (key[0] & 0xffffffff, key[1], key[2], key[3]) == (FEED, 3, 2, rpc.AUTH_NONE) and idx.numel() == n
    args = s.args_fields(FEED, 3, 2)
    batch, st = dec.decode(rpc.AUTH_NONE, args, dev, len(stream), n, ro, {7: 16, 9: 16})
    assert st == (0, n, 0)
    hb = batch.to_host()
    assert np.array_equal(hb.arrays[10].view(np.uint32), sensor)
    assert np.array_equal(hb.arrays[11], a) and np.array_equal(hb.arrays[12], b)


# ---- conditional tapes: unions and optional data (Spec.tape) -------------------------
def _walk(s, t, vals, emit, p):
    """Consume one value per tape field of type t (in tape order) and pack the
    ones the generated xdrEncode would write: a union packs its discriminant
    and the matching arm / default arm (jrpcgen.java:1240-1340), optional
    data packs a bool and the value if true (INDIRECTION)."""
    d = s.types.get(t)
    if isinstance(d, rpcgen.Union):
        disc = vals[0]
        _walk_decl(s, d.disc, vals, emit, p)
        hit = False
        for labels, arm in d.arms:
            m = disc in [s.value(v) for v in labels]
            hit |= m
            _walk_decl(s, arm, vals, emit and m, p)
        if d.default is not None:
            _walk_decl(s, d.default, vals, emit and not hit, p)
        return
    if isinstance(d, rpcgen.Struct):
        for sub in d.decls:
            _walk_decl(s, sub, vals, emit, p)
        return
    _walk_decl(s, rpcgen.Decl("x", t, rpcgen.SCALAR), vals, emit, p)


class _Null:
    def __getattr__(self, name):
        return lambda *a, **k: None


def _walk_decl(s, decl, vals, emit, p):
    if decl.kind == rpcgen.VOID:
        return
    if decl.kind == rpcgen.OPTIONAL:
        present = vals[0] != 0
        v = vals.pop(0)
        (p if emit else _Null()).pack_bool(bool(v))
        _walk(s, decl.type, vals, emit and present, p)
        return
    t = decl.type
    if isinstance(t, str) and isinstance(s.types.get(t), (rpcgen.Union, rpcgen.Struct)) \
            and decl.kind == rpcgen.SCALAR:
        _walk(s, t, vals, emit, p)
        return
    if isinstance(t, str) and isinstance(s.types.get(t), rpcgen.Decl) and decl.kind == rpcgen.SCALAR:
        td = s.types[t]
        _walk_decl(s, rpcgen.Decl(decl.name, td.type, td.kind, td.size), vals, emit, p)
        return
    _pack_decl(s, p if emit else _Null(), decl, vals)


def _cond_batch(fields, conds, n, seed):
    hb = random_batch(fields, n, seed=seed, dyn_len=(0, 9), special_floats=False)
    rng = np.random.default_rng(seed)
    for k, (t, kind, c) in enumerate(fields):
        if t == B:
            hb.arrays[k][:] = rng.integers(0, 2, n, dtype=np.uint8)
        elif t == E and kind == SC:   # enums / int discriminants take their case values mostly
            hb.arrays[k][:] = rng.choice(np.array([0, 1, 2, 5, 9], np.int32), n)
    for _, d, _, _ in conds:
        if fields[d][0] == I:
            hb.arrays[d][:] = rng.choice(np.array([0, 0, 1, 70], np.int32), n)
    return hb


@pytest.mark.parametrize("type_name", ["lookup_res", "entry", "kind_res", "listing"])
def test_conditional_tape_matches_generated_encode(type_name):
    s = spec("batch_types.x")
    with pytest.raises(rpcgen.NotBatchable):
        s.fields(type_name)
    fields, conds = s.tape(type_name)
    n = 200
    hb = _cond_batch(fields, conds, n, seed=5)
    rc, xdr, offs = oracle.encode_batch(fields, hb.columns(), n, hb.xdr_total() + 8, conds=conds)
    assert rc == 0
    for i in range(n):
        p = xdrlib.Packer()
        vals = _record_values(fields, hb, i)
        _walk(s, type_name, vals, True, p)
        assert not vals
        assert xdr[offs[i]:offs[i + 1]] == p.get_buffer(), f"record {i}"


def test_conditional_tape_shapes():
    s = spec("batch_types.x")
    f, c = s.tape("lookup_res")
    assert f == [(I, SC, 0)] + FATTR and c == [(k, 0, False, [0]) for k in range(1, 11)]
    f, c = s.tape("kind_res")
    # kind, size (REG|LNK), entry{id, name, bool, seconds, useconds} (DIR), why (default)
    assert f == [(E, SC, 0), (H, SC, 0), (U, SC, 0), (STR, DY, 0), (B, SC, 0), (U, SC, 0), (U, SC, 0),
                 (STR, DY, 0)]
    assert c == [(1, 0, False, [1, 5]), (2, 0, False, [2]), (3, 0, False, [2]), (4, 0, False, [2]),
                 (5, 4, True, [0]), (6, 4, True, [0]), (7, 0, True, [1, 5, 2])]
    f, c = s.args_tape(400123, 1, 7)           # LIST(fhandle, kind_res): arguments back to back
    assert f[0] == (O, FX, 32) and c[0] == (2, 1, False, [1, 5])
    f, c = s.tape("optional_next")           # a list node: a repeated group, no conditions
    assert f == [(I, SC, 0), (G, LS, 0, 1), (I, SC, 0)] and c == []


def test_lease_release_tape():
    """RELEASE(lease_key, lease_state): an int union argument; the two-label
    arm carries both case values, the void default adds no field."""
    s = spec("lease_cache.x")
    f, c = s.args_tape(LEASE, 1, 2)
    assert f == [(UH, SC, 0), (STR, DY, 0), (I, SC, 0), (O, DY, 0), (U, SC, 0)]
    assert c == [(3, 2, False, [0]), (4, 2, False, [1, 70])]


@pytest.mark.gpu
def test_gpu_lease_release_args(gpu_ctx):
    """RELEASE(lease_key, lease_state) argument batches through the engine
    with the conditional tape, checked against xdrlib packing of the
    generated order."""
    import torch
    from oncrpc4j_amd import engine
    from oncrpc4j_amd.columns import DeviceBatch, HostBatch
    s = spec("lease_cache.x")
    fields, conds = s.args_tape(LEASE, 1, 2)
    n = 5000
    hb = _cond_batch(fields, conds, n, seed=118)
    want = b""
    offs = [0]
    for i in range(n):
        p = xdrlib.Packer()
        vals = _record_values(fields, hb, i)
        _walk(s, "lease_key", vals, True, p)
        _walk(s, "lease_state", vals, True, p)
        want += p.get_buffer()
        offs.append(len(want))
    sch = engine.Schema(fields, conds)
    db = DeviceBatch.from_host(hb)
    out = torch.zeros(hb.xdr_total(), dtype=torch.uint8, device="cuda")
    ro = torch.zeros(n + 1, dtype=torch.int64, device="cuda")
    ln = gpu_ctx.encode(sch, db.columns(), n, out, hb.xdr_total(), rec_offsets=ro)
    assert out[:ln].cpu().numpy().tobytes() == want
    assert ro.cpu().tolist() == offs
    back = DeviceBatch.empty(fields, n, hb.dyn_caps())
    rc, fb, err = gpu_ctx.decode(sch, out, ln, n, back.columns(), rec_offsets=ro)
    assert (rc, fb, err) == (0, n, 0)
    ref = HostBatch.empty(fields, n, hb.dyn_caps())
    assert oracle.decode_batch(fields, want, np.array(offs, np.uint64), n, ref.columns(),
                               conds=conds) == (0, n, 0)
    assert back.to_host().equal(ref)


# ---- repeated groups: arrays of structs and recursive lists ---------------------------
MAPPING = [(U, SC, 0)] * 4
DIRENT = [(UH, SC, 0), (STR, DY, 0), (UH, SC, 0)]
LIST_TAPES = {
    "dump_res": [(G, LS, 0, 4)] + MAPPING,
    "dir_list": [(G, LS, 0, 3)] + DIRENT + [(B, SC, 0)],
    "readdir_ok": [(O, FX, 8), (G, LS, 0, 3)] + DIRENT + [(B, SC, 0)],
    "tagged": [(I, SC, 0), (G, DY, 0, 2), (U, SC, 0), (U, SC, 0), (G, FX, 2, 2), (U, SC, 0), (U, SC, 0),
               (STR, DY, 0)],
    # `map_node first` (not a pointer): its fields, then its `next` chain
    "chain_head": [(I, SC, 0)] + MAPPING + [(G, LS, 0, 4)] + MAPPING,
}


def test_group_tapes():
    s = spec("list_types.x")
    for t, want in LIST_TAPES.items():
        assert s.fields(t) == want, t
    assert s.result_fields(400124, 1, 4) == LIST_TAPES["dump_res"]        # DUMP
    assert s.args_fields(400124, 1, 16) == LIST_TAPES["dir_list"]         # READDIR(dir_list)
    bad = rpcgen.parse("struct u { int a; }; union v switch (int d) { case 1: int x; default: void; };"
                       "struct w { v items<>; }; struct n { int a; n *next; int b; };")
    with pytest.raises(rpcgen.NotBatchable):
        bad.fields("w")                      # union elements: no one-level group
    with pytest.raises(rpcgen.NotBatchable, match="contains itself"):
        bad.fields("n")                      # recursion that is not the last declaration


def _pack_tape(p, fields, hb, i):
    """xdrlib, driven by the tape: a group packs its count (dynamic) / TRUE
    before each element and FALSE after (list) and each element's members."""
    def one(k, row):
        t, kind = fields[k][0], fields[k][1]
        a = hb.arrays[k]
        if kind == DY:
            vals, offs = a
            v = vals[int(offs[row]):int(offs[row + 1])]
            if t in (O, STR):
                p.pack_opaque(bytes(np.asarray(v, np.uint8)))
            else:
                p.pack_array([int(x) for x in v], p.pack_int if t != U else p.pack_uint)
            return
        if t == O:
            p.pack_fopaque(fields[k][2], bytes(np.asarray(a[row], np.uint8)))
            return
        pk = {I: p.pack_int, U: p.pack_uint, B: p.pack_bool, H: p.pack_hyper, UH: p.pack_uhyper}[t]
        pk(int(a[row]))
    k = 0
    while k < len(fields):
        f = fields[k]
        if f[0] != G:
            one(k, i)
            k += 1
            continue
        e0, e1 = (i * f[2], (i + 1) * f[2]) if f[1] == FX else (int(hb.arrays[k][i]), int(hb.arrays[k][i + 1]))
        if f[1] == DY:
            p.pack_uint(e1 - e0)
        for e in range(e0, e1):
            if f[1] == LS:
                p.pack_bool(True)
            for j in range(1, f[3] + 1):
                one(k + j, e)
        if f[1] == LS:
            p.pack_bool(False)
        k += 1 + f[3]


def _group_batch(fields, n, seed):
    hb = random_batch(fields, n, seed=seed, dyn_len=(0, 11), group_len=(0, 7), special_floats=False)
    for k, f in enumerate(fields):
        if f[0] == B:
            hb.arrays[k] = (hb.arrays[k] != 0).astype(np.uint8)
    return hb


@pytest.mark.parametrize("type_name", list(LIST_TAPES))
def test_group_tape_matches_xdrlib(type_name):
    fields = LIST_TAPES[type_name]
    n = 300
    hb = _group_batch(fields, n, seed=len(type_name))
    rc, xdr, offs = oracle.encode_batch(fields, hb.columns(), n, hb.xdr_total())
    assert rc == 0
    for i in range(n):
        p = xdrlib.Packer()
        _pack_tape(p, fields, hb, i)
        assert xdr[offs[i]:offs[i + 1]] == p.get_buffer(), f"record {i}"


@pytest.mark.gpu
def test_gpu_portmap_dump_and_readdir(gpu_ctx):
    """DUMP reply bodies (mapping lists) encoded on the GPU with the generated
    tape equal xdrlib's; READDIR(dir_list) arguments decode like the oracle."""
    import torch
    from oncrpc4j_amd import engine
    from oncrpc4j_amd.columns import DeviceBatch, HostBatch
    s = spec("list_types.x")
    for fields, n in ((s.result_fields(400124, 1, 4), 20000), (s.args_fields(400124, 1, 16), 8000)):
        hb = _group_batch(fields, n, seed=n)
        want, offs = b"", [0]
        for i in range(n):
            p = xdrlib.Packer()
            _pack_tape(p, fields, hb, i)
            want += p.get_buffer()
            offs.append(len(want))
        sch = engine.Schema(fields)
        db = DeviceBatch.from_host(hb)
        out = torch.zeros(len(want), dtype=torch.uint8, device="cuda")
        ro = torch.zeros(n + 1, dtype=torch.int64, device="cuda")
        ln = gpu_ctx.encode(sch, db.columns(), n, out, len(want), rec_offsets=ro)
        assert out[:ln].cpu().numpy().tobytes() == want
        assert ro.cpu().tolist() == offs
        back = DeviceBatch.empty(fields, n, hb.dyn_caps())
        assert gpu_ctx.decode(sch, out, ln, n, back.columns(), rec_offsets=ro) == (0, n, 0)
        ref = HostBatch.empty(fields, n, hb.dyn_caps())
        assert oracle.decode_batch(fields, want, np.array(offs, np.uint64), n, ref.columns()) == (0, n, 0)
        assert back.to_host().equal(ref) and ref.equal(hb)
