"""rpcgen .x -> engine field tapes (oncrpc4j_amd/rpcgen.py).

Fixtures: the reference's rpcgen test inputs (oncrpc4j-rpcgen/src/test/xdr/
Calculator.x, BlobStore.x — data files the reference's own tests hold) and
tests/golden/rpcgen/batch_types.x.  The tape order is checked against an
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


def spec(name):
    return rpcgen.parse_file(os.path.join(HERE, name))


def test_calculator_consts_and_tapes():
    s = spec("Calculator.x")
    assert s.value("PLAIN_ZERO") == 0 and s.value("HEX_ZERO") == 0
    assert s.value("SMALL_CONST") == 0xFF00
    assert s.value("LARGE_CONST") == 0xFFF000000000
    assert s.value("HUGE_CONST") == 0xFFF000000000000000000
    assert s.value("UNSIGNED_LONG_HEX_CONST") == s.value("UNSIGNED_LONG_OCT_CONST") == \
        s.value("UNSIGNED_LONG_DEC_CONST") == 2**64 - 1
    assert s.value("UNSIGNED_INT_HEX_CONST") == s.value("UNSIGNED_INT_OCT_CONST") == 2**32 - 1
    assert s.fields("CalculationResult") == [(H, SC, 0), (UH, SC, 0), (UH, SC, 0)]
    procs = s.procedures()
    assert {k: p.name for k, p in procs.items()} == {(117, 1, 1): "add", (117, 1, 2): "addSimple"}
    assert s.args_fields(117, 1, 1) == [(H, SC, 0), (H, SC, 0)]   # add(hyper, hyper)
    assert s.result_fields(117, 1, 1) == s.fields("CalculationResult")
    assert s.result_fields(117, 1, 2) == [(H, SC, 0)]


def test_blobstore_union_is_not_one_tape():
    s = spec("BlobStore.x")
    assert s.fields("Key") == [(O, DY, 0)]
    assert s.args_fields(118, 1, 2) == [(O, DY, 0)]                 # get(Key)
    with pytest.raises(rpcgen.NotBatchable, match="union Value"):
        s.fields("Value")
    with pytest.raises(rpcgen.NotBatchable):
        s.args_fields(118, 1, 1)                                    # put(Key, Value)
    u = s.types["Value"]
    assert u.disc.name == "notNull" and u.disc.type == "bool"
    assert [(v, d.kind, d.type) for v, d in u.arms] == [(["TRUE"], "dynamic", "opaque"), (["FALSE"], "void", "void")]
    assert s.result_fields(118, 1, 1) == []                          # void put


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
    with pytest.raises(rpcgen.NotBatchable, match="optional"):
        s.fields("optional_next")
    with pytest.raises(rpcgen.NotBatchable, match="array"):
        s.fields("with_array_of_structs")


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
def test_calculator_calls_decode_with_generated_tape(gpu_ctx):
    import torch
    from oncrpc4j_amd import rpc
    s = spec("Calculator.x")
    rng = np.random.default_rng(117)
    n = 4000
    a = rng.integers(-2**63, 2**63, n, dtype=np.int64)
    b = rng.integers(-2**63, 2**63, n, dtype=np.int64)
    stream, offs = b"", [0]
    for i in range(n):
        p = xdrlib.Packer()
        for v in (i, rpc.CALL, rpc.RPCVERS, 117, 1, 1, rpc.AUTH_NONE):
            p.pack_int(v)
        p.pack_opaque(b"")
        p.pack_int(rpc.AUTH_NONE)
        p.pack_opaque(b"")
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
    assert key == (117, 1, 1, rpc.AUTH_NONE) and idx.numel() == n
    args = s.args_fields(*key[:3])
    batch, st = dec.decode(rpc.AUTH_NONE, args, dev, len(stream), n, ro, {7: 16, 9: 16})
    assert st == (0, n, 0)
    hb = batch.to_host()
    assert np.array_equal(hb.arrays[10], a) and np.array_equal(hb.arrays[11], b)
