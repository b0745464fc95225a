"""Extent-derived decode counts (tuning key 31, kernels_rec.hip spec_mode):
the sizes pass (or, key 31 = 2, the sweep block itself, with a decoupled
look-back for its native offsets) derives the last dynamic field's count (a vector of 4-byte
elements followed only by fixed fields) from the record extent, the sweep
place kernel checks every count word, and anything the derivation cannot
settle reruns the exact walk.  Every case is compared with the oracle (values,
first bad record, code) and with the same decode with the derivation off
(key 31 = 0): clean batches (the derivation holds), count words that disagree
with the extent (smaller: trailing bytes the reference leaves unread; larger:
"xdr stream too short"), extents with trailing bytes (whole words and odd
bytes), errors before the count word (reported by the derived pass itself),
capacity errors, records larger than the tile (the per-record path's check)
and blocks of big records (group kernel: exact rerun)."""
import zlib

import numpy as np
import pytest

import oracle
from oncrpc4j_amd import abi
from oncrpc4j_amd.columns import random_batch
from test_gpu_parity import gpu_decode, oracle_decode

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

I, U, E, F, H = abi.T_INT, abi.T_UINT, abi.T_ENUM, abi.T_FLOAT, abi.T_HYPER
STR, O = abi.T_STRING, abi.T_OPAQUE
SC, FX, DY = abi.K_SCALAR, abi.K_FIXED, abi.K_DYNAMIC

SCHEMAS = {
    "cfg4": [(I, SC, 0), (STR, DY, 0), (I, DY, 0)],
    "tail": [(I, SC, 0), (O, DY, 0), (U, DY, 0), (I, SC, 0), (H, SC, 0), (I, FX, 3)],
    "vec_only": [(E, DY, 0)],
    "hdr_floats": [(I, FX, 2), (F, DY, 0), (I, SC, 0)],
}


def _count_word_pos(fields, hb, offs, r, framed):
    """Stream offset of record r's last dynamic field's count word."""
    pos = int(offs[r]) + (4 if framed else 0)
    last = max(k for k, f in enumerate(fields) if f[1] == DY)
    for k, f in enumerate(fields[:last]):
        t, kind, c = f
        if kind == DY:
            n = int(hb.arrays[k][1][r + 1] - hb.arrays[k][1][r])
            pos += 4 + ((n + 3) & ~3 if t in (O, STR) else 4 * n)
        else:
            w = {H: 8}.get(t, 4)
            pos += (c if kind == FX else 1) * w if t not in (O,) else (c + 3) & ~3
    return pos


MODES = (1, 2, 0)   # key 31: derived counts (two passes), derived in one pass (look-back), off


def _both(ctx, fields, xdr, n, ro, caps, framed):
    """(oracle, [decode under each key-31 mode]) of the same input."""
    o = oracle_decode(fields, xdr, n, ro, caps, framed)
    gs = []
    try:
        for m in MODES:
            ctx.tune(31, m)
            gs.append(gpu_decode(ctx, fields, xdr, n, ro, caps, framed))
    finally:
        ctx.tune(31, 2)   # the default
    return o, gs, None


def _check(o, gs, _unused=None, what=""):
    upto = o[1]
    for m, g in zip(MODES, gs):
        assert g[:3] == o[:3], (what, m)
        assert g[3].equal(o[3], upto=upto), (what, m)


def _encode(fields, hb, framed):
    rc, xdr, offs = oracle.encode_batch(fields, hb.columns(), hb.n, hb.xdr_total(framed) + 8, framed=framed)
    assert rc == 0
    return xdr, np.asarray(offs, dtype=np.uint64)


@pytest.mark.parametrize("framed", [False, True], ids=["raw", "rm"])
@pytest.mark.parametrize("n", [1, 5, 3000, 20000])
@pytest.mark.parametrize("name", sorted(SCHEMAS))
def test_clean(gpu_ctx, name, n, framed):
    fields = SCHEMAS[name]
    hb = random_batch(fields, n, seed=zlib.crc32(f"spec/{name}/{n}/{framed}".encode()), dyn_len=(0, 40))
    xdr, offs = _encode(fields, hb, framed)
    o, g, g0 = _both(gpu_ctx, fields, xdr, n, offs, hb.dyn_caps(), framed)
    assert o[:3] == (0, n, 0)
    _check(o, g, g0)


@pytest.mark.parametrize("framed", [False, True], ids=["raw", "rm"])
@pytest.mark.parametrize("delta", [-1, -3, 1, 2], ids=lambda d: f"count{d:+d}")
@pytest.mark.parametrize("name", ["cfg4", "tail"])
def test_count_word_disagrees(gpu_ctx, name, delta, framed):
    """One record's count word != what its extent holds: smaller leaves whole
    trailing words the reference does not read (no error), larger is "xdr
    stream too short" at that record."""
    fields = SCHEMAS[name]
    n = 5000
    hb = random_batch(fields, n, seed=zlib.crc32(f"disagree/{name}/{delta}".encode()), dyn_len=(3, 30))
    xdr, offs = _encode(fields, hb, framed)
    b = bytearray(xdr)
    for r in (7, 2600, n - 1):
        p = _count_word_pos(fields, hb, offs, r, framed)
        c = int.from_bytes(b[p:p + 4], "big")
        b[p:p + 4] = (c + delta).to_bytes(4, "big")
    o, g, g0 = _both(gpu_ctx, fields, bytes(b), n, offs, hb.dyn_caps(), framed)
    if delta > 0:
        assert o[0] == abi.E_SHORT and o[1] == 7
    else:
        assert o[:3] == (0, n, 0)
    _check(o, g, g0, what=f"delta {delta}")


@pytest.mark.parametrize("junk", [1, 2, 4, 12], ids=lambda j: f"junk{j}")
@pytest.mark.parametrize("name", ["cfg4", "tail", "vec_only"])
def test_trailing_bytes(gpu_ctx, name, junk):
    """Extents longer than their records (RpcCall leaves the rest unread): odd
    tails cannot be a count, whole words give a count that the word refutes."""
    fields = SCHEMAS[name]
    n = 4000
    hb = random_batch(fields, n, seed=junk, dyn_len=(0, 25))
    xdr, offs = _encode(fields, hb, False)
    rng = np.random.default_rng(junk)
    parts, ro, pos = [], [0], 0
    for r in range(n):
        rec = xdr[int(offs[r]):int(offs[r + 1])]
        extra = junk if r % 97 == 5 else 0
        parts.append(rec + bytes(rng.integers(0, 256, extra, dtype=np.uint8)))
        pos += len(rec) + extra
        ro.append(pos)
    o, g, g0 = _both(gpu_ctx, fields, b"".join(parts), n, ro, hb.dyn_caps(), False)
    assert o[:3] == (0, n, 0)
    _check(o, g, g0)


@pytest.mark.parametrize("framed", [False, True], ids=["raw", "rm"])
def test_errors_before_the_count_word(gpu_ctx, framed):
    """Negative / huge string lengths and a broken mark: the derived pass
    reports them itself (no count word involved) — first bad record and code
    as the oracle, records before it decoded."""
    fields = SCHEMAS["cfg4"]
    n = 6000
    hb = random_batch(fields, n, seed=99, dyn_len=(0, 30))
    xdr, offs = _encode(fields, hb, framed)
    for r, val in ((4321, 0xfffffff0), (1234, 0x7fff0000)):
        b = bytearray(xdr)
        p = int(offs[r]) + (4 if framed else 0) + 4
        b[p:p + 4] = val.to_bytes(4, "big")
        o, g, g0 = _both(gpu_ctx, fields, bytes(b), n, offs, hb.dyn_caps(), framed)
        assert o[0] in (abi.E_CORRUPT, abi.E_SHORT) and o[1] == r
        _check(o, g, g0, what=f"record {r}")
    if framed:
        b = bytearray(xdr)
        b[int(offs[3333])] ^= 0x80
        o, g, g0 = _both(gpu_ctx, fields, bytes(b), n, offs, hb.dyn_caps(), True)
        assert (o[0], o[1]) == (abi.E_FRAME, 3333)
        _check(o, g, g0, what="mark")
    # a truncated stream: the last records' extents run past in_len
    o, g, g0 = _both(gpu_ctx, fields, xdr[:len(xdr) * 2 // 3], n, offs, hb.dyn_caps(), framed)
    assert o[0] != 0
    _check(o, g, g0, what="truncated")


def test_capacity(gpu_ctx):
    fields = SCHEMAS["cfg4"]
    n = 3000
    hb = random_batch(fields, n, seed=5, dyn_len=(1, 20))
    xdr, offs = _encode(fields, hb, False)
    for k in (1, 2):
        caps = dict(hb.dyn_caps())
        caps[k] = caps[k] * 2 // 3
        o, g, g0 = _both(gpu_ctx, fields, xdr, n, offs, caps, False)
        assert o[0] == abi.E_CAPACITY
        _check(o, g, g0, what=f"field {k}")


@pytest.mark.parametrize("delta", [0, -1, 1], ids=lambda d: f"count{d:+d}")
def test_records_beyond_the_tile(gpu_ctx, delta):
    """Small sweep tile: records larger than it take the per-record path, which
    checks the count word from HBM."""
    fields = SCHEMAS["cfg4"]
    n = 1500
    hb = random_batch(fields, n, seed=17, dyn_len=(0, 700))
    xdr, offs = _encode(fields, hb, False)
    b = bytearray(xdr)
    if delta:
        cnt = np.diff(np.asarray(hb.arrays[2][1], dtype=np.int64))
        r = int(np.argmax(cnt))   # one of the biggest records
        p = _count_word_pos(fields, hb, offs, r, False)
        c = int.from_bytes(b[p:p + 4], "big")
        b[p:p + 4] = (c + delta).to_bytes(4, "big")
    gpu_ctx.tune(25, 1024)
    gpu_ctx.tune(13, 0)
    try:
        o, g, g0 = _both(gpu_ctx, fields, bytes(b), n, offs, hb.dyn_caps(), False)
    finally:
        gpu_ctx.tune(0)
    _check(o, g, g0, what=f"delta {delta}")


def test_big_record_blocks(gpu_ctx):
    """Blocks averaging >= key 13 bytes per record go to the group kernel, which
    does not check count words: the derived pass hands the batch to the walk."""
    fields = SCHEMAS["cfg4"]
    n = 5000
    hb = random_batch(fields, n, seed=23, dyn_len=(0, 60))
    xdr, offs = _encode(fields, hb, False)
    b = bytearray(xdr)
    p = _count_word_pos(fields, hb, offs, 2100, False)
    c = int.from_bytes(b[p:p + 4], "big")
    if c:
        b[p:p + 4] = (c - 1).to_bytes(4, "big")
    gpu_ctx.tune(13, 120)
    try:
        o, g, g0 = _both(gpu_ctx, fields, bytes(b), n, offs, hb.dyn_caps(), False)
    finally:
        gpu_ctx.tune(0)
    assert o[:3] == (0, n, 0)
    _check(o, g, g0)


def test_rerun_over_many_blocks(gpu_ctx):
    """More than 1024 record blocks: the exact rerun's kernels run on a small
    grid and loop over the blocks."""
    fields = SCHEMAS["cfg4"]
    n = 1_200_000
    hb = random_batch(fields, n, seed=31, dyn_len=(1, 6))
    xdr, offs = _encode(fields, hb, False)
    b = bytearray(xdr)
    p = _count_word_pos(fields, hb, offs, n - 5, False)
    c = int.from_bytes(b[p:p + 4], "big")
    b[p:p + 4] = (c - 1).to_bytes(4, "big")   # whole trailing word: the walk decides
    o, g, g0 = _both(gpu_ctx, fields, bytes(b), n, offs, hb.dyn_caps(), False)
    assert o[:3] == (0, n, 0)
    _check(o, g, g0)
