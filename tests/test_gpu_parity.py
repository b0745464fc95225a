"""GPU parity: libxdrgpu.so (HIP, gfx950) against the pinned CPU oracle and the
golden fixtures.  Bit-exact for every byte and every decoded value; error
parity = same first failing record and same code as a sequential reference
decode (Xdr.java:1028-1037)."""
import zlib

import numpy as np
import pytest

import gold
import oracle
from oncrpc4j_amd import abi, engine
from oncrpc4j_amd.columns import DeviceBatch, HostBatch, aos_columns, random_batch, xdr_word_offsets

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

I, U, E, B = abi.T_INT, abi.T_UINT, abi.T_ENUM, abi.T_BOOL
H, UH, F, D = abi.T_HYPER, abi.T_UHYPER, abi.T_FLOAT, abi.T_DOUBLE
S, BY, O, STR = abi.T_SHORT, abi.T_BYTE, abi.T_OPAQUE, abi.T_STRING
SC, FX, DY = abi.K_SCALAR, abi.K_FIXED, abi.K_DYNAMIC

SCHEMAS = {
    "cfg2_8xint": [(I, SC, 0)] * 8,
    "cfg1_int_int_string": [(I, SC, 0), (I, SC, 0), (STR, DY, 0)],
    "cfg3_6xint_opaque": [(I, SC, 0)] * 6 + [(O, DY, 0)],
    "cfg4_int_string_intvec": [(I, SC, 0), (STR, DY, 0), (I, DY, 0)],
    "all_scalars": [(I, SC, 0), (U, SC, 0), (E, SC, 0), (B, SC, 0), (H, SC, 0), (UH, SC, 0),
                    (F, SC, 0), (D, SC, 0), (S, SC, 0), (BY, SC, 0)],
    "fixed_arrays": [(I, FX, 3), (H, FX, 2), (F, FX, 2), (D, FX, 1), (S, FX, 3), (BY, FX, 5),
                     (O, FX, 5), (O, FX, 8), (U, FX, 1), (O, FX, 0)],
    "dyn_vectors": [(H, DY, 0), (UH, DY, 0), (F, DY, 0), (D, DY, 0), (S, DY, 0), (BY, DY, 0),
                    (U, DY, 0), (O, DY, 0), (E, DY, 0), (STR, DY, 0)],
    "words_mixed": [(I, SC, 0), (F, SC, 0), (H, SC, 0), (D, SC, 0), (O, FX, 8), (I, FX, 2)],
    "odd_words": [(I, SC, 0)] * 3,
    "big_fixed": [(I, FX, 200), (O, FX, 37)],   # beyond the word-map limit -> record path
    # one dynamic byte field between fixed fields of every width: the payload
    # kernels decode head and tail words around it
    "head_payload_tail": [(I, SC, 0), (H, SC, 0), (O, FX, 3), (O, DY, 0), (D, SC, 0), (S, SC, 0), (I, FX, 2)],
}


# Record-path implementations (kernels_rec.hip launch_rec_phase), as tuning
# (key, value) pairs: "staged" = the defaults (key 9 = 4: sub-batches through
# an LDS tile, the output-stationary sweep decode with one-pass derived counts
# where it applies, large-record blocks on the group kernels), "staged_walk"
# the exact walk instead of derived counts (key 31 = 0, the fallback the
# derived counts rerun), "staged_lean" the record-group staged decode that
# schemas of 3-4 dynamic fields take (key 20 = 1), "group" the group kernels
# for every block (key 9 = 0).  Tests taking `rec_kernel` run under each.
REC_KERNELS = {"staged": ((9, 4),), "staged_walk": ((9, 4), (31, 0)), "staged_lean": ((9, 4), (20, 1)),
               "group": ((9, 0),)}


@pytest.fixture(params=sorted(REC_KERNELS), ids=str)
def rec_kernel(request, gpu_ctx):
    for k, v in REC_KERNELS[request.param]:
        gpu_ctx.tune(k, v)
    yield request.param
    gpu_ctx.tune(0)


# ---- helpers ----------------------------------------------------------------
def gpu_encode(ctx, fields, hb, framed=False, cap_slack=0):
    sch = engine.Schema(fields)
    db = DeviceBatch.from_host(hb)
    total = hb.xdr_total(framed)
    out = torch.zeros(total + 64, dtype=torch.uint8, device="cuda")
    offs = torch.zeros(hb.n + 1, dtype=torch.int64, device="cuda")
    ln = ctx.encode(sch, db.columns(), hb.n, out, total + cap_slack, rec_offsets=offs, framed=framed)
    assert ln == total
    assert not out[total:].any(), "engine wrote past the stream end"
    return out[:ln].cpu().numpy().tobytes(), offs.cpu().numpy().view(np.uint64)


def gpu_decode(ctx, fields, xdr, n, rec_offsets, caps, framed=False, use_offsets=True):
    sch = engine.Schema(fields)
    db = DeviceBatch.empty(fields, n, caps)
    buf = torch.from_numpy(np.frombuffer(xdr, dtype=np.uint8).copy()).cuda() if xdr else \
        torch.zeros(4, dtype=torch.uint8, device="cuda")
    ro = None
    if use_offsets and rec_offsets is not None:
        ro = torch.from_numpy(np.asarray(rec_offsets, dtype=np.uint64).view(np.int64)).cuda()
    rc, fb, err = ctx.decode(sch, buf, len(xdr), n, db.columns(), rec_offsets=ro, framed=framed,
                             raise_on_error=False)
    return rc, fb, err, db.to_host()


def oracle_decode(fields, xdr, n, rec_offsets, caps, framed=False):
    out = HostBatch.empty(fields, n, caps)
    ro = None if rec_offsets is None else np.asarray(rec_offsets, dtype=np.uint64)
    rc, fb, err = oracle.decode_batch(fields, xdr, ro, n, out.columns(), framed=framed)
    return rc, fb, err, out


# ---- golden fixtures ------------------------------------------------------------
@pytest.mark.parametrize("b", gold.load("xdrlib_vectors.json")["batches"],
                         ids=lambda b: f'{b["name"]}-{"rm" if b["framed"] else "raw"}')
def test_golden_xdrlib(gpu_ctx, rec_kernel, b):
    fields = [tuple(f) for f in b["fields"]]
    hb = gold.batch_from_records(fields, b["records"])
    xdr, offs = gpu_encode(gpu_ctx, fields, hb, b["framed"])
    assert xdr.hex() == b["xdr"]
    assert offs.tolist() == b["rec_offsets"]
    rc, fb, err, out = gpu_decode(gpu_ctx, fields, xdr, hb.n, offs, hb.dyn_caps(), b["framed"])
    assert (rc, fb, err) == (0, hb.n, 0)
    assert out.equal(hb)


@pytest.mark.parametrize("case", gold.load("kat_reference.json")["scalars"], ids=lambda c: c["name"])
def test_golden_kat(gpu_ctx, case):
    fields = [tuple(f) for f in case["fields"]]
    hb = gold.batch_from_records(fields, [case["values"]])
    xdr, offs = gpu_encode(gpu_ctx, fields, hb)
    assert xdr.hex() == case["xdr"]
    rc, fb, err, out = gpu_decode(gpu_ctx, fields, xdr, 1, offs, hb.dyn_caps())
    assert rc == 0 and out.equal(hb)


@pytest.mark.parametrize("case", gold.load("kat_reference.json")["errors"], ids=lambda c: c["name"])
def test_golden_kat_errors(gpu_ctx, case):
    fields = [tuple(f) for f in case["fields"]]
    xdr = bytes.fromhex(case["xdr"])
    rc, fb, err, _ = gpu_decode(gpu_ctx, fields, xdr, 1, [0, len(xdr)], {0: 64})
    assert (rc, fb, err) == (case["code"], 0, case["code"])


def test_jdk_nan(gpu_ctx):
    d = gold.load("kat_jdk_nan.json")
    for t, key in ((F, "float"), (D, "double")):
        fields = [(t, SC, 0)]
        hb = gold.batch_from_records(fields, [[int(c["bits"], 16)] for c in d[key]])
        xdr, _ = gpu_encode(gpu_ctx, fields, hb)
        assert xdr.hex() == "".join(c["xdr"] for c in d[key])


# ---- random batches vs the oracle ---------------------------------------------------
@pytest.mark.parametrize("framed", [False, True], ids=["raw", "rm"])
@pytest.mark.parametrize("n", [1, 7, 2049, 20000])
@pytest.mark.parametrize("name", sorted(SCHEMAS))
def test_random_parity(gpu_ctx, rec_kernel, name, n, framed):
    fields = SCHEMAS[name]
    hb = random_batch(fields, n, seed=zlib.crc32(f"{name}/{n}/{framed}".encode()), dyn_len=(0, 40))
    rc, want, want_offs = oracle.encode_batch(fields, hb.columns(), n, hb.xdr_total(framed) + 8,
                                              framed=framed)
    assert rc == 0
    xdr, offs = gpu_encode(gpu_ctx, fields, hb, framed)
    assert xdr == want
    assert np.array_equal(offs, want_offs)
    caps = hb.dyn_caps()
    g = gpu_decode(gpu_ctx, fields, xdr, n, offs, caps, framed)
    o = oracle_decode(fields, xdr, n, offs, caps, framed)
    assert g[:3] == o[:3] == (0, n, 0)
    assert g[3].equal(o[3])
    if all(k != DY for _, k, _ in fields):   # fixed-stride decode without offsets
        g2 = gpu_decode(gpu_ctx, fields, xdr, n, None, caps, framed, use_offsets=False)
        assert g2[:3] == (0, n, 0) and g2[3].equal(o[3])


AOS_EXTRA = {"float_words": [(F, SC, 0), (I, SC, 0), (O, FX, 4)] * 2,
             "one_word": [(I, SC, 0)], "wide_words": [(I, FX, 37)]}


FRAMED_KERNELS = {"lds": 1, "lean": 2}


@pytest.fixture(params=sorted(FRAMED_KERNELS))
def framed_kernel(request, gpu_ctx):
    """Record-marked streaming decode kernels (kernels_fixed.hip, tuning key
    14): the wave-local LDS transpose (records under 3 words always take it)
    or the lean kernels (wave-uniform divmod, no op table for plain int words)."""
    gpu_ctx.tune(14, FRAMED_KERNELS[request.param])
    yield request.param
    gpu_ctx.tune(0)


@pytest.mark.parametrize("framed", [False, True], ids=["raw", "rm"])
@pytest.mark.parametrize("n", [4099, 4100, 70001])
@pytest.mark.parametrize("name", ["cfg2_8xint", "words_mixed", "odd_words", "float_words", "one_word",
                                  "wide_words"])
def test_aos_layout(gpu_ctx, framed_kernel, name, n, framed):
    """Array-of-structs native records (one struct per record, fields at their
    XDR word positions): the streaming paths (raw: n*words a multiple of 4;
    record-marked: single-word types) and the word-map path otherwise."""
    fields = SCHEMAS.get(name) or AOS_EXTRA[name]
    hb = random_batch(fields, n, seed=7)
    total = hb.xdr_total(framed)
    rc, want, _ = oracle.encode_batch(fields, hb.columns(), n, total + 8, framed=framed)
    assert rc == 0
    offs = xdr_word_offsets(fields)
    rec = hb.xdr_total() // n
    # pack the SoA host batch into one AoS buffer (native little-endian values)
    aos = np.zeros((n, rec), dtype=np.uint8)
    for k, a in enumerate(hb.arrays):
        raw = np.ascontiguousarray(a).view(np.uint8).reshape(n, -1)
        aos[:, offs[k]:offs[k] + raw.shape[1]] = raw
    dev = torch.from_numpy(aos).cuda()
    sch = engine.Schema(fields)
    cols = aos_columns(fields, dev.data_ptr(), rec, offs)
    out = torch.zeros(total + 16, dtype=torch.uint8, device="cuda")
    assert gpu_ctx.encode(sch, cols, n, out, total, framed=framed) == total
    assert out[:total].cpu().numpy().tobytes() == want
    assert not out[total:].any()
    back = torch.zeros_like(dev)
    cols2 = aos_columns(fields, back.data_ptr(), rec, offs)
    gpu_ctx.decode(sch, out, total, n, cols2, framed=framed)
    o = oracle_decode(fields, want, n, None, {}, framed)[3]
    ob = np.zeros((n, rec), dtype=np.uint8)
    for k, a in enumerate(o.arrays):
        raw = np.ascontiguousarray(a).view(np.uint8).reshape(n, -1)
        ob[:, offs[k]:offs[k] + raw.shape[1]] = raw
    assert np.array_equal(back.cpu().numpy(), ob)
    if framed:   # a corrupted mark: same first bad record and code as the oracle
        bad = bytearray(want)
        r = n // 3
        bad[r * (rec + 4) + 3] ^= 0x10
        tb = torch.from_numpy(np.frombuffer(bytes(bad), dtype=np.uint8).copy()).cuda()
        rc, fb, err = gpu_ctx.decode(sch, tb, total, n, cols2, framed=True, raise_on_error=False)
        oo = oracle_decode(fields, bytes(bad), n, None, {}, True)
        assert (rc, fb, err) == oo[:3] == (abi.E_FRAME, r, abi.E_FRAME)


# ---- error parity ------------------------------------------------------------------
def _corrupt_cases(fields, hb, xdr, offs, framed):
    """(description, bytes, rec_offsets) with one defect each."""
    rng = np.random.default_rng(1)
    cases = []
    n = hb.n
    b = bytearray(xdr)
    cases.append(("truncated", bytes(b[:len(b) - 3]), offs))
    cases.append(("truncated-half", bytes(b[:len(b) // 2]), offs))
    dyn = [k for k, f in enumerate(fields) if f[1] == DY]
    if dyn:
        for val, desc in ((0xfffffffe, "negative"), (0x7ffffff0, "huge")):
            bb = bytearray(xdr)
            r = int(rng.integers(0, n))
            pos = int(offs[r]) + (4 if framed else 0)
            for k, f in enumerate(fields):
                if f[1] == DY:
                    break
                pos += 4 * (f[2] if f[1] == FX else 1)   # only int fields precede it here
            bb[pos:pos + 4] = val.to_bytes(4, "big")
            cases.append((desc, bytes(bb), offs))
    if framed:
        bb = bytearray(xdr)
        r = int(rng.integers(0, n))
        bb[int(offs[r])] ^= 0x80   # clear LAST_FRAG
        cases.append(("bad-mark", bytes(bb), offs))
    return cases


@pytest.mark.parametrize("framed", [False, True], ids=["raw", "rm"])
@pytest.mark.parametrize("name", ["cfg2_8xint", "cfg4_int_string_intvec", "cfg3_6xint_opaque",
                                  "cfg1_int_int_string"])
def test_error_parity(gpu_ctx, rec_kernel, name, framed):
    fields = SCHEMAS[name]
    n = 3000
    hb = random_batch(fields, n, seed=11, dyn_len=(0, 20))
    rc, xdr, offs = oracle.encode_batch(fields, hb.columns(), n, hb.xdr_total(framed), framed=framed)
    caps = hb.dyn_caps()
    for desc, bad, ro in _corrupt_cases(fields, hb, xdr, offs, framed):
        o = oracle_decode(fields, bad, n, ro, caps, framed)
        g = gpu_decode(gpu_ctx, fields, bad, n, ro, caps, framed)
        assert o[0] != 0, desc
        assert g[:3] == o[:3], desc
        assert g[3].equal(o[3], upto=o[1]), desc   # records before first_bad decoded
        if all(k != DY for _, k, _ in fields):
            g2 = gpu_decode(gpu_ctx, fields, bad, n, None, caps, framed, use_offsets=False)
            o2 = oracle_decode(fields, bad, n, None, caps, framed)
            assert g2[:3] == o2[:3], desc


@pytest.mark.parametrize("lean", [1, 2], ids=["lean", "sweep"])
@pytest.mark.parametrize("tile", [1024, 4096])
@pytest.mark.parametrize("framed", [False, True], ids=["raw", "rm"])
@pytest.mark.parametrize("name", ["cfg1_int_int_string", "cfg3_6xint_opaque", "cfg4_int_string_intvec",
                                  "dyn_vectors"])
def test_staged_tile_sizes(gpu_ctx, name, framed, tile, lean):
    """Staged place kernels with small LDS tiles: records whose staged bytes
    exceed the tile take the whole-block direct path, the others form
    sub-batches of every size (dyn_vectors has non-stageable vector types and
    runs the group kernels)."""
    fields = SCHEMAS[name]
    n = 2500
    hb = random_batch(fields, n, seed=zlib.crc32(f"tile/{name}/{framed}/{tile}".encode()), dyn_len=(0, 3000))
    rc, want, want_offs = oracle.encode_batch(fields, hb.columns(), n, hb.xdr_total(framed) + 8, framed=framed)
    assert rc == 0
    gpu_ctx.tune(9, 4)
    gpu_ctx.tune(12, tile)
    gpu_ctx.tune(25, tile)   # the sweep decode's own tile
    gpu_ctx.tune(13, 0)   # every block staged (no split of large-record blocks to the group kernel)
    gpu_ctx.tune(20, lean)
    try:
        xdr, offs = gpu_encode(gpu_ctx, fields, hb, framed)
        assert xdr == want
        assert np.array_equal(offs, want_offs)
        caps = hb.dyn_caps()
        g = gpu_decode(gpu_ctx, fields, xdr, n, offs, caps, framed)
        o = oracle_decode(fields, xdr, n, offs, caps, framed)
        assert g[:3] == o[:3] == (0, n, 0)
        assert g[3].equal(o[3])
    finally:
        gpu_ctx.tune(0)


def test_decode_capacity(gpu_ctx, rec_kernel):
    fields = SCHEMAS["cfg4_int_string_intvec"]
    hb = random_batch(fields, 500, seed=3, dyn_len=(1, 20))
    rc, xdr, offs = oracle.encode_batch(fields, hb.columns(), 500, hb.xdr_total())
    caps = hb.dyn_caps()
    small = dict(caps)
    small[1] = caps[1] // 2
    o = oracle_decode(fields, xdr, 500, offs, small)
    g = gpu_decode(gpu_ctx, fields, xdr, 500, offs, small)
    assert o[0] == abi.E_CAPACITY
    assert g[:3] == o[:3]


def test_encode_capacity(gpu_ctx, rec_kernel):
    for name in ("cfg2_8xint", "cfg4_int_string_intvec"):
        fields = SCHEMAS[name]
        hb = random_batch(fields, 100, seed=5, dyn_len=(1, 9))
        total = hb.xdr_total()
        sch = engine.Schema(fields)
        db = DeviceBatch.from_host(hb)
        out = torch.zeros(total, dtype=torch.uint8, device="cuda")
        with pytest.raises(engine.CapacityError):
            gpu_ctx.encode(sch, db.columns(), 100, out, total - 4)
        assert not out.any(), "nothing may be written on XDRG_E_CAPACITY"


@pytest.mark.parametrize("junk", [1, 3, 4, 8], ids=lambda j: f"junk{j}")
@pytest.mark.parametrize("name", ["cfg4_int_string_intvec", "dyn_vectors", "fixed_arrays"])
def test_decode_extents_with_unread_bytes(gpu_ctx, rec_kernel, name, junk):
    """Record extents longer than the record: the reference decodes each
    message from its own Xdr and leaves the rest unread
    (RpcMessageParserTCP.java:109-140).  junk % 4 != 0 puts the records off
    one dword grid (segment kernel: per-record path)."""
    fields = SCHEMAS[name]
    n = 1500
    hb = random_batch(fields, n, seed=junk, dyn_len=(0, 33))
    rc, xdr, offs = oracle.encode_batch(fields, hb.columns(), n, hb.xdr_total())
    rng = np.random.default_rng(junk)
    parts, ro, pos = [], [0], 0
    for r in range(n):
        rec = xdr[int(offs[r]):int(offs[r + 1])]
        extra = int(rng.integers(0, junk + 1)) if junk % 4 else junk
        parts.append(rec + bytes(rng.integers(0, 256, extra, dtype=np.uint8)))
        pos += len(rec) + extra
        ro.append(pos)
    stream = b"".join(parts)
    caps = hb.dyn_caps()
    o = oracle_decode(fields, stream, n, ro, caps)
    g = gpu_decode(gpu_ctx, fields, stream, n, ro, caps)
    assert o[:3] == (0, n, 0)
    assert g[:3] == o[:3]
    assert g[3].equal(o[3])


def test_empty_batch(gpu_ctx):
    for name in ("cfg2_8xint", "cfg4_int_string_intvec"):
        fields = SCHEMAS[name]
        hb = random_batch(fields, 0, seed=1)
        xdr, offs = gpu_encode(gpu_ctx, fields, hb)
        assert xdr == b"" and offs.tolist() == [0]
        g = gpu_decode(gpu_ctx, fields, b"", 0, [0], {})
        assert g[:3] == (0, 0, 0)


# ---- framing ------------------------------------------------------------------------
@pytest.mark.parametrize("case", gold.load("framing.json")["cases"], ids=lambda c: c["name"])
def test_frame_scan(gpu_ctx, case):
    stream = bytes.fromhex(case["stream"])
    dev = torch.from_numpy(np.frombuffer(stream, dtype=np.uint8).copy()).cuda() if stream else \
        torch.zeros(4, dtype=torch.uint8, device="cuda")
    offs = torch.zeros(17, dtype=torch.int64, device="cuda")
    k = gpu_ctx.frame_scan(dev, len(stream), offs, 16)
    assert k == case["complete"]
    assert offs[:k + 1].cpu().tolist() == case["offsets"]
    rc, want = oracle.frame_scan(stream, 16)
    assert want == case["offsets"]


# ---- BASELINE-size properties (size-independent checks) -------------------------------
@pytest.mark.slow
def test_cfg2_full_size_roundtrip(gpu_ctx):
    """configs[1]: 64 Mi records of 8 x int32: XDR == per-word byte reversal of
    the native records, and decode(encode(x)) == x bit for bit."""
    n = 64 << 20
    fields = SCHEMAS["cfg2_8xint"]
    g = torch.Generator(device="cuda").manual_seed(0x0DCAC4E5 + 2)
    nat = torch.randint(-2**31, 2**31 - 1, (n, 8), dtype=torch.int32, device="cuda", generator=g)
    sch = engine.Schema(fields)
    cols = aos_columns(fields, nat.data_ptr(), 32, xdr_word_offsets(fields))
    out = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    assert gpu_ctx.encode(sch, cols, n, out, n * 32) == n * 32
    assert torch.equal(out.view(-1, 4), nat.view(torch.uint8).view(-1, 4).flip(1))
    back = torch.empty_like(nat)
    gpu_ctx.decode(sch, out, n * 32, n, aos_columns(fields, back.data_ptr(), 32,
                                                    xdr_word_offsets(fields)))
    assert torch.equal(back, nat)
    # framed variant: every 36-byte record = mark + the same 32 bytes
    outf = torch.empty(n * 36, dtype=torch.uint8, device="cuda")
    assert gpu_ctx.encode(sch, cols, n, outf, n * 36, framed=True) == n * 36
    v = outf.view(n, 36)
    assert torch.equal(v[:, 4:], out.view(n, 32))
    mark = torch.tensor([0x80, 0, 0, 32], dtype=torch.uint8, device="cuda")
    assert torch.equal(v[:, :4], mark.expand(n, 4))


# ---- big records (blocks averaging >= 1 KiB: the group kernels) and mixed blocks
@pytest.mark.parametrize("framed", [False, True], ids=["raw", "rm"])
@pytest.mark.parametrize("name", ["cfg3_6xint_opaque", "cfg4_int_string_intvec", "cfg1_int_int_string",
                                  "head_payload_tail"])
def test_big_records(gpu_ctx, rec_kernel, name, framed):
    """Records of 1-6 KiB (every block big) and a mix of small and big blocks:
    bytes, offsets and values against the oracle; then error parity (cut
    stream, negative / huge length) and a too-small native column.  Under
    every record-path kernel."""
    fields = SCHEMAS[name]
    for n, dyn in ((3000, (1000, 6000)), (5000, (0, 2600))):
        hb = random_batch(fields, n, seed=zlib.crc32(f"big/{name}/{framed}/{n}".encode()), dyn_len=dyn)
        rc, want, want_offs = oracle.encode_batch(fields, hb.columns(), n, hb.xdr_total(framed) + 8,
                                                  framed=framed)
        assert rc == 0
        xdr, offs = gpu_encode(gpu_ctx, fields, hb, framed)
        assert xdr == want
        assert np.array_equal(offs, want_offs)
        caps = hb.dyn_caps()
        g = gpu_decode(gpu_ctx, fields, xdr, n, offs, caps, framed)
        o = oracle_decode(fields, xdr, n, offs, caps, framed)
        assert g[:3] == o[:3] == (0, n, 0)
        assert g[3].equal(o[3])
        for desc, bad, ro in _corrupt_cases(fields, hb, xdr, offs, framed):
            o = oracle_decode(fields, bad, n, ro, caps, framed)
            g = gpu_decode(gpu_ctx, fields, bad, n, ro, caps, framed)
            assert g[:3] == o[:3], desc
            assert g[3].equal(o[3], upto=o[1]), desc
        small = {k: v // 2 for k, v in caps.items()}
        o = oracle_decode(fields, xdr, n, offs, small, framed)
        g = gpu_decode(gpu_ctx, fields, xdr, n, offs, small, framed)
        assert o[0] == abi.E_CAPACITY and g[:3] == o[:3]
        assert g[3].equal(o[3], upto=o[1])


# ---- lane-per-record word kernels (kernels_fixed.hip k_words_lane_*, tuning key 16)
@pytest.mark.parametrize("lane_kernel", [2, 1, 0], ids=["lds", "lane", "wordmap"])
@pytest.mark.parametrize("framed", [False, True], ids=["raw", "rm"])
@pytest.mark.parametrize("name,fields", [
    ("ints8", [(I, SC, 0)] * 8),
    ("mixed_words", [(I, SC, 0), (F, SC, 0), (H, SC, 0), (U, FX, 3), (O, FX, 8), (E, SC, 0)]),
    ("one_word", [(U, SC, 0)]),
    ("wide", [(I, FX, 15)]),
    ("past_lane_limit", [(I, FX, 31)]),   # > 16 words: the word-map kernels
])
def test_words_lane(gpu_ctx, lane_kernel, framed, name, fields):
    """Struct-of-arrays and padded-stride columns of 4-byte words, raw and
    record-marked: bytes and values against the oracle, a cut stream and a
    corrupted mark against the oracle's first error."""
    gpu_ctx.tune(16, lane_kernel)
    try:
        n = 70001
        hb = random_batch(fields, n, seed=zlib.crc32(f"lane/{name}/{framed}".encode()), special_floats=False)
        total = hb.xdr_total(framed)
        rc, want, want_offs = oracle.encode_batch(fields, hb.columns(), n, total + 8, framed=framed)
        assert rc == 0
        xdr, _ = gpu_encode(gpu_ctx, fields, hb, framed)
        assert xdr == want
        g = gpu_decode(gpu_ctx, fields, xdr, n, None, {}, framed, use_offsets=False)
        o = oracle_decode(fields, xdr, n, None, {}, framed)
        assert g[:3] == o[:3] == (0, n, 0) and g[3].equal(o[3])
        # strided columns: every field of record i at base + 48*i (a padded struct)
        sch = engine.Schema(fields)
        rec_native = sum(abi.NATIVE_SIZE[t] * (c if k == FX else 1) for t, k, c in fields)
        stride = ((rec_native + 47) // 48) * 48
        offs = [int(x) for x in np.cumsum([0] + [abi.NATIVE_SIZE[t] * (c if k == FX else 1) for t, k, c in fields])[:-1]]
        buf = np.zeros((n, stride), dtype=np.uint8)
        expect = np.zeros((n, stride), dtype=np.uint8)
        for k, a in enumerate(hb.arrays):
            raw = np.ascontiguousarray(a).view(np.uint8).reshape(n, -1)
            buf[:, offs[k]:offs[k] + raw.shape[1]] = raw
            if fields[k][0] == F:   # encode canonicalises NaNs (Xdr.java:674-676); decode keeps those bits
                bits = np.ascontiguousarray(a).view(np.uint32).copy()
                bits[np.isnan(np.ascontiguousarray(a))] = 0x7fc00000
                raw = bits.view(np.uint8).reshape(n, -1)
            expect[:, offs[k]:offs[k] + raw.shape[1]] = raw
        dev = torch.from_numpy(buf).cuda()
        out = torch.zeros(total, dtype=torch.uint8, device="cuda")
        assert gpu_ctx.encode(sch, aos_columns(fields, dev.data_ptr(), stride, list(offs)), n, out, total,
                              framed=framed) == total
        assert out.cpu().numpy().tobytes() == want
        back = torch.zeros_like(dev)
        gpu_ctx.decode(sch, out, total, n, aos_columns(fields, back.data_ptr(), stride, list(offs)), framed=framed)
        assert torch.equal(back.cpu(), torch.from_numpy(expect))
        # first error: a cut stream (SHORT) and, framed, a corrupted mark (FRAME)
        cut = want[:len(want) - 5]
        g = gpu_decode(gpu_ctx, fields, cut, n, None, {}, framed, use_offsets=False)
        assert g[:3] == oracle_decode(fields, cut, n, None, {}, framed)[:3]
        if framed:
            bad = bytearray(want)
            bad[int(want_offs[n // 2])] ^= 0x80
            g = gpu_decode(gpu_ctx, fields, bytes(bad), n, None, {}, True, use_offsets=False)
            assert g[:3] == oracle_decode(fields, bytes(bad), n, None, {}, True)[:3] == (abi.E_FRAME, n // 2, abi.E_FRAME)
    finally:
        gpu_ctx.tune(16, 2)


@pytest.mark.parametrize("shift", [0, 1, 2, 3])
@pytest.mark.parametrize("name", ["cfg4_int_string_intvec", "cfg1_int_int_string", "dyn_vectors"])
def test_decode_packed_bytes_unaligned_base(gpu_ctx, rec_kernel, name, shift):
    """Packed byte columns (string<> / opaque<>) decoded at every base
    misalignment: the staged kernel writes each whole word of a sub-batch's
    column range once (composing the next records' bytes) and byte-stores
    only the words shared with neighbouring sub-batches.  Short (0..5 byte)
    and long strings mixed; guard bytes around the column stay untouched."""
    fields = SCHEMAS[name]
    n = 5000
    hb = random_batch(fields, n, seed=zlib.crc32(f"pack/{name}/{shift}".encode()), dyn_len=(0, 5))
    rng = np.random.default_rng(shift)
    for k, (t, kind, _) in enumerate(fields):   # every 7th record long, so sub-batches split
        if kind == DY and t in (O, STR):
            vals, offs = hb.arrays[k]
            lens = np.diff(offs.astype(np.int64))
            lens[::7] = rng.integers(6, 300, size=lens[::7].size)
            no = np.zeros(n + 1, dtype=offs.dtype)
            no[1:] = np.cumsum(lens)
            hb.arrays[k] = (rng.integers(0, 256, size=int(no[-1]), dtype=np.uint8).astype(vals.dtype), no)
    rc, want, want_offs = oracle.encode_batch(fields, hb.columns(), n, hb.xdr_total(False), framed=False)
    assert rc == 0
    caps = hb.dyn_caps()
    db = DeviceBatch.empty(fields, n, caps)
    guard = {}
    for k, (t, kind, _) in enumerate(fields):
        if kind == DY and t in (O, STR):
            tv, to = db.tensors[k]
            big = torch.full((tv.numel() + 8,), 0x5A, dtype=tv.dtype, device="cuda")
            guard[k] = big
            db.tensors[k] = (big[shift:shift + tv.numel()], to)
    buf = torch.from_numpy(np.frombuffer(want, dtype=np.uint8).copy()).cuda()
    ro = torch.from_numpy(np.asarray(want_offs, dtype=np.uint64).view(np.int64)).cuda()
    rc, fb, err = gpu_ctx.decode(engine.Schema(fields), buf, len(want), n, db.columns(), rec_offsets=ro,
                                 raise_on_error=False)
    o = oracle_decode(fields, want, n, want_offs, caps)
    assert (rc, fb, err) == o[:3] == (0, n, 0)
    for k, big in guard.items():
        g = big.cpu().numpy().view(np.uint8)
        assert (g[:shift] == 0x5A).all() and (g[shift + db.tensors[k][0].numel():] == 0x5A).all()
    assert db.to_host().equal(o[3])


@pytest.mark.parametrize("framed", [False, True], ids=["raw", "rm"])
@pytest.mark.parametrize("name", ["cfg4_int_string_intvec", "cfg1_int_int_string", "dyn_vectors", "cfg3_6xint_opaque"])
def test_resident_decode_fallback_blocks(gpu_ctx, name, framed):
    """Default decode over mixed blocks: small records, except a run of 14
    records of ~3000 bytes whose block averages >= 1 KiB per record, so that
    block goes to the group kernel while its neighbours take the staged sweep;
    a second pass plants a corrupt length word in a staged block (first-bad
    record, error code and the records before it)."""
    fields = SCHEMAS[name]
    n = 3000
    hb = random_batch(fields, n, seed=zlib.crc32(f"res/{name}/{framed}".encode()), dyn_len=(0, 24))
    rng = np.random.default_rng(7)
    for k, (t, kind, _) in enumerate(fields):
        if kind == DY and t in (O, STR):
            vals, offs = hb.arrays[k]
            lens = np.diff(offs.astype(np.int64))
            lens[1300:1314] = rng.integers(2900, 3100, size=14)
            no = np.zeros(n + 1, dtype=offs.dtype)
            no[1:] = np.cumsum(lens)
            hb.arrays[k] = (rng.integers(0, 256, size=int(no[-1]), dtype=np.uint8).astype(vals.dtype), no)
    rc, want, want_offs = oracle.encode_batch(fields, hb.columns(), n, hb.xdr_total(framed), framed=framed)
    assert rc == 0
    caps = hb.dyn_caps()
    gpu_ctx.tune(9, 4)
    try:
        g = gpu_decode(gpu_ctx, fields, want, n, want_offs, caps, framed)
        o = oracle_decode(fields, want, n, want_offs, caps, framed)
        assert g[:3] == o[:3] == (0, n, 0)
        assert g[3].equal(o[3])
        bad = bytearray(want)
        p = int(want_offs[2000]) + (4 if framed else 0) + 4 * sum(
            f[2] if f[1] == FX else 1 for f in fields[:next(i for i, f in enumerate(fields) if f[1] == DY)])
        bad[p:p + 4] = (0x7FFFFFF0).to_bytes(4, "big")   # first dynamic length word of record 2000
        g = gpu_decode(gpu_ctx, fields, bytes(bad), n, want_offs, caps, framed)
        o = oracle_decode(fields, bytes(bad), n, want_offs, caps, framed)
        assert g[:3] == o[:3] and o[1] == 2000
        assert g[3].equal(o[3], upto=2000)   # records before first_bad decoded
    finally:
        gpu_ctx.tune(0)
