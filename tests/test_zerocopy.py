"""Zero-copy payloads: a payload field encoded by
reference (xdrEncodeFileChunk / xdrEncodeShallowByteBuffer, Xdr.java:839-866,
978-988, sent as separate writable messages, :579-597 and
GrizzlyRpcTransport.sendRawTCP :130-168) and decoded as a slice of the stream
(xdrDecodeByteBuffer, :423-439).

The contract the reference's own tests pin (ctest/xdr/XdrTest.java:743-790,
testMergeFileChunkOnAsBuffer / testOpaqueAndFileChunkCompatibility): the
message assembled from the buffer, the chunk and its zero padding equals the
dynamic-opaque encoding of the same bytes.  Checked for the oracle on the
CPU and for the HIP engine on the GPU, whose payload column is passed as a
NULL data pointer: the device never reads it."""
import numpy as np
import pytest

import oracle
from oncrpc4j_amd import abi
from oncrpc4j_amd.columns import HostBatch, random_batch

I, B, O, STR = abi.T_INT, abi.T_BOOL, abi.T_OPAQUE, abi.T_STRING
SC, DY = abi.K_SCALAR, abi.K_DYNAMIC

NFS_WRITE = [(I, SC, 0)] * 6 + [(O, DY, 0)]                       # config 3 shape
READ_RES = [(I, SC, 0), (B, SC, 0), (I, SC, 0), (STR, DY, 0), (O, DY, 0), (I, SC, 0)]
READ_CONDS = [(1, 0, False, [0]), (2, 0, False, [0]), (3, 0, False, [0]), (4, 0, False, [0])]


def payload_of(hb, k, i):
    vals, offs = hb.arrays[k]
    return vals[int(offs[i]):int(offs[i + 1])].tobytes()


def assemble(buf, offs, splice, hb, field):
    """The messages a sender writes: buffer head, payload, zero pad, buffer tail."""
    out = []
    for i in range(hb.n):
        a, b, s = int(offs[i]), int(offs[i + 1]), int(splice[i])
        if s == (1 << 64) - 1:
            out.append(buf[a:b])
            continue
        p = payload_of(hb, field, i)
        out.append(buf[a:s] + p + bytes((4 - (len(p) & 3)) & 3) + buf[s:b])
    return b"".join(out)


def _batch(fields, n, seed, dyn_len):
    hb = random_batch(fields, n, seed=seed, dyn_len=dyn_len)
    if fields is READ_RES:
        rng = np.random.default_rng(seed)
        hb.arrays[0][:] = rng.choice(np.array([0, 0, 0, 5], np.int32), n)
        hb.arrays[1][:] = rng.integers(0, 2, n, dtype=np.uint8)
    return hb


CASES = [("nfs_write", NFS_WRITE, None, 6), ("read_res", READ_RES, READ_CONDS, 4)]


# ---- oracle (CPU) -------------------------------------------------------------------------
def test_oracle_file_chunk_matches_opaque_reference_test():
    """XdrTest.testOpaqueAndFileChunkCompatibility (:764-790): int 42 + a
    64 KiB + 3 chunk merges into the dynamic-opaque bytes (1 pad byte)."""
    fields = [(I, SC, 0), (O, DY, 0)]
    data = np.random.default_rng(0).integers(0, 256, 64 * 1024 + 3, dtype=np.uint8)
    hb = HostBatch(fields, 1, [np.array([42], np.int32),
                               (data, np.array([0, data.size], np.uint64))])
    cap = hb.xdr_total()
    rc, deep, offs = oracle.encode_batch(fields, hb.columns(), 1, cap)
    rc2, buf, offs2, splice = oracle.encode_batch_shallow(fields, hb.columns(), 1, cap, 1)
    assert rc == rc2 == 0
    assert buf == bytes.fromhex("0000002a" "00010003") and splice.tolist() == [8]
    assert assemble(buf, offs2, splice, hb, 1) == deep
    assert deep[8:8 + data.size] == data.tobytes() and deep[-1:] == b"\0"   # testMergeFileChunkOnAsBuffer


@pytest.mark.parametrize("name,fields,conds,field", CASES, ids=[c[0] for c in CASES])
@pytest.mark.parametrize("framed", [False, True], ids=["raw", "rm"])
def test_oracle_shallow_and_view(name, fields, conds, field, framed):
    n = 300
    hb = _batch(fields, n, 3, (0, 70))
    cap = hb.xdr_total(framed)
    rc, deep, deep_offs = oracle.encode_batch(fields, hb.columns(), n, cap, framed=framed, conds=conds)
    assert rc == 0
    rc, buf, offs, splice = oracle.encode_batch_shallow(fields, hb.columns(), n, cap, field,
                                                        framed=framed, conds=conds)
    assert rc == 0
    assert assemble(buf, offs, splice, hb, field) == deep
    # view decode of the full stream: slices point at the payloads, nothing copied
    out = HostBatch.empty(fields, n, hb.dyn_caps())
    rc, fb, err, pos = oracle.decode_batch_view(fields, deep, deep_offs, n, out.columns(), field,
                                                framed=framed, conds=conds)
    assert (rc, fb, err) == (0, n, 0)
    ref = HostBatch.empty(fields, n, hb.dyn_caps())
    assert oracle.decode_batch(fields, deep, deep_offs, n, ref.columns(), framed=framed,
                               conds=conds) == (0, n, 0)
    lens = np.diff(out.arrays[field][1].astype(np.int64))
    assert np.array_equal(out.arrays[field][1], ref.arrays[field][1])
    for i in range(n):
        if pos[i] == (1 << 64) - 1:
            assert lens[i] == 0
            continue
        assert deep[int(pos[i]):int(pos[i]) + int(lens[i])] == payload_of(ref, field, i)
    for k in range(len(fields)):
        if k != field:
            assert np.array_equal(np.asarray(out.arrays[k][0] if fields[k][1] == DY else out.arrays[k]),
                                  np.asarray(ref.arrays[k][0] if fields[k][1] == DY else ref.arrays[k]))


def test_oracle_byref_field_must_be_bytes():
    fields = [(I, SC, 0), (I, DY, 0)]
    hb = random_batch(fields, 4, seed=1)
    rc, *_ = oracle.encode_batch_shallow(fields, hb.columns(), 4, hb.xdr_total(), 1)
    assert rc == oracle.E_INVAL


# ---- the HIP engine (GPU) -----------------------------------------------------------------
def _dev():
    torch = pytest.importorskip("torch")
    from oncrpc4j_amd import engine
    from oncrpc4j_amd.columns import DeviceBatch
    return torch, engine, DeviceBatch


@pytest.mark.gpu
@pytest.mark.parametrize("name,fields,conds,field", CASES, ids=[c[0] for c in CASES])
@pytest.mark.parametrize("framed", [False, True], ids=["raw", "rm"])
def test_gpu_shallow_encode_vs_oracle(gpu_ctx, name, fields, conds, field, framed):
    torch, engine, DeviceBatch = _dev()
    n = 20000
    hb = _batch(fields, n, 5, (0, 300))
    cap = hb.xdr_total(framed)
    rc, want, want_offs, want_splice = oracle.encode_batch_shallow(fields, hb.columns(), n, cap,
                                                                   field, framed=framed, conds=conds)
    assert rc == 0
    sch = engine.Schema(fields, conds)
    db = DeviceBatch.from_host(hb)
    cols = db.columns()
    cols[field].data = None            # the payload is never read by the device
    out = torch.zeros(cap + 64, dtype=torch.uint8, device="cuda")
    offs = torch.zeros(n + 1, dtype=torch.int64, device="cuda")
    splice = torch.zeros(n, dtype=torch.int64, device="cuda")
    ln = gpu_ctx.encode_shallow(sch, cols, n, out, cap, field, splice, rec_offsets=offs,
                                framed=framed)
    got = out[:ln].cpu().numpy().tobytes()
    assert not out[ln:].any()
    assert got == want
    assert np.array_equal(offs.cpu().numpy().view(np.uint64), want_offs)
    assert np.array_equal(splice.cpu().numpy().view(np.uint64), want_splice)
    rc, deep, _ = oracle.encode_batch(fields, hb.columns(), n, cap, framed=framed, conds=conds)
    assert assemble(got, want_offs, want_splice, hb, field) == deep


@pytest.mark.gpu
@pytest.mark.parametrize("name,fields,conds,field", CASES, ids=[c[0] for c in CASES])
@pytest.mark.parametrize("framed", [False, True], ids=["raw", "rm"])
def test_gpu_view_decode_vs_oracle(gpu_ctx, name, fields, conds, field, framed):
    torch, engine, DeviceBatch = _dev()
    n = 20000
    hb = _batch(fields, n, 9, (0, 300))
    cap = hb.xdr_total(framed)
    rc, xdr, offs = oracle.encode_batch(fields, hb.columns(), n, cap, framed=framed, conds=conds)
    assert rc == 0
    ref = HostBatch.empty(fields, n, hb.dyn_caps())
    rc, fb, err, want_pos = oracle.decode_batch_view(fields, xdr, offs, n, ref.columns(), field,
                                                     framed=framed, conds=conds)
    assert (rc, fb, err) == (0, n, 0)
    sch = engine.Schema(fields, conds)
    caps = hb.dyn_caps()
    caps[field] = 1                   # the payload column holds nothing: views only
    db = DeviceBatch.empty(fields, n, caps)
    buf = torch.from_numpy(np.frombuffer(xdr, dtype=np.uint8).copy()).cuda()
    ro = torch.from_numpy(offs.view(np.int64)).cuda()
    pos = torch.zeros(n, dtype=torch.int64, device="cuda")
    rc, fb, err = gpu_ctx.decode_view(sch, buf, len(xdr), n, db.columns(), field, pos,
                                      rec_offsets=ro, framed=framed)
    assert (rc, fb, err) == (0, n, 0)
    assert np.array_equal(pos.cpu().numpy().view(np.uint64), want_pos)
    got = db.to_host()
    for k, f in enumerate(fields):
        if f[1] == DY:
            assert np.array_equal(got.arrays[k][1], ref.arrays[k][1]), k
            if k != field:
                m = int(ref.arrays[k][1][-1])
                assert np.array_equal(got.arrays[k][0][:m], ref.arrays[k][0][:m]), k
        else:
            assert np.array_equal(got.arrays[k], ref.arrays[k]), k


@pytest.mark.gpu
def test_gpu_view_decode_errors(gpu_ctx):
    """A payload cut short / a negative length: same first record and code
    as the sequential decode (Xdr.java:1028-1037)."""
    torch, engine, DeviceBatch = _dev()
    fields, field, n = NFS_WRITE, 6, 4000
    hb = _batch(fields, n, 13, (1, 64))
    rc, xdr, offs = oracle.encode_batch(fields, hb.columns(), n, hb.xdr_total())
    sch = engine.Schema(fields)
    for r, mode in ((1234, "cut"), (2500, "neg"), (17, "cut")):
        buf = bytearray(xdr)
        o = offs.copy()
        lw = int(o[r]) + 24                        # record r's length word
        if mode == "neg":
            buf[lw:lw + 4] = b"\x80\x00\x00\x01"
        else:
            o[r + 1] = o[r] + 24 + 4 + 1           # extent ends one payload byte in
        data = bytes(buf)
        ref = HostBatch.empty(fields, n, hb.dyn_caps())
        want = oracle.decode_batch_view(fields, data, o, n, ref.columns(), field)[:3]
        db = DeviceBatch.empty(fields, n, {field: 1})
        pos = torch.zeros(n, dtype=torch.int64, device="cuda")
        got = gpu_ctx.decode_view(sch, torch.from_numpy(np.frombuffer(data, np.uint8).copy()).cuda(),
                                  len(data), n, db.columns(), field, pos,
                                  rec_offsets=torch.from_numpy(o.view(np.int64)).cuda(),
                                  raise_on_error=False)
        assert got == want and got[1] == r, (mode, r)


@pytest.mark.gpu
def test_gpu_byref_rejects_non_bytes(gpu_ctx):
    torch, engine, DeviceBatch = _dev()
    fields = [(I, SC, 0), (I, DY, 0)]
    sch = engine.Schema(fields)
    hb = random_batch(fields, 8, seed=2)
    db = DeviceBatch.from_host(hb)
    out = torch.zeros(1024, dtype=torch.uint8, device="cuda")
    sp = torch.zeros(8, dtype=torch.int64, device="cuda")
    with pytest.raises(engine.XdrgError) as ei:
        gpu_ctx.encode_shallow(sch, db.columns(), 8, out, 1024, 1, sp)
    assert ei.value.code == abi.E_INVAL


WIDE_RES = [(I, SC, 0), (STR, DY, 0), (I, DY, 0), (O, DY, 0), (STR, DY, 0), (O, DY, 0), (I, SC, 0)]


@pytest.mark.gpu
@pytest.mark.parametrize("framed", [False, True], ids=["raw", "rm"])
def test_gpu_byref_wide_schema(gpu_ctx, framed):
    """By-reference payload in a schema with more dynamic fields than the lane
    kernels stage (wave-per-record path): encode and view decode vs oracle."""
    torch, engine, DeviceBatch = _dev()
    fields, field, n = WIDE_RES, 3, 4001
    hb = random_batch(fields, n, seed=21, dyn_len=(0, 90))
    cap = hb.xdr_total(framed)
    rc, want, want_offs, want_splice = oracle.encode_batch_shallow(fields, hb.columns(), n, cap, field,
                                                                   framed=framed)
    assert rc == 0
    sch = engine.Schema(fields)
    db = DeviceBatch.from_host(hb)
    cols = db.columns()
    cols[field].data = None
    out = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    offs = torch.zeros(n + 1, dtype=torch.int64, device="cuda")
    splice = torch.zeros(n, dtype=torch.int64, device="cuda")
    ln = gpu_ctx.encode_shallow(sch, cols, n, out, cap, field, splice, rec_offsets=offs, framed=framed)
    assert out[:ln].cpu().numpy().tobytes() == want
    assert np.array_equal(splice.cpu().numpy().view(np.uint64), want_splice)
    rc, deep, deep_offs = oracle.encode_batch(fields, hb.columns(), n, cap, framed=framed)
    ref = HostBatch.empty(fields, n, hb.dyn_caps())
    rc, fb, err, want_pos = oracle.decode_batch_view(fields, deep, deep_offs, n, ref.columns(), field,
                                                     framed=framed)
    caps = hb.dyn_caps()
    caps[field] = 1
    back = DeviceBatch.empty(fields, n, caps)
    pos = torch.zeros(n, dtype=torch.int64, device="cuda")
    buf = torch.from_numpy(np.frombuffer(deep, np.uint8).copy()).cuda()
    got = gpu_ctx.decode_view(sch, buf, len(deep), n, back.columns(), field, pos,
                              rec_offsets=torch.from_numpy(deep_offs.view(np.int64)).cuda(),
                              framed=framed)
    assert got == (0, n, 0)
    assert np.array_equal(pos.cpu().numpy().view(np.uint64), want_pos)
    h = back.to_host()
    for k, f in enumerate(fields):
        if k == field:
            assert np.array_equal(h.arrays[k][1], ref.arrays[k][1])
        elif f[1] == DY:
            m = int(ref.arrays[k][1][-1])
            assert np.array_equal(h.arrays[k][1], ref.arrays[k][1])
            assert np.array_equal(h.arrays[k][0][:m], ref.arrays[k][0][:m])
        else:
            assert np.array_equal(h.arrays[k], ref.arrays[k])
