"""Host-memory forms of the zero-copy calls:
xdrg_encode_batch_shallow / xdrg_decode_batch_view with XDRG_HOST_PTRS
(staging ring) and XDRG_HOST_PTRS | XDRG_HOST_MAPPED (registered memory in
place) — what a JNI caller holding direct ByteBuffers reaches.

The reference's zero-copy send (xdrEncodeShallowByteBuffer / FileChunk,
xdr/Xdr.java:839-866, 978-988, sent as separate writable messages :582-597,
grizzly/GrizzlyRpcTransport.java:130-168) keeps the payload where it is; here
the payload column's data pointer is NULL on every call (never read, never
staged), so only the heads cross PCIe.  xdrDecodeByteBuffer (:423-439)
returns slices of the host buffer: payload_pos comes back as offsets into the
caller's own stream.  Every case is checked against the oracle
(xo_encode_batch_shallow / xo_decode_batch_view), with a ring of 64 KiB slots
so batches cut into many chunks and records straddle them; the staging
bookkeeping runs under ASan/UBSan in tests/test_sanitize.py (by-reference
rounds of tests/cpp/san_stage.cpp)."""
import zlib

import numpy as np
import pytest

import oracle
from hostmem import KINDS, Registered, moved
from oncrpc4j_amd import abi, engine
from oncrpc4j_amd.columns import HostBatch, random_batch
from test_zerocopy import CASES, NFS_WRITE, _batch, assemble

pytestmark = pytest.mark.gpu
SLOT = 64 << 10
U64MAX = (1 << 64) - 1
# (memory kind, mapped)
MODES = [("pageable", False), ("registered", False), ("torch_pinned", False), ("registered", True),
         ("torch_pinned", True)]
MODE_IDS = [f"{k}{'-mapped' if m else ''}" for k, m in MODES]


@pytest.fixture(scope="module")
def hctx():
    import torch
    assert torch.cuda.is_available()
    c = engine.Context(0)
    c.host_staging(SLOT, 3)
    yield c
    c.close()


def _no_payload(cols, field):
    cols[field].data = None   # the payload column: never dereferenced
    return cols


@pytest.mark.parametrize("mode", MODES, ids=MODE_IDS)
@pytest.mark.parametrize("framed", [False, True], ids=["raw", "rm"])
@pytest.mark.parametrize("name,fields,conds,field", CASES, ids=[c[0] for c in CASES])
def test_host_shallow_encode_vs_oracle(hctx, name, fields, conds, field, framed, mode):
    kind, mapped = mode
    n = 3001
    hb0 = _batch(fields, n, zlib.crc32(f"{name}{framed}{kind}".encode()) & 0xffff, (0, 900))
    cap = hb0.xdr_total(framed)
    rc, want, want_offs, want_splice = oracle.encode_batch_shallow(fields, hb0.columns(), n, cap, field,
                                                                   framed=framed, conds=conds)
    assert rc == 0
    mem = KINDS[kind]()
    try:
        hb = moved(hb0, mem)
        sch = engine.Schema(fields, conds)
        out = mem.array(np.full(cap + 64, 0xee, np.uint8))
        ro = mem.array(np.zeros(n + 1, np.uint64))
        spl = mem.array(np.zeros(n, np.uint64))
        ln = hctx.encode_shallow(sch, _no_payload(hb.columns(), field), n, out, cap, field, spl, rec_offsets=ro,
                                 framed=framed, host=True, mapped=mapped)
        assert ln == len(want)
        assert out[:ln].tobytes() == want
        assert (out[ln:] == 0xee).all()
        assert np.array_equal(ro, want_offs)
        assert np.array_equal(spl, want_splice)
        rc, deep, _ = oracle.encode_batch(fields, hb0.columns(), n, cap, framed=framed, conds=conds)
        assert assemble(out[:ln].tobytes(), want_offs, want_splice, hb0, field) == deep
    finally:
        mem.close()


@pytest.mark.parametrize("mode", MODES, ids=MODE_IDS)
@pytest.mark.parametrize("framed", [False, True], ids=["raw", "rm"])
@pytest.mark.parametrize("name,fields,conds,field", CASES, ids=[c[0] for c in CASES])
def test_host_view_decode_vs_oracle(hctx, name, fields, conds, field, framed, mode):
    kind, mapped = mode
    n = 3001
    hb0 = _batch(fields, n, zlib.crc32(f"v{name}{framed}{kind}".encode()) & 0xffff, (0, 900))
    cap = hb0.xdr_total(framed)
    rc, xdr, offs = oracle.encode_batch(fields, hb0.columns(), n, cap, framed=framed, conds=conds)
    assert rc == 0
    ref = HostBatch.empty(fields, n, hb0.dyn_caps())
    rc, fb, err, want_pos = oracle.decode_batch_view(fields, xdr, offs, n, ref.columns(), field,
                                                     framed=framed, conds=conds)
    assert (rc, fb, err) == (0, n, 0)
    mem = KINDS[kind]()
    try:
        caps = hb0.dyn_caps()
        caps[field] = 0
        back = moved(HostBatch.empty(fields, n, caps), mem)
        stream = mem.array(np.frombuffer(xdr, np.uint8))
        ro = mem.array(offs)
        pos = mem.array(np.full(n, 7, np.uint64))
        cols = _no_payload(back.columns(), field)
        cols[field].cap = 0
        st = hctx.decode_view(engine.Schema(fields, conds), stream, len(xdr), n, cols, field, pos,
                              rec_offsets=ro, framed=framed, host=True, mapped=mapped)
        assert st == (0, n, 0)
        assert np.array_equal(pos, want_pos)
        for i in range(0, n, 97):   # the slices are the payloads, in the caller's own buffer
            if want_pos[i] != U64MAX:
                a = int(pos[i])
                ln = int(ref.arrays[field][1][i + 1] - ref.arrays[field][1][i])
                assert stream[a:a + ln].tobytes() == xdr[a:a + ln]
        for k, f in enumerate(fields):
            if f[1] == abi.K_DYNAMIC:
                assert np.array_equal(back.arrays[k][1], ref.arrays[k][1]), k
                if k != field:
                    m = int(ref.arrays[k][1][-1])
                    assert np.array_equal(back.arrays[k][0][:m], ref.arrays[k][0][:m]), k
            else:
                assert np.array_equal(back.arrays[k], ref.arrays[k]), k
    finally:
        mem.close()


@pytest.mark.parametrize("mode", [("pageable", False), ("registered", False), ("registered", True)],
                         ids=["pageable", "registered", "registered-mapped"])
def test_host_view_decode_errors_vs_oracle(hctx, mode):
    """A payload cut short / a negative length: the first failing record and
    code of the sequential decode (Xdr.java:1028-1037), records spread over
    many staging chunks."""
    kind, mapped = mode
    fields, field, n = NFS_WRITE, 6, 4000
    hb0 = _batch(fields, n, 13, (1, 200))
    rc, xdr, offs = oracle.encode_batch(fields, hb0.columns(), n, hb0.xdr_total())
    sch = engine.Schema(fields)
    for r, what in ((3210, "cut"), (2500, "neg"), (17, "cut"), (n - 1, "neg")):
        buf = bytearray(xdr)
        o = offs.copy()
        lw = int(o[r]) + 24
        if what == "neg":
            buf[lw:lw + 4] = b"\x80\x00\x00\x01"
        else:
            o[r + 1] = o[r] + 24 + 4 + 1
        data = bytes(buf)
        ref = HostBatch.empty(fields, n, hb0.dyn_caps())
        want = oracle.decode_batch_view(fields, data, o, n, ref.columns(), field)
        mem = KINDS[kind]()
        try:
            caps = hb0.dyn_caps()
            caps[field] = 0
            back = moved(HostBatch.empty(fields, n, caps), mem)
            pos = mem.array(np.zeros(n, np.uint64))
            cols = _no_payload(back.columns(), field)
            cols[field].cap = 0
            got = hctx.decode_view(sch, mem.array(np.frombuffer(data, np.uint8)), len(data), n, cols, field, pos,
                                   rec_offsets=mem.array(o), host=True, mapped=mapped, raise_on_error=False)
            assert got == tuple(want[:3]) and got[1] == r, (what, r)
            assert np.array_equal(pos[:r], want[3][:r])
            for k in range(6):   # the records before the bad one are delivered
                assert np.array_equal(back.arrays[k][:r], ref.arrays[k][:r])
        finally:
            mem.close()


def test_host_shallow_heads_only_cross(hctx):
    """Config-3 records (24-B head + 4 KiB payload) by reference: the staged
    call moves the heads (and offsets) through a ring far smaller than the
    payloads, which are never read — the payload array is unreadable (an
    address no process may touch), so a read would fault the copy."""
    fields, field, n = NFS_WRITE, 6, 20000
    rng = np.random.default_rng(3)
    hb0 = random_batch(fields, n, seed=4)
    offs = np.arange(n + 1, dtype=np.uint64) * 4096   # 80 MiB of payload, never allocated
    hb0.arrays[field] = (np.zeros(1, np.uint8), offs)
    for k in range(6):
        hb0.arrays[k][:] = rng.integers(-2**31, 2**31, n, dtype=np.int64).astype(np.int32)
    small = HostBatch(fields, n, [a if k != field else (np.zeros(1, np.uint8), np.zeros(n + 1, np.uint64))
                                  for k, a in enumerate(hb0.arrays)])
    # the oracle on zero-length payloads gives the heads; splice and marks follow from the lengths
    heads = 32 * n   # mark + six ints + length word per message
    out = np.zeros(heads + 64, np.uint8)
    spl = np.zeros(n, np.uint64)
    ro = np.zeros(n + 1, np.uint64)
    cols = _no_payload(hb0.columns(), field)
    cols[field].data = 1 << 47   # non-canonical-ish host address: never dereferenced
    sch = engine.Schema(fields)
    ln = hctx.encode_shallow(sch, cols, n, out, heads + 64, field, spl, rec_offsets=ro, framed=True, host=True)
    assert ln == 32 * n
    rc, want, want_offs = oracle.encode_batch(fields, small.columns(), n, 32 * n, framed=True)
    got = out[:ln].copy().reshape(n, 32)
    exp = np.frombuffer(want, np.uint8).reshape(n, 32).copy()
    exp[:, 28:32] = np.frombuffer(np.full(n, 4096, ">u4").tobytes(), np.uint8).reshape(n, 4)   # length words
    exp[:, 0:4] = np.frombuffer(np.full(n, 0x80000000 | (28 + 4096), ">u4").tobytes(), np.uint8).reshape(n, 4)
    assert np.array_equal(got, exp)
    assert np.array_equal(spl, np.arange(n, dtype=np.uint64) * 32 + 32)
    assert np.array_equal(ro, np.arange(n + 1, dtype=np.uint64) * 32)


# ---- flags a call does not take: XDRG_E_INVAL before any pointer is used ----------------
def test_unknown_flags_refused(gpu_ctx):
    import ctypes
    L = engine.lib()
    fields = NFS_WRITE
    sch = engine.Schema(fields)
    hb = random_batch(fields, 4, seed=1, dyn_len=(1, 8))
    cols = hb.columns()
    junk = np.zeros(256, np.uint8)
    ol = ctypes.c_uint64(0)
    fb = ctypes.c_uint64(0)
    er = ctypes.c_int(0)
    h = gpu_ctx.handle
    for bad in (0x10, 0x100, 0x80000000, abi.HOST_MAPPED, abi.HOST_MAPPED | abi.FRAME_RM):
        # host pointers everywhere: a kernel that read them would fault, so only a refusal passes
        assert L.xdrg_encode_batch(h, sch.handle, cols, 4, junk.ctypes.data, 256, None, bad,
                                   ctypes.addressof(ol)) == abi.E_INVAL
        assert L.xdrg_decode_batch(h, sch.handle, junk.ctypes.data, 256, None, 4, cols, bad,
                                   ctypes.addressof(fb), ctypes.addressof(er)) == abi.E_INVAL
        assert L.xdrg_encode_batch_shallow(h, sch.handle, cols, 4, junk.ctypes.data, 256, None, bad,
                                           ctypes.addressof(ol), 6, junk.ctypes.data) == abi.E_INVAL
        assert L.xdrg_decode_batch_view(h, sch.handle, junk.ctypes.data, 256, None, 4, cols, bad,
                                        ctypes.addressof(fb), ctypes.addressof(er), 6,
                                        junk.ctypes.data) == abi.E_INVAL
    # the multi-GPU calls take device memory only
    for bad in (abi.HOST_PTRS, abi.HOST_PTRS | abi.HOST_MAPPED, abi.ASYNC):
        ctxs = (ctypes.c_void_p * 1)(h.value)
        cptr = (ctypes.c_void_p * 1)(ctypes.addressof(cols))
        outs = (ctypes.c_void_p * 1)(junk.ctypes.data)
        assert L.xdrg_encode_batch_multi(ctxs, 1, sch.handle, cptr, (ctypes.c_uint64 * 1)(4), outs, 256, None,
                                         bad, ctypes.byref(ol)) == abi.E_INVAL
        assert L.xdrg_decode_batch_multi(ctxs, 1, sch.handle, outs, 256, None, (ctypes.c_uint64 * 1)(4), cptr,
                                         bad, ctypes.byref(fb), ctypes.byref(er)) == abi.E_INVAL


def test_device_alloc_copy_roundtrip(gpu_ctx):
    """xdrg_device_alloc / xdrg_copy: a caller with no device allocator (a
    JVM) stages a batch in HBM itself and runs the device form of a call."""
    fields = [(abi.T_INT, abi.K_SCALAR, 0)] * 8
    n = 10007
    hb = random_batch(fields, n, seed=8)
    rc, want, _ = oracle.encode_batch(fields, hb.columns(), n, 32 * n)
    sch = engine.Schema(fields)
    bufs = []
    try:
        dcols = []
        for k in range(8):
            p = gpu_ctx.device_alloc(4 * n)
            bufs.append(p)
            gpu_ctx.copy(p, hb.arrays[k], 4 * n, abi.COPY_H2D)
            dcols.append((p, 0, None, 0))
        out = gpu_ctx.device_alloc(32 * n)
        bufs.append(out)
        assert gpu_ctx.encode(sch, dcols, n, out, 32 * n) == 32 * n
        host = np.zeros(32 * n, np.uint8)
        gpu_ctx.copy(host, out, 32 * n, abi.COPY_D2H)
        assert host.tobytes() == want
        out2 = gpu_ctx.device_alloc(0)   # 0 bytes: a valid buffer
        bufs.append(out2)
        with pytest.raises(engine.XdrgError) as ei:
            gpu_ctx.copy(host, out, 16, 9)
        assert ei.value.code == abi.E_INVAL
    finally:
        for p in bufs:
            gpu_ctx.device_free(p)
