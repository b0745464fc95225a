"""XDRG_HOST_PTRS: batches in HOST memory through the C-ABI (include/xdrg.h),
the boundary a JNI caller with Grizzly host buffers reaches
(xdr/Xdr.java:115-119, grizzly/GrizzlyMemoryManager.java:42-57,
grizzly/GrizzlyRpcTransport.java:97-112).

Every case compares the staged host call with the oracle (oracle/xdr_oracle.c,
the restatement of Xdr.java) on the same records: stream bytes, record
offsets, decoded columns, first-bad record and error code, CAPACITY.  The
context's ring is a few slots of 64 KiB, so every batch is cut into many
chunks and records straddle chunk boundaries; a record larger than a slot
grows the ring.  Host memory comes as plain pageable numpy buffers (bounce
copies), buffers registered with xdrg_host_register (direct DMA, and
XDRG_HOST_MAPPED: kernels on the host buffers in place) and hipHostMalloc'd
torch pinned memory.  The staging bookkeeping itself runs under ASan/UBSan
on the CPU in tests/test_sanitize.py."""
import ctypes
import threading
import zlib

import numpy as np
import pytest

import oracle
from oncrpc4j_amd import abi, engine
from oncrpc4j_amd.columns import HostBatch, aos_columns, random_batch

I, U, B, H, F, D = abi.T_INT, abi.T_UINT, abi.T_BOOL, abi.T_HYPER, abi.T_FLOAT, abi.T_DOUBLE
S, BY, O, STR, G = abi.T_SHORT, abi.T_BYTE, abi.T_OPAQUE, abi.T_STRING, abi.T_GROUP
SC, FX, DY, LS = abi.K_SCALAR, abi.K_FIXED, abi.K_DYNAMIC, abi.K_LIST

SCHEMAS = {
    "cfg2_8xint32": [(I, SC, 0)] * 8,
    "mixed_fixed": [(I, SC, 0), (H, SC, 0), (F, SC, 0), (D, SC, 0), (B, SC, 0), (S, SC, 0), (BY, SC, 0),
                    (O, FX, 5), (I, FX, 3)],
    "cfg4_shape": [(I, SC, 0), (STR, DY, 0), (I, DY, 0)],
    "cfg3_shape": [(I, SC, 0)] * 6 + [(O, DY, 0)],
    "many_dynamic": [(H, SC, 0), (STR, DY, 0), (D, DY, 0), (S, DY, 0), (O, FX, 3), (BY, DY, 0), (U, SC, 0)],
}
SLOT = 64 << 10

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hctx():
    import torch
    assert torch.cuda.is_available()   # torch's runtime first (its pinned allocator serves TorchPinned)
    c = engine.Context(0)
    c.host_staging(SLOT, 3)
    yield c
    c.close()


from hostmem import KINDS, Pageable, Registered, TorchPinned, moved  # noqa: E402,F401


def oracle_encode(fields, hb, framed, conds=None):
    rc, want, offs = oracle.encode_batch(fields, hb.columns(), hb.n, hb.xdr_total(framed) + 64, framed=framed,
                                         conds=conds)
    assert rc == 0
    return want, offs


def oracle_decode(fields, xdr, offs, n, caps, framed, conds=None):
    ref = HostBatch.empty(fields, n, caps)
    st = oracle.decode_batch(fields, xdr, offs, n, ref.columns(), framed=framed, conds=conds)
    return ref, st


# ---- round trips ----------------------------------------------------------------------
@pytest.mark.parametrize("kind", list(KINDS))
@pytest.mark.parametrize("framed", [False, True], ids=["raw", "rm"])
@pytest.mark.parametrize("name", list(SCHEMAS))
def test_host_roundtrip_vs_oracle(hctx, name, framed, kind):
    fields = SCHEMAS[name]
    n = 700 if name == "cfg3_shape" else 5003
    hb0 = random_batch(fields, n, seed=zlib.crc32(f"{name}{framed}".encode()) & 0xffff,
                       dyn_len=(0, 300) if name == "cfg3_shape" else (0, 40))
    want, want_offs = oracle_encode(fields, hb0, framed)
    mem = KINDS[kind]()
    try:
        hb = moved(hb0, mem)
        sch = engine.Schema(fields)
        out = mem.array(np.zeros(len(want) + 64, np.uint8))
        ro = mem.array(np.zeros(n + 1, np.uint64))
        ln = hctx.encode(sch, hb.columns(), n, out, len(want) + 64, rec_offsets=ro, framed=framed, host=True)
        assert ln == len(want)
        assert out[:ln].tobytes() == want, "staged encode differs from the oracle"
        assert np.array_equal(ro, want_offs)
        back = HostBatch.empty(fields, n, hb0.dyn_caps())
        back = moved(back, mem)
        var = not sch.is_fixed
        st = hctx.decode(sch, out, ln, n, back.columns(), rec_offsets=ro if var else None, framed=framed,
                         host=True)
        assert st == (0, n, 0)
        ref, rst = oracle_decode(fields, want, want_offs, n, hb0.dyn_caps(), framed)
        assert rst == (0, n, 0)
        assert back.equal(ref), "staged decode differs from the oracle"
    finally:
        mem.close()


@pytest.mark.parametrize("name", ["cfg2_8xint32", "cfg4_shape", "mixed_fixed"])
def test_host_mapped_vs_oracle(hctx, name):
    """XDRG_HOST_MAPPED: the kernels read and write registered host buffers in place."""
    fields = SCHEMAS[name]
    n = 4099
    hb0 = random_batch(fields, n, seed=11, dyn_len=(0, 40))
    want, want_offs = oracle_encode(fields, hb0, False)
    mem = Registered()
    try:
        hb = moved(hb0, mem)
        sch = engine.Schema(fields)
        out = mem.array(np.zeros(len(want) + 64, np.uint8))
        ro = mem.array(np.zeros(n + 1, np.uint64))
        ln = hctx.encode(sch, hb.columns(), n, out, len(want) + 64, rec_offsets=ro, mapped=True)
        assert out[:ln].tobytes() == want and np.array_equal(ro, want_offs)
        back = moved(HostBatch.empty(fields, n, hb0.dyn_caps()), mem)
        st = hctx.decode(sch, out, ln, n, back.columns(), rec_offsets=ro, mapped=True)
        assert st == (0, n, 0)
        ref, _ = oracle_decode(fields, want, want_offs, n, hb0.dyn_caps(), False)
        assert back.equal(ref)
        with pytest.raises(engine.XdrgError):   # pageable memory is not device-reachable
            hctx.encode(sch, hb0.columns(), n, np.zeros(len(want), np.uint8), len(want), mapped=True)
    finally:
        mem.close()


# ---- errors: the reference's first failing record and code ---------------------------
@pytest.mark.parametrize("kind", ["pageable", "registered"])
def test_host_decode_errors_vs_oracle(hctx, kind):
    fields = SCHEMAS["cfg4_shape"]
    n = 6000
    hb0 = random_batch(fields, n, seed=5, dyn_len=(0, 60))
    want, offs = oracle_encode(fields, hb0, False)
    sch = engine.Schema(fields)
    rng = np.random.default_rng(9)
    mem = KINDS[kind]()
    try:
        for case in range(6):
            x = bytearray(want)
            ro = offs.copy()
            in_len = len(x)
            r = int(rng.integers(n // 3, n))   # deep inside a later chunk
            if case == 0:    # a string length past its record: SHORT
                x[int(ro[r]) + 4:int(ro[r]) + 8] = (0x7ffffff0).to_bytes(4, "big")
            elif case == 1:  # a negative vector count: CORRUPT (checkArraySize, Xdr.java:1034-1037)
                slen = int.from_bytes(x[int(ro[r]) + 4:int(ro[r]) + 8], "big")
                p = int(ro[r]) + 8 + slen + ((4 - slen & 3) & 3)
                x[p:p + 4] = (0xfffffffe).to_bytes(4, "big")
            elif case == 2:  # the stream ends inside record r
                in_len = int(ro[r]) + 6
            elif case == 3:  # a record extent cut short
                ro[r + 1] = ro[r] + 4
            caps = hb0.dyn_caps()
            if case == 4:    # the string column holds the records before r only: CAPACITY
                caps[1] = int(hb0.arrays[1][1][r])
            if case == 5:    # and the int<> column
                caps[2] = int(hb0.arrays[2][1][r]) + 1
            xs = mem.array(np.frombuffer(bytes(x), np.uint8))
            ros = mem.array(ro)
            back = moved(HostBatch.empty(fields, n, caps), mem)
            st = hctx.decode(sch, xs, in_len, n, back.columns(), rec_offsets=ros, host=True, raise_on_error=False)
            ref, rst = oracle_decode(fields, bytes(x[:in_len]), ro, n, caps, False)
            assert st == rst, (case, st, rst)
            assert st[0] != 0 and st[1] <= r
            assert back.equal(ref, upto=st[1]), f"case {case}: records before first_bad differ"
    finally:
        mem.close()


def test_host_fixed_decode_errors_vs_oracle(hctx):
    """Fixed-size chunks leave without waiting; their status is still the batch's first error."""
    fields = SCHEMAS["cfg2_8xint32"]
    n = 9000
    hb = random_batch(fields, n, seed=3)
    sch = engine.Schema(fields)
    for framed in (False, True):
        want, offs = oracle_encode(fields, hb, framed)
        x = bytearray(want)
        in_len = len(x)
        if framed:   # a mark that does not frame its record: FRAME
            r = 7777
            x[int(offs[r]):int(offs[r]) + 4] = (0x80000010).to_bytes(4, "big")
        else:        # truncated: SHORT at the first incomplete record
            in_len = len(x) - 37
        back = HostBatch.empty(fields, n)
        st = hctx.decode(sch, np.frombuffer(bytes(x), np.uint8), in_len, n, back.columns(), framed=framed,
                         host=True, raise_on_error=False)
        ref, rst = oracle_decode(fields, bytes(x[:in_len]), None, n, None, framed)
        assert st == rst and st[0] != 0
        assert back.equal(ref, upto=st[1])


def test_host_encode_capacity(hctx):
    L = engine.lib()
    for name in ("cfg2_8xint32", "cfg4_shape"):
        fields = SCHEMAS[name]
        n = 3000
        hb = random_batch(fields, n, seed=2, dyn_len=(0, 50))
        want, _ = oracle_encode(fields, hb, True)
        sch = engine.Schema(fields)
        out = np.zeros(len(want), np.uint8)
        ol = ctypes.c_uint64(0)
        rc = L.xdrg_encode_batch(hctx.handle, sch.handle, hb.columns(), n, out.ctypes.data, len(want) - 4,
                                 None, abi.FRAME_RM | abi.HOST_PTRS, ctypes.byref(ol))
        assert rc == abi.E_CAPACITY and ol.value == len(want)   # the bytes the batch needs
        rc = L.xdrg_encode_batch(hctx.handle, sch.handle, hb.columns(), n, out.ctypes.data, len(want),
                                 None, abi.FRAME_RM | abi.HOST_PTRS | abi.ASYNC, ctypes.byref(ol))
        assert rc == abi.E_INVAL   # host calls are synchronous


# ---- layouts: records larger than a slot, array-of-structs, constants, unions ----------
def test_host_records_larger_than_a_slot():
    """opaque<> records of up to 300 KiB through 64 KiB slots: the ring grows."""
    fields = SCHEMAS["cfg3_shape"]
    n = 40
    hb = random_batch(fields, n, seed=4, dyn_len=(0, 300 << 10))
    want, offs = oracle_encode(fields, hb, False)
    with engine.Context(0) as c:
        c.host_staging(SLOT, 2)
        sch = engine.Schema(fields)
        out = np.zeros(len(want), np.uint8)
        ro = np.zeros(n + 1, np.uint64)
        assert c.encode(sch, hb.columns(), n, out, len(want), rec_offsets=ro, host=True) == len(want)
        assert out.tobytes() == want and np.array_equal(ro, offs)
        back = HostBatch.empty(fields, n, hb.dyn_caps())
        assert c.decode(sch, out, len(want), n, back.columns(), rec_offsets=ro, host=True) == (0, n, 0)
        assert back.equal(hb)


def test_host_aos_partial_coverage(hctx):
    """Array-of-structs records with bytes no field covers (a gap and a tail):
    decode writes the fields only, the caller's other bytes stay."""
    fields = [(I, SC, 0)] * 4 + [(H, SC, 0), (I, SC, 0)]
    offs = [0, 4, 8, 12, 24, 32]           # 16..24 and 36..48 are the caller's
    rec = 48
    n = 5000
    rng = np.random.default_rng(8)
    aos = rng.integers(0, 256, n * rec, dtype=np.uint8)
    cols = aos_columns(fields, aos.ctypes.data, rec, offs)
    sch = engine.Schema(fields)
    xb = n * sch.fixed_size   # 28 B records
    rc, want, _ = oracle.encode_batch(fields, cols, n, xb)
    assert rc == 0
    out = np.zeros(xb, np.uint8)
    assert hctx.encode(sch, cols, n, out, xb, host=True) == xb
    assert out.tobytes() == want
    back = np.full(n * rec, 0xAB, np.uint8)
    assert hctx.decode(sch, out, xb, n, aos_columns(fields, back.ctypes.data, rec, offs), host=True) == (0, n, 0)
    b2, a2 = back.reshape(n, rec), aos.reshape(n, rec)
    covered = np.zeros(rec, bool)
    for o, w in zip(offs, [4, 4, 4, 4, 8, 4]):
        covered[o:o + w] = True
    assert np.array_equal(b2[:, covered], a2[:, covered])
    assert (b2[:, ~covered] == 0xAB).all()


def test_host_constant_columns(hctx):
    """XDRG_STRIDE_CONST columns (the reply prelude words, RpcCall.java:328-332) from host memory."""
    fields = [(I, SC, 0), (I, SC, 0), (I, SC, 0), (STR, DY, 0)]
    n = 4000
    hb = random_batch(fields, n, seed=6, dyn_len=(0, 30))
    const = np.array([1, 0], np.int32)
    cols = hb.columns()
    cols[1].data, cols[1].stride = const.ctypes.data, abi.STRIDE_CONST
    cols[2].data, cols[2].stride = const.ctypes.data + 4, abi.STRIDE_CONST
    rc, want, offs = oracle.encode_batch(fields, cols, n, hb.xdr_total() + 64)
    assert rc == 0
    out = np.zeros(len(want), np.uint8)
    ro = np.zeros(n + 1, np.uint64)
    assert hctx.encode(engine.Schema(fields), cols, n, out, len(want), rec_offsets=ro, host=True) == len(want)
    assert out.tobytes() == want and np.array_equal(ro, offs)


def test_host_conditional_schema(hctx):
    """A union-shaped tape (rpcgen READ-like result) through the staging ring."""
    fields = [(I, SC, 0), (B, SC, 0), (I, SC, 0), (STR, DY, 0), (O, DY, 0), (I, SC, 0)]
    conds = [(1, 0, False, [0]), (2, 0, False, [0]), (3, 0, False, [0]), (4, 0, False, [0])]
    n = 5000
    hb = random_batch(fields, n, seed=12, dyn_len=(0, 50))
    rng = np.random.default_rng(12)
    hb.arrays[0][:] = rng.choice(np.array([0, 0, 0, 5], np.int32), n)
    hb.arrays[1][:] = rng.integers(0, 2, n, dtype=np.uint8)
    rc, want, offs = oracle.encode_batch(fields, hb.columns(), n, hb.xdr_total() + 64, conds=conds)
    assert rc == 0
    sch = engine.Schema(fields, conds)
    out = np.zeros(len(want) + 16, np.uint8)
    ro = np.zeros(n + 1, np.uint64)
    assert hctx.encode(sch, hb.columns(), n, out, len(out), rec_offsets=ro, host=True) == len(want)
    assert out[:len(want)].tobytes() == want and np.array_equal(ro, offs)
    back = HostBatch.empty(fields, n, hb.dyn_caps())
    assert hctx.decode(sch, out, len(want), n, back.columns(), rec_offsets=ro, host=True) == (0, n, 0)
    ref = HostBatch.empty(fields, n, hb.dyn_caps())
    assert oracle.decode_batch(fields, want, offs, n, ref.columns(), conds=conds) == (0, n, 0)
    assert back.equal(ref)


GROUP_SHAPES = {
    # portmap DUMP's pmaplist (a T *next list), an array of structs with strings
    # and vectors inside, a fixed array of structs; a top-level string beside them
    "list": [(I, SC, 0), (G, LS, 0, 2), (U, SC, 0), (STR, DY, 0), (I, SC, 0)],
    "array": [(STR, DY, 0), (G, DY, 0, 4), (H, SC, 0), (O, DY, 0), (I, DY, 0), (O, FX, 3)],
    "fixed": [(U, SC, 0), (G, FX, 3, 2), (S, SC, 0), (STR, DY, 0), (D, SC, 0)],
}


@pytest.mark.parametrize("kind", ["pageable", "registered", "mapped"])
@pytest.mark.parametrize("framed", [False, True], ids=["raw", "rm"])
@pytest.mark.parametrize("shape", list(GROUP_SHAPES))
def test_host_groups_vs_oracle(hctx, shape, framed, kind):
    """Repeated groups on host memory: staged (a chunk of records moves its
    elements' member rows with it; 64 KiB slots, so lists straddle many
    chunks) and mapped in place, encode and decode equal to the oracle;
    then a decode with too few element slots (CAPACITY at the oracle's
    record)."""
    fields = GROUP_SHAPES[shape]
    n = 3000
    hb0 = random_batch(fields, n, seed=13 + len(shape), dyn_len=(0, 12), group_len=(0, 9), special_floats=False)
    rc, want, offs = oracle.encode_batch(fields, hb0.columns(), n, hb0.xdr_total(framed) + 64, framed=framed)
    assert rc == 0
    sch = engine.Schema(fields)
    mem = Registered() if kind != "pageable" else Pageable()
    host, mapped = kind != "mapped", kind == "mapped"
    try:
        hb = moved(hb0, mem)
        out = mem.array(np.zeros(len(want), np.uint8))
        ro = mem.array(np.zeros(n + 1, np.uint64))
        assert hctx.encode(sch, hb.columns(), n, out, len(want), rec_offsets=ro, framed=framed, host=host,
                           mapped=mapped) == len(want)
        assert out.tobytes() == want
        assert np.array_equal(ro, offs)
        for caps in (hb0.dyn_caps(), {k: v // 2 for k, v in hb0.dyn_caps().items()}):
            back = moved(HostBatch.empty(fields, n, caps), mem)
            st = hctx.decode(sch, out, len(want), n, back.columns(), rec_offsets=ro, framed=framed, host=host,
                             mapped=mapped, raise_on_error=False)
            ref = HostBatch.empty(fields, n, caps)
            wst = oracle.decode_batch(fields, want, offs, n, ref.columns(), framed=framed)
            assert st == wst
            assert back.equal(ref, upto=wst[1])
    finally:
        mem.close()


def test_host_two_contexts_concurrently():
    """A server's two directions at once, one context per thread (Xdr's single
    owner, Xdr.java:56,71): replies encode while requests decode."""
    fields = SCHEMAS["cfg4_shape"]
    n = 20000
    hb = random_batch(fields, n, seed=21, dyn_len=(0, 60))
    want, offs = oracle_encode(fields, hb, True)
    sch = engine.Schema(fields)
    res = {}

    def enc():
        with engine.Context(0) as c:
            c.host_staging(256 << 10, 3)
            out = np.zeros(len(want), np.uint8)
            ro = np.zeros(n + 1, np.uint64)
            for _ in range(3):
                ln = c.encode(sch, hb.columns(), n, out, len(want), rec_offsets=ro, framed=True, host=True)
            res["enc"] = (ln, out.tobytes(), ro.copy())

    def dec():
        with engine.Context(0) as c:
            c.host_staging(256 << 10, 3)
            buf = np.frombuffer(want, np.uint8)
            for _ in range(3):
                back = HostBatch.empty(fields, n, hb.dyn_caps())
                st = c.decode(sch, buf, len(want), n, back.columns(), rec_offsets=offs, framed=True, host=True)
            res["dec"] = (st, back)

    ts = [threading.Thread(target=enc), threading.Thread(target=dec)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    ln, got, ro = res["enc"]
    assert ln == len(want) and got == want and np.array_equal(ro, offs)
    st, back = res["dec"]
    assert st == (0, n, 0) and back.equal(hb)
