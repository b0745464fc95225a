"""The receive side on socket buffers (include/xdrg.h "receive on host socket
buffers"): xdrg_receive_batch, xdrg_frame_scan_ex, xdrg_deframe_ex.

The reference walks the marks of the host Grizzly Buffer its selector thread
filled and hands every complete message on (rpc/RpcMessageParserTCP.java:
44-61 handleRead, :63-99 isAllFragmentsArrived, :109-140 assembleXdr, the
remainder split :57-60); the next filter decodes each message body
(XdrAble.xdrDecode; RpcCall.java:351-354 leaves trailing bytes unread).  The
oracle restates exactly that (oracle/xdr_oracle.c xo_receive_batch:
xo_all_fragments_arrived / xo_assemble per message, then the per-record
decode).  Every case here compares the engine with it on the same stream:
status, messages delivered, consumed bytes (where the remainder starts),
message offsets, first failing message and code, and the decoded columns.

Streams: every record of a random batch is one message, sent as one
fragment (GrizzlyRpcTransport.java:103-110) or re-fragmented the way
ctest/rpc/RpcMessageParserTCPTest.java:161-181 does, with fragment sizes
that are multiples of 4 or not; an incomplete message at the end (STOP for
it, the remainder split before it); corrupted bodies; a message cap; too
small columns (CAPACITY).  Memory: device (HBM), pageable host memory and
registered host memory through the staging ring (64 KiB slots: every stream
spans many windows, messages straddle them, long ones grow the ring), and
registered host memory mapped in place."""
import zlib

import numpy as np
import pytest

import oracle
from hostmem import Pageable, Registered, moved
from oncrpc4j_amd import abi, engine
from oncrpc4j_amd.columns import DeviceBatch, HostBatch, random_batch

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

I, U, B, H, F, D = abi.T_INT, abi.T_UINT, abi.T_BOOL, abi.T_HYPER, abi.T_FLOAT, abi.T_DOUBLE
S, BY, O, STR = abi.T_SHORT, abi.T_BYTE, abi.T_OPAQUE, abi.T_STRING
SC, FX, DY = abi.K_SCALAR, abi.K_FIXED, abi.K_DYNAMIC

SCHEMAS = {
    "cfg2_8xint32": ([(I, SC, 0)] * 8, None),
    "cfg4_shape": ([(I, SC, 0), (STR, DY, 0), (I, DY, 0)], None),
    "cfg3_shape": ([(I, SC, 0)] * 6 + [(O, DY, 0)], None),
    "many_dynamic": ([(H, SC, 0), (STR, DY, 0), (D, DY, 0), (S, DY, 0), (O, FX, 3), (BY, DY, 0), (U, SC, 0)], None),
    # an optional string and an int union (void / hyper / opaque<> arms): rpcgen's
    # optional data and unions as a conditional tape (include/xdrg.h xdrg_cond)
    "cond_union": ([(U, SC, 0), (B, SC, 0), (STR, DY, 0), (I, SC, 0), (H, SC, 0), (O, DY, 0)],
                   [(2, 1, 0, [1]), (4, 3, 0, [1, 2]), (5, 3, 0, [7])]),
    # repeated groups (READDIR-like list of {fileid, name<>, cookie, bool}; a
    # counted array of {int, string<>} between scalars): on host memory the
    # walk, the deframe and the decode of the bodies are three staged passes
    "dirlist_group": ([(abi.T_GROUP, abi.K_LIST, 0, 4), (H, SC, 0), (STR, DY, 0), (H, SC, 0), (B, SC, 0),
                       (I, SC, 0)], None),
    "items_group": ([(I, SC, 0), (abi.T_GROUP, DY, 0, 2), (I, SC, 0), (STR, DY, 0), (I, SC, 0)], None),
}
SLOT = 64 << 10
MEMS = ["device", "pageable", "registered", "mapped"]


@pytest.fixture(scope="module")
def rctx():
    assert torch.cuda.is_available()
    c = engine.Context(0)
    c.set_stream(torch.cuda.current_stream())
    c.host_staging(SLOT, 3)
    yield c
    c.close()


def _sane(hb, conds):
    """Discriminants that pick every arm; bools 0 / 1."""
    rng = np.random.default_rng(hb.n)
    for k, f in enumerate(hb.fields):
        if f[0] == B:   # (a group member's array holds one value per element)
            hb.arrays[k][:] = rng.integers(0, 2, len(hb.arrays[k]), dtype=np.uint8)
    for _, d, _, vals in conds or ():
        if hb.fields[d][0] != B:
            pool = np.array(list(vals) + [0, 5], dtype=np.int64)
            hb.arrays[d][:] = pool[rng.integers(0, pool.size, hb.n)].astype(hb.arrays[d].dtype)
    return hb


def build_stream(fields, conds, hb, style, seed, tail=False, corrupt=0):
    """One message per record -> (stream bytes, body offsets).  style: 'single'
    one fragment each, 'multi' re-fragmented (sizes % 4 == 0), 'odd' fragment
    sizes % 4 != 0 (later marks off 4-byte alignment), 'mixed'."""
    rc, raw, ro = oracle.encode_batch(fields, hb.columns(), hb.n, hb.xdr_total(False) + 64, conds=conds)
    assert rc == 0
    rng = np.random.default_rng(seed)
    parts = []
    for i in range(hb.n):
        body = bytearray(raw[int(ro[i]):int(ro[i + 1])])
        if corrupt and rng.integers(0, corrupt) == 0 and len(body) >= 8:
            body[int(rng.integers(0, len(body) // 4)) * 4] = 0xff   # a length / count word turns negative or huge
        st = style if style != "mixed" else ("single", "multi", "odd")[int(rng.integers(0, 3))]
        if st == "single":
            frag = len(body) + 1
        elif st == "multi":
            frag = 4 * int(rng.integers(1, 40))
        else:
            frag = int(rng.integers(1, 90)) | 1
        parts.append(oracle.fragment(bytes(body), frag))
    if tail and hb.n:
        i = int(rng.integers(0, hb.n))
        t = oracle.fragment(raw[int(ro[i]):int(ro[i + 1])], 64)
        parts.append(t[:max(1, int(rng.integers(1, max(len(t), 2))))])
    return b"".join(parts)


def oracle_receive(fields, conds, stream, cap, caps):
    ref = HostBatch.empty(fields, cap, caps)
    rc, n, used, offs, fb, err = oracle.receive_batch(fields, stream, cap, ref.columns(), conds=conds)
    return (rc, n, used, fb, err), offs, ref


def engine_receive(ctx, fields, conds, stream, cap, caps, mem):
    """-> ((status, delivered, consumed, first_bad, err), message offsets, decoded HostBatch)."""
    sch = engine.Schema(fields, conds)
    if mem == "device":
        buf = torch.zeros(len(stream) + 16, dtype=torch.uint8, device="cuda")
        if stream:
            buf[:len(stream)] = torch.from_numpy(np.frombuffer(stream, np.uint8).copy()).cuda()
        db = DeviceBatch.empty(fields, cap, caps)
        offs = torch.zeros(cap + 1, dtype=torch.int64, device="cuda")
        res = ctx.receive(sch, buf, len(stream), cap, db.columns(), msg_offsets=offs, raise_on_error=False)
        return res, offs.cpu().numpy().view(np.uint64), db.to_host(), None
    host = Registered() if mem in ("registered", "mapped") else Pageable()
    data = host.array(np.frombuffer(stream, np.uint8).copy() if stream else np.zeros(1, np.uint8))
    out = moved(HostBatch.empty(fields, cap, caps), host)
    offs = host.array(np.zeros(cap + 1, np.uint64))
    res = ctx.receive(sch, data, len(stream), cap, out.columns(), msg_offsets=offs, host=mem != "mapped",
                      mapped=mem == "mapped", raise_on_error=False)
    return res, offs.copy(), out, host


def check_receive(ctx, name, stream, cap, caps, mem):
    fields, conds = SCHEMAS[name]
    want, woffs, ref = oracle_receive(fields, conds, stream, cap, caps)
    got, goffs, out, host = engine_receive(ctx, fields, conds, stream, cap, caps, mem)
    try:
        rc, n, used, fb, err = want
        assert got[0] == rc, (got, want)
        assert got[1:3] == (n, used), (got, want)
        if rc != abi.E_INCOMPLETE:
            assert got[3:] == (fb, err), (got, want)
            assert goffs[:n + 1].tolist() == woffs[:n + 1]
            assert out.equal(ref, upto=fb if err else n)
    finally:
        if host is not None:
            host.close()
    return want


@pytest.mark.parametrize("mem", MEMS)
@pytest.mark.parametrize("style", ["single", "multi", "odd", "mixed"])
@pytest.mark.parametrize("name", sorted(SCHEMAS))
def test_receive_vs_oracle(rctx, name, style, mem):
    """Every message complete but one cut tail: all delivered, the tail left
    (consumed = where it starts), values as the oracle's handleRead + decode."""
    fields, conds = SCHEMAS[name]
    n = 300 if name == "cfg3_shape" else 3000
    hb = _sane(random_batch(fields, n, seed=zlib.crc32(f"rx/{name}".encode()) & 0xffff,
                            dyn_len=(0, 600) if name == "cfg3_shape" else (0, 40), special_floats=False), conds)
    stream = build_stream(fields, conds, hb, style, seed=n, tail=True)
    want = check_receive(rctx, name, stream, n + 3, hb.dyn_caps(), mem)
    assert want[0] == 0 and want[1] == n and want[2] < len(stream)


@pytest.mark.parametrize("mem", MEMS)
@pytest.mark.parametrize("cap", [1, 7, 1000])
def test_receive_cap_and_remainder(rctx, cap, mem):
    """At most cap messages; the call returns where the remainder starts, and
    resuming there delivers the rest (handleRead's split, :57-60)."""
    name = "cfg4_shape"
    fields, conds = SCHEMAS[name]
    hb = random_batch(fields, 600 if cap == 1 else 2500, seed=cap, dyn_len=(0, 30))
    stream = build_stream(fields, conds, hb, "mixed", seed=cap, tail=True)
    pos, total = 0, 0
    for _ in range(4000):
        want = check_receive(rctx, name, stream[pos:], cap, hb.dyn_caps(), mem)
        if want[0] == abi.E_INCOMPLETE:
            break
        assert want[1] == min(cap, hb.n - total)
        total += want[1]
        pos += want[2]
    assert total == hb.n


@pytest.mark.parametrize("mem", MEMS)
@pytest.mark.parametrize("name", ["cfg4_shape", "many_dynamic", "cond_union", "dirlist_group"])
def test_receive_errors_vs_oracle(rctx, name, mem):
    """Corrupted bodies: the first bad message and its code; the call delivers
    through it (consumed = its end) and the columns hold the messages before."""
    fields, conds = SCHEMAS[name]
    hb = _sane(random_batch(fields, 2000, seed=17, dyn_len=(0, 30), special_floats=False), conds)
    bad = 0
    for corrupt in (400, 30, 5):
        stream = build_stream(fields, conds, hb, "mixed", seed=corrupt, corrupt=corrupt)
        want = check_receive(rctx, name, stream, hb.n, hb.dyn_caps(), mem)
        if want[0]:
            assert want[1] == want[3] + 1
            bad += 1
    assert bad


@pytest.mark.parametrize("mem", MEMS)
def test_receive_capacity(rctx, mem):
    """Columns too small for the messages: CAPACITY at the first message that
    does not fit, delivered up to it (retry with larger columns)."""
    name = "cfg4_shape"
    fields, conds = SCHEMAS[name]
    hb = random_batch(fields, 3000, seed=3, dyn_len=(1, 30))
    stream = build_stream(fields, conds, hb, "multi", seed=4)
    caps = {k: v // 2 for k, v in hb.dyn_caps().items()}
    want = check_receive(rctx, name, stream, hb.n, caps, mem)
    assert want[0] == abi.E_CAPACITY and want[1] == want[3]


@pytest.mark.parametrize("mem", MEMS)
def test_receive_stop_and_empty(rctx, mem):
    """No complete message (nothing, a lone mark, a cut first message): STOP."""
    name = "cfg2_8xint32"
    fields, conds = SCHEMAS[name]
    hb = random_batch(fields, 3, seed=1)
    stream = build_stream(fields, conds, hb, "multi", seed=2)
    for cut in (b"", stream[:3], stream[:4], stream[:20]):
        want = check_receive(rctx, name, cut, 4, hb.dyn_caps(), mem)
        assert want[0] == abi.E_INCOMPLETE and want[1:3] == (0, 0)


def test_receive_large_messages_grow_the_ring(rctx):
    """Messages larger than a 64 KiB slot's window: the ring grows."""
    name = "cfg3_shape"
    fields, conds = SCHEMAS[name]
    hb = random_batch(fields, 40, seed=8, dyn_len=(50000, 300000))
    stream = build_stream(fields, conds, hb, "mixed", seed=9, tail=True)
    for mem in ("pageable", "registered"):
        want = check_receive(rctx, name, stream, hb.n, hb.dyn_caps(), mem)
        assert want[0] == 0 and want[1] == hb.n


# ---- xdrg_frame_scan_ex / xdrg_deframe_ex on host memory --------------------------------
def _streams():
    fields, conds = SCHEMAS["cfg4_shape"]
    out = []
    for style in ("single", "multi", "odd"):
        hb = random_batch(fields, 1500, seed=len(style), dyn_len=(0, 50))
        out.append((style, build_stream(fields, conds, hb, style, seed=5, tail=True)))
    return out


@pytest.mark.parametrize("mem", ["pageable", "registered", "mapped"])
def test_frame_scan_ex_host_vs_oracle(rctx, mem):
    for style, stream in _streams():
        for cap in (1, 99, 1 << 20):
            rc, want = oracle.frame_scan(stream, cap)
            host = Registered() if mem != "pageable" else Pageable()
            try:
                data = host.array(np.frombuffer(stream, np.uint8).copy())
                offs = host.array(np.zeros(min(cap, 4000) + 1, np.uint64))
                k, used = rctx.frame_scan(data, len(stream), offs, min(cap, 4000), host=mem != "mapped",
                                          mapped=mem == "mapped", with_consumed=True)
                rc2, want2 = oracle.frame_scan(stream, min(cap, 4000))
                assert k == len(want2) - 1, style
                assert offs[:k + 1].tolist() == want2
                assert used == want2[-1]
            finally:
                host.close()


@pytest.mark.parametrize("mem", ["pageable", "registered", "mapped"])
def test_deframe_ex_host_vs_oracle(rctx, mem):
    for style, stream in _streams():
        rc, want = oracle.frame_scan(stream, 1 << 20)
        k_want = len(want) - 1
        bodies = []
        for i in range(k_want):   # assembleXdr of each message: the concatenated fragment bodies
            seg, p, body = stream[want[i]:want[i + 1]], 0, b""
            while True:
                m = int.from_bytes(seg[p:p + 4], "big")
                body += seg[p + 4:p + 4 + (m & abi.RPC_SIZE_MASK)]
                p += 4 + (m & abi.RPC_SIZE_MASK)
                if m & abi.RPC_LAST_FRAG:
                    break
            bodies.append(body)
        total = sum(len(b) for b in bodies)
        for room in (total, total // 3):
            host = Registered() if mem != "pageable" else Pageable()
            try:
                data = host.array(np.frombuffer(stream, np.uint8).copy())
                pay = host.array(np.zeros(max(room, 1), np.uint8))
                offs = host.array(np.zeros(k_want + 1, np.uint64))
                k, used, rc = rctx.deframe(data, len(stream), pay, room, offs, k_want, host=mem != "mapped",
                                           mapped=mem == "mapped", raise_on_error=False)
                if room == total:
                    assert rc == 0 and k == k_want and used == want[-1], style
                elif mem == "mapped":   # the device form: nothing delivered, the bytes needed
                    assert rc == abi.E_CAPACITY
                    continue
                else:   # the bodies that fit
                    assert rc == abi.E_CAPACITY and 0 < k < k_want and used == want[k]
                got = [pay[int(offs[i]):int(offs[i + 1])].tobytes() for i in range(k)]
                assert got == bodies[:k]
            finally:
                host.close()


@pytest.mark.parametrize("win", [1, 0], ids=["windows", "three_pass"])
@pytest.mark.parametrize("mem", ["pageable", "registered"])
@pytest.mark.parametrize("name", ["dirlist_group", "items_group"])
def test_receive_groups_staged_vs_oracle(rctx, name, mem, win):
    """Repeated groups on host memory: the staging windows carry each
    message's element rows (tuning key 42 = 1, one PCIe crossing) or the
    staged walk, deframe and body decode run (key 42 = 0); both equal the
    oracle's handleRead + decode, with element capacities that run out
    mid-stream (CAPACITY, delivered up to it) and messages over many 64 KiB
    windows."""
    fields, conds = SCHEMAS[name]
    rctx.tune(42, win)
    try:
        n = 4000
        hb = _sane(random_batch(fields, n, seed=zlib.crc32(f"grx/{name}".encode()) & 0xffff, dyn_len=(0, 40),
                                special_floats=False), conds)
        for style in ("single", "mixed"):
            stream = build_stream(fields, conds, hb, style, seed=n + len(style), tail=True)
            want = check_receive(rctx, name, stream, n + 3, hb.dyn_caps(), mem)
            assert want[0] == 0 and want[1] == n
        g = next(k for k, f in enumerate(fields) if f[0] == abi.T_GROUP)
        caps = hb.dyn_caps()
        caps[g] = caps[g] * 2 // 3   # the group's elements run out two thirds in
        stream = build_stream(fields, conds, hb, "single", seed=7)
        want = check_receive(rctx, name, stream, n, caps, mem)
        assert want[0] == abi.E_CAPACITY and want[1] == want[3] < n
    finally:
        rctx.tune(0)
