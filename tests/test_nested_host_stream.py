"""XDRG_HOST_PTRS on schemas whose group elements hold groups (SURVEY.md §8f
row 2; include/xdrg.h "Host memory"): the staging ring moves every level's
element rows with their records (host_stage.h chunk_rows / dec_layout, a
nested group's totals read at its parent's element total), so such batches
stream through small slots instead of bouncing whole through device scratch.

The reference decodes any XdrAble, nested or not, straight from the host
Grizzly buffer (rpc/RpcMessageParserTCP.java:44-61, 109-140; jrpcgen.java:
856-906 calls the inner elements' xdrDecode).  Here: volume_index (lists
inside list elements, an optional and a union inside them), acl_tree (four
group levels) and seg_lists (arrays of list heads), random batches far
larger than slot x slots, pageable and registered memory, against the oracle
encode and round trip, and a cut stream's first bad record deep in a later
chunk (Xdr.java:1028-1031)."""
import numpy as np
import pytest

import oracle
import test_acl_tree as acl
import test_list_heads as seg
import test_volume_index as vol
from oncrpc4j_amd import abi
from oncrpc4j_amd.columns import HostBatch

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

SLOT = 64 << 10   # small slots: records and their elements straddle chunks

CASES = {
    "volume_index": (vol.FIELDS, vol.CONDS, vol._random),
    "acl_tree": (acl.FIELDS, acl.CONDS, acl._random),
    "seg_lists": (seg.FIELDS, None, seg._random),
}


@pytest.mark.parametrize("kind", ["pageable", "registered"])
@pytest.mark.parametrize("name", sorted(CASES))
def test_nested_host_streams(name, kind):
    from oncrpc4j_amd import engine
    from hostmem import Pageable, Registered, moved
    fields, conds, make = CASES[name]
    hb0 = make(4000, 77)
    rc, want, offs = oracle.encode_batch(fields, hb0.columns(), hb0.n, hb0.xdr_total() + 64, conds=conds)
    assert rc == 0
    assert len(want) > 3 * SLOT, "the batch must not fit the ring at once"
    n = hb0.n
    c = engine.Context(0)
    mem = Registered() if kind == "registered" else Pageable()
    try:
        c.host_staging(SLOT, 3)
        b0 = c.internal_stat(4)
        hb = moved(hb0, mem)
        sch = engine.Schema(fields, conds)
        out = mem.array(np.zeros(len(want) + 64, np.uint8))
        ro = mem.array(np.zeros(n + 1, np.uint64))
        ln = c.encode(sch, hb.columns(), n, out, len(want) + 64, rec_offsets=ro, host=True)
        assert ln == len(want)
        assert out[:ln].tobytes() == want and np.array_equal(ro, offs)
        back = moved(HostBatch.empty(fields, n, hb0.dyn_caps()), mem)
        assert c.decode(sch, out, ln, n, back.columns(), rec_offsets=ro, host=True) == (0, n, 0)
        dec = HostBatch.empty(fields, n, hb0.dyn_caps())   # absent optional / union arms read as 0
        assert oracle.decode_batch(fields, want, offs, n, dec.columns(), conds=conds) == (0, n, 0)
        assert back.equal(dec)
        # a stream cut inside a record of a late chunk: status and the records before it
        cut = int(offs[n - 40]) + 6
        xin = mem.array(np.frombuffer(want[:cut] + bytes(64), np.uint8).copy())
        got = moved(HostBatch.empty(fields, n, hb0.dyn_caps()), mem)
        st = c.decode(sch, xin, cut, n, got.columns(), rec_offsets=ro, host=True, raise_on_error=False)
        ref = HostBatch.empty(fields, n, hb0.dyn_caps())
        rst = oracle.decode_batch(fields, want[:cut], offs, n, ref.columns(), conds=conds)
        assert st == rst and st[1] == n - 40
        assert got.equal(ref, upto=st[1])
        assert c.internal_stat(4) == b0, "streamed, not bounced through device scratch"
    finally:
        mem.close()
        c.close()


@pytest.mark.parametrize("name", sorted(CASES))
def test_nested_host_capacity(name):
    """Too few inner elements in the host columns: CAPACITY at the oracle's
    record, the records before it decoded (a chunk's grant is the remainder
    of the host column)."""
    from oncrpc4j_amd import engine
    from hostmem import Pageable, moved
    fields, conds, make = CASES[name]
    hb0 = make(3000, 91)
    rc, want, offs = oracle.encode_batch(fields, hb0.columns(), hb0.n, hb0.xdr_total() + 64, conds=conds)
    n = hb0.n
    caps = hb0.dyn_caps()
    inner = [k for k, f in enumerate(fields) if f[0] == abi.T_GROUP and hb0.parent[k] >= 0 and f[1] != abi.K_FIXED and caps.get(k)]
    if not inner:
        pytest.skip("no counted inner group")
    k = inner[0]
    caps[k] = caps[k] * 2 // 3
    c = engine.Context(0)
    mem = Pageable()
    try:
        c.host_staging(SLOT, 2)
        sch = engine.Schema(fields, conds)
        xin = mem.array(np.frombuffer(want + bytes(64), np.uint8).copy())
        ro = mem.array(offs.copy())
        got = moved(HostBatch.empty(fields, n, caps), mem)
        st = c.decode(sch, xin, len(want), n, got.columns(), rec_offsets=ro, host=True, raise_on_error=False)
        ref = HostBatch.empty(fields, n, caps)
        rst = oracle.decode_batch(fields, want, offs, n, ref.columns(), conds=conds)
        assert st == rst and st[0] != 0
        assert got.equal(ref, upto=st[1])
    finally:
        mem.close()
        c.close()


@pytest.mark.parametrize("win,budget", [(1, 20), (1, 2), (0, 20)], ids=["windows", "windows_tight", "three_pass"])
@pytest.mark.parametrize("kind", ["pageable", "registered"])
@pytest.mark.parametrize("name", sorted(CASES))
def test_nested_host_receive(name, kind, win, budget):
    """xdrg_receive_batch on a host socket buffer of nested-group messages:
    the receive windows carry every level's element rows with their messages
    (tuning key 42 = 1: one PCIe crossing, no three-pass fallback taken) or
    the staged walk, deframe and body decode run (key 42 = 0); windows_tight
    reserves a fifth of a window's bytes for its columns (key 49 = 2), so
    windows deliver fewer messages than they hold and single messages grow
    the ring (host_stage.h stage_receive's two halves).  All equal
    the oracle's handleRead + decode (RpcMessageParserTCP.java:44-61,
    109-140) on single-fragment and re-fragmented streams with a cut tail,
    on corrupted bodies (first bad message delivered, GARBAGE_ARGS) and with
    an inner group's elements running out (CAPACITY)."""
    from oncrpc4j_amd import engine
    from test_receive import build_stream, engine_receive, oracle_receive
    fields, conds, make = CASES[name]
    n = 3000
    hb = make(n, 123)
    c = engine.Context(0)
    try:
        c.host_staging(SLOT, 3)
        c.tune(42, win)
        c.tune(49, budget)
        t0 = c.internal_stat(5)
        inner = [k for k, f in enumerate(fields)
                 if f[0] == abi.T_GROUP and hb.parent[k] >= 0 and f[1] != abi.K_FIXED]
        small = hb.dyn_caps()
        small[inner[0]] = small[inner[0]] * 2 // 3
        cases = [("single", 0, hb.dyn_caps()), ("mixed", 0, hb.dyn_caps()), ("single", 1500, hb.dyn_caps()),
                 ("single", 0, small)]
        for style, corrupt, caps in cases:
            stream = build_stream(fields, conds, hb, style, seed=n + len(style) + corrupt, tail=True,
                                  corrupt=corrupt)
            want, woffs, ref = oracle_receive(fields, conds, stream, n + 3, caps)
            got, goffs, out, host = engine_receive(c, fields, conds, stream, n + 3, caps, kind)
            try:
                rc, got_n, used, fb, err = want
                assert got[:3] == (rc, got_n, used), (style, corrupt, got, want)
                assert got[3:] == (fb, err), (style, corrupt, got, want)
                assert goffs[:got_n + 1].tolist() == woffs[:got_n + 1]
                assert out.equal(ref, upto=fb if err else got_n)
                if caps is small:
                    assert err == abi.E_CAPACITY and 0 < got_n < n
                elif corrupt:
                    assert err != 0
                else:
                    assert (rc, got_n) == (0, n)
            finally:
                host.close()
        if win:
            assert c.internal_stat(5) == t0, "the receive windows carried the nested schema"
        else:
            assert c.internal_stat(5) == t0 + len(cases)
    finally:
        c.close()


@pytest.mark.parametrize("name", sorted(CASES))
def test_first_record_bad_member_offsets(name):
    """A batch whose record 0 fails delivers no records, and every offsets
    column holds its one entry, 0 (Xdr.java:1028-1031: nothing decoded):
    the members' first entries too, which only record 0's place wrote — the
    staging ring starts a chunk at any record, so a chunk whose first record
    is the batch's first bad one returned stale slot bytes there.  Device
    columns filled with a sentinel first."""
    from oncrpc4j_amd import engine
    from oncrpc4j_amd.columns import DeviceBatch
    fields, conds, make = CASES[name]
    hb = make(200, 5)
    rc, want, offs = oracle.encode_batch(fields, hb.columns(), hb.n, hb.xdr_total() + 64, conds=conds)
    c = engine.Context(0)
    try:
        for cut in (0, 2, 6):   # record 0 cut inside its first words
            db = DeviceBatch.empty(fields, hb.n, hb.dyn_caps())
            cnt = []   # every counted column's offsets: dynamic fields and DYNAMIC / LIST groups
            for k, f in enumerate(fields):
                t = db.tensors[k]
                if isinstance(t, tuple):
                    cnt.append((k, t[1]))
                elif f[0] == abi.T_GROUP and f[1] != abi.K_FIXED:
                    cnt.append((k, t))
            for _, o in cnt:
                o.fill_(0x5a5a5a5a)
            x = torch.zeros(len(want) + 64, dtype=torch.uint8, device="cuda")
            if cut:
                x[:cut] = torch.from_numpy(np.frombuffer(want[:cut], np.uint8).copy()).cuda()
            ro = torch.from_numpy(offs.view(np.int64).copy()).cuda()
            st = c.decode(engine.Schema(fields, conds), x, cut, hb.n, db.columns(), rec_offsets=ro,
                          raise_on_error=False)
            assert st[1] == 0 and st[0] != 0
            for k, o in cnt:
                assert int(o[0]) == 0, (cut, k, fields[k])
    finally:
        c.close()
