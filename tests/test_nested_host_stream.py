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
