"""Arrays of list heads: a list node type's generated
xdrEncode is a do/while over its chain — the node's fields, then
xdrEncodeBoolean(next != null), then the next node's fields, ... until a FALSE
(jrpcgen.java:1103-1121, xdrDecode :1133-1150) — so `T x<>` / `T x[N]` of a
list node T writes a count (dynamic) and, per element, a whole chain
(jrpcgen.java:856-906 calling each element's xdrEncode), and a `T` held by
value writes one chain.

tests/golden/rpcgen/seg_lists.x `seg_map` holds all three.  On the tape
(oncrpc4j_amd.rpcgen) an element of such an array is the head node's fields
followed by the chain's remaining nodes as an inner list group — the same
words in the same order, with one group level per chain.  The fixtures
(tests/golden/seg_lists_vectors.json) were packed by CPython's stdlib xdrlib
from the declarations; the oracle is checked against them on the CPU, the HIP
engine against them and against the oracle on the GPU."""
import os

import numpy as np
import pytest

import gold
import oracle
from oncrpc4j_amd import abi, rpcgen
from oncrpc4j_amd.columns import HostBatch, random_batch

FIX = gold.load("seg_lists_vectors.json")
FIELDS = [tuple(f) for f in FIX["fields"]]
SPEC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "rpcgen", "seg_lists.x")
CHAINS, CH_REST, SPARE, SP_REST, FIRST_REST, DONE = 1, 5, 9, 13, 20, 24


def _ids(b):
    return "rm" if b["framed"] else "raw"


def _batch(b):
    hb = gold.batch_from_records(FIELDS, b["records"])
    return hb, bytes.fromhex(b["xdr"]), np.asarray(b["rec_offsets"], np.uint64)


def test_seg_lists_tape():
    G, FX, DY, LS = abi.T_GROUP, abi.K_FIXED, abi.K_DYNAMIC, abi.K_LIST
    node = [(abi.T_UHYPER, abi.K_SCALAR, 0), (abi.T_UINT, abi.K_SCALAR, 0), (abi.T_OPAQUE, DY, 0)]
    f, c = rpcgen.parse_file(SPEC).tape("seg_map")
    assert [tuple(x) for x in f] == FIELDS and c == []
    assert FIELDS == ([(abi.T_UINT, abi.K_SCALAR, 0), (G, DY, 0, 7)] + node + [(G, LS, 0, 3)] + node +
                      [(G, FX, 2, 7)] + node + [(G, LS, 0, 3)] + node +
                      node + [(G, LS, 0, 3)] + node + [(abi.T_BOOL, abi.K_SCALAR, 0)])


def test_batch_layout():
    hb, want, offs = _batch(FIX["batches"][0])
    assert hb.rows(CH_REST) == hb.elems(CHAINS) > 0   # one chain per array element
    assert hb.rows(SP_REST) == hb.elems(SPARE) == 2 * hb.n
    assert hb.rows(FIRST_REST) == hb.n
    assert hb.elems(CH_REST) > 0 and hb.elems(FIRST_REST) > 0
    s = hb.slice(7, 31)
    rc, xdr, _ = oracle.encode_batch(FIELDS, s.columns(), s.n, len(want))
    assert rc == 0 and xdr == want[int(offs[7]):int(offs[31])]


@pytest.mark.parametrize("b", FIX["batches"], ids=_ids)
def test_oracle_seg_lists_fixture(b):
    hb, want, offs = _batch(b)
    rc, xdr, ro = oracle.encode_batch(FIELDS, hb.columns(), hb.n, len(want) + 64, framed=b["framed"])
    assert rc == 0
    assert xdr == want, "oracle encode differs from xdrlib"
    assert ro.tolist() == b["rec_offsets"]
    out = HostBatch.empty(FIELDS, hb.n, hb.dyn_caps())
    assert oracle.decode_batch(FIELDS, want, offs, hb.n, out.columns(), framed=b["framed"]) == (0, hb.n, 0)
    assert out.equal(hb)


def _mutations(b, want, rng):
    """(name, stream, in_len, code, record): errors inside the chains."""
    out = []
    r, _, at = b["probes"][[p[1] for p in b["probes"]].index("chains_count")]
    y = bytearray(want)
    y[at:at + 4] = b"\xff\xff\xff\xfc"          # `new seg_node[-4]`: NegativeArraySizeException
    out.append(("negative_chains_count", bytes(y), len(y), abi.E_NEG_SIZE, r))
    tags = [p for p in b["probes"] if p[1] == "tag_len"]
    r, _, at = tags[int(rng.integers(0, len(tags)))]
    y = bytearray(want)
    y[at:at + 4] = b"\x80\x00\x00\x03"          # a negative opaque length inside a chain
    out.append(("tag_corrupt", bytes(y), len(y), abi.E_CORRUPT, r))
    nexts = [p for p in b["probes"] if p[1] == "next_bool"]
    r, _, at = nexts[int(rng.integers(0, len(nexts)))]
    y = bytearray(want)
    y[at:at + 4] = b"\x00\x00\x00\x01"          # a chain continues where it ended: later bytes misparse
    out.append(("chain_extended", bytes(y), len(y), None, r))
    r, _, at = nexts[int(rng.integers(0, len(nexts)))]
    out.append(("truncated_in_chain", bytes(want), at + 2, None, r))
    return out


def test_oracle_seg_lists_errors():
    b = FIX["batches"][0]
    hb, want, offs = _batch(b)
    for name, x, in_len, code, r in _mutations(b, want, np.random.default_rng(5)):
        ref = HostBatch.empty(FIELDS, hb.n, hb.dyn_caps())
        rc, fb, err = oracle.decode_batch(FIELDS, x[:in_len], offs, hb.n, ref.columns())
        if code is not None:
            assert err == code, (name, rc, fb, err)
        assert err != 0 or code == 0 or code is None, name
        assert ref.equal(hb, upto=min(fb, r)), name


def _random(n, seed):
    hb = random_batch(FIELDS, n, seed=seed, dyn_len=(0, 8), group_len=(0, 5), inner_len=(0, 4))
    hb.arrays[DONE][:] = np.random.default_rng(seed).integers(0, 2, n, dtype=np.uint8)
    return hb


def test_oracle_random_roundtrip():
    hb = _random(400, 9)
    rc, want, offs = oracle.encode_batch(FIELDS, hb.columns(), hb.n, hb.xdr_total() + 64)
    assert rc == 0
    out = HostBatch.empty(FIELDS, hb.n, hb.dyn_caps())
    assert oracle.decode_batch(FIELDS, want, offs, hb.n, out.columns()) == (0, hb.n, 0)
    assert out.equal(hb)


# ---- GPU ---------------------------------------------------------------------
@pytest.fixture(params=[(8, 32768), (8, 0), (64, 0)], ids=lambda p: f"enc{p[0]}-dtile{p[1]}")
def grp_tune(request, gpu_ctx):
    """Group kernels under each production choice (tuning keys 32 / 33)."""
    gpu_ctx.tune(32, request.param[0])
    gpu_ctx.tune(33, request.param[1])
    yield request.param
    gpu_ctx.tune(0)


def _gpu_roundtrip(gpu_ctx, hb, want, offs, framed):
    import torch
    from oncrpc4j_amd import engine
    from oncrpc4j_amd.columns import DeviceBatch
    sch = engine.Schema(FIELDS)
    db = DeviceBatch.from_host(hb)
    out = torch.zeros(len(want) + 64, dtype=torch.uint8, device="cuda")
    ro = torch.zeros(hb.n + 1, dtype=torch.int64, device="cuda")
    ln = gpu_ctx.encode(sch, db.columns(), hb.n, out, len(want) + 64, rec_offsets=ro, framed=framed)
    assert out[:ln].cpu().numpy().tobytes() == want, "GPU encode differs"
    assert not out[ln:].any(), "engine wrote past the stream end"
    assert ro.cpu().numpy().astype(np.uint64).tolist() == offs.tolist()
    back = DeviceBatch.empty(FIELDS, hb.n, hb.dyn_caps())
    assert gpu_ctx.decode(sch, out, ln, hb.n, back.columns(), rec_offsets=ro, framed=framed) == (0, hb.n, 0)
    assert back.to_host().equal(hb)


@pytest.mark.gpu
@pytest.mark.parametrize("b", FIX["batches"], ids=_ids)
def test_gpu_seg_lists_fixture(gpu_ctx, grp_tune, b):
    hb, want, offs = _batch(b)
    _gpu_roundtrip(gpu_ctx, hb, want, offs, b["framed"])


@pytest.mark.gpu
def test_gpu_seg_lists_errors_vs_oracle(gpu_ctx, grp_tune):
    import torch
    from oncrpc4j_amd import engine
    from oncrpc4j_amd.columns import DeviceBatch
    b = FIX["batches"][0]
    hb, want, offs = _batch(b)
    sch = engine.Schema(FIELDS)
    for name, x, in_len, _, _ in _mutations(b, want, np.random.default_rng(7)):
        dev = torch.from_numpy(np.frombuffer(x, np.uint8).copy()).cuda()
        ro = torch.from_numpy(offs.astype(np.int64)).cuda()
        back = DeviceBatch.empty(FIELDS, hb.n, hb.dyn_caps())
        st = gpu_ctx.decode(sch, dev, in_len, hb.n, back.columns(), rec_offsets=ro, raise_on_error=False)
        ref = HostBatch.empty(FIELDS, hb.n, hb.dyn_caps())
        rst = oracle.decode_batch(FIELDS, x[:in_len], offs, hb.n, ref.columns())
        assert st == rst, (name, st, rst)
        assert back.to_host().equal(ref, upto=st[1]), name


@pytest.mark.gpu
@pytest.mark.parametrize("framed", [False, True], ids=["raw", "rm"])
def test_gpu_seg_lists_random_vs_oracle(gpu_ctx, grp_tune, framed):
    hb = _random(3000, 17)
    rc, want, offs = oracle.encode_batch(FIELDS, hb.columns(), hb.n, hb.xdr_total(framed) + 64, framed=framed)
    assert rc == 0
    _gpu_roundtrip(gpu_ctx, hb, want, offs, framed)
