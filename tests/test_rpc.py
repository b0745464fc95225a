"""RPC message batching (oncrpc4j_amd/rpc.py): accepted
replies (RpcCall.acceptedReply, rpc/RpcCall.java:323-343) and incoming calls
(RpcProtocolFilter.handleRead + RpcCall.accept, RpcCall.java:206-216) as
device batches.  Fixtures: tests/golden/rpc_vectors.json (xdrlib-packed in the
reference's field order, tests/golden/make_golden.py)."""
import numpy as np
import pytest

import gold
import oracle
from oncrpc4j_amd import abi, rpc
from oncrpc4j_amd.columns import HostBatch, random_batch

V = gold.load("rpc_vectors.json")


# ---- host helpers (oracle side) --------------------------------------------------
def _const_cols(words):
    """Constant columns over one int32 array (XDRG_STRIDE_CONST)."""
    arr = np.array(words, dtype=np.int32)
    return arr, [(arr.ctypes.data + 4 * i, abi.STRIDE_CONST, None, 0) for i in range(len(words))]


def _host_cols(tuples, keep):
    out = (abi.Column * len(tuples))()
    for i, (data, stride, offs, cap) in enumerate(tuples):
        out[i].data = data
        out[i].stride = stride
        out[i].offsets = offs
        out[i].cap = cap
    out._keep = keep
    return out


def _body_host_tuples(hb):
    cols = hb.columns()
    return [(cols[k].data, cols[k].stride, cols[k].offsets, cols[k].cap) for k in range(len(hb.fields))], cols


def reply_host_columns(xids, body_hb, stat=rpc.SUCCESS):
    xa = np.array(xids, dtype=np.int32)
    carr, consts = _const_cols([rpc.REPLY, rpc.MSG_ACCEPTED, rpc.AUTH_NONE, 0, stat])
    body, bkeep = _body_host_tuples(body_hb)
    tuples = [(xa.ctypes.data, 4, None, 0)] + consts + body
    return _host_cols(tuples, (xa, carr, bkeep, body_hb))


def call_records_batch(records):
    """rpc_vectors.json calls -> HostBatch of rpc.call_fields(AUTH_UNIX, (int, string))."""
    rows = []
    for r in records:
        machine = bytes.fromhex(r["machine"])
        body_len = 4 + 4 + len(machine) + (-len(machine)) % 4 + 4 + 4 + 4 + 4 * len(r["gids"])
        rows.append([r["xid"], rpc.CALL, r["rpcvers"], r["prog"], r["vers"], r["proc"],
                     rpc.AUTH_UNIX, body_len, r["stamp"], r["machine"], r["uid"], r["gid"], r["gids"],
                     rpc.AUTH_NONE, "", r["arg_int"], r["arg_str"]])
    return gold.batch_from_records(rpc.call_fields(rpc.AUTH_UNIX, ARGS), rows)


ARGS = [rpc.INT, rpc.STRING_DYN]


# ---- CPU: field tapes and the oracle against the fixtures ---------------------------
def test_reply_prelude_is_24_bytes():
    assert sum(4 for _ in rpc.REPLY_PRELUDE_NONE) == 24
    assert rpc.accepted_reply_fields([])[:6] == rpc.REPLY_PRELUDE_NONE
    with pytest.raises(ValueError):
        rpc.call_fields(rpc.RPCSEC_GSS)


@pytest.mark.parametrize("case", V["replies"], ids=lambda c: c["name"])
def test_oracle_reply_vectors(case):
    body_fields = [tuple(f) for f in case["body_fields"]]
    fields = rpc.accepted_reply_fields(body_fields)
    n = len(case["xids"])
    body = gold.batch_from_records(body_fields, case["bodies"])
    cols = reply_host_columns(case["xids"], body)
    want = bytes.fromhex(case["stream"])
    rc, xdr, offs = oracle.encode_batch(fields, cols, n, len(want) + 16, framed=True)
    assert rc == 0
    assert xdr == want
    assert offs.tolist() == case["rec_offsets"]


def test_oracle_call_vectors():
    c = V["calls"]
    fields = rpc.call_fields(rpc.AUTH_UNIX, ARGS)
    want = call_records_batch(c["records"])
    stream = bytes.fromhex(c["stream"])
    n = len(c["records"])
    out = HostBatch.empty(fields, n, want.dyn_caps())
    rc, fb, err = oracle.decode_batch(fields, stream, np.array(c["rec_offsets"], dtype=np.uint64), n,
                                      out.columns(), framed=True)
    assert (rc, fb, err) == (0, n, 0)
    assert out.equal(want)


def test_oracle_rejects_constant_column_on_decode():
    fields = [rpc.INT]
    _, consts = _const_cols([7])
    cols = _host_cols(consts, None)
    rc, fb, err = oracle.decode_batch(fields, b"\x00\x00\x00\x07", None, 1, cols)
    assert rc == abi.E_INVAL


# ---- GPU: the engine path ----------------------------------------------------------
torch = pytest.importorskip("torch")


def _dev_bytes(b):
    return torch.from_numpy(np.frombuffer(b, dtype=np.uint8).copy()).cuda()


def _dev_body_cols(body_hb):
    from oncrpc4j_amd.columns import DeviceBatch
    db = DeviceBatch.from_host(body_hb)
    cols = db.columns()
    return [(cols[k].data, cols[k].stride, cols[k].offsets, cols[k].cap) for k in range(len(body_hb.fields))], db


@pytest.mark.gpu
@pytest.mark.parametrize("case", V["replies"], ids=lambda c: c["name"])
def test_reply_encoder_golden(gpu_ctx, case):
    body_fields = [tuple(f) for f in case["body_fields"]]
    n = len(case["xids"])
    enc = rpc.ReplyEncoder(gpu_ctx, body_fields)
    xids = torch.tensor(case["xids"], dtype=torch.int32, device="cuda")
    body, keep = _dev_body_cols(gold.batch_from_records(body_fields, case["bodies"]))
    want = bytes.fromhex(case["stream"])
    out = torch.zeros(len(want) + 64, dtype=torch.uint8, device="cuda")
    offs = torch.zeros(n + 1, dtype=torch.int64, device="cuda")
    ln = enc.encode(xids, body, n, out, out.numel(), rec_offsets=offs)
    assert ln == len(want)
    assert out[:ln].cpu().numpy().tobytes() == want
    assert offs.cpu().tolist() == case["rec_offsets"]
    assert not out[ln:].any()


@pytest.mark.gpu
@pytest.mark.parametrize("per_reply_stat", [False, True], ids=["const-stat", "per-reply-stat"])
@pytest.mark.parametrize("body", ["none", "int_string_intvec", "fixed_words"])
def test_reply_encoder_random_vs_oracle(gpu_ctx, body, per_reply_stat):
    body_fields = {"none": [], "int_string_intvec": [rpc.INT, rpc.STRING_DYN, rpc.INT_DYN],
                   "fixed_words": [rpc.INT, (abi.T_HYPER, abi.K_SCALAR, 0), (abi.T_OPAQUE, abi.K_FIXED, 6)]}[body]
    n = 20011
    rng = np.random.default_rng(n)
    xids = rng.integers(-2**31, 2**31, n, dtype=np.int64).astype(np.int32)
    stats = rng.integers(0, 6, n, dtype=np.int32) if per_reply_stat else None
    hb = random_batch(body_fields, n, seed=3, dyn_len=(0, 30)) if body_fields else HostBatch([], n, [])
    # oracle: the same tape with host columns (constants and all)
    fields = rpc.accepted_reply_fields(body_fields)
    hcols = reply_host_columns(xids, hb)
    if per_reply_stat:
        hcols[5].data = stats.ctypes.data
        hcols[5].stride = 4
    total = n * 28 + sum(hb.xdr_sizes()) if body_fields else n * 28
    rc, want, want_offs = oracle.encode_batch(fields, hcols, n, total + 16, framed=True)
    assert rc == 0
    enc = rpc.ReplyEncoder(gpu_ctx, body_fields)
    body_cols, keep = _dev_body_cols(hb) if body_fields else ([], None)
    dx = torch.from_numpy(xids).cuda()
    ds = torch.from_numpy(stats).cuda() if per_reply_stat else None
    out = torch.zeros(len(want) + 64, dtype=torch.uint8, device="cuda")
    offs = torch.zeros(n + 1, dtype=torch.int64, device="cuda")
    ln = enc.encode(dx, body_cols, n, out, out.numel(), rec_offsets=offs, accept_stats=ds)
    assert ln == len(want)
    assert out[:ln].cpu().numpy().tobytes() == want
    assert np.array_equal(offs.cpu().numpy().view(np.uint64), want_offs)


@pytest.mark.gpu
def test_reply_encoder_verifier_bodies(gpu_ctx):
    """Per-reply verifier bodies (e.g. RPCSEC_GSS MICs, RpcAuthVerifier.java:58-61)."""
    n = 3001
    rng = np.random.default_rng(7)
    lens = rng.integers(0, 40, n)
    offs = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(lens, out=offs[1:])
    vals = rng.integers(0, 256, int(offs[-1]), dtype=np.uint8)
    xids = rng.integers(0, 2**31, n, dtype=np.int64).astype(np.int32)
    enc = rpc.ReplyEncoder(gpu_ctx, [rpc.INT], verifier_flavor=rpc.RPCSEC_GSS, verifier_body=True)
    body = np.arange(n, dtype=np.int32)
    out = torch.zeros(n * 80, dtype=torch.uint8, device="cuda")
    ln = enc.encode(torch.from_numpy(xids).cuda(), [(torch.from_numpy(body).cuda(), 4, None, 0)], n, out,
                    out.numel(), verifier=(torch.from_numpy(vals).cuda(),
                                           torch.from_numpy(offs.view(np.int64)).cuda()))
    got = out[:ln].cpu().numpy().tobytes()
    # restated per message in the reference's order (RpcCall.java:328-333)
    exp = b""
    for i in range(n):
        v = vals[offs[i]:offs[i + 1]].tobytes()
        msg = (int(xids[i]).to_bytes(4, "big", signed=True) + (1).to_bytes(4, "big") + bytes(4) +
               rpc.RPCSEC_GSS.to_bytes(4, "big") + len(v).to_bytes(4, "big") + v + bytes((-len(v)) % 4) +
               bytes(4) + int(body[i]).to_bytes(4, "big"))
        exp += (len(msg) | 0x80000000).to_bytes(4, "big") + msg
    assert got == exp


@pytest.mark.gpu
def test_call_decoder_golden(gpu_ctx):
    c = V["calls"]
    n = len(c["records"])
    stream = bytes.fromhex(c["stream"])
    xdr = _dev_bytes(stream)
    ro = torch.tensor(c["rec_offsets"], dtype=torch.int64, device="cuda")
    dec = rpc.CallDecoder(gpu_ctx)
    hdr, st = dec.decode_headers(xdr, len(stream), n, ro)
    assert st == (0, n, 0)
    h = hdr.cpu().numpy()
    for i, r in enumerate(c["records"]):
        assert h[i].tolist() == [r["xid"], rpc.CALL, r["rpcvers"], r["prog"], r["vers"], r["proc"], rpc.AUTH_UNIX]
    m = rpc.CallDecoder.check(hdr)
    assert m["rpc_mismatch"].nonzero().flatten().tolist() == [5, 17]
    assert not m["not_call"].any() and not m["unsupported_flavor"].any()
    groups = rpc.CallDecoder.group_by_procedure(hdr)
    assert list(groups) == [(100003, 4, 1, rpc.AUTH_UNIX)]
    want = call_records_batch(c["records"])
    batch, st = dec.decode(rpc.AUTH_UNIX, ARGS, xdr, len(stream), n, ro, want.dyn_caps())
    assert st == (0, n, 0)
    assert batch.to_host().equal(want)


@pytest.mark.gpu
def test_reply_decoder_roundtrip(gpu_ctx):
    case = V["replies"][2]   # string bodies
    n = len(case["xids"])
    stream = bytes.fromhex(case["stream"])
    body_fields = [tuple(f) for f in case["body_fields"]]
    dec = rpc.ReplyDecoder(gpu_ctx, body_fields)
    ro = torch.tensor(case["rec_offsets"], dtype=torch.int64, device="cuda")
    batch, st = dec.decode(_dev_bytes(stream), len(stream), n, ro, {4: 16, 6: 64 * n})
    assert st == (0, n, 0)
    hb = batch.to_host()
    assert hb.arrays[0].tolist() == case["xids"]
    assert set(hb.arrays[1].tolist()) == {rpc.REPLY} and set(hb.arrays[2].tolist()) == {rpc.MSG_ACCEPTED}
    assert [bytes(hb.record(i, 6)).hex() for i in range(n)] == [b[0] for b in case["bodies"]]


@pytest.mark.gpu
def test_constant_column_rejected_on_decode(gpu_ctx):
    from oncrpc4j_amd import engine
    sch = engine.Schema([rpc.INT])
    c = torch.zeros(4, dtype=torch.int32, device="cuda")
    xdr = torch.zeros(4, dtype=torch.uint8, device="cuda")
    rc, _, _ = gpu_ctx.decode(sch, xdr, 4, 1, [(c, abi.STRIDE_CONST, None, 0)], raise_on_error=False)
    assert rc == abi.E_INVAL
