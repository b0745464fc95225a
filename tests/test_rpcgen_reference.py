"""The reference's own rpcgen inputs: BlobStore.x and
Calculator.x of oncrpc4j-rpcgen/src/test/xdr/, the two programs the
reference's build runs jrpcgen on (oncrpc4j-rpcgen/pom.xml:38-96) and its
loopback tests call (gtest/java/.../SyncBlobStoreTest.java:8-29,
AbstractCalculatorTest.java:19-39).

* The .x files are parsed UNCHANGED from /root/reference (skipped where the
  reference is absent, as on the GPU box; they are never copied) and their
  tapes checked against the ones the fixture records:
  put(Key, Value) / get(Key) -> Value with Value a bool union
  (notNull: TRUE -> opaque<1024>, FALSE -> void), add(hyper, hyper) ->
  CalculationResult {hyper, unsigned hyper, unsigned hyper},
  addSimple(hyper, hyper) -> hyper, and Calculator.x's constants in every
  literal form.
* tests/golden/reference_rpcgen_vectors.json (tests/golden/make_golden.py)
  holds those messages packed by CPython's stdlib xdrlib from the
  declarations, both Value arms included; the oracle must reproduce the
  bytes on the CPU, the HIP engine on the GPU, encode and decode, raw and
  record-marked."""
import os

import numpy as np
import pytest

import gold
import oracle
from oncrpc4j_amd import abi, rpcgen
from oncrpc4j_amd.columns import HostBatch

FIX = gold.load("reference_rpcgen_vectors.json")
REF_X = "/root/reference/oncrpc4j-rpcgen/src/test/xdr"
MSGS = FIX["messages"]


def _ids(m):
    return f"{m['name']}-{'rm' if m['framed'] else 'raw'}"


def _tape(m):
    return [tuple(f) for f in m["fields"]], [(a, b, bool(n), list(v)) for a, b, n, v in m["conds"]]


def _batch(m):
    fields, _ = _tape(m)
    hb = gold.batch_from_records(fields, m["records"])
    return hb, bytes.fromhex(m["xdr"]), np.asarray(m["rec_offsets"], np.uint64)


@pytest.mark.skipif(not os.path.isdir(REF_X), reason="the reference tree is not present")
def test_reference_x_files_parse_to_the_fixture_tapes():
    specs = {name: rpcgen.parse_file(os.path.join(REF_X, name)) for name in ("BlobStore.x", "Calculator.x")}
    seen = set()
    for m in MSGS:
        s = specs["BlobStore.x" if m["program"] == 118 else "Calculator.x"]
        key = (m["program"], m["version"], m["procedure"])
        p = s.procedures()[key]
        assert p.name == m["name"].split(".")[1].split()[0]
        got = s.args_tape(*key) if m["which"] == "args" else s.result_tape(*key)
        assert ([tuple(f) for f in got[0]], [tuple(c) for c in got[1]]) == \
            ([tuple(f) for f in _tape(m)[0]], [tuple(c) for c in _tape(m)[1]]), m["name"]
        seen.add((key, m["which"]))
    # every procedure's arguments and result (put's result is void: an empty tape)
    put = specs["BlobStore.x"]
    assert put.result_tape(118, 1, 1) == ([], [])
    assert len(seen) == 7
    c = specs["Calculator.x"]
    assert c.value("PLAIN_ZERO") == c.value("HEX_ZERO") == 0
    assert c.value("SMALL_CONST") == 0xFF00 and c.value("LARGE_CONST") == 0xFFF000000000
    assert c.value("HUGE_CONST") == 0xFFF000000000000000000
    for k in ("UNSIGNED_LONG_HEX_CONST", "UNSIGNED_LONG_OCT_CONST", "UNSIGNED_LONG_DEC_CONST"):
        assert c.value(k) == 2**64 - 1, k
    for k in ("UNSIGNED_INT_HEX_CONST", "UNSIGNED_INT_OCT_CONST", "UNSIGNED_INT_DEC_CONST"):
        assert c.value(k) == 2**32 - 1, k


def test_fixture_covers_both_value_arms():
    for m in MSGS:
        if m["name"] not in ("BlobStore.put args", "BlobStore.get result"):
            continue
        k = 1 if m["name"] == "BlobStore.put args" else 0   # the notNull discriminant
        arms = {r[k] for r in m["records"]}
        assert arms == {0, 1}, m["name"]


@pytest.mark.parametrize("m", MSGS, ids=_ids)
def test_oracle_reference_rpcgen_vectors(m):
    fields, conds = _tape(m)
    hb, want, offs = _batch(m)
    rc, xdr, ro = oracle.encode_batch(fields, hb.columns(), hb.n, len(want) + 64, framed=m["framed"],
                                      conds=conds or None)
    assert rc == 0 and xdr == want and np.array_equal(ro, offs)
    out = HostBatch.empty(fields, hb.n, hb.dyn_caps())
    assert oracle.decode_batch(fields, want, offs, hb.n, out.columns(), framed=m["framed"],
                               conds=conds or None) == (0, hb.n, 0)
    assert out.equal(hb)


@pytest.mark.gpu
@pytest.mark.parametrize("m", MSGS, ids=_ids)
def test_gpu_reference_rpcgen_vectors(gpu_ctx, m):
    import torch
    from oncrpc4j_amd import engine
    from oncrpc4j_amd.columns import DeviceBatch
    fields, conds = _tape(m)
    hb, want, offs = _batch(m)
    sch = engine.Schema(fields, conds or None)
    db = DeviceBatch.from_host(hb)
    out = torch.zeros(len(want) + 64, dtype=torch.uint8, device="cuda")
    ro = torch.zeros(hb.n + 1, dtype=torch.int64, device="cuda")
    ln = gpu_ctx.encode(sch, db.columns(), hb.n, out, len(want) + 64, rec_offsets=ro, framed=m["framed"])
    assert out[:ln].cpu().numpy().tobytes() == want
    assert np.array_equal(ro.cpu().numpy().view(np.uint64), offs)
    back = DeviceBatch.empty(fields, hb.n, hb.dyn_caps())
    assert gpu_ctx.decode(sch, out, ln, hb.n, back.columns(), rec_offsets=ro, framed=m["framed"]) == (0, hb.n, 0)
    assert back.to_host().equal(hb)
    # the stream as the fixture holds it, decoded from a fresh device copy
    dev = torch.from_numpy(np.frombuffer(want, np.uint8).copy()).cuda()
    back2 = DeviceBatch.empty(fields, hb.n, hb.dyn_caps())
    assert gpu_ctx.decode(sch, dev, len(want), hb.n, back2.columns(),
                          rec_offsets=torch.from_numpy(offs.view(np.int64)).cuda(), framed=m["framed"]) == (0, hb.n, 0)
    assert back2.to_host().equal(hb)


@pytest.mark.gpu
def test_gpu_blobstore_value_errors_vs_oracle(gpu_ctx):
    """get's result (Value) cut inside a TRUE arm's opaque / with a negative
    length: the first failing record and code equal the oracle's."""
    import torch
    from oncrpc4j_amd import engine
    from oncrpc4j_amd.columns import DeviceBatch
    m = next(x for x in MSGS if x["name"] == "BlobStore.get result" and not x["framed"])
    fields, conds = _tape(m)
    hb, want, offs = _batch(m)
    sch = engine.Schema(fields, conds)
    full = [i for i, r in enumerate(m["records"]) if r[0] and len(r[1]) >= 8]
    for r, what in ((full[3], "cut"), (full[-1], "neg")):
        buf = bytearray(want)
        o = offs.copy()
        if what == "neg":
            buf[int(o[r]) + 4:int(o[r]) + 8] = b"\xff\xff\xff\xf0"
        else:
            o[r + 1] = o[r] + 9
        data = bytes(buf)
        ref = HostBatch.empty(fields, hb.n, hb.dyn_caps())
        rst = oracle.decode_batch(fields, data, o, hb.n, ref.columns(), conds=conds)
        back = DeviceBatch.empty(fields, hb.n, hb.dyn_caps())
        st = gpu_ctx.decode(sch, torch.from_numpy(np.frombuffer(data, np.uint8).copy()).cuda(), len(data), hb.n,
                            back.columns(), rec_offsets=torch.from_numpy(o.view(np.int64)).cuda(),
                            raise_on_error=False)
        assert st == rst and st[1] == r and st[2] in (abi.E_SHORT, abi.E_CORRUPT), (what, st, rst)
        assert back.to_host().equal(ref, upto=r)
