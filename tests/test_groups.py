"""Repeated groups: arrays of structs and recursive lists (include/xdrg.h
"Repeated groups").

rpcgen encodes `T x<>` of a struct T as the element count and then every
element's fields, `T x[N]` without the count (jrpcgen.java:856-906), and a
recursive optional list `T *x` (struct T { ...; T *next; }) as TRUE +
element for each element, then FALSE (INDIRECTION, jrpcgen.java:835-851) —
the bytes oncrpc4j's own portmap/pmaplist.java:63-70 and rpcb_list.java
write.  Decoding a negative count is `new T[-2]`: NegativeArraySizeException
(XDRG_E_NEG_SIZE).  The fixtures (tests/golden/group_vectors.json) were
packed by CPython's stdlib xdrlib; the oracle is checked against them on the
CPU, the HIP engine against them and against the oracle on the GPU."""
import numpy as np
import pytest

import gold
import oracle
from oncrpc4j_amd import abi
from oncrpc4j_amd.columns import HostBatch, random_batch

I, U, B, H, F = abi.T_INT, abi.T_UINT, abi.T_BOOL, abi.T_HYPER, abi.T_FLOAT
O, STR, G = abi.T_OPAQUE, abi.T_STRING, abi.T_GROUP
SC, FX, DY, LS = abi.K_SCALAR, abi.K_FIXED, abi.K_DYNAMIC, abi.K_LIST

BATCHES = gold.load("group_vectors.json")["batches"]


def _ids(b):
    return f'{b["name"]}-{"rm" if b["framed"] else "raw"}'


def _fields(b):
    return [tuple(f) for f in b["fields"]]


def _offs(v):
    return np.asarray(v, dtype=np.uint64)


# ---- oracle vs the xdrlib fixtures (CPU) ---------------------------------------------
@pytest.mark.parametrize("b", BATCHES, ids=_ids)
def test_oracle_group_fixture(b):
    fields = _fields(b)
    hb = gold.batch_from_records(fields, b["records"])
    assert hb.xdr_sizes(b["framed"]).tolist() == np.diff(b["rec_offsets"]).tolist()
    rc, xdr, offs = oracle.encode_batch(fields, hb.columns(), hb.n, hb.xdr_total(b["framed"]),
                                        framed=b["framed"])
    assert rc == 0
    assert xdr.hex() == b["xdr"]
    assert offs.tolist() == b["rec_offsets"]
    out = HostBatch.empty(fields, hb.n, hb.dyn_caps())
    rc, fb, err = oracle.decode_batch(fields, xdr, offs, hb.n, out.columns(), framed=b["framed"])
    assert (rc, fb, err) == (0, hb.n, 0)
    assert out.equal(hb)


PMAP = [(G, LS, 0, 4), (I, SC, 0), (I, SC, 0), (I, SC, 0), (I, SC, 0)]
ITEMS = [(I, SC, 0), (G, DY, 0, 2), (I, SC, 0), (STR, DY, 0), (I, SC, 0)]


def _decode(fields, xdr, n=1, caps=None):
    out = HostBatch.empty(fields, n, caps or {k: 64 for k in range(len(fields))})
    offs = _offs([0, len(xdr)]) if n == 1 else None
    return oracle.decode_batch(fields, xdr, offs, n, out.columns()), out


ERROR_CASES = [
    # count -2: new item[-2] -> NegativeArraySizeException (jrpcgen.java:886-906)
    ("negative_count", ITEMS, "00000001" "fffffffe", abi.E_NEG_SIZE),
    # count 2, one element present -> the second element's int is short
    ("short_element", ITEMS, "00000001" "00000002" "00000007" "00000001" "61000000", abi.E_SHORT),
    # element string length -1 -> checkArraySize (Xdr.java:1034-1037)
    ("corrupt_member", ITEMS, "00000001" "00000001" "00000007" "ffffffff", abi.E_CORRUPT),
    # a list whose closing bool is missing
    ("list_unterminated", PMAP, "00000001" "00000001" "00000002" "00000003" "00000004", abi.E_SHORT),
    # the count word itself missing
    ("missing_count", ITEMS, "00000001", abi.E_SHORT),
]


@pytest.mark.parametrize("name,fields,hexs,code", ERROR_CASES, ids=[c[0] for c in ERROR_CASES])
def test_oracle_group_errors(name, fields, hexs, code):
    (rc, fb, err), _ = _decode(fields, bytes.fromhex(hexs))
    assert (rc, fb, err) == (code, 0, code)


def test_oracle_list_bool_any_nonzero():
    """xdrDecodeBoolean: any non-zero word continues the list (Xdr.java:404-407)."""
    xdr = bytes.fromhex("00000007" "00000001" "00000002" "00000003" "00000004" "00000000")
    (rc, fb, err), out = _decode(PMAP, xdr)
    assert (rc, fb, err) == (0, 1, 0)
    assert out.arrays[0].tolist() == [0, 1] and out.arrays[4][0] == 4


def test_oracle_group_capacity_after_walk():
    """Capacity is reported only when the group's walk succeeds: a SHORT
    element wins over too few element slots."""
    xdr = bytes.fromhex("00000001" "00000003" + "00000007" "00000000" * 2)   # 3rd element short
    (rc, _, _), _ = _decode(ITEMS, xdr, caps={1: 1, 3: 8})
    assert rc == abi.E_SHORT
    xdr = bytes.fromhex("00000001" "00000002" + "00000007" "00000000" * 2 + "00000009")
    (rc, _, _), _ = _decode(ITEMS, xdr, caps={1: 1, 3: 8})
    assert rc == abi.E_CAPACITY


@pytest.mark.parametrize("fields", [
    [(G, DY, 0, 0), (I, SC, 0)],               # no members
    [(G, DY, 0, 3), (I, SC, 0)],               # members past the tape
    [(G, LS, 2, 1), (I, SC, 0)],               # a list has no count
    [(G, DY, 0, 2), (G, DY, 0, 1), (I, SC, 0)],   # nested group
    [(G, FX, 4, 1), (I, FX, 0)],               # elements of no bytes
])
def test_oracle_group_invalid(fields):
    hb = HostBatch.empty([(I, SC, 0)], 1)
    flat = [tuple(f) for f in fields]
    arr = oracle.fields_array(flat)
    cols = (oracle.Column * len(flat))()
    out = np.zeros(64, np.uint8)
    L = oracle.lib()
    rc = L.xo_encode_batch(arr, len(flat), __import__("ctypes").addressof(cols), 0, out.ctypes.data, 64,
                           None, 0, None)
    assert rc == abi.E_INVAL
    del hb


def test_oracle_group_random_roundtrip():
    fields = [(H, SC, 0), (G, DY, 0, 3), (U, SC, 0), (STR, DY, 0), (I, FX, 2),
              (G, LS, 0, 2), (B, SC, 0), (O, DY, 0), (I, DY, 0)]
    hb = random_batch(fields, 300, seed=11, dyn_len=(0, 9), group_len=(0, 6), special_floats=False)
    for framed in (False, True):
        rc, xdr, offs = oracle.encode_batch(fields, hb.columns(), hb.n, hb.xdr_total(framed), framed=framed)
        assert rc == 0 and len(xdr) == hb.xdr_total(framed)
        out = HostBatch.empty(fields, hb.n, hb.dyn_caps())
        rc, fb, err = oracle.decode_batch(fields, xdr, offs, hb.n, out.columns(), framed=framed)
        assert (rc, fb, err) == (0, hb.n, 0)
        # bools decode as 0/1 (Xdr.java:404-407)
        want = hb.arrays[6].copy()
        hb2 = HostBatch(hb.fields, hb.n, list(hb.arrays))
        hb2.arrays[6] = (want != 0).astype(np.uint8)
        assert out.equal(hb2)
