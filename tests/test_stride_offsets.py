"""Fixed-size decode at explicit record extents (the receive pipeline: a frame
scan's offsets handed to xdrg_decode_batch).  When every extent is the fixed
stride the engine checks that on the device and takes the stride kernels
(tuning key 29 = 1, the default); otherwise, or with key 29 = 0, the record
path decodes each extent.  Both must equal the oracle's decode at the same
offsets (Xdr.java:1028-1037 error order), including streams that start past
byte 0, corrupted record marks, invalid values and short streams."""
import zlib

import numpy as np
import pytest

import oracle
from oncrpc4j_amd import abi, engine
from oncrpc4j_amd.columns import DeviceBatch, HostBatch, random_batch

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

I, B, H, F, D, O = abi.T_INT, abi.T_BOOL, abi.T_HYPER, abi.T_FLOAT, abi.T_DOUBLE, abi.T_OPAQUE
SC, FX = abi.K_SCALAR, abi.K_FIXED

SCHEMAS = {
    "cfg2_8xint": [(I, SC, 0)] * 8,
    "bool_hyper": [(I, SC, 0), (B, SC, 0), (H, SC, 0), (D, SC, 0)],
    "fixed_opaque": [(I, FX, 3), (O, FX, 5), (F, SC, 0)],
    "big_fixed": [(I, FX, 200), (O, FX, 37)],
}


@pytest.fixture(params=[1, 0], ids=["check", "record_path"])
def stride_check(request, gpu_ctx):
    gpu_ctx.tune(29, request.param)
    yield request.param
    gpu_ctx.tune(0)


def _stream(fields, n, framed, seed, lead):
    hb = random_batch(fields, n, seed=seed)
    rc, xdr, ro = oracle.encode_batch(fields, hb.columns(), n, hb.xdr_total(framed) + 8, framed=framed)
    assert rc == 0
    return hb, b"\xa5" * lead + xdr, ro.astype(np.uint64) + np.uint64(lead)


def _both(ctx, fields, x, in_len, ro, n, framed):
    sch = engine.Schema(fields)
    caps = {}
    db = DeviceBatch.empty(fields, n, caps)
    buf = torch.from_numpy(np.frombuffer(x, np.uint8).copy()).cuda()
    dro = torch.from_numpy(ro.view(np.int64).copy()).cuda()
    st = ctx.decode(sch, buf, in_len, n, db.columns(), rec_offsets=dro, framed=framed, raise_on_error=False)
    ref = HostBatch.empty(fields, n, caps)
    rst = oracle.decode_batch(fields, x[:in_len], ro, n, ref.columns(), framed=framed)
    return st, rst, db.to_host(), ref


@pytest.mark.parametrize("framed", [False, True], ids=["raw", "rm"])
@pytest.mark.parametrize("lead", [0, 12])
@pytest.mark.parametrize("n", [1, 2049, 70001])
@pytest.mark.parametrize("name", sorted(SCHEMAS))
def test_uniform_extents(gpu_ctx, stride_check, name, n, lead, framed):
    fields = SCHEMAS[name]
    hb, x, ro = _stream(fields, n, framed, zlib.crc32(f"{name}/{n}/{lead}".encode()), lead)
    st, rst, got, ref = _both(gpu_ctx, fields, x, len(x), ro, n, framed)
    assert st == rst == (0, n, 0)
    assert got.equal(ref)


@pytest.mark.parametrize("framed", [False, True], ids=["raw", "rm"])
@pytest.mark.parametrize("name", sorted(SCHEMAS))
def test_extent_errors(gpu_ctx, stride_check, name, framed):
    """Non-uniform extents, a bad mark / value inside one record, a short
    stream: same first bad record, code and earlier values as the oracle."""
    fields = SCHEMAS[name]
    n = 5000
    hb, x, ro = _stream(fields, n, framed, 7, 8)
    rng = np.random.default_rng(zlib.crc32(name.encode()))
    r = int(rng.integers(1, n - 1))
    cases = []
    # one extent 4 bytes longer (record r followed by a stray word), the rest shifted
    y = x[:int(ro[r + 1])] + b"\x00\x00\x00\x00" + x[int(ro[r + 1]):]
    ro2 = ro.copy()
    ro2[r + 1:] += np.uint64(4)
    cases.append(("longer_extent", y, len(y), ro2))
    # the stream ends inside record r
    cases.append(("short", x, int(ro[r]) + 4, ro))
    # the first word of record r changed: a record mark (rm) or the first value (raw)
    y = bytearray(x)
    y[int(ro[r]):int(ro[r]) + 4] = b"\x7f\x00\x00\x09"
    cases.append(("first_word", bytes(y), len(y), ro))
    if name == "bool_hyper":   # an invalid bool
        y = bytearray(x)
        p = int(ro[r]) + (4 if framed else 0) + 4
        y[p:p + 4] = b"\x00\x00\x00\x02"
        cases.append(("bad_bool", bytes(y), len(y), ro))
    for what, y, in_len, offs in cases:
        st, rst, got, ref = _both(gpu_ctx, fields, y, in_len, offs, n, framed)
        assert st == rst, (what, st, rst)
        assert got.equal(ref, upto=st[1]), what
