"""oracle.py — TEST INFRASTRUCTURE ONLY: ctypes binding of libxdr_oracle.so.

The plain-C CPU restatement of org.dcache.oncrpc4j.xdr.Xdr and of the
RFC 1831 record-mark framing (oracle/xdr_oracle.c cites the reference
file:line of every function).  Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import this module, and only as the checker
or the timed CPU baseline; the product package (oncrpc4j_amd) never does.
"""
import ctypes
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libxdr_oracle.so")

# mirrors include/xdrg.h (kept local so the oracle does not import the product)
OK, E_SHORT, E_CORRUPT, E_FIXED_LEN, E_CAPACITY, E_FRAME, E_INVAL = 0, 1, 2, 3, 4, 5, 6
E_INCOMPLETE = 9
E_NEG_SIZE = 10
FRAME_RM = 0x1


class Field(ctypes.Structure):
    _fields_ = [("type", ctypes.c_uint32), ("kind", ctypes.c_uint32),
                ("count", ctypes.c_uint32), ("reserved", ctypes.c_uint32)]


class Cond(ctypes.Structure):
    _fields_ = [("field", ctypes.c_uint32), ("disc", ctypes.c_uint32), ("negate", ctypes.c_uint32),
                ("nvalues", ctypes.c_uint32), ("values", ctypes.c_void_p)]


class Column(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("stride", ctypes.c_int64),
                ("offsets", ctypes.c_void_p), ("cap", ctypes.c_uint64)]


class XoStream(ctypes.Structure):
    _fields_ = [("buf", ctypes.c_void_p), ("cap", ctypes.c_size_t), ("pos", ctypes.c_size_t),
                ("limit", ctypes.c_size_t), ("in_use", ctypes.c_int), ("growable", ctypes.c_int)]


_P = ctypes.c_void_p
_U64 = ctypes.c_uint64
_SZ = ctypes.c_size_t
_PS = ctypes.POINTER(XoStream)
_PF = ctypes.POINTER(Field)
_PC = ctypes.c_void_p  # any ctypes xdrg_column array (passed by address)

_SIGS = {
    "xo_stream_alloc": (ctypes.c_int, [_PS, _SZ]),
    "xo_stream_wrap": (None, [_PS, _P, _SZ]),
    "xo_stream_free": (None, [_PS]),
    "xo_begin_encoding": (None, [_PS]),
    "xo_end_encoding": (None, [_PS]),
    "xo_begin_decoding": (None, [_PS]),
    "xo_end_decoding": (None, [_PS]),
    "xo_has_more_data": (ctypes.c_int, [_PS]),
    "xo_remaining": (_SZ, [_PS]),
    "xo_encode_int": (ctypes.c_int, [_PS, ctypes.c_int32]),
    "xo_encode_long": (ctypes.c_int, [_PS, ctypes.c_int64]),
    "xo_encode_float": (ctypes.c_int, [_PS, ctypes.c_float]),
    "xo_encode_double": (ctypes.c_int, [_PS, ctypes.c_double]),
    "xo_encode_boolean": (ctypes.c_int, [_PS, ctypes.c_int]),
    "xo_encode_opaque": (ctypes.c_int, [_PS, _P, _SZ, _SZ]),
    "xo_encode_dynamic_opaque": (ctypes.c_int, [_PS, _P, _SZ]),
    "xo_encode_string": (ctypes.c_int, [_PS, _P, _SZ]),
    "xo_encode_int_vector": (ctypes.c_int, [_PS, _P, _SZ]),
    "xo_encode_int_fixed_vector": (ctypes.c_int, [_PS, _P, _SZ, ctypes.c_int32]),
    "xo_decode_int": (ctypes.c_int, [_PS, ctypes.POINTER(ctypes.c_int32)]),
    "xo_decode_long": (ctypes.c_int, [_PS, ctypes.POINTER(ctypes.c_int64)]),
    "xo_decode_boolean": (ctypes.c_int, [_PS, ctypes.POINTER(ctypes.c_int)]),
    "xo_decode_opaque": (ctypes.c_int, [_PS, _P, _SZ]),
    "xo_decode_dynamic_opaque": (ctypes.c_int, [_PS, ctypes.POINTER(_P), ctypes.POINTER(_SZ)]),
    "xo_decode_int_vector": (ctypes.c_int, [_PS, _P, _SZ, ctypes.POINTER(_SZ)]),
    "xo_record_mark": (ctypes.c_uint32, [ctypes.c_uint32]),
    "xo_all_fragments_arrived": (ctypes.c_int, [_P, _SZ]),
    "xo_assemble": (ctypes.c_int, [_P, _SZ, _P, _SZ, ctypes.POINTER(_SZ), ctypes.POINTER(_SZ)]),
    "xo_frame_scan": (ctypes.c_int, [_P, _SZ, _P, _U64, ctypes.POINTER(_U64)]),
    "xo_fragment": (_SZ, [_P, _SZ, _SZ, _P, _SZ]),
    "xo_receive_batch": (ctypes.c_int, [_PF, _SZ, _P, _SZ, _P, _U64, _U64, _PC, _P, ctypes.POINTER(_U64),
                                        ctypes.POINTER(_U64), ctypes.POINTER(_U64), ctypes.POINTER(ctypes.c_int)]),
    "xo_encode_batch": (ctypes.c_int, [_PF, _SZ, _PC, _U64, _P, _U64, _P, ctypes.c_uint32, _P]),
    "xo_decode_batch": (ctypes.c_int, [_PF, _SZ, _P, _U64, _P, _U64, _PC, ctypes.c_uint32, _P, _P]),
    "xo_encode_batch_cond": (ctypes.c_int, [_PF, _SZ, _P, _SZ, _PC, _U64, _P, _U64, _P,
                                            ctypes.c_uint32, _P]),
    "xo_decode_batch_cond": (ctypes.c_int, [_PF, _SZ, _P, _SZ, _P, _U64, _P, _U64, _PC,
                                            ctypes.c_uint32, _P, _P]),
    "xo_encode_batch_shallow": (ctypes.c_int, [_PF, _SZ, _P, _SZ, _PC, _U64, _P, _U64, _P,
                                               ctypes.c_uint32, _P, ctypes.c_uint32, _P]),
    "xo_decode_batch_view": (ctypes.c_int, [_PF, _SZ, _P, _SZ, _P, _U64, _P, _U64, _PC,
                                            ctypes.c_uint32, _P, _P, ctypes.c_uint32, _P]),
    "xo_encode_batch_mt": (ctypes.c_int, [_PF, _SZ, _PC, _U64, _P, _U64, ctypes.c_uint32, _P,
                                          ctypes.c_int]),
    "xo_decode_batch_mt": (ctypes.c_int, [_PF, _SZ, _P, _U64, _U64, _PC, ctypes.c_uint32, _P, _P,
                                          ctypes.c_int]),
}

_LIB = None


def build():
    """Compile the restatement (oracle/Makefile); building the checker is not using it."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = L
    return _LIB


def fields_array(fields):
    """[(type, kind, count)] or, for a repeated group, (T_GROUP, kind, count, members)."""
    arr = (Field * len(fields))()
    for i, f in enumerate(fields):
        arr[i].type, arr[i].kind, arr[i].count = f[0], f[1], f[2]
        arr[i].reserved = f[3] if len(f) > 3 else 0
    return arr


def conds_array(conds):
    """[(field, disc, negate, [values])] -> (ctypes xdrg_cond array or None, keep-alive)."""
    if not conds:
        return None, None
    arr = (Cond * len(conds))()
    keep = []
    for i, (f, d, neg, vals) in enumerate(conds):
        v = (ctypes.c_int32 * max(len(vals), 1))(*vals)
        keep.append(v)
        arr[i].field, arr[i].disc, arr[i].negate, arr[i].nvalues = f, d, int(neg), len(vals)
        arr[i].values = ctypes.addressof(v)
    return arr, keep


def encode_batch(fields, cols, n, out_cap, framed=False, conds=None):
    """-> (status, xdr bytes, record offsets[n+1])"""
    import numpy as np
    L = lib()
    fa = fields_array(fields)
    ca, keep = conds_array(conds)
    out = np.zeros(max(out_cap, 1), dtype=np.uint8)
    offs = np.zeros(n + 1, dtype=np.uint64)
    out_len = _U64(0)
    rc = L.xo_encode_batch_cond(fa, len(fields), ca, len(conds or ()), ctypes.addressof(cols), n,
                                out.ctypes.data, out_cap, offs.ctypes.data,
                                FRAME_RM if framed else 0, ctypes.byref(out_len))
    del keep
    return rc, out[:out_len.value].tobytes() if rc == OK else b"", offs


def decode_batch(fields, xdr, rec_offsets, n, cols, framed=False, conds=None):
    """-> (status, first_bad, err); cols (host Column array) receives the values."""
    import numpy as np
    L = lib()
    fa = fields_array(fields)
    ca, keep = conds_array(conds)
    buf = np.frombuffer(xdr, dtype=np.uint8) if len(xdr) else np.zeros(1, np.uint8)
    fb = _U64(0)
    err = ctypes.c_int(0)
    ro = rec_offsets.ctypes.data if rec_offsets is not None else None
    rc = L.xo_decode_batch_cond(fa, len(fields), ca, len(conds or ()), buf.ctypes.data, len(xdr), ro,
                                n, ctypes.addressof(cols), FRAME_RM if framed else 0,
                                ctypes.byref(fb), ctypes.byref(err))
    del keep
    return rc, fb.value, err.value


def frame_scan(data, cap):
    import numpy as np
    L = lib()
    buf = np.frombuffer(data, dtype=np.uint8) if len(data) else np.zeros(1, np.uint8)
    offs = np.zeros(cap + 1, dtype=np.uint64)
    nm = _U64(0)
    rc = L.xo_frame_scan(buf.ctypes.data, len(data), offs.ctypes.data, cap, ctypes.byref(nm))
    return rc, offs[:nm.value + 1].tolist()


def receive_batch(fields, data, cap, cols, conds=None):
    """handleRead + per-message decode (xdrg_receive_batch's contract) ->
    (status, messages delivered, consumed bytes, message offsets, first_bad, err)."""
    import numpy as np
    L = lib()
    fa = fields_array(fields)
    ca, keep = conds_array(conds)
    buf = np.frombuffer(data, dtype=np.uint8) if len(data) else np.zeros(1, np.uint8)
    offs = np.zeros(len(data) // 4 + 2, dtype=np.uint64)
    nm, used, fb, err = _U64(0), _U64(0), _U64(0), ctypes.c_int(0)
    rc = L.xo_receive_batch(fa, len(fields), ca, len(conds or ()), buf.ctypes.data, len(data), cap,
                            ctypes.addressof(cols), offs.ctypes.data, ctypes.byref(nm), ctypes.byref(used),
                            ctypes.byref(fb), ctypes.byref(err))
    del keep
    return rc, nm.value, used.value, offs[:nm.value + 1].tolist(), fb.value, err.value


def fragment(payload, frag):
    """Re-fragment a payload into record-marked fragments of <= frag bytes."""
    import numpy as np
    L = lib()
    src = np.frombuffer(payload, dtype=np.uint8) if payload else np.zeros(1, np.uint8)
    cap = len(payload) + 4 * (len(payload) // frag + 1)
    out = np.zeros(cap, dtype=np.uint8)
    w = L.xo_fragment(src.ctypes.data, len(payload), frag, out.ctypes.data, cap)
    return out[:w].tobytes()


def encode_batch_shallow(fields, cols, n, out_cap, field, framed=False, conds=None):
    """-> (status, buffer bytes, record offsets[n+1], splice[n]) — xdrEncodeFileChunk form."""
    import numpy as np
    L = lib()
    fa = fields_array(fields)
    ca, keep = conds_array(conds)
    out = np.zeros(max(out_cap, 1), dtype=np.uint8)
    offs = np.zeros(n + 1, dtype=np.uint64)
    splice = np.zeros(max(n, 1), dtype=np.uint64)
    out_len = _U64(0)
    rc = L.xo_encode_batch_shallow(fa, len(fields), ca, len(conds or ()), ctypes.addressof(cols), n,
                                   out.ctypes.data, out_cap, offs.ctypes.data,
                                   FRAME_RM if framed else 0, ctypes.byref(out_len), field,
                                   splice.ctypes.data)
    del keep
    return rc, out[:out_len.value].tobytes() if rc == OK else b"", offs, splice[:n]


def decode_batch_view(fields, xdr, rec_offsets, n, cols, field, framed=False, conds=None):
    """-> (status, first_bad, err, payload_pos[n]) — xdrDecodeByteBuffer form."""
    import numpy as np
    L = lib()
    fa = fields_array(fields)
    ca, keep = conds_array(conds)
    buf = np.frombuffer(xdr, dtype=np.uint8) if len(xdr) else np.zeros(1, np.uint8)
    pos = np.zeros(max(n, 1), dtype=np.uint64)
    fb = _U64(0)
    err = ctypes.c_int(0)
    rc = L.xo_decode_batch_view(fa, len(fields), ca, len(conds or ()), buf.ctypes.data, len(xdr),
                                rec_offsets.ctypes.data, n, ctypes.addressof(cols),
                                FRAME_RM if framed else 0, ctypes.byref(fb), ctypes.byref(err),
                                field, pos.ctypes.data)
    del keep
    return rc, fb.value, err.value, pos[:n]
