"""ctypes mirror of include/xdrg.h — the C-ABI of libxdrgpu.so.

Constants and struct layouts here must match include/xdrg.h exactly; the
reference interface each one stands for is cited there.
"""
import ctypes

ABI_VERSION = 1

# status codes (include/xdrg.h; Xdr.java:1028-1037)
OK = 0
E_SHORT = 1
E_CORRUPT = 2
E_FIXED_LEN = 3
E_CAPACITY = 4
E_FRAME = 5
E_INVAL = 6
E_HIP = 7
E_NOMEM = 8
E_INCOMPLETE = 9
E_NEG_SIZE = 10

STATUS_NAMES = {
    OK: "OK", E_SHORT: "SHORT", E_CORRUPT: "CORRUPT", E_FIXED_LEN: "FIXED_LEN",
    E_CAPACITY: "CAPACITY", E_FRAME: "FRAME", E_INVAL: "INVAL", E_HIP: "HIP",
    E_NOMEM: "NOMEM", E_INCOMPLETE: "INCOMPLETE", E_NEG_SIZE: "NEG_SIZE",
}

# base types (rpcgen baseTypes, jrpcgen.java:608-618)
T_INT, T_UINT, T_ENUM, T_BOOL, T_HYPER, T_UHYPER = 1, 2, 3, 4, 5, 6
T_FLOAT, T_DOUBLE, T_SHORT, T_BYTE, T_OPAQUE, T_STRING = 7, 8, 9, 10, 11, 12
T_GROUP = 13   # repeated group: the next `reserved` fields are its members

# declaration kinds (JrpcgenDeclaration.java:64-81)
K_SCALAR, K_FIXED, K_DYNAMIC = 0, 1, 2
K_LIST = 3     # XDRG_T_GROUP only: recursive optional list (BE(1) + element ..., BE(0))

# flags
FRAME_RM = 0x1
ASYNC = 0x2
HOST_PTRS = 0x4     # every pointer of the call is host memory (staging ring, include/xdrg.h)
HOST_MAPPED = 0x8   # with HOST_PTRS: kernels access the registered host buffers in place
STRIDE_CONST = -(1 << 63)   # XDRG_STRIDE_CONST: every record reads element run 0 (encode only)
CTX_TIMING = 0x1
COPY_H2D, COPY_D2H, COPY_D2D = 1, 2, 3   # xdrg_copy kinds

# kernel ids for xdrg_ctx_kernel_stats
KERNEL_FIXED_ENCODE = 0
KERNEL_FIXED_DECODE = 1
KERNEL_VAR_SIZE = 2
KERNEL_VAR_SCAN = 3
KERNEL_VAR_ENCODE = 4
KERNEL_VAR_DECODE = 5
KERNEL_FRAME_SCAN = 6
KERNEL_COUNT = 7

RPC_LAST_FRAG = 0x80000000  # RpcMessageParserTCP.java:37
RPC_SIZE_MASK = 0x7FFFFFFF  # RpcMessageParserTCP.java:41

NATIVE_SIZE = {
    T_INT: 4, T_UINT: 4, T_ENUM: 4, T_FLOAT: 4, T_HYPER: 8, T_UHYPER: 8, T_DOUBLE: 8,
    T_SHORT: 2, T_BYTE: 1, T_BOOL: 1, T_OPAQUE: 1, T_STRING: 1,
}
XDR_SIZE = {
    T_INT: 4, T_UINT: 4, T_ENUM: 4, T_FLOAT: 4, T_HYPER: 8, T_UHYPER: 8, T_DOUBLE: 8,
    T_SHORT: 4, T_BYTE: 4, T_BOOL: 4, T_OPAQUE: 1, T_STRING: 1,
}


class Field(ctypes.Structure):
    _fields_ = [("type", ctypes.c_uint32), ("kind", ctypes.c_uint32),
                ("count", ctypes.c_uint32), ("reserved", ctypes.c_uint32)]


class Cond(ctypes.Structure):
    """xdrg_cond: field `field` present iff (value(disc) in values) != negate."""
    _fields_ = [("field", ctypes.c_uint32), ("disc", ctypes.c_uint32), ("negate", ctypes.c_uint32),
                ("nvalues", ctypes.c_uint32), ("values", ctypes.c_void_p)]


MAX_DISC = 8
MAX_CASES = 64


class Column(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("stride", ctypes.c_int64),
                ("offsets", ctypes.c_void_p), ("cap", ctypes.c_uint64)]


# every function include/xdrg.h declares: name -> (restype, argtypes)
_P = ctypes.c_void_p
_U64 = ctypes.c_uint64
_PU64 = ctypes.POINTER(ctypes.c_uint64)
FUNCTIONS = {
    "xdrg_abi_version": (ctypes.c_int, []),
    "xdrg_status_string": (ctypes.c_char_p, [ctypes.c_int]),
    "xdrg_last_error": (ctypes.c_char_p, [_P]),
    "xdrg_ctx_create": (ctypes.c_int, [ctypes.c_int, ctypes.c_uint32, ctypes.POINTER(_P)]),
    "xdrg_ctx_destroy": (ctypes.c_int, [_P]),
    "xdrg_ctx_set_stream": (ctypes.c_int, [_P, _P]),
    "xdrg_ctx_kernel_stats": (ctypes.c_int, [_P, ctypes.c_int, _PU64,
                                             ctypes.POINTER(ctypes.c_double)]),
    "xdrg_ctx_reset_stats": (ctypes.c_int, [_P]),
    "xdrg_ctx_host_staging": (ctypes.c_int, [_P, _U64, ctypes.c_uint32]),
    "xdrg_host_register": (ctypes.c_int, [_P, _P, _U64]),
    "xdrg_host_unregister": (ctypes.c_int, [_P, _P]),
    "xdrg_device_alloc": (ctypes.c_int, [_P, _U64, ctypes.POINTER(_P)]),
    "xdrg_device_free": (ctypes.c_int, [_P, _P]),
    "xdrg_copy": (ctypes.c_int, [_P, _P, _P, _U64, ctypes.c_int]),
    "xdrg_schema_create": (ctypes.c_int, [ctypes.POINTER(Field), ctypes.c_size_t,
                                          ctypes.POINTER(_P)]),
    "xdrg_schema_create_cond": (ctypes.c_int, [ctypes.POINTER(Field), ctypes.c_size_t,
                                               ctypes.POINTER(Cond), ctypes.c_size_t,
                                               ctypes.POINTER(_P)]),
    "xdrg_schema_destroy": (ctypes.c_int, [_P]),
    "xdrg_schema_fixed_size": (ctypes.c_uint64, [_P]),
    "xdrg_encode_batch": (ctypes.c_int, [_P, _P, ctypes.POINTER(Column), _U64, _P, _U64, _P,
                                         ctypes.c_uint32, _P]),
    "xdrg_decode_batch": (ctypes.c_int, [_P, _P, _P, _U64, _P, _U64, ctypes.POINTER(Column),
                                         ctypes.c_uint32, _P, _P]),
    "xdrg_encode_batch_shallow": (ctypes.c_int, [_P, _P, ctypes.POINTER(Column), _U64, _P, _U64, _P,
                                                 ctypes.c_uint32, _P, ctypes.c_uint32, _P]),
    "xdrg_decode_batch_view": (ctypes.c_int, [_P, _P, _P, _U64, _P, _U64, ctypes.POINTER(Column),
                                              ctypes.c_uint32, _P, _P, ctypes.c_uint32, _P]),
    "xdrg_frame_scan": (ctypes.c_int, [_P, _P, _U64, _P, _U64, _PU64]),
    "xdrg_deframe": (ctypes.c_int, [_P, _P, _U64, _P, _U64, _P, _U64, _PU64, _PU64]),
    "xdrg_frame_scan_ex": (ctypes.c_int, [_P, _P, _U64, _P, _U64, _PU64, _PU64, ctypes.c_uint32]),
    "xdrg_deframe_ex": (ctypes.c_int, [_P, _P, _U64, _P, _U64, _P, _U64, _PU64, _PU64, ctypes.c_uint32]),
    "xdrg_receive_batch": (ctypes.c_int, [_P, _P, _P, _U64, _U64, ctypes.POINTER(Column), ctypes.c_uint32, _P,
                                          _PU64, _PU64, _PU64, ctypes.POINTER(ctypes.c_int)]),
    "xdrg_encode_batch_multi": (ctypes.c_int, [_P, ctypes.c_uint32, _P, _P, _P, _P, _U64, _P,
                                               ctypes.c_uint32, _PU64]),
    "xdrg_decode_batch_multi": (ctypes.c_int, [_P, ctypes.c_uint32, _P, _P, _U64, _P, _P, _P,
                                               ctypes.c_uint32, _PU64, ctypes.POINTER(ctypes.c_int)]),
}


def bind(lib):
    """Attach restype/argtypes for every exported C-ABI function."""
    for name, (res, args) in FUNCTIONS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def pad4(n):
    """(4 - (len & 3)) & 3 — Xdr.java:777."""
    return (4 - (n & 3)) & 3
