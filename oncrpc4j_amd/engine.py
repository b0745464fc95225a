"""engine.py — Python host binding of libxdrgpu.so (the C-ABI of include/xdrg.h).

This is the drop-in boundary seen from Python: the same entry points a JNI or
Panama shim in oncrpc4j-core binds.  The library is the only
compute path; if it is missing or no GPU is present the calls raise — there is
no CPU fallback.

Error mapping mirrors the reference: XDRG_E_SHORT / XDRG_E_CORRUPT raise
BadXdrOncRpcException with the reference's messages (xdr/Xdr.java:1028-1037,
xdr/BadXdrOncRpcException.java:24), XDRG_E_FIXED_LEN raises ValueError
(IllegalArgumentException, Xdr.java:625-627).
"""
import ctypes
import os

from . import abi

# XDRG_LIBRARY: another build of the same C-ABI (measurement tools A/B kernel variants)
LIB_PATH = os.environ.get("XDRG_LIBRARY") or os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                          "libxdrgpu.so")

_LIB = None



def lib():
    """Load libxdrgpu.so (raises if it has not been built)."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                "libxdrgpu.so is not built (run `python -c 'import __graft_entry__ as g; g.build()'`)")
        _LIB = abi.bind(ctypes.CDLL(LIB_PATH))
        # not in include/xdrg.h: per-context kernel choices (xdrg_internal.h Tuning)
        _LIB.xdrg_internal_tune.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong]
        _LIB.xdrg_internal_tune.restype = ctypes.c_int
        _LIB.xdrg_internal_stat.argtypes = [ctypes.c_void_p, ctypes.c_int]
        _LIB.xdrg_internal_stat.restype = ctypes.c_longlong
        v = _LIB.xdrg_abi_version()
        if v != abi.ABI_VERSION:
            raise RuntimeError(f"libxdrgpu.so ABI {v} != {abi.ABI_VERSION}")
    return _LIB


class XdrgError(Exception):
    """A non-OK engine status.  .code = XDRG_E_*, .first_bad = record index."""

    def __init__(self, code, msg, first_bad=None):
        super().__init__(msg)
        self.code = code
        self.first_bad = first_bad


class BadXdrOncRpcException(XdrgError, IOError):
    """org.dcache.oncrpc4j.xdr.BadXdrOncRpcException (an IOException)."""


class CapacityError(XdrgError):
    pass


class NegativeArraySizeException(XdrgError):
    """java.lang.NegativeArraySizeException: an array of structs decoded with a
    negative count (rpcgen's `new T[xdr.xdrDecodeInt()]`, jrpcgen.java:886-906)."""


def _raise(code, ctx=None, first_bad=None):
    L = lib()
    msg = L.xdrg_status_string(code).decode()
    if ctx is not None:
        detail = L.xdrg_last_error(ctx).decode()
        if detail and detail != msg:
            msg = f"{msg} ({detail})"
    if code in (abi.E_SHORT, abi.E_CORRUPT):
        raise BadXdrOncRpcException(code, msg, first_bad)
    if code == abi.E_FIXED_LEN:
        raise ValueError(msg)
    if code == abi.E_NEG_SIZE:
        raise NegativeArraySizeException(code, msg, first_bad)
    if code == abi.E_CAPACITY:
        raise CapacityError(code, msg, first_bad)
    raise XdrgError(code, msg, first_bad)


class Schema:
    """A compiled field tape (rpcgen struct body).  fields: [(type, kind, count)].

    conds: optional [(field, disc, negate, [case values])] — rpcgen unions and
    optional data (include/xdrg.h xdrg_cond): field `field` is present iff
    field `disc` is and (value(disc) in values) != negate."""

    def __init__(self, fields, conds=None):
        self.fields = [tuple(int(x) for x in f) for f in fields]
        self.conds = [(int(f), int(d), int(n), [int(v) for v in vals])
                      for f, d, n, vals in (conds or ())]
        arr = (abi.Field * len(self.fields))()
        for i, f in enumerate(self.fields):   # (type, kind, count[, members of a group])
            arr[i].type, arr[i].kind, arr[i].count = f[0], f[1], f[2]
            arr[i].reserved = f[3] if len(f) > 3 else 0
        h = ctypes.c_void_p()
        if self.conds:
            ca = (abi.Cond * len(self.conds))()
            keep = []
            for i, (f, d, n, vals) in enumerate(self.conds):
                v = (ctypes.c_int32 * max(len(vals), 1))(*vals)
                keep.append(v)
                ca[i].field, ca[i].disc, ca[i].negate, ca[i].nvalues = f, d, int(n), len(vals)
                ca[i].values = ctypes.addressof(v)
            rc = lib().xdrg_schema_create_cond(arr, len(self.fields), ca, len(self.conds),
                                               ctypes.byref(h))
        else:
            rc = lib().xdrg_schema_create(arr, len(self.fields), ctypes.byref(h))
        if rc:
            _raise(rc)
        self._h = h

    @property
    def handle(self):
        return self._h

    @property
    def fixed_size(self):
        """XDR bytes per record for fixed-size schemas, 0 otherwise."""
        return int(lib().xdrg_schema_fixed_size(self._h))

    @property
    def is_fixed(self):
        return not self.conds and all(f[1] != abi.K_DYNAMIC and f[0] != abi.T_GROUP for f in self.fields)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and _LIB is not None:
            _LIB.xdrg_schema_destroy(h)
            self._h = None


def _ptr(x):
    """Address of a torch tensor, a numpy array, an int or None."""
    if x is None:
        return None
    if isinstance(x, int):
        return x
    if hasattr(x, "data_ptr"):
        return x.data_ptr()
    return x.ctypes.data


def host_register(ptr, nbytes, ctx=None):
    """xdrg_host_register: pin (and map) a host buffer once, as a caller's
    pooled direct buffers would be; registered spans skip the staging
    ring's bounce copy and may take mapped=True."""
    rc = lib().xdrg_host_register(ctx.handle if ctx is not None else None, _ptr(ptr), int(nbytes))
    if rc:
        _raise(rc, ctx.handle if ctx is not None else None)


def host_unregister(ptr, ctx=None):
    rc = lib().xdrg_host_unregister(ctx.handle if ctx is not None else None, _ptr(ptr))
    if rc:
        _raise(rc, ctx.handle if ctx is not None else None)


def columns_array(cols):
    """[(data, stride, offsets, cap)] -> ctypes xdrg_column array."""
    arr = (abi.Column * len(cols))()
    for i, (data, stride, offsets, cap) in enumerate(cols):
        arr[i].data = _ptr(data)
        arr[i].stride = int(stride)
        arr[i].offsets = _ptr(offsets)
        arr[i].cap = int(cap)
    return arr


class Context:
    """xdrg_ctx: one device, one stream, its own workspace (Xdr.java:56,71:
    one owner at a time — use one Context per thread)."""

    def __init__(self, device=0, timing=False):
        L = lib()
        h = ctypes.c_void_p()
        rc = L.xdrg_ctx_create(int(device), abi.CTX_TIMING if timing else 0, ctypes.byref(h))
        if rc:
            _raise(rc)
        self._h = h
        self.device = device

    @property
    def handle(self):
        return self._h

    def set_stream(self, stream):
        """stream: a torch.cuda.Stream, a raw hipStream_t (int) or None."""
        raw = getattr(stream, "cuda_stream", stream)
        rc = lib().xdrg_ctx_set_stream(self._h, raw)
        if rc:
            _raise(rc, self._h)

    def host_staging(self, slot_bytes, slots):
        """xdrg_ctx_host_staging: the ring the host=True calls move through."""
        rc = lib().xdrg_ctx_host_staging(self._h, int(slot_bytes), int(slots))
        if rc:
            _raise(rc, self._h)

    @staticmethod
    def _flags(framed, async_, host, mapped):
        return ((abi.FRAME_RM if framed else 0) | (abi.ASYNC if async_ else 0) |
                (abi.HOST_PTRS if host or mapped else 0) | (abi.HOST_MAPPED if mapped else 0))

    def encode(self, schema, cols, n, out, out_cap, rec_offsets=None, framed=False, async_=False,
               out_len=None, host=False, mapped=False):
        """xdrg_encode_batch -> bytes written (sync mode).  host=True: every
        pointer is host memory (XDRG_HOST_PTRS, the staging ring); mapped=True:
        registered host memory accessed in place (XDRG_HOST_MAPPED)."""
        flags = self._flags(framed, async_, host, mapped)
        carr = cols if isinstance(cols, ctypes.Array) else columns_array(cols)
        ol = ctypes.c_uint64(0)
        olp = _ptr(out_len) if async_ else ctypes.addressof(ol)
        rc = lib().xdrg_encode_batch(self._h, schema.handle, carr, int(n), _ptr(out), int(out_cap),
                                     _ptr(rec_offsets), flags, olp)
        if rc:
            _raise(rc, self._h)
        return None if async_ else ol.value

    def decode(self, schema, xdr, xdr_len, n, cols, rec_offsets=None, framed=False, async_=False,
               first_bad=None, err=None, raise_on_error=True, host=False, mapped=False):
        """xdrg_decode_batch -> (status, first_bad, err) in sync mode (host /
        mapped as for encode)."""
        flags = self._flags(framed, async_, host, mapped)
        carr = cols if isinstance(cols, ctypes.Array) else columns_array(cols)
        fb = ctypes.c_uint64(0)
        er = ctypes.c_int(0)
        fbp = _ptr(first_bad) if async_ else ctypes.addressof(fb)
        erp = _ptr(err) if async_ else ctypes.addressof(er)
        rc = lib().xdrg_decode_batch(self._h, schema.handle, _ptr(xdr), int(xdr_len),
                                     _ptr(rec_offsets), int(n), carr, flags, fbp, erp)
        if rc and raise_on_error:
            _raise(rc, self._h, None if async_ else fb.value)
        return rc, (None if async_ else fb.value), (None if async_ else er.value)

    def encode_shallow(self, schema, cols, n, out, out_cap, field, splice, rec_offsets=None,
                       framed=False, host=False, mapped=False):
        """xdrg_encode_batch_shallow: field `field` travels by reference
        (xdrEncodeFileChunk, Xdr.java:978-988); splice[i] = where record i's
        payload + zero pad go in its message.  -> bytes written to out.
        host / mapped as for encode (the payload's values never cross)."""
        flags = self._flags(framed, False, host, mapped)
        carr = cols if isinstance(cols, ctypes.Array) else columns_array(cols)
        ol = ctypes.c_uint64(0)
        rc = lib().xdrg_encode_batch_shallow(self._h, schema.handle, carr, int(n), _ptr(out),
                                             int(out_cap), _ptr(rec_offsets), flags,
                                             ctypes.addressof(ol), int(field), _ptr(splice))
        if rc:
            _raise(rc, self._h)
        return ol.value

    def decode_view(self, schema, xdr, xdr_len, n, cols, field, payload_pos, rec_offsets=None,
                    framed=False, raise_on_error=True, host=False, mapped=False):
        """xdrg_decode_batch_view: field `field` decodes as a stream slice
        (xdrDecodeByteBuffer, Xdr.java:423-439) -> (status, first_bad, err).
        host / mapped as for decode."""
        flags = self._flags(framed, False, host, mapped)
        carr = cols if isinstance(cols, ctypes.Array) else columns_array(cols)
        fb = ctypes.c_uint64(0)
        er = ctypes.c_int(0)
        rc = lib().xdrg_decode_batch_view(self._h, schema.handle, _ptr(xdr), int(xdr_len),
                                          _ptr(rec_offsets), int(n), carr, flags,
                                          ctypes.addressof(fb), ctypes.addressof(er), int(field),
                                          _ptr(payload_pos))
        if rc and raise_on_error:
            _raise(rc, self._h, fb.value)
        return rc, fb.value, er.value

    def device_alloc(self, nbytes):
        """xdrg_device_alloc -> device address (int); free with device_free."""
        p = ctypes.c_void_p()
        rc = lib().xdrg_device_alloc(self._h, int(nbytes), ctypes.byref(p))
        if rc:
            _raise(rc, self._h)
        return p.value

    def device_free(self, ptr):
        rc = lib().xdrg_device_free(self._h, _ptr(ptr))
        if rc:
            _raise(rc, self._h)

    def copy(self, dst, src, nbytes, kind):
        """xdrg_copy (kind: abi.COPY_H2D / COPY_D2H / COPY_D2D), synchronous."""
        rc = lib().xdrg_copy(self._h, _ptr(dst), _ptr(src), int(nbytes), int(kind))
        if rc:
            _raise(rc, self._h)

    def frame_scan(self, data, length, msg_offsets, cap, host=False, mapped=False, with_consumed=False):
        """xdrg_frame_scan (device) / xdrg_frame_scan_ex (host=True: a host socket
        buffer through the staging ring, mapped=True: registered host memory in
        place) -> number of complete messages (0 = STOP), or (messages,
        consumed) with with_consumed."""
        nm = ctypes.c_uint64(0)
        used = ctypes.c_uint64(0)
        if host or mapped or with_consumed:
            rc = lib().xdrg_frame_scan_ex(self._h, _ptr(data), int(length), _ptr(msg_offsets), int(cap),
                                          ctypes.byref(nm), ctypes.byref(used), self._flags(False, False, host, mapped))
        else:
            rc = lib().xdrg_frame_scan(self._h, _ptr(data), int(length), _ptr(msg_offsets), int(cap),
                                       ctypes.byref(nm))
        if rc not in (abi.OK, abi.E_INCOMPLETE):
            _raise(rc, self._h)
        return (nm.value, used.value) if with_consumed else nm.value

    def deframe(self, data, length, payload, payload_cap, msg_offsets, cap, host=False, mapped=False,
                raise_on_error=True):
        """xdrg_deframe / xdrg_deframe_ex -> (messages, consumed stream bytes);
        (0, 0) = STOP.  On host memory a payload that fills up delivers the
        bodies that fit (XDRG_E_CAPACITY, raised unless raise_on_error=False:
        then (messages, consumed, status))."""
        nm = ctypes.c_uint64(0)
        used = ctypes.c_uint64(0)
        if host or mapped:
            rc = lib().xdrg_deframe_ex(self._h, _ptr(data), int(length), _ptr(payload), int(payload_cap),
                                       _ptr(msg_offsets), int(cap), ctypes.byref(nm), ctypes.byref(used),
                                       self._flags(False, False, host, mapped))
        else:
            rc = lib().xdrg_deframe(self._h, _ptr(data), int(length), _ptr(payload), int(payload_cap),
                                    _ptr(msg_offsets), int(cap), ctypes.byref(nm), ctypes.byref(used))
        if not raise_on_error:
            return nm.value, used.value, rc
        if rc not in (abi.OK, abi.E_INCOMPLETE):
            _raise(rc, self._h)
        return nm.value, used.value

    def receive(self, schema, data, length, cap, cols, msg_offsets=None, host=False, mapped=False,
                raise_on_error=True):
        """xdrg_receive_batch: RpcMessageParserTCP.handleRead over a socket
        buffer plus the decode of every complete message as one record ->
        (status, messages delivered, consumed bytes, first_bad, err)."""
        carr = cols if isinstance(cols, ctypes.Array) else columns_array(cols)
        nm, used, fb = ctypes.c_uint64(0), ctypes.c_uint64(0), ctypes.c_uint64(0)
        er = ctypes.c_int(0)
        rc = lib().xdrg_receive_batch(self._h, schema.handle, _ptr(data), int(length), int(cap), carr,
                                      self._flags(False, False, host, mapped), _ptr(msg_offsets),
                                      ctypes.byref(nm), ctypes.byref(used), ctypes.byref(fb), ctypes.byref(er))
        if rc and rc != abi.E_INCOMPLETE and raise_on_error:
            _raise(rc, self._h, fb.value)
        return rc, nm.value, used.value, fb.value, er.value

    def apply_tuning(self, spec):
        """Measurement tools only (bench.py, tools/): force kernel choices from
        a "key=value,key=value" string such as the XDRG_TUNE variable those
        tools read.  A context never reads the environment by itself."""
        for kv in filter(None, (x.strip() for x in (spec or "").split(","))):
            k, sep, v = kv.partition("=")
            try:
                if not sep:
                    raise ValueError
                key, value = int(k), int(v)
            except ValueError:
                raise ValueError(f"tuning entry {kv!r}: expected key=value with integers") from None
            self.tune(key, value)

    def tune(self, key, value=0):
        """Force one of this context's kernel choices (xdrg_internal.h Tuning:
        the parity tests run every production path; key 0 restores the
        defaults).  Not part of the drop-in boundary."""
        rc = lib().xdrg_internal_tune(self._h, int(key), int(value))
        if rc:
            raise ValueError(f"tuning key {key} = {value} rejected")

    def internal_stat(self, key):
        """Internal counters (xdrg_internal_stat: 1 speculative frame walks,
        2 of them walked again by the exact kernels, 3 super-chunks re-walked
        by their fix-up, 4 host-memory calls bounced whole through device
        scratch, 5 host receives taken in three passes).  Not part of the drop-in boundary."""
        return int(lib().xdrg_internal_stat(self._h, int(key)))

    def kernel_stats(self, kernel):
        """-> (launches, total_ms) for one XDRG_KERNEL_* id (needs timing=True)."""
        n = ctypes.c_uint64(0)
        ms = ctypes.c_double(0)
        lib().xdrg_ctx_kernel_stats(self._h, int(kernel), ctypes.byref(n), ctypes.byref(ms))
        return n.value, ms.value

    def reset_stats(self):
        lib().xdrg_ctx_reset_stats(self._h)

    def close(self):
        if getattr(self, "_h", None) is not None:
            lib().xdrg_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


# ---- multi-GPU, one process (xdrg_encode_batch_multi / xdrg_decode_batch_multi) ----
def _ptr_array(ctype, items):
    arr = (ctype * len(items))()
    for i, x in enumerate(items):
        arr[i] = _ptr(x) if not isinstance(x, ctypes.Array) else ctypes.addressof(x)
    return arr


def encode_multi(ctxs, schema, cols, counts, outs, out_cap, rec_offsets=None, framed=False):
    """Shard-parallel encode + xGMI all-gather over len(ctxs) contexts ->
    stream bytes; every outs[i] then holds the whole stream."""
    k = len(ctxs)
    carrs = [c if isinstance(c, ctypes.Array) else columns_array(c) for c in cols]
    ol = ctypes.c_uint64(0)
    ro = _ptr_array(ctypes.c_void_p, rec_offsets) if rec_offsets is not None else None
    rc = lib().xdrg_encode_batch_multi(_ptr_array(ctypes.c_void_p, [c.handle.value for c in ctxs]), k,
                                       schema.handle, _ptr_array(ctypes.c_void_p, carrs),
                                       (ctypes.c_uint64 * k)(*counts), _ptr_array(ctypes.c_void_p, outs),
                                       int(out_cap), ro, abi.FRAME_RM if framed else 0, ctypes.byref(ol))
    if rc:
        _raise(rc, ctxs[0].handle)
    return ol.value


def decode_multi(ctxs, schema, ins, in_len, counts, cols, rec_offsets=None, framed=False,
                 raise_on_error=True):
    """Shard-parallel decode -> (status, first_bad, err) over the whole batch."""
    k = len(ctxs)
    carrs = [c if isinstance(c, ctypes.Array) else columns_array(c) for c in cols]
    fb = ctypes.c_uint64(0)
    er = ctypes.c_int(0)
    ro = _ptr_array(ctypes.c_void_p, rec_offsets) if rec_offsets is not None else None
    rc = lib().xdrg_decode_batch_multi(_ptr_array(ctypes.c_void_p, [c.handle.value for c in ctxs]), k,
                                       schema.handle, _ptr_array(ctypes.c_void_p, ins), int(in_len), ro,
                                       (ctypes.c_uint64 * k)(*counts), _ptr_array(ctypes.c_void_p, carrs),
                                       abi.FRAME_RM if framed else 0, ctypes.byref(fb), ctypes.byref(er))
    if rc and raise_on_error:
        _raise(rc, ctxs[0].handle, fb.value)
    return rc, fb.value, er.value
