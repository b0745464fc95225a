"""columns.py — native (columnar) record batches on the host and in HBM.

The reference encodes one XdrAble at a time (xdr/XdrAble.java:40,49); the
engine works on a batch of N records of one schema laid out as columns
(include/xdrg.h, xdrg_column):

* fixed field (SCALAR / FIXED): an array of shape (n,) or (n, count) —
  struct-of-arrays; or one field of an array-of-structs via (data, stride);
* dynamic field (T<> / opaque<> / string<>): (values, offsets[n+1]) —
  record i owns values[offsets[i]:offsets[i+1]].

HostBatch holds numpy arrays (fixtures, the oracle's host pointers);
DeviceBatch holds torch tensors in HBM (the engine's device pointers).
torch is only the device-memory allocator here.
"""
import ctypes

import numpy as np

from . import abi

NP_DTYPE = {
    abi.T_INT: np.int32, abi.T_UINT: np.uint32, abi.T_ENUM: np.int32, abi.T_BOOL: np.uint8,
    abi.T_HYPER: np.int64, abi.T_UHYPER: np.uint64, abi.T_FLOAT: np.float32,
    abi.T_DOUBLE: np.float64, abi.T_SHORT: np.int16, abi.T_BYTE: np.int8,
    abi.T_OPAQUE: np.uint8, abi.T_STRING: np.uint8,
}
# same-width integer view used to compare floats bit for bit
_BITS = {4: np.uint32, 8: np.uint64, 2: np.uint16, 1: np.uint8}


def pad4(n):
    return (4 - (n & 3)) & 3


def field_xdr_bytes(field, cnt=None):
    """XDR bytes of one field of one record (cnt = dynamic element count)."""
    t, k, c = field
    if k == abi.K_DYNAMIC:
        return 4 + (cnt + pad4(cnt) if abi.XDR_SIZE[t] == 1 else cnt * abi.XDR_SIZE[t])
    n = c if k == abi.K_FIXED else 1
    if t == abi.T_OPAQUE:
        return n + pad4(n)
    return n * abi.XDR_SIZE[t]


def _bits(a):
    a = np.ascontiguousarray(a)
    return a.view(_BITS[a.dtype.itemsize]) if a.dtype.kind == "f" else a


class HostBatch:
    """n records of `fields` as numpy columns."""

    def __init__(self, fields, n, arrays):
        self.fields = [tuple(f) for f in fields]
        self.n = int(n)
        self.arrays = arrays

    # ---- construction ----------------------------------------------------
    @classmethod
    def empty(cls, fields, n, dyn_caps=None):
        """Zeroed output columns for a decode; dyn_caps[k] = element capacity."""
        arrays = []
        for k, (t, kind, c) in enumerate(fields):
            dt = NP_DTYPE[t]
            if kind == abi.K_DYNAMIC:
                cap = (dyn_caps or {}).get(k, 0)
                arrays.append((np.zeros(max(cap, 1), dtype=dt), np.zeros(n + 1, dtype=np.uint64)))
            elif kind == abi.K_FIXED:
                arrays.append(np.zeros((n, c), dtype=dt))
            else:
                arrays.append(np.zeros(n, dtype=dt))
        return cls(fields, n, arrays)

    def columns(self):
        """ctypes xdrg_column array with HOST pointers (for the oracle)."""
        arr = (abi.Column * len(self.fields))()
        for k, (t, kind, c) in enumerate(self.fields):
            if kind == abi.K_DYNAMIC:
                vals, offs = self.arrays[k]
                arr[k].data = vals.ctypes.data
                arr[k].offsets = offs.ctypes.data
                arr[k].cap = vals.size
                arr[k].stride = 0
            else:
                a = self.arrays[k]
                arr[k].data = a.ctypes.data
                arr[k].stride = 0
                arr[k].offsets = None
                arr[k].cap = 0
        arr._keep = self.arrays  # keep the numpy buffers alive with the array
        return arr

    def dyn_caps(self):
        return {k: int(self.arrays[k][1][-1]) for k, f in enumerate(self.fields)
                if f[1] == abi.K_DYNAMIC}

    def xdr_sizes(self, framed=False):
        """Per-record XDR size (numpy uint64)."""
        s = np.full(self.n, 4 if framed else 0, dtype=np.uint64)
        for k, f in enumerate(self.fields):
            if f[1] == abi.K_DYNAMIC:
                offs = self.arrays[k][1].astype(np.uint64)
                cnt = offs[1:] - offs[:-1]
                if abi.XDR_SIZE[f[0]] == 1:
                    s += 4 + cnt + ((4 - (cnt & 3)) & 3)
                else:
                    s += 4 + cnt * abi.XDR_SIZE[f[0]]
            else:
                s += field_xdr_bytes(f)
        return s

    def xdr_total(self, framed=False):
        return int(self.xdr_sizes(framed).sum())

    def native_bytes(self):
        """Algorithmic native bytes of the batch (values actually present)."""
        tot = 0
        for k, f in enumerate(self.fields):
            if f[1] == abi.K_DYNAMIC:
                vals, offs = self.arrays[k]
                tot += int(offs[-1]) * vals.dtype.itemsize
            else:
                tot += self.arrays[k].nbytes
        return tot

    def record(self, i, k):
        """Value(s) of field k of record i."""
        f = self.fields[k]
        if f[1] == abi.K_DYNAMIC:
            vals, offs = self.arrays[k]
            return vals[int(offs[i]):int(offs[i + 1])]
        return self.arrays[k][i]

    def slice(self, lo, hi):
        """Records [lo, hi) as a new batch (dynamic offsets rebased)."""
        arrays = []
        for k, f in enumerate(self.fields):
            if f[1] == abi.K_DYNAMIC:
                vals, offs = self.arrays[k]
                a, b = int(offs[lo]), int(offs[hi])
                arrays.append((vals[a:b].copy(), (offs[lo:hi + 1] - offs[lo]).astype(np.uint64)))
            else:
                arrays.append(self.arrays[k][lo:hi].copy())
        return HostBatch(self.fields, hi - lo, arrays)

    def equal(self, other, upto=None):
        """Bit-exact equality of the first `upto` records (floats by bits)."""
        n = self.n if upto is None else upto
        for k, f in enumerate(self.fields):
            if f[1] == abi.K_DYNAMIC:
                va, oa = self.arrays[k]
                vb, ob = other.arrays[k]
                if not np.array_equal(oa[:n + 1], ob[:n + 1]):
                    return False
                e = int(oa[n])
                if not np.array_equal(_bits(va[:e]), _bits(vb[:e])):
                    return False
            else:
                if not np.array_equal(_bits(self.arrays[k][:n]), _bits(other.arrays[k][:n])):
                    return False
        return True


# ---- synthetic batches (seeded) -------------------------------------------
def random_batch(fields, n, seed, dyn_len=(0, 16), string_alphabet=b"abcdefghijklmnopqrstuvwxyz",
                 special_floats=True):
    """Seeded synthetic batch: ints uniform over their full range, floats as
    random bit patterns (NaNs with payloads included), bools 0/1/other
    non-zero bytes, dynamic lengths uniform in dyn_len (inclusive)."""
    rng = np.random.default_rng(seed)
    arrays = []
    for t, kind, c in fields:
        dt = np.dtype(NP_DTYPE[t])
        if kind == abi.K_DYNAMIC:
            lo, hi = dyn_len
            cnt = rng.integers(lo, hi + 1, size=n, dtype=np.uint64)
            offs = np.zeros(n + 1, dtype=np.uint64)
            np.cumsum(cnt, out=offs[1:])
            total = int(offs[-1])
            if t == abi.T_STRING:
                alpha = np.frombuffer(string_alphabet, dtype=np.uint8)
                vals = alpha[rng.integers(0, len(alpha), size=total)]
            else:
                vals = _random_values(rng, dt, total, t, special_floats)
            arrays.append((vals, offs))
        else:
            shape = (n, c) if kind == abi.K_FIXED else (n,)
            size = int(np.prod(shape))
            arrays.append(_random_values(rng, dt, size, t, special_floats).reshape(shape))
    return HostBatch(fields, n, arrays)


def _random_values(rng, dt, size, t, special_floats):
    raw = rng.integers(0, 256, size=size * dt.itemsize, dtype=np.uint8)
    v = raw.view(dt).copy() if size else np.zeros(0, dtype=dt)
    if t == abi.T_BOOL:
        v = np.where(rng.random(size) < 0.25, v, (v & 1)).astype(np.uint8)
    if dt.kind == "f" and special_floats and size:
        u = v.view(_BITS[dt.itemsize])
        sp = (np.array([0x7fc00000, 0x7f800001, 0xffc00001, 0x7f800000, 0xff800000, 0, 0x80000000],
                       dtype=np.uint32) if dt.itemsize == 4 else
              np.array([0x7ff8000000000000, 0x7ff0000000000001, 0xfff8000000000123,
                        0x7ff0000000000000, 0xfff0000000000000, 0, 0x8000000000000000],
                       dtype=np.uint64))
        pick = rng.random(size) < 0.1
        u[pick] = sp[rng.integers(0, len(sp), size=int(pick.sum()))]
    return v


# ---- device batches (torch HBM) --------------------------------------------
_TORCH_DTYPE = None


def _torch_dtype(np_dt):
    import torch
    global _TORCH_DTYPE
    if _TORCH_DTYPE is None:
        _TORCH_DTYPE = {
            np.dtype(np.int32): torch.int32, np.dtype(np.uint32): torch.int32,
            np.dtype(np.int64): torch.int64, np.dtype(np.uint64): torch.int64,
            np.dtype(np.float32): torch.int32, np.dtype(np.float64): torch.int64,
            np.dtype(np.int16): torch.int16, np.dtype(np.int8): torch.int8,
            np.dtype(np.uint8): torch.uint8,
        }
    return _TORCH_DTYPE[np.dtype(np_dt)]


def _signed_view(a):
    """numpy array -> same-bits array of a torch-supported dtype."""
    a = np.ascontiguousarray(a)
    m = {np.dtype(np.uint32): np.int32, np.dtype(np.uint64): np.int64,
         np.dtype(np.float32): np.int32, np.dtype(np.float64): np.int64}
    return a.view(m[a.dtype]) if a.dtype in m else a


class DeviceBatch:
    """n records of `fields` as torch tensors in HBM (same structure as HostBatch)."""

    def __init__(self, fields, n, tensors, np_dtypes):
        self.fields = [tuple(f) for f in fields]
        self.n = int(n)
        self.tensors = tensors
        self._np = np_dtypes

    @classmethod
    def from_host(cls, hb, device="cuda"):
        import torch
        tensors, dts = [], []
        for k, f in enumerate(hb.fields):
            if f[1] == abi.K_DYNAMIC:
                vals, offs = hb.arrays[k]
                tv = torch.from_numpy(_signed_view(vals if vals.size else np.zeros(1, vals.dtype)))
                to = torch.from_numpy(offs.astype(np.uint64).view(np.int64))
                tensors.append((tv.to(device), to.to(device)))
                dts.append(vals.dtype)
            else:
                a = hb.arrays[k]
                tensors.append(torch.from_numpy(_signed_view(a)).to(device))
                dts.append(a.dtype)
        return cls(hb.fields, hb.n, tensors, dts)

    @classmethod
    def empty(cls, fields, n, dyn_caps=None, device="cuda"):
        import torch
        tensors, dts = [], []
        for k, (t, kind, c) in enumerate(fields):
            dt = np.dtype(NP_DTYPE[t])
            tdt = _torch_dtype(dt)
            if kind == abi.K_DYNAMIC:
                cap = max((dyn_caps or {}).get(k, 0), 1)
                tensors.append((torch.zeros(cap, dtype=tdt, device=device),
                                torch.zeros(n + 1, dtype=torch.int64, device=device)))
            elif kind == abi.K_FIXED:
                tensors.append(torch.zeros((n, c), dtype=tdt, device=device))
            else:
                tensors.append(torch.zeros(n, dtype=tdt, device=device))
            dts.append(dt)
        return cls(fields, n, tensors, dts)

    def columns(self):
        """ctypes xdrg_column array with DEVICE pointers."""
        arr = (abi.Column * len(self.fields))()
        for k, f in enumerate(self.fields):
            if f[1] == abi.K_DYNAMIC:
                tv, to = self.tensors[k]
                arr[k].data = tv.data_ptr()
                arr[k].offsets = to.data_ptr()
                arr[k].cap = tv.numel()
                arr[k].stride = 0
            else:
                arr[k].data = self.tensors[k].data_ptr()
                arr[k].stride = 0
                arr[k].offsets = None
                arr[k].cap = 0
        arr._keep = self.tensors
        return arr

    def to_host(self):
        arrays = []
        for k, f in enumerate(self.fields):
            dt = self._np[k]
            if f[1] == abi.K_DYNAMIC:
                tv, to = self.tensors[k]
                vals = tv.cpu().numpy().view(dt)
                offs = to.cpu().numpy().view(np.uint64)
                arrays.append((vals, offs))
            else:
                arrays.append(self.tensors[k].cpu().numpy().view(dt))
        return HostBatch(self.fields, self.n, arrays)


def aos_columns(fields, base_ptr, record_bytes, field_offsets):
    """Columns of an array-of-structs: field k of record i at
    base + i*record_bytes + field_offsets[k] (a C struct array / direct
    ByteBuffer of packed records)."""
    arr = (abi.Column * len(fields))()
    for k in range(len(fields)):
        arr[k].data = base_ptr + field_offsets[k]
        arr[k].stride = record_bytes
        arr[k].offsets = None
        arr[k].cap = 0
    return arr


def xdr_word_offsets(fields):
    """Byte offset of every fixed field inside its XDR record (the AoS layout
    that is word-for-word the XDR record)."""
    offs, pos = [], 0
    for f in fields:
        offs.append(pos)
        pos += field_xdr_bytes(f) if f[1] != abi.K_DYNAMIC else 0
    return offs
