"""columns.py — native (columnar) record batches on the host and in HBM.

The reference encodes one XdrAble at a time (xdr/XdrAble.java:40,49); the
engine works on a batch of N records of one schema laid out as columns
(include/xdrg.h, xdrg_column):

* fixed field (SCALAR / FIXED): an array of shape (n,) or (n, count) —
  struct-of-arrays; or one field of an array-of-structs via (data, stride);
* dynamic field (T<> / opaque<> / string<>): (values, offsets[n+1]) —
  record i owns values[offsets[i]:offsets[i+1]].

* repeated group (array of structs / linked list, include/xdrg.h): the field
  tuple is (T_GROUP, kind, count, members) and the next `members` fields are
  its members; the group's array is offsets[n+1] (element ranges; None for
  a FIXED group: record i owns elements i*count ...), and every member array
  is indexed by ELEMENT (fixed: (E,) / (E, count); dynamic: (values,
  offsets[E+1])).  A member may itself be a group (up to four group levels
  in all, its members counted in the outer `members`): its array is indexed
  by the enclosing group's elements (offsets[E+1]) and its own members by
  its elements.

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


def parents(fields):
    """parent[k] = index of the group field k is an immediate member of, or -1
    (an inner group claims its own members after its parent's span)."""
    par = [-1] * len(fields)
    for k, f in enumerate(fields):
        if f[0] == abi.T_GROUP:
            for j in range(1, f[3] + 1):
                par[k + j] = k
    return par


def direct_members(fields, g):
    """Indices of group g's immediate members (an inner group's members skipped)."""
    out, j = [], g + 1
    while j <= g + fields[g][3]:
        out.append(j)
        j += 1 + (fields[j][3] if fields[j][0] == abi.T_GROUP else 0)
    return out


def _is_group(f):
    return f[0] == abi.T_GROUP


def _counted(f):
    """Fields whose array carries offsets: dynamic fields, DYNAMIC / LIST groups."""
    return f[1] == abi.K_DYNAMIC or (_is_group(f) and f[1] == abi.K_LIST)


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
        self.parent = parents(self.fields)

    # ---- element bookkeeping of repeated groups ----------------------------
    def elems(self, g, upto=None):
        """Elements of group g in records [0, upto)."""
        f = self.fields[g]
        rows = self.rows(g, upto)
        if f[1] == abi.K_FIXED:
            return rows * f[2]
        return int(self.arrays[g][rows])

    def rows(self, k, upto=None):
        """Rows of field k's array in records [0, upto): records, or its group's elements."""
        g = self.parent[k]
        n = self.n if upto is None else upto
        return n if g < 0 else self.elems(g, n)

    def _elem_cap(self, g):
        """Element capacity of group g: the smallest over its members (fixed
        members are indexed by element with no capacity of their own)."""
        caps = []
        for j in direct_members(self.fields, g):
            m = self.arrays[j]
            f = self.fields[j]
            if _is_group(f):
                caps.append(len(m) - 1 if m is not None else self._elem_cap(j) // max(f[2], 1))
            else:
                caps.append((len(m[1]) - 1) if f[1] == abi.K_DYNAMIC else m.shape[0])
        return min(caps)

    # ---- construction ----------------------------------------------------
    @classmethod
    def empty(cls, fields, n, dyn_caps=None):
        """Zeroed output columns for a decode; dyn_caps[k] = element capacity
        (of a dynamic field, of a group, or of a group's dynamic member)."""
        fields = [tuple(f) for f in fields]
        caps = dyn_caps or {}
        rows_of = _cap_rows(fields, n, caps)
        arrays = []
        for k, f in enumerate(fields):
            t, kind, c = f[0], f[1], f[2]
            rows = rows_of[k]
            if _is_group(f):
                arrays.append(None if kind == abi.K_FIXED else np.zeros(rows + 1, dtype=np.uint64))
                continue
            dt = NP_DTYPE[t]
            if kind == abi.K_DYNAMIC:
                cap = caps.get(k, 0)
                arrays.append((np.zeros(max(cap, 1), dtype=dt), np.zeros(rows + 1, dtype=np.uint64)))
            elif kind == abi.K_FIXED:
                arrays.append(np.zeros((max(rows, 1), c), dtype=dt))
            else:
                arrays.append(np.zeros(max(rows, 1), dtype=dt))
        return cls(fields, n, arrays)

    def columns(self):
        """ctypes xdrg_column array with HOST pointers (for the oracle)."""
        arr = (abi.Column * len(self.fields))()
        for k, f in enumerate(self.fields):
            kind = f[1]
            arr[k].stride = 0
            if _is_group(f):
                offs = self.arrays[k]
                arr[k].data = None
                arr[k].offsets = None if offs is None else offs.ctypes.data
                arr[k].cap = self._elem_cap(k)
            elif kind == abi.K_DYNAMIC:
                vals, offs = self.arrays[k]
                arr[k].data = vals.ctypes.data
                arr[k].offsets = offs.ctypes.data
                arr[k].cap = vals.size
            else:
                a = self.arrays[k]
                arr[k].data = a.ctypes.data
                arr[k].offsets = None
                arr[k].cap = 0
        arr._keep = self.arrays  # keep the numpy buffers alive with the array
        return arr

    def dyn_caps(self):
        caps = {}
        for k, f in enumerate(self.fields):
            if _is_group(f):
                caps[k] = self.elems(k)
            elif f[1] == abi.K_DYNAMIC:
                caps[k] = int(self.arrays[k][1][self.rows(k)])
        return caps

    def _field_sizes(self, k, rows):
        """XDR bytes of field k for each of its `rows` rows (numpy uint64)."""
        f = self.fields[k]
        if f[1] == abi.K_DYNAMIC:
            offs = self.arrays[k][1][:rows + 1].astype(np.uint64)
            cnt = offs[1:] - offs[:-1]
            if abi.XDR_SIZE[f[0]] == 1:
                return 4 + cnt + ((4 - (cnt & 3)) & 3)
            return 4 + cnt * abi.XDR_SIZE[f[0]]
        return np.full(rows, field_xdr_bytes(f[:3]), dtype=np.uint64)

    def _group_sizes(self, k, rows):
        """XDR bytes of group k at each of its `rows` rows (its count / closing
        bool and every element, inner groups included)."""
        f = self.fields[k]
        E = self.elems(k)
        es = np.full(E, 4 if f[1] == abi.K_LIST else 0, dtype=np.uint64)
        for j in direct_members(self.fields, k):
            es += self._group_sizes(j, E) if _is_group(self.fields[j]) else self._field_sizes(j, E)
        ce = np.zeros(E + 1, dtype=np.uint64)
        np.cumsum(es, out=ce[1:])
        if f[1] == abi.K_FIXED:
            bounds = np.arange(rows + 1, dtype=np.uint64) * f[2]
        else:
            bounds = self.arrays[k][:rows + 1].astype(np.uint64)
        return ce[bounds[1:]] - ce[bounds[:-1]] + {abi.K_DYNAMIC: 4, abi.K_LIST: 4, abi.K_FIXED: 0}[f[1]]

    def xdr_sizes(self, framed=False):
        """Per-record XDR size (numpy uint64)."""
        s = np.full(self.n, 4 if framed else 0, dtype=np.uint64)
        k = 0
        while k < len(self.fields):
            f = self.fields[k]
            if not _is_group(f):
                s += self._field_sizes(k, self.n)
                k += 1
                continue
            s += self._group_sizes(k, self.n)
            k += 1 + f[3]
        return s

    def xdr_total(self, framed=False):
        return int(self.xdr_sizes(framed).sum())

    def native_bytes(self):
        """Algorithmic native bytes of the batch (values actually present)."""
        tot = 0
        for k, f in enumerate(self.fields):
            if _is_group(f):
                if self.arrays[k] is not None:
                    tot += 8 * self.rows(k)
            elif f[1] == abi.K_DYNAMIC:
                vals, offs = self.arrays[k]
                tot += int(offs[self.rows(k)]) * vals.dtype.itemsize
            else:
                a = self.arrays[k]
                tot += a[:self.rows(k)].nbytes
        return tot

    def record(self, i, k):
        """Value(s) of top-level field k of record i."""
        f = self.fields[k]
        if f[1] == abi.K_DYNAMIC:
            vals, offs = self.arrays[k]
            return vals[int(offs[i]):int(offs[i + 1])]
        return self.arrays[k][i]

    def slice(self, lo, hi):
        """Records [lo, hi) as a new batch (offsets rebased)."""
        arrays = []
        rng = {}
        for k, f in enumerate(self.fields):
            g = self.parent[k]
            a, b = (lo, hi) if g < 0 else rng[g]
            if _is_group(f):
                if f[1] == abi.K_FIXED:
                    arrays.append(None)
                    rng[k] = (a * f[2], b * f[2])
                else:
                    offs = self.arrays[k]
                    arrays.append((offs[a:b + 1] - offs[a]).astype(np.uint64))
                    rng[k] = (int(offs[a]), int(offs[b]))
            elif f[1] == abi.K_DYNAMIC:
                vals, offs = self.arrays[k]
                x, y = int(offs[a]), int(offs[b])
                arrays.append((vals[x:y].copy(), (offs[a:b + 1] - offs[a]).astype(np.uint64)))
            else:
                arrays.append(self.arrays[k][a:b].copy())
        return HostBatch(self.fields, hi - lo, arrays)

    def equal(self, other, upto=None):
        """Bit-exact equality of the first `upto` records (floats by bits)."""
        n = self.n if upto is None else upto
        for k, f in enumerate(self.fields):
            g = self.parent[k]
            rows = n if g < 0 else self.elems(g, n)
            if _is_group(f):
                if f[1] != abi.K_FIXED and not np.array_equal(self.arrays[k][:rows + 1],
                                                                other.arrays[k][:rows + 1]):
                    return False
            elif f[1] == abi.K_DYNAMIC:
                va, oa = self.arrays[k]
                vb, ob = other.arrays[k]
                if not np.array_equal(oa[:rows + 1], ob[:rows + 1]):
                    return False
                e = int(oa[rows])
                if not np.array_equal(_bits(va[:e]), _bits(vb[:e])):
                    return False
            else:
                if not np.array_equal(_bits(self.arrays[k][:rows]), _bits(other.arrays[k][:rows])):
                    return False
        return True


# ---- synthetic batches (seeded) -------------------------------------------
def random_batch(fields, n, seed, dyn_len=(0, 16), string_alphabet=b"abcdefghijklmnopqrstuvwxyz",
                 special_floats=True, group_len=(0, 4), inner_len=(0, 3)):
    """Seeded synthetic batch: ints uniform over their full range, floats as
    random bit patterns (NaNs with payloads included), bools 0/1/other
    non-zero bytes, dynamic lengths uniform in dyn_len, DYNAMIC / LIST group
    element counts uniform in group_len (inner groups: inner_len; both
    inclusive)."""
    rng = np.random.default_rng(seed)
    fields = [tuple(f) for f in fields]
    par = parents(fields)
    arrays = []
    elems = {}
    for k, f in enumerate(fields):
        t, kind, c = f[0], f[1], f[2]
        rows = n if par[k] < 0 else elems[par[k]]
        if t == abi.T_GROUP:
            if kind == abi.K_FIXED:
                arrays.append(None)
                elems[k] = rows * c
            else:
                lo, hi = group_len if par[k] < 0 else inner_len
                cnt = rng.integers(lo, hi + 1, size=rows, dtype=np.uint64)
                offs = np.zeros(rows + 1, dtype=np.uint64)
                np.cumsum(cnt, out=offs[1:])
                arrays.append(offs)
                elems[k] = int(offs[-1])
            continue
        dt = np.dtype(NP_DTYPE[t])
        if kind == abi.K_DYNAMIC:
            lo, hi = dyn_len
            cnt = rng.integers(lo, hi + 1, size=rows, dtype=np.uint64)
            offs = np.zeros(rows + 1, dtype=np.uint64)
            np.cumsum(cnt, out=offs[1:])
            total = int(offs[-1])
            if t == abi.T_STRING:
                alpha = np.frombuffer(string_alphabet, dtype=np.uint8)
                vals = alpha[rng.integers(0, len(alpha), size=total)]
            else:
                vals = _random_values(rng, dt, total, t, special_floats)
            arrays.append((vals, offs))
        else:
            shape = (rows, c) if kind == abi.K_FIXED else (rows,)
            size = int(np.prod(shape))
            arrays.append(_random_values(rng, dt, size, t, special_floats).reshape(shape))
    return HostBatch(fields, n, arrays)


def _cap_rows(fields, n, caps):
    """Rows of every field's array in an empty (decode output) batch: records
    at top level, a FIXED group's rows x count, else caps[group]."""
    par = parents(fields)
    rows = [0] * len(fields)
    for k in range(len(fields)):
        p = par[k]
        if p < 0:
            rows[k] = n
        elif fields[p][1] == abi.K_FIXED:
            rows[k] = rows[p] * fields[p][2]
        else:
            rows[k] = caps.get(p, 0)
    return rows


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
        self.parent = parents(self.fields)

    @classmethod
    def from_host(cls, hb, device="cuda"):
        import torch
        tensors, dts = [], []
        for k, f in enumerate(hb.fields):
            if _is_group(f):
                offs = hb.arrays[k]
                tensors.append(None if offs is None else
                               torch.from_numpy(offs.astype(np.uint64).view(np.int64)).to(device))
                dts.append(None)
            elif f[1] == abi.K_DYNAMIC:
                vals, offs = hb.arrays[k]
                tv = torch.from_numpy(_signed_view(vals if vals.size else np.zeros(1, vals.dtype)))
                to = torch.from_numpy(offs.astype(np.uint64).view(np.int64))
                tensors.append((tv.to(device), to.to(device)))
                dts.append(vals.dtype)
            else:
                a = hb.arrays[k]
                tensors.append(torch.from_numpy(_signed_view(a if a.size else
                                                             np.zeros((1,) + a.shape[1:], a.dtype))).to(device))
                dts.append(a.dtype)
        return cls(hb.fields, hb.n, tensors, dts)

    @classmethod
    def empty(cls, fields, n, dyn_caps=None, device="cuda"):
        import torch
        fields = [tuple(f) for f in fields]
        caps = dyn_caps or {}
        rows_of = _cap_rows(fields, n, caps)
        tensors, dts = [], []
        for k, f in enumerate(fields):
            t, kind, c = f[0], f[1], f[2]
            rows = rows_of[k]
            if _is_group(f):
                tensors.append(None if kind == abi.K_FIXED else
                               torch.zeros(rows + 1, dtype=torch.int64, device=device))
                dts.append(None)
                continue
            dt = np.dtype(NP_DTYPE[t])
            tdt = _torch_dtype(dt)
            if kind == abi.K_DYNAMIC:
                cap = max(caps.get(k, 0), 1)
                tensors.append((torch.zeros(cap, dtype=tdt, device=device),
                                torch.zeros(rows + 1, dtype=torch.int64, device=device)))
            elif kind == abi.K_FIXED:
                tensors.append(torch.zeros((max(rows, 1), c), dtype=tdt, device=device))
            else:
                tensors.append(torch.zeros(max(rows, 1), dtype=tdt, device=device))
            dts.append(dt)
        return cls(fields, n, tensors, dts)

    def _elem_cap(self, g):
        """Element capacity of group g: the smallest over its members."""
        caps = []
        for j in direct_members(self.fields, g):
            m = self.tensors[j]
            f = self.fields[j]
            if _is_group(f):
                caps.append(m.numel() - 1 if m is not None else self._elem_cap(j) // max(f[2], 1))
            else:
                caps.append((m[1].numel() - 1) if f[1] == abi.K_DYNAMIC else m.shape[0])
        return min(caps)

    def columns(self):
        """ctypes xdrg_column array with DEVICE pointers."""
        arr = (abi.Column * len(self.fields))()
        for k, f in enumerate(self.fields):
            arr[k].stride = 0
            if _is_group(f):
                arr[k].data = None
                arr[k].offsets = None if self.tensors[k] is None else self.tensors[k].data_ptr()
                arr[k].cap = self._elem_cap(k)
            elif f[1] == abi.K_DYNAMIC:
                tv, to = self.tensors[k]
                arr[k].data = tv.data_ptr()
                arr[k].offsets = to.data_ptr()
                arr[k].cap = tv.numel()
            else:
                arr[k].data = self.tensors[k].data_ptr()
                arr[k].offsets = None
                arr[k].cap = 0
        arr._keep = self.tensors
        return arr

    def to_host(self):
        arrays = []
        for k, f in enumerate(self.fields):
            dt = self._np[k]
            if _is_group(f):
                arrays.append(None if self.tensors[k] is None else
                              self.tensors[k].cpu().numpy().view(np.uint64))
            elif f[1] == abi.K_DYNAMIC:
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
