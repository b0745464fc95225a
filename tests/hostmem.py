"""Host memory of the three kinds a caller of the XDRG_HOST_PTRS calls holds
(tests only): pageable buffers, buffers pinned with xdrg_host_register, and
hipHostMalloc'd torch pinned memory."""
import ctypes
import mmap

import numpy as np

from oncrpc4j_amd import engine
from oncrpc4j_amd.columns import HostBatch


class Registered:
    """Page-aligned anonymous mappings pinned with xdrg_host_register."""

    def __init__(self):
        self.maps, self.ptrs = [], []

    def array(self, like):
        nbytes = max(like.nbytes, 1)
        m = mmap.mmap(-1, nbytes)
        a = np.frombuffer(m, dtype=np.uint8, count=like.nbytes).view(like.dtype).reshape(like.shape)
        a[...] = like
        engine.host_register(ctypes.addressof(ctypes.c_char.from_buffer(m)), nbytes)
        self.maps.append(m)
        self.ptrs.append(ctypes.addressof(ctypes.c_char.from_buffer(m)))
        return a

    def close(self):
        for p in self.ptrs:
            engine.host_unregister(p)
        self.ptrs = []


class TorchPinned:
    """hipHostMalloc'd buffers (torch pin_memory): pinned without registration."""

    def __init__(self):
        self.keep = []

    def array(self, like):
        import torch
        t = torch.empty(max(like.nbytes, 1), dtype=torch.uint8).pin_memory()
        self.keep.append(t)
        a = t.numpy()[:like.nbytes].view(like.dtype).reshape(like.shape)
        a[...] = like
        return a

    def close(self):
        self.keep = []


class Pageable:
    def array(self, like):
        return like.copy()

    def close(self):
        pass


KINDS = {"pageable": Pageable, "registered": Registered, "torch_pinned": TorchPinned}


def moved(hb, mem):
    """hb with every array in memory of kind `mem`."""
    arrays = []
    for a in hb.arrays:
        if a is None:
            arrays.append(None)
        elif isinstance(a, tuple):
            arrays.append((mem.array(a[0]), mem.array(a[1])))
        else:
            arrays.append(mem.array(a))
    return HostBatch(hb.fields, hb.n, arrays)


