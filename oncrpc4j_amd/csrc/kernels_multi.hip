// kernels_multi.hip — the exchange step of the multi-GPU entry points
// (xdrg_encode_batch_multi, include/xdrg.h).
//
// After every device has encoded its record shard in place, each device
// PULLS the other shards straight out of its peers' HBM over xGMI with one
// k_gather launch: all peers' segments in one grid, so on an 8-GPU node the
// copy engages the 7 point-to-point links to the 7 peers at once (a ring
// would serialise them).  Segments keep their stream offset, so source and
// destination share their alignment inside the 16-byte grid.
#include <hip/hip_runtime.h>

#include "xdrg_internal.h"

namespace xdrg {

typedef uint32_t u32x4g __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_gather(const GatherArgs a) {
    const uint32_t s = blockIdx.y;
    const uint8_t *src = a.src[s];
    uint8_t *dst = a.dst[s];
    const uint64_t bytes = a.bytes[s];
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t nthr = (uint64_t)gridDim.x * blockDim.x;
    const uint32_t mis = (uint32_t)((uintptr_t)dst & 15);
    if (((uintptr_t)src & 15) != mis) {   // different grids: byte copy (never for stream shards)
        for (uint64_t i = tid; i < bytes; i += nthr) dst[i] = src[i];
        return;
    }
    uint64_t head = mis ? 16 - mis : 0;
    if (head > bytes) head = bytes;
    if (tid < head) dst[tid] = src[tid];
    const uint64_t nv = (bytes - head) >> 4;
    const u32x4g *sv = (const u32x4g *)(src + head);
    u32x4g *dv = (u32x4g *)(dst + head);
    for (uint64_t i = tid; i < nv; i += nthr) __builtin_nontemporal_store(__builtin_nontemporal_load(sv + i), dv + i);
    const uint64_t done = head + 16 * nv;
    if (tid < bytes - done) dst[done + tid] = src[done + tid];
}

int launch_gather(const GatherArgs &a, void *stream) {
    if (!a.nseg) return 0;
    uint64_t most = 0;
    for (uint32_t s = 0; s < a.nseg; ++s) most = a.bytes[s] > most ? a.bytes[s] : most;
    uint64_t blocks = (most / 16 + 255) / 256;
    if (blocks > 2048) blocks = 2048;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(k_gather, dim3((uint32_t)blocks, a.nseg), dim3(256), 0, (hipStream_t)stream, a);
    return (int)hipGetLastError();
}

// ---- host link copies (XDRG_HOST_PTRS staging, host_stage.h) ----------------
// One span between HBM and host memory the device maps (registered or
// hipHostMalloc'd), copied by the CUs instead of the DMA engines: copies of
// both directions then run as kernels on their own streams, so the PCIe
// link carries H2D and D2H traffic at once (the DMA engines took turns,
// DESIGN.md §5.1).  Each lane stores one destination-aligned 16-B chunk; the
// source is read as aligned 16-B vectors when it shares the destination's
// grid (every H2D span: the ring places it congruent mod 16), else as the
// aligned dwords under the chunk, realigned with v_alignbyte.
__device__ __forceinline__ u32x4g load16_from(const uint8_t *s) {
    const uintptr_t a = (uintptr_t)s;
    if ((a & 15) == 0) return __builtin_nontemporal_load((const u32x4g *)s);
    const uint32_t sh = (uint32_t)(a & 3);
    const uint32_t *q = (const uint32_t *)(a - sh);
    const uint32_t w0 = q[0], w1 = q[1], w2 = q[2], w3 = q[3];
    u32x4g v;
    if (!sh) {
        v.x = w0; v.y = w1; v.z = w2; v.w = w3;
        return v;
    }
    const uint32_t w4 = q[4];
    v.x = __builtin_amdgcn_alignbyte(w1, w0, sh);
    v.y = __builtin_amdgcn_alignbyte(w2, w1, sh);
    v.z = __builtin_amdgcn_alignbyte(w3, w2, sh);
    v.w = __builtin_amdgcn_alignbyte(w4, w3, sh);
    return v;
}

__global__ __launch_bounds__(256) void k_copy_link(uint8_t *dst, const uint8_t *src, uint64_t bytes) {
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t nthr = (uint64_t)gridDim.x * blockDim.x;
    const uint32_t mis = (uint32_t)((uintptr_t)dst & 15);
    uint64_t head = mis ? 16 - mis : 0;
    if (head > bytes) head = bytes;
    if (tid < head) dst[tid] = src[tid];
    const uint64_t nv = (bytes - head) >> 4;
    u32x4g *dv = (u32x4g *)(dst + head);
    const uint8_t *s0 = src + head;
    for (uint64_t i = tid; i < nv; i += nthr) __builtin_nontemporal_store(load16_from(s0 + 16 * i), dv + i);
    const uint64_t done = head + 16 * nv;
    if (tid < bytes - done) dst[done + tid] = src[done + tid];
}

int launch_copy_link(uint8_t *dst, const uint8_t *src, uint64_t bytes, void *stream) {
    if (!bytes) return 0;
    uint64_t blocks = (bytes / 16 + 255) / 256;
    if (blocks > 1024) blocks = 1024;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(k_copy_link, dim3((uint32_t)blocks), dim3(256), 0, (hipStream_t)stream, dst, src, bytes);
    return (int)hipGetLastError();
}

__global__ void k_pick_u64(uint64_t *dst, const uint64_t *base, const uint64_t *index, uint64_t limit) {
    if (threadIdx.x || blockIdx.x) return;
    const uint64_t i = *index;
    *dst = i <= limit ? base[i] : 0;
}
int launch_pick_u64(uint64_t *dst, const uint64_t *base, const uint64_t *index, uint64_t limit, void *stream) {
    hipLaunchKernelGGL(k_pick_u64, dim3(1), dim3(64), 0, (hipStream_t)stream, dst, base, index, limit);
    return (int)hipGetLastError();
}

__global__ void k_add_u64(uint64_t *p, uint64_t n, uint64_t delta) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        p[i] += delta;
}

int launch_add_u64(uint64_t *p, uint64_t n, uint64_t delta, void *stream) {
    if (!n || !delta) return 0;
    uint64_t blocks = (n + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(k_add_u64, dim3((uint32_t)blocks), dim3(256), 0, (hipStream_t)stream, p, n, delta);
    return (int)hipGetLastError();
}

__global__ void k_add_pos(uint64_t *p, uint64_t n, uint64_t delta) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t v = p[i];
        if (v != ~0ull) p[i] = v + delta;
    }
}

int launch_add_pos(uint64_t *p, uint64_t n, uint64_t delta, void *stream) {
    if (!n || !delta) return 0;
    uint64_t blocks = (n + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(k_add_pos, dim3((uint32_t)blocks), dim3(256), 0, (hipStream_t)stream, p, n, delta);
    return (int)hipGetLastError();
}

}  // namespace xdrg
