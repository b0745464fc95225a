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

}  // namespace xdrg
