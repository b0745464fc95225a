// kernels_frame.hip — record-mark walk of a received TCP byte stream, in
// parallel.  Reference: RpcMessageParserTCP.java
// (paths under /root/reference/oncrpc4j-core/src/main/java/org/dcache/
// oncrpc4j/rpc/): isAllFragmentsArrived :63-99 walks marks BE(size | LAST)
// until a last fragment, STOPping when fewer than 4 bytes or fewer than
// `size` bytes remain; assembleXdr :109-140 concatenates the fragment
// bodies; handleRead :44-61 repeats on the remainder.
//
// The marks form a linked list (mark at p -> next mark at p + 4 + size), so
// the walk is a dependent chain.  On the GPU it becomes list ranking over
// every 4-byte position of the stream (fragment sizes are multiples of 4 in
// XDR traffic; a stream whose real chain meets another size falls back to
// the exact serial walk):
//   L1  k_frame_l1     per 16 KiB chunk, in LDS: every word position's exit =
//                      first chain position at or past the chunk end (12
//                      rounds of pointer jumping).
//   L2  k_frame_l2 x6  per 1 MiB super-chunk, in HBM: pointer doubling of the
//                      L1 exits (a hop crosses >= 1 chunk, so 6 rounds).
//   L3  k_frame_fix    one lane hops super-chunk to super-chunk from offset 0
//                      (<= len / 1 MiB dependent loads), k_frame_entries one
//                      lane per super-chunk hops its chunks (<= 64), giving
//                      every chunk's true entry; k_frame_count/emit walk each
//                      chunk's own marks in parallel.
// Fragments are then grouped into messages with two scans (rocPRIM) and the
// bodies copied out by k_frame_copy.
#include <cstring>

#include <hip/hip_runtime.h>
#include <rocprim/rocprim.hpp>

#include "xdrg_internal.h"

namespace xdrg {

__device__ __forceinline__ uint32_t fr_bswap(uint32_t x) { return __builtin_bswap32(x); }

// Next chain word index after the mark at word q (q < Q = len / 4), or a
// terminal: kFStop (fragment not fully received), kFUnal (size % 4 != 0).
__device__ __forceinline__ uint32_t frag_next(const uint32_t *w, uint64_t len, uint64_t q) {
    const uint64_t p = 4 * q;
    const uint32_t m = fr_bswap(w[q]);
    const uint64_t size = m & kSizeMask;
    if (size > len - p - 4) return kFStop;   // RpcMessageParserTCP.java:77-79
    if (size & 3) return kFUnal;
    return (uint32_t)((p + 4 + size) >> 2);
}

// L1: exit of every word position of one chunk.
__global__ __launch_bounds__(256) void k_frame_l1(const uint32_t *w, uint64_t len, uint64_t Q,
                                                   uint32_t *exit1, uint32_t *exit2) {
    __shared__ uint32_t J[kFChunk];
    const uint64_t c0 = (uint64_t)blockIdx.x * kFChunk;
    const uint64_t c1 = c0 + kFChunk;
    for (uint32_t i = threadIdx.x; i < kFChunk; i += blockDim.x) {
        const uint64_t q = c0 + i;
        J[i] = q < Q ? frag_next(w, len, q) : kFStop;
    }
    __syncthreads();
    for (int round = 0; round < kFChunkLog2; ++round) {   // chains inside a chunk have <= kFChunk hops
        uint32_t v[kFChunk / 256];
#pragma unroll
        for (int k = 0; k < kFChunk / 256; ++k) {
            const uint32_t j = J[threadIdx.x + 256 * k];
            v[k] = (j >= c0 && j < c1) ? J[j - c0] : j;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kFChunk / 256; ++k) J[threadIdx.x + 256 * k] = v[k];
        __syncthreads();
    }
    for (uint32_t i = threadIdx.x; i < kFChunk; i += blockDim.x) {
        const uint64_t q = c0 + i;
        if (q < Q) { exit1[q] = J[i]; exit2[q] = J[i]; }
    }
}

// L2: one doubling round of the super-chunk exits (in place: a value read
// early is still a successor on the same chain, so rounds only get faster).
__global__ __launch_bounds__(256) void k_frame_l2(uint32_t *exit2, uint64_t Q) {
    const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= Q) return;
    const uint32_t v = exit2[q];
    if (v < Q && v / kFSuper == q / kFSuper) exit2[q] = exit2[v];
}

// L3a: super-chunk entries along the real chain from offset 0.
__global__ void k_frame_fix(const uint32_t *exit2, uint64_t Q, uint32_t *sentry, uint64_t *res) {
    if (threadIdx.x || blockIdx.x) return;
    uint64_t e = 0;
    while (e < Q) {
        sentry[e / kFSuper] = (uint32_t)e;
        e = exit2[e];
    }
    res[0] = e;   // >= Q: ran to the end; kFStop / kFUnal: terminal met on the real chain
}

// L3b: chunk entries inside each super-chunk.
__global__ void k_frame_entries(const uint32_t *exit1, uint64_t Q, uint64_t nsuper, const uint32_t *sentry,
                                uint32_t *centry) {
    const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nsuper || sentry[s] == kFNone) return;
    uint64_t e = sentry[s];
    while (e < Q && e / kFSuper == s) {
        centry[e / kFChunk] = (uint32_t)e;
        e = exit1[e];
    }
}

// Walk the real chain inside chunk c: count (emit == false) or write the
// complete fragments (word index, raw mark).
template <bool kEmit>
__global__ void k_frame_walk(const uint32_t *w, uint64_t len, uint64_t Q, uint64_t nchunks,
                             const uint32_t *centry, uint32_t *counts, const uint32_t *base,
                             uint64_t *frag_pos, uint32_t *frag_mark) {
    const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= nchunks) return;
    uint32_t n = 0;
    const uint32_t e = centry[c];
    if (e != kFNone) {
        const uint64_t c1 = (c + 1) * kFChunk;
        uint64_t q = e;
        const uint32_t b = kEmit ? base[c] : 0;
        while (q < Q && q < c1) {
            const uint32_t nx = frag_next(w, len, q);
            if (nx == kFStop || nx == kFUnal) break;
            if (kEmit) {
                frag_pos[b + n] = 4 * q;
                frag_mark[b + n] = fr_bswap(w[q]);
            }
            ++n;
            q = nx;
        }
    }
    if (!kEmit) counts[c] = n;
}

// Exact serial walk (any fragment sizes): the fallback.  res[0] = fragments.
__global__ void k_frame_serial(const uint8_t *in, uint64_t len, uint64_t *frag_pos, uint32_t *frag_mark,
                               uint64_t *res) {
    if (threadIdx.x || blockIdx.x) return;
    uint64_t p = 0, n = 0;
    while (len - p >= 4) {
        const uint32_t m = ((uint32_t)in[p] << 24) | ((uint32_t)in[p + 1] << 16) | ((uint32_t)in[p + 2] << 8) | in[p + 3];
        const uint64_t size = m & kSizeMask;
        if (size > len - p - 4) break;
        frag_pos[n] = p;
        frag_mark[n] = m;
        ++n;
        p += 4 + size;
    }
    res[0] = n;
}

// Complete fragments end with the last LAST mark: res[1] = its index + 1
// (grid-stride max, one atomic per block).
__global__ __launch_bounds__(256) void k_frame_lastmsg(const uint32_t *frag_mark, uint64_t nfrag,
                                                        unsigned long long *res) {
    __shared__ unsigned long long wmax[4];
    unsigned long long m = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nfrag; i += (uint64_t)gridDim.x * blockDim.x)
        if (frag_mark[i] & kLastFrag) m = i + 1;
    for (int d = 32; d > 0; d >>= 1) {
        const unsigned long long o = __shfl_down(m, d, 64);
        m = o > m ? o : m;
    }
    if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 4; ++w) m = wmax[w] > m ? wmax[w] : m;
        if (m) atomicMax(res, m);
    }
}

// Per-fragment scan inputs: body size and last flag.
__global__ void k_frame_prep(const uint32_t *frag_mark, uint64_t nf, uint64_t *size, uint32_t *last) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nf) return;
    size[i] = frag_mark[i] & kSizeMask;
    last[i] = frag_mark[i] >> 31;
}

// Message i's first fragment writes msg_offsets[i] (payload or stream
// offset); the tail entry is the end of message `cap` (or of the last).
// consumed[0] = stream bytes of messages < cap (handleRead's split point).
__global__ void k_frame_msgs(const uint64_t *frag_pos, const uint32_t *frag_mark, uint64_t nf,
                             const uint32_t *msg_id, const uint64_t *pay_off, uint64_t cap, bool stream_offsets,
                             uint64_t *msg_offsets, uint64_t *consumed) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nf) return;
    const bool first = i == 0 || (frag_mark[i - 1] & kLastFrag);
    const uint64_t m = msg_id[i];
    const uint64_t v = stream_offsets ? frag_pos[i] : pay_off[i];
    if (first && m <= cap) msg_offsets[m] = v;
    if (first && m == cap) consumed[0] = frag_pos[i];
    if (i + 1 == nf && m + 1 <= cap) {   // end of the last message
        const uint64_t sz = frag_mark[i] & kSizeMask;
        msg_offsets[m + 1] = stream_offsets ? frag_pos[i] + 4 + sz : pay_off[i] + sz;
        consumed[0] = frag_pos[i] + 4 + sz;
    }
}

// A group of G lanes per fragment copies its body (G sized by the host from
// the average fragment): 16-byte accesses (dword-aligned, so unaligned
// vectors on gfx950) with a dword tail; byte copies on the fallback path.
typedef uint32_t u32x4f __attribute__((ext_vector_type(4), aligned(4)));
__global__ __launch_bounds__(256) void k_frame_copy(const uint8_t *in, const uint64_t *frag_pos,
                                                     const uint32_t *frag_mark, const uint64_t *pay_off,
                                                     const uint32_t *msg_id, uint64_t nf, uint64_t cap,
                                                     uint32_t G, uint8_t *payload) {
    const uint32_t gl = threadIdx.x & (G - 1);
    const uint64_t ngroups = (uint64_t)gridDim.x * (blockDim.x / G);
    for (uint64_t f = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / G; f < nf; f += ngroups) {
        if (msg_id[f] >= cap) return;   // fragments are in message order
        const uint8_t *src = in + frag_pos[f] + 4;
        uint8_t *dst = payload + pay_off[f];
        const uint64_t n = frag_mark[f] & kSizeMask;
        if ((((uintptr_t)src | (uintptr_t)dst | n) & 3) == 0) {
            const uint64_t nv = n >> 4;
            for (uint64_t i = gl; i < nv; i += G) *(u32x4f *)(dst + 16 * i) = *(const u32x4f *)(src + 16 * i);
            for (uint64_t i = 4 * nv + gl; i < n / 4; i += G) ((uint32_t *)dst)[i] = ((const uint32_t *)src)[i];
        } else {
            for (uint64_t i = gl; i < n; i += G) dst[i] = src[i];
        }
    }
}

// ---- launchers -------------------------------------------------------------------
static inline dim3 grid1(uint64_t n, uint32_t t) { return dim3((uint32_t)((n + t - 1) / t)); }

int frame_levels(const uint8_t *in, uint64_t len, FrameWs &ws, void *stream) {
    hipStream_t st = (hipStream_t)stream;
    const uint32_t *w = (const uint32_t *)in;
    const uint64_t Q = len / 4, nch = (Q + kFChunk - 1) / kFChunk, nsup = (Q + kFSuper - 1) / kFSuper;
    hipLaunchKernelGGL(k_frame_l1, dim3((uint32_t)nch), dim3(256), 0, st, w, len, Q, ws.exit1, ws.exit2);
    for (uint32_t r = 0; r < kFSuperLog2; ++r) hipLaunchKernelGGL(k_frame_l2, grid1(Q, 256), dim3(256), 0, st, ws.exit2, Q);
    if (hipMemsetAsync(ws.sentry, 0xff, nsup * 4, st) != hipSuccess) return (int)hipErrorUnknown;
    if (hipMemsetAsync(ws.centry, 0xff, nch * 4, st) != hipSuccess) return (int)hipErrorUnknown;
    hipLaunchKernelGGL(k_frame_fix, dim3(1), dim3(64), 0, st, ws.exit2, Q, ws.sentry, ws.res);
    hipLaunchKernelGGL(k_frame_entries, grid1(nsup, 64), dim3(64), 0, st, ws.exit1, Q, nsup, ws.sentry, ws.centry);
    hipLaunchKernelGGL(k_frame_walk<false>, grid1(nch, 64), dim3(64), 0, st, w, len, Q, nch, ws.centry, ws.counts,
                       nullptr, nullptr, nullptr);
    // fragment base per chunk; res[2] = fragments
    size_t tb = ws.tmp_bytes;
    if (rocprim::exclusive_scan(ws.tmp, tb, ws.counts, ws.base, 0u, nch, rocprim::plus<uint32_t>(), st) != hipSuccess)
        return (int)hipErrorUnknown;
    hipLaunchKernelGGL(k_frame_walk<true>, grid1(nch, 64), dim3(64), 0, st, w, len, Q, nch, ws.centry, nullptr,
                       ws.base, ws.frag_pos, ws.frag_mark);
    return (int)hipGetLastError();
}

size_t frame_scan_tmp_bytes(uint64_t n) {
    size_t a = 0, b = 0;
    (void)rocprim::exclusive_scan(nullptr, a, (const uint32_t *)nullptr, (uint32_t *)nullptr, 0u, n,
                                  rocprim::plus<uint32_t>());
    (void)rocprim::exclusive_scan(nullptr, b, (const uint64_t *)nullptr, (uint64_t *)nullptr, (uint64_t)0, n,
                                  rocprim::plus<uint64_t>());
    return (a > b ? a : b) + 256;
}

int frame_serial(const uint8_t *in, uint64_t len, FrameWs &ws, void *stream) {
    hipLaunchKernelGGL(k_frame_serial, dim3(1), dim3(64), 0, (hipStream_t)stream, in, len, ws.frag_pos, ws.frag_mark,
                       ws.res + 2);
    return (int)hipGetLastError();
}

int frame_last(FrameWs &ws, uint64_t nfrag, void *stream) {
    hipStream_t st = (hipStream_t)stream;
    if (hipMemsetAsync(ws.res + 1, 0, 8, st) != hipSuccess) return (int)hipErrorUnknown;
    uint64_t blocks = (nfrag + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    if (nfrag) hipLaunchKernelGGL(k_frame_lastmsg, dim3((uint32_t)blocks), dim3(256), 0, st, ws.frag_mark, nfrag,
                                  (unsigned long long *)ws.res + 1);
    return (int)hipGetLastError();
}

int frame_messages(const uint8_t *in, FrameWs &ws, uint64_t nf, uint64_t cap, bool stream_offsets,
                   uint64_t *msg_offsets, void *stream) {
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(k_frame_prep, grid1(nf, 256), dim3(256), 0, st, ws.frag_mark, nf, ws.size, ws.last);
    size_t tb = ws.tmp_bytes;
    if (rocprim::exclusive_scan(ws.tmp, tb, ws.last, ws.msg_id, 0u, nf, rocprim::plus<uint32_t>(), st) != hipSuccess)
        return (int)hipErrorUnknown;
    tb = ws.tmp_bytes;
    if (rocprim::exclusive_scan(ws.tmp, tb, ws.size, ws.pay_off, (uint64_t)0, nf, rocprim::plus<uint64_t>(), st) !=
        hipSuccess)
        return (int)hipErrorUnknown;
    hipLaunchKernelGGL(k_frame_msgs, grid1(nf, 256), dim3(256), 0, st, ws.frag_pos, ws.frag_mark, nf, ws.msg_id,
                       ws.pay_off, cap, stream_offsets, msg_offsets, ws.res + 3);
    (void)in;
    return (int)hipGetLastError();
}

int frame_copy(const uint8_t *in, FrameWs &ws, uint64_t nf, uint64_t cap, uint64_t payload_bytes, uint8_t *payload,
               void *stream) {
    uint32_t G = 1;   // lanes per fragment: ~16 bytes per lane for the average fragment
    while (G < 64 && 16ull * G * nf < payload_bytes) G <<= 1;
    uint64_t blocks = (nf + 256 / G - 1) / (256 / G);
    if (blocks > 65536) blocks = 65536;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(k_frame_copy, dim3((uint32_t)blocks), dim3(256), 0, (hipStream_t)stream, in, ws.frag_pos,
                       ws.frag_mark, ws.pay_off, ws.msg_id, nf, cap, G, payload);
    return (int)hipGetLastError();
}

}  // namespace xdrg
