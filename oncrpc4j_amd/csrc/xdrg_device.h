// xdrg_device.h — device helpers shared by the record-path kernels
// (kernels_rec.hip) and the repeated-group kernels (kernels_group.hip):
// element <-> XDR word conversions with the reference's semantics and the
// block-wide scans.  Reference lines are cited at each helper.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "xdrg_internal.h"

namespace xdrg {

// Debug builds (make debug: -DXDRG_DEBUG) check the invariants the kernels
// trust (element descriptors, tile windows): a broken one stops the kernel
// with its condition printed instead of becoming a wild access.  Product
// builds compile the checks out.
#ifdef XDRG_DEBUG
#define XDRG_DCHECK(c)                                                                         \
    do {                                                                                       \
        if (!(c)) {                                                                            \
            printf("XDRG_DCHECK failed %s:%d: %s (block %u thread %u)\n", __FILE__, __LINE__, #c, \
                   blockIdx.x, threadIdx.x);                                                   \
            __builtin_trap();                                                                  \
        }                                                                                      \
    } while (0)
#else
#define XDRG_DCHECK(c) do {} while (0)
#endif

__device__ __forceinline__ uint32_t bswap32r(uint32_t x) { return __builtin_bswap32(x); }
__device__ __forceinline__ uint32_t pad4(uint64_t n) { return (uint32_t)((4 - (n & 3)) & 3); }

__device__ __forceinline__ uint32_t canon_f32r(uint32_t u) {
    return ((u & 0x7fffffffu) > 0x7f800000u) ? 0x7fc00000u : u;
}
__device__ __forceinline__ void canon_f64r(uint32_t &hi, uint32_t &lo) {
    const uint32_t h = hi & 0x7fffffffu;
    if (h > 0x7ff00000u || (h == 0x7ff00000u && lo != 0)) { hi = 0x7ff80000u; lo = 0; }
}

// ---- element words ---------------------------------------------------------
// XDR word `half` (0 = first) of one native element at p.
__device__ __forceinline__ uint32_t enc_elem(uint32_t type, const uint8_t *p, uint32_t half) {
    switch (type) {
    case XDRG_T_INT: case XDRG_T_UINT: case XDRG_T_ENUM: return bswap32r(*(const uint32_t *)p);
    case XDRG_T_FLOAT: return bswap32r(canon_f32r(*(const uint32_t *)p));
    case XDRG_T_HYPER: case XDRG_T_UHYPER: return bswap32r(*(const uint32_t *)(p + (half ? 0 : 4)));
    case XDRG_T_DOUBLE: {
        uint32_t lo = *(const uint32_t *)p, hi = *(const uint32_t *)(p + 4);
        canon_f64r(hi, lo);
        return bswap32r(half ? lo : hi);
    }
    case XDRG_T_BOOL: return *p ? 0x01000000u : 0u;
    case XDRG_T_SHORT: return bswap32r((uint32_t)(int32_t)*(const int16_t *)p);
    case XDRG_T_BYTE: return bswap32r((uint32_t)(int32_t)*(const int8_t *)p);
    default: return 0;
    }
}
__device__ __forceinline__ void dec_elem(uint32_t type, uint8_t *p, uint32_t half, uint32_t v) {
    switch (type) {
    case XDRG_T_INT: case XDRG_T_UINT: case XDRG_T_ENUM: case XDRG_T_FLOAT:
        *(uint32_t *)p = bswap32r(v); break;
    case XDRG_T_HYPER: case XDRG_T_UHYPER: case XDRG_T_DOUBLE:
        *(uint32_t *)(p + (half ? 0 : 4)) = bswap32r(v); break;
    case XDRG_T_BOOL: *p = v != 0; break;
    case XDRG_T_SHORT: *(uint16_t *)p = (uint16_t)bswap32r(v); break;
    case XDRG_T_BYTE: *p = (uint8_t)bswap32r(v); break;
    default: break;
    }
}

// k (1..4) bytes starting at an arbitrarily aligned p, as they sit in memory
// (little-endian word).  Only dwords that hold a requested byte are read, so
// no access leaves the page of a valid byte.
__device__ __forceinline__ uint32_t load_bytes(const uint8_t *p, uint32_t k) {
    const uintptr_t a = (uintptr_t)p;
    const uint32_t sh = (uint32_t)(a & 3);
    const uint32_t *q = (const uint32_t *)(a - sh);
    const uint32_t lo = q[0];
    const uint32_t hi = (sh + k > 4) ? q[1] : 0u;
    uint32_t v = sh ? __builtin_amdgcn_alignbyte(hi, lo, sh) : lo;
    if (k < 4) v &= (1u << (8 * k)) - 1u;
    return v;
}

// ---- block-wide exclusive scan (256 threads = 4 waves of 64) ----------------
__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t t = __shfl_up(v, d, 64);
        if (lane >= d) v += t;
    }
    return v;
}
// Returns the exclusive prefix of v over the block; *total = block sum.
__device__ __forceinline__ uint64_t block_excl_scan(uint64_t v, uint64_t *total) {
    __shared__ uint64_t wsum[kRecThreads / 64];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint64_t incl = wave_incl_scan(v);
    if (lane == 63) wsum[wid] = incl;
    __syncthreads();
    uint64_t before = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < kRecThreads / 64; ++w) {
        if (w < wid) before += wsum[w];
        tot += wsum[w];
    }
    __syncthreads();
    *total = tot;
    return before + incl - v;
}
__device__ __forceinline__ uint64_t block_sum(uint64_t v) {
    uint64_t tot;
    (void)block_excl_scan(v, &tot);
    return tot;
}

// ---- XCD-aware block order ----------------------------------------------------
// Blocks are dealt round-robin over the 8 XCDs (b and b + 8 share one; each
// XCD has its own L2; MI355X_MICROARCH.md "Workgroup dispatch").  Block b of a
// one-pass grid of nb blocks takes logical block xcd_block(b, nb): XCD slot
// x = b % 8 owns the contiguous logical range [x*q + min(x, r), ...), q = nb/8,
// r = nb % 8, so the blocks resident on one XCD work on neighbouring records
// and a 128-byte line that straddles two of them is completed in one L2
// (else each XCD writes back its own partial copy of the line).  A bijection
// of [0, nb) for speed only: correctness never depends on the placement.
__device__ __forceinline__ uint64_t xcd_block(uint64_t b, uint64_t nb) {
    const uint64_t x = b & 7, q = nb >> 3, r = nb & 7;
    return x * q + (x < r ? x : r) + (b >> 3);
}

}  // namespace xdrg
