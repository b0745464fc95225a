// kernels_rec.hip — record path of the MI355X XDR engine: schemas with
// dynamic fields (opaque<>, string<>, T<> vectors), where every record has
// its own encoded size and the batch needs a prefix scan to place records.
//
// Encode (native columns -> one contiguous XDR stream):
//   1. k_enc_sizes   per block: sum of the XDR sizes of its kRecPerBlock
//                    records (computed from the dynamic columns' offsets).
//   2. k_scan_rows   one block per row: exclusive scan of the block sums.
//   3. k_enc_place   per block: recompute sizes, block-wide wavefront scan
//                    (DPP/shuffle inside a wave, LDS across waves) + block
//                    prefix -> record offsets; then one wavefront per record
//                    writes the record (header words, length words, payload
//                    realigned with v_alignbyte, zero pad).
// Decode (XDR stream + record extents -> native columns):
//   1. k_dec_sizes   per block, per dynamic column: walk each record's
//                    length words with the reference's check order
//                    (Xdr.java:171-531, 1028-1037), sum element counts and
//                    report the first failing check (atomicMin error key).
//   2. k_scan_rows   exclusive scan per dynamic column.
//   3. k_dec_place   per block: native offsets (written to the columns'
//                    offsets arrays), capacity check, then one wavefront per
//                    record copies every field out.
// Only agent-scope kernel boundaries separate the passes (no in-launch
// inter-workgroup hand-off), so nothing depends on XCD placement.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "xdrg_internal.h"

namespace xdrg {

__device__ __forceinline__ uint32_t bswap32r(uint32_t x) { return __builtin_bswap32(x); }
__device__ __forceinline__ uint32_t pad4(uint64_t n) { return (uint32_t)((4 - (n & 3)) & 3); }

__device__ __forceinline__ uint32_t canon_f32r(uint32_t u) {
    return ((u & 0x7fffffffu) > 0x7f800000u) ? 0x7fc00000u : u;
}
__device__ __forceinline__ void canon_f64r(uint32_t &hi, uint32_t &lo) {
    const uint32_t h = hi & 0x7fffffffu;
    if (h > 0x7ff00000u || (h == 0x7ff00000u && lo != 0)) { hi = 0x7ff80000u; lo = 0; }
}

// XDR bytes of a dynamic field holding `cnt` elements (length word included).
__device__ __forceinline__ uint64_t dyn_xdr_bytes(const VField &f, uint64_t cnt) {
    return 4 + (f.xsz == 1 ? cnt + pad4(cnt) : cnt * f.xsz);
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

// ---- scan of per-block sums: one block (1024 threads) per row ---------------
__global__ __launch_bounds__(1024) void k_scan_rows(uint64_t *sums, uint64_t nblocks,
                                                    uint64_t *totals) {
    __shared__ uint64_t wsum[16];
    __shared__ uint64_t carry_s;
    uint64_t *row = sums + (uint64_t)blockIdx.x * nblocks;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (threadIdx.x == 0) carry_s = 0;
    __syncthreads();
    for (uint64_t base = 0; base < nblocks; base += 1024) {
        const uint64_t i = base + threadIdx.x;
        const uint64_t v = i < nblocks ? row[i] : 0;
        const uint64_t incl = wave_incl_scan(v);
        if (lane == 63) wsum[wid] = incl;
        __syncthreads();
        uint64_t before = carry_s, tot = 0;
        for (int w = 0; w < 16; ++w) {
            if (w < wid) before += wsum[w];
            tot += wsum[w];
        }
        if (i < nblocks) row[i] = before + incl - v;
        __syncthreads();
        if (threadIdx.x == 0) carry_s += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) totals[blockIdx.x] = carry_s;
}

// ===========================================================================
// Encode
// ===========================================================================
__device__ __forceinline__ uint64_t enc_rec_size(const RecArgs &a, uint64_t r) {
    uint64_t s = a.fixed_xdr;
    for (uint32_t d = 0; d < a.ndyn; ++d) {
        const VField &f = a.f[a.dyn_idx[d]];
        s += dyn_xdr_bytes(f, f.offsets[r + 1] - f.offsets[r]);
    }
    return s;
}

__global__ __launch_bounds__(kRecThreads) void k_enc_sizes(const RecArgs a) {
    const uint64_t r0 = (uint64_t)blockIdx.x * kRecPerBlock + (uint64_t)threadIdx.x * kRecPerThread;
    uint64_t s = 0;
    for (int j = 0; j < kRecPerThread; ++j)
        if (r0 + j < a.n) s += enc_rec_size(a, r0 + j);
    const uint64_t tot = block_sum(s);
    if (threadIdx.x == 0) a.block_sums[blockIdx.x] = tot;
}

// One wavefront writes record r at byte offset pos of the stream.
__device__ void enc_record_wave(const RecArgs &a, uint64_t r, uint64_t pos, uint64_t size) {
    const uint32_t lane = threadIdx.x & 63;
    uint8_t *out = a.xdr;
    if (a.framed) {
        if (lane == 0)
            *(uint32_t *)(out + pos) = bswap32r((uint32_t)(size - 4) | kLastFrag);
        pos += 4;
    }
    for (uint32_t k = 0; k < a.nf; ++k) {
        const VField &f = a.f[k];
        if (f.kind != XDRG_K_DYNAMIC) {
            const uint8_t *base = f.data + (int64_t)r * f.stride;
            const uint32_t nw = f.xbytes >> 2;
            for (uint32_t i = lane; i < nw; i += 64) {
                uint32_t v;
                if (f.type == XDRG_T_OPAQUE) {
                    const uint32_t rem = f.count - 4 * i;
                    v = load_bytes(base + 4 * i, rem < 4 ? rem : 4);
                } else if (f.xsz == 8) {
                    v = enc_elem(f.type, base + (uint64_t)(i >> 1) * 8, i & 1);
                } else {
                    v = enc_elem(f.type, base + (uint64_t)i * f.nsz, 0);
                }
                *(uint32_t *)(out + pos + 4 * (uint64_t)i) = v;
            }
            pos += f.xbytes;
        } else {
            const uint64_t e0 = f.offsets[r], cnt = f.offsets[r + 1] - e0;
            if (lane == 0) *(uint32_t *)(out + pos) = bswap32r((uint32_t)cnt);
            pos += 4;
            if (f.xsz == 1) {  // opaque<> / string<>: bytes + zero pad (Xdr.java:776-800)
                const uint8_t *src = f.data + e0;
                const uint64_t nw = (cnt + 3) >> 2;
                for (uint64_t i = lane; i < nw; i += 64) {
                    const uint64_t rem = cnt - 4 * i;
                    *(uint32_t *)(out + pos + 4 * i) = load_bytes(src + 4 * i, rem < 4 ? (uint32_t)rem : 4u);
                }
                pos += 4 * nw;
            } else {           // T<> vectors (Xdr.java:607-613, 641-647, ...)
                const uint8_t *src = f.data + e0 * f.nsz;
                const uint64_t nw = cnt * (f.xsz >> 2);
                for (uint64_t i = lane; i < nw; i += 64) {
                    uint32_t v = f.xsz == 8 ? enc_elem(f.type, src + (i >> 1) * 8, (uint32_t)(i & 1))
                                            : enc_elem(f.type, src + i * f.nsz, 0);
                    *(uint32_t *)(out + pos + 4 * i) = v;
                }
                pos += 4 * nw;
            }
        }
    }
}

__global__ __launch_bounds__(kRecThreads) void k_enc_place_wave(const RecArgs a) {
    __shared__ uint64_t soff[kRecPerBlock + 1];
    const uint64_t total = a.totals[0];
    if (total > a.xdr_cap) return;  // XDRG_E_CAPACITY: write nothing
    const uint64_t rb = (uint64_t)blockIdx.x * kRecPerBlock;
    const uint32_t t0 = threadIdx.x * kRecPerThread;
    uint64_t sz[kRecPerThread];
    uint64_t s = 0;
#pragma unroll
    for (int j = 0; j < kRecPerThread; ++j) {
        sz[j] = (rb + t0 + j < a.n) ? enc_rec_size(a, rb + t0 + j) : 0;
        s += sz[j];
    }
    uint64_t btot;
    uint64_t off = a.block_sums[blockIdx.x] + block_excl_scan(s, &btot);
#pragma unroll
    for (int j = 0; j < kRecPerThread; ++j) {
        soff[t0 + j] = off;
        if (a.rec_out && rb + t0 + j < a.n) a.rec_out[rb + t0 + j] = off;
        off += sz[j];
    }
    if (threadIdx.x == kRecThreads - 1) soff[kRecPerBlock] = off;
    if (a.rec_out && blockIdx.x == 0 && threadIdx.x == 0) a.rec_out[a.n] = total;
    __syncthreads();
    const uint32_t wid = threadIdx.x >> 6;
    uint64_t nrec = a.n - rb;
    if (nrec > kRecPerBlock) nrec = kRecPerBlock;
    for (uint32_t j = wid; j < nrec; j += kRecThreads / 64)
        enc_record_wave(a, rb + j, soff[j], soff[j + 1] - soff[j]);
}

// ===========================================================================
// Decode
// ===========================================================================
struct Extent { uint64_t a, b; };

__device__ __forceinline__ Extent rec_extent(const RecArgs &a, uint64_t r) {
    Extent e;
    if (a.rec_in) { e.a = a.rec_in[r]; e.b = a.rec_in[r + 1]; }
    else { e.a = r * a.rec_stride; e.b = e.a + a.rec_stride; }
    if (e.b > a.xdr_cap) e.b = a.xdr_cap;
    if (e.a > e.b) e.a = e.b;
    return e;
}

__device__ __forceinline__ uint32_t ld_be32(const uint8_t *p) { return bswap32r(*(const uint32_t *)p); }

// Walk record r with the reference's check order.  Returns 0 or an error
// code (with *sub = check position); *cnt = element count of dynamic field
// `want` (field index), if reached.
__device__ uint32_t walk_record(const RecArgs &a, uint64_t r, uint32_t want, uint64_t *cnt,
                                uint32_t *sub) {
    const Extent e = rec_extent(a, r);
    uint64_t pos = e.a;
    *cnt = 0;
    if (a.framed) {  // one single-fragment message per record (GrizzlyRpcTransport:103-110)
        *sub = 0;
        if (e.b - pos < 4) return XDRG_E_SHORT;
        const uint32_t m = ld_be32(a.xdr + pos);
        const uint64_t want_len = a.rec_in ? e.b - pos - 4 : a.rec_stride - 4;
        if (!(m & kLastFrag) || (uint64_t)(m & kSizeMask) != want_len) return XDRG_E_FRAME;
        pos += 4;
    }
    for (uint32_t k = 0; k < a.nf; ++k) {
        const VField &f = a.f[k];
        *sub = 2 * k + 1;
        if (f.kind != XDRG_K_DYNAMIC) {
            // ensureBytes per element / per opaque (Xdr.java:1028-1032)
            if (e.b - pos < f.xbytes) return XDRG_E_SHORT;
            pos += f.xbytes;
            continue;
        }
        if (e.b - pos < 4) return XDRG_E_SHORT;  // length word (Xdr.java:171-175)
        const int32_t len = (int32_t)ld_be32(a.xdr + pos);
        pos += 4;
        uint64_t need;
        if (f.xsz == 1) {
            if (len == 0) need = 0;                      // Xdr.java:376-378 / :395-397
            else if (len < 0) return XDRG_E_CORRUPT;     // checkArraySize :1034-1037
            else need = (uint64_t)len + pad4((uint64_t)len);
        } else {
            if (len < 0) return XDRG_E_CORRUPT;          // checkArraySize before new T[len]
            need = (uint64_t)len * f.xsz;
        }
        if (e.b - pos < need) return XDRG_E_SHORT;
        pos += need;
        if (k == want) *cnt = (uint64_t)len;
    }
    return 0;
}

__global__ __launch_bounds__(kRecThreads) void k_dec_sizes_wave(const RecArgs a) {
    const uint64_t r0 = (uint64_t)blockIdx.x * kRecPerBlock + (uint64_t)threadIdx.x * kRecPerThread;
    // first pass (row 0 only) reports errors; every row sums its column
    for (uint32_t d = 0; d < (a.ndyn ? a.ndyn : 1); ++d) {
        const uint32_t want = a.ndyn ? a.dyn_idx[d] : 0xffffffffu;
        uint64_t s = 0;
        for (int j = 0; j < kRecPerThread; ++j) {
            const uint64_t r = r0 + j;
            if (r >= a.n) break;
            uint64_t c;
            uint32_t sub;
            const uint32_t err = walk_record(a, r, want, &c, &sub);
            if (err) {
                if (d == 0) atomicMin(a.errkey, err_key(r, sub, err));
                break;  // later records of this thread are past the error
            }
            s += c;
        }
        const uint64_t tot = block_sum(s);
        if (a.ndyn && threadIdx.x == 0) a.block_sums[(uint64_t)d * a.nblocks + blockIdx.x] = tot;
    }
}

// One wavefront decodes record r (already validated up to `upto` fields).
__device__ void dec_record_wave(const RecArgs &a, uint64_t r, uint32_t upto) {
    const uint32_t lane = threadIdx.x & 63;
    const Extent e = rec_extent(a, r);
    uint64_t pos = e.a + (a.framed ? 4 : 0);
    const uint8_t *__restrict__ in = a.xdr;
    for (uint32_t k = 0; k < upto; ++k) {
        const VField &f = a.f[k];
        if (f.kind != XDRG_K_DYNAMIC) {
            uint8_t *base = f.data + (int64_t)r * f.stride;
            const uint32_t nw = f.xbytes >> 2;
            for (uint32_t i = lane; i < nw; i += 64) {
                const uint32_t v = *(const uint32_t *)(in + pos + 4 * (uint64_t)i);
                if (f.type == XDRG_T_OPAQUE) {
                    const uint32_t rem = f.count - 4 * i, kb = rem < 4 ? rem : 4;
                    for (uint32_t b = 0; b < kb; ++b) base[4 * i + b] = (uint8_t)(v >> (8 * b));
                } else if (f.xsz == 8) {
                    dec_elem(f.type, base + (uint64_t)(i >> 1) * 8, i & 1, v);
                } else {
                    dec_elem(f.type, base + (uint64_t)i * f.nsz, 0, v);
                }
            }
            pos += f.xbytes;
            continue;
        }
        const int32_t len = (int32_t)ld_be32(in + pos);
        pos += 4;
        const uint64_t cnt = len > 0 ? (uint64_t)len : 0;
        const uint64_t e0 = f.offsets[r];
        if (f.xsz == 1) {
            // bytes to an arbitrarily aligned native destination: each lane
            // owns one aligned destination dword; partial head/tail dwords
            // are written byte by byte (neighbours belong to other records).
            uint8_t *dst = f.data + e0;
            const uintptr_t d0 = (uintptr_t)dst;
            const uint32_t sh = (uint32_t)(d0 & 3);
            const uintptr_t D = d0 - sh;
            const uint64_t nd = (sh + cnt + 3) >> 2;
            const uint64_t src_words = (cnt + 3) >> 2;
            const uint32_t *q = (const uint32_t *)(in + pos);
            for (uint64_t i = lane; i < nd; i += 64) {
                const uint32_t cur = i < src_words ? q[i] : 0u;
                uint32_t v;
                if (sh) {
                    const uint32_t prev = i > 0 ? q[i - 1] : 0u;
                    v = __builtin_amdgcn_alignbyte(cur, prev, 4 - sh);
                } else {
                    v = cur;
                }
                const uint64_t lo = i == 0 ? sh : 0;              // first valid byte in dword
                const uint64_t hi_end = sh + cnt - 4 * i;          // bytes valid below this
                const uint32_t hi = hi_end < 4 ? (uint32_t)hi_end : 4u;
                uint8_t *dd = (uint8_t *)(D + 4 * i);
                if (lo == 0 && hi == 4) {
                    *(uint32_t *)dd = v;
                } else {
                    for (uint32_t b = (uint32_t)lo; b < hi; ++b) dd[b] = (uint8_t)(v >> (8 * b));
                }
            }
            pos += cnt + pad4(cnt);
        } else {
            uint8_t *dst = f.data + e0 * f.nsz;
            const uint64_t nw = cnt * (f.xsz >> 2);
            for (uint64_t i = lane; i < nw; i += 64) {
                const uint32_t v = *(const uint32_t *)(in + pos + 4 * i);
                if (f.xsz == 8) dec_elem(f.type, dst + (i >> 1) * 8, (uint32_t)(i & 1), v);
                else dec_elem(f.type, dst + i * f.nsz, 0, v);
            }
            pos += cnt * f.xsz;
        }
    }
}

__global__ __launch_bounds__(kRecThreads) void k_dec_place_wave(const RecArgs a) {
    __shared__ uint32_t s_upto[kRecPerBlock];
    const uint64_t rb = (uint64_t)blockIdx.x * kRecPerBlock;
    const uint32_t t0 = threadIdx.x * kRecPerThread;
    const unsigned long long walk_key = *a.errkey;  // final after k_dec_sizes
    const uint64_t bad = walk_key == kNoError ? a.n : (uint64_t)(walk_key >> 16);
    // fields decodable per record: all for records before the first walk
    // error, none after; native capacity may cut a record short.
#pragma unroll
    for (int j = 0; j < kRecPerThread; ++j) s_upto[t0 + j] = (rb + t0 + j < bad) ? a.nf : 0;
    for (uint32_t d = 0; d < a.ndyn; ++d) {
        const uint32_t k = a.dyn_idx[d];
        const VField &f = a.f[k];
        uint64_t c[kRecPerThread];
        uint64_t s = 0;
#pragma unroll
        for (int j = 0; j < kRecPerThread; ++j) {
            const uint64_t r = rb + t0 + j;
            c[j] = 0;
            if (r < a.n && r < bad) {
                uint32_t sub;
                (void)walk_record(a, r, k, &c[j], &sub);
            }
            s += c[j];
        }
        uint64_t btot;
        uint64_t off = a.block_sums[(uint64_t)d * a.nblocks + blockIdx.x] + block_excl_scan(s, &btot);
#pragma unroll
        for (int j = 0; j < kRecPerThread; ++j) {
            const uint64_t r = rb + t0 + j;
            if (r < a.n) {
                f.offsets[r] = off;
                if (r < bad && off + c[j] > f.cap) {   // native column too small
                    atomicMin(a.errkey, err_key(r, 2 * k + 2, XDRG_E_CAPACITY));
                    if (s_upto[t0 + j] > k) s_upto[t0 + j] = k;
                }
            }
            off += c[j];
        }
        if (blockIdx.x == 0 && threadIdx.x == 0) f.offsets[a.n] = a.totals[d];
    }
    __syncthreads();
    const uint32_t wid = threadIdx.x >> 6;
    uint64_t nrec = a.n > rb ? a.n - rb : 0;
    if (nrec > kRecPerBlock) nrec = kRecPerBlock;
    for (uint32_t j = wid; j < nrec; j += kRecThreads / 64)
        if (s_upto[j]) dec_record_wave(a, rb + j, s_upto[j]);
}

// ===========================================================================
// Shared helpers of the place kernels (schemas with <= kMaxDynLds dynamic
// fields).  Byte-unaligned global dword / dwordx4 accesses are used where
// a payload moves between the 4-aligned stream and byte-packed native
// columns: gfx950 supports them under the HSA unaligned-access mode
// (tools/probes/unaligned.hip).
// ===========================================================================
typedef uint32_t u32x4a __attribute__((ext_vector_type(4), aligned(4)));
typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(1)));
typedef uint32_t u32u __attribute__((aligned(1)));

__device__ __forceinline__ bool is_word4(const VField &f) {
    return f.type == XDRG_T_INT || f.type == XDRG_T_UINT || f.type == XDRG_T_ENUM ||
           f.type == XDRG_T_FLOAT;
}

// XDR word at byte offset rel (multiple of 4) of fixed field f, record r.
__device__ __forceinline__ uint32_t fixed_word(const VField &f, uint64_t r, uint64_t rel) {
    const uint8_t *base = f.data + (int64_t)r * f.stride;
    const uint32_t i = (uint32_t)(rel >> 2);
    if (f.type == XDRG_T_OPAQUE) {
        const uint32_t rem = f.count - 4 * i;
        return load_bytes(base + 4 * i, rem < 4 ? rem : 4);
    }
    if (f.xsz == 8) return enc_elem(f.type, base + (uint64_t)(i >> 1) * 8, i & 1);
    return enc_elem(f.type, base + (uint64_t)i * f.nsz, 0);
}
__device__ __forceinline__ void fixed_store(const VField &f, uint64_t r, uint64_t rel, uint32_t v) {
    uint8_t *base = f.data + (int64_t)r * f.stride;
    const uint32_t i = (uint32_t)(rel >> 2);
    if (f.type == XDRG_T_OPAQUE) {
        const uint32_t rem = f.count - 4 * i, kb = rem < 4 ? rem : 4;
        if (kb == 4) *(u32u *)(base + 4 * i) = v;
        else for (uint32_t b = 0; b < kb; ++b) base[4 * i + b] = (uint8_t)(v >> (8 * b));
        return;
    }
    if (f.xsz == 8) dec_elem(f.type, base + (uint64_t)(i >> 1) * 8, i & 1, v);
    else dec_elem(f.type, base + (uint64_t)i * f.nsz, 0, v);
}

// XDR word at byte offset rel of dynamic field f (element count cnt, first
// element e0 of its native run).  rel < 4 is the length word.
__device__ __forceinline__ uint32_t dyn_word(const VField &f, uint64_t e0, uint64_t cnt, uint64_t rel) {
    if (rel < 4) return bswap32r((uint32_t)cnt);
    const uint64_t b = rel - 4;
    if (f.xsz == 1) {
        if (b >= cnt) return 0u;   // zero pad (Xdr.java:765-781)
        const uint8_t *src = f.data + e0 + b;
        const uint64_t nb = cnt - b;
        return nb >= 4 ? *(const u32u *)src : load_bytes(src, (uint32_t)nb);
    }
    if (f.xsz == 8) return enc_elem(f.type, f.data + (e0 + (b >> 3)) * 8, (uint32_t)((b >> 2) & 1));
    return enc_elem(f.type, f.data + (e0 + (b >> 2)) * f.nsz, 0);
}
__device__ __forceinline__ void dyn_store(const VField &f, uint64_t e0, uint64_t cnt, uint64_t rel, uint32_t v) {
    if (rel < 4) return;   // the count is known from the walk
    const uint64_t b = rel - 4;
    if (f.xsz == 1) {
        if (b >= cnt) return;   // pad
        uint8_t *dst = f.data + e0 + b;
        const uint64_t nb = cnt - b;
        if (nb >= 4) *(u32u *)dst = v;
        else for (uint32_t i = 0; i < nb; ++i) dst[i] = (uint8_t)(v >> (8 * i));
        return;
    }
    if (f.xsz == 8) dec_elem(f.type, f.data + (e0 + (b >> 3)) * 8, (uint32_t)((b >> 2) & 1), v);
    else dec_elem(f.type, f.data + (e0 + (b >> 2)) * f.nsz, 0, v);
}

// ---- encode -------------------------------------------------------------------
// LDS: soff[RPB + 2] u64 | ssrc[ND][RPB] u64 | scnt[ND][RPB] u32
__host__ __device__ constexpr size_t enc_lds_bytes(uint32_t nd) {
    return (size_t)(kRecPerBlock + 2) * 8 + (size_t)nd * kRecPerBlock * 12;
}

// ---- decode ------------------------------------------------------------------------
// Walk record r (known valid) and store each dynamic field's count at
// cnt_row[d * kRecPerBlock]; returns the record's first payload byte.
__device__ __forceinline__ uint32_t walk_counts(const RecArgs &a, uint64_t r, uint32_t *cnt_row,
                                                uint32_t *sub, uint64_t *start, uint64_t *bytes) {
    const Extent e = rec_extent(a, r);
    uint64_t pos = e.a;
    *start = e.a;
    *bytes = e.b - e.a;
    if (a.framed) {
        *sub = 0;
        if (e.b - pos < 4) return XDRG_E_SHORT;
        const uint32_t m = ld_be32(a.xdr + pos);
        const uint64_t want_len = a.rec_in ? e.b - pos - 4 : a.rec_stride - 4;
        if (!(m & kLastFrag) || (uint64_t)(m & kSizeMask) != want_len) return XDRG_E_FRAME;
        pos += 4;
    }
    uint32_t d = 0;
    for (uint32_t k = 0; k < a.nf; ++k) {
        const VField &f = a.f[k];
        *sub = 2 * k + 1;
        if (f.kind != XDRG_K_DYNAMIC) {
            if (e.b - pos < f.xbytes) return XDRG_E_SHORT;
            pos += f.xbytes;
            continue;
        }
        if (e.b - pos < 4) return XDRG_E_SHORT;
        const int32_t len = (int32_t)ld_be32(a.xdr + pos);
        pos += 4;
        uint64_t need;
        if (f.xsz == 1) {
            if (len == 0) need = 0;
            else if (len < 0) return XDRG_E_CORRUPT;
            else need = (uint64_t)len + pad4((uint64_t)len);
        } else {
            if (len < 0) return XDRG_E_CORRUPT;
            need = (uint64_t)len * f.xsz;
        }
        if (e.b - pos < need) return XDRG_E_SHORT;
        pos += need;
        cnt_row[(size_t)d * kRecPerBlock] = (uint32_t)len;
        ++d;
    }
    return 0;
}

// LDS: scnt[ND][RPB] u32.  Also stores every record's counts in
// a.rec_cnt[d * n + r] so the place kernel never walks the stream again.
__global__ __launch_bounds__(kRecThreads) void k_dec_sizes_g(const RecArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint32_t *scnt = (uint32_t *)smem;
    const uint64_t rb = (uint64_t)blockIdx.x * kRecPerBlock;
    const uint32_t t0 = threadIdx.x * kRecPerThread;
    bool dead = false;
#pragma unroll
    for (int j = 0; j < kRecPerThread; ++j) {
        const uint64_t r = rb + t0 + j;
        for (uint32_t d = 0; d < a.ndyn; ++d) scnt[(size_t)d * kRecPerBlock + t0 + j] = 0;
        if (r >= a.n || dead) continue;
        uint32_t sub;
        uint64_t st, by;
        const uint32_t err = walk_counts(a, r, scnt + t0 + j, &sub, &st, &by);
        if (err) {
            atomicMin(a.errkey, err_key(r, sub, err));
            dead = true;  // later records of this thread are past the error
            for (uint32_t d = 0; d < a.ndyn; ++d) scnt[(size_t)d * kRecPerBlock + t0 + j] = 0;
        }
    }
    __syncthreads();
    // coalesced copy of the block's counts to the workspace
    uint64_t nrec = a.n > rb ? a.n - rb : 0;
    if (nrec > kRecPerBlock) nrec = kRecPerBlock;
    for (uint32_t d = 0; d < a.ndyn; ++d)
        for (uint32_t i = threadIdx.x; i < nrec; i += kRecThreads)
            a.rec_cnt[(uint64_t)d * a.n + rb + i] = scnt[(size_t)d * kRecPerBlock + i];
    for (uint32_t d = 0; d < a.ndyn; ++d) {
        uint64_t s = 0;
#pragma unroll
        for (int j = 0; j < kRecPerThread; ++j) s += scnt[(size_t)d * kRecPerBlock + t0 + j];
        const uint64_t tot = block_sum(s);
        if (threadIdx.x == 0) a.block_sums[(uint64_t)d * a.nblocks + blockIdx.x] = tot;
    }
}

// ===========================================================================
// Group-per-record place kernels (the default; field-major)
//
// Phase 1, one thread per kRecPerThread records: sizes / counts, block scan,
// and every record's metadata (stream offset, dynamic counts, native offsets)
// staged in LDS.  Phase 2 walks the fields
// in schema order; for each field every record of the block is handled by a
// group of G lanes, G (1..64) chosen per field from that field's average size
// in the block.  Opaque/string fields move as one blob [length][payload][zero
// pad] in 16-byte chunks, kCopyU chunks per lane in flight, realigned with
// v_alignbyte_b32 so every global access is dword-aligned.  Measured on
// MI355X this beat a flat (output-stationary chunk sweep), a column-major, a
// segment-table and a lane-per-record design on configs 3 and 4 (DESIGN.md
// §5.3).
// ===========================================================================
__device__ __forceinline__ uint32_t mask_bytes(uint32_t v, int64_t valid) {
    if (valid >= 4) return v;
    if (valid <= 0) return 0;
    return v & ((1u << (8 * valid)) - 1u);
}

struct Chunk5 { uint32_t q0, q1, q2, q3, q4; };

__device__ __forceinline__ uint32_t pow2_lanes(uint64_t bytes_per_rec, uint32_t bytes_per_lane) {
    uint32_t g = 1;
    while (g < 64 && (uint64_t)g * bytes_per_lane < bytes_per_rec) g <<= 1;
    return g;
}

// One opaque/string field as one blob: [BE length][payload][zero pad] (Xdr.java:776-800).
template <int kCopyU>
__device__ __forceinline__ void enc_blob_bytes(uint8_t *__restrict__ dst, const uint8_t *__restrict__ src,
                                               uint64_t cnt, uint32_t G, uint32_t gl) {
    const uint64_t nwb = 1 + ((cnt + 3) >> 2), nch = (nwb + 3) >> 2;
    const uint32_t sh = (uint32_t)((uintptr_t)src & 3);
    const uint8_t *sa = src - sh;
    const uint8_t *end = src + cnt;
    const uint32_t lenw = bswap32r((uint32_t)cnt);
    for (uint64_t c0 = gl; c0 < nch; c0 += (uint64_t)G * kCopyU) {
        Chunk5 ch[kCopyU];
#pragma unroll
        for (int u = 0; u < kCopyU; ++u) {
            const uint64_t c = c0 + (uint64_t)u * G;
            if (c >= nch) continue;
            const uint8_t *p = sa + 16 * c;   // words at p - 4 + 4m, m = 0..4
            if (c > 0 && p + 16 <= end) {
                const u32x4a v = *(const u32x4a *)(p - 4);
                ch[u].q0 = v.x; ch[u].q1 = v.y; ch[u].q2 = v.z; ch[u].q3 = v.w;
                ch[u].q4 = sh ? *(const uint32_t *)(p + 12) : 0u;
            } else {
                ch[u].q0 = (c > 0 && p - 4 < end) ? *(const uint32_t *)(p - 4) : 0u;
                ch[u].q1 = p < end ? *(const uint32_t *)p : 0u;
                ch[u].q2 = p + 4 < end ? *(const uint32_t *)(p + 4) : 0u;
                ch[u].q3 = p + 8 < end ? *(const uint32_t *)(p + 8) : 0u;
                ch[u].q4 = (sh && p + 12 < end) ? *(const uint32_t *)(p + 12) : 0u;
            }
        }
#pragma unroll
        for (int u = 0; u < kCopyU; ++u) {
            const uint64_t c = c0 + (uint64_t)u * G;
            if (c >= nch) break;
            const Chunk5 &q = ch[u];
            uint32_t o0 = sh ? __builtin_amdgcn_alignbyte(q.q1, q.q0, sh) : q.q0;
            uint32_t o1 = sh ? __builtin_amdgcn_alignbyte(q.q2, q.q1, sh) : q.q1;
            uint32_t o2 = sh ? __builtin_amdgcn_alignbyte(q.q3, q.q2, sh) : q.q2;
            uint32_t o3 = sh ? __builtin_amdgcn_alignbyte(q.q4, q.q3, sh) : q.q3;
            const int64_t rem = 4 + (int64_t)cnt - 16 * (int64_t)c;   // blob bytes from chunk start
            if (rem < 16) {
                o0 = mask_bytes(o0, rem); o1 = mask_bytes(o1, rem - 4);
                o2 = mask_bytes(o2, rem - 8); o3 = mask_bytes(o3, rem - 12);
            }
            if (c == 0) o0 = lenw;
            uint8_t *d = dst + 16 * c;
            if (4 * c + 4 <= nwb) {
                u32x4a o; o.x = o0; o.y = o1; o.z = o2; o.w = o3;
                *(u32x4a *)d = o;
            } else {
                const uint64_t left = nwb - 4 * c;
                *(uint32_t *)d = o0;
                if (left > 1) *(uint32_t *)(d + 4) = o1;
                if (left > 2) *(uint32_t *)(d + 8) = o2;
            }
        }
    }
}

// int/uint/enum/float vector as one blob: [BE count][BE elements...].
__device__ __forceinline__ void enc_blob_words4(uint8_t *__restrict__ dst, const uint8_t *__restrict__ src,
                                                uint64_t cnt, bool fl, uint32_t G, uint32_t gl) {
    const uint64_t nwb = 1 + cnt, nch = (nwb + 3) >> 2;
    const uint32_t *p0 = (const uint32_t *)src;   // element e = blob word e + 1
    for (uint64_t c = gl; c < nch; c += G) {
        uint32_t w[4];
        if (c > 0 && 4 * c + 4 <= nwb) {
            const u32x4a v = *(const u32x4a *)(p0 + 4 * c - 1);
            w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint64_t b = 4 * c + j;   // blob word
                w[j] = (b >= 1 && b < nwb) ? p0[b - 1] : 0u;
            }
        }
        uint32_t o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = bswap32r(fl ? canon_f32r(w[j]) : w[j]);
        if (c == 0) o[0] = bswap32r((uint32_t)cnt);
        uint32_t *d = (uint32_t *)(dst + 16 * c);
        if (4 * c + 4 <= nwb) {
            u32x4a ov; ov.x = o[0]; ov.y = o[1]; ov.z = o[2]; ov.w = o[3];
            *(u32x4a *)d = ov;
        } else {
            for (uint64_t j = 0; 4 * c + j < nwb; ++j) d[j] = o[j];
        }
    }
}

// XDR payload (4-aligned src, cnt bytes) -> native bytes at any alignment.
// Partial head/tail dwords are written byte by byte: their other bytes
// belong to neighbouring records.
template <int kCopyU>
__device__ __forceinline__ void dec_bytes(uint8_t *__restrict__ dst, const uint8_t *__restrict__ src,
                                          uint64_t cnt, uint32_t G, uint32_t gl) {
    if (!cnt) return;
    const uint32_t sh = (uint32_t)((uintptr_t)dst & 3);
    uint8_t *da = dst - sh;
    const uint64_t nd = (sh + cnt + 3) >> 2, nch = (nd + 3) >> 2, nsw = (cnt + 3) >> 2;
    const uint32_t *q = (const uint32_t *)src;
    for (uint64_t c0 = gl; c0 < nch; c0 += (uint64_t)G * kCopyU) {
        Chunk5 ch[kCopyU];   // q0 = word before the chunk, q1..q4 = the chunk's source words
#pragma unroll
        for (int u = 0; u < kCopyU; ++u) {
            const uint64_t i0 = 4 * (c0 + (uint64_t)u * G);
            if (i0 >= 4 * nch) continue;
            if (i0 + 4 <= nsw) {
                const u32x4a v = *(const u32x4a *)(q + i0);
                ch[u].q1 = v.x; ch[u].q2 = v.y; ch[u].q3 = v.z; ch[u].q4 = v.w;
            } else {
                ch[u].q1 = i0 < nsw ? q[i0] : 0u;
                ch[u].q2 = i0 + 1 < nsw ? q[i0 + 1] : 0u;
                ch[u].q3 = i0 + 2 < nsw ? q[i0 + 2] : 0u;
                ch[u].q4 = i0 + 3 < nsw ? q[i0 + 3] : 0u;
            }
            ch[u].q0 = (sh && i0) ? q[i0 - 1] : 0u;
        }
#pragma unroll
        for (int u = 0; u < kCopyU; ++u) {
            const uint64_t c = c0 + (uint64_t)u * G;
            if (c >= nch) break;
            const uint64_t i0 = 4 * c;
            const Chunk5 &w = ch[u];
            uint32_t v[4];
            if (sh) {
                const uint32_t s = 4 - sh;
                v[0] = __builtin_amdgcn_alignbyte(w.q1, w.q0, s); v[1] = __builtin_amdgcn_alignbyte(w.q2, w.q1, s);
                v[2] = __builtin_amdgcn_alignbyte(w.q3, w.q2, s); v[3] = __builtin_amdgcn_alignbyte(w.q4, w.q3, s);
            } else {
                v[0] = w.q1; v[1] = w.q2; v[2] = w.q3; v[3] = w.q4;
            }
            uint8_t *d = da + 16 * c;
            if ((i0 > 0 || sh == 0) && 4 * (i0 + 4) <= sh + cnt) {
                u32x4a o; o.x = v[0]; o.y = v[1]; o.z = v[2]; o.w = v[3];
                *(u32x4a *)d = o;
                continue;
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint64_t i = i0 + j;
                if (i >= nd) break;
                const uint32_t lo = i == 0 ? sh : 0;
                const uint64_t he = sh + cnt - 4 * i;
                const uint32_t hi = he < 4 ? (uint32_t)he : 4u;
                if (lo == 0 && hi == 4) *(uint32_t *)(d + 4 * j) = v[j];
                else for (uint32_t b = lo; b < hi; ++b) d[4 * j + b] = (uint8_t)(v[j] >> (8 * b));
            }
        }
    }
}

__device__ __forceinline__ void dec_words4(uint8_t *__restrict__ dst, const uint8_t *__restrict__ src,
                                           uint64_t cnt, uint32_t G, uint32_t gl) {
    const uint64_t nch = (cnt + 3) >> 2;
    for (uint64_t c = gl; c < nch; c += G) {
        const uint32_t *p = (const uint32_t *)(src + 16 * c);
        uint32_t *d = (uint32_t *)(dst + 16 * c);
        if (4 * c + 4 <= cnt) {
            const u32x4a v = *(const u32x4a *)p;
            u32x4a o; o.x = bswap32r(v.x); o.y = bswap32r(v.y); o.z = bswap32r(v.z); o.w = bswap32r(v.w);
            *(u32x4a *)d = o;
        } else {
            for (uint64_t j = 0; 4 * c + j < cnt; ++j) d[j] = bswap32r(p[j]);
        }
    }
}

template <int U>
__global__ __launch_bounds__(kRecThreads) void k_enc_place_g(const RecArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint64_t *soff = (uint64_t *)smem;
    uint64_t *ssrc = soff + kRecPerBlock + 2;
    uint32_t *scnt = (uint32_t *)(ssrc + (size_t)a.ndyn * kRecPerBlock);
    const uint64_t total = a.totals[0];
    if (total > a.xdr_cap) return;  // XDRG_E_CAPACITY: write nothing
    const uint64_t rb = (uint64_t)blockIdx.x * kRecPerBlock;
    const uint32_t t0 = threadIdx.x * kRecPerThread;
    uint64_t sz[kRecPerThread];
    uint64_t s = 0;
#pragma unroll
    for (int j = 0; j < kRecPerThread; ++j) {
        const uint64_t r = rb + t0 + j;
        uint64_t size = 0;
        if (r < a.n) {
            size = a.fixed_xdr;
            for (uint32_t d = 0; d < a.ndyn; ++d) {
                const VField &f = a.f[a.dyn_idx[d]];
                const uint64_t o0 = f.offsets[r], cnt = f.offsets[r + 1] - o0;
                ssrc[(size_t)d * kRecPerBlock + t0 + j] = o0;
                scnt[(size_t)d * kRecPerBlock + t0 + j] = (uint32_t)cnt;
                size += dyn_xdr_bytes(f, cnt);
            }
        } else {
            for (uint32_t d = 0; d < a.ndyn; ++d) scnt[(size_t)d * kRecPerBlock + t0 + j] = 0;
        }
        sz[j] = size;
        s += size;
    }
    uint64_t btot;
    uint64_t off = a.block_sums[blockIdx.x] + block_excl_scan(s, &btot);
#pragma unroll
    for (int j = 0; j < kRecPerThread; ++j) {
        soff[t0 + j] = off;
        if (a.rec_out && rb + t0 + j < a.n) a.rec_out[rb + t0 + j] = off;
        off += sz[j];
    }
    if (threadIdx.x == kRecThreads - 1) soff[kRecPerBlock] = off;
    if (a.rec_out && blockIdx.x == 0 && threadIdx.x == 0) a.rec_out[a.n] = total;
    __syncthreads();
    uint64_t nrec = a.n - rb;
    if (nrec > kRecPerBlock) nrec = kRecPerBlock;
    uint8_t *out = a.xdr;
    const uint32_t tid = threadIdx.x;
    if (a.framed) {   // one single-fragment message per record (GrizzlyRpcTransport:103-110)
        for (uint32_t j = tid; j < nrec; j += kRecThreads)
            *(uint32_t *)(out + soff[j]) = bswap32r((uint32_t)(soff[j + 1] - soff[j] - 4) | kLastFrag);
    }
    uint64_t fixed_delta = a.framed ? 4 : 0;
    uint32_t d = 0;
    for (uint32_t k = 0; k < a.nf; ++k) {
        const VField &f = a.f[k];
        if (f.kind != XDRG_K_DYNAMIC) {
            const uint32_t nw = f.xbytes >> 2;
            if (nw) {
                const uint32_t G = a.force_g ? a.force_g : pow2_lanes((uint64_t)nw * 4, 16);
                const uint32_t gl = tid & (G - 1), ng = kRecThreads / G;
                for (uint32_t j = tid / G; j < nrec; j += ng) {
                    uint8_t *dst = out + soff[j] + fixed_delta;
                    for (uint32_t i = gl; i < nw; i += G) *(uint32_t *)(dst + 4 * i) = fixed_word(f, rb + j, 4 * i);
                }
            }
            fixed_delta += f.xbytes;
            continue;
        }
        const uint32_t *cn = scnt + (size_t)d * kRecPerBlock;
        const uint64_t *sr = ssrc + (size_t)d * kRecPerBlock;
        uint64_t ps = 0;
        for (uint32_t j = tid; j < nrec; j += kRecThreads) ps += cn[j];
        const uint64_t fbytes = block_sum(ps) * (f.xsz == 1 ? 1 : f.xsz) + 4 * nrec;
        const uint32_t G = a.force_g ? a.force_g : pow2_lanes(nrec ? fbytes / nrec : 0, a.lane_bytes_enc);
        const uint32_t gl = tid & (G - 1), ng = kRecThreads / G;
        for (uint32_t j = tid / G; j < nrec; j += ng) {
            const uint64_t cnt = cn[j], e0 = sr[j];
            uint8_t *dst = out + soff[j] + fixed_delta;
            if (f.xsz == 1) {
                enc_blob_bytes<U>(dst, f.data + e0, cnt, G, gl);
            } else if (is_word4(f)) {
                enc_blob_words4(dst, f.data + e0 * 4, cnt, f.type == XDRG_T_FLOAT, G, gl);
            } else {
                if (gl == 0) *(uint32_t *)dst = bswap32r((uint32_t)cnt);
                const uint64_t nw = cnt * (f.xsz >> 2);
                for (uint64_t i = gl; i < nw; i += G) *(uint32_t *)(dst + 4 + 4 * i) = dyn_word(f, e0, cnt, 4 + 4 * i);
            }
        }
        __syncthreads();
        for (uint32_t j = tid; j < nrec; j += kRecThreads) soff[j] += dyn_xdr_bytes(f, cn[j]);
        __syncthreads();
        ++d;
    }
}

// LDS: sstart[RPB] u64 | snoff[ND][RPB] u64 | scnt[ND][RPB] u32 | supto[RPB] u32
__host__ __device__ constexpr size_t dec_g_lds_bytes(uint32_t nd) {
    return (size_t)kRecPerBlock * 12 + (size_t)nd * kRecPerBlock * 12;
}

template <int U>
__global__ __launch_bounds__(kRecThreads) void k_dec_place_g(const RecArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint64_t *sstart = (uint64_t *)smem;
    uint64_t *snoff = sstart + kRecPerBlock;
    uint32_t *scnt = (uint32_t *)(snoff + (size_t)a.ndyn * kRecPerBlock);
    uint32_t *supto = scnt + (size_t)a.ndyn * kRecPerBlock;
    const uint64_t rb = (uint64_t)blockIdx.x * kRecPerBlock;
    const uint32_t t0 = threadIdx.x * kRecPerThread;
    const unsigned long long walk_key = *a.errkey;  // final after k_dec_sizes_g
    const uint64_t bad = walk_key == kNoError ? a.n : (uint64_t)(walk_key >> 16);
    for (uint32_t i = threadIdx.x; i < kRecPerBlock; i += kRecThreads) {
        const uint64_t r = rb + i;
        const bool live = r < a.n && r < bad;
        for (uint32_t d = 0; d < a.ndyn; ++d)
            scnt[(size_t)d * kRecPerBlock + i] = live ? a.rec_cnt[(uint64_t)d * a.n + r] : 0u;
        supto[i] = live ? a.nf : 0u;
        if (live) sstart[i] = rec_extent(a, r).a + (a.framed ? 4 : 0);
    }
    __syncthreads();
    for (uint32_t d = 0; d < a.ndyn; ++d) {
        const uint32_t k = a.dyn_idx[d];
        const VField &f = a.f[k];
        uint64_t s = 0;
#pragma unroll
        for (int j = 0; j < kRecPerThread; ++j) s += scnt[(size_t)d * kRecPerBlock + t0 + j];
        uint64_t btot;
        uint64_t off = a.block_sums[(uint64_t)d * a.nblocks + blockIdx.x] + block_excl_scan(s, &btot);
#pragma unroll
        for (int j = 0; j < kRecPerThread; ++j) {
            const uint64_t r = rb + t0 + j;
            const uint64_t c = scnt[(size_t)d * kRecPerBlock + t0 + j];
            snoff[(size_t)d * kRecPerBlock + t0 + j] = off;
            if (r < a.n) {
                f.offsets[r] = off;
                if (r < bad && off + c > f.cap) {   // native column too small
                    atomicMin(a.errkey, err_key(r, 2 * k + 2, XDRG_E_CAPACITY));
                    atomicMin(&supto[t0 + j], k);
                }
            }
            off += c;
        }
        if (blockIdx.x == 0 && threadIdx.x == 0) f.offsets[a.n] = a.totals[d];
    }
    __syncthreads();
    uint64_t nrec = a.n > rb ? a.n - rb : 0;
    if (nrec > kRecPerBlock) nrec = kRecPerBlock;
    const uint8_t *in = a.xdr;
    const uint32_t tid = threadIdx.x;
    uint64_t fixed_delta = 0;
    uint32_t d = 0;
    for (uint32_t k = 0; k < a.nf; ++k) {
        const VField &f = a.f[k];
        if (f.kind != XDRG_K_DYNAMIC) {
            const uint32_t nw = f.xbytes >> 2;
            if (nw) {
                const uint32_t G = a.force_g ? a.force_g : pow2_lanes((uint64_t)nw * 4, 16);
                const uint32_t gl = tid & (G - 1), ng = kRecThreads / G;
                for (uint32_t j = tid / G; j < nrec; j += ng) {
                    if (k >= supto[j]) continue;
                    const uint8_t *src = in + sstart[j] + fixed_delta;
                    for (uint32_t i = gl; i < nw; i += G) fixed_store(f, rb + j, 4 * i, *(const uint32_t *)(src + 4 * i));
                }
            }
            fixed_delta += f.xbytes;
            continue;
        }
        const uint32_t *cn = scnt + (size_t)d * kRecPerBlock;
        const uint64_t *no = snoff + (size_t)d * kRecPerBlock;
        uint64_t ps = 0;
        for (uint32_t j = tid; j < nrec; j += kRecThreads) ps += cn[j];
        const uint64_t fbytes = block_sum(ps) * (f.xsz == 1 ? 1 : f.xsz) + 4 * nrec;
        const uint32_t G = a.force_g ? a.force_g : pow2_lanes(nrec ? fbytes / nrec : 0, a.lane_bytes_dec);
        const uint32_t gl = tid & (G - 1), ng = kRecThreads / G;
        for (uint32_t j = tid / G; j < nrec; j += ng) {
            if (k >= supto[j]) continue;
            const uint64_t cnt = cn[j];
            const uint8_t *src = in + sstart[j] + fixed_delta + 4;
            if (f.xsz == 1) {
                dec_bytes<U>(f.data + no[j], src, cnt, G, gl);
            } else if (is_word4(f)) {
                dec_words4(f.data + no[j] * 4, src, cnt, G, gl);
            } else {
                const uint64_t nw = cnt * (f.xsz >> 2);
                for (uint64_t i = gl; i < nw; i += G) dyn_store(f, no[j], cnt, 4 + 4 * i, *(const uint32_t *)(src + 4 * i));
            }
        }
        __syncthreads();
        for (uint32_t j = tid; j < nrec; j += kRecThreads) sstart[j] += dyn_xdr_bytes(f, cn[j]);
        __syncthreads();
        ++d;
    }
}

// ===========================================================================
// Lane-per-record kernels (small records).  The group kernels above give a
// record a group of lanes per field and so keep only one or two 16-byte
// loads per lane in flight; here every lane owns whole records and issues up
// to kLaneU unaligned 16-byte loads of a payload before its stores, the
// pattern that measured 4.4-5.5 TB/s for 128-192 B records on MI355X
// (tools/probes/pattern_bw.hip, B vs D).  Records are taken strided
// (thread t: block records t, t + 256, ...), so neighbouring lanes write
// neighbouring records.  The prologue (block scan, LDS layout) is the group
// kernels'.
// ===========================================================================
constexpr int kLaneU = 4;   // 16-byte chunks per lane in flight

// [BE count][payload][zero pad] from bytes at any alignment to a 4-aligned dst.
__device__ __forceinline__ void lane_enc_bytes(uint8_t *__restrict__ dst, const uint8_t *__restrict__ src,
                                               uint32_t cnt) {
    *(uint32_t *)dst = bswap32r(cnt);
    dst += 4;
    const uint32_t nfull = cnt >> 4;
    for (uint32_t c = 0; c < nfull; c += kLaneU) {
        u32x4u v[kLaneU];
#pragma unroll
        for (int u = 0; u < kLaneU; ++u)
            if (c + u < nfull) v[u] = *(const u32x4u *)(src + 16 * (c + u));
#pragma unroll
        for (int u = 0; u < kLaneU; ++u)
            if (c + u < nfull) *(u32x4u *)(dst + 16 * (c + u)) = v[u];
    }
    const uint32_t rem = cnt & 15, o = 16 * nfull;
    for (uint32_t i = 0; 4 * i < rem; ++i) {
        const uint32_t k = rem - 4 * i;
        *(uint32_t *)(dst + o + 4 * i) = load_bytes(src + o + 4 * i, k < 4 ? k : 4u);   // zero pad (Xdr.java:765-781)
    }
}

// [BE count][BE elements] from a 4-aligned native int/uint/enum/float run.
__device__ __forceinline__ void lane_enc_words(uint8_t *__restrict__ dst, const uint32_t *__restrict__ src,
                                               uint32_t cnt, bool fl) {
    *(uint32_t *)dst = bswap32r(cnt);
    dst += 4;
    const uint32_t nfull = cnt >> 2;
    for (uint32_t c = 0; c < nfull; c += kLaneU) {
        u32x4a v[kLaneU];
#pragma unroll
        for (int u = 0; u < kLaneU; ++u)
            if (c + u < nfull) v[u] = *(const u32x4a *)(src + 4 * (c + u));
#pragma unroll
        for (int u = 0; u < kLaneU; ++u) {
            if (c + u >= nfull) continue;
            u32x4a o;
            o.x = bswap32r(fl ? canon_f32r(v[u].x) : v[u].x); o.y = bswap32r(fl ? canon_f32r(v[u].y) : v[u].y);
            o.z = bswap32r(fl ? canon_f32r(v[u].z) : v[u].z); o.w = bswap32r(fl ? canon_f32r(v[u].w) : v[u].w);
            *(u32x4u *)(dst + 16 * (c + u)) = o;
        }
    }
    for (uint32_t i = 4 * nfull; i < cnt; ++i) {
        const uint32_t w = src[i];
        *(uint32_t *)(dst + 4 * i) = bswap32r(fl ? canon_f32r(w) : w);
    }
}

// XDR payload (4-aligned) -> native bytes at any alignment; exactly cnt
// bytes are written (the next record's bytes follow in the column).
__device__ __forceinline__ void lane_dec_bytes(uint8_t *__restrict__ dst, const uint8_t *__restrict__ src,
                                               uint32_t cnt) {
    const uint32_t nfull = cnt >> 4;
    for (uint32_t c = 0; c < nfull; c += kLaneU) {
        u32x4a v[kLaneU];
#pragma unroll
        for (int u = 0; u < kLaneU; ++u)
            if (c + u < nfull) v[u] = *(const u32x4a *)(src + 16 * (c + u));
#pragma unroll
        for (int u = 0; u < kLaneU; ++u)
            if (c + u < nfull) *(u32x4u *)(dst + 16 * (c + u)) = v[u];
    }
    const uint32_t rem = cnt & 15, o = 16 * nfull;
    for (uint32_t i = 0; 4 * i < rem; ++i) {
        const uint32_t w = *(const uint32_t *)(src + o + 4 * i), k = rem - 4 * i;
        if (k >= 4) *(u32u *)(dst + o + 4 * i) = w;
        else for (uint32_t b = 0; b < k; ++b) dst[o + 4 * i + b] = (uint8_t)(w >> (8 * b));
    }
}

__device__ __forceinline__ void lane_dec_words(uint32_t *__restrict__ dst, const uint8_t *__restrict__ src,
                                               uint32_t cnt) {
    const uint32_t nfull = cnt >> 2;
    for (uint32_t c = 0; c < nfull; c += kLaneU) {
        u32x4a v[kLaneU];
#pragma unroll
        for (int u = 0; u < kLaneU; ++u)
            if (c + u < nfull) v[u] = *(const u32x4a *)(src + 16 * (c + u));
#pragma unroll
        for (int u = 0; u < kLaneU; ++u) {
            if (c + u >= nfull) continue;
            u32x4a o;
            o.x = bswap32r(v[u].x); o.y = bswap32r(v[u].y); o.z = bswap32r(v[u].z); o.w = bswap32r(v[u].w);
            *(u32x4a *)(dst + 4 * (c + u)) = o;
        }
    }
    for (uint32_t i = 4 * nfull; i < cnt; ++i) dst[i] = bswap32r(*(const uint32_t *)(src + 4 * i));
}

__global__ __launch_bounds__(kRecThreads) void k_enc_lane(const RecArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint64_t *soff = (uint64_t *)smem;
    uint64_t *ssrc = soff + kRecPerBlock + 2;
    uint32_t *scnt = (uint32_t *)(ssrc + (size_t)a.ndyn * kRecPerBlock);
    const uint64_t total = a.totals[0];
    if (total > a.xdr_cap) return;  // XDRG_E_CAPACITY: write nothing
    const uint64_t rb = (uint64_t)blockIdx.x * kRecPerBlock;
    const uint32_t t0 = threadIdx.x * kRecPerThread;
    uint64_t sz[kRecPerThread];
    uint64_t s = 0;
#pragma unroll
    for (int j = 0; j < kRecPerThread; ++j) {
        const uint64_t r = rb + t0 + j;
        uint64_t size = 0;
        if (r < a.n) {
            size = a.fixed_xdr;
            for (uint32_t d = 0; d < a.ndyn; ++d) {
                const VField &f = a.f[a.dyn_idx[d]];
                const uint64_t o0 = f.offsets[r], cnt = f.offsets[r + 1] - o0;
                ssrc[(size_t)d * kRecPerBlock + t0 + j] = o0;
                scnt[(size_t)d * kRecPerBlock + t0 + j] = (uint32_t)cnt;
                size += dyn_xdr_bytes(f, cnt);
            }
        }
        sz[j] = size;
        s += size;
    }
    uint64_t btot;
    uint64_t off = a.block_sums[blockIdx.x] + block_excl_scan(s, &btot);
#pragma unroll
    for (int j = 0; j < kRecPerThread; ++j) {
        soff[t0 + j] = off;
        if (a.rec_out && rb + t0 + j < a.n) a.rec_out[rb + t0 + j] = off;
        off += sz[j];
    }
    if (threadIdx.x == kRecThreads - 1) soff[kRecPerBlock] = off;
    if (a.rec_out && blockIdx.x == 0 && threadIdx.x == 0) a.rec_out[a.n] = total;
    __syncthreads();
    const uint64_t nrec = a.n - rb < (uint64_t)kRecPerBlock ? a.n - rb : (uint64_t)kRecPerBlock;
    for (uint32_t j = threadIdx.x; j < nrec; j += kRecThreads) {
        const uint64_t r = rb + j;
        uint8_t *dst = a.xdr + soff[j];
        if (a.framed) {   // GrizzlyRpcTransport.java:103-110
            *(uint32_t *)dst = bswap32r((uint32_t)(soff[j + 1] - soff[j] - 4) | kLastFrag);
            dst += 4;
        }
        uint32_t d = 0;
        for (uint32_t k = 0; k < a.nf; ++k) {
            const VField &f = a.f[k];
            if (f.kind != XDRG_K_DYNAMIC) {
                const uint32_t nw = f.xbytes >> 2;
                for (uint32_t i = 0; i < nw; ++i) *(uint32_t *)(dst + 4 * i) = fixed_word(f, r, 4 * i);
                dst += f.xbytes;
                continue;
            }
            const uint32_t cnt = scnt[(size_t)d * kRecPerBlock + j];
            const uint64_t e0 = ssrc[(size_t)d * kRecPerBlock + j];
            if (f.xsz == 1) {
                lane_enc_bytes(dst, f.data + e0, cnt);
            } else if (is_word4(f)) {
                lane_enc_words(dst, (const uint32_t *)(f.data + e0 * 4), cnt, f.type == XDRG_T_FLOAT);
            } else {
                *(uint32_t *)dst = bswap32r(cnt);
                const uint64_t nw = (uint64_t)cnt * (f.xsz >> 2);
                for (uint64_t i = 0; i < nw; ++i) *(uint32_t *)(dst + 4 + 4 * i) = dyn_word(f, e0, cnt, 4 + 4 * i);
            }
            dst += dyn_xdr_bytes(f, cnt);
            ++d;
        }
    }
}

__global__ __launch_bounds__(kRecThreads) void k_dec_lane(const RecArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint64_t *sstart = (uint64_t *)smem;
    uint64_t *snoff = sstart + kRecPerBlock;
    uint32_t *scnt = (uint32_t *)(snoff + (size_t)a.ndyn * kRecPerBlock);
    uint32_t *supto = scnt + (size_t)a.ndyn * kRecPerBlock;
    const uint64_t rb = (uint64_t)blockIdx.x * kRecPerBlock;
    const uint32_t t0 = threadIdx.x * kRecPerThread;
    const unsigned long long walk_key = *a.errkey;  // final after k_dec_sizes_g
    const uint64_t bad = walk_key == kNoError ? a.n : (uint64_t)(walk_key >> 16);
    for (uint32_t i = threadIdx.x; i < kRecPerBlock; i += kRecThreads) {
        const uint64_t r = rb + i;
        const bool live = r < a.n && r < bad;
        for (uint32_t d = 0; d < a.ndyn; ++d)
            scnt[(size_t)d * kRecPerBlock + i] = live ? a.rec_cnt[(uint64_t)d * a.n + r] : 0u;
        supto[i] = live ? a.nf : 0u;
        if (live) sstart[i] = rec_extent(a, r).a + (a.framed ? 4 : 0);
    }
    __syncthreads();
    for (uint32_t d = 0; d < a.ndyn; ++d) {
        const uint32_t k = a.dyn_idx[d];
        const VField &f = a.f[k];
        uint64_t s = 0;
#pragma unroll
        for (int j = 0; j < kRecPerThread; ++j) s += scnt[(size_t)d * kRecPerBlock + t0 + j];
        uint64_t btot;
        uint64_t off = a.block_sums[(uint64_t)d * a.nblocks + blockIdx.x] + block_excl_scan(s, &btot);
#pragma unroll
        for (int j = 0; j < kRecPerThread; ++j) {
            const uint64_t r = rb + t0 + j;
            const uint64_t c = scnt[(size_t)d * kRecPerBlock + t0 + j];
            snoff[(size_t)d * kRecPerBlock + t0 + j] = off;
            if (r < a.n) {
                f.offsets[r] = off;
                if (r < bad && off + c > f.cap) {   // native column too small
                    atomicMin(a.errkey, err_key(r, 2 * k + 2, XDRG_E_CAPACITY));
                    atomicMin(&supto[t0 + j], k);
                }
            }
            off += c;
        }
        if (blockIdx.x == 0 && threadIdx.x == 0) f.offsets[a.n] = a.totals[d];
    }
    __syncthreads();
    const uint64_t nrec = a.n > rb ? (a.n - rb < (uint64_t)kRecPerBlock ? a.n - rb : (uint64_t)kRecPerBlock) : 0;
    for (uint32_t j = threadIdx.x; j < nrec; j += kRecThreads) {
        const uint32_t upto = supto[j];
        if (!upto) continue;
        const uint64_t r = rb + j;
        const uint8_t *src = a.xdr + sstart[j];
        uint32_t d = 0;
        for (uint32_t k = 0; k < upto; ++k) {
            const VField &f = a.f[k];
            if (f.kind != XDRG_K_DYNAMIC) {
                const uint32_t nw = f.xbytes >> 2;
                for (uint32_t i = 0; i < nw; ++i) fixed_store(f, r, 4 * i, *(const uint32_t *)(src + 4 * i));
                src += f.xbytes;
                continue;
            }
            const uint32_t cnt = scnt[(size_t)d * kRecPerBlock + j];
            const uint64_t no = snoff[(size_t)d * kRecPerBlock + j];
            if (f.xsz == 1) lane_dec_bytes(f.data + no, src + 4, cnt);
            else if (is_word4(f)) lane_dec_words((uint32_t *)(f.data + no * 4), src + 4, cnt);
            else {
                const uint64_t nw = (uint64_t)cnt * (f.xsz >> 2);
                for (uint64_t i = 0; i < nw; ++i) dyn_store(f, no, cnt, 4 + 4 * i, *(const uint32_t *)(src + 4 + 4 * i));
            }
            src += dyn_xdr_bytes(f, cnt);
            ++d;
        }
    }
}

// ===========================================================================
// Launchers
// ===========================================================================
__global__ void k_debug_recargs(const RecArgs a) {
    if (threadIdx.x || blockIdx.x) return;
    printf("RecArgs n=%llu nf=%u framed=%u fixed_xdr=%u ndyn=%u xdr=%p cap=%llu rec_in=%p stride=%llu "
           "nblocks=%llu\n", (unsigned long long)a.n, a.nf, a.framed, a.fixed_xdr, a.ndyn, a.xdr,
           (unsigned long long)a.xdr_cap, a.rec_in, (unsigned long long)a.rec_stride,
           (unsigned long long)a.nblocks);
    if (a.rec_in) printf("  rec_in[0..2]=%llu %llu %llu\n", (unsigned long long)a.rec_in[0],
                         (unsigned long long)a.rec_in[1], (unsigned long long)a.rec_in[2]);
    for (uint32_t k = 0; k < a.nf; ++k)
        printf("  f%u type=%u kind=%u nsz=%u xsz=%u count=%u xbytes=%u data=%p off=%p cap=%llu\n", k,
               a.f[k].type, a.f[k].kind, a.f[k].nsz, a.f[k].xsz, a.f[k].count, a.f[k].xbytes,
               a.f[k].data, a.f[k].offsets, (unsigned long long)a.f[k].cap);
    uint64_t c;
    uint32_t sub;
    const uint32_t e = walk_record(a, 0, a.ndyn ? a.dyn_idx[0] : 0, &c, &sub);
    printf("  walk(0) -> err=%u sub=%u cnt=%llu\n", e, sub, (unsigned long long)c);
    const uint32_t *w = (const uint32_t *)a.xdr;
    printf("  xdr words: %08x %08x %08x %08x  be: %u %u %u\n", w[0], w[1], w[2], w[3], ld_be32(a.xdr),
           ld_be32(a.xdr + 4), ld_be32(a.xdr + 8));
    const Extent ex = rec_extent(a, 0);
    uint64_t pos = ex.a + 8;
    const int32_t len = (int32_t)ld_be32(a.xdr + pos);
    pos += 4;
    const uint64_t need = (uint64_t)len + pad4((uint64_t)len);
    printf("  ext=[%llu,%llu) len=%d need=%llu room=%llu pad=%u\n", (unsigned long long)ex.a,
           (unsigned long long)ex.b, len, (unsigned long long)need, (unsigned long long)(ex.b - pos),
           pad4((uint64_t)len));
}

// copy unroll of the group kernels (tools/tune_rec.py; set_tuning keys 4 and 5)
static int g_enc_u = 2, g_dec_u = 2;
static uint32_t g_force_g = 0;
static int g_rec_kernel = 0;   // 0 = group per record (default), 3 = lane per record
static uint32_t g_lane_bytes_enc = 32, g_lane_bytes_dec = 32;
int set_rec_tuning(int key, long long value) {
    if (key == 9) {
        if (value != 0 && value != 3) return -1;
        g_rec_kernel = (int)value;
        return 0;
    }
    if (key == 7 || key == 8) {   // target payload bytes per lane when sizing groups
        if (value < 4 || value > 65536) return -1;
        (key == 7 ? g_lane_bytes_enc : g_lane_bytes_dec) = (uint32_t)value;
        return 0;
    }
    if (key == 6) {   // lanes per record: 0 = automatic, else a power of two <= 64
        if (value < 0 || value > 64 || (value & (value - 1))) return -1;
        g_force_g = (uint32_t)value;
        return 0;
    }
    if (value != 1 && value != 2 && value != 4) return -1;
    if (key == 4) g_enc_u = (int)value;
    else if (key == 5) g_dec_u = (int)value;
    else return -1;
    return 0;
}

int launch_rec_phase(const RecArgs &args, int phase, void *stream) {
    RecArgs a = args;
    a.force_g = g_force_g;
    a.lane_bytes_enc = g_lane_bytes_enc;
    a.lane_bytes_dec = g_lane_bytes_dec;
    if (phase == REC_DEC_SIZES && getenv("XDRG_DEBUG"))
        hipLaunchKernelGGL(k_debug_recargs, dim3(1), dim3(64), 0, (hipStream_t)stream, a);
    hipStream_t st = (hipStream_t)stream;
    const uint64_t nb = a.nblocks;
    const bool grp = a.ndyn <= (uint32_t)kMaxDynLds;
    switch (phase) {
    case REC_ENC_SIZES: hipLaunchKernelGGL(k_enc_sizes, dim3(nb), dim3(kRecThreads), 0, st, a); break;
    case REC_ENC_SCAN:
        hipLaunchKernelGGL(k_scan_rows, dim3(1), dim3(1024), 0, st, a.block_sums, nb, a.totals);
        break;
    case REC_ENC_PLACE:
        if (grp && g_rec_kernel == 3) {
            hipLaunchKernelGGL(k_enc_lane, dim3(nb), dim3(kRecThreads), enc_lds_bytes(a.ndyn), st, a);
        } else if (grp) {
            if (g_enc_u == 1) hipLaunchKernelGGL(k_enc_place_g<1>, dim3(nb), dim3(kRecThreads), enc_lds_bytes(a.ndyn), st, a);
            else hipLaunchKernelGGL(k_enc_place_g<2>, dim3(nb), dim3(kRecThreads), enc_lds_bytes(a.ndyn), st, a);
        }
        else hipLaunchKernelGGL(k_enc_place_wave, dim3(nb), dim3(kRecThreads), 0, st, a);
        break;
    case REC_DEC_SIZES:
        if (grp) hipLaunchKernelGGL(k_dec_sizes_g, dim3(nb), dim3(kRecThreads),
                                    (size_t)a.ndyn * kRecPerBlock * 4, st, a);
        else hipLaunchKernelGGL(k_dec_sizes_wave, dim3(nb), dim3(kRecThreads), 0, st, a);
        break;
    case REC_DEC_SCAN:
        if (a.ndyn)
            hipLaunchKernelGGL(k_scan_rows, dim3(a.ndyn), dim3(1024), 0, st, a.block_sums, nb, a.totals);
        break;
    case REC_DEC_PLACE:
        if (grp && g_rec_kernel == 3) {
            hipLaunchKernelGGL(k_dec_lane, dim3(nb), dim3(kRecThreads), dec_g_lds_bytes(a.ndyn), st, a);
        } else if (grp) {
            if (g_dec_u == 1) hipLaunchKernelGGL(k_dec_place_g<1>, dim3(nb), dim3(kRecThreads), dec_g_lds_bytes(a.ndyn), st, a);
            else hipLaunchKernelGGL(k_dec_place_g<2>, dim3(nb), dim3(kRecThreads), dec_g_lds_bytes(a.ndyn), st, a);
        }
        else hipLaunchKernelGGL(k_dec_place_wave, dim3(nb), dim3(kRecThreads), 0, st, a);
        break;
    default: return (int)hipErrorInvalidValue;
    }
    return (int)hipGetLastError();
}



}  // namespace xdrg
