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
__device__ void enc_record(const RecArgs &a, uint64_t r, uint64_t pos, uint64_t size) {
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

__global__ __launch_bounds__(kRecThreads) void k_enc_place(const RecArgs a) {
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
        enc_record(a, rb + j, soff[j], soff[j + 1] - soff[j]);
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

__global__ __launch_bounds__(kRecThreads) void k_dec_sizes(const RecArgs a) {
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
__device__ void dec_record(const RecArgs &a, uint64_t r, uint32_t upto) {
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

__global__ __launch_bounds__(kRecThreads) void k_dec_place(const RecArgs a) {
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
        if (s_upto[j]) dec_record(a, rb + j, s_upto[j]);
}

// ===========================================================================
// Frame walk (RpcMessageParserTCP.isAllFragmentsArrived/assembleXdr :63-140)
// ===========================================================================
__device__ __forceinline__ uint32_t ld_be32_u(const uint8_t *p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

// Serial mark walk by one lane (marks form a dependent chain).  result[0] =
// complete messages found.
__global__ void k_frame_scan(const uint8_t *in, uint64_t len, uint64_t *msg_offsets, uint64_t cap,
                             uint64_t *result) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    uint64_t pos = 0, k = 0;
    while (k < cap) {
        uint64_t p = pos;
        bool complete = false;
        if (len - p < 4) break;
        do {
            const uint32_t m = ld_be32_u(in + p);
            p += 4;
            const uint64_t size = m & kSizeMask;
            if (size > len - p) break;           // fragment not fully received
            p += size;
            if (m & kLastFrag) { complete = true; break; }
        } while (len - p >= 4);
        if (!complete) break;
        msg_offsets[k++] = pos;
        pos = p;
    }
    msg_offsets[k] = pos;
    result[0] = k;
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

int launch_rec_phase(const RecArgs &a, int phase, void *stream) {
    if (phase == REC_DEC_SIZES && getenv("XDRG_DEBUG"))
        hipLaunchKernelGGL(k_debug_recargs, dim3(1), dim3(64), 0, (hipStream_t)stream, a);
    hipStream_t st = (hipStream_t)stream;
    const uint64_t nb = a.nblocks;
    switch (phase) {
    case REC_ENC_SIZES: hipLaunchKernelGGL(k_enc_sizes, dim3(nb), dim3(kRecThreads), 0, st, a); break;
    case REC_ENC_SCAN:
        hipLaunchKernelGGL(k_scan_rows, dim3(1), dim3(1024), 0, st, a.block_sums, nb, a.totals);
        break;
    case REC_ENC_PLACE: hipLaunchKernelGGL(k_enc_place, dim3(nb), dim3(kRecThreads), 0, st, a); break;
    case REC_DEC_SIZES: hipLaunchKernelGGL(k_dec_sizes, dim3(nb), dim3(kRecThreads), 0, st, a); break;
    case REC_DEC_SCAN:
        if (a.ndyn)
            hipLaunchKernelGGL(k_scan_rows, dim3(a.ndyn), dim3(1024), 0, st, a.block_sums, nb, a.totals);
        break;
    case REC_DEC_PLACE: hipLaunchKernelGGL(k_dec_place, dim3(nb), dim3(kRecThreads), 0, st, a); break;
    default: return (int)hipErrorInvalidValue;
    }
    return (int)hipGetLastError();
}

int launch_frame_scan(const uint8_t *in, uint64_t len, uint64_t *msg_offsets, uint64_t cap,
                      uint64_t *result, void *stream) {
    hipLaunchKernelGGL(k_frame_scan, dim3(1), dim3(64), 0, (hipStream_t)stream, in, len,
                       msg_offsets, cap, result);
    return (int)hipGetLastError();
}

}  // namespace xdrg
