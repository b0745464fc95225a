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
// Flat place kernels (schemas with <= kMaxDynLds dynamic fields)
//
// Phase 1, one thread per record: sizes / counts, block scan, and every
// record's metadata (stream offset, dynamic counts, native offsets) staged in
// LDS.  Phase 2 sweeps the block's contiguous XDR byte range in 16-byte
// chunks, one chunk per lane per step, so the stream side is perfectly
// coalesced (aligned dwordx4).  A lane finds its chunk's record by binary
// search over the LDS offsets and the field by walking the schema; a chunk
// that lies inside one dynamic payload moves with one 16-byte access on the
// native side (byte-unaligned global accesses are supported on gfx950 under
// the HSA unaligned-access mode, tools/probes/unaligned.hip); other chunks are
// assembled dword by dword.  Measured pattern ceilings that chose this shape
// (tools/probes/pattern_bw.hip, MI355X): coalesced stream + misaligned other
// side 6.1-6.3 TB/s; record-at-a-time groups 2.4-5.4 TB/s.
// ===========================================================================
typedef uint32_t u32x4a __attribute__((ext_vector_type(4), aligned(4)));
typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(1)));
typedef uint32_t u32u __attribute__((aligned(1)));

__device__ __forceinline__ bool is_word4(const VField &f) {
    return f.type == XDRG_T_INT || f.type == XDRG_T_UINT || f.type == XDRG_T_ENUM ||
           f.type == XDRG_T_FLOAT;
}

// Last j in [0, n) with key[j] <= q (key non-decreasing, key[0] <= q).
__device__ __forceinline__ uint32_t find_rec(const uint64_t *key, uint32_t n, uint64_t q) {
    uint32_t lo = 0, hi = n;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (key[mid] <= q) lo = mid;
        else hi = mid;
    }
    return lo;
}

// Coarse chunk -> record table: entry e holds the record containing chunk
// cbase + (e << shift), so a chunk's record is found by a short binary search
// between two neighbouring entries instead of over the whole block.
constexpr int kLookup = 256;
constexpr int kFlatU = 4;     // chunks per lane in flight in the flat kernels

__device__ __forceinline__ void build_lookup(const uint64_t *key, uint32_t n, uint64_t cbase, uint32_t shift,
                                             uint64_t lo_byte, uint32_t *tab) {
    for (uint32_t e = threadIdx.x; e <= kLookup; e += blockDim.x) {
        uint64_t q = (cbase + ((uint64_t)e << shift)) << 4;
        if (q < lo_byte) q = lo_byte;
        tab[e] = find_rec(key, n, q);
    }
}
__device__ __forceinline__ uint32_t lookup_rec(const uint64_t *key, uint32_t n, const uint32_t *tab,
                                               uint64_t cbase, uint32_t shift, uint64_t q) {
    const uint64_t e = ((q >> 4) - cbase) >> shift;
    uint32_t lo = tab[e], hi = e + 1 <= (uint64_t)kLookup ? tab[e + 1] + 1 : n;
    if (hi > n) hi = n;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (key[mid] <= q) lo = mid;
        else hi = mid;
    }
    return lo;
}
__device__ __forceinline__ uint32_t lookup_shift(uint64_t nchunks) {
    uint32_t sh = 0;
    while ((nchunks >> sh) > (uint64_t)kLookup - 1) ++sh;
    return sh;
}

// Where byte o of a record falls: segment kind, field, dynamic index, offset
// inside the field's XDR bytes.  cnt(d) gives dynamic field d's count.
enum SegKind : uint32_t { SEG_NONE = 0, SEG_MARK = 1, SEG_FIXED = 2, SEG_DYN = 3 };
struct Seg {
    uint32_t kind, k, d;
    uint64_t rel;   // byte offset inside the field's XDR bytes
    uint64_t cnt;   // SEG_DYN: element count
    uint64_t len;   // XDR bytes of the field
};

template <class CntFn>
__device__ __forceinline__ Seg locate(const RecArgs &a, const VField *F, uint64_t o, CntFn cnt_of) {
    Seg s;
    s.kind = SEG_NONE; s.k = 0; s.d = 0; s.rel = 0; s.cnt = 0; s.len = 0;
    uint64_t pos = 0;
    if (a.framed) {
        if (o < 4) { s.kind = SEG_MARK; s.rel = o; return s; }
        pos = 4;
    }
    uint32_t d = 0;
    for (uint32_t k = 0; k < a.nf; ++k) {
        const VField &f = F[k];
        uint64_t len, c = 0;
        if (f.kind != XDRG_K_DYNAMIC) {
            len = f.xbytes;
        } else {
            c = cnt_of(d);
            len = dyn_xdr_bytes(f, c);
        }
        if (o < pos + len) {
            s.kind = f.kind != XDRG_K_DYNAMIC ? SEG_FIXED : SEG_DYN;
            s.k = k; s.d = d; s.rel = o - pos; s.cnt = c; s.len = len;
            return s;
        }
        pos += len;
        if (f.kind == XDRG_K_DYNAMIC) ++d;
    }
    return s;
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

// Field descriptors staged in LDS: phase 2 indexes them with per-lane field
// numbers, which on the kernel-argument struct would become per-lane global
// loads of the kernarg segment.
__device__ __forceinline__ void stage_fields(const RecArgs &a, VField *sf) {
    for (uint32_t k = threadIdx.x; k < a.nf; k += blockDim.x) sf[k] = a.f[k];
}

// ---- encode -------------------------------------------------------------------
// LDS: soff[RPB + 2] u64 | ssrc[ND][RPB] u64 | scnt[ND][RPB] u32
__host__ __device__ constexpr size_t enc_lds_bytes(uint32_t nd) {
    return (size_t)(kRecPerBlock + 2) * 8 + (size_t)nd * kRecPerBlock * 12;
}

__global__ __launch_bounds__(kRecThreads) void k_enc_flat(const RecArgs a) {
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
    uint32_t nrec = (uint32_t)(a.n - rb < kRecPerBlock ? a.n - rb : kRecPerBlock);
    const uint64_t O0 = soff[0], O1 = soff[nrec];   // entries past nrec hold the end
    const uint64_t cbase = O0 >> 4, cend = (O1 + 15) >> 4;
    const uint32_t lsh = lookup_shift(cend - cbase);
    __shared__ uint32_t tab[kLookup + 1];
    __shared__ VField sf[kMaxFields];
    build_lookup(soff, nrec, cbase, lsh, O0, tab);
    stage_fields(a, sf);
    __syncthreads();
    uint8_t *out = a.xdr;
    for (uint64_t c0 = cbase + threadIdx.x; c0 < cend; c0 += (uint64_t)kRecThreads * kFlatU) {
        // A: classify kFlatU chunks and issue their fast-path loads
        u32x4a fv[kFlatU];
        uint32_t jj[kFlatU];
        bool fast[kFlatU];
#pragma unroll
        for (int u = 0; u < kFlatU; ++u) {
            const uint64_t c = c0 + (uint64_t)u * kRecThreads;
            fast[u] = false;
            jj[u] = 0;
            if (c >= cend) continue;
            const uint64_t p = c << 4;
            const uint64_t q0 = p > O0 ? p : O0;
            const uint32_t j = lookup_rec(soff, nrec, tab, cbase, lsh, q0);
            jj[u] = j;
            if (p < O0 || p + 16 > soff[j + 1]) continue;
            auto cnt_of = [&](uint32_t d) -> uint64_t { return scnt[(size_t)d * kRecPerBlock + j]; };
            const Seg g = locate(a, sf, p - soff[j], cnt_of);
            if (g.kind != SEG_DYN || g.rel < 4 || g.rel + 16 > g.len) continue;
            const VField &f = sf[g.k];
            const uint64_t e0 = ssrc[(size_t)g.d * kRecPerBlock + j];
            const uint64_t b = g.rel - 4;
            if (f.xsz == 1 && b + 16 <= g.cnt) {
                const u32x4u v = *(const u32x4u *)(f.data + e0 + b);
                fv[u].x = v.x; fv[u].y = v.y; fv[u].z = v.z; fv[u].w = v.w;
                fast[u] = true;
            } else if (is_word4(f)) {
                const u32x4a v = *(const u32x4a *)(f.data + (e0 + (b >> 2)) * 4);
                const bool fl = f.type == XDRG_T_FLOAT;
                fv[u].x = bswap32r(fl ? canon_f32r(v.x) : v.x); fv[u].y = bswap32r(fl ? canon_f32r(v.y) : v.y);
                fv[u].z = bswap32r(fl ? canon_f32r(v.z) : v.z); fv[u].w = bswap32r(fl ? canon_f32r(v.w) : v.w);
                fast[u] = true;
            }
        }
        // B: store; general chunks are assembled dword by dword
#pragma unroll
        for (int u = 0; u < kFlatU; ++u) {
            const uint64_t c = c0 + (uint64_t)u * kRecThreads;
            if (c >= cend) break;
            const uint64_t p = c << 4;
            if (fast[u]) {
                *(u32x4a *)(out + p) = fv[u];
                continue;
            }
            uint32_t j = jj[u];
            uint32_t w[4];
            uint32_t valid = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint64_t q = p + 4 * i;
                w[i] = 0;
                if (q < O0 || q >= O1) continue;
                while (j + 1 < nrec && q >= soff[j + 1]) ++j;
                auto cnt_j = [&](uint32_t d) -> uint64_t { return scnt[(size_t)d * kRecPerBlock + j]; };
                const Seg gg = locate(a, sf, q - soff[j], cnt_j);
                valid |= 1u << i;
                const uint64_t r = rb + j;
                if (gg.kind == SEG_MARK) {
                    w[i] = bswap32r((uint32_t)(soff[j + 1] - soff[j] - 4) | kLastFrag);
                } else if (gg.kind == SEG_FIXED) {
                    w[i] = fixed_word(sf[gg.k], r, gg.rel);
                } else if (gg.kind == SEG_DYN) {
                    w[i] = dyn_word(sf[gg.k], ssrc[(size_t)gg.d * kRecPerBlock + j], gg.cnt, gg.rel);
                }
            }
            if (valid == 0xf) {
                u32x4a o; o.x = w[0]; o.y = w[1]; o.z = w[2]; o.w = w[3];
                *(u32x4a *)(out + p) = o;
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    if (valid & (1u << i)) *(uint32_t *)(out + p + 4 * i) = w[i];
            }
        }
    }
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

// LDS: sstart[RPB + 2] u64 | snoff[ND][RPB] u64 | scnt[ND][RPB] u32 | supto[RPB] u32
__host__ __device__ constexpr size_t dec_lds_bytes(uint32_t nd) {
    return (size_t)(kRecPerBlock + 2) * 8 + (size_t)kRecPerBlock * 4 + (size_t)nd * kRecPerBlock * 12;
}

__global__ __launch_bounds__(kRecThreads) void k_dec_flat(const RecArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint64_t *sstart = (uint64_t *)smem;                         // record start in the stream
    uint64_t *snoff = sstart + kRecPerBlock + 2;
    uint32_t *scnt = (uint32_t *)(snoff + (size_t)a.ndyn * kRecPerBlock);
    uint32_t *supto = scnt + (size_t)a.ndyn * kRecPerBlock;
    __shared__ uint64_t s_end;
    const uint64_t rb = (uint64_t)blockIdx.x * kRecPerBlock;
    const uint32_t t0 = threadIdx.x * kRecPerThread;
    const unsigned long long walk_key = *a.errkey;  // final after k_dec_sizes_g
    const uint64_t bad = walk_key == kNoError ? a.n : (uint64_t)(walk_key >> 16);
    // live records of the block: validated by k_dec_sizes_g (before `bad`)
    const uint64_t lim = bad < a.n ? bad : a.n;
    const uint32_t nlive = (uint32_t)(lim > rb ? (lim - rb < kRecPerBlock ? lim - rb : kRecPerBlock) : 0);
    for (uint32_t i = threadIdx.x; i < kRecPerBlock; i += kRecThreads) {
        const bool live = i < nlive;
        const uint64_t r = rb + i;
        for (uint32_t d = 0; d < a.ndyn; ++d)
            scnt[(size_t)d * kRecPerBlock + i] = live ? a.rec_cnt[(uint64_t)d * a.n + r] : 0u;
        supto[i] = live ? a.nf : 0u;
        if (live) {
            const Extent e = rec_extent(a, r);
            sstart[i] = e.a;
            if (i + 1 == nlive) s_end = e.b;
        }
    }
    __syncthreads();
    for (uint32_t d = 0; d < a.ndyn; ++d) {
        const uint32_t k = a.dyn_idx[d];
        const VField &f = a.f[k];
        uint64_t ps = 0;
#pragma unroll
        for (int j = 0; j < kRecPerThread; ++j) ps += scnt[(size_t)d * kRecPerBlock + t0 + j];
        uint64_t btot;
        uint64_t off = a.block_sums[(uint64_t)d * a.nblocks + blockIdx.x] + block_excl_scan(ps, &btot);
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
    if (!nlive) return;
    const uint64_t I0 = sstart[0], I1 = s_end;
    const uint64_t cbase = I0 >> 4, cend = (I1 + 15) >> 4;
    const uint32_t lsh = lookup_shift(cend - cbase);
    __shared__ uint32_t tab[kLookup + 1];
    __shared__ VField sf[kMaxFields];
    build_lookup(sstart, nlive, cbase, lsh, I0, tab);
    stage_fields(a, sf);
    __syncthreads();
    const uint8_t *in = a.xdr;
    const uint64_t in_words = a.xdr_cap >> 2;
    for (uint64_t c0 = cbase + threadIdx.x; c0 < cend; c0 += (uint64_t)kRecThreads * kFlatU) {
        uint32_t w[kFlatU][4];
        uint32_t jj[kFlatU];
#pragma unroll
        for (int u = 0; u < kFlatU; ++u) {   // A: loads and record lookups
            const uint64_t c = c0 + (uint64_t)u * kRecThreads;
            jj[u] = 0;
            if (c >= cend) continue;
            const uint64_t p = c << 4;
            if (4 * c + 4 <= in_words) {
                const u32x4a v = *(const u32x4a *)(in + p);
                w[u][0] = v.x; w[u][1] = v.y; w[u][2] = v.z; w[u][3] = v.w;
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    w[u][i] = 4 * c + i < in_words ? *(const uint32_t *)(in + p + 4 * i) : 0u;
            }
            jj[u] = lookup_rec(sstart, nlive, tab, cbase, lsh, p > I0 ? p : I0);
        }
#pragma unroll
        for (int u = 0; u < kFlatU; ++u) {   // B: scatter to the native columns
            const uint64_t c = c0 + (uint64_t)u * kRecThreads;
            if (c >= cend) break;
            const uint64_t p = c << 4;
            uint32_t j = jj[u];
            const uint64_t rend0 = j + 1 < nlive ? sstart[j + 1] : I1;
            if (p >= I0 && p + 16 <= rend0) {
                auto cnt_of = [&](uint32_t d) -> uint64_t { return scnt[(size_t)d * kRecPerBlock + j]; };
                const Seg g = locate(a, sf, p - sstart[j], cnt_of);
                if (g.kind == SEG_DYN && g.rel >= 4 && g.rel + 16 <= g.len && g.k < supto[j]) {
                    const VField &f = sf[g.k];
                    const uint64_t no = snoff[(size_t)g.d * kRecPerBlock + j];
                    const uint64_t b = g.rel - 4;
                    if (f.xsz == 1 && b + 16 <= g.cnt) {
                        u32x4u o; o.x = w[u][0]; o.y = w[u][1]; o.z = w[u][2]; o.w = w[u][3];
                        *(u32x4u *)(f.data + no + b) = o;
                        continue;
                    }
                    if (is_word4(f)) {
                        u32x4a o;
                        o.x = bswap32r(w[u][0]); o.y = bswap32r(w[u][1]);
                        o.z = bswap32r(w[u][2]); o.w = bswap32r(w[u][3]);
                        *(u32x4a *)(f.data + (no + (b >> 2)) * 4) = o;
                        continue;
                    }
                }
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint64_t q = p + 4 * i;
                if (q < I0 || q >= I1) continue;
                while (j + 1 < nlive && q >= sstart[j + 1]) ++j;
                auto cnt_j = [&](uint32_t d) -> uint64_t { return scnt[(size_t)d * kRecPerBlock + j]; };
                const Seg gg = locate(a, sf, q - sstart[j], cnt_j);
                if (gg.kind == SEG_NONE || gg.kind == SEG_MARK || gg.k >= supto[j]) continue;
                const uint64_t r = rb + j;
                if (gg.kind == SEG_FIXED) fixed_store(sf[gg.k], r, gg.rel, w[u][i]);
                else dyn_store(sf[gg.k], snoff[(size_t)gg.d * kRecPerBlock + j], gg.cnt, gg.rel, w[u][i]);
            }
        }
    }
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

// copy unroll of the group kernels (tools/tune_rec.py; set_tuning keys 4 and 5)
static int g_enc_u = 2, g_dec_u = 2;
static uint32_t g_force_g = 0;
static uint32_t g_lane_bytes_enc = 32, g_lane_bytes_dec = 32;
int set_rec_tuning(int key, long long value) {
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
        if (grp) hipLaunchKernelGGL(k_enc_flat, dim3(nb), dim3(kRecThreads), enc_lds_bytes(a.ndyn), st, a);
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
        if (grp) hipLaunchKernelGGL(k_dec_flat, dim3(nb), dim3(kRecThreads), dec_lds_bytes(a.ndyn), st, a);
        else hipLaunchKernelGGL(k_dec_place_wave, dim3(nb), dim3(kRecThreads), 0, st, a);
        break;
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
