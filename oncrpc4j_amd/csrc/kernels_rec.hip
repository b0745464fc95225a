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

#include "xdrg_device.h"
#include "xdrg_internal.h"

namespace xdrg {

// XDR bytes of a dynamic field holding `cnt` elements (length word included).
__device__ __forceinline__ uint64_t dyn_xdr_bytes(const VField &f, uint64_t cnt) {
    return 4 + (f.xsz == 1 ? cnt + pad4(cnt) : cnt * f.xsz);
}

// ---- conditional fields (rpcgen unions / optional data, xdrg_cond) ----------
// Field k with f.cond = d + 1 is present iff field d is present and d's value
// is / is not in its case list: the switch jrpcgen emits for a union
// (jrpcgen.java:1240-1340; no matching arm and no default = nothing) and the
// bool-then-value of optional data.  Discriminant values live in up to
// XDRG_MAX_DISC slots; slot indices are uniform, so the selects below are
// unrolled over constant register indices (no scratch).
struct Disc {
    uint32_t pres;              // bit k: field k present in this record
    int32_t v[XDRG_MAX_DISC];
    __device__ __forceinline__ int32_t get(uint32_t slot) const {
        int32_t r = 0;
#pragma unroll
        for (int i = 0; i < XDRG_MAX_DISC; ++i) if ((uint32_t)i == slot) r = v[i];
        return r;
    }
    __device__ __forceinline__ void set(uint32_t slot, int32_t x) {
#pragma unroll
        for (int i = 0; i < XDRG_MAX_DISC; ++i) if ((uint32_t)i == slot) v[i] = x;
    }
};
// Is field k present, given the discriminants seen so far?
__device__ __forceinline__ bool cond_present(const RecArgs &a, const VField &f, const Disc &dv) {
    if (!f.cond) return true;
    const uint32_t d = f.cond - 1;
    if (!((dv.pres >> d) & 1u)) return false;
    const int32_t x = dv.get(a.f[d].slot - 1);
    bool in = false;
    for (uint32_t i = 0; i < f.cnum; ++i) in |= a.cvals[f.cfirst + i] == x;
    return in != (f.cneg != 0);
}
// Record field k as present with (discriminant) value x; bools count as 0/1
// (Xdr.java:803-805 encode, :404-407 decode any non-zero = true).
__device__ __forceinline__ void cond_mark(const VField &f, uint32_t k, int32_t x, Disc &dv) {
    dv.pres |= 1u << k;
    if (f.slot) dv.set(f.slot - 1, f.type == XDRG_T_BOOL ? (x != 0) : x);
}
// Native value of discriminant field f of record r (encode side).
__device__ __forceinline__ int32_t disc_native(const VField &f, uint64_t r) {
    const uint8_t *p = f.data + (int64_t)r * f.stride;
    return f.type == XDRG_T_BOOL ? (int32_t)(*p != 0) : *(const int32_t *)p;
}

// ---- extent-derived decode counts (tuning key 31) ----------------------------
// When a schema's last dynamic field is a vector of 4-byte elements followed
// only by fixed fields (config 4: int, string<>, int<>), a record whose extent
// holds no trailing bytes has count = (extent left after the count word -
// fixed tail) / 4, so the sizes pass reads one length word per record fewer
// (the string's, at a fixed offset from the record start) and the place
// kernel, which stages every byte anyway, checks each decoded record's count
// word against the derived count.  Any record the derivation cannot settle
// (trailing bytes, a short tail, a mismatching count word, a capacity error, a
// block of big records) clears *spec, and the exact walk reruns the decode
// (spec_mode 2) from a reset error key: results and first-bad errors are then
// exactly the walk's.  The derived pass reports only errors of checks that
// come before the derived count word in Xdr's order (Xdr.java:171-531).
// (spec_mode 3, one pass: every block runs, its look-back chain needs them all)
__device__ __forceinline__ bool spec_skip(const RecArgs &a) {
    if (a.spec_mode != 1 && a.spec_mode != 2) return false;
    const uint32_t s = __hip_atomic_load(a.spec, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return a.spec_mode == 1 ? s == 0 : s != 0;
}
__device__ __forceinline__ void spec_fail(const RecArgs &a) { atomicAnd(a.spec, 0u); }

__global__ void k_spec_reset(const uint32_t *spec, unsigned long long *errkey) {
    if (threadIdx.x == 0 && *spec == 0) *errkey = kNoError;
}

// ---- scan of per-block sums: one block (1024 threads) per row ---------------
// gate (nullable): the exact rerun's scan runs only when *gate == 0 (spec failed)
__global__ __launch_bounds__(1024) void k_scan_rows(uint64_t *sums, uint64_t nblocks,
                                                    uint64_t *totals, const uint32_t *gate) {
    if (gate && *gate != 0) return;
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
// XDR size of record r of a schema with conditional fields (mark included).
__device__ uint64_t enc_rec_size_cond(const RecArgs &a, uint64_t r) {
    uint64_t s = a.framed ? 4 : 0;
    Disc dv;
    dv.pres = 0;
    for (uint32_t k = 0; k < a.nf; ++k) {
        const VField &f = a.f[k];
        if (!cond_present(a, f, dv)) continue;
        cond_mark(f, k, f.slot ? disc_native(f, r) : 0, dv);
        if (k + 1 == a.byref) { s += 4; continue; }   // by reference: the length word only
        s += f.kind != XDRG_K_DYNAMIC ? (uint64_t)f.xbytes
                                      : dyn_xdr_bytes(f, f.offsets[r + 1] - f.offsets[r]);
    }
    return s;
}

__device__ __forceinline__ uint64_t enc_rec_size(const RecArgs &a, uint64_t r) {
    if (a.ncond || a.byref) return enc_rec_size_cond(a, r);
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
    const uint64_t mark_at = pos;
    uint64_t ref_bytes = 0;   // payload + pad of a by-reference field (not in `out`)
    if (a.framed) pos += 4;
    Disc dv;
    dv.pres = 0;
    for (uint32_t k = 0; k < a.nf; ++k) {
        const VField &f = a.f[k];
        if (a.ncond) {   // absent union arm / optional value: nothing on the wire
            if (!cond_present(a, f, dv)) {
                if (k + 1 == a.byref && lane == 0) a.ref_pos[r] = ~0ull;
                continue;
            }
            cond_mark(f, k, f.slot ? disc_native(f, r) : 0, dv);
        }
        if (k + 1 == a.byref) {
            // xdrEncodeFileChunk (Xdr.java:978-988): the length word here, the
            // payload and its padding spliced in by the sender at pos + 4
            const uint64_t cnt = f.offsets[r + 1] - f.offsets[r];
            if (lane == 0) {
                *(uint32_t *)(out + pos) = bswap32r((uint32_t)cnt);
                a.ref_pos[r] = pos + 4;
            }
            ref_bytes = cnt + pad4(cnt);
            pos += 4;
            continue;
        }
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
    // one mark over every part of the message (GrizzlyRpcTransport.java:103-110,
    // sendRawTCP :135-139 with a file chunk)
    if (a.framed && lane == 0)
        *(uint32_t *)(out + mark_at) = bswap32r((uint32_t)(size - 4 + ref_bytes) | kLastFrag);
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
    Disc dv;
    dv.pres = 0;
    for (uint32_t k = 0; k < a.nf; ++k) {
        const VField &f = a.f[k];
        *sub = 2 * k + 1;
        if (a.ncond && !cond_present(a, f, dv)) continue;
        if (f.kind != XDRG_K_DYNAMIC) {
            // ensureBytes per element / per opaque (Xdr.java:1028-1032)
            if (e.b - pos < f.xbytes) return XDRG_E_SHORT;
            if (a.ncond) cond_mark(f, k, f.slot ? (int32_t)ld_be32(a.xdr + pos) : 0, dv);
            pos += f.xbytes;
            continue;
        }
        if (a.ncond) cond_mark(f, k, 0, dv);
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
    Disc dv;
    dv.pres = 0;
    for (uint32_t k = 0; k < upto; ++k) {
        const VField &f = a.f[k];
        if (a.ncond) {
            if (!cond_present(a, f, dv)) {
                if (k + 1 == a.byref && lane == 0) a.ref_pos[r] = ~0ull;
                // absent: a fixed field reads as zero (a fresh rpcgen object's
                // default); a dynamic one has an empty run (count 0 from the walk)
                if (f.kind != XDRG_K_DYNAMIC) {
                    uint8_t *base = f.data + (int64_t)r * f.stride;
                    const uint32_t nb = f.type == XDRG_T_OPAQUE ? f.count
                                      : (f.kind == XDRG_K_FIXED ? f.count : 1u) * f.nsz;
                    for (uint32_t i = lane; i < nb; i += 64) base[i] = 0;
                }
                continue;
            }
            cond_mark(f, k, f.slot ? (int32_t)ld_be32(in + pos) : 0, dv);
        }
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
        if (k + 1 == a.byref) {   // xdrDecodeByteBuffer (Xdr.java:423-439): a slice, no copy
            if (lane == 0) a.ref_pos[r] = pos;
            pos += cnt + pad4(cnt);
            continue;
        }
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
                if (r < bad && k + 1 != a.byref && off + c[j] > f.cap) {   // native column too small
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
typedef uint32_t u32x4n __attribute__((ext_vector_type(4)));   // 16-byte aligned

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

// Average XDR bytes per record of this block >= a.big_rec (the split between
// the group and the staged kernels, both launched over the whole grid).
// Encode reads the scanned block sums, decode the record extents.
__device__ __forceinline__ bool block_is_big_at(const RecArgs &a, uint64_t b, bool decode) {
    const uint64_t rb = b * kRecPerBlock;
    const uint64_t nrec = a.n - rb < (uint64_t)kRecPerBlock ? a.n - rb : (uint64_t)kRecPerBlock;
    uint64_t bytes;
    if (!decode) bytes = (b + 1 < a.nblocks ? a.block_sums[b + 1] : a.totals[0]) - a.block_sums[b];
    else if (a.rec_in) bytes = a.rec_in[rb + nrec] - a.rec_in[rb];
    else bytes = a.rec_stride * nrec;
    return bytes >= (uint64_t)a.big_rec * nrec;
}
__device__ __forceinline__ bool block_is_big(const RecArgs &a, bool decode) {
    return block_is_big_at(a, blockIdx.x, decode);
}

// ---- decode ------------------------------------------------------------------------
// Walk record r (known valid) and store each dynamic field's count at
// cnt_row[d * kRecPerBlock]; returns the record's first payload byte.
__device__ __forceinline__ uint32_t walk_counts(const RecArgs &a, uint64_t r, uint32_t *cnt_row,
                                                uint32_t *sub, uint64_t *start, uint64_t *bytes,
                                                uint32_t stride = kRecPerBlock) {
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
    Disc dv;
    dv.pres = 0;
    for (uint32_t k = 0; k < a.nf; ++k) {
        const VField &f = a.f[k];
        *sub = 2 * k + 1;
        if (a.ncond && !cond_present(a, f, dv)) {   // absent arm: count 0
            if (f.kind == XDRG_K_DYNAMIC) ++d;
            continue;
        }
        if (f.kind != XDRG_K_DYNAMIC) {
            if (e.b - pos < f.xbytes) return XDRG_E_SHORT;
            if (a.ncond) cond_mark(f, k, f.slot ? (int32_t)ld_be32(a.xdr + pos) : 0, dv);
            pos += f.xbytes;
            continue;
        }
        if (a.ncond) cond_mark(f, k, 0, dv);
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
        cnt_row[(size_t)d * stride] = (uint32_t)len;
        ++d;
    }
    return 0;
}

// The kRecPerThread records r0 + j * rs of a thread walked in lockstep, field by field
// (schemas without conditional fields): their length words are independent
// loads, issued together (clamped addresses, no per-load guard) before any
// is used, so a thread waits once per dynamic field instead of once per
// record and field as the serial walk_counts does.  Per record the checks
// and their order are walk_counts' (Xdr.java:171-531, 1028-1037): err[j] =
// 0 or the code of its first failing check, sub[j] that check's position;
// counts are stored for the dynamic fields the walk passed.
// SPEC (extent-derived counts, key 31): the last dynamic field's count word
// is not read; the count is what the extent leaves after it and the fixed
// tail (`tail` bytes), and *unc is set when that is not a whole count.
template <bool SPEC = false>
__device__ __forceinline__ void walk_counts_lockstep(const RecArgs &a, uint64_t r0, uint32_t nj,
                                                     uint32_t *cnt_row, uint32_t (&err)[kRecPerThread],
                                                     uint32_t (&sub)[kRecPerThread], uint32_t rs = 1,
                                                     uint32_t tail = 0, bool *unc = nullptr) {
    constexpr uint32_t kNone = 0xffu;                         // slot past the batch end
    const uint8_t *dummy = (const uint8_t *)a.block_sums;     // any 4 readable bytes
    uint64_t pos[kRecPerThread], end[kRecPerThread];
#pragma unroll
    for (int j = 0; j < kRecPerThread; ++j) {
        sub[j] = 0;
        if ((uint32_t)j < nj) {
            const Extent e = rec_extent(a, r0 + (uint64_t)j * rs);
            pos[j] = e.a; end[j] = e.b; err[j] = 0;
        } else {
            pos[j] = end[j] = 0; err[j] = kNone;
        }
    }
    if (a.framed) {   // one single-fragment message per record (GrizzlyRpcTransport:103-110)
        uint32_t m[kRecPerThread];
#pragma unroll
        for (int j = 0; j < kRecPerThread; ++j) {
            const bool ok = !err[j] && end[j] - pos[j] >= 4;
            m[j] = *(const uint32_t *)(ok ? a.xdr + pos[j] : dummy);
        }
        // branch-free: the per-record branches of this check, inlined into the
        // one-pass sweep (and into a device-function form of the sizes
        // kernel), lost the FRAME error of a record cut short by in_len on
        // this compiler (ROCm 7.2; a printf in the branch made it correct):
        // the join after the size compare runs the matched edge's phi copy
        // of err under the restored exec of every LAST-set lane, see
        // profiles/r04_compiler/README.md; selects keep one straight-line
        // form (tests/test_spec_counts.py)
#ifndef XDRG_BRANCHY_MARK
#pragma unroll
        for (int j = 0; j < kRecPerThread; ++j) {
            const uint64_t left = end[j] - pos[j];
            const uint32_t mk = bswap32r(m[j]);
            const uint64_t want_len = a.rec_in ? left - 4 : a.rec_stride - 4;
            const bool frame_ok = (mk & kLastFrag) && (uint64_t)(mk & kSizeMask) == want_len;
            const uint32_t e = left < 4 ? (uint32_t)XDRG_E_SHORT : (frame_ok ? 0u : (uint32_t)XDRG_E_FRAME);
            const bool live = err[j] == 0;
            err[j] = live ? e : err[j];
            pos[j] += (live && !e) ? 4 : 0;
        }
#else   // experiment build (tools/mkexp.sh branchy -DXDRG_BRANCHY_MARK): round 3's branchy form
#pragma unroll
        for (int j = 0; j < kRecPerThread; ++j) {
            if (err[j]) continue;
            if (end[j] - pos[j] < 4) { err[j] = XDRG_E_SHORT; continue; }
            const uint32_t mk = bswap32r(m[j]);
            const uint64_t want_len = a.rec_in ? end[j] - pos[j] - 4 : a.rec_stride - 4;
#ifdef XDRG_BRANCHY_PRINTF
            if (!(mk & kLastFrag) || (uint64_t)(mk & kSizeMask) != want_len) {
                if (r0 + (uint64_t)j * rs + 1 == a.n) printf("frame r=%llu\n", (unsigned long long)(r0 + j * rs));
                err[j] = XDRG_E_FRAME;
                continue;
            }
#else
            if (!(mk & kLastFrag) || (uint64_t)(mk & kSizeMask) != want_len) { err[j] = XDRG_E_FRAME; continue; }
#endif
            pos[j] += 4;
        }
#endif
    }
    uint32_t d = 0;
    for (uint32_t k = 0; k < a.nf; ++k) {
        const VField &f = a.f[k];
        if (f.kind != XDRG_K_DYNAMIC) {
#pragma unroll
            for (int j = 0; j < kRecPerThread; ++j) {
                if (err[j]) continue;
                sub[j] = 2 * k + 1;
                if (end[j] - pos[j] < f.xbytes) err[j] = XDRG_E_SHORT;   // ensureBytes
                else pos[j] += f.xbytes;
            }
            continue;
        }
        const bool derive = SPEC && d + 1 == a.ndyn;   // count from the extent, word not read
        uint32_t w[kRecPerThread];
#pragma unroll
        for (int j = 0; j < kRecPerThread; ++j) {   // all length words in flight
            const bool ok = !derive && !err[j] && end[j] - pos[j] >= 4;
            w[j] = derive ? 0u : *(const uint32_t *)(ok ? a.xdr + pos[j] : dummy);
        }
#pragma unroll
        for (int j = 0; j < kRecPerThread; ++j) {
            if (err[j]) continue;
            sub[j] = 2 * k + 1;
            if (end[j] - pos[j] < 4) { err[j] = XDRG_E_SHORT; continue; }   // length word (Xdr.java:171-175)
            int32_t len;
            if (derive) {
                const uint64_t left = end[j] - pos[j] - 4;   // after the count word
                const uint64_t body = left - tail;
                if (left < tail || body % f.xsz || body / f.xsz > 0x7fffffffull) {
                    *unc = true;        // the count word decides: exact rerun
                    err[j] = kNone;     // (reported as no error; the rerun reports)
                    continue;
                }
                len = (int32_t)(body / f.xsz);
            } else {
                len = (int32_t)bswap32r(w[j]);
            }
            pos[j] += 4;
            uint64_t need;
            if (f.xsz == 1) {
                if (len == 0) need = 0;                                      // Xdr.java:376-378
                else if (len < 0) { err[j] = XDRG_E_CORRUPT; continue; }     // checkArraySize :1034-1037
                else need = (uint64_t)len + pad4((uint64_t)len);
            } else {
                if (len < 0) { err[j] = XDRG_E_CORRUPT; continue; }
                need = (uint64_t)len * f.xsz;
            }
            if (end[j] - pos[j] < need) { err[j] = XDRG_E_SHORT; continue; }
            pos[j] += need;
            cnt_row[(size_t)d * kRecPerBlock + j * rs] = (uint32_t)len;
        }
        ++d;
    }
#pragma unroll
    for (int j = 0; j < kRecPerThread; ++j)
        if (err[j] == kNone) err[j] = 0;
}

// LDS: scnt[ND][RPB] u32.  Also stores every record's counts in
// a.rec_cnt[d * n + r] so the place kernel never walks the stream again.
// SPEC: the extent-derived pass (tuning key 31, spec_mode 1).
// Blocks loop over record blocks b = blockIdx.x + k * gridDim.x when LOOP
// (the derived-count decode's exact rerun launches a small grid, so a rerun
// that is not needed costs a few microseconds); otherwise one block each.
template <bool SPEC, bool LOOP = false>
__global__ __launch_bounds__(kRecThreads) void k_dec_sizes_g(const RecArgs a) {
    if (!SPEC && spec_skip(a)) return;   // the exact rerun, and the derived counts held
    for (uint64_t bid = blockIdx.x; bid < a.nblocks; bid += gridDim.x) {
        extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
        uint32_t *scnt = (uint32_t *)smem;
        const uint64_t rb = bid * kRecPerBlock;
        const uint32_t t0 = threadIdx.x * kRecPerThread;
        bool dead = false;
        // a block of big records goes to the group kernel, which does not verify: exact rerun
        if (SPEC && threadIdx.x == 0 && a.big_rec && block_is_big_at(a, bid, true)) spec_fail(a);
        if (!a.ncond) {
            // thread t walks records rb + t + 256 j: each length-word load of a
            // wave covers 64 consecutive records, so neighbouring records' words
            // share cache lines inside one instruction (one line fetch each)
            const uint32_t t = threadIdx.x;
#pragma unroll
            for (int j = 0; j < kRecPerThread; ++j)
                for (uint32_t d = 0; d < a.ndyn; ++d) scnt[(size_t)d * kRecPerBlock + t + j * kRecThreads] = 0;
            const uint64_t r0 = rb + t;
            const uint32_t nj = r0 < a.n ? (uint32_t)((a.n - r0 + kRecThreads - 1) / kRecThreads < (uint64_t)kRecPerThread
                                                      ? (a.n - r0 + kRecThreads - 1) / kRecThreads : (uint64_t)kRecPerThread)
                                         : 0u;
            uint32_t err[kRecPerThread], sub[kRecPerThread];
            uint32_t tail = 0;   // fixed XDR bytes after the last dynamic field
            for (uint32_t k = a.dyn_idx[a.ndyn ? a.ndyn - 1 : 0] + 1; SPEC && k < a.nf; ++k) tail += a.f[k].xbytes;
            bool unc = false;
            walk_counts_lockstep<SPEC>(a, r0, nj, scnt + t, err, sub, kRecThreads, tail, &unc);
            if (SPEC && unc) spec_fail(a);
#pragma unroll
            for (int j = 0; j < kRecPerThread; ++j) {
                if (!dead && err[j]) {
                    atomicMin(a.errkey, err_key(r0 + (uint64_t)j * kRecThreads, sub[j], err[j]));
                    dead = true;   // later records of this thread are past the error
                }
                if (dead)
                    for (uint32_t d = 0; d < a.ndyn; ++d) scnt[(size_t)d * kRecPerBlock + t + j * kRecThreads] = 0;
            }
        }
        for (int j = 0; a.ncond && j < kRecPerThread; ++j) {   // conditional schemas: serial walk
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
            if (threadIdx.x == 0) a.block_sums[(uint64_t)d * a.nblocks + bid] = tot;
        }
        if (!LOOP) break;
        __syncthreads();   // (LDS reuse by the next block)
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

// The low `n` bytes of a dword (n clamped to 0..4), in 32-bit arithmetic.
__device__ __forceinline__ uint32_t lo_mask(int32_t n) {
    return n <= 0 ? 0u : n >= 4 ? ~0u : (1u << (8 * n)) - 1u;
}

struct Chunk5 { uint32_t q0, q1, q2, q3, q4; };

__device__ __forceinline__ uint32_t pow2_lanes(uint64_t bytes_per_rec, uint32_t bytes_per_lane) {
    uint32_t g = 1;
    while (g < 64 && (uint64_t)g * bytes_per_lane < bytes_per_rec) g <<= 1;
    return g;
}

// ---- 16-byte chunk helpers ---------------------------------------------------
// A lane moves one 16-byte chunk of a record's field at a time.  The copy
// loops keep U chunks of each of R records (R iterations of the group's
// record loop) in flight per lane: every load of an iteration is issued
// unconditionally, before any value is used, so the wave waits once per
// iteration instead of once per load.  (Loads guarded by per-lane
// conditions were each followed by their own s_waitcnt vmcnt(0), one
// outstanding load per wave)
//
// A Span is the 4-aligned extent [loA, endA) holding a source's valid bytes
// (a native column or the XDR stream).  A chunk reads a 20-byte window at a
// 4-aligned address w; the load is clamped into [loA, hi = endA - 20] so it
// never touches a page without valid bytes.  Windows that had to be clamped
// (the first/last chunks of a span, or a span shorter than 20 bytes: then
// every load reads `dummy`, any 20 readable bytes) are re-read word by word
// after all loads of the iteration are in flight.  Bytes a window holds
// beyond its record belong to neighbouring records and are masked on store.
struct Span {
    const uint8_t *loA, *endA, *hi, *dummy;
};
__device__ __forceinline__ Span make_span(const uint8_t *first, const uint8_t *end, const uint8_t *dummy) {
    Span s;
    s.loA = (const uint8_t *)((uintptr_t)first & ~(uintptr_t)3);
    s.endA = (const uint8_t *)(((uintptr_t)end + 3) & ~(uintptr_t)3);
    s.hi = (uintptr_t)s.endA >= (uintptr_t)s.loA + 20 ? s.endA - 20 : nullptr;
    s.dummy = dummy;
    return s;
}
__device__ __forceinline__ const uint8_t *span_clamp(const Span &s, const uint8_t *w) {
    if (!s.hi) return s.dummy;
    return w < s.loA ? s.loA : (w > s.hi ? s.hi : w);
}
__device__ __forceinline__ uint32_t span_word(const Span &s, const uint8_t *a) {
    return (a >= s.loA && a < s.endA) ? *(const uint32_t *)a : 0u;
}
// Unconditional window load (+ the fifth word when five are needed).
__device__ __forceinline__ void win_load(Chunk5 &q, const Span &s, const uint8_t *w, bool five) {
    const uint8_t *pa = span_clamp(s, w);
    const u32x4a v = *(const u32x4a *)pa;
    q.q0 = v.x; q.q1 = v.y; q.q2 = v.z; q.q3 = v.w;
    q.q4 = five ? *(const uint32_t *)(pa + 16) : 0u;
}
// After the wait: redo a clamped window word by word.
__device__ __forceinline__ void win_fix(Chunk5 &q, const Span &s, const uint8_t *w, bool five) {
    if (span_clamp(s, w) == w) return;
    q.q0 = span_word(s, w); q.q1 = span_word(s, w + 4);
    q.q2 = span_word(s, w + 8); q.q3 = span_word(s, w + 12);
    q.q4 = five ? span_word(s, w + 16) : 0u;
}

// Blob [BE length][payload][zero pad] of an opaque/string field
// (Xdr.java:776-800): chunk c covers blob bytes [16c, 16c + 16).  The
// payload starts at src (any alignment, sh = src & 3); q0..q4 are the words
// at src - sh + 16c - 4 + 4m.
__device__ __forceinline__ const uint8_t *blob_win(const uint8_t *src, uint64_t c) {
    return src - ((uintptr_t)src & 3) + 16 * c - 4;
}
template <bool NT = false>
__device__ __forceinline__ void blob_store(uint8_t *dst, const Chunk5 &q, uint32_t sh, uint64_t c, uint64_t cnt) {
    const uint64_t nwb = 1 + ((cnt + 3) >> 2);
    uint32_t o0 = sh ? __builtin_amdgcn_alignbyte(q.q1, q.q0, sh) : q.q0;
    uint32_t o1 = sh ? __builtin_amdgcn_alignbyte(q.q2, q.q1, sh) : q.q1;
    uint32_t o2 = sh ? __builtin_amdgcn_alignbyte(q.q3, q.q2, sh) : q.q2;
    uint32_t o3 = sh ? __builtin_amdgcn_alignbyte(q.q4, q.q3, sh) : q.q3;
    const int64_t rem = 4 + (int64_t)cnt - 16 * (int64_t)c;   // blob bytes from chunk start
    if (rem < 16) {   // zero pad (Xdr.java:765)
        o0 = mask_bytes(o0, rem); o1 = mask_bytes(o1, rem - 4);
        o2 = mask_bytes(o2, rem - 8); o3 = mask_bytes(o3, rem - 12);
    }
    if (c == 0) o0 = bswap32r((uint32_t)cnt);
    uint8_t *d = dst + 16 * c;
    if (4 * c + 4 <= nwb) {
        u32x4a o; o.x = o0; o.y = o1; o.z = o2; o.w = o3;
        if (NT) __builtin_nontemporal_store(o, (u32x4a *)d);
        else *(u32x4a *)d = o;
    } else {
        const uint64_t left = nwb - 4 * c;
        *(uint32_t *)d = o0;
        if (left > 1) *(uint32_t *)(d + 4) = o1;
        if (left > 2) *(uint32_t *)(d + 8) = o2;
    }
}

// Chunk index a slot loads: inactive slots (c >= nch) re-read their
// record's last chunk (a line the active slots fetch anyway).
__device__ __forceinline__ uint64_t ld_chunk(uint64_t c, uint64_t nch) {
    return c < nch ? c : (nch ? nch - 1 : 0);
}

// Chunks of R opaque/string blobs; nch[r] = 0 marks an unused slot.
template <int U, int R>
__device__ __forceinline__ void enc_blob_bytes(uint8_t *const (&dst)[R], const uint8_t *const (&src)[R],
                                               const uint64_t (&cnt)[R], const uint64_t (&nch)[R],
                                               const Span &sp, uint32_t G, uint32_t gl) {
    uint64_t mx = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) mx = nch[r] > mx ? nch[r] : mx;
    for (uint64_t c0 = gl; c0 < mx; c0 += (uint64_t)G * U) {
        Chunk5 ch[R][U];
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int u = 0; u < U; ++u)
                win_load(ch[r][u], sp, blob_win(src[r], ld_chunk(c0 + (uint64_t)u * G, nch[r])), true);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint32_t sh = (uint32_t)((uintptr_t)src[r] & 3);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint64_t c = c0 + (uint64_t)u * G;
                if (c >= nch[r]) continue;
                win_fix(ch[r][u], sp, blob_win(src[r], c), true);
                blob_store(dst[r], ch[r][u], sh, c, cnt[r]);
            }
        }
    }
}

// int/uint/enum/float vector as one blob: [BE count][BE elements...]; blob
// word b is element b - 1 of the 4-aligned native run src, so chunk c
// reads the words at src + 16c - 4.
template <bool NT = false>
__device__ __forceinline__ void w4_store(uint8_t *dst, const Chunk5 &q, uint64_t c, uint64_t cnt, bool fl) {
    const uint64_t nwb = 1 + cnt;
    uint32_t o[4] = {q.q0, q.q1, q.q2, q.q3};
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = bswap32r(fl ? canon_f32r(o[j]) : o[j]);
    if (c == 0) o[0] = bswap32r((uint32_t)cnt);
    uint32_t *d = (uint32_t *)(dst + 16 * c);
    if (4 * c + 4 <= nwb) {
        u32x4a ov; ov.x = o[0]; ov.y = o[1]; ov.z = o[2]; ov.w = o[3];
        if (NT) __builtin_nontemporal_store(ov, (u32x4a *)d);
        else *(u32x4a *)d = ov;
    } else {
        for (uint64_t j = 0; 4 * c + j < nwb; ++j) d[j] = o[j];
    }
}
template <int U, int R>
__device__ __forceinline__ void enc_blob_words4(uint8_t *const (&dst)[R], const uint8_t *const (&src)[R],
                                                const uint64_t (&cnt)[R], const uint64_t (&nch)[R], bool fl,
                                                const Span &sp, uint32_t G, uint32_t gl) {
    uint64_t mx = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) mx = nch[r] > mx ? nch[r] : mx;
    for (uint64_t c0 = gl; c0 < mx; c0 += (uint64_t)G * U) {
        Chunk5 ch[R][U];
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int u = 0; u < U; ++u)
                win_load(ch[r][u], sp, src[r] + 16 * ld_chunk(c0 + (uint64_t)u * G, nch[r]) - 4, false);
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint64_t c = c0 + (uint64_t)u * G;
                if (c >= nch[r]) continue;
                win_fix(ch[r][u], sp, src[r] + 16 * c - 4, false);
                w4_store(dst[r], ch[r][u], c, cnt[r], fl);
            }
    }
}

// XDR payload (4-aligned src, cnt bytes) -> native bytes at any alignment.
// Destination dwords are aligned: da = dst - sh; chunk c covers native
// dwords 4c..4c+3 and reads the stream words at src + 16c - 4 (q0 = the
// word before the chunk, q1..q4 its words).  Partial head/tail dwords are
// written byte by byte: their other bytes belong to neighbouring records.
__device__ __forceinline__ void dec_store(uint8_t *da, const Chunk5 &w, uint64_t c, uint64_t cnt, uint32_t sh) {
    const uint64_t i0 = 4 * c, nd = (sh + cnt + 3) >> 2;
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
        return;
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
template <int U, int R>
__device__ __forceinline__ void dec_bytes(uint8_t *const (&dst)[R], const uint8_t *const (&src)[R],
                                          const uint64_t (&cnt)[R], const uint64_t (&nch)[R],
                                          const Span &sp, uint32_t G, uint32_t gl) {
    uint64_t mx = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) mx = nch[r] > mx ? nch[r] : mx;
    for (uint64_t c0 = gl; c0 < mx; c0 += (uint64_t)G * U) {
        Chunk5 ch[R][U];
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int u = 0; u < U; ++u)
                win_load(ch[r][u], sp, src[r] + 16 * ld_chunk(c0 + (uint64_t)u * G, nch[r]) - 4, true);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint32_t sh = (uint32_t)((uintptr_t)dst[r] & 3);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint64_t c = c0 + (uint64_t)u * G;
                if (c >= nch[r]) continue;
                win_fix(ch[r][u], sp, src[r] + 16 * c - 4, true);
                dec_store(dst[r] - sh, ch[r][u], c, cnt[r], sh);
            }
        }
    }
}

// [BE elements] (4-aligned stream) -> native int/uint/enum/float run.
template <int U, int R>
__device__ __forceinline__ void dec_words4(uint8_t *const (&dst)[R], const uint8_t *const (&src)[R],
                                           const uint64_t (&cnt)[R], const uint64_t (&nch)[R],
                                           const Span &sp, uint32_t G, uint32_t gl) {
    uint64_t mx = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) mx = nch[r] > mx ? nch[r] : mx;
    for (uint64_t c0 = gl; c0 < mx; c0 += (uint64_t)G * U) {
        Chunk5 ch[R][U];
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int u = 0; u < U; ++u)
                win_load(ch[r][u], sp, src[r] + 16 * ld_chunk(c0 + (uint64_t)u * G, nch[r]), false);
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint64_t c = c0 + (uint64_t)u * G;
                if (c >= nch[r]) continue;
                win_fix(ch[r][u], sp, src[r] + 16 * c, false);
                const uint32_t w[4] = {ch[r][u].q0, ch[r][u].q1, ch[r][u].q2, ch[r][u].q3};
                uint32_t *d = (uint32_t *)(dst[r] + 16 * c);
                if (4 * c + 4 <= cnt[r]) {
                    u32x4a o;
                    o.x = bswap32r(w[0]); o.y = bswap32r(w[1]); o.z = bswap32r(w[2]); o.w = bswap32r(w[3]);
                    *(u32x4a *)d = o;
                } else {
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        if (4 * c + j < cnt[r]) d[j] = bswap32r(w[j]);
                }
            }
    }
}


template <int U, int R>
__global__ __launch_bounds__(kRecThreads) void k_enc_place_g(const RecArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint64_t *soff = (uint64_t *)smem;
    uint64_t *ssrc = soff + kRecPerBlock + 2;
    uint32_t *scnt = (uint32_t *)(ssrc + (size_t)a.ndyn * kRecPerBlock);
    const uint64_t total = a.totals[0];
    if (total > a.xdr_cap) return;  // XDRG_E_CAPACITY: write nothing
    if (a.big_rec && !block_is_big(a, false)) return;   // the staged kernel's block
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
    if (a.payk) {   // k_enc_payload writes these records whole: hand over the payload positions
        for (uint32_t j = tid; j < nrec; j += kRecThreads) a.pay_pos[rb + j] = soff[j] + a.pay_fb;
        return;
    }
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
                for (uint32_t j0 = tid / G; j0 < nrec; j0 += ng * R) {
                    for (uint32_t i = gl; i < nw; i += G) {
                        uint32_t v[R];
#pragma unroll
                        for (int r = 0; r < R; ++r) {   // unconditional: a past-the-end slot re-reads the last record
                            const uint32_t j = j0 + r * ng < nrec ? j0 + r * ng : (uint32_t)nrec - 1;
                            v[r] = fixed_word(f, rb + j, 4 * i);
                        }
#pragma unroll
                        for (int r = 0; r < R; ++r) {
                            const uint32_t j = j0 + r * ng;
                            if (j < nrec) *(uint32_t *)(out + soff[j] + fixed_delta + 4 * i) = v[r];
                        }
                    }
                }
            }
            fixed_delta += f.xbytes;
            continue;
        }
        const uint32_t *cn = scnt + (size_t)d * kRecPerBlock;
        const uint64_t *sr = ssrc + (size_t)d * kRecPerBlock;
        if (a.payk == d + 1) {   // k_enc_payload moves this field: hand over its position
            for (uint32_t j = tid; j < nrec; j += kRecThreads) a.pay_pos[rb + j] = soff[j] + fixed_delta;
            __syncthreads();
            for (uint32_t j = tid; j < nrec; j += kRecThreads) soff[j] += dyn_xdr_bytes(f, cn[j]);
            __syncthreads();
            ++d;
            continue;
        }
        uint64_t ps = 0;
        for (uint32_t j = tid; j < nrec; j += kRecThreads) ps += cn[j];
        const uint64_t fbytes = block_sum(ps) * (f.xsz == 1 ? 1 : f.xsz) + 4 * nrec;
        const uint32_t G = a.force_g ? a.force_g : pow2_lanes(nrec ? fbytes / nrec : 0, a.lane_bytes_enc);
        const uint32_t gl = tid & (G - 1), ng = kRecThreads / G;
        const bool bytes = f.xsz == 1, w4 = is_word4(f);
        const uint64_t esz = bytes ? 1 : f.nsz;
        const Span sp = make_span(f.data + f.offsets[0] * esz, f.data + f.offsets[a.n] * esz,
                                  (const uint8_t *)a.block_sums);
        for (uint32_t j0 = tid / G; j0 < nrec; j0 += ng * R) {
            uint8_t *dst[R];
            const uint8_t *src[R];
            uint64_t cnt[R], nch[R];
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const uint32_t j = j0 + r * ng;
                const bool live = j < nrec;
                cnt[r] = live ? cn[j] : 0;
                const uint64_t e0 = live ? sr[j] : 0;
                dst[r] = out + (live ? soff[j] : 0) + fixed_delta;
                src[r] = f.data + (bytes ? e0 : e0 * f.nsz);
                const uint64_t nwb = 1 + (bytes ? (cnt[r] + 3) >> 2 : cnt[r] * (f.xsz >> 2));
                nch[r] = live ? (nwb + 3) >> 2 : 0;
            }
            if (bytes) {
                enc_blob_bytes<U, R>(dst, src, cnt, nch, sp, G, gl);
            } else if (w4) {
                enc_blob_words4<U, R>(dst, src, cnt, nch, f.type == XDRG_T_FLOAT, sp, G, gl);
            } else {
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    if (!nch[r]) continue;
                    const uint64_t e0 = sr[j0 + r * ng];
                    if (gl == 0) *(uint32_t *)dst[r] = bswap32r((uint32_t)cnt[r]);
                    const uint64_t nw = cnt[r] * (f.xsz >> 2);
                    for (uint64_t i = gl; i < nw; i += G)
                        *(uint32_t *)(dst[r] + 4 + 4 * i) = dyn_word(f, e0, cnt[r], 4 + 4 * i);
                }
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

constexpr int kHeadRecs = 4, kHeadWords = 8;   // dec_place_g_block's head words: records per lane, words
template <int U, int R>
__device__ __forceinline__ void dec_place_g_block(const RecArgs &a, uint64_t bid) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint64_t *sstart = (uint64_t *)smem;
    uint64_t *snoff = sstart + kRecPerBlock;
    uint32_t *scnt = (uint32_t *)(snoff + (size_t)a.ndyn * kRecPerBlock);
    uint32_t *supto = scnt + (size_t)a.ndyn * kRecPerBlock;
    if (a.big_rec && !block_is_big_at(a, bid, true)) return;   // the staged kernel's block
    const uint64_t rb = bid * kRecPerBlock;
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
        uint64_t off = a.block_sums[(uint64_t)d * a.nblocks + bid] + block_excl_scan(s, &btot);
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
        if (bid == 0 && threadIdx.x == 0) f.offsets[a.n] = a.totals[d];
    }
    __syncthreads();
    uint64_t nrec = a.n > rb ? a.n - rb : 0;
    if (nrec > kRecPerBlock) nrec = kRecPerBlock;
    const uint8_t *in = a.xdr;
    const uint32_t tid = threadIdx.x;
    uint64_t fixed_delta = 0;
    uint32_t d = 0, k = 0;
    {   // The fixed fields before the first dynamic one (config 3's head words):
        // a lane per record, every head word of kHeadRecs records in flight
        // before the column stores.  The field loop below keeps one load per
        // lane in flight, and these heads sit a record apart (4 KiB in config 3).
        uint32_t hw = 0, kd = 0;
        for (; kd < a.nf && a.f[kd].kind != XDRG_K_DYNAMIC; ++kd) hw += a.f[kd].xbytes >> 2;
        if (kd > 0 && hw <= kHeadWords) {
            for (uint32_t j0 = tid; j0 < nrec; j0 += kHeadRecs * kRecThreads) {
                uint32_t v[kHeadRecs][kHeadWords];
#pragma unroll
                for (int m = 0; m < kHeadRecs; ++m) {   // unconditional: dead slots read the workspace
                    const uint32_t j = j0 + m * kRecThreads;
                    const bool live = j < nrec && supto[j] != 0;
                    const uint8_t *p = live ? in + sstart[j] : (const uint8_t *)a.block_sums;
#pragma unroll
                    for (int i = 0; i < kHeadWords; ++i)
                        if (i < (int)hw) v[m][i] = *(const uint32_t *)(p + (live ? 4 * i : 0));
                }
#pragma unroll
                for (int i = 0; i < kHeadWords; ++i) {
                    if (i >= (int)hw) break;
                    uint32_t q = 0, w0 = 0;   // head word i is word i - w0 of field q
                    while (w0 + (a.f[q].xbytes >> 2) <= (uint32_t)i) w0 += a.f[q++].xbytes >> 2;
                    const VField &f = a.f[q];
#pragma unroll
                    for (int m = 0; m < kHeadRecs; ++m) {
                        const uint32_t j = j0 + m * kRecThreads;
                        if (j < nrec && q < supto[j]) fixed_store(f, rb + j, 4 * (i - w0), v[m][i]);
                    }
                }
            }
            k = kd;
            fixed_delta = 4 * (uint64_t)hw;
        }
    }
    for (; k < a.nf; ++k) {
        const VField &f = a.f[k];
        if (f.kind != XDRG_K_DYNAMIC) {
            const uint32_t nw = f.xbytes >> 2;
            if (nw) {
                const uint32_t G = a.force_g ? a.force_g : pow2_lanes((uint64_t)nw * 4, 16);
                const uint32_t gl = tid & (G - 1), ng = kRecThreads / G;
                for (uint32_t j0 = tid / G; j0 < nrec; j0 += ng * R) {
                    for (uint32_t i = gl; i < nw; i += G) {
                        uint32_t v[R];
#pragma unroll
                        for (int r = 0; r < R; ++r) {   // unconditional: dead slots read the workspace
                            const uint32_t j = j0 + r * ng;
                            const bool live = j < nrec && k < supto[j];
                            v[r] = *(const uint32_t *)(live ? in + sstart[j] + fixed_delta + 4 * i
                                                            : (const uint8_t *)a.block_sums);
                        }
#pragma unroll
                        for (int r = 0; r < R; ++r) {
                            const uint32_t j = j0 + r * ng;
                            if (j < nrec && k < supto[j]) fixed_store(f, rb + j, 4 * i, v[r]);
                        }
                    }
                }
            }
            fixed_delta += f.xbytes;
            continue;
        }
        const uint32_t *cn = scnt + (size_t)d * kRecPerBlock;
        const uint64_t *no = snoff + (size_t)d * kRecPerBlock;
        if (a.payk == d + 1) {   // k_dec_payload moves this field (records the walk passed only)
            for (uint32_t j = tid; j < nrec; j += kRecThreads)
                a.pay_pos[rb + j] = k < supto[j] ? sstart[j] + fixed_delta : ~0ull;
            __syncthreads();
            for (uint32_t j = tid; j < nrec; j += kRecThreads) sstart[j] += dyn_xdr_bytes(f, cn[j]);
            __syncthreads();
            ++d;
            continue;
        }
        uint64_t ps = 0;
        for (uint32_t j = tid; j < nrec; j += kRecThreads) ps += cn[j];
        const uint64_t fbytes = block_sum(ps) * (f.xsz == 1 ? 1 : f.xsz) + 4 * nrec;
        const uint32_t G = a.force_g ? a.force_g : pow2_lanes(nrec ? fbytes / nrec : 0, a.lane_bytes_dec);
        const uint32_t gl = tid & (G - 1), ng = kRecThreads / G;
        const bool bytes = f.xsz == 1, w4 = is_word4(f);
        const Span sp = make_span(in, in + a.xdr_cap, (const uint8_t *)a.block_sums);
        for (uint32_t j0 = tid / G; j0 < nrec; j0 += ng * R) {
            uint8_t *dst[R];
            const uint8_t *src[R];
            uint64_t cnt[R], nch[R];
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const uint32_t j = j0 + r * ng;
                const bool live = j < nrec && k < supto[j];
                cnt[r] = live ? cn[j] : 0;
                const uint64_t e0 = live ? no[j] : 0;
                src[r] = in + (live ? sstart[j] : 0) + fixed_delta + 4;
                dst[r] = f.data + (bytes ? e0 : e0 * f.nsz);
                const uint32_t sh = (uint32_t)((uintptr_t)dst[r] & 3);
                const uint64_t nd = bytes ? (sh + cnt[r] + 3) >> 2 : cnt[r] * (f.xsz >> 2);
                nch[r] = (live && cnt[r]) ? (nd + 3) >> 2 : 0;
            }
            if (bytes) {
                dec_bytes<U, R>(dst, src, cnt, nch, sp, G, gl);
            } else if (w4) {
                dec_words4<U, R>(dst, src, cnt, nch, sp, G, gl);
            } else {
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    if (!nch[r]) continue;
                    const uint64_t e0 = no[j0 + r * ng];
                    const uint64_t nw = cnt[r] * (f.xsz >> 2);
                    for (uint64_t i = gl; i < nw; i += G)
                        dyn_store(f, e0, cnt[r], 4 + 4 * i, *(const uint32_t *)(src[r] + 4 * i));
                }
            }
        }
        __syncthreads();
        for (uint32_t j = tid; j < nrec; j += kRecThreads) sstart[j] += dyn_xdr_bytes(f, cn[j]);
        __syncthreads();
        ++d;
    }
}
template <int U, int R, bool LOOP = false>
__global__ __launch_bounds__(kRecThreads) void k_dec_place_g(const RecArgs a) {
    if (spec_skip(a)) return;   // (a big block already cleared *spec in the derived pass)
    if (!LOOP) { dec_place_g_block<U, R>(a, blockIdx.x); return; }
    for (uint64_t b = blockIdx.x; b < a.nblocks; b += gridDim.x) {   // as k_dec_sizes_g
        dec_place_g_block<U, R>(a, b);
        __syncthreads();
    }
}

// ---- payload kernels (large byte payloads of the group kernels' blocks) -----
// Config 3's payload copy bound (tools/probes/record_copy.hip,
// profiles/r01_configs/record_copy_probe.txt): a block that owns 1024
// consecutive 4 KiB records keeps the records in flight at any moment 4 MB
// apart (28-31 ms per 64 GiB copy); only grids whose neighbouring blocks
// copy neighbouring records reach 23.5 ms.  The group kernels compute every
// record's placement (block scan) and write the other fields; for one dynamic
// byte field (opaque<> / string<>) they only store the field's stream
// position (pay_pos), and these kernels move it: a wave per record, four
// consecutive records per block, a one-pass grid, 16-byte accesses with
// four in flight per lane.  Same bytes as enc_blob_bytes / dec_bytes
// (Xdr.java:765-800 length, bytes, zero pad; :341-383 decode).
__device__ __forceinline__ bool payload_block(const RecArgs &a, uint64_t r, bool decode) {
    return !a.big_rec || block_is_big_at(a, r / kRecPerBlock, decode);
}
// XDR word at byte o (4-aligned) of record r in a schema whose one dynamic
// field is the byte field f (cnt bytes at src): the mark, the fixed fields
// before f, f's length word, its payload and zero pad (Xdr.java:776-800),
// the fixed fields after f.
__device__ uint32_t payload_rec_word(const RecArgs &a, uint64_t r, uint64_t o, uint64_t size, const uint8_t *src,
                                     uint64_t cnt) {
    const uint64_t fb = a.pay_fb, P = cnt + pad4(cnt);
    if (a.framed && o == 0) return bswap32r((uint32_t)(size - 4) | kLastFrag);   // GrizzlyRpcTransport:103-110
    if (o >= fb && o < fb + 4) return bswap32r((uint32_t)cnt);
    if (o >= fb + 4 && o < fb + 4 + P) {
        const uint64_t b = o - fb - 4;
        return b >= cnt ? 0u : (cnt - b >= 4 ? *(const u32u *)(src + b) : load_bytes(src + b, (uint32_t)(cnt - b)));
    }
    uint64_t q = a.framed ? 4 : 0;   // a fixed field's word
    if (o >= fb) o -= 4 + P;
    const uint64_t j = (o - q) >> 2;
    if (j < a.pay_nw) {   // its direct rule (fill_rec)
        const PayWord w = a.pw[j];
        const uint8_t *p = w.data + (int64_t)r * w.stride + w.off;
        return w.type == XDRG_T_OPAQUE ? load_bytes(p, w.rem) : enc_elem(w.type, p, w.half);
    }
    for (uint32_t k = 0; k < a.nf; ++k) {
        const VField &f = a.f[k];
        if (f.kind == XDRG_K_DYNAMIC) continue;
        if (o < q + f.xbytes) return fixed_word(f, r, o - q);
        q += f.xbytes;
    }
    return 0;
}

// A wave writes record r whole — mark, fixed fields, length word, payload,
// zero pad, trailing fixed fields.  Chunk c covers stream bytes
// [A + 16c, A + 16c + 16), A = the record start rounded down to 16; chunks
// inside the payload are one aligned 16-byte store from a 4-aligned load,
// the record's other words go out a dword per lane after them (the edge
// lines are shared with the neighbouring records, whose waves run alongside
// and complete them in L2).  One pass over each line: the group kernel only
// hands over the payload positions (pay_pos).
// Nontemporal 16-byte loads and stores; every metadata load is issued
// together, before the checks that use them (24.8 vs 25.6 ms with the checks
// first, profiles/r02_c3_hoist_ab.jsonl); plain stores and a smaller grid whose
// blocks stride over the records measured slower.
constexpr uint32_t kPayLanes = 64;   // lanes per record: a wave
__device__ __forceinline__ void enc_payload_rec(const RecArgs &a, uint64_t r) {
    if (r >= a.n) return;
    const VField &f = a.f[a.dyn_idx[a.payk - 1]];
    const uint64_t total = a.totals[0], e0 = f.offsets[r], e1 = f.offsets[r + 1], pp = a.pay_pos[r];
    const bool mine = payload_block(a, r, false);
    if (total > a.xdr_cap || !mine) return;
    const uint64_t cnt = e1 - e0;
    const uint64_t R = pp - a.pay_fb;   // record start
    const uint64_t P = cnt + pad4(cnt), size = a.fixed_xdr + 4 + P;
    const uint8_t *src = f.data + e0;
    constexpr uint32_t LPR = kPayLanes;
    const uint32_t lane = threadIdx.x % LPR;
    uint8_t *const A = a.xdr + (R & ~(uint64_t)15);
    const uint64_t sh = R & 15;                    // record start inside chunk 0
    const uint64_t p0 = sh + a.pay_fb + 4;         // payload start, chunk coordinates
    const uint64_t cf = (p0 + 15) >> 4, cl = (p0 + cnt) >> 4;   // payload-only chunks: [cf, cl)
    for (uint64_t c0 = cf + lane; c0 < cl; c0 += 4 * LPR) {   // payload-only chunks
        u32x4a v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {   // all loads in flight first
            const uint64_t c = c0 + LPR * u;
            if (c < cl) {
                v[u] = __builtin_nontemporal_load((const u32x4a *)(src + 16 * c - p0));   // 4-aligned
            }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint64_t c = c0 + LPR * u;
            if (c >= cl) continue;
            // the chunks of the record's first and last 128-byte lines, which
            // it shares with its own and its neighbours' head / tail words,
            // go through L2 as plain stores (var_encode 22.69 vs 23.15 ms on
            // config 3, profiles/r06_c3/edge_plain_ab.jsonl)
            if (c < ((cf + 7) & ~7ull) || c >= (cl & ~7ull)) {
                *(u32x4n *)(A + 16 * c) = v[u];
                continue;
            }
            __builtin_nontemporal_store(v[u], (u32x4n *)(A + 16 * c));
        }
    }
    // the record's words outside those chunks (mark, fixed fields, length,
    // the payload's first and last bytes, pad, trailing fixed fields): a word
    // per lane, their loads in parallel.  (Loading them before the payload
    // loop, to overlap the two round trips, measured slower: 6.41 vs 6.32 ms
    // on 4 Mi config-3 records, profiles/r05_c3/pay_head_hoist_ab.jsonl.)
    const uint64_t hw = cl > cf ? (16 * cf - sh) >> 2 : (size >> 2);   // head words
    const uint64_t tw0 = cl > cf ? (16 * cl - sh) >> 2 : (size >> 2);  // first tail word
    const uint64_t nslow = hw + (size >> 2) - tw0;
    for (uint64_t i = lane; i < nslow; i += LPR) {
        const uint64_t wi = i < hw ? i : tw0 + (i - hw);
        *(uint32_t *)(a.xdr + R + 4 * wi) = payload_rec_word(a, r, 4 * wi, size, src, cnt);
    }
}
// a block per 4 records (a wave each): neighbouring blocks on neighbouring records
// (a.xcd: blocks in XCD order, xcd_block; one pass below 2^32 records)
// (key 37 bit 0 encode, bit 1 decode: encode 24.31 ms in XCD order, decode
// 21.06 ms in block order vs 22.37 in XCD order on config 3, profiles/r04_configs)
__device__ __forceinline__ uint64_t pay_block(const RecArgs &a, uint32_t bit) {
    return (a.xcd & bit) ? xcd_block(blockIdx.x, gridDim.x) : (uint64_t)blockIdx.x;
}
__global__ __launch_bounds__(256) void k_enc_payload(const RecArgs a) {
    const uint64_t step = (uint64_t)gridDim.x * (256 / kPayLanes);
    for (uint64_t r = pay_block(a, 1) * (256 / kPayLanes) + threadIdx.x / kPayLanes; r < a.n; r += step)
        enc_payload_rec(a, r);
}
__device__ __forceinline__ void dec_payload_rec(const RecArgs &a, uint64_t r) {
    if (r >= a.n) return;
    const uint32_t d = a.payk - 1;
    const VField &f = a.f[a.dyn_idx[d]];
    // metadata loads issued together, before the checks (one round trip ahead of the data)
    const uint64_t pos = a.pay_pos[r], cnt = a.rec_cnt[(uint64_t)d * a.n + r], o = f.offsets[r];
    if (pos == ~0ull || !payload_block(a, r, true)) return;
    const uint8_t *src = a.xdr + pos + 4;
    uint8_t *dst = f.data + o;
    constexpr uint32_t LPR = kPayLanes;
    const uint32_t lane = threadIdx.x % LPR;
    // (the record's fixed fields are the group kernel's, k_dec_place_g: a wave
    // per record writing its six head words measured slower, 29.1 vs 25.2 ms
    // on config 3)
    const uint64_t nch = (cnt + 15) >> 4;
    for (uint64_t c0 = lane; c0 < nch; c0 += 4 * LPR) {
        u32x4a v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint64_t c = c0 + LPR * u;
            if (16 * c + 16 <= cnt)
                v[u] = __builtin_nontemporal_load((const u32x4a *)(src + 16 * c));
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint64_t c = c0 + LPR * u;
            if (c >= nch) continue;
            if (16 * c + 16 <= cnt) {
                __builtin_nontemporal_store(v[u], (u32x4u *)(dst + 16 * c));
                continue;
            }
            for (uint64_t b = 16 * c; b < cnt; b += 4) {   // last chunk (stream words are 4-aligned)
                const uint32_t w = *(const uint32_t *)(src + b);
                const uint64_t k = cnt - b;
                if (k >= 4) *(u32u *)(dst + b) = w;
                else for (uint32_t i = 0; i < k; ++i) dst[b + i] = (uint8_t)(w >> (8 * i));
            }
        }
    }
}
__global__ __launch_bounds__(256) void k_dec_payload(const RecArgs a) {
    const uint64_t step = (uint64_t)gridDim.x * (256 / kPayLanes);
    for (uint64_t r = pay_block(a, 2) * (256 / kPayLanes) + threadIdx.x / kPayLanes; r < a.n; r += step)
        dec_payload_rec(a, r);
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
            if (a.ncond || a.byref) size = enc_rec_size_cond(a, r);   // arms / by-reference payload
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
        uint8_t *const mark = dst;
        uint64_t ref_bytes = 0;   // by-reference payload + pad (sent beside `out`)
        if (a.framed) dst += 4;
        uint32_t d = 0;
        Disc dv;
        dv.pres = 0;
        for (uint32_t k = 0; k < a.nf; ++k) {
            const VField &f = a.f[k];
            if (a.ncond) {   // union arm / optional value not taken: nothing on the wire
                if (!cond_present(a, f, dv)) {
                    if (k + 1 == a.byref) a.ref_pos[r] = ~0ull;
                    if (f.kind == XDRG_K_DYNAMIC) ++d;
                    continue;
                }
                cond_mark(f, k, f.slot ? disc_native(f, r) : 0, dv);
            }
            if (k + 1 == a.byref) {   // xdrEncodeFileChunk (Xdr.java:978-988)
                const uint32_t cnt = scnt[(size_t)d * kRecPerBlock + j];
                *(uint32_t *)dst = bswap32r(cnt);
                dst += 4;
                a.ref_pos[r] = (uint64_t)(dst - a.xdr);
                ref_bytes = cnt + pad4(cnt);
                ++d;
                continue;
            }
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
        if (a.framed)   // GrizzlyRpcTransport.java:103-110 (sendRawTCP :135-139: every part)
            *(uint32_t *)mark = bswap32r((uint32_t)(soff[j + 1] - soff[j] - 4 + ref_bytes) | kLastFrag);
    }
}

// Lane j of the block decodes record r = rb + j from src (its first field's
// bytes in the stream), fields [0, upto).  (An LDS-tiled variant, records
// staged in sub-batches, measured slower at every tile size: DESIGN.md §5.7.)
__device__ __forceinline__ void lane_dec_record(const RecArgs &a, uint64_t r, uint32_t j, uint32_t upto,
                                                const uint8_t *src, const uint64_t *snoff, const uint32_t *scnt) {
    uint32_t d = 0;
    Disc dv;
    dv.pres = 0;
    for (uint32_t k = 0; k < upto; ++k) {
        const VField &f = a.f[k];
        if (a.ncond) {
            if (!cond_present(a, f, dv)) {
                // absent: fixed fields read as zero (a fresh rpcgen object), dynamic
                // ones have an empty run (count 0 from the walk)
                if (k + 1 == a.byref) a.ref_pos[r] = ~0ull;
                if (f.kind == XDRG_K_DYNAMIC) { ++d; continue; }
                uint8_t *base = f.data + (int64_t)r * f.stride;
                const uint32_t nb = f.type == XDRG_T_OPAQUE ? f.count
                                  : (f.kind == XDRG_K_FIXED ? f.count : 1u) * f.nsz;
                for (uint32_t i = 0; i < nb; ++i) base[i] = 0;
                continue;
            }
            cond_mark(f, k, f.slot ? (int32_t)ld_be32(src) : 0, dv);
        }
        if (f.kind != XDRG_K_DYNAMIC) {
            const uint32_t nw = f.xbytes >> 2;
            for (uint32_t i = 0; i < nw; ++i) fixed_store(f, r, 4 * i, *(const uint32_t *)(src + 4 * i));
            src += f.xbytes;
            continue;
        }
        const uint32_t cnt = scnt[(size_t)d * kRecPerBlock + j];
        if (k + 1 == a.byref) {   // xdrDecodeByteBuffer (Xdr.java:423-439): a slice
            a.ref_pos[r] = (uint64_t)(src + 4 - a.xdr);
            src += 4 + cnt + pad4(cnt);
            ++d;
            continue;
        }
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
                if (r < bad && k + 1 != a.byref && off + c > f.cap) {   // native column too small
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
        if (upto) lane_dec_record(a, rb + j, j, upto, a.xdr + sstart[j], snoff, scnt);
    }
}

// ===========================================================================
// Staged place kernels (the default for schemas whose dynamic fields are all
// opaque/string or int/uint/enum/float vectors, at most kMaxDynLds of them).
//
// Counters on config 4 (rocprofv3 FETCH_SIZE / WRITE_SIZE)
// showed that the group kernels' field-major passes over a 1024-record block
// (~180 KB of XDR) fall out of L2 between passes: encode wrote 1.5x its XDR
// bytes to HBM (partial lines written back more than once) and decode
// fetched the stream once per field.  Here a block works through its records
// in sub-batches (at most kRecThreads records) whose dynamic source bytes fit
// one LDS tile:
//   1. stage: the sub-batch's source bytes are one contiguous range per
//      column (encode: each dynamic native column; decode: the XDR stream)
//      and are copied into LDS with coalesced 16-byte loads, all in flight;
//   2. scatter: field-major over the sub-batch, a group of G lanes per record
//      reads its field from LDS and writes it with 16-byte global stores; a
//      sub-batch's output is written within one short window, so its lines
//      merge in L2 before they are written back, and no global load waits
//      behind these stores.
// Fixed fields read (encode) or write (decode) their native columns
// directly.  A record whose staged bytes exceed the tile, and every record of
// a block whose column ranges do not fit 31-bit offsets, is moved by the
// whole block straight between global buffers (enc/dec_record_block).
// ===========================================================================
constexpr uint32_t kStageSlack = 64;           // LDS bytes a chunk window may read past the tile

__host__ __device__ inline bool stage_type(uint32_t type, uint32_t xsz) {
    return xsz == 1 || type == XDRG_T_INT || type == XDRG_T_UINT || type == XDRG_T_ENUM || type == XDRG_T_FLOAT;
}

// 16-aligned global extent [*a0, *a0 + 16 * chunks) covering [p0, p1).
__device__ __forceinline__ uint32_t stage_chunks(const uint8_t *p0, const uint8_t *p1, const uint8_t **a0) {
    const uintptr_t x0 = (uintptr_t)p0 & ~(uintptr_t)15, x1 = ((uintptr_t)p1 + 15) & ~(uintptr_t)15;
    *a0 = (const uint8_t *)x0;
    return p1 > p0 ? (uint32_t)((x1 - x0) >> 4) : 0u;
}

// Copy the staged ranges into the tile: range d is cb[d+1] - cb[d] chunks
// from the 16-aligned a0[d] to tile offset 16 * cb[d].  Four loads per lane
// are issued before their LDS writes.  A 16-byte aligned chunk that holds a
// valid byte never leaves that byte's page.
__device__ __forceinline__ void stage_copy(uint8_t *tile, const uint8_t *const (&a0)[kMaxDynLds],
                                           const uint32_t (&cb)[kMaxDynLds + 1], uint32_t nd) {
    const uint32_t total = cb[nd];
    if (!total) return;
    for (uint32_t i0 = threadIdx.x; i0 < total; i0 += 4 * kRecThreads) {
        u32x4n v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t i = i0 + u * kRecThreads < total ? i0 + u * kRecThreads : total - 1;
            const uint8_t *src = a0[0] + 16 * (uint64_t)i;
#pragma unroll
            for (int d = 1; d < kMaxDynLds; ++d)
                if ((uint32_t)d < nd && i >= cb[d]) src = a0[d] + 16 * (uint64_t)(i - cb[d]);
            v[u] = __builtin_nontemporal_load((const u32x4n *)src);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t i = i0 + u * kRecThreads;
            if (i < total) *(u32x4n *)(tile + 16 * (size_t)i) = v[u];
        }
    }
}

// stage_copy by LDS-DMA (global_load_lds_dwordx4): chunk i lands at tile +
// 16 i straight from memory, no registers, so the block can do other work
// (the sweep's metadata) while the loads fly; the caller's barrier waits for
// them.  A wave's 64 chunks are contiguous in the tile (the instruction's LDS
// address is wave-uniform base + 16 * lane).
__device__ __forceinline__ void stage_dma(uint8_t *tile, const uint8_t *const (&a0)[kMaxDynLds],
                                          const uint32_t (&cb)[kMaxDynLds + 1], uint32_t nd) {
    const uint32_t total = cb[nd], lane = threadIdx.x & 63;
    for (uint32_t i0 = (threadIdx.x >> 6) * 64; i0 < total; i0 += kRecThreads) {
        const uint32_t i = i0 + lane;
        if (i >= total) continue;
        const uint8_t *src = a0[0] + 16 * (uint64_t)i;
#pragma unroll
        for (int d = 1; d < kMaxDynLds; ++d)
            if ((uint32_t)d < nd && i >= cb[d]) src = a0[d] + 16 * (uint64_t)(i - cb[d]);
        __builtin_amdgcn_global_load_lds((const void *)src, (__attribute__((address_space(3))) void *)(tile + 16 * (size_t)i0),
                                         16, 0, 0);
    }
}

// XDR bytes of record j's dynamic fields d < nd (counts from a rel table:
// row d holds element offsets relative to the block's first record).
__device__ __forceinline__ uint64_t dyn_before(const RecArgs &a, const uint32_t *rel, uint32_t j, uint32_t nd,
                                               uint32_t rs = kRecPerBlock + 1) {
    uint64_t s = 0;
#pragma unroll
    for (int d = 0; d < kMaxDynLds; ++d) {
        if ((uint32_t)d >= nd) continue;
        const uint32_t *r = rel + d * rs;
        s += dyn_xdr_bytes(a.f[a.dyn_idx[d]], r[j + 1] - r[j]);
    }
    return s;
}

// ---- encode -------------------------------------------------------------------
// LDS: soff[RPB + 1] u32 (record offset - block offset) | srel[ND][RPB + 1] u32 |
// pad masks [17][4] u32 | tile
constexpr uint32_t kPadMasks = 17 * 16;   // row i: the dwords of 16 bytes whose first i are kept
__host__ __device__ constexpr size_t enc_stage_rows(uint32_t nd) {
    return ((size_t)(nd + 1) * (kRecPerBlock + 1) * 4 + 15) & ~(size_t)15;
}
__host__ __device__ constexpr size_t enc_stage_meta(uint32_t nd) { return enc_stage_rows(nd) + kPadMasks; }

// The whole block writes record r at stream offset pos from the native
// columns (records too large for the tile).
__device__ void enc_record_block(const RecArgs &a, uint64_t r, uint64_t pos) {
    const uint32_t tid = threadIdx.x;
    uint8_t *out = a.xdr;
    if (a.framed) pos += 4;   // the mark is written by the caller
    for (uint32_t k = 0; k < a.nf; ++k) {
        const VField &f = a.f[k];
        if (f.kind != XDRG_K_DYNAMIC) {
            const uint32_t nw = f.xbytes >> 2;
            for (uint32_t i = tid; i < nw; i += kRecThreads) *(uint32_t *)(out + pos + 4 * i) = fixed_word(f, r, 4 * i);
            pos += f.xbytes;
            continue;
        }
        const bool bytes = f.xsz == 1;
        const uint64_t esz = bytes ? 1 : f.nsz;
        const uint64_t e0 = f.offsets[r], cnt1 = f.offsets[r + 1] - e0;
        const Span sp = make_span(f.data + f.offsets[0] * esz, f.data + f.offsets[a.n] * esz,
                                  (const uint8_t *)a.block_sums);
        uint8_t *dst[1] = {out + pos};
        const uint8_t *src[1] = {f.data + e0 * esz};
        const uint64_t cnt[1] = {cnt1};
        const uint64_t nwb = 1 + (bytes ? (cnt1 + 3) >> 2 : cnt1);
        const uint64_t nch[1] = {(nwb + 3) >> 2};
        if (bytes) enc_blob_bytes<2, 1>(dst, src, cnt, nch, sp, kRecThreads, tid);
        else enc_blob_words4<2, 1>(dst, src, cnt, nch, f.type == XDRG_T_FLOAT, sp, kRecThreads, tid);
        pos += dyn_xdr_bytes(f, cnt1);
    }
}

// Records the sub-batch starting at js can take: [js, js + k) fit the tile
// iff staging [js, js + 1 + t) fits for every t < k (monotone), counted with
// one barrier (which also ends every use of the tile before it).  0 = record
// js alone exceeds the tile.
__device__ __forceinline__ uint32_t enc_fit(const RecArgs &a, const uint64_t (&base)[kMaxDynLds],
                                            const uint32_t *srel, uint32_t js, uint32_t nrec) {
    const uint32_t je = js + 1 + threadIdx.x;
    bool fits = false;
    if (je <= nrec) {
        uint32_t need = 0;
#pragma unroll
        for (int d = 0; d < kMaxDynLds; ++d) {
            if ((uint32_t)d >= a.ndyn) continue;
            const VField &f = a.f[a.dyn_idx[d]];
            const uint64_t esz = f.xsz == 1 ? 1 : f.nsz;
            const uint32_t *rel = srel + d * (kRecPerBlock + 1);
            const uint8_t *a0;
            need += 16 * stage_chunks(f.data + (base[d] + rel[js]) * esz, f.data + (base[d] + rel[je]) * esz, &a0);
        }
        fits = need <= a.tile_bytes;
    }
    return (uint32_t)__syncthreads_count(fits);
}

// Input-staged encode with a record-major scatter: a group of lanes writes
// all of a record's fields, so its output lines are completed together and
// leave L2 whole (WRITE 1.00x algorithmic on config 4).  Measured and removed
// (git history): the field-major scatter (1.23x WRITE), the
// same with nontemporal stores, an LDS output image composed from HBM inputs
// or from the staged tile.
__global__ __launch_bounds__(kRecThreads) void k_enc_stage_rm(const RecArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr uint32_t RS = kRecPerBlock + 1;   // row stride of soff / srel
    uint32_t *soff = (uint32_t *)smem;
    uint32_t *srel = soff + RS;
    uint32_t *padm = (uint32_t *)(smem + enc_stage_rows(a.ndyn));
    uint8_t *tile = smem + enc_stage_meta(a.ndyn);
    if (threadIdx.x < kPadMasks / 4)   // (read after the prologue's barrier)
        padm[threadIdx.x] = lo_mask((int32_t)(threadIdx.x >> 2) - 4 * (int32_t)(threadIdx.x & 3));
    const uint64_t total = a.totals[0];
    if (total > a.xdr_cap) return;  // XDRG_E_CAPACITY: write nothing
    if (a.big_rec && block_is_big(a, false)) return;   // the group kernel's block
    const uint64_t rb = (uint64_t)blockIdx.x * kRecPerBlock;
    const uint32_t tid = threadIdx.x, t0 = tid * kRecPerThread;
    const uint32_t nrec = (uint32_t)(a.n - rb < (uint64_t)kRecPerBlock ? a.n - rb : (uint64_t)kRecPerBlock);
    // ---- prologue: record sizes, column offsets relative to record rb, block scan
    uint64_t sz[kRecPerThread];
#pragma unroll
    for (int j = 0; j < kRecPerThread; ++j) sz[j] = t0 + j < nrec ? a.fixed_xdr : 0;
    uint64_t base[kMaxDynLds];
    bool wide = false;
#pragma unroll
    for (int d = 0; d < kMaxDynLds; ++d) {
        base[d] = 0;
        if ((uint32_t)d >= a.ndyn) continue;
        const VField &f = a.f[a.dyn_idx[d]];
        const uint64_t esz = f.xsz == 1 ? 1 : f.nsz;
        base[d] = f.offsets[rb];
        wide |= (f.offsets[rb + nrec] - base[d]) * esz >= (1ull << 31);
        uint64_t o[kRecPerThread + 1];
#pragma unroll
        for (int j = 0; j <= kRecPerThread; ++j) {   // unconditional loads, index clamped
            const uint64_t r = rb + t0 + j;
            o[j] = f.offsets[r < a.n ? r : a.n];
        }
#pragma unroll
        for (int j = 0; j < kRecPerThread; ++j) {
            if (t0 + j < nrec) sz[j] += dyn_xdr_bytes(f, o[j + 1] - o[j]);
            srel[d * RS + t0 + j] = (uint32_t)(o[j] - base[d]);
        }
        if (tid == kRecThreads - 1) srel[d * RS + kRecPerBlock] = (uint32_t)(o[kRecPerThread] - base[d]);
    }
    uint64_t s = 0;
#pragma unroll
    for (int j = 0; j < kRecPerThread; ++j) s += sz[j];
    uint64_t btot;
    const uint64_t bbase = a.block_sums[blockIdx.x];   // stream offset of record rb
    uint64_t off = block_excl_scan(s, &btot);
    wide |= btot >= (1ull << 32);
#pragma unroll
    for (int j = 0; j < kRecPerThread; ++j) {
        soff[t0 + j] = (uint32_t)off;
        if (a.rec_out && t0 + j < nrec) a.rec_out[rb + t0 + j] = bbase + off;
        off += sz[j];
    }
    if (tid == kRecThreads - 1) soff[kRecPerBlock] = (uint32_t)off;
    if (a.rec_out && blockIdx.x == 0 && tid == 0) a.rec_out[a.n] = total;
    __syncthreads();
    if (wide) {   // block offsets beyond 32 bits: record by record, straight from global
        uint64_t pos = bbase;
        for (uint32_t j = 0; j < nrec; ++j) {
            const uint64_t r = rb + j;
            uint64_t size = a.fixed_xdr;
            for (uint32_t d = 0; d < a.ndyn; ++d) {
                const VField &f = a.f[a.dyn_idx[d]];
                size += dyn_xdr_bytes(f, f.offsets[r + 1] - f.offsets[r]);
            }
            if (a.framed && tid == 0)   // GrizzlyRpcTransport:103-110
                *(uint32_t *)(a.xdr + pos) = bswap32r((uint32_t)(size - 4) | kLastFrag);
            enc_record_block(a, r, pos);
            pos += size;
        }
        return;
    }
    uint8_t *const out = a.xdr + bbase;   // block-relative stream
    // ---- sub-batches
    uint32_t js = 0;
    uint32_t k1 = enc_fit(a, base, srel, js, nrec);
    while (js < nrec) {
        if (k1 == 0) {   // too large for the tile: the whole block writes record js
            if (a.framed && tid == 0)
                *(uint32_t *)(out + soff[js]) = bswap32r((soff[js + 1] - soff[js] - 4) | kLastFrag);
            enc_record_block(a, rb + js, bbase + soff[js]);
            ++js;
            k1 = js < nrec ? enc_fit(a, base, srel, js, nrec) : 0;
            continue;
        }
        const uint32_t je = js + k1;
        // stage every dynamic column's range of the sub-batch
        const uint8_t *a0[kMaxDynLds];
        uint32_t cb[kMaxDynLds + 1];
        cb[0] = 0;
#pragma unroll
        for (int d = 0; d < kMaxDynLds; ++d) {
            a0[d] = nullptr;
            cb[d + 1] = cb[d];
            if ((uint32_t)d >= a.ndyn) continue;
            const VField &f = a.f[a.dyn_idx[d]];
            const uint64_t esz = f.xsz == 1 ? 1 : f.nsz;
            cb[d + 1] += stage_chunks(f.data + (base[d] + srel[d * RS + js]) * esz,
                                      f.data + (base[d] + srel[d * RS + je]) * esz, &a0[d]);
        }
        stage_copy(tile, a0, cb, a.ndyn);   // (stage_dma measured 3.70 vs 3.62 ms here: nothing to overlap)
        __syncthreads();
        const uint32_t m = je - js;
        // tile offset of element 0 of the block's dynamic column d, minus its
        // 16-aligned staged start (wave-uniform): element e of the column sits
        // at tile byte tadj[d] + e * esz.  Everything below is 32-bit
        // (block-relative offsets < 2^32, the `wide` check), stores address
        // the block's output as a uniform base + 32-bit lane offset.
        int32_t tadj[kMaxDynLds];
#pragma unroll
        for (int d = 0; d < kMaxDynLds; ++d) {
            tadj[d] = 0;
            if ((uint32_t)d >= a.ndyn) continue;
            const VField &f = a.f[a.dyn_idx[d]];
            const uint64_t esz = f.xsz == 1 ? 1 : f.nsz;
            tadj[d] = (int32_t)(16 * cb[d]) + (int32_t)((uintptr_t)(f.data + base[d] * esz) - (uintptr_t)a0[d]);
        }
        {   // record-major scatter: a group of lanes writes all of a record
            const uint32_t rbytes = (soff[je] - soff[js]) / m;
            const uint32_t G = a.force_g ? a.force_g : pow2_lanes(rbytes, a.lane_bytes_enc);
            const uint32_t gl = tid & (G - 1), ng = kRecThreads / G;
            for (uint32_t j = js + tid / G; j < je; j += ng) {
                const uint32_t r0 = soff[j];
                uint32_t o = r0 + (a.framed ? 4u : 0u), d = 0;   // output offset of the next field
                if (a.framed && gl == 0)   // the record's mark with its bytes (GrizzlyRpcTransport:103-110)
                    *(uint32_t *)(out + r0) = bswap32r((soff[j + 1] - r0 - 4) | kLastFrag);
                for (uint32_t k = 0; k < a.nf; ++k) {
                    const VField &f = a.f[k];
                    if (f.kind != XDRG_K_DYNAMIC) {
                        const uint32_t nw = f.xbytes >> 2;
                        for (uint32_t i = gl; i < nw; i += G)
                            *(uint32_t *)(out + (o + 4 * i)) = fixed_word(f, rb + j, 4 * i);
                        o += f.xbytes;
                        continue;
                    }
                    const uint32_t *rel = srel + d * RS;
                    const uint32_t e0 = rel[j], cnt = rel[j + 1] - e0;
                    if (f.xsz == 1) {
                        // blob [BE length][bytes][zero pad] (Xdr.java:776-800): chunk c =
                        // blob bytes [16c, 16c + 16) from the five tile words at w + 16c
                        const int32_t t = tadj[d] + (int32_t)e0;   // tile byte of the payload
                        const uint32_t sh = (uint32_t)t & 3u;     // (a0 is 16-aligned)
                        const int32_t w = t - (int32_t)sh - 4;
                        const uint32_t nwb = 1 + ((cnt + 3) >> 2), nch = (nwb + 3) >> 2;
                        for (uint32_t c = gl; c < nch; c += G) {
                            const uint32_t *q = (const uint32_t *)(tile + (w + 16 * (int32_t)c));
                            const uint32_t q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3], q4 = q[4];
                            // (alignbyte by 0 is the low word: no select for aligned payloads)
                            uint32_t o0 = __builtin_amdgcn_alignbyte(q1, q0, sh);
                            uint32_t o1 = __builtin_amdgcn_alignbyte(q2, q1, sh);
                            uint32_t o2 = __builtin_amdgcn_alignbyte(q3, q2, sh);
                            uint32_t o3 = __builtin_amdgcn_alignbyte(q4, q3, sh);
                            // blob bytes from the chunk start: the last chunk's zero pad
                            // (Xdr.java:765) by a mask row (every other chunk: row 16)
                            const int32_t rem = 4 + (int32_t)cnt - 16 * (int32_t)c;
                            const u32x4a pm = *(const u32x4a *)(padm + 4 * (rem < 16 ? rem : 16));
                            o0 &= pm.x;
                            o1 &= pm.y;
                            o2 &= pm.z;
                            o3 &= pm.w;
                            if (c == 0) o0 = bswap32r(cnt);
                            uint8_t *dd = out + (o + 16 * c);
                            if (4 * c + 4 <= nwb) {
                                u32x4a v; v.x = o0; v.y = o1; v.z = o2; v.w = o3;
                                *(u32x4a *)dd = v;
                            } else {
                                const uint32_t left = nwb - 4 * c;
                                *(uint32_t *)dd = o0;
                                if (left > 1) *(uint32_t *)(dd + 4) = o1;
                                if (left > 2) *(uint32_t *)(dd + 8) = o2;
                            }
                        }
                        o += 4 + ((cnt + 3) & ~3u);
                    } else {
                        // [BE count][BE elements] (Xdr.java:607-613): blob word b is element
                        // b - 1, chunk c reads the four tile words at t - 4 + 16c
                        const int32_t t = tadj[d] + 4 * (int32_t)e0 - 4;
                        const bool fl = f.type == XDRG_T_FLOAT;
                        const uint32_t nwb = 1 + cnt, nch = (nwb + 3) >> 2;
                        for (uint32_t c = gl; c < nch; c += G) {
                            const uint32_t *q = (const uint32_t *)(tile + (t + 16 * (int32_t)c));
                            uint32_t v[4] = {q[0], q[1], q[2], q[3]};
#pragma unroll
                            for (int i = 0; i < 4; ++i) v[i] = bswap32r(fl ? canon_f32r(v[i]) : v[i]);
                            if (c == 0) v[0] = bswap32r(cnt);
                            uint32_t *dd = (uint32_t *)(out + (o + 16 * c));
                            if (4 * c + 4 <= nwb) {
                                u32x4a x; x.x = v[0]; x.y = v[1]; x.z = v[2]; x.w = v[3];
                                *(u32x4a *)dd = x;
                            } else {
                                for (uint32_t i = 0; 4 * c + i < nwb; ++i) dd[i] = v[i];
                            }
                        }
                        o += 4 * nwb;
                    }
                    ++d;
                }
            }
        }
        js = je;
        k1 = js < nrec ? enc_fit(a, base, srel, js, nrec) : 0;   // its barrier ends the tile's use
    }
}

// ---- decode -------------------------------------------------------------------
// LDS: sstart[RPB + 1] u32 (record start - the block's first start) | snrel[ND][RPB + 1] u32 |
// supto[RPB] u8 | tile[tile_bytes + slack]: 29.4 KB with two dynamic fields, so
// five blocks fit a CU (the u64 starts and u32 field limits of the first
// version held it at four)
__host__ __device__ constexpr size_t dec_stage_meta(uint32_t nd) {
    return ((size_t)(kRecPerBlock + 1) * 4 + (size_t)nd * (kRecPerBlock + 1) * 4 + (size_t)kRecPerBlock +
            16 + 15) & ~(size_t)15;   // + 16: the sweep's meta sentinels after supto (kSweepMetaPad words)
}

// Threads tid < nthr of the block decode fields [0, upto) of record r (the
// block's record j) whose first field starts at stream offset pos (records
// too large for the tile).  Counts come from the block's relative native offsets snrel, native
// offsets from the columns' offsets arrays this block just wrote.
__device__ __forceinline__ void dec_record_block(const RecArgs &a, uint64_t r, uint64_t pos, uint32_t upto,
                                 const uint32_t *snrel, uint32_t j, uint32_t tid, uint32_t nthr,
                                 uint32_t rs = kRecPerBlock + 1) {
    const uint8_t *in = a.xdr;
    const Span sp = make_span(in, in + a.xdr_cap, (const uint8_t *)a.block_sums);
    uint32_t d = 0;
    for (uint32_t k = 0; k < upto; ++k) {
        const VField &f = a.f[k];
        if (f.kind != XDRG_K_DYNAMIC) {
            const uint32_t nw = f.xbytes >> 2;
            for (uint32_t i = tid; i < nw; i += nthr) fixed_store(f, r, 4 * i, *(const uint32_t *)(in + pos + 4 * i));
            pos += f.xbytes;
            continue;
        }
        const bool bytes = f.xsz == 1;
        const uint32_t *rel = snrel + (size_t)d * rs;
        const uint64_t cnt1 = rel[j + 1] - rel[j];
        // extent-derived count (key 31): the count word must say the same
        if ((a.spec_mode & 1) && d + 1 == a.ndyn && tid == 0 && bswap32r(*(const uint32_t *)(in + pos)) != (uint32_t)cnt1)
            spec_fail(a);
        uint8_t *dst[1] = {f.data + f.offsets[r] * (bytes ? 1 : f.nsz)};
        const uint8_t *src[1] = {in + pos + 4};
        const uint64_t cnt[1] = {cnt1};
        const uint32_t sh = (uint32_t)((uintptr_t)dst[0] & 3);
        const uint64_t nd = bytes ? (sh + cnt1 + 3) >> 2 : cnt1;
        const uint64_t nch[1] = {cnt1 ? (nd + 3) >> 2 : 0};
        if (bytes) dec_bytes<2, 1>(dst, src, cnt, nch, sp, nthr, tid);
        else dec_words4<2, 1>(dst, src, cnt, nch, sp, nthr, tid);
        pos += dyn_xdr_bytes(f, cnt1);
        ++d;
    }
}

// Unaligned dword of the tile at byte offset o.
__device__ __forceinline__ uint32_t tile_word(const uint8_t *tile, int64_t o) {
    const uint32_t *w = (const uint32_t *)(tile + (o & ~(int64_t)3));
    const uint32_t s = (uint32_t)(o & 3);
    return s ? __builtin_amdgcn_alignbyte(w[1], w[0], s) : w[0];
}
// XDR bytes of record j's dynamic fields before d (xs: their element sizes).
__device__ __forceinline__ uint32_t dyn_before_xs(const uint32_t (&xs)[kMaxDynLds], const uint32_t *rel,
                                                  uint32_t j, uint32_t d, uint32_t rs = kRecPerBlock + 1) {
    uint32_t s = 0;
#pragma unroll
    for (int e = 0; e < kMaxDynLds - 1; ++e) {
        if ((uint32_t)e >= d) continue;
        const uint32_t *r = rel + e * rs;
        const uint32_t c = r[j + 1] - r[j];
        s += 4 + (xs[e] == 1 ? (c + 3) & ~3u : c * xs[e]);
    }
    return s;
}
// Byte field of one staged record, lean form (tuning key 20): cnt bytes
// at tile offset L (4-aligned) to dst (any alignment), chunk c of the
// 4-aligned da = dst - sh by lane c % G.  The dword a record boundary falls
// in is written once, whole, by the later record's first lane when both
// records fill their side of it (own_head: hv is the composed dword; the
// earlier record then skips it, skip_tail); otherwise each side byte-stores
// its own bytes.  Every other store is a whole dword or 16 bytes.
__device__ __forceinline__ void dec_bytes_lean(uint8_t *dst, const uint8_t *tile, uint32_t L, uint32_t cnt,
                                               bool own_head, uint32_t hv, bool skip_tail, uint32_t gl, uint32_t G) {
    const uint32_t sh = (uint32_t)((uintptr_t)dst & 3), end = sh + cnt, nch = (end + 15) >> 4;
    uint8_t *da = dst - sh;
    const uint32_t rs = (4 - sh) & 3;   // source misalignment of dest dwords
    for (uint32_t c = gl; c < nch; c += G) {
        const uint32_t b0 = 16 * c;
        const uint32_t *w = (const uint32_t *)(tile + (L + b0 - sh - rs));   // 4-aligned
        const uint32_t q0 = w[0], q1 = w[1], q2 = w[2], q3 = w[3], q4 = w[4];
        uint32_t v[4];
        v[0] = rs ? __builtin_amdgcn_alignbyte(q1, q0, rs) : q0;
        v[1] = rs ? __builtin_amdgcn_alignbyte(q2, q1, rs) : q1;
        v[2] = rs ? __builtin_amdgcn_alignbyte(q3, q2, rs) : q2;
        v[3] = rs ? __builtin_amdgcn_alignbyte(q4, q3, rs) : q3;
        const bool head = c == 0 && sh != 0;
        if (head && own_head) v[0] = hv;
        uint8_t *d = da + b0;
        if ((!head || own_head) && b0 + 16 <= end) {
            u32x4a o; o.x = v[0]; o.y = v[1]; o.z = v[2]; o.w = v[3];
            *(u32x4a *)d = o;
            continue;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t lo = b0 + 4 * k;
            if (lo >= end) continue;
            const bool hd = lo < sh, tl = lo + 4 > end;
            if ((!hd || own_head) && !tl) { *(uint32_t *)(d + 4 * k) = v[k]; continue; }
            if (tl && skip_tail) continue;
            const uint32_t bs = hd ? sh : 0u, be = tl ? end - lo : 4u;
            uint8_t *p = d + 4 * k;
            if (bs == 0 && be > 0) p[0] = (uint8_t)v[k];
            if (bs <= 1 && be > 1) p[1] = (uint8_t)(v[k] >> 8);
            if (bs <= 2 && be > 2) p[2] = (uint8_t)(v[k] >> 16);
            if (be > 3) p[3] = (uint8_t)(v[k] >> 24);
        }
    }
}

// Records [js, je) of a staged decode sub-batch, whose XDR bytes the tile
// holds (stream offset sb + x at tile offset lds0 + x), decoded by threads
// ctid < nthr: every field by groups of lanes per record; byte fields of
// error-free blocks with whole boundary dwords (dec_bytes_lean).
template <uint32_t RS>
__device__ __forceinline__ void dec_stage_batch(const RecArgs &a, const uint8_t *tile, int64_t lds0, uint64_t rb,
                                                uint32_t js, uint32_t je, const uint32_t *sstart,
                                                const uint32_t *snrel, const uint8_t *supto, const uint64_t *s_base,
                                                const uint32_t (&xs)[kMaxDynLds], bool lean, uint32_t ctid,
                                                uint32_t nthr) {
    uint32_t fpre = 0;
    uint32_t d = 0;
    const uint32_t m = je - js;
    for (uint32_t k = 0; k < a.nf; ++k) {
        const VField &f = a.f[k];
        if (f.kind != XDRG_K_DYNAMIC) {
            const uint32_t nw = f.xbytes >> 2;
            if (nw) {
                const uint32_t G = a.force_g ? a.force_g : pow2_lanes((uint64_t)nw * 4, 16);
                const uint32_t gl = ctid & (G - 1), ng = nthr / G;
                for (uint32_t j = js + ctid / G; j < je; j += ng) {
                    if (k >= supto[j]) continue;
                    const uint32_t *w = (const uint32_t *)(tile + (lds0 + (int64_t)(sstart[j] + fpre +
                                                                               dyn_before(a, snrel, j, d, RS))));
                    for (uint32_t i = gl; i < nw; i += G) fixed_store(f, rb + j, 4 * i, w[i]);
                }
            }
            fpre += f.xbytes;
            continue;
        }
        const bool bytes = f.xsz == 1;
        const uint64_t esz = bytes ? 1 : f.nsz;
        const uint32_t *rel = snrel + d * RS;
        const uint64_t base = s_base[d];
        const uint64_t fbytes = (uint64_t)(rel[je] - rel[js]) * esz + 4ull * m;
        const uint32_t G = a.force_g ? a.force_g : pow2_lanes(fbytes / m, a.lane_bytes_dec);
        const uint32_t gl = ctid & (G - 1), ng = nthr / G;
        for (uint32_t j = js + ctid / G; j < je; j += ng) {
            if (k >= supto[j]) continue;
            const uint64_t cnt = rel[j + 1] - rel[j];
            if (!cnt) continue;
            // tile offset of the payload (after the length word)
            const int64_t L = lds0 + (int64_t)(sstart[j] + fpre + dyn_before(a, snrel, j, d, RS) + 4);
            uint8_t *dst = f.data + (base + rel[j]) * esz;
            if (bytes && lean) {
                // the boundary dwords with records j - 1 and j + 1 (within the sub-batch)
                const uint32_t sh = (uint32_t)((uintptr_t)dst & 3);
                const uint32_t tb = (sh + (uint32_t)cnt) & 3;   // record j's bytes in its last dword
                bool own = false, skip = false;
                uint32_t hv = 0;
                if (sh && j > js) {
                    const uint32_t cp = rel[j] - rel[j - 1];
                    if (cp >= sh && cnt >= 4 - sh) {
                        own = true;
                        const int64_t Lp = lds0 + (int64_t)(sstart[j - 1] + fpre + dyn_before_xs(xs, snrel, j - 1, d, RS) + 4);
                        const uint32_t pw = tile_word(tile, Lp + cp - sh), hw = tile_word(tile, L);
                        hv = (pw & ((1u << (8 * sh)) - 1u)) | (hw << (8 * sh));
                    }
                }
                if (tb && j + 1 < je && cnt >= tb && rel[j + 2] - rel[j + 1] >= 4 - tb) skip = true;
                dec_bytes_lean(dst, tile, (uint32_t)L, (uint32_t)cnt, own, hv, skip, gl, G);
            } else if (bytes) {
                const uint32_t sh = (uint32_t)((uintptr_t)dst & 3);
                const uint64_t nch = (((sh + cnt + 3) >> 2) + 3) >> 2;
                for (uint64_t c = gl; c < nch; c += G) {
                    const uint32_t *w = (const uint32_t *)(tile + (L + 16 * (int64_t)c - 4));
                    Chunk5 q;
                    q.q0 = w[0]; q.q1 = w[1]; q.q2 = w[2]; q.q3 = w[3]; q.q4 = w[4];
                    dec_store(dst - sh, q, c, cnt, sh);
                }
            } else {
                const uint64_t nch = (cnt + 3) >> 2;
                for (uint64_t c = gl; c < nch; c += G) {
                    const uint32_t *w = (const uint32_t *)(tile + (L + 16 * (int64_t)c));
                    uint32_t *o = (uint32_t *)(dst + 16 * c);
                    if (4 * c + 4 <= cnt) {
                        u32x4a v;
                        v.x = bswap32r(w[0]); v.y = bswap32r(w[1]); v.z = bswap32r(w[2]); v.w = bswap32r(w[3]);
                        *(u32x4a *)o = v;
                    } else {
                        for (uint64_t e = 0; 4 * c + e < cnt; ++e) o[e] = bswap32r(w[e]);
                    }
                }
            }
        }
        ++d;
    }
}

// ---- output-stationary sweep of a staged sub-batch (tuning key 20 = 2) --------
// The dynamic fields of an error-free sub-batch are written by destination
// chunks instead of by records: lane q writes the q-th 16-byte chunk of the
// sub-batch's column range (aligned in global memory: one coalesced store per
// lane, no partial lines) and composes it from the records whose bytes it
// holds.  Before the stage barrier every record lane describes its record in
// meta (start, end and tile offset: one word, read as consecutive words) and
// writes its index into the chunk map for the chunks whose first element it
// holds (about length / 16 byte stores per record).  A chunk reads its owner
// from the map and the next records' words in one go, so the common chunks
// (inside one record, or across one record edge) are straight-line code with
// no dependent LDS round trips beyond map -> meta -> tile; the per-record
// control flow of groups of lanes (what bounds dec_stage_batch, DESIGN.md
// §5.3) is gone.  Byte fields: Xdr.java:760-763 / :797-800 (bytes, pad
// skipped); int vectors: Xdr.java:607-613 (one bswap per element).
constexpr uint32_t kSweepMetaPad = 4;   // meta sentinels after the sub-batch's last record

// LDS the sweep adds after the tile: the second field's meta, the chunk
// map of both fields (their chunks together cover at most the tile's bytes)
// and the byte-mask rows (kPadMasks: row i keeps the first i bytes of 16).
__host__ __device__ constexpr size_t dec_sweep_map(uint32_t tile_bytes) {
    return ((size_t)(tile_bytes >> 4) + 32 + 15) & ~(size_t)15;
}
__host__ __device__ constexpr size_t dec_sweep_extra(uint32_t tile_bytes) {
    return (((size_t)kRecThreads + kSweepMetaPad) * 4 + 15 & ~(size_t)15) + dec_sweep_map(tile_bytes) + kPadMasks;
}

// Record lanes of the sub-batch [js, js + m): meta[t] = (start - x0) | tile
// offset << 16 (elements relative to chunk 0, which starts at x0),
// meta[m .. m + pad) = the end (empty records); map[c] = the record holding
// chunk c's first element, for every c in [1, nq) (chunk 0: record 0 or the
// first non-empty one after it).
template <uint32_t RS>
__device__ __forceinline__ void sweep_build(uint32_t *meta, uint8_t *map, const uint32_t *rel,
                                            const uint32_t *sstart, const uint32_t *snrel,
                                            const uint32_t (&xs)[kMaxDynLds], uint32_t d, int32_t tb, int32_t x0,
                                            uint32_t cs, uint32_t js, uint32_t m, uint32_t nq) {
    const uint32_t t = threadIdx.x;
    if (t >= m) return;
    const uint32_t j = js + t;
    const uint32_t lo = (uint32_t)((int32_t)rel[j] - x0), hi = (uint32_t)((int32_t)rel[j + 1] - x0);
    const uint32_t T = (uint32_t)(tb + (int32_t)(sstart[j] + dyn_before_xs(xs, snrel, j, d, RS)));
    meta[t] = lo | T << 16;
    if (t + 1 == m)
#pragma unroll
        for (uint32_t k = 0; k < kSweepMetaPad; ++k) meta[m + k] = hi;
    const uint32_t r = (1u << cs) - 1;
    const uint32_t c1 = min((hi + r) >> cs, nq);
    for (uint32_t c = (lo + r) >> cs; c < c1; ++c) map[c] = (uint8_t)t;
}

// Byte mask of bytes [lo, hi) (clamped to 0..4) of a dword.
__device__ __forceinline__ uint32_t byte_mask(int32_t lo, int32_t hi) {
    lo = lo < 0 ? 0 : lo;
    hi = hi > 4 ? 4 : hi;
    return hi > lo ? (uint32_t)((1ull << (8 * hi)) - (1ull << (8 * lo))) : 0u;
}

// Bytes [lo, hi) of the aligned 16-byte chunk at g (g + 4 k: dword k = v[k]),
// by whole dwords where a dword is covered and byte stores at the ends.
__device__ __forceinline__ void store_chunk_part(uint8_t *g, const uint32_t (&v)[4], int32_t lo, int32_t hi) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int32_t b0 = lo - 4 * k < 0 ? 0 : lo - 4 * k, b1 = hi - 4 * k > 4 ? 4 : hi - 4 * k;
        if (b1 <= b0) continue;
        uint8_t *p = g + 4 * k;
        if (b0 == 0 && b1 == 4) { *(uint32_t *)p = v[k]; continue; }
        for (int32_t b = b0; b < b1; ++b) p[b] = (uint8_t)(v[k] >> (8 * b));
    }
}

// The 16 tile bytes from tile offset w (any alignment; the tile's slack and
// the meta region before it make every such window readable).
__device__ __forceinline__ void tile16(const uint8_t *tile, int32_t w, uint32_t (&u)[4]) {
    const uint32_t *p = (const uint32_t *)(tile + (w & ~3));
    const uint32_t s = (uint32_t)w & 3u;
    const uint32_t q0 = p[0], q1 = p[1], q2 = p[2], q3 = p[3], q4 = p[4];
    u[0] = __builtin_amdgcn_alignbyte(q1, q0, s);
    u[1] = __builtin_amdgcn_alignbyte(q2, q1, s);
    u[2] = __builtin_amdgcn_alignbyte(q3, q2, s);
    u[3] = __builtin_amdgcn_alignbyte(q4, q3, s);
}

// Byte field: col = the column at block-relative element 0, chunk q = bytes
// [x0 + 16 q, + 16) with col + x0 16-aligned, [xb, xe) = the sub-batch's bytes.
__device__ __forceinline__ void sweep_bytes(uint8_t *col, const uint8_t *tile, const uint32_t *meta,
                                            const uint8_t *map, const uint32_t *padm, int32_t x0, uint32_t nq,
                                            uint32_t m, int32_t xb, int32_t xe) {
    for (uint32_t q = threadIdx.x; q < nq; q += kRecThreads) {
        const int32_t xr = 16 * (int32_t)q;   // chunk start relative to x0
        uint32_t j = q ? map[q] : 0u;
        uint32_t m0 = meta[j], m1 = meta[j + 1], m2 = meta[j + 2];
        while ((int32_t)(m1 & 0xffffu) <= xr && j + 1 < m) {   // chunk 0: empty records first
            ++j;
            m0 = m1;
            m1 = m2;
            m2 = meta[j + 2];
        }
        // record A = j holds the chunk's first byte, record B = j + 1 starts where A ends
        const int32_t loA = (int32_t)(m0 & 0xffffu), hiA = (int32_t)(m1 & 0xffffu), hiB = (int32_t)(m2 & 0xffffu);
        uint32_t a[4], b[4], v[4];
        tile16(tile, (int32_t)(m0 >> 16) + (xr - loA), a);
        // B's window: when A is the sub-batch's last record (m1 is then the
        // sentinel) or covers the whole chunk, B's bytes are masked out below;
        // clamp the window so the read stays inside the block's LDS
        const int32_t wb = (int32_t)(m1 >> 16) + (xr - hiA);
        tile16(tile, wb < 0 ? 0 : wb, b);
        const int32_t sp = hiA - xr;   // chunk bytes [0, sp) from A, [sp, ..) from B (sp >= 1)
        const u32x4a mk = *(const u32x4a *)(padm + 4 * (sp < 16 ? sp : 16));   // (a mask row: one LDS read)
        v[0] = (a[0] & mk.x) | (b[0] & ~mk.x);
        v[1] = (a[1] & mk.y) | (b[1] & ~mk.y);
        v[2] = (a[2] & mk.z) | (b[2] & ~mk.z);
        v[3] = (a[3] & mk.w) | (b[3] & ~mk.w);
        if (hiB < xr + 16) {   // a third record (or more) inside the chunk: B was short or empty
            int32_t lo = hiB;
            for (uint32_t jj = j + 2; lo < xr + 16 && jj < m; ++jj) {
                const uint32_t e0 = meta[jj];
                const int32_t hi = (int32_t)(meta[jj + 1] & 0xffffu);
                if (hi > lo) {
                    uint32_t c[4];
                    tile16(tile, (int32_t)(e0 >> 16) + (xr - lo), c);
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const uint32_t mk = byte_mask(lo - xr - 4 * k, hi - xr - 4 * k);
                        v[k] = (v[k] & ~mk) | (c[k] & mk);
                    }
                }
                lo = hi;
            }
        }
        const int32_t x = x0 + xr;
        uint8_t *g = col + x;
        if (x >= xb && x + 16 <= xe) {
            u32x4n o;
            o.x = v[0]; o.y = v[1]; o.z = v[2]; o.w = v[3];
            *(u32x4n *)g = o;
        } else {   // the sub-batch's first / last chunk: its neighbours own the other bytes
            store_chunk_part(g, v, xb - x, xe - x);
        }
    }
}

// Word field (4-byte elements, XDR big-endian): chunk q = elements
// [x0 + 4 q, + 4), col + x0 16-aligned; up to four records per chunk in
// straight-line code.
__device__ __forceinline__ void sweep_words(uint32_t *col, const uint8_t *tile, const uint32_t *meta,
                                            const uint8_t *map, int32_t x0, uint32_t nq, uint32_t m, int32_t xb,
                                            int32_t xe) {
    for (uint32_t q = threadIdx.x; q < nq; q += kRecThreads) {
        const int32_t xr = 4 * (int32_t)q;
        uint32_t j = q ? map[q] : 0u;
        uint32_t e[kSweepMetaPad + 1];
#pragma unroll
        for (uint32_t k = 0; k <= kSweepMetaPad; ++k) e[k] = meta[j + k];
        uint32_t v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int32_t x = xr + k;
            int32_t src = -1;
#pragma unroll
            for (int r = kSweepMetaPad - 1; r >= 0; --r) {   // the record among j .. j + 3 holding x
                const int32_t lo = (int32_t)(e[r] & 0xffffu), hi = (int32_t)(e[r + 1] & 0xffffu);
                if (x >= lo && x < hi) src = (int32_t)(e[r] >> 16) + 4 * (x - lo);
            }
            if (src < 0)   // beyond record j + 3 (short or empty records; rare)
                for (uint32_t jj = j + kSweepMetaPad; jj < m; ++jj) {
                    const uint32_t f0 = meta[jj];
                    const int32_t lo = (int32_t)(f0 & 0xffffu), hi = (int32_t)(meta[jj + 1] & 0xffffu);
                    if (x >= lo && x < hi) { src = (int32_t)(f0 >> 16) + 4 * (x - lo); break; }
                    if (lo > x) break;
                }
            v[k] = src >= 0 ? bswap32r(*(const uint32_t *)(tile + src)) : 0u;
        }
        const int32_t x = x0 + xr;
        uint32_t *g = col + x;
        if (x >= xb && x + 4 <= xe) {
            u32x4n o;
            o.x = v[0]; o.y = v[1]; o.z = v[2]; o.w = v[3];
            *(u32x4n *)g = o;
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (x + k >= xb && x + k < xe) g[k] = v[k];
        }
    }
}

// Per dynamic field (at most two) of a sweep sub-batch: the column at
// block-relative element 0, chunk 0's element x0, chunks, sub-batch range.
struct SweepField {
    uint8_t *col;
    int32_t x0, xb, xe;
    uint32_t nq, moff;   // chunks; the field's first entry in the shared chunk map
};

// Before the stage barrier: meta and chunk maps of the (at most two) dynamic
// fields of records [js, je).  meta0 / meta1 hold kRecThreads + pad words.
template <uint32_t RS>
__device__ __forceinline__ void dec_sweep_prep(const RecArgs &a, int64_t lds0, uint32_t js, uint32_t je,
                                               const uint32_t *sstart, const uint32_t *snrel,
                                               const uint64_t *s_base, const uint32_t (&xs)[kMaxDynLds],
                                               uint32_t *meta0, uint32_t *meta1, uint8_t *map,
                                               SweepField *sf) {
    uint32_t fpre = 0, d = 0, moff = 0;
    for (uint32_t k = 0; k < a.nf; ++k) {
        const VField &f = a.f[k];
        if (f.kind != XDRG_K_DYNAMIC) {
            fpre += f.xbytes;
            continue;
        }
        const uint32_t *rel = snrel + d * RS;
        const bool bytes = f.xsz == 1;
        SweepField s;
        s.col = f.data + s_base[d] * (bytes ? 1 : 4);
        const uint32_t cs = bytes ? 4u : 2u;   // log2 of a chunk's elements
        s.xb = (int32_t)rel[js];
        s.xe = (int32_t)rel[je];
        s.x0 = bytes ? s.xb - (int32_t)((uintptr_t)(s.col + s.xb) & 15)
                     : s.xb - (int32_t)(((uintptr_t)(s.col + 4 * (int64_t)s.xb) >> 2) & 3);
        s.nq = s.xe > s.xb ? (uint32_t)(s.xe - s.x0 + (1 << cs) - 1) >> cs : 0u;
        s.moff = moff;
        sweep_build<RS>(d ? meta1 : meta0, map + moff, rel, sstart, snrel, xs, d, (int32_t)lds0 + (int32_t)fpre + 4,
                        s.x0, cs, js, je - js, s.nq);
        if (threadIdx.x == 0) sf[d] = s;   // read after the stage barrier
        moff += s.nq;
        ++d;
    }
}

// After the stage barrier: every field of records [js, je), fixed fields by
// groups of lanes per record as dec_stage_batch, dynamic fields by the sweep.
template <uint32_t RS>
__device__ __forceinline__ void dec_stage_sweep(const RecArgs &a, const uint8_t *tile, int64_t lds0, uint64_t rb,
                                                uint32_t js, uint32_t je, const uint32_t *sstart,
                                                const uint32_t *snrel, const uint32_t *meta0, const uint32_t *meta1,
                                                const uint8_t *map, const uint32_t *padm, const SweepField *sf) {
    const uint32_t tid = threadIdx.x, m = je - js;
    uint32_t fpre = 0, d = 0;
    for (uint32_t k = 0; k < a.nf; ++k) {
        const VField &f = a.f[k];
        if (f.kind != XDRG_K_DYNAMIC) {
            const uint32_t nw = f.xbytes >> 2;
            if (nw) {
                const uint32_t G = a.force_g ? a.force_g : pow2_lanes((uint64_t)nw * 4, 16);
                const uint32_t gl = tid & (G - 1), ng = kRecThreads / G;
                for (uint32_t j = js + tid / G; j < je; j += ng) {
                    const uint32_t *w = (const uint32_t *)(tile + (lds0 + (int64_t)(sstart[j] + fpre +
                                                                               dyn_before(a, snrel, j, d, RS))));
                    for (uint32_t i = gl; i < nw; i += G) fixed_store(f, rb + j, 4 * i, w[i]);
                }
            }
            fpre += f.xbytes;
            continue;
        }
        const SweepField &s = sf[d];
        if (f.xsz == 1) {
            sweep_bytes(s.col, tile, d ? meta1 : meta0, map + s.moff, padm, s.x0, s.nq, m, s.xb, s.xe);
        } else {
            sweep_words((uint32_t *)s.col, tile, d ? meta1 : meta0, map + s.moff, s.x0, s.nq, m, s.xb, s.xe);
        }
        ++d;
    }
}

// As enc_fit, over the XDR stream range of records [js, js + 1 + t).
__device__ __forceinline__ uint32_t dec_fit(const RecArgs &a, const uint32_t *sstart, uint64_t sb,
                                            const uint32_t *snrel, uint32_t js, uint32_t nlive) {
    const uint32_t je = js + 1 + threadIdx.x;
    bool fits = false;
    if (je <= nlive) {
        const uint8_t *a0;
        const uint64_t e = sb + sstart[je - 1] + (a.fixed_xdr - (a.framed ? 4 : 0)) + dyn_before(a, snrel, je - 1, a.ndyn);
        fits = 16 * stage_chunks(a.xdr + sb + sstart[js], a.xdr + e, &a0) <= a.tile_bytes;
    }
    return (uint32_t)__syncthreads_count(fits);
}

// ---- one-pass derived counts (tuning key 31 = 2, spec_mode 3) ---------------
// The sweep block walks its own records (the derived pass's one length-word
// gather per record), publishes its count totals and learns the native
// offset of its first element per dynamic field from its predecessors: a
// decoupled look-back over one status word per block and dynamic field, flag
// in bits 62-63 (1 = the block's own total, 2 = the inclusive prefix over
// blocks [0, b]) | value, stored and polled with agent-scope atomics (a tagged
// word needs no fence).  Blocks take tickets in start order, so every block
// waited on is running and publishes its total without waiting.  Errors stay
// local: a block decodes its records before its own first walk error, and
// the error key (atomicMin) orders them over the batch as the walk does.
constexpr uint64_t kLbOwn = 1ull << 62, kLbIncl = 2ull << 62, kLbVal = kLbOwn - 1;

__device__ __forceinline__ void lb_put(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t lb_get(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
    for (int o = 32; o; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
// Wave 0 of block b: publish agg (lb_publish, as soon as the walk has the
// block's totals); later (lb_wait, after the block's offset-free prologue, so
// the predecessors' totals arrive meanwhile) look back over the predecessors
// 64 at a time down to the nearest inclusive prefix of each field, publish
// the inclusive prefix; s_base[d] = the exclusive prefix of field d.
__device__ __forceinline__ void lb_publish(const RecArgs &a, uint64_t b, const uint64_t (&agg)[kMaxDynLds]) {
    if ((threadIdx.x & 63) == 0)
#pragma unroll
        for (int d = 0; d < kMaxDynLds; ++d)
            if ((uint32_t)d < a.ndyn) lb_put(a.block_sums + (uint64_t)d * a.nblocks + b, (b ? kLbOwn : kLbIncl) | agg[d]);
}
__device__ __forceinline__ void lb_wait(const RecArgs &a, uint64_t b, const uint64_t (&agg)[kMaxDynLds],
                                        uint64_t *s_base) {
    const uint32_t lane = threadIdx.x & 63, nd = a.ndyn;
    const uint64_t nb = a.nblocks;
    uint64_t *st = a.block_sums;
    uint64_t pre[kMaxDynLds] = {0, 0, 0, 0};
    uint32_t done = 0;
    const uint32_t all = (1u << nd) - 1;
    int64_t p = (int64_t)b - 1 - (int64_t)lane;
    while (b && done != all) {
        uint64_t v[kMaxDynLds];
        for (;;) {
            bool ready = true;
#pragma unroll
            for (int d = 0; d < kMaxDynLds; ++d) {
                if ((uint32_t)d >= nd) { v[d] = kLbIncl; continue; }
                const uint64_t x = p >= 0 ? lb_get(st + (uint64_t)d * nb + (uint64_t)p) : kLbIncl;
                v[d] = x;
                ready = ready && (x >> 62) != 0;
            }
            if (__all(ready)) break;
            __builtin_amdgcn_s_sleep(2);
        }
#pragma unroll
        for (int d = 0; d < kMaxDynLds; ++d) {
            if ((uint32_t)d >= nd || ((done >> d) & 1)) continue;
            const uint64_t pm = __ballot((v[d] >> 62) == 2);
            const uint32_t first = pm ? (uint32_t)__builtin_ctzll(pm) : 63u;   // nearest inclusive predecessor
            pre[d] += wave_sum64(lane <= first ? (v[d] & kLbVal) : 0);
            if (pm) done |= 1u << d;
        }
        p -= 64;
    }
    if (lane == 0)
#pragma unroll
        for (int d = 0; d < kMaxDynLds; ++d) {
            if ((uint32_t)d >= nd) continue;
            if (b) lb_put(st + (uint64_t)d * nb + b, kLbIncl | (pre[d] + agg[d]));
            s_base[d] = pre[d];
            if (b + 1 == nb) {
                a.totals[d] = pre[d] + agg[d];
                a.f[a.dyn_idx[d]].offsets[a.n] = pre[d] + agg[d];
            }
        }
}

// The one-pass sweep's walk of its block (k_dec_sizes_g<true>'s, over records
// rb + tid + 256 j): counts into scnt, errors into the error key and the
// block's first failing record into *s_bad.  (Its record-mark check is the
// branch-free one of walk_counts_lockstep: the branchy form, inlined here as
// in round 2's look-back decode, lost FRAME errors; tools/diag_trunc.py.)
__device__ __forceinline__ void one_pass_walk(const RecArgs &a, uint64_t rb, uint32_t *scnt, uint32_t *s_bad) {
    const uint32_t tid = threadIdx.x;
#pragma unroll
    for (int j = 0; j < kRecPerThread; ++j)
        for (uint32_t d = 0; d < a.ndyn; ++d) scnt[(size_t)d * kRecPerBlock + tid + j * kRecThreads] = 0;
    const uint64_t r0 = rb + tid;
    const uint32_t nj = r0 < a.n ? (uint32_t)((a.n - r0 + kRecThreads - 1) / kRecThreads < (uint64_t)kRecPerThread
                                              ? (a.n - r0 + kRecThreads - 1) / kRecThreads : (uint64_t)kRecPerThread)
                                 : 0u;
    uint32_t err[kRecPerThread], sub[kRecPerThread];
    uint32_t tail = 0;   // fixed XDR bytes after the last dynamic field
    for (uint32_t k = a.dyn_idx[a.ndyn - 1] + 1; k < a.nf; ++k) tail += a.f[k].xbytes;
    bool unc = false, dead = false;
    walk_counts_lockstep<true>(a, r0, nj, scnt + tid, err, sub, kRecThreads, tail, &unc);
    if (unc) spec_fail(a);
#pragma unroll
    for (int j = 0; j < kRecPerThread; ++j) {
        if (!dead && err[j]) {
            atomicMin(a.errkey, err_key(r0 + (uint64_t)j * kRecThreads, sub[j], err[j]));
            atomicMin(s_bad, tid + j * kRecThreads);
            dead = true;   // later records of this thread are past the error
        }
        if (dead)
            for (uint32_t d = 0; d < a.ndyn; ++d) scnt[(size_t)d * kRecPerBlock + tid + j * kRecThreads] = 0;
    }
}

#ifndef XDRG_DEC_STAGE_OCC
#define XDRG_DEC_STAGE_OCC 5   // blocks per CU the register budget is sized for
#endif
template <bool SW, bool ONE = false>
__device__ __forceinline__ void dec_stage_body(const RecArgs &a, uint64_t bid) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr uint32_t RS = kRecPerBlock + 1;
    uint32_t *sstart = (uint32_t *)smem;
    uint32_t *snrel = sstart + RS;
    uint8_t *supto = (uint8_t *)(snrel + (size_t)a.ndyn * RS);
    uint8_t *tile = smem + dec_stage_meta(a.ndyn);
    __shared__ uint32_t s_wide;
    __shared__ uint64_t s_base[kMaxDynLds];   // native offset of the block's first element, per dynamic field
    const uint32_t tid = threadIdx.x, t0 = tid * kRecPerThread;
    const uint64_t nb = a.nblocks;
    uint32_t *scnt1 = (uint32_t *)tile;   // ONE: the block's walked counts [ndyn][RPB], read before staging
    uint32_t nlive;
    uint64_t agg1[kMaxDynLds] = {0, 0, 0, 0};   // ONE: the block's totals (published, waited on below)
    if (ONE) {
        __shared__ unsigned long long s_tk;
        __shared__ uint32_t s_bad1;
        if (tid == 0) {
            s_tk = atomicAdd(a.lb_ticket, 1ull) + 1ull;   // (the ticket word starts at ~0)
            s_bad1 = kRecPerBlock;
        }
        __syncthreads();
        bid = s_tk;
        const uint64_t rb = bid * kRecPerBlock;
        one_pass_walk(a, rb, scnt1, &s_bad1);
        uint64_t agg[kMaxDynLds] = {0, 0, 0, 0};
#pragma unroll
        for (int d = 0; d < kMaxDynLds; ++d) {
            if ((uint32_t)d >= a.ndyn) continue;
            uint64_t sv = 0;
#pragma unroll
            for (int j = 0; j < kRecPerThread; ++j) sv += scnt1[(size_t)d * kRecPerBlock + tid + j * kRecThreads];
            agg[d] = block_sum(sv);   // (its barriers also publish s_bad1 and the counts)
        }
        if (tid < 64) lb_publish(a, bid, agg);
        // a block of big records would be the group kernel's, which is not
        // launched here: the exact rerun decodes the batch (the block still
        // settles its prefix: its successors wait for it)
        if (a.big_rec && block_is_big_at(a, bid, true)) {
            if (tid < 64) lb_wait(a, bid, agg, s_base);
            if (tid == 0) spec_fail(a);
            return;
        }
#pragma unroll
        for (int d = 0; d < kMaxDynLds; ++d) agg1[d] = agg[d];
        const uint32_t nr = (uint32_t)(a.n > rb ? (a.n - rb < (uint64_t)kRecPerBlock ? a.n - rb : (uint64_t)kRecPerBlock) : 0);
        nlive = s_bad1 < nr ? s_bad1 : nr;
    } else {
        if (a.big_rec && block_is_big_at(a, bid, true)) return;   // the group kernel's block
    }
    const uint64_t rb = bid * kRecPerBlock;
    const uint32_t nrec = (uint32_t)(a.n > rb ? (a.n - rb < (uint64_t)kRecPerBlock ? a.n - rb : (uint64_t)kRecPerBlock) : 0);
    uint32_t xs[kMaxDynLds];             // XDR element size per dynamic field (1: padded bytes)
#pragma unroll
    for (int e = 0; e < kMaxDynLds; ++e) xs[e] = (uint32_t)e < a.ndyn ? a.f[a.dyn_idx[e]].xsz : 0u;
    if (!ONE) {
        const unsigned long long walk_key = *a.errkey;  // final after k_dec_sizes_g
        const uint64_t bad = walk_key == kNoError ? a.n : (uint64_t)(walk_key >> 16);
        if (tid < a.ndyn) s_base[tid] = a.block_sums[(uint64_t)tid * nb + bid];
        nlive = bad > rb ? (uint32_t)(bad - rb < (uint64_t)nrec ? bad - rb : (uint64_t)nrec) : 0;
    }
    if (tid == 0) s_wide = 0;
    // ---- prologue: counts, native offsets (written to the columns), capacity,
    // extents; block-relative first (ONE: while the look-back's predecessors settle)
    const uint64_t sb = nlive ? rec_extent(a, rb).a + (a.framed ? 4 : 0) : 0;   // stream offset of sstart 0
    uint32_t upto[kRecPerThread];
    bool wide = false;
#pragma unroll
    for (int j = 0; j < kRecPerThread; ++j) {
        const bool live = t0 + j < nlive;
        upto[j] = live ? a.nf : 0u;
        if (live) {
            const uint64_t st = rec_extent(a, rb + t0 + j).a + (a.framed ? 4 : 0);
            wide |= st < sb || st - sb >= (1ull << 31);   // out of order or beyond 31 bits: direct path
            sstart[t0 + j] = (uint32_t)(st - sb);
        }
    }
#pragma unroll
    for (int d = 0; d < kMaxDynLds; ++d) {
        if ((uint32_t)d >= a.ndyn) continue;
        const uint32_t k = a.dyn_idx[d];
        const VField &f = a.f[k];
        uint32_t c[kRecPerThread];
        uint64_t s = 0;
#pragma unroll
        for (int j = 0; j < kRecPerThread; ++j) {
            const uint64_t r = rb + t0 + j;
            c[j] = t0 + j < nlive ? (ONE ? scnt1[(size_t)d * kRecPerBlock + t0 + j] : a.rec_cnt[(uint64_t)d * a.n + r]) : 0u;
            s += c[j];
        }
        uint64_t btot;
        uint64_t off = block_excl_scan(s, &btot);   // block-relative
        wide |= btot * (f.xsz == 1 ? 1 : f.nsz) >= (1ull << 31);
#pragma unroll
        for (int j = 0; j < kRecPerThread; ++j) {
            snrel[d * RS + t0 + j] = (uint32_t)off;
            off += c[j];
        }
        if (tid == kRecThreads - 1) snrel[d * RS + kRecPerBlock] = (uint32_t)off;
    }
    if (ONE) {
        if (tid < 64) lb_wait(a, bid, agg1, s_base);
        __syncthreads();   // s_base; snrel
    } else {
        __syncthreads();   // snrel
    }
#pragma unroll
    for (int d = 0; d < kMaxDynLds; ++d) {   // native offsets and capacity, now absolute
        if ((uint32_t)d >= a.ndyn) continue;
        const uint32_t k = a.dyn_idx[d];
        const VField &f = a.f[k];
        const uint64_t base = ONE ? s_base[d] : a.block_sums[(uint64_t)d * nb + bid];
        const uint32_t *rel = snrel + d * RS;
#pragma unroll
        for (int j = 0; j < kRecPerThread; ++j) {
            const uint64_t r = rb + t0 + j;
            const uint64_t off = base + rel[t0 + j];
            if (t0 + j < nrec) {
                f.offsets[r] = off;
                if (t0 + j < nlive && off + (rel[t0 + j + 1] - rel[t0 + j]) > f.cap) {   // native column too small
                    atomicMin(a.errkey, err_key(r, 2 * k + 2, XDRG_E_CAPACITY));
                    if (upto[j] > k) upto[j] = k;
                    if (a.spec_mode & 1) spec_fail(a);   // on derived counts: the exact walk decides
                }
            }
        }
        if (!ONE && tid == 0 && bid == 0) f.offsets[a.n] = a.totals[d];   // (ONE: lb_wait)
    }
#pragma unroll
    for (int j = 0; j < kRecPerThread; ++j) supto[t0 + j] = (uint8_t)upto[j];
    bool full = true;   // every live record decodes every field: byte fields take dec_bytes_lean
#pragma unroll
    for (int j = 0; j < kRecPerThread; ++j) full &= t0 + j >= nlive || upto[j] == a.nf;
    const bool lean = __syncthreads_and(full);
    // SW: the output-stationary sweep (key 20 = 2; the launcher checked the
    // word columns' alignment and ndyn <= 2) for error-free blocks, record by
    // record otherwise.  meta0 reuses supto (an error-free block's records all
    // decode every field); meta1 and the chunk map follow the tile.
    const bool sweep = SW && lean;
    uint32_t *smeta1 = (uint32_t *)(tile + a.tile_bytes + kStageSlack);
    uint8_t *smap = (uint8_t *)smeta1 + ((((size_t)kRecThreads + kSweepMetaPad) * 4 + 15) & ~(size_t)15);
    uint32_t *spadm = (uint32_t *)(smap + dec_sweep_map(a.tile_bytes));
    if (SW && threadIdx.x < kPadMasks / 4)   // (read after the sub-batches' stage barriers)
        spadm[threadIdx.x] = lo_mask((int32_t)(threadIdx.x >> 2) - 4 * (int32_t)(threadIdx.x & 3));
    __shared__ SweepField sf[2];
    // staging needs every record's fields to end where the next begins or
    // before (records in stream order); otherwise the block goes direct
    const uint32_t fx = a.fixed_xdr - (a.framed ? 4 : 0);   // fixed XDR bytes of the fields
    if (!wide) {
#pragma unroll
        for (int j = 0; j < kRecPerThread; ++j) {
            const uint32_t i = t0 + j;
            if (i + 1 < nlive && (sstart[i + 1] < sstart[i] || sstart[i] + fx + dyn_before(a, snrel, i, a.ndyn) > sstart[i + 1]))
                wide = true;
        }
    }
    if (wide) s_wide = 1;
    __syncthreads();
    wide = s_wide != 0;
    const uint8_t *in = a.xdr;

    if (wide) {
        for (uint32_t j = 0; j < nlive; ++j)
            dec_record_block(a, rb + j, rec_extent(a, rb + j).a + (a.framed ? 4 : 0), supto[j], snrel, j, tid, kRecThreads);
        return;
    }
    // ---- sub-batches
    uint32_t js = 0;
    uint32_t k1 = nlive ? dec_fit(a, sstart, sb, snrel, js, nlive) : 0;
    while (js < nlive) {
        if (k1 == 0) {   // too large for the tile: the whole block decodes record js
            // (an error-free block's every record decodes all fields; the sweep keeps its metadata in supto)
            dec_record_block(a, rb + js, sb + sstart[js], sweep ? a.nf : supto[js], snrel, js, tid, kRecThreads);
            ++js;
            k1 = js < nlive ? dec_fit(a, sstart, sb, snrel, js, nlive) : 0;
            continue;
        }
        const uint32_t je = js + k1;
        const uint8_t *a0[kMaxDynLds] = {nullptr, nullptr, nullptr, nullptr};
        uint32_t cb[kMaxDynLds + 1] = {0, 0, 0, 0, 0};
        cb[1] = stage_chunks(in + sb + sstart[js], in + sb + sstart[je - 1] + fx + dyn_before(a, snrel, je - 1, a.ndyn),
                             &a0[0]);
        const int64_t lds0 = -(int64_t)(a0[0] - (in + sb));   // tile offset of sstart value x: lds0 + x
        if (SW) {   // stage by LDS-DMA while the record lanes build the sweep's metadata
            // (blocks that decode record by record from HBM below never read the tile)
            if (sweep) {
                stage_dma(tile, a0, cb, 1);
                dec_sweep_prep<RS>(a, lds0, js, je, sstart, snrel, s_base, xs, (uint32_t *)supto, smeta1, smap, sf);
                // LDS-DMA writes retire on vmcnt, not lgkmcnt: every wave waits for
                // its own DMA before the barrier, so no wave reads a chunk that
                // another wave's load has not landed yet
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
        } else {
            stage_copy(tile, a0, cb, 1);
        }
        __syncthreads();
        if (!SW) dec_stage_batch<RS>(a, tile, lds0, rb, js, je, sstart, snrel, supto, s_base, xs, lean, tid, kRecThreads);
        else if (sweep) {
            if ((a.spec_mode & 1) && tid < je - js) {   // derived counts (key 31): check the count words
                const uint32_t j = js + tid, dl = a.ndyn - 1;
                uint32_t fb = 0;   // fixed XDR bytes before the last dynamic field
                for (uint32_t k = 0; k < a.dyn_idx[dl]; ++k) fb += a.f[k].kind != XDRG_K_DYNAMIC ? a.f[k].xbytes : 0u;
                const uint32_t *rel = snrel + dl * RS;
                const uint32_t cw = tile_word(tile, lds0 + (int64_t)(sstart[j] + fb + dyn_before_xs(xs, snrel, j, dl, RS)));
                if (bswap32r(cw) != rel[j + 1] - rel[j]) spec_fail(a);
            }
            dec_stage_sweep<RS>(a, tile, lds0, rb, js, je, sstart, snrel, (uint32_t *)supto, smeta1, smap, spadm, sf);
        } else
            for (uint32_t j = js; j < je; ++j)
                dec_record_block(a, rb + j, sb + sstart[j], supto[j], snrel, j, tid, kRecThreads);
        js = je;
        k1 = js < nlive ? dec_fit(a, sstart, sb, snrel, js, nlive) : 0;   // its barrier ends the tile's use
    }
}

#ifndef XDRG_DEC_SWEEP_OCC
#define XDRG_DEC_SWEEP_OCC 4   // blocks per CU the sweep kernel's register budget is sized for (5: 96 VGPRs
                               // with spills, 3.71 ms vs 3.18 ms on config 4 at its best tile)
#endif
// (LOOP: blocks loop over record blocks as k_dec_sizes_g)
template <bool LOOP>
__global__ __launch_bounds__(kRecThreads, XDRG_DEC_STAGE_OCC) void k_dec_stage(const RecArgs a) {
    if (spec_skip(a)) return;
    if (!LOOP) { dec_stage_body<false>(a, blockIdx.x); return; }
    for (uint64_t b = blockIdx.x; b < a.nblocks; b += gridDim.x) {
        dec_stage_body<false>(a, b);
        __syncthreads();
    }
}
// MODE 0: a block per record block; 1 (LOOP): blocks loop over record blocks;
// 2: one pass with derived counts (spec_mode 3: walk + look-back in the block)
template <int MODE>
__global__ __launch_bounds__(kRecThreads, XDRG_DEC_SWEEP_OCC) void k_dec_sweep(const RecArgs a) {
    if (MODE == 2) { dec_stage_body<true, true>(a, 0); return; }
    if (spec_skip(a)) return;   // derived counts already failed / held (key 31)
    if (MODE == 0) { dec_stage_body<true>(a, blockIdx.x); return; }
    for (uint64_t b = blockIdx.x; b < a.nblocks; b += gridDim.x) {
        dec_stage_body<true>(a, b);
        __syncthreads();
    }
}

// ===========================================================================
// Launchers
// ===========================================================================
// Group kernels: U 16-byte chunks per lane and R records per lane in flight
// (a U x R sweep on configs 3 and 4 stayed within 5 %: tools/sweep_rec.py).
constexpr int kGroupU = 2, kGroupR = 1;

int launch_scan_rows(uint64_t *sums, uint64_t nblocks, uint64_t *totals, uint32_t rows, void *stream) {
    if (!rows) return hipSuccess;
    hipLaunchKernelGGL(k_scan_rows, dim3(rows), dim3(1024), 0, (hipStream_t)stream, sums, nblocks, totals,
                       (const uint32_t *)nullptr);
    return (int)hipGetLastError();
}

int launch_spec_reset(const uint32_t *spec, unsigned long long *errkey, void *stream) {
    hipLaunchKernelGGL(k_spec_reset, dim3(1), dim3(64), 0, (hipStream_t)stream, spec, errkey);
    return (int)hipGetLastError();
}

// The staged decode takes the output-stationary sweep (k_dec_sweep).
static bool dec_sweep_ok(const RecArgs &a, const Tuning &t) {
    bool sw = t.dec_lean == 2 && t.sweep_tile <= 32768 && a.ndyn <= 2;   // (16-bit tile offsets in meta)
    for (uint32_t d = 0; d < a.ndyn && sw; ++d) {   // word columns take 16-byte stores of 4-byte elements
        const VField &f = a.f[a.dyn_idx[d]];
        sw = f.xsz == 1 || (f.nsz == 4 && ((uintptr_t)f.data & 3) == 0);
    }
    return sw;
}

bool rec_spec_ok(const RecArgs &a, const Tuning &t) {
    if (!t.spec_sizes || t.rec != 4 || a.ncond || a.byref || !a.rec_in || !a.ndyn || a.ndyn > 2) return false;
    for (uint32_t d = 0; d < a.ndyn; ++d)
        if (!stage_type(a.f[a.dyn_idx[d]].type, a.f[a.dyn_idx[d]].xsz)) return false;
    return a.f[a.dyn_idx[a.ndyn - 1]].xsz == 4 && dec_sweep_ok(a, t);   // a word vector last
}

int launch_rec_phase(const RecArgs &args, int phase, const Tuning &t, void *stream) {
    RecArgs a = args;
    a.force_g = t.force_g;
    a.lane_bytes_enc = t.lane_bytes_enc;
    a.lane_bytes_dec = t.lane_bytes_dec;
    a.tile_bytes = t.tile_bytes;
    a.big_rec = 0;
    a.xcd = (uint32_t)t.xcd_order;
    hipStream_t st = (hipStream_t)stream;
    const uint64_t nb = a.nblocks;
    // conditional schemas (unions / optional data) and by-reference payloads take
    // the lane-per-record kernels (wave per record beyond kMaxDynLds dynamic fields)
    const bool special = a.ncond || a.byref;
    const bool grp = a.ndyn <= (uint32_t)kMaxDynLds && !special;
    const bool lane = a.ndyn <= (uint32_t)kMaxDynLds && special;
    bool stage = grp && t.rec == 4;
    for (uint32_t d = 0; d < a.ndyn && stage; ++d)
        stage = stage_type(a.f[a.dyn_idx[d]].type, a.f[a.dyn_idx[d]].xsz);
    // one dynamic byte field, blocks on the group kernels: the payload kernels move it
    const bool pay = a.pay_pos && a.ndyn == 1 && a.f[a.dyn_idx[0]].xsz == 1 && ((stage && t.big_rec) || (grp && !stage));
    a.payk = pay ? 1u : 0u;
    // the derived-count decode's exact rerun (spec_mode 2) runs on a small grid
    // whose blocks loop over the record blocks: when the rerun is not needed
    // its kernels return at once for a few microseconds each
    const dim3 dgrid((unsigned)(a.spec_mode == 2 && nb > 1024 ? 1024 : nb));
    const uint64_t pblk = (a.n + 3) / 4;   // payload kernels: a wave per record, 4 records per block
    const dim3 pgrid((unsigned)(pblk < (1ull << 30) ? pblk : (1ull << 30)));
    switch (phase) {
    case REC_ENC_SIZES: hipLaunchKernelGGL(k_enc_sizes, dim3(nb), dim3(kRecThreads), 0, st, a); break;
    case REC_ENC_SCAN:
        hipLaunchKernelGGL(k_scan_rows, dim3(1), dim3(1024), 0, st, a.block_sums, nb, a.totals,
                           (const uint32_t *)nullptr);
        break;
    case REC_ENC_PLACE:
        if (stage) {   // small-record blocks staged, large-record blocks by the group kernel
            a.big_rec = t.big_rec;
            hipLaunchKernelGGL(k_enc_stage_rm, dim3(nb), dim3(kRecThreads),
                               enc_stage_meta(a.ndyn) + a.tile_bytes + kStageSlack, st, a);
            if (a.big_rec) hipLaunchKernelGGL((k_enc_place_g<kGroupU, kGroupR>), dim3(nb), dim3(kRecThreads), enc_lds_bytes(a.ndyn), st, a);
            if (a.big_rec && pay) hipLaunchKernelGGL(k_enc_payload, pgrid, dim3(256), 0, st, a);
        } else if (lane) {
            hipLaunchKernelGGL(k_enc_lane, dim3(nb), dim3(kRecThreads), enc_lds_bytes(a.ndyn), st, a);
        } else if (grp) {
            hipLaunchKernelGGL((k_enc_place_g<kGroupU, kGroupR>), dim3(nb), dim3(kRecThreads), enc_lds_bytes(a.ndyn), st, a);
            if (pay) hipLaunchKernelGGL(k_enc_payload, pgrid, dim3(256), 0, st, a);
        }
        else hipLaunchKernelGGL(k_enc_place_wave, dim3(nb), dim3(kRecThreads), 0, st, a);
        break;
    case REC_DEC_SIZES:
        if (a.spec_mode == 3) break;   // one pass: the sweep walks its own block
        if (a.spec_mode == 1) {   // extent-derived counts (key 31; rec_spec_ok held)
            a.big_rec = t.big_rec;
            hipLaunchKernelGGL(k_dec_sizes_g<true>, dim3(nb), dim3(kRecThreads), (size_t)a.ndyn * kRecPerBlock * 4, st, a);
        } else if (a.spec_mode == 2) {
            hipLaunchKernelGGL((k_dec_sizes_g<false, true>), dgrid, dim3(kRecThreads), (size_t)a.ndyn * kRecPerBlock * 4, st, a);
        } else if (grp || lane) hipLaunchKernelGGL(k_dec_sizes_g<false>, dim3(nb), dim3(kRecThreads),
                                    (size_t)a.ndyn * kRecPerBlock * 4, st, a);
        else hipLaunchKernelGGL(k_dec_sizes_wave, dim3(nb), dim3(kRecThreads), 0, st, a);
        break;
    case REC_DEC_SCAN:
        if (a.ndyn && a.spec_mode != 3)
            hipLaunchKernelGGL(k_scan_rows, dim3(a.ndyn), dim3(1024), 0, st, a.block_sums, nb, a.totals,
                               (const uint32_t *)(a.spec_mode == 2 ? a.spec : nullptr));
        break;
    case REC_DEC_PLACE:
        if (stage) {
            a.big_rec = t.big_rec;
            const bool sw = dec_sweep_ok(a, t);
            if (sw) a.tile_bytes = t.sweep_tile;
            const size_t lds = dec_stage_meta(a.ndyn) + a.tile_bytes + kStageSlack + (sw ? dec_sweep_extra(a.tile_bytes) : 0);
            const bool loop = a.spec_mode == 2;
            if (sw && a.spec_mode == 3) hipLaunchKernelGGL(k_dec_sweep<2>, dim3(nb), dim3(kRecThreads), lds, st, a);
            else if (sw && loop) hipLaunchKernelGGL(k_dec_sweep<1>, dgrid, dim3(kRecThreads), lds, st, a);
            else if (sw) hipLaunchKernelGGL(k_dec_sweep<0>, dim3(nb), dim3(kRecThreads), lds, st, a);
            else if (loop) hipLaunchKernelGGL(k_dec_stage<true>, dgrid, dim3(kRecThreads), lds, st, a);
            else hipLaunchKernelGGL(k_dec_stage<false>, dim3(nb), dim3(kRecThreads), lds, st, a);
            // (the derived-count pass hands any big-record block to the exact rerun)
            if (a.big_rec && loop) hipLaunchKernelGGL((k_dec_place_g<kGroupU, kGroupR, true>), dgrid, dim3(kRecThreads), dec_g_lds_bytes(a.ndyn), st, a);
            else if (a.big_rec && !(a.spec_mode & 1)) hipLaunchKernelGGL((k_dec_place_g<kGroupU, kGroupR>), dim3(nb), dim3(kRecThreads), dec_g_lds_bytes(a.ndyn), st, a);
            if (a.big_rec && pay) hipLaunchKernelGGL(k_dec_payload, pgrid, dim3(256), 0, st, a);
        } else if (lane) {
            hipLaunchKernelGGL(k_dec_lane, dim3(nb), dim3(kRecThreads), dec_g_lds_bytes(a.ndyn), st, a);
        } else if (grp) {
            hipLaunchKernelGGL((k_dec_place_g<kGroupU, kGroupR>), dim3(nb), dim3(kRecThreads), dec_g_lds_bytes(a.ndyn), st, a);
            if (pay) hipLaunchKernelGGL(k_dec_payload, pgrid, dim3(256), 0, st, a);
        }
        else hipLaunchKernelGGL(k_dec_place_wave, dim3(nb), dim3(kRecThreads), 0, st, a);
        break;
    default: return (int)hipErrorInvalidValue;
    }
    return (int)hipGetLastError();
}

}  // namespace xdrg
