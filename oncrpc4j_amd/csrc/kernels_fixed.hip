// kernels_fixed.hip — fixed-size record kernels of the MI355X XDR engine.
//
// A fixed-size XDR record (no dynamic field) is a sequence of 4-byte
// big-endian words (RFC 4506 §3; oncrpc4j xdr/Xdr.java:545-548, 812-815).
// Two kernels cover every fixed schema:
//
//  * k_stream_*  — the native record is word-for-word the XDR record
//    (array-of-structs whose fields sit at their XDR word positions: int,
//    float, hyper, double, 4-multiple opaque).  The batch is then one flat
//    stream of 16-byte vectors; each lane byte-swaps (v_perm_b32) whole
//    dwordx4 vectors, U vectors in flight per lane.  Pure HBM streaming: 1
//    read + 1 write of every byte, the copy-kernel roofline.
//
//  * k_wordmap_* — any other fixed layout (struct-of-arrays columns,
//    strided columns, bool/short/byte, odd opaque sizes, record marks).
//    Each lane owns 4 consecutive XDR words (one dwordx4 of the stream) and
//    maps each to its native column through a per-word op table held in
//    LDS.  XDR side: coalesced 16-byte accesses; native side: per-element.
#include <hip/hip_runtime.h>

#include "xdrg_internal.h"

namespace xdrg {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// Float.floatToIntBits: every NaN -> 0x7fc00000 (Xdr.java:674-676).
__device__ __forceinline__ uint32_t canon_f32(uint32_t u) {
    return ((u & 0x7fffffffu) > 0x7f800000u) ? 0x7fc00000u : u;
}
// Double.doubleToLongBits: every NaN -> 0x7ff8000000000000 (Xdr.java:685-687).
__device__ __forceinline__ void canon_f64(uint32_t &hi, uint32_t &lo) {
    const uint32_t h = hi & 0x7fffffffu;
    if (h > 0x7ff00000u || (h == 0x7ff00000u && lo != 0)) { hi = 0x7ff80000u; lo = 0; }
}

template <bool NT>
__device__ __forceinline__ u32x4 ld4(const u32x4 *p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT>
__device__ __forceinline__ void st4(u32x4 *p, u32x4 v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// ---------------------------------------------------------------------------
// Streaming kernels (AoS-dense layouts).
// ---------------------------------------------------------------------------
template <int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void k_stream_bswap(const u32x4 *__restrict__ src,
                                                      u32x4 *__restrict__ dst, uint64_t nvec) {
    const uint64_t step = (uint64_t)gridDim.x * (256 * U);
    for (uint64_t i = (uint64_t)blockIdx.x * (256 * U) + threadIdx.x; i < nvec; i += step) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t k = i + (uint64_t)u * 256;
            if (k < nvec) v[u] = ld4<NTL>(src + k);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t k = i + (uint64_t)u * 256;
            if (k < nvec) {
                u32x4 o;
                o.x = bswap32(v[u].x); o.y = bswap32(v[u].y);
                o.z = bswap32(v[u].z); o.w = bswap32(v[u].w);
                st4<NTS>(dst + k, o);
            }
        }
    }
}

// One XDR/native word of a mixed AoS-dense record.  x[] holds the 4 words of
// the vector; q is the record word position of x[j].  HYPER/DOUBLE pairs are
// guaranteed (host check) to sit in one vector: HI at an even j, LO at j+1.
__device__ __forceinline__ uint32_t stream_word(uint8_t op, const uint32_t *x, int j) {
    switch (op) {
    case OP_FLOAT: return bswap32(canon_f32(x[j]));
    case OP_HYPER_HI: return bswap32(x[j + 1]);
    case OP_HYPER_LO: return bswap32(x[j - 1]);
    case OP_DOUBLE_HI: { uint32_t hi = x[j + 1], lo = x[j]; canon_f64(hi, lo); return bswap32(hi); }
    case OP_DOUBLE_LO: { uint32_t hi = x[j], lo = x[j - 1]; canon_f64(hi, lo); return bswap32(lo); }
    case OP_OPAQUE: return x[j];
    default: return bswap32(x[j]);
    }
}

template <int U, bool NT>
__global__ __launch_bounds__(256) void k_stream_ops(const StreamArgs a) {
    __shared__ uint8_t sops[kMaxWords];
    for (int t = threadIdx.x; t < (int)a.w; t += 256) sops[t] = a.ops[t];
    __syncthreads();
    const u32x4 *__restrict__ src = (const u32x4 *)a.src;
    u32x4 *__restrict__ dst = (u32x4 *)a.dst;
    const uint64_t step = (uint64_t)gridDim.x * (256 * U);
    for (uint64_t i = (uint64_t)blockIdx.x * (256 * U) + threadIdx.x; i < a.nvec; i += step) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t k = i + (uint64_t)u * 256;
            if (k < a.nvec) v[u] = ld4<NT>(src + k);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t k = i + (uint64_t)u * 256;
            if (k < a.nvec) {
                uint32_t p = (uint32_t)((k * 4) % a.w);
                const uint32_t x[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
                uint32_t o[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    o[j] = stream_word(sops[p], x, j);
                    if (++p == a.w) p = 0;
                }
                u32x4 ov; ov.x = o[0]; ov.y = o[1]; ov.z = o[2]; ov.w = o[3];
                st4<NT>(dst + k, ov);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Record-marked streaming kernels (AoS-dense records of 4-byte words: int,
// uint, enum, float, 4-multiple opaque).  XDR record = mark + W words, native
// record = W words.  One lane per 16-byte chunk of the destination: it reads
// the (at most 5) source words its chunk needs with one 4-byte-aligned
// 16-byte load plus one dword, inserts or skips the record mark, and writes
// one aligned 16-byte vector.  Decode checks every mark (the lane whose
// chunk holds a record's first native word checks that record's mark).
// ---------------------------------------------------------------------------
typedef uint32_t u32x4w __attribute__((ext_vector_type(4), aligned(4)));

__device__ __forceinline__ uint32_t pick5(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t e, uint32_t i) {
    return i == 0 ? a : i == 1 ? b : i == 2 ? c : i == 3 ? d : e;
}
__device__ __forceinline__ uint32_t word_op(uint8_t op, uint32_t x) {
    return op == OP_FLOAT ? bswap32(canon_f32(x)) : op == OP_OPAQUE ? x : bswap32(x);
}
// q = x / d, r = x % d for x < 2^52 (double reciprocal + one correction)
__device__ __forceinline__ void divmod(uint64_t x, uint32_t d, double inv, uint64_t &q, uint32_t &r) {
    q = (uint64_t)((double)x * inv);
    int64_t rr = (int64_t)(x - q * d);
    if (rr < 0) { --q; rr += d; }
    else if (rr >= (int64_t)d) { ++q; rr -= d; }
    r = (uint32_t)rr;
}

// ---- wave-local LDS transpose (decode of records under 3 words) --------------
// Each wavefront owns 256 consecutive destination words: it loads the source
// words they need as 16-byte ALIGNED vectors (coalesced, one per lane,
// nontemporal) into its own LDS slice, then every lane gathers its 4
// destination words from LDS and writes one aligned 16-byte vector.  Only
// the wave synchronises (no block barrier after the op-table staging).  The
// lean kernels below are faster; this one stays for records
// whose 4 native words can span two marks.
constexpr int kFrDecWords = 4 * 130;     // decode: <= 256 * (W+1)/W + 4 <= 516 source words

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Stage source words [B, B + 4*nv) (B a multiple of 4) into t; words past
// `limit` read as 0.
__device__ __forceinline__ void wave_stage(uint32_t *t, const uint32_t *src, uint64_t B, uint32_t nv,
                                           uint64_t limit, uint32_t lane) {
    for (uint32_t v = lane; v < nv; v += 64) {
        const uint64_t wi = B + 4 * (uint64_t)v;
        u32x4 x;
        if (wi + 4 <= limit) {
            x = __builtin_nontemporal_load((const u32x4 *)(src + wi));
        } else {
            x.x = wi < limit ? src[wi] : 0u; x.y = wi + 1 < limit ? src[wi + 1] : 0u;
            x.z = wi + 2 < limit ? src[wi + 2] : 0u; x.w = 0u;
        }
        *(u32x4 *)(t + 4 * v) = x;
    }
}

__global__ __launch_bounds__(256) void k_stream_framed_dec_lds(const StreamArgs a, uint64_t n,
                                                               uint32_t mark_le, double inv_w,
                                                               unsigned long long *errkey) {
    __shared__ uint8_t sops[kMaxWords];
    __shared__ __attribute__((aligned(16))) uint32_t sbuf[4][kFrDecWords];
    for (int t = threadIdx.x; t < (int)a.w; t += 256) sops[t] = a.ops[t];
    __syncthreads();
    const uint32_t W = a.w, Wt = a.w + 1, lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint64_t total = n * W;                           // native words
    const uint64_t g_first = ((uint64_t)blockIdx.x * 4 + wid) * 256;
    if (g_first >= total) return;
    uint64_t r0; uint32_t w0;
    divmod(g_first, W, inv_w, r0, w0);
    uint64_t g_last = g_first + 255;
    if (g_last >= total) g_last = total - 1;
    uint64_t rl; uint32_t wl;
    divmod(g_last, W, inv_w, rl, wl);
    const uint64_t B = (r0 * Wt + w0) & ~3ull;             // covers the first record's mark
    const uint64_t x_last = rl * Wt + 1 + wl;
    uint32_t *t = sbuf[wid];
    wave_stage(t, (const uint32_t *)a.src, B, (uint32_t)((x_last - B) / 4 + 1), n * Wt, lane);
    wave_lds_sync();
    const uint64_t g0 = g_first + 4 * (uint64_t)lane;
    if (g0 >= total) return;
    uint64_t r; uint32_t w;
    divmod(g0, W, inv_w, r, w);
    uint32_t o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (g0 + k >= total) { o[k] = 0; continue; }
        const uint64_t x = r * Wt + 1 + w - B;
        // first native word of record r: check its mark (RpcMessageParserTCP.java:63-99)
        if (w == 0 && t[x - 1] != mark_le) atomicMin(errkey, err_key(r, 0, XDRG_E_FRAME));
        o[k] = word_op(sops[w], t[x]);
        if (++w == W) { w = 0; ++r; }
    }
    uint8_t *dst = a.dst + g0 * 4;
    if (g0 + 4 <= total) {
        u32x4 ov; ov.x = o[0]; ov.y = o[1]; ov.z = o[2]; ov.w = o[3];
        __builtin_nontemporal_store(ov, (u32x4 *)dst);
    } else {
        for (uint64_t k = 0; g0 + k < total; ++k) ((uint32_t *)dst)[k] = o[k];
    }
}

// ---- lean kernels (default) ------------------------------------------------------
// A per-lane 64-bit double-reciprocal divmod and an LDS op-table read per
// word made the first direct kernels VALU-bound.  Here the
// division happens once per wave on uniform values (scalar unit); a lane
// only adds its 32-bit offset (4 * lane < 256 words) and splits it with a
// float reciprocal; schemas of plain int/uint/enum words (ALLB) skip the op
// table entirely.
__device__ __forceinline__ void split_small(uint32_t x, uint32_t d, float inv, uint32_t &q, uint32_t &r) {
    // x < 2^24: q = x / d, r = x % d
    q = (uint32_t)((float)x * inv);
    int32_t rr = (int32_t)(x - q * d);
    if (rr < 0) { --q; rr += (int32_t)d; }
    else if (rr >= (int32_t)d) { ++q; rr -= (int32_t)d; }
    r = (uint32_t)rr;
}

template <bool ALLB>
__global__ __launch_bounds__(256) void k_stream_framed_enc_lean(const StreamArgs a, uint64_t n, uint32_t mark_le) {
    __shared__ uint8_t sops[kMaxWords];
    if constexpr (!ALLB) {
        for (int t = threadIdx.x; t < (int)a.w; t += 256) sops[t] = a.ops[t];
        __syncthreads();
    }
    const uint32_t W = a.w, Wt = a.w + 1, lane = threadIdx.x & 63;
    const uint64_t total = n * Wt;                                   // XDR words
    const uint64_t gw = ((uint64_t)blockIdx.x * 256 + __builtin_amdgcn_readfirstlane(threadIdx.x & ~63u)) * 4;
    if (gw >= total) return;
    const uint64_t r0 = gw / Wt;                                     // wave-uniform
    const uint32_t j0 = (uint32_t)(gw - r0 * Wt);
    uint32_t q, j;
    split_small(j0 + 4 * lane, Wt, 1.0f / (float)Wt, q, j);
    const uint64_t g0 = gw + 4 * lane;
    if (g0 >= total) return;
    const uint64_t r = r0 + q;
    const uint64_t i0 = r * W + (j ? j - 1 : 0);                     // first native word used
    const uint64_t nin = n * W;
    const uint32_t *src = (const uint32_t *)a.src;
    uint32_t x0, x1, x2, x3;
    if (i0 + 4 <= nin) {
        const u32x4w v = __builtin_nontemporal_load((const u32x4w *)(src + i0));
        x0 = v.x; x1 = v.y; x2 = v.z; x3 = v.w;
    } else {
        x0 = i0 < nin ? src[i0] : 0u; x1 = i0 + 1 < nin ? src[i0 + 1] : 0u;
        x2 = i0 + 2 < nin ? src[i0 + 2] : 0u; x3 = 0u;
    }
    uint32_t o[4];
    uint32_t k = 0, w = j;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        if (w == 0) {
            o[t] = mark_le;                       // GrizzlyRpcTransport.java:103-110
        } else {
            const uint32_t x = k == 0 ? x0 : k == 1 ? x1 : k == 2 ? x2 : x3;
            o[t] = ALLB ? bswap32(x) : word_op(sops[w - 1], x);
            ++k;
        }
        if (++w == Wt) w = 0;
    }
    uint8_t *dst = a.dst + g0 * 4;
    if (g0 + 4 <= total) {
        u32x4 ov; ov.x = o[0]; ov.y = o[1]; ov.z = o[2]; ov.w = o[3];
        __builtin_nontemporal_store(ov, (u32x4 *)dst);
    } else {
        for (uint64_t t = 0; g0 + t < total; ++t) ((uint32_t *)dst)[t] = o[t];
    }
}

template <bool ALLB>
__global__ __launch_bounds__(256) void k_stream_framed_dec_lean(const StreamArgs a, uint64_t n, uint32_t mark_le,
                                                                unsigned long long *errkey) {
    __shared__ uint8_t sops[kMaxWords];
    if constexpr (!ALLB) {
        for (int t = threadIdx.x; t < (int)a.w; t += 256) sops[t] = a.ops[t];
        __syncthreads();
    }
    const uint32_t W = a.w, Wt = a.w + 1, lane = threadIdx.x & 63;
    const uint64_t total = n * W;                                    // native words
    const uint64_t gw = ((uint64_t)blockIdx.x * 256 + __builtin_amdgcn_readfirstlane(threadIdx.x & ~63u)) * 4;
    if (gw >= total) return;
    const uint64_t r0 = gw / W;
    const uint32_t w0 = (uint32_t)(gw - r0 * W);
    uint32_t q, w;
    split_small(w0 + 4 * lane, W, 1.0f / (float)W, q, w);
    const uint64_t n0 = gw + 4 * lane;
    if (n0 >= total) return;
    uint64_t r = r0 + q;
    const uint64_t x0i = r * Wt + 1 + w;                             // XDR word of native word n0
    const uint64_t nx = n * Wt;
    const uint32_t *src = (const uint32_t *)a.src;
    // the 4 native words span at most 5 XDR words (W >= 3: one mark at most)
    uint32_t y0, y1, y2, y3, y4;   // selects, not an indexed array (no scratch)
    if (x0i + 5 <= nx) {
        const u32x4w v = __builtin_nontemporal_load((const u32x4w *)(src + x0i));
        y0 = v.x; y1 = v.y; y2 = v.z; y3 = v.w;
        y4 = src[x0i + 4];
    } else {
        y0 = x0i < nx ? src[x0i] : 0u; y1 = x0i + 1 < nx ? src[x0i + 1] : 0u;
        y2 = x0i + 2 < nx ? src[x0i + 2] : 0u; y3 = x0i + 3 < nx ? src[x0i + 3] : 0u;
        y4 = x0i + 4 < nx ? src[x0i + 4] : 0u;
    }
    uint32_t o[4];
    uint32_t k = 0;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        if (n0 + t >= total) { o[t] = 0; continue; }
        if (w == 0) {   // first word of record r: check its mark (RpcMessageParserTCP.java:63-99)
            const uint32_t m = k == 0 ? src[x0i - 1] : pick5(y0, y1, y2, y3, y4, k - 1);
            if (m != mark_le) atomicMin(errkey, err_key(r, 0, XDRG_E_FRAME));
        }
        const uint32_t x = pick5(y0, y1, y2, y3, y4, k);
        o[t] = ALLB ? bswap32(x) : word_op(sops[w], x);
        ++k;
        if (++w == W) { w = 0; ++r; ++k; }   // skip the next record's mark
    }
    uint8_t *dst = a.dst + n0 * 4;
    if (n0 + 4 <= total) {
        u32x4 ov; ov.x = o[0]; ov.y = o[1]; ov.z = o[2]; ov.w = o[3];
        __builtin_nontemporal_store(ov, (u32x4 *)dst);
    } else {
        for (uint64_t t = 0; n0 + t < total; ++t) ((uint32_t *)dst)[t] = o[t];
    }
}

int launch_stream_framed(const StreamArgs &a, uint64_t n, uint32_t mark_le, bool decode,
                         unsigned long long *errkey, const Tuning &t, void *stream) {
    if (!n || !a.w) return hipSuccess;
    hipStream_t st = (hipStream_t)stream;
    // the lean decode kernel holds 5 source words per lane: 4 native words of
    // records of W < 3 words can span more (two marks), so those take the
    // wave-LDS variant (tuning key 14 = 1 forces it for every decode)
    if (decode && (t.framed == 1 || a.w < 3)) {
        const uint64_t words = n * a.w;
        const uint64_t blocks = (words + 1023) / 1024;     // 4 waves x 256 words
        hipLaunchKernelGGL(k_stream_framed_dec_lds, dim3(blocks), dim3(256), 0, st, a, n, mark_le,
                           1.0 / (double)a.w, errkey);
        return (int)hipGetLastError();
    }
    const uint64_t words = decode ? n * a.w : n * (a.w + 1);
    const uint64_t blocks = (((words + 3) >> 2) + 255) / 256;
    if (decode) {
        if (a.all_bswap)
            hipLaunchKernelGGL(k_stream_framed_dec_lean<true>, dim3(blocks), dim3(256), 0, st, a, n, mark_le, errkey);
        else
            hipLaunchKernelGGL(k_stream_framed_dec_lean<false>, dim3(blocks), dim3(256), 0, st, a, n, mark_le, errkey);
    } else {
        if (a.all_bswap)
            hipLaunchKernelGGL(k_stream_framed_enc_lean<true>, dim3(blocks), dim3(256), 0, st, a, n, mark_le);
        else
            hipLaunchKernelGGL(k_stream_framed_enc_lean<false>, dim3(blocks), dim3(256), 0, st, a, n, mark_le);
    }
    return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// Word-map kernels (any fixed layout).
// ---------------------------------------------------------------------------
struct WordMapShared {
    WordOp ops[kMaxWords];
    uint8_t *base[kMaxCols];
    int64_t stride[kMaxCols];
};

__device__ __forceinline__ void wordmap_stage(const WordMapArgs &a, WordMapShared &s) {
    for (int t = threadIdx.x; t < (int)a.nops; t += blockDim.x) s.ops[t] = a.ops[t];
    if (threadIdx.x < kMaxCols) {
        s.base[threadIdx.x] = a.base[threadIdx.x];
        s.stride[threadIdx.x] = a.stride[threadIdx.x];
    }
    __syncthreads();
}

// Encode one XDR word of record r (Xdr.java encoders, see WordOpKind).
__device__ __forceinline__ uint32_t enc_word(const WordMapShared &s, const WordOp o, uint64_t r,
                                             uint32_t mark) {
    if (o.op == OP_MARK) return mark;
    const uint8_t *p = s.base[o.col] + (int64_t)r * s.stride[o.col] + o.off;
    switch (o.op) {
    case OP_BSWAP: return bswap32(*(const uint32_t *)p);
    case OP_FLOAT: return bswap32(canon_f32(*(const uint32_t *)p));
    case OP_HYPER_HI: return bswap32(*(const uint32_t *)(p + 4));
    case OP_HYPER_LO: return bswap32(*(const uint32_t *)p);
    case OP_DOUBLE_HI:
    case OP_DOUBLE_LO: {
        uint32_t lo = *(const uint32_t *)p, hi = *(const uint32_t *)(p + 4);
        canon_f64(hi, lo);
        return bswap32(o.op == OP_DOUBLE_HI ? hi : lo);
    }
    case OP_BOOL: return *p ? 0x01000000u : 0u;
    case OP_SHORT: return bswap32((uint32_t)(int32_t)*(const int16_t *)p);
    case OP_BYTE: return bswap32((uint32_t)(int32_t)*(const int8_t *)p);
    case OP_OPAQUE: {
        uint32_t v = 0;
        for (uint32_t b = 0; b < o.aux; ++b) v |= (uint32_t)p[b] << (8 * b);
        return v;
    }
    default: return 0;
    }
}

// Decode one XDR word v of record r into its native column.
__device__ __forceinline__ void dec_word(const WordMapShared &s, const WordOp o, uint64_t r,
                                         uint32_t w, uint32_t v, const WordMapArgs &a) {
    if (o.op == OP_MARK) {
        if (v != a.mark_le) atomicMin(a.errkey, err_key(r, w, XDRG_E_FRAME));
        return;
    }
    uint8_t *p = s.base[o.col] + (int64_t)r * s.stride[o.col] + o.off;
    switch (o.op) {
    case OP_BSWAP:
    case OP_FLOAT:      // intBitsToFloat keeps the raw bits (Xdr.java:255-257)
    case OP_HYPER_LO:
    case OP_DOUBLE_LO: *(uint32_t *)p = bswap32(v); break;
    case OP_HYPER_HI:
    case OP_DOUBLE_HI: *(uint32_t *)(p + 4) = bswap32(v); break;
    case OP_BOOL: *p = v != 0; break;
    case OP_SHORT: *(uint16_t *)p = (uint16_t)bswap32(v); break;
    case OP_BYTE: *p = (uint8_t)bswap32(v); break;
    case OP_OPAQUE:
        for (uint32_t b = 0; b < o.aux; ++b) p[b] = (uint8_t)(v >> (8 * b));
        break;
    default: break;
    }
}

template <bool A16>
__global__ __launch_bounds__(256) void k_wordmap_encode(const WordMapArgs a) {
    __shared__ WordMapShared s;
    wordmap_stage(a, s);
    const uint64_t total = a.n * a.wt;
    const uint64_t nchunks = (total + 3) >> 2;
    const uint64_t S = (uint64_t)gridDim.x * blockDim.x;
    uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= nchunks) return;
    uint64_t r = (c * 4) / a.wt;
    uint32_t w = (uint32_t)(c * 4 - r * a.wt);
    for (; c < nchunks; c += S) {
        uint32_t v[4];
        uint64_t rr = r;
        uint32_t ww = w;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            v[j] = rr < a.n ? enc_word(s, s.ops[ww], rr, a.mark_le) : 0u;
            if (++ww == a.wt) { ww = 0; ++rr; }
        }
        const uint64_t g = c * 4;
        if (A16 && g + 4 <= total) {
            u32x4 o; o.x = v[0]; o.y = v[1]; o.z = v[2]; o.w = v[3];
            *(u32x4 *)(a.xdr + g * 4) = o;
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (g + j < total) *(uint32_t *)(a.xdr + (g + j) * 4) = v[j];
        }
        r += a.dr; w += a.dw;
        if (w >= a.wt) { w -= a.wt; ++r; }
    }
}

template <bool A16>
__global__ __launch_bounds__(256) void k_wordmap_decode(const WordMapArgs a) {
    __shared__ WordMapShared s;
    wordmap_stage(a, s);
    const uint64_t total = a.n * a.wt;
    const uint64_t avail = a.xdr_len >> 2;  // whole words present in the input
    const uint64_t valid = total < avail ? total : avail;
    const uint64_t nchunks = (valid + 3) >> 2;
    const uint64_t S = (uint64_t)gridDim.x * blockDim.x;
    uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= nchunks) return;
    uint64_t r = (c * 4) / a.wt;
    uint32_t w = (uint32_t)(c * 4 - r * a.wt);
    for (; c < nchunks; c += S) {
        const uint64_t g = c * 4;
        uint32_t v[4];
        if (A16 && g + 4 <= valid) {
            const u32x4 x = *(const u32x4 *)(a.xdr + g * 4);
            v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                v[j] = g + j < valid ? *(const uint32_t *)(a.xdr + (g + j) * 4) : 0u;
        }
        uint64_t rr = r;
        uint32_t ww = w;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (g + j < valid) dec_word(s, s.ops[ww], rr, ww, v[j], a);
            if (++ww == a.wt) { ww = 0; ++rr; }
        }
        r += a.dr; w += a.dw;
        if (w >= a.wt) { w -= a.wt; ++r; }
    }
}

// ---------------------------------------------------------------------------
// Launchers.
// ---------------------------------------------------------------------------
static int g_num_cu = 0;
static int num_cu() {
    if (!g_num_cu) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&g_num_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            g_num_cu <= 0)
            g_num_cu = 256;
    }
    return g_num_cu;
}

static uint64_t grid_for(uint64_t work_items, uint64_t per_block, uint64_t max_blocks) {
    uint64_t b = (work_items + per_block - 1) / per_block;
    if (b > max_blocks) b = max_blocks;
    return b ? b : 1;
}

// Streaming kernels: one 16-byte vector per lane, one pass over the batch
// (no grid-stride loop), nontemporal loads and stores — the shape a sweep of
// unroll x nontemporal x grid chose on MI355X.
int launch_stream_words(const StreamArgs &a, void *stream) {
    if (!a.nvec) return hipSuccess;
    hipStream_t st = (hipStream_t)stream;
    if (a.all_bswap) {
        const uint64_t blocks = grid_for(a.nvec, 256, ~0ull);
        hipLaunchKernelGGL((k_stream_bswap<1, true, true>), dim3(blocks), dim3(256), 0, st,
                           (const u32x4 *)a.src, (u32x4 *)a.dst, a.nvec);
    } else {
        const uint64_t b4 = grid_for(a.nvec, 256 * 4, ~0ull);
        hipLaunchKernelGGL((k_stream_ops<4, true>), dim3(b4), dim3(256), 0, st, a);
    }
    return (int)hipGetLastError();
}

static void wordmap_grid(WordMapArgs &a, uint64_t words, uint64_t *blocks) {
    const uint64_t chunks = (words + 3) >> 2;
    *blocks = grid_for(chunks, 256, (uint64_t)num_cu() * 16);
    const uint64_t adv = *blocks * 256 * 4;  // words advanced per grid-stride step
    a.dr = adv / a.wt;
    a.dw = (uint32_t)(adv % a.wt);
}

int launch_wordmap_encode(const WordMapArgs &args, bool aligned16, void *stream) {
    WordMapArgs a = args;
    if (!a.n) return hipSuccess;
    uint64_t blocks;
    wordmap_grid(a, a.n * a.wt, &blocks);
    hipStream_t st = (hipStream_t)stream;
    if (aligned16) hipLaunchKernelGGL(k_wordmap_encode<true>, dim3(blocks), dim3(256), 0, st, a);
    else hipLaunchKernelGGL(k_wordmap_encode<false>, dim3(blocks), dim3(256), 0, st, a);
    return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// Lane-per-record word kernels: fixed schemas whose every XDR word is one
// 4-byte native word (int/uint/enum/float, hyper halves, 4-byte opaque runs)
// in any column layout — struct-of-arrays above all, the layout a Java
// BatchXdrEncoder fills (one direct buffer per field).  A lane owns a record:
// its native words are loads at uniform column bases (consecutive lanes,
// consecutive elements: coalesced per column), its XDR record one contiguous
// run written with 16-byte stores when records are 16-byte multiples.  The
// word table is read at compile-time positions (the loop over the record's
// words is unrolled), so no LDS and no per-word table lookup: the word-map
// kernels' per-word LDS reads, 64-bit address math and op switch made them
// VALU-bound (config 2 SoA: 1.11 / 0.96 ms vs 0.66 for the AoS stream).
// ---------------------------------------------------------------------------
constexpr int kLaneWords = 16;   // XDR words per record (incl. the mark) on these kernels

__device__ __forceinline__ void lane_op(const WordMapArgs &a, int w, uint32_t &op, uint32_t &col, uint32_t &off) {
    // the 8-byte WordOp as one aligned 64-bit kernel-argument load (no byte-wide
    // member read at its own address: the SMEM base hazard of DESIGN.md §8)
    const uint64_t raw = *(const uint64_t *)&a.ops[w];
    op = (uint32_t)(raw & 0xff);
    col = (uint32_t)((raw >> 8) & 0xff);
    off = (uint32_t)(raw >> 32) + (op == OP_HYPER_HI ? 4u : 0u);   // HI: native bytes [off+4, off+8)
}

__device__ __forceinline__ uint32_t lane_enc_word(const WordMapArgs &a, int w, uint64_t r) {
    uint32_t op, col, off;
    lane_op(a, w, op, col, off);
    if (op == OP_MARK) return a.mark_le;   // GrizzlyRpcTransport.java:103-110
    const uint32_t x = *(const uint32_t *)(a.base[col] + (int64_t)r * a.stride[col] + off);
    return op == OP_OPAQUE ? x : bswap32(op == OP_FLOAT ? canon_f32(x) : x);   // Xdr.java:545, :674
}

template <bool V16>
__global__ __launch_bounds__(256) void k_words_lane_enc(const WordMapArgs a) {
    const uint64_t r = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= a.n) return;
    const uint32_t wt = a.wt;
    uint32_t v[kLaneWords];
#pragma unroll
    for (int w = 0; w < kLaneWords; ++w)   // every load of the record in flight before the stores
        v[w] = (uint32_t)w < wt ? lane_enc_word(a, w, r) : 0u;
    uint8_t *dst = a.xdr + r * wt * 4;
    if (V16) {
#pragma unroll
        for (int q = 0; q < kLaneWords / 4; ++q)
            if ((uint32_t)(4 * q) < wt) {
                u32x4 o; o.x = v[4 * q]; o.y = v[4 * q + 1]; o.z = v[4 * q + 2]; o.w = v[4 * q + 3];
                __builtin_nontemporal_store(o, (u32x4 *)(dst + 16 * q));
            }
    } else {
#pragma unroll
        for (int w = 0; w < kLaneWords; ++w)
            if ((uint32_t)w < wt) *(uint32_t *)(dst + 4 * w) = v[w];
    }
}

template <bool V16>
__global__ __launch_bounds__(256) void k_words_lane_dec(const WordMapArgs a) {
    const uint64_t r = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint32_t wt = a.wt;
    // records wholly inside xdr_len; the first one that is not is the host's SHORT key
    if (r >= a.n || (r + 1) * wt * 4 > a.xdr_len) return;
    const uint8_t *src = a.xdr + r * wt * 4;
    uint32_t v[kLaneWords];
    if (V16) {
#pragma unroll
        for (int q = 0; q < kLaneWords / 4; ++q)
            if ((uint32_t)(4 * q) < wt) {
                const u32x4 x = __builtin_nontemporal_load((const u32x4 *)(src + 16 * q));
                v[4 * q] = x.x; v[4 * q + 1] = x.y; v[4 * q + 2] = x.z; v[4 * q + 3] = x.w;
            }
    } else {
#pragma unroll
        for (int w = 0; w < kLaneWords; ++w)
            v[w] = (uint32_t)w < wt ? *(const uint32_t *)(src + 4 * w) : 0u;
    }
#pragma unroll
    for (int w = 0; w < kLaneWords; ++w) {
        if ((uint32_t)w >= wt) continue;
        uint32_t op, col, off;
        lane_op(a, w, op, col, off);
        if (op == OP_MARK) {   // RpcMessageParserTCP.java:63-99
            if (v[w] != a.mark_le) atomicMin(a.errkey, err_key(r, (uint32_t)w, XDRG_E_FRAME));
            continue;
        }
        // decode keeps raw float bits (Xdr.java:255-257); opaque bytes as they are
        *(uint32_t *)(a.base[col] + (int64_t)r * a.stride[col] + off) = op == OP_OPAQUE ? v[w] : bswap32(v[w]);
    }
}

// LDS-staged form of the lane kernels: the block's 256 records sit in LDS as
// rows of kRowPad (odd) words, so a lane's row writes / reads hit distinct
// banks, and the block's XDR span — contiguous, 16-byte aligned because it
// starts at record 256*blockIdx.x of a 16-byte-aligned stream — moves as
// coalesced 16-byte accesses whatever the record size (the lane kernels' own
// record stores stride wt*4 bytes per lane: 9-word framed records took
// scalar stores, 1.95 ms on config 2).
constexpr int kRowPad = kLaneWords + 1;

__device__ __forceinline__ uint32_t lds_word(const uint32_t *t, uint32_t j, uint32_t wt) {
    const uint32_t rr = j / wt;
    return t[rr * kRowPad + (j - rr * wt)];
}

// Column side, for both directions: quad q of the block is word w = q / 64 of
// records 4*(q % 64) .. +3 — w is wave-uniform, so its WordOp is a scalar
// load and a dense 4-byte column (stride 4, 16-byte aligned run) moves as one
// 16-byte access per lane; other strides take four 4-byte accesses.
__device__ __forceinline__ void wave_op(const WordMapArgs &a, uint32_t w, uint32_t &op, uint32_t &col, uint32_t &off) {
    const uint64_t raw = *(const uint64_t *)&a.ops[__builtin_amdgcn_readfirstlane(w)];
    op = (uint32_t)(raw & 0xff);
    col = (uint32_t)((raw >> 8) & 0xff);
    off = (uint32_t)(raw >> 32) + (op == OP_HYPER_HI ? 4u : 0u);
}

__device__ __forceinline__ uint32_t enc_xform(uint32_t op, uint32_t x) {
    return op == OP_OPAQUE ? x : bswap32(op == OP_FLOAT ? canon_f32(x) : x);   // Xdr.java:545, :674
}

__global__ __launch_bounds__(256) void k_words_lds_enc(const WordMapArgs a) {
    __shared__ uint32_t t[256 * kRowPad];
    const uint64_t r0 = (uint64_t)blockIdx.x * 256;
    const uint32_t wt = a.wt;
    const uint32_t nr = (uint32_t)min<uint64_t>(256, a.n - r0);
    for (uint32_t q = threadIdx.x; q < 64 * wt; q += 256) {
        const uint32_t w = q >> 6, i = 4 * (q & 63);
        uint32_t op, col, off;
        wave_op(a, w, op, col, off);
        uint32_t *row = t + i * kRowPad + w;
        if (op == OP_MARK) {   // GrizzlyRpcTransport.java:103-110
            row[0] = row[kRowPad] = row[2 * kRowPad] = row[3 * kRowPad] = a.mark_le;
            continue;
        }
        const int64_t st = a.stride[col];
        const uint8_t *p = a.base[col] + (int64_t)(r0 + i) * st + off;
        if (i + 4 <= nr && st == 4 && ((uintptr_t)p & 15) == 0) {
            const u32x4 x = __builtin_nontemporal_load((const u32x4 *)p);
            row[0] = enc_xform(op, x.x); row[kRowPad] = enc_xform(op, x.y);
            row[2 * kRowPad] = enc_xform(op, x.z); row[3 * kRowPad] = enc_xform(op, x.w);
        } else {
            for (uint32_t k = 0; k < 4 && i + k < nr; ++k) row[k * kRowPad] = enc_xform(op, *(const uint32_t *)(p + k * st));
        }
    }
    __syncthreads();
    const uint32_t words = nr * wt, quads = words >> 2;
    uint8_t *dst = a.xdr + r0 * wt * 4;
    for (uint32_t q = threadIdx.x; q < quads; q += 256) {
        u32x4 o;
        o.x = lds_word(t, 4 * q, wt); o.y = lds_word(t, 4 * q + 1, wt);
        o.z = lds_word(t, 4 * q + 2, wt); o.w = lds_word(t, 4 * q + 3, wt);
        __builtin_nontemporal_store(o, (u32x4 *)(dst + 16 * q));
    }
    for (uint32_t j = 4 * quads + threadIdx.x; j < words; j += 256) *(uint32_t *)(dst + 4 * j) = lds_word(t, j, wt);
}

__global__ __launch_bounds__(256) void k_words_lds_dec(const WordMapArgs a) {
    __shared__ uint32_t t[256 * kRowPad];
    const uint64_t r0 = (uint64_t)blockIdx.x * 256;
    const uint32_t wt = a.wt;
    // records wholly inside xdr_len; the first one that is not is the host's SHORT key
    const uint64_t whole = a.xdr_len / ((uint64_t)wt * 4);
    const uint64_t lim = min<uint64_t>(a.n, whole);
    if (r0 >= lim) return;   // block-uniform
    const uint32_t nr = (uint32_t)min<uint64_t>(256, lim - r0);
    const uint32_t words = nr * wt, quads = words >> 2;
    const uint8_t *src = a.xdr + r0 * wt * 4;
    for (uint32_t q = threadIdx.x; q < quads; q += 256) {
        const u32x4 x = __builtin_nontemporal_load((const u32x4 *)(src + 16 * q));
        const uint32_t j = 4 * q;
        uint32_t rr = j / wt, c = j - rr * wt;
        t[rr * kRowPad + c] = x.x; if (++c == wt) { c = 0; ++rr; }
        t[rr * kRowPad + c] = x.y; if (++c == wt) { c = 0; ++rr; }
        t[rr * kRowPad + c] = x.z; if (++c == wt) { c = 0; ++rr; }
        t[rr * kRowPad + c] = x.w;
    }
    for (uint32_t j = 4 * quads + threadIdx.x; j < words; j += 256) {
        const uint32_t rr = j / wt;
        t[rr * kRowPad + (j - rr * wt)] = *(const uint32_t *)(src + 4 * j);
    }
    __syncthreads();
    for (uint32_t q = threadIdx.x; q < 64 * wt; q += 256) {
        const uint32_t w = q >> 6, i = 4 * (q & 63);
        if (i >= nr) continue;
        uint32_t op, col, off;
        wave_op(a, w, op, col, off);
        const uint32_t *row = t + i * kRowPad + w;
        if (op == OP_MARK) {   // RpcMessageParserTCP.java:63-99; the min key is the first bad record
            for (uint32_t k = 0; k < 4 && i + k < nr; ++k)
                if (row[k * kRowPad] != a.mark_le) {
                    atomicMin(a.errkey, err_key(r0 + i + k, w, XDRG_E_FRAME));
                    break;
                }
            continue;
        }
        // decode keeps raw float bits (Xdr.java:255-257); opaque bytes as they are
        const int64_t st = a.stride[col];
        uint8_t *p = a.base[col] + (int64_t)(r0 + i) * st + off;
        if (i + 4 <= nr && st == 4 && ((uintptr_t)p & 15) == 0) {
            u32x4 o;
            o.x = row[0]; o.y = row[kRowPad]; o.z = row[2 * kRowPad]; o.w = row[3 * kRowPad];
            if (op != OP_OPAQUE) { o.x = bswap32(o.x); o.y = bswap32(o.y); o.z = bswap32(o.z); o.w = bswap32(o.w); }
            __builtin_nontemporal_store(o, (u32x4 *)p);
        } else {
            for (uint32_t k = 0; k < 4 && i + k < nr; ++k) {
                const uint32_t v = row[k * kRowPad];
                *(uint32_t *)(p + k * st) = op == OP_OPAQUE ? v : bswap32(v);
            }
        }
    }
}

bool words_lane_ok(const WordOp *ops, uint32_t nops) {
    if (!nops || nops > (uint32_t)kLaneWords) return false;
    for (uint32_t w = 0; w < nops; ++w) {
        const uint8_t op = ops[w].op;
        if (op == OP_OPAQUE ? ops[w].aux != 4
                            : !(op == OP_BSWAP || op == OP_FLOAT || op == OP_HYPER_HI || op == OP_HYPER_LO ||
                                op == OP_MARK))
            return false;
    }
    return true;
}

int launch_words_lane(const WordMapArgs &a, bool decode, bool v16, const Tuning &t, void *stream) {
    if (!t.words) return -1;   // the caller falls back to the word-map kernels
    if (!a.n) return hipSuccess;
    hipStream_t st = (hipStream_t)stream;
    const dim3 grid((unsigned)((a.n + 255) / 256));
    if (t.words == 2 && ((uintptr_t)a.xdr & 15) == 0) {
        if (decode) hipLaunchKernelGGL(k_words_lds_dec, grid, dim3(256), 0, st, a);
        else hipLaunchKernelGGL(k_words_lds_enc, grid, dim3(256), 0, st, a);
        return (int)hipGetLastError();
    }
    if (decode) {
        if (v16) hipLaunchKernelGGL(k_words_lane_dec<true>, grid, dim3(256), 0, st, a);
        else hipLaunchKernelGGL(k_words_lane_dec<false>, grid, dim3(256), 0, st, a);
    } else {
        if (v16) hipLaunchKernelGGL(k_words_lane_enc<true>, grid, dim3(256), 0, st, a);
        else hipLaunchKernelGGL(k_words_lane_enc<false>, grid, dim3(256), 0, st, a);
    }
    return (int)hipGetLastError();
}

int launch_wordmap_decode(const WordMapArgs &args, bool aligned16, void *stream) {
    WordMapArgs a = args;
    const uint64_t total = a.n * a.wt, avail = a.xdr_len >> 2;
    const uint64_t valid = total < avail ? total : avail;
    if (!valid) return hipSuccess;
    uint64_t blocks;
    wordmap_grid(a, valid, &blocks);
    hipStream_t st = (hipStream_t)stream;
    if (aligned16) hipLaunchKernelGGL(k_wordmap_decode<true>, dim3(blocks), dim3(256), 0, st, a);
    else hipLaunchKernelGGL(k_wordmap_decode<false>, dim3(blocks), dim3(256), 0, st, a);
    return (int)hipGetLastError();
}

}  // namespace xdrg

namespace xdrg {

__global__ void k_iota(uint64_t *dst, uint64_t n, uint64_t stride) {
    const uint64_t S = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= n; i += S) dst[i] = i * stride;
}

int launch_iota(uint64_t *dst, uint64_t n, uint64_t stride, void *stream) {
    const uint64_t blocks = grid_for(n + 1, 256, (uint64_t)num_cu() * 8);
    hipLaunchKernelGGL(k_iota, dim3(blocks), dim3(256), 0, (hipStream_t)stream, dst, n, stride);
    return (int)hipGetLastError();
}

__global__ void k_finalize(const unsigned long long *errkey, unsigned long long extra, uint64_t n,
                           uint64_t *first_bad, int *err) {
    if (threadIdx.x || blockIdx.x) return;
    unsigned long long k = errkey ? *errkey : kNoError;
    if (extra < k) k = extra;
    if (first_bad) *first_bad = k == kNoError ? n : (uint64_t)(k >> 16);
    if (err) *err = k == kNoError ? 0 : (int)(k & 0xf);
}

int launch_finalize(const unsigned long long *errkey, unsigned long long extra_key, uint64_t n,
                    uint64_t *first_bad, int *err, void *stream) {
    hipLaunchKernelGGL(k_finalize, dim3(1), dim3(64), 0, (hipStream_t)stream, errkey, extra_key, n,
                       first_bad, err);
    return (int)hipGetLastError();
}

}  // namespace xdrg

namespace xdrg {
// out[0] |= 1 when some record extent of ro (n + 1 offsets) is not `stride`
// bytes; out[1] = ro[0].  Decides whether fixed-size records at explicit
// extents (a frame scan's offsets) can take the fixed-stride kernels.
__global__ void k_check_stride(const uint64_t *ro, uint64_t n, uint64_t stride, unsigned long long *out) {
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool bad = false;
    for (uint64_t i = tid; i < n; i += (uint64_t)gridDim.x * blockDim.x) bad |= ro[i + 1] - ro[i] != stride;
    if (__ballot(bad) && (threadIdx.x & 63) == 0) atomicOr(out, 1ull);
    if (tid == 0) out[1] = ro[0];
}
int launch_check_stride(const uint64_t *ro, uint64_t n, uint64_t stride, unsigned long long *out, void *stream) {
    const uint64_t blocks = grid_for(n, 256, (uint64_t)num_cu() * 8);
    hipLaunchKernelGGL(k_check_stride, dim3(blocks), dim3(256), 0, (hipStream_t)stream, ro, n, stride, out);
    return (int)hipGetLastError();
}

__global__ void k_store_u64(uint64_t *dst, uint64_t v) {
    if (threadIdx.x == 0 && blockIdx.x == 0) *dst = v;
}
int launch_store_u64(uint64_t *dst, uint64_t value, void *stream) {
    hipLaunchKernelGGL(k_store_u64, dim3(1), dim3(64), 0, (hipStream_t)stream, dst, value);
    return (int)hipGetLastError();
}
}  // namespace xdrg
