// kernels_group.hip — repeated groups: arrays of structs and recursive
// lists (include/xdrg.h "Repeated groups").
//
// rpcgen encodes `T x<>` of a struct T as xdrEncodeInt(x.length) and then
// each element's fields, `T x[N]` without the count, and decodes with
// `new T[xdr.xdrDecodeInt()]` and no checkArraySize
// (oncrpc4j-rpcgen .../jrpcgen/jrpcgen.java:856-906).  A recursive list
// `T *x` (struct T { ...; T *next; }) is xdrEncodeBoolean(true) + element
// while there is one, then xdrEncodeBoolean(false) (INDIRECTION,
// jrpcgen.java:835-851; oncrpc4j-core portmap/pmaplist.java:50-69).
//
// Encode: k_grp_enc_sizes (a lane per record sums its fields, elements
// included) -> k_scan_rows -> k_grp_enc_place (a wave per record; elements
// of fixed size go a lane per element at computed positions, others a lane
// per element after a wave scan of their sizes).
// Decode: k_grp_dec_walk (a lane per record walks every count, list bool
// and member length in the reference's order and reports the first failing
// check) -> k_scan_rows over the counted columns -> k_grp_dec_offsets
// (native offsets, capacity) -> k_grp_dec_place (a lane per record walks
// it again and stores every value).
#include <hip/hip_runtime.h>

#include <type_traits>

#include "xdrg_device.h"
#include "xdrg_internal.h"

namespace xdrg {

// A field-table index every live lane of the wave holds (the walks step
// through the schema in lockstep; only the number of elements differs):
// said so to the compiler, the table is read with scalar loads instead of a
// vector load in every member's dependent chain.
__device__ __forceinline__ uint32_t g_uni(uint32_t k) { return __builtin_amdgcn_readfirstlane(k); }

typedef uint32_t u32g __attribute__((aligned(1)));
typedef uint32_t u32x4g __attribute__((ext_vector_type(4)));   // 16-byte aligned

__device__ __forceinline__ uint64_t g_dyn_bytes(const GField &f, uint64_t cnt) {
    return 4 + (f.xsz == 1 ? cnt + pad4(cnt) : cnt * f.xsz);
}
__device__ __forceinline__ uint32_t g_ld(const uint8_t *p) { return bswap32r(*(const uint32_t *)p); }

// Elements [e0, e0 + cnt) of group g in record r (DYNAMIC / LIST: its
// offsets; FIXED: r * count on).
__device__ __forceinline__ void g_range(const GField &g, uint64_t r, uint64_t &e0, uint64_t &cnt) {
    if (g.kind == XDRG_K_FIXED) {
        e0 = r * g.count;
        cnt = g.count;
    } else {
        e0 = g.offsets[r];
        cnt = g.offsets[r + 1] - e0;
    }
}

// XDR word w of fixed field f at row i (a record, or an element of a group).
__device__ __forceinline__ uint32_t g_fixed_word(const GField &f, uint64_t i, uint32_t w) {
    const uint8_t *base = f.data + (int64_t)i * f.stride;
    if (f.type == XDRG_T_OPAQUE) {   // bytes + zero pad (Xdr.java:776-781)
        const uint32_t rem = f.count - 4 * w;
        return load_bytes(base + 4 * w, rem < 4 ? rem : 4);
    }
    if (f.xsz == 8) return enc_elem(f.type, base + (uint64_t)(w >> 1) * 8, w & 1);
    return enc_elem(f.type, base + (uint64_t)w * f.nsz, 0);
}
__device__ __forceinline__ void g_fixed_store(const GField &f, uint64_t i, uint32_t w, uint32_t v) {
    uint8_t *base = f.data + (int64_t)i * f.stride;
    if (f.type == XDRG_T_OPAQUE) {   // pad skipped unchecked (Xdr.java:341-349)
        const uint32_t rem = f.count - 4 * w, kb = rem < 4 ? rem : 4;
        if (kb == 4) *(u32g *)(base + 4 * w) = v;
        else for (uint32_t b = 0; b < kb; ++b) base[4 * w + b] = (uint8_t)(v >> (8 * b));
        return;
    }
    if (f.xsz == 8) dec_elem(f.type, base + (uint64_t)(w >> 1) * 8, w & 1, v);
    else dec_elem(f.type, base + (uint64_t)w * f.nsz, 0, v);
}
// Payload word w (after the length word) of a dynamic field whose row owns
// elements [e0, e0 + cnt).
__device__ __forceinline__ uint32_t g_dyn_word(const GField &f, uint64_t e0, uint64_t cnt, uint64_t w) {
    if (f.xsz == 1) {
        const uint64_t b = 4 * w;
        const uint8_t *src = f.data + e0 + b;
        return cnt - b >= 4 ? *(const u32g *)src : load_bytes(src, (uint32_t)(cnt - b));
    }
    if (f.xsz == 8) return enc_elem(f.type, f.data + (e0 + (w >> 1)) * 8, (uint32_t)(w & 1));
    return enc_elem(f.type, f.data + (e0 + w) * f.nsz, 0);
}
__device__ __forceinline__ void g_dyn_store(const GField &f, uint64_t e0, uint64_t cnt, uint64_t w, uint32_t v) {
    if (f.xsz == 1) {
        const uint64_t b = 4 * w;
        uint8_t *dst = f.data + e0 + b;
        if (cnt - b >= 4) *(u32g *)dst = v;
        else for (uint64_t i = 0; i < cnt - b; ++i) dst[i] = (uint8_t)(v >> (8 * i));
        return;
    }
    if (f.xsz == 8) dec_elem(f.type, f.data + (e0 + (w >> 1)) * 8, (uint32_t)(w & 1), v);
    else dec_elem(f.type, f.data + (e0 + w) * f.nsz, 0, v);
}
// len payload bytes from the 4-aligned src (stream or LDS tile) to dst at any
// alignment: byte stores only for the head and tail of the destination,
// aligned dwords composed from two source words in between (g_dyn_store
// stored a byte-aligned dword per word, which the compiler splits into bytes).
__device__ __forceinline__ void g_dec_bytes(uint8_t *dst, const uint8_t *src, uint64_t len) {
    const uint32_t sh = (uint32_t)((uintptr_t)dst & 3);
    const uint32_t head = (4 - sh) & 3;   // bytes before dst's first aligned dword
    const uint32_t hb = head < len ? head : (uint32_t)len;
    if (hb) {
        const uint32_t w0 = *(const uint32_t *)src;
        for (uint32_t b = 0; b < hb; ++b) dst[b] = (uint8_t)(w0 >> (8 * b));
    }
    if (len <= head) return;
    const uint64_t body = (len - head) >> 2;   // whole aligned dwords
    uint32_t *da = (uint32_t *)(dst + head);
    const uint32_t *sw = (const uint32_t *)src;
    for (uint64_t k = 0; k < body; ++k) {   // source bytes [head + 4k, head + 4k + 4)
        const uint32_t lo = sw[k], hi = head ? sw[k + 1] : 0u;
        da[k] = head ? __builtin_amdgcn_alignbyte(hi, lo, head) : lo;
    }
    const uint64_t t0 = head + 4 * body;
    for (uint64_t b = t0; b < len; ++b) {   // tail bytes
        const uint32_t w = sw[b >> 2];
        dst[b] = (uint8_t)(w >> (8 * (b & 3)));
    }
}
__device__ __forceinline__ uint64_t g_dyn_words(const GField &f, uint64_t cnt) {
    return f.xsz == 1 ? (cnt + 3) >> 2 : cnt * (f.xsz >> 2);
}

// ---- conditions (unions / optional data) on their own level -------------------
// A field's presence follows its discriminant (an earlier field of the same
// level: top-level fields per record, a group's members per element), as the
// generated xdrEncode / xdrDecode switch on it (jrpcgen.java:1240-1340).
// pres: bit k = discriminant k present; v: discriminant values by slot
// (uniform slot indices, unrolled selects: no scratch).  ccid / cp: the last
// condition evaluated (GField::cneg >> 8, its class: fields whose conditions
// are the same test) and its result — the members of an optional struct or a
// union arm share one test, evaluated once per element; noting a
// discriminant forgets it.
struct GDisc {
    uint32_t pres;
    int32_t v[XDRG_MAX_DISC];
    uint32_t ccid, cp;
};
__device__ __forceinline__ int32_t gd_get(const GDisc &d, uint32_t slot) {
    int32_t r = 0;
#pragma unroll
    for (int j = 0; j < XDRG_MAX_DISC; ++j) r = slot == (uint32_t)j ? d.v[j] : r;
    return r;
}
__device__ __forceinline__ bool g_present(const GroupArgs &a, const GField &f, GDisc &d) {
    if (!f.cond) return true;
    const uint32_t cid = f.cneg >> 8;   // (wave-uniform: the field is)
    if (d.ccid == cid) return d.cp != 0;
    const uint32_t dk = f.cond - 1;
    bool p = false;
    if ((d.pres >> dk) & 1u) {
        const int32_t v = gd_get(d, a.f[dk].dslot - 1);
        bool in = false;
        for (uint32_t j = 0; j < f.cnum; ++j) in |= a.cvals[f.cfirst + j] == v;
        p = in != ((f.cneg & 1u) != 0);
    }
    d.ccid = cid;
    d.cp = p;
    return p;
}
// A discriminant's presence and value into d (only discriminants are read
// back: a condition names one, which has a value slot).
__device__ __forceinline__ void g_note(GDisc &d, uint32_t k, const GField &f, bool present, int32_t val) {
    if (f.dslot) {
        d.pres = present ? (d.pres | (1u << k)) : (d.pres & ~(1u << k));
#pragma unroll
        for (int j = 0; j < XDRG_MAX_DISC; ++j)
            if (f.dslot - 1 == (uint32_t)j) d.v[j] = present ? val : 0;
        d.ccid = 0;
    }
}
// A discriminant's value: from its native row (encode; bool as 0 / 1) or
// from the word about to be decoded (any non-zero bool is true, Xdr.java:404-407).
__device__ __forceinline__ int32_t g_enc_dval(const GField &f, uint64_t i) {
    const uint8_t *p = f.data + (int64_t)i * f.stride;
    return f.type == XDRG_T_BOOL ? (int32_t)(*p != 0) : *(const int32_t *)p;
}
__device__ __forceinline__ int32_t g_dec_dval(const GField &f, const uint8_t *in, uint64_t pos, uint64_t end) {
    if (end - pos < 4) return 0;   // the field's own check fails first
    const int32_t w = (int32_t)g_ld(in + pos);
    return f.type == XDRG_T_BOOL ? (int32_t)(w != 0) : w;
}
// Presence of field k on encode at row i (notes it into d).
__device__ __forceinline__ bool g_enc_field_present(const GroupArgs &a, uint32_t k, uint64_t i, GDisc &d) {
    const GField &f = a.f[k];
    if (!a.ncond) return true;
    const bool p = g_present(a, f, d);
    g_note(d, k, f, p, p && f.dslot ? g_enc_dval(f, i) : 0);
    return p;
}
__device__ __forceinline__ bool g_dec_field_present(const GroupArgs &a, uint32_t k, const uint8_t *in, uint64_t pos,
                                                    uint64_t end, GDisc &d) {
    const GField &f = a.f[k];
    if (!a.ncond) return true;
    const bool p = g_present(a, f, d);
    g_note(d, k, f, p, p && f.dslot ? g_dec_dval(f, in, pos, end) : 0);
    return p;
}

// XDR bytes of element e of group g (its list bool included).  L = the
// group's depth: an element at depth 0 may hold an inner array of structs /
// list (a member group), whose count word, elements and closing bool are the
// element's bytes too, as the element's generated xdrEncode writes them
// (jrpcgen.java:856-906, 835-851).
template <int L, int D>
__device__ __forceinline__ uint64_t g_group_bytes(const GroupArgs &a, uint32_t g, uint64_t row, GDisc &d);
template <int L, int D>
__device__ __forceinline__ uint64_t g_elem_bytes(const GroupArgs &a, uint32_t g, uint64_t e, GDisc d) {
    g = g_uni(g);
    const GField &G = a.f[g];
    if (!G.ncm && !G.ngm) {
        uint64_t s = G.efix;
        for (uint32_t j = 1; j <= G.nmem; ++j) {
            j = g_uni(j);
            const GField &m = a.f[g + j];
            if (m.kind == XDRG_K_DYNAMIC) s += g_dyn_bytes(m, m.offsets[e + 1] - m.offsets[e]);
        }
        return s;
    }
    uint64_t s = G.kind == XDRG_K_LIST ? 4 : 0;
    for (uint32_t j = 1; j <= G.nmem; ++j) {
        j = g_uni(j);
        const GField &m = a.f[g + j];
        const bool p = !G.ncm || g_enc_field_present(a, g + j, e, d);
        if (m.type == XDRG_T_GROUP) {
            if constexpr (L + 1 < D) {
                if (p) s += g_group_bytes<L + 1, D>(a, g + j, e, d);
            }
            j += m.nmem;
            continue;
        }
        if (m.kind != XDRG_K_DYNAMIC) {   // (a run of fixed members of one condition: at once)
            if (p) s += m.run ? m.run >> 8 : m.xbytes;
            j += m.run ? (m.run & 0xffu) - 1 : 0;
            continue;
        }
        if (p) s += g_dyn_bytes(m, m.offsets[e + 1] - m.offsets[e]);
    }
    return s;
}
// XDR bytes of group g at row `row` of its column (a record, or an element
// of the enclosing group): its count / closing bool and every element.
template <int L, int D>
__device__ __forceinline__ uint64_t g_group_bytes(const GroupArgs &a, uint32_t g, uint64_t row, GDisc &d) {
    g = g_uni(g);
    const GField &G = a.f[g];
    uint64_t e0, cnt;
    g_range(G, row, e0, cnt);
    uint64_t s = G.kind == XDRG_K_FIXED ? 0 : 4;   // the count, or a list's closing bool
    if (G.ndm && g + 1 == a.lay_g) {   // one layout: the fixed bytes, and each dynamic member's from its offsets
        s += cnt * (uint64_t)(G.efix + 4 * G.ndm);
        const uint64_t *o0 = a.f[a.slot_field[a.lay_s0 - 1]].offsets;
        const uint32_t z0 = a.lay_z0;
        uint64_t p0 = o0[e0];
        for (uint64_t e = e0; e < e0 + cnt; ++e) {
            const uint64_t q0 = o0[e + 1], c = q0 - p0;
            s += z0 == 1 ? c + pad4(c) : c * z0;
            p0 = q0;
        }
        if (G.ndm > 1) {
            const uint64_t *o1 = a.f[a.slot_field[a.lay_s1 - 1]].offsets;
            const uint32_t z1 = a.lay_z1;
            uint64_t p1 = o1[e0];
            for (uint64_t e = e0; e < e0 + cnt; ++e) {
                const uint64_t q1 = o1[e + 1], c = q1 - p1;
                s += z1 == 1 ? c + pad4(c) : c * z1;
                p1 = q1;
            }
        }
    } else if (G.ndm || G.ncm) {
        for (uint64_t e = e0; e < e0 + cnt; ++e) s += g_elem_bytes<L, D>(a, g, e, d);
    } else {
        s += cnt * G.efix;
    }
    return s;
}

// The kernels' GroupArgs (one by-value kernel argument, 4 KB).  The deepest
// instances (D = kGrpLevels) and the element-parallel kernels (g_kargs<
// kGrpLevels>) read it in place in the kernarg segment: their inlined code
// makes the compiler give the argument a private copy otherwise (4 KB of
// scratch per lane, a 4 KB copy per lane at entry).  The others keep the
// plain argument (no change in their code).
template <int D>
__device__ __forceinline__ const GroupArgs &g_kargs(const GroupArgs &a) {
    if constexpr (D > 2) return *(const GroupArgs *)__builtin_amdgcn_kernarg_segment_ptr();
    else return a;
}

// ===========================================================================
// Encode
// ===========================================================================
template <int D>
__device__ __forceinline__ uint64_t g_rec_size(const GroupArgs &a, uint64_t r) {
    uint64_t s = a.framed ? 4 : 0;
    GDisc d{};
    for (uint32_t k = 0; k < a.nf;) {
        k = g_uni(k);
        const GField &f = a.f[k];
        if (!g_enc_field_present(a, k, r, d)) {   // an absent field / array / list writes nothing
            k += f.type == XDRG_T_GROUP ? 1 + f.nmem : 1;
            continue;
        }
        if (f.type == XDRG_T_GROUP) {
            s += g_group_bytes<0, D>(a, k, r, d);
            k += 1 + f.nmem;
            continue;
        }
        s += f.kind == XDRG_K_DYNAMIC ? g_dyn_bytes(f, f.offsets[r + 1] - f.offsets[r]) : (uint64_t)f.xbytes;
        ++k;
    }
    return s;
}

// The walk (and the encode sizes pass) is a dependent chain of loads per
// record: kWalkSplit blocks share
// one scan block's kRecPerBlock records (fewer records per lane, more waves
// in flight), and add their totals into its block_sums entry (zeroed first).
// One record per lane (4) against four (1), decode / encode ms
// (`profiles/r04_groups/walk_split_ab.jsonl`): READDIRPLUS 1.40 -> 1.23 /
// 1.81 -> 1.67, chunk_map 3.04 -> 2.75 / 1.89 -> 1.77, volume_index 2.80 ->
// 2.67 / 1.77 -> 1.65, DUMP 1.13 -> 1.06, READDIR 2.33 -> 2.25 / 2.61 -> 2.49.
#ifndef XDRG_WALK_SPLIT
#define XDRG_WALK_SPLIT 4
#endif
constexpr int kWalkSplit = XDRG_WALK_SPLIT;
static_assert(kRecPerThread % kWalkSplit == 0, "records per lane");
template <int D>
__global__ __launch_bounds__(kRecThreads) void k_grp_enc_sizes(const GroupArgs a_) {
    const GroupArgs &a = g_kargs<D>(a_);
    constexpr int per = kRecPerThread / kWalkSplit;
    const uint64_t blk = blockIdx.x / kWalkSplit;
    const uint64_t r0 = blk * kRecPerBlock + (uint64_t)(blockIdx.x % kWalkSplit) * (kRecPerBlock / kWalkSplit) +
                        (uint64_t)threadIdx.x * per;
    uint64_t s = 0;
    for (int j = 0; j < per; ++j) {
        const uint64_t r = r0 + j;
        if (r >= a.n) break;
        const uint64_t z = g_rec_size<D>(a, r);
        a.rec_size[r] = z;
        s += z;
    }
    const uint64_t tot = block_sum(s);
    if (threadIdx.x == 0) {
        if (kWalkSplit == 1) a.block_sums[blk] = tot;
        else atomicAdd((unsigned long long *)&a.block_sums[blk], (unsigned long long)tot);
    }
}

// One lane writes element e of group g at byte p of out (the stream, or an
// LDS image of a sub-batch's stream bytes); returns its end.
template <int L, int D>
__device__ __forceinline__ uint64_t g_enc_group(const GroupArgs &a, uint8_t *out, uint32_t g, uint64_t row, uint64_t p,
                                                GDisc &d);
template <int L, int D>
__device__ __forceinline__ uint64_t g_enc_elem(const GroupArgs &a, uint8_t *out, uint32_t g, uint64_t e, uint64_t p,
                                               GDisc d) {
    g = g_uni(g);
    const GField &G = a.f[g];
    if (G.kind == XDRG_K_LIST) {   // xdrEncodeBoolean(true) (pmaplist.java:65-67)
        *(uint32_t *)(out + p) = bswap32r(1u);
        p += 4;
    }
    for (uint32_t j = 1; j <= G.nmem; ++j) {
        j = g_uni(j);
        const GField &m = a.f[g + j];
        const bool present = !G.ncm || g_enc_field_present(a, g + j, e, d);   // an element's absent arm
        if (m.type == XDRG_T_GROUP) {   // an inner array / list: this lane writes it whole
            if constexpr (L + 1 < D) {
                if (present) p = g_enc_group<L + 1, D>(a, out, g + j, e, p, d);
            }
            j += m.nmem;
            continue;
        }
        if (!present) continue;
        if (m.kind != XDRG_K_DYNAMIC) {
            for (uint32_t w = 0; w < m.xbytes >> 2; ++w) *(uint32_t *)(out + p + 4 * w) = g_fixed_word(m, e, w);
            p += m.xbytes;
            continue;
        }
        const uint64_t e0 = m.offsets[e], cnt = m.offsets[e + 1] - e0;
        *(uint32_t *)(out + p) = bswap32r((uint32_t)cnt);
        const uint64_t nw = g_dyn_words(m, cnt);
        for (uint64_t w = 0; w < nw; ++w) *(uint32_t *)(out + p + 4 + 4 * w) = g_dyn_word(m, e0, cnt, w);
        p += 4 + 4 * nw;
    }
    return p;
}
// Group g at row `row` of its column, by one lane from stream byte p.
template <int L, int D>
__device__ __forceinline__ uint64_t g_enc_group(const GroupArgs &a, uint8_t *out, uint32_t g, uint64_t row, uint64_t p,
                                                GDisc &d) {
    g = g_uni(g);
    const GField &G = a.f[g];
    uint64_t e0, cnt;
    g_range(G, row, e0, cnt);
    if (G.kind == XDRG_K_DYNAMIC) {   // xdrEncodeInt($size) (jrpcgen.java:866-876)
        *(uint32_t *)(out + p) = bswap32r((uint32_t)cnt);
        p += 4;
    }
    for (uint64_t e = e0; e < e0 + cnt; ++e) p = g_enc_elem<L, D>(a, out, g, e, p, d);
    if (G.kind == XDRG_K_LIST) {      // xdrEncodeBoolean(false)
        *(uint32_t *)(out + p) = 0;
        p += 4;
    }
    return p;
}

// G lanes (a wave or a part of one: G divides 64) write record r at stream
// byte pos; ln = the lane's index in its group.  Fixed-size elements go a lane
// per element at computed positions, others a lane per element after a
// G-lane scan of their sizes.  G = 64 kept a wave per record (round 2); most
// records hold a handful of elements, so a wave of 8-lane groups writes
// eight records at once (tuning key 32; DUMP encode 7.1 -> 2.0 ms, READDIR
// 8.7 -> 5.0, READDIRPLUS 9.0 -> 3.7).
template <uint32_t G>
__device__ __forceinline__ uint64_t g_incl_scan(uint64_t v, uint32_t ln) {
#pragma unroll
    for (uint32_t d = 1; d < G; d <<= 1) {
        const uint64_t t = __shfl_up(v, d, G);
        if (ln >= d) v += t;
    }
    return v;
}
template <uint32_t G, int D>
__device__ __forceinline__ void g_enc_record(const GroupArgs &a, uint64_t r, uint64_t pos, uint64_t size, uint32_t ln) {
    uint8_t *out = a.xdr;
    if (a.framed) {   // GrizzlyRpcTransport.java:103-110
        if (ln == 0) *(uint32_t *)(out + pos) = bswap32r((uint32_t)(size - 4) | kLastFrag);
        pos += 4;
    }
    GDisc d{};
    for (uint32_t k = 0; k < a.nf;) {
        k = g_uni(k);
        const GField &f = a.f[k];
        if (!g_enc_field_present(a, k, r, d)) {   // the record's absent arm / optional value
            k += f.type == XDRG_T_GROUP ? 1 + f.nmem : 1;
            continue;
        }
        if (f.type == XDRG_T_GROUP) {
            uint64_t e0, cnt;
            g_range(f, r, e0, cnt);
            if (f.kind == XDRG_K_DYNAMIC) {   // xdrEncodeInt($size) (jrpcgen.java:866-876)
                if (ln == 0) *(uint32_t *)(out + pos) = bswap32r((uint32_t)cnt);
                pos += 4;
            }
            if (!f.ndm && !f.ncm) {   // elements of one size: a lane per element
                for (uint64_t i = ln; i < cnt; i += G) g_enc_elem<0, D>(a, out, k, e0 + i, pos + i * f.efix, d);
                pos += cnt * f.efix;
            } else {        // a lane per element at its scanned position
                // (the group's lanes stay together: the scan's shuffles need all G)
                for (uint64_t b = 0; b < cnt; b += G) {
                    const uint64_t i = b + ln;
                    const uint64_t z = i < cnt ? g_elem_bytes<0, D>(a, k, e0 + i, d) : 0;
                    const uint64_t incl = g_incl_scan<G>(z, ln);
                    if (i < cnt) g_enc_elem<0, D>(a, out, k, e0 + i, pos + incl - z, d);
                    pos += __shfl(incl, G - 1, G);
                }
            }
            if (f.kind == XDRG_K_LIST) {   // xdrEncodeBoolean(false): the list ends
                if (ln == 0) *(uint32_t *)(out + pos) = 0;
                pos += 4;
            }
            k += 1 + f.nmem;
            continue;
        }
        if (f.kind != XDRG_K_DYNAMIC) {
            for (uint32_t w = ln; w < f.xbytes >> 2; w += G) *(uint32_t *)(out + pos + 4 * w) = g_fixed_word(f, r, w);
            pos += f.xbytes;
        } else {
            const uint64_t e0 = f.offsets[r], cnt = f.offsets[r + 1] - e0;
            if (ln == 0) *(uint32_t *)(out + pos) = bswap32r((uint32_t)cnt);
            const uint64_t nw = g_dyn_words(f, cnt);
            for (uint64_t w = ln; w < nw; w += G) *(uint32_t *)(out + pos + 4 + 4 * w) = g_dyn_word(f, e0, cnt, w);
            pos += 4 + 4 * nw;
        }
        ++k;
    }
}

template <uint32_t G, int D>
__global__ __launch_bounds__(kRecThreads) void k_grp_enc_place(const GroupArgs a_) {
    const GroupArgs &a = g_kargs<D>(a_);
    __shared__ uint64_t soff[kRecPerBlock + 1];
    const uint64_t total = a.totals[0];
    if (total > a.xdr_cap) return;   // XDRG_E_CAPACITY: write nothing
    const uint64_t rb = (uint64_t)blockIdx.x * kRecPerBlock;
    const uint32_t t0 = threadIdx.x * kRecPerThread;
    uint64_t sz[kRecPerThread], s = 0;
#pragma unroll
    for (int j = 0; j < kRecPerThread; ++j) {
        sz[j] = rb + t0 + j < a.n ? a.rec_size[rb + t0 + j] : 0;
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
    const uint64_t nrec = a.n - rb < (uint64_t)kRecPerBlock ? a.n - rb : (uint64_t)kRecPerBlock;
    // groups of G lanes take records in turn; a group past the end idles
    // through its last rounds (uniform loop bound: the scans' shuffles)
    const uint32_t ng = kRecThreads / G, ln = threadIdx.x & (G - 1);
    for (uint32_t j0 = 0; j0 < nrec; j0 += ng) {
        const uint32_t j = j0 + threadIdx.x / G;
        if (j < nrec) g_enc_record<G, D>(a, rb + j, soff[j], soff[j + 1] - soff[j], ln);
    }
}

// Element-parallel encode place (tuning key 41 = bytes of an LDS image of the
// output, 0: off) for schemas without conditional fields whose one top-level
// group has a layout (GroupArgs::lay_g).  The lane-group place above writes a
// record's elements from its own lanes as scattered dwords.  Here a sub-batch
// of records whose XDR fits the image is composed in LDS: every lane sizes
// elements (the layout and the dynamic members' offsets), a block scan places
// them, record lanes write the top-level fields, counts and list ends, every
// lane writes elements (consecutive lanes, consecutive elements), and the
// block copies the image out with 16-byte stores.  Same words as
// g_enc_record (jrpcgen.java:835-906 counts / list bools, Xdr.java:765-800).
constexpr uint32_t kEncElCap = 1024;   // elements per sub-batch
constexpr uint16_t kNoOwner = 0xffff;   // an element of a record whose group is absent
__host__ __device__ constexpr size_t enc_el_lds_bytes(uint32_t img) {
    return (size_t)(kRecPerBlock + 1) * 8 + (size_t)(kEncElCap + 1) * 4 + (size_t)kRecPerBlock * 4 +
           (size_t)kEncElCap * 2 + (size_t)(kRecPerBlock + 1) * 2 + 16 + img;
}
__device__ __forceinline__ void g_st_img(uint8_t *img, uint32_t p, uint32_t v) { *(uint32_t *)(img + p) = v; }
// XDR bytes of element e of the layout group g
__device__ __forceinline__ uint32_t g_lay_elem_bytes(const GroupArgs &a, const GField &G, uint64_t e) {
    uint64_t z = (G.kind == XDRG_K_LIST ? 4 : 0) + a.lay_pre;
    if (G.ndm > 0) {
        const GField &m0 = a.f[a.slot_field[a.lay_s0 - 1]];
        const uint64_t c0 = m0.offsets[e + 1] - m0.offsets[e];
        z += 4 + (a.lay_z0 == 1 ? c0 + pad4(c0) : c0 * a.lay_z0) + a.lay_mid;
        if (G.ndm > 1) {
            const GField &m1 = a.f[a.slot_field[a.lay_s1 - 1]];
            const uint64_t c1 = m1.offsets[e + 1] - m1.offsets[e];
            z += 4 + (a.lay_z1 == 1 ? c1 + pad4(c1) : c1 * a.lay_z1) + a.lay_post;
        }
    }
    return (uint32_t)z;
}
// Element e of group g into the image at p (its list bool, then every member)
template <bool COND>
__device__ __forceinline__ void g_enc_elem_img(const GroupArgs &a, uint32_t g, uint64_t e, uint8_t *img, uint32_t p) {
    g = g_uni(g);
    const GField &G = a.f[g];
    if (G.kind == XDRG_K_LIST) {   // xdrEncodeBoolean(true) (pmaplist.java:65-67)
        g_st_img(img, p, bswap32r(1u));
        p += 4;
    }
    GDisc d{};   // (a member's condition names an earlier member of its element)
    for (uint32_t j = 1; j <= G.nmem; ++j) {
        j = g_uni(j);
        const GField &m = a.f[g + j];
        if (COND && G.ncm && !g_enc_field_present(a, g + j, e, d)) continue;   // an element's absent arm
        if (m.kind != XDRG_K_DYNAMIC) {
            for (uint32_t w = 0; w < m.xbytes >> 2; ++w) g_st_img(img, p + 4 * w, g_fixed_word(m, e, w));
            p += m.xbytes;
            continue;
        }
        const uint64_t e0 = m.offsets[e], cnt = m.offsets[e + 1] - e0;
        g_st_img(img, p, bswap32r((uint32_t)cnt));
        const uint32_t nw = (uint32_t)g_dyn_words(m, cnt);
        for (uint32_t w = 0; w < nw; ++w) g_st_img(img, p + 4 + 4 * w, g_dyn_word(m, e0, cnt, w));
        p += 4 + 4 * nw;
    }
}
// Record r's own words into the image at p (its mark, top-level fields, the
// group's count and list end); returns the image offset of its first element
// (its elements take gbytes there).
template <bool COND>
__device__ __forceinline__ uint32_t g_enc_top_img(const GroupArgs &a, uint64_t r, uint8_t *img, uint32_t p,
                                                  uint64_t size, uint32_t gbytes) {
    uint32_t first = p;
    if (a.framed) {   // GrizzlyRpcTransport.java:103-110
        g_st_img(img, p, bswap32r((uint32_t)(size - 4) | kLastFrag));
        p += 4;
    }
    GDisc d{};
    for (uint32_t k = 0; k < a.nf;) {
        k = g_uni(k);
        const GField &f = a.f[k];
        if (COND && !g_enc_field_present(a, k, r, d)) {   // the record's absent arm / optional value
            k += f.type == XDRG_T_GROUP ? 1 + f.nmem : 1;
            continue;
        }
        if (f.type == XDRG_T_GROUP) {
            uint64_t e0, cnt;
            g_range(f, r, e0, cnt);
            if (f.kind == XDRG_K_DYNAMIC) {   // xdrEncodeInt($size) (jrpcgen.java:866-876)
                g_st_img(img, p, bswap32r((uint32_t)cnt));
                p += 4;
            }
            first = p;
            p += gbytes;
            if (f.kind == XDRG_K_LIST) {   // xdrEncodeBoolean(false): the list ends
                g_st_img(img, p, 0u);
                p += 4;
            }
            k += 1 + f.nmem;
            continue;
        }
        if (f.kind != XDRG_K_DYNAMIC) {
            for (uint32_t w = 0; w < f.xbytes >> 2; ++w) g_st_img(img, p + 4 * w, g_fixed_word(f, r, w));
            p += f.xbytes;
        } else {
            const uint64_t e0 = f.offsets[r], cnt = f.offsets[r + 1] - e0;
            g_st_img(img, p, bswap32r((uint32_t)cnt));
            const uint32_t nw = (uint32_t)g_dyn_words(f, cnt);
            for (uint32_t w = 0; w < nw; ++w) g_st_img(img, p + 4 + 4 * w, g_dyn_word(f, e0, cnt, w));
            p += 4 + 4 * nw;
        }
        ++k;
    }
    return first;
}
// Small batches: gridDim.x / nblocks (1, 2 or 4, enc_el_split) blocks share a
// scan block's records; each scans all of its sizes (the offsets need them)
// and composes its own share.  512 Ki READDIRPLUS replies are 512 scan
// blocks, two per CU: two blocks per scan block take their encode place from
// 1.68 to 1.11 ms; batches of 1,024 scan blocks and more lose 1-3 % when split
// (`profiles/r04_groups/enc_el_split_ab.jsonl`), so they are not.
__host__ __device__ inline uint32_t enc_el_split(uint64_t nblocks) { return nblocks >= 1024 ? 1u : nblocks >= 512 ? 2u : 4u; }
// D > 1: the group's elements hold inner groups (their sizes and words by the
// recursive element functions, into the image as into the stream).
template <bool COND, bool SHARE, int D>   // COND: the schema has conditional fields; SHARE: split > 1
__global__ __launch_bounds__(kRecThreads) void k_grp_enc_place_el(const GroupArgs a_) {
    const GroupArgs &a = g_kargs<kGrpLevels>(a_);
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint64_t *soff = (uint64_t *)smem;                       // [RPB + 1] record offsets in the stream
    uint32_t *xs = (uint32_t *)(soff + kRecPerBlock + 1);    // [cap + 1] element offsets in the sub-batch's elements
    uint32_t *rst = xs + kEncElCap + 1;                      // [RPB] image offset of a record's first element
    uint16_t *own = (uint16_t *)(rst + kRecPerBlock);        // [cap] an element's record (sub-batch index)
    uint16_t *fj = own + kEncElCap;                          // [RPB + 1] a record's first element (sub-batch index)
    uint8_t *img = smem + ((enc_el_lds_bytes(0) - 16 + 15) & ~(size_t)15);
    const uint64_t total = a.totals[0];
    if (total > a.xdr_cap) return;   // XDRG_E_CAPACITY: write nothing
    const uint32_t split = SHARE ? gridDim.x / (uint32_t)a.nblocks : 1u, kShare = kRecPerBlock / split;
    const uint64_t blk = blockIdx.x / split, q = blockIdx.x % split;
    const uint64_t rb0 = blk * kRecPerBlock;
    const uint32_t tid = threadIdx.x, t0 = tid * kRecPerThread;
    uint64_t sz[kRecPerThread], s = 0;
#pragma unroll
    for (int j = 0; j < kRecPerThread; ++j) {
        sz[j] = rb0 + t0 + j < a.n ? a.rec_size[rb0 + t0 + j] : 0;
        s += sz[j];
    }
    uint64_t btot;
    uint64_t off = a.block_sums[blk] + block_excl_scan(s, &btot);
#pragma unroll
    for (int j = 0; j < kRecPerThread; ++j) {
        soff[t0 + j] = off;
        if (a.rec_out && rb0 + t0 + j < a.n && (t0 + j) / kShare == q) a.rec_out[rb0 + t0 + j] = off;
        off += sz[j];
    }
    if (tid == kRecThreads - 1) soff[kRecPerBlock] = off;
    if (a.rec_out && blockIdx.x == 0 && tid == 0) a.rec_out[a.n] = total;
    __syncthreads();
    // this block's share: records rb .. rb + nrec, offsets from soff[0]
    const uint64_t rb = rb0 + q * kShare;
    if (rb >= a.n) return;
    if (SHARE) soff += q * kShare;
    const uint32_t nrec = (uint32_t)(a.n - rb < (uint64_t)kShare ? a.n - rb : (uint64_t)kShare);
    const uint32_t g = a.el_g;
    const GField &G = a.f[g];
    const bool lay = a.lay_g == g + 1;   // (no conditional member: every element has the layout)
    auto gfirst = [&](uint32_t j) -> uint64_t {   // the group's first element of block record j (j <= nrec)
        const uint64_t r = rb + j;
        return G.kind == XDRG_K_FIXED ? r * G.count : G.offsets[r];
    };
    uint32_t js = 0;
    while (js < nrec) {
        // records [js, js + 1 + tid) fit iff their bytes and elements do (monotone)
        const uint32_t je1 = js + 1 + tid;
        bool fits = false;
        if (je1 <= nrec)
            fits = soff[je1] - soff[js] <= a.enc_img && gfirst(je1) - gfirst(js) <= kEncElCap;
        const uint32_t k1 = (uint32_t)__syncthreads_count(fits);
        if (k1 == 0) {   // one record larger than the image: wave 0 writes it to the stream
            if (tid < 64) g_enc_record<64, D>(a, rb + js, soff[js], soff[js + 1] - soff[js], tid);
            ++js;
            continue;
        }
        const uint32_t je = js + k1, m = k1;
        const uint64_t E0 = gfirst(js);
        const uint32_t nel = (uint32_t)(gfirst(je) - E0);
        // record lanes: the first element and the element owner map; an element
        // of a record whose group is absent (its arm / optional value not
        // taken) is owned by no record (kNoOwner) and writes nothing
        for (uint32_t t = tid; t < m; t += kRecThreads) {
            const uint32_t f0 = (uint32_t)(gfirst(js + t) - E0), f1 = (uint32_t)(gfirst(js + t + 1) - E0);
            bool gp = true;
            if (COND) {   // the top-level fields up to the group, for its condition
                GDisc d{};
                for (uint32_t k = 0; k <= g;) {
                    const GField &f = a.f[k];
                    const bool p = g_enc_field_present(a, k, rb + js + t, d);
                    if (k == g) { gp = p; break; }
                    k += f.type == XDRG_T_GROUP ? 1 + f.nmem : 1;
                }
            }
            fj[t] = (uint16_t)f0;
            for (uint32_t i = f0; i < f1; ++i) own[i] = gp ? (uint16_t)t : kNoOwner;
        }
        if (tid == 0) fj[m] = (uint16_t)nel;
        __syncthreads();
        // element sizes, four consecutive elements per lane, placed by a block scan
        uint32_t z[4], zs = 0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t i = 4 * tid + u;
            z[u] = 0;
            if (i < nel && own[i] != kNoOwner)
                z[u] = lay ? g_lay_elem_bytes(a, G, E0 + i) : (uint32_t)g_elem_bytes<0, D>(a, g, E0 + i, GDisc{});
            zs += z[u];
        }
        uint64_t ztot;
        uint32_t x = (uint32_t)block_excl_scan(zs, &ztot);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t i = 4 * tid + u;
            if (i < nel) xs[i] = x;
            x += z[u];
        }
        if (tid == 0) xs[nel] = (uint32_t)ztot;
        __syncthreads();
        // record lanes: their own words; the image starts at record js
        const uint64_t ib = soff[js];
        for (uint32_t t = tid; t < m; t += kRecThreads) {
            const uint32_t j = js + t;
            rst[t] = g_enc_top_img<COND>(a, rb + j, img, (uint32_t)(soff[j] - ib), soff[j + 1] - soff[j],
                                   xs[fj[t + 1]] - xs[fj[t]]);
        }
        __syncthreads();
        for (uint32_t i = tid; i < nel; i += kRecThreads) {
            const uint32_t t = own[i];
            if (t == kNoOwner) continue;
            if constexpr (D == 1) g_enc_elem_img<COND>(a, g, E0 + i, img, rst[t] + xs[i] - xs[fj[t]]);
            else (void)g_enc_elem<0, D>(a, img, g, E0 + i, rst[t] + xs[i] - xs[fj[t]], GDisc{});
        }
        __syncthreads();
        // the image out: dwords up to a 16-byte boundary, 16-byte stores, dwords
        const uint32_t nb = (uint32_t)(soff[je] - ib);
        uint8_t *dst = a.xdr + ib;   // (4-aligned: XDR words)
        const uint32_t head = (uint32_t)((16 - ((uintptr_t)dst & 15)) & 15) < nb ? (uint32_t)((16 - ((uintptr_t)dst & 15)) & 15) : nb;
        const uint32_t nchunk = (nb - head) >> 4;
        for (uint32_t i = tid; i < nchunk; i += kRecThreads) {
            const uint32_t *w = (const uint32_t *)(img + head + 16 * i);
            u32x4g o;
            o.x = w[0]; o.y = w[1]; o.z = w[2]; o.w = w[3];
            *(u32x4g *)(dst + head + 16 * i) = o;
        }
        const uint32_t tail0 = head + 16 * nchunk;
        if (tid < (head >> 2)) *(uint32_t *)(dst + 4 * tid) = *(const uint32_t *)(img + 4 * tid);
        if (tid < ((nb - tail0) >> 2)) *(uint32_t *)(dst + tail0 + 4 * tid) = *(const uint32_t *)(img + tail0 + 4 * tid);
        js = je;   // (the next fit's barrier ends the image's use)
    }
}

// ===========================================================================
// Decode
// ===========================================================================
struct GExtent { uint64_t a, b; };
__device__ __forceinline__ GExtent g_extent(const GroupArgs &a, uint64_t r) {
    GExtent e{a.rec_in[r], a.rec_in[r + 1]};
    if (e.b > a.xdr_cap) e.b = a.xdr_cap;
    if (e.a > e.b) e.a = e.b;
    return e;
}

// A dynamic field's length word at pos, then its payload: the reference's
// check order (Xdr.java:171-175 length, :374-383 / :392-401 len == 0 first,
// checkArraySize :1034-1037, ensureBytes :1028-1032).  Returns 0 or an error.
__device__ __forceinline__ uint32_t g_walk_dyn_z(uint32_t xsz, const uint8_t *in, uint64_t end, uint64_t &pos,
                                                 uint32_t &len_out) {
    if (end - pos < 4) return XDRG_E_SHORT;
    const int32_t len = (int32_t)g_ld(in + pos);
    pos += 4;
    uint64_t need;
    if (xsz == 1) {
        if (len == 0) { len_out = 0; return 0; }
        if (len < 0) return XDRG_E_CORRUPT;
        need = (uint64_t)len + pad4((uint64_t)len);
    } else {
        if (len < 0) return XDRG_E_CORRUPT;
        need = (uint64_t)len * xsz;
    }
    if (end - pos < need) return XDRG_E_SHORT;
    pos += need;
    len_out = (uint32_t)len;
    return 0;
}
__device__ __forceinline__ uint32_t g_walk_dyn(const GField &f, const uint8_t *in, uint64_t end, uint64_t &pos,
                                               uint32_t &len_out) {
    return g_walk_dyn_z(f.xsz, in, end, pos, len_out);
}

// Walk group g from pos (its count word or list bools and every element, each
// member's checks in the reference's order: jrpcgen.java:886-906 reads the
// count with no checkArraySize, so a negative one is NegativeArraySizeException;
// a list reads xdrDecodeBoolean() before every element, any non-zero = another,
// Xdr.java:404-407); cnt[s] += the counts of the counted columns it meets.
// L = depth: an element at depth 0 may hold an inner group, walked the same way.
// emap (the element-parallel place's group, GroupArgs::emap): a 1 at the
// stream word of every element start.
// The walk's per-slot counts: registers (slot-indexed selects) or an LDS
// column per lane (WCntL).  The LDS form frees 16 registers (walk<1> 125 ->
// 82 VGPRs, walk<2> 158 -> 99, walk<4> 222 -> 129): READDIRPLUS decode 0.864
// -> 0.833 ms, volume_index 2.25 -> 2.16; a schema with a layout group keeps
// registers (READDIR 2.22 vs 2.31 ms; profiles/r05_groups/walk_cnt_ab.jsonl).
struct WCntL {   // slot s of lane t at p[s * kRecThreads], p = base + t
    uint32_t *p;
    __device__ __forceinline__ uint32_t &operator[](uint32_t s) const { return p[s * kRecThreads]; }
};
struct WCntNull {   // counts nobody reads (a walk for the position only)
    uint32_t x;
    __device__ __forceinline__ uint32_t &operator[](uint32_t) { return x; }
};
template <int L, int D, class C>
__device__ __forceinline__ uint32_t g_walk_group(const GroupArgs &a, uint32_t g, const uint8_t *in, uint64_t end, uint64_t &pos,
                                 C &cnt, GDisc &d, uint8_t *emap = nullptr);
// The members of one element of group g (after a list element's TRUE), inner
// groups included: pos past it, cnt[s] += its counts of counted column s.
template <int L, int D, class C>
__device__ __forceinline__ uint32_t g_walk_elem(const GroupArgs &a, uint32_t g, const uint8_t *in, uint64_t end,
                                                uint64_t &pos, C &cnt, GDisc &d) {
    const GField &f = a.f[g];
    for (uint32_t j = 1; j <= f.nmem; ++j) {
        j = g_uni(j);
        const GField &m = a.f[g + j];
        const bool present = !f.ncm || g_dec_field_present(a, g + j, in, pos, end, d);
        if (m.type == XDRG_T_GROUP) {   // an inner array / list of this element
            if constexpr (L + 1 < D) {
                if (present) {
                    const uint32_t err = g_walk_group<L + 1, D, C>(a, g + j, in, end, pos, cnt, d);
                    if (err) return err;
                }
            }
            j += m.nmem;
            continue;
        }
        if (m.kind != XDRG_K_DYNAMIC) {   // (a run of fixed members of one condition: at once)
            const uint32_t nb = m.run ? m.run >> 8 : m.xbytes;
            j += m.run ? (m.run & 0xffu) - 1 : 0;
            if (!present) continue;
            if (end - pos < nb) return XDRG_E_SHORT;
            pos += nb;
        } else if (present) {
            uint32_t len = 0;
            const uint32_t err = g_walk_dyn(m, in, end, pos, len);
            if (err) return err;
            cnt[m.slot - 1] += len;
        }
    }
    return 0;
}
template <int L, int D, class C>
__device__ __forceinline__ uint32_t g_walk_group(const GroupArgs &a, uint32_t g, const uint8_t *in, uint64_t end, uint64_t &pos,
                                 C &cnt, GDisc &d, uint8_t *emap) {
    g = g_uni(g);
    const GField &f = a.f[g];
    uint64_t n;
    if (f.kind == XDRG_K_DYNAMIC) {   // int $size = xdr.xdrDecodeInt(); new T[$size]
        if (end - pos < 4) return XDRG_E_SHORT;
        const int32_t c = (int32_t)g_ld(in + pos);
        pos += 4;
        if (c < 0) return XDRG_E_NEG_SIZE;
        n = (uint64_t)c;
    } else {
        n = f.kind == XDRG_K_FIXED ? f.count : ~0ull;
    }
    if (!f.ndm && !f.ncm && f.kind != XDRG_K_LIST) {   // elements of one size
        if ((end - pos) / f.efix < n) return XDRG_E_SHORT;
        if (emap)
            for (uint64_t i = 0; i < n; ++i) emap[(pos + i * f.efix) >> 2] = 1;
        pos += n * f.efix;
    } else if (g + 1 == a.lay_g) {   // one layout: the same checks, member descriptors not read
        // (a run of fixed members is SHORT iff one of them is, with the same sub)
        const uint32_t pre = a.lay_pre, mid = a.lay_mid, post = a.lay_post, nd = f.ndm;
        uint64_t c0 = 0, c1 = 0, i = 0;
        for (;; ++i) {
            if (f.kind == XDRG_K_LIST) {   // xdrDecodeBoolean(): any non-zero = another
                if (end - pos < 4) return XDRG_E_SHORT;
                const uint32_t more = g_ld(in + pos);
                pos += 4;
                if (!more) break;
            } else if (i == n) {
                break;
            }
            if (emap) emap[pos >> 2] = 1;
            if (end - pos < pre) return XDRG_E_SHORT;
            pos += pre;
            if (nd > 0) {
                uint32_t len = 0;
                uint32_t err = g_walk_dyn_z(a.lay_z0, in, end, pos, len);
                if (err) return err;
                c0 += len;
                if (end - pos < mid) return XDRG_E_SHORT;
                pos += mid;
                if (nd > 1) {
                    err = g_walk_dyn_z(a.lay_z1, in, end, pos, len);
                    if (err) return err;
                    c1 += len;
                    if (end - pos < post) return XDRG_E_SHORT;
                    pos += post;
                }
            }
        }
        if (nd > 0) cnt[a.lay_s0 - 1] += (uint32_t)c0;
        if (nd > 1) cnt[a.lay_s1 - 1] += (uint32_t)c1;
        n = i;
    } else {
        uint64_t i = 0;
        for (;; ++i) {
            if (f.kind == XDRG_K_LIST) {   // xdrDecodeBoolean(): any non-zero = another
                if (end - pos < 4) return XDRG_E_SHORT;
                const uint32_t more = g_ld(in + pos);
                pos += 4;
                if (!more) break;
            } else if (i == n) {
                break;
            }
            if (emap) emap[pos >> 2] = 1;
            const uint32_t err = g_walk_elem<L, D, C>(a, g, in, end, pos, cnt, d);
            if (err) return err;
        }
        n = i;
    }
    if (f.slot) cnt[f.slot - 1] += (uint32_t)n;   // (an inner group: summed over the outer elements)
    return 0;
}

// Walk record r; cnt[s] = the record's count of counted column s.
template <int D, class C>
__device__ __forceinline__ uint32_t g_walk(const GroupArgs &a, uint64_t r, C &cnt, uint32_t *sub) {
    const GExtent e = g_extent(a, r);
    const uint8_t *in = a.xdr;
    uint64_t pos = e.a;
    *sub = 0;
    if (a.framed) {   // one single-fragment message per record (GrizzlyRpcTransport:103-110)
        if (e.b - pos < 4) return XDRG_E_SHORT;
        const uint32_t m = g_ld(in + pos);
        if (!(m & kLastFrag) || (uint64_t)(m & kSizeMask) != e.b - pos - 4) return XDRG_E_FRAME;
        pos += 4;
    }
    GDisc d{};
    for (uint32_t k = 0; k < a.nf;) {
        k = g_uni(k);   // (every live lane is at the same field: scalar field-table loads)
        const GField &f = a.f[k];
        *sub = 2 * k + 1;
        if (!g_dec_field_present(a, k, in, pos, e.b, d)) {   // absent: nothing on the wire
            k += f.type == XDRG_T_GROUP ? 1 + f.nmem : 1;
            continue;
        }
        if (f.type == XDRG_T_GROUP) {
            const uint32_t err = g_walk_group<0, D, C>(a, k, in, e.b, pos, cnt, d, k == a.el_g ? a.emap : nullptr);
            if (err) return err;
            k += 1 + f.nmem;
            continue;
        }
        if (f.kind != XDRG_K_DYNAMIC) {
            if (e.b - pos < f.xbytes) return XDRG_E_SHORT;   // ensureBytes (Xdr.java:1028-1032)
            pos += f.xbytes;
        } else {
            uint32_t len = 0;
            const uint32_t err = g_walk_dyn(f, in, e.b, pos, len);
            if (err) return err;
            cnt[f.slot - 1] = len;
        }
        ++k;
    }
    return 0;
}

template <int D, bool CL>   // CL: the counts in LDS (WCntL)
__global__ __launch_bounds__(kRecThreads) void k_grp_dec_walk(const GroupArgs a_) {
    const GroupArgs &a = g_kargs<D>(a_);
    constexpr int per = kRecPerThread / kWalkSplit;
    const uint64_t blk = blockIdx.x / kWalkSplit;
    const uint64_t r0 = blk * kRecPerBlock + (uint64_t)(blockIdx.x % kWalkSplit) * (kRecPerBlock / kWalkSplit) +
                        (uint64_t)threadIdx.x * per;
    uint64_t sums[kMaxSlots];
    for (uint32_t s = 0; s < a.nslot; ++s) sums[s] = 0;
    for (int j = 0; j < per; ++j) {
        const uint64_t r = r0 + j;
        if (r >= a.n) break;
        __shared__ uint32_t wcnt[CL ? kMaxSlots * kRecThreads : 1];
        typename std::conditional<CL, WCntL, uint32_t[kMaxSlots]>::type cnt;
        if constexpr (CL) cnt.p = wcnt + threadIdx.x;
        for (uint32_t s = 0; s < a.nslot; ++s) cnt[s] = 0;
        uint32_t sub;
        const uint32_t err = g_walk<D>(a, r, cnt, &sub);
        if (err) {
            atomicMin(a.errkey, err_key(r, sub, err));
            for (uint32_t s = 0; s < a.nslot; ++s) cnt[s] = 0;   // a failed record owns nothing
        }
        for (uint32_t s = 0; s < a.nslot; ++s) {
            a.rec_cnt[(uint64_t)s * a.n + r] = cnt[s];
            sums[s] += cnt[s];
        }
    }
    for (uint32_t s = 0; s < a.nslot; ++s) {
        const uint64_t tot = block_sum(sums[s]);
        if (threadIdx.x == 0) {
            if (kWalkSplit == 1) a.block_sums[(uint64_t)s * a.nblocks + blk] = tot;
            else atomicAdd((unsigned long long *)&a.block_sums[(uint64_t)s * a.nblocks + blk], (unsigned long long)tot);
        }
    }
}

// Elements of group g over the whole batch (the rows of its members'
// columns): a FIXED group multiplies its parent's rows, others have their
// column total; false when a level's total exceeds its capacity (the
// capacity error stands and no offsets[rows] entry is in bounds).
__device__ __forceinline__ bool g_batch_rows(const GroupArgs &a, uint32_t g, uint64_t &rows) {
    uint64_t mult = 1;
    for (;;) {
        const GField &G = a.f[g];
        if (G.kind != XDRG_K_FIXED) {
            const uint64_t t = a.totals[G.slot - 1];
            rows = t * mult;
            return t <= G.cap;
        }
        mult *= G.count;
        if (!G.grp) { rows = a.n * mult; return true; }
        g = G.grp - 1;
    }
}

// Native offsets of every counted column (the columns' offsets arrays for
// top-level fields and groups, rec_base for all), capacity per record.
__global__ __launch_bounds__(kRecThreads) void k_grp_dec_offsets(const GroupArgs a) {
    const uint64_t rb = (uint64_t)blockIdx.x * kRecPerBlock;
    const uint32_t t0 = threadIdx.x * kRecPerThread;
    for (uint32_t s = 0; s < a.nslot; ++s) {
        const uint32_t k = a.slot_field[s];
        const GField &f = a.f[k];
        uint32_t c[kRecPerThread];
        uint64_t sum = 0;
#pragma unroll
        for (int j = 0; j < kRecPerThread; ++j) {
            const uint64_t r = rb + t0 + j;
            c[j] = r < a.n ? a.rec_cnt[(uint64_t)s * a.n + r] : 0u;
            sum += c[j];
        }
        uint64_t btot;
        uint64_t off = a.block_sums[(uint64_t)s * a.nblocks + blockIdx.x] + block_excl_scan(sum, &btot);
#pragma unroll
        for (int j = 0; j < kRecPerThread; ++j) {
            const uint64_t r = rb + t0 + j;
            if (r < a.n) {
                a.rec_base[(uint64_t)s * a.n + r] = off;
                if (!f.grp) f.offsets[r] = off;   // members: per element, by the place kernel
                if (off + c[j] > f.cap) atomicMin(a.errkey, err_key(r, 2 * f.top + 2, XDRG_E_CAPACITY));
            }
            off += c[j];
        }
        if (blockIdx.x == 0 && threadIdx.x == 0) {   // offsets[rows] = the column's total
            uint64_t rows;
            if (!f.grp) {
                f.offsets[a.n] = a.totals[s];
            } else {
                // a member's first entry: record 0's place writes it, but a
                // batch whose record 0 fails places nothing (the staging ring
                // cuts batches anywhere, so that is any chunk's first record)
                f.offsets[0] = 0;
                if (a.totals[s] <= f.cap && g_batch_rows(a, f.grp - 1, rows)) f.offsets[rows] = a.totals[s];
            }
        }
    }
}

// One lane decodes record r (walked clean, capacity checked), field by
// field in stream order: a wave keeps 64 records' loads in flight instead of
// one record's chain of dependent length words.
// The defaults of a freshly constructed rpcgen object for an absent fixed
// field at row i: zeros.
__device__ __forceinline__ void g_zero_fixed(const GField &f, uint64_t i) {
    uint8_t *p = f.data + (int64_t)i * f.stride;
    const uint64_t nb = (uint64_t)f.nsz * (f.kind == XDRG_K_FIXED ? f.count : 1);
    for (uint64_t b = 0; b < nb; ++b) p[b] = 0;
}

// Running native offsets of the counted columns of one record's group, in
// registers (slot-indexed selects): reading back the offsets just stored made
// every element wait for the previous one's store (READDIR decode 9.5 ->
// DESIGN.md §5.7).
struct GRun {
    uint64_t v[kMaxSlots];
    __device__ __forceinline__ uint64_t get(uint32_t slot) const {   // slot = GField::slot (1-based)
        uint64_t x = 0;
#pragma unroll
        for (int q = 0; q < kMaxSlots; ++q) x = (uint32_t)q + 1 == slot ? v[q] : x;
        return x;
    }
    __device__ __forceinline__ void set(uint32_t slot, uint64_t x) {
#pragma unroll
        for (int q = 0; q < kMaxSlots; ++q) v[q] = (uint32_t)q + 1 == slot ? x : v[q];
    }
    __device__ __forceinline__ void zero(uint32_t = kMaxSlots) {
#pragma unroll
        for (int q = 0; q < kMaxSlots; ++q) v[q] = 0;
    }
};
// The same in LDS, a column per lane (slot q of lane t at v[q * kRecThreads],
// v = base + t), for the deepest instances (D > 2): their inlined levels left
// no registers for 16 running offsets and their selects (dec place 245-256
// VGPRs, one wave per SIMD).
// n: the columns behind v (k_grp_dec_place_eln reserves max(nslot, 1) of
// them, the NEST kernels' static array kMaxSlots); zero(n) clears the
// schema's nslot columns only.
struct GRunL {
    uint64_t *v;
    uint32_t n = kMaxSlots;
    __device__ __forceinline__ uint64_t get(uint32_t slot) const {
        XDRG_DCHECK(slot <= n);
        return slot ? v[(slot - 1) * kRecThreads] : 0;
    }
    __device__ __forceinline__ void set(uint32_t slot, uint64_t x) {
        XDRG_DCHECK(slot <= n);
        if (slot) v[(slot - 1) * kRecThreads] = x;
    }
    __device__ __forceinline__ void zero(uint32_t nslot) {
        XDRG_DCHECK(nslot <= kMaxSlots);
        n = nslot ? nslot : 1u;
        for (uint32_t q = 0; q < nslot; ++q) v[q * kRecThreads] = 0;
    }
};
#ifndef XDRG_RUN_LDS_D
#define XDRG_RUN_LDS_D 1   // instances deeper than this keep their running offsets in LDS
#endif
constexpr bool g_run_lds(int D) { return D > XDRG_RUN_LDS_D; }
template <int D>
using GRunOf = typename std::conditional<g_run_lds(D), GRunL, GRun>::type;
// The running offsets of an element of the one-level element-parallel place:
// its (at most two) dynamic members' slots and offsets, two compares instead
// of a 16-way select per access.
struct GRun2 {
    uint32_t s0, s1;
    uint64_t v0, v1;
    __device__ __forceinline__ uint64_t get(uint32_t slot) const { return slot == s0 ? v0 : slot == s1 ? v1 : 0; }
    __device__ __forceinline__ void set(uint32_t slot, uint64_t x) {   // (selects: kept in registers)
        v1 = slot == s1 && slot != s0 ? x : v1;
        v0 = slot == s0 ? x : v0;
    }
};
__device__ __forceinline__ void g_run_bind(GRun &, uint64_t *) {}
__device__ __forceinline__ void g_run_bind(GRunL &run, uint64_t *rl) { run.v = rl; }
constexpr uint32_t kRunLds = kMaxSlots * kRecThreads;   // GRunL words of a block
__device__ __forceinline__ uint64_t g_rec_base(const GroupArgs &a, uint32_t slot, uint64_t r) {
    return a.rec_base[(uint64_t)(slot - 1) * a.n + r];
}
// The first element (row of its members' columns) of group g for record r,
// inside top-level group k whose first element is e0.
__device__ __forceinline__ uint64_t g_first_row(const GroupArgs &a, uint32_t k, uint64_t e0, uint32_t g, uint64_t r) {
    uint64_t mult = 1;
    for (;;) {
        if (g == k) return e0 * mult;
        const GField &G = a.f[g];
        if (G.kind != XDRG_K_FIXED) return g_rec_base(a, G.slot, r) * mult;
        mult *= G.count;
        g = G.grp - 1;
    }
}
// Top-level group k at record r, first element e0: every counted column of
// its span starts at the record's base (a direct member at row e0, an inner
// group's member at its record's first inner element), and its first offsets
// entry is written (an empty record leaves the next record's entry the same).
template <class R>
__device__ __forceinline__ void g_run_init(const GroupArgs &a, uint32_t k, uint64_t r, uint64_t e0, R &run) {
    run.zero(a.nslot);
    const GField &f = a.f[k];
    for (uint32_t j = 1; j <= f.nmem; ++j) {
        j = g_uni(j);
        const GField &m = a.f[k + j];
        if (!m.slot) continue;
        const uint64_t b0 = g_rec_base(a, m.slot, r);
        run.set(m.slot, b0);
        // a member of an inner group: rows are that group's elements, whose
        // first for record r its parents give (counted ones from their
        // record base, a T x[N] as N times its parent's first row)
        const uint64_t row = m.grp == k + 1 ? e0 : g_first_row(a, k, e0, m.grp - 1, r);
        m.offsets[row] = b0;
    }
}

// Element e of group g with no bytes on the wire (an absent T x[N]'s N
// elements): fixed members zero, dynamic members and inner arrays empty.
template <int L, int D, class R>
__device__ __forceinline__ void g_absent_elem(const GroupArgs &a, uint32_t g, uint64_t e, R &run) {
    g = g_uni(g);
    const GField &G = a.f[g];
    for (uint32_t j = 1; j <= G.nmem; ++j) {
        j = g_uni(j);
        const GField &m = a.f[g + j];
        if (m.type == XDRG_T_GROUP) {
            if constexpr (L + 1 < D) {
                if (m.kind != XDRG_K_FIXED) m.offsets[e + 1] = run.get(m.slot);
                else for (uint64_t i = e * m.count; i < (e + 1) * m.count; ++i) g_absent_elem<L + 1, D>(a, g + j, i, run);
            }
            j += m.nmem;
            continue;
        }
        if (m.kind != XDRG_K_DYNAMIC) g_zero_fixed(m, e);
        else m.offsets[e + 1] = run.get(m.slot);
    }
}

template <int L, int D, class R>
__device__ __forceinline__ void g_dec_elem(const GroupArgs &a, uint32_t g, uint64_t e, const uint8_t *in, uint64_t &pos,
                           uint64_t end, GDisc &d, R &run);
// Inner group g (at depth L, a member of an element at depth L - 1) of outer
// element e: its count word or list bools, read as the walk checked them,
// then its elements.
template <int L, int D, class R>
__device__ __forceinline__ void g_dec_inner(const GroupArgs &a, uint32_t g, uint64_t e, const uint8_t *in,
                                            uint64_t &pos, uint64_t end, GDisc &d, R &run) {
    g = g_uni(g);
    const GField &G = a.f[g];
    const uint64_t i0 = G.kind == XDRG_K_FIXED ? e * G.count : run.get(G.slot);
    uint64_t n = G.count;
    if (G.kind == XDRG_K_DYNAMIC) {
        n = g_ld(in + pos);
        pos += 4;
    }
    uint64_t i = 0;
    for (;; ++i) {
        if (G.kind == XDRG_K_LIST) {
            const uint32_t more = g_ld(in + pos);
            pos += 4;
            if (!more) break;
        } else if (i == n) {
            break;
        }
        g_dec_elem<L, D>(a, g, i0 + i, in, pos, end, d, run);
    }
    if (G.kind != XDRG_K_FIXED) {
        G.offsets[e + 1] = i0 + i;
        run.set(G.slot, i0 + i);
    }
}

// The members of element e of group g (after a list element's TRUE).
template <int L, int D, class R>
__device__ __forceinline__ void g_dec_elem(const GroupArgs &a, uint32_t g, uint64_t e, const uint8_t *in, uint64_t &pos,
                           uint64_t end, GDisc &d, R &run) {
    g = g_uni(g);
    const GField &f = a.f[g];
    for (uint32_t j = 1; j <= f.nmem; ++j) {
        j = g_uni(j);
        const GField &m = a.f[g + j];
        const bool present = !f.ncm || g_dec_field_present(a, g + j, in, pos, end, d);   // an element's absent arm
        if (m.type == XDRG_T_GROUP) {
            if constexpr (L + 1 < D) {
                if (present) {
                    g_dec_inner<L + 1, D>(a, g + j, e, in, pos, end, d, run);
                } else if (m.kind != XDRG_K_FIXED) {
                    m.offsets[e + 1] = run.get(m.slot);
                } else {
                    for (uint64_t i = e * m.count; i < (e + 1) * m.count; ++i) g_absent_elem<L + 1, D>(a, g + j, i, run);
                }
            }
            j += m.nmem;
            continue;
        }
        if (m.kind != XDRG_K_DYNAMIC) {   // a run of fixed members of one condition: one test
            const uint32_t nr = m.run ? (m.run & 0xffu) : 1u;
            for (uint32_t q = 0; q < nr; ++q) {
                const GField &mq = a.f[g + j + q];
                if (!present) {
                    g_zero_fixed(mq, e);
                    continue;
                }
                for (uint32_t w = 0; w < mq.xbytes >> 2; ++w)
                    g_fixed_store(mq, e, w, *(const uint32_t *)(in + pos + 4 * w));
                pos += mq.xbytes;
            }
            j += nr - 1;
            continue;
        }
        const uint64_t v0 = run.get(m.slot);
        if (!present) {
            m.offsets[e + 1] = v0;
            continue;
        }
        const uint64_t len = g_ld(in + pos);
        m.offsets[e + 1] = v0 + len;
        run.set(m.slot, v0 + len);
        const uint64_t nw = g_dyn_words(m, len);
        if (m.xsz == 1) g_dec_bytes(m.data + v0, in + pos + 4, len);
        else for (uint64_t w = 0; w < nw; ++w) g_dyn_store(m, v0, len, w, *(const uint32_t *)(in + pos + 4 + 4 * w));
        pos += 4 + 4 * nw;
    }
}

// Element e's members parsed without storing (the element-parallel place's
// record walk): pos past the element, run past its dynamic members.
template <class R>
__device__ __forceinline__ void g_elem_skip(const GroupArgs &a, uint32_t g, const uint8_t *in, uint64_t &pos,
                                            uint64_t end, GDisc &d, R &run) {
    g = g_uni(g);
    const GField &f = a.f[g];
    if (!f.ndm && !f.ncm) {   // elements of one size (a list's TRUE is already past)
        pos += f.efix - (f.kind == XDRG_K_LIST ? 4 : 0);
        return;
    }
    for (uint32_t j = 1; j <= f.nmem; ++j) {
        j = g_uni(j);
        const GField &m = a.f[g + j];
        const bool present = !f.ncm || g_dec_field_present(a, g + j, in, pos, end, d);
        if (m.kind != XDRG_K_DYNAMIC) {   // (a run of fixed members of one condition: at once)
            const uint32_t nb = m.run ? m.run >> 8 : m.xbytes;
            j += m.run ? (m.run & 0xffu) - 1 : 0;
            if (present) pos += nb;
            continue;
        }
        if (!present) continue;
        const uint64_t len = g_ld(in + pos);
        run.set(m.slot, run.get(m.slot) + len);
        pos += 4 + 4 * g_dyn_words(m, len);
    }
}

#ifndef XDRG_EL_RUN2
#define XDRG_EL_RUN2 1   // the element decode's running offsets as GRun2 (0: the 16-slot GRun)
#endif
// Element-parallel place (tuning key 38): the element descriptors a record
// lane leaves for a sub-batch — element i (= e - E0) starts at tile offset
// pos[i], and dynamic member q (of at most 2) at native offset sb[q] +
// rel[q * cap + i].
struct GElDesc {   // (scalar members: an indexed array here went to scratch)
    uint32_t *pos, *rel;
    uint32_t cap;                 // descriptors per sub-batch
    uint64_t E0;                  // the sub-batch's first element
    uint32_t nm;                  // dynamic members
    uint32_t ms0, ms1;            // their slots
    uint32_t mk0, mk1;            // their field indices
    uint64_t sb0, sb1;            // their native offsets at E0
    const uint8_t *tile;
    uint64_t rb;                  // the block's first record; per block record j (LDS, prefetched):
    const uint64_t *mE;           //   the group's first element of record rb + j (j <= 256)
    const uint64_t *mb0, *mb1;    //   the dynamic members' native offsets at it
    // an element without conditional members as a layout (lay = 1): fixed
    // bytes pre, dynamic member 0 (XDR element size z0), fixed bytes mid,
    // member 1 (z1), fixed bytes post; the record walk then reads one length
    // word per dynamic member and no member descriptor
    uint32_t lay, pre, mid, post, z0, z1;
};
// XDR words of cnt elements of XDR size z (g_dyn_words by size alone)
__device__ __forceinline__ uint64_t g_dyn_words_z(uint32_t z, uint64_t cnt) {
    return z == 1 ? (cnt + 3) >> 2 : cnt * (z >> 2);
}
// The lengths of one element's (at most two) dynamic members, by slot: the
// run g_elem_skip advances when only the element's own lengths matter.
struct GLen2 {
    uint32_t s0, s1;
    uint64_t l0, l1;
    __device__ __forceinline__ uint64_t get(uint32_t slot) const { return slot == s0 ? l0 : slot == s1 ? l1 : 0; }
    __device__ __forceinline__ void set(uint32_t slot, uint64_t x) {
        if (slot == s0) l0 = x;
        else if (slot == s1) l1 = x;
    }
};
// Element at tile offset pos of the element-parallel group: pos past it and
// its dynamic members' lengths (LAY: the layout's one length word each).
template <bool LAY>
__device__ __forceinline__ void g_el_parse(const GroupArgs &a, const GElDesc &el, uint32_t g, const uint8_t *in,
                                           uint64_t &pos, uint64_t &l0, uint64_t &l1) {
    l0 = l1 = 0;
    if constexpr (LAY) {
        pos += el.pre;
        if (el.nm > 0) {
            l0 = g_ld(in + pos);
            pos += 4 + 4 * g_dyn_words_z(el.z0, l0) + el.mid;
            if (el.nm > 1) {
                l1 = g_ld(in + pos);
                pos += 4 + 4 * g_dyn_words_z(el.z1, l1) + el.post;
            }
        }
    } else {
        GLen2 len{el.ms0 ? el.ms0 : ~0u, el.ms1 ? el.ms1 : ~0u, 0, 0};
        GDisc d{};
        g_elem_skip(a, g, in, pos, ~0ull, d, len);
        l0 = len.l0;
        l1 = len.l1;
    }
}

// in: where stream offset x is read, in + (x - base) (the stream with base 0,
// or an LDS tile holding this record's bytes whose first byte is stream offset
// base: k_grp_dec_place_lds).  Positions are tile-relative so that no pointer
// into the tile ever lies below it: a generic (flat) access through a tile
// pointer moved below the tile's 32-bit LDS address wraps out of the LDS
// aperture (the place kernels' former tile + (uint32_t)(xb - a0) faulted so).
// EL (element-parallel place): the record's one group leaves descriptors in
// *el instead of decoding its elements (the block decodes them afterwards,
// a lane per element).
// rl: the lane's GRunL column (D > 2).
// MAP (with EL): the elements' positions and member offsets are already in
// *el (found from GroupArgs::emap); the record lane steps over its group
// from its last element's position.
template <int D, bool EL = false, bool MAP = false>
__device__ __forceinline__ void g_dec_record(const GroupArgs &a, uint64_t r, const uint8_t *in, uint64_t base = 0,
                                             const GElDesc &el = GElDesc{}, uint64_t *rl = nullptr) {
    const GExtent ex = g_extent(a, r);   // the extent the walk checked (clamped to in_len)
    const uint64_t end = ex.b - base;
    uint64_t pos = ex.a + (a.framed ? 4 : 0) - base;
    GDisc d{};
    for (uint32_t k = 0; k < a.nf;) {
        k = g_uni(k);
        const GField &f = a.f[k];
        if (!g_dec_field_present(a, k, in, pos, end, d)) {
            if (f.type != XDRG_T_GROUP) {
                if (f.kind != XDRG_K_DYNAMIC) g_zero_fixed(f, r);   // dynamic: count 0 (offsets kernel)
                ++k;
                continue;
            }
            if (f.kind == XDRG_K_FIXED) {   // an absent T x[N]: N zero / empty elements
                GRunOf<D> run;
                g_run_bind(run, rl);
                g_run_init(a, k, r, r * f.count, run);
                for (uint64_t e = r * f.count; e < (r + 1) * f.count; ++e) g_absent_elem<0, D>(a, k, e, run);
            }
            k += 1 + f.nmem;
            continue;
        }
        if (f.type == XDRG_T_GROUP) {
            uint64_t e0, cnt;
            GRunOf<D> run;
            g_run_bind(run, rl);
            if constexpr (EL) {   // the block's metadata, prefetched into LDS
                const uint32_t j = (uint32_t)(r - el.rb);
                e0 = el.mE[j];
                cnt = el.mE[j + 1] - e0;
                if constexpr (D > 1) {   // (k_grp_dec_place_eln) every counted column of the span
                    g_run_init(a, k, r, e0, run);
                } else {
                    run.zero();
                    if (el.nm > 0) { run.set(el.ms0, el.mb0[j]); a.f[el.mk0].offsets[e0] = el.mb0[j]; }
                    if (el.nm > 1) { run.set(el.ms1, el.mb1[j]); a.f[el.mk1].offsets[e0] = el.mb1[j]; }
                }
            } else {
                e0 = f.kind == XDRG_K_FIXED ? r * f.count : g_rec_base(a, f.slot, r);
                cnt = f.kind == XDRG_K_FIXED ? f.count : a.rec_cnt[(uint64_t)(f.slot - 1) * a.n + r];
                g_run_init(a, k, r, e0, run);
            }
            if (f.kind == XDRG_K_DYNAMIC) pos += 4;
            if constexpr (EL && MAP) {
                if (cnt) {   // past the last element (its TRUE is before its position)
                    pos = el.pos[e0 + cnt - 1 - el.E0];
                    if constexpr (D > 1) {   // inner groups included
                        WCntNull nc;
                        GDisc de{};
                        (void)g_walk_elem<0, D>(a, k, in, ~0ull, pos, nc, de);
                    } else {
                        uint64_t l0, l1;
                        if (el.lay) g_el_parse<true>(a, el, k, in, pos, l0, l1);
                        else g_el_parse<false>(a, el, k, in, pos, l0, l1);
                    }
                }
                if (f.kind == XDRG_K_LIST) pos += 4;   // its FALSE
                k += 1 + f.nmem;
                continue;
            }
            if constexpr (EL) {
                if (el.lay) {   // elements of a fixed layout: one length word per dynamic member
                    const uint32_t lb = f.kind == XDRG_K_LIST ? 4u : 0u;
                    uint64_t r0 = el.nm > 0 ? run.get(el.ms0) : 0, r1 = el.nm > 1 ? run.get(el.ms1) : 0;
                    for (uint64_t e = e0; e < e0 + cnt; ++e) {
                        pos += lb;   // a list's TRUE
                        const uint32_t i = (uint32_t)(e - el.E0);
                        el.pos[i] = (uint32_t)pos;   // (in is the tile)
                        pos += el.pre;
                        if (el.nm > 0) {
                            el.rel[i] = (uint32_t)(r0 - el.sb0);
                            const uint64_t len = g_ld(in + pos);
                            r0 += len;
                            pos += 4 + 4 * g_dyn_words_z(el.z0, len) + el.mid;
                            if (el.nm > 1) {
                                el.rel[el.cap + i] = (uint32_t)(r1 - el.sb1);
                                const uint64_t len1 = g_ld(in + pos);
                                r1 += len1;
                                pos += 4 + 4 * g_dyn_words_z(el.z1, len1) + el.post;
                            }
                        }
                    }
                    if (f.kind == XDRG_K_LIST) pos += 4;   // its FALSE
                    k += 1 + f.nmem;
                    continue;
                }
            }
            for (uint64_t e = e0; e < e0 + cnt; ++e) {
                if (f.kind == XDRG_K_LIST) pos += 4;   // its TRUE
                if constexpr (EL) {
                    const uint32_t i = (uint32_t)(e - el.E0);
                    el.pos[i] = (uint32_t)(in + pos - el.tile);
                    if (el.nm > 0) el.rel[i] = (uint32_t)(run.get(el.ms0) - el.sb0);
                    if (el.nm > 1) el.rel[el.cap + i] = (uint32_t)(run.get(el.ms1) - el.sb1);
                    g_elem_skip(a, k, in, pos, end, d, run);
                } else {
                    g_dec_elem<0, D>(a, k, e, in, pos, end, d, run);
                }
            }
            if (f.kind == XDRG_K_LIST) pos += 4;   // its FALSE
            k += 1 + f.nmem;
            continue;
        }
        if (f.kind != XDRG_K_DYNAMIC) {
            for (uint32_t w = 0; w < f.xbytes >> 2; ++w) g_fixed_store(f, r, w, *(const uint32_t *)(in + pos + 4 * w));
            pos += f.xbytes;
        } else {
            const uint64_t len = g_ld(in + pos);
            const uint64_t e0 = g_rec_base(a, f.slot, r);
            const uint64_t nw = g_dyn_words(f, len);
            if (f.xsz == 1) g_dec_bytes(f.data + e0, in + pos + 4, len);
            else for (uint64_t w = 0; w < nw; ++w) g_dyn_store(f, e0, len, w, *(const uint32_t *)(in + pos + 4 + 4 * w));
            pos += 4 + 4 * nw;
        }
        ++k;
    }
}

template <int D>
__global__ __launch_bounds__(kRecThreads) void k_grp_dec_place(const GroupArgs a_) {
    const GroupArgs &a = g_kargs<D>(a_);
    const unsigned long long key = *a.errkey;   // final: walk and capacity kernels ran before
    const uint64_t bad = key == kNoError ? a.n : (uint64_t)(key >> 16);
    const uint64_t r = (uint64_t)blockIdx.x * kRecThreads + threadIdx.x;
    __shared__ uint64_t runs[g_run_lds(D) ? kRunLds : 1];
    if (r < bad) g_dec_record<D>(a, r, a.xdr, 0, GElDesc{}, runs + threadIdx.x);
}

// nch 16-byte chunks from the 16-aligned global address a0 into the tile by
// LDS-DMA (global_load_lds_dwordx4: every load of the block in flight at once,
// no registers; a copy loop through registers waited one memory round trip
// per 4 KiB of tile).  A wave's 64 chunks land contiguously (the LDS address
// is wave-uniform base + 16 * lane).  Each wave waits for its own DMA before
// the caller's barrier: LDS-DMA retires on vmcnt, not lgkmcnt.
__device__ __forceinline__ void g_stage_tile(uint8_t *tile, uintptr_t a0, uint32_t nch) {
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t i0 = (threadIdx.x >> 6) * 64; i0 < nch; i0 += kRecThreads) {
        if (i0 + lane < nch)
            __builtin_amdgcn_global_load_lds((const void *)(a0 + 16 * (uintptr_t)(i0 + lane)),
                                             (__attribute__((address_space(3))) void *)(tile + 16 * (size_t)i0), 16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Staged place (tuning key 33): the block's records go through an LDS tile in
// sub-batches [js, je) whose stream bytes fit it (16-byte aligned, coalesced
// 16-B loads), and each lane decodes its record from the tile: the walk's
// dependent length words and list bools become LDS reads instead of HBM
// round trips.  A record larger than the tile decodes from HBM.
template <int D>
__global__ __launch_bounds__(kRecThreads) void k_grp_dec_place_lds(const GroupArgs a_) {
    const GroupArgs &a = g_kargs<D>(a_);
    extern __shared__ __attribute__((aligned(16))) uint8_t tile[];
    __shared__ uint64_t runs[g_run_lds(D) ? kRunLds : 1];
    const unsigned long long key = *a.errkey;   // final: walk and capacity kernels ran before
    const uint64_t bad = key == kNoError ? a.n : (uint64_t)(key >> 16);
    const uint64_t rb = (uint64_t)blockIdx.x * kRecThreads;
    const uint32_t tid = threadIdx.x;
    const uint64_t lim = bad < a.n ? bad : a.n;
    const uint32_t nlive = lim > rb ? (uint32_t)(lim - rb < (uint64_t)kRecThreads ? lim - rb : (uint64_t)kRecThreads) : 0u;
    const uintptr_t xb = (uintptr_t)a.xdr;
    // the walk reads no byte at or past in_len (g_dec_record clamps each record's
    // end): the staged range is clamped the same way, so a record whose extent
    // runs past the stream (a cut tail that still parses) never stages bytes
    // beyond it — in XDRG_HOST_MAPPED mode those would be unmapped host memory
    auto ext = [&](uint64_t r) -> uint64_t { const uint64_t x = a.rec_in[r]; return x < a.xdr_cap ? x : a.xdr_cap; };
    uint32_t js = 0;
    while (js < nlive) {
        // records [js, js + 1 + tid) fit iff their aligned byte range does (monotone)
        const uint32_t je1 = js + 1 + tid;
        bool fits = false;
        if (je1 <= nlive) {
            const uintptr_t lo = (xb + ext(rb + js)) & ~(uintptr_t)15;
            const uintptr_t hi = (xb + ext(rb + je1) + 15) & ~(uintptr_t)15;
            fits = hi >= lo && hi - lo <= a.dec_tile;
        }
        const uint32_t k1 = (uint32_t)__syncthreads_count(fits);
        if constexpr (D > 1) {
            // one call site of the record decode (two inlined copies of the nested
            // form kept the kernel arguments in 4 KB of scratch): a record larger
            // than the tile (k1 = 0) decodes from the stream through the same
            // generic pointer, tile-relative positions keep both in range
            const uint32_t je = js + (k1 ? k1 : 1);
            const uintptr_t a0 = (xb + ext(rb + js)) & ~(uintptr_t)15;
            const uintptr_t a1 = (xb + ext(rb + je) + 15) & ~(uintptr_t)15;
            g_stage_tile(tile, a0, k1 && a1 > a0 ? (uint32_t)((a1 - a0) >> 4) : 0u);
            __syncthreads();
            if (js + tid < je)
                g_dec_record<D>(a, rb + js + tid, k1 ? tile : a.xdr, k1 ? a0 - xb : 0, GElDesc{}, runs + tid);
            __syncthreads();   // the tile's next use
            js = je;
            continue;
        }
        if (k1 == 0) {   // one record larger than the tile: its lane decodes from HBM
            if (tid == 0) g_dec_record<D>(a, rb + js, a.xdr, 0, GElDesc{}, runs + tid);
            ++js;
            continue;
        }
        const uint32_t je = js + k1;
        const uintptr_t a0 = (xb + ext(rb + js)) & ~(uintptr_t)15;
        const uintptr_t a1 = (xb + ext(rb + je) + 15) & ~(uintptr_t)15;
        g_stage_tile(tile, a0, a1 > a0 ? (uint32_t)((a1 - a0) >> 4) : 0u);
        __syncthreads();
        // stream offset x of these records is at tile + (x - (a0 - xb))
        if (js + tid < je) g_dec_record<D>(a, rb + js + tid, tile, a0 - xb, GElDesc{}, runs + tid);
        __syncthreads();   // the tile's next use
        js = je;
    }
}

// Element-parallel place (tuning key 38 > 0: at most that many elements per
// sub-batch; schemas with one top-level group, no inner groups, at most two
// dynamic members).  The lane-per-record place wrote each element's members
// at the lane's own record: the 64 stores of one instruction hit 64 rows
// far apart.  Here a sub-batch of records is staged in the LDS tile as in
// k_grp_dec_place_lds, each record lane walks its record once (top-level
// fields decoded, the group's elements parsed for their tile offsets and
// member native offsets: descriptors in LDS), and then every lane of the
// block decodes an element: consecutive lanes, consecutive elements, so the
// member stores of an instruction fall on consecutive rows.
// LDS of k_grp_dec_place_el: per-block metadata (extents, the group's first
// elements, the dynamic members' bases: 4 x 257 u64) | tile | descriptors
constexpr size_t kElMeta = 4 * (kRecThreads + 1) * 8;
#ifndef XDRG_EL_OCC
#define XDRG_EL_OCC 1   // blocks per CU the register budget is sized for (experiment builds: 2, 3)
#endif
// MAP (GroupArgs::emap, tuning key 44): the walk left a 1 at the stream word
// of every element start, so a sub-batch finds its elements' positions by a
// block scan over the map, every lane parses a run of elements for their
// dynamic members' lengths, a block scan places those, and a record lane only
// steps over its group from its last element: no serial walk through the
// elements.  A block with a record not 4-aligned takes the record walk.
template <bool LAY, bool MAP>   // LAY: the group is GroupArgs::lay_g (the record walk reads the layout)
__global__ __launch_bounds__(kRecThreads, XDRG_EL_OCC) void k_grp_dec_place_el(const GroupArgs a_) {
    const GroupArgs &a = g_kargs<kGrpLevels>(a_);
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint64_t *mx = (uint64_t *)smem;             // [257] record extents (clamped to in_len)
    uint64_t *mE = mx + (kRecThreads + 1);       // [257] the group's first element of each record
    uint64_t *mb0 = mE + (kRecThreads + 1);      // [257] dynamic member 0's base
    uint64_t *mb1 = mb0 + (kRecThreads + 1);     // [257] dynamic member 1's base
    uint8_t *tile = smem + kElMeta;
    __shared__ uint64_t runs[g_run_lds(1) ? kRunLds : 1];
    uint32_t *dpos = (uint32_t *)(tile + a.dec_tile);
    uint32_t *drel = dpos + a.dec_el;
    const unsigned long long key = *a.errkey;   // final: walk and capacity kernels ran before
    const uint64_t bad = key == kNoError ? a.n : (uint64_t)(key >> 16);
    const uint64_t rb = (uint64_t)blockIdx.x * kRecThreads;
    const uint32_t tid = threadIdx.x;
    const uint64_t lim = bad < a.n ? bad : a.n;
    const uint32_t nlive = lim > rb ? (uint32_t)(lim - rb < (uint64_t)kRecThreads ? lim - rb : (uint64_t)kRecThreads) : 0u;
    const uintptr_t xb = (uintptr_t)a.xdr;
    const uint32_t g = a.el_g;
    const GField &G = a.f[g];
    GElDesc el;
    el.pos = dpos;
    el.rel = drel;
    el.cap = a.dec_el;
    el.tile = tile;
    el.nm = 0;
    el.ms0 = el.ms1 = el.mk0 = el.mk1 = 0;
    el.sb0 = el.sb1 = 0;
    for (uint32_t j = 1; j <= G.nmem; ++j) {
        j = g_uni(j);
        if (a.f[g + j].kind != XDRG_K_DYNAMIC) continue;
        if (el.nm == 0) { el.ms0 = a.f[g + j].slot; el.mk0 = g + j; }
        else { el.ms1 = a.f[g + j].slot; el.mk1 = g + j; }
        ++el.nm;
    }
    // the element layout (GroupArgs::lay_g: every element has the same fields)
    el.lay = LAY;
    el.pre = a.lay_pre;
    el.mid = a.lay_mid;
    el.post = a.lay_post;
    el.z0 = a.lay_z0;
    el.z1 = a.lay_z1;
    el.rb = rb;
    el.mE = mE;
    el.mb0 = mb0;
    el.mb1 = mb1;
    // the block's metadata in one round trip (records rb .. rb + nlive, one past the last)
    for (uint32_t j = tid; j <= nlive; j += kRecThreads) {
        const uint64_t r = rb + j;
        const uint64_t x = a.rec_in[r];
        mx[j] = x < a.xdr_cap ? x : a.xdr_cap;
        mE[j] = G.kind == XDRG_K_FIXED ? r * G.count : (r < a.n ? g_rec_base(a, G.slot, r) : a.totals[G.slot - 1]);
        if (el.nm > 0) mb0[j] = r < a.n ? g_rec_base(a, el.ms0, r) : a.totals[el.ms0 - 1];
        if (el.nm > 1) mb1[j] = r < a.n ? g_rec_base(a, el.ms1, r) : a.totals[el.ms1 - 1];
    }
    bool use_map = false;
    if constexpr (MAP) {   // element starts map to words exactly when records are 4-aligned
        bool al = true;
        for (uint32_t j = tid; j <= nlive; j += kRecThreads) {
            const uint64_t x = a.rec_in[rb + j];
            al = al && (x & 3) == 0;
        }
        use_map = __syncthreads_and(al);
    } else {
        __syncthreads();
    }
    uint32_t js = 0;
    while (js < nlive) {
        const uint32_t je1 = js + 1 + tid;
        bool fits = false;
        if (je1 <= nlive) {
            const uintptr_t lo = (xb + mx[js]) & ~(uintptr_t)15;
            const uintptr_t hi = (xb + mx[je1] + 15) & ~(uintptr_t)15;
            fits = hi >= lo && hi - lo <= a.dec_tile && mE[je1] - mE[js] <= a.dec_el;
        }
        const uint32_t k1 = (uint32_t)__syncthreads_count(fits);
        if (k1 == 0) {   // one record larger than the tile or the descriptors: its lane decodes from HBM
            if (tid == 0) g_dec_record<1>(a, rb + js, a.xdr, 0, GElDesc{}, runs + tid);
            ++js;
            continue;
        }
        const uint32_t je = js + k1;
        const uintptr_t a0 = (xb + mx[js]) & ~(uintptr_t)15;
        const uintptr_t a1 = (xb + mx[je] + 15) & ~(uintptr_t)15;
        const uint32_t nch = a1 > a0 ? (uint32_t)((a1 - a0) >> 4) : 0u;
        g_stage_tile(tile, a0, nch);
        el.E0 = mE[js];
        el.sb0 = mb0[js];
        el.sb1 = mb1[js];
        __syncthreads();
        // stream offset x at tile + (x - (a0 - xb))
        const uint32_t nel_sb = (uint32_t)(mE[je] - el.E0);
        bool mapped = false;
        if (MAP && use_map) {
            // positions: the flagged words of the sub-batch's records, in order
            const uint64_t tb = a0 - xb;
            const uint64_t wlo = mx[js] >> 2, whi = mx[je] >> 2;
            uint32_t found = 0;
            for (uint64_t cw = wlo & ~15ull; cw < whi; cw += 16 * kRecThreads) {   // (block-uniform)
                const uint64_t w0 = cw + 16ull * tid;
                typedef uint32_t u32x4g __attribute__((ext_vector_type(4)));
                u32x4g v = {0u, 0u, 0u, 0u};
                if (w0 < whi) v = *(const u32x4g *)(a.emap + w0);
                uint32_t fl = 0;   // bit b: word w0 + b starts an element
#pragma unroll
                for (int b = 0; b < 16; ++b) {
                    const uint64_t w = w0 + b;
                    if (((v[b >> 2] >> (8 * (b & 3))) & 0xffu) && w >= wlo && w < whi) fl |= 1u << b;
                }
                uint64_t tot;
                uint32_t idx = found + (uint32_t)block_excl_scan(__popc(fl), &tot);
                for (uint32_t m = fl; m; m &= m - 1, ++idx)
                    if (idx < nel_sb) dpos[idx] = (uint32_t)(4 * (w0 + __ffs(m) - 1) - tb);
                found += (uint32_t)tot;
            }
            XDRG_DCHECK(found == nel_sb);
            mapped = found == nel_sb;   // (block-uniform; else the record walk below)
            __syncthreads();   // dpos
        }
        if (MAP && mapped) {
            // the dynamic members' native offsets: each lane a run of elements
            const uint64_t tb = a0 - xb;
            const uint32_t nel = nel_sb;
            const uint32_t per = (nel + kRecThreads - 1) / kRecThreads;
            uint64_t sum = 0;
            for (uint32_t u = 0; u < per; ++u) {
                const uint32_t i = tid * per + u;
                if (i >= nel) break;
                uint64_t pos = dpos[i], l0, l1;
                if constexpr (LAY) g_el_parse<true>(a, el, g, tile, pos, l0, l1);
                else g_el_parse<false>(a, el, g, tile, pos, l0, l1);
                drel[i] = (uint32_t)l0;
                drel[el.cap + i] = (uint32_t)l1;
                sum += l0 | l1 << 32;   // (a sub-batch's lengths fit 32 bits each)
            }
            uint64_t tot;
            const uint64_t pre = block_excl_scan(sum, &tot);
            uint32_t r0 = (uint32_t)pre, r1 = (uint32_t)(pre >> 32);
            for (uint32_t u = 0; u < per; ++u) {
                const uint32_t i = tid * per + u;
                if (i >= nel) break;
                const uint32_t l0 = drel[i], l1 = drel[el.cap + i];
                drel[i] = r0;
                drel[el.cap + i] = r1;
                r0 += l0;
                r1 += l1;
            }
            if (js + tid < je) g_dec_record<1, true, true>(a, rb + js + tid, tile, tb, el, runs + tid);
        } else {
            if (js + tid < je) g_dec_record<1, true>(a, rb + js + tid, tile, a0 - xb, el, runs + tid);
        }
        __syncthreads();   // descriptors
        const uint64_t nel = mE[je] - el.E0;
        XDRG_DCHECK(nel <= a.dec_el);   // (the fit count bounded the sub-batch's elements)
        for (uint32_t i = tid; i < nel; i += kRecThreads) {
#if XDRG_EL_RUN2
            GRun2 run{el.ms0 ? el.ms0 : ~0u, el.ms1 ? el.ms1 : ~0u, 0, 0};
#else
            GRunOf<1> run;
            g_run_bind(run, runs + tid);
            run.zero();
#endif
            // the record walk left every element a tile position inside the staged
            // bytes and member offsets inside the members' capacities
            XDRG_DCHECK(dpos[i] < 16u * nch);
            XDRG_DCHECK(el.nm < 1 || el.sb0 + drel[i] <= a.f[el.mk0].cap);
            XDRG_DCHECK(el.nm < 2 || el.sb1 + drel[el.cap + i] <= a.f[el.mk1].cap);
            if (el.nm > 0) run.set(el.ms0, el.sb0 + drel[i]);
            if (el.nm > 1) run.set(el.ms1, el.sb1 + drel[el.cap + i]);
            GDisc d{};
            uint64_t pos = dpos[i];
            g_dec_elem<0, 1>(a, g, el.E0 + i, tile, pos, ~0ull, d, run);
        }
        __syncthreads();   // the tile's and the descriptors' next use
        js = je;
    }
}

// Element-parallel place for a schema whose one top-level group holds inner
// groups (D > 1; GroupArgs::emap set, tuning keys 38 / 44): a sub-batch of
// records is staged as in k_grp_dec_place_el and its elements found from the
// walk's element-start map; every lane walks a run of elements (inner groups
// included) for their counts of every counted column of the group's span, a
// block scan per column places them, a record lane writes its first rows'
// offsets and steps over its group from its last element, and every lane
// then decodes elements, inner groups included, from running offsets that
// start at its element's scanned positions (GRunL columns).  A block with a
// record not 4-aligned, or a sub-batch whose map count differs, decodes a
// record per lane from the tile (k_grp_dec_place_lds).
// LDS: eln_lds_bytes (xdrg_internal.h).
template <int D>
__global__ __launch_bounds__(kRecThreads) void k_grp_dec_place_eln(const GroupArgs a_) {
    const GroupArgs &a = g_kargs<kGrpLevels>(a_);
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    __shared__ uint64_t sbase[kMaxSlots];   // each column's native offset at the sub-batch's first record
    uint64_t *mx = (uint64_t *)smem;             // [257] record extents (clamped to in_len)
    uint64_t *mE = mx + (kRecThreads + 1);       // [257] the group's first element of each record
    uint8_t *tile = smem + kElnMeta;
    const uint32_t cap = a.dec_el;
    uint32_t *dpos = (uint32_t *)(tile + a.dec_tile);
    uint32_t *drel = dpos + cap;
    const uint32_t g = a.el_g;
    const GField &G = a.f[g];
    uint32_t ns = 0;   // counted columns of the group's span
    for (uint32_t j = 1; j <= G.nmem; ++j) ns += a.f[g_uni(g + j)].slot ? 1u : 0u;
    uint64_t *runs = (uint64_t *)(dpos + (((size_t)cap * (1 + ns) + 1) & ~(size_t)1));   // (8-aligned)
    uint64_t *const rl = runs + threadIdx.x;
    const unsigned long long key = *a.errkey;   // final: walk and capacity kernels ran before
    const uint64_t bad = key == kNoError ? a.n : (uint64_t)(key >> 16);
    const uint64_t rb = (uint64_t)blockIdx.x * kRecThreads;
    const uint32_t tid = threadIdx.x;
    const uint64_t lim = bad < a.n ? bad : a.n;
    const uint32_t nlive = lim > rb ? (uint32_t)(lim - rb < (uint64_t)kRecThreads ? lim - rb : (uint64_t)kRecThreads) : 0u;
    const uintptr_t xb = (uintptr_t)a.xdr;
    GElDesc el{};
    el.pos = dpos;
    el.cap = cap;
    el.tile = tile;
    el.rb = rb;
    el.mE = mE;
    bool al = true;
    for (uint32_t j = tid; j <= nlive; j += kRecThreads) {
        const uint64_t r = rb + j;
        const uint64_t x = a.rec_in[r];
        al = al && (x & 3) == 0;
        mx[j] = x < a.xdr_cap ? x : a.xdr_cap;
        mE[j] = G.kind == XDRG_K_FIXED ? r * G.count : (r < a.n ? g_rec_base(a, G.slot, r) : a.totals[G.slot - 1]);
    }
    const bool use_map = __syncthreads_and(al);
    uint32_t js = 0;
    while (js < nlive) {
        const uint32_t je1 = js + 1 + tid;
        bool fits = false;
        if (je1 <= nlive) {
            const uintptr_t lo = (xb + mx[js]) & ~(uintptr_t)15;
            const uintptr_t hi = (xb + mx[je1] + 15) & ~(uintptr_t)15;
            fits = hi >= lo && hi - lo <= a.dec_tile && mE[je1] - mE[js] <= cap;
        }
        const uint32_t k1 = (uint32_t)__syncthreads_count(fits);
        if (k1 == 0) {   // one record larger than the tile or the positions: its lane decodes from HBM
            if (tid == 0) g_dec_record<D>(a, rb + js, a.xdr, 0, GElDesc{}, rl);
            ++js;
            continue;
        }
        const uint32_t je = js + k1;
        const uintptr_t a0 = (xb + mx[js]) & ~(uintptr_t)15;
        const uintptr_t a1 = (xb + mx[je] + 15) & ~(uintptr_t)15;
        const uint64_t tb = a0 - xb;
        g_stage_tile(tile, a0, a1 > a0 ? (uint32_t)((a1 - a0) >> 4) : 0u);
        el.E0 = mE[js];
        if (tid < a.nslot) {
            const uint64_t r = rb + js;
            sbase[tid] = r < a.n ? g_rec_base(a, tid + 1, r) : a.totals[tid];
        }
        __syncthreads();
        const uint32_t nel = (uint32_t)(mE[je] - el.E0);
        bool mapped = false;
        if (use_map) {   // positions: the flagged words of the sub-batch's records, in order
            const uint64_t wlo = mx[js] >> 2, whi = mx[je] >> 2;
            uint32_t found = 0;
            for (uint64_t cw = wlo & ~15ull; cw < whi; cw += 16 * kRecThreads) {   // (block-uniform)
                const uint64_t w0 = cw + 16ull * tid;
                typedef uint32_t u32x4g __attribute__((ext_vector_type(4)));
                u32x4g v = {0u, 0u, 0u, 0u};
                if (w0 < whi) v = *(const u32x4g *)(a.emap + w0);
                uint32_t fl = 0;   // bit b: word w0 + b starts an element
#pragma unroll
                for (int b = 0; b < 16; ++b) {
                    const uint64_t w = w0 + b;
                    if (((v[b >> 2] >> (8 * (b & 3))) & 0xffu) && w >= wlo && w < whi) fl |= 1u << b;
                }
                uint64_t tot;
                uint32_t idx = found + (uint32_t)block_excl_scan(__popc(fl), &tot);
                for (uint32_t m = fl; m; m &= m - 1, ++idx)
                    if (idx < nel) dpos[idx] = (uint32_t)(4 * (w0 + __ffs(m) - 1) - tb);
                found += (uint32_t)tot;
            }
            XDRG_DCHECK(found == nel);
            mapped = found == nel;   // (block-uniform)
            __syncthreads();   // dpos
        }
        if (!mapped) {   // a record per lane from the tile
            if (js + tid < je) g_dec_record<D>(a, rb + js + tid, tile, tb, GElDesc{}, rl);
            __syncthreads();   // the tile's next use
            js = je;
            continue;
        }
        // each lane's run of elements: their counts of every span column
        const uint32_t per = (nel + kRecThreads - 1) / kRecThreads;
        WCntL cnt{(uint32_t *)runs + tid};   // (the lane's GRunL column as counters until the decode)
        for (uint32_t u = 0; u < per; ++u) {
            const uint32_t i = tid * per + u;
            if (i >= nel) break;
            for (uint32_t s = 0; s < a.nslot; ++s) cnt[s] = 0;
            uint64_t pos = dpos[i];
            GDisc d{};
            (void)g_walk_elem<0, D>(a, g, tile, ~0ull, pos, cnt, d);
            uint32_t q = 0;
            for (uint32_t j = 1; j <= G.nmem; ++j) {
                const uint32_t sl = a.f[g_uni(g + j)].slot;
                if (sl) drel[(size_t)q++ * cap + i] = cnt[sl - 1];
            }
        }
        // a block scan per column: counts -> positions relative to sbase
        for (uint32_t q = 0; q < ns; ++q) {
            uint32_t *c = drel + (size_t)q * cap;
            uint64_t sum = 0;
            for (uint32_t u = 0; u < per; ++u) {
                const uint32_t i = tid * per + u;
                if (i < nel) sum += c[i];
            }
            uint64_t tot;
            uint32_t p = (uint32_t)block_excl_scan(sum, &tot);
            for (uint32_t u = 0; u < per; ++u) {
                const uint32_t i = tid * per + u;
                if (i >= nel) break;
                const uint32_t x = c[i];
                c[i] = p;
                p += x;
            }
        }
        if (js + tid < je) g_dec_record<D, true, true>(a, rb + js + tid, tile, tb, el, rl);
        __syncthreads();   // positions, scanned counts
        for (uint32_t i = tid; i < nel; i += kRecThreads) {
            GRunL run{rl};
            uint32_t q = 0;
            for (uint32_t j = 1; j <= G.nmem; ++j) {
                const uint32_t sl = a.f[g_uni(g + j)].slot;
                if (sl) run.set(sl, sbase[sl - 1] + drel[(size_t)q++ * cap + i]);
            }
            GDisc d{};
            uint64_t pos = dpos[i];
            g_dec_elem<0, D>(a, g, el.E0 + i, tile, pos, ~0ull, d, run);
        }
        __syncthreads();   // the tile's and the positions' next use
        js = je;
    }
}

// Kernels are instantiated per group levels D: 1 (no group inside an element:
// the inner-group code compiled out, running offsets in registers), 2 (one
// level of groups inside elements, the common nested shapes) and kGrpLevels
// (deeper schemas; their inlined levels take more registers).
template <int D>
static hipError_t launch_group_phase_t(const GroupArgs &a, int phase, hipStream_t st) {
    const dim3 grid((uint32_t)a.nblocks), block(kRecThreads);
    const dim3 rgrid((uint32_t)((a.n + kRecThreads - 1) / kRecThreads));
    const uint32_t split = a.enc_split ? a.enc_split : enc_el_split(a.nblocks);
    const dim3 egrid((uint32_t)a.nblocks * split);
    const bool esh = split > 1;
    switch (phase) {
    case GRP_ENC_SIZES:
        if (kWalkSplit > 1) {
            const hipError_t e = hipMemsetAsync(a.block_sums, 0, (size_t)a.nblocks * 8, st);
            if (e != hipSuccess) return e;
        }
        hipLaunchKernelGGL(k_grp_enc_sizes<D>, dim3((uint32_t)a.nblocks * kWalkSplit), block, 0, st, a);
        break;
    case GRP_ENC_PLACE:   // element-parallel (key 41) or G lanes per record (key 32)
        if constexpr (D > 2) {   // deep schemas' records are large: a 32 KiB image at least (acl_tree
                                 // encode 3.49 ms at 16 KiB, 2.15 at 32; volume_index keeps 16 KiB:
                                 // 1.04 vs 1.28 ms, profiles/r05_groups/enc_nest_ab.txt)
            if (a.enc_img && a.enc_img < 32768) {
                GroupArgs b = a;
                b.enc_img = 32768;
                return launch_group_phase_t<D>(b, phase, st);
            }
        }
        if (a.enc_img && a.ncond && esh) hipLaunchKernelGGL((k_grp_enc_place_el<true, true, D>), egrid, block, enc_el_lds_bytes(a.enc_img), st, a);
        else if (a.enc_img && a.ncond) hipLaunchKernelGGL((k_grp_enc_place_el<true, false, D>), egrid, block, enc_el_lds_bytes(a.enc_img), st, a);
        else if (a.enc_img && esh) hipLaunchKernelGGL((k_grp_enc_place_el<false, true, D>), egrid, block, enc_el_lds_bytes(a.enc_img), st, a);
        else if (a.enc_img) hipLaunchKernelGGL((k_grp_enc_place_el<false, false, D>), egrid, block, enc_el_lds_bytes(a.enc_img), st, a);
        else if (a.enc_lanes == 4) hipLaunchKernelGGL((k_grp_enc_place<4, D>), grid, block, 0, st, a);
        else if (a.enc_lanes == 8) hipLaunchKernelGGL((k_grp_enc_place<8, D>), grid, block, 0, st, a);
        else if (a.enc_lanes == 16) hipLaunchKernelGGL((k_grp_enc_place<16, D>), grid, block, 0, st, a);
        else if (a.enc_lanes == 32) hipLaunchKernelGGL((k_grp_enc_place<32, D>), grid, block, 0, st, a);
        else hipLaunchKernelGGL((k_grp_enc_place<64, D>), grid, block, 0, st, a);
        break;
    case GRP_DEC_WALK:
        if (kWalkSplit > 1 && a.nslot) {
            const hipError_t e = hipMemsetAsync(a.block_sums, 0, (size_t)a.nslot * a.nblocks * 8, st);
            if (e != hipSuccess) return e;
        }
        if constexpr (D == 1) {
            if (a.lay_g) hipLaunchKernelGGL((k_grp_dec_walk<1, false>), dim3((uint32_t)a.nblocks * kWalkSplit), block, 0, st, a);
            else hipLaunchKernelGGL((k_grp_dec_walk<1, true>), dim3((uint32_t)a.nblocks * kWalkSplit), block, 0, st, a);
        } else {
            hipLaunchKernelGGL((k_grp_dec_walk<D, true>), dim3((uint32_t)a.nblocks * kWalkSplit), block, 0, st, a);
        }
        break;
    case GRP_DEC_OFFSETS: if (a.nslot) hipLaunchKernelGGL(k_grp_dec_offsets, grid, block, 0, st, a); break;
    case GRP_DEC_PLACE:   // a lane per record, from an LDS tile (tuning key 33 > 0) or from HBM
        if (D > 1 && a.emap && a.dec_el && a.dec_tile) {   // element-parallel, inner groups
            uint32_t ns = 0;
            for (uint32_t j = 1; j <= a.f[a.el_g].nmem; ++j) ns += a.f[a.el_g + j].slot ? 1u : 0u;
            if constexpr (D > 1)
                hipLaunchKernelGGL(k_grp_dec_place_eln<D>, rgrid, block, eln_lds_bytes(a.dec_tile, a.dec_el, ns, a.nslot), st, a);
        } else if (D == 1 && a.dec_el && a.dec_tile) {
            const size_t lds = kElMeta + a.dec_tile + 12 * (size_t)a.dec_el;
            if (a.lay_g == a.el_g + 1 && a.emap) hipLaunchKernelGGL((k_grp_dec_place_el<true, true>), rgrid, block, lds, st, a);
            else if (a.lay_g == a.el_g + 1) hipLaunchKernelGGL((k_grp_dec_place_el<true, false>), rgrid, block, lds, st, a);
            else if (a.emap) hipLaunchKernelGGL((k_grp_dec_place_el<false, true>), rgrid, block, lds, st, a);
            else hipLaunchKernelGGL((k_grp_dec_place_el<false, false>), rgrid, block, lds, st, a);
        }
        else if (a.dec_tile) hipLaunchKernelGGL(k_grp_dec_place_lds<D>, rgrid, block, a.dec_tile, st, a);
        else hipLaunchKernelGGL(k_grp_dec_place<D>, rgrid, block, 0, st, a);
        break;
    default: break;
    }
    return hipSuccess;
}

int launch_group_phase(const GroupArgs &a, int phase, void *stream) {
    if (phase < GRP_ENC_SIZES || phase > GRP_DEC_PLACE) return (int)hipErrorInvalidValue;
    const hipError_t e = a.levels > 2 ? launch_group_phase_t<kGrpLevels>(a, phase, (hipStream_t)stream)
                       : a.levels == 2 ? launch_group_phase_t<2>(a, phase, (hipStream_t)stream)
                                       : launch_group_phase_t<1>(a, phase, (hipStream_t)stream);
    return (int)(e != hipSuccess ? e : hipGetLastError());
}

}  // namespace xdrg
