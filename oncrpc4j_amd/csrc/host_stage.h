// host_stage.h — the XDRG_HOST_PTRS pipeline of the C-ABI (include/xdrg.h):
// batches whose columns and stream live in HOST memory, moved through a
// context-owned ring of device slots chunk by chunk.
//
// The reference builds every Xdr on a host Grizzly Buffer
// (xdr/Xdr.java:115-119, grizzly/GrizzlyMemoryManager.java:42-57) and sends
// from it (grizzly/GrizzlyRpcTransport.java:97-112); a caller of the engine
// therefore starts and ends in host memory.  A batch is cut into record
// ranges (chunks) that fit one slot; chunk k of a direction goes
//     H2D (copy stream)  ->  codec kernels (compute stream)  ->  D2H (copy stream)
// in slot k mod S, so the H2D of one chunk, the kernels of another and the
// D2H of a third are in flight together.  Host spans that are not pinned
// (xdrg_host_register / hipHostMalloc) go through the slot's pinned bounce
// buffer: a CPU copy before the H2D, after the D2H.
//
// This header is plain C++17 (no HIP): the pipeline is a template over an
// executor, so the same planning and bookkeeping runs on the GPU
// (xdrg_abi.cpp, HipExec) and under ASan/UBSan on the CPU with the oracle as
// the "kernels" (tests/cpp/san_stage.cpp).  Executor interface:
//   uint32_t nslots(); uint64_t slot_bytes(); uint8_t *slot(uint32_t s);
//   uint8_t *bounce(uint32_t s);                 // pinned mirror of slot s (lazily allocated)
//   bool pinned(const void *p, uint64_t bytes);  // host span the DMA engines can read / write
//   int wait_slot(uint32_t s);                   // host-blocking: slot s's last D2H has landed
//   int dma_h2d(uint8_t *dev, const void *host, uint64_t bytes);         // copy stream
//   int h2d_done(uint32_t s);                    // event: slot s's inputs are on the device
//   int kernel_begin(uint32_t s);                // compute stream waits h2d_done(s)
//   int add_u64(int on_d2h, uint64_t *dev, uint64_t n, uint64_t delta);  // dev[0..n) += delta
//   int add_pos(uint64_t *dev, uint64_t n, uint64_t delta);   // copy stream: the same, UINT64_MAX kept
//   int encode(uint32_t s, const xdrg_column *dcols, uint64_t m, uint8_t *out, uint64_t cap,
//              uint64_t *rec, uint32_t flags, uint32_t byref, uint64_t *ref);
//                                                // async; result word 0 = stream bytes; byref = 0 or
//                                                // 1 + the field encoded by reference, ref its splice
//                                                // positions (xdrg_encode_batch_shallow)
//   int decode(uint32_t s, const uint8_t *in, uint64_t len, const uint64_t *rec, uint64_t m,
//              xdrg_column *dcols, uint32_t flags, uint32_t byref, uint64_t *ref);
//                                                // async; words 0 / 1 = first_bad / err; byref: the
//                                                // field decoded as a view, ref its payload positions
//                                                // (xdrg_decode_batch_view)
//   int kernel_end(uint32_t s, const uint64_t *const *extra, const uint64_t *const *index,
//                  const uint64_t *limit, uint32_t nextra);
//                                                // result words 2 + i = index[i] ? (*index[i] <= limit[i] ?
//                                                // extra[i][*index[i]] : 0) : *extra[i] (device words); event
//   const uint64_t *res_word(uint32_t s, uint32_t i);  // device address of slot s's result word 2 + i
//                                                // (an index of a later kernel_end entry: the totals
//                                                // of an inner group's members follow its own)
//   int wait_kernel(uint32_t s, uint64_t *words); // host-blocking; words[0 .. 2 + nextra)
//   int d2h_begin(uint32_t s);                   // copy stream waits slot s's kernels
//   int dma_d2h(void *host, const uint8_t *dev, uint64_t bytes);
//   int dma_d2h_2d(void *host, uint64_t hpitch, const uint8_t *dev, uint64_t dpitch,
//                  uint64_t width, uint64_t rows);
//   int d2h_done(uint32_t s);                    // event: slot s's outputs have left
//   int grow(uint64_t slot_bytes);               // reallocate the ring (idle) for a larger chunk
// and, for the receive pipeline (stage_receive):
//   int scan(uint32_t s, const uint8_t *win, uint64_t wlen, uint64_t cap, uint64_t *offs, int bodies,
//            uint8_t *body_dst, uint64_t *boffs, uint64_t *res);
//       host-blocking, on the compute stream (after kernel_begin(s)): the record-mark walk of
//       win[0, wlen) (RpcMessageParserTCP.java:63-140).  res[0] = complete messages (<= cap),
//       res[1] = the stream bytes they occupy, res[2] = 1 if every one is a single fragment,
//       offs[0..res[0]] = their offsets in win.  With bodies == 2 (or 1 and res[2] == 0) their
//       bodies are also assembled, marks stripped (assembleXdr :109-140), into body_dst (NULL:
//       the executor's own body buffer, body()), boffs[0..res[0]] = body offsets, res[3] = bytes.
//   const uint8_t *body();                       // the executor's body buffer (device)
//   int d2d(uint8_t *dst, const uint8_t *src, uint64_t bytes);   // copy stream, in order with dma_h2d
//   int offs_copy(uint64_t *dst, const uint64_t *src, uint64_t n, uint64_t delta);   // compute stream:
//                                                // dst[i] = src[i] + delta
//   int decode_count(uint32_t s, const uint8_t *in, uint64_t len, const uint64_t *rec, uint64_t m,
//                    uint32_t flags, uint64_t *tot, uint64_t *bad);
//       host-blocking, compute stream: the first half of a repeated-group schema's decode (its
//       walk): tot[i] = values / elements of the i-th counted field (dynamic fields and DYNAMIC /
//       LIST groups, in field order) over the m records, at least what the place writes for
//       the records before the first bad one (*bad, m if none)
//   int decode_place(<decode's arguments>);      // async: the rest of that decode (the walk's
//                                                // counts, dcols sized by tot)
// Every call returns XDRG_OK or an XDRG_E_* status.
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <algorithm>
#include <cstring>
#include <deque>
#include <functional>
#include <vector>

#include "../../include/xdrg.h"

namespace xdrg {
namespace hs {

constexpr uint32_t kMaxSlots = 8;
constexpr uint64_t kSpanAlign = 256;   // every span starts on its own 256-B boundary ...
constexpr uint64_t kSpanSlack = 64;    // ... followed by slack the 16-B window loads may touch

// One schema field as the pipeline sees it (the compiled xdrg_schema's view).
// Repeated groups (include/xdrg.h): a group field (XDRG_T_GROUP) has no data
// of its own (DYNAMIC / LIST: per-record element offsets), its members are
// columns indexed by ELEMENT, so a chunk of records [lo, lo + m) moves the
// member rows of its elements.
struct Field {
    uint32_t type, kind, count;
    uint32_t nsz;      // native element bytes
    uint32_t xsz;      // XDR element bytes (1: opaque / string bytes)
    uint32_t xbytes;   // fixed fields: XDR bytes of the field
    uint32_t grp = 0;  // member: its group's field index + 1
    uint32_t emin = 0; // group: fewest XDR bytes of one element (0: elements may be empty)
};
struct Schema {
    std::vector<Field> f;
    uint64_t fixed_part = 0;   // XDR bytes of the fixed fields
    bool var_size = false;     // dynamic or conditional fields
    uint64_t min_xdr = 0;      // fewest XDR bytes a well-formed record has (receive: rows per window)
    bool groups = false;
};
inline bool is_group(const Field &f) { return f.type == XDRG_T_GROUP; }

// Rows of each field's column in a chunk: records [lo, lo + m) for top-level
// fields, the chunk's elements for a group's members.
struct Rows {
    std::vector<uint64_t> lo, n;   // per field
};

inline uint64_t up(uint64_t v, uint64_t a) { return (v + a - 1) / a * a; }

// Fixed-size columns that share one host window per record: the fields of an
// array-of-structs record (same stride, within one stride of the lowest),
// or one struct-of-arrays column, or a constant column (stride 0).
struct Region {
    const uint8_t *base = nullptr;   // lowest field address (row 0)
    int64_t stride = 0;              // bytes per row; 0 = constant (encode only)
    uint32_t space = 0;              // 0: records; g + 1: the elements of group field g
    uint64_t row_end = 0;            // bytes of a row that fields cover, from base
    bool full = false;               // fields cover every byte of a row (decode: one contiguous D2H)
    std::vector<uint32_t> fields;
    std::vector<std::pair<uint64_t, uint64_t>> segs;   // covered [a, b) inside a row, merged
};

inline uint64_t fixed_elem_bytes(const Field &f) {
    return (uint64_t)f.nsz * (f.kind == XDRG_K_FIXED ? f.count : 1);
}

// Group the fixed columns into regions.  Returns XDRG_E_INVAL for layouts the
// pipeline does not take (negative or overlapping strides).
inline int build_regions(const Schema &s, const xdrg_column *cols, std::vector<Region> &out) {
    out.clear();
    struct C { const uint8_t *p; int64_t st; uint64_t e; uint32_t k, sp; };
    std::vector<C> v;
    for (uint32_t k = 0; k < s.f.size(); ++k) {
        const Field &f = s.f[k];
        if (f.kind == XDRG_K_DYNAMIC || is_group(f)) continue;
        const uint64_t e = fixed_elem_bytes(f);
        if (!e) continue;   // T x[0]: no bytes on either side
        int64_t st = cols[k].stride;
        if (st == XDRG_STRIDE_CONST) st = 0;
        else if (st == 0) st = (int64_t)e;
        else if (st < 0 || (uint64_t)st < e) return XDRG_E_INVAL;
        v.push_back({(const uint8_t *)cols[k].data, st, e, k, f.grp});
    }
    std::sort(v.begin(), v.end(), [](const C &a, const C &b) {
        return a.sp != b.sp ? a.sp < b.sp : a.st != b.st ? a.st < b.st : a.p < b.p;
    });
    for (const C &c : v) {   // (a region's fields share one row space: records, or one group's elements)
        Region *r = out.empty() ? nullptr : &out.back();
        const bool joins = r && c.st && r->stride == c.st && r->space == c.sp && c.p >= r->base &&
                           (uint64_t)(c.p - r->base) + c.e <= (uint64_t)c.st;
        if (!joins) {
            out.push_back(Region());
            r = &out.back();
            r->base = c.p;
            r->stride = c.st;
            r->space = c.sp;
        }
        const uint64_t a = (uint64_t)(c.p - r->base);
        r->fields.push_back(c.k);
        r->row_end = std::max(r->row_end, a + c.e);
        r->segs.push_back({a, a + c.e});
    }
    for (Region &r : out) {
        std::sort(r.segs.begin(), r.segs.end());
        std::vector<std::pair<uint64_t, uint64_t>> m;
        for (auto &g : r.segs) {
            if (!m.empty() && g.first <= m.back().second) m.back().second = std::max(m.back().second, g.second);
            else m.push_back(g);
        }
        r.segs = m;
        r.full = r.stride && m.size() == 1 && m[0].first == 0 && m[0].second == (uint64_t)r.stride;
    }
    return XDRG_OK;
}

// Bump allocation of one chunk's spans inside a slot; `mod` keeps a span's
// address congruent to its host address modulo 16, so a host-aligned column
// stays aligned on the device (the kernels check native alignment).
struct Bump {
    uint64_t used = 0;
    uint64_t take(uint64_t bytes, uint64_t mod = 0) {
        const uint64_t o = up(used, kSpanAlign) + (mod & 15);
        used = o + bytes + kSpanSlack;
        return o;
    }
};

// Where one chunk's data sits inside its slot.
struct Layout {
    uint64_t lo = 0, m = 0, need = 0;
    std::vector<uint64_t> reg;               // per region: slot offset of row 0's base
    std::vector<uint64_t> val, off, vcap;    // per field (dynamic, group offsets): values / offsets, value capacity
    std::vector<uint64_t> rows;              // decode: per field, the rows laid out (members: element bound)
    uint64_t xdr = 0, xcap = 0, rec = 0;     // stream span, its capacity, record offsets (m + 1)
    uint64_t ref = 0;                        // by-reference field: splice / payload positions (m)
    uint64_t win = 0, wlen = 0;              // decode: host window [win, win + wlen) of the stream
};

// Rows of a chunk of records [lo, lo + m): records for top-level fields, the
// chunk's elements for group members (encode: from the host group offsets).
// Groups nest (a group's members may hold groups): the tape is in pre-order,
// so a group's own rows (records, or its parent's elements) are known when
// its turn comes, and its element offsets are indexed by them.
inline void chunk_rows(const Schema &s, const xdrg_column *cols, uint64_t lo, uint64_t m, Rows &R) {
    R.lo.assign(s.f.size(), lo);
    R.n.assign(s.f.size(), m);
    for (uint32_t g = 0; g < s.f.size(); ++g) {
        const Field &f = s.f[g];
        if (!is_group(f)) continue;
        uint64_t elo, em;
        if (f.kind == XDRG_K_FIXED) {
            elo = R.lo[g] * f.count;
            em = R.n[g] * f.count;
        } else {
            elo = cols[g].offsets[R.lo[g]];
            em = cols[g].offsets[R.lo[g] + R.n[g]] - elo;
        }
        for (uint32_t k = g + 1; k < s.f.size(); ++k)
            if (s.f[k].grp == g + 1) {
                R.lo[k] = elo;
                R.n[k] = em;
            }
    }
}
// Whether the pipeline moves a schema's element rows: groups at any depth,
// except a T x[N] group whose rows are another group's elements (its member
// rows would be N times a device total).
inline bool stage_groups_ok(const Schema &s) {
    for (uint32_t k = 0; k < s.f.size(); ++k) {
        const Field &f = s.f[k];
        if (!is_group(f) || f.kind != XDRG_K_FIXED) continue;
        for (uint32_t p = f.grp; p; p = s.f[p - 1].grp)
            if (s.f[p - 1].kind != XDRG_K_FIXED) return false;
    }
    return true;
}
// Elements of group g in a chunk (encode), from its first member's rows.
inline uint64_t group_elems(const Rows &R, uint32_t g) { return R.n[g + 1]; }

// Bound on a chunk's XDR bytes (conditional fields may take some away).
inline uint64_t bound_xdr(const Schema &s, bool framed, uint64_t m, const xdrg_column *cols, const Rows &R,
                          uint32_t byref = 0) {
    uint64_t b = m * (framed ? 4 : 0);
    for (uint32_t k = 0; k < s.f.size(); ++k) {
        const Field &f = s.f[k];
        if (k + 1 == byref) {   // by reference: the length word stays, the payload goes out on its own
            b += 4 * R.n[k];
        } else if (is_group(f)) {   // a count word, or a bool per element and the closing one
            if (f.kind == XDRG_K_DYNAMIC) b += 4 * R.n[k];
            if (f.kind == XDRG_K_LIST) b += 4 * R.n[k] + 4 * group_elems(R, k);
        } else if (f.kind != XDRG_K_DYNAMIC) {
            b += (uint64_t)f.xbytes * R.n[k];
        } else {
            const uint64_t *o = cols[k].offsets;
            b += R.n[k] * (4 + (f.xsz == 1 ? 3 : 0)) + (o[R.lo[k] + R.n[k]] - o[R.lo[k]]) * f.xsz;
        }
    }
    return b;
}

// A region's host span over `rows` rows (0 rows: nothing).
inline uint64_t region_span(const Region &g, uint64_t rows) {
    return rows ? (uint64_t)g.stride * (rows - 1) + g.row_end : 0;
}
inline uint32_t region_field0(const Region &g) { return g.fields.front(); }

// ---------------------------------------------------------------------------
// encode
// ---------------------------------------------------------------------------
struct EncPlan {
    const Schema &s;
    const xdrg_column *cols;
    uint64_t n;
    bool framed, want_rec;
    std::vector<Region> regs;
    uint32_t byref = 0;   // 1 + the field encoded by reference (its values never move), or 0
};

inline void enc_layout(const EncPlan &p, uint64_t lo, uint64_t m, Layout &L, Rows &R) {
    const Schema &s = p.s;
    Bump b;
    L.lo = lo;
    L.m = m;
    chunk_rows(s, p.cols, lo, m, R);
    L.reg.assign(p.regs.size(), 0);
    for (size_t r = 0; r < p.regs.size(); ++r) {
        const Region &g = p.regs[r];
        const uint32_t k0 = region_field0(g);
        const uint8_t *h = g.base + (uint64_t)g.stride * R.lo[k0];
        L.reg[r] = b.take(region_span(g, R.n[k0]), (uintptr_t)h);
    }
    L.val.assign(s.f.size(), 0);
    L.off.assign(s.f.size(), 0);
    L.vcap.assign(s.f.size(), 0);
    for (uint32_t k = 0; k < s.f.size(); ++k) {
        const Field &f = s.f[k];
        if (is_group(f)) {   // the group's element offsets per row (record, or parent element)
            if (f.kind != XDRG_K_FIXED)
                L.off[k] = b.take((R.n[k] + 1) * 8, (uintptr_t)(p.cols[k].offsets + R.lo[k]));
            continue;
        }
        if (f.kind != XDRG_K_DYNAMIC) continue;
        const uint64_t a = p.cols[k].offsets[R.lo[k]], e = p.cols[k].offsets[R.lo[k] + R.n[k]];
        if (k + 1 != p.byref) {
            L.vcap[k] = e - a;
            L.val[k] = b.take((e - a) * f.nsz, (uintptr_t)((const uint8_t *)p.cols[k].data + a * f.nsz));
        }
        L.off[k] = b.take((R.n[k] + 1) * 8, (uintptr_t)(p.cols[k].offsets + R.lo[k]));
    }
    L.xcap = bound_xdr(s, p.framed, m, p.cols, R, p.byref);
    L.xdr = b.take(L.xcap);
    L.rec = (p.want_rec || s.var_size) ? b.take((m + 1) * 8) : 0;
    L.ref = p.byref ? b.take(m * 8) : 0;
    L.need = b.used;
}

// Dynamic offsets (and group element offsets) must not decrease over the
// batch (the device call has the same precondition); the pipeline checks the
// ends it cuts at.
inline bool dyn_offsets_sane(const Schema &s, const xdrg_column *cols, uint64_t n) {
    Rows R;
    R.lo.assign(s.f.size(), 0);
    R.n.assign(s.f.size(), n);
    for (uint32_t g = 0; g < s.f.size(); ++g) {   // each group's range before its members' rows come from it
        const Field &f = s.f[g];
        if (!is_group(f)) continue;
        if (f.kind != XDRG_K_FIXED && cols[g].offsets[R.lo[g] + R.n[g]] < cols[g].offsets[R.lo[g]]) return false;
        const uint64_t elo = f.kind == XDRG_K_FIXED ? R.lo[g] * f.count : cols[g].offsets[R.lo[g]];
        const uint64_t em = f.kind == XDRG_K_FIXED ? R.n[g] * f.count : cols[g].offsets[R.lo[g] + R.n[g]] - elo;
        for (uint32_t k = g + 1; k < s.f.size(); ++k)
            if (s.f[k].grp == g + 1) {
                R.lo[k] = elo;
                R.n[k] = em;
            }
    }
    for (uint32_t k = 0; k < s.f.size(); ++k)
        if (!is_group(s.f[k]) && s.f[k].kind == XDRG_K_DYNAMIC &&
            cols[k].offsets[R.lo[k] + R.n[k]] < cols[k].offsets[R.lo[k]])
            return false;
    return true;
}

// Largest record count from lo whose layout fits `cap` bytes: first guess
// from the batch's average record, then shrink.  Returns 0 when one record
// does not fit (the caller grows the ring).
template <class LayoutFn>
uint64_t fit_chunk(uint64_t lo, uint64_t n, uint64_t guess, uint64_t cap, LayoutFn &&lay, Layout &L) {
    uint64_t m = std::min<uint64_t>(n - lo, std::max<uint64_t>(guess, 1));
    for (;;) {
        lay(lo, m, L);
        if (L.need <= cap) return m;
        if (m == 1) return 0;
        uint64_t nm = (uint64_t)((double)m * (double)cap / (double)L.need * 0.97);
        if (nm >= m) nm = m - 1;
        if (nm > 256) nm &= ~(uint64_t)63;
        m = std::max<uint64_t>(nm, 1);
    }
}

// Bytes per record of a batch, averaged (chunk-size guess).
inline double enc_avg_bytes(const EncPlan &p) {
    if (!p.n) return 1.0;
    Layout L;
    Rows R;
    enc_layout(p, 0, p.n, L, R);
    return (double)L.need / (double)p.n;
}

// A chunk in flight.
struct Flight {
    uint32_t slot;
    Layout L;
    Rows R;
    std::vector<uint64_t> base;   // decode: per field, rows / values before this chunk (dynamic: values,
                                  // group: elements)
    std::vector<uint64_t> cap;    // decode: per field, device capacity granted to the chunk (values / elements)
};

template <class X>
struct Stager {
    X &x;
    // pending CPU copy-outs of each slot's bounce buffer (D2H into pageable memory)
    struct Out {
        uint8_t *host;
        const uint8_t *src;
        uint64_t width, rows, hpitch, spitch;
    };
    std::vector<Out> outs[kMaxSlots];
    bool busy[kMaxSlots] = {};

    explicit Stager(X &e) : x(e) {}

    // Slot s reusable: its last D2H landed and the bounce copies ran.
    int acquire(uint32_t s) {
        if (!busy[s]) return XDRG_OK;
        int rc = x.wait_slot(s);
        if (rc) return rc;
        for (const Out &o : outs[s])
            for (uint64_t r = 0; r < o.rows; ++r) std::memcpy(o.host + r * o.hpitch, o.src + r * o.spitch, o.width);
        outs[s].clear();
        busy[s] = false;
        return XDRG_OK;
    }
    int drain() {
        for (uint32_t s = 0; s < x.nslots(); ++s) {
            const int rc = acquire(s);
            if (rc) return rc;
        }
        return XDRG_OK;
    }
    uint8_t *bounce_of(uint32_t s, const uint8_t *dev) { return x.bounce(s) + (dev - x.slot(s)); }

    int h2d(uint32_t s, uint8_t *dev, const void *host, uint64_t bytes) {
        if (!bytes) return XDRG_OK;
        if (x.pinned(host, bytes)) return x.dma_h2d(dev, host, bytes);
        uint8_t *bb = x.bounce(s);
        if (!bb) return XDRG_E_NOMEM;
        uint8_t *b = bounce_of(s, dev);
        std::memcpy(b, host, bytes);
        return x.dma_h2d(dev, b, bytes);
    }
    int d2h(uint32_t s, void *host, const uint8_t *dev, uint64_t bytes) {
        busy[s] = true;
        if (!bytes) return XDRG_OK;
        if (x.pinned(host, bytes)) return x.dma_d2h(host, dev, bytes);
        if (!x.bounce(s)) return XDRG_E_NOMEM;
        uint8_t *b = bounce_of(s, dev);
        outs[s].push_back({(uint8_t *)host, b, bytes, 1, 0, 0});
        return x.dma_d2h(b, dev, bytes);
    }
    int d2h_2d(uint32_t s, uint8_t *host, uint64_t pitch, const uint8_t *dev, uint64_t width, uint64_t rows) {
        busy[s] = true;
        if (!rows || !width) return XDRG_OK;
        const uint64_t span = pitch * (rows - 1) + width;
        if (x.pinned(host, span)) return x.dma_d2h_2d(host, pitch, dev, pitch, width, rows);
        if (!x.bounce(s)) return XDRG_E_NOMEM;
        uint8_t *b = bounce_of(s, dev);
        outs[s].push_back({host, b, width, rows, pitch, pitch});
        return x.dma_d2h_2d(b, pitch, dev, pitch, width, rows);
    }
    // decoded fixed columns of `rows` rows from row `first` (regions of one row space)
    int d2h_region(uint32_t s, const Region &g, uint64_t first, const uint8_t *dev, uint64_t rows) {
        uint8_t *h = (uint8_t *)g.base + (uint64_t)g.stride * first;
        if (g.full) return d2h(s, h, dev, (uint64_t)g.stride * rows);
        for (auto &sg : g.segs) {
            const int rc = d2h_2d(s, h + sg.first, (uint64_t)g.stride, dev + sg.first, sg.second - sg.first, rows);
            if (rc) return rc;
        }
        return XDRG_OK;
    }
};

#define HS_TRY(x)                 \
    do {                          \
        const int rc_ = (x);      \
        if (rc_) return rc_;      \
    } while (0)

// Encode n host records into the host stream `out` (xdrg_encode_batch
// contract).  Chunk results arrive in record order, so chunk k's stream
// bytes land at the sum of the earlier chunks' sizes and its record offsets
// are rebased by it.  A variable-size batch that overruns out_cap keeps
// sizing the remaining chunks and returns XDRG_E_CAPACITY with the bytes it
// needs (the chunks before the overrun have been written).  Repeated groups:
// a chunk moves its records' elements with them (the members' rows between
// the group offsets of its first and last record, rebased to the chunk).
// By reference (byref = 1 + field, xdrg_encode_batch_shallow): that field's
// values stay on the host — only its offsets cross — and splice (host, n)
// receives each record's splice position, rebased like its record offset.
template <class X>
int stage_encode(X &x, const Schema &s, const xdrg_column *cols, uint64_t n, uint8_t *out, uint64_t out_cap,
                 uint64_t *rec_offsets, uint32_t flags, uint64_t *out_len, uint32_t byref = 0,
                 uint64_t *splice = nullptr) {
    const bool framed = flags & XDRG_FRAME_RM;
    EncPlan p{s, cols, n, framed, rec_offsets != nullptr, {}, byref};
    HS_TRY(build_regions(s, cols, p.regs));
    if (!dyn_offsets_sane(s, cols, n)) return XDRG_E_INVAL;
    const uint64_t stride = s.fixed_part + (framed ? 4 : 0);
    if (!s.var_size) {
        const uint64_t total = n * stride;
        if (n && total / n != stride) return XDRG_E_INVAL;
        if (out_len) *out_len = total;
        if (total > out_cap) return XDRG_E_CAPACITY;
    }
    if (n == 0) {
        if (rec_offsets) rec_offsets[0] = 0;
        if (out_len) *out_len = 0;
        return XDRG_OK;
    }
    Stager<X> st(x);
    Rows Rl;   // rows of the layout being sized
    auto lay = [&](uint64_t lo, uint64_t m, Layout &L) { enc_layout(p, lo, m, L, Rl); };
    uint64_t guess = (uint64_t)((double)x.slot_bytes() / enc_avg_bytes(p));
    std::deque<Flight> q;
    uint64_t base = 0;   // stream bytes of the retired chunks
    bool over = false;
    // D2H of the oldest chunk in flight (its kernels done for a variable-size batch)
    auto retire = [&]() -> int {
        Flight &f = q.front();
        const uint32_t s_ = f.slot;
        const Layout &L = f.L;
        uint64_t size = L.m * stride;
        if (s.var_size) {
            uint64_t w[2];
            HS_TRY(x.wait_kernel(s_, w));
            size = w[0];
        }
        if (!over && base + size > out_cap) over = true;
        HS_TRY(x.d2h_begin(s_));
        if (!over) {
            uint8_t *slot = x.slot(s_);
            HS_TRY(st.d2h(s_, out + base, slot + L.xdr, size));
            if (rec_offsets) {
                HS_TRY(x.add_u64(1, (uint64_t *)(slot + L.rec), L.m + 1, base));
                HS_TRY(st.d2h(s_, rec_offsets + L.lo, slot + L.rec, (L.m + 1) * 8));
            }
            if (byref) {
                HS_TRY(x.add_pos((uint64_t *)(slot + L.ref), L.m, base));
                HS_TRY(st.d2h(s_, splice + L.lo, slot + L.ref, L.m * 8));
            }
        } else {
            st.busy[s_] = true;
        }
        HS_TRY(x.d2h_done(s_));
        base += size;
        q.pop_front();
        return XDRG_OK;
    };
    uint64_t lo = 0;
    for (uint64_t k = 0; lo < n; ++k) {
        Flight f;
        f.slot = (uint32_t)(k % x.nslots());
        uint64_t m = fit_chunk(lo, n, guess, x.slot_bytes(), lay, f.L);
        if (!m) {   // one record exceeds a slot: let the ring drain and grow it
            while (!q.empty()) HS_TRY(retire());
            HS_TRY(st.drain());
            HS_TRY(x.grow(up(f.L.need + f.L.need / 4, 1 << 20)));
            m = fit_chunk(lo, n, 1, x.slot_bytes(), lay, f.L);
            if (!m) return XDRG_E_NOMEM;
        }
        f.R = Rl;   // (fit_chunk's last layout is the chunk's)
        guess = std::max<uint64_t>(m, 1);
        const uint32_t s_ = f.slot;
        while (!q.empty() && q.front().slot == s_) HS_TRY(retire());   // a one-slot ring: the chunk before leaves first
        HS_TRY(st.acquire(s_));
        uint8_t *slot = x.slot(s_);
        const Layout &L = f.L;
        const Rows &R = f.R;
        std::vector<xdrg_column> dc(s.f.size());
        for (size_t r = 0; r < p.regs.size(); ++r) {
            const Region &g = p.regs[r];
            const uint32_t k0 = region_field0(g);
            HS_TRY(st.h2d(s_, slot + L.reg[r], g.base + (uint64_t)g.stride * R.lo[k0], region_span(g, R.n[k0])));
            for (uint32_t k2 : g.fields) {
                dc[k2].data = slot + L.reg[r] + ((const uint8_t *)cols[k2].data - g.base);
                dc[k2].stride = cols[k2].stride;
            }
        }
        for (uint32_t k2 = 0; k2 < s.f.size(); ++k2) {
            const Field &fd = s.f[k2];
            if (is_group(fd)) {
                if (fd.kind != XDRG_K_FIXED) {
                    HS_TRY(st.h2d(s_, slot + L.off[k2], cols[k2].offsets + R.lo[k2], (R.n[k2] + 1) * 8));
                    dc[k2].offsets = (uint64_t *)(slot + L.off[k2]);
                }
                dc[k2].cap = group_elems(R, k2);
            } else if (fd.kind == XDRG_K_DYNAMIC) {
                const uint64_t a = cols[k2].offsets[R.lo[k2]];
                if (k2 + 1 != byref)
                    HS_TRY(st.h2d(s_, slot + L.val[k2], (const uint8_t *)cols[k2].data + a * fd.nsz, L.vcap[k2] * fd.nsz));
                HS_TRY(st.h2d(s_, slot + L.off[k2], cols[k2].offsets + R.lo[k2], (R.n[k2] + 1) * 8));
                dc[k2].data = k2 + 1 == byref ? nullptr : slot + L.val[k2];
                dc[k2].offsets = (uint64_t *)(slot + L.off[k2]);
                dc[k2].cap = L.vcap[k2];
            } else if (!fixed_elem_bytes(fd)) {
                dc[k2].data = slot;   // no bytes: any valid, aligned pointer
                dc[k2].stride = 0;
            }
        }
        HS_TRY(x.h2d_done(s_));
        HS_TRY(x.kernel_begin(s_));
        for (uint32_t k2 = 0; k2 < s.f.size(); ++k2) {   // offsets relative to the chunk's first value / element
            const Field &fd = s.f[k2];
            if (is_group(fd) && fd.kind != XDRG_K_FIXED && cols[k2].offsets[R.lo[k2]])
                HS_TRY(x.add_u64(0, dc[k2].offsets, R.n[k2] + 1, (uint64_t)0 - cols[k2].offsets[R.lo[k2]]));
            else if (!is_group(fd) && fd.kind == XDRG_K_DYNAMIC && cols[k2].offsets[R.lo[k2]])
                HS_TRY(x.add_u64(0, dc[k2].offsets, R.n[k2] + 1, (uint64_t)0 - cols[k2].offsets[R.lo[k2]]));
        }
        HS_TRY(x.encode(s_, dc.data(), m, slot + L.xdr, L.xcap, L.rec ? (uint64_t *)(slot + L.rec) : nullptr,
                        flags & XDRG_FRAME_RM, byref, byref ? (uint64_t *)(slot + L.ref) : nullptr));
        HS_TRY(x.kernel_end(s_, nullptr, nullptr, nullptr, 0));
        q.push_back(std::move(f));
        // fixed-size chunks leave at once; a variable-size chunk waits for its
        // kernels while the next chunk's H2D and kernels are already queued
        while (q.size() > (s.var_size ? 1u : 0u)) HS_TRY(retire());
        lo += m;
    }
    while (!q.empty()) HS_TRY(retire());
    HS_TRY(st.drain());
    if (out_len) *out_len = base;
    return over ? XDRG_E_CAPACITY : XDRG_OK;
}

// ---------------------------------------------------------------------------
// decode
// ---------------------------------------------------------------------------
struct DecPlan {
    const Schema &s;
    const uint8_t *in;
    uint64_t in_len;
    const uint64_t *ro;   // record extents (n + 1) or NULL (fixed stride)
    uint64_t n;
    bool framed;
    xdrg_column *cols;
    std::vector<Region> regs;
    uint32_t byref = 0;   // 1 + the field decoded as a view (its values are never written), or 0
};

// The chunk's stream window: [min, max] of its record extents (rebased by
// the window start, rounded down to 16 relative to `in`), or the chunk's
// records at the fixed stride; clamped to in_len.
inline void dec_window(const DecPlan &p, uint64_t lo, uint64_t m, uint64_t &win, uint64_t &wlen) {
    uint64_t a, e;
    if (p.ro) {
        a = UINT64_MAX;
        e = 0;
        for (uint64_t i = lo; i <= lo + m; ++i) {
            a = std::min(a, p.ro[i]);
            e = std::max(e, p.ro[i]);
        }
    } else {
        const uint64_t stride = p.s.fixed_part + (p.framed ? 4 : 0);
        a = lo * stride;
        e = (lo + m) * stride;
    }
    a = std::min(a, p.in_len);
    if (p.ro) a &= ~(uint64_t)15;   // extents are rebased; a fixed stride is not
    e = std::min(e, p.in_len);
    win = a;
    wlen = e > a ? e - a : 0;
}

// Element rows a decode window may produce for group g: each element takes
// at least emin XDR bytes (a LIST's TRUE, the unconditional members); a
// group whose elements may be empty is bounded by its column's capacity.
inline uint64_t elem_bound(const Schema &s, const xdrg_column *cols, uint32_t g, uint64_t rows, uint64_t wlen) {
    const Field &f = s.f[g];
    if (f.kind == XDRG_K_FIXED) return rows * f.count;   // rows: records, or (nested) the parent's elements
    return f.emin ? wlen / f.emin + 1 : cols[g].cap;
}

inline void dec_layout(const DecPlan &p, uint64_t lo, uint64_t m, Layout &L) {
    const Schema &s = p.s;
    Bump b;
    L.lo = lo;
    L.m = m;
    dec_window(p, lo, m, L.win, L.wlen);
    L.xdr = b.take(L.wlen, (uintptr_t)(p.in + L.win));
    L.rec = p.ro ? b.take((m + 1) * 8, (uintptr_t)(p.ro + lo)) : 0;
    L.rows.assign(s.f.size(), m);
    for (uint32_t g = 0; g < s.f.size(); ++g)   // (pre-order: a group's rows are set before its members')
        if (is_group(s.f[g])) {
            const uint64_t eb = elem_bound(s, p.cols, g, L.rows[g], L.wlen);
            for (uint32_t k = g + 1; k < s.f.size(); ++k)
                if (s.f[k].grp == g + 1) L.rows[k] = eb;
        }
    L.reg.assign(p.regs.size(), 0);
    for (size_t r = 0; r < p.regs.size(); ++r) {
        const Region &g = p.regs[r];
        const uint64_t rows = L.rows[region_field0(g)];
        L.reg[r] = b.take(region_span(g, rows), g.space ? 0 : (uintptr_t)(g.base + (uint64_t)g.stride * lo));
    }
    L.val.assign(s.f.size(), 0);
    L.off.assign(s.f.size(), 0);
    L.vcap.assign(s.f.size(), 0);
    for (uint32_t k = 0; k < s.f.size(); ++k) {
        const Field &f = s.f[k];
        if (is_group(f)) {
            if (f.kind != XDRG_K_FIXED) L.off[k] = b.take((L.rows[k] + 1) * 8);
            continue;
        }
        if (f.kind != XDRG_K_DYNAMIC) continue;
        // a record's elements are bounded by the bytes its stream holds
        if (k + 1 != p.byref) {
            const uint64_t cap = L.wlen / f.xsz + 1;
            L.vcap[k] = cap;
            L.val[k] = b.take(cap * f.nsz);
        }
        L.off[k] = b.take((L.rows[k] + 1) * 8);
    }
    L.ref = p.byref ? b.take(m * 8) : 0;
    L.need = b.used;
}

// Decode n records of the host stream into host columns (xdrg_decode_batch
// contract).  A variable-size batch needs chunk k-1's element totals before
// chunk k's kernels run (its values land after them and its capacity is the
// host column's remainder); that wait overlaps chunk k's H2D.  Fixed-size
// chunks leave as soon as they are queued; their status is read when their
// slot comes round again.  The first chunk (in record order) that reports an
// error ends the walk: its first failing record is the batch's.  Repeated
// groups: a chunk's elements follow the previous chunks' (the group column's
// total per chunk), and its members' values follow theirs.  As a view
// (byref = 1 + field, xdrg_decode_batch_view): that field's offsets are
// written as for a copy, its values are not, and payload_pos (host, n)
// receives each payload's offset in `in` (the chunk's window start added).
template <class X>
int stage_decode(X &x, const Schema &s, const uint8_t *in, uint64_t in_len, const uint64_t *rec_offsets,
                 uint64_t n, xdrg_column *cols, uint32_t flags, uint64_t *first_bad, int *err,
                 uint32_t byref = 0, uint64_t *payload_pos = nullptr) {
    const bool framed = flags & XDRG_FRAME_RM;
    DecPlan p{s, in, in_len, rec_offsets, n, framed, cols, {}, byref};
    HS_TRY(build_regions(s, cols, p.regs));
    // the counted columns whose totals place the next chunk: dynamic fields
    // (their values) and DYNAMIC / LIST groups (their elements)
    std::vector<uint32_t> cnt;
    for (uint32_t k = 0; k < s.f.size(); ++k)
        if (s.f[k].kind == XDRG_K_DYNAMIC || (is_group(s.f[k]) && s.f[k].kind != XDRG_K_FIXED)) cnt.push_back(k);
    if (cnt.size() > 32) return XDRG_E_INVAL;
    if (first_bad) *first_bad = n;
    if (err) *err = XDRG_OK;
    if (n == 0) {
        for (uint32_t k : cnt) cols[k].offsets[0] = 0;
        return XDRG_OK;
    }
    Stager<X> st(x);
    auto lay = [&](uint64_t lo, uint64_t m, Layout &L) { dec_layout(p, lo, m, L); };
    uint64_t guess;
    {
        const uint64_t stride = s.fixed_part + (framed ? 4 : 0);
        double per = (double)std::max<uint64_t>(stride, 4);
        if (rec_offsets && rec_offsets[n] > rec_offsets[0]) per = (double)(rec_offsets[n] - rec_offsets[0]) / (double)n;
        per = per * (1.0 + (double)cnt.size()) + 24.0 * (double)cnt.size() + (rec_offsets ? 8.0 : 0.0);
        for (const Region &g : p.regs) per += (double)g.stride;
        guess = std::max<uint64_t>((uint64_t)((double)x.slot_bytes() / per), 1);
    }
    std::vector<uint64_t> next_base(s.f.size(), 0);   // values / elements of the chunks before the next one
    std::deque<Flight> q;                              // variable-size: the chunk whose kernels run
    std::deque<std::pair<uint32_t, uint64_t>> pend;   // fixed-size: (slot, first record) awaiting status
    uint64_t fb = n;
    int code = XDRG_OK;
    bool stop = false;
    auto status = [&](uint32_t s_, uint64_t lo_, uint64_t *w) -> int {
        HS_TRY(x.wait_kernel(s_, w));
        if (w[1] && !stop) {
            fb = lo_ + w[0];
            code = (int)w[1];
            stop = true;
        }
        return XDRG_OK;
    };
    // D2H of a chunk; tot[k] = its totals (values of a dynamic field, elements of a group)
    auto retire = [&](const Flight &f, const std::vector<uint64_t> &tot) -> int {
        const uint32_t s_ = f.slot;
        const Layout &L = f.L;
        uint8_t *slot = x.slot(s_);
        // rows of a field's column in this chunk and the first of them
        // (a T x[N] group's rows are records or T x[M] elements: stage_groups_ok)
        std::function<uint64_t(uint32_t)> rows_of = [&](uint32_t k) -> uint64_t {
            if (!s.f[k].grp) return L.m;
            const uint32_t g = s.f[k].grp - 1;
            return s.f[g].kind == XDRG_K_FIXED ? rows_of(g) * s.f[g].count : tot[g];
        };
        std::function<uint64_t(uint32_t)> first_of = [&](uint32_t k) -> uint64_t {
            if (!s.f[k].grp) return L.lo;
            const uint32_t g = s.f[k].grp - 1;
            return s.f[g].kind == XDRG_K_FIXED ? first_of(g) * s.f[g].count : f.base[g];
        };
        HS_TRY(x.d2h_begin(s_));
        for (size_t r = 0; r < p.regs.size(); ++r) {
            const uint32_t k0 = region_field0(p.regs[r]);
            HS_TRY(st.d2h_region(s_, p.regs[r], first_of(k0), slot + L.reg[r], rows_of(k0)));
        }
        for (uint32_t k : cnt) {   // a group's offsets: one per row of its own (records, or parent elements)
            const uint64_t rows = rows_of(k);
            const uint64_t first = first_of(k);
            HS_TRY(x.add_u64(1, (uint64_t *)(slot + L.off[k]), rows + 1, f.base[k]));
            HS_TRY(st.d2h(s_, cols[k].offsets + first, slot + L.off[k], (rows + 1) * 8));
            if (!is_group(s.f[k]) && k + 1 != byref)
                HS_TRY(st.d2h(s_, (uint8_t *)cols[k].data + f.base[k] * s.f[k].nsz, slot + L.val[k], tot[k] * s.f[k].nsz));
        }
        if (byref) {   // payload positions: window-relative on the device, stream offsets on the host
            HS_TRY(x.add_pos((uint64_t *)(slot + L.ref), L.m, L.win));
            HS_TRY(st.d2h(s_, payload_pos + L.lo, slot + L.ref, L.m * 8));
        }
        st.busy[s_] = true;
        return x.d2h_done(s_);
    };
    // the running variable-size chunk: status, totals (which place the next
    // chunk), then its D2H
    auto settle = [&]() -> int {
        const Flight &f = q.front();
        uint64_t w[2 + 32];
        HS_TRY(status(f.slot, f.L.lo, w));
        std::vector<uint64_t> tot(s.f.size(), 0);
        for (size_t i = 0; i < cnt.size(); ++i) {
            // a failing chunk's totals may not cover its valid prefix (a decode
            // stops at the error): it hands back every value / element it was granted
            const uint32_t k = cnt[i];
            tot[k] = k + 1 == byref ? (w[1] ? 0 : w[2 + i])   // (a view's values are never placed)
                                    : w[1] ? f.cap[k] : std::min(w[2 + i], f.cap[k]);
            next_base[k] = f.base[k] + tot[k];
        }
        HS_TRY(retire(f, tot));
        q.pop_front();
        return XDRG_OK;
    };
    uint64_t lo = 0;
    for (uint64_t k = 0; lo < n && !stop; ++k) {
        Flight f;
        f.slot = (uint32_t)(k % x.nslots());
        uint64_t m = fit_chunk(lo, n, guess, x.slot_bytes(), lay, f.L);
        if (!m) {   // one record exceeds a slot: let the ring drain and grow it
            while (!q.empty()) HS_TRY(settle());
            while (!pend.empty()) {
                uint64_t w[2];
                HS_TRY(status(pend.front().first, pend.front().second, w));
                pend.pop_front();
            }
            HS_TRY(st.drain());
            if (stop) break;
            HS_TRY(x.grow(up(f.L.need + f.L.need / 4, 1 << 20)));
            m = fit_chunk(lo, n, 1, x.slot_bytes(), lay, f.L);
            if (!m) return XDRG_E_NOMEM;
        }
        guess = std::max<uint64_t>(m, 1);
        const uint32_t s_ = f.slot;
        if (!pend.empty() && pend.front().first == s_) {   // the slot's last chunk: its status
            uint64_t w[2];
            HS_TRY(status(s_, pend.front().second, w));
            pend.pop_front();
            if (stop) break;
        }
        if (!q.empty() && q.front().slot == s_) {   // a one-slot ring: the chunk before leaves first
            HS_TRY(settle());
            if (stop) break;
        }
        HS_TRY(st.acquire(s_));
        uint8_t *slot = x.slot(s_);
        const Layout &L = f.L;
        HS_TRY(st.h2d(s_, slot + L.xdr, in + L.win, L.wlen));
        if (rec_offsets) HS_TRY(st.h2d(s_, slot + L.rec, rec_offsets + lo, (m + 1) * 8));
        HS_TRY(x.h2d_done(s_));
        if (!q.empty()) {   // the previous chunk's totals place this one
            HS_TRY(settle());
            if (stop) break;
        }
        std::vector<xdrg_column> dc(s.f.size());
        for (size_t r = 0; r < p.regs.size(); ++r) {
            const Region &g = p.regs[r];
            for (uint32_t k2 : g.fields) {
                dc[k2].data = slot + L.reg[r] + ((const uint8_t *)cols[k2].data - g.base);
                dc[k2].stride = cols[k2].stride;
            }
        }
        f.base.assign(s.f.size(), 0);
        f.cap.assign(s.f.size(), 0);
        for (uint32_t k2 = 0; k2 < s.f.size(); ++k2) {
            const Field &fd = s.f[k2];
            if (is_group(fd)) {   // elements: after the chunks before, within the window's bound
                if (fd.kind == XDRG_K_FIXED) {
                    f.cap[k2] = L.rows[k2] * fd.count;
                    dc[k2].cap = f.cap[k2];
                    continue;
                }
                f.base[k2] = next_base[k2];
                const uint64_t left = cols[k2].cap > f.base[k2] ? cols[k2].cap - f.base[k2] : 0;
                f.cap[k2] = std::min(left, L.rows[k2 + 1]);
                dc[k2].offsets = (uint64_t *)(slot + L.off[k2]);
                dc[k2].cap = f.cap[k2];
            } else if (k2 + 1 == byref) {   // a view: offsets only, no capacity
                f.base[k2] = next_base[k2];
                dc[k2].data = nullptr;
                dc[k2].offsets = (uint64_t *)(slot + L.off[k2]);
                dc[k2].cap = 0;
            } else if (fd.kind == XDRG_K_DYNAMIC) {
                f.base[k2] = next_base[k2];
                const uint64_t left = cols[k2].cap > f.base[k2] ? cols[k2].cap - f.base[k2] : 0;
                f.cap[k2] = std::min(left, L.vcap[k2]);
                dc[k2].data = slot + L.val[k2];
                dc[k2].offsets = (uint64_t *)(slot + L.off[k2]);
                dc[k2].cap = f.cap[k2];
            } else if (!fixed_elem_bytes(fd)) {
                dc[k2].data = slot;
                dc[k2].stride = 0;
            }
        }
        HS_TRY(x.kernel_begin(s_));
        if (rec_offsets && L.win) HS_TRY(x.add_u64(0, (uint64_t *)(slot + L.rec), m + 1, (uint64_t)0 - L.win));
        HS_TRY(x.decode(s_, slot + L.xdr, L.wlen, rec_offsets ? (uint64_t *)(slot + L.rec) : nullptr, m, dc.data(),
                        flags & XDRG_FRAME_RM, byref, byref ? (uint64_t *)(slot + L.ref) : nullptr));
        // totals: a dynamic field's offsets at its last row (a member's: at the
        // chunk's element total, read on the device), a group's at record m
        // (the element total is read on the device only when within the member's
        // laid-out rows: a failing decode may leave it anywhere, and then the
        // totals are the grants anyway)
        // (nested: a column whose rows are a DYNAMIC / LIST group's elements is
        // read at that group's total, an earlier entry's result word)
        std::vector<const uint64_t *> extra, index;
        std::vector<uint64_t> limit;
        std::vector<uint32_t> pos(s.f.size(), 0);   // counted field -> its entry
        for (uint32_t i = 0; i < cnt.size(); ++i) pos[cnt[i]] = i;
        for (uint32_t k2 : cnt) {
            const Field &fd = s.f[k2];
            const uint64_t *o = (const uint64_t *)(slot + L.off[k2]);
            limit.push_back(L.rows[k2]);
            uint32_t g = fd.grp;   // the nearest DYNAMIC / LIST ancestor whose elements index this column
            uint64_t mult = 1;
            while (g && s.f[g - 1].kind == XDRG_K_FIXED) {
                mult *= s.f[g - 1].count;
                g = s.f[g - 1].grp;
            }
            if (!g) {   // rows: records (times the T x[N] counts above it)
                extra.push_back(o + m * mult);
                index.push_back(nullptr);
            } else {    // rows: group g - 1's elements in this chunk (mult == 1: stage_groups_ok)
                extra.push_back(o);
                index.push_back(x.res_word(s_, pos[g - 1]));
            }
        }
        HS_TRY(x.kernel_end(s_, extra.data(), index.data(), limit.data(), (uint32_t)extra.size()));
        if (cnt.empty()) {
            HS_TRY(retire(f, std::vector<uint64_t>(s.f.size(), 0)));
            pend.push_back({s_, lo});
        } else {
            q.push_back(std::move(f));
        }
        lo += m;
    }
    while (!q.empty()) HS_TRY(settle());
    while (!pend.empty()) {
        uint64_t w[2];
        HS_TRY(status(pend.front().first, pend.front().second, w));
        pend.pop_front();
    }
    HS_TRY(st.drain());
    if (first_bad) *first_bad = fb;
    if (err) *err = code;
    return code;
}

// ---------------------------------------------------------------------------
// receive: a host socket buffer's record-mark walk, then (DECODE) every
// complete message decoded as one record, or (DEFRAME) the bodies assembled
// ---------------------------------------------------------------------------
// RpcMessageParserTCP.handleRead (rpc/RpcMessageParserTCP.java:44-61) walks
// the marks of the bytes a selector thread read, hands every complete message
// on (assembleXdr :109-140) and keeps the remainder (:57-60).  Here the host
// stream moves through the ring in windows; window k is scanned on the device
// (its complete messages, at most the rows its slot holds), its messages
// decoded from the same slot, and window k+1 starts at the first byte window k
// did not consume: its fresh bytes were copied to the next slot already
// (behind `H` bytes of room), and window k's unconsumed tail is copied device
// to device in front of them, so every stream byte crosses PCIe once.  A tail
// longer than the room restages the window from the host; a message longer
// than a window grows the ring.  A window starts at a message boundary, so it
// is as aligned on the device as the message is in the stream (XDR: 4 bytes;
// the parallel walk needs that, an odd-sized fragment before it means the
// serial walk).
enum RecvMode { RECV_SCAN = 0, RECV_DEFRAME = 1, RECV_DECODE = 2 };

// Schemas whose decode a receive window carries: repeated groups at any
// level the staging ring moves (stage_groups_ok) whose counted elements take
// at least one XDR byte each, so a window's bytes bound every level's element
// rows.
inline bool recv_groups_ok(const Schema &s) {
    if (!stage_groups_ok(s)) return false;
    for (const Field &f : s.f)
        if (is_group(f) && f.kind != XDRG_K_FIXED && f.emin == 0) return false;
    return true;
}

// Rows of field k's column for `msgs` messages in a receive window of W
// bytes: messages, or the elements of its group (FIXED: the group's rows x
// count; else at most one per emin bytes of the window, at any depth, as
// stage_decode's elem_bound).
inline uint64_t recv_rows_bound(const Schema &s, uint32_t k, uint64_t msgs, uint64_t W) {
    if (!s.f[k].grp) return msgs;
    const uint32_t g = s.f[k].grp - 1;
    const Field &gf = s.f[g];
    return gf.kind == XDRG_K_FIXED ? recv_rows_bound(s, g, msgs, W) * gf.count : W / gf.emin + 1;
}

struct RecvResult {
    uint64_t n_msgs = 0, consumed = 0, first_bad = 0, payload = 0;
    int err = XDRG_OK;
};

// mode RECV_SCAN: message offsets only; RECV_DEFRAME: bodies into the host
// payload (payload_cap; messages whose bodies do not fit stay undelivered,
// XDRG_E_CAPACITY); RECV_DECODE: each message one record of *sp into the
// host columns (xdrg_decode_batch's column contract, rows = messages).
// msg_offsets (host, nullable): stream offsets of the delivered messages and
// the end of the last (DEFRAME: body offsets in payload).
template <class X>
int stage_receive(X &x, int mode, const Schema *sp, const uint8_t *in, uint64_t len, uint64_t cap,
                  xdrg_column *cols, uint8_t *payload, uint64_t payload_cap, uint64_t *msg_offsets,
                  RecvResult &out, double col_budget = 2.0) {
    out = RecvResult();
    std::vector<Region> regs;
    // the counted columns (stage_decode's): dynamic fields (values) and
    // DYNAMIC / LIST groups (elements, whose member rows ride with the window)
    std::vector<uint32_t> dyn;
    uint64_t minmsg = 4;   // a mark
    if (mode == RECV_DECODE) {
        if (!recv_groups_ok(*sp)) return XDRG_E_INVAL;
        HS_TRY(build_regions(*sp, cols, regs));
        for (const Region &g : regs)
            if (!g.stride) return XDRG_E_INVAL;   // constant columns are encode-only
        for (uint32_t k = 0; k < sp->f.size(); ++k)
            if (sp->f[k].kind == XDRG_K_DYNAMIC || (is_group(sp->f[k]) && sp->f[k].kind != XDRG_K_FIXED))
                dyn.push_back(k);
        if (dyn.size() > 32) return XDRG_E_INVAL;
        minmsg += sp->min_xdr;
    }
    auto rows_in = [&](uint32_t k, uint64_t msgs, uint64_t W) { return recv_rows_bound(*sp, k, msgs, W); };
    // A repeated-group schema decodes in two halves (decode_count, then
    // decode_place): the columns are laid out for the window's counted rows
    // and values, not for the bounds above (for nested groups those reserve
    // several times the window), so a window can take most of its slot.  The
    // geometry then reserves col_budget column bytes per window byte; a
    // window whose columns need more delivers fewer messages.
    const bool two = mode == RECV_DECODE && sp->groups;
    const double kColBudget = col_budget > 0 ? col_budget : 2.0;
    if (msg_offsets) msg_offsets[0] = 0;
    if (cap == 0 || len < 4) return XDRG_E_INCOMPLETE;
    Stager<X> st(x);
    // window geometry for the ring's slot size (reserving every region's worst
    // alignment, so a window that fills G.rows rows fits): room H and fresh bytes F
    // (multiples of 16), the rows a window may deliver, and where the message
    // offsets, body offsets, bodies (DEFRAME) and columns (DECODE) sit
    struct Geo { uint64_t H, F, W, rows, offs, boffs, body, cols, need; };
    auto geo_for = [&](uint64_t F) {
        Geo g;
        g.F = F;
        g.H = std::max<uint64_t>(up(F / 8, 16), 64);
        g.W = g.H + g.F;
        g.rows = std::max<uint64_t>(g.W / minmsg, 1);
        Bump b;
        b.take(g.W);
        g.offs = b.take((g.rows + 1) * 8);
        g.boffs = b.take((g.rows + 1) * 8);
        g.body = mode == RECV_DEFRAME ? b.take(g.W) : 0;
        g.cols = b.used;
        if (two) {
            b.take((uint64_t)(kColBudget * (double)g.W));
        } else if (mode == RECV_DECODE) {
            // (a window's regions keep their host address modulo 16: the worst case)
            for (const Region &r : regs) b.take((uint64_t)r.stride * rows_in(region_field0(r), g.rows, g.W), 15);
            for (uint32_t k : dyn) {
                b.take((rows_in(k, g.rows, g.W) + 1) * 8);
                if (is_group(sp->f[k])) continue;
                b.take((g.W / sp->f[k].xsz + 1) * sp->f[k].nsz);
            }
        }
        g.need = b.used;
        return g;
    };
    auto fit_geo = [&]() {
        uint64_t F = std::max<uint64_t>(up(x.slot_bytes() / 2, 16), 16);
        Geo g = geo_for(F);
        while (g.need > x.slot_bytes() && F > 16) {
            uint64_t nf = up((uint64_t)((double)F * (double)x.slot_bytes() / (double)g.need * 0.97), 16);
            F = std::max<uint64_t>(std::min<uint64_t>(nf, F - 16), 16);
            g = geo_for(F);
        }
        return g;
    };
    Geo G = fit_geo();
    if (G.need > x.slot_bytes()) {
        HS_TRY(x.grow(up(G.need + G.need / 2, 1 << 12)));
        G = fit_geo();
        if (G.need > x.slot_bytes()) return XDRG_E_NOMEM;
    }

    struct Win {               // one window: its slot, where it sits, what it holds
        uint32_t slot = 0;
        uint64_t off = 0;      // slot offset of window byte 0
        uint64_t hpos = 0;     // host stream offset of window byte 0
        uint64_t wl = 0;       // bytes in the window
        uint64_t fresh_at = 0; // prefetched fresh bytes: host [fresh_at, fresh_end) at slot offset H
        uint64_t fresh_end = 0;
        bool prefetched = false;
    };
    struct Chunk {             // a decoded window awaiting its status
        uint32_t slot;
        uint64_t lo, m;        // first message index, messages
        Layout L;              // its columns in the slot
        std::vector<uint64_t> base, capg;
        uint64_t hpos;         // host stream offset of its window
        const uint64_t *doffs; // its messages' window offsets (device, in its slot)
        uint64_t *hoffs;       // host message offsets [lo, lo + m] (msg_offsets), or NULL
    };
    std::deque<Chunk> pend;
    bool stop = false;
    std::vector<uint64_t> next_base(mode == RECV_DECODE ? sp->f.size() : 0, 0);
    auto stage_fresh = [&](Win &w, uint64_t from) -> int {   // the F bytes after `from`, at slot offset H
        w.fresh_at = from;
        w.fresh_end = std::min(len, from + G.F);
        w.prefetched = true;
        return st.h2d(w.slot, x.slot(w.slot) + G.H, in + from, w.fresh_end - from);
    };
    // the oldest decoded window (its kernels are done): status, then its columns out
    auto settle = [&]() -> int {
        Chunk &c = pend.front();
        uint64_t w[2 + 32];
        HS_TRY(x.wait_kernel(c.slot, w));
        std::vector<uint64_t> tot(sp->f.size(), 0);   // per counted field: values / elements
        for (size_t i = 0; i < dyn.size(); ++i) {
            // a failing window's totals may not cover its valid prefix (a decode
            // stops at the error): it hands back every value it was granted
            const uint32_t k = dyn[i];
            tot[k] = w[1] ? c.capg[k] : std::min(w[2 + i], c.capg[k]);
            next_base[k] = c.base[k] + tot[k];
        }
        // rows of a field's column in this window and the first of them
        // (a group's own rows: messages, or its parent group's elements)
        std::function<uint64_t(uint32_t)> rows_of = [&](uint32_t k) -> uint64_t {
            if (!sp->f[k].grp) return c.m;
            const uint32_t g = sp->f[k].grp - 1;
            return sp->f[g].kind == XDRG_K_FIXED ? rows_of(g) * sp->f[g].count : tot[g];
        };
        std::function<uint64_t(uint32_t)> first_of = [&](uint32_t k) -> uint64_t {
            if (!sp->f[k].grp) return c.lo;
            const uint32_t g = sp->f[k].grp - 1;
            return sp->f[g].kind == XDRG_K_FIXED ? first_of(g) * sp->f[g].count : c.base[g];
        };
        uint8_t *slot = x.slot(c.slot);
        HS_TRY(x.d2h_begin(c.slot));
        for (size_t r = 0; r < regs.size(); ++r) {
            const uint32_t k0 = region_field0(regs[r]);
            HS_TRY(st.d2h_region(c.slot, regs[r], first_of(k0), slot + c.L.reg[r], rows_of(k0)));
        }
        for (uint32_t k : dyn) {
            const uint64_t rows = rows_of(k), first = first_of(k);
            HS_TRY(x.add_u64(1, (uint64_t *)(slot + c.L.off[k]), rows + 1, c.base[k]));
            HS_TRY(st.d2h(c.slot, cols[k].offsets + first, slot + c.L.off[k], (rows + 1) * 8));
            if (!is_group(sp->f[k]))
                HS_TRY(st.d2h(c.slot, (uint8_t *)cols[k].data + c.base[k] * sp->f[k].nsz, slot + c.L.val[k],
                              tot[k] * sp->f[k].nsz));
        }
        st.busy[c.slot] = true;
        HS_TRY(x.d2h_done(c.slot));
        if (w[1] && !stop) {   // the batch's first failing message (windows are in message order)
            stop = true;
            const uint64_t fb = c.lo + w[0];
            const int e = (int)w[1];
            // a bad message is delivered (and rejected: GARBAGE_ARGS, RpcDispatcher.java:126-131);
            // one that did not fit the columns is not
            const uint64_t upto = e == XDRG_E_CAPACITY ? fb : fb + 1;
            uint64_t end = 0;
            if (c.hoffs) {
                HS_TRY(st.acquire(c.slot));   // its message offsets have landed on the host
                end = c.hoffs[upto - c.lo];
            } else {   // the one offset it needs, from the slot
                HS_TRY(x.d2h_begin(c.slot));
                HS_TRY(st.d2h(c.slot, &end, (const uint8_t *)(c.doffs + (upto - c.lo)), 8));
                HS_TRY(x.d2h_done(c.slot));
                HS_TRY(st.acquire(c.slot));
                end += c.hpos;
            }
            out.first_bad = fb;
            out.err = e;
            out.n_msgs = upto;
            out.consumed = end;
        }
        pend.pop_front();
        return XDRG_OK;
    };

    // two halves: rows of field k's column for m messages whose counted
    // fields hold t[] values / elements, and the slot bytes of that layout
    std::function<uint64_t(uint32_t, uint64_t, const std::vector<uint64_t> &)> rows_counted =
        [&](uint32_t k, uint64_t m, const std::vector<uint64_t> &t) -> uint64_t {
        if (!sp->f[k].grp) return m;
        const uint32_t g = sp->f[k].grp - 1;
        return sp->f[g].kind == XDRG_K_FIXED ? rows_counted(g, m, t) * sp->f[g].count : t[g];
    };
    auto col_need = [&](uint64_t m, const std::vector<uint64_t> &t) -> uint64_t {
        Bump b;
        b.used = G.cols;
        for (const Region &r : regs) b.take((uint64_t)r.stride * rows_counted(region_field0(r), m, t), 15);
        for (uint32_t k2 : dyn) {
            b.take((rows_counted(k2, m, t) + 1) * 8);
            if (!is_group(sp->f[k2])) b.take(t[k2] * sp->f[k2].nsz);
        }
        return b.used;
    };

    const uint32_t S = x.nslots();
    Win cur;
    HS_TRY(st.acquire(0));
    HS_TRY(stage_fresh(cur, 0));
    cur.off = G.H;
    cur.wl = cur.fresh_end;
    HS_TRY(x.h2d_done(0));
    uint64_t pos = 0, k = 0, pbytes = 0, chunk_no = 0;
    int rc_final = XDRG_OK;
    for (;;) {
        Win nxt;
        nxt.slot = (uint32_t)((chunk_no + 1) % S);
        const uint64_t wend = cur.hpos + cur.wl;   // == cur's fresh end
        // the next window's fresh bytes go out before this walk when its slot is free already
        if (S >= 3 && wend < len) {
            HS_TRY(st.acquire(nxt.slot));
            HS_TRY(stage_fresh(nxt, wend));
        }
        uint8_t *slot = x.slot(cur.slot);
        uint64_t *doffs = (uint64_t *)(slot + G.offs), *dboffs = (uint64_t *)(slot + G.boffs);
        uint8_t *dbody = mode == RECV_DEFRAME ? slot + G.body : nullptr;
        const int bodies = mode == RECV_DEFRAME ? 2 : (mode == RECV_DECODE ? 1 : 0);
        uint64_t want0 = std::min<uint64_t>(cap - k, G.rows);
        uint64_t want = want0;
        uint64_t res[4] = {0, 0, 1, 0};
        HS_TRY(x.kernel_begin(cur.slot));
        HS_TRY(x.scan(cur.slot, slot + cur.off, cur.wl, want, doffs, bodies, dbody, dboffs, res));
        bool room_limited = false;
        if (mode == RECV_DEFRAME)
            while (res[0] > 1 && pbytes + res[3] > payload_cap) {   // the bodies that fit
                room_limited = true;
                want = std::min<uint64_t>(res[0] - 1, std::max<uint64_t>(1, (uint64_t)((double)res[0] *
                       (double)(payload_cap - pbytes) / (double)res[3])));
                HS_TRY(x.scan(cur.slot, slot + cur.off, cur.wl, want, doffs, bodies, dbody, dboffs, res));
            }
        // the previous window's kernels ran before this walk (one compute stream): settle it
        while (!pend.empty()) HS_TRY(settle());
        if (stop) break;
        uint64_t m = res[0], used = res[1];
        if (mode == RECV_DEFRAME && m && pbytes + res[3] > payload_cap) {
            rc_final = XDRG_E_CAPACITY;   // not one more body fits the payload buffer
            break;
        }
        // two halves: the window's counts, then (if its columns do not fit the
        // slot) fewer messages, or for one message a larger ring
        std::vector<uint64_t> tot2;
        uint64_t grow_to = 0;
        if (two && m) {
            for (;;) {
                if (res[2]) HS_TRY(x.offs_copy(dboffs, doffs, m + 1, cur.off));   // window -> slot offsets
                std::vector<uint64_t> t(dyn.size(), 0);
                uint64_t bad = m;
                HS_TRY(x.decode_count(cur.slot, res[2] ? slot : x.body(), res[2] ? cur.off + cur.wl : res[3], dboffs,
                                      m, res[2] ? XDRG_FRAME_RM : 0, t.data(), &bad));
                tot2.assign(sp->f.size(), 0);
                for (size_t i = 0; i < dyn.size(); ++i) tot2[dyn[i]] = t[i];
                const uint64_t need = col_need(m, tot2);
                if (need <= x.slot_bytes()) break;
                if (m == 1) {
                    grow_to = up(need + need / 2, 1 << 12);
                    break;
                }
                want = std::max<uint64_t>(1, std::min<uint64_t>(m - 1, (uint64_t)((double)m * 0.9 *
                       (double)(x.slot_bytes() - G.cols) / (double)(need - G.cols))));
                want0 = want;   // (fewer by choice: not the stream's end)
                HS_TRY(x.scan(cur.slot, slot + cur.off, cur.wl, want, doffs, bodies, dbody, dboffs, res));
                m = res[0];
                used = res[1];
            }
        }
        if (m == 0 || grow_to) {
            if (m == 0 && wend == len) break;   // the remainder is not a complete message: STOP (:51-53)
            // the message at pos is longer than a window (or its columns than a
            // slot): drain, grow the ring, restage
            HS_TRY(st.drain());
            HS_TRY(x.grow(std::max<uint64_t>(grow_to, up(x.slot_bytes() * 2, 1 << 12))));
            G = fit_geo();
            chunk_no = 0;
            cur = Win();
            cur.hpos = pos;
            cur.wl = std::min(len - pos, G.W);
            cur.fresh_end = pos + cur.wl;
            HS_TRY(st.h2d(0, x.slot(0), in + pos, cur.wl));
            HS_TRY(x.h2d_done(0));
            continue;
        }
        // deliver: message offsets, then the bodies or the decoded records
        const uint64_t lo = k;
        Chunk c;
        c.slot = cur.slot;
        c.lo = lo;
        c.m = m;
        c.hpos = cur.hpos;
        c.doffs = doffs;
        c.hoffs = msg_offsets ? msg_offsets + lo : nullptr;
        if (mode == RECV_DECODE) {
            Bump b;
            b.used = G.cols;
            c.L.reg.assign(regs.size(), 0);
            c.L.off.assign(sp->f.size(), 0);
            c.L.val.assign(sp->f.size(), 0);
            c.L.rows.assign(sp->f.size(), 0);
            c.base.assign(sp->f.size(), 0);
            c.capg.assign(sp->f.size(), 0);
            for (uint32_t k2 = 0; k2 < sp->f.size(); ++k2)
                c.L.rows[k2] = two ? rows_counted(k2, m, tot2) : rows_in(k2, m, cur.wl);
            std::vector<xdrg_column> dc(sp->f.size());
            for (size_t r = 0; r < regs.size(); ++r) {
                // (group members: the elements of the window's messages; a
                // member region's host address is not known yet, so no modulus)
                const uint32_t k0 = region_field0(regs[r]);
                c.L.reg[r] = b.take((uint64_t)regs[r].stride * c.L.rows[k0],
                                    regs[r].space ? 0 : (uintptr_t)(regs[r].base + (uint64_t)regs[r].stride * lo));
                for (uint32_t k2 : regs[r].fields) {
                    dc[k2].data = slot + c.L.reg[r] + ((const uint8_t *)cols[k2].data - regs[r].base);
                    dc[k2].stride = cols[k2].stride;
                }
            }
            for (uint32_t k2 = 0; k2 < sp->f.size(); ++k2) {
                const Field &fd = sp->f[k2];
                if (is_group(fd)) {   // elements: after the windows before, within the window's bound
                    if (fd.kind == XDRG_K_FIXED) {
                        c.capg[k2] = c.L.rows[k2] * fd.count;
                        dc[k2].cap = c.capg[k2];
                        continue;
                    }
                    c.L.off[k2] = b.take((c.L.rows[k2] + 1) * 8);
                    c.base[k2] = next_base[k2];
                    const uint64_t left = cols[k2].cap > c.base[k2] ? cols[k2].cap - c.base[k2] : 0;
                    c.capg[k2] = std::min(left, two ? tot2[k2] : c.L.rows[k2 + 1]);
                    dc[k2].offsets = (uint64_t *)(slot + c.L.off[k2]);
                    dc[k2].cap = c.capg[k2];
                } else if (fd.kind == XDRG_K_DYNAMIC) {
                    c.L.off[k2] = b.take((c.L.rows[k2] + 1) * 8);
                    // a window holds at most this many elements (two halves: its count)
                    const uint64_t vc = two ? tot2[k2] : cur.wl / fd.xsz + 1;
                    c.L.val[k2] = b.take(vc * fd.nsz);
                    c.base[k2] = next_base[k2];
                    const uint64_t left = cols[k2].cap > c.base[k2] ? cols[k2].cap - c.base[k2] : 0;
                    c.capg[k2] = std::min(left, vc);
                    dc[k2].data = slot + c.L.val[k2];
                    dc[k2].offsets = (uint64_t *)(slot + c.L.off[k2]);
                    dc[k2].cap = c.capg[k2];
                } else if (!fixed_elem_bytes(fd)) {
                    dc[k2].data = slot;
                    dc[k2].stride = 0;
                }
            }
            if (b.used > x.slot_bytes()) return XDRG_E_NOMEM;   // (the geometry reserved G.rows rows)
            // single fragments decode in place, record-marked (one mark per message,
            // GrizzlyRpcTransport.java:103-110); assembled bodies without marks
            if (two) {
                HS_TRY(x.decode_place(cur.slot, res[2] ? slot : x.body(), res[2] ? cur.off + cur.wl : res[3], dboffs,
                                      m, dc.data(), res[2] ? XDRG_FRAME_RM : 0, 0, nullptr));
            } else if (res[2]) {
                HS_TRY(x.offs_copy(dboffs, doffs, m + 1, cur.off));   // window -> slot offsets
                HS_TRY(x.decode(cur.slot, slot, cur.off + cur.wl, dboffs, m, dc.data(), XDRG_FRAME_RM, 0, nullptr));
            } else {
                HS_TRY(x.decode(cur.slot, x.body(), res[3], dboffs, m, dc.data(), 0, 0, nullptr));
            }
            // totals (stage_decode's): a column whose rows are messages (times
            // the T x[N] counts above it) at its last row; one whose rows are a
            // DYNAMIC / LIST group's elements at that group's window total, an
            // earlier entry's result word, read on the device when within the
            // column's laid-out rows
            std::vector<const uint64_t *> extra, index;
            std::vector<uint64_t> limit;
            std::vector<uint32_t> pos(sp->f.size(), 0);   // counted field -> its entry
            for (uint32_t i = 0; i < dyn.size(); ++i) pos[dyn[i]] = i;
            for (uint32_t k2 : dyn) {
                const uint64_t *o = (const uint64_t *)(slot + c.L.off[k2]);
                limit.push_back(c.L.rows[k2]);
                uint32_t g = sp->f[k2].grp;
                uint64_t mult = 1;
                while (g && sp->f[g - 1].kind == XDRG_K_FIXED) {
                    mult *= sp->f[g - 1].count;
                    g = sp->f[g - 1].grp;
                }
                extra.push_back(g ? o : o + m * mult);
                index.push_back(g ? x.res_word(cur.slot, pos[g - 1]) : nullptr);
            }
            HS_TRY(x.kernel_end(cur.slot, extra.data(), index.data(), limit.data(), (uint32_t)extra.size()));
            if (c.hoffs) {   // the caller's message offsets (without them the device copy stays
                HS_TRY(x.d2h_begin(cur.slot));   // window-relative: an error reads one entry, settle)
                HS_TRY(x.add_u64(1, doffs, m + 1, cur.hpos));
                HS_TRY(st.d2h(cur.slot, c.hoffs, (const uint8_t *)doffs, (m + 1) * 8));
                HS_TRY(x.d2h_done(cur.slot));
            }
            pend.push_back(std::move(c));
        } else {
            HS_TRY(x.kernel_end(cur.slot, nullptr, nullptr, nullptr, 0));
            HS_TRY(x.d2h_begin(cur.slot));
            if (mode == RECV_DEFRAME) {
                HS_TRY(st.d2h(cur.slot, payload + pbytes, dbody, res[3]));
                HS_TRY(x.add_u64(1, dboffs, m + 1, pbytes));
                if (c.hoffs) HS_TRY(st.d2h(cur.slot, c.hoffs, (const uint8_t *)dboffs, (m + 1) * 8));
                pbytes += res[3];
            } else if (c.hoffs) {
                HS_TRY(x.add_u64(1, doffs, m + 1, cur.hpos));
                HS_TRY(st.d2h(cur.slot, c.hoffs, (const uint8_t *)doffs, (m + 1) * 8));
            }
            st.busy[cur.slot] = true;
            HS_TRY(x.d2h_done(cur.slot));
        }
        k += m;
        pos += used;
        if (room_limited) { rc_final = XDRG_E_CAPACITY; break; }
        if (k == cap || pos == len || (wend == len && m < want0)) break;
        // the next window: this one's unconsumed tail, then the fresh bytes
        if (S == 1) {   // one slot: this window leaves first, the next restages from the host
            while (!pend.empty()) HS_TRY(settle());
            HS_TRY(st.drain());
            if (stop) break;
        }
        const uint64_t tail = wend - pos;
        if (S >= 2 && wend < len && !nxt.prefetched) {
            HS_TRY(st.acquire(nxt.slot));
            HS_TRY(stage_fresh(nxt, wend));
        }
        if (S >= 2 && tail <= G.H && (nxt.prefetched || wend == len)) {
            if (!nxt.prefetched) {   // the stream ends in this window: the tail alone
                HS_TRY(st.acquire(nxt.slot));
                nxt.fresh_at = nxt.fresh_end = wend;
            }
            HS_TRY(x.d2d(x.slot(nxt.slot) + G.H - tail, slot + cur.off + used, tail));
            nxt.off = G.H - tail;
            nxt.wl = tail + (nxt.fresh_end - nxt.fresh_at);
        } else {   // a long tail (or one slot): the window again from the host
            if (S >= 2) HS_TRY(st.acquire(nxt.slot));
            nxt.off = 0;
            nxt.wl = std::min(len - pos, G.W);
            HS_TRY(st.h2d(nxt.slot, x.slot(nxt.slot), in + pos, nxt.wl));
        }
        nxt.hpos = pos;
        HS_TRY(x.h2d_done(nxt.slot));
        cur = nxt;
        ++chunk_no;
    }
    while (!pend.empty()) HS_TRY(settle());
    HS_TRY(st.drain());
    if (!stop) {
        out.n_msgs = k;
        out.consumed = pos;
        out.first_bad = k;
    }
    out.payload = pbytes;
    if (out.err) return out.err;
    if (rc_final) return rc_final;
    return out.n_msgs ? XDRG_OK : XDRG_E_INCOMPLETE;
}

#undef HS_TRY

}  // namespace hs
}  // namespace xdrg
