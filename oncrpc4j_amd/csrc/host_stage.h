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
//   int encode(uint32_t s, const xdrg_column *dcols, uint64_t m, uint8_t *out, uint64_t cap,
//              uint64_t *rec, uint32_t flags);   // async; result word 0 = stream bytes
//   int decode(uint32_t s, const uint8_t *in, uint64_t len, const uint64_t *rec, uint64_t m,
//              xdrg_column *dcols, uint32_t flags);   // async; words 0 / 1 = first_bad / err
//   int kernel_end(uint32_t s, const uint64_t *const *extra, uint32_t nextra);
//                                                // result words 2.. = *extra[i]; event
//   int wait_kernel(uint32_t s, uint64_t *words); // host-blocking; words[0 .. 2 + nextra)
//   int d2h_begin(uint32_t s);                   // copy stream waits slot s's kernels
//   int dma_d2h(void *host, const uint8_t *dev, uint64_t bytes);
//   int dma_d2h_2d(void *host, uint64_t hpitch, const uint8_t *dev, uint64_t dpitch,
//                  uint64_t width, uint64_t rows);
//   int d2h_done(uint32_t s);                    // event: slot s's outputs have left
//   int grow(uint64_t slot_bytes);               // reallocate the ring (idle) for a larger chunk
// Every call returns XDRG_OK or an XDRG_E_* status.
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <algorithm>
#include <cstring>
#include <deque>
#include <vector>

#include "../../include/xdrg.h"

namespace xdrg {
namespace hs {

constexpr uint32_t kMaxSlots = 8;
constexpr uint64_t kSpanAlign = 256;   // every span starts on its own 256-B boundary ...
constexpr uint64_t kSpanSlack = 64;    // ... followed by slack the 16-B window loads may touch

// One schema field as the pipeline sees it (the compiled xdrg_schema's view).
struct Field {
    uint32_t type, kind, count;
    uint32_t nsz;      // native element bytes
    uint32_t xsz;      // XDR element bytes (1: opaque / string bytes)
    uint32_t xbytes;   // fixed fields: XDR bytes of the field
};
struct Schema {
    std::vector<Field> f;
    uint64_t fixed_part = 0;   // XDR bytes of the fixed fields
    bool var_size = false;     // dynamic or conditional fields
};

inline uint64_t up(uint64_t v, uint64_t a) { return (v + a - 1) / a * a; }

// Fixed-size columns that share one host window per record: the fields of an
// array-of-structs record (same stride, within one stride of the lowest),
// or one struct-of-arrays column, or a constant column (stride 0).
struct Region {
    const uint8_t *base = nullptr;   // lowest field address (row 0)
    int64_t stride = 0;              // bytes per row; 0 = constant (encode only)
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
    struct C { const uint8_t *p; int64_t st; uint64_t e; uint32_t k; };
    std::vector<C> v;
    for (uint32_t k = 0; k < s.f.size(); ++k) {
        const Field &f = s.f[k];
        if (f.kind == XDRG_K_DYNAMIC) continue;
        const uint64_t e = fixed_elem_bytes(f);
        if (!e) continue;   // T x[0]: no bytes on either side
        int64_t st = cols[k].stride;
        if (st == XDRG_STRIDE_CONST) st = 0;
        else if (st == 0) st = (int64_t)e;
        else if (st < 0 || (uint64_t)st < e) return XDRG_E_INVAL;
        v.push_back({(const uint8_t *)cols[k].data, st, e, k});
    }
    std::sort(v.begin(), v.end(), [](const C &a, const C &b) { return a.st != b.st ? a.st < b.st : a.p < b.p; });
    for (const C &c : v) {
        Region *r = out.empty() ? nullptr : &out.back();
        const bool joins = r && c.st && r->stride == c.st && c.p >= r->base &&
                           (uint64_t)(c.p - r->base) + c.e <= (uint64_t)c.st;
        if (!joins) {
            out.push_back(Region());
            r = &out.back();
            r->base = c.p;
            r->stride = c.st;
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
    std::vector<uint64_t> val, off, vcap;    // per field (dynamic): values / offsets offset, value capacity
    uint64_t xdr = 0, xcap = 0, rec = 0;     // stream span, its capacity, record offsets (m + 1)
    uint64_t win = 0, wlen = 0;              // decode: host window [win, win + wlen) of the stream
};

inline uint64_t bound_xdr(const Schema &s, bool framed, uint64_t m, const xdrg_column *cols, uint64_t lo,
                          uint64_t hi) {
    uint64_t b = m * (s.fixed_part + (framed ? 4 : 0));
    for (uint32_t k = 0; k < s.f.size(); ++k) {
        const Field &f = s.f[k];
        if (f.kind != XDRG_K_DYNAMIC) continue;
        b += m * (4 + (f.xsz == 1 ? 3 : 0)) + (cols[k].offsets[hi] - cols[k].offsets[lo]) * f.xsz;
    }
    return b;
}

// ---------------------------------------------------------------------------
// encode
// ---------------------------------------------------------------------------
struct EncPlan {
    const Schema &s;
    const xdrg_column *cols;
    uint64_t n;
    bool framed, want_rec;
    std::vector<Region> regs;
};

inline void enc_layout(const EncPlan &p, uint64_t lo, uint64_t m, Layout &L) {
    const Schema &s = p.s;
    Bump b;
    L.lo = lo;
    L.m = m;
    L.reg.assign(p.regs.size(), 0);
    for (size_t r = 0; r < p.regs.size(); ++r) {
        const Region &g = p.regs[r];
        const uint8_t *h = g.base + (uint64_t)g.stride * lo;
        L.reg[r] = b.take((uint64_t)g.stride * (m - 1) + g.row_end, (uintptr_t)h);
    }
    L.val.assign(s.f.size(), 0);
    L.off.assign(s.f.size(), 0);
    L.vcap.assign(s.f.size(), 0);
    for (uint32_t k = 0; k < s.f.size(); ++k) {
        if (s.f[k].kind != XDRG_K_DYNAMIC) continue;
        const uint64_t a = p.cols[k].offsets[lo], e = p.cols[k].offsets[lo + m];
        L.vcap[k] = e - a;
        L.val[k] = b.take((e - a) * s.f[k].nsz, (uintptr_t)((const uint8_t *)p.cols[k].data + a * s.f[k].nsz));
        L.off[k] = b.take((m + 1) * 8, (uintptr_t)(p.cols[k].offsets + lo));
    }
    L.xcap = bound_xdr(s, p.framed, m, p.cols, lo, lo + m);
    L.xdr = b.take(L.xcap);
    L.rec = (p.want_rec || s.var_size) ? b.take((m + 1) * 8) : 0;
    L.need = b.used;
}

// Dynamic offsets must not decrease over the batch (the device call has the
// same precondition); the pipeline checks the ends it cuts at.
inline bool dyn_offsets_sane(const Schema &s, const xdrg_column *cols, uint64_t lo, uint64_t hi) {
    for (uint32_t k = 0; k < s.f.size(); ++k)
        if (s.f[k].kind == XDRG_K_DYNAMIC && cols[k].offsets[hi] < cols[k].offsets[lo]) return false;
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
    enc_layout(p, 0, p.n, L);
    return (double)L.need / (double)p.n;
}

// A chunk in flight.
struct Flight {
    uint32_t slot;
    Layout L;
    std::vector<uint64_t> base;   // decode: per field, elements before this chunk (dynamic fields)
    std::vector<uint64_t> cap;    // decode: per field, device value capacity granted to the chunk
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
// needs (the chunks before the overrun have been written).
template <class X>
int stage_encode(X &x, const Schema &s, const xdrg_column *cols, uint64_t n, uint8_t *out, uint64_t out_cap,
                 uint64_t *rec_offsets, uint32_t flags, uint64_t *out_len) {
    const bool framed = flags & XDRG_FRAME_RM;
    EncPlan p{s, cols, n, framed, rec_offsets != nullptr, {}};
    HS_TRY(build_regions(s, cols, p.regs));
    if (!dyn_offsets_sane(s, cols, 0, n)) return XDRG_E_INVAL;
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
    auto lay = [&](uint64_t lo, uint64_t m, Layout &L) { enc_layout(p, lo, m, L); };
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
        guess = std::max<uint64_t>(m, 1);
        const uint32_t s_ = f.slot;
        while (!q.empty() && q.front().slot == s_) HS_TRY(retire());   // a one-slot ring: the chunk before leaves first
        HS_TRY(st.acquire(s_));
        uint8_t *slot = x.slot(s_);
        const Layout &L = f.L;
        std::vector<xdrg_column> dc(s.f.size());
        for (size_t r = 0; r < p.regs.size(); ++r) {
            const Region &g = p.regs[r];
            HS_TRY(st.h2d(s_, slot + L.reg[r], g.base + (uint64_t)g.stride * lo, (uint64_t)g.stride * (m - 1) + g.row_end));
            for (uint32_t k2 : g.fields) {
                dc[k2].data = slot + L.reg[r] + ((const uint8_t *)cols[k2].data - g.base);
                dc[k2].stride = cols[k2].stride;
            }
        }
        for (uint32_t k2 = 0; k2 < s.f.size(); ++k2) {
            const Field &fd = s.f[k2];
            if (fd.kind == XDRG_K_DYNAMIC) {
                const uint64_t a = cols[k2].offsets[lo];
                HS_TRY(st.h2d(s_, slot + L.val[k2], (const uint8_t *)cols[k2].data + a * fd.nsz, L.vcap[k2] * fd.nsz));
                HS_TRY(st.h2d(s_, slot + L.off[k2], cols[k2].offsets + lo, (m + 1) * 8));
                dc[k2].data = slot + L.val[k2];
                dc[k2].offsets = (uint64_t *)(slot + L.off[k2]);
                dc[k2].cap = L.vcap[k2];
            } else if (!fixed_elem_bytes(fd)) {
                dc[k2].data = slot;   // no bytes: any valid, aligned pointer
                dc[k2].stride = 0;
            }
        }
        HS_TRY(x.h2d_done(s_));
        HS_TRY(x.kernel_begin(s_));
        for (uint32_t k2 = 0; k2 < s.f.size(); ++k2)   // offsets relative to the chunk's first value
            if (s.f[k2].kind == XDRG_K_DYNAMIC && cols[k2].offsets[lo])
                HS_TRY(x.add_u64(0, dc[k2].offsets, m + 1, (uint64_t)0 - cols[k2].offsets[lo]));
        HS_TRY(x.encode(s_, dc.data(), m, slot + L.xdr, L.xcap, L.rec ? (uint64_t *)(slot + L.rec) : nullptr,
                        flags & XDRG_FRAME_RM));
        HS_TRY(x.kernel_end(s_, nullptr, 0));
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

inline void dec_layout(const DecPlan &p, uint64_t lo, uint64_t m, Layout &L) {
    const Schema &s = p.s;
    Bump b;
    L.lo = lo;
    L.m = m;
    dec_window(p, lo, m, L.win, L.wlen);
    L.xdr = b.take(L.wlen, (uintptr_t)(p.in + L.win));
    L.rec = p.ro ? b.take((m + 1) * 8, (uintptr_t)(p.ro + lo)) : 0;
    L.reg.assign(p.regs.size(), 0);
    for (size_t r = 0; r < p.regs.size(); ++r) {
        const Region &g = p.regs[r];
        L.reg[r] = b.take((uint64_t)g.stride * (m - 1) + g.row_end, (uintptr_t)(g.base + (uint64_t)g.stride * lo));
    }
    L.val.assign(s.f.size(), 0);
    L.off.assign(s.f.size(), 0);
    L.vcap.assign(s.f.size(), 0);
    for (uint32_t k = 0; k < s.f.size(); ++k) {
        const Field &f = s.f[k];
        if (f.kind != XDRG_K_DYNAMIC) continue;
        // a record's elements are bounded by the bytes its stream holds
        const uint64_t cap = L.wlen / f.xsz + 1;
        L.vcap[k] = cap;
        L.val[k] = b.take(cap * f.nsz);
        L.off[k] = b.take((m + 1) * 8);
    }
    L.need = b.used;
}

// Decode n records of the host stream into host columns (xdrg_decode_batch
// contract).  A variable-size batch needs chunk k-1's element totals before
// chunk k's kernels run (its values land after them and its capacity is the
// host column's remainder); that wait overlaps chunk k's H2D.  Fixed-size
// chunks leave as soon as they are queued; their status is read when their
// slot comes round again.  The first chunk (in record order) that reports an
// error ends the walk: its first failing record is the batch's.
template <class X>
int stage_decode(X &x, const Schema &s, const uint8_t *in, uint64_t in_len, const uint64_t *rec_offsets,
                 uint64_t n, xdrg_column *cols, uint32_t flags, uint64_t *first_bad, int *err) {
    const bool framed = flags & XDRG_FRAME_RM;
    DecPlan p{s, in, in_len, rec_offsets, n, framed, cols, {}};
    HS_TRY(build_regions(s, cols, p.regs));
    std::vector<uint32_t> dyn;
    for (uint32_t k = 0; k < s.f.size(); ++k)
        if (s.f[k].kind == XDRG_K_DYNAMIC) dyn.push_back(k);
    if (dyn.size() > 32) return XDRG_E_INVAL;
    if (first_bad) *first_bad = n;
    if (err) *err = XDRG_OK;
    if (n == 0) {
        for (uint32_t k : dyn) cols[k].offsets[0] = 0;
        return XDRG_OK;
    }
    Stager<X> st(x);
    auto lay = [&](uint64_t lo, uint64_t m, Layout &L) { dec_layout(p, lo, m, L); };
    uint64_t guess;
    {
        const uint64_t stride = s.fixed_part + (framed ? 4 : 0);
        double per = (double)std::max<uint64_t>(stride, 4);
        if (rec_offsets && rec_offsets[n] > rec_offsets[0]) per = (double)(rec_offsets[n] - rec_offsets[0]) / (double)n;
        per = per * (1.0 + (double)dyn.size()) + 24.0 * (double)dyn.size() + (rec_offsets ? 8.0 : 0.0);
        for (const Region &g : p.regs) per += (double)g.stride;
        guess = std::max<uint64_t>((uint64_t)((double)x.slot_bytes() / per), 1);
    }
    std::vector<uint64_t> next_base(s.f.size(), 0);   // elements of the chunks before the next one
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
    // D2H of a chunk; `tot` = its element totals (variable-size)
    auto retire = [&](const Flight &f, const uint64_t *tot) -> int {
        const uint32_t s_ = f.slot;
        const Layout &L = f.L;
        uint8_t *slot = x.slot(s_);
        HS_TRY(x.d2h_begin(s_));
        for (size_t r = 0; r < p.regs.size(); ++r) {
            const Region &g = p.regs[r];
            uint8_t *h = (uint8_t *)g.base + (uint64_t)g.stride * L.lo;
            if (g.full) {
                HS_TRY(st.d2h(s_, h, slot + L.reg[r], (uint64_t)g.stride * L.m));
            } else {
                for (auto &sg : g.segs)
                    HS_TRY(st.d2h_2d(s_, h + sg.first, (uint64_t)g.stride, slot + L.reg[r] + sg.first,
                                     sg.second - sg.first, L.m));
            }
        }
        for (size_t i = 0; i < dyn.size(); ++i) {
            const uint32_t k = dyn[i];
            HS_TRY(x.add_u64(1, (uint64_t *)(slot + L.off[k]), L.m + 1, f.base[k]));
            HS_TRY(st.d2h(s_, cols[k].offsets + L.lo, slot + L.off[k], (L.m + 1) * 8));
            HS_TRY(st.d2h(s_, (uint8_t *)cols[k].data + f.base[k] * s.f[k].nsz, slot + L.val[k],
                          tot[i] * s.f[k].nsz));
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
        uint64_t tot[32];
        for (size_t i = 0; i < dyn.size(); ++i) {
            // a failing chunk's totals may not cover its valid prefix (a decode
            // stops at the error): it hands back every value it was granted
            tot[i] = w[1] ? f.cap[dyn[i]] : std::min(w[2 + i], f.cap[dyn[i]]);
            next_base[dyn[i]] = f.base[dyn[i]] + tot[i];
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
            if (fd.kind == XDRG_K_DYNAMIC) {
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
                        flags & XDRG_FRAME_RM));
        std::vector<const uint64_t *> extra;
        for (uint32_t k2 : dyn) extra.push_back((const uint64_t *)(slot + L.off[k2]) + m);   // element totals
        HS_TRY(x.kernel_end(s_, extra.data(), (uint32_t)extra.size()));
        if (dyn.empty()) {
            HS_TRY(retire(f, nullptr));
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

#undef HS_TRY

}  // namespace hs
}  // namespace xdrg
