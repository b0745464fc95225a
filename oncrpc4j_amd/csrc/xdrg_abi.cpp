// xdrg_abi.cpp — host side of libxdrgpu.so: the C-ABI of include/xdrg.h.
//
// Owns schema compilation (rpcgen field tape -> word program / record
// descriptors), per-call validation with the reference's error contract,
// path selection (streaming / word-map / record path), device workspace and
// per-kernel HIP-event timing.  Every entry point cites the reference
// interface it replaces in include/xdrg.h.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "host_stage.h"
#include "xdrg_internal.h"

using namespace xdrg;

// ---------------------------------------------------------------------------
// schema
// ---------------------------------------------------------------------------
struct xdrg_schema {
    std::vector<xdrg_field> f;
    std::vector<uint32_t> nsz;      // native element bytes per field
    std::vector<uint32_t> xsz;      // XDR element bytes per field (1 = bytes)
    std::vector<uint32_t> xbytes;   // fixed fields: XDR bytes of the field
    std::vector<uint32_t> wpos;     // fixed fields: XDR word position in the record
    std::vector<WordOp> ops;        // fixed schemas: one op per XDR word
    uint64_t fixed_size = 0;        // XDR bytes per record (no dynamic field), else 0
    uint64_t fixed_part = 0;        // XDR bytes of the fixed fields
    bool var_size = false;          // records differ in size (dynamic or conditional fields)
    // conditional fields (xdrg_cond), per field; cvals = all case values
    std::vector<uint32_t> cond, cneg, cfirst, cnum, slot;
    std::vector<int32_t> cvals;
    uint32_t ncond = 0;
    bool stream_types = true;       // every field is word-for-word (int/float/hyper/double/opaque%4)
    uint32_t nwords = 0;
    // repeated groups (include/xdrg.h): grp[k] = its immediate group's index
    // + 1 for a member, 0 otherwise; such schemas take the group kernels.
    // nested: a group sits inside another group's element
    std::vector<uint32_t> grp;
    uint32_t ngroups = 0;
    bool nested = false;
};

static uint32_t native_size(uint32_t t) {
    switch (t) {
    case XDRG_T_INT: case XDRG_T_UINT: case XDRG_T_ENUM: case XDRG_T_FLOAT: return 4;
    case XDRG_T_HYPER: case XDRG_T_UHYPER: case XDRG_T_DOUBLE: return 8;
    case XDRG_T_SHORT: return 2;
    case XDRG_T_BYTE: case XDRG_T_BOOL: case XDRG_T_OPAQUE: case XDRG_T_STRING: return 1;
    default: return 0;
    }
}
static uint32_t xdr_elem_size(uint32_t t) {
    switch (t) {
    case XDRG_T_HYPER: case XDRG_T_UHYPER: case XDRG_T_DOUBLE: return 8;
    case XDRG_T_OPAQUE: case XDRG_T_STRING: return 1;
    default: return native_size(t) ? 4 : 0;
    }
}
// (type, kind) pairs rpcgen emits against the Xdr surface (jrpcgen.java:661-739).
static bool field_valid(const xdrg_field &f) {
    if (!native_size(f.type) || f.kind > XDRG_K_DYNAMIC || f.reserved) return false;
    if (f.type == XDRG_T_BOOL && f.kind != XDRG_K_SCALAR) return false;
    if (f.type == XDRG_T_STRING && f.kind != XDRG_K_DYNAMIC) return false;
    if (f.type == XDRG_T_OPAQUE && f.kind == XDRG_K_SCALAR) return false;
    if (f.kind == XDRG_K_FIXED && f.count > 0x7fffffffu) return false;
    return true;
}
// The group at fs[k] spanning at most `lim` fields (depth 0 = top level,
// groups nest down to depth kGrpLevels - 1): grp[] of its members (its
// immediate members get k + 1, an inner group's members that group),
// *sized = an element encodes to >= 1 XDR word.
static bool group_valid(const xdrg_field *fs, size_t k, size_t lim, int depth, std::vector<uint32_t> &grp,
                        bool *sized) {
    const xdrg_field &g = fs[k];
    const uint32_t m = g.reserved;
    if (!(g.kind >= XDRG_K_FIXED && g.kind <= XDRG_K_LIST && m >= 1 && (size_t)m < lim) ||
        (g.kind == XDRG_K_FIXED && g.count > 0x7fffffffu) || (g.kind == XDRG_K_LIST && g.count))
        return false;
    bool sz = g.kind == XDRG_K_LIST;
    for (uint32_t j = 1; j <= m; ++j) {
        const xdrg_field &f = fs[k + j];
        grp[k + j] = (uint32_t)k + 1;
        if (f.type == XDRG_T_GROUP) {   // an array of structs / list inside the element
            bool s2 = false;
            if (depth + 1 >= kGrpLevels || !group_valid(fs, k + j, (size_t)m + 1 - j, depth + 1, grp, &s2) || !s2)
                return false;
            sz |= f.kind != XDRG_K_FIXED || f.count > 0;
            j += f.reserved;
            continue;
        }
        if (!field_valid(f)) return false;
        sz |= f.kind != XDRG_K_FIXED || f.count > 0;
    }
    *sized = sz;
    return true;
}

static uint8_t scalar_op(uint32_t t, bool second_half) {
    switch (t) {
    case XDRG_T_FLOAT: return OP_FLOAT;
    case XDRG_T_HYPER: case XDRG_T_UHYPER: return second_half ? OP_HYPER_LO : OP_HYPER_HI;
    case XDRG_T_DOUBLE: return second_half ? OP_DOUBLE_LO : OP_DOUBLE_HI;
    case XDRG_T_BOOL: return OP_BOOL;
    case XDRG_T_SHORT: return OP_SHORT;
    case XDRG_T_BYTE: return OP_BYTE;
    default: return OP_BSWAP;
    }
}

extern "C" int xdrg_schema_create_cond(const xdrg_field *fields, size_t nfields,
                                       const xdrg_cond *conds, size_t nconds, xdrg_schema **out) {
    if (!out) return XDRG_E_INVAL;
    if (nconds && !conds) return XDRG_E_INVAL;
    *out = nullptr;
    if (!fields || !nfields || nfields > (size_t)kMaxFields) return XDRG_E_INVAL;
    xdrg_schema *s = new (std::nothrow) xdrg_schema();
    if (!s) return XDRG_E_NOMEM;
    uint64_t words = 0;
    // repeated groups: {XDRG_T_GROUP, FIXED / DYNAMIC / LIST, count, m} and m
    // member fields of the base types or groups of them (down to kGrpLevels
    // levels), an element of at least one XDR word
    s->grp.assign(nfields, 0);
    for (size_t k = 0; k < nfields; ++k) {
        if (fields[k].type != XDRG_T_GROUP) continue;
        bool sized = false;
        if (!group_valid(fields, k, nfields - k, 0, s->grp, &sized) || !sized) { delete s; return XDRG_E_INVAL; }
        for (size_t j = k + 1; j <= k + fields[k].reserved; ++j)
            if (fields[j].type == XDRG_T_GROUP) s->nested = true;
        ++s->ngroups;
        k += fields[k].reserved;
    }
    for (size_t k = 0; k < nfields; ++k) {
        const xdrg_field &f = fields[k];
        if (f.type == XDRG_T_GROUP) {   // a record's elements: counted on the device
            s->f.push_back(f);
            s->nsz.push_back(0);
            s->xsz.push_back(0);
            s->wpos.push_back((uint32_t)words);
            s->xbytes.push_back(0);
            s->var_size = true;
            s->stream_types = false;
            continue;
        }
        if (!field_valid(f)) { delete s; return XDRG_E_INVAL; }
        s->f.push_back(f);
        s->nsz.push_back(native_size(f.type));
        s->xsz.push_back(xdr_elem_size(f.type));
        s->wpos.push_back((uint32_t)words);
        if (f.kind == XDRG_K_DYNAMIC) {
            s->var_size = true;
            s->xbytes.push_back(0);
            s->stream_types = false;
            continue;
        }
        const uint64_t cnt = f.kind == XDRG_K_FIXED ? f.count : 1;
        uint64_t xb;
        if (f.type == XDRG_T_OPAQUE) {
            xb = cnt + ((4 - (cnt & 3)) & 3);  // Xdr.java:776-781
            if (cnt & 3) s->stream_types = false;
            for (uint64_t i = 0; i < xb / 4 && words + i < kMaxWords; ++i) {
                const uint64_t rem = cnt - 4 * i;
                s->ops.push_back({OP_OPAQUE, (uint8_t)k, (uint8_t)(rem < 4 ? rem : 4), 0, (uint32_t)(4 * i)});
            }
        } else {
            const uint32_t xs = xdr_elem_size(f.type), ns = native_size(f.type);
            xb = cnt * xs;
            if (ns != xs) s->stream_types = false;  // bool/short/byte widen on the wire
            for (uint64_t e = 0; e < cnt && words + (e * xs) / 4 < kMaxWords; ++e) {
                s->ops.push_back({scalar_op(f.type, false), (uint8_t)k, 0, 0, (uint32_t)(e * ns)});
                if (xs == 8) s->ops.push_back({scalar_op(f.type, true), (uint8_t)k, 0, 0, (uint32_t)(e * ns)});
            }
        }
        if (xb > 0xffffffffull) { delete s; return XDRG_E_INVAL; }
        s->xbytes.push_back((uint32_t)xb);
        s->fixed_part += xb;
        words += xb / 4;
    }
    s->nwords = (uint32_t)(words < 0xffffffffull ? words : 0xffffffffull);
    s->cond.assign(nfields, 0);
    s->cneg.assign(nfields, 0);
    s->cfirst.assign(nfields, 0);
    s->cnum.assign(nfields, 0);
    s->slot.assign(nfields, 0);
    uint32_t nslots = 0;
    for (size_t i = 0; i < nconds; ++i) {
        const xdrg_cond &cd = conds[i];
        const size_t k = cd.field, d = cd.disc;
        // the discriminant: an earlier scalar int / unsigned / enum / bool
        // (RFC 4506 §4.15; jrpcgen.java:1240-1340, JrpcgenDeclaration INDIRECTION)
        if (k >= nfields || d >= k || s->cond[k] || cd.negate > 1 || (cd.nvalues && !cd.values) ||
            s->cvals.size() + cd.nvalues > (size_t)XDRG_MAX_CASES) {
            delete s;
            return XDRG_E_INVAL;
        }
        const xdrg_field &df = fields[d];
        if (df.kind != XDRG_K_SCALAR || (df.type != XDRG_T_INT && df.type != XDRG_T_UINT &&
                                         df.type != XDRG_T_ENUM && df.type != XDRG_T_BOOL)) {
            delete s;
            return XDRG_E_INVAL;
        }
        // with repeated groups a condition stays on its level: top-level on
        // top-level, a member on an earlier member of its own group (per element)
        if (s->grp[k] != s->grp[d]) {
            delete s;
            return XDRG_E_INVAL;
        }
        if (!s->slot[d]) {
            if (nslots == (uint32_t)XDRG_MAX_DISC) { delete s; return XDRG_E_INVAL; }
            s->slot[d] = ++nslots;
        }
        s->cond[k] = (uint32_t)d + 1;
        s->cneg[k] = cd.negate;
        s->cfirst[k] = (uint32_t)s->cvals.size();
        s->cnum[k] = cd.nvalues;
        for (uint32_t j = 0; j < cd.nvalues; ++j) s->cvals.push_back(cd.values[j]);
        ++s->ncond;
    }
    if (s->ncond) s->var_size = true;   // records of one schema now differ in shape
    s->fixed_size = s->var_size ? 0 : s->fixed_part;
    if (s->var_size || words > kMaxWords) s->ops.clear();
    *out = s;
    return XDRG_OK;
}

extern "C" int xdrg_schema_create(const xdrg_field *fields, size_t nfields, xdrg_schema **out) {
    return xdrg_schema_create_cond(fields, nfields, nullptr, 0, out);
}

extern "C" int xdrg_schema_destroy(xdrg_schema *s) {
    delete s;
    return XDRG_OK;
}

extern "C" uint64_t xdrg_schema_fixed_size(const xdrg_schema *s) { return s ? s->fixed_size : 0; }

// ---------------------------------------------------------------------------
// context
// ---------------------------------------------------------------------------
struct Timed {
    int kernel;
    hipEvent_t a, b;
    bool count;   // adds a launch (false: time only, e.g. the derived-count decode's rerun)
};

// Staging ring of the XDRG_HOST_PTRS calls (host_stage.h): device slots, a
// pinned bounce mirror, the copy / compute streams and per-slot events and
// status words.
struct StageRing {
    uint64_t want_slot = 64ull << 20;   // xdrg_ctx_host_staging
    uint32_t want_n = 4;
    uint8_t *dev = nullptr;
    uint64_t slot = 0;                  // allocated bytes per slot
    uint32_t n = 0;
    uint8_t *bounce = nullptr;          // pinned, n * slot (first pageable span)
    hipStream_t h2d = nullptr, d2h = nullptr, comp = nullptr;
    hipEvent_t e_h2d[hs::kMaxSlots] = {}, e_kern[hs::kMaxSlots] = {}, e_d2h[hs::kMaxSlots] = {};
    bool d2h_rec[hs::kMaxSlots] = {};
    uint32_t nres[hs::kMaxSlots] = {};
    uint64_t *d_res = nullptr, *h_res = nullptr;   // [kMaxSlots][kResWords]
};
constexpr uint32_t kResWords = 64;

struct xdrg_ctx {
    int device = 0;
    uint32_t flags = 0;
    hipStream_t stream = nullptr;
    // device status block: [0] error key, [1] frame-scan result
    unsigned long long *d_stat = nullptr;
    unsigned long long *h_stat = nullptr;  // pinned mirror
    uint64_t *d_ws = nullptr;
    size_t ws_words = 0;
    void *d_fws = nullptr;      // frame-walk workspace (kernels_frame.hip)
    size_t fws_bytes = 0;
    std::string err;
    std::deque<Timed> pending;
    std::vector<hipEvent_t> pool;
    uint64_t launches[XDRG_KERNEL_COUNT] = {};
    double ms[XDRG_KERNEL_COUNT] = {};
    Tuning tune;                // this context's kernel choices (xdrg_internal_tune)
    StageRing ring;             // XDRG_HOST_PTRS staging (allocated on first use)
    uint8_t *d_rx = nullptr;    // receive scratch: assembled message bodies / message offsets
    size_t rx_bytes = 0;
    uint64_t frame_spec_calls = 0;     // speculative word walks (xdrg_internal_stat 1)
    uint64_t frame_spec_gave_up = 0;   // ... of them walked again by the exact kernels (key 2)
    uint64_t frame_spec_rewalks = 0;   // super-chunks k_fs_fix walked again (key 3)
    uint64_t host_bounces = 0;         // XDRG_HOST_PTRS calls moved whole through device scratch (key 4)
    uint64_t recv_three_pass = 0;      // host receives by walk, deframe, decode (key 5)
};

static int hip_fail(xdrg_ctx *c, hipError_t e, const char *what) {
    if (c) {
        char buf[256];
        snprintf(buf, sizeof buf, "%s: %s", what, hipGetErrorString(e));
        c->err = buf;
    }
    return XDRG_E_HIP;
}
static int inval(xdrg_ctx *c, const char *what) {
    if (c) c->err = what;
    return XDRG_E_INVAL;
}
#define HIPCHK(c, x)                                       \
    do {                                                   \
        hipError_t e_ = (x);                               \
        if (e_ != hipSuccess) return hip_fail(c, e_, #x);  \
    } while (0)

// Every entry point that selects a device puts the caller thread's current
// device back on every return path: a JVM or torch caller driving another
// GPU must not find its device switched under it.
struct DeviceGuard {
    int prev = -1;
    DeviceGuard() {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
    DeviceGuard(const DeviceGuard &) = delete;
    DeviceGuard &operator=(const DeviceGuard &) = delete;
};

static hipEvent_t ev_get(xdrg_ctx *c) {
    if (!c->pool.empty()) {
        hipEvent_t e = c->pool.back();
        c->pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}
static void resolve_one(xdrg_ctx *c) {
    Timed t = c->pending.front();
    c->pending.pop_front();
    float ms = 0.f;
    if (hipEventSynchronize(t.b) == hipSuccess && hipEventElapsedTime(&ms, t.a, t.b) == hipSuccess) {
        c->launches[t.kernel] += t.count ? 1 : 0;
        c->ms[t.kernel] += ms;
    }
    c->pool.push_back(t.a);
    c->pool.push_back(t.b);
}

// Bracket one launch with timing events when XDRG_CTX_TIMING is set.
struct TimedLaunch {
    xdrg_ctx *c;
    int kernel;
    bool count;
    hipEvent_t a = nullptr, b = nullptr;
    TimedLaunch(xdrg_ctx *c_, int k, bool count_ = true) : c(c_), kernel(k), count(count_) {
        if (!(c->flags & XDRG_CTX_TIMING)) return;
        if (c->pending.size() > 4096) resolve_one(c);
        a = ev_get(c);
        b = ev_get(c);
        if (a) (void)hipEventRecord(a, c->stream);
    }
    ~TimedLaunch() {
        if (!a || !b) return;
        (void)hipEventRecord(b, c->stream);
        c->pending.push_back({kernel, a, b, count});
    }
};

extern "C" int xdrg_abi_version(void) { return XDRG_ABI_VERSION; }

int xdrg::set_tuning(Tuning &t, int key, long long v) {
    auto in = [&](long long lo, long long hi) { return v >= lo && v <= hi; };
    switch (key) {
    case 6: if (!in(0, 64) || (v & (v - 1))) return -1; t.force_g = (uint32_t)v; return 0;
    case 7: case 8: if (!in(4, 65536)) return -1; (key == 7 ? t.lane_bytes_enc : t.lane_bytes_dec) = (uint32_t)v; return 0;
    case 9: if (v != 0 && v != 4) return -1; t.rec = (int32_t)v; return 0;
    case 12: if (!in(1024, 98304) || (v & 15)) return -1; t.tile_bytes = (uint32_t)v; return 0;
    case 13: if (!in(0, 1ll << 31)) return -1; t.big_rec = (uint32_t)v; return 0;
    case 14: if (!in(1, 2)) return -1; t.framed = (int32_t)v; return 0;
    case 16: if (!in(0, 2)) return -1; t.words = (int32_t)v; return 0;
    case 20: if (!in(1, 2)) return -1; t.dec_lean = (int32_t)v; return 0;
    case 25: if (!in(1024, 32768) || (v & 15)) return -1; t.sweep_tile = (uint32_t)v; return 0;
    case 26: if (!in(0, 1)) return -1; t.stage_copy = (int32_t)v; return 0;
    case 29: if (!in(0, 1)) return -1; t.stride_check = (int32_t)v; return 0;
    case 31: if (!in(0, 2)) return -1; t.spec_sizes = (int32_t)v; return 0;
    case 32: if (v != 64 && v != 32 && v != 16 && v != 8 && v != 4) return -1; t.grp_enc_lanes = (int32_t)v; return 0;
    case 33: if (v && (!in(1024, 65536) || (v & 15))) return -1; t.grp_dec_tile = (int32_t)v; return 0;
    case 36: if (!in(1, 64)) return -1; t.emit_per = (int32_t)v; return 0;
    case 37: if (!in(0, 3)) return -1; t.xcd_order = (int32_t)v; return 0;
    case 38: if (v && !in(64, 4096)) return -1; t.grp_dec_el = (int32_t)v; return 0;
    case 41: if (v && (!in(4096, 49152) || (v & 15))) return -1; t.grp_enc_img = (int32_t)v; return 0;
    case 42: if (!in(0, 1)) return -1; t.recv_win = (int32_t)v; return 0;
    case 43: if (v != 0 && v != 1 && v != 2 && v != 4) return -1; t.grp_enc_split = (int32_t)v; return 0;
    case 44: if (!in(0, 1)) return -1; t.grp_dec_emap = (int32_t)v; return 0;
    case 45: if (!in(0, 1)) return -1; t.grp_enc_img_nest = (int32_t)v; return 0;
    case 47: if (!in(0, 1)) return -1; t.frame_spec = (int32_t)v; return 0;
    case 48: if (!in(0, 1)) return -1; t.emit_wave = (int32_t)v; return 0;
    case 49: if (!in(1, 100)) return -1; t.recv_budget = (int32_t)v; return 0;
    default: return -1;
    }
}

// Not part of include/xdrg.h: per-context kernel choices (xdrg_internal.h
// Tuning) for the parity tests, which force every production path, and for
// tools/sweep_rec.py.  Key 0 restores the defaults.
extern "C" int xdrg_internal_tune(xdrg_ctx *c, int key, long long value) {
    if (!c) return XDRG_E_INVAL;
    if (key == 0) { c->tune = Tuning(); return XDRG_OK; }
    return set_tuning(c->tune, key, value) ? XDRG_E_INVAL : XDRG_OK;
}

// Not part of include/xdrg.h: counters for the parity tests (1: speculative
// frame walks, 2: those that gave up and ran the exact kernels, 3: super-
// chunks their fix-up walked again, 4: host-memory calls that bounced whole
// through device scratch instead of streaming through the staging ring, 5:
// host receives that took three passes instead of the receive windows).
extern "C" long long xdrg_internal_stat(xdrg_ctx *c, int key) {
    if (!c) return -1;
    switch (key) {
    case 1: return (long long)c->frame_spec_calls;
    case 2: return (long long)c->frame_spec_gave_up;
    case 3: return (long long)c->frame_spec_rewalks;
    case 4: return (long long)c->host_bounces;
    case 5: return (long long)c->recv_three_pass;
    default: return -1;
    }
}

extern "C" const char *xdrg_status_string(int status) {
    switch (status) {
    case XDRG_OK: return "ok";
    case XDRG_E_SHORT: return "xdr stream too short";        // Xdr.java:1030
    case XDRG_E_CORRUPT: return "corrupted xdr";              // Xdr.java:1036
    case XDRG_E_FIXED_LEN: return "array size does not match protocol specification";  // :625-627
    case XDRG_E_CAPACITY: return "output buffer too small";
    case XDRG_E_FRAME: return "record mark does not frame the record";
    case XDRG_E_INVAL: return "invalid argument";
    case XDRG_E_HIP: return "HIP runtime error";
    case XDRG_E_NOMEM: return "out of memory";
    case XDRG_E_INCOMPLETE: return "not all fragments arrived";
    case XDRG_E_NEG_SIZE: return "negative array size";   // NegativeArraySizeException
    default: return "unknown status";
    }
}

extern "C" const char *xdrg_last_error(xdrg_ctx *c) { return c ? c->err.c_str() : ""; }

extern "C" int xdrg_ctx_create(int device, uint32_t flags, xdrg_ctx **out) {
    if (!out) return XDRG_E_INVAL;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return XDRG_E_HIP;
    DeviceGuard dg;
    if (hipSetDevice(device) != hipSuccess) return XDRG_E_HIP;
    xdrg_ctx *c = new (std::nothrow) xdrg_ctx();
    if (!c) return XDRG_E_NOMEM;
    c->device = device;
    c->flags = flags;
    if (hipMalloc(&c->d_stat, 64) != hipSuccess ||
        hipHostMalloc(&c->h_stat, 128, hipHostMallocDefault) != hipSuccess) {
        if (c->d_stat) (void)hipFree(c->d_stat);
        delete c;
        return XDRG_E_HIP;
    }
    *out = c;
    return XDRG_OK;
}

static void ring_free(xdrg_ctx *c);

extern "C" int xdrg_ctx_destroy(xdrg_ctx *c) {
    if (!c) return XDRG_OK;
    DeviceGuard dg;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    ring_free(c);
    while (!c->pending.empty()) resolve_one(c);
    for (hipEvent_t e : c->pool) (void)hipEventDestroy(e);
    if (c->d_ws) (void)hipFree(c->d_ws);
    if (c->d_fws) (void)hipFree(c->d_fws);
    if (c->d_rx) (void)hipFree(c->d_rx);
    if (c->d_stat) (void)hipFree(c->d_stat);
    if (c->h_stat) (void)hipHostFree(c->h_stat);
    delete c;
    return XDRG_OK;
}

extern "C" int xdrg_ctx_set_stream(xdrg_ctx *c, void *stream) {
    if (!c) return XDRG_E_INVAL;
    c->stream = (hipStream_t)stream;
    return XDRG_OK;
}

extern "C" int xdrg_ctx_kernel_stats(xdrg_ctx *c, int kernel, uint64_t *launches, double *total_ms) {
    if (!c || kernel < 0 || kernel >= XDRG_KERNEL_COUNT) return XDRG_E_INVAL;
    DeviceGuard dg;
    (void)hipSetDevice(c->device);
    while (!c->pending.empty()) resolve_one(c);
    if (launches) *launches = c->launches[kernel];
    if (total_ms) *total_ms = c->ms[kernel];
    return XDRG_OK;
}

extern "C" int xdrg_ctx_reset_stats(xdrg_ctx *c) {
    if (!c) return XDRG_E_INVAL;
    DeviceGuard dg;
    (void)hipSetDevice(c->device);
    while (!c->pending.empty()) resolve_one(c);
    for (int k = 0; k < XDRG_KERNEL_COUNT; ++k) { c->launches[k] = 0; c->ms[k] = 0; }
    return XDRG_OK;
}

static int ensure_ws(xdrg_ctx *c, size_t words) {
    if (words <= c->ws_words) return XDRG_OK;
    if (c->d_ws) {
        HIPCHK(c, hipStreamSynchronize(c->stream));
        HIPCHK(c, hipFree(c->d_ws));
        c->d_ws = nullptr;
        c->ws_words = 0;
    }
    HIPCHK(c, hipMalloc(&c->d_ws, words * sizeof(uint64_t)));
    c->ws_words = words;
    return XDRG_OK;
}

// Receive scratch (assembled bodies, message offsets): grown on demand, after
// the work that may still read it (the context's stream and its ring's
// compute stream) has finished.
static int ensure_rx(xdrg_ctx *c, size_t bytes) {
    if (bytes <= c->rx_bytes) return XDRG_OK;
    if (c->d_rx) {
        HIPCHK(c, hipStreamSynchronize(c->stream));
        if (c->ring.comp) HIPCHK(c, hipStreamSynchronize(c->ring.comp));
        HIPCHK(c, hipFree(c->d_rx));
        c->d_rx = nullptr;
        c->rx_bytes = 0;
    }
    const size_t want = bytes + bytes / 4 + 4096;
    HIPCHK(c, hipMalloc(&c->d_rx, want));
    c->rx_bytes = want;
    return XDRG_OK;
}

// ---------------------------------------------------------------------------
// helpers
// ---------------------------------------------------------------------------
static inline bool aligned(const void *p, uintptr_t a) { return ((uintptr_t)p & (a - 1)) == 0; }

static int64_t eff_stride(const xdrg_schema *s, size_t k, const xdrg_column &col) {
    if (col.stride == XDRG_STRIDE_CONST) return 0;   // every record reads element run 0
    if (col.stride) return col.stride;
    const uint64_t cnt = s->f[k].kind == XDRG_K_FIXED ? s->f[k].count : 1;
    return (int64_t)(s->nsz[k] * cnt);
}

// Native element alignment the kernels rely on (4-byte units for hyper/double).
static int check_columns(xdrg_ctx *c, const xdrg_schema *s, const xdrg_column *cols, uint64_t n,
                         bool decode) {
    if (!cols) return inval(c, "columns are NULL");
    for (size_t k = 0; k < s->f.size(); ++k) {
        const xdrg_field &f = s->f[k];
        if (f.type == XDRG_T_GROUP) {
            if (f.kind != XDRG_K_FIXED && !cols[k].offsets) return inval(c, "group column without offsets");
            continue;
        }
        if (s->grp[k] && f.kind != XDRG_K_DYNAMIC && !cols[k].data) return inval(c, "group member data is NULL");
        const uint32_t al = s->nsz[k] >= 4 ? 4 : s->nsz[k];
        if (f.kind == XDRG_K_DYNAMIC) {
            if (!cols[k].offsets) return inval(c, "dynamic column without offsets");
            if (n && !cols[k].data && !decode) { /* all-empty columns may have no data */ }
            if (!aligned(cols[k].data, al)) return inval(c, "dynamic column data misaligned");
        } else {
            if (decode && cols[k].stride == XDRG_STRIDE_CONST) return inval(c, "constant column on decode");
            const int64_t st = eff_stride(s, k, cols[k]);
            if (s->xbytes[k] && n && !cols[k].data) return inval(c, "fixed column data is NULL");
            if (!aligned(cols[k].data, al) || (st % (int64_t)al)) return inval(c, "fixed column misaligned");
        }
    }
    return XDRG_OK;
}

// Streaming path eligibility: unframed, array-of-structs whose fields sit at
// their XDR word positions, 16-byte aligned ends, 2-word types even-aligned.
static bool stream_eligible(const xdrg_schema *s, const xdrg_column *cols, uint64_t n,
                            const void *xdr, const uint8_t **base_out) {
    if (s->var_size || !s->stream_types || s->ops.empty() || !s->nwords) return false;
    if (((n * s->nwords) & 3) != 0) return false;
    const int64_t rec = (int64_t)s->nwords * 4;
    const uint8_t *base = nullptr;
    for (size_t k = 0; k < s->f.size(); ++k) {
        if (!s->xbytes[k]) continue;
        const uint8_t *b = (const uint8_t *)cols[k].data - 4 * (uint64_t)s->wpos[k];
        if (!base) base = b;
        if (b != base) return false;
        if (eff_stride(s, k, cols[k]) != rec) return false;
    }
    if (!base || !aligned(base, 16) || !aligned(xdr, 16)) return false;
    for (size_t w = 0; w < s->ops.size(); ++w) {
        const uint8_t op = s->ops[w].op;
        if ((op == OP_HYPER_HI || op == OP_DOUBLE_HI) && ((w & 1) || (s->nwords & 1))) return false;
    }
    *base_out = base;
    return true;
}

// Framed streaming path: as stream_eligible (layout) but only single-word
// ops (no hyper/double pairs) and any word count; the XDR side may be only
// 4-byte aligned.
static bool framed_stream_eligible(const xdrg_schema *s, const xdrg_column *cols, uint64_t n,
                                   const void *xdr, const uint8_t **base_out) {
    if (s->var_size || !s->stream_types || s->ops.empty() || !s->nwords) return false;
    const int64_t rec = (int64_t)s->nwords * 4;
    const uint8_t *base = nullptr;
    for (size_t k = 0; k < s->f.size(); ++k) {
        if (!s->xbytes[k]) continue;
        const uint8_t *b = (const uint8_t *)cols[k].data - 4 * (uint64_t)s->wpos[k];
        if (!base) base = b;
        if (b != base) return false;
        if (eff_stride(s, k, cols[k]) != rec) return false;
    }
    if (!base || !aligned(base, 16) || !aligned(xdr, 16)) return false;
    for (const WordOp &o : s->ops)
        if (o.op != OP_BSWAP && o.op != OP_FLOAT && o.op != OP_OPAQUE) return false;
    (void)n;
    *base_out = base;
    return true;
}

static void fill_stream_ops(const xdrg_schema *s, bool decode, StreamArgs &a) {
    a.all_bswap = 1;
    for (size_t w = 0; w < s->ops.size(); ++w) {
        uint8_t op = s->ops[w].op;
        if (decode) {  // decode keeps raw float/double bits (Xdr.java:255-269)
            if (op == OP_FLOAT) op = OP_BSWAP;
            else if (op == OP_DOUBLE_HI) op = OP_HYPER_HI;
            else if (op == OP_DOUBLE_LO) op = OP_HYPER_LO;
        }
        a.ops[w] = op;
        if (op != OP_BSWAP) a.all_bswap = 0;
    }
}

static void fill_wordmap(const xdrg_schema *s, const xdrg_column *cols, bool framed, WordMapArgs &a) {
    memset(&a, 0, sizeof a);
    uint32_t w = 0;
    if (framed) a.ops[w++] = {OP_MARK, 0, 0, 0, 0};
    for (const WordOp &o : s->ops) a.ops[w++] = o;
    a.wt = w;
    a.nops = w;
    const uint32_t m = (uint32_t)(s->fixed_size | kLastFrag);
    a.mark_le = __builtin_bswap32(m);
    for (size_t k = 0; k < s->f.size(); ++k) {
        a.base[k] = (uint8_t *)cols[k].data;
        a.stride[k] = eff_stride(s, k, cols[k]);
    }
}

static int fill_rec(xdrg_ctx *c, const xdrg_schema *s, xdrg_column *cols, uint64_t n, bool framed,
                    RecArgs &a) {
    memset(&a, 0, sizeof a);
    a.n = n;
    a.nf = (uint32_t)s->f.size();
    a.framed = framed;
    a.fixed_xdr = (uint32_t)(s->fixed_part + (framed ? 4 : 0));
    for (size_t k = 0; k < s->f.size(); ++k) {
        VField &v = a.f[k];
        const xdrg_field &f = s->f[k];
        v.type = f.type;
        v.kind = f.kind;
        v.nsz = s->nsz[k];
        v.xsz = s->xsz[k];
        v.count = f.count;
        v.xbytes = s->xbytes[k];
        v.data = (uint8_t *)cols[k].data;
        v.stride = f.kind == XDRG_K_DYNAMIC ? 0 : eff_stride(s, k, cols[k]);
        v.offsets = cols[k].offsets;
        v.cap = cols[k].cap;
        v.cond = s->cond[k];
        v.cneg = s->cneg[k];
        v.cfirst = s->cfirst[k];
        v.cnum = s->cnum[k];
        v.slot = s->slot[k];
        if (f.kind == XDRG_K_DYNAMIC) a.dyn_idx[a.ndyn++] = (uint32_t)k;
        else if (!a.ndyn) a.pay_fb += s->xbytes[k];
    }
    a.pay_fb += framed ? 4 : 0;   // bytes before the first dynamic field (the payload kernels' field)
    a.ncond = s->ncond;
    // the fixed words as direct rules (VField::xbytes words of each fixed field)
    if (!s->ncond && s->fixed_part / 4 <= (uint64_t)kPayWords) {
        uint32_t j = 0;
        for (size_t k = 0; k < s->f.size(); ++k) {
            const VField &v = a.f[k];
            if (v.kind == XDRG_K_DYNAMIC) continue;
            for (uint32_t i = 0; i < v.xbytes / 4; ++i, ++j) {
                PayWord &w = a.pw[j];
                w.data = v.data;
                w.stride = v.stride;
                w.type = v.type;
                w.half = v.xsz == 8 ? (uint8_t)(i & 1) : 0;
                w.off = (uint16_t)(v.type == XDRG_T_OPAQUE ? 4 * i : v.xsz == 8 ? (i >> 1) * 8 : i * v.nsz);
                w.rem = (uint8_t)(v.type == XDRG_T_OPAQUE ? std::min<uint32_t>(v.count - 4 * i, 4u) : 0u);
            }
        }
        a.pay_nw = j;
    }
    for (size_t i = 0; i < s->cvals.size(); ++i) a.cvals[i] = s->cvals[i];
    a.nblocks = (n + kRecPerBlock - 1) / kRecPerBlock;
    if (!a.nblocks) a.nblocks = 1;
    const size_t rows = a.ndyn ? a.ndyn : 1;
    // block sums [rows][nblocks] | totals [rows] (+ pad) | per-record counts u32 [ndyn][n]
    const size_t sums_words = rows * a.nblocks + rows + 8;
    const size_t cnt_words = (a.ndyn * n + 1) / 2;
    // | per-record payload positions u64 [n] (one dynamic byte field: k_enc/dec_payload)
    const size_t pay_words = (a.ndyn == 1 && a.f[a.dyn_idx[0]].xsz == 1) ? n : 0;
    int rc = ensure_ws(c, sums_words + cnt_words + pay_words);
    if (rc) return rc;
    a.block_sums = c->d_ws;
    a.totals = c->d_ws + rows * a.nblocks;
    a.rec_cnt = (uint32_t *)(c->d_ws + sums_words);
    a.pay_pos = pay_words ? c->d_ws + sums_words + cnt_words : nullptr;
    a.errkey = c->d_stat;
    return XDRG_OK;
}

// Kernel arguments and workspace of a schema with repeated groups.
// map_bytes (decode): workspace for GroupArgs::emap, 16-byte aligned after the rest.
// The class of field k's condition for the group kernels (GField::cneg >> 8):
// 1 + the first field whose condition is the same test (same discriminant,
// negation and case values), 0 for an unconditional field.
static uint32_t cond_class(const xdrg_schema *s, size_t k) {
    if (!s->cond[k]) return 0;
    for (size_t i = 0; i <= k; ++i) {
        if (s->cond[i] != s->cond[k] || s->cneg[i] != s->cneg[k] || s->cnum[i] != s->cnum[k]) continue;
        bool same = true;
        for (uint32_t j = 0; j < s->cnum[k] && same; ++j) same = s->cvals[s->cfirst[i] + j] == s->cvals[s->cfirst[k] + j];
        if (same) return (uint32_t)i + 1;
    }
    return (uint32_t)k + 1;
}

static int fill_group(xdrg_ctx *c, const xdrg_schema *s, const xdrg_column *cols, uint64_t n, bool framed,
                      bool decode, GroupArgs &a, uint64_t map_bytes = 0) {
    memset(&a, 0, sizeof a);
    a.n = n;
    a.nf = (uint32_t)s->f.size();
    a.framed = framed;
    for (size_t k = 0; k < s->f.size(); ++k) {
        GField &v = a.f[k];
        const xdrg_field &f = s->f[k];
        v.type = f.type;
        v.kind = f.kind;
        v.nsz = s->nsz[k];
        v.xsz = s->xsz[k];
        v.count = f.count;
        v.xbytes = s->xbytes[k];
        v.grp = s->grp[k];
        v.top = (uint32_t)k;   // the top-level field that owns it (an inner group's member: two levels up)
        while (s->grp[v.top]) v.top = s->grp[v.top] - 1;
        v.data = (uint8_t *)cols[k].data;
        v.stride = (f.kind == XDRG_K_DYNAMIC || f.type == XDRG_T_GROUP) ? 0 : eff_stride(s, k, cols[k]);
        v.offsets = cols[k].offsets;
        v.cap = cols[k].cap;
        const bool counted = (f.type == XDRG_T_GROUP && f.kind != XDRG_K_FIXED) ||
                             (f.type != XDRG_T_GROUP && f.kind == XDRG_K_DYNAMIC);
        if (counted) {
            if (a.nslot == (uint32_t)kMaxSlots) return inval(c, "too many counted columns in a group schema");
            a.slot_field[a.nslot] = (uint32_t)k;
            v.slot = ++a.nslot;
        }
        if (f.type == XDRG_T_GROUP) {
            v.nmem = f.reserved;
            v.efix = f.kind == XDRG_K_LIST ? 4 : 0;
            for (uint32_t j = 1; j <= f.reserved; ++j) {   // its immediate members
                const xdrg_field &m = s->f[k + j];
                if (m.type == XDRG_T_GROUP) {   // an inner array / list: elements of varying size
                    ++v.ndm;
                    ++v.ngm;
                    if (s->cond[k + j]) ++v.ncm;
                    j += m.reserved;
                    continue;
                }
                if (m.kind == XDRG_K_DYNAMIC) ++v.ndm;
                else v.efix += s->xbytes[k + j];
                if (s->cond[k + j]) ++v.ncm;
            }
        }
        v.cond = s->cond[k];
        v.cneg = s->cneg[k] | (cond_class(s, k) << 8);
        v.cfirst = s->cfirst[k];
        v.cnum = s->cnum[k];
        v.dslot = s->slot[k];
    }
    // runs of fixed members (GField::run)
    for (uint32_t k = 0; k < a.nf; ++k) {
        GField &v = a.f[k];
        auto runnable = [&](const GField &w) {
            return w.grp == v.grp && w.type != XDRG_T_GROUP && w.kind != XDRG_K_DYNAMIC && !w.dslot &&
                   (w.cneg >> 8) == (v.cneg >> 8);
        };
        if (!v.grp || !runnable(v)) continue;
        uint32_t n = 1;
        uint64_t bytes = v.xbytes;
        while (k + n < a.nf && n < 255 && runnable(a.f[k + n])) bytes += a.f[k + n++].xbytes;
        if (n >= 2 && bytes < (1u << 24)) v.run = (uint32_t)bytes << 8 | n;
    }
    a.ncond = s->ncond;
    a.nest = s->nested ? 1u : 0u;
    a.levels = 1;
    for (size_t k = 0; k < s->f.size(); ++k) {   // a group's level = its group ancestors
        if (s->f[k].type != XDRG_T_GROUP) continue;
        uint32_t lv = 1;
        for (uint32_t g = s->grp[k]; g; g = s->grp[g - 1]) ++lv;
        if (lv > a.levels) a.levels = lv;
    }
    // the element layout of a schema's one top-level group (GroupArgs::lay_g)
    a.lay_g = 0;
    for (uint32_t k = 0; k < a.nf && s->ngroups == 1 && !a.nest; ++k) {
        const GField &G = a.f[k];
        if (G.type != XDRG_T_GROUP || G.grp || G.ncm || G.ngm || G.ndm > 2) continue;
        uint32_t q = 0, fb[3] = {0, 0, 0}, z[2] = {4, 4}, sl[2] = {0, 0};
        for (uint32_t j = 1; j <= G.nmem; ++j) {
            const GField &m = a.f[k + j];
            if (m.kind == XDRG_K_DYNAMIC) { z[q] = m.xsz; sl[q] = m.slot; ++q; }
            else fb[q] += m.xbytes;
        }
        a.lay_g = k + 1;
        a.lay_pre = fb[0]; a.lay_mid = fb[1]; a.lay_post = fb[2];
        a.lay_z0 = z[0]; a.lay_z1 = z[1];
        a.lay_s0 = sl[0]; a.lay_s1 = sl[1];
    }
    for (size_t i = 0; i < s->cvals.size(); ++i) a.cvals[i] = s->cvals[i];
    a.nblocks = (n + kRecPerBlock - 1) / kRecPerBlock;
    if (!a.nblocks) a.nblocks = 1;
    const size_t rows = a.nslot ? a.nslot : 1;
    // block sums [rows][nblocks] | totals [rows] | encode: sizes [n] / decode: counts u32 [nslot][n]
    // and native offsets [nslot][n]
    const size_t sums = rows * a.nblocks + rows + 8;
    const size_t per_rec = decode ? (a.nslot * n + 1) / 2 + a.nslot * n : n;
    const size_t map_words = (map_bytes + 7) / 8 + 2;
    int rc = ensure_ws(c, sums + per_rec + 1 + map_words);
    if (rc) return rc;
    a.emap = map_bytes ? (uint8_t *)(((uintptr_t)(c->d_ws + sums + per_rec + 1) + 15) & ~(uintptr_t)15) : nullptr;
    a.block_sums = c->d_ws;
    a.totals = c->d_ws + rows * a.nblocks;
    if (decode) {
        a.rec_cnt = (uint32_t *)(c->d_ws + sums);
        a.rec_base = c->d_ws + sums + (a.nslot * n + 1) / 2;
    } else {
        a.rec_size = c->d_ws + sums;
    }
    a.errkey = c->d_stat;
    return XDRG_OK;
}

static int group_encode(xdrg_ctx *c, const xdrg_schema *s, const xdrg_column *cols, uint64_t n, uint8_t *out,
                        uint64_t out_cap, uint64_t *rec_offsets, bool framed, bool async, uint64_t *out_len) {
    if (n == 0) {
        if (rec_offsets) HIPCHK(c, hipMemsetAsync(rec_offsets, 0, 8, c->stream));
        if (out_len && !async) *out_len = 0;
        if (out_len && async) HIPCHK(c, (hipError_t)launch_store_u64(out_len, 0, c->stream));
        if (!async) HIPCHK(c, hipStreamSynchronize(c->stream));
        return XDRG_OK;
    }
    GroupArgs a;
    int rc = fill_group(c, s, cols, n, framed, false, a);
    if (rc) return rc;
    a.enc_lanes = (uint32_t)c->tune.grp_enc_lanes;
    a.enc_split = (uint32_t)c->tune.grp_enc_split;
    // the element-parallel place: one top-level group (inner groups included)
    if (c->tune.grp_enc_img && s->ngroups == 1 && (!a.nest || c->tune.grp_enc_img_nest))
        for (uint32_t k = 0; k < a.nf; ++k)
            if (a.f[k].type == XDRG_T_GROUP && !a.f[k].grp) {
                a.enc_img = (uint32_t)c->tune.grp_enc_img;
                a.el_g = k;
            }
    a.xdr = out;
    a.xdr_cap = out_cap;
    a.rec_out = rec_offsets;
    {
        TimedLaunch t(c, XDRG_KERNEL_VAR_SIZE);
        HIPCHK(c, (hipError_t)launch_group_phase(a, GRP_ENC_SIZES, c->stream));
    }
    {
        TimedLaunch t(c, XDRG_KERNEL_VAR_SCAN);
        HIPCHK(c, (hipError_t)launch_scan_rows(a.block_sums, a.nblocks, a.totals, 1, c->stream));
    }
    {
        TimedLaunch t(c, XDRG_KERNEL_VAR_ENCODE);
        HIPCHK(c, (hipError_t)launch_group_phase(a, GRP_ENC_PLACE, c->stream));
    }
    if (async) {
        if (out_len) HIPCHK(c, hipMemcpyAsync(out_len, a.totals, 8, hipMemcpyDeviceToDevice, c->stream));
        return XDRG_OK;
    }
    HIPCHK(c, hipMemcpyAsync(c->h_stat, a.totals, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const uint64_t total = c->h_stat[0];
    if (out_len) *out_len = total;
    if (total > out_cap) {
        c->err = "output buffer too small";
        return XDRG_E_CAPACITY;
    }
    return XDRG_OK;
}

// ---------------------------------------------------------------------------
// encode
// ---------------------------------------------------------------------------
// byref = 0, or 1 + the field encoded by reference (xdrg_encode_batch_shallow).
static int encode_impl(xdrg_ctx *c, const xdrg_schema *s, const xdrg_column *cols, uint64_t n,
                       uint8_t *out, uint64_t out_cap, uint64_t *rec_offsets, uint32_t flags,
                       uint64_t *out_len, uint32_t byref, uint64_t *ref_pos) {
    if (!c || !s) return XDRG_E_INVAL;
    DeviceGuard dg;
    HIPCHK(c, hipSetDevice(c->device));
    const bool framed = flags & XDRG_FRAME_RM;
    const bool async = flags & XDRG_ASYNC;
    if (!aligned(out, 4)) return inval(c, "XDR buffer not 4-byte aligned");
    if (n && !out) return inval(c, "XDR buffer is NULL");
    int rc = check_columns(c, s, cols, n, false);
    if (rc) return rc;
    if (s->ngroups) {
        if (byref) return inval(c, "by-reference payloads in a schema with repeated groups");
        return group_encode(c, s, cols, n, out, out_cap, rec_offsets, framed, async, out_len);
    }

    if (!s->var_size) {
        const uint64_t stride = s->fixed_size + (framed ? 4 : 0);
        const uint64_t total = n * stride;
        if (n && total / n != stride) return inval(c, "batch size overflows");
        if (total > out_cap) {
            if (out_len && !async) *out_len = total;
            c->err = "output buffer too small";
            return XDRG_E_CAPACITY;
        }
        if (rec_offsets) {
            TimedLaunch t(c, XDRG_KERNEL_FIXED_ENCODE);
            HIPCHK(c, (hipError_t)launch_iota(rec_offsets, n, stride, c->stream));
        }
        const uint8_t *base = nullptr;
        if (n && !framed && stream_eligible(s, cols, n, out, &base)) {
            StreamArgs a;
            memset(&a, 0, sizeof a);
            a.src = base;
            a.dst = out;
            a.nvec = total / 16;
            a.w = s->nwords;
            fill_stream_ops(s, false, a);
            TimedLaunch t(c, XDRG_KERNEL_FIXED_ENCODE);
            HIPCHK(c, (hipError_t)launch_stream_words(a, c->stream));
        } else if (n && framed && framed_stream_eligible(s, cols, n, out, &base)) {
            StreamArgs a;
            memset(&a, 0, sizeof a);
            a.src = base;
            a.dst = out;
            a.w = s->nwords;
            fill_stream_ops(s, false, a);
            TimedLaunch t(c, XDRG_KERNEL_FIXED_ENCODE);
            HIPCHK(c, (hipError_t)launch_stream_framed(a, n, __builtin_bswap32((uint32_t)(s->fixed_size | kLastFrag)),
                                                       false, nullptr, c->tune, c->stream));
        } else if (n && s->nwords + (framed ? 1 : 0) <= (uint32_t)kMaxWords && !s->ops.empty() &&
                   s->f.size() <= (size_t)kMaxCols) {
            WordMapArgs a;
            fill_wordmap(s, cols, framed, a);
            a.n = n;
            a.xdr = out;
            TimedLaunch t(c, XDRG_KERNEL_FIXED_ENCODE);
            int lr = -1;
            if (words_lane_ok(a.ops, a.nops))
                lr = launch_words_lane(a, false, aligned(out, 16) && (a.wt % 4) == 0, c->tune, c->stream);
            if (lr > 0) HIPCHK(c, (hipError_t)lr);
            if (lr < 0) HIPCHK(c, (hipError_t)launch_wordmap_encode(a, aligned(out, 16), c->stream));
        } else if (n && total) {
            RecArgs a;
            rc = fill_rec(c, s, (xdrg_column *)cols, n, framed, a);
            if (rc) return rc;
            a.xdr = out;
            a.xdr_cap = out_cap;
            a.rec_out = nullptr;
            for (int ph = REC_ENC_SIZES; ph <= REC_ENC_PLACE; ++ph) {
                TimedLaunch t(c, XDRG_KERNEL_VAR_SIZE + ph);
                HIPCHK(c, (hipError_t)launch_rec_phase(a, ph, c->tune, c->stream));
            }
        }
        if (out_len) {
            if (async) HIPCHK(c, (hipError_t)launch_store_u64(out_len, total, c->stream));
            else *out_len = total;
        }
        if (!async) HIPCHK(c, hipStreamSynchronize(c->stream));
        return XDRG_OK;
    }

    // variable-size records: size -> scan -> place
    if (n == 0) {
        if (rec_offsets) HIPCHK(c, hipMemsetAsync(rec_offsets, 0, 8, c->stream));
        if (out_len && !async) *out_len = 0;
        if (out_len && async) HIPCHK(c, (hipError_t)launch_store_u64(out_len, 0, c->stream));
        if (!async) HIPCHK(c, hipStreamSynchronize(c->stream));
        return XDRG_OK;
    }
    RecArgs a;
    rc = fill_rec(c, s, (xdrg_column *)cols, n, framed, a);
    if (rc) return rc;
    a.xdr = out;
    a.xdr_cap = out_cap;
    a.rec_out = rec_offsets;
    a.byref = byref;
    a.ref_pos = ref_pos;
    for (int ph = REC_ENC_SIZES; ph <= REC_ENC_PLACE; ++ph) {
        TimedLaunch t(c, XDRG_KERNEL_VAR_SIZE + ph);
        HIPCHK(c, (hipError_t)launch_rec_phase(a, ph, c->tune, c->stream));
    }
    if (async) {
        if (out_len) HIPCHK(c, hipMemcpyAsync(out_len, a.totals, 8, hipMemcpyDeviceToDevice, c->stream));
        return XDRG_OK;
    }
    HIPCHK(c, hipMemcpyAsync(c->h_stat, a.totals, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const uint64_t total = c->h_stat[0];
    if (out_len) *out_len = total;
    if (total > out_cap) {
        c->err = "output buffer too small";
        return XDRG_E_CAPACITY;
    }
    return XDRG_OK;
}

static int host_encode(xdrg_ctx *c, const xdrg_schema *s, const xdrg_column *cols, uint64_t n, uint8_t *out,
                       uint64_t out_cap, uint64_t *rec_offsets, uint32_t flags, uint64_t *out_len,
                       uint32_t byref, uint64_t *splice);
static int host_decode(xdrg_ctx *c, const xdrg_schema *s, const uint8_t *in, uint64_t in_len,
                       const uint64_t *rec_offsets, uint64_t n, xdrg_column *cols, uint32_t flags,
                       uint64_t *first_bad, int *err, uint32_t byref, uint64_t *payload_pos);

// The flags of the codec calls (encode / decode, their by-reference forms);
// any other bit is refused before a pointer is looked at, so a caller's host
// buffer never reaches a kernel under a flag the call does not know.
static int codec_flags(xdrg_ctx *c, uint32_t flags) {
    if (flags & ~(XDRG_FRAME_RM | XDRG_ASYNC | XDRG_HOST_PTRS | XDRG_HOST_MAPPED))
        return inval(c, "unknown flag bits");
    if ((flags & XDRG_HOST_MAPPED) && !(flags & XDRG_HOST_PTRS)) return inval(c, "XDRG_HOST_MAPPED without XDRG_HOST_PTRS");
    return XDRG_OK;
}

extern "C" int xdrg_encode_batch(xdrg_ctx *c, const xdrg_schema *s, const xdrg_column *cols,
                                 uint64_t n, uint8_t *out, uint64_t out_cap, uint64_t *rec_offsets,
                                 uint32_t flags, uint64_t *out_len) {
    const int rc = codec_flags(c, flags);
    if (rc) return rc;
    if (flags & XDRG_HOST_PTRS) return host_encode(c, s, cols, n, out, out_cap, rec_offsets, flags, out_len, 0, nullptr);
    return encode_impl(c, s, cols, n, out, out_cap, rec_offsets, flags, out_len, 0, nullptr);
}

// A dynamic opaque / string field may travel by reference (Xdr.java:839-866, 978-988).
static int check_byref(xdrg_ctx *c, const xdrg_schema *s, uint32_t field, const void *pos) {
    if (!c || !s) return XDRG_E_INVAL;
    if (field >= s->f.size()) return inval(c, "by-reference field index out of range");
    const xdrg_field &f = s->f[field];
    if (f.kind != XDRG_K_DYNAMIC || (f.type != XDRG_T_OPAQUE && f.type != XDRG_T_STRING))
        return inval(c, "by-reference field must be a dynamic opaque or string");
    if (!pos) return inval(c, "splice / payload position array is NULL");
    return XDRG_OK;
}

extern "C" int xdrg_encode_batch_shallow(xdrg_ctx *c, const xdrg_schema *s, const xdrg_column *cols,
                                         uint64_t n, uint8_t *out, uint64_t out_cap,
                                         uint64_t *rec_offsets, uint32_t flags, uint64_t *out_len,
                                         uint32_t field, uint64_t *splice) {
    int rc = codec_flags(c, flags);
    if (!rc) rc = check_byref(c, s, field, n ? splice : (void *)1);
    if (rc) return rc;
    if (flags & XDRG_HOST_PTRS)
        return host_encode(c, s, cols, n, out, out_cap, rec_offsets, flags, out_len, field + 1, splice);
    return encode_impl(c, s, cols, n, out, out_cap, rec_offsets, flags, out_len, field + 1, splice);
}

// ---------------------------------------------------------------------------
// decode
// ---------------------------------------------------------------------------
static int rec_dec_kernel_id(int ph) {
    return ph == REC_DEC_SIZES ? XDRG_KERNEL_VAR_SIZE
         : ph == REC_DEC_SCAN ? XDRG_KERNEL_VAR_SCAN : XDRG_KERNEL_VAR_DECODE;
}

static int finish_decode(xdrg_ctx *c, uint64_t n, unsigned long long host_key, bool used_dev_key,
                         bool async, uint64_t *first_bad, int *err) {
    if (async) {
        if (first_bad || err)
            HIPCHK(c, (hipError_t)launch_finalize(used_dev_key ? c->d_stat : nullptr, host_key, n,
                                                  first_bad, err, c->stream));
        return XDRG_OK;
    }
    unsigned long long key = host_key;
    if (used_dev_key) {
        HIPCHK(c, hipMemcpyAsync(c->h_stat, c->d_stat, 8, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        if (c->h_stat[0] < key) key = c->h_stat[0];
    } else {
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    if (key == kNoError) {
        if (first_bad) *first_bad = n;
        if (err) *err = XDRG_OK;
        return XDRG_OK;
    }
    const int code = (int)(key & 0xf);
    if (first_bad) *first_bad = (uint64_t)(key >> 16);
    if (err) *err = code;
    c->err = xdrg_status_string(code);
    return code;
}

// k_grp_dec_place_eln's sub-batch: at most this tile (key 33) and these
// elements (key 38).  volume_index / acl_tree decode ms: 16 KiB / 512
// elements 1.39 / 3.59, 16 KiB / 256 1.15 / 3.59, 8 KiB / 256 1.71 / 5.87,
// 32 KiB / 256 1.11 / 2.36 (profiles/r05_groups/eln_tune*.txt)
#ifndef XDRG_ELN_TILE
#define XDRG_ELN_TILE 32768
#endif
constexpr uint32_t kElnTile = XDRG_ELN_TILE, kElnCap = 256;

// A repeated-group schema's decode in two halves (the receive windows,
// hs::stage_receive, lay their columns out for the counted rows): kDecCount
// runs the walk and the row scan only, its columns are not touched (may be
// dummies), and copies the error key and every counted column's total to
// count_out[0], count_out[1 ..] (host, pinned; ready after the stream
// synchronises); kDecPlace then runs the rest on the same workspace (same
// schema, records and stream, nothing else on the context's stream between).
constexpr uint32_t kDecCount = 1u << 30;
constexpr uint32_t kDecPlace = 1u << 29;

static int decode_impl(xdrg_ctx *c, const xdrg_schema *s, const uint8_t *in, uint64_t in_len,
                       const uint64_t *rec_offsets, uint64_t n, xdrg_column *cols, uint32_t flags,
                       uint64_t *first_bad, int *err, uint32_t byref, uint64_t *ref_pos,
                       uint64_t *count_out = nullptr) {
    if (!c || !s) return XDRG_E_INVAL;
    DeviceGuard dg;
    HIPCHK(c, hipSetDevice(c->device));
    const bool framed = flags & XDRG_FRAME_RM;
    const bool async = flags & XDRG_ASYNC;
    const bool count_half = flags & kDecCount, place_half = flags & kDecPlace;
    if ((count_half || place_half) && (!s->ngroups || !async || byref || (count_half && !count_out)))
        return inval(c, "two-half decode: repeated-group schemas, asynchronous");
    if (!aligned(in, 4)) return inval(c, "XDR buffer not 4-byte aligned");
    if (n && in_len && !in) return inval(c, "XDR buffer is NULL");
    if (s->var_size && !rec_offsets) return inval(c, "variable-size schema needs record offsets");
    int rc = count_half ? XDRG_OK : check_columns(c, s, cols, n, true);
    if (rc) return rc;
    if (s->ngroups) {
        if (byref) return inval(c, "payload views in a schema with repeated groups");
        GroupArgs a;
        // the element-start map: a byte per stream word, read 16 at a time
        const uint64_t map_bytes = c->tune.grp_dec_emap && c->tune.grp_dec_el && s->ngroups == 1 ? in_len / 4 + 32 : 0;
        rc = fill_group(c, s, cols, n, framed, true, a, map_bytes);
        if (rc) return rc;
        uint8_t *const emap = a.emap;
        a.emap = nullptr;
        a.dec_tile = (uint32_t)c->tune.grp_dec_tile;
        // the element-parallel place: one top-level group without inner groups,
        // at most two dynamic members, LDS for the tile and the descriptors
        if (c->tune.grp_dec_el && a.dec_tile && !a.nest && s->ngroups == 1 &&
            8224ull + a.dec_tile + 12ull * (uint64_t)c->tune.grp_dec_el <= 65536) {   // (+ kElMeta)
            for (uint32_t k = 0; k < a.nf; ++k)
                if (a.f[k].type == XDRG_T_GROUP && !a.f[k].grp && a.f[k].ndm <= 2 &&
                    !(a.f[k].kind == XDRG_K_FIXED && a.f[k].cond)) {   // (an absent T x[N] has no descriptors)
                    a.dec_el = (uint32_t)c->tune.grp_dec_el;
                    a.el_g = k;
                }
        }
        // elements found by their start words: each element has a word of its own
        // (a list's TRUE before it, else at least 4 unconditional bytes).  Not for
        // a group with a layout: its record walk reads one length word per
        // dynamic member, cheaper than the map's stores and scan (DUMP decode
        // 1.05 -> 1.60 ms, READDIR 2.22 -> 3.13 with it)
        auto own_word = [&](uint32_t g) {
            const GField &G = a.f[g];
            uint64_t minb = 0;
            for (uint32_t j = 1; j <= G.nmem; ++j) {
                const GField &m = a.f[g + j];
                if (!m.cond) minb += m.type == XDRG_T_GROUP ? (m.kind == XDRG_K_FIXED ? 0 : 4)
                                                            : m.kind == XDRG_K_DYNAMIC ? 4 : m.xbytes;
                if (m.type == XDRG_T_GROUP) j += m.nmem;
            }
            return G.kind == XDRG_K_LIST || minb >= 4;
        };
        if (a.dec_el && emap && a.lay_g != a.el_g + 1 && own_word(a.el_g)) a.emap = emap;
        // the element-parallel place of a group holding inner groups
        // (k_grp_dec_place_eln): a smaller tile and fewer elements per sub-batch,
        // its LDS also holding every span column's positions and running offsets
        if (!a.dec_el && emap && a.nest && c->tune.grp_dec_el && a.dec_tile)
            for (uint32_t k = 0; k < a.nf; ++k) {
                const GField &G = a.f[k];
                if (G.type != XDRG_T_GROUP || G.grp || (G.kind == XDRG_K_FIXED && G.cond) || !own_word(k)) continue;
                uint32_t ns = 0;
                for (uint32_t j = 1; j <= G.nmem; ++j) ns += a.f[k + j].slot ? 1u : 0u;
                uint32_t tile = a.dec_tile < kElnTile ? a.dec_tile : kElnTile;
                uint32_t cap = (uint32_t)c->tune.grp_dec_el < kElnCap ? (uint32_t)c->tune.grp_dec_el : kElnCap;
                const size_t budget = kPlaceLdsBudget - kPlaceStaticLds;
                while (eln_lds_bytes(tile, cap, ns, a.nslot) > budget && tile > 4096) {
                    tile /= 2;
                    cap = cap > 128 ? cap / 2 : cap;
                }
                if (eln_lds_bytes(tile, cap, ns, a.nslot) > budget) break;
                a.dec_tile = tile;
                a.dec_el = cap;
                a.el_g = k;
                a.emap = emap;
            }
        // a nested schema's lane-per-record places (k_grp_dec_place_lds<D > 1>)
        // keep their running-offset columns in static LDS beside the tile
        if (a.levels > 1 && !(a.emap && a.dec_el) && a.dec_tile &&
            a.dec_tile + kNestRunLdsBytes + kPlaceStaticLds > kPlaceLdsBudget)
            a.dec_tile = (uint32_t)((kPlaceLdsBudget - kNestRunLdsBytes - kPlaceStaticLds) & ~(size_t)15);
        if (n == 0 && count_half) {
            memset(count_out, 0, 8 * (1 + (size_t)a.nslot));
            count_out[0] = kNoError;
            return XDRG_OK;
        }
        if (n == 0) {
            for (uint32_t q = 0; q < a.nslot; ++q)   // (members too: zero rows, offsets[0] = 0)
                HIPCHK(c, hipMemsetAsync(cols[a.slot_field[q]].offsets, 0, 8, c->stream));
            return finish_decode(c, n, kNoError, false, async, first_bad, err);
        }
        a.xdr = (uint8_t *)in;
        a.xdr_cap = in_len;
        a.rec_in = rec_offsets;
        if (!place_half) {
            HIPCHK(c, hipMemsetAsync(c->d_stat, 0xff, 8, c->stream));
            if (a.emap) HIPCHK(c, hipMemsetAsync(a.emap, 0, in_len / 4 + 32, c->stream));
            {
                TimedLaunch t(c, XDRG_KERNEL_VAR_SIZE);
                HIPCHK(c, (hipError_t)launch_group_phase(a, GRP_DEC_WALK, c->stream));
            }
            {
                TimedLaunch t(c, XDRG_KERNEL_VAR_SCAN);
                HIPCHK(c, (hipError_t)launch_scan_rows(a.block_sums, a.nblocks, a.totals, a.nslot, c->stream));
            }
        }
        if (count_half) {
            HIPCHK(c, hipMemcpyAsync(count_out, c->d_stat, 8, hipMemcpyDeviceToHost, c->stream));
            if (a.nslot)
                HIPCHK(c, hipMemcpyAsync(count_out + 1, a.totals, 8 * (size_t)a.nslot, hipMemcpyDeviceToHost, c->stream));
            return XDRG_OK;
        }
        {
            TimedLaunch t(c, XDRG_KERNEL_VAR_DECODE);
            HIPCHK(c, (hipError_t)launch_group_phase(a, GRP_DEC_OFFSETS, c->stream));
            HIPCHK(c, (hipError_t)launch_group_phase(a, GRP_DEC_PLACE, c->stream));
        }
        return finish_decode(c, n, kNoError, true, async, first_bad, err);
    }

    // Fixed-size records at explicit extents that turn out to be the fixed
    // stride — a frame scan of uniform single-fragment messages, the receive
    // side of GrizzlyRpcTransport's one mark per reply — take the stride
    // kernels after one device check of the offsets (sync calls; one round
    // trip).  Same records, same checks: record i is [ro[0] + i*stride, +stride).
    if (!s->var_size && rec_offsets && n && !async && !byref && c->tune.stride_check) {
        const uint64_t stride = s->fixed_size + (framed ? 4 : 0);
        HIPCHK(c, hipMemsetAsync(c->d_stat + 6, 0, 16, c->stream));
        HIPCHK(c, (hipError_t)launch_check_stride(rec_offsets, n, stride, c->d_stat + 6, c->stream));
        HIPCHK(c, hipMemcpyAsync(c->h_stat + 6, c->d_stat + 6, 16, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        const uint64_t o0 = c->h_stat[7];
        if (!c->h_stat[6] && stride && o0 <= in_len && n * stride <= in_len - o0 && n * stride / n == stride &&
            aligned(in + o0, 4)) {
            in += o0;
            in_len -= o0;
            rec_offsets = nullptr;
        }
    }
    if (!s->var_size && !rec_offsets) {
        const uint64_t stride = s->fixed_size + (framed ? 4 : 0);
        const uint64_t total = n * stride;
        if (n && total / n != stride) return inval(c, "batch size overflows");
        // records wholly inside in_len decode; the first one that is not
        // fails "xdr stream too short" at its first missing word (Xdr.java:1028-1031)
        unsigned long long host_key = kNoError;
        if (stride && in_len < total) {
            const uint64_t rs = in_len / stride;
            const uint64_t ws = (in_len - rs * stride) / 4;
            host_key = err_key(rs, (uint32_t)ws, XDRG_E_SHORT);
        }
        bool dev_key = false;
        const uint8_t *base = nullptr;
        if (n && !framed && in_len >= total && stream_eligible(s, cols, n, in, &base)) {
            StreamArgs a;
            memset(&a, 0, sizeof a);
            a.src = in;
            a.dst = (uint8_t *)base;
            a.nvec = total / 16;
            a.w = s->nwords;
            fill_stream_ops(s, true, a);
            TimedLaunch t(c, XDRG_KERNEL_FIXED_DECODE);
            HIPCHK(c, (hipError_t)launch_stream_words(a, c->stream));
        } else if (n && framed && in_len >= total && framed_stream_eligible(s, cols, n, in, &base)) {
            StreamArgs a;
            memset(&a, 0, sizeof a);
            a.src = in;
            a.dst = (uint8_t *)base;
            a.w = s->nwords;
            fill_stream_ops(s, true, a);
            dev_key = true;
            HIPCHK(c, hipMemsetAsync(c->d_stat, 0xff, 8, c->stream));
            TimedLaunch t(c, XDRG_KERNEL_FIXED_DECODE);
            HIPCHK(c, (hipError_t)launch_stream_framed(a, n, __builtin_bswap32((uint32_t)(s->fixed_size | kLastFrag)),
                                                       true, c->d_stat, c->tune, c->stream));
        } else if (n && stride && s->nwords + (framed ? 1 : 0) <= (uint32_t)kMaxWords &&
                   !s->ops.empty() && s->f.size() <= (size_t)kMaxCols) {
            WordMapArgs a;
            fill_wordmap(s, cols, framed, a);
            a.n = n;
            a.xdr = (uint8_t *)in;
            a.xdr_len = in_len;
            a.errkey = c->d_stat;
            dev_key = framed;
            if (dev_key) HIPCHK(c, hipMemsetAsync(c->d_stat, 0xff, 8, c->stream));
            TimedLaunch t(c, XDRG_KERNEL_FIXED_DECODE);
            int lr = -1;
            if (words_lane_ok(a.ops, a.nops))
                lr = launch_words_lane(a, true, aligned(in, 16) && (a.wt % 4) == 0, c->tune, c->stream);
            if (lr > 0) HIPCHK(c, (hipError_t)lr);
            if (lr < 0) HIPCHK(c, (hipError_t)launch_wordmap_decode(a, aligned(in, 16), c->stream));
        } else if (n && stride) {
            RecArgs a;
            rc = fill_rec(c, s, cols, n, framed, a);
            if (rc) return rc;
            a.xdr = (uint8_t *)in;
            a.xdr_cap = in_len;
            a.rec_in = nullptr;
            a.rec_stride = stride;
            HIPCHK(c, hipMemsetAsync(c->d_stat, 0xff, 8, c->stream));
            dev_key = true;
            for (int ph = REC_DEC_SIZES; ph <= REC_DEC_PLACE; ++ph) {
                TimedLaunch t(c, rec_dec_kernel_id(ph));
                HIPCHK(c, (hipError_t)launch_rec_phase(a, ph, c->tune, c->stream));
            }
        }
        return finish_decode(c, n, host_key, dev_key, async, first_bad, err);
    }

    // record path: extents from rec_offsets
    RecArgs a;
    rc = fill_rec(c, s, cols, n, framed, a);
    if (rc) return rc;
    if (n == 0) {
        for (uint32_t d = 0; d < a.ndyn; ++d)
            HIPCHK(c, hipMemsetAsync(cols[a.dyn_idx[d]].offsets, 0, 8, c->stream));
        return finish_decode(c, n, kNoError, false, async, first_bad, err);
    }
    a.xdr = (uint8_t *)in;
    a.xdr_cap = in_len;
    a.rec_in = rec_offsets;
    a.byref = byref;
    a.ref_pos = ref_pos;
    // extent-derived counts (tuning key 31): the derived pass, then the exact
    // walk's kernels, which return at once unless the derived counts failed
    // (device flag, no host round trip: XDRG_ASYNC and graph capture keep working)
    const bool spec = rec_spec_ok(a, c->tune) && (!c->tune.big_rec || in_len / n < c->tune.big_rec);
    a.spec = spec ? (uint32_t *)(c->d_stat + 1) : nullptr;   // word 1: ~0 = derived counts hold
    a.spec_mode = spec ? (c->tune.spec_sizes == 2 ? 3 : 1) : 0;
    a.lb_ticket = c->d_stat + 2;                              // word 2: one-pass block tickets
    HIPCHK(c, hipMemsetAsync(c->d_stat, 0xff, spec ? 24 : 8, c->stream));
    if (a.spec_mode == 3)   // the look-back status words (in the block sums' place)
        HIPCHK(c, hipMemsetAsync(a.block_sums, 0, (size_t)a.ndyn * a.nblocks * 8, c->stream));
    for (int ph = REC_DEC_SIZES; ph <= REC_DEC_PLACE; ++ph) {
        TimedLaunch t(c, rec_dec_kernel_id(ph));
        HIPCHK(c, (hipError_t)launch_rec_phase(a, ph, c->tune, c->stream));
    }
    if (spec && !async) {   // one round trip reads the error key and the spec word together
        HIPCHK(c, hipMemcpyAsync(c->h_stat, c->d_stat, 16, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        if ((uint32_t)c->h_stat[1] != 0)   // the derived counts held: the key is final
            return finish_decode(c, n, c->h_stat[0], false, false, first_bad, err);
        HIPCHK(c, hipMemsetAsync(c->d_stat, 0xff, 8, c->stream));   // the exact walk, from scratch
        a.spec = nullptr;
        a.spec_mode = 0;
        for (int ph = REC_DEC_SIZES; ph <= REC_DEC_PLACE; ++ph) {
            TimedLaunch t(c, rec_dec_kernel_id(ph), false);
            HIPCHK(c, (hipError_t)launch_rec_phase(a, ph, c->tune, c->stream));
        }
    } else if (spec) {   // XDRG_ASYNC: no host round trip, the rerun's kernels check the word
        HIPCHK(c, (hipError_t)launch_spec_reset(a.spec, c->d_stat, c->stream));
        a.spec_mode = 2;
        for (int ph = REC_DEC_SIZES; ph <= REC_DEC_PLACE; ++ph) {   // (their time, not extra launches)
            TimedLaunch t(c, rec_dec_kernel_id(ph), false);
            HIPCHK(c, (hipError_t)launch_rec_phase(a, ph, c->tune, c->stream));
        }
    }
    return finish_decode(c, n, kNoError, true, async, first_bad, err);
}

extern "C" int xdrg_decode_batch(xdrg_ctx *c, const xdrg_schema *s, const uint8_t *in,
                                 uint64_t in_len, const uint64_t *rec_offsets, uint64_t n,
                                 xdrg_column *cols, uint32_t flags, uint64_t *first_bad, int *err) {
    const int rc = codec_flags(c, flags);
    if (rc) return rc;
    if (flags & XDRG_HOST_PTRS)
        return host_decode(c, s, in, in_len, rec_offsets, n, cols, flags, first_bad, err, 0, nullptr);
    return decode_impl(c, s, in, in_len, rec_offsets, n, cols, flags, first_bad, err, 0, nullptr);
}

extern "C" int xdrg_decode_batch_view(xdrg_ctx *c, const xdrg_schema *s, const uint8_t *in,
                                      uint64_t in_len, const uint64_t *rec_offsets, uint64_t n,
                                      xdrg_column *cols, uint32_t flags, uint64_t *first_bad,
                                      int *err, uint32_t field, uint64_t *payload_pos) {
    int rc = codec_flags(c, flags);
    if (!rc) rc = check_byref(c, s, field, n ? payload_pos : (void *)1);
    if (rc) return rc;
    if (flags & XDRG_HOST_PTRS)
        return host_decode(c, s, in, in_len, rec_offsets, n, cols, flags, first_bad, err, field + 1, payload_pos);
    return decode_impl(c, s, in, in_len, rec_offsets, n, cols, flags, first_bad, err, field + 1,
                       payload_pos);
}

// ---------------------------------------------------------------------------
// host memory (XDRG_HOST_PTRS): registry, staging ring, executor
// ---------------------------------------------------------------------------
// Buffers pinned through xdrg_host_register: host base -> (bytes, device view).
namespace {
struct HostReg {
    uint64_t bytes;
    uint8_t *dev;
};
std::mutex g_reg_mu;
std::map<uintptr_t, HostReg> g_reg;

// The registration holding [p, p + n), or nullptr.
bool reg_find(const void *p, uint64_t n, uintptr_t *base, HostReg *out) {
    std::lock_guard<std::mutex> lk(g_reg_mu);
    const uintptr_t a = (uintptr_t)p;
    auto it = g_reg.upper_bound(a);
    if (it == g_reg.begin()) return false;
    --it;
    if (a + n > it->first + it->second.bytes) return false;
    if (base) *base = it->first;
    if (out) *out = it->second;
    return true;
}

// hipPointerGetAttributes: 1 pinned / mapped host memory, 2 device memory, 0 other
int host_kind(const void *p) {
    hipPointerAttribute_t a;
    memset(&a, 0, sizeof a);
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    if (a.type == hipMemoryTypeHost) return 1;
    if (a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged) return 2;
    return 0;
}
}  // namespace

// A host span the DMA engines and kernels can reach without staging.
static bool span_pinned(const void *p, uint64_t n) {
    if (!n) return true;
    if (reg_find(p, n, nullptr, nullptr)) return true;
    return host_kind(p) == 1 && host_kind((const uint8_t *)p + n - 1) == 1;
}

// Device address of a pinned host span (XDRG_HOST_MAPPED), or nullptr.
static void *span_device(const void *p, uint64_t n) {
    if (!p) return nullptr;
    uintptr_t base = 0;
    HostReg r;
    if (reg_find(p, n ? n : 1, &base, &r)) return r.dev + ((uintptr_t)p - base);
    if (!span_pinned(p, n ? n : 1)) return nullptr;
    void *d = nullptr;
    if (hipHostGetDevicePointer(&d, (void *)p, 0) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    return d;
}

extern "C" int xdrg_host_register(xdrg_ctx *c, void *ptr, uint64_t bytes) {
    if (!ptr || !bytes) return inval(c, "nothing to register");
    DeviceGuard dg;
    if (c) HIPCHK(c, hipSetDevice(c->device));
    if (reg_find(ptr, 1, nullptr, nullptr)) return inval(c, "buffer already registered");
    HIPCHK(c, hipHostRegister(ptr, bytes, hipHostRegisterMapped | hipHostRegisterPortable));
    void *d = nullptr;
    const hipError_t e = hipHostGetDevicePointer(&d, ptr, 0);
    if (e != hipSuccess) {
        (void)hipHostUnregister(ptr);
        return hip_fail(c, e, "hipHostGetDevicePointer");
    }
    std::lock_guard<std::mutex> lk(g_reg_mu);
    g_reg[(uintptr_t)ptr] = HostReg{bytes, (uint8_t *)d};
    return XDRG_OK;
}

extern "C" int xdrg_host_unregister(xdrg_ctx *c, void *ptr) {
    {
        std::lock_guard<std::mutex> lk(g_reg_mu);
        auto it = g_reg.find((uintptr_t)ptr);
        if (it == g_reg.end()) return inval(c, "buffer not registered");
        g_reg.erase(it);
    }
    DeviceGuard dg;
    if (c) HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipHostUnregister(ptr));
    return XDRG_OK;
}

// Device buffers for a caller without a device allocator (GrizzlyMemoryManager
// allocate / wrap, grizzly/GrizzlyMemoryManager.java:42-57, in HBM).
extern "C" int xdrg_device_alloc(xdrg_ctx *c, uint64_t bytes, void **out) {
    if (!c || !out) return XDRG_E_INVAL;
    *out = nullptr;
    DeviceGuard dg;
    HIPCHK(c, hipSetDevice(c->device));
    void *p = nullptr;
    const hipError_t e = hipMalloc(&p, bytes ? bytes : 256);
    if (e != hipSuccess) {
        (void)hip_fail(c, e, "hipMalloc");
        return XDRG_E_NOMEM;
    }
    *out = p;
    return XDRG_OK;
}

extern "C" int xdrg_device_free(xdrg_ctx *c, void *p) {
    if (!c) return XDRG_E_INVAL;
    if (!p) return XDRG_OK;
    DeviceGuard dg;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamSynchronize(c->stream));   // (work queued on it may still read the buffer)
    HIPCHK(c, hipFree(p));
    return XDRG_OK;
}

extern "C" int xdrg_copy(xdrg_ctx *c, void *dst, const void *src, uint64_t bytes, int kind) {
    if (!c) return XDRG_E_INVAL;
    const hipMemcpyKind k = kind == XDRG_COPY_H2D ? hipMemcpyHostToDevice
                          : kind == XDRG_COPY_D2H ? hipMemcpyDeviceToHost
                          : kind == XDRG_COPY_D2D ? hipMemcpyDeviceToDevice : hipMemcpyDefault;
    if (k == hipMemcpyDefault) return inval(c, "xdrg_copy: kind must be XDRG_COPY_H2D / D2H / D2D");
    if (!bytes) return XDRG_OK;
    if (!dst || !src) return inval(c, "xdrg_copy: NULL buffer");
    DeviceGuard dg;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipMemcpyAsync(dst, src, bytes, k, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return XDRG_OK;
}

extern "C" int xdrg_ctx_host_staging(xdrg_ctx *c, uint64_t slot_bytes, uint32_t slots) {
    if (!c) return XDRG_E_INVAL;
    if (slots < 1 || slots > hs::kMaxSlots || slot_bytes < (1u << 16)) return inval(c, "staging: 1..8 slots of >= 64 KiB");
    c->ring.want_slot = slot_bytes;
    c->ring.want_n = slots;
    return XDRG_OK;
}

static void ring_free(xdrg_ctx *c) {
    StageRing &r = c->ring;
    if (r.comp) (void)hipStreamSynchronize(r.comp);
    if (r.h2d) (void)hipStreamSynchronize(r.h2d);
    if (r.d2h) (void)hipStreamSynchronize(r.d2h);
    if (r.dev) (void)hipFree(r.dev);
    if (r.bounce) (void)hipHostFree(r.bounce);
    r.dev = r.bounce = nullptr;
    r.slot = 0;
    r.n = 0;
    for (uint32_t i = 0; i < hs::kMaxSlots; ++i) {
        if (r.e_h2d[i]) (void)hipEventDestroy(r.e_h2d[i]);
        if (r.e_kern[i]) (void)hipEventDestroy(r.e_kern[i]);
        if (r.e_d2h[i]) (void)hipEventDestroy(r.e_d2h[i]);
        r.e_h2d[i] = r.e_kern[i] = r.e_d2h[i] = nullptr;
        r.d2h_rec[i] = false;
    }
    for (hipStream_t *st : {&r.h2d, &r.d2h, &r.comp})
        if (*st) {
            (void)hipStreamDestroy(*st);
            *st = nullptr;
        }
    if (r.d_res) (void)hipFree(r.d_res);
    if (r.h_res) (void)hipHostFree(r.h_res);
    r.d_res = r.h_res = nullptr;
}

// Slots of `slot` bytes; streams, events and status words on first use.
static int ring_ready(xdrg_ctx *c, uint64_t slot) {
    StageRing &r = c->ring;
    if (!r.comp) {
        HIPCHK(c, hipStreamCreateWithFlags(&r.h2d, hipStreamNonBlocking));
        HIPCHK(c, hipStreamCreateWithFlags(&r.d2h, hipStreamNonBlocking));
        HIPCHK(c, hipStreamCreateWithFlags(&r.comp, hipStreamNonBlocking));
        for (uint32_t i = 0; i < hs::kMaxSlots; ++i) {
            HIPCHK(c, hipEventCreateWithFlags(&r.e_h2d[i], hipEventDisableTiming));
            HIPCHK(c, hipEventCreateWithFlags(&r.e_kern[i], hipEventDisableTiming));
            HIPCHK(c, hipEventCreateWithFlags(&r.e_d2h[i], hipEventDisableTiming));
        }
        HIPCHK(c, hipMalloc(&r.d_res, sizeof(uint64_t) * kResWords * hs::kMaxSlots));
        HIPCHK(c, hipHostMalloc(&r.h_res, sizeof(uint64_t) * kResWords * hs::kMaxSlots, hipHostMallocDefault));
    }
    slot = hs::up(slot, 1 << 16);
    if (r.dev && r.slot == slot && r.n == r.want_n) return XDRG_OK;
    HIPCHK(c, hipStreamSynchronize(r.h2d));
    HIPCHK(c, hipStreamSynchronize(r.d2h));
    HIPCHK(c, hipStreamSynchronize(r.comp));
    if (r.dev) HIPCHK(c, hipFree(r.dev));
    if (r.bounce) HIPCHK(c, hipHostFree(r.bounce));
    r.dev = r.bounce = nullptr;
    for (uint32_t i = 0; i < hs::kMaxSlots; ++i) r.d2h_rec[i] = false;
    r.n = r.want_n;
    r.slot = slot;
    const hipError_t e = hipMalloc(&r.dev, r.slot * r.n);
    if (e != hipSuccess) {
        r.dev = nullptr;
        r.slot = 0;
        return hip_fail(c, e, "staging ring hipMalloc");
    }
    return XDRG_OK;
}

static int frame_walk(xdrg_ctx *c, const uint8_t *in, uint64_t len, uint8_t *payload, uint64_t payload_cap,
                      uint64_t *msg_offsets, uint64_t cap, uint64_t *n_msgs, uint64_t *consumed,
                      uint64_t *frags = nullptr, uint64_t *body_bytes = nullptr, uint64_t stride = 0,
                      bool *uniform = nullptr);

// host_stage.h executor on one context: copies on the ring's H2D / D2H
// streams, kernels on its compute stream, ordered by per-slot events.
struct HipExec {
    xdrg_ctx *c;
    const xdrg_schema *s;
    StageRing &r;
    HipExec(xdrg_ctx *c_, const xdrg_schema *s_) : c(c_), s(s_), r(c_->ring) {}

    uint32_t nslots() const { return r.n; }
    uint64_t slot_bytes() const { return r.slot; }
    uint8_t *slot(uint32_t i) const { return r.dev + (uint64_t)i * r.slot; }
    uint8_t *bounce(uint32_t i) {
        if (!r.bounce && hipHostMalloc(&r.bounce, r.slot * r.n, hipHostMallocDefault) != hipSuccess) {
            (void)hipGetLastError();
            r.bounce = nullptr;
            c->err = "staging bounce hipHostMalloc failed";
            return nullptr;
        }
        return r.bounce + (uint64_t)i * r.slot;
    }
    bool pinned(const void *p, uint64_t n) const { return span_pinned(p, n); }
    int wait_slot(uint32_t i) {
        if (r.d2h_rec[i]) HIPCHK(c, hipEventSynchronize(r.e_d2h[i]));
        return XDRG_OK;
    }
    // the device's view of a host span when the copy kernels move it (tuning key 26)
    const uint8_t *link_view(const void *host, uint64_t n) const {
        return c->tune.stage_copy ? (const uint8_t *)span_device(host, n) : nullptr;
    }
    int dma_h2d(uint8_t *dev, const void *host, uint64_t n) {
        if (const uint8_t *v = link_view(host, n)) {
            HIPCHK(c, (hipError_t)launch_copy_link(dev, v, n, r.h2d));
            return XDRG_OK;
        }
        HIPCHK(c, hipMemcpyAsync(dev, host, n, hipMemcpyHostToDevice, r.h2d));
        return XDRG_OK;
    }
    int h2d_done(uint32_t i) {
        HIPCHK(c, hipEventRecord(r.e_h2d[i], r.h2d));
        return XDRG_OK;
    }
    int kernel_begin(uint32_t i) {
        HIPCHK(c, hipStreamWaitEvent(r.comp, r.e_h2d[i], 0));
        HIPCHK(c, hipMemsetAsync(r.d_res + (uint64_t)i * kResWords, 0, 16, r.comp));
        return XDRG_OK;
    }
    int add_u64(int on_d2h, uint64_t *p, uint64_t n, uint64_t delta) {
        HIPCHK(c, (hipError_t)launch_add_u64(p, n, delta, on_d2h ? r.d2h : r.comp));
        return XDRG_OK;
    }
    int add_pos(uint64_t *p, uint64_t n, uint64_t delta) {
        HIPCHK(c, (hipError_t)launch_add_pos(p, n, delta, r.d2h));
        return XDRG_OK;
    }
    int encode(uint32_t i, const xdrg_column *dc, uint64_t m, uint8_t *out, uint64_t cap, uint64_t *rec,
               uint32_t flags, uint32_t byref, uint64_t *ref) {
        hipStream_t keep = c->stream;
        c->stream = r.comp;
        const int rc = encode_impl(c, s, dc, m, out, cap, rec, flags | XDRG_ASYNC, r.d_res + (uint64_t)i * kResWords,
                                   byref, ref);
        c->stream = keep;
        return rc;
    }
    int decode(uint32_t i, const uint8_t *in, uint64_t len, const uint64_t *rec, uint64_t m, xdrg_column *dc,
               uint32_t flags, uint32_t byref, uint64_t *ref) {
        hipStream_t keep = c->stream;
        c->stream = r.comp;
        uint64_t *w = r.d_res + (uint64_t)i * kResWords;
        const int rc = decode_impl(c, s, in, len, rec, m, dc, flags | XDRG_ASYNC, w, (int *)(w + 1), byref, ref);
        c->stream = keep;
        return rc;
    }
    // the two halves of a repeated-group decode (hs::stage_receive); the counts
    // land in the slot's result words 47.. (kernel_end writes at most 2 + 32)
    int decode_count(uint32_t i, const uint8_t *in, uint64_t len, const uint64_t *rec, uint64_t m, uint32_t flags,
                     uint64_t *tot, uint64_t *bad) {
        hipStream_t keep = c->stream;
        c->stream = r.comp;
        std::vector<xdrg_column> dummy(s->f.size());
        uint64_t *h = r.h_res + (uint64_t)i * kResWords + (kResWords - 1 - kMaxSlots);
        int rc = decode_impl(c, s, in, len, rec, m, dummy.data(), flags | XDRG_ASYNC | kDecCount, nullptr, nullptr, 0,
                             nullptr, h);
        c->stream = keep;
        if (rc) return rc;
        HIPCHK(c, hipStreamSynchronize(r.comp));
        uint32_t ns = 0;
        for (size_t k = 0; k < s->f.size(); ++k)
            ns += (s->f[k].type == XDRG_T_GROUP) ? s->f[k].kind != XDRG_K_FIXED : s->f[k].kind == XDRG_K_DYNAMIC;
        memcpy(tot, h + 1, 8 * (size_t)ns);
        *bad = h[0] == kNoError ? m : (uint64_t)(h[0] >> 16);
        return XDRG_OK;
    }
    int decode_place(uint32_t i, const uint8_t *in, uint64_t len, const uint64_t *rec, uint64_t m, xdrg_column *dc,
                     uint32_t flags, uint32_t, uint64_t *) {
        return decode(i, in, len, rec, m, dc, flags | kDecPlace, 0, nullptr);
    }
    int kernel_end(uint32_t i, const uint64_t *const *extra, const uint64_t *const *index, const uint64_t *limit,
                   uint32_t nextra) {
        if (nextra + 2 > kResWords) return inval(c, "too many dynamic fields for the staging status");
        uint64_t *w = r.d_res + (uint64_t)i * kResWords;
        for (uint32_t j = 0; j < nextra; ++j) {
            if (index && index[j])
                HIPCHK(c, (hipError_t)launch_pick_u64(w + 2 + j, extra[j], index[j], limit[j], r.comp));
            else HIPCHK(c, hipMemcpyAsync(w + 2 + j, extra[j], 8, hipMemcpyDeviceToDevice, r.comp));
        }
        HIPCHK(c, hipMemcpyAsync(r.h_res + (uint64_t)i * kResWords, w, 8 * (2 + nextra), hipMemcpyDeviceToHost, r.comp));
        r.nres[i] = 2 + nextra;
        HIPCHK(c, hipEventRecord(r.e_kern[i], r.comp));
        return XDRG_OK;
    }
    const uint64_t *res_word(uint32_t i, uint32_t j) const { return r.d_res + (uint64_t)i * kResWords + 2 + j; }
    int wait_kernel(uint32_t i, uint64_t *w) {
        HIPCHK(c, hipEventSynchronize(r.e_kern[i]));
        memcpy(w, r.h_res + (uint64_t)i * kResWords, 8 * r.nres[i]);
        w[1] &= 0xffffffffull;   // err is an int (the upper half was zeroed)
        return XDRG_OK;
    }
    int d2h_begin(uint32_t i) {
        HIPCHK(c, hipStreamWaitEvent(r.d2h, r.e_kern[i], 0));
        return XDRG_OK;
    }
    int dma_d2h(void *host, const uint8_t *dev, uint64_t n) {
        if (const uint8_t *v = link_view(host, n)) {
            HIPCHK(c, (hipError_t)launch_copy_link((uint8_t *)v, dev, n, r.d2h));
            return XDRG_OK;
        }
        HIPCHK(c, hipMemcpyAsync(host, dev, n, hipMemcpyDeviceToHost, r.d2h));
        return XDRG_OK;
    }
    int dma_d2h_2d(void *host, uint64_t hp, const uint8_t *dev, uint64_t dp, uint64_t w, uint64_t rows) {
        HIPCHK(c, hipMemcpy2DAsync(host, hp, dev, dp, w, rows, hipMemcpyDeviceToHost, r.d2h));
        return XDRG_OK;
    }
    int d2h_done(uint32_t i) {
        HIPCHK(c, hipEventRecord(r.e_d2h[i], r.d2h));
        r.d2h_rec[i] = true;
        return XDRG_OK;
    }
    int grow(uint64_t slot) { return ring_ready(c, slot > r.slot ? slot : r.slot); }
    // receive (hs::stage_receive): the record-mark walk of a slot window on the
    // compute stream (host-blocking), bodies assembled by a second walk when asked
    int scan(uint32_t, const uint8_t *win, uint64_t wlen, uint64_t cap, uint64_t *offs, int bodies,
             uint8_t *body_dst, uint64_t *boffs, uint64_t *res) {
        hipStream_t keep = c->stream;
        c->stream = r.comp;
        uint64_t nm = 0, used = 0, nf = 0;
        int rc = frame_walk(c, win, wlen, nullptr, 0, offs, cap, &nm, &used, &nf, nullptr);
        res[0] = res[1] = res[3] = 0;
        res[2] = 1;
        if (rc == XDRG_E_INCOMPLETE) rc = XDRG_OK;
        if (!rc && nm) {
            res[0] = nm;
            res[1] = used;
            res[2] = nf == nm;
            if (bodies == 2 || (bodies == 1 && nf != nm)) {
                uint8_t *dst = body_dst;
                if (!dst) {
                    rc = ensure_rx(c, used + 64);
                    dst = c->d_rx;
                }
                uint64_t nm2 = 0, used2 = 0, bytes = 0;
                if (!rc) rc = frame_walk(c, win, wlen, dst, used, boffs, nm, &nm2, &used2, nullptr, &bytes);
                res[3] = bytes;
            }
        }
        c->stream = keep;
        return rc;
    }
    const uint8_t *body() const { return c->d_rx; }
    int d2d(uint8_t *dst, const uint8_t *src, uint64_t n) {
        if (n) HIPCHK(c, hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToDevice, r.h2d));
        return XDRG_OK;
    }
    int offs_copy(uint64_t *dst, const uint64_t *src, uint64_t n, uint64_t delta) {
        HIPCHK(c, hipMemcpyAsync(dst, src, n * 8, hipMemcpyDeviceToDevice, r.comp));
        HIPCHK(c, (hipError_t)launch_add_u64(dst, n, delta, r.comp));
        return XDRG_OK;
    }
    // every copy and kernel of the call has finished (the caller's buffers are free again)
    int finish() {
        HIPCHK(c, hipStreamSynchronize(r.h2d));
        HIPCHK(c, hipStreamSynchronize(r.comp));
        HIPCHK(c, hipStreamSynchronize(r.d2h));
        return XDRG_OK;
    }
};

static void stage_schema(const xdrg_schema *s, hs::Schema &v) {
    v.f.resize(s->f.size());
    uint64_t ndyn = 0;
    for (size_t k = 0; k < s->f.size(); ++k) {
        const xdrg_field &f = s->f[k];
        v.f[k] = hs::Field{f.type, f.kind, f.count, s->nsz[k], s->xsz[k], s->xbytes[k], s->grp[k], 0};
        ndyn += f.kind == XDRG_K_DYNAMIC;
        if (f.type != XDRG_T_GROUP) continue;
        // fewest XDR bytes of an element: a list's TRUE, its unconditional
        // direct members (an inner group: its count word or its closing FALSE)
        uint32_t e = f.kind == XDRG_K_LIST ? 4 : 0;
        for (uint32_t j = 1; j <= f.reserved; ++j) {
            const xdrg_field &m = s->f[k + j];
            if (s->grp[k + j] != k + 1 || s->cond[k + j]) continue;
            if (m.type == XDRG_T_GROUP) e += m.kind == XDRG_K_FIXED ? 0 : 4;
            else e += m.kind == XDRG_K_DYNAMIC ? 4 : s->xbytes[k + j];
        }
        v.f[k].emin = e;
        v.groups = true;
    }
    v.fixed_part = s->fixed_part;
    v.var_size = s->var_size;
    // a well-formed record: every fixed field, a length word per dynamic field
    // (absent arms of a conditional schema may take any of it away)
    v.min_xdr = s->ncond || s->ngroups ? 0 : s->fixed_part + 4 * ndyn;
}

// Device views of host columns (XDRG_HOST_MAPPED).  Every span a kernel may
// touch must lie inside one registration (or one pinned allocation): a fixed
// column's rows, a dynamic column's n + 1 offsets and its values (encode:
// offsets[n] elements; decode: cap), a group member's rows over the batch's
// elements (encode: the group's offsets[n]; decode: the group's element
// capacity).  A buffer registered shorter than its use is refused.
// Every column's host span (bytes the call touches: rows x stride, values,
// offsets + 1) mapped by fn(ptr, bytes) -> the device address (nullptr: not
// covered).  XDRG_HOST_MAPPED maps through the registrations; the bounce path
// through device scratch.
// byref = 1 + a field whose values the call never touches (a by-reference
// payload, a view): its offsets map, its data is NULL.
template <typename F>
static int map_cols(xdrg_ctx *c, const xdrg_schema *s, const xdrg_column *cols, uint64_t n, bool decode,
                    std::vector<xdrg_column> &out, F fn, uint32_t byref = 0) {
    out.assign(cols, cols + s->f.size());
    // native rows of every field's column (a group precedes its members):
    // records, a FIXED group's rows x count, else the group's elements
    std::vector<uint64_t> rows_of(s->f.size(), n);
    for (size_t k = 0; k < s->f.size(); ++k) {
        if (!s->grp[k]) continue;
        const size_t g = s->grp[k] - 1;
        const xdrg_field &gf = s->f[g];
        if (gf.kind == XDRG_K_FIXED) rows_of[k] = rows_of[g] * gf.count;
        else if (decode) rows_of[k] = cols[g].cap;
        else rows_of[k] = rows_of[g] ? cols[g].offsets[rows_of[g]] : 0;   // host memory: the caller's offsets
    }
    for (size_t k = 0; k < s->f.size(); ++k) {
        xdrg_column &d = out[k];
        const xdrg_field &f = s->f[k];
        const uint64_t rows = rows_of[k];
        if (f.type == XDRG_T_GROUP) {
            if (d.offsets && f.kind != XDRG_K_FIXED) {
                d.offsets = (uint64_t *)fn(cols[k].offsets, (rows + 1) * 8);
                if (!d.offsets) return inval(c, "XDRG_HOST_MAPPED: group offsets not registered for every row + 1");
            }
            continue;
        }
        if (f.kind == XDRG_K_DYNAMIC) {
            d.offsets = (uint64_t *)fn(cols[k].offsets, (rows + 1) * 8);
            if (!d.offsets) return inval(c, "XDRG_HOST_MAPPED: column offsets not registered for every row + 1");
            if (k + 1 == byref) {
                d.data = nullptr;
                d.cap = 0;
                continue;
            }
            const uint64_t vals = decode ? cols[k].cap : (rows ? cols[k].offsets[rows] : 0);
            if (d.data || vals) {
                d.data = fn(cols[k].data, vals * s->nsz[k]);
                if (!d.data) return inval(c, "XDRG_HOST_MAPPED: column values not registered for their extent");
            }
            continue;
        }
        if (!d.data) continue;
        const uint64_t elem = (uint64_t)s->nsz[k] * (f.kind == XDRG_K_FIXED ? f.count : 1);
        const int64_t st = eff_stride(s, k, cols[k]);
        // no rows: no bytes (a member column of a group without elements may be
        // a zero-length allocation); a constant column (stride 0): one row
        const uint64_t span = rows == 0 ? 0 : st == 0 ? elem : (uint64_t)st * (rows - 1) + elem;
        d.data = fn(cols[k].data, span);
        if (!d.data) return inval(c, "XDRG_HOST_MAPPED: column data not registered for every row");
    }
    return XDRG_OK;
}
static int mapped_cols(xdrg_ctx *c, const xdrg_schema *s, const xdrg_column *cols, uint64_t n, bool decode,
                       std::vector<xdrg_column> &out, uint32_t byref = 0) {
    // a span of no bytes is never dereferenced: any valid device address stands in
    return map_cols(c, s, cols, n, decode, out, [c](const void *p, uint64_t b) -> void * {
        void *d = span_device(p, b);
        return d || b ? d : (void *)c->d_stat;
    }, byref);
}

// Host memory of a schema the staging ring does not window (a T x[N] group
// inside a counted group's elements, hs::stage_groups_ok) goes whole through
// device scratch: the host spans the call touches — columns, stream, offsets;
// overlapping ones merged (array-of-structs columns share bytes) — are copied
// in, the device call runs, and the spans it writes are copied back.
struct Bounce {
    struct Span { const uint8_t *h; uint64_t len; bool out; };
    struct Reg { uint8_t *h; uint64_t len; uint8_t *d; bool out; };
    std::vector<Span> spans;
    std::vector<Reg> regs;
    uint8_t *empty = nullptr;   // stands in for every span of no bytes (never dereferenced)
    void add(const void *p, uint64_t len, bool out) { if (p && len) spans.push_back({(const uint8_t *)p, len, out}); }
    // merge the spans, allocate and fill the device regions
    int place(xdrg_ctx *c) {
        std::sort(spans.begin(), spans.end(), [](const Span &a, const Span &b) { return a.h < b.h; });
        for (const Span &sp : spans) {
            if (!regs.empty() && sp.h <= regs.back().h + regs.back().len) {
                Reg &r = regs.back();
                const uint8_t *e = std::max<const uint8_t *>(r.h + r.len, sp.h + sp.len);
                r.len = (uint64_t)(e - r.h);
                r.out |= sp.out;
            } else {
                regs.push_back({(uint8_t *)sp.h, sp.len, nullptr, sp.out});
            }
        }
        for (Reg &r : regs) {
            HIPCHK(c, hipMallocAsync((void **)&r.d, r.len, c->stream));
            HIPCHK(c, hipMemcpyAsync(r.d, r.h, r.len, hipMemcpyHostToDevice, c->stream));
        }
        HIPCHK(c, hipMallocAsync((void **)&empty, 256, c->stream));
        return XDRG_OK;
    }
    // the device address of host p, a span of `len` bytes (0: the stand-in)
    void *dev(const void *p, uint64_t len) const {
        if (!p) return nullptr;
        const uint8_t *q = (const uint8_t *)p;
        for (const Reg &r : regs)
            if (q >= r.h && q < r.h + r.len) return r.d + (q - r.h);
        return len ? nullptr : empty;
    }
    int finish(xdrg_ctx *c, bool copy_back) {
        int rc = XDRG_OK;
        for (Reg &r : regs) {
            if (copy_back && r.out && hipMemcpyAsync(r.h, r.d, r.len, hipMemcpyDeviceToHost, c->stream) != hipSuccess)
                rc = XDRG_E_HIP;
            (void)hipFreeAsync(r.d, c->stream);
        }
        if (empty) (void)hipFreeAsync(empty, c->stream);
        if (hipStreamSynchronize(c->stream) != hipSuccess) rc = XDRG_E_HIP;
        return rc;
    }
};
static int bounce_encode(xdrg_ctx *c, const xdrg_schema *s, const xdrg_column *cols, uint64_t n, uint8_t *out,
                         uint64_t out_cap, uint64_t *rec_offsets, uint32_t dflags, uint64_t *out_len) {
    Bounce B;
    std::vector<xdrg_column> dc;
    c->host_bounces++;
    int rc = map_cols(c, s, cols, n, false, dc, [&](const void *p, uint64_t b) { B.add(p, b, false); return (void *)p; });
    if (rc) return rc;
    B.add(out, out_cap, true);
    B.add(rec_offsets, (n + 1) * 8, true);
    HIPCHK(c, hipStreamSynchronize(c->stream));   // the caller's earlier work on this context
    rc = B.place(c);
    if (rc) { (void)B.finish(c, false); return rc; }
    rc = map_cols(c, s, cols, n, false, dc, [&](const void *p, uint64_t b) { return B.dev(p, b); });
    uint64_t len = 0;
    if (!rc) rc = encode_impl(c, s, dc.data(), n, (uint8_t *)B.dev(out, out_cap), out_cap,
                              (uint64_t *)B.dev(rec_offsets, (n + 1) * 8), dflags, &len, 0, nullptr);
    const int fr = B.finish(c, rc == XDRG_OK);
    if (!rc && out_len) *out_len = len;
    return rc ? rc : fr;
}
static int bounce_decode(xdrg_ctx *c, const xdrg_schema *s, const uint8_t *in, uint64_t in_len,
                         const uint64_t *rec_offsets, uint64_t n, xdrg_column *cols, uint32_t dflags,
                         uint64_t *first_bad, int *err) {
    Bounce B;
    std::vector<xdrg_column> dc;
    c->host_bounces++;
    int rc = map_cols(c, s, cols, n, true, dc, [&](const void *p, uint64_t b) { B.add(p, b, true); return (void *)p; });
    if (rc) return rc;
    B.add(in, in_len, false);
    B.add(rec_offsets, (n + 1) * 8, false);
    HIPCHK(c, hipStreamSynchronize(c->stream));
    rc = B.place(c);
    if (rc) { (void)B.finish(c, false); return rc; }
    rc = map_cols(c, s, cols, n, true, dc, [&](const void *p, uint64_t b) { return B.dev(p, b); });
    if (!rc) rc = decode_impl(c, s, (const uint8_t *)B.dev(in, in_len), in_len,
                              (const uint64_t *)B.dev(rec_offsets, (n + 1) * 8), n,
                              dc.data(), dflags, first_bad, err, 0, nullptr);
    const bool dec_err = rc && *err;   // a decode error: the records before it are delivered
    const int fr = B.finish(c, rc == XDRG_OK || dec_err);
    return rc ? rc : fr;
}

static int host_common(xdrg_ctx *c, const xdrg_schema *s, uint32_t flags) {
    if (!c || !s) return XDRG_E_INVAL;
    if (flags & XDRG_ASYNC) return inval(c, "XDRG_HOST_PTRS calls are synchronous (no XDRG_ASYNC)");
    return XDRG_OK;
}

// byref / splice: xdrg_encode_batch_shallow on host memory — the payload
// field's values are never read (nor staged: only the heads cross PCIe), its
// offsets are; splice is a host array of n entries.
static int host_encode(xdrg_ctx *c, const xdrg_schema *s, const xdrg_column *cols, uint64_t n, uint8_t *out,
                       uint64_t out_cap, uint64_t *rec_offsets, uint32_t flags, uint64_t *out_len,
                       uint32_t byref, uint64_t *splice) {
    int rc = host_common(c, s, flags);
    if (rc) return rc;
    DeviceGuard dg;
    HIPCHK(c, hipSetDevice(c->device));
    if (!aligned(out, 4)) return inval(c, "XDR buffer not 4-byte aligned");
    if (n && !out) return inval(c, "XDR buffer is NULL");
    rc = check_columns(c, s, cols, n, false);
    if (rc) return rc;
    const uint32_t dflags = flags & XDRG_FRAME_RM;
    if (byref && s->ngroups) return inval(c, "by-reference payloads in a schema with repeated groups");
    if (flags & XDRG_HOST_MAPPED) {
        std::vector<xdrg_column> dc;
        rc = mapped_cols(c, s, cols, n, false, dc, byref);
        if (rc) return rc;
        uint8_t *dout = n ? (uint8_t *)span_device(out, out_cap) : out;
        uint64_t *drec = rec_offsets ? (uint64_t *)span_device(rec_offsets, (n + 1) * 8) : nullptr;
        if ((n && !dout) || (rec_offsets && !drec)) return inval(c, "XDRG_HOST_MAPPED: stream / offsets not registered");
        uint64_t *dspl = byref && n ? (uint64_t *)span_device(splice, n * 8) : splice;
        if (byref && n && !dspl) return inval(c, "XDRG_HOST_MAPPED: splice positions not registered");
        return encode_impl(c, s, dc.data(), n, dout, out_cap, drec, dflags, out_len, byref, dspl);
    }
    hs::Schema v;
    stage_schema(s, v);
    if (!hs::stage_groups_ok(v)) return bounce_encode(c, s, cols, n, out, out_cap, rec_offsets, dflags, out_len);
    rc = ring_ready(c, c->ring.slot > c->ring.want_slot ? c->ring.slot : c->ring.want_slot);
    if (rc) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));   // the caller's earlier work on this context
    HipExec x(c, s);
    rc = hs::stage_encode(x, v, cols, n, out, out_cap, rec_offsets, dflags, out_len, byref, splice);
    const int fr = x.finish();
    if (rc == XDRG_E_CAPACITY) c->err = "output buffer too small";
    else if (rc == XDRG_E_INVAL && c->err.empty()) c->err = "host columns: unsupported layout";
    return rc ? rc : fr;
}

// byref / payload_pos: xdrg_decode_batch_view on host memory — the stream
// is staged, the payload field's offsets come back as for a copy, its values
// are never written, payload_pos (host, n) = offsets in `in`.
static int host_decode(xdrg_ctx *c, const xdrg_schema *s, const uint8_t *in, uint64_t in_len,
                       const uint64_t *rec_offsets, uint64_t n, xdrg_column *cols, uint32_t flags,
                       uint64_t *first_bad, int *err, uint32_t byref, uint64_t *payload_pos) {
    int rc = host_common(c, s, flags);
    if (rc) return rc;
    DeviceGuard dg;
    HIPCHK(c, hipSetDevice(c->device));
    if (!aligned(in, 4)) return inval(c, "XDR buffer not 4-byte aligned");
    if (n && in_len && !in) return inval(c, "XDR buffer is NULL");
    if (s->var_size && !rec_offsets) return inval(c, "variable-size schema needs record offsets");
    rc = check_columns(c, s, cols, n, true);
    if (rc) return rc;
    const uint32_t dflags = flags & XDRG_FRAME_RM;
    if (byref && s->ngroups) return inval(c, "payload views in a schema with repeated groups");
    if (flags & XDRG_HOST_MAPPED) {
        std::vector<xdrg_column> dc;
        rc = mapped_cols(c, s, cols, n, true, dc, byref);
        if (rc) return rc;
        const uint8_t *din = in_len ? (const uint8_t *)span_device(in, in_len) : in;
        const uint64_t *drec = rec_offsets ? (const uint64_t *)span_device(rec_offsets, (n + 1) * 8) : nullptr;
        if ((in_len && !din) || (rec_offsets && !drec)) return inval(c, "XDRG_HOST_MAPPED: stream / offsets not registered");
        uint64_t *dpos = byref && n ? (uint64_t *)span_device(payload_pos, n * 8) : payload_pos;
        if (byref && n && !dpos) return inval(c, "XDRG_HOST_MAPPED: payload positions not registered");
        return decode_impl(c, s, din, in_len, drec, n, dc.data(), dflags, first_bad, err, byref, dpos);
    }
    hs::Schema v;
    stage_schema(s, v);
    if (!hs::stage_groups_ok(v)) return bounce_decode(c, s, in, in_len, rec_offsets, n, cols, dflags, first_bad, err);
    rc = ring_ready(c, c->ring.slot > c->ring.want_slot ? c->ring.slot : c->ring.want_slot);
    if (rc) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HipExec x(c, s);
    rc = hs::stage_decode(x, v, in, in_len, rec_offsets, n, cols, dflags, first_bad, err, byref, payload_pos);
    const int fr = x.finish();
    if (rc && rc != XDRG_E_INVAL && rc != XDRG_E_HIP && rc != XDRG_E_NOMEM) c->err = xdrg_status_string(rc);
    else if (rc == XDRG_E_INVAL && c->err.empty()) c->err = "host columns: unsupported layout";
    return rc ? rc : fr;
}

// ---------------------------------------------------------------------------
// framing
// ---------------------------------------------------------------------------
// Carve the frame-walk workspace for a stream of Q words (the fragment list:
// one entry per word at most).  The speculative walk needs neither the exact
// kernels' tables (exact: the 2-B exit table and the active-word lists,
// 6 B per word) nor, for stream offsets, the fragment list (frags: 8 B per
// word): without them the workspace is ~0.3 B per word instead of ~14.
static int frame_ws(xdrg_ctx *c, uint64_t Q, FrameWs &ws, bool exact = true, bool frags = true) {
    const uint64_t nsup = (Q + kFSuper - 1) / kFSuper + 1, nsub = nsup * (kFSuper / kFChunk);
    const uint64_t ngrp = nsup / 64 + 2;
    const uint64_t F = Q + 2;
    size_t off = 0;
    auto take = [&](size_t bytes) { const size_t o = off; off += (bytes + 255) & ~(size_t)255; return o; };
    const size_t o_ex = take(exact ? 2 * Q : 0), o_al = take(exact ? 4 * (size_t)kFChunk * nsub : 0), o_ac = take(4 * nsub), o_se = take(4 * nsup), o_wt = take(4 * 256 * nsup), o_gs = take(4 * 256 * (nsup + 64)), o_ge = take(4 * 256 * ngrp), o_gn = take(4 * ngrp), o_sb = take(sizeof(FrameSub) * nsub),
                 o_fb = take(512 * nsub), o_lb = take(512 * nsub), o_su = take(sizeof(FrameSuper) * nsup),
                 o_ba = take(sizeof(FrameBase) * nsup), o_fp = take(frags ? 8 * F : 0), o_sx = take(8 * nsup), o_lw = take(8 * (5 * nsup + 1)), o_re = take(64);
    if (off > c->fws_bytes) {
        if (c->d_fws) {
            HIPCHK(c, hipStreamSynchronize(c->stream));
            HIPCHK(c, hipFree(c->d_fws));
            c->d_fws = nullptr;
            c->fws_bytes = 0;
        }
        HIPCHK(c, hipMalloc(&c->d_fws, off));
        c->fws_bytes = off;
    }
    uint8_t *b = (uint8_t *)c->d_fws;
    ws.exitR = (uint16_t *)(b + o_ex);
    ws.alist = (uint32_t *)(b + o_al);
    ws.acnt = (uint32_t *)(b + o_ac);
    ws.sentry = (uint32_t *)(b + o_se);
    ws.wtab = (uint32_t *)(b + o_wt);
    ws.gsx = (uint32_t *)(b + o_gs);
    ws.gexit = (uint32_t *)(b + o_ge);
    ws.gentry = (uint32_t *)(b + o_gn);
    ws.sub = (FrameSub *)(b + o_sb);
    ws.fbits = (uint32_t *)(b + o_fb);
    ws.lbits = (uint32_t *)(b + o_lb);
    ws.sup = (FrameSuper *)(b + o_su);
    ws.bases = (FrameBase *)(b + o_ba);
    ws.frag_pos = (uint64_t *)(b + o_fp);
    ws.sx = (uint32_t *)(b + o_sx);
    ws.lbw = (uint64_t *)(b + o_lw);
    ws.res = (uint64_t *)(b + o_re);
    return XDRG_OK;
}

// RpcMessageParserTCP.handleRead over a whole buffer: the complete messages
// (at most cap) as stream offsets (payload == NULL) or assembled bodies.
// One host round trip for xdrg_frame_scan (two for xdrg_deframe: the payload
// size is checked before the bodies move).
// stride > 0 (stream offsets): *uniform = every delivered message starts at
// its index x stride (checked by k_fr_emit as it writes the offsets; the
// parallel walk only).
static int frame_walk(xdrg_ctx *c, const uint8_t *in, uint64_t len, uint8_t *payload, uint64_t payload_cap,
                      uint64_t *msg_offsets, uint64_t cap, uint64_t *n_msgs, uint64_t *consumed,
                      uint64_t *frags, uint64_t *body_bytes, uint64_t stride, bool *uniform) {
    if (uniform) *uniform = false;
    if (!c || !msg_offsets || !n_msgs) return XDRG_E_INVAL;
    if (len && !in) return inval(c, "stream is NULL");
    if (len > kFMaxLen) return inval(c, "stream longer than 16 GiB");
    DeviceGuard dg;
    HIPCHK(c, hipSetDevice(c->device));
    *n_msgs = 0;
    if (consumed) *consumed = 0;
    TimedLaunch t(c, XDRG_KERNEL_FRAME_SCAN);
    HIPCHK(c, hipMemsetAsync(msg_offsets, 0, 8, c->stream));
    const uint64_t Q = len / 4;
    FrameWs ws;
    const bool stream_offsets = payload == nullptr;
    bool serial = !aligned(in, 4) || Q == 0;
    bool exact = !c->tune.frame_spec;
    int rc = frame_ws(c, Q, ws, exact || serial, !stream_offsets || serial);
    if (rc) return rc;
    if (!serial) {   // parallel walk over words; a real chain meeting a size % 4 != 0 walks again over bytes
        if (!exact) {   // the speculative walk; the exact kernels when it gives up (res[7])
            ++c->frame_spec_calls;
            HIPCHK(c, (hipError_t)frame_spec(in, len, ws, cap, stream_offsets, msg_offsets, !stream_offsets,
                                             c->tune.emit_per, c->tune.emit_wave, stride, false, c->stream));
            HIPCHK(c, hipMemcpyAsync(c->h_stat + 2, ws.res, 64, hipMemcpyDeviceToHost, c->stream));
            HIPCHK(c, hipStreamSynchronize(c->stream));
            if ((c->h_stat[2 + 7] & 2) && c->h_stat[2] != kFUnal) {   // a failed entry check: re-walks
                HIPCHK(c, (hipError_t)frame_spec(in, len, ws, cap, stream_offsets, msg_offsets, !stream_offsets,
                                                 c->tune.emit_per, c->tune.emit_wave, stride, true, c->stream));
                HIPCHK(c, hipMemcpyAsync(c->h_stat + 2, ws.res, 64, hipMemcpyDeviceToHost, c->stream));
                HIPCHK(c, hipStreamSynchronize(c->stream));
            }
            c->frame_spec_rewalks += c->h_stat[2 + 7] >> 8;
            if (c->h_stat[2 + 7] & 1) {
                ++c->frame_spec_gave_up;
                exact = true;
                HIPCHK(c, hipMemsetAsync(msg_offsets, 0, 8, c->stream));
                rc = frame_ws(c, Q, ws);   // (the exact kernels' tables)
                if (rc) return rc;
            }
        }
        if (exact) {
            HIPCHK(c, (hipError_t)frame_parallel(in, len, 4, ws, cap, stream_offsets, msg_offsets, !stream_offsets,
                                                 c->tune.emit_per, c->tune.emit_wave, stride, c->stream));
            HIPCHK(c, hipMemcpyAsync(c->h_stat + 2, ws.res, 56, hipMemcpyDeviceToHost, c->stream));
            HIPCHK(c, hipStreamSynchronize(c->stream));
        }
        if (c->h_stat[2] == kFUnal) {
            if (len < kFByteMaxLen) {
                rc = frame_ws(c, frame_positions(len, 1), ws);
                if (rc) return rc;
                HIPCHK(c, hipMemsetAsync(msg_offsets, 0, 8, c->stream));
                HIPCHK(c, (hipError_t)frame_parallel(in, len, 1, ws, cap, stream_offsets, msg_offsets,
                                                     !stream_offsets, c->tune.emit_per, c->tune.emit_wave, stride,
                                                     c->stream));
                HIPCHK(c, hipMemcpyAsync(c->h_stat + 2, ws.res, 56, hipMemcpyDeviceToHost, c->stream));
                HIPCHK(c, hipStreamSynchronize(c->stream));
            } else {
                serial = true;
                rc = frame_ws(c, Q, ws);
                if (rc) return rc;
            }
        }
    }
    if (serial) {
        if (len < 4) {
            c->h_stat[2 + 1] = c->h_stat[2 + 3] = c->h_stat[2 + 4] = c->h_stat[2 + 5] = 0;
        } else {
            HIPCHK(c, (hipError_t)frame_serial(in, len, ws, cap, stream_offsets, msg_offsets, c->stream));
            HIPCHK(c, hipMemcpyAsync(c->h_stat + 2, ws.res, 48, hipMemcpyDeviceToHost, c->stream));
            HIPCHK(c, hipStreamSynchronize(c->stream));
        }
    }
    // h_stat[2 + k] = res[k]: [1] complete fragments, [3] consumed, [4] complete messages,
    // [5] fragments of the first cap messages
    const uint64_t M = c->h_stat[2 + 4];
    const uint64_t nout = M < cap ? M : cap;
    if (frags) *frags = nout ? c->h_stat[2 + 5] : 0;
    if (nout == 0) return XDRG_E_INCOMPLETE;   // NextAction STOP (RpcMessageParserTCP.java:51-53)
    *n_msgs = nout;
    if (consumed) *consumed = c->h_stat[2 + 3];
    if (uniform) *uniform = stride && !serial && c->h_stat[2 + 6] == 0 && c->h_stat[2 + 3] == nout * stride;
    if (payload) {
        const uint64_t nfc = c->h_stat[2 + 5];
        HIPCHK(c, hipMemcpyAsync(c->h_stat + 1, msg_offsets + nout, 8, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        const uint64_t bytes = c->h_stat[1];
        if (body_bytes) *body_bytes = bytes;
        if (bytes > payload_cap) {
            c->err = "payload buffer too small";
            if (consumed) *consumed = bytes;
            return XDRG_E_CAPACITY;
        }
        HIPCHK(c, (hipError_t)frame_copy(in, ws, nfc, bytes, payload, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    return XDRG_OK;
}

extern "C" int xdrg_frame_scan(xdrg_ctx *c, const uint8_t *in, uint64_t len, uint64_t *msg_offsets,
                               uint64_t cap, uint64_t *n_msgs) {
    return frame_walk(c, in, len, nullptr, 0, msg_offsets, cap, n_msgs, nullptr);
}

extern "C" int xdrg_deframe(xdrg_ctx *c, const uint8_t *in, uint64_t len, uint8_t *payload,
                            uint64_t payload_cap, uint64_t *msg_offsets, uint64_t cap, uint64_t *n_msgs,
                            uint64_t *consumed) {
    if (!payload && payload_cap) return XDRG_E_INVAL;
    uint8_t dummy = 0;
    return frame_walk(c, in, len, payload ? payload : &dummy, payload_cap, msg_offsets, cap, n_msgs, consumed);
}

// ---------------------------------------------------------------------------
// receive: host socket buffers (RpcMessageParserTCP.handleRead) and the
// decode of every complete message
// ---------------------------------------------------------------------------
static int recv_flags(xdrg_ctx *c, uint32_t flags) {
    if (flags & ~(XDRG_HOST_PTRS | XDRG_HOST_MAPPED)) return inval(c, "receive calls take XDRG_HOST_PTRS / XDRG_HOST_MAPPED only");
    if ((flags & XDRG_HOST_MAPPED) && !(flags & XDRG_HOST_PTRS)) return inval(c, "XDRG_HOST_MAPPED without XDRG_HOST_PTRS");
    return XDRG_OK;
}

// Device-resident receive (device pointers, or mapped views of registered
// host memory): one walk of the whole stream, then one decode of its
// messages — in place and record-marked when every message is one fragment
// (the common case: GrizzlyRpcTransport sends one, :103-110), else from the
// assembled bodies.  offs: device, cap + 1 entries.
static int recv_device(xdrg_ctx *c, const xdrg_schema *s, const uint8_t *in, uint64_t len, uint64_t cap,
                       xdrg_column *cols, uint64_t *offs, uint64_t *n_msgs, uint64_t *consumed, uint64_t *first_bad,
                       int *err) {
    *n_msgs = *consumed = 0;
    *first_bad = 0;
    *err = XDRG_OK;
    uint64_t nm = 0, used = 0, nf = 0;
    // fixed-size records: the walk's emit also checks the offsets against the
    // stride (single-fragment messages back to back decode by the stride
    // kernels with no separate pass over the offsets, tuning key 29)
    const uint64_t stride = !s->var_size && c->tune.stride_check ? s->fixed_size + 4 : 0;
    bool uniform = false;
    int rc = frame_walk(c, in, len, nullptr, 0, offs, cap, &nm, &used, &nf, nullptr, stride, &uniform);
    if (rc) return rc;   // XDRG_E_INCOMPLETE: STOP
    uint64_t fb = nm;
    int e = XDRG_OK;
    if (nf == nm && uniform && aligned(in, 4)) {
        rc = decode_impl(c, s, in, nm * stride, nullptr, nm, cols, XDRG_FRAME_RM, &fb, &e, 0, nullptr);
    } else if (nf == nm) {
        rc = decode_impl(c, s, in, len, offs, nm, cols, XDRG_FRAME_RM, &fb, &e, 0, nullptr);
    } else {   // multi-fragment messages: bodies assembled behind their offsets in the scratch
        const size_t ob = ((nm + 1) * 8 + 255) & ~(size_t)255;
        rc = ensure_rx(c, ob + used + 64);
        if (rc) return rc;
        uint64_t *boffs = (uint64_t *)c->d_rx;
        uint8_t *body = c->d_rx + ob;
        uint64_t nm2 = 0, used2 = 0, bytes = 0;
        rc = frame_walk(c, in, len, body, used, boffs, nm, &nm2, &used2, nullptr, &bytes);
        if (rc) return rc;
        rc = decode_impl(c, s, body, bytes, boffs, nm, cols, 0, &fb, &e, 0, nullptr);
    }
    if (rc && !e) return rc;   // an argument / HIP failure, not a decode error
    *n_msgs = nm;
    *consumed = used;
    *first_bad = fb;
    *err = e;
    if (e) {   // deliver through the bad message (CAPACITY: up to it)
        const uint64_t upto = e == XDRG_E_CAPACITY ? fb : fb + 1;
        DeviceGuard dg;
        HIPCHK(c, hipSetDevice(c->device));
        HIPCHK(c, hipMemcpyAsync(c->h_stat + 1, offs + upto, 8, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        *n_msgs = upto;
        *consumed = c->h_stat[1];
        c->err = xdrg_status_string(e);
        return e;
    }
    return XDRG_OK;
}

// Host memory through the staging ring (hs::stage_receive).
static int recv_staged(xdrg_ctx *c, int mode, const xdrg_schema *s, const uint8_t *in, uint64_t len, uint64_t cap,
                       xdrg_column *cols, uint8_t *payload, uint64_t payload_cap, uint64_t *msg_offsets,
                       hs::RecvResult &R) {
    hs::Schema v;
    if (s) stage_schema(s, v);
    int rc = ring_ready(c, c->ring.slot > c->ring.want_slot ? c->ring.slot : c->ring.want_slot);
    if (rc) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));   // the caller's earlier work on this context
    HipExec x(c, s);
    rc = hs::stage_receive(x, mode, s ? &v : nullptr, in, len, cap, cols, payload, payload_cap, msg_offsets, R,
                           c->tune.recv_budget / 10.0);
    const int fr = x.finish();
    if (rc && rc != XDRG_E_INCOMPLETE && rc != XDRG_E_HIP && c->err.empty()) c->err = xdrg_status_string(rc);
    return rc ? rc : fr;
}

// Schemas the receive windows do not carry (a T x[N] group inside a counted
// group's elements, group elements of no XDR bytes: hs::recv_groups_ok) on
// host memory: the staged walk (stream
// offsets of the complete messages), the staged deframe of those messages
// (their bodies into host scratch), then the staged decode of the bodies
// (xdrg_decode_batch with XDRG_HOST_PTRS).  The same results as the device
// receive; each stream byte crosses PCIe three times here.  Every other
// schema, nested repeated groups included, goes through hs::stage_receive's
// windows (one crossing).
static int recv_staged_groups(xdrg_ctx *c, const xdrg_schema *s, const uint8_t *in, uint64_t len, uint64_t cap,
                              xdrg_column *cols, uint64_t *msg_offsets, uint64_t *n_msgs, uint64_t *consumed,
                              uint64_t *first_bad, int *err) {
    c->recv_three_pass++;
    std::vector<uint64_t> so(cap + 1, 0);
    hs::RecvResult R;
    int rc = recv_staged(c, hs::RECV_SCAN, nullptr, in, len, cap, nullptr, nullptr, 0, so.data(), R);
    if (rc) return rc;   // XDRG_E_INCOMPLETE: STOP
    const uint64_t nm = R.n_msgs, used = R.consumed;
    std::vector<uint8_t> body(used + 16);
    std::vector<uint64_t> bo(nm + 1, 0);
    hs::RecvResult D;
    rc = recv_staged(c, hs::RECV_DEFRAME, nullptr, in, used, nm, nullptr, body.data(), used, bo.data(), D);
    if (rc) return rc;
    if (D.n_msgs != nm || D.consumed != used) {
        c->err = "receive: the deframe of the scanned messages disagrees with the scan";
        return XDRG_E_HIP;
    }
    uint64_t fb = nm;
    int e = XDRG_OK;
    rc = xdrg_decode_batch(c, s, body.data(), bo[nm], bo.data(), nm, cols, XDRG_HOST_PTRS, &fb, &e);
    if (rc && !e) return rc;   // an argument / HIP failure, not a decode error
    const uint64_t upto = !e ? nm : (e == XDRG_E_CAPACITY ? fb : fb + 1);   // (recv_device's delivery)
    if (msg_offsets) memcpy(msg_offsets, so.data(), (nm + 1) * 8);
    *n_msgs = upto;
    *consumed = so[upto];
    *first_bad = e ? fb : nm;
    *err = e;
    if (e) c->err = xdrg_status_string(e);
    return e;
}

extern "C" int xdrg_frame_scan_ex(xdrg_ctx *c, const uint8_t *in, uint64_t len, uint64_t *msg_offsets,
                                  uint64_t cap, uint64_t *n_msgs, uint64_t *consumed, uint32_t flags) {
    if (!c || !msg_offsets || !n_msgs) return XDRG_E_INVAL;
    int rc = recv_flags(c, flags);
    if (rc) return rc;
    uint64_t used = 0;
    *n_msgs = 0;
    if (consumed) *consumed = 0;
    if (len && !in) return inval(c, "stream is NULL");
    if (!(flags & XDRG_HOST_PTRS)) {
        rc = frame_walk(c, in, len, nullptr, 0, msg_offsets, cap, n_msgs, &used, nullptr, nullptr);
        if (consumed) *consumed = used;
        return rc;
    }
    DeviceGuard dg;
    HIPCHK(c, hipSetDevice(c->device));
    if (flags & XDRG_HOST_MAPPED) {
        const uint8_t *din = len ? (const uint8_t *)span_device(in, len) : in;
        uint64_t *doffs = (uint64_t *)span_device(msg_offsets, (cap + 1) * 8);
        if ((len && !din) || !doffs) return inval(c, "XDRG_HOST_MAPPED: stream / offsets not registered");
        rc = frame_walk(c, din, len, nullptr, 0, doffs, cap, n_msgs, &used, nullptr, nullptr);
        if (consumed) *consumed = used;
        return rc;
    }
    hs::RecvResult R;
    rc = recv_staged(c, hs::RECV_SCAN, nullptr, in, len, cap, nullptr, nullptr, 0, msg_offsets, R);
    *n_msgs = R.n_msgs;
    if (consumed) *consumed = R.consumed;
    return rc;
}

extern "C" int xdrg_deframe_ex(xdrg_ctx *c, const uint8_t *in, uint64_t len, uint8_t *payload, uint64_t payload_cap,
                               uint64_t *msg_offsets, uint64_t cap, uint64_t *n_msgs, uint64_t *consumed,
                               uint32_t flags) {
    if (!c || !msg_offsets || !n_msgs || (!payload && payload_cap)) return XDRG_E_INVAL;
    int rc = recv_flags(c, flags);
    if (rc) return rc;
    *n_msgs = 0;
    if (consumed) *consumed = 0;
    if (len && !in) return inval(c, "stream is NULL");
    if (!(flags & XDRG_HOST_PTRS)) return xdrg_deframe(c, in, len, payload, payload_cap, msg_offsets, cap, n_msgs, consumed);
    DeviceGuard dg;
    HIPCHK(c, hipSetDevice(c->device));
    if (flags & XDRG_HOST_MAPPED) {
        const uint8_t *din = len ? (const uint8_t *)span_device(in, len) : in;
        uint8_t *dpay = payload_cap ? (uint8_t *)span_device(payload, payload_cap) : nullptr;
        uint64_t *doffs = (uint64_t *)span_device(msg_offsets, (cap + 1) * 8);
        if ((len && !din) || (payload_cap && !dpay) || !doffs)
            return inval(c, "XDRG_HOST_MAPPED: stream / payload / offsets not registered");
        uint8_t dummy = 0;
        return frame_walk(c, din, len, dpay ? dpay : &dummy, payload_cap, doffs, cap, n_msgs, consumed, nullptr, nullptr);
    }
    hs::RecvResult R;
    rc = recv_staged(c, hs::RECV_DEFRAME, nullptr, in, len, cap, nullptr, payload, payload_cap, msg_offsets, R);
    *n_msgs = R.n_msgs;
    if (consumed) *consumed = R.consumed;
    return rc;
}

extern "C" int xdrg_receive_batch(xdrg_ctx *c, const xdrg_schema *s, const uint8_t *in, uint64_t len, uint64_t cap,
                                  xdrg_column *cols, uint32_t flags, uint64_t *msg_offsets, uint64_t *n_msgs,
                                  uint64_t *consumed, uint64_t *first_bad, int *err) {
    if (!c || !s || !n_msgs || !consumed) return XDRG_E_INVAL;
    int rc = recv_flags(c, flags);
    if (rc) return rc;
    *n_msgs = *consumed = 0;
    uint64_t fb_ = 0;
    int e_ = XDRG_OK;
    if (!first_bad) first_bad = &fb_;
    if (!err) err = &e_;
    *first_bad = 0;
    *err = XDRG_OK;
    if (len && !in) return inval(c, "stream is NULL");
    DeviceGuard dg;
    HIPCHK(c, hipSetDevice(c->device));
    rc = check_columns(c, s, cols, cap, true);
    if (rc) return rc;
    if ((flags & XDRG_HOST_PTRS) && !(flags & XDRG_HOST_MAPPED)) {
        hs::Schema v;
        stage_schema(s, v);
        if (!hs::recv_groups_ok(v) || (s->ngroups && !c->tune.recv_win))   // T x[N] under a counted group /
                                                                            // elements of no bytes: walk,
                                                                            // deframe, decode
            return recv_staged_groups(c, s, in, len, cap, cols, msg_offsets, n_msgs, consumed, first_bad, err);
        hs::RecvResult R;
        rc = recv_staged(c, hs::RECV_DECODE, s, in, len, cap, cols, nullptr, 0, msg_offsets, R);
        *n_msgs = R.n_msgs;
        *consumed = R.consumed;
        *first_bad = R.first_bad;
        *err = R.err;
        if (rc == XDRG_E_INVAL && c->err.empty()) c->err = "host columns: unsupported layout";
        return rc;
    }
    const uint8_t *din = in;
    xdrg_column *dcols = cols;
    std::vector<xdrg_column> mc;
    uint64_t *doffs = msg_offsets;
    if (flags & XDRG_HOST_MAPPED) {
        rc = mapped_cols(c, s, cols, cap, true, mc);
        if (rc) return rc;
        dcols = mc.data();
        din = len ? (const uint8_t *)span_device(in, len) : in;
        doffs = msg_offsets ? (uint64_t *)span_device(msg_offsets, (cap + 1) * 8) : nullptr;
        if ((len && !din) || (msg_offsets && !doffs)) return inval(c, "XDRG_HOST_MAPPED: stream / offsets not registered");
    }
    uint64_t *tmp = nullptr;   // no caller array: the offsets in stream-ordered scratch
    if (!doffs) {
        HIPCHK(c, hipMallocAsync((void **)&tmp, (cap + 1) * 8, c->stream));
        doffs = tmp;
    }
    rc = recv_device(c, s, din, len, cap, dcols, doffs, n_msgs, consumed, first_bad, err);
    if (tmp) (void)hipFreeAsync(tmp, c->stream);
    return rc;
}

// ---------------------------------------------------------------------------
// multi-GPU, one process
// ---------------------------------------------------------------------------
// Peer access from `dev` to `peer`, enabled once per pair.
static int enable_peer(xdrg_ctx *c, int dev, int peer) {
    if (dev == peer) return XDRG_OK;
    int can = 0;
    HIPCHK(c, hipDeviceCanAccessPeer(&can, dev, peer));
    if (!can) {
        c->err = "device pair has no peer access";
        return XDRG_E_HIP;
    }
    HIPCHK(c, hipSetDevice(dev));
    const hipError_t e = hipDeviceEnablePeerAccess(peer, 0);
    if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) return hip_fail(c, e, "hipDeviceEnablePeerAccess");
    (void)hipGetLastError();   // clear a sticky "already enabled"
    return XDRG_OK;
}

static int multi_args(xdrg_ctx *const *ctxs, uint32_t nctx, const xdrg_schema *s, const uint64_t *counts,
                      uint32_t flags) {
    if (!ctxs || !s || !counts || nctx == 0 || nctx > (uint32_t)kMaxGatherSeg / 2) return XDRG_E_INVAL;
    for (uint32_t i = 0; i < nctx; ++i)
        if (!ctxs[i]) return XDRG_E_INVAL;
    if (flags & ~XDRG_FRAME_RM)   // synchronous, device memory (xdrg_device_alloc / xdrg_copy for a JVM)
        return inval(ctxs[0], "multi-GPU calls take XDRG_FRAME_RM only (device memory, synchronous)");
    return XDRG_OK;
}

// XDR bytes of one shard: closed form for fixed-size schemas, else the size
// and scan passes on the context's stream (result in c->h_stat[2] after a sync).
static int shard_size_launch(xdrg_ctx *c, const xdrg_schema *s, const xdrg_column *cols, uint64_t n,
                             bool framed, uint64_t *size, bool *on_device) {
    *on_device = false;
    if (!s->var_size || n == 0) {
        *size = s->var_size ? 0 : n * (s->fixed_size + (framed ? 4 : 0));
        return XDRG_OK;
    }
    HIPCHK(c, hipSetDevice(c->device));
    if (s->ngroups) {   // repeated groups: the group size pass and its scan (group_encode's first two)
        GroupArgs g;
        int rc = fill_group(c, s, cols, n, framed, false, g);
        if (rc) return rc;
        g.enc_lanes = (uint32_t)c->tune.grp_enc_lanes;
        g.enc_split = (uint32_t)c->tune.grp_enc_split;
        HIPCHK(c, (hipError_t)launch_group_phase(g, GRP_ENC_SIZES, c->stream));
        HIPCHK(c, (hipError_t)launch_scan_rows(g.block_sums, g.nblocks, g.totals, 1, c->stream));
        HIPCHK(c, hipMemcpyAsync(c->h_stat + 2, g.totals, 8, hipMemcpyDeviceToHost, c->stream));
        *on_device = true;
        return XDRG_OK;
    }
    RecArgs a;
    int rc = fill_rec(c, s, (xdrg_column *)cols, n, framed, a);
    if (rc) return rc;
    for (int ph = REC_ENC_SIZES; ph <= REC_ENC_SCAN; ++ph) HIPCHK(c, (hipError_t)launch_rec_phase(a, ph, c->tune, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->h_stat + 2, a.totals, 8, hipMemcpyDeviceToHost, c->stream));
    *on_device = true;
    return XDRG_OK;
}

extern "C" int xdrg_encode_batch_multi(xdrg_ctx *const *ctxs, uint32_t nctx, const xdrg_schema *s,
                                       const xdrg_column *const *cols, const uint64_t *counts,
                                       uint8_t *const *out, uint64_t out_cap, uint64_t *const *rec_offsets,
                                       uint32_t flags, uint64_t *out_len) {
    int rc = multi_args(ctxs, nctx, s, counts, flags);
    if (rc) return rc;
    DeviceGuard dg;
    if (!cols || !out) return inval(ctxs[0], "columns / outputs are NULL");
    const bool framed = flags & XDRG_FRAME_RM;
    // 1. shard sizes (all devices in flight, then one sync each)
    std::vector<uint64_t> size(nctx), base(nctx + 1, 0), first(nctx + 1, 0);
    std::vector<char> dev(nctx);
    for (uint32_t i = 0; i < nctx; ++i) {
        rc = check_columns(ctxs[i], s, cols[i], counts[i], false);
        if (rc) return rc;
        bool d = false;
        rc = shard_size_launch(ctxs[i], s, cols[i], counts[i], framed, &size[i], &d);
        if (rc) return rc;
        dev[i] = d;
    }
    for (uint32_t i = 0; i < nctx; ++i) {
        if (dev[i]) {
            HIPCHK(ctxs[i], hipSetDevice(ctxs[i]->device));
            HIPCHK(ctxs[i], hipStreamSynchronize(ctxs[i]->stream));
            size[i] = ctxs[i]->h_stat[2];
        }
        base[i + 1] = base[i] + size[i];
        first[i + 1] = first[i] + counts[i];
    }
    const uint64_t total = base[nctx];
    if (out_len) *out_len = total;
    if (total > out_cap) {
        ctxs[0]->err = "output buffer too small";
        return XDRG_E_CAPACITY;
    }
    // 2. every context encodes its shard in place, at the shard's stream offset
    for (uint32_t i = 0; i < nctx; ++i) {
        xdrg_ctx *c = ctxs[i];
        uint64_t *ro = rec_offsets && rec_offsets[i] ? rec_offsets[i] + first[i] : nullptr;
        rc = xdrg_encode_batch(c, s, cols[i], counts[i], out[i] + base[i], out_cap - base[i], ro,
                               (framed ? XDRG_FRAME_RM : 0) | XDRG_ASYNC, nullptr);
        if (rc) return rc;
    }
    for (uint32_t i = 0; i < nctx; ++i) {
        HIPCHK(ctxs[i], hipSetDevice(ctxs[i]->device));
        HIPCHK(ctxs[i], hipStreamSynchronize(ctxs[i]->stream));
    }
    // Rebase the shard-relative record offsets.  Shards sharing one offsets
    // array both wrote entry first[i+1] (shard i its size, shard i+1 its 0),
    // so that entry is stored, never read-modified: shard i stores base[i] at
    // first[i] and base[i+1] at first[i+1] (the same value its neighbour
    // stores) and adds base[i] only to its interior entries, which no other
    // shard touches.  Every encode above has finished before these run.
    if (rec_offsets) {
        for (uint32_t i = 0; i < nctx; ++i) {
            if (!rec_offsets[i]) continue;
            xdrg_ctx *c = ctxs[i];
            uint64_t *ro = rec_offsets[i] + first[i];
            HIPCHK(c, hipSetDevice(c->device));
            HIPCHK(c, (hipError_t)launch_store_u64(ro, base[i], c->stream));
            HIPCHK(c, (hipError_t)launch_store_u64(ro + counts[i], base[i + 1], c->stream));
            if (counts[i] > 1) HIPCHK(c, (hipError_t)launch_add_u64(ro + 1, counts[i] - 1, base[i], c->stream));
        }
        for (uint32_t i = 0; i < nctx; ++i) {
            HIPCHK(ctxs[i], hipSetDevice(ctxs[i]->device));
            HIPCHK(ctxs[i], hipStreamSynchronize(ctxs[i]->stream));
        }
    }
    if (nctx == 1) return XDRG_OK;
    // 3. full-mesh all-gather: context i pulls every peer's shard (and offsets)
    for (uint32_t i = 0; i < nctx; ++i) {
        xdrg_ctx *c = ctxs[i];
        GatherArgs g;
        memset(&g, 0, sizeof g);
        for (uint32_t j = 0; j < nctx; ++j) {
            if (j == i) continue;
            if (out[j] != out[i] && size[j]) {
                rc = enable_peer(c, c->device, ctxs[j]->device);
                if (rc) return rc;
                g.src[g.nseg] = out[j] + base[j];
                g.dst[g.nseg] = out[i] + base[j];
                g.bytes[g.nseg++] = size[j];
            }
            if (rec_offsets && rec_offsets[i] && rec_offsets[j] && rec_offsets[j] != rec_offsets[i]) {
                rc = enable_peer(c, c->device, ctxs[j]->device);
                if (rc) return rc;
                g.src[g.nseg] = (const uint8_t *)(rec_offsets[j] + first[j]);
                g.dst[g.nseg] = (uint8_t *)(rec_offsets[i] + first[j]);
                g.bytes[g.nseg++] = (counts[j] + 1) * 8;
            }
        }
        HIPCHK(c, hipSetDevice(c->device));
        HIPCHK(c, (hipError_t)launch_gather(g, c->stream));
    }
    for (uint32_t i = 0; i < nctx; ++i) {
        HIPCHK(ctxs[i], hipSetDevice(ctxs[i]->device));
        HIPCHK(ctxs[i], hipStreamSynchronize(ctxs[i]->stream));
    }
    return XDRG_OK;
}

extern "C" int xdrg_decode_batch_multi(xdrg_ctx *const *ctxs, uint32_t nctx, const xdrg_schema *s,
                                       const uint8_t *const *in, uint64_t in_len,
                                       const uint64_t *const *rec_offsets, const uint64_t *counts,
                                       xdrg_column *const *cols, uint32_t flags, uint64_t *first_bad, int *err) {
    int rc = multi_args(ctxs, nctx, s, counts, flags);
    if (rc) return rc;
    DeviceGuard dg;
    if (!cols || !in) return inval(ctxs[0], "columns / inputs are NULL");
    const bool framed = flags & XDRG_FRAME_RM;
    const uint64_t stride = s->fixed_size + (framed ? 4 : 0);
    uint64_t first = 0, n_total = 0;
    for (uint32_t i = 0; i < nctx; ++i) n_total += counts[i];
    // every shard in flight; results land in each context's pinned status block
    for (uint32_t i = 0; i < nctx; ++i) {
        xdrg_ctx *c = ctxs[i];
        const uint64_t *ro = rec_offsets ? rec_offsets[i] : nullptr;
        const uint8_t *src = in[i];
        uint64_t len = in_len;
        if (ro) {
            ro += first;
        } else {   // fixed stride: the shard starts at record `first`
            const uint64_t skip = first * stride;
            src += skip < in_len ? skip : in_len;
            len = in_len > skip ? in_len - skip : 0;
        }
        rc = xdrg_decode_batch(c, s, src, len, ro, counts[i], cols[i],
                               (framed ? XDRG_FRAME_RM : 0) | XDRG_ASYNC,
                               (uint64_t *)(c->d_stat + 4), (int *)(c->d_stat + 5));
        if (rc) return rc;
        HIPCHK(c, hipMemcpyAsync(c->h_stat + 4, c->d_stat + 4, 16, hipMemcpyDeviceToHost, c->stream));
        first += counts[i];
    }
    uint64_t fb = n_total;
    int code = XDRG_OK;
    first = 0;
    for (uint32_t i = 0; i < nctx; ++i) {
        xdrg_ctx *c = ctxs[i];
        HIPCHK(c, hipSetDevice(c->device));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        const uint64_t f = c->h_stat[4];
        const int e = (int)(uint32_t)c->h_stat[5];
        if (e != XDRG_OK && first + f < fb) {   // the sequential reference stops at the smallest
            fb = first + f;
            code = e;
        }
        first += counts[i];
    }
    if (first_bad) *first_bad = fb;
    if (err) *err = code;
    if (code) ctxs[0]->err = xdrg_status_string(code);
    return code;
}
