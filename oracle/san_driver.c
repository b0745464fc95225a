/*
 * san_driver.c — TEST INFRASTRUCTURE: drives the oracle (xdr_oracle.c) under
 * AddressSanitizer + UndefinedBehaviorSanitizer (oracle/Makefile `sanitize`,
 * run by tests/test_sanitize.py).  Every stream codec, the batch drivers
 * (plain, conditional, shallow, view, multithreaded) and the record-mark
 * walk run over seeded random schemas and records, then over truncated and
 * corrupted streams: the checker itself must never read or write out of
 * bounds, whatever bytes it is handed.  Exit 0 = every round trip matched.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "xdr_oracle.h"

static uint64_t rng_state = 0x0DCAC4E5u;
static uint64_t rnd(void) {   /* splitmix64 */
    uint64_t z = (rng_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static uint32_t rnd_below(uint32_t n) { return n ? (uint32_t)(rnd() % n) : 0; }

#define CHECK(c)                                                          \
    do {                                                                  \
        if (!(c)) {                                                       \
            fprintf(stderr, "%s:%d: check failed: %s\n", __FILE__, __LINE__, #c); \
            exit(1);                                                      \
        }                                                                 \
    } while (0)

static uint32_t nsize(uint32_t t) {
    switch (t) {
    case XDRG_T_HYPER: case XDRG_T_UHYPER: case XDRG_T_DOUBLE: return 8;
    case XDRG_T_SHORT: return 2;
    case XDRG_T_BYTE: case XDRG_T_BOOL: case XDRG_T_OPAQUE: case XDRG_T_STRING: return 1;
    default: return 4;
    }
}
static uint32_t xsize(uint32_t t) {
    switch (t) {
    case XDRG_T_HYPER: case XDRG_T_UHYPER: case XDRG_T_DOUBLE: return 8;
    case XDRG_T_OPAQUE: case XDRG_T_STRING: return 1;
    default: return 4;
    }
}

/* the known answers of the reference's own tests (tests/golden/kat_reference.json) */
static void stream_kats(void) {
    xo_stream s;
    CHECK(xo_stream_alloc(&s, 4) == XDRG_OK);   /* grows (Xdr.java:1020-1026) */
    xo_begin_encoding(&s);
    CHECK(xo_encode_int(&s, 17) == XDRG_OK);
    CHECK(xo_encode_long(&s, 297519060383110161ll) == XDRG_OK);
    const uint8_t op[8] = {0x0C, 0x0A, 0x0F, 0x0E, 0x0B, 0x0A, 0x0B, 0x0E};
    CHECK(xo_encode_dynamic_opaque(&s, op, 8) == XDRG_OK);
    xo_end_encoding(&s);
    const uint8_t want[] = {0, 0, 0, 0x11, 0x04, 0x21, 0x00, 0x02, 0x54, 0x0b, 0x14, 0x11,
                            0, 0, 0, 8, 0x0C, 0x0A, 0x0F, 0x0E, 0x0B, 0x0A, 0x0B, 0x0E};
    CHECK(s.limit == sizeof want && memcmp(s.buf, want, sizeof want) == 0);
    xo_begin_decoding(&s);
    int32_t i; int64_t l; const uint8_t *p; size_t n;
    CHECK(xo_decode_int(&s, &i) == XDRG_OK && i == 17);
    CHECK(xo_decode_long(&s, &l) == XDRG_OK && l == 297519060383110161ll);
    CHECK(xo_decode_dynamic_opaque(&s, &p, &n) == XDRG_OK && n == 8 && memcmp(p, op, 8) == 0);
    CHECK(!xo_has_more_data(&s));
    CHECK(xo_decode_int(&s, &i) == XDRG_E_SHORT);   /* past the end */
    xo_stream_free(&s);
    /* int then long: too short; count -2: corrupted */
    uint8_t b4[4] = {0, 0, 0, 1};
    xo_stream w;
    xo_stream_wrap(&w, b4, 4);
    xo_begin_decoding(&w);
    CHECK(xo_decode_long(&w, &l) == XDRG_E_SHORT);
    uint8_t neg[8] = {0xff, 0xff, 0xff, 0xfe, 0, 0, 0, 0};
    xo_stream_wrap(&w, neg, 8);
    xo_begin_decoding(&w);
    int32_t iv[4];
    CHECK(xo_decode_int_vector(&w, iv, 4, &n) == XDRG_E_CORRUPT);
    int32_t fv[3] = {1, 2, 3};
    CHECK(xo_stream_alloc(&s, 16) == XDRG_OK);
    xo_begin_encoding(&s);
    CHECK(xo_encode_int_fixed_vector(&s, fv, 3, 4) == XDRG_E_FIXED_LEN);
    xo_stream_free(&s);
}

/* ---- random batches ---------------------------------------------------------- */
typedef struct {
    xdrg_field f[12];
    size_t nf;
    xdrg_column col[12];
    void *mem[12];
    uint64_t *offs[12];
} batch;

static const uint32_t kTypes[] = {XDRG_T_INT, XDRG_T_UINT, XDRG_T_ENUM, XDRG_T_BOOL, XDRG_T_HYPER,
                                  XDRG_T_UHYPER, XDRG_T_FLOAT, XDRG_T_DOUBLE, XDRG_T_SHORT,
                                  XDRG_T_BYTE, XDRG_T_OPAQUE, XDRG_T_STRING};

static void random_schema(batch *b) {
    memset(b, 0, sizeof *b);
    b->nf = 1 + rnd_below(10);
    for (size_t k = 0; k < b->nf; ++k) {
        const uint32_t t = kTypes[rnd_below(12)];
        uint32_t kind = rnd_below(3);
        if (t == XDRG_T_BOOL) kind = XDRG_K_SCALAR;
        if (t == XDRG_T_STRING) kind = XDRG_K_DYNAMIC;
        if (t == XDRG_T_OPAQUE && kind == XDRG_K_SCALAR) kind = XDRG_K_FIXED;
        b->f[k].type = t;
        b->f[k].kind = kind;
        b->f[k].count = kind == XDRG_K_FIXED ? rnd_below(7) : 0;
    }
}

/* n records of random values; dynamic counts in [0, maxlen] */
static void fill(batch *b, uint64_t n, uint32_t maxlen) {
    for (size_t k = 0; k < b->nf; ++k) {
        const xdrg_field *f = &b->f[k];
        const uint32_t es = nsize(f->type);
        uint64_t elems;
        if (f->kind == XDRG_K_DYNAMIC) {
            b->offs[k] = calloc(n + 1, 8);
            for (uint64_t i = 0; i < n; ++i) b->offs[k][i + 1] = b->offs[k][i] + rnd_below(maxlen + 1);
            elems = b->offs[k][n];
            b->col[k].offsets = b->offs[k];
            b->col[k].cap = elems;
        } else {
            elems = n * (f->kind == XDRG_K_FIXED ? f->count : 1);
        }
        uint8_t *m = malloc(elems * es + 1);
        for (uint64_t i = 0; i < elems * es; ++i) m[i] = (uint8_t)rnd();
        if (f->type == XDRG_T_BOOL)
            for (uint64_t i = 0; i < elems; ++i) m[i] &= 1;
        b->mem[k] = m;
        b->col[k].data = m;
    }
}

/* empty output columns shaped like `in` (dynamic capacity = in's counts) */
static void shape_like(batch *o, const batch *in, uint64_t n) {
    memset(o, 0, sizeof *o);
    o->nf = in->nf;
    memcpy(o->f, in->f, sizeof in->f);
    for (size_t k = 0; k < in->nf; ++k) {
        const xdrg_field *f = &in->f[k];
        const uint32_t es = nsize(f->type);
        uint64_t elems;
        if (f->kind == XDRG_K_DYNAMIC) {
            elems = in->offs[k][n];
            o->offs[k] = calloc(n + 1, 8);
            o->col[k].offsets = o->offs[k];
            o->col[k].cap = elems;
        } else {
            elems = n * (f->kind == XDRG_K_FIXED ? f->count : 1);
        }
        o->mem[k] = calloc(elems * es + 1, 1);
        o->col[k].data = o->mem[k];
    }
}

static void release(batch *b) {
    for (size_t k = 0; k < b->nf; ++k) {
        free(b->mem[k]);
        free(b->offs[k]);
    }
}

static uint64_t xdr_total(const batch *b, uint64_t n, int framed) {
    uint64_t t = framed ? 4 * n : 0;
    for (size_t k = 0; k < b->nf; ++k) {
        const xdrg_field *f = &b->f[k];
        const uint32_t xs = xsize(f->type);
        if (f->kind == XDRG_K_DYNAMIC) {
            const uint64_t e = b->offs[k][n];
            t += 4 * n + (xs == 1 ? 0 : xs * e);
            if (xs == 1)
                for (uint64_t i = 0; i < n; ++i) {
                    const uint64_t c = b->offs[k][i + 1] - b->offs[k][i];
                    t += c + ((4 - (c & 3)) & 3);
                }
        } else {
            const uint64_t c = f->kind == XDRG_K_FIXED ? f->count : 1;
            t += n * (xs == 1 ? c + ((4 - (c & 3)) & 3) : xs * c);
        }
    }
    return t;
}

static void batch_round(int framed) {
    batch in, out;
    random_schema(&in);
    const uint64_t n = rnd_below(300);
    fill(&in, n, rnd_below(2) ? 9 : 70);
    const uint64_t total = xdr_total(&in, n, framed);
    uint8_t *xdr = malloc(total + 1);
    uint64_t *ro = calloc(n + 1, 8), len = 0;
    const uint32_t fl = framed ? XDRG_FRAME_RM : 0;
    CHECK(xo_encode_batch(in.f, in.nf, in.col, n, xdr, total, ro, fl, &len) == XDRG_OK);
    CHECK(len == total && ro[n] == total);
    /* too small an output: capacity, no overrun */
    if (total >= 4) CHECK(xo_encode_batch(in.f, in.nf, in.col, n, xdr, total - 4, ro, fl, &len) != XDRG_OK);
    CHECK(xo_encode_batch(in.f, in.nf, in.col, n, xdr, total, ro, fl, &len) == XDRG_OK);
    shape_like(&out, &in, n);
    uint64_t fb = 0;
    int err = 0;
    CHECK(xo_decode_batch(in.f, in.nf, xdr, total, ro, n, out.col, fl, &fb, &err) == XDRG_OK && fb == n);
    for (size_t k = 0; k < in.nf; ++k) {   /* values back (bool: any non-zero -> 1; floats by bits) */
        const xdrg_field *f = &in.f[k];
        const uint64_t elems = f->kind == XDRG_K_DYNAMIC ? in.offs[k][n]
                                                         : n * (f->kind == XDRG_K_FIXED ? f->count : 1);
        if (f->type == XDRG_T_FLOAT || f->type == XDRG_T_DOUBLE) continue;   /* NaNs canonicalised */
        CHECK(memcmp(in.mem[k], out.mem[k], elems * nsize(f->type)) == 0);
        if (f->kind == XDRG_K_DYNAMIC) CHECK(memcmp(in.offs[k], out.offs[k], 8 * (n + 1)) == 0);
    }
    /* every truncation and a few corruptions: any status, never a stray access */
    for (int r = 0; r < 24 && total; ++r) {
        const uint64_t cut = rnd_below((uint32_t)total);
        uint8_t *t = malloc(cut + 1);
        memcpy(t, xdr, cut);
        (void)xo_decode_batch(in.f, in.nf, t, cut, ro, n, out.col, fl, &fb, &err);
        (void)xo_decode_batch(in.f, in.nf, t, cut, NULL, n, out.col, fl, &fb, &err);
        free(t);
        uint8_t *c = malloc(total);
        memcpy(c, xdr, total);
        for (int j = 0; j < 4; ++j) c[rnd_below((uint32_t)total)] = (uint8_t)rnd();
        (void)xo_decode_batch(in.f, in.nf, c, total, ro, n, out.col, fl, &fb, &err);
        free(c);
    }
    /* the record-mark walk over the framed stream, then re-fragmented */
    if (framed && total) {
        uint64_t *mo = calloc(n + 2, 8), nm = 0;
        CHECK(xo_frame_scan(xdr, total, mo, n + 1, &nm) == XDRG_OK && nm == n);
        const size_t fcap = total + 4 * (total / 8 + 2);
        uint8_t *fr = malloc(fcap), *pay = malloc(total + 1);
        const size_t w = xo_fragment(xdr, total, 8 + rnd_below(64), fr, fcap);
        size_t plen = 0, used = 0;
        CHECK(xo_all_fragments_arrived(fr, w));
        CHECK(xo_assemble(fr, w, pay, total, &plen, &used) == XDRG_OK && plen == total && used == w);
        CHECK(memcmp(pay, xdr, total) == 0);
        for (int r = 0; r < 16; ++r) {
            const size_t cut = rnd_below((uint32_t)w);
            (void)xo_all_fragments_arrived(fr, cut);
            (void)xo_frame_scan(fr, cut, mo, n + 1, &nm);
        }
        free(mo);
        free(fr);
        free(pay);
    }
    free(xdr);
    free(ro);
    release(&in);
    release(&out);
}

static void mt_round(void) {
    batch in, out;
    memset(&in, 0, sizeof in);
    in.nf = 8;
    for (int k = 0; k < 8; ++k) in.f[k].type = XDRG_T_INT;
    const uint64_t n = 1000 + rnd_below(5000);
    fill(&in, n, 0);
    const uint64_t total = 32 * n;
    uint8_t *xdr = malloc(total);
    uint64_t len = 0, fb = 0;
    int err = 0;
    CHECK(xo_encode_batch_mt(in.f, 8, in.col, n, xdr, total, 0, &len, 4) == XDRG_OK && len == total);
    shape_like(&out, &in, n);
    CHECK(xo_decode_batch_mt(in.f, 8, xdr, total, n, out.col, 0, &fb, &err, 4) == XDRG_OK && fb == n);
    for (int k = 0; k < 8; ++k) CHECK(memcmp(in.mem[k], out.mem[k], 4 * n) == 0);
    CHECK(xo_decode_batch_mt(in.f, 8, xdr, total - 7, n, out.col, 0, &fb, &err, 4) == XDRG_E_SHORT);
    free(xdr);
    release(&in);
    release(&out);
}

int main(int argc, char **argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 300;
    stream_kats();
    for (int r = 0; r < rounds; ++r) batch_round(r & 1);
    for (int r = 0; r < 4; ++r) mt_round();
    printf("san_driver: %d batch rounds ok\n", rounds);
    return 0;
}
