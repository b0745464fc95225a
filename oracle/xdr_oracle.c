/*
 * xdr_oracle.c — TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline).
 *
 * Plain-C restatement of org.dcache.oncrpc4j.xdr.Xdr and of the RFC 1831
 * record-mark framing of oncrpc4j.  Each function cites the reference lines
 * it follows; paths are relative to
 * /root/reference/oncrpc4j-core/src/main/java/org/dcache/oncrpc4j/.
 * Never linked into the product library.
 */
#include "xdr_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ---- big-endian helpers (util/Bytes.java:39-107) ------------------------ */
static inline void put_be32(uint8_t *p, uint32_t v) {
    p[0] = (uint8_t)(v >> 24); p[1] = (uint8_t)(v >> 16);
    p[2] = (uint8_t)(v >> 8);  p[3] = (uint8_t)v;
}
static inline uint32_t get_be32(const uint8_t *p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
static inline void put_be64(uint8_t *p, uint64_t v) {   /* Bytes.putLong :39-54 */
    put_be32(p, (uint32_t)(v >> 32)); put_be32(p + 4, (uint32_t)v);
}
static inline uint64_t get_be64(const uint8_t *p) {     /* Bytes.getLong :84-93 */
    return ((uint64_t)get_be32(p) << 32) | get_be32(p + 4);
}

/* ---- stream state (Xdr.java:82-154) ------------------------------------ */
int xo_stream_alloc(xo_stream *s, size_t size) {
    s->buf = (uint8_t *)calloc(size ? size : 1, 1);   /* fresh heap buffer: zeroed */
    if (!s->buf) return XDRG_E_NOMEM;
    s->cap = size; s->pos = 0; s->limit = size; s->in_use = 0; s->growable = 1;
    return XDRG_OK;
}
void xo_stream_wrap(xo_stream *s, uint8_t *buf, size_t len) {
    s->buf = buf; s->cap = len; s->pos = 0; s->limit = len; s->in_use = 0; s->growable = 0;
}
void xo_stream_free(xo_stream *s) {
    if (s->growable) free(s->buf);
    s->buf = NULL; s->cap = s->pos = s->limit = 0;
}
void xo_begin_encoding(xo_stream *s) { s->pos = 0; s->limit = s->cap; s->in_use = 1; } /* clear() :138 */
void xo_end_encoding(xo_stream *s)   { s->limit = s->pos; s->pos = 0; s->in_use = 0; } /* flip()  :144 */
void xo_begin_decoding(xo_stream *s) { s->pos = 0; s->in_use = 1; }                    /* rewind():126 */
void xo_end_decoding(xo_stream *s)   { s->pos = 0; s->in_use = 0; }                    /* rewind():132 */
size_t xo_remaining(const xo_stream *s) { return s->limit - s->pos; }
int xo_has_more_data(const xo_stream *s) { return s->pos < s->limit; }                /* :152-154 */

/* ensureCapacity (Xdr.java:1020-1026): grow to max(cap*3/2+1, cap+size). */
static int ensure_capacity(xo_stream *s, size_t size) {
    if (xo_remaining(s) >= size) return XDRG_OK;
    if (!s->growable) return XDRG_E_CAPACITY;
    size_t old = s->cap;
    size_t ncap = old * 3 / 2 + 1;
    if (ncap < old + size) ncap = old + size;
    uint8_t *nb = (uint8_t *)realloc(s->buf, ncap);
    if (!nb) return XDRG_E_NOMEM;
    memset(nb + old, 0, ncap - old);
    s->buf = nb; s->cap = ncap; s->limit = ncap;
    return XDRG_OK;
}
/* ensureBytes (Xdr.java:1028-1032) */
static inline int ensure_bytes(const xo_stream *s, size_t size) {
    return xo_remaining(s) < size ? XDRG_E_SHORT : XDRG_OK;
}
/* checkArraySize (Xdr.java:1034-1038) */
static inline int check_array_size(int32_t len) { return len < 0 ? XDRG_E_CORRUPT : XDRG_OK; }

static inline uint32_t pad4(size_t len) { return (uint32_t)((4 - (len & 3)) & 3); } /* :777 */

/* ---- encoders ------------------------------------------------------------ */
int xo_encode_int(xo_stream *s, int32_t v) {                 /* Xdr.java:545-548 */
    int rc = ensure_capacity(s, 4); if (rc) return rc;
    put_be32(s->buf + s->pos, (uint32_t)v); s->pos += 4;
    return XDRG_OK;
}
int xo_encode_long(xo_stream *s, int64_t v) {                /* Xdr.java:812-815 */
    int rc = ensure_capacity(s, 8); if (rc) return rc;
    put_be64(s->buf + s->pos, (uint64_t)v); s->pos += 8;
    return XDRG_OK;
}
/* Float.floatToIntBits: every NaN collapses to 0x7fc00000 (Xdr.java:674-676). */
static inline uint32_t float_to_int_bits(float f) {
    uint32_t u; memcpy(&u, &f, 4);
    if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x007fffffu)) return 0x7fc00000u;
    return u;
}
/* Double.doubleToLongBits: every NaN collapses to 0x7ff8000000000000 (:685-687). */
static inline uint64_t double_to_long_bits(double d) {
    uint64_t u; memcpy(&u, &d, 8);
    if ((u & 0x7ff0000000000000ull) == 0x7ff0000000000000ull && (u & 0x000fffffffffffffull))
        return 0x7ff8000000000000ull;
    return u;
}
int xo_encode_float(xo_stream *s, float v)   { return xo_encode_int(s, (int32_t)float_to_int_bits(v)); }
int xo_encode_double(xo_stream *s, double v) { return xo_encode_long(s, (int64_t)double_to_long_bits(v)); }
int xo_encode_boolean(xo_stream *s, int v)   { return xo_encode_int(s, v ? 1 : 0); }       /* :803-805 */
int xo_encode_byte(xo_stream *s, int8_t v)   { return xo_encode_int(s, (int32_t)v); }      /* :919-925 */
int xo_encode_short(xo_stream *s, int16_t v) { return xo_encode_int(s, (int32_t)v); }      /* :934-936 */

/* xdrEncodeOpaque(bytes, offset, len) (Xdr.java:776-781): bytes then zero pad. */
int xo_encode_opaque(xo_stream *s, const uint8_t *b, size_t off, size_t len) {
    uint32_t pad = pad4(len);
    int rc = ensure_capacity(s, len + pad); if (rc) return rc;
    if (len) memcpy(s->buf + s->pos, b + off, len);
    s->pos += len;
    memset(s->buf + s->pos, 0, pad);                 /* paddingZeros :765 */
    s->pos += pad;
    return XDRG_OK;
}
int xo_encode_dynamic_opaque(xo_stream *s, const uint8_t *b, size_t len) { /* :797-800 */
    int rc = xo_encode_int(s, (int32_t)len); if (rc) return rc;
    return xo_encode_opaque(s, b, 0, len);
}
int xo_encode_string(xo_stream *s, const uint8_t *utf8, size_t len) {    /* :760-763 */
    if (!utf8) len = 0;                              /* null -> "" */
    return xo_encode_dynamic_opaque(s, utf8, len);
}
/* xdrEncodeByteBuffer (Xdr.java:824-831): the pad is a position skip, not a
 * write; a fresh (zeroed) buffer therefore carries zero pad bytes.            */
int xo_encode_byte_buffer(xo_stream *s, const uint8_t *b, size_t len) {
    uint32_t pad = pad4(len);
    int rc = xo_encode_int(s, (int32_t)len); if (rc) return rc;
    rc = ensure_capacity(s, len + pad); if (rc) return rc;
    if (len) memcpy(s->buf + s->pos, b, len);
    s->pos += len + pad;
    return XDRG_OK;
}
/* xdrEncodeFileChunk (Xdr.java:978-988): the length word only; the chunk and
 * its zero padding stay outside the buffer and travel as their own writable
 * messages (asBufferWritableMessages :579-597).                              */
int xo_encode_file_chunk(xo_stream *s, size_t len, uint32_t *padding) {
    int rc = xo_encode_int(s, (int32_t)len); if (rc) return rc;
    *padding = pad4(len);
    return XDRG_OK;
}
/* xdrEncodeIntVector (Xdr.java:607-613): one capacity check, count + ints. */
int xo_encode_int_vector(xo_stream *s, const int32_t *v, size_t n) {
    int rc = ensure_capacity(s, 4 + 4 * n); if (rc) return rc;
    put_be32(s->buf + s->pos, (uint32_t)n); s->pos += 4;
    for (size_t i = 0; i < n; i++) { put_be32(s->buf + s->pos, (uint32_t)v[i]); s->pos += 4; }
    return XDRG_OK;
}
/* Fixed-vector encoders reject value.length != length (Xdr.java:624-631 etc.). */
#define FIXED_CHECK(n, length) if ((size_t)(length) != (n) || (length) < 0) return XDRG_E_FIXED_LEN
int xo_encode_int_fixed_vector(xo_stream *s, const int32_t *v, size_t n, int32_t length) {
    FIXED_CHECK(n, length);
    for (size_t i = 0; i < n; i++) { int rc = xo_encode_int(s, v[i]); if (rc) return rc; }
    return XDRG_OK;
}
int xo_encode_long_vector(xo_stream *s, const int64_t *v, size_t n) {    /* :641-647 */
    int rc = ensure_capacity(s, 4 + 8 * n); if (rc) return rc;
    put_be32(s->buf + s->pos, (uint32_t)n); s->pos += 4;
    for (size_t i = 0; i < n; i++) { put_be64(s->buf + s->pos, (uint64_t)v[i]); s->pos += 8; }
    return XDRG_OK;
}
int xo_encode_long_fixed_vector(xo_stream *s, const int64_t *v, size_t n, int32_t length) {
    FIXED_CHECK(n, length);                                             /* :658-665 */
    for (size_t i = 0; i < n; i++) { int rc = xo_encode_long(s, v[i]); if (rc) return rc; }
    return XDRG_OK;
}
int xo_encode_float_vector(xo_stream *s, const float *v, size_t n) {     /* :696-702 */
    int rc = xo_encode_int(s, (int32_t)n); if (rc) return rc;
    for (size_t i = 0; i < n; i++) { rc = xo_encode_float(s, v[i]); if (rc) return rc; }
    return XDRG_OK;
}
int xo_encode_float_fixed_vector(xo_stream *s, const float *v, size_t n, int32_t length) {
    FIXED_CHECK(n, length);                                             /* :713-720 */
    for (size_t i = 0; i < n; i++) { int rc = xo_encode_float(s, v[i]); if (rc) return rc; }
    return XDRG_OK;
}
int xo_encode_double_vector(xo_stream *s, const double *v, size_t n) {   /* :729-735 */
    int rc = xo_encode_int(s, (int32_t)n); if (rc) return rc;
    for (size_t i = 0; i < n; i++) { rc = xo_encode_double(s, v[i]); if (rc) return rc; }
    return XDRG_OK;
}
int xo_encode_double_fixed_vector(xo_stream *s, const double *v, size_t n, int32_t length) {
    FIXED_CHECK(n, length);                                             /* :746-753 */
    for (size_t i = 0; i < n; i++) { int rc = xo_encode_double(s, v[i]); if (rc) return rc; }
    return XDRG_OK;
}
int xo_encode_short_vector(xo_stream *s, const int16_t *v, size_t n) {   /* :945-951 */
    int rc = xo_encode_int(s, (int32_t)n); if (rc) return rc;
    for (size_t i = 0; i < n; i++) { rc = xo_encode_short(s, v[i]); if (rc) return rc; }
    return XDRG_OK;
}
int xo_encode_short_fixed_vector(xo_stream *s, const int16_t *v, size_t n, int32_t length) {
    FIXED_CHECK(n, length);                                             /* :962-969 */
    for (size_t i = 0; i < n; i++) { int rc = xo_encode_short(s, v[i]); if (rc) return rc; }
    return XDRG_OK;
}
int xo_encode_byte_vector(xo_stream *s, const int8_t *v, size_t n) {     /* :878-888 */
    int rc = xo_encode_int(s, (int32_t)n); if (rc) return rc;
    for (size_t i = 0; i < n; i++) { rc = xo_encode_byte(s, v[i]); if (rc) return rc; }
    return XDRG_OK;
}
int xo_encode_byte_fixed_vector(xo_stream *s, const int8_t *v, size_t n, int32_t length) {
    FIXED_CHECK(n, length);                                             /* :900-911 */
    for (size_t i = 0; i < n; i++) { int rc = xo_encode_int(s, (int32_t)v[i]); if (rc) return rc; }
    return XDRG_OK;
}

/* ---- decoders ------------------------------------------------------------ */
int xo_decode_int(xo_stream *s, int32_t *v) {                 /* Xdr.java:171-175 */
    int rc = ensure_bytes(s, 4); if (rc) return rc;
    *v = (int32_t)get_be32(s->buf + s->pos); s->pos += 4;
    return XDRG_OK;
}
int xo_decode_long(xo_stream *s, int64_t *v) {                /* Xdr.java:417-420 */
    int rc = ensure_bytes(s, 8); if (rc) return rc;
    *v = (int64_t)get_be64(s->buf + s->pos); s->pos += 8;
    return XDRG_OK;
}
int xo_decode_float(xo_stream *s, float *v) {                 /* :255-257 intBitsToFloat */
    int32_t i; int rc = xo_decode_int(s, &i); if (rc) return rc;
    memcpy(v, &i, 4); return XDRG_OK;
}
int xo_decode_double(xo_stream *s, double *v) {               /* :267-269 longBitsToDouble */
    int64_t l; int rc = xo_decode_long(s, &l); if (rc) return rc;
    memcpy(v, &l, 8); return XDRG_OK;
}
int xo_decode_boolean(xo_stream *s, int *v) {                 /* :404-407 any non-zero */
    int32_t i; int rc = xo_decode_int(s, &i); if (rc) return rc;
    *v = i != 0; return XDRG_OK;
}
int xo_decode_byte(xo_stream *s, int8_t *v) {                 /* :485-487 (byte) */
    int32_t i; int rc = xo_decode_int(s, &i); if (rc) return rc;
    *v = (int8_t)i; return XDRG_OK;
}
int xo_decode_short(xo_stream *s, int16_t *v) {               /* :497-499 (short) */
    int32_t i; int rc = xo_decode_int(s, &i); if (rc) return rc;
    *v = (int16_t)i; return XDRG_OK;
}
/* xdrDecodeOpaque(buf, off, len) (Xdr.java:341-349): len 0 returns at once;
 * the pad is skipped without being checked.                                  */
int xo_decode_opaque(xo_stream *s, uint8_t *dst, size_t len) {
    if (len == 0) return XDRG_OK;
    uint32_t pad = pad4(len);
    int rc = ensure_bytes(s, len + pad); if (rc) return rc;
    if (dst) memcpy(dst, s->buf + s->pos, len);
    s->pos += len + pad;
    return XDRG_OK;
}
/* xdrDecodeDynamicOpaque (Xdr.java:374-383) and xdrDecodeString (:392-401):
 * length; 0 -> empty before any sign check; negative -> corrupted; bytes.    */
static int decode_counted_bytes(xo_stream *s, const uint8_t **p, size_t *len) {
    int32_t l; int rc = xo_decode_int(s, &l); if (rc) return rc;
    *p = s->buf + s->pos; *len = 0;
    if (l == 0) return XDRG_OK;
    rc = check_array_size(l); if (rc) return rc;
    *p = s->buf + s->pos;
    rc = xo_decode_opaque(s, NULL, (size_t)l); if (rc) return rc;
    *len = (size_t)l;
    return XDRG_OK;
}
int xo_decode_dynamic_opaque(xo_stream *s, const uint8_t **p, size_t *len) { return decode_counted_bytes(s, p, len); }
int xo_decode_string(xo_stream *s, const uint8_t **p, size_t *len)         { return decode_counted_bytes(s, p, len); }
/* xdrDecodeByteBuffer (Xdr.java:423-439): sign check first (0 passes), then
 * ensureBytes(len + pad); returns a view.                                     */
int xo_decode_byte_buffer(xo_stream *s, const uint8_t **p, size_t *len) {
    int32_t l; int rc = xo_decode_int(s, &l); if (rc) return rc;
    rc = check_array_size(l); if (rc) return rc;
    uint32_t pad = pad4((size_t)l);
    rc = ensure_bytes(s, (size_t)l + pad); if (rc) return rc;
    *p = s->buf + s->pos; *len = (size_t)l;
    s->pos += (size_t)l + pad;
    return XDRG_OK;
}
/* Dynamic vectors (Xdr.java:184-193, 219-228, 278-282, 308-312, 452-456,
 * 509-513): count; negative -> corrupted; then element by element, each
 * running ensureBytes.  The reference allocates `new T[count]` before the
 * first element check; for an absurd count that is an OutOfMemoryError in
 * the JVM where this restatement (and the engine) report "too short".      */
#define DECODE_VECTOR(NAME, T, XSZ, GET)                                        \
int NAME(xo_stream *s, T *out, size_t cap, size_t *n) {                          \
    int32_t l; int rc = xo_decode_int(s, &l); if (rc) return rc;                 \
    rc = check_array_size(l); if (rc) return rc;                                 \
    *n = 0;                                                                       \
    if (xo_remaining(s) < (size_t)l * (XSZ)) return XDRG_E_SHORT;                \
    if ((size_t)l > cap) return XDRG_E_CAPACITY;                                 \
    for (int32_t i = 0; i < l; i++) { GET; s->pos += (XSZ); }                    \
    *n = (size_t)l;                                                               \
    return XDRG_OK;                                                              \
}
DECODE_VECTOR(xo_decode_int_vector, int32_t, 4, out[i] = (int32_t)get_be32(s->buf + s->pos))
DECODE_VECTOR(xo_decode_long_vector, int64_t, 8, out[i] = (int64_t)get_be64(s->buf + s->pos))
DECODE_VECTOR(xo_decode_float_vector, float, 4,
              { uint32_t u = get_be32(s->buf + s->pos); memcpy(&out[i], &u, 4); })
DECODE_VECTOR(xo_decode_double_vector, double, 8,
              { uint64_t u = get_be64(s->buf + s->pos); memcpy(&out[i], &u, 8); })
DECODE_VECTOR(xo_decode_short_vector, int16_t, 4, out[i] = (int16_t)get_be32(s->buf + s->pos))
DECODE_VECTOR(xo_decode_byte_vector, int8_t, 4, out[i] = (int8_t)get_be32(s->buf + s->pos))

/* ---- record marking (RFC 1831 §10, docs/rfc1831.txt:688-707) ------------- */
#define RPC_LAST_FRAG 0x80000000u   /* RpcMessageParserTCP.java:37 */
#define RPC_SIZE_MASK 0x7fffffffu   /* RpcMessageParserTCP.java:41 */

uint32_t xo_record_mark(uint32_t payload_len) {             /* GrizzlyRpcTransport:104 */
    return payload_len | RPC_LAST_FRAG;
}
/* isAllFragmentsArrived (RpcMessageParserTCP.java:63-99). */
int xo_all_fragments_arrived(const uint8_t *buf, size_t len) {
    size_t pos = 0;
    if (len < 4) return 0;
    do {
        uint32_t m = get_be32(buf + pos); pos += 4;
        size_t size = m & RPC_SIZE_MASK;
        if (size > len - pos) return 0;          /* fragment bigger than received */
        if (m & RPC_LAST_FRAG) return 1;         /* complete message */
        pos += size;
    } while (len - pos >= 4);
    return 0;
}
/* assembleXdr (RpcMessageParserTCP.java:109-140): the payload is the
 * concatenation of the fragment bodies.                                      */
int xo_assemble(const uint8_t *buf, size_t len, uint8_t *payload, size_t payload_cap,
                size_t *payload_len, size_t *consumed) {
    size_t pos = 0, out = 0; int complete;
    do {
        if (len - pos < 4) return XDRG_E_INCOMPLETE;
        uint32_t m = get_be32(buf + pos); pos += 4;
        size_t size = m & RPC_SIZE_MASK;
        complete = (m & RPC_LAST_FRAG) != 0;
        if (size > len - pos) return XDRG_E_INCOMPLETE;
        if (out + size > payload_cap) return XDRG_E_CAPACITY;
        memcpy(payload + out, buf + pos, size);
        out += size; pos += size;
    } while (!complete);
    *payload_len = out; *consumed = pos;
    return XDRG_OK;
}
/* Repeated handleRead over one socket buffer (:44-61): every complete message
 * is one INVOKE; the remainder is split off (:57-60).                        */
int xo_frame_scan(const uint8_t *buf, size_t len, uint64_t *msg_offsets, uint64_t cap,
                  uint64_t *n_msgs) {
    size_t pos = 0; uint64_t k = 0;
    while (k < cap && xo_all_fragments_arrived(buf + pos, len - pos)) {
        if (msg_offsets) msg_offsets[k] = pos;
        int last = 0;
        while (!last) {
            uint32_t m = get_be32(buf + pos); pos += 4;
            last = (m & RPC_LAST_FRAG) != 0;
            pos += m & RPC_SIZE_MASK;
        }
        k++;
    }
    if (msg_offsets) msg_offsets[k] = pos;
    *n_msgs = k;
    return k ? XDRG_OK : XDRG_E_INCOMPLETE;
}
/* handleRead over one socket buffer followed by the decode of every complete
 * message (RpcMessageParserTCP.java:44-61; assembleXdr :109-140 hands each
 * message body to the next filter as one Xdr, which XdrAble.xdrDecode reads:
 * RpcCall.java:351-354 leaves trailing bytes unread).  Restates the contract
 * of xdrg_receive_batch (include/xdrg.h): at most cap messages; a decode
 * error at message i delivers messages 0..i (CAPACITY: 0..i-1), so the
 * caller resumes after the bad one (RpcDispatcher.java:126-131 answers it
 * GARBAGE_ARGS) or retries it with larger columns.  Bodies go through one
 * concatenated buffer; the per-message extents index it.                   */
int xo_receive_batch(const xdrg_field *fs, size_t nf, const xdrg_cond *conds, size_t nconds,
                     const uint8_t *in, uint64_t len, uint64_t cap, xdrg_column *cols,
                     uint64_t *msg_offsets, uint64_t *n_msgs, uint64_t *consumed,
                     uint64_t *first_bad, int *err) {
    uint64_t k = 0;
    size_t pos = 0;
    uint8_t *body = (uint8_t *)malloc(len + 1);
    uint64_t *ext = (uint64_t *)malloc(sizeof(uint64_t) * (len / 4 + 2));
    uint64_t *mo = (uint64_t *)malloc(sizeof(uint64_t) * (len / 4 + 2));
    if (!body || !ext || !mo) { free(body); free(ext); free(mo); return XDRG_E_NOMEM; }
    size_t blen = 0;
    ext[0] = 0;
    while (k < cap && xo_all_fragments_arrived(in + pos, len - pos)) {
        size_t plen = 0, used = 0;
        if (xo_assemble(in + pos, len - pos, body + blen, len - blen, &plen, &used) != XDRG_OK) break;
        mo[k] = pos;
        pos += used;
        blen += plen;
        ext[++k] = blen;
    }
    mo[k] = pos;
    *n_msgs = k;
    *consumed = pos;
    if (first_bad) *first_bad = k;
    if (err) *err = XDRG_OK;
    int rc = k ? XDRG_OK : XDRG_E_INCOMPLETE;
    if (k) {
        uint64_t fb = k;
        int e = XDRG_OK;
        rc = xo_decode_batch_cond(fs, nf, conds, nconds, body, blen, ext, k, cols, 0, &fb, &e);
        if (rc == XDRG_E_INVAL || rc == XDRG_E_NOMEM) { free(body); free(ext); free(mo); return rc; }
        if (e) {
            const uint64_t upto = e == XDRG_E_CAPACITY ? fb : fb + 1;   /* messages delivered */
            *n_msgs = upto;
            *consumed = mo[upto];
        }
        if (first_bad) *first_bad = fb;
        if (err) *err = e;
    }
    if (msg_offsets)
        for (uint64_t i = 0; i <= *n_msgs; i++) msg_offsets[i] = mo[i];
    free(body); free(ext); free(mo);
    return rc;
}
/* toFragmentedBuffer (ctest/rpc/RpcMessageParserTCPTest.java:161-181). */
size_t xo_fragment(const uint8_t *payload, size_t len, size_t frag, uint8_t *out, size_t cap) {
    size_t nfrag = len / frag + 1, pos = 0, o = 0;
    if (cap < len + 4 * nfrag) return 0;
    do {
        --nfrag;
        size_t fs = len - pos < frag ? len - pos : frag;
        uint32_t m = nfrag > 0 ? (uint32_t)fs : ((uint32_t)fs | RPC_LAST_FRAG);
        put_be32(out + o, m); o += 4;
        if (fs) memcpy(out + o, payload + pos, fs);
        o += fs; pos += fs;
    } while (nfrag > 0);
    return o;
}

/* ---- batch driver -------------------------------------------------------- */
static size_t native_size(uint32_t t) {
    switch (t) {
    case XDRG_T_INT: case XDRG_T_UINT: case XDRG_T_ENUM: case XDRG_T_FLOAT: return 4;
    case XDRG_T_HYPER: case XDRG_T_UHYPER: case XDRG_T_DOUBLE: return 8;
    case XDRG_T_SHORT: return 2;
    case XDRG_T_BYTE: case XDRG_T_BOOL: case XDRG_T_OPAQUE: case XDRG_T_STRING: return 1;
    default: return 0;
    }
}
/* Which (type, kind) pairs rpcgen can emit against the Xdr surface
 * (jrpcgen.java:661-739): no boolean vectors, strings only as string<>,
 * opaque only as opaque[N] / opaque<>.                                       */
static int field_valid(const xdrg_field *f) {
    if (f->type == XDRG_T_GROUP) return 0;   /* checked by check_schema with its members */
    if (!native_size(f->type) || f->kind > XDRG_K_DYNAMIC || f->reserved) return 0;
    if (f->type == XDRG_T_BOOL && f->kind != XDRG_K_SCALAR) return 0;
    if (f->type == XDRG_T_STRING && f->kind != XDRG_K_DYNAMIC) return 0;
    if (f->type == XDRG_T_OPAQUE && f->kind == XDRG_K_SCALAR) return 0;
    if (f->kind == XDRG_K_FIXED && f->count > 0x7fffffffu) return 0;
    return 1;
}
static inline int64_t col_stride(const xdrg_field *f, const xdrg_column *c) {
    size_t cnt = f->kind == XDRG_K_FIXED ? f->count : 1;
    if (c->stride == XDRG_STRIDE_CONST) return 0;   /* constant field (encode only) */
    return c->stride ? c->stride : (int64_t)(native_size(f->type) * cnt);
}
static inline const uint8_t *fixed_ptr(const xdrg_field *f, const xdrg_column *c, uint64_t i) {
    return (const uint8_t *)c->data + (int64_t)i * col_stride(f, c);
}

/* One record's fields, in declaration order, through the stream encoders —
 * what an rpcgen XdrAble.xdrEncode does (jrpcgen.java:788-808).              */
/* Conditional fields (include/xdrg.h xdrg_cond): what rpcgen emits for a
 * union — `switch (disc) { case v: arm; ... default: arm }` with no code for
 * an unmatched value (jrpcgen.java:1240-1340) — and for optional data, a
 * bool and then the value (JrpcgenDeclaration INDIRECTION).  cond_of[k]
 * points at field k's condition or is NULL.                                 */
typedef struct { const xdrg_cond *cond_of[64]; } xo_conds;

static int has_group(const xdrg_field *fs, size_t nf);
/* grp_of[k] = index + 1 of the group field k is an immediate member of, 0
 * at top level (a group inside an element claims its own members after its
 * parent has claimed the whole span) */
static void group_of(const xdrg_field *fs, size_t nf, uint32_t *grp_of) {
    for (size_t k = 0; k < nf; k++) grp_of[k] = 0;
    for (size_t k = 0; k < nf; k++)
        if (fs[k].type == XDRG_T_GROUP)
            for (uint32_t j = 1; j <= fs[k].reserved && k + j < nf; j++) grp_of[k + j] = (uint32_t)k + 1;
}
/* With repeated groups a condition stays on its level: a top-level field
 * (a group included: the whole array / list present or not) on an earlier
 * top-level discriminant, a member (a union or optional inside an element,
 * e.g. READDIRPLUS's post_op_attr in entryplus3) on an earlier member of
 * its own group, evaluated per element.                                      */
static int cond_table(const xdrg_field *fs, size_t nf, const xdrg_cond *conds, size_t nc,
                      xo_conds *t) {
    memset(t, 0, sizeof *t);
    if (nf > 64) return nc ? XDRG_E_INVAL : XDRG_OK;
    uint32_t grp_of[64];
    group_of(fs, nf, grp_of);
    for (size_t i = 0; i < nc; i++) {
        const xdrg_cond *c = &conds[i];
        if (c->field >= nf || c->disc >= c->field || t->cond_of[c->field]) return XDRG_E_INVAL;
        if (grp_of[c->field] != grp_of[c->disc]) return XDRG_E_INVAL;
        const xdrg_field *d = &fs[c->disc];
        if (d->kind != XDRG_K_SCALAR || !(d->type == XDRG_T_INT || d->type == XDRG_T_UINT ||
                                          d->type == XDRG_T_ENUM || d->type == XDRG_T_BOOL))
            return XDRG_E_INVAL;
        t->cond_of[c->field] = c;
    }
    return XDRG_OK;
}
/* Is field k present, given the presence and values of the fields before it? */
static int present(const xo_conds *t, size_t k, const int *pres, const int32_t *val) {
    const xdrg_cond *c = t ? t->cond_of[k] : NULL;
    if (!c) return 1;
    if (!pres[c->disc]) return 0;
    int in = 0;
    for (uint32_t j = 0; j < c->nvalues; j++) in |= c->values[j] == val[c->disc];
    return in != (c->negate != 0);
}

/* Field f of row i of its column — a record for a top-level field, an
 * element for a group member — through the stream encoders. */
static int encode_field(xo_stream *s, const xdrg_field *f, const xdrg_column *c, uint64_t i) {
    int rc = XDRG_OK;
    if (f->kind == XDRG_K_DYNAMIC) {
        uint64_t a = c->offsets[i], b = c->offsets[i + 1];
        const uint8_t *base = (const uint8_t *)c->data + a * native_size(f->type);
        size_t n = (size_t)(b - a);
        switch (f->type) {
        case XDRG_T_INT: case XDRG_T_UINT: case XDRG_T_ENUM:
            rc = xo_encode_int_vector(s, (const int32_t *)base, n); break;
        case XDRG_T_HYPER: case XDRG_T_UHYPER:
            rc = xo_encode_long_vector(s, (const int64_t *)base, n); break;
        case XDRG_T_FLOAT:  rc = xo_encode_float_vector(s, (const float *)base, n); break;
        case XDRG_T_DOUBLE: rc = xo_encode_double_vector(s, (const double *)base, n); break;
        case XDRG_T_SHORT:  rc = xo_encode_short_vector(s, (const int16_t *)base, n); break;
        case XDRG_T_BYTE:   rc = xo_encode_byte_vector(s, (const int8_t *)base, n); break;
        case XDRG_T_OPAQUE: rc = xo_encode_dynamic_opaque(s, base, n); break;
        case XDRG_T_STRING: rc = xo_encode_string(s, base, n); break;
        default: rc = XDRG_E_INVAL;
        }
    } else if (f->kind == XDRG_K_FIXED) {
        const uint8_t *p = fixed_ptr(f, c, i);
        size_t n = f->count; int32_t len = (int32_t)f->count;
        switch (f->type) {
        case XDRG_T_INT: case XDRG_T_UINT: case XDRG_T_ENUM:
            rc = xo_encode_int_fixed_vector(s, (const int32_t *)p, n, len); break;
        case XDRG_T_HYPER: case XDRG_T_UHYPER:
            rc = xo_encode_long_fixed_vector(s, (const int64_t *)p, n, len); break;
        case XDRG_T_FLOAT:  rc = xo_encode_float_fixed_vector(s, (const float *)p, n, len); break;
        case XDRG_T_DOUBLE: rc = xo_encode_double_fixed_vector(s, (const double *)p, n, len); break;
        case XDRG_T_SHORT:  rc = xo_encode_short_fixed_vector(s, (const int16_t *)p, n, len); break;
        case XDRG_T_BYTE:   rc = xo_encode_byte_fixed_vector(s, (const int8_t *)p, n, len); break;
        case XDRG_T_OPAQUE: rc = xo_encode_opaque(s, p, 0, n); break;
        default: rc = XDRG_E_INVAL;
        }
    } else {
        const uint8_t *p = fixed_ptr(f, c, i);
        switch (f->type) {
        case XDRG_T_INT: case XDRG_T_UINT: case XDRG_T_ENUM: {
            int32_t v; memcpy(&v, p, 4); rc = xo_encode_int(s, v); break; }
        case XDRG_T_HYPER: case XDRG_T_UHYPER: {
            int64_t v; memcpy(&v, p, 8); rc = xo_encode_long(s, v); break; }
        case XDRG_T_FLOAT:  { float v; memcpy(&v, p, 4); rc = xo_encode_float(s, v); break; }
        case XDRG_T_DOUBLE: { double v; memcpy(&v, p, 8); rc = xo_encode_double(s, v); break; }
        case XDRG_T_BOOL:   rc = xo_encode_boolean(s, *p != 0); break;
        case XDRG_T_SHORT:  { int16_t v; memcpy(&v, p, 2); rc = xo_encode_short(s, v); break; }
        case XDRG_T_BYTE:   rc = xo_encode_byte(s, (int8_t)*p); break;
        default: rc = XDRG_E_INVAL;
        }
    }
    return rc;
}

/* A repeated group (include/xdrg.h): rpcgen's array-of-structs loop
 * `xdrEncodeInt($size); for (...) x[$idx].xdrEncode(xdr)` (jrpcgen.java:
 * 856-880; no count for T x[N]), or a recursive list: xdrEncodeBoolean(true)
 * and the element while there is one, then xdrEncodeBoolean(false)
 * (portmap/pmaplist.java:63-70).  g[0] is the group, g[1..m] its members. */
/* Presence and discriminant value of member / field k (absolute index gk)
 * at row e, from the native columns (encode). */
static void enc_presence(const xo_conds *cc, size_t gk, const xdrg_field *f, const xdrg_column *c, uint64_t e,
                         int *pres, int32_t *val) {
    pres[gk] = present(cc, gk, pres, val);
    val[gk] = 0;
    if (pres[gk] && f->kind == XDRG_K_SCALAR) {
        const uint8_t *p = fixed_ptr(f, c, e);
        if (f->type == XDRG_T_BOOL) val[gk] = *p != 0;
        else if (native_size(f->type) == 4) memcpy(&val[gk], p, 4);
    }
}

static int encode_group(xo_stream *s, const xdrg_field *g, const xdrg_column *gc, uint64_t i,
                        const xo_conds *cc, size_t gk, int *pres, int32_t *val) {
    const uint32_t m = g->reserved;
    uint64_t e0, cnt;
    if (g->kind == XDRG_K_FIXED) { e0 = i * g->count; cnt = g->count; }
    else { e0 = gc->offsets[i]; cnt = gc->offsets[i + 1] - e0; }
    int rc = XDRG_OK;
    if (g->kind == XDRG_K_DYNAMIC) rc = xo_encode_int(s, (int32_t)cnt);
    for (uint64_t e = e0; !rc && e < e0 + cnt; e++) {
        if (g->kind == XDRG_K_LIST) rc = xo_encode_boolean(s, 1);
        for (uint32_t j = 1; !rc && j <= m; j++) {
            /* an element's union arms / optional data (jrpcgen.java:1240-1340) */
            enc_presence(cc, gk + j, &g[j], &gc[j], e, pres, val);
            const uint32_t span = g[j].type == XDRG_T_GROUP ? g[j].reserved : 0;
            if (pres[gk + j]) {
                /* an array of structs / list inside the element: its own count
                 * and elements, as the element's generated xdrEncode calls the
                 * inner elements' (jrpcgen.java:856-906, 835-851); its column
                 * is indexed by this group's element e */
                rc = span ? encode_group(s, &g[j], &gc[j], e, cc, gk + j, pres, val)
                          : encode_field(s, &g[j], &gc[j], e);
            }
            j += span;
        }
    }
    if (!rc && g->kind == XDRG_K_LIST) rc = xo_encode_boolean(s, 0);
    return rc;
}

/* shallow >= 0: that dynamic opaque/string field is encoded by reference
 * (xdrEncodeFileChunk); *chunk_at = its splice position in the record's
 * buffer, *chunk_len = its bytes (padding implied), or *chunk_at = ~0 when
 * the field is absent.                                                       */
static int encode_record_ex(xo_stream *s, const xdrg_field *fs, size_t nf, const xdrg_column *cols,
                            uint64_t i, const xo_conds *cc, int shallow, uint64_t *chunk_at,
                            uint64_t *chunk_len) {
    int pres[64]; int32_t val[64];
    for (size_t k = 0; k < nf; k++) {
        const xdrg_field *f = &fs[k];
        const xdrg_column *c = &cols[k];
        int rc = XDRG_OK;
        if (k < 64) {
            pres[k] = present(cc, k, pres, val);
            if (!pres[k]) {
                if (f->type == XDRG_T_GROUP) k += f->reserved;   /* nothing of the array / list */
                continue;
            }
            val[k] = 0;
            if (f->kind == XDRG_K_SCALAR) {
                const uint8_t *p = fixed_ptr(f, c, i);
                if (f->type == XDRG_T_BOOL) val[k] = *p != 0;
                else if (native_size(f->type) == 4) memcpy(&val[k], p, 4);
            }
        }
        if (f->kind == XDRG_K_DYNAMIC && (int)k == shallow) {
            uint64_t a = c->offsets[i], b = c->offsets[i + 1];
            uint32_t padding;
            rc = xo_encode_file_chunk(s, (size_t)(b - a), &padding);
            if (rc) return rc;
            *chunk_at = s->pos;
            *chunk_len = b - a;
            continue;
        }
        if (f->type == XDRG_T_GROUP) {
            rc = encode_group(s, fs + k, cols + k, i, cc, k, pres, val);
            if (rc) return rc;
            k += f->reserved;   /* its members */
            continue;
        }
        rc = encode_field(s, f, c, i);
        if (rc) return rc;
    }
    return XDRG_OK;
}

static int encode_record(xo_stream *s, const xdrg_field *fs, size_t nf, const xdrg_column *cols,
                         uint64_t i, const xo_conds *cc) {
    uint64_t at, len;
    return encode_record_ex(s, fs, nf, cols, i, cc, -1, &at, &len);
}

/* Repeated groups (include/xdrg.h): the group field, then `reserved` member
 * fields of the base types or groups of them, down to XO_GROUP_LEVELS levels
 * (an inner group's own span counted in the outer `reserved`); an element
 * that encodes to at least one byte (list elements carry their bool, a
 * counted inner array its count). */
#define XO_GROUP_LEVELS 4
static int has_group(const xdrg_field *fs, size_t nf) {
    for (size_t k = 0; k < nf; k++) if (fs[k].type == XDRG_T_GROUP) return 1;
    return 0;
}
/* The group at g (a span of `lim` fields from g on, depth 0 = top level):
 * XDRG_OK and *sized = whether an element encodes to >= 1 byte. */
static int check_group(const xdrg_field *g, size_t lim, int depth, int *sized_out) {
    const uint32_t m = g->reserved;
    if (g->kind < XDRG_K_FIXED || g->kind > XDRG_K_LIST || m == 0 || m > lim - 1) return XDRG_E_INVAL;
    if ((g->kind == XDRG_K_FIXED && g->count > 0x7fffffffu) || (g->kind == XDRG_K_LIST && g->count))
        return XDRG_E_INVAL;
    int sized = g->kind == XDRG_K_LIST;
    for (uint32_t j = 1; j <= m; j++) {
        const xdrg_field *f = &g[j];
        if (f->type == XDRG_T_GROUP) {
            int s2 = 0;
            if (depth + 1 >= XO_GROUP_LEVELS || check_group(f, (size_t)m + 1 - j, depth + 1, &s2) || !s2)
                return XDRG_E_INVAL;
            sized |= f->kind != XDRG_K_FIXED || f->count > 0;
            j += f->reserved;
            continue;
        }
        if (!field_valid(f)) return XDRG_E_INVAL;
        sized |= f->kind == XDRG_K_DYNAMIC || f->kind == XDRG_K_SCALAR || f->count > 0;
    }
    *sized_out = sized;
    return XDRG_OK;
}
static int check_schema(const xdrg_field *fs, size_t nf) {
    if (!fs || !nf || nf > 64) return XDRG_E_INVAL;
    for (size_t k = 0; k < nf; k++) {
        const xdrg_field *g = &fs[k];
        if (g->type != XDRG_T_GROUP) {
            if (!field_valid(g)) return XDRG_E_INVAL;
            continue;
        }
        int sized = 0;
        if (check_group(g, nf - k, 0, &sized) || !sized) return XDRG_E_INVAL;
        k += g->reserved;
    }
    return XDRG_OK;
}

int xo_encode_batch(const xdrg_field *fs, size_t nf, const xdrg_column *cols, uint64_t n,
                    uint8_t *out, uint64_t out_cap, uint64_t *rec_offsets, uint32_t flags,
                    uint64_t *out_len) {
    return xo_encode_batch_cond(fs, nf, NULL, 0, cols, n, out, out_cap, rec_offsets, flags, out_len);
}
int xo_encode_batch_cond(const xdrg_field *fs, size_t nf, const xdrg_cond *conds, size_t nconds,
                         const xdrg_column *cols, uint64_t n, uint8_t *out, uint64_t out_cap,
                         uint64_t *rec_offsets, uint32_t flags, uint64_t *out_len) {
    int rc = check_schema(fs, nf); if (rc) return rc;
    xo_conds cc;
    rc = cond_table(fs, nf, conds, nconds, &cc); if (rc) return rc;
    const int framed = (flags & XDRG_FRAME_RM) != 0;
    uint64_t pos = 0;
    for (uint64_t i = 0; i < n; i++) {
        if (rec_offsets) rec_offsets[i] = pos;
        uint64_t body = pos + (framed ? 4 : 0);
        if (body > out_cap) return XDRG_E_CAPACITY;
        /* the record is encoded as its own Xdr message (RpcCall.acceptedReply
         * encodes one message per Xdr, RpcCall.java:323-343) ...            */
        xo_stream s;
        xo_stream_wrap(&s, out + body, (size_t)(out_cap - body));
        xo_begin_encoding(&s);
        rc = encode_record(&s, fs, nf, cols, i, nconds ? &cc : NULL);
        if (rc) return rc;
        xo_end_encoding(&s);
        /* ... and framed as GrizzlyRpcTransport.sendDefault does (:103-110). */
        if (framed) put_be32(out + pos, xo_record_mark((uint32_t)s.limit));
        pos = body + s.limit;
    }
    if (rec_offsets) rec_offsets[n] = pos;
    if (out_len) *out_len = pos;
    return XDRG_OK;
}

/* Batch of messages each carrying one payload by reference: the buffer part
 * of every record back to back in `out` (record offsets in rec_offsets),
 * splice[i] = where record i's payload (then its zero padding) goes, or
 * UINT64_MAX when the field is absent.  With XDRG_FRAME_RM the mark counts
 * every part, as sendRawTCP does (GrizzlyRpcTransport.java:130-139,
 * 224-231).                                                                  */
int xo_encode_batch_shallow(const xdrg_field *fs, size_t nf, const xdrg_cond *conds, size_t nconds,
                            const xdrg_column *cols, uint64_t n, uint8_t *out, uint64_t out_cap,
                            uint64_t *rec_offsets, uint32_t flags, uint64_t *out_len,
                            uint32_t field, uint64_t *splice) {
    int rc = check_schema(fs, nf); if (rc) return rc;
    if (has_group(fs, nf)) return XDRG_E_INVAL;
    if (field >= nf || fs[field].kind != XDRG_K_DYNAMIC ||
        (fs[field].type != XDRG_T_OPAQUE && fs[field].type != XDRG_T_STRING)) return XDRG_E_INVAL;
    xo_conds cc;
    rc = cond_table(fs, nf, conds, nconds, &cc); if (rc) return rc;
    const int framed = (flags & XDRG_FRAME_RM) != 0;
    uint64_t pos = 0;
    for (uint64_t i = 0; i < n; i++) {
        if (rec_offsets) rec_offsets[i] = pos;
        uint64_t body = pos + (framed ? 4 : 0);
        if (body > out_cap) return XDRG_E_CAPACITY;
        xo_stream s;
        xo_stream_wrap(&s, out + body, (size_t)(out_cap - body));
        xo_begin_encoding(&s);
        uint64_t at = UINT64_MAX, len = 0;
        rc = encode_record_ex(&s, fs, nf, cols, i, nconds ? &cc : NULL, (int)field, &at, &len);
        if (rc) return rc;
        xo_end_encoding(&s);
        uint64_t chunk = at == UINT64_MAX ? 0 : len + pad4((size_t)len);
        if (framed) put_be32(out + pos, xo_record_mark((uint32_t)(s.limit + chunk)));
        splice[i] = at == UINT64_MAX ? UINT64_MAX : body + at;
        pos = body + s.limit;
    }
    if (rec_offsets) rec_offsets[n] = pos;
    if (out_len) *out_len = pos;
    return XDRG_OK;
}

/* Field f of row i of its column (a record, or an element of a group)
 * through the stream decoders; dynamic fields append at offsets[i]. */
static int decode_field(xo_stream *s, const xdrg_field *f, xdrg_column *c, uint64_t i) {
    int rc = XDRG_OK;
    if (f->kind == XDRG_K_DYNAMIC) {
        size_t es = native_size(f->type);
        uint64_t a = c->offsets[i];
        uint8_t *base = (uint8_t *)c->data + a * es;
        size_t cap = c->cap > a ? (size_t)(c->cap - a) : 0, got = 0;
        switch (f->type) {
        case XDRG_T_INT: case XDRG_T_UINT: case XDRG_T_ENUM:
            rc = xo_decode_int_vector(s, (int32_t *)base, cap, &got); break;
        case XDRG_T_HYPER: case XDRG_T_UHYPER:
            rc = xo_decode_long_vector(s, (int64_t *)base, cap, &got); break;
        case XDRG_T_FLOAT:  rc = xo_decode_float_vector(s, (float *)base, cap, &got); break;
        case XDRG_T_DOUBLE: rc = xo_decode_double_vector(s, (double *)base, cap, &got); break;
        case XDRG_T_SHORT:  rc = xo_decode_short_vector(s, (int16_t *)base, cap, &got); break;
        case XDRG_T_BYTE:   rc = xo_decode_byte_vector(s, (int8_t *)base, cap, &got); break;
        case XDRG_T_OPAQUE: case XDRG_T_STRING: {
            const uint8_t *p; size_t len;
            rc = f->type == XDRG_T_OPAQUE ? xo_decode_dynamic_opaque(s, &p, &len)
                                          : xo_decode_string(s, &p, &len);
            if (!rc && len > cap) rc = XDRG_E_CAPACITY;
            if (!rc) { memcpy(base, p, len); got = len; }
            break; }
        default: rc = XDRG_E_INVAL;
        }
        if (rc) return rc;
        c->offsets[i + 1] = a + got;
    } else {
        size_t cnt = f->kind == XDRG_K_FIXED ? f->count : 1;
        uint8_t *p = (uint8_t *)fixed_ptr(f, c, i);
        if (f->type == XDRG_T_OPAQUE) return xo_decode_opaque(s, p, cnt);
        for (size_t e = 0; e < cnt && !rc; e++) {
            switch (f->type) {
            case XDRG_T_INT: case XDRG_T_UINT: case XDRG_T_ENUM: {
                int32_t v; rc = xo_decode_int(s, &v); if (!rc) memcpy(p + 4 * e, &v, 4); break; }
            case XDRG_T_FLOAT: {
                float v; rc = xo_decode_float(s, &v); if (!rc) memcpy(p + 4 * e, &v, 4); break; }
            case XDRG_T_HYPER: case XDRG_T_UHYPER: {
                int64_t v; rc = xo_decode_long(s, &v); if (!rc) memcpy(p + 8 * e, &v, 8); break; }
            case XDRG_T_DOUBLE: {
                double v; rc = xo_decode_double(s, &v); if (!rc) memcpy(p + 8 * e, &v, 8); break; }
            case XDRG_T_BOOL: { int v; rc = xo_decode_boolean(s, &v); if (!rc) p[e] = (uint8_t)v; break; }
            case XDRG_T_SHORT: {
                int16_t v; rc = xo_decode_short(s, &v); if (!rc) memcpy(p + 2 * e, &v, 2); break; }
            case XDRG_T_BYTE: { int8_t v; rc = xo_decode_byte(s, &v); if (!rc) p[e] = (uint8_t)v; break; }
            default: rc = XDRG_E_INVAL;
            }
        }
        if (rc) return rc;
    }
    return XDRG_OK;
}

/* Count of a repeated group's elements as its decoder meets them: rpcgen's
 * `int $size = xdr.xdrDecodeInt(); x = new T[$size]` — no checkArraySize, so
 * a negative count is NegativeArraySizeException (jrpcgen.java:886-906) —
 * or a list's `xdrDecodeBoolean()` before every element (pmaplist.java:
 * 52-61).  The first pass walks the group with every member's checks on a
 * copy of the stream (walk errors come first, in the reference's order);
 * then the element and member capacities; then the second pass decodes.   */
/* Presence and discriminant value of field k (absolute index gk) as a
 * decoder meets it: the value is the word about to be decoded. */
static void dec_presence(const xo_conds *cc, size_t gk, const xdrg_field *f, const xo_stream *s, int *pres,
                         int32_t *val) {
    pres[gk] = present(cc, gk, pres, val);
    val[gk] = 0;
    if (pres[gk] && f->kind == XDRG_K_SCALAR && xo_remaining(s) >= 4) {
        const int32_t w = (int32_t)get_be32(s->buf + s->pos);
        val[gk] = f->type == XDRG_T_BOOL ? (w != 0) : w;
    }
}

static int walk_group(xo_stream *s, const xdrg_field *g, uint64_t *cnt_out, uint64_t *mcnt,
                      const xo_conds *cc, size_t gk, int *pres, int32_t *val) {
    const uint32_t m = g->reserved;
    for (uint32_t j = 1; j <= m; j++) mcnt[j] = 0;
    uint64_t cnt = 0;
    int rc = XDRG_OK;
    if (g->kind == XDRG_K_DYNAMIC) {
        int32_t v;
        rc = xo_decode_int(s, &v);
        if (rc) return rc;
        if (v < 0) return XDRG_E_NEG_SIZE;
        cnt = (uint64_t)v;
    } else if (g->kind == XDRG_K_FIXED) {
        cnt = g->count;
    }
    for (uint64_t e = 0;; e++) {
        if (g->kind == XDRG_K_LIST) {
            int more;
            rc = xo_decode_boolean(s, &more);
            if (rc) return rc;
            if (!more) break;
        } else if (e == cnt) {
            break;
        }
        for (uint32_t j = 1; j <= m; j++) {
            const xdrg_field *f = &g[j];
            dec_presence(cc, gk + j, f, s, pres, val);
            if (f->type == XDRG_T_GROUP) {   /* an inner array / list: its elements and members */
                if (pres[gk + j]) {
                    uint64_t icnt = 0, imcnt[64];
                    rc = walk_group(s, f, &icnt, imcnt, cc, gk + j, pres, val);
                    if (rc) return rc;
                    mcnt[j] += icnt;
                    for (uint32_t jj = 1; jj <= f->reserved; jj++) mcnt[j + jj] += imcnt[jj];
                }
                j += f->reserved;
                continue;
            }
            if (!pres[gk + j]) continue;
            if (f->kind == XDRG_K_DYNAMIC) {
                int32_t len;
                rc = xo_decode_int(s, &len);
                if (rc) return rc;
                size_t need;
                if (f->type == XDRG_T_OPAQUE || f->type == XDRG_T_STRING) {
                    if (len == 0) continue;                       /* Xdr.java:376-378 */
                    if (len < 0) return XDRG_E_CORRUPT;           /* checkArraySize :1034-1037 */
                    need = (size_t)len + pad4((size_t)len);
                } else {
                    if (len < 0) return XDRG_E_CORRUPT;
                    need = (size_t)len * (native_size(f->type) == 8 ? 8 : 4);
                }
                rc = ensure_bytes(s, need);
                if (rc) return rc;
                s->pos += need;
                mcnt[j] += (uint64_t)len;
            } else {
                size_t n = f->kind == XDRG_K_FIXED ? f->count : 1;
                size_t need = f->type == XDRG_T_OPAQUE ? n + pad4(n)
                            : n * ((f->type == XDRG_T_HYPER || f->type == XDRG_T_UHYPER || f->type == XDRG_T_DOUBLE) ? 8 : 4);
                rc = ensure_bytes(s, need);
                if (rc) return rc;
                s->pos += need;
            }
        }
        if (g->kind == XDRG_K_LIST) cnt++;
    }
    *cnt_out = cnt;
    return XDRG_OK;
}

/* The defaults of a freshly constructed rpcgen object for an absent field
 * at row e: zero, or an empty run (its offsets entry repeats). */
static void absent_field(const xdrg_field *f, xdrg_column *c, uint64_t e) {
    if (f->kind == XDRG_K_DYNAMIC) c->offsets[e + 1] = c->offsets[e];
    else {
        size_t cnt = f->kind == XDRG_K_FIXED ? f->count : 1;
        memset((uint8_t *)fixed_ptr(f, c, e), 0, cnt * native_size(f->type));
    }
}
/* An absent array / list at row i of its column: no elements, or a T x[N]'s
 * N zero / empty elements (inner arrays in them empty too). */
static void absent_group(const xdrg_field *g, xdrg_column *gc, uint64_t i) {
    if (g->kind != XDRG_K_FIXED) { gc->offsets[i + 1] = gc->offsets[i]; return; }
    for (uint64_t e = i * g->count; e < (i + 1) * g->count; e++)
        for (uint32_t j = 1; j <= g->reserved; j++) {
            if (g[j].type == XDRG_T_GROUP) {
                absent_group(&g[j], &gc[j], e);
                j += g[j].reserved;
            } else {
                absent_field(&g[j], &gc[j], e);
            }
        }
}

/* Capacity of every column in group g's span for the rows one record adds:
 * its members' from row e0 on (the group's first element for the record),
 * an inner group's elements from its first row i0 and, recursively, its own
 * members; mcnt[j] = what the record's walk counted for member j. */
static int members_fit(const xdrg_field *g, const xdrg_column *gc, uint64_t e0, const uint64_t *mcnt) {
    for (uint32_t j = 1; j <= g->reserved; j++) {
        if (g[j].type == XDRG_T_GROUP) {   /* an inner array: its elements start at row i0 */
            const xdrg_field *ig = &g[j];
            const xdrg_column *ic = &gc[j];
            const uint64_t i0 = ig->kind == XDRG_K_FIXED ? e0 * ig->count : ic->offsets[e0];
            if (ig->kind != XDRG_K_FIXED && i0 + mcnt[j] > ic->cap) return XDRG_E_CAPACITY;
            int rc = members_fit(ig, ic, i0, mcnt + j);
            if (rc) return rc;
            j += ig->reserved;
            continue;
        }
        if (g[j].kind == XDRG_K_DYNAMIC && gc[j].offsets[e0] + mcnt[j] > gc[j].cap) return XDRG_E_CAPACITY;
    }
    return XDRG_OK;
}

static int decode_group(xo_stream *s, const xdrg_field *g, xdrg_column *gc, uint64_t i,
                        const xo_conds *cc, size_t gk, int *pres, int32_t *val) {
    const uint32_t m = g->reserved;
    uint64_t mcnt[64], cnt = 0;
    xo_stream w = *s;
    int rc = walk_group(&w, g, &cnt, mcnt, cc, gk, pres, val);
    if (rc) return rc;
    const uint64_t e0 = g->kind == XDRG_K_FIXED ? i * g->count : gc->offsets[i];
    if (g->kind != XDRG_K_FIXED && e0 + cnt > gc->cap) return XDRG_E_CAPACITY;
    rc = members_fit(g, gc, e0, mcnt);
    if (rc) return rc;
    if (g->kind == XDRG_K_DYNAMIC) s->pos += 4;
    for (uint64_t e = e0; e < e0 + cnt; e++) {
        if (g->kind == XDRG_K_LIST) s->pos += 4;
        for (uint32_t j = 1; j <= m; j++) {
            dec_presence(cc, gk + j, &g[j], s, pres, val);
            const uint32_t span = g[j].type == XDRG_T_GROUP ? g[j].reserved : 0;
            if (!pres[gk + j]) {
                if (span) absent_group(&g[j], &gc[j], e);
                else absent_field(&g[j], &gc[j], e);
                j += span;
                continue;
            }
            rc = span ? decode_group(s, &g[j], &gc[j], e, cc, gk + j, pres, val)
                      : decode_field(s, &g[j], &gc[j], e);
            if (rc) return rc;
            j += span;
        }
    }
    if (g->kind == XDRG_K_LIST) s->pos += 4;
    if (g->kind != XDRG_K_FIXED) gc->offsets[i + 1] = e0 + cnt;
    return XDRG_OK;
}

/* One record's fields through the stream decoders (XdrAble.xdrDecode). */
static int decode_record(xo_stream *s, const xdrg_field *fs, size_t nf, xdrg_column *cols,
                         uint64_t i, const xo_conds *cc, int view, const uint8_t *base_in,
                         uint64_t *view_pos) {
    int pres[64]; int32_t val[64];
    for (size_t k = 0; k < nf; k++) {
        const xdrg_field *f = &fs[k];
        xdrg_column *c = &cols[k];
        int rc = XDRG_OK;
        if (k < 64) {
            pres[k] = present(cc, k, pres, val);
            val[k] = 0;
            if (pres[k] && f->kind == XDRG_K_SCALAR && xo_remaining(s) >= 4) {
                int32_t w = (int32_t)get_be32(s->buf + s->pos);   /* the value about to decode */
                val[k] = f->type == XDRG_T_BOOL ? (w != 0) : w;
            }
            if (!pres[k]) {   /* absent: the defaults of a new rpcgen object */
                if ((int)k == view) view_pos[i] = UINT64_MAX;
                if (f->type == XDRG_T_GROUP) {   /* no elements (a FIXED group's are zero / empty) */
                    absent_group(f, c, i);
                    k += f->reserved;
                    continue;
                }
                absent_field(f, c, i);
                continue;
            }
        }
        if (f->kind == XDRG_K_DYNAMIC && (int)k == view) {
            /* xdrDecodeByteBuffer (Xdr.java:423-439): a slice of the stream */
            const uint8_t *p; size_t len;
            rc = xo_decode_byte_buffer(s, &p, &len);
            if (rc) return rc;
            view_pos[i] = (uint64_t)(p - base_in);
            c->offsets[i + 1] = c->offsets[i] + len;
            continue;
        }
        if (f->type == XDRG_T_GROUP) {
            rc = decode_group(s, fs + k, cols + k, i, cc, k, pres, val);
            if (rc) return rc;
            k += f->reserved;   /* its members */
            continue;
        }
        rc = decode_field(s, f, c, i);
        if (rc) return rc;
    }
    return XDRG_OK;
}

static uint64_t schema_fixed_size(const xdrg_field *fs, size_t nf) {
    uint64_t sz = 0;
    if (has_group(fs, nf)) return 0;   /* repeated groups: record offsets, like dynamic fields */
    for (size_t k = 0; k < nf; k++) {
        const xdrg_field *f = &fs[k];
        if (f->kind == XDRG_K_DYNAMIC) return 0;
        uint64_t cnt = f->kind == XDRG_K_FIXED ? f->count : 1;
        if (f->type == XDRG_T_OPAQUE) sz += cnt + pad4((size_t)cnt);
        else if (f->type == XDRG_T_HYPER || f->type == XDRG_T_UHYPER || f->type == XDRG_T_DOUBLE) sz += 8 * cnt;
        else sz += 4 * cnt;
    }
    return sz;
}

int xo_decode_batch(const xdrg_field *fs, size_t nf, const uint8_t *in, uint64_t in_len,
                    const uint64_t *rec_offsets, uint64_t n, xdrg_column *cols, uint32_t flags,
                    uint64_t *first_bad, int *err) {
    return xo_decode_batch_cond(fs, nf, NULL, 0, in, in_len, rec_offsets, n, cols, flags,
                                first_bad, err);
}
int xo_decode_batch_cond(const xdrg_field *fs, size_t nf, const xdrg_cond *conds, size_t nconds,
                         const uint8_t *in, uint64_t in_len, const uint64_t *rec_offsets,
                         uint64_t n, xdrg_column *cols, uint32_t flags, uint64_t *first_bad,
                         int *err) {
    return xo_decode_batch_view(fs, nf, conds, nconds, in, in_len, rec_offsets, n, cols, flags,
                                first_bad, err, UINT32_MAX, NULL);
}
/* view < nfields: that dynamic opaque/string field decodes as a slice of the
 * stream (xdrDecodeByteBuffer): view_pos[i] = its payload's offset in `in`,
 * offsets[] as if copied; nothing is copied.                                 */
int xo_decode_batch_view(const xdrg_field *fs, size_t nf, const xdrg_cond *conds, size_t nconds,
                         const uint8_t *in, uint64_t in_len, const uint64_t *rec_offsets,
                         uint64_t n, xdrg_column *cols, uint32_t flags, uint64_t *first_bad,
                         int *err, uint32_t field, uint64_t *view_pos) {
    int rc = check_schema(fs, nf); if (rc) return rc;
    const int view = field < nf ? (int)field : -1;
    if (view >= 0 && has_group(fs, nf)) return XDRG_E_INVAL;
    if (field != UINT32_MAX && (view < 0 || fs[field].kind != XDRG_K_DYNAMIC || !view_pos ||
        (fs[field].type != XDRG_T_OPAQUE && fs[field].type != XDRG_T_STRING))) return XDRG_E_INVAL;
    xo_conds cc;
    rc = cond_table(fs, nf, conds, nconds, &cc); if (rc) return rc;
    const int framed = (flags & XDRG_FRAME_RM) != 0;
    const uint64_t fixed = nconds ? 0 : schema_fixed_size(fs, nf);
    if (!rec_offsets && !fixed) return XDRG_E_INVAL;
    for (size_t k = 0; k < nf; k++)
        if (fs[k].kind != XDRG_K_DYNAMIC && cols[k].stride == XDRG_STRIDE_CONST) return XDRG_E_INVAL;
    for (size_t k = 0; k < nf; k++)
        if ((fs[k].kind == XDRG_K_DYNAMIC || (fs[k].type == XDRG_T_GROUP && fs[k].kind == XDRG_K_LIST)) && n)
            cols[k].offsets[0] = 0;
    const uint64_t stride = fixed + (framed ? 4 : 0);
    for (uint64_t i = 0; i < n; i++) {
        uint64_t a, b;
        if (rec_offsets) { a = rec_offsets[i]; b = rec_offsets[i + 1]; }
        else { a = i * stride; b = a + stride; }
        if (b > in_len) b = in_len;
        if (a > b) a = b;
        rc = XDRG_OK;
        if (framed) {
            /* one record = one single-fragment message (GrizzlyRpcTransport:104) */
            if (b - a < 4) rc = XDRG_E_SHORT;
            else {
                uint32_t m = get_be32(in + a);
                uint64_t want = rec_offsets ? (b - a - 4) : fixed;
                if (!(m & RPC_LAST_FRAG) || (m & RPC_SIZE_MASK) != want) rc = XDRG_E_FRAME;
                a += 4;
            }
        }
        if (!rc) {
            xo_stream s;
            xo_stream_wrap(&s, (uint8_t *)in + a, (size_t)(b - a));
            xo_begin_decoding(&s);
            rc = decode_record(&s, fs, nf, cols, i, nconds ? &cc : NULL, view, in, view_pos);
        }
        if (rc) {
            if (first_bad) *first_bad = i;
            if (err) *err = rc;
            return rc;
        }
    }
    if (first_bad) *first_bad = n;
    if (err) *err = XDRG_OK;
    return XDRG_OK;
}

/* ---- multithreaded driver (all-cores CPU baseline) ------------------------- */
typedef struct {
    const xdrg_field *fs; size_t nf; const xdrg_column *cols; xdrg_column *ocols;
    uint64_t lo, hi; uint8_t *buf; uint64_t stride; uint64_t in_len;
    uint32_t flags; int rc; uint64_t first_bad; int err;
} mt_job;

static void *enc_worker(void *arg) {
    mt_job *j = (mt_job *)arg;
    xdrg_column sub[64];
    for (size_t k = 0; k < j->nf; k++) {
        sub[k] = j->cols[k];
        sub[k].data = (uint8_t *)sub[k].data + (int64_t)j->lo * col_stride(&j->fs[k], &sub[k]);
    }
    uint64_t len;
    j->rc = xo_encode_batch(j->fs, j->nf, sub, j->hi - j->lo, j->buf + j->lo * j->stride,
                            (j->hi - j->lo) * j->stride, NULL, j->flags, &len);
    return NULL;
}
static void *dec_worker(void *arg) {
    mt_job *j = (mt_job *)arg;
    xdrg_column sub[64];
    for (size_t k = 0; k < j->nf; k++) {
        sub[k] = j->ocols[k];
        sub[k].data = (uint8_t *)sub[k].data + (int64_t)j->lo * col_stride(&j->fs[k], &sub[k]);
    }
    uint64_t start = j->lo * j->stride;
    uint64_t avail = j->in_len > start ? j->in_len - start : 0;
    j->rc = xo_decode_batch(j->fs, j->nf, j->buf + start, avail, NULL, j->hi - j->lo, sub,
                            j->flags, &j->first_bad, &j->err);
    j->first_bad += j->lo;
    return NULL;
}
static int run_mt(void *(*fn)(void *), mt_job *proto, uint64_t n, int threads) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256]; mt_job jobs[256];
    for (int t = 0; t < threads; t++) {
        jobs[t] = *proto;
        jobs[t].lo = n * (uint64_t)t / (uint64_t)threads;
        jobs[t].hi = n * (uint64_t)(t + 1) / (uint64_t)threads;
        if (pthread_create(&th[t], NULL, fn, &jobs[t])) { threads = t; break; }
    }
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    int rc = XDRG_OK; uint64_t fb = n; int err = XDRG_OK;
    for (int t = 0; t < threads; t++) {
        if (jobs[t].rc && jobs[t].first_bad < fb) { fb = jobs[t].first_bad; err = jobs[t].err; rc = jobs[t].rc; }
        else if (jobs[t].rc && !rc) rc = jobs[t].rc;
    }
    proto->first_bad = fb; proto->err = err;
    return rc;
}
int xo_encode_batch_mt(const xdrg_field *fs, size_t nf, const xdrg_column *cols, uint64_t n,
                       uint8_t *out, uint64_t out_cap, uint32_t flags, uint64_t *out_len,
                       int threads) {
    int rc = check_schema(fs, nf); if (rc) return rc;
    if (nf > 64) return XDRG_E_INVAL;
    uint64_t fixed = schema_fixed_size(fs, nf);
    if (!fixed) return XDRG_E_INVAL;
    uint64_t stride = fixed + ((flags & XDRG_FRAME_RM) ? 4 : 0);
    if (out_cap < n * stride) return XDRG_E_CAPACITY;
    mt_job p; memset(&p, 0, sizeof p);
    p.fs = fs; p.nf = nf; p.cols = cols; p.buf = out; p.stride = stride; p.flags = flags;
    p.first_bad = n;
    rc = run_mt(enc_worker, &p, n, threads);
    if (!rc && out_len) *out_len = n * stride;
    return rc;
}
int xo_decode_batch_mt(const xdrg_field *fs, size_t nf, const uint8_t *in, uint64_t in_len,
                       uint64_t n, xdrg_column *cols, uint32_t flags, uint64_t *first_bad,
                       int *err, int threads) {
    int rc = check_schema(fs, nf); if (rc) return rc;
    if (nf > 64) return XDRG_E_INVAL;
    uint64_t fixed = schema_fixed_size(fs, nf);
    if (!fixed) return XDRG_E_INVAL;
    mt_job p; memset(&p, 0, sizeof p);
    p.fs = fs; p.nf = nf; p.ocols = cols; p.buf = (uint8_t *)in; p.in_len = in_len;
    p.stride = fixed + ((flags & XDRG_FRAME_RM) ? 4 : 0); p.flags = flags; p.first_bad = n;
    rc = run_mt(dec_worker, &p, n, threads);
    if (first_bad) *first_bad = p.first_bad;
    if (err) *err = p.err;
    return rc;
}
