/*
 * xdr_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C CPU restatement of the reference codec, used as the parity
 * checker for the HIP engine and as the CPU baseline in bench.py.  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * it; the product path (oncrpc4j_amd/, libxdrgpu.so) never does.
 *
 * Restated sources (under /root/reference/oncrpc4j-core/src/main/java/
 * org/dcache/oncrpc4j/):
 *   xdr/Xdr.java:39-1039                    stream codec, bounds/error order
 *   grizzly/GrizzlyRpcTransport.java:97-110 record mark on send
 *   rpc/RpcMessageParserTCP.java:44-140     record-mark walk / assembly
 *   util/Bytes.java:39-107                  big-endian helpers
 * Pinned by the reference's own known-answer tests (tests/golden/
 * kat_reference.json, from ctest/xdr/Xdr{Int,Long,Opaque}Test.java and
 * XdrTest.java) and by vectors from an independent RFC 1014 implementation
 * (tests/golden/xdrlib_vectors.json).
 */
#ifndef XDR_ORACLE_H
#define XDR_ORACLE_H

#include <stddef.h>
#include <stdint.h>
#include "../include/xdrg.h"

#ifdef __cplusplus
extern "C" {
#endif

/* A Grizzly-Buffer-like byte stream: position / limit / capacity, BIG_ENDIAN
 * (Xdr.java:115-119).  `growable` mirrors GrizzlyMemoryManager.reallocate
 * (Xdr.java:1020-1026); a wrapped caller buffer is not growable.            */
typedef struct xo_stream {
    uint8_t *buf;
    size_t   cap;
    size_t   pos;
    size_t   limit;
    int      in_use;
    int      growable;
} xo_stream;

int  xo_stream_alloc(xo_stream *s, size_t size);          /* new Xdr(size)   Xdr.java:82  */
void xo_stream_wrap(xo_stream *s, uint8_t *buf, size_t len); /* new Xdr(bytes) Xdr.java:96 */
void xo_stream_free(xo_stream *s);
void xo_begin_encoding(xo_stream *s);   /* clear  Xdr.java:137 */
void xo_end_encoding(xo_stream *s);     /* flip   Xdr.java:143 */
void xo_begin_decoding(xo_stream *s);   /* rewind Xdr.java:122 */
void xo_end_decoding(xo_stream *s);     /* rewind Xdr.java:131 */
int  xo_has_more_data(const xo_stream *s);               /* Xdr.java:152 */
size_t xo_remaining(const xo_stream *s);

/* encoders: return XDRG_OK / XDRG_E_NOMEM / XDRG_E_CAPACITY / XDRG_E_FIXED_LEN */
int xo_encode_int(xo_stream *s, int32_t v);
int xo_encode_long(xo_stream *s, int64_t v);
int xo_encode_float(xo_stream *s, float v);
int xo_encode_double(xo_stream *s, double v);
int xo_encode_boolean(xo_stream *s, int v);
int xo_encode_byte(xo_stream *s, int8_t v);
int xo_encode_short(xo_stream *s, int16_t v);
int xo_encode_opaque(xo_stream *s, const uint8_t *b, size_t off, size_t len);
int xo_encode_dynamic_opaque(xo_stream *s, const uint8_t *b, size_t len);
int xo_encode_string(xo_stream *s, const uint8_t *utf8, size_t len); /* NULL -> "" */
int xo_encode_byte_buffer(xo_stream *s, const uint8_t *b, size_t len);
int xo_encode_int_vector(xo_stream *s, const int32_t *v, size_t n);
int xo_encode_int_fixed_vector(xo_stream *s, const int32_t *v, size_t n, int32_t length);
int xo_encode_long_vector(xo_stream *s, const int64_t *v, size_t n);
int xo_encode_long_fixed_vector(xo_stream *s, const int64_t *v, size_t n, int32_t length);
int xo_encode_float_vector(xo_stream *s, const float *v, size_t n);
int xo_encode_float_fixed_vector(xo_stream *s, const float *v, size_t n, int32_t length);
int xo_encode_double_vector(xo_stream *s, const double *v, size_t n);
int xo_encode_double_fixed_vector(xo_stream *s, const double *v, size_t n, int32_t length);
int xo_encode_short_vector(xo_stream *s, const int16_t *v, size_t n);
int xo_encode_short_fixed_vector(xo_stream *s, const int16_t *v, size_t n, int32_t length);
int xo_encode_byte_vector(xo_stream *s, const int8_t *v, size_t n);
int xo_encode_byte_fixed_vector(xo_stream *s, const int8_t *v, size_t n, int32_t length);

/* decoders: return XDRG_OK / XDRG_E_SHORT / XDRG_E_CORRUPT.  Variable-length
 * results are returned as (pointer into the stream, length) views; *_vector
 * decoders write at most `cap` elements into `out` and report the count.     */
int xo_decode_int(xo_stream *s, int32_t *v);
int xo_decode_long(xo_stream *s, int64_t *v);
int xo_decode_float(xo_stream *s, float *v);
int xo_decode_double(xo_stream *s, double *v);
int xo_decode_boolean(xo_stream *s, int *v);
int xo_decode_byte(xo_stream *s, int8_t *v);
int xo_decode_short(xo_stream *s, int16_t *v);
int xo_decode_opaque(xo_stream *s, uint8_t *dst, size_t len);            /* fixed len  */
int xo_decode_dynamic_opaque(xo_stream *s, const uint8_t **p, size_t *len);
int xo_decode_string(xo_stream *s, const uint8_t **p, size_t *len);
int xo_decode_byte_buffer(xo_stream *s, const uint8_t **p, size_t *len);
int xo_decode_int_vector(xo_stream *s, int32_t *out, size_t cap, size_t *n);
int xo_decode_long_vector(xo_stream *s, int64_t *out, size_t cap, size_t *n);
int xo_decode_float_vector(xo_stream *s, float *out, size_t cap, size_t *n);
int xo_decode_double_vector(xo_stream *s, double *out, size_t cap, size_t *n);
int xo_decode_short_vector(xo_stream *s, int16_t *out, size_t cap, size_t *n);
int xo_decode_byte_vector(xo_stream *s, int8_t *out, size_t cap, size_t *n);

/* ---- record marking ---------------------------------------------------- */
/* GrizzlyRpcTransport.sendDefault (:103-110): BE(remaining | LAST_FRAG).   */
uint32_t xo_record_mark(uint32_t payload_len);
/* RpcMessageParserTCP.isAllFragmentsArrived (:63-99) on buf[0..len).       */
int  xo_all_fragments_arrived(const uint8_t *buf, size_t len);
/* RpcMessageParserTCP.assembleXdr (:109-140): consume one message starting
 * at buf, copy the concatenated fragment bodies into payload (capacity
 * payload_cap), return bytes consumed from buf in *consumed and the payload
 * length in *payload_len.  Precondition: xo_all_fragments_arrived.          */
int  xo_assemble(const uint8_t *buf, size_t len, uint8_t *payload, size_t payload_cap,
                 size_t *payload_len, size_t *consumed);
/* Host restatement of xdrg_frame_scan (see include/xdrg.h).                 */
int  xo_frame_scan(const uint8_t *buf, size_t len, uint64_t *msg_offsets, uint64_t cap,
                   uint64_t *n_msgs);
/* handleRead + the decode of each complete message as one record (the
 * contract of xdrg_receive_batch, include/xdrg.h; HOST pointers).           */
int  xo_receive_batch(const xdrg_field *fields, size_t nfields, const xdrg_cond *conds, size_t nconds,
                      const uint8_t *in, uint64_t len, uint64_t cap, xdrg_column *cols,
                      uint64_t *msg_offsets, uint64_t *n_msgs, uint64_t *consumed,
                      uint64_t *first_bad, int *err);
/* Split a payload into record-marked fragments of at most frag bytes each
 * (fixture generator restating ctest/rpc/RpcMessageParserTCPTest.java:161-181).
 * Returns bytes written into out (cap must be >= len + 4*(len/frag+1)).      */
size_t xo_fragment(const uint8_t *payload, size_t len, size_t frag, uint8_t *out, size_t cap);

/* ---- batch driver over the stream codec ---------------------------------- */
/* Same contract as xdrg_encode_batch / xdrg_decode_batch in include/xdrg.h,
 * with HOST pointers.  Each record is encoded into its own Xdr exactly as an
 * XdrAble would be (per-field calls in declaration order), and framed as
 * GrizzlyRpcTransport would frame the message.                              */
int xo_encode_batch(const xdrg_field *fields, size_t nfields, const xdrg_column *cols,
                    uint64_t n, uint8_t *out, uint64_t out_cap, uint64_t *rec_offsets,
                    uint32_t flags, uint64_t *out_len);
int xo_decode_batch(const xdrg_field *fields, size_t nfields, const uint8_t *in,
                    uint64_t in_len, const uint64_t *rec_offsets, uint64_t n,
                    xdrg_column *cols, uint32_t flags, uint64_t *first_bad, int *err);
/* Same, with conditional fields (include/xdrg.h xdrg_cond: rpcgen unions
 * and optional data, jrpcgen.java:1240-1340).                               */
int xo_encode_batch_cond(const xdrg_field *fields, size_t nfields, const xdrg_cond *conds,
                         size_t nconds, const xdrg_column *cols, uint64_t n, uint8_t *out,
                         uint64_t out_cap, uint64_t *rec_offsets, uint32_t flags,
                         uint64_t *out_len);
int xo_decode_batch_cond(const xdrg_field *fields, size_t nfields, const xdrg_cond *conds,
                         size_t nconds, const uint8_t *in, uint64_t in_len,
                         const uint64_t *rec_offsets, uint64_t n, xdrg_column *cols,
                         uint32_t flags, uint64_t *first_bad, int *err);
/* Zero-copy forms (include/xdrg.h
 * xdrg_encode_batch_shallow / xdrg_decode_batch_view): a payload field
 * encoded by reference (xdrEncodeFileChunk, Xdr.java:978-988, with
 * asBufferWritableMessages :579-597) and decoded as a stream slice
 * (xdrDecodeByteBuffer, :423-439).                                          */
int xo_encode_file_chunk(xo_stream *s, size_t len, uint32_t *padding);
int xo_encode_batch_shallow(const xdrg_field *fields, size_t nfields, const xdrg_cond *conds,
                            size_t nconds, const xdrg_column *cols, uint64_t n, uint8_t *out,
                            uint64_t out_cap, uint64_t *rec_offsets, uint32_t flags,
                            uint64_t *out_len, uint32_t field, uint64_t *splice);
int xo_decode_batch_view(const xdrg_field *fields, size_t nfields, const xdrg_cond *conds,
                         size_t nconds, const uint8_t *in, uint64_t in_len,
                         const uint64_t *rec_offsets, uint64_t n, xdrg_column *cols,
                         uint32_t flags, uint64_t *first_bad, int *err, uint32_t field,
                         uint64_t *view_pos);
/* Same, split over `threads` POSIX threads by contiguous record ranges (each
 * range encodes into its own slice; fixed-size schemas only for encode).  The
 * all-cores CPU baseline of SURVEY.md §8(d).                                  */
int xo_encode_batch_mt(const xdrg_field *fields, size_t nfields, const xdrg_column *cols,
                       uint64_t n, uint8_t *out, uint64_t out_cap, uint32_t flags,
                       uint64_t *out_len, int threads);
int xo_decode_batch_mt(const xdrg_field *fields, size_t nfields, const uint8_t *in,
                       uint64_t in_len, uint64_t n, xdrg_column *cols, uint32_t flags,
                       uint64_t *first_bad, int *err, int threads);

#ifdef __cplusplus
}
#endif
#endif
