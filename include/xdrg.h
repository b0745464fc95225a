/*
 * xdrg.h — C-ABI of the MI355X XDR batch engine (libxdrgpu.so).
 *
 * This is the drop-in boundary for the oncrpc4j XDR hot path.  Every entry
 * point below names the reference interface it replaces (paths are relative
 * to /root/reference/oncrpc4j-core/src/main/java/org/dcache/oncrpc4j/):
 *
 *   xdr/XdrEncodingStream.java:32-57   per-field encode surface  -> xdrg_encode_batch
 *   xdr/XdrDecodingStream.java:33-58   per-field decode surface  -> xdrg_decode_batch
 *   xdr/Xdr.java:39-1039               concrete codec semantics (bit-exact contract)
 *   grizzly/GrizzlyRpcTransport.java:97-110   record-mark prepend on send -> XDRG_FRAME_RM
 *   rpc/RpcMessageParserTCP.java:63-140       record-mark walk on receive -> xdrg_frame_scan
 *   rpc/RpcMessageParserTCP.java:44-61 + XdrAble.xdrDecode of each message
 *                                             (host socket buffer)   -> xdrg_receive_batch
 *
 * The reference is per-field and per-record (an XdrAble encodes its fields in
 * declaration order into one Xdr; xdr/XdrAble.java:40,49).  The engine works on
 * a BATCH of N records of one schema.  A schema is the field tape rpcgen emits
 * for a struct (oncrpc4j-rpcgen .../jrpcgen/jrpcgen.java:661-913): each field is
 * a base type (jrpcgen.java:608-618, plus enum/unsigned/opaque) with a
 * declaration kind (JrpcgenDeclaration.java:64-81: SCALAR, FIXEDVECTOR,
 * DYNAMICVECTOR).  Records live natively as columns (one per field, native
 * little-endian), the XDR side is one contiguous big-endian byte stream.
 *
 * Conventions
 *   - plain C types only; no C++ or torch types cross this boundary;
 *   - every call returns an int status (XDRG_OK or an XDRG_E_* code) and never
 *     throws; the Java/JNI side rethrows;
 *   - the caller owns every buffer; the engine keeps no pointer past return
 *     except its context's own device workspace;
 *   - a context is used by one thread at a time (mirrors Xdr's single-owner
 *     model, xdr/Xdr.java:56,71); use one context per worker thread;
 *   - all data pointers are DEVICE pointers (HBM) unless a call says otherwise
 *     or carries XDRG_HOST_PTRS (host memory through the staging ring).
 */
#ifndef XDRG_H
#define XDRG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define XDRG_ABI_VERSION 1

/* ---- status codes ------------------------------------------------------ */
/* Error parity with the reference (xdr/Xdr.java:1028-1037,
 * xdr/BadXdrOncRpcException.java:24):                                       */
#define XDRG_OK           0
#define XDRG_E_SHORT      1  /* BadXdrOncRpcException("xdr stream too short")  Xdr.java:1030 */
#define XDRG_E_CORRUPT    2  /* BadXdrOncRpcException("corrupted xdr")         Xdr.java:1036 */
#define XDRG_E_FIXED_LEN  3  /* IllegalArgumentException("array size does not match
                                protocol specification")                       Xdr.java:625-627 */
#define XDRG_E_CAPACITY   4  /* output buffer too small (the reference grows: Xdr.java:1020-1026) */
#define XDRG_E_FRAME      5  /* fixed-stride framed decode met a record mark that is not
                                (LAST | record size) — a multi-fragment or foreign record */
#define XDRG_E_INVAL      6  /* bad argument / unsupported schema */
#define XDRG_E_HIP        7  /* HIP runtime error (see xdrg_last_error) */
#define XDRG_E_NOMEM      8  /* allocation failed */
#define XDRG_E_INCOMPLETE 9  /* frame scan: not all fragments arrived -> NextAction STOP
                                (RpcMessageParserTCP.java:51-53) */
#define XDRG_E_NEG_SIZE   10 /* NegativeArraySizeException: a negative element count of an
                                array of structs, which jrpcgen decodes as
                                `new T[xdr.xdrDecodeInt()]` with no checkArraySize
                                (oncrpc4j-rpcgen .../jrpcgen/jrpcgen.java:886-906) */

/* ---- schema vocabulary (rpcgen) ------------------------------------------ */
/* Base types.  Native element sizes: INT/UINT/ENUM/FLOAT 4, HYPER/UHYPER/
 * DOUBLE 8, SHORT 2, BYTE/BOOL/OPAQUE/STRING 1.  XDR element sizes: 4 for
 * every scalar type (BYTE and SHORT are sign-extended to an XDR int,
 * Xdr.java:919-936; byte vectors use 4 bytes per element, Xdr.java:878-888),
 * 8 for HYPER/UHYPER/DOUBLE, and 1 byte + trailing zero pad to a multiple of
 * 4 for OPAQUE/STRING (Xdr.java:776-781).                                   */
#define XDRG_T_INT     1   /* xdrEncodeInt            Xdr.java:545  / xdrDecodeInt     :171 */
#define XDRG_T_UINT    2   /* rpcgen "unsigned int" -> int  (JrpcgenParser.cup:658)         */
#define XDRG_T_ENUM    3   /* enums are ints           (jrpcgen.java:688-695)                */
#define XDRG_T_BOOL    4   /* xdrEncodeBoolean         Xdr.java:803  / decode != 0     :404 */
#define XDRG_T_HYPER   5   /* xdrEncodeLong            Xdr.java:812  / xdrDecodeLong   :417 */
#define XDRG_T_UHYPER  6
#define XDRG_T_FLOAT   7   /* floatToIntBits (NaN canonical) Xdr.java:674 / raw bits :255 */
#define XDRG_T_DOUBLE  8   /* doubleToLongBits (NaN canonical) Xdr.java:685 / raw  :267 */
#define XDRG_T_SHORT   9   /* sign-extend / truncate   Xdr.java:934 / :497               */
#define XDRG_T_BYTE   10   /* sign-extend / truncate   Xdr.java:919 / :485               */
#define XDRG_T_OPAQUE 11   /* opaque x[N] / x<>        Xdr.java:776, :797 / :341, :374     */
#define XDRG_T_STRING 12   /* string s<> as UTF-8 bytes Xdr.java:760 / :392              */
#define XDRG_T_GROUP  13   /* a repeated group of member fields (array of structs / linked
                              list); see "Repeated groups" below                     */

/* Declaration kinds (JrpcgenDeclaration.java:64-81).                         */
#define XDRG_K_SCALAR  0   /* one element                                              */
#define XDRG_K_FIXED   1   /* T x[count]: count elements, no length word               */
#define XDRG_K_DYNAMIC 2   /* T x<count?>: 4-byte BE length word + elements (count = max,
                              0 = unbounded; the reference never enforces a max)       */
#define XDRG_K_LIST    3   /* XDRG_T_GROUP only: a recursive list `T *x` with
                              struct T { ...; T *next; }: BE(1) before every element,
                              BE(0) after the last (INDIRECTION, jrpcgen.java:835-851;
                              portmap/pmaplist.java:50-69, rpcb_list.java:55-78)     */

typedef struct xdrg_field {
    uint32_t type;      /* XDRG_T_* */
    uint32_t kind;      /* XDRG_K_* */
    uint32_t count;     /* FIXED: element count; DYNAMIC: max (0 = none); SCALAR: ignored */
    uint32_t reserved;  /* XDRG_T_GROUP: number of member fields that follow; else 0 */
} xdrg_field;

/* Repeated groups (arrays of structs, linked lists).  rpcgen encodes
 * `T x<>` / `T x[N]` for a struct T as a count word (dynamic only) and then
 * each element's fields (jrpcgen.java:856-906), and a recursive optional list
 * (struct T { ...; T *next; }, used as `T *x`) as BE(1) + element for every
 * element and a closing BE(0).  On the tape a group is one field
 * {XDRG_T_GROUP, kind FIXED / DYNAMIC / LIST, count, reserved = m} followed
 * by its m member fields (SCALAR, FIXED or DYNAMIC of the base types) or
 * inner groups (an array of structs / list inside the element,
 * jrpcgen.java:856-906 calling the inner elements' xdrEncode), recursively
 * up to four group levels in all; an outer m counts every inner group's
 * whole span.  A condition (xdrg_cond below) stays on its level: a top-level
 * field (the group field included) on a top-level discriminant, a member (an
 * inner group included) on an earlier member of its own group, evaluated per
 * element.  Columns: the group's own column has offsets[rows + 1] (DYNAMIC /
 * LIST: row i owns elements [offsets[i], offsets[i+1]); FIXED: element
 * i*count + j, offsets unused) where rows are the records (top level) or the
 * outer group's elements (an inner group), and, on decode, cap = element
 * capacity; data is unused.  A member's column is indexed by ELEMENT of its
 * own group: fixed members at data + e*stride, dynamic members own
 * [offsets[e], offsets[e+1]) (offsets has elements + 1 entries).  Decode
 * errors keep the reference's order: the count / list bools / member checks
 * as the element loops meet them; a negative count is XDRG_E_NEG_SIZE.
 * A deeper inner group's column is indexed by the elements of the group
 * that holds it, the same way.  XDRG_HOST_PTRS staging moves every level's
 * element rows with their records; only a FIXED (T x[N]) group inside a
 * DYNAMIC / LIST group's elements goes through device scratch whole (the
 * spans the call touches copied in and back, overlapping spans merged).    */

/* One native column.  Fixed-size fields (SCALAR / FIXED): record i's first
 * element is at  data + i*stride  (stride 0 = packed = elem_size*count), so
 * both struct-of-arrays (stride = element bytes) and array-of-structs
 * (data = &recs[0].field, stride = sizeof(rec)) describe the same batch.
 * DYNAMIC fields: record i owns elements [offsets[i], offsets[i+1]) of data
 * (element units: bytes for OPAQUE/STRING).  On decode the engine writes
 * offsets[0..n] (offsets[0] = 0) and needs cap >= total elements.           */
typedef struct xdrg_column {
    void     *data;
    int64_t   stride;
    uint64_t *offsets;
    uint64_t  cap;
} xdrg_column;

/* Encode only: a SCALAR / FIXED column whose records all read the element
 * run at `data` — a constant field such as the msg_type, reply_stat,
 * verifier and accept_stat words every accepted reply carries
 * (rpc/RpcCall.java:328-332) or a call's rpcvers/prog/vers
 * (RpcCall.java:462-467).  Decode rejects it with XDRG_E_INVAL.            */
#define XDRG_STRIDE_CONST INT64_MIN

/* ---- flags --------------------------------------------------------------- */
/* Prepend one RFC 1831 record mark per record: BE(len | 0x80000000), one
 * last fragment per message (GrizzlyRpcTransport.java:103-110,
 * RpcMessageParserTCP.java:37-41, docs/rfc1831.txt:696-705).  On decode the
 * engine expects and strips one mark per record.                             */
#define XDRG_FRAME_RM      0x1u
/* out_len / first_bad / err are DEVICE pointers; the call does not
 * synchronise the stream (graph-capturable).                                  */
#define XDRG_ASYNC         0x2u
/* Host memory (SURVEY.md §8b HOST_PTRS): every pointer of an
 * xdrg_encode_batch / xdrg_decode_batch call — column data and offsets, the
 * stream, rec_offsets, out_len / first_bad / err — is a HOST pointer, as the
 * reference's Xdr works on a host Grizzly buffer (xdr/Xdr.java:115-119,
 * grizzly/GrizzlyMemoryManager.java:42-57) and sends from it
 * (grizzly/GrizzlyRpcTransport.java:97-112).  The batch moves through the
 * context's staging ring (xdrg_ctx_host_staging) in record chunks:
 * H2D / kernels / D2H of consecutive chunks overlap on the context's own
 * copy and compute streams; spans that are not pinned (xdrg_host_register,
 * hipHostMalloc) pass through the ring's pinned bounce buffers.  The call
 * is synchronous (XDRG_ASYNC is refused).  Results are those of the device
 * call on the same records, except that a variable-size encode that
 * overruns out_cap may have written the records before the overrun.
 * Repeated groups: a chunk of records moves its elements' member rows with
 * it (rows between the group offsets of its first and last record).        */
#define XDRG_HOST_PTRS     0x4u
/* With XDRG_HOST_PTRS: no staging — the kernels read and write the host
 * buffers in place over PCIe.  Every buffer must be registered
 * (xdrg_host_register) or allocated pinned (hipHostMalloc); a variable-size
 * decode then reads the stream twice over the link (sizes, then place).     */
#define XDRG_HOST_MAPPED   0x8u

/* ---- opaque handles ------------------------------------------------------- */
typedef struct xdrg_ctx    xdrg_ctx;
typedef struct xdrg_schema xdrg_schema;

/* ---- version / diagnostics ------------------------------------------------ */
int         xdrg_abi_version(void);
const char *xdrg_status_string(int status);   /* reference exception message */
const char *xdrg_last_error(xdrg_ctx *ctx);   /* last HIP / argument detail   */

/* ---- context -------------------------------------------------------------- */
/* A context binds one device and one stream and owns scratch workspace.
 * Replaces the per-call `new Xdr(...)` buffer ownership of the reference
 * (Xdr.java:82-119, RpcCall.java:460).                                        */
#define XDRG_CTX_TIMING 0x1u    /* record HIP events around every kernel launch */
int  xdrg_ctx_create(int device, uint32_t flags, xdrg_ctx **out);
int  xdrg_ctx_destroy(xdrg_ctx *ctx);
/* stream is a hipStream_t (NULL = the default stream). */
int  xdrg_ctx_set_stream(xdrg_ctx *ctx, void *stream);
/* Per-kernel launch statistics (only with XDRG_CTX_TIMING): kernel ids below. */
#define XDRG_KERNEL_FIXED_ENCODE 0
#define XDRG_KERNEL_FIXED_DECODE 1
#define XDRG_KERNEL_VAR_SIZE     2
#define XDRG_KERNEL_VAR_SCAN     3
#define XDRG_KERNEL_VAR_ENCODE   4
#define XDRG_KERNEL_VAR_DECODE   5
#define XDRG_KERNEL_FRAME_SCAN   6
#define XDRG_KERNEL_COUNT        7
int  xdrg_ctx_kernel_stats(xdrg_ctx *ctx, int kernel, uint64_t *launches, double *total_ms);
int  xdrg_ctx_reset_stats(xdrg_ctx *ctx);

/* Staging ring of the XDRG_HOST_PTRS calls: `slots` (1..8) device slots of
 * `slot_bytes` each, plus a pinned bounce mirror allocated on first use by
 * a span that is not pinned.  Default 4 x 64 MiB.  A chunk is as many
 * records as fit one slot (inputs, outputs and offsets together); a record
 * larger than a slot grows the ring.  Takes effect at the next host call.  */
int  xdrg_ctx_host_staging(xdrg_ctx *ctx, uint64_t slot_bytes, uint32_t slots);
/* Pin a caller buffer for the DMA engines and map it for the kernels
 * (hipHostRegister): the reference's direct / pooled Grizzly buffers
 * (rpc/MemoryAllocator, grizzly/GrizzlyUtils.java:140-156) registered once
 * and reused.  Registered spans skip the bounce copy and may take
 * XDRG_HOST_MAPPED.  ctx may be NULL (current device).                      */
int  xdrg_host_register(xdrg_ctx *ctx, void *ptr, uint64_t bytes);
int  xdrg_host_unregister(xdrg_ctx *ctx, void *ptr);

/* Device buffers for a caller with no device allocator of its own (a JVM):
 * the HBM counterpart of GrizzlyMemoryManager.allocate / wrap
 * (grizzly/GrizzlyMemoryManager.java:42-57).  The pointers these return are
 * what the device forms of every call take (no flags; the multi-GPU calls;
 * XDRG_ASYNC result words).  xdrg_device_alloc: `bytes` on the context's
 * device (256-byte aligned; 0 bytes gives a valid 256-byte buffer).
 * xdrg_copy: `bytes` from src to dst on the context's stream, then a
 * synchronise; kind says which side is which.  A host side may be any host
 * memory (pinned or registered spans move at DMA speed).                    */
#define XDRG_COPY_H2D 1
#define XDRG_COPY_D2H 2
#define XDRG_COPY_D2D 3
int  xdrg_device_alloc(xdrg_ctx *ctx, uint64_t bytes, void **out);
int  xdrg_device_free(xdrg_ctx *ctx, void *ptr);
int  xdrg_copy(xdrg_ctx *ctx, void *dst, const void *src, uint64_t bytes, int kind);

/* ---- schema ----------------------------------------------------------------- */
/* Compile a field tape (rpcgen struct body, jrpcgen.java:758-913) into an
 * engine schema.  Host-side object; may be shared by contexts.                 */
int  xdrg_schema_create(const xdrg_field *fields, size_t nfields, xdrg_schema **out);
int  xdrg_schema_destroy(xdrg_schema *schema);

/* Conditional fields: rpcgen unions and optional data, whose records of one
 * type differ in shape.  A union (jrpcgen.java:1240-1340) encodes its
 * discriminant and then the one arm whose case list holds the value (or the
 * default arm, or nothing); optional data `T *x` (JrpcgenDeclaration
 * INDIRECTION) encodes a bool and then T only when it is true.  Both flatten
 * to one tape in which some fields carry a condition on an earlier
 * discriminant field:
 *   field k is present  iff  field `disc` is present  and
 *                            (value(disc) in values[0..nvalues))  !=  negate
 * value(disc) is the int / unsigned / enum as an int32, a bool as 0 or 1
 * (decode: any non-zero word is true, Xdr.java:404-407).  Nested unions /
 * optionals chain: an absent discriminant makes its dependants absent.
 * Encode writes nothing for an absent field (its native slot is ignored);
 * decode writes zero into an absent fixed field's native slot and an empty
 * run (offsets[i+1] == offsets[i]) for an absent dynamic field — the
 * defaults of a freshly constructed rpcgen object.  A schema with any
 * condition is variable-size (xdrg_schema_fixed_size() == 0).  At most
 * XDRG_MAX_DISC distinct discriminant fields and XDRG_MAX_CASES case values
 * per schema.                                                                 */
#define XDRG_MAX_DISC  8
#define XDRG_MAX_CASES 64
typedef struct xdrg_cond {
    uint32_t field;          /* the conditional field (index into fields)                 */
    uint32_t disc;           /* its discriminant: an earlier SCALAR INT/UINT/ENUM/BOOL field */
    uint32_t negate;         /* 0: case arm (value in list); 1: default arm / optional (not in) */
    uint32_t nvalues;
    const int32_t *values;   /* host pointer, copied at schema creation                   */
} xdrg_cond;
int  xdrg_schema_create_cond(const xdrg_field *fields, size_t nfields, const xdrg_cond *conds,
                             size_t nconds, xdrg_schema **out);
/* XDR bytes of one record when every field is fixed-size (no DYNAMIC field),
 * excluding any record mark; 0 for variable-size schemas.                      */
uint64_t xdrg_schema_fixed_size(const xdrg_schema *schema);

/* ---- encode ------------------------------------------------------------------ */
/* Encode n records into one contiguous XDR stream `out` (capacity out_cap
 * bytes).  The stream is the concatenation of every record's encoding in
 * record order, each record the concatenation of its fields' encodings in
 * declaration order (XdrAble.xdrEncode via rpcgen codingMethod), prefixed per
 * record by a record mark when XDRG_FRAME_RM is set.  rec_offsets (n+1
 * entries, nullable) receives the byte offset of each record (of its mark
 * when framed) and the total.  *out_len receives the total byte count.
 * Pad bytes are written as zeros (RFC 4506; Xdr.java:765-781).
 * Returns XDRG_E_CAPACITY (and writes nothing) if out_cap is too small.     */
int  xdrg_encode_batch(xdrg_ctx *ctx, const xdrg_schema *schema,
                       const xdrg_column *cols, uint64_t n,
                       uint8_t *out, uint64_t out_cap,
                       uint64_t *rec_offsets, uint32_t flags,
                       uint64_t *out_len);

/* ---- decode ------------------------------------------------------------------ */
/* Decode n records from `in` (in_len bytes) into native columns.
 * rec_offsets (n+1 entries): record i occupies [rec_offsets[i],
 * rec_offsets[i+1]) (its mark first when XDRG_FRAME_RM); NULL is allowed for
 * fixed-size schemas (records back to back at the fixed stride).  Records
 * are decoded independently with the reference's check order
 * (Xdr.java:171-531, 1028-1037); trailing bytes inside a record's extent are
 * ignored as RpcCall.retrieveCall does (RpcCall.java:351-354).  On error the
 * status is returned, *first_bad = the smallest failing record index and
 * *err = its code — what a sequential reference decode would throw first.
 * Columns of records before first_bad hold their decoded values.           */
int  xdrg_decode_batch(xdrg_ctx *ctx, const xdrg_schema *schema,
                       const uint8_t *in, uint64_t in_len,
                       const uint64_t *rec_offsets, uint64_t n,
                       xdrg_column *cols, uint32_t flags,
                       uint64_t *first_bad, int *err);

/* ---- zero-copy payloads -------------------------------------
 * Send side — xdrEncodeFileChunk (xdr/Xdr.java:978-988) and
 * xdrEncodeShallowByteBuffer (:839-866): the payload of one dynamic
 * OPAQUE/STRING field per record is encoded BY REFERENCE.  The device writes
 * every other byte of each message (the length word included) into `out`;
 * the payload and its zero padding stay where they are and go out as their
 * own writable messages, as asBufferWritableMessages (:579-597) and
 * GrizzlyRpcTransport.sendRawTCP (grizzly/GrizzlyRpcTransport.java:130-168)
 * do.  Message i on the wire is
 *     out[rec_offsets[i], splice[i])  payload(i)  zero pad(len_i)  out[splice[i], rec_offsets[i+1])
 * with len_i = offsets[i+1] - offsets[i] of the field's column, pad =
 * (4 - (len & 3)) & 3.  splice[i] = UINT64_MAX when the field is absent
 * (conditional schemas): the message is out[rec_offsets[i], rec_offsets[i+1]).
 * The field column's `data` is never dereferenced (it may be a host
 * buffer, a file mapping or NULL).
 * With XDRG_FRAME_RM each mark counts every part (sendRawTCP :135-139,
 * getMessagesSize :224-231).  splice: an array of n entries.
 * Memory: device pointers (flags 0, XDRG_ASYNC); or, as for
 * xdrg_encode_batch, XDRG_HOST_PTRS — every other column, out, rec_offsets,
 * splice and out_len host memory moved through the staging ring, the payload
 * column's values never read nor staged (only the heads cross PCIe: the
 * Grizzly buffer a sender writes around the payload, Xdr.java:582-597) — or
 * XDRG_HOST_PTRS | XDRG_HOST_MAPPED (registered host memory in place).     */
int  xdrg_encode_batch_shallow(xdrg_ctx *ctx, const xdrg_schema *schema,
                               const xdrg_column *cols, uint64_t n,
                               uint8_t *out, uint64_t out_cap,
                               uint64_t *rec_offsets, uint32_t flags, uint64_t *out_len,
                               uint32_t field, uint64_t *splice);

/* Receive side — xdrDecodeByteBuffer (xdr/Xdr.java:423-439): the payload of
 * one dynamic OPAQUE/STRING field per record is returned as a slice of the
 * stream instead of a copy.  payload_pos[i] (device, n entries) = offset in
 * `in` of record i's payload (UINT64_MAX if absent); the column's offsets
 * are written as for a copy (len_i = offsets[i+1] - offsets[i]); its data
 * and cap are ignored.  Checks and error parity as xdrg_decode_batch.
 * Memory as xdrg_decode_batch: device pointers, XDRG_HOST_PTRS (the stream
 * staged, payload_pos and the columns returned to host memory: the slices
 * then point into the caller's own host buffer, as Xdr's do), or
 * XDRG_HOST_PTRS | XDRG_HOST_MAPPED.  Any other flag bit, on this and every
 * codec call, is XDRG_E_INVAL.                                              */
int  xdrg_decode_batch_view(xdrg_ctx *ctx, const xdrg_schema *schema,
                            const uint8_t *in, uint64_t in_len,
                            const uint64_t *rec_offsets, uint64_t n,
                            xdrg_column *cols, uint32_t flags,
                            uint64_t *first_bad, int *err,
                            uint32_t field, uint64_t *payload_pos);

/* ---- framing (receive side) ----------------------------------------------------- */
/* Walk the record marks of a TCP byte stream (RpcMessageParserTCP.java:63-99):
 * writes msg_offsets[k] = offset of message k's first mark for every complete
 * message (all fragments present), msg_offsets[*n_msgs] = offset just past the
 * last complete message (the "reminder" split point, :57-58).  Returns
 * XDRG_OK, or XDRG_E_INCOMPLETE when no complete message is present (STOP).
 * `in` is a device pointer; msg_offsets is a device array of cap+1 entries;
 * *n_msgs is a host pointer.                                                     */
int  xdrg_frame_scan(xdrg_ctx *ctx, const uint8_t *in, uint64_t len,
                     uint64_t *msg_offsets, uint64_t cap, uint64_t *n_msgs);

/* Deframe a received TCP byte stream: RpcMessageParserTCP.handleRead for a
 * whole socket-buffer batch (isAllFragmentsArrived :63-99 and assembleXdr
 * :109-140, repeated while complete messages remain).  The fragment bodies
 * of each complete message (at most cap) are concatenated, marks stripped,
 * into `payload` (device, payload_cap bytes) back to back; message i is
 * payload[msg_offsets[i], msg_offsets[i+1]) (device, cap + 1 entries).
 * *n_msgs (host) = messages delivered; *consumed (host) = stream bytes they
 * occupied — the remainder starts there (handleRead's split, :57-60).
 * Returns XDRG_OK, XDRG_E_INCOMPLETE (no complete message: STOP), or
 * XDRG_E_CAPACITY (payload_cap too small; *consumed = bytes needed).  The
 * messages then decode from payload + msg_offsets without XDRG_FRAME_RM.
 * xdrg_frame_scan is the zero-copy form: stream offsets of each message's
 * first mark (single-fragment messages decode in place with XDRG_FRAME_RM).
 * Both walk the marks in parallel (list ranking over 4-byte positions); a
 * stream whose chain meets a fragment size that is not a multiple of 4 is
 * walked serially, with the same result.                                    */
int  xdrg_deframe(xdrg_ctx *ctx, const uint8_t *in, uint64_t len, uint8_t *payload,
                  uint64_t payload_cap, uint64_t *msg_offsets, uint64_t cap, uint64_t *n_msgs,
                  uint64_t *consumed);

/* ---- receive on host socket buffers --------------------
 * The reference walks the marks of the host Grizzly Buffer its selector thread
 * filled (rpc/RpcMessageParserTCP.java:44-61: isAllFragmentsArrived :63-99,
 * assembleXdr :109-140, the remainder split :57-60) and hands each complete
 * message to the next filter, whose XdrAble.xdrDecode reads it
 * (rpc/RpcCall.java:351-354 leaves trailing bytes unread).  These calls take
 * that buffer where it lives:
 *   flags 0                                  device pointers (HBM);
 *   XDRG_HOST_PTRS                           host memory moved through the context's
 *                                            staging ring in windows: each window is
 *                                            walked and decoded on the device, and the
 *                                            next starts at the first byte not consumed
 *                                            (its tail copied device to device), so each
 *                                            stream byte crosses PCIe once;
 *   XDRG_HOST_PTRS | XDRG_HOST_MAPPED        registered host memory (xdrg_host_register)
 *                                            read and written in place over PCIe.
 * Every pointer of the call follows the flags (n_msgs, consumed, first_bad and
 * err are always host pointers).  The calls are synchronous.
 *
 * xdrg_frame_scan_ex / xdrg_deframe_ex: xdrg_frame_scan / xdrg_deframe with
 * those flags and *consumed (the remainder starts there).  On host memory a
 * deframe delivers the messages whose bodies fit payload_cap and returns
 * XDRG_E_CAPACITY when a complete message was left for lack of room (the
 * device form returns XDRG_E_CAPACITY with *consumed = the bytes needed and
 * delivers nothing).
 *
 * xdrg_receive_batch: the walk, then every complete message (at most cap)
 * decoded as one record of `schema` into cols (xdrg_decode_batch's column
 * contract; rows = messages, fixed columns hold cap rows): a single-fragment
 * message decodes in place with its mark checked (XDRG_FRAME_RM), a
 * multi-fragment one from its assembled body.  *n_msgs = messages delivered,
 * *consumed = stream bytes they occupy, msg_offsets (nullable, cap + 1
 * entries) = each delivered message's first mark and *consumed.  Returns
 * XDRG_OK, XDRG_E_INCOMPLETE (no complete message: STOP), or the first
 * message's decode error: *first_bad = its index, *err = its code, columns
 * hold the messages before it, and the call has delivered through it
 * (*n_msgs = first_bad + 1, *consumed = its end: RpcDispatcher answers such a
 * call GARBAGE_ARGS, RpcDispatcher.java:126-131, and the caller resumes at
 * *consumed) — except XDRG_E_CAPACITY, which delivers up to it (*n_msgs =
 * first_bad) so the caller can retry it with larger columns.  Host staging
 * streams every schema through the staging windows in one crossing, a
 * window's group element rows (every level) placed by the previous window's
 * totals — except a schema with a FIXED (T x[N]) group inside a DYNAMIC /
 * LIST group's elements, or with group elements of no XDR bytes, which is
 * walked, deframed and then decoded (three staged passes; same results).   */
int  xdrg_frame_scan_ex(xdrg_ctx *ctx, const uint8_t *in, uint64_t len, uint64_t *msg_offsets,
                        uint64_t cap, uint64_t *n_msgs, uint64_t *consumed, uint32_t flags);
int  xdrg_deframe_ex(xdrg_ctx *ctx, const uint8_t *in, uint64_t len, uint8_t *payload,
                     uint64_t payload_cap, uint64_t *msg_offsets, uint64_t cap, uint64_t *n_msgs,
                     uint64_t *consumed, uint32_t flags);
int  xdrg_receive_batch(xdrg_ctx *ctx, const xdrg_schema *schema, const uint8_t *in, uint64_t len,
                        uint64_t cap, xdrg_column *cols, uint32_t flags, uint64_t *msg_offsets,
                        uint64_t *n_msgs, uint64_t *consumed, uint64_t *first_bad, int *err);

/* ---- multi-GPU, one process ---------------------------
 * For a caller that drives several devices from one process (a JVM with one
 * context per GPU).  Records are independent (xdr/XdrAble.java:40,49), so a
 * batch shards into consecutive record ranges, context i owning counts[i]
 * records in context order (first_i = counts[0] + ... + counts[i-1]).  At
 * most 8 contexts; contexts may share a device.  Both calls synchronise.
 *
 * Encode: context i encodes its shard from its own device columns cols[i]
 * straight into out[i] (device of context i, out_cap bytes) at the shard's
 * stream offset, then every context pulls its peers' shards out of their
 * HBM over xGMI (peer access is enabled on first use).  On return every
 * out[i] holds the whole stream — byte-identical to one context encoding
 * all records — and rec_offsets[i] (nullable; n_total + 1 entries) its
 * record offsets.  *out_len (host) = stream bytes.
 *
 * Decode: context i decodes records [first_i, first_i + counts[i]) of the
 * stream in[i] resident on its device (in_len bytes; rec_offsets[i] = the
 * stream's n_total + 1 record offsets, or NULL for fixed-size schemas) into
 * its shard's columns cols[i].  *first_bad / *err (host) = the reference's
 * first error over the whole batch: the smallest failing record.
 *
 * Any schema shards, repeated groups and conditional members included: a
 * shard's columns are the columns one context would hold for its records
 * alone (group element rows and member offsets counted from the shard's
 * first record), as xdrg_encode_batch / xdrg_decode_batch take them.      */
int  xdrg_encode_batch_multi(xdrg_ctx *const *ctxs, uint32_t nctx, const xdrg_schema *schema,
                             const xdrg_column *const *cols, const uint64_t *counts,
                             uint8_t *const *out, uint64_t out_cap, uint64_t *const *rec_offsets,
                             uint32_t flags, uint64_t *out_len);
int  xdrg_decode_batch_multi(xdrg_ctx *const *ctxs, uint32_t nctx, const xdrg_schema *schema,
                             const uint8_t *const *in, uint64_t in_len,
                             const uint64_t *const *rec_offsets, const uint64_t *counts,
                             xdrg_column *const *cols, uint32_t flags,
                             uint64_t *first_bad, int *err);

#ifdef __cplusplus
}
#endif
#endif /* XDRG_H */
