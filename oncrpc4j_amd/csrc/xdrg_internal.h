// xdrg_internal.h — shared definitions of the MI355X XDR batch engine
// (libxdrgpu.so).  Host and device code include this; nothing here crosses
// the C-ABI (include/xdrg.h is the boundary).
//
// Reference semantics restated here (paths under /root/reference/
// oncrpc4j-core/src/main/java/org/dcache/oncrpc4j/):
//   xdr/Xdr.java:545-548 / :171-175   int  <-> 4 bytes big-endian
//   xdr/Xdr.java:812-815 / :417-420   long <-> 8 bytes BE, high word first
//   xdr/Xdr.java:674-687              float/double via floatToIntBits /
//                                     doubleToLongBits (every NaN canonical)
//   xdr/Xdr.java:803-805 / :404-407   boolean 1/0, decode any non-zero = true
//   xdr/Xdr.java:919-936 / :485-499   byte/short sign-extended / truncated
//   xdr/Xdr.java:776-781 / :341-349   opaque bytes + zero pad to 4
//   grizzly/GrizzlyRpcTransport.java:103-110  record mark BE(len | LAST)
#pragma once

#include <stddef.h>
#include <stdint.h>

#include "../../include/xdrg.h"

namespace xdrg {

// ---- limits of the kernel-argument descriptors --------------------------
constexpr int kMaxWords  = 128;  // XDR words per record on the word-map path
constexpr int kMaxCols   = 32;   // fields per schema on the word-map path
constexpr int kMaxFields = 32;   // fields per schema on the record path

constexpr uint32_t kLastFrag = 0x80000000u;  // RpcMessageParserTCP.java:37
constexpr uint32_t kSizeMask = 0x7fffffffu;  // RpcMessageParserTCP.java:41

// ---- one XDR word of a fixed-size record --------------------------------
// Every fixed-size XDR record is a sequence of 4-byte words (RFC 4506 §3);
// each word is produced (encode) or consumed (decode) by one WordOp that
// names the native column, the byte offset inside that record's native
// element run, and the conversion.
enum WordOpKind : uint8_t {
    OP_BSWAP = 0,     // int/uint/enum: u32 native <-> BE word
    OP_FLOAT = 1,     // float: encode canonicalises NaN (Xdr.java:674-676)
    OP_HYPER_HI = 2,  // long high word: native bytes [off+4, off+8)
    OP_HYPER_LO = 3,  // long low word:  native bytes [off,   off+4)
    OP_DOUBLE_HI = 4, // double: as HYPER, encode canonicalises NaN (:685-687)
    OP_DOUBLE_LO = 5,
    OP_BOOL = 6,      // native u8: encode 0/1, decode != 0 (:803, :404)
    OP_SHORT = 7,     // native i16: sign-extend / truncate (:934, :497)
    OP_BYTE = 8,      // native i8 : sign-extend / truncate (:919, :485)
    OP_OPAQUE = 9,    // aux = 1..4 payload bytes copied raw, rest zero pad
    OP_MARK = 10,     // record mark (encode: write, decode: check)
};

struct WordOp {
    uint8_t op;
    uint8_t col;   // field index
    uint8_t aux;   // OP_OPAQUE: payload bytes in this word
    uint8_t rsv;
    uint32_t off;  // byte offset inside the record's native element run
};

// Word-map kernel arguments (passed by value; < 2 KiB of kernarg).
struct WordMapArgs {
    uint64_t n;                  // records
    uint32_t wt;                 // XDR words per record (incl. mark when framed)
    uint32_t mark_le;            // record mark as it sits in memory (BE bytes)
    uint64_t dr;                 // grid-stride advance of the record index ...
    uint32_t dw;                 // ... and of the word index (per 4*stride words)
    uint32_t nops;               // == wt
    uint8_t *xdr;                // XDR stream
    uint64_t xdr_len;            // decode: valid input bytes
    unsigned long long *errkey;  // decode: min error key
    uint8_t *base[kMaxCols];     // native column bases
    int64_t stride[kMaxCols];    // native column strides (bytes per record)
    WordOp ops[kMaxWords];
};

// Streaming (register) kernel arguments: AoS-dense records whose native
// layout is word-for-word the XDR layout.
struct StreamArgs {
    const uint8_t *src;
    uint8_t *dst;
    uint64_t nvec;        // 16-byte vectors
    uint32_t w;           // words per record
    uint32_t all_bswap;   // 1: every word is a plain byte swap
    uint8_t ops[kMaxWords];  // per record word: OP_BSWAP/FLOAT/HYPER_*/DOUBLE_*/OPAQUE
};

// ---- record path (variable-size schemas) --------------------------------
// Every member is 32 or 64 bits wide: the record kernels read these
// descriptors with scalar (SMEM) loads at uniform field indices, and a
// byte-wide member lets the compiler form a misaligned SMEM base whose low
// address bits the scalar unit drops (observed on gfx950: a dword load at
// base 0x81 + 7 returned the dword at 0x84).
struct VField {
    uint32_t type;    // XDRG_T_*
    uint32_t kind;    // XDRG_K_*
    uint32_t nsz;     // native element bytes
    uint32_t xsz;     // XDR element bytes (1 for opaque/string)
    uint32_t count;   // FIXED count
    uint32_t xbytes;  // fixed fields: XDR bytes of the field (incl. pad)
    uint8_t *data;
    int64_t stride;
    uint64_t *offsets;
    uint64_t cap;
    // conditional fields (xdrg_cond): present iff field cond-1 is present and
    // its value is (cneg = 0) / is not (cneg = 1) in cvals[cfirst, cfirst + cnum)
    uint32_t cond;    // 0 = unconditional, else discriminant field index + 1
    uint32_t cneg;
    uint32_t cfirst;
    uint32_t cnum;
    uint32_t slot;    // 0, or 1 + this field's discriminant value slot
    uint32_t rsv;
};

// One fixed XDR word of a record: field data + r * stride + off, converted
// as enc_elem(type, ., half) (XDRG_T_OPAQUE: load_bytes of min(rem, 4)).
constexpr int kPayWords = 16;
struct PayWord {
    const uint8_t *data;
    int64_t stride;
    uint32_t type;
    uint16_t off;
    uint8_t half, rem;
};
struct RecArgs {
    uint64_t n;
    uint32_t nf;
    uint32_t framed;
    uint32_t fixed_xdr;        // XDR bytes of all fixed fields (plus mark)
    uint32_t ndyn;
    uint8_t *xdr;
    uint64_t xdr_cap;          // encode: out_cap; decode: in_len
    const uint64_t *rec_in;    // decode: record extents (n+1), or NULL (fixed stride)
    uint64_t rec_stride;       // decode with rec_in == NULL
    uint64_t *rec_out;         // encode: record offsets (n+1), nullable
    uint64_t *block_sums;      // workspace [ndyn+1][nblocks]
    uint64_t nblocks;
    uint64_t *totals;          // workspace [ndyn+1]: scanned totals
    unsigned long long *errkey;
    uint32_t *rec_cnt;         // decode workspace [ndyn][n]: element count per record
    uint32_t force_g;          // 0 = group size from the average field size, else lanes per record
    uint32_t lane_bytes_enc;   // group sizing: target XDR bytes per lane (encode / decode)
    uint32_t lane_bytes_dec;
    uint32_t tile_bytes;       // staged place kernels: LDS tile per sub-batch
    uint32_t big_rec;          // blocks averaging >= big_rec XDR bytes per record take the group
                               // kernels, the others the staged ones (0: one kernel for all)
    uint32_t ncond;            // conditional fields in the schema (0: every record has all fields)
    uint32_t byref;            // 0, or 1 + the field encoded by reference / decoded as a view
    uint32_t xcd;              // payload kernels: blocks in XCD order (xcd_block)
    uint64_t *ref_pos;         // byref: encode splice[n] / decode payload_pos[n]
    uint32_t payk;             // 0, or 1 + the dynamic byte field the payload kernels move for the
                               // group kernels' blocks (k_enc/dec_payload)
    uint32_t pay_fb;           // payk: XDR bytes before that field in a record (mark + fixed fields)
    uint64_t *pay_pos;         // payk: per record, stream offset of that field's length word
                               // (decode: ~0 = not to be written)
    uint32_t *spec;            // decode, extent-derived counts (spec_mode != 0): ~0 = the derived
                               // counts hold so far, 0 = a kernel found they do not (exact rerun)
    uint32_t spec_mode;        // 0 off; 1 the derived-count pass (sizes, place verifying the count
                               // words); 2 the exact rerun (its kernels return unless *spec == 0);
                               // 3 the derived counts in one pass (k_dec_sweep walks and looks back)
    unsigned long long *lb_ticket;   // spec_mode 3: block tickets in start order (starts at ~0)
    uint32_t dyn_idx[kMaxFields]; // dynamic field -> field index
    VField f[kMaxFields];
    int32_t cvals[XDRG_MAX_CASES];  // case values of the conditional fields
    // the fixed XDR words of a record (mark excluded, in stream order, the
    // dynamic field skipped) as direct element rules, so k_enc_payload's head
    // and tail words need no walk over the fields (pay_nw = 0: schemas with
    // more words or conditional fields walk them)
    uint32_t pay_nw;
    PayWord pw[kPayWords];
};
static_assert(sizeof(RecArgs) <= 4096, "RecArgs must fit the kernel-argument segment");

// Error key: smaller = what a sequential reference decode throws first.
//   key = record << 16 | sub << 4 | code
// sub orders the checks inside a record (word index on the word-map path;
// 2*field+1 / 2*field+2 on the record path, 0 for the record mark).
__host__ __device__ inline unsigned long long err_key(uint64_t rec, uint32_t sub, uint32_t code) {
    return ((unsigned long long)rec << 16) | ((unsigned long long)(sub & 0xfffu) << 4) |
           (code & 0xfu);
}
constexpr unsigned long long kNoError = ~0ull;

// ---- per-context kernel choices -----------------------------------------
// Every value selects among production kernels (each of which some input
// takes anyway) or sizes one; the defaults are the measured winners
// (DESIGN.md §5).  A context owns its own copy (one context per thread), set
// through xdrg_internal_tune() — not part of include/xdrg.h; the parity tests
// force each path and tools/sweep_rec.py sweeps the sizes.
struct Tuning {
    int32_t words = 2;              // key 16: fixed 4-byte-word schemas: 2 LDS-staged, 1 lane per record, 0 word-map
    int32_t framed = 2;             // key 14: record-marked AoS decode: 2 lean, 1 wave-LDS transpose
    int32_t rec = 4;                // key 9: record path: 4 staged sub-batches (large-record blocks on the
                                    // group kernels), 0 group kernels for every block
    int32_t dec_lean = 2;           // key 20: staged decode of <= 2 dynamic fields: 2 the output-stationary
                                    // sweep (k_dec_sweep), 1 record groups writing whole boundary dwords
                                    // (k_dec_stage, the kernel of 3-4 dynamic fields)
    uint32_t force_g = 0;           // key 6: lanes per record (0 = sized from the field)
    uint32_t lane_bytes_enc = 64;   // keys 7/8: group sizing, XDR bytes per lane (encode 64: the
                                    // record-major staged encode's 4 lanes per config-4 record)
    uint32_t lane_bytes_dec = 32;
    uint32_t tile_bytes = 16384;    // key 12: staged kernels, LDS tile per sub-batch
    uint32_t sweep_tile = 21504;    // key 25: the sweep decode's LDS tile (k_dec_sweep, 4 blocks per CU)
    uint32_t big_rec = 1024;        // key 13: blocks averaging >= this many XDR bytes per record
                                    // take the group kernels (0 = never)
    int32_t stride_check = 1;       // key 29: fixed-size decode at rec_offsets: 1 check for the fixed
                                    // stride and take the stride kernels (sync calls), 0 the record path
    int32_t stage_copy = 1;         // key 26: XDRG_HOST_PTRS copies of device-mapped host spans:
                                    // 1 copy kernels (k_copy_link), 0 the DMA engines (hipMemcpyAsync)
    int32_t xcd_order = 1;          // key 37: payload kernels walk the records in XCD order (xcd_block):
                                    // bit 0 encode, bit 1 decode (0 in block order)
    int32_t emit_per = 4;           // key 36: frame walk, sub-chunks per k_fr_emit block (at most;
                                    // halved until the grid has >= 64 blocks)
    int32_t emit_wave = 1;          // key 48: frame walk emit: 1 a wave per sub-chunk (k_fr_emit_w), 0 k_fr_emit
    int32_t recv_budget = 20;       // key 49: receive windows of group schemas: column bytes reserved per
                                    // window byte, in tenths (hs::stage_receive; tests force the paths
                                    // that deliver fewer messages or grow the ring with small values)
    int32_t frame_spec = 1;         // key 47: word-mode frame walk: 1 the speculative walk (k_fs_*,
                                    // the exact kernels when it gives up), 0 the exact kernels only
    int32_t grp_dec_tile = 32768;   // key 33: repeated-group decode place, LDS tile per sub-batch of
                                    // records (0: each lane walks its record in HBM)
    int32_t grp_enc_lanes = 8;      // key 32: repeated-group encode, lanes per record (64 = a wave)
    int32_t grp_enc_img = 16384;    // key 41: repeated-group encode place element-parallel through an LDS
                                    // image of this many bytes (schemas without conditional fields whose
                                    // group has a layout; 0: lanes per record, key 32).  DUMP encode 2.19 ->
                                    // 0.83 ms, READDIR 5.07 -> 3.03 (32 KiB: 0.92 / 2.99), DESIGN.md §5.7
    int32_t grp_dec_el = 1024;      // key 38: repeated-group decode place element-parallel (one top-level
                                    // group, no inner groups, <= 2 dynamic members), at most this many
                                    // elements per sub-batch (0: a lane per record; READDIR decode 9.3 ->
                                    // 5.5 ms, DUMP 3.0 -> 1.9)
    int32_t recv_win = 1;           // key 42: XDRG_HOST_PTRS receive of repeated-group schemas: 1 the
                                    // staging windows carry the element rows (one PCIe crossing), 0 the
                                    // staged walk, deframe and body decode (three; A/B only)
    int32_t grp_enc_split = 0;      // key 43: element-parallel group encode, blocks per scan block (1, 2,
                                    // 4; 0 = by batch size, enc_el_split)
    int32_t grp_dec_emap = 1;       // key 44: element-parallel group decode finds its elements from the
                                    // walk's element-start map (0: each record lane walks its elements)
    int32_t grp_enc_img_nest = 1;   // key 45: the element-parallel encode (key 41) for a group holding inner
                                    // groups too (0: lanes per record, key 32)
    int32_t spec_sizes = 2;         // key 31: sweep decode whose last dynamic field is a word vector
                                    // followed by fixed fields only: 1 derive its counts from the record
                                    // extents (sizes reads one length word per record, the place kernel
                                    // verifies every count word, exact rerun on a mismatch), 2 the same
                                    // in one pass (the sweep walks its block and looks back for its
                                    // native offsets: no sizes or scan kernel), 0 walk all
};
// Kernel variants measured slower in every A/B and removed (DESIGN.md §5,
// git history): keys 4/5/10/11 (group kernels' loads in flight), 18 (payload
// in the group kernels), 20 = 0 (byte-stored record edges), 24 (payload
// checks before loads), 27 = 0-3 (field-major / output-image / nontemporal
// staged encode), 28 (plain payload stores), 30 (serial frame walk for odd
// fragment sizes), 34 (payload grid stride), 35 (LDS-tiled lane decode),
// key 9 = 3 (lane-per-record kernels for unconditional schemas).
int set_tuning(Tuning &t, int key, long long value);   // 0, or -1 for an unknown key / bad value

// ---- launchers (kernels_*.hip) -----------------------------------------
// All launches go on `stream`; each returns hipSuccess or the launch error.
int launch_stream_words(const StreamArgs &a, void *stream);
// record-marked AoS-dense stream (words: BSWAP / FLOAT / OPAQUE only)
int launch_stream_framed(const StreamArgs &a, uint64_t n, uint32_t mark_le, bool decode,
                         unsigned long long *errkey, const Tuning &t, void *stream);
int launch_wordmap_encode(const WordMapArgs &a, bool aligned16, void *stream);
// lane-per-record word kernels (every XDR word one 4-byte native word, <= 32
// words per record incl. the mark); returns -1 when switched off (tuning)
bool words_lane_ok(const WordOp *ops, uint32_t nops);
int launch_words_lane(const WordMapArgs &a, bool decode, bool v16, const Tuning &t, void *stream);
int launch_wordmap_decode(const WordMapArgs &a, bool aligned16, void *stream);
enum RecPhase { REC_ENC_SIZES, REC_ENC_SCAN, REC_ENC_PLACE, REC_DEC_SIZES, REC_DEC_SCAN, REC_DEC_PLACE };
int launch_rec_phase(const RecArgs &a, int phase, const Tuning &t, void *stream);
// *dst = value (stream-ordered)
int launch_store_u64(uint64_t *dst, uint64_t value, void *stream);
// rec_offsets[i] = i * stride for i in [0, n]
int launch_iota(uint64_t *dst, uint64_t n, uint64_t stride, void *stream);
// out[0] |= 1 if some extent ro[i+1] - ro[i] != stride (i < n); out[1] = ro[0]
int launch_check_stride(const uint64_t *ro, uint64_t n, uint64_t stride, unsigned long long *out, void *stream);
// Combine the device error key with a host-side key and write the public
// results (async mode); any output pointer may be NULL.
int launch_finalize(const unsigned long long *errkey, unsigned long long extra_key, uint64_t n,
                    uint64_t *first_bad, int *err, void *stream);

// ---- parallel record-mark walk (kernels_frame.hip) ------------------------
constexpr uint32_t kFChunkLog2 = 12;
constexpr uint32_t kFChunk = 1u << kFChunkLog2;      // words per sub-chunk (16 KiB of stream)
constexpr uint32_t kFSuperLog2 = 4;                  // sub-chunks per super-chunk, log2
constexpr uint32_t kFSuper = kFChunk << kFSuperLog2; // words per super-chunk (256 KiB)
static_assert(kFSuper <= 65536, "super-local chain words are 16-bit (FrameWs::exitR)");
constexpr uint32_t kFStop = 0xffffffffu;      // chain ends: fragment not fully received
constexpr uint32_t kFUnal = 0xfffffffeu;      // chain meets a size % 4 != 0 (serial fallback)
constexpr uint32_t kFNone = 0xffffffffu;      // no entry
constexpr uint64_t kFMaxLen = (1ull << 34) - (1ull << 21);   // 32-bit word positions below the terminals
struct FrameSub {                             // one sub-chunk's share of the real chain
    uint32_t nfrag, nlast;                    // complete fragments starting in it, LAST flags among them
    uint32_t pre_frag, pre_last;              // exclusive prefixes inside its super-chunk
    uint32_t prev_tail;                       // LAST flag of the super's previous fragment (2: none)
    uint32_t upto_ll, has_ll, rsv;            // fragments through its last LAST one
};
struct FrameSuper {
    uint32_t nfrag, nlast, tail, has_ll;      // tail: LAST flag of its last fragment
    uint64_t upto_ll;                         // in-super fragments through its last LAST one
};
struct FrameBase {                            // super-chunk exclusive prefixes
    uint64_t frag, last;
    uint32_t prev_tail, rsv;                  // LAST flag of the fragment before it
};
struct FrameWs {                              // device workspace of one walk
    uint16_t *exitR;                          // [Q] last chain word inside the super-chunk (super-
                                              // local): the exit is that word's next mark
    uint32_t *alist, *acnt;                   // [nsub][kFChunk], [nsub]: active words of each sub-chunk
                                              // (position | next << 12 | LAST << 24), their count
    uint32_t *sentry;                         // [nsup] super-chunk entries on the real chain
    uint32_t *wtab;                           // [nsup][256] super-chunk exits of each one's first words
    uint32_t *gsx;                            // [nsup][256] walk from each window entry to the group end
    uint32_t *gexit;                          // [ngrp][256] group exits of the first super's first words
    uint32_t *gentry;                         // [ngrp] group entries on the real chain
    FrameSub *sub;                            // [nsub]
    uint32_t *fbits, *lbits;                  // [nsub][128] complete-fragment / LAST bitmaps
    FrameSuper *sup;                          // [nsup]
    FrameBase *bases;                         // [nsup]
    uint64_t *frag_pos;                       // [Q + 2] stream offset of each complete fragment's mark
                                              // (xdrg_deframe; one entry past the last copied fragment)
    uint32_t *sx;                             // [nsup][2] speculative walk: each super-chunk's entry
                                              // guess and exit
    uint64_t *lbw;                            // [5 nsup + 1] its look-back words and block ticket
    uint64_t *res;                            // [0] chain terminal [1] complete fragments (through the
                                              // last LAST one) [3] consumed bytes [4] complete messages
                                              // [5] fragments of the first `cap` messages [6] off-stride
                                              // [7] bit 0: the speculative walk gave up, bit 1:
                                              // its checks failed (k_fs_fix next), bits 8+: re-walks
};
// Walk positions of a len-byte stream: B = 4 words (len / 4), B = 1 bytes a
// whole mark can start at (len - 3).
inline uint32_t frame_positions(uint64_t len, int B) {
    return B == 4 ? (uint32_t)(len / 4) : (uint32_t)(len >= 4 ? len - 3 : 0);
}
constexpr uint64_t kFByteMaxLen = 1ull << 31;   // byte-mode walks (positions and chain values < 2^32)
// Parallel walk over positions of B bytes (4: words, 1: bytes): every result
// in ws.res / msg_offsets (stream or payload offsets); the fragment list too
// when frag_list.  res[0] == kFUnal (word mode only): the real chain met a
// size % 4 != 0 — walk again in byte mode.
// stride > 0 (stream offsets): res[6] = 1 when some message does not start at
// message index x stride (xdrg_receive_batch's fixed-size decode skips its own
// check of the offsets when none is off)
int frame_parallel(const uint8_t *in, uint64_t len, int B, const FrameWs &ws, uint64_t cap, bool stream_offsets,
                   uint64_t *msg_offsets, bool frag_list, int emit_per, int emit_wave, uint64_t stride,
                   void *stream);
int frame_serial(const uint8_t *in, uint64_t len, const FrameWs &ws, uint64_t cap, bool stream_offsets,
                 uint64_t *msg_offsets, void *stream);
// The speculative word walk (k_fs_walk + look-back, k_fr_emit): the same
// results as frame_parallel(B = 4) unless res[7] & 2 (a failed check:
// nothing emitted; call again with fix = true, k_fs_fix + k_fr_emit) or,
// after the fix, res[7] & 1 (it gave up; frame_parallel runs).
int frame_spec(const uint8_t *in, uint64_t len, const FrameWs &ws, uint64_t cap, bool stream_offsets,
               uint64_t *msg_offsets, bool frag_list, int emit_per, int emit_wave, uint64_t stride, bool fix,
               void *stream);
// Bodies of the first nf fragments into payload (marks stripped).
int frame_copy(const uint8_t *in, const FrameWs &ws, uint64_t nf, uint64_t payload_bytes, uint8_t *payload,
               void *stream);

// ---- multi-GPU exchange (kernels_multi.hip) -------------------------------
constexpr int kMaxGatherSeg = 16;
struct GatherArgs {             // copy bytes[s] from src[s] (a peer's HBM) to dst[s]
    uint32_t nseg;
    uint32_t rsv;
    const uint8_t *src[kMaxGatherSeg];
    uint8_t *dst[kMaxGatherSeg];
    uint64_t bytes[kMaxGatherSeg];
};
int launch_gather(const GatherArgs &a, void *stream);
int launch_add_u64(uint64_t *p, uint64_t n, uint64_t delta, void *stream);   // p[0..n) += delta
// p[i] += delta for every p[i] != UINT64_MAX (splice / payload positions: UINT64_MAX = absent)
int launch_add_pos(uint64_t *p, uint64_t n, uint64_t delta, void *stream);
// *dst = *index <= limit ? base[*index] : 0
int launch_pick_u64(uint64_t *dst, const uint64_t *base, const uint64_t *index, uint64_t limit, void *stream);
// dst[0..bytes) = src[0..bytes) by the CUs, one side host memory the device maps
int launch_copy_link(uint8_t *dst, const uint8_t *src, uint64_t bytes, void *stream);

// ---- repeated groups (kernels_group.hip) --------------------------------
// Arrays of structs and recursive lists (include/xdrg.h "Repeated groups").
// A counted column ("slot") is one whose per-record element count the decode
// walk reports and a scan turns into native offsets: a top-level dynamic
// field, a DYNAMIC / LIST group (its elements) or a group's dynamic member
// (its values over the record's elements).
constexpr int kMaxSlots = 16;
// Group nesting levels: a top-level group (level 0) and groups inside its
// elements down to level kGrpLevels - 1 (jrpcgen nests arrays of structs and
// lists without a limit, jrpcgen.java:856-906; the kernels are instantiated
// per level, kGrpLast = the innermost, whose elements hold no group).
constexpr int kGrpLevels = 4;
constexpr int kGrpLast = kGrpLevels - 1;
struct GField {
    uint32_t type, kind, nsz, xsz;
    uint32_t count;   // FIXED count (of a field's elements or a group's)
    uint32_t xbytes;  // fixed field: XDR bytes (incl. pad)
    uint32_t grp;     // member: its immediate group's field index + 1; top level: 0
    uint32_t nmem;    // group: member fields that follow it
    uint32_t efix;    // group: XDR bytes of an element's fixed members (+ 4: a list's bool)
    uint32_t ndm;     // group: dynamic members
    uint32_t slot;    // counted column: slot + 1, else 0
    uint32_t top;     // top-level field index that owns it (the group for a member)
    uint32_t ncm;     // group: conditional members (elements then differ in size)
    uint32_t ngm;     // group: inner groups among its immediate members (one level down)
    // conditional fields (xdrg_cond) on their own level: a top-level field on
    // an earlier top-level discriminant, a member on an earlier member of its
    // group (per element): present iff field cond-1 is present and its value
    // is (cneg = 0) / is not (cneg = 1) in cvals[cfirst, cfirst + cnum)
    uint32_t cond, cneg, cfirst, cnum;
    uint32_t dslot;   // 0, or 1 + this field's discriminant value slot
    // a group member that starts a run of fixed members of one condition
    // class with no discriminant among them (the walks skip such a run as
    // one: a member's SHORT carries its group's sub either way): run bytes
    // << 8 | members (>= 2), else 0 (fill_group; in GField's padding)
    uint32_t run;
    uint8_t *data;
    int64_t stride;
    uint64_t *offsets;
    uint64_t cap;
};
struct GroupArgs {
    uint64_t n;
    uint32_t nf;
    uint32_t framed;
    uint32_t nslot;
    uint32_t enc_lanes;          // encode place: lanes per record (64, 16, 8; tuning key 32)
    uint8_t *xdr;
    uint64_t xdr_cap;            // encode: out_cap; decode: in_len
    const uint64_t *rec_in;      // decode: record extents (n+1)
    uint64_t *rec_out;           // encode: record offsets (n+1), nullable
    uint64_t *rec_size;          // encode workspace [n]: record sizes
    uint64_t *block_sums;        // [max(nslot, 1)][nblocks]
    uint64_t nblocks;
    uint64_t *totals;            // [max(nslot, 1)]
    uint32_t *rec_cnt;           // decode workspace [nslot][n]: counts per record
    uint64_t *rec_base;          // decode workspace [nslot][n]: native offset per record
    unsigned long long *errkey;
    uint32_t slot_field[kMaxSlots];
    uint32_t ncond;              // conditional fields (0: every record / element has all of them)
    uint32_t dec_tile;           // decode place: LDS tile bytes (0: records read from HBM; key 33)
    uint32_t nest;               // some group holds an inner group
    uint32_t levels;             // group levels of the schema (1 + the deepest nesting; the kernels' D)
    uint32_t dec_el;             // decode place: element-parallel, descriptors per sub-batch (0: off; key 38)
    uint32_t el_g;               // the element-parallel place's group (the schema's one top-level group)
    uint8_t *emap;               // decode, element-parallel place (key 44): a byte per stream word, 1 where
                                 // the walk met an element of group el_g (zeroed first; null: off)
    // 1 + the top-level group whose elements have one layout (no conditional
    // members, no inner groups, at most two dynamic members), 0: none.  The walk
    // and the element-parallel place then read one length word per dynamic
    // member of an element and no member descriptor.
    uint32_t lay_g;
    uint32_t lay_pre, lay_mid, lay_post;   // fixed member bytes before / between / after the dynamic members
    uint32_t lay_z0, lay_z1;               // the dynamic members' XDR element sizes
    uint32_t lay_s0, lay_s1;               // their counted-column slots
    uint32_t enc_img;            // encode place: element-parallel, LDS image bytes (0: off; key 41)
    uint32_t enc_split;          // its blocks per scan block (0: enc_el_split; key 43)
    int32_t cvals[XDRG_MAX_CASES];
    GField f[kMaxFields];
};
static_assert(sizeof(GroupArgs) <= 4096, "GroupArgs must fit the kernel-argument segment");
enum GroupPhase { GRP_ENC_SIZES, GRP_ENC_PLACE, GRP_DEC_WALK, GRP_DEC_OFFSETS, GRP_DEC_PLACE };
int launch_group_phase(const GroupArgs &a, int phase, void *stream);
// exclusive scan of `rows` rows of nblocks block sums each (k_scan_rows)
int launch_scan_rows(uint64_t *sums, uint64_t nblocks, uint64_t *totals, uint32_t rows, void *stream);
// extent-derived decode counts failed (*spec == 0): reset the error key for the exact rerun
int launch_spec_reset(const uint32_t *spec, unsigned long long *errkey, void *stream);
// Can this decode derive its last dynamic field's counts from the record extents?
bool rec_spec_ok(const RecArgs &a, const Tuning &t);

constexpr int kRecThreads = 256;   // record path: threads per block
constexpr int kRecPerThread = 4;   // records per thread in the size/scan pass
constexpr int kRecPerBlock = kRecThreads * kRecPerThread;
constexpr int kMaxDynLds = 4;      // dynamic fields whose per-record metadata is staged in LDS
// LDS of k_grp_dec_place_eln (element-parallel place of a nested group):
// extents and first elements (2 x 257 u64) | tile | positions [cap] | scanned
// counts [ns span columns][cap] | GRunL columns [nslot][256 lanes].
constexpr size_t kElnMeta = 2 * (kRecThreads + 1) * 8 + 16;
// LDS budget of one group place block (dynamic + static): two blocks per CU.
// The static parts: k_grp_dec_place_eln's sbase and scan words (416 B at
// round 6, kept under kPlaceStaticLds), and for D > 1 the lane-per-record
// places' running-offset columns (kMaxSlots x kRecThreads words).
constexpr size_t kPlaceLdsBudget = 65536;
constexpr size_t kPlaceStaticLds = 512;
constexpr size_t kNestRunLdsBytes = 8 * (size_t)kMaxSlots * kRecThreads;
inline size_t eln_lds_bytes(uint32_t tile, uint32_t cap, uint32_t ns, uint32_t nslot) {
    return kElnMeta + tile + 4 * (size_t)cap * (1 + ns) + 8 + 8 * (size_t)kRecThreads * (nslot ? nslot : 1);
}


}  // namespace xdrg
