// kernels_frame.hip — record-mark walk of a received TCP byte stream, in
// parallel.  Reference: RpcMessageParserTCP.java
// (paths under /root/reference/oncrpc4j-core/src/main/java/org/dcache/
// oncrpc4j/rpc/): isAllFragmentsArrived :63-99 walks marks BE(size | LAST)
// until a last fragment, STOPping when fewer than 4 bytes or fewer than
// `size` bytes remain; assembleXdr :109-140 concatenates the fragment
// bodies; handleRead :44-61 repeats on the remainder.
//
// The marks form a chain (mark at word q -> next mark at q + 1 + size / 4),
// so the walk is a dependent chain; every word of the stream may be the one
// the chain enters a region at, so a region's "exit" (the first chain word
// at or past its end) is computed for every word.  Fragment sizes of XDR
// traffic are multiples of 4; a stream whose real chain meets another size
// is walked serially (k_fr_serial), with the same result.
//
//   k_fr_exits  block per super-chunk (16 sub-chunks of 4096 words), sub-
//               chunks from last to first: stage the words, point every word
//               at its next mark, resolve pointers into later sub-chunks
//               through their finished results, pointer-jump the pointers
//               that stay inside (active words, compacted) -> exitR[q] = the
//               last chain word inside the super-chunk (16-bit, super-local);
//               the super-chunk exit of q is that word's next mark, which the
//               readers recompute (fr_exit).  One read of the stream, 2 B per
//               word written.
//   k_fr_fix_* each super-chunk's true entry: groups of 64 super-chunks
//               resolve the exit of every entry in their first words in
//               parallel (windows of exits in LDS), one wave hops group to
//               group from word 0, each group fills in its super-chunks.
//   k_fr_mark   block per super-chunk, sub-chunks first to last from its
//               entry: stage, mark the chain by pointer doubling (round r
//               marks the successors 2^r hops on, so round r covers hops
//               < 2^(r+1)), count complete fragments and LAST flags, keep the
//               two bitmaps and the in-super prefixes.
//   k_fr_bases  one block: super-chunk prefixes, the last complete message.
//   k_fr_emit   block per sub-chunk: message offsets (stream or payload
//               coordinates) and, for xdrg_deframe, the fragment list.
//   k_fr_copy   fragment bodies into the payload (marks stripped).
// Chain fragments tile the stream from offset 0, so the payload offset of
// fragment f at stream offset p is p - 4 f and its body size is the gap to
// the next fragment minus 4: no scan over sizes is needed.
// Word positions are 32-bit (streams < 16 GiB - 2 MiB, kFMaxLen).
#include <hip/hip_runtime.h>

#include <utility>

#include "xdrg_internal.h"

namespace xdrg {

__device__ __forceinline__ uint32_t fr_bswap(uint32_t x) { return __builtin_bswap32(x); }
// Order one wave's LDS accesses across lanes (a one-wave block needs no barrier).
__device__ __forceinline__ void sp_fence() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// Positions: the walk runs in word mode (B = 4: position q = stream word q,
// Q = len / 4 words, tb = len % 4 trailing bytes) and, when the real chain
// meets a fragment size that is not a multiple of 4, again in byte mode (B =
// 1: position p = stream byte p, Q = len - 3 = the positions a whole mark can
// start at, marks read unaligned; streams < 2 GiB).  A chain value >= Q ends
// the walk in both.
//
// Next chain position after the mark m at position q < Q, or a terminal:
// kFStop (fragment not fully received: size > remaining - 4,
// RpcMessageParserTCP.java:77-79), kFUnal (word mode: size % 4 != 0).
template <int B>
__device__ __forceinline__ uint32_t fr_next(uint32_t m, uint32_t q, uint32_t Q, uint32_t tb) {
    const uint32_t size = m & kSizeMask;
    if (B == 1) return size + 1 <= Q - q ? q + 4 + size : kFStop;   // Q + 3 - q bytes left
    const uint32_t R = Q - q;   // whole words left, >= 1
    const bool fits = R >= (1u << 30) || size + 4 <= 4 * R + tb;
    if (!fits) return kFStop;
    if (size & 3) return kFUnal;
    return q + 1 + (size >> 2);
}

// The raw (memory-order) mark word at position p < Q.  Byte mode: bytes p ..
// p + 3 from the two words around them (the second one byte by byte where it
// passes the stream's end, len = Q + 3).
template <int B>
__device__ __forceinline__ uint32_t fr_at(const uint32_t *w, uint32_t Q, uint32_t p) {
    if (B == 4) return w[p];
    const uint32_t i = p >> 2, s = p & 3;
    const uint32_t a = w[i];
    if (s == 0) return a;
    const uint64_t len = (uint64_t)Q + 3;
    uint32_t b = 0;
    if (4 * (uint64_t)i + 8 <= len) {
        b = w[i + 1];
    } else {
        const uint8_t *c = (const uint8_t *)w;
        for (uint32_t j = 0; j < 4; ++j)
            if (4 * (uint64_t)i + 4 + j < len) b |= (uint32_t)c[4 * (uint64_t)i + 4 + j] << (8 * j);
    }
    return __builtin_amdgcn_alignbyte(b, a, s);
}

// Word layout of a sub-chunk (kFChunk = 4096 words, 256 threads): thread t
// owns words 4 t + 1024 k + c (k, c < 4), so every 16-byte load and store of
// a wave covers 1 KiB contiguously and the own-word LDS accesses of
// neighbouring lanes fall in neighbouring banks.  (Sixteen consecutive words
// per thread measured slower: 16-byte accesses 64 bytes apart.)
typedef uint32_t u32x4f __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint32_t fr_cw(uint32_t tid, int i) { return 4 * tid + 1024 * (i >> 2) + (i & 3); }
// Whether a sub-chunk's marks load without guards: word mode every word
// inside; byte mode the 1025 words under it inside the stream.
template <int B>
__device__ __forceinline__ bool fr_full(uint32_t base, uint32_t Q) {
    return B == 4 ? base + kFChunk <= Q : (uint64_t)base + kFChunk + 4 <= (uint64_t)Q + 3;
}
template <int B>
__device__ __forceinline__ void fr_cload(const uint32_t *w, uint32_t Q, uint32_t base, uint32_t tid, uint32_t (&r)[16]) {
    if (B == 4 && fr_full<B>(base, Q)) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const u32x4f v = __builtin_nontemporal_load((const u32x4f *)(w + base + 4 * tid + 1024 * k));
            r[4 * k] = v.x; r[4 * k + 1] = v.y; r[4 * k + 2] = v.z; r[4 * k + 3] = v.w;
        }
    } else if (B == 1 && fr_full<B>(base, Q)) {   // positions 4 tid + 1024 k + c: word wb + tid + 256 k, byte c
        const uint32_t wb = base >> 2;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t a = w[wb + tid + 256 * k], b = w[wb + tid + 256 * k + 1];
            r[4 * k] = a;
            r[4 * k + 1] = __builtin_amdgcn_alignbyte(b, a, 1);
            r[4 * k + 2] = __builtin_amdgcn_alignbyte(b, a, 2);
            r[4 * k + 3] = __builtin_amdgcn_alignbyte(b, a, 3);
        }
    } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) r[i] = base + fr_cw(tid, i) < Q ? fr_at<B>(w, Q, base + fr_cw(tid, i)) : 0u;
    }
}

// Block-wide "any" with one barrier: each wave's ballot lands in one of two
// alternating flag rows (a row is rewritten only two rounds later, after
// every thread has read it).
struct FrAny {
    uint32_t f[2][4];
};
__device__ __forceinline__ bool fr_block_any(bool p, FrAny &a, uint32_t &par) {
    const bool w = __ballot(p) != 0;
    a.f[par][threadIdx.x >> 6] = w ? 1u : 0u;   // every lane of the wave stores the same value
    __syncthreads();
    const u32x4f v = *(const u32x4f *)a.f[par];
    par ^= 1u;
    return (v.x | v.y | v.z | v.w) != 0;
}

// Inclusive prefix sum over the wave.
__device__ __forceinline__ uint32_t fr_wave_incl(uint32_t v) {
    const uint32_t lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t a = __shfl_up(v, d, 64);
        if (lane >= (uint32_t)d) v += a;
    }
    return v;
}

// ---------------------------------------------------------------------------
// k_fr_exits
// ---------------------------------------------------------------------------
// Sub-chunks from last to first.  J holds, per word, either a sub-chunk-local
// pointer (< kFChunk: the word's chain goes on inside the sub-chunk) or a
// result kFRes | r (r = super-local last chain word inside the super-chunk).
// A word whose next mark stays inside the sub-chunk is active: its pointer
// jumps (in place: a value read early is still a successor on the same chain)
// until it holds a result.  The active words are compacted into a list first,
// so every thread jumps ceil(active / 256) of them per round whatever the
// layout of the marks.  A next mark in a later sub-chunk of the super-chunk
// takes that word's result from exitR, which this block already wrote (L2;
// never read before, so no stale L1 line).  24 KiB of LDS.  (The next
// sub-chunk's results kept in LDS instead measured slower: 32 KiB, fewer
// blocks per CU.)  The compacted list goes out too, for k_fr_mark: per
// sub-chunk alist[sub][k] = position | next << 12 | LAST << 24 of its active
// words (complete fragments all), acnt[sub] of them.
constexpr uint32_t kFRes = 0x10000u;
constexpr uint32_t kFPtr = 0xfffu;     // the local pointer of a J value (bit 12: the word's LAST flag)
template <int B>
__global__ __launch_bounds__(256, 6) void k_fr_exits(const uint32_t *__restrict__ w, uint32_t Q, uint32_t tb,
                                                      uint16_t *exitR, uint32_t *alist, uint32_t *acnt,
                                                      uint32_t *sentry, uint32_t *gentry, uint32_t ngrp) {
    __shared__ __attribute__((aligned(16))) uint32_t J[kFChunk];
    __shared__ __attribute__((aligned(16))) uint16_t L[kFChunk];   // active positions (sub-chunk local)
    __shared__ uint32_t wtot[4];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint32_t sbeg = blockIdx.x * kFSuper;
    const uint32_t send = min(sbeg + kFSuper, Q);   // chain words past it leave the super-chunk
    const uint32_t nsub = (send - sbeg + kFChunk - 1) / kFChunk;
    // the entries k_fr_fix_* fill in start as "none" (one vector store a block)
    if (tid == 0) {
        sentry[blockIdx.x] = ~0u;
        if (blockIdx.x < ngrp) gentry[blockIdx.x] = ~0u;
    }
    uint32_t x[16], y[16];
    fr_cload<B>(w, Q, sbeg + (nsub - 1) * kFChunk, tid, x);
    for (int j = (int)nsub - 1; j >= 0; --j) {
        const uint32_t base = sbeg + (uint32_t)j * kFChunk;
        const uint32_t bend = base + kFChunk;
        if (j > 0) fr_cload<B>(w, Q, base - kFChunk, tid, y);   // next sub-chunk's words in flight
        // J: a local pointer with the word's LAST flag (next mark inside), the
        // next mark's offset past bend when it lies in a later sub-chunk
        // [bend, send) (looked up below), else the word itself as the last one
        // (next mark past the super-chunk, or a terminal)
        const uint32_t lim = send > bend ? send - bend : 0u;
        const uint32_t own0 = kFRes | (base - sbeg + 4 * tid);
        uint32_t act = 0, look = 0;
        if (bend <= Q && fr_full<B>(base, Q)) {
            // a full sub-chunk: d = local position of the next mark.  A size
            // that is not a multiple of 4 ends the chain (word mode terminal),
            // and a fragment that does not fit reaches past Q >= send, so
            // neither needs its own test here.  One band of 4 words at a time
            // (few live registers: occupancy bounds this kernel)
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                uint32_t t[4];
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const int i = 4 * k + c;
                    const uint32_t m = fr_bswap(x[i]);
                    const uint32_t d = B == 4 ? ((m >> 2) & 0x1fffffffu) + 4 * tid + 1024 * k + c + 1
                                              : (m & kSizeMask) + 4 * tid + 1024 * k + c + 4;
                    const bool al = B == 1 || (m & 3u) == 0;
                    const bool in = al && d < kFChunk, lk = al && d - kFChunk < lim;
                    act |= (in ? 1u : 0u) << i;
                    look |= (lk ? 1u : 0u) << i;
                    t[c] = in ? d | (x[i] & 0x80u) << 5 : lk ? d - kFChunk : own0 + 1024 * k + c;
                }
                *(u32x4f *)&J[4 * tid + 1024 * k] = u32x4f{t[0], t[1], t[2], t[3]};
            }
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                uint32_t t[4];
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const int i = 4 * k + c;
                    const uint32_t q = base + fr_cw(tid, i);
                    const uint32_t v = q < Q ? fr_next<B>(fr_bswap(x[i]), q, Q, tb) : kFStop;
                    act |= (v < bend ? 1u : 0u) << i;   // a word inside (terminals are >= kFUnal)
                    const bool lk = v - bend < lim;
                    look |= (lk ? 1u : 0u) << i;
                    t[c] = v < bend ? (v - base) | (x[i] & 0x80u) << 5 : lk ? v - bend : own0 + 1024 * k + c;
                }
                *(u32x4f *)&J[4 * tid + 1024 * k] = u32x4f{t[0], t[1], t[2], t[3]};
            }
        }
        for (uint32_t m = look; m; m &= m - 1) {   // own words: no barrier needed
            const uint32_t li = fr_cw(tid, __ffs(m) - 1);
            J[li] = kFRes | exitR[bend + J[li]];
        }
        const uint32_t cnt = __popc(act);
        const uint32_t incl = fr_wave_incl(cnt);
        if (lane == 63) wtot[wv] = incl;
        __syncthreads();   // J, wtot
        const uint32_t t0 = wtot[0], t1 = wtot[1], t2 = wtot[2], t3 = wtot[3];
        const uint32_t A = t0 + t1 + t2 + t3;   // active words of the sub-chunk
        uint32_t pos = incl - cnt + (wv > 0 ? t0 : 0u) + (wv > 1 ? t1 : 0u) + (wv > 2 ? t2 : 0u);
        const uint64_t sub = (uint64_t)blockIdx.x * (kFSuper / kFChunk) + (uint32_t)j;
        for (uint32_t m = act; m; m &= m - 1) L[pos++] = (uint16_t)fr_cw(tid, __ffs(m) - 1);
        if (tid == 0) acnt[sub] = A;
        if (A) {
            __syncthreads();   // L
            // the list out (coalesced), before this thread's own entries jump
            uint32_t *al = alist + sub * kFChunk;
            for (uint32_t k = tid; k < A; k += 256) {
                const uint32_t li = L[k];
                al[k] = li | (J[li] & 0x1fffu) << 12;
            }
            // this thread's list entries: tid + 256 c, c < ceil((A - tid) / 256).
            // Asynchronous pointer jumping: a thread jumps its own entries until
            // they hold results, reading whatever the other threads have written
            // meanwhile (LDS words are read and written whole, and every value a
            // word ever holds is a successor on its chain), so no barrier per
            // round.  Positions only grow, so a pointer resolves within kFChunk
            // jumps (the bound is a guard).
            const uint32_t mine = A > tid ? (A - tid - 1) / 256 + 1 : 0u;
            uint32_t pend = mine >= 32 ? ~0u : (1u << mine) - 1u;
            for (uint32_t it = 0; pend && it < kFChunk; ++it) {
                for (uint32_t m = pend; m; m &= m - 1) {
                    const uint32_t c = __ffs(m) - 1;
                    const uint32_t li = L[tid + 256 * c];
                    const uint32_t u = J[J[li] & kFPtr];
                    J[li] = u;
                    if (u >= kFRes) pend &= ~(1u << c);
                }
            }
            __syncthreads();   // every entry holds its result
        }
        typedef uint16_t u16x4f __attribute__((ext_vector_type(4)));
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const u32x4f v = *(const u32x4f *)&J[4 * tid + 1024 * k];
            const u16x4f h = u16x4f{(uint16_t)v.x, (uint16_t)v.y, (uint16_t)v.z, (uint16_t)v.w};
            if (bend <= Q) {
                *(u16x4f *)(exitR + base + 4 * tid + 1024 * k) = h;
            } else {
#pragma unroll
                for (int c = 0; c < 4; ++c)
                    if (base + 4 * tid + 1024 * k + c < Q) exitR[base + 4 * tid + 1024 * k + c] = h[c];
            }
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) x[i] = y[i];
        __syncthreads();   // this sub-chunk's exitR visible to the block; J, L, wtot free again
    }
}

// The super-chunk exit of word q < Q: the next mark after its chain's last
// word inside the super-chunk (a word >= min(super end, Q), or a terminal).
template <int B>
__device__ __forceinline__ uint32_t fr_exit(const uint32_t *w, const uint16_t *exitR, uint32_t Q, uint32_t tb,
                                            uint32_t q) {
    const uint32_t r = (q & ~(kFSuper - 1)) + exitR[q];
    return fr_next<B>(fr_bswap(fr_at<B>(w, Q, r)), r, Q, tb);
}

// ---------------------------------------------------------------------------
// k_fr_fix: super-chunk entries along the real chain from word 0.
// ---------------------------------------------------------------------------
// Two levels: a group is 64 consecutive super-chunks.
//   k_fr_fix_grp   block per group: the group's exit for every entry word in
//                  the first kFixWin words of its first super-chunk (a lane
//                  per entry hops super-chunk to super-chunk through windows
//                  of exits staged in LDS; an entry deeper than the window
//                  recomputes its exit from exitR);
//   k_fr_fix_top   one wave hops group to group from word 0 (a deep group
//                  entry walks that group's super-chunks through fr_exit);
//   k_fr_fix_fill  block per group: from its true entry, every super-chunk
//                  entry of the group (sentry).
constexpr uint32_t kFixWin = 256;   // entry words per super-chunk window
constexpr uint32_t kFixGrp = 64;    // super-chunks per group
template <int B>
struct FrExits {   // what fr_exit reads
    const uint32_t *w;
    const uint16_t *exitR;
    uint32_t Q, tb;
    __device__ __forceinline__ uint32_t operator()(uint32_t q) const { return fr_exit<B>(w, exitR, Q, tb, q); }
};
// k_fr_win: the window table, wtab[s][d] = exit of word d < kFixWin of
// super-chunk s (kFStop past Q), every entry in parallel.
template <int B>
__global__ __launch_bounds__(256) void k_fr_win(FrExits<B> ex, uint32_t nsup, uint32_t *wtab) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (uint64_t)nsup * kFixWin) return;
    const uint64_t q = (i / kFixWin) * kFSuper + i % kFixWin;
    wtab[i] = q < ex.Q ? ex((uint32_t)q) : kFStop;
}
// Group g's windows from the table (kFStop past the last super-chunk).
__device__ __forceinline__ void fix_stage(const uint32_t *wtab, uint32_t nsup, uint32_t g, uint32_t *win) {
    typedef uint32_t u32x4w __attribute__((ext_vector_type(4)));
    const uint64_t n = (uint64_t)min(kFixGrp, nsup - g * kFixGrp) * kFixWin;
    const u32x4w *src = (const u32x4w *)(wtab + (uint64_t)g * kFixGrp * kFixWin);
    for (uint32_t k = threadIdx.x; k < kFixGrp * kFixWin / 4; k += blockDim.x)
        ((u32x4w *)win)[k] = 4 * (uint64_t)k < n ? src[k] : u32x4w{kFStop, kFStop, kFStop, kFStop};
    __syncthreads();
}
// One hop from chain word e inside group g: the exit of e's super-chunk.
template <int B>
__device__ __forceinline__ uint32_t fix_hop(const FrExits<B> &ex, const uint32_t *win, uint32_t g, uint32_t e) {
    const uint32_t s = e >> (kFChunkLog2 + kFSuperLog2), d = e & (kFSuper - 1);
    return d < kFixWin ? win[(s - g * kFixGrp) * kFixWin + d] : ex(e);
}

// k_fr_fix_grp: per group, a backward sweep over its super-chunks gives, for
// every window entry (k, d < kFixWin), the first chain word that is past the
// group, a terminal, or a deep word (depth >= kFixWin) inside the group where
// a walk must go on through fr_exit: gsx[g][k][d] (k_fr_fix_top uses it for
// deep group entries).  Then the group exits of the first super-chunk's
// window, gexit[g][d], resolved through the deep words.  128 KiB of LDS.
template <int B>
__global__ __launch_bounds__(256) void k_fr_fix_grp(FrExits<B> ex, const uint32_t *wtab, uint32_t nsup,
                                                    uint32_t *gsx, uint32_t *gexit) {
    __shared__ __attribute__((aligned(16))) uint32_t win[kFixGrp * kFixWin];
    __shared__ __attribute__((aligned(16))) uint32_t sg[kFixGrp * kFixWin];
    const uint32_t g = blockIdx.x, d = threadIdx.x;
    const uint32_t Q = ex.Q;
    fix_stage(wtab, nsup, g, win);
    const uint32_t gbeg = g * kFixGrp * kFSuper;
    const uint64_t gend64 = (uint64_t)gbeg + (uint64_t)kFixGrp * kFSuper;
    const uint32_t gend = gend64 < Q ? (uint32_t)gend64 : Q;
    const uint32_t nk = min(kFixGrp, nsup - g * kFixGrp);
    for (int k = (int)nk - 1; k >= 0; --k) {
        uint32_t x = win[k * kFixWin + d];
        if (x < gend) {   // inside the group, in a later super-chunk
            const uint32_t k2 = (x - gbeg) >> (kFChunkLog2 + kFSuperLog2), d2 = (x - gbeg) & (kFSuper - 1);
            if (d2 < kFixWin) x = sg[k2 * kFixWin + d2];
        }
        sg[k * kFixWin + d] = x;
        __syncthreads();
    }
    uint32_t *out = gsx + (uint64_t)g * kFixGrp * kFixWin;
    for (uint32_t k = 0; k < nk; ++k) out[k * kFixWin + d] = sg[k * kFixWin + d];
    uint32_t e = gbeg + d;   // this lane's entry word
    if (e < gend) {
        e = sg[d];
        while (e < gend) {   // a deep word: one super-chunk through fr_exit, then the table again
            e = ex(e);
            if (e >= gend) break;
            const uint32_t k2 = (e - gbeg) >> (kFChunkLog2 + kFSuperLog2), d2 = (e - gbeg) & (kFSuper - 1);
            if (d2 < kFixWin) e = sg[k2 * kFixWin + d2];
        }
    } else {
        e = kFStop;
    }
    gexit[(uint64_t)g * kFixWin + d] = e;
}

// The group exits go through LDS when they fit (a stream up to kFTopLds
// groups, 2.5 GiB): the hop chain then costs LDS latency per group.
constexpr uint32_t kFTopLds = 160;
template <int B>
__global__ __launch_bounds__(1024) void k_fr_fix_top(FrExits<B> ex, const uint32_t *gsx, const uint32_t *gexit,
                                                     uint32_t ngrp, uint32_t *gentry, uint64_t *res) {
    __shared__ __attribute__((aligned(16))) uint32_t gl[kFTopLds * kFixWin];
    const uint32_t Q = ex.Q;
    const bool lds = ngrp <= kFTopLds;
    if (lds) {
        typedef uint32_t u32x4w __attribute__((ext_vector_type(4)));
        for (uint32_t k = threadIdx.x; k < ngrp * kFixWin / 4; k += blockDim.x)
            ((u32x4w *)gl)[k] = ((const u32x4w *)gexit)[k];
        __syncthreads();
    }
    if (threadIdx.x >= 64) return;
    uint32_t e = 0;
    while (e < Q) {
        const uint32_t g = e / (kFixGrp * kFSuper), d = e - g * kFixGrp * kFSuper;
        gentry[g] = e;   // one address for the whole wave
        if (d < kFixWin) {
            e = lds ? gl[g * kFixWin + d] : gexit[(uint64_t)g * kFixWin + d];
        } else {         // a deep group entry: fr_exit to the next super-chunk, then the sweep's table
            const uint32_t gbeg = g * kFixGrp * kFSuper;
            const uint64_t gend = (uint64_t)gbeg + (uint64_t)kFixGrp * kFSuper;
            while (e < Q && e < gend) {
                e = ex(e);
                if (e >= kFUnal || e >= Q || e >= gend) break;
                const uint32_t k2 = (e - gbeg) >> (kFChunkLog2 + kFSuperLog2), d2 = (e - gbeg) & (kFSuper - 1);
                if (d2 < kFixWin) e = gsx[((uint64_t)g * kFixGrp + k2) * kFixWin + d2];
            }
        }
        if (e >= kFUnal) break;
    }
    if (threadIdx.x == 0) res[0] = e;   // >= Q: ran to the end; kFStop / kFUnal: terminal met on the real chain
}

template <int B>
__global__ __launch_bounds__(256) void k_fr_fix_fill(FrExits<B> ex, const uint32_t *wtab, const uint32_t *gentry,
                                                     uint32_t nsup, uint32_t *sentry) {
    __shared__ __attribute__((aligned(16))) uint32_t win[kFixGrp * kFixWin];
    const uint32_t g = blockIdx.x;
    const uint32_t Q = ex.Q;
    uint32_t e = gentry[g];
    if (e == kFNone) return;   // the chain skips this group (block-uniform)
    fix_stage(wtab, nsup, g, win);
    if (threadIdx.x) return;
    const uint64_t gend64 = (uint64_t)(g + 1) * kFixGrp * kFSuper;
    const uint32_t gend = gend64 < Q ? (uint32_t)gend64 : Q;
    while (e < gend) {
        sentry[e >> (kFChunkLog2 + kFSuperLog2)] = e;
        e = fix_hop(ex, win, g, e);
        if (e >= kFUnal) break;
    }
}

// ---------------------------------------------------------------------------
// k_fr_mark: per sub-chunk bitmaps of the complete chain fragments and their
// LAST flags, counts and in-super prefixes.
// ---------------------------------------------------------------------------
// Works on k_fr_exits' list of active words (the words whose next mark stays
// inside the sub-chunk) instead of the stream: the chain inside a sub-chunk
// is its entry, list entries, and one last word whose next mark leaves (or
// ends the chain), read from the stream by one thread.  The chain is found by
// pruning (below), or by pointer doubling over sub-chunk-local u16 pointers
// (kFOut = no pointer inside) when pruning has not settled in kFPruneRounds.
// Marks are LDS bitmaps (bit b of word k = position 32 k + b), written out
// whole.
constexpr uint32_t kFOut = 0xffffu;
constexpr int kFPruneRounds = 4;   // then pointer doubling
constexpr int kFMaxEnt = kFChunk / 256;   // list entries per thread (at most)
struct FrWaveStat {       // waves 0 and 1 (bitmap words 64 v .. 64 v + 63)
    uint32_t nfrag;       // complete fragments
    uint32_t nlast;       // LAST ones among them
    uint32_t cand;        // (1 + position of its last LAST fragment) << 16 | its complete fragments through it
    uint32_t tail;        // 1 + (position << 1 | LAST flag) of its last complete fragment (0: none)
};
// bytes b0..b3 of w, each 0 or 1, as bits 0..3
__device__ __forceinline__ uint32_t fr_bytes01(uint32_t w) { return (w * 0x01020408u) >> 24 & 0xfu; }
__device__ __forceinline__ uint32_t fr_wave_sum(uint32_t v) {
#pragma unroll
    for (int d = 32; d; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}
__device__ __forceinline__ uint32_t fr_wave_max(uint32_t v) {
#pragma unroll
    for (int d = 32; d; d >>= 1) v = max(v, (uint32_t)__shfl_xor(v, d, 64));
    return v;
}
__device__ __forceinline__ uint32_t fr_wave_min(uint32_t v) {
#pragma unroll
    for (int d = 32; d; d >>= 1) v = min(v, (uint32_t)__shfl_xor(v, d, 64));
    return v;
}

template <int B>
__global__ __launch_bounds__(256, 4) void k_fr_mark(const uint32_t *__restrict__ w, uint32_t Q, uint32_t tb,
                                                     const uint32_t *sentry, const uint64_t *res,
                                                     const uint32_t *alist, const uint32_t *acnt, FrameSub *sub,
                                                     uint32_t *fbits, uint32_t *lbits, FrameSuper *sup) {
    // J[1] (pointer doubling) and pred (pruning) are never live together: one
    // buffer; a doubling pass clears it afterwards, as pred's stamps expect
    __shared__ __attribute__((aligned(16))) uint16_t J[2][kFChunk];
    __shared__ __attribute__((aligned(16))) uint8_t on[kFChunk + 64];   // + one dummy byte per lane
    uint8_t *const pred = (uint8_t *)J[1];                              // round stamps (else never cleared)
    __shared__ __attribute__((aligned(16))) uint32_t fb[128], lb[128];
    __shared__ __attribute__((aligned(16))) FrAny any;
    __shared__ FrWaveStat ws[2];
    __shared__ uint32_t wmax[4], e_next;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint32_t s = blockIdx.x;
    const uint32_t sbeg = s * kFSuper;
    const uint32_t send = min(sbeg + kFSuper, Q);
    const uint32_t nsub = (send - sbeg + kFChunk - 1) / kFChunk;
    const uint64_t sub0 = (uint64_t)s * (kFSuper / kFChunk);
    uint32_t e = res[0] == kFUnal ? kFNone : sentry[s];   // kFNone: no chain word in this super-chunk
    uint32_t pre_f = 0, pre_l = 0, tail = 2;   // tail: LAST flag of the super's last fragment (2 = none yet)
    uint32_t lastlast = 0, has_ll = 0;         // in-super count up to and including its last LAST fragment
    uint32_t par = 0;
    // empty state: J no pointers, on / pred / bitmaps clear
    typedef uint32_t u32x4m __attribute__((ext_vector_type(4)));
    const u32x4m z4 = {0u, 0u, 0u, 0u}, o4 = {~0u, ~0u, ~0u, ~0u};
    *(u32x4m *)&J[0][8 * tid] = o4;
    *(u32x4m *)&J[0][8 * tid + 2048] = o4;
    *(u32x4m *)&on[16 * tid] = z4;
    *(u32x4m *)&J[1][8 * tid] = z4;
    *(u32x4m *)&J[1][8 * tid + 2048] = z4;
    if (tid < 128) fb[tid] = 0; else lb[tid - 128] = 0;
    __syncthreads();
    // the next sub-chunk's list count and first two entries, loaded one ahead
    uint32_t nA = acnt[sub0], n0 = alist[sub0 * kFChunk + tid], n1 = alist[sub0 * kFChunk + 256 + tid];
    for (uint32_t j = 0; j < nsub; ++j) {
        const uint32_t base = sbeg + j * kFChunk;
        const uint32_t bend = base + kFChunk;
        const uint64_t sj = sub0 + j;
        const uint32_t A = nA, p0 = n0, p1 = n1;
        if (j + 1 < nsub) {
            nA = acnt[sj + 1];
            n0 = alist[(sj + 1) * kFChunk + tid];
            n1 = alist[(sj + 1) * kFChunk + 256 + tid];
        }
        FrameSub info;
        info.pre_frag = pre_f;
        info.pre_last = pre_l;
        info.prev_tail = tail;
        info.nfrag = info.nlast = info.upto_ll = info.has_ll = info.rsv = 0;
        if (e >= bend || e >= Q) {   // the chain skips this sub-chunk (or has ended); state stays empty
            if (tid == 0) sub[sj] = info;
            if (tid < 128) fbits[sj * 128 + tid] = 0; else lbits[sj * 128 + tid - 128] = 0;
            continue;
        }
        const uint32_t el = e - base;   // the entry, sub-chunk local
        const uint32_t Cmax = (A + 255) / 256;
        const uint32_t *al = alist + sj * kFChunk;
        uint32_t ent[kFMaxEnt], mine = 0;   // entries tid + 256 c: position | next << 12 | LAST << 24
#pragma unroll
        for (int c = 0; c < kFMaxEnt; ++c) {
            if ((uint32_t)c >= Cmax) break;
            const uint32_t k = tid + 256 * c;
            ent[c] = c == 0 ? p0 : c == 1 ? p1 : k < A ? al[k] : 0u;
            mine |= (k < A ? 1u : 0u) << c;
        }
        // S = the entry and every list target; the largest target (or the
        // entry) is most likely the chain's last word: its stream word is
        // loaded ahead of the pruning
        uint32_t tmax = el;
#pragma unroll
        for (int c = 0; c < kFMaxEnt; ++c) {
            if ((uint32_t)c >= Cmax) break;
            if ((mine >> c) & 1) {
                const uint32_t pos = ent[c] & 0xfffu, nx = (ent[c] >> 12) & 0xfffu;
                J[0][pos] = (uint16_t)nx;
                on[nx] = 1;
                tmax = max(tmax, nx);
            }
        }
        tmax = fr_wave_max(tmax);
        if (lane == 0) wmax[wv] = tmax;
        if (tid == 0) on[el] = 1;
        __syncthreads();
        uint32_t guess = 0, gword = 0;
        if (tid == 0) {
            guess = max(max(wmax[0], wmax[1]), max(wmax[2], wmax[3]));
            if (base + guess < Q) gword = fr_at<B>(w, Q, base + guess);
        }
        // drop the nodes with no predecessor in S until nothing changes; every
        // node left reaches back to the entry (positions fall along
        // predecessors), every chain node stays: S is the chain.  Rounds = the
        // longest false chain + 1.  pred holds round stamps, so it is never
        // cleared.
        bool settled = false;
        for (int r = 0; r < kFPruneRounds; ++r) {
            const uint8_t stamp = (uint8_t)(1 + j * kFPruneRounds + r);
#pragma unroll
            for (int c = 0; c < kFMaxEnt; ++c) {
                if ((uint32_t)c >= Cmax) break;
                if (((mine >> c) & 1) && on[ent[c] & 0xfffu]) pred[(ent[c] >> 12) & 0xfffu] = stamp;
            }
            __syncthreads();
            bool ch = false;
#pragma unroll
            for (int c = 0; c < kFMaxEnt; ++c) {
                if ((uint32_t)c >= Cmax) break;
                const uint32_t nx = (ent[c] >> 12) & 0xfffu;
                if (((mine >> c) & 1) && nx != el && on[nx] && pred[nx] != stamp) {
                    on[nx] = 0;
                    ch = true;
                }
            }
            if (!fr_block_any(ch, any, par)) { settled = true; break; }
        }
        if (!settled) {
            // long false chains (bodies full of small integers): pointer
            // doubling with marking, double-buffered: round r reads J^(2^r) and
            // marks the node 2^r hops past every marked node, so after round r
            // every chain node < 2^(r+1) hops from the entry is marked.  An
            // entry whose pointer left copies the sentinel into the other buffer
            // once more before it drops out, so both buffers agree on it.
            *(u32x4m *)&J[1][8 * tid] = o4;
            *(u32x4m *)&J[1][8 * tid + 2048] = o4;
            *(u32x4m *)&on[16 * tid] = z4;
            __syncthreads();
#pragma unroll
            for (int c = 0; c < kFMaxEnt; ++c) {
                if ((uint32_t)c >= Cmax) break;
                if ((mine >> c) & 1) J[1][ent[c] & 0xfffu] = (uint16_t)((ent[c] >> 12) & 0xfffu);
            }
            if (tid == 0) on[el] = 1;
            __syncthreads();
            uint32_t cur = 0, live = mine;
            for (;;) {
                bool mv = false;
                const uint16_t *Jc = J[cur];
                uint16_t *Jn = J[cur ^ 1];
#pragma unroll
                for (int c = 0; c < kFMaxEnt; ++c) {
                    if ((uint32_t)c >= Cmax) break;
                    if (!((live >> c) & 1)) continue;
                    const uint32_t li = ent[c] & 0xfffu;
                    const uint32_t v = Jc[li];
                    const bool in = v != kFOut;
                    const uint32_t vv = in ? v : li;
                    const bool o = on[li] != 0;
                    on[in && o ? v : kFChunk + lane] = 1;
                    const uint32_t u = Jc[vv];
                    Jn[li] = (uint16_t)(in ? u : kFOut);
                    live &= in ? ~0u : ~(1u << c);
                    mv |= in && u != kFOut;
                }
                cur ^= 1;
                if (!fr_block_any(mv, any, par)) break;
            }
            // leave J[0] with no pointers for the next sub-chunk, J[1] clear
            // for pred's stamps
            *(u32x4m *)&J[0][8 * tid] = o4;
            *(u32x4m *)&J[0][8 * tid + 2048] = o4;
            *(u32x4m *)&J[1][8 * tid] = z4;
            *(u32x4m *)&J[1][8 * tid + 2048] = z4;
        }
        // marks of the chain's list words; its last word = the largest chain position
        uint32_t lmax = el;
#pragma unroll
        for (int c = 0; c < kFMaxEnt; ++c) {
            if ((uint32_t)c >= Cmax) break;
            const uint32_t pos = ent[c] & 0xfffu;
            if (((mine >> c) & 1) && on[pos]) {
                atomicOr(&fb[pos >> 5], 1u << (pos & 31));
                if ((ent[c] >> 24) & 1) atomicOr(&lb[pos >> 5], 1u << (pos & 31));
                lmax = max(lmax, (ent[c] >> 12) & 0xfffu);
            }
        }
        lmax = fr_wave_max(lmax);
        if (lane == 0) wmax[wv] = lmax;   // (thread 0 read the previous values before the pruning's barriers)
        __syncthreads();   // marks, wmax; on / J free again
        const uint32_t last = max(max(wmax[0], wmax[1]), max(wmax[2], wmax[3]));
        // back to the empty state for the next sub-chunk (the list entries only)
#pragma unroll
        for (int c = 0; c < kFMaxEnt; ++c) {
            if ((uint32_t)c >= Cmax) break;
            if ((mine >> c) & 1) {
                J[0][ent[c] & 0xfffu] = (uint16_t)kFOut;
                on[(ent[c] >> 12) & 0xfffu] = 0;
            }
        }
        if (tid == 0) {   // the last word: its next mark is the next sub-chunk's entry
            const uint32_t q = base + last;
            uint32_t v = kFStop;
            if (q < Q) {
                const uint32_t m = fr_bswap(last == guess ? gword : fr_at<B>(w, Q, q));
                v = fr_next<B>(m, q, Q, tb);
                if (v < kFUnal) {
                    atomicOr(&fb[last >> 5], 1u << (last & 31));
                    if (m >> 31) atomicOr(&lb[last >> 5], 1u << (last & 31));
                }
            }
            on[el] = 0;
            e_next = v;
        }
        __syncthreads();   // bitmaps final, e_next
        const uint32_t fw = tid < 128 ? fb[tid] : 0u, lw = tid < 128 ? lb[tid] : 0u;
        if (tid < 128) fbits[sj * 128 + tid] = fw; else lbits[sj * 128 + tid - 128] = lb[tid - 128];
        if (wv < 2) {   // bitmap word tid: counts, the last LAST fragment, the last fragment
            const uint32_t pc = __popc(fw);
            const uint32_t incl = fr_wave_incl(pc);
            uint32_t cand = 0, tl = 0;
            if (lw) {
                const uint32_t hb = 31 - __clz(lw);
                cand = (32 * tid + hb + 1) << 16 | (incl - pc + __popc(fw & ((2u << hb) - 1u)));
            }
            if (fw) {
                const uint32_t hb = 31 - __clz(fw);
                tl = 1 + ((32 * tid + hb) << 1 | ((lw >> hb) & 1u));
            }
            cand = fr_wave_max(cand);
            tl = fr_wave_max(tl);
            const uint32_t nl = fr_wave_sum(__popc(lw));
            if (lane == 63) ws[wv] = FrWaveStat{incl, nl, cand, tl};
        }
        __syncthreads();   // ws; bitmaps read
        if (tid < 128) fb[tid] = 0; else lb[tid - 128] = 0;
        const FrWaveStat w0 = ws[0], w1 = ws[1];
        const uint32_t tnf = w0.nfrag + w1.nfrag, tnl = w0.nlast + w1.nlast;
        uint32_t lp = 0, up = 0;
        if (w1.cand) { lp = w1.cand >> 16; up = (w1.cand & 0xffffu) + w0.nfrag; }
        else if (w0.cand) { lp = w0.cand >> 16; up = w0.cand & 0xffffu; }
        const uint32_t tlp = max(w0.tail, w1.tail);
        const uint32_t tl = tlp ? (tlp - 1) & 1u : tail;
        info.nfrag = tnf;
        info.nlast = tnl;
        if (lp) {
            info.has_ll = 1;
            info.upto_ll = up;
            has_ll = 1;
            lastlast = pre_f + up;
        }
        if (tid == 0) sub[sj] = info;
        e = e_next;
        tail = tl;
        pre_f += tnf;
        pre_l += tnl;
    }
    if (tid == 0) {
        FrameSuper v;
        v.nfrag = pre_f;
        v.nlast = pre_l;
        v.tail = tail;
        v.has_ll = has_ll;
        v.upto_ll = lastlast;
        sup[s] = v;
    }
}

// ---------------------------------------------------------------------------
// k_fr_bases: super-chunk exclusive prefixes (fragments, LAST flags, the LAST
// flag of the fragment before each super-chunk) and the batch totals:
// res[1] = complete fragments (through the last LAST one), res[4] = complete
// messages, res[5] = fragments of the first `cap` messages (k_fr_emit lowers
// it), res[3] = consumed stream bytes (set by k_fr_emit).
// ---------------------------------------------------------------------------
// Super-chunks at or past nv are off the real chain (the speculative walk's
// supers after its terminal) and count as empty; bases[] is written for all.
__device__ __forceinline__ void fr_bases_block(const FrameSuper *sup, uint64_t nsup, uint64_t nv, FrameBase *bases,
                                               uint64_t *res) {
    // thread t takes the run of super-chunks [t R, t R + R): its sums and
    // "last non-empty tail" in registers, one block scan of the runs, then the
    // run again with the carried prefix
    __shared__ uint64_t sf[1024], sl[1024];
    __shared__ uint32_t st[1024];
    __shared__ uint64_t fc;
    const uint32_t tid = threadIdx.x;
    if (tid == 0) fc = 0;
    const FrameSuper none = {0, 0, 2, 0, 0};
    auto get = [&](uint64_t s) { return s < nv ? sup[s] : none; };
    const uint64_t R = (nsup + 1023) / 1024;
    const uint64_t s0 = tid * R, s1 = min(s0 + R, nsup);
    uint64_t f = 0, l = 0;
    uint32_t t = 2u;
    constexpr int kRun = 12;   // runs up to this long load at once (registers)
    FrameSuper run[kRun];
    if (R <= kRun) {
#pragma unroll
        for (int i = 0; i < kRun; ++i)
            if (s0 + i < s1) run[i] = get(s0 + i);
#pragma unroll
        for (int i = 0; i < kRun; ++i)
            if (s0 + i < s1) {
                f += run[i].nfrag;
                l += run[i].nlast;
                if (run[i].nfrag) t = run[i].tail;
            }
    } else {
        for (uint64_t s = s0; s < s1; ++s) {
            const FrameSuper v = get(s);
            f += v.nfrag;
            l += v.nlast;
            if (v.nfrag) t = v.tail;
        }
    }
    sf[tid] = f;
    sl[tid] = l;
    st[tid] = t;
    __syncthreads();
    for (uint32_t d = 1; d < 1024; d <<= 1) {   // inclusive scans: sums, "last non-empty tail"
        const uint64_t af = tid >= d ? sf[tid - d] : 0, al = tid >= d ? sl[tid - d] : 0;
        const uint32_t at = tid >= d ? st[tid - d] : 2u;
        __syncthreads();
        sf[tid] += af;
        sl[tid] += al;
        if (st[tid] == 2u) st[tid] = at;
        __syncthreads();
    }
    uint64_t cf = sf[tid] - f, cl = sl[tid] - l;
    uint32_t ct = tid ? st[tid - 1] : 2u;
    if (ct == 2u) ct = 1u;   // fragment 0 starts a message
    uint64_t best = 0;
    auto emit = [&](uint64_t s, const FrameSuper &v) {
        FrameBase o;
        o.frag = cf;
        o.last = cl;
        o.prev_tail = ct;
        o.rsv = 0;
        bases[s] = o;
        if (v.has_ll) best = max(best, (uint64_t)(cf + v.upto_ll));
        cf += v.nfrag;
        cl += v.nlast;
        if (v.nfrag) ct = v.tail;
    };
    if (R <= kRun) {
#pragma unroll
        for (int i = 0; i < kRun; ++i)
            if (s0 + i < s1) emit(s0 + i, run[i]);
    } else {
        for (uint64_t s = s0; s < s1; ++s) emit(s, get(s));
    }
    if (best) atomicMax((unsigned long long *)&fc, (unsigned long long)best);
    __syncthreads();
    if (tid == 0) {
        res[1] = fc;            // complete fragments: through the last LAST fragment
        res[4] = sl[1023];      // complete messages
        res[5] = fc;
        res[3] = 0;
        res[6] = 0;             // k_fr_emit: a message offset off the expected stride
    }
}
__global__ __launch_bounds__(1024) void k_fr_bases(const FrameSuper *sup, uint64_t nsup, FrameBase *bases,
                                                    uint64_t *res) {
    if (threadIdx.x == 0) res[7] = 0;   // (a speculative walk that gave up may have set it)
    if (res[0] == kFUnal) return;       // block-uniform
    fr_bases_block(sup, nsup, nsup, bases, res);
}

// ---------------------------------------------------------------------------
// k_fr_emit: block (128 threads, two waves) per sub-chunk, thread t owns
// bitmap word t.
// frag_pos (xdrg_deframe only): stream offset of every fragment of the first
// `cap` messages, plus the entry after the last one (the next fragment's
// offset, or the end of the last complete message) so k_fr_copy reads body
// sizes as gaps.
// ---------------------------------------------------------------------------
template <int B>
__device__ __forceinline__ void fr_emit_sub(const uint32_t *__restrict__ w, uint32_t Q, const FrameSub *sub,
                                            const FrameBase *bases, const uint32_t *fbits, const uint32_t *lbits,
                                            uint64_t cap, int stream_offsets, uint64_t *msg_offsets,
                                            uint64_t *frag_pos, uint64_t *res, uint64_t F, uint64_t M, uint64_t k,
                                            uint64_t stride, uint16_t *so, uint32_t (&wsum)[2][2],
                                            uint32_t (&wtail)[2], uint32_t (&wlo)[2], uint32_t (&whi)[2]) {
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint64_t s = k / (kFSuper / kFChunk);
    // every load issued before the first test: the workspace arrays cover the
    // whole grid (frame_ws), so a sub-chunk skipped here read in-bounds words only
    const FrameSub info = sub[k];
    const FrameBase b = bases[s];
    const uint32_t fw = fbits[k * 128 + tid], lw = lbits[k * 128 + tid];
    if (k * kFChunk >= Q) return;
    if (!info.nfrag) return;
    const uint64_t fb0 = b.frag + info.pre_frag, lb0 = b.last + info.pre_last;
    if (fb0 >= F) return;                          // past the last complete message
    const uint32_t in_tail = info.prev_tail != 2u ? info.prev_tail : b.prev_tail;
    // exclusive prefixes over the block's words (wave scans + one barrier),
    // and the LAST flag of the fragment before each word ("last non-empty")
    uint32_t cf = __popc(fw), cl = __popc(lw);
    uint32_t lt = fw ? 1 + (tid << 1 | ((lw >> (31 - __clz(fw))) & 1u)) : 0u;   // max = the latest
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t a1 = __shfl_up(cf, d, 64), a2 = __shfl_up(cl, d, 64), a3 = __shfl_up(lt, d, 64);
        if (lane >= (uint32_t)d) { cf += a1; cl += a2; lt = max(lt, a3); }
    }
    if (lane == 63) { wsum[wv][0] = cf; wsum[wv][1] = cl; wtail[wv] = lt; }
    __syncthreads();
    const uint32_t pf_incl = cf + (wv ? wsum[0][0] : 0u), pl_incl = cl + (wv ? wsum[0][1] : 0u);
    uint32_t lt_excl = __shfl_up(lt, 1, 64);
    if (lane == 0) lt_excl = 0;
    if (wv) lt_excl = max(lt_excl, wtail[0]);
    uint64_t f = fb0 + pf_incl - __popc(fw);
    uint64_t m = lb0 + pl_incl - __popc(lw);
    uint32_t prev_last = lt_excl ? (lt_excl - 1) & 1u : in_tail;
    const uint64_t base = k * kFChunk;
    // message starts (m in [lb0, lb0 + LAST flags]) go through LDS as 16-bit
    // offsets from the sub-chunk, then out coalesced
    const uint64_t mlim = min(M, cap + 1);   // msg_offsets[m] is written for m < mlim
    uint32_t klo = ~0u, khi = 0;
    for (uint32_t bits = fw; bits; bits &= bits - 1) {
        if (f >= F) break;
        const uint32_t bt = __ffs(bits) - 1;
        const uint32_t lp = 32 * tid + bt;
        const uint64_t p = B * (base + lp);   // stream byte of the mark
        const bool last = (lw >> bt) & 1;
        const bool first = f == 0 || prev_last;
        if (first && m < mlim) {   // payload offsets: fragments tile the stream (p - 4 f)
            const uint32_t kk = (uint32_t)(m - lb0);
            so[kk] = (uint16_t)(stream_offsets ? B * lp : B * lp - 4 * (uint32_t)(f - fb0));
            klo = min(klo, kk);
            khi = max(khi, kk + 1);
        }
        if (first && m == cap) { res[3] = p; res[5] = f; }   // handleRead's split point (:57-60)
        if (frag_pos && m <= cap) frag_pos[f] = p;
        if (f + 1 == F) {   // the last LAST fragment closes the last complete message
            const uint64_t size = fr_bswap(fr_at<B>(w, Q, (uint32_t)(base + lp))) & kSizeMask;
            if (m + 1 <= cap) msg_offsets[m + 1] = stream_offsets ? p + 4 + size : p - 4 * f + size;
            if (M <= cap) {
                res[3] = p + 4 + size;
                if (frag_pos) frag_pos[F] = p + 4 + size;
            }
        }
        prev_last = last;
        m += last;
        ++f;
    }
    klo = fr_wave_min(klo);
    khi = fr_wave_max(khi);
    if (lane == 0) { wlo[wv] = klo; whi[wv] = khi; }
    __syncthreads();
    klo = min(wlo[0], wlo[1]);
    khi = max(whi[0], whi[1]);
    const uint64_t vbase = stream_offsets ? B * base : B * base - 4 * fb0;
    bool off_stride = false;   // stride > 0: message m should start at m * stride (the receive's fixed-size decode)
    for (uint32_t kk = klo + tid; kk < khi; kk += 128) {
        const uint64_t o = vbase + so[kk];
        msg_offsets[lb0 + kk] = o;
        off_stride |= stride && o != (lb0 + kk) * stride;
    }
    if (__ballot(off_stride) && lane == 0) atomicOr((unsigned long long *)(res + 6), 1ull);
    __syncthreads();   // so / wsum / wlo free for the block's next sub-chunk
}

template <int B>
__global__ __launch_bounds__(128) void k_fr_emit(const uint32_t *__restrict__ w, uint32_t Q, const FrameSub *sub,
                                                  const FrameBase *bases, const uint32_t *fbits,
                                                  const uint32_t *lbits, uint64_t cap, int stream_offsets,
                                                  uint64_t *msg_offsets, uint64_t *frag_pos, uint64_t *res,
                                                  uint64_t nsub, uint32_t per, uint64_t stride) {
    __shared__ uint32_t wsum[2][2], wtail[2], wlo[2], whi[2];
    __shared__ uint16_t so[kFChunk + 1];           // staged message offsets
    const uint64_t r0 = res[0], F = res[1], M = res[4];
    if (r0 == kFUnal || (res[7] & 3)) return;   // byte walk next, the walk's checks failed or it gave up
    // `per` consecutive sub-chunks per block (fewer, longer blocks: the
    // per-sub-chunk work is a few hundred stores)
    const uint64_t k0 = (uint64_t)blockIdx.x * per;
    const uint64_t k1 = min(k0 + per, nsub);
    for (uint64_t k = k0; k < k1; ++k)
        fr_emit_sub<B>(w, Q, sub, bases, fbits, lbits, cap, stream_offsets, msg_offsets, frag_pos, res, F, M, k,
                       stride, so, wsum, wtail, wlo, whi);
}

// k_fr_emit_w: the same results from one wave per sub-chunk, lane l owning
// bitmap words 2 l and 2 l + 1 (positions 64 l .. 64 l + 63): no cross-wave
// exchange, and the per-fragment loop in 32-bit sub-chunk-relative counters
// (fragment and message indices relative to fb0 / lb0, limits clamped).
__device__ __forceinline__ uint32_t fr_wave_incl_max(uint32_t v) {
    const uint32_t lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t a = __shfl_up(v, d, 64);
        if (lane >= (uint32_t)d) v = max(v, a);
    }
    return v;
}
__device__ __forceinline__ uint32_t fr_rel(uint64_t x, uint64_t base) {   // x - base clamped to [0, 2^32 - 1]
    return x <= base ? 0u : x - base >= 0xffffffffull ? 0xffffffffu : (uint32_t)(x - base);
}
template <int B>
__device__ __forceinline__ void fr_emit_wave(const uint32_t *__restrict__ w, uint32_t Q, const FrameSub *sub,
                                             const FrameBase *bases, const uint64_t *fb64, const uint64_t *lb64,
                                             uint64_t cap, int stream_offsets, uint64_t *msg_offsets,
                                             uint64_t *frag_pos, uint64_t *res, uint64_t F, uint64_t M, uint64_t k,
                                             uint64_t stride, uint16_t *so) {
    const uint32_t l = threadIdx.x & 63;
    const uint64_t s = k / (kFSuper / kFChunk);
    const FrameSub info = sub[k];
    const FrameBase b = bases[s];
    const uint64_t Fl = fb64[k * 64 + l], Ll = lb64[k * 64 + l];
    if (k * kFChunk >= Q || !info.nfrag) return;
    const uint64_t fb0 = b.frag + info.pre_frag, lb0 = b.last + info.pre_last;
    if (fb0 >= F) return;   // past the last complete message
    const uint32_t in_tail = info.prev_tail != 2u ? info.prev_tail : b.prev_tail;
    const uint32_t pf = __popcll(Fl), pl = __popcll(Ll);
    uint32_t rf = fr_wave_incl(pf) - pf, rm = fr_wave_incl(pl) - pl;   // relative f, m of the lane's first
    // the LAST flag of the fragment before the lane's first: the latest lane below with one
    const uint32_t tag = Fl ? 1u + (l << 1 | (uint32_t)((Ll >> (63 - __builtin_clzll(Fl))) & 1u)) : 0u;
    uint32_t tex = __shfl_up(fr_wave_incl_max(tag), 1, 64);
    if (l == 0) tex = 0;
    bool prev_last = tex ? ((tex - 1) & 1u) != 0 : in_tail != 0;
    const uint64_t mlim = min(M, cap + 1);           // msg_offsets[m] is written for m < mlim
    const uint32_t rF = fr_rel(F, fb0), rmlim = fr_rel(mlim, lb0);
    const bool capin = cap >= lb0;                    // m == cap / m <= cap possible in this sub-chunk
    const uint32_t rcap = capin ? fr_rel(cap, lb0) : 0u;
    const bool first0 = fb0 == 0;
    const uint64_t base = k * kFChunk;
    uint32_t klo = ~0u, khi = 0;
    for (uint64_t bits = Fl; bits; bits &= bits - 1) {
        if (rf >= rF) break;
        const uint32_t bt = (uint32_t)__builtin_ctzll(bits);
        const uint32_t lp = 64 * l + bt;
        const bool last = (Ll >> bt) & 1ull;
        const bool first = prev_last || (first0 && rf == 0);
        if (first && rm < rmlim) {   // payload offsets: fragments tile the stream (p - 4 f)
            so[rm] = (uint16_t)(stream_offsets ? B * lp : B * lp - 4 * rf);
            klo = min(klo, rm);
            khi = max(khi, rm + 1);
        }
        if (capin && rm <= rcap) {
            const uint64_t p = B * (base + lp);   // stream byte of the mark
            if (first && rm == rcap) { res[3] = p; res[5] = fb0 + rf; }   // handleRead's split point (:57-60)
            if (frag_pos) frag_pos[fb0 + rf] = p;
        }
        if (rf + 1 == rF) {   // the last LAST fragment closes the last complete message
            const uint64_t p = B * (base + lp), f = fb0 + rf, m = lb0 + rm;
            const uint64_t size = fr_bswap(fr_at<B>(w, Q, (uint32_t)(base + lp))) & kSizeMask;
            if (m + 1 <= cap) msg_offsets[m + 1] = stream_offsets ? p + 4 + size : p - 4 * f + size;
            if (M <= cap) {
                res[3] = p + 4 + size;
                if (frag_pos) frag_pos[F] = p + 4 + size;
            }
        }
        prev_last = last;
        rm += last ? 1u : 0u;
        ++rf;
    }
    klo = fr_wave_min(klo);
    khi = fr_wave_max(khi);
    sp_fence();
    const uint64_t vbase = stream_offsets ? B * base : B * base - 4 * fb0;
    bool off_stride = false;   // stride > 0: message m should start at m * stride (the receive's fixed-size decode)
    for (uint32_t kk = klo + l; kk < khi; kk += 64) {
        const uint64_t o = vbase + so[kk];
        msg_offsets[lb0 + kk] = o;
        off_stride |= stride && o != (lb0 + kk) * stride;
    }
    if (__ballot(off_stride) && l == 0) atomicOr((unsigned long long *)(res + 6), 1ull);
    sp_fence();   // so free for the block's next sub-chunk
}

template <int B>
__global__ __launch_bounds__(64) void k_fr_emit_w(const uint32_t *__restrict__ w, uint32_t Q, const FrameSub *sub,
                                                  const FrameBase *bases, const uint32_t *fbits,
                                                  const uint32_t *lbits, uint64_t cap, int stream_offsets,
                                                  uint64_t *msg_offsets, uint64_t *frag_pos, uint64_t *res,
                                                  uint64_t nsub, uint32_t per, uint64_t stride) {
    __shared__ uint16_t so[kFChunk + 1];           // staged message offsets
    const uint64_t r0 = res[0], F = res[1], M = res[4];
    if (r0 == kFUnal || (res[7] & 3)) return;
    const uint64_t k0 = (uint64_t)blockIdx.x * per;
    const uint64_t k1 = min(k0 + per, nsub);
    for (uint64_t k = k0; k < k1; ++k)
        fr_emit_wave<B>(w, Q, sub, bases, (const uint64_t *)fbits, (const uint64_t *)lbits, cap, stream_offsets,
                        msg_offsets, frag_pos, res, F, M, k, stride, so);
}
// Emit with the context's variant (tuning key 48: 1 a wave per sub-chunk, 0 k_fr_emit).
template <int B>
static void fr_emit_launch(const uint32_t *w, uint32_t Q, const FrameWs &ws, uint64_t cap, bool stream_offsets,
                           uint64_t *msg_offsets, bool frag_list, int emit_per, int emit_wave, uint64_t stride,
                           uint64_t nsub, hipStream_t st) {
    uint32_t per = emit_per > 0 ? (uint32_t)emit_per : 1u;
    const uint64_t minb = emit_wave ? 256 : 64;   // keep the grid wide for short streams
    while (per > 1 && nsub / per < minb) per >>= 1;
    const dim3 grid((uint32_t)((nsub + per - 1) / per));
    if (emit_wave)
        hipLaunchKernelGGL(k_fr_emit_w<B>, grid, dim3(64), 0, st, w, Q, ws.sub, ws.bases, ws.fbits, ws.lbits, cap,
                           stream_offsets ? 1 : 0, msg_offsets, frag_list ? ws.frag_pos : nullptr, ws.res, nsub, per,
                           stream_offsets ? stride : 0ull);
    else
        hipLaunchKernelGGL(k_fr_emit<B>, grid, dim3(128), 0, st, w, Q, ws.sub, ws.bases, ws.fbits, ws.lbits, cap,
                           stream_offsets ? 1 : 0, msg_offsets, frag_list ? ws.frag_pos : nullptr, ws.res, nsub, per,
                           stream_offsets ? stride : 0ull);
}

// ---------------------------------------------------------------------------
// Exact serial walk (any fragment sizes): the fallback.  Same results as the
// parallel path (fragment list with its end entry, message offsets).
// ---------------------------------------------------------------------------
__global__ void k_fr_serial(const uint8_t *in, uint64_t len, uint64_t cap, int stream_offsets,
                            uint64_t *msg_offsets, uint64_t *frag_pos, uint64_t *res) {
    if (threadIdx.x || blockIdx.x) return;
    uint64_t p = 0, n = 0, F = 0, M = 0, endF = 0;
    while (len - p >= 4) {
        const uint32_t mk = ((uint32_t)in[p] << 24) | ((uint32_t)in[p + 1] << 16) | ((uint32_t)in[p + 2] << 8) | in[p + 3];
        const uint64_t size = mk & kSizeMask;
        if (size > len - p - 4) break;
        frag_pos[n++] = p;
        p += 4 + size;
        if (mk & kLastFrag) { F = n; ++M; endF = p; }
    }
    frag_pos[n] = p;
    // messages of the complete fragments (isAllFragmentsArrived :82-85)
    uint64_t m = 0, body = 0, consumed = 0, fcap = F;
    bool first = true;
    for (uint64_t f = 0; f < F; ++f) {
        const uint64_t pos = frag_pos[f], size = frag_pos[f + 1] - pos - 4;
        if (first && m <= cap) {
            if (m < M) msg_offsets[m] = stream_offsets ? pos : body;
            if (m == cap) { consumed = pos; fcap = f; }
        }
        body += size;
        const uint32_t mk = ((uint32_t)in[pos] << 24);
        first = (mk & kLastFrag) != 0;
        if (first) {
            ++m;
            if (m <= cap) msg_offsets[m] = stream_offsets ? pos + 4 + size : body;
        }
    }
    if (M <= cap) consumed = endF;
    res[1] = F;
    res[3] = consumed;
    res[4] = M;
    res[5] = fcap;
}

// A group of G lanes per fragment copies its body (the gap to the next
// fragment minus the mark) to payload[p - 4 f): 16-byte accesses (dword-
// aligned, so unaligned vectors on gfx950) with a dword tail; byte copies
// when a body is not a 4-multiple (serial path).
typedef uint32_t u32x4c __attribute__((ext_vector_type(4), aligned(4)));
__global__ __launch_bounds__(256) void k_fr_copy(const uint8_t *in, const uint64_t *frag_pos, uint64_t nf, uint32_t G,
                                                 uint8_t *payload) {
    const uint32_t gl = threadIdx.x & (G - 1);
    const uint64_t ngroups = (uint64_t)gridDim.x * (blockDim.x / G);
    for (uint64_t f = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / G; f < nf; f += ngroups) {
        const uint64_t p = frag_pos[f];
        const uint64_t n = frag_pos[f + 1] - p - 4;
        const uint8_t *src = in + p + 4;
        uint8_t *dst = payload + (p - 4 * f);
        if ((((uintptr_t)src | (uintptr_t)dst | n) & 3) == 0) {
            const uint64_t nv = n >> 4;
            for (uint64_t i = gl; i < nv; i += G) *(u32x4c *)(dst + 16 * i) = *(const u32x4c *)(src + 16 * i);
            for (uint64_t i = 4 * nv + gl; i < n / 4; i += G) ((uint32_t *)dst)[i] = ((const uint32_t *)src)[i];
        } else {
            for (uint64_t i = gl; i < n; i += G) dst[i] = src[i];
        }
    }
}

// ---------------------------------------------------------------------------
// Speculative walk (word mode, round 6): one read of the stream, chain work
// in proportion to the marks, no per-word exit table.
// ---------------------------------------------------------------------------
// One wave per super-chunk (k_fs_walk), its sub-chunks in order; a sub-chunk
// is a tile of 64 segments of 64 words, lane l owning segment l:
//   1. each lane walks its segment from its first word whose chain leaves the
//      segment plausibly (exit in the next kSpWin words, or exactly at the
//      stream end); words of rejected chains are skipped (same exit).  The
//      accepted chain: its complete words S, their LAST flags, the last word
//      T and the exit X.  Payload read as a mark almost always jumps far, so
//      the accepted chain is normally the real one from the segment's first
//      mark on.
//   2. from the sub-chunk's entry e (exact inside a super-chunk: the previous
//      sub-chunk's exit), the segments the real chain visits are found by
//      binary lifting over the segment successors (lane shuffles): a segment
//      is on the path when its predecessor's exit lands in it, and its
//      landing must lie on its accepted chain (or be its last word).  All
//      landings on their chains: the marks are the chains from the landings
//      on.  Otherwise (rare: a false chain accepted before the landing, a
//      landing on an incomplete last fragment) one exact walk from e that
//      takes a segment's chain wherever the walk meets it.
//   3. bitmaps and counts as k_fr_mark leaves them (k_fr_emit reads both).
// A super-chunk's own entry is the one guess: the exit of the first
// plausible chain through the last kSpHalo words of the previous super-chunk
// (else its first accepted segment chain).  k_fs_fix checks every guess
// against the previous super-chunk's exit (both in sx), walks the first
// wrong one again from its true entry, and repeats, at most kSpFixIters
// times; then the bases.  A stream it cannot settle (fragments longer than a
// super-chunk, bodies of mark-like words everywhere) sets res[7] and is
// walked again by the exact kernels above.
constexpr uint32_t kSpWin = 2048;    // plausible exits: the next kSpWin words past a segment
constexpr uint32_t kSpHalo = 128;    // words of the previous super-chunk walked for the entry guess
constexpr uint32_t kSpNoT = 0xffu;   // a segment without an accepted chain
constexpr int kSpFixIters = 4;
constexpr uint32_t kSpRow = 65;      // LDS words per segment row (one pad word)
struct SpLds {                       // one wave's share (19 KiB)
    uint32_t tile[64 * kSpRow];      // the sub-chunk, segment l in row l (sp_idx)
    uint64_t nS[64], nLM[64];        // accepted chains (the exact walk's shortcuts)
    uint32_t nX[64], nT[64];
    uint32_t fb[128], lb[128];       // the exact walk's bitmaps
};
// Word q of a tile: segment l = q / 64 in row l, kSpRow words apart, so the
// 32 lanes of a half-wave reading offset c of their own segments hit 32
// banks ((65 l + c) % 32), and lane l staging word l of every segment writes
// consecutive banks.
__device__ __forceinline__ uint32_t sp_idx(uint32_t q) { return (q >> 6) * kSpRow + (q & 63u); }
__device__ __forceinline__ uint64_t sp_shfl64(uint64_t v, uint32_t src) {
    const uint32_t lo = __shfl((uint32_t)v, (int)src, 64), hi = __shfl((uint32_t)(v >> 32), (int)src, 64);
    return (uint64_t)hi << 32 | lo;
}
// Loads of a sub-chunk: word base + 64 k + l into y[k] (k < 64), one
// coalesced 256-byte dword load per k, so that lane l holds word l of every
// segment k; words past Q read as 0 (never walked).
__device__ __forceinline__ void sp_load(const uint32_t *w, uint32_t Q, uint32_t base, uint32_t l, uint32_t (&y)[64]) {
    if (base + kFChunk <= Q) {
#pragma unroll
        for (int k = 0; k < 64; ++k) y[k] = __builtin_nontemporal_load(w + base + 64 * k + l);
    } else {
#pragma unroll
        for (int k = 0; k < 64; ++k) {
            const uint32_t q = base + 64 * k + l;
            y[k] = q < Q ? w[q] : 0u;
        }
    }
}
// Stage y into the tile and return this lane's segment's candidate starts:
// bit c = word c of segment l could be a mark whose fragment is shorter than
// 16 KiB (size < 2^14, size % 4 == 0: in the raw big-endian word, bits 0-6,
// 8-15, 22-23 and 24-25 clear).  One ballot per segment k is segment k's
// mask; lane k keeps it.
constexpr uint32_t kSpCandMask = 0x03C0FF7Fu;
template <int K>
__device__ __forceinline__ void sp_stage1(uint32_t *tile, uint32_t l, uint32_t v, uint32_t &lo, uint32_t &hi) {
    tile[kSpRow * K + l] = v;
    const uint64_t b = __ballot((v & kSpCandMask) == 0);
    const uint32_t blo = (uint32_t)b, bhi = (uint32_t)(b >> 32);
    asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(lo) : "s"(blo), "n"(K));
    asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(hi) : "s"(bhi), "n"(K));
}
template <int... K>
__device__ __forceinline__ uint64_t sp_stage_seq(uint32_t *tile, uint32_t l, const uint32_t (&y)[64],
                                                 std::integer_sequence<int, K...>) {
    uint32_t lo = 0, hi = 0;
    (sp_stage1<K>(tile, l, y[K], lo, hi), ...);
    return (uint64_t)hi << 32 | lo;
}
__device__ __forceinline__ uint64_t sp_stage(uint32_t *tile, uint32_t l, const uint32_t (&y)[64]) {
    return sp_stage_seq(tile, l, y, std::make_integer_sequence<int, 64>{});
}

// A lane's segment chain: candidate starts in order, the words of a
// rejected chain dropped with it (they share its exit).
// INTERIOR (the sub-chunk ends kSpWin words or more before the stream's end):
// every next mark that stays in the segment or exits plausibly is inside the
// stream, so no fit test.
template <bool INTERIOR>
__device__ __forceinline__ void sp_lane_walk(const uint32_t *tile, uint32_t l, uint32_t gsb, uint32_t nval,
                                             uint64_t cand, uint32_t Q, uint32_t tb, uint64_t &S, uint64_t &LM,
                                             uint32_t &X, uint32_t &T, uint32_t &sig) {
    const uint64_t valid = nval >= 64 ? ~0ull : ((1ull << nval) - 1ull);
    uint64_t avail = cand & valid, ms = 0, ml = 0;
    const uint32_t row = l * kSpRow;
    bool act = avail != 0;
    uint32_t c = act ? (uint32_t)__builtin_ctzll(avail) : 0u, cur = c;
    // The loop follows each lane's chain one mark a step (lean: a mark that
    // stays in the segment is the common step); a chain's end, taken or
    // rejected, is handled under a wave-uniform branch.  Rejected: its words
    // share its exit, so the walk resumes at the next candidate past them.
    while (__ballot(act)) {
        const uint32_t m = fr_bswap(tile[row + cur]);
        bool cm;
        uint32_t d;
        if (INTERIOR) {
            cm = (m & 3u) == 0;
            d = cur + 1 + ((m >> 2) & 0x1fffffffu);
        } else {
            const uint32_t nx = fr_next<4>(m, gsb + cur, Q, tb);
            cm = nx < kFUnal;
            d = nx - gsb;
        }
        const uint64_t bit = act && cm ? 1ull << cur : 0ull;
        ms |= bit;
        ml |= (m >> 31) ? bit : 0ull;
        const bool cont = act && cm && d < nval;
        const bool end = act && !cont;
        if (__ballot(end)) {
            const bool take = end && cm && (gsb + d == Q || (d >= 64 && d - 64 < kSpWin));
            if (take) {
                S = ms;
                LM = ml;
                X = gsb + d;
                T = cur;
                sig = c;
            }
            const bool rej = end && !take;
            avail = rej ? avail & ~(ms | (1ull << cur)) & ~((2ull << c) - 1ull) : avail;
            const uint32_t nc = avail ? (uint32_t)__builtin_ctzll(avail) : 0u;
            c = rej ? nc : c;
            ms = rej ? 0ull : ms;
            ml = rej ? 0ull : ml;
            act = act && !take && !(rej && !avail);
            cur = rej ? nc : cur;
        }
        cur = cont ? d : cur;
    }
}

// The wave's walk of super-chunk s (lane = threadIdx.x % 64).  given: the
// entry is gent (a re-walk from k_fs_fix); else 0 for s = 0 and guessed for
// the others.  Writes the 16 FrameSub of s, the bitmaps of its sub-chunks
// with marks, sup[s] and sx[2 s] = entry (kFNone: none found), sx[2 s + 1] =
// exit (the first chain word past the super-chunk, or a terminal).
struct SpRec {                       // a run of super-chunks (k_fs_walk's look-back)
    uint64_t nf, nl, up;             // complete fragments, LAST ones, fragments through the last LAST one
    uint32_t E, X;                   // the first one's entry, the last one's exit
    uint32_t fl;                     // kSpTail bits: LAST flag of the last fragment (2: none); kSpHas ..
};
constexpr uint32_t kSpTail = 3u, kSpHas = 4u, kSpTerm = 8u, kSpFail = 16u, kSpEmpty = 32u;
__device__ __forceinline__ SpRec fs_super(const uint32_t *__restrict__ w, uint32_t Q, uint32_t tb, uint32_t s, bool given,
                         uint32_t gent, FrameSub *sub, uint32_t *fbits, uint32_t *lbits, FrameSuper *sup,
                         uint32_t *sx, SpLds *sp) {
    const uint32_t l = threadIdx.x & 63;
    uint32_t *const tile = sp->tile;
    const uint32_t sbeg = s * kFSuper;
    const uint32_t send = min(sbeg + kFSuper, Q);
    const uint32_t nsub = (send - sbeg + kFChunk - 1) / kFChunk;
    bool known = true;
    uint32_t e = given ? gent : 0u;
    if (!given && s > 0) {
        // the entry guess: chains through the last kSpHalo words of s - 1,
        // lane l from word l, then l + 64; the lowest accepted start's exit
        const uint32_t hb = sbeg - kSpHalo;
        tile[l] = w[hb + l];
        tile[l + 64] = w[hb + l + 64];
        sp_fence();
        uint32_t c = l, cur = l, hx = 0, key = 0xffu;
        bool act = true;
        while (__ballot(act)) {
            if (act) {
                const uint32_t m = fr_bswap(tile[cur]);
                const uint32_t nx = fr_next<4>(m, hb + cur, Q, tb);
                const bool comp = nx < kFUnal;
                const uint32_t d = nx - hb;
                if (comp && d < kSpHalo) {
                    cur = d;
                } else {
                    if (comp && nx - sbeg < kSpWin) {
                        hx = nx;
                        key = c;
                        act = false;
                    } else if (c < 64) {
                        c += 64;
                        cur = c;
                    } else {
                        act = false;
                    }
                }
            }
        }
        const uint32_t kmin = fr_wave_min(key);
        if (kmin != 0xffu) {
            const uint32_t src = __builtin_ctzll(__ballot(key == kmin));
            e = __shfl(hx, (int)src, 64);
        } else {
            known = false;
        }
        sp_fence();
    }
    const uint32_t E0 = known ? e : kFNone;
    uint32_t entry = E0;
    uint32_t pre_f = 0, pre_l = 0, tail = 2, lastlast = 0, has_ll = 0;
    uint32_t y[64];
    sp_load(w, Q, sbeg, l, y);
    const uint64_t sub0 = (uint64_t)s * (kFSuper / kFChunk);
    for (uint32_t j = 0; j < kFSuper / kFChunk; ++j) {
        const uint32_t base = sbeg + j * kFChunk;
        const uint32_t bend = base + kFChunk;
        const uint64_t sj = sub0 + j;
        FrameSub info;
        info.nfrag = info.nlast = info.upto_ll = info.has_ll = info.rsv = 0;
        info.pre_frag = pre_f;
        info.pre_last = pre_l;
        info.prev_tail = tail;
        const bool need = j < nsub && (!known || (e >= base && e < bend && e < Q));
        if (!need) {
            if (j + 1 < nsub) sp_load(w, Q, base + kFChunk, l, y);
            if (l == 0) sub[sj] = info;
            continue;
        }
        const uint64_t cand = sp_stage(tile, l, y);
        if (j + 1 < nsub) sp_load(w, Q, base + kFChunk, l, y);
        sp_fence();
        // 1. the segment's accepted chain: candidate starts in order, the
        // words of a rejected chain dropped with it (they share its exit)
        const uint32_t gsb = base + 64 * l;
        const uint32_t nval = Q > gsb ? min(Q - gsb, 64u) : 0u;
        uint64_t S = 0, LM = 0;
        uint32_t X = 0, T = kSpNoT, sig = 0;
        if ((uint64_t)bend + kSpWin <= Q)
            sp_lane_walk<true>(tile, l, gsb, nval, cand, Q, tb, S, LM, X, T, sig);
        else
            sp_lane_walk<false>(tile, l, gsb, nval, cand, Q, tb, S, LM, X, T, sig);
        const bool acc = T != kSpNoT;
        if (!known) {   // no guess yet: the first accepted chain of this sub-chunk
            const uint64_t am = __ballot(acc);
            if (!am) {
                if (l == 0) sub[sj] = info;
                sp_fence();
                continue;
            }
            const uint32_t ka = __builtin_ctzll(am);
            e = base + 64 * ka + __shfl(sig, (int)ka, 64);
            entry = e;
            known = true;
        }
        // 2. the path from e
        const uint32_t el = e - base, ke = el >> 6;
        const uint32_t succ = acc && X < Q && X < bend ? (X - base) >> 6 : 64u;
        uint32_t J[6];
        J[0] = succ;
#pragma unroll
        for (int r = 1; r < 6; ++r) {
            const uint32_t t = __shfl(J[r - 1], (int)(J[r - 1] & 63u), 64);
            J[r] = J[r - 1] < 64 ? t : 64u;
        }
        uint32_t p = ke;   // the last path segment before l (for l > ke)
#pragma unroll
        for (int r = 5; r >= 0; --r) {
            const uint32_t n = __shfl(J[r], (int)p, 64);
            if (n + 1 <= l) p = n;
        }
        const uint32_t sp_ = __shfl(succ, (int)p, 64), xp = __shfl(X, (int)p, 64);
        const bool on = l == ke || (l > ke && sp_ == l);
        const uint32_t lam = l == ke ? (el & 63u) : xp - gsb;
        bool ok = true;
        if (on) ok = acc && (((S >> lam) & 1ull) || lam == T);
        uint64_t F, Lb;
        uint32_t exitv;
        if (__ballot(!ok) == 0) {
            F = on ? S & (~0ull << lam) : 0ull;
            Lb = F & LM;
            const uint64_t onm = __ballot(on);
            exitv = __shfl(X, 63 - __builtin_clzll(onm), 64);
        } else {
            // the exact walk from e, through accepted chains where it meets them
            sp->nS[l] = S;
            sp->nLM[l] = LM;
            sp->nX[l] = X;
            sp->nT[l] = acc ? T : kSpNoT;
            sp->fb[l] = 0;
            sp->fb[l + 64] = 0;
            sp->lb[l] = 0;
            sp->lb[l + 64] = 0;
            sp_fence();
            uint32_t x = e;
            while (x < bend && x < Q) {
                const uint32_t q = x - base, k = q >> 6, lm = q & 63u;
                const uint32_t Tk = sp->nT[k];
                const uint64_t Sk = sp->nS[k];
                if (Tk != kSpNoT && (((Sk >> lm) & 1ull) || lm == Tk)) {
                    const uint64_t f = Sk & (~0ull << lm), lf = f & sp->nLM[k];
                    if (l == 0) {
                        sp->fb[2 * k] |= (uint32_t)f;
                        sp->fb[2 * k + 1] |= (uint32_t)(f >> 32);
                        sp->lb[2 * k] |= (uint32_t)lf;
                        sp->lb[2 * k + 1] |= (uint32_t)(lf >> 32);
                    }
                    x = sp->nX[k];
                } else {
                    const uint32_t m = fr_bswap(tile[sp_idx(q)]);
                    const uint32_t nx = fr_next<4>(m, x, Q, tb);
                    if (nx < kFUnal && l == 0) {
                        sp->fb[q >> 5] |= 1u << (q & 31);
                        if (m >> 31) sp->lb[q >> 5] |= 1u << (q & 31);
                    }
                    x = nx;
                }
                sp_fence();
            }
            exitv = x;
            F = (uint64_t)sp->fb[2 * l + 1] << 32 | sp->fb[2 * l];
            Lb = (uint64_t)sp->lb[2 * l + 1] << 32 | sp->lb[2 * l];
            sp_fence();
        }
        // 3. bitmaps and counts
        ((uint64_t *)fbits)[sj * 64 + l] = F;
        ((uint64_t *)lbits)[sj * 64 + l] = Lb;
        const uint32_t pf = __popcll(F), pl = __popcll(Lb);
        const uint32_t incl = fr_wave_incl(pf);
        const uint32_t nf = __shfl(incl, 63, 64);
        const uint32_t nl = fr_wave_sum(pl);
        const uint64_t lmask = __ballot(Lb != 0), fmask = __ballot(F != 0);
        uint32_t upto = 0, tl = 2;
        if (lmask) {
            const uint32_t hl = 63 - __builtin_clzll(lmask);
            uint32_t v = 0;
            if (Lb) {
                const uint32_t bl = 63 - __builtin_clzll(Lb);
                v = incl - pf + __popcll(F & (bl == 63 ? ~0ull : (2ull << bl) - 1ull));
            }
            upto = __shfl(v, (int)hl, 64);
        }
        if (fmask) {
            const uint32_t hf = 63 - __builtin_clzll(fmask);
            const uint32_t tv = F ? (uint32_t)(Lb >> (63 - __builtin_clzll(F))) & 1u : 0u;
            tl = __shfl(tv, (int)hf, 64);
        }
        info.nfrag = nf;
        info.nlast = nl;
        if (nl) {
            info.has_ll = 1;
            info.upto_ll = upto;
            has_ll = 1;
            lastlast = pre_f + upto;
        }
        if (l == 0) sub[sj] = info;
        pre_f += nf;
        pre_l += nl;
        if (nf) tail = tl;
        e = exitv;
        sp_fence();
    }
    const uint32_t X = known ? e : kFNone;
    if (l == 0) {
        FrameSuper v;
        v.nfrag = pre_f;
        v.nlast = pre_l;
        v.tail = tail;
        v.has_ll = has_ll;
        v.upto_ll = lastlast;
        sup[s] = v;
        sx[2 * (uint64_t)s] = entry;
        sx[2 * (uint64_t)s + 1] = X;
    }
    SpRec r;
    r.nf = pre_f;
    r.nl = pre_l;
    r.up = lastlast;
    r.E = entry;
    r.X = X;
    r.fl = tail | (has_ll ? kSpHas : 0u) | (X >= kFUnal || X >= Q ? kSpTerm : 0u);
    return r;
}

// ---- the walk's look-back: each super-chunk's bases and the entry checks --
// A run's record: its counts, first entry, last exit and whether it stops (a
// terminal or the stream's end: later super-chunks are off the chain; a
// failed check: the speculative results are void).  Records combine in
// stream order (associative): a stopped left run absorbs the right one; else
// the right run's entry must be the left run's exit, landing in the right
// run's first super-chunk r0.
__device__ __forceinline__ SpRec sp_combine(const SpRec &L, const SpRec &R, uint32_t r0) {
    if (L.fl & kSpEmpty) return R;
    if (R.fl & kSpEmpty) return L;
    if (L.fl & (kSpTerm | kSpFail)) return L;
    SpRec o = L;
    if (!(R.E == L.X && (uint64_t)L.X < (uint64_t)r0 * kFSuper + kFSuper)) {
        o.fl |= kSpFail;
        return o;
    }
    const uint32_t rt = R.fl & kSpTail;
    o.X = R.X;
    o.nf = L.nf + R.nf;
    o.nl = L.nl + R.nl;
    o.up = (R.fl & kSpHas) ? L.nf + R.up : L.up;
    o.fl = (rt != 2u ? rt : (L.fl & kSpTail)) | ((L.fl | R.fl) & kSpHas) | (R.fl & (kSpTerm | kSpFail));
    return o;
}
__device__ __forceinline__ SpRec sp_shfl_rec(const SpRec &r, uint32_t src) {
    SpRec o;
    o.nf = sp_shfl64(r.nf, src);
    o.nl = sp_shfl64(r.nl, src);
    o.up = sp_shfl64(r.up, src);
    o.E = __shfl(r.E, (int)src, 64);
    o.X = __shfl(r.X, (int)src, 64);
    o.fl = __shfl(r.fl, (int)src, 64);
    return o;
}
// Five tagged words per super-chunk (flag in bits 62-63: 1 its own record,
// 2 the record of [0, s]), word k of super-chunk s at lbw[k nsup + s], stored
// and polled with agent-scope atomics.  A reader takes a record whose five
// flags agree (an upgrade from own to inclusive is five stores).
__device__ __forceinline__ void sp_put(uint64_t *lbw, uint64_t ns, uint32_t s, const SpRec &r, uint64_t flag) {
    const uint64_t f = flag << 62;
    const uint64_t v[5] = {f | r.X | (uint64_t)(r.fl & 31u) << 32, f | r.nf, f | r.nl, f | r.up, f | r.E};
#pragma unroll
    for (int k = 0; k < 5; ++k) __hip_atomic_store(lbw + k * ns + s, v[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Decoupled look-back over block records (wave 0 of the block): record b
// covers super-chunks [b span, b span + span); publish agg (own), look back
// 64 records at a time down to the nearest inclusive one, waiting only for
// the records up to it (an ordered lane reduction), publish [0, b] and return
// the exclusive prefix.  Every block of the small k_fs_scan grid is resident,
// so the records waited on are being computed.
__device__ __forceinline__ SpRec sp_lookback(const SpRec &agg, uint32_t b, uint32_t nrec, uint32_t span,
                                             uint64_t *lbw) {
    const uint32_t l = threadIdx.x & 63;
    const uint64_t ns = nrec;
    if (l == 0) sp_put(lbw, ns, b, agg, b ? 1u : 2u);
    SpRec P;
    P.nf = P.nl = P.up = 0;
    P.E = P.X = 0;
    P.fl = kSpEmpty;
    if (b) {
        SpRec acc = P;
        uint32_t acc_first = b;   // (records)
        int64_t p0 = (int64_t)b - 1;
        for (;;) {
            const int64_t p = p0 - (int64_t)l;
            uint64_t v[5] = {0, 0, 0, 0, 0};
            uint64_t im;
            for (;;) {
                bool ready = true;
                if (p >= 0) {
#pragma unroll
                    for (int k = 0; k < 5; ++k)
                        v[k] = __hip_atomic_load(lbw + k * ns + (uint64_t)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    const uint64_t f = v[0] >> 62;
                    ready = f != 0;
#pragma unroll
                    for (int k = 1; k < 5; ++k) ready = ready && (v[k] >> 62) == f;
                }
                const uint64_t rm = __ballot(ready);
                im = __ballot(ready && p >= 0 && (v[0] >> 62) == 2);
                const uint64_t below = ~rm ? (1ull << __builtin_ctzll(~rm)) - 1ull : ~0ull;   // the ready prefix
                if ((im & below) || !~rm) {
                    im &= below;
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
            const uint32_t lim = im ? (uint32_t)__builtin_ctzll(im) : (uint32_t)(p0 < 63 ? p0 : 63);
            constexpr uint64_t kV = (1ull << 62) - 1;
            SpRec r;
            r.X = (uint32_t)v[0];
            r.fl = p >= 0 ? (uint32_t)(v[0] >> 32) & 31u : kSpEmpty;
            r.nf = v[1] & kV;
            r.nl = v[2] & kV;
            r.up = v[3] & kV;
            r.E = (uint32_t)v[4];
            for (uint32_t d = 1; d < 64; d <<= 1) {   // lane i: records [p0 - min(i + 2d - 1, lim), p0 - i]
                const SpRec o = sp_shfl_rec(r, (l + d) & 63u);
                if (l + d <= lim) r = sp_combine(o, r, (uint32_t)(p0 - (int64_t)(l + d - 1)) * span);
            }
            const SpRec bb = sp_shfl_rec(r, 0);   // records [p0 - lim, p0]
            acc = sp_combine(bb, acc, acc_first * span);
            acc_first = (uint32_t)(p0 - (int64_t)lim);
            if (im) break;
            p0 -= 64;
        }
        P = acc;
        if (l == 0) sp_put(lbw, ns, b, sp_combine(P, agg, b * span), 2u);
    }
    return P;
}

// The super-chunk records after the walk: a thread per super-chunk (its
// FrameSuper and sx pair), an ordered block scan, the look-back over blocks,
// then bases[s] (the exclusive prefix) and, from the last super-chunk, the
// walk's results (res[7] = 2: some entry check failed, k_fs_fix next).
constexpr uint32_t kSpScan = 256;
__global__ __launch_bounds__(kSpScan) void k_fs_scan(uint32_t Q, uint32_t nsup, const FrameSuper *sup,
                                                      const uint32_t *sx, uint64_t *lbw, FrameBase *bases,
                                                      uint64_t *res) {
    __shared__ SpRec wt[kSpScan / 64];
    __shared__ SpRec bp;
    const uint32_t tid = threadIdx.x, l = tid & 63, wv = tid >> 6;
    const uint32_t b = blockIdx.x, nrec = gridDim.x;
    const uint32_t s = b * kSpScan + tid;
    SpRec r;
    r.fl = kSpEmpty;
    r.nf = r.nl = r.up = 0;
    r.E = r.X = 0;
    if (s < nsup) {
        const FrameSuper v = sup[s];
        const uint2 e = ((const uint2 *)sx)[s];
        r.nf = v.nfrag;
        r.nl = v.nlast;
        r.up = v.upto_ll;
        r.E = e.x;
        r.X = e.y;
        r.fl = (v.tail & kSpTail) | (v.has_ll ? kSpHas : 0u) | (e.y >= kFUnal || e.y >= Q ? kSpTerm : 0u);
    }
    // inclusive scan in the wave (lane i: supers [s - 2d + 1, s] after step d)
    for (uint32_t d = 1; d < 64; d <<= 1) {
        const SpRec o = sp_shfl_rec(r, (l - d) & 63u);
        if (l >= d) r = sp_combine(o, r, s - d + 1);
    }
    if (l == 63) wt[wv] = r;
    __syncthreads();
    SpRec wp;   // waves before this one
    wp.fl = kSpEmpty;
    wp.nf = wp.nl = wp.up = 0;
    wp.E = wp.X = 0;
    for (uint32_t k = 0; k < wv; ++k) wp = sp_combine(wp, wt[k], b * kSpScan + 64 * k);
    const SpRec incl = sp_combine(wp, r, b * kSpScan + 64 * wv);   // supers [b kSpScan, s]
    if (tid == kSpScan - 1) bp = incl;                              // the block's aggregate
    __syncthreads();
    if (wv == 0) {
        const SpRec P = sp_lookback(bp, b, nrec, kSpScan, lbw);
        if (l == 0) wt[0] = P;   // (wave 0 read wt[*] above; the barrier below orders the rest)
    }
    __syncthreads();
    const SpRec P = wt[0];
    // exclusive prefix of s: P + the in-block inclusive of s - 1
    SpRec ex = sp_shfl_rec(incl, (l - 1) & 63u);
    if (l == 0) ex = wp;
    const SpRec E = sp_combine(P, ex, b * kSpScan);
    if (s < nsup) {
        FrameBase fb;
        const uint32_t pt = E.fl & kSpTail;
        fb.frag = E.nf;
        fb.last = E.nl;
        fb.prev_tail = (E.fl & kSpEmpty) || pt == 2u ? 1u : pt;   // fragment 0 starts a message
        fb.rsv = 0;
        bases[s] = fb;
    }
    if (s + 1 == nsup) {
        const SpRec I = sp_combine(P, incl, b * kSpScan);
        res[0] = I.X;          // >= Q, kFStop or kFUnal (the byte walk next)
        res[1] = I.up;         // complete fragments: through the last LAST one
        res[4] = I.nl;         // complete messages
        res[5] = I.up;
        res[3] = 0;
        res[6] = 0;
        res[7] = (I.fl & kSpFail) ? 2u : 0u;
    }
}

// Block = one wave = one super-chunk.
__global__ __launch_bounds__(64) void k_fs_walk(const uint32_t *__restrict__ w, uint32_t Q, uint32_t tb,
                                                FrameSub *sub, uint32_t *fbits, uint32_t *lbits, FrameSuper *sup,
                                                uint32_t *sx) {
    __shared__ SpLds sp;
    (void)fs_super(w, Q, tb, blockIdx.x, false, 0u, sub, fbits, lbits, sup, sx, &sp);
}

// One block: check every super-chunk's entry guess against its predecessor's
// exit, walk the first wrong one again from its true entry (wave 0), repeat;
// then the bases over the super-chunks the real chain reaches (res[0] = the
// chain's end: >= Q, kFStop or kFUnal).  res[7] = re-walks << 8 | 1 when it
// gave up.
__global__ __launch_bounds__(1024) void k_fs_fix(const uint32_t *__restrict__ w, uint32_t Q, uint32_t tb,
                                                 uint32_t nsup, FrameSub *sub, uint32_t *fbits, uint32_t *lbits,
                                                 FrameSuper *sup, uint32_t *sx, FrameBase *bases, uint64_t *res) {
    __shared__ SpLds sp;
    __shared__ uint32_t s_fail, s_term;
    const uint32_t tid = threadIdx.x;
    bool done = false;
    uint32_t term = ~0u;
    int it = 0;
    for (;; ++it) {
        if (tid == 0) {
            s_fail = ~0u;
            s_term = ~0u;
        }
        __syncthreads();
        uint32_t f = ~0u, t = ~0u;
        // thread tid checks super-chunks [s0, s1) (the bases' runs below):
        // super-chunk s against s - 1, the pairs loaded at once (uint2: entry, exit)
        const uint32_t R = (nsup + 1023) / 1024, s0 = tid * R, s1 = min(s0 + R, nsup);
        auto check = [&](uint32_t s, uint2 p, uint32_t Es) {   // p = (entry, exit) of s - 1
            if (p.x == kFNone) return;              // s - 1 has no chain: if the chain reaches it, s - 1 fails
            if (p.y >= kFUnal || p.y >= Q) {        // the chain ends in s - 1
                t = min(t, s);
                return;
            }
            if (!(p.y < s * kFSuper + kFSuper && Es == p.y)) f = min(f, s);
        };
        const uint2 *px = (const uint2 *)sx;
        constexpr uint32_t kRun = 12;
        if (R <= kRun) {
            uint2 pr[kRun + 1];
#pragma unroll
            for (uint32_t i = 0; i <= kRun; ++i)
                if (s0 + i >= 1 && s0 + i - 1 < s1 && i <= R) pr[i] = px[s0 + i - 1];
#pragma unroll
            for (uint32_t i = 1; i <= kRun; ++i)
                if (s0 + i - 1 < s1 && s0 + i - 1 >= 1) check(s0 + i - 1, pr[i - 1], pr[i].x);
        } else {
            for (uint32_t s = max(s0, 1u); s < s1; ++s) check(s, px[s - 1], px[s].x);
        }
        f = fr_wave_min(f);
        t = fr_wave_min(t);
        if ((tid & 63) == 0) {
            if (f != ~0u) atomicMin(&s_fail, f);
            if (t != ~0u) atomicMin(&s_term, t);
        }
        __syncthreads();
        const uint32_t F = s_fail, T = s_term;
        if (F == ~0u || T < F) {
            done = true;
            term = T;
            break;
        }
        if (it == kSpFixIters) break;
        if (tid < 64) (void)fs_super(w, Q, tb, F, true, sx[2 * (uint64_t)(F - 1) + 1], sub, fbits, lbits, sup, sx, &sp);
        __threadfence_block();
        __syncthreads();
    }
    if (!done) {
        if (tid == 0) res[7] = (uint64_t)it << 8 | 1u;
        return;
    }
    const uint32_t nv = min(term, nsup);
    if (tid == 0) {
        res[0] = sx[2 * (uint64_t)(nv - 1) + 1];
        res[7] = (uint64_t)it << 8;
    }
    __syncthreads();
    if (sx[2 * (uint64_t)(nv - 1) + 1] == kFUnal) return;   // the byte walk next (block-uniform)
    fr_bases_block(sup, nsup, nv, bases, res);
}

// ---- launchers -------------------------------------------------------------------
template <int B>
static int frame_launch(const uint8_t *in, uint64_t len, const FrameWs &ws, uint64_t cap, bool stream_offsets,
                        uint64_t *msg_offsets, bool frag_list, int emit_per, int emit_wave, uint64_t stride,
                        hipStream_t st) {
    const uint32_t *w = (const uint32_t *)in;
    const uint32_t Q = frame_positions(len, B), tb = B == 4 ? (uint32_t)(len & 3) : 0u;
    const uint64_t nsup = (Q + kFSuper - 1) / kFSuper, nsub = nsup * (kFSuper / kFChunk);
    const uint64_t ngrp = (nsup + kFixGrp - 1) / kFixGrp;   // <= nsup: k_fr_exits sets every gentry
    hipLaunchKernelGGL(k_fr_exits<B>, dim3((uint32_t)nsup), dim3(256), 0, st, w, Q, tb, ws.exitR, ws.alist, ws.acnt,
                       ws.sentry, ws.gentry, (uint32_t)ngrp);
    const FrExits<B> ex{w, ws.exitR, Q, tb};
    hipLaunchKernelGGL(k_fr_win<B>, dim3((uint32_t)((nsup * kFixWin + 255) / 256)), dim3(256), 0, st, ex,
                       (uint32_t)nsup, ws.wtab);
    hipLaunchKernelGGL(k_fr_fix_grp<B>, dim3((uint32_t)ngrp), dim3(kFixWin), 0, st, ex, ws.wtab, (uint32_t)nsup,
                       ws.gsx, ws.gexit);
    hipLaunchKernelGGL(k_fr_fix_top<B>, dim3(1), dim3(1024), 0, st, ex, ws.gsx, ws.gexit, (uint32_t)ngrp, ws.gentry,
                       ws.res);
    hipLaunchKernelGGL(k_fr_fix_fill<B>, dim3((uint32_t)ngrp), dim3(256), 0, st, ex, ws.wtab, ws.gentry,
                       (uint32_t)nsup, ws.sentry);
    hipLaunchKernelGGL(k_fr_mark<B>, dim3((uint32_t)nsup), dim3(256), 0, st, w, Q, tb, ws.sentry, ws.res, ws.alist,
                       ws.acnt, ws.sub, ws.fbits, ws.lbits, ws.sup);
    hipLaunchKernelGGL(k_fr_bases, dim3(1), dim3(1024), 0, st, ws.sup, nsup, ws.bases, ws.res);
    // several sub-chunks per block, while the grid stays wide (short streams
    // keep their parallelism)
    fr_emit_launch<B>(w, Q, ws, cap, stream_offsets, msg_offsets, frag_list, emit_per, emit_wave, stride, nsub, st);
    return (int)hipGetLastError();
}

int frame_parallel(const uint8_t *in, uint64_t len, int B, const FrameWs &ws, uint64_t cap, bool stream_offsets,
                   uint64_t *msg_offsets, bool frag_list, int emit_per, int emit_wave, uint64_t stride,
                   void *stream) {
    return B == 1 ? frame_launch<1>(in, len, ws, cap, stream_offsets, msg_offsets, frag_list, emit_per, emit_wave,
                                    stride, (hipStream_t)stream)
                  : frame_launch<4>(in, len, ws, cap, stream_offsets, msg_offsets, frag_list, emit_per, emit_wave,
                                    stride, (hipStream_t)stream);
}

int frame_spec(const uint8_t *in, uint64_t len, const FrameWs &ws, uint64_t cap, bool stream_offsets,
               uint64_t *msg_offsets, bool frag_list, int emit_per, int emit_wave, uint64_t stride, bool fix,
               void *stream) {
    const hipStream_t st = (hipStream_t)stream;
    const uint32_t *w = (const uint32_t *)in;
    const uint32_t Q = frame_positions(len, 4), tb = (uint32_t)(len & 3);
    const uint64_t nsup = (Q + kFSuper - 1) / kFSuper, nsub = nsup * (kFSuper / kFChunk);
    if (fix) {   // the walk's checks failed: settle the stream, bases again
        hipLaunchKernelGGL(k_fs_fix, dim3(1), dim3(1024), 0, st, w, Q, tb, (uint32_t)nsup, ws.sub, ws.fbits,
                           ws.lbits, ws.sup, ws.sx, ws.bases, ws.res);
    } else {
        const uint32_t nrec = (uint32_t)((nsup + kSpScan - 1) / kSpScan);
        const hipError_t e = hipMemsetAsync(ws.lbw, 0, 8 * 5 * (size_t)nrec, st);
        if (e != hipSuccess) return (int)e;
        hipLaunchKernelGGL(k_fs_walk, dim3((uint32_t)nsup), dim3(64), 0, st, w, Q, tb, ws.sub, ws.fbits, ws.lbits,
                           ws.sup, ws.sx);
        hipLaunchKernelGGL(k_fs_scan, dim3(nrec), dim3(kSpScan), 0, st, Q, (uint32_t)nsup, ws.sup, ws.sx, ws.lbw,
                           ws.bases, ws.res);
    }
    fr_emit_launch<4>(w, Q, ws, cap, stream_offsets, msg_offsets, frag_list, emit_per, emit_wave, stride, nsub, st);
    return (int)hipGetLastError();
}

int frame_serial(const uint8_t *in, uint64_t len, const FrameWs &ws, uint64_t cap, bool stream_offsets,
                 uint64_t *msg_offsets, void *stream) {
    hipLaunchKernelGGL(k_fr_serial, dim3(1), dim3(64), 0, (hipStream_t)stream, in, len, cap, stream_offsets ? 1 : 0,
                       msg_offsets, ws.frag_pos, ws.res);
    return (int)hipGetLastError();
}

int frame_copy(const uint8_t *in, const FrameWs &ws, uint64_t nf, uint64_t payload_bytes, uint8_t *payload,
               void *stream) {
    if (!nf) return hipSuccess;
    uint32_t G = 1;   // lanes per fragment: ~16 bytes per lane for the average fragment
    while (G < 64 && 16ull * G * nf < payload_bytes) G <<= 1;
    uint64_t blocks = (nf + 256 / G - 1) / (256 / G);
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(k_fr_copy, dim3((uint32_t)blocks), dim3(256), 0, (hipStream_t)stream, in, ws.frag_pos, nf, G,
                       payload);
    return (int)hipGetLastError();
}

}  // namespace xdrg
