// Probe: the config-3 encode copy shape (16 Mi payloads of 4096 B from a
// 16-aligned native column into 4124-B XDR records at +28, a group of 64
// lanes per record, 1024 records per 256-thread block), with the 16-byte
// chunk grid placed three ways:
//  F1 source-aligned grid: aligned 16-B loads, 4-aligned (misaligned) stores
//     (the blob copy of k_enc_place_g: chunk c at blob byte 16c)
//  F2 destination-aligned grid: 4-aligned 16-B loads, aligned stores
//  F3 destination-aligned grid, aligned loads: each lane loads its aligned
//     source vector and takes the words it lacks from the next lane
//     (__shfl_down), aligned stores
// and the decode shape (4124-B XDR records at +28 -> 16-aligned native):
//  G1 4-aligned 16-B loads + the fifth word as a second load (dec_bytes)
//  G2 4-aligned 16-B loads only (no fifth word: the shape when the native
//     destination is 16-aligned and the stream is 4-aligned)
//  G3 aligned loads + __shfl_down for the misaligned words, aligned stores
// Prints ms and GB/s of payload read+write.  hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef uint32_t v4 __attribute__((ext_vector_type(4)));
typedef uint32_t v4w __attribute__((ext_vector_type(4), aligned(4)));

constexpr size_t N = 16u << 20, SREC = 4096, DREC = 4124, DOFF = 28;

__device__ __forceinline__ uint32_t pick(const v4 &a, const v4 &b, uint32_t i) {   // word i of a:b
    const uint32_t x = i == 0 ? a.x : i == 1 ? a.y : i == 2 ? a.z : a.w;
    const uint32_t y = i == 4 ? b.x : i == 5 ? b.y : i == 6 ? b.z : b.w;
    return i < 4 ? x : y;
}

template <int MODE, int RPB = 1024>
__global__ __launch_bounds__(256) void kF(const uint8_t *s, uint8_t *d) {
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (size_t r = (size_t)blockIdx.x * RPB + w; r < ((size_t)blockIdx.x + 1) * RPB && r < N; r += 4) {
        const uint8_t *src = s + r * SREC;
        uint8_t *dst = d + r * DREC + DOFF;
        if (MODE == 1) {   // chunks on the source grid
            for (uint32_t c = lane; c < SREC / 16; c += 64)
                *(v4w *)(dst + 16 * c) = *(const v4 *)(src + 16 * c);
        } else if (MODE == 4) {   // F1, the record's chunks visited from a per-record rotation
            const uint32_t rot = (uint32_t)((r * 37) & (SREC / 16 - 1));
            for (uint32_t i = lane; i < SREC / 16; i += 64) {
                const uint32_t c = (i + rot) & (SREC / 16 - 1);
                *(v4w *)(dst + 16 * c) = *(const v4 *)(src + 16 * c);
            }
        } else if (MODE == 6) {   // F1, the wave's whole record in flight (4 chunks per lane)
            v4 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = *(const v4 *)(src + 16 * (lane + 64 * u));
#pragma unroll
            for (int u = 0; u < 4; ++u) *(v4w *)(dst + 16 * (lane + 64 * u)) = v[u];
        } else if (MODE == 5) {   // F1 with a padded source stride (4096 + 16)
            const uint8_t *sp = s + r * (SREC + 16);
            for (uint32_t c = lane; c < SREC / 16; c += 64)
                *(v4w *)(dst + 16 * c) = *(const v4 *)(sp + 16 * c);
        } else {
            const uint32_t m = (uint32_t)((uintptr_t)dst & 15);   // 0, 4, 8, 12
            uint8_t *A = dst - m;
            const uint32_t nch = (SREC + m + 15) / 16;
            for (uint32_t c0 = 0; c0 < nch; c0 += 64) {
                const uint32_t c = c0 + lane;
                // destination chunk c holds source bytes [16c - m, 16c - m + 16)
                v4 o;
                if (MODE == 2) {
                    const int64_t sb = (int64_t)16 * c - m;
                    const int64_t cl = sb < 0 ? 0 : (sb > (int64_t)SREC - 16 ? (int64_t)SREC - 16 : sb);
                    o = *(const v4w *)(src + cl);
                } else {
                    const int64_t sv = (int64_t)c - 1;   // aligned source vector holding byte 16c - m (m > 0)
                    const uint32_t vi = sv < 0 ? 0 : (sv > (int64_t)(SREC / 16 - 1) ? SREC / 16 - 1 : (uint32_t)sv);
                    const v4 a = *(const v4 *)(src + 16 * vi);
                    v4 b;
                    b.x = __shfl_down(a.x, 1, 64); b.y = __shfl_down(a.y, 1, 64);
                    b.z = __shfl_down(a.z, 1, 64); b.w = __shfl_down(a.w, 1, 64);
                    if (lane == 63) b = *(const v4 *)(src + 16 * (vi + 1 < SREC / 16 ? vi + 1 : vi));
                    const uint32_t sh = m ? 4 - m / 4 : 0;   // first word of the chunk inside a:b
                    o.x = pick(a, b, sh); o.y = pick(a, b, sh + 1); o.z = pick(a, b, sh + 2); o.w = pick(a, b, sh + 3);
                }
                if (c < nch) {
                    if (c > 0 && c + 1 < nch) *(v4 *)(A + 16 * c) = o;
                    else {   // head / tail chunk: only the record's words
                        const int64_t lo = (int64_t)16 * c, hi = lo + 16;
                        for (int t = 0; t < 4; ++t) {
                            const int64_t b = lo + 4 * t;
                            if (b >= m && b < (int64_t)SREC + m && b < hi)
                                ((uint32_t *)(A + 16 * c))[t] = t == 0 ? o.x : t == 1 ? o.y : t == 2 ? o.z : o.w;
                        }
                    }
                }
            }
        }
    }
}

// F8 / G8: the whole block per record (256 lanes, one 16-B chunk each), the
// block's 1024 records in order
template <bool DEC, int U, int RPB = 1024>
__global__ __launch_bounds__(256) void kBlk(const uint8_t *s, uint8_t *d) {
    for (size_t r = (size_t)blockIdx.x * RPB; r < ((size_t)blockIdx.x + 1) * RPB && r < N; r += U) {
        v4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t rr = r + u, c = threadIdx.x;
            v[u] = DEC ? *(const v4w *)(s + rr * DREC + DOFF + 16 * c) : *(const v4 *)(s + rr * SREC + 16 * c);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t rr = r + u, c = threadIdx.x;
            if (DEC) *(v4 *)(d + rr * SREC + 16 * c) = v[u];
            else *(v4w *)(d + rr * DREC + DOFF + 16 * c) = v[u];
        }
    }
}

// F9 / G9: block per record, each block's records N/S apart (S slices)
template <bool DEC, int S>
__global__ __launch_bounds__(256) void kSl(const uint8_t *s, uint8_t *d) {
    for (int k = 0; k < S; ++k) {
        const size_t rr = (size_t)blockIdx.x + (size_t)k * (N / S), c = threadIdx.x;
        if (DEC) *(v4 *)(d + rr * SREC + 16 * c) = *(const v4w *)(s + rr * DREC + DOFF + 16 * c);
        else *(v4w *)(d + rr * DREC + DOFF + 16 * c) = *(const v4 *)(s + rr * SREC + 16 * c);
    }
}

// F7 / G7: flat one-pass grid, one 16-B chunk per lane (the kA shape), the
// chunk's record and offset from its global index (256 chunks per record)
template <bool DEC>
__global__ __launch_bounds__(256) void kFlat(const uint8_t *s, uint8_t *d) {
    for (size_t q = (size_t)blockIdx.x * 256 + threadIdx.x; q < N * 256; q += (size_t)gridDim.x * 256) {
        const size_t r = q >> 8, c = q & 255;
        if (!DEC) *(v4w *)(d + r * DREC + DOFF + 16 * c) = *(const v4 *)(s + r * SREC + 16 * c);
        else *(v4 *)(d + r * SREC + 16 * c) = *(const v4w *)(s + r * DREC + DOFF + 16 * c);
    }
}

template <int MODE, int RPB = 1024>
__global__ __launch_bounds__(256) void kG(const uint8_t *s, uint8_t *d) {
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (size_t r = (size_t)blockIdx.x * RPB + w; r < ((size_t)blockIdx.x + 1) * RPB && r < N; r += 4) {
        const uint8_t *src = s + r * DREC + DOFF;     // 4-aligned
        uint8_t *dst = d + r * SREC;                  // 16-aligned
        if (MODE == 4) {   // G2, the record's chunks visited from a per-record rotation
            const uint32_t rot = (uint32_t)((r * 37) & (SREC / 16 - 1));
            for (uint32_t i = lane; i < SREC / 16; i += 64) {
                const uint32_t c = (i + rot) & (SREC / 16 - 1);
                *(v4 *)(dst + 16 * c) = *(const v4w *)(src + 16 * c);
            }
            continue;
        }
        if (MODE == 5) {   // G2 with a padded destination stride (4096 + 16)
            uint8_t *dp = d + r * (SREC + 16);
            for (uint32_t c = lane; c < SREC / 16; c += 64) *(v4 *)(dp + 16 * c) = *(const v4w *)(src + 16 * c);
            continue;
        }
        if (MODE == 3) {
            const uint32_t m = (uint32_t)((uintptr_t)src & 15);
            const uint8_t *A = src - m;
            for (uint32_t c0 = 0; c0 < SREC / 16; c0 += 64) {
                const uint32_t c = c0 + lane;
                const v4 a = *(const v4 *)(A + 16 * c);           // aligned, may read past the record
                v4 b;
                b.x = __shfl_down(a.x, 1, 64); b.y = __shfl_down(a.y, 1, 64);
                b.z = __shfl_down(a.z, 1, 64); b.w = __shfl_down(a.w, 1, 64);
                if (lane == 63) b = *(const v4 *)(A + 16 * (c + 1));
                const uint32_t sh = m / 4;
                v4 o;
                o.x = pick(a, b, sh); o.y = pick(a, b, sh + 1); o.z = pick(a, b, sh + 2); o.w = pick(a, b, sh + 3);
                *(v4 *)(dst + 16 * c) = o;
            }
        } else {
            for (uint32_t c = lane; c < SREC / 16; c += 64) {
                v4 o = *(const v4w *)(src + 16 * c);
                if (MODE == 1) {   // the fifth-word load (data-dependent use: never true here)
                    const uint32_t q4 = *(const uint32_t *)(src + 16 * c + 16);
                    if (q4 == 0x12345678u && o.x == 0x9abcdef0u) o.y ^= 1u;
                }
                *(v4 *)(dst + 16 * c) = o;
            }
        }
    }
}

int main() {
    uint8_t *s, *d;
    const size_t big = N * DREC + 4096;
    hipMalloc(&s, big); hipMalloc(&d, big);
    hipMemset(s, 1, big); hipMemset(d, 0, big);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    auto timeit = [&](const char *name, auto launch) {
        launch(); hipDeviceSynchronize();
        float best = 1e9;
        for (int it = 0; it < 7; ++it) {
            hipEventRecord(e0); launch(); hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1); if (ms < best) best = ms;
        }
        printf("%-58s %8.3f ms  %7.1f GB/s (payload read+write)\n", name, best, 2.0 * N * SREC / best / 1e6);
    };
    const dim3 grid(N / 1024), blk(256);
    timeit("F1 enc: aligned loads, misaligned stores", [&] { hipLaunchKernelGGL(kF<1>, grid, blk, 0, 0, s, d); });
    timeit("F2 enc: misaligned loads, aligned stores", [&] { hipLaunchKernelGGL(kF<2>, grid, blk, 0, 0, s, d); });
    timeit("F3 enc: aligned loads + shfl, aligned stores", [&] { hipLaunchKernelGGL(kF<3>, grid, blk, 0, 0, s, d); });
    timeit("G1 dec: misaligned loads + 5th word, aligned stores", [&] { hipLaunchKernelGGL(kG<1>, grid, blk, 0, 0, s, d); });
    timeit("G2 dec: misaligned loads, aligned stores", [&] { hipLaunchKernelGGL(kG<2>, grid, blk, 0, 0, s, d); });
    timeit("G3 dec: aligned loads + shfl, aligned stores", [&] { hipLaunchKernelGGL(kG<3>, grid, blk, 0, 0, s, d); });
    timeit("F4 enc: F1 + per-record chunk rotation", [&] { hipLaunchKernelGGL(kF<4>, grid, blk, 0, 0, s, d); });
    timeit("F5 enc: F1 with source stride 4112", [&] { hipLaunchKernelGGL(kF<5>, grid, blk, 0, 0, s, d); });
    timeit("G4 dec: G2 + per-record chunk rotation", [&] { hipLaunchKernelGGL(kG<4>, grid, blk, 0, 0, s, d); });
    timeit("G5 dec: G2 with destination stride 4112", [&] { hipLaunchKernelGGL(kG<5>, grid, blk, 0, 0, s, d); });
    timeit("F6 enc: F1 with 4 chunks per lane in flight", [&] { hipLaunchKernelGGL(kF<6>, grid, blk, 0, 0, s, d); });
    timeit("F7 enc: flat one-pass grid, 1 chunk per lane", [&] { hipLaunchKernelGGL(kFlat<false>, dim3(N / 4), blk, 0, 0, s, d); });
    timeit("G7 dec: flat one-pass grid, 1 chunk per lane", [&] { hipLaunchKernelGGL(kFlat<true>, dim3(N / 4), blk, 0, 0, s, d); });
    timeit("F1 enc, 64 records per block", [&] { hipLaunchKernelGGL((kF<1, 64>), dim3(N / 64), blk, 0, 0, s, d); });
    timeit("F1 enc, 16 records per block", [&] { hipLaunchKernelGGL((kF<1, 16>), dim3(N / 16), blk, 0, 0, s, d); });
    timeit("F6 enc, 16 records per block", [&] { hipLaunchKernelGGL((kF<6, 16>), dim3(N / 16), blk, 0, 0, s, d); });
    timeit("G2 dec, 64 records per block", [&] { hipLaunchKernelGGL((kG<2, 64>), dim3(N / 64), blk, 0, 0, s, d); });
    timeit("G2 dec, 16 records per block", [&] { hipLaunchKernelGGL((kG<2, 16>), dim3(N / 16), blk, 0, 0, s, d); });
    timeit("F8 enc: block per record, 1 record in flight", [&] { hipLaunchKernelGGL((kBlk<false, 1>), grid, blk, 0, 0, s, d); });
    timeit("F8 enc: block per record, 2 records in flight", [&] { hipLaunchKernelGGL((kBlk<false, 2>), grid, blk, 0, 0, s, d); });
    timeit("G8 dec: block per record, 1 record in flight", [&] { hipLaunchKernelGGL((kBlk<true, 1>), grid, blk, 0, 0, s, d); });
    timeit("G8 dec: block per record, 2 records in flight", [&] { hipLaunchKernelGGL((kBlk<true, 2>), grid, blk, 0, 0, s, d); });
    timeit("F8 enc: block per record, 2 records per block", [&] { hipLaunchKernelGGL((kBlk<false, 1, 2>), dim3(N / 2), blk, 0, 0, s, d); });
    timeit("F8 enc: block per record, 8 records per block", [&] { hipLaunchKernelGGL((kBlk<false, 1, 8>), dim3(N / 8), blk, 0, 0, s, d); });
    timeit("F8 enc: block per record, 64 records per block", [&] { hipLaunchKernelGGL((kBlk<false, 1, 64>), dim3(N / 64), blk, 0, 0, s, d); });
    timeit("G8 dec: block per record, 2 records per block", [&] { hipLaunchKernelGGL((kBlk<true, 1, 2>), dim3(N / 2), blk, 0, 0, s, d); });
    timeit("G8 dec: block per record, 8 records per block", [&] { hipLaunchKernelGGL((kBlk<true, 1, 8>), dim3(N / 8), blk, 0, 0, s, d); });
    timeit("F9 enc: block per record, 4 slices N/4 apart", [&] { hipLaunchKernelGGL((kSl<false, 4>), dim3(N / 4), blk, 0, 0, s, d); });
    timeit("F9 enc: block per record, 2 slices N/2 apart", [&] { hipLaunchKernelGGL((kSl<false, 2>), dim3(N / 2), blk, 0, 0, s, d); });
    timeit("F9 enc: block per record, 8 slices N/8 apart", [&] { hipLaunchKernelGGL((kSl<false, 8>), dim3(N / 8), blk, 0, 0, s, d); });
    timeit("G9 dec: block per record, 4 slices N/4 apart", [&] { hipLaunchKernelGGL((kSl<true, 4>), dim3(N / 4), blk, 0, 0, s, d); });
    hipError_t e = hipGetLastError();
    printf("status: %s\n", hipGetErrorString(e));
    return 0;
}
