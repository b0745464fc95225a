// Probe: copy bandwidth of access patterns the record kernels can use.
//  A coalesced: lane i copies 16-B vector i (+ grid stride)
//  B lane-per-record: lane copies its own REC-byte record with 16-B vectors
//  C lane-per-record, unaligned: as B, source and destination offset by 4 and 7 bytes
//  D group of G lanes per record, sequential records per group
#include <hip/hip_runtime.h>
#include <cstdio>
typedef uint32_t v4 __attribute__((ext_vector_type(4)));
typedef uint32_t v4u __attribute__((ext_vector_type(4), aligned(1)));

__global__ void kA(const v4 *s, v4 *d, size_t n) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i < n) __builtin_nontemporal_store(__builtin_nontemporal_load(s + i), d + i);
}
template <int REC, int SOFF, int DOFF>
__global__ void kB(const uint8_t *s, uint8_t *d, size_t nrec) {
    size_t r = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (r >= nrec) return;
    const uint8_t *sp = s + r * REC + SOFF;
    uint8_t *dp = d + r * REC + DOFF;
    v4u buf[REC / 16];
#pragma unroll
    for (int k = 0; k < REC / 16; ++k) buf[k] = *(const v4u *)(sp + 16 * k);
#pragma unroll
    for (int k = 0; k < REC / 16; ++k) *(v4u *)(dp + 16 * k) = buf[k];
}
template <int REC, int G>
__global__ void kD(const uint8_t *s, uint8_t *d, size_t nrec) {
    const int gl = threadIdx.x % G, grp = threadIdx.x / G, ng = blockDim.x / G;
    size_t r0 = blockIdx.x * (size_t)1024;
    for (size_t j = grp; j < 1024; j += ng) {
        size_t r = r0 + j;
        if (r >= nrec) break;
        const uint8_t *sp = s + r * REC + 4;
        uint8_t *dp = d + r * REC + 4;
        for (int c = gl; c < (REC - 16) / 16; c += G) *(v4u *)(dp + 16 * c) = *(const v4u *)(sp + 16 * c);
    }
}
// A2: coalesced output, source shifted by SOFF bytes (unaligned 16-B loads)
template <int SOFF>
__global__ void kA2(const uint8_t *s, v4 *d, size_t n) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i < n) __builtin_nontemporal_store(*(const v4u *)(s + 16 * i + SOFF), d + i);
}
// E: one block (256 lanes) per record, sequential records per block
template <int REC>
__global__ void kE(const uint8_t *s, uint8_t *d, size_t nrec, int per_block) {
    for (int j = 0; j < per_block; ++j) {
        size_t r = (size_t)blockIdx.x * per_block + j;
        if (r >= nrec) return;
        const uint8_t *sp = s + r * REC + 4;
        uint8_t *dp = d + r * REC + 4;
        for (int c = threadIdx.x; c < (REC - 16) / 16; c += blockDim.x) *(v4u *)(dp + 16 * c) = *(const v4u *)(sp + 16 * c);
    }
}
int main() {
    const size_t bytes = (size_t)6 << 30;
    uint8_t *s, *d;
    hipMalloc(&s, bytes + 64); hipMalloc(&d, bytes + 64);
    hipMemset(s, 1, bytes); hipMemset(d, 0, bytes);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    auto timeit = [&](const char *name, auto launch) {
        launch(); hipDeviceSynchronize();
        float best = 1e9;
        for (int it = 0; it < 5; ++it) {
            hipEventRecord(e0); launch(); hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1); if (ms < best) best = ms;
        }
        printf("%-44s %8.3f ms  %7.1f GB/s (read+write)\n", name, best, 2.0 * bytes / best / 1e6);
    };
    const size_t nv = bytes / 16;
    timeit("A coalesced 16B/lane, nt", [&] { hipLaunchKernelGGL(kA, dim3(nv / 256), dim3(256), 0, 0, (const v4 *)s, (v4 *)d, nv); });
    const size_t n192 = bytes / 192, n4k = bytes / 4096, n64 = bytes / 64;
    timeit("B lane/record 192B aligned", [&] { hipLaunchKernelGGL((kB<192, 0, 0>), dim3(n192 / 256 + 1), dim3(256), 0, 0, s, d, n192); });
    timeit("C lane/record 192B src+4 dst+7", [&] { hipLaunchKernelGGL((kB<192, 4, 7>), dim3(n192 / 256 + 1), dim3(256), 0, 0, s, d, n192 - 1); });
    timeit("B lane/record 64B aligned", [&] { hipLaunchKernelGGL((kB<64, 0, 0>), dim3(n64 / 256 + 1), dim3(256), 0, 0, s, d, n64); });
    timeit("C lane/record 64B src+4 dst+7", [&] { hipLaunchKernelGGL((kB<64, 4, 7>), dim3(n64 / 256 + 1), dim3(256), 0, 0, s, d, n64 - 1); });
    timeit("D G=4 per 192B record, +4", [&] { hipLaunchKernelGGL((kD<192, 4>), dim3(n192 / 1024 + 1), dim3(256), 0, 0, s, d, n192 - 1); });
    timeit("D G=16 per 192B record, +4", [&] { hipLaunchKernelGGL((kD<192, 16>), dim3(n192 / 1024 + 1), dim3(256), 0, 0, s, d, n192 - 1); });
    timeit("D G=64 per 4096B record, +4", [&] { hipLaunchKernelGGL((kD<4096, 64>), dim3(n4k / 1024 + 1), dim3(256), 0, 0, s, d, n4k - 1); });
    timeit("D G=16 per 4096B record, +4", [&] { hipLaunchKernelGGL((kD<4096, 16>), dim3(n4k / 1024 + 1), dim3(256), 0, 0, s, d, n4k - 1); });
    timeit("A2 coalesced out, src+4", [&] { hipLaunchKernelGGL((kA2<4>), dim3(nv / 256 - 1), dim3(256), 0, 0, s, (v4 *)d, nv - 256); });
    timeit("A2 coalesced out, src+7", [&] { hipLaunchKernelGGL((kA2<7>), dim3(nv / 256 - 1), dim3(256), 0, 0, s, (v4 *)d, nv - 256); });
    timeit("E block/record 4096B, 1 per block", [&] { hipLaunchKernelGGL((kE<4096>), dim3(n4k - 1), dim3(256), 0, 0, s, d, n4k - 1, 1); });
    timeit("E block/record 4096B, 16 per block", [&] { hipLaunchKernelGGL((kE<4096>), dim3(n4k / 16), dim3(256), 0, 0, s, d, n4k - 1, 16); });
    timeit("B lane/record 128B src+4 dst+4", [&] { hipLaunchKernelGGL((kB<128, 4, 4>), dim3(n192 / 256 + 1), dim3(256), 0, 0, s, d, n192 - 1); });
    timeit("B lane/record 256B src+4 dst+4", [&] { hipLaunchKernelGGL((kB<256, 4, 4>), dim3(bytes / 256 / 256 + 1), dim3(256), 0, 0, s, d, bytes / 256 - 1); });
    return 0;
}
