// gather_fetch.hip — calibration probe for the config-4 decode traffic question
// ("Config 4 decode: one read of the stream, measured
// honestly"; MI355X_MICROARCH.md: FETCH_SIZE is calibrated only for wide
// streaming reads, other widths must be calibrated on a known byte count).
//
// Kernels over a 4 GiB buffer (record-like 180-byte stride, as config 4's
// average record):
//   k_stream      every 16-byte chunk once, coalesced (the reference count)
//   k_gather      one dword per 180-byte "record" (the one-pass walk's length
//                 word gather), all blocks
//   k_walk_stage  per block of 1024 "records" (184 KB): the gather, then the
//                 block's bytes staged in 21 KiB pieces (the sweep's stage):
//                 the one-pass decode's read pattern without its compute
//   k_stage       the same staging without the gather
// Each kernel's time is printed (HIP events, median of 5); rocprofv3 --pmc
// FETCH_SIZE on this binary gives each kernel's fetch count.  Build:
//   hipcc --offload-arch=gfx950 -O3 -o gather_fetch tools/probes/gather_fetch.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr uint64_t kRec = 180, kRecPerBlock = 1024, kTile = 21504;

__global__ void k_stream(const u32x4 *p, uint64_t n16, uint32_t *sink) {
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
        const u32x4 v = __builtin_nontemporal_load(p + i);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9e3779b9u) sink[0] = acc;
}

__global__ void k_gather(const uint8_t *p, uint64_t nrec, uint32_t *sink) {
    uint32_t acc = 0;
    for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < nrec; r += (uint64_t)gridDim.x * blockDim.x)
        acc ^= *(const uint32_t *)(p + r * kRec + 4);
    if (acc == 0x9e3779b9u) sink[0] = acc;
}

// block b: records [b * 1024, (b + 1) * 1024); 256 threads
template <bool GATHER>
__global__ __launch_bounds__(256) void k_walk_stage(const uint8_t *p, uint64_t nrec, uint32_t *sink) {
    __shared__ __attribute__((aligned(16))) uint8_t tile[kTile];
    const uint64_t r0 = (uint64_t)blockIdx.x * kRecPerBlock;
    if (r0 >= nrec) return;
    const uint64_t r1 = std::min<uint64_t>(r0 + kRecPerBlock, nrec);
    uint32_t acc = 0;
    if (GATHER) {
        uint32_t w[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint64_t r = r0 + threadIdx.x + 256 * j;
            w[j] = r < r1 ? *(const uint32_t *)(p + r * kRec + 4) : 0u;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) acc ^= w[j];
    }
    __shared__ uint32_t s_acc;
    if (threadIdx.x == 0) s_acc = 0;
    __syncthreads();
    atomicXor(&s_acc, acc);
    const uint64_t b0 = r0 * kRec, b1 = r1 * kRec;
    for (uint64_t s = b0 & ~(uint64_t)15; s < b1; s += kTile) {
        const uint64_t e = std::min<uint64_t>(s + kTile, (b1 + 15) & ~(uint64_t)15);
        const uint32_t nch = (uint32_t)((e - s) >> 4);
        for (uint32_t i = threadIdx.x; i < nch; i += 256)
            *(u32x4 *)(tile + 16 * i) = __builtin_nontemporal_load((const u32x4 *)(p + s) + i);
        __syncthreads();
        uint32_t x = 0;
        for (uint32_t i = threadIdx.x; i < nch * 4; i += 256) x ^= ((const uint32_t *)tile)[i];
        atomicXor(&s_acc, x);
        __syncthreads();
    }
    if (threadIdx.x == 0 && s_acc == 0x9e3779b9u) sink[0] = s_acc;
}

template <typename F>
static float timed(F f) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    std::vector<float> ts;
    f();
    (void)hipDeviceSynchronize();
    for (int i = 0; i < 5; ++i) {
        (void)hipEventRecord(a, 0);
        f();
        (void)hipEventRecord(b, 0);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    return ts[2];
}

int main() {
    const uint64_t bytes = 4ull << 30;
    const uint64_t nrec = bytes / kRec;
    uint8_t *p;
    uint32_t *sink;
    CK(hipMalloc(&p, bytes + 4096));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(p, 0x5a, bytes + 4096));
    const uint64_t nblk = (nrec + kRecPerBlock - 1) / kRecPerBlock;
    const float t_s = timed([&] { k_stream<<<1024 * 256, 256>>>((const u32x4 *)p, bytes / 16, sink); });
    const float t_g = timed([&] { k_gather<<<(nrec + 255) / 256, 256>>>(p, nrec, sink); });
    const float t_ws = timed([&] { k_walk_stage<true><<<nblk, 256>>>(p, nrec, sink); });
    const float t_st = timed([&] { k_walk_stage<false><<<nblk, 256>>>(p, nrec, sink); });
    CK(hipDeviceSynchronize());
    const double gb = bytes / 1e9;
    printf("{\"buffer_GB\": %.3f, \"records\": %llu, \"record_bytes\": %llu,\n", gb, (unsigned long long)nrec,
           (unsigned long long)kRec);
    printf(" \"k_stream_ms\": %.4f, \"k_stream_TBps\": %.3f,\n", t_s, gb / t_s);
    printf(" \"k_gather_ms\": %.4f, \"k_gather_lines_GB\": %.3f,\n", t_g, nrec * 128.0 / 1e9);
    printf(" \"k_walk_stage_ms\": %.4f, \"k_stage_ms\": %.4f, \"walk_stage_over_stage\": %.3f}\n", t_ws, t_st, t_ws / t_st);
    return 0;
}
