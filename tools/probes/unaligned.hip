// Probe: do byte-unaligned dword / dwordx4 global loads and stores return
// and write the right bytes on this GPU (HSA unaligned access mode)?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(1)));
typedef uint32_t u32u __attribute__((aligned(1)));
__global__ void k(const uint8_t *src, uint8_t *dst, uint32_t *ld_out) {
    const int t = threadIdx.x;  // t = byte offset 0..15
    if (t >= 16) return;
    const u32x4u v = *(const u32x4u *)(src + 64 * t + t);
    ld_out[4 * t + 0] = v.x; ld_out[4 * t + 1] = v.y; ld_out[4 * t + 2] = v.z; ld_out[4 * t + 3] = v.w;
    *(u32x4u *)(dst + 64 * t + t) = v;
    *(u32u *)(dst + 64 * t + 32 + t) = v.x;
}
int main() {
    uint8_t h[1024], out[1024];
    uint32_t ld[64];
    for (int i = 0; i < 1024; ++i) h[i] = (uint8_t)(i * 7 + 3);
    uint8_t *ds, *dd; uint32_t *dl;
    hipMalloc(&ds, 1024); hipMalloc(&dd, 1024); hipMalloc(&dl, 256);
    hipMemcpy(ds, h, 1024, hipMemcpyHostToDevice);
    hipMemset(dd, 0, 1024);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, ds, dd, dl);
    hipMemcpy(out, dd, 1024, hipMemcpyDeviceToHost);
    hipMemcpy(ld, dl, 256, hipMemcpyDeviceToHost);
    int bad_ld = 0, bad_st = 0;
    for (int t = 0; t < 16; ++t) {
        uint32_t want[4];
        memcpy(want, h + 64 * t + t, 16);
        for (int j = 0; j < 4; ++j) bad_ld += ld[4 * t + j] != want[j];
        bad_st += memcmp(out + 64 * t + t, h + 64 * t + t, 16) != 0;
        bad_st += memcmp(out + 64 * t + 32 + t, h + 64 * t + t, 4) != 0;
        for (int b = 0; b < t; ++b) bad_st += out[64 * t + b] != 0;   // no bytes before
    }
    printf("unaligned probe: bad loads=%d bad stores=%d\n", bad_ld, bad_st);
    return 0;
}
