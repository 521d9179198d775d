// klines.hip -- line-request microbenchmark (not product code).
//
// Question (C3/C5 line waste): a 64-B header window that lies
// alone in its 128-B line costs a whole 128-B EA read request. Can a load
// with another cache policy be served by a 64-B request, and is the limit
// the rate of requests (then a 64-B request gains nothing) or of bytes?
// Reads N 64-B pieces per launch, 4 lanes x 16 B each through LDS-DMA (as
// k_rx loads its windows), either packed (stride 64: two pieces per line) or
// each alone in its line (stride 128), with cpol 0 / nt / sc0 / sc1 / sc0 sc1
// (gfx940+ bits: sc0 = 1, nt = 2, sc1 = 16). Launches walk a 2 GB buffer so
// the Infinity Cache does not hold the pieces. A rocprofv3 --pmc pass with
// TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum over the same
// binary gives each variant's request sizes (kernel names carry the variant).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/klines.hip -o scripts/klines
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

template <int STRIDE, int CPOL>
__global__ __launch_bounds__(256) void k_lines(const uint8_t *base, uint32_t n, uint32_t *out) {
    __shared__ __attribute__((aligned(16))) uint8_t s_win[4 * 64 * 64];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    uint8_t *wl = s_win + wave * 4096;
    const uint32_t fbase = blockIdx.x * 256 + wave * 64;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t p = fbase + k * 16 + (lane >> 2);
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(base + (size_t)p * STRIDE + (lane & 3) * 16),
                                         (__attribute__((address_space(3))) void *)(wl + k * 1024), 16, 0, CPOL);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    const uint4 *row = reinterpret_cast<const uint4 *>(wl + (lane >> 4) * 1024 + (lane & 15) * 64);
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) { const uint4 q = row[k]; x ^= q.x ^ q.y ^ q.z ^ q.w; }
    if (i < n) out[i] = x;
}

typedef void (*Kern)(const uint8_t *, uint32_t, uint32_t *);

int main(int argc, char **argv) {
    const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : (2u << 20);   // pieces per launch (multiple of 256)
    const size_t total = 2ull << 30;
    uint8_t *buf;
    uint32_t *out;
    CK(hipMalloc(&buf, total));
    CK(hipMemset(buf, 3, total));
    CK(hipMalloc(&out, 4ull * n));
    struct V { const char *name; int stride; Kern k; } vs[] = {
        {"packed  cpol 0    ", 64, k_lines<64, 0>},
        {"alone   cpol 0    ", 128, k_lines<128, 0>},
        {"alone   nt        ", 128, k_lines<128, 2>},
        {"alone   sc0       ", 128, k_lines<128, 1>},
        {"alone   sc1       ", 128, k_lines<128, 16>},
        {"alone   sc0 sc1   ", 128, k_lines<128, 17>},
        {"alone   sc0 sc1 nt", 128, k_lines<128, 19>},
        {"packed  nt        ", 64, k_lines<64, 2>},
    };
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int reps = 40;
    printf("# %u pieces of 64 B per launch, 2 GB walked\n", n);
    for (const V &v : vs) {
        const size_t span = (size_t)n * v.stride;
        const size_t nspan = total / span;
        hipLaunchKernelGGL(v.k, dim3(n / 256), dim3(256), 0, 0, buf, n, out);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a, 0));
        for (int r = 0; r < reps; ++r)
            hipLaunchKernelGGL(v.k, dim3(n / 256), dim3(256), 0, 0, buf + (r % nspan) * span, n, out);
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        const double us = ms * 1e3 / reps;
        const double lines = v.stride == 64 ? n / 2.0 : (double)n;
        printf("%s stride %3d: %7.2f us/launch, %6.1f G pieces/s, %6.1f G lines/s, %6.2f TB/s of lines\n", v.name,
               v.stride, us, n / us / 1e3, lines / us / 1e3, lines * 128 / us / 1e6);
    }
    return 0;
}
