// kgather.hip -- header-window gather microbenchmark (not product code).
//
// Question: with frames in slots larger than 64 B (N1 frame-size sweep, IMIX),
// k_rx reads one 64-B window per 128-B line or more and runs at ~46 G
// windows/s, well under the HBM byte rate. Which load shape gathers sparse
// 64-B windows fastest? 1M windows per launch, 16 rotating buffers (> MALL).
//   glds   : k_rx's LDS-DMA (4 x 16 B per frame, 4 lanes per frame), cpol 0/nt
//   vec4   : plain global_load_dwordx4, 4 lanes per frame, cpol default
//   lane64 : one lane per frame, 4 x dwordx4 from the same lane
// Each kernel xors its window into a 4-B output per frame (so nothing is
// optimised away). Prints us per launch per (stride, method).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/kgather.hip -o scripts/kgather
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

template <int CPOL>
__global__ __launch_bounds__(256) void k_glds(const uint8_t *arena, uint32_t stride, uint32_t n, uint32_t *out) {
    __shared__ __attribute__((aligned(16))) uint8_t s_win[4 * 64 * 64];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    uint8_t *wl = s_win + wave * 4096;
    const uint32_t fbase = blockIdx.x * 256 + wave * 64;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t p = fbase + k * 16 + (lane >> 2);
        const uint8_t *src = arena + (size_t)p * stride + (lane & 3) * 16;
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                         (__attribute__((address_space(3))) void *)(wl + k * 1024), 16, 0, CPOL);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint4 *row = reinterpret_cast<const uint4 *>(wl + lane * 64);
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        uint4 q = row[k];
        x ^= q.x ^ q.y ^ q.z ^ q.w;
    }
    if (i < n) out[i] = x;
}

__global__ __launch_bounds__(256) void k_vec4(const uint8_t *arena, uint32_t stride, uint32_t n, uint32_t *out) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t fbase = blockIdx.x * 256 + wave * 64;
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t p = fbase + k * 16 + (lane >> 2);
        const uint4 q = *reinterpret_cast<const uint4 *>(arena + (size_t)p * stride + (lane & 3) * 16);
        uint32_t x = q.x ^ q.y ^ q.z ^ q.w;
        x ^= __shfl_xor(x, 1);
        x ^= __shfl_xor(x, 2);
        if ((lane & 3) == 0 && (lane >> 2) == (lane >> 2)) acc = (k == (int)((lane >> 4) & 3)) ? x : acc;
    }
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) out[i] = acc;
}

__global__ __launch_bounds__(256) void k_lane64(const uint8_t *arena, uint32_t stride, uint32_t n, uint32_t *out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint4 *w = reinterpret_cast<const uint4 *>(arena + (size_t)i * stride);
    uint4 a = w[0], b = w[1], c = w[2], d = w[3];
    out[i] = a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w ^ c.x ^ c.y ^ c.z ^ c.w ^ d.x ^ d.y ^ d.z ^ d.w;
}

int main(int argc, char **argv) {
    const uint32_t n = 1u << 20, NB = 16;
    const int iters = argc > 1 ? atoi(argv[1]) : 64;
    uint32_t *out;
    CK(hipMalloc(&out, 4ull * n));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (uint32_t stride : {64u, 128u, 256u, 1536u}) {
        std::vector<uint8_t *> buf(NB);
        for (auto &b : buf) {
            CK(hipMalloc(&b, (size_t)n * stride + 256));
            CK(hipMemset(b, 1, (size_t)n * stride + 256));
        }
        CK(hipDeviceSynchronize());
        auto run = [&](const char *name, auto launch) {
            for (int w = 0; w < 16; ++w) launch(buf[w % NB]);
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0, 0));
            for (int k = 0; k < iters; ++k) launch(buf[k % NB]);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            const double us = ms * 1e3 / iters;
            printf("stride %5u %-10s %8.2f us/launch  %7.1f G windows/s  %6.2f TB/s (64 B/window)\n", stride, name, us,
                   n / us / 1e3, 64.0 * n / us / 1e6);
        };
        const dim3 g(n / 256), b(256);
        run("glds", [&](uint8_t *a) { hipLaunchKernelGGL(k_glds<0>, g, b, 0, 0, a, stride, n, out); });
        run("glds_nt", [&](uint8_t *a) { hipLaunchKernelGGL(k_glds<2>, g, b, 0, 0, a, stride, n, out); });
        run("vec4", [&](uint8_t *a) { hipLaunchKernelGGL(k_vec4, g, b, 0, 0, a, stride, n, out); });
        run("lane64", [&](uint8_t *a) { hipLaunchKernelGGL(k_lane64, g, b, 0, 0, a, stride, n, out); });
        for (auto &bb : buf) CK(hipFree(bb));
    }
    return 0;
}
