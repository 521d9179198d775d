// khostgather.hip -- zero-copy gather microbenchmark over PCIe (not product code).
//
// Question: the mbuf ingress (fcgpu_process_mbufs) reads one 64-B mbuf header
// and one 64-B header window per packet from page-locked host memory and
// tops out at ~155 Mpps whether the descriptors are built on the GPU or on
// the host. Which load shape reads scattered 64-B pieces of host memory
// fastest? 256K pieces per launch at a 2304-B stride (rte_mbuf element
// size), in shuffled order, in memory registered with hipHostRegister
// (mapped) as fcgpu_pool_register does, and in hipHostMalloc memory.
//   glds   : 4 lanes x 16 B per piece via LDS-DMA (k_rx / k_mbuf_desc today)
//   vec4   : 4 lanes x 16 B, plain global_load_dwordx4
//   lane64 : one lane per piece, 4 x dwordx4
//   lane16 : one lane per piece, 16 B only (request count vs bytes)
//   w8x8   : 8 lanes x 8 B per piece
// Prints us per launch and M pieces/s per method.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/khostgather.hip -o scripts/khostgather
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ __launch_bounds__(256) void k_glds(const uint8_t *base, const uint32_t *off, uint32_t n, uint32_t *out) {
    __shared__ __attribute__((aligned(16))) uint8_t s_win[4 * 64 * 64];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    const uint32_t o = i < n ? off[i] : 0u;
    uint8_t *wl = s_win + wave * 4096;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t po = __shfl(o, k * 16 + (lane >> 2));
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(base + po + (lane & 3) * 16),
                                         (__attribute__((address_space(3))) void *)(wl + k * 1024), 16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    const uint4 *row = reinterpret_cast<const uint4 *>(wl + (lane >> 4) * 1024 + (lane & 15) * 64);
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) { uint4 q = row[k]; x ^= q.x ^ q.y ^ q.z ^ q.w; }
    if (i < n) out[i] = x;
}

__global__ __launch_bounds__(256) void k_vec4(const uint8_t *base, const uint32_t *off, uint32_t n, uint32_t *out) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    const uint32_t o = i < n ? off[i] : 0u;
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t po = __shfl(o, (int)((threadIdx.x & ~63u) % 64 + k * 16 + (lane >> 2)));
        const uint4 q = *reinterpret_cast<const uint4 *>(base + po + (lane & 3) * 16);
        uint32_t x = q.x ^ q.y ^ q.z ^ q.w;
        x ^= __shfl_xor(x, 1);
        x ^= __shfl_xor(x, 2);
        if ((lane >> 4) == (uint32_t)k) acc = x;
    }
    if (i < n) out[i] = acc;
}

__global__ __launch_bounds__(256) void k_lane64(const uint8_t *base, const uint32_t *off, uint32_t n, uint32_t *out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint4 *p = reinterpret_cast<const uint4 *>(base + off[i]);
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) { uint4 q = p[k]; x ^= q.x ^ q.y ^ q.z ^ q.w; }
    out[i] = x;
}

__global__ __launch_bounds__(256) void k_lane16(const uint8_t *base, const uint32_t *off, uint32_t n, uint32_t *out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint4 q = *reinterpret_cast<const uint4 *>(base + off[i]);
    out[i] = q.x ^ q.y ^ q.z ^ q.w;
}

__global__ __launch_bounds__(256) void k_w8x8(const uint8_t *base, const uint32_t *off, uint32_t n, uint32_t *out) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    const uint32_t o = i < n ? off[i] : 0u;
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const uint32_t po = __shfl(o, k * 8 + (lane >> 3));
        const uint2 q = *reinterpret_cast<const uint2 *>(base + po + (lane & 7) * 8);
        uint32_t x = q.x ^ q.y;
        x ^= __shfl_xor(x, 1);
        x ^= __shfl_xor(x, 2);
        x ^= __shfl_xor(x, 4);
        if ((lane >> 3) == (uint32_t)k) acc = x;
    }
    if (i < n) out[i] = acc;
}

typedef void (*Kern)(const uint8_t *, const uint32_t *, uint32_t, uint32_t *);

static double run(Kern k, const uint8_t *base, const uint32_t *doff, uint32_t n, uint32_t *dout, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    hipLaunchKernelGGL(k, dim3((n + 255) / 256), dim3(256), 0, 0, base, doff, n, dout);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a, 0));
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k, dim3((n + 255) / 256), dim3(256), 0, 0, base, doff, n, dout);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms * 1e3 / reps;
}

int main(int argc, char **argv) {
    const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : (1u << 18);
    // argv[2]: stride between pieces (2304 = rte_mbuf element; 64 = the
    // element's packed staging records); argv[3] = 0: pieces in address order
    const size_t stride = argc > 2 ? (size_t)atoi(argv[2]) : 2304;
    const bool shuffled = argc > 3 ? atoi(argv[3]) != 0 : true;
    // argv[4]: bytes each 64-B read starts before its piece (16: a window
    // that starts 16 B early, as k_rx's does for a record staged from frame
    // byte 14 at a 16-B aligned address -- neighbouring windows overlap when
    // the stride is < 64)
    const uint32_t lead = argc > 4 ? (uint32_t)atoi(argv[4]) : 0u;
    const size_t bytes = stride * n + 4096 + 128;
    std::vector<uint32_t> off(n);
    for (uint32_t i = 0; i < n; ++i) off[i] = (uint32_t)(i * stride + (stride >= 2304 ? 256 : 0) + 64 - lead);
    std::mt19937 rng(1);
    if (shuffled) std::shuffle(off.begin(), off.end(), rng);
    printf("# %u pieces, stride %zu B, %s, reads start %u B before each piece\n", n, stride,
           shuffled ? "shuffled" : "in address order", lead);
    uint32_t *doff, *dout;
    CK(hipMalloc(&doff, 4ull * n));
    CK(hipMalloc(&dout, 4ull * n));
    CK(hipMemcpy(doff, off.data(), 4ull * n, hipMemcpyHostToDevice));
    struct M { const char *name; Kern k; } ms[] = {
        {"glds", k_glds}, {"vec4", k_vec4}, {"lane64", k_lane64}, {"lane16", k_lane16}, {"w8x8", k_w8x8}};
    for (int mem = 0; mem < 3; ++mem) {
        uint8_t *host = nullptr, *dev = nullptr;
        if (mem == 0) {
            host = static_cast<uint8_t *>(aligned_alloc(4096, (bytes + 4095) / 4096 * 4096));
            for (size_t j = 0; j < bytes; j += 4096) host[j] = (uint8_t)j;
            CK(hipHostRegister(host, (bytes + 4095) / 4096 * 4096, hipHostRegisterMapped));
            CK(hipHostGetDevicePointer((void **)&dev, host, 0));
        } else {
            // 1: coherent (hipHostMallocDefault); 2: non-coherent -- the GPU's
            // L2 may keep its lines within a kernel (written by the host
            // before the launch, read by the kernel only)
            CK(hipHostMalloc((void **)&host, bytes, mem == 1 ? hipHostMallocDefault : hipHostMallocNonCoherent));
            for (size_t j = 0; j < bytes; j += 4096) host[j] = (uint8_t)j;
            CK(hipHostGetDevicePointer((void **)&dev, host, 0));
        }
        for (auto &m : ms) {
            const double us = run(m.k, dev, doff, n, dout, 10);
            printf("%s %-7s %8.1f us  %7.1f M pieces/s\n",
                   mem == 0 ? "registered" : mem == 1 ? "hostmalloc" : "noncoherent", m.name, us, n / us);
        }
        if (mem == 0) {
            CK(hipHostUnregister(host));
            free(host);
        } else {  // 1, 2
            CK(hipHostFree(host));
        }
    }
    return 0;
}
