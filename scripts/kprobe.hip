// kprobe.hip -- flow-table probe microbenchmark (not product code).
//
// Question: the 1M-flow C4 case of k_rx costs one random 128-B line fill per
// packet for its 16-B slot probe, on top of the 0.56 line of header window
// and descriptor, and the launch runs at the chip's line-fill rate. Does a
// probe with another cache policy (non-temporal, or scoped so that it need
// not allocate in the XCD's L2) cost less? 1M random 16-B probes per launch
// into a 128 MB slot array (the --flow-capacity 2000000 table), each lane one
// probe into LDS (global_load_lds, as k_rx loads its windows), alone and
// together with the C2 window gather of 16 rotating 72 MB batches.
// cpol bits (gfx940+): sc0 = 1, nt = 2, sc1 = 16.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/kprobe.hip -o scripts/kprobe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

template <int CPOL, bool WIN, bool PROBE>
__global__ __launch_bounds__(256) void k_probe(const uint8_t *arena, const uint4 *slots, const uint32_t *pos,
                                               uint32_t n, uint32_t *out) {
    __shared__ __attribute__((aligned(16))) uint8_t s_win[4 * 64 * 64];
    __shared__ __attribute__((aligned(16))) uint4 s_sl[256];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    uint8_t *wl = s_win + wave * 4096;
    if (WIN) {
        const uint32_t fbase = blockIdx.x * 256 + wave * 64;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t p = fbase + k * 16 + (lane >> 2);
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(arena + (size_t)p * 64 + (lane & 3) * 16),
                                             (__attribute__((address_space(3))) void *)(wl + k * 1024), 16, 0, 2);
        }
    }
    if (PROBE) {
        const uint32_t q = i < n ? pos[i] : 0u;
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(slots + q),
                                         (__attribute__((address_space(3))) void *)(s_sl + wave * 64), 16, 0, CPOL);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    uint32_t x = 0;
    if (WIN) {
        const uint4 *row = reinterpret_cast<const uint4 *>(wl + (lane >> 4) * 1024 + (lane & 15) * 64);
        const uint4 a = row[0];
        x ^= a.x ^ a.w;
    }
    if (PROBE) {
        const uint4 s = s_sl[threadIdx.x];
        x ^= s.x ^ s.y ^ s.z ^ s.w;
    }
    if (i < n) out[i] = x;
}

typedef void (*Kern)(const uint8_t *, const uint4 *, const uint32_t *, uint32_t, uint32_t *);

int main() {
    const uint32_t n = 1u << 20, nslots = 8u << 20, nbuf = 16;
    std::vector<uint32_t> pos(n);
    std::mt19937 rng(7);
    for (auto &p : pos) p = rng() & (nslots - 1);
    uint4 *slots;
    uint32_t *dpos, *dout;
    CK(hipMalloc(&slots, 16ull * nslots));
    CK(hipMemset(slots, 1, 16ull * nslots));
    CK(hipMalloc(&dpos, 4ull * n));
    CK(hipMalloc(&dout, 4ull * n));
    CK(hipMemcpy(dpos, pos.data(), 4ull * n, hipMemcpyHostToDevice));
    std::vector<uint8_t *> arenas(nbuf);
    for (auto &a : arenas) {
        CK(hipMalloc(&a, 64ull * n + 256));
        CK(hipMemset(a, 2, 64ull * n + 256));
    }
    struct V { const char *name; Kern k; } vs[] = {
        {"windows only            ", k_probe<0, true, false>},
        {"probe cpol 0            ", k_probe<0, false, true>},
        {"probe nt                ", k_probe<2, false, true>},
        {"probe sc0               ", k_probe<1, false, true>},
        {"probe sc1               ", k_probe<16, false, true>},
        {"probe sc0 sc1           ", k_probe<17, false, true>},
        {"probe nt sc0 sc1        ", k_probe<19, false, true>},
        {"windows + probe cpol 0  ", k_probe<0, true, true>},
        {"windows + probe nt      ", k_probe<2, true, true>},
        {"windows + probe sc1     ", k_probe<16, true, true>},
        {"windows + probe sc0 sc1 ", k_probe<17, true, true>},
        {"windows + probe nt sc0sc1", k_probe<19, true, true>},
    };
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int reps = 32;
    for (auto &v : vs) {
        for (int r = 0; r < 4; ++r)
            hipLaunchKernelGGL(v.k, dim3(n / 256), dim3(256), 0, 0, arenas[r % nbuf], slots, dpos, n, dout);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a, 0));
        for (int r = 0; r < reps; ++r)
            hipLaunchKernelGGL(v.k, dim3(n / 256), dim3(256), 0, 0, arenas[r % nbuf], slots, dpos, n, dout);
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        printf("%s %7.2f us/launch\n", v.name, ms * 1e3 / reps);
    }
    return 0;
}
