// kvariants.hip -- kernel experiments for the receive-path hot path (not product code).
//
// Times, on 1M-packet C2 batches rotated over 16 HBM buffers (> Infinity Cache):
//   stream   : contiguous dwordx4 read of the same 72 MB (HBM ceiling for the bytes)
//   direct   : per-lane desc + 4 x dwordx4 window loads, fold, write 6 B/pkt
//   glds     : desc + LDS-DMA gather (k_rx's load path), fold, write 6 B/pkt
//   k_rx/none, k_rx/tile at several grid sizes (grid-stride persistent variants)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include scripts/kvariants.hip -o /tmp/kv
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include "../fastclick_amd/csrc/fcgpu_device.hh"

using namespace fcgpu;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ __launch_bounds__(256) void k_stream(const uint4 *p, size_t n16, uint32_t *out) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) {
        uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ __launch_bounds__(256) void k_direct(const uint8_t *arena, const uint2 *desc, uint32_t n,
                                                uint16_t *v, uint32_t *h) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    uint2 d = desc[i];
    const uint4 *w = reinterpret_cast<const uint4 *>(arena + d.x);
    uint4 a = w[0], b = w[1], c = w[2], e = w[3];
    uint32_t x = a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w ^ c.x ^ c.y ^ c.z ^ c.w ^ e.x ^ e.y ^ e.z ^ e.w;
    v[i] = (uint16_t)(x ^ d.y);
    h[i] = x;
}

__global__ __launch_bounds__(256) void k_glds(const uint8_t *arena, const uint2 *desc, uint32_t n,
                                              uint16_t *v, uint32_t *h) {
    __shared__ __attribute__((aligned(16))) uint8_t s_win[4 * 64 * 64];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    uint2 d = make_uint2(0, 0);
    if (i < n) d = desc[i];
    uint8_t *wl = s_win + wave * 4096;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t p = k * 16 + (lane >> 2);
        const uint32_t poff = __shfl(d.x, (int)p);
        const uint32_t c = (lane & 3) ^ ((p >> 2) & 3);
        glds16(arena + (poff & ~15u) + c * 16, wl + k * 1024);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint4 *row = reinterpret_cast<const uint4 *>(wl + lane * 64);
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        uint4 q = row[k];
        x ^= q.x ^ q.y ^ q.z ^ q.w;
    }
    if (i < n) {
        v[i] = (uint16_t)(x ^ d.y);
        h[i] = x;
    }
}

int main(int argc, char **argv) {
    const uint32_t n = 1u << 20, nports = 16;
    const uint32_t NB = argc > 2 ? (uint32_t)atoi(argv[2]) : 16;
    const int iters = argc > 1 ? atoi(argv[1]) : 200;
    // C2 frames: 60-B UDP/IPv4 in 64-B slots
    std::vector<uint8_t> host((size_t)n * 64 + 256, 0);
    std::vector<uint32_t> desc(2 * n);
    uint8_t f[60] = {2, 0, 0, 0, 0, 2, 2, 0, 0, 0, 0, 1, 8, 0, 0x45, 0, 0, 46, 0, 0, 0, 0, 64, 17, 0, 0,
                     10, 0, 0, 1, 10, 0, 0, 2, 0x04, 0xd2, 0x16, 0x2e, 0, 26};
    uint32_t sum = 0;
    for (int k = 0; k < 20; k += 2) sum += (f[14 + k] << 8) | f[15 + k];
    while (sum >> 16) sum = (sum & 0xffff) + (sum >> 16);
    sum = ~sum & 0xffff;
    f[24] = sum >> 8;
    f[25] = sum & 0xff;
    for (uint32_t i = 0; i < n; ++i) {
        memcpy(&host[(size_t)i * 64], f, 60);
        desc[2 * i] = i * 64;
        desc[2 * i + 1] = 60;
    }
    std::vector<uint8_t *> arena(NB);
    std::vector<uint2 *> dd(NB);
    for (uint32_t b = 0; b < NB; ++b) {
        CK(hipMalloc(&arena[b], host.size()));
        CK(hipMalloc(&dd[b], 8ull * n));
        CK(hipMemcpy(arena[b], host.data(), host.size(), hipMemcpyHostToDevice));
        CK(hipMemcpy(dd[b], desc.data(), 8ull * n, hipMemcpyHostToDevice));
    }
    uint16_t *v;
    uint32_t *h, *perm, *tilecnt, *sink;
    uint16_t *tc;
    unsigned long long *ctr;
    const uint32_t ntiles = n / 256;
    CK(hipMalloc(&v, 2ull * n));
    CK(hipMalloc(&h, 4ull * n));
    CK(hipMalloc(&perm, 4ull * n));
    CK(hipMalloc(&tilecnt, 4ull * 65 * ntiles));
    CK(hipMalloc(&tc, 2ull * 17 * ntiles));
    CK(hipMalloc(&ctr, 8ull * FCGPU_CTR_SHARDS * FCGPU_NCOUNTERS));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(ctr, 0, 8ull * FCGPU_CTR_SHARDS * FCGPU_NCOUNTERS));
    hipEvent_t e0, e1, k0, k1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventCreateWithFlags(&k0, hipEventDisableSystemFence));
    CK(hipEventCreateWithFlags(&k1, hipEventDisableSystemFence));

    RxArgs A{};
    A.n = n;
    A.ntiles = ntiles;
    A.verdict = v;
    A.hash = h;
    A.anno = nullptr;
    A.tilecnt = tilecnt;
    const bool tp = argc > 3 && !strcmp(argv[3], "tp");
    A.perm = tp ? nullptr : perm;
    A.tile_perm = tp ? (uint8_t *)perm : nullptr;
    A.tile_count = tc;
    A.ctr = ctr;
    memset(&A.cfg, 0, sizeof(A.cfg));
    A.cfg.offset = 14;
    A.cfg.nports = nports;
    A.cfg.lb_magic = (uint32_t)((((uint64_t)1 << 32) + nports - 1) / nports);
    A.cfg.hash_mode = FCGPU_HASH_FLOWID;
    A.cfg.classify = FCGPU_CLS_LB_HASH;
    const double bytes = 72.0 * n;

    auto run = [&](const char *name, auto launch) {
        for (int w = 0; w < 20; ++w) launch(w % NB, nullptr, nullptr);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, 0));
        for (int it = 0; it < iters; ++it) launch(it % NB, nullptr, nullptr);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        // kernel-only duration via ext-launch events, averaged over 20 launches
        float kt = 0;
        for (int it = 0; it < 20; ++it) {
            launch(it % NB, k0, k1);
            CK(hipEventSynchronize(k1));
            float t = 0;
            CK(hipEventElapsedTime(&t, k0, k1));
            kt += t;
        }
        kt /= 20;
        const double us = ms * 1e3 / iters;
        printf("%-28s back-to-back %7.2f us/launch  %7.0f Mpps  %6.0f GB/s | kernel %7.2f us  %6.0f GB/s\n", name,
               us, n / us, bytes / us / 1e3, kt * 1e3, bytes / (kt * 1e3) / 1e3);
    };

    run("stream (contiguous 72 MB)", [&](int b, hipEvent_t a, hipEvent_t c) {
        // 72 B/pkt of contiguous bytes: the arena (64 MB) + desc (8 MB) as one read set
        if (a) {
            hipExtLaunchKernelGGL(k_stream, dim3(4096), dim3(256), 0, 0, a, nullptr, 0, (const uint4 *)arena[b],
                                  (size_t)n * 4, sink);
            hipExtLaunchKernelGGL(k_stream, dim3(512), dim3(256), 0, 0, nullptr, c, 0, (const uint4 *)dd[b],
                                  (size_t)n / 2, sink);
        } else {
            hipLaunchKernelGGL(k_stream, dim3(4096), dim3(256), 0, 0, (const uint4 *)arena[b], (size_t)n * 4, sink);
            hipLaunchKernelGGL(k_stream, dim3(512), dim3(256), 0, 0, (const uint4 *)dd[b], (size_t)n / 2, sink);
        }
    });
    run("direct 4x dwordx4", [&](int b, hipEvent_t a, hipEvent_t c) {
        if (a) hipExtLaunchKernelGGL(k_direct, dim3(ntiles), dim3(256), 0, 0, a, c, 0, arena[b], dd[b], n, v, h);
        else hipLaunchKernelGGL(k_direct, dim3(ntiles), dim3(256), 0, 0, arena[b], dd[b], n, v, h);
    });
    run("glds gather", [&](int b, hipEvent_t a, hipEvent_t c) {
        if (a) hipExtLaunchKernelGGL(k_glds, dim3(ntiles), dim3(256), 0, 0, a, c, 0, arena[b], dd[b], n, v, h);
        else hipLaunchKernelGGL(k_glds, dim3(ntiles), dim3(256), 0, 0, arena[b], dd[b], n, v, h);
    });
    auto rx = [&](auto kern, uint32_t grid) {
        return [&, kern, grid](int b, hipEvent_t a, hipEvent_t c) {
            RxArgs X = A;
            X.arena = arena[b];
            X.desc = dd[b];
            if (a) hipExtLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, a, c, 0, X);
            else hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, X);
        };
    };
    run("k_rx none", rx(k_rx<FCGPU_CHECK_IP4, true, kPartNone, false, false>, ntiles));
    run("k_rx none fast", rx(k_rx<FCGPU_CHECK_IP4, true, kPartNone, false, false, false, true>, ntiles));
    run("k_rx tile", rx(k_rx<FCGPU_CHECK_IP4, true, kPartTile, false, false>, ntiles));
    run("k_rx tile fast", rx(k_rx<FCGPU_CHECK_IP4, true, kPartTile, false, false, false, true>, ntiles));
    run("k_rx global", rx(k_rx<FCGPU_CHECK_IP4, true, kPartGlobal, false, false>, ntiles));
    run("k_rx global fast", rx(k_rx<FCGPU_CHECK_IP4, true, kPartGlobal, false, false, false, true>, ntiles));
    return 0;
}
