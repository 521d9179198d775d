// kcopy.hip -- pinned host -> device copy rate by copy size and stream count
// (not product code). The element's host path copies one 1.2-MB block per
// 16K-packet batch per thread; a trace of 8 threads showed ~18 us between
// back-to-back H2D copies. This times R copies of S bytes from hipHostMalloc
// memory, issued round-robin over K streams, and prints the aggregate GB/s
// and us per copy.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/kcopy.hip -o scripts/kcopy
#include <hip/hip_runtime.h>
#include <chrono>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
int main() {
    const size_t maxb = 8u << 20;
    const int maxk = 16;
    std::vector<uint8_t *> h(maxk), d(maxk);
    std::vector<hipStream_t> s(maxk);
    for (int k = 0; k < maxk; ++k) {
        CK(hipHostMalloc((void **)&h[k], maxb, hipHostMallocDefault));
        CK(hipMalloc((void **)&d[k], maxb));
        CK(hipStreamCreateWithFlags(&s[k], hipStreamNonBlocking));
    }
    const size_t sizes[] = {256u << 10, 1200u << 10, 2400u << 10, 8u << 20};
    const int ks[] = {1, 2, 4, 8, 16};
    for (size_t b : sizes)
        for (int K : ks) {
            const int R = 256;
            for (int w = 0; w < 2; ++w) {   // warm, then timed
                CK(hipDeviceSynchronize());
                auto t0 = std::chrono::steady_clock::now();
                for (int r = 0; r < R; ++r) CK(hipMemcpyAsync(d[r % K], h[r % K], b, hipMemcpyHostToDevice, s[r % K]));
                CK(hipDeviceSynchronize());
                double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
                if (w) printf("H2D %7zu KB x %d streams: %6.1f GB/s, %6.1f us per copy\n", b >> 10, K, (double)b * R / us / 1e3, us / R);
            }
        }
    return 0;
}
