// mock_element_bench.cc -- profiling aid (not product code): the element's
// host-side ceiling with scripts/mock_fcgpu.cc standing in for the GPU.
// A 64K-packet C2-shaped trace (60-B frames in 64-B slots) through
// GPUIPCheckClassify behind a BURST-32 source, as scripts/element_threads.py
// does on the GPU box.  Usage: element_bench THREADS [BATCH] [REPS] [CONF]
// (CONF: another GPUIPCheckClassify configuration; tests/test_host_sanitizers.py
// runs the element's data path under ASan/UBSan this way).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "fcclick.h"

int main(int argc, char **argv) {
    const uint32_t threads = argc > 1 ? (uint32_t)atoi(argv[1]) : 1;
    const std::string batch = argc > 2 ? argv[2] : "16384";     // a number or "auto"
    const uint32_t reps = argc > 3 ? (uint32_t)atoi(argv[3]) : 40;   // 0: pushed for 2 s (fcclick_bench_timed)
    const uint32_t n = 1u << 16;
    std::vector<uint8_t> arena((size_t)n * 64 + 256, 0);
    std::vector<uint32_t> desc(2ull * n);
    for (uint32_t i = 0; i < n; ++i) {
        uint8_t *f = arena.data() + (size_t)i * 64;
        f[12] = 0x08;                       // IPv4 ethertype
        f[14] = 0x45;                       // version 4, ihl 5
        f[17] = 46;                         // ip_len
        f[22] = 64;                         // ttl
        f[23] = 17;                         // UDP
        desc[2 * i] = i * 64;
        desc[2 * i + 1] = 60;
    }
    std::string conf = argc > 4 ? std::string(argv[4])
                                : "GPUIPCheckClassify(OFFSET 14, CHECKSUM true, N 16, LB_MODE hash, BATCH " + batch + ")";
    auto run = [&](const char *c, double *pps, char *err) {
        return reps ? fcclick_bench_threads(c, arena.data(), desc.data(), n, 32, reps, threads, pps, err, 512)
                    : fcclick_bench_timed(c, arena.data(), desc.data(), n, 32, 2.0, threads, pps, err, 512);
    };
    double pps = 0;
    char err[512] = {0};
    const int rc = run(conf.c_str(), &pps, err);
    if (rc) {
        fprintf(stderr, "error %d: %s\n", rc, err);
        return 1;
    }
    double floor = 0;
    run("Pass", &floor, err);
    printf("{\"threads\": %u, \"batch\": \"%s\", \"method\": \"%s\", \"element_mpps\": %.1f, \"floor_mpps\": %.1f, "
           "\"element_ns_per_pkt_per_thread\": %.2f}\n",
           threads, batch.c_str(), reps ? "passes" : "timed 2 s", pps / 1e6, floor / 1e6, threads * 1e9 / pps);
    return 0;
}
