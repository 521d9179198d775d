// fcgpu_part.hh -- the whole-batch partition passes after k_rx
// (FCGPU_PART_GLOBAL: k_scan / k_scan_multi, k_part_multi) and the mbuf
// descriptor pass ahead of it (k_mbuf_desc, fcgpu_process_mbufs). Included by
// fcgpu_process.hip alone, which launches them.
#pragma once
#include "fcgpu_device.hh"

namespace fcgpu {

// Exclusive scan of one output's per-tile counts (in place) and its total.
// grid = nports+1 blocks of 1024 threads.
__device__ __forceinline__ void scan_column(uint32_t *tilecnt, uint32_t ntiles, uint32_t *totals, uint32_t b) {
    __shared__ uint32_t s_w[16];
    uint32_t *col = tilecnt + (size_t)b * ntiles;
    const uint32_t per = (ntiles + 1023) / 1024;
    const uint32_t beg = threadIdx.x * per;
    // a thread's first kScanRegs counts stay in registers for the second
    // pass (a 1M-packet batch has 4 per thread): one round trip to memory
    constexpr uint32_t kScanRegs = 8;
    uint32_t keep[kScanRegs];
    uint32_t sum = 0;
#pragma unroll
    for (uint32_t j = 0; j < kScanRegs; ++j) {
        const uint32_t t = beg + j;
        keep[j] = j < per && t < ntiles ? col[t] : 0u;
        sum += keep[j];
    }
    for (uint32_t j = kScanRegs; j < per; ++j) {
        const uint32_t t = beg + j;
        if (t < ntiles) sum += col[t];
    }
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t incl = sum;
#pragma unroll
    for (int dlt = 1; dlt < 64; dlt <<= 1) {
        const uint32_t v = __shfl_up(incl, dlt);
        if (lane >= (uint32_t)dlt) incl += v;
    }
    if (lane == 63) s_w[wave] = incl;
    __syncthreads();
    uint32_t wpre = 0, total = 0;
    for (uint32_t w = 0; w < 16; ++w) {
        const uint32_t v = s_w[w];
        if (w < wave) wpre += v;
        total += v;
    }
    uint32_t run = wpre + incl - sum;
#pragma unroll
    for (uint32_t j = 0; j < kScanRegs; ++j) {
        const uint32_t t = beg + j;
        if (j < per && t < ntiles) {
            col[t] = run;
            run += keep[j];
        }
    }
    for (uint32_t j = kScanRegs; j < per; ++j) {
        const uint32_t t = beg + j;
        if (t < ntiles) {
            const uint32_t v = col[t];
            col[t] = run;
            run += v;
        }
    }
    if (threadIdx.x == 0) totals[b] = total;
}
__global__ __launch_bounds__(1024) void k_scan(uint32_t *tilecnt, uint32_t ntiles, uint32_t *totals) {
    scan_column(tilecnt, ntiles, totals, blockIdx.x);
}
// The batches of a fused launch (fcgpu_process_jobs): block (b, j) scans
// output b of batch j.
struct ScanMulti {
    uint32_t *tilecnt[kMaxFuseJobs];
    uint32_t *totals[kMaxFuseJobs];
    uint32_t ntiles[kMaxFuseJobs];
};
__global__ __launch_bounds__(1024) void k_scan_multi(ScanMulti M) {
    const uint32_t j = blockIdx.y;
    scan_column(M.tilecnt[j], M.ntiles[j], M.totals[j], blockIdx.x);
}

// The scatter pass of the dense whole-batch partition (CLASSIFY_EACH_PACKET
// order over each batch): perm[start[bin] + tile offset + rank] = i, for one
// batch or the batches of a fused launch; the grid is their tile groups end to
// end (a batch without perm has one workgroup, for its port_start).
struct PartMulti {
    const uint16_t *verdict[kMaxFuseJobs];
    const uint32_t *tileoff[kMaxFuseJobs];
    const uint32_t *totals[kMaxFuseJobs];
    uint32_t *perm[kMaxFuseJobs];
    uint32_t *port_start[kMaxFuseJobs];
    uint32_t n[kMaxFuseJobs];        // 0 for a batch without perm
    uint32_t ntiles[kMaxFuseJobs];   // the batch's tile count (its tileoff columns)
    uint32_t wg0[kMaxFuseJobs];      // first workgroup of the batch
    uint32_t g, nports;
    uint32_t tpw;                    // tiles per workgroup (1..kPartTiles)
};
// Each workgroup scatters tpw consecutive tiles of its batch (one tile per
// workgroup left the pass bound by the workgroup dispatch rate: 7 us per
// 1M-packet batch for 6 MB of traffic; the host picks tpw so the grid still
// fills the machine), the next tile's verdicts and column offsets loaded while
// the current one is ranked and scattered.
constexpr uint32_t kPartTiles = 8;
__global__ __launch_bounds__(kTile) void k_part_multi(PartMulti M) {
    __shared__ uint32_t s_cnt[4][FCGPU_MAX_PORTS + 1];
    __shared__ uint32_t s_base[FCGPU_MAX_PORTS + 2];
    __shared__ uint32_t s_off[2][FCGPU_MAX_PORTS + 1];
    uint32_t j = 0;
    for (uint32_t k = 1; k < M.g; ++k) j = blockIdx.x >= M.wg0[k] ? k : j;   // workgroup-uniform
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6, tid = threadIdx.x;
    const uint32_t nb = M.nports + 1, n = M.n[j], ntiles = M.ntiles[j];
    const uint32_t t0 = (blockIdx.x - M.wg0[j]) * M.tpw;
    const uint32_t nt = n ? ntiles : 1u;
    const uint16_t *verdict = M.verdict[j];
    const uint32_t *tileoff = M.tileoff[j];
    // the outputs' starts, from the batch's totals
    if (tid < nb) s_cnt[0][tid] = M.totals[j][tid];
    __syncthreads();
    if (tid == 0) {
        uint32_t acc = 0;
        for (uint32_t b = 0; b < nb; ++b) { s_base[b] = acc; acc += s_cnt[0][b]; }
        s_base[nb] = acc;
    }
    __syncthreads();
    if (t0 == 0 && M.port_start[j] && tid <= nb) M.port_start[j][tid] = s_base[tid];
    const uint64_t lt = (1ull << lane) - 1ull;
    const uint32_t nbits = 32 - __clz(nb - 1 | 1);
    // every tile's verdicts and offsets are loaded up front (registers, the
    // loops unrolled over kPartTiles): the tiles' work then waits for memory
    // once, not once per tile
    uint32_t vv[kPartTiles], oo[kPartTiles];
#pragma unroll
    for (uint32_t u = 0; u < kPartTiles; ++u) {
        vv[u] = 0xffffu;
        oo[u] = 0;
        if (u < M.tpw && t0 + u < nt) {
            const uint32_t i = (t0 + u) * kTile + tid;
            if (i < n) vv[u] = verdict[i];
            if (tid < nb && n) oo[u] = tileoff[(size_t)tid * ntiles + t0 + u];
        }
    }
#pragma unroll
    for (uint32_t u = 0; u < kPartTiles; ++u) {
        if (u >= M.tpw || t0 + u >= nt) break;   // workgroup-uniform
        const uint32_t tile = t0 + u, i = tile * kTile + tid;
        const uint32_t v = vv[u], off = oo[u];
        const bool live = i < n;
        const uint32_t bin = live ? (v >> 8) : 0xffffffffu;
        const uint64_t grp = match_any(bin, nbits, __ballot(live));
        const uint32_t rank = (uint32_t)__popcll(grp & lt);
        for (uint32_t b = lane; b < nb; b += 64) s_cnt[wave][b] = 0;
        if (tid < nb) s_off[u & 1][tid] = off;
        __builtin_amdgcn_wave_barrier();
        if (live && rank == 0) s_cnt[wave][bin] = (uint32_t)__popcll(grp);
        __syncthreads();
        if (live) {
            uint32_t wpre = 0;
            for (uint32_t w = 0; w < wave; ++w) wpre += s_cnt[w][bin];
            M.perm[j][s_base[bin] + s_off[u & 1][bin] + wpre + rank] = i;
        }
        __syncthreads();   // the counts are read before the next tile resets them
    }
}

// ---- mbuf ingress: descriptors from the mbufs themselves -------------------
// One lane per mbuf pointer (host virtual address). The pointer and the frame
// are checked against the registered pool before anything is dereferenced;
// the header fields are read from host memory over PCIe (header_bytes <= 64). desc[i] = (frame
// offset from the pool base, data_len), or (0, 0) for a pointer or frame
// outside the pool (or too close to its end for the header-window read).
struct MbufArgs {
    const uint64_t *ptrs;     // [n] host virtual addresses of the mbufs (device copy)
    uint32_t n;
    uint64_t pool_host;       // registered pool: host VA
    uint64_t pool_bytes;
    const uint8_t *pool_dev;  // its device address
    uint32_t f_buf, f_off, f_len, hdr;   // fcgpu_mbuf_layout
    uint2 *desc;              // [n] out
};
// The mbuf headers travel over PCIe: each wave fetches its 64 mbufs' first 64
// bytes as whole 64-B segments (4 lanes x 16 B per mbuf, LDS-DMA, the k_rx
// window pattern) -- one read request per mbuf instead of one per field --
// then each lane takes its fields from LDS.
__global__ __launch_bounds__(256) void k_mbuf_desc(MbufArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t s_hdr[4 * kWave * 64];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    uint64_t m = i < a.n ? a.ptrs[i] : 0;
    // a pointer outside the pool is never dereferenced: read the pool's first
    // header instead and discard it
    const bool inpool = m >= a.pool_host && m - a.pool_host + 64 <= a.pool_bytes && a.hdr <= 64;
    const uint64_t src = inpool ? m - a.pool_host : 0;
    uint8_t *hl = s_hdr + wave * (kWave * 64);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t p = k * 16 + (lane >> 2);
        const uint32_t lo = __shfl((uint32_t)src, (int)p), hi = __shfl((uint32_t)(src >> 32), (int)p);
        const uint64_t o = ((uint64_t)hi << 32 | lo) + (lane & 3) * 16;
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(a.pool_dev + o),
                                         (__attribute__((address_space(3))) void *)(hl + k * 1024), 16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    if (i >= a.n) return;
    // row p of instruction k sits at k*1024 + (p%16)*64: this lane's is lane/16, lane%16
    const uint8_t *h = hl + (lane >> 4) * 1024 + (lane & 15) * 64;
    uint2 d = make_uint2(0, 0);
    if (inpool) {
        uint64_t buf;
        uint16_t off, len;
        memcpy(&buf, h + a.f_buf, 8);
        memcpy(&off, h + a.f_off, 2);
        memcpy(&len, h + a.f_len, 2);
        const uint64_t f = buf + off;
        // the ABI's over-read allowance (128 B past the start, 16 B past the
        // end of every frame) must stay inside the registered pool too
        const uint64_t reach = len + 16u > 128u ? len + 16u : 128u;
        if (f >= a.pool_host && f - a.pool_host + reach <= a.pool_bytes)
            d = make_uint2((uint32_t)(f - a.pool_host), len);
    }
    a.desc[i] = d;
}

}  // namespace fcgpu
