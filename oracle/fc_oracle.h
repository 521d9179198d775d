/*
 * fc_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * Scalar CPU restatement of the FastClick receive-path elements, used as the
 * parity checker for the HIP path (tests/, __graft_entry__.smoke(), and
 * bench.py's cpu_baseline leg). Nothing in fastclick_amd/ may include, link or
 * call this code. Each function cites the reference file:line it restates.
 *
 * Parity pin: the restatement is checked against golden vectors produced by the
 * compiled reference (tests/golden/, generator tests/golden/gen_golden.py).
 */
#ifndef FC_ORACLE_H
#define FC_ORACLE_H
#include <stdint.h>
#include "../include/fastclick_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* A1: lib/in_cksum.c:20-51 */
uint16_t fco_in_cksum_pseudohdr(uint16_t data_csum, const uint8_t *iph, int packet_len);
uint16_t fco_in_cksum(const uint8_t *addr, int len);

/* Per-packet result of the fused chain (same meaning as the GPU outputs). */
typedef struct fco_result {
    uint8_t    reason;   /* FCGPU_R_* */
    uint8_t    port;     /* output index; nports for the invalid list */
    uint32_t   hash;
    fcgpu_anno anno;
    uint32_t   ip_rw;    /* IP header bytes 8..11 as a packet that leaves with R_OK leaves (cfg.rewrite), else 0 */
} fco_result;

/* A2 (+A4/A13/A14): one packet through the configured check chain, then
 * A5-A7/A15 hashing and A8/A9 classification. */
void fco_process_packet(const fcgpu_cfg *cfg, const uint8_t *frame, uint32_t len,
                        fco_result *r);

/* Batch driver over the arena+descriptor layout, same outputs as the device
 * path: verdict/hash/anno arrays may be NULL. perm/port_start as A10
 * (CLASSIFY_EACH_PACKET stable partition, include/click/packetbatch.hh:259-307).
 * counters (FCGPU_NCOUNTERS) are accumulated (not reset). */
void fco_process_batch(const fcgpu_cfg *cfg, const uint8_t *arena, const uint32_t *desc,
                       uint32_t n, uint16_t *verdict, uint32_t *hash, fcgpu_anno *anno,
                       uint32_t *perm, uint32_t *port_start, uint64_t *counters);

/* Same, plus the FCGPU_PART_TILE outputs (perm_tile, tile_count) and the
 * header rewrites (ip_rw, may be NULL). */
void fco_process_batch2(const fcgpu_cfg *cfg, const uint8_t *arena, const uint32_t *desc,
                        uint32_t n, uint16_t *verdict, uint32_t *hash, fcgpu_anno *anno,
                        uint32_t *perm, uint32_t *port_start, uint32_t *perm_tile,
                        uint16_t *tile_count, uint64_t *counters, uint32_t *ip_rw);

/* Decision program for FCGPU_CLS_PROGRAM (A11): the oracle keeps one
 * (process-global; test use is single-threaded). Same step format as the ABI. */
void fco_set_program(uint32_t kind, const fcgpu_step *steps, uint32_t nsteps, int32_t all);
/* IPFilter::match / Classifier Program::match on one packet whose anno holds
 * nh/th/length (after the check): returns the output, or 0x7fff if none. */
uint32_t fco_run_program(const uint8_t *frame, const fcgpu_anno *a);

/* Flow table (FlowIPManagerHMP, elements/research/flowipmanagerhmp.cc:96-126):
 * IDs in order of first appearance, persistent across fco_flow_batch calls.
 * verdict/anno are this batch's fco_process_batch outputs. */
typedef struct fco_flowtab fco_flowtab;
fco_flowtab *fco_flow_new(uint32_t max_flows);
void fco_flow_free(fco_flowtab *t);
uint32_t fco_flow_count(const fco_flowtab *t);
void fco_flow_batch(fco_flowtab *t, const uint8_t *arena, const uint32_t *desc, uint32_t n,
                    const uint16_t *verdict, const fcgpu_anno *anno, uint32_t *flowid);

/* Flow table with timeouts (VirtualFlowManagerIMP + FlowManagerIMPState,
 * include/click/flow/virtualflowmanager.hh): IDs from a LIFO free-ID stack,
 * a timer wheel expiring idle flows, released IDs reused one maintainer run
 * later. Times in ms. See fc_oracle.c for the rules. */
typedef struct fco_imp fco_imp;
fco_imp *fco_imp_new(uint32_t capacity, uint32_t timeout_s, uint32_t recycle_ms);
void fco_imp_free(fco_imp *t);
void fco_imp_batch(fco_imp *t, const uint8_t *arena, const uint32_t *desc, uint32_t n,
                   const uint16_t *verdict, const fcgpu_anno *anno, uint32_t now_ms, uint32_t *flowid);
uint32_t fco_imp_maintain(fco_imp *t, uint32_t now_ms);
void fco_imp_stats(const fco_imp *t, uint32_t *count, uint32_t *free_ids, uint32_t *pending);

/* Individual pieces, exposed for known-answer tests. */
uint32_t fco_ipflowid_hash(uint32_t saddr_raw, uint16_t sport_net,
                           uint32_t daddr_raw, uint16_t dport_net);  /* A6 */
uint32_t fco_ip6flowid_hash(const uint8_t src[16], uint16_t sport_net,
                            const uint8_t dst[16], uint16_t dport_net); /* A15 */
int fco_lb_hash_port(uint32_t h, int n);                         /* A8 direct_hash */
uint32_t fco_crc32c_u32(uint32_t data, uint32_t crc);           /* rte_hash_crc_4byte */
int fco_lb_crc_port(uint32_t proto, uint32_t saddr, uint32_t daddr, uint32_t ports, int n); /* A8 direct_hash_crc */
int fco_hash_ip_port(const uint8_t *data, uint32_t len, int n);  /* A8 hash_ip */
int fco_hashswitch_port(const uint8_t *data, uint32_t len, int off, int l, int n); /* A9 */
void fco_lb_hash_ring(uint32_t nsel, uint32_t size, uint32_t *ring);  /* A8 cst_hash_agg ring */
void fco_set_lb_table(const uint8_t *t, uint32_t n);
int fco_lb_table_port(uint32_t h);
void fco_classify_each_packet(int nbatches, const int *port, uint32_t n,
                              uint32_t *perm, uint32_t *start); /* A10 */
/* A10 applied to consecutive `tile`-packet batches (FCGPU_PART_TILE layout):
 * perm[t*tile ...] = tile t's packet indices grouped by output, tile_count
 * [t*nbatches + b] = run sizes. */
void fco_partition_tiles(int nbatches, const int *port, uint32_t n, uint32_t tile,
                         uint32_t *perm, uint16_t *tile_count);

#ifdef __cplusplus
}
#endif
#endif
