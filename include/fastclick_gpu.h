/*
 * fastclick_gpu.h -- C ABI of the MI355X receive-path element library
 * (libfcgpu.so, HIP for gfx950).
 *
 * One call processes one batch of packets through the fused chain
 *
 *     [StripEtherVLANHeader] -> CheckIPHeader | CheckIP6Header | MarkIPHeader
 *         -> AggregateHash (IPFlowID / IPFlow5ID / IP6FlowID low-32 hash)
 *         -> per-port classify (FlowSwitch LB hash, LB hash_ip, HashSwitch)
 *         -> stable per-port partition (CLASSIFY_EACH_PACKET)
 *
 * and replaces, for a FastClick BatchElement, the per-packet loops
 *   - CheckIPHeader::valid            elements/ip/checkipheader.cc:163-226
 *   - click_in_cksum                  lib/in_cksum.c:20-51
 *   - IPFlowID::hashcode              include/click/ipflowid.hh:153-164
 *   - IPFlow5ID::hashcode             include/click/ipflowid.hh:242-251
 *   - AggregateHash::simple_action    elements/analysis/aggregatehash.cc:49-55
 *   - LoadBalancer::pick_server       include/click/loadbalancer.hh:553-584
 *   - HashSwitch::process             elements/standard/hashswitch.cc:50-66
 *   - StripEtherVLANHeader::simple_action elements/ethernet/stripethervlanheader.cc:48-61
 *   - CheckIP6Header::simple_action   elements/ip6/checkip6header.cc:105-168
 *   - IP6FlowID::hashcode             include/click/ip6flowid.hh:220-230
 *   - CLASSIFY_EACH_PACKET            include/click/packetbatch.hh:259-307
 * (SURVEY.md section 8(a) rows A1-A15). The FastClick-side caller is the
 * GPUIPCheckClassify element (fastclick_amd/csrc/host/), which keeps the
 * Element::push_batch API (include/click/element.hh:53-54) and calls this ABI.
 *
 * Batch layout ("arena + descriptor"):
 *   arena : bytes; packet i's frame starts at arena + desc[2i] and is
 *           desc[2i+1] bytes long. The arena must stay readable for 128 bytes
 *           past every frame start and 16 bytes past every frame end
 *           (header-window over-read; bytes outside the frame never decide a
 *           verdict).
 *   desc  : uint32 pairs (offset, length), 8 bytes per packet.
 * Results are per-packet structure-of-arrays; every output pointer may be NULL
 * (that output is then not produced).
 *
 * Errors: every int-returning entry point returns FCGPU_OK (0) or a negative
 * FCGPU_E* code; fcgpu_last_error() gives the message. There is no silent
 * fallback: a missing device or a failed launch is an error return.
 */
#ifndef FASTCLICK_GPU_H
#define FASTCLICK_GPU_H

#ifndef __HIPCC_RTC__   /* hiprtc (fcgpu_set_program's compiled programs) has its own */
#include <stddef.h>
#include <stdint.h>
#endif

#ifdef __cplusplus
extern "C" {
#endif

#define FCGPU_ABI_VERSION 25

#define FCGPU_OK          0
#define FCGPU_EINVAL     -1   /* bad argument / configuration            */
#define FCGPU_ENODEV     -2   /* no HIP device / device not usable       */
#define FCGPU_ENOMEM     -3   /* allocation failed / batch > max_batch   */
#define FCGPU_ERUNTIME   -4   /* HIP runtime or kernel launch failure    */

/* Verdict reason codes. 0..6 are CheckIPHeader::Reason
 * (elements/ip/checkipheader.hh:139-147); 6 = NREASONS = valid. */
#define FCGPU_R_MINISCULE   0
#define FCGPU_R_BAD_VERSION 1
#define FCGPU_R_BAD_HLEN    2
#define FCGPU_R_BAD_IP_LEN  3
#define FCGPU_R_BAD_CKSUM   4
#define FCGPU_R_BAD_SADDR   5
#define FCGPU_R_OK          6
#define FCGPU_R_BAD_IP6     7   /* CheckIP6Header's single drop reason      */
#define FCGPU_R_VLAN_REJECT 8   /* StripEtherVLANHeader output 1 (untagged, NATIVE_VLAN < 0) */
#define FCGPU_R_NO_MATCH    9   /* valid, but the classifier program matched no output:
                                   CLASSIFY_EACH_PACKET kills it (packetbatch.hh:268)  */
/* CheckUDPHeader / CheckTCPHeader::Reason (elements/tcpudp/checkudpheader.hh:83-87,
 * checktcpheader.hh:83-87) for IPv4-valid packets, when l4_mode is set: */
#define FCGPU_R_L4_PROTO    10  /* NOT_UDP / NOT_TCP                         */
#define FCGPU_R_L4_LENGTH   11  /* BAD_LENGTH                                */
#define FCGPU_R_L4_CKSUM    12  /* BAD_CHECKSUM (pseudo-header checksum)     */
/* Header rewrite stage (cfg.rewrite), after the classifier, on packets it let through: */
#define FCGPU_R_TTL_EXPIRED 13  /* DecIPTTL output 1: ip_ttl <= 1 (decipttl.cc:62-65)          */
#define FCGPU_R_SETCKSUM_BAD 14 /* SetIPChecksum "bad input packet": kill (setipchecksum.cc:44-56) */
#define FCGPU_NREASON_SLOTS 14  /* counters for reasons 0-5, 7-14            */
/* Reasons >= FCGPU_R_NO_MATCH are decided after CheckIPHeader accepted the
 * packet: they count in "count", not in "drops". */

/* check_mode */
#define FCGPU_CHECK_IP4   0   /* CheckIPHeader(OFFSET o[, CHECKSUM c, BADSRC, GOODDST]) */
#define FCGPU_MARK_IP4    1   /* MarkIPHeader(o): no validation                         */
#define FCGPU_CHECK_AUTO  2   /* StripEtherVLANHeader(NATIVE_VLAN) at o, then by IP version
                                 nibble: 6 -> CheckIP6Header, else -> CheckIPHeader.
                                 With vlan_ethertype: VLANDecap(ETHERTYPE) + Strip(14)
                                 (elements/ethernet/vlandecap.cc:49-70): same offsets,
                                 untagged -> tci 0 (native_vlan 0)                     */
#define FCGPU_MARK_IP6    3   /* MarkIP6Header(o) (elements/ip6/markip6header.cc:43-48): no
                                 validation, nh = o, th = o + 40; IP6FlowID hash        */
/* hash_mode (written to the AGGREGATE annotation output) */
#define FCGPU_HASH_NONE     0
#define FCGPU_HASH_FLOWID   1   /* IPFlowID(p).hashcode() low 32 (AggregateHash); v6: IP6FlowID */
#define FCGPU_HASH_FLOW5ID  2   /* IPFlow5ID(p).hashcode() low 32 (adds ip_p)               */
/* classify */
#define FCGPU_CLS_NONE       0  /* every valid packet -> port 0                          */
#define FCGPU_CLS_LB_HASH    1  /* LoadBalancer direct_hash / direct_hash_agg:
                                   ((H>>16) ^ (H&0xffff)) % nports                       */
#define FCGPU_CLS_HASH_IP    2  /* LoadBalancer direct_hash_ip (frame bytes 26..33)      */
#define FCGPU_CLS_HASHSWITCH 3  /* HashSwitch(hs_offset, hs_length), nports = MAX        */
#define FCGPU_CLS_PROGRAM    4  /* decision program set by fcgpu_set_program: IPFilter /
                                   IPClassifier or Classifier                          */
#define FCGPU_CLS_LB_CRC     5  /* LoadBalancer direct_hash_crc (DPDK builds,
                                   include/click/loadbalancer.hh:563-569): c = CRC32-C of
                                   the IPFlow5ID words proto, saddr, daddr, ports from 0
                                   (ipv4_hash_crc, include/click/dpdk_glue.hh:13-27, via
                                   rte_hash_crc_4byte = the SSE4.2 crc32 instruction), port =
                                   ((c>>16) ^ (c&0xffff)) % nports. IPv4 check modes only */
#define FCGPU_CLS_LB_TABLE   6  /* LoadBalancer constant_hash_agg (include/click/
                                   loadbalancer.hh:585-589): port = table[((H>>16) ^
                                   (H&0xffff)) % buckets], H the hash_mode hash; the table
                                   (the reference's consistent-hash ring, :170-189) is set
                                   by fcgpu_set_lb_table */

/* l4_mode: a CheckUDPHeader / CheckTCPHeader after the IPv4 check (CHECK_IP4 or
 * MARK_IP4 only). The checksum covers the whole L4 segment, so with
 * l4_checksum the device reads every byte of the packet, not only the header
 * window. */
#define FCGPU_L4_NONE 0
#define FCGPU_L4_UDP  1
#define FCGPU_L4_TCP  2

/* rewrite flags: header rewrites after the classifier on IPv4 packets it sent
 * to an output. The rewritten bytes 8..11 of the IP header
 * (ttl, protocol, checksum) come back in fcgpu_out.ip_rw; with
 * FCGPU_RW_INPLACE they are also stored into the arena (device path). */
#define FCGPU_RW_DECTTL   1u  /* DecIPTTL: ttl <= 1 -> FCGPU_R_TTL_EXPIRED, else ttl-1 and the
                                 RFC 1624 incremental checksum (elements/ip/decipttl.cc:52-78) */
#define FCGPU_RW_SETCKSUM 2u  /* SetIPChecksum: full header checksum (elements/ip/setipchecksum.cc:38-58),
                                 after DecIPTTL when both are set                          */
#define FCGPU_RW_INPLACE  4u

#define FCGPU_MAX_PORTS   64
#define FCGPU_MAX_ADDRS   16

typedef struct fcgpu_cfg {
    uint32_t size;            /* = sizeof(fcgpu_cfg)                                     */
    uint32_t check_mode;      /* FCGPU_CHECK_*                                           */
    int32_t  offset;          /* OFFSET: frame start -> IP header (CHECK_IP4/MARK_IP4),
                                 or frame start -> Ethernet header (CHECK_AUTO)          */
    uint32_t checksum;        /* CHECKSUM; the reference default is FALSE
                                 (elements/ip/checkipheader.cc:110)          */
    uint32_t hash_mode;       /* FCGPU_HASH_*                                            */
    uint32_t classify;        /* FCGPU_CLS_*                                             */
    uint32_t nports;          /* classify outputs N (1..FCGPU_MAX_PORTS)                 */
    int32_t  hs_offset;       /* HashSwitch OFFSET (frame-relative)                      */
    int32_t  hs_length;       /* HashSwitch LENGTH (> 0)                                 */
    int32_t  native_vlan;     /* StripEtherVLANHeader NATIVE_VLAN (default 0; <0 reject) */
    uint32_t nbadsrc;         /* BADSRC list (raw network-order s_addr words)            */
    uint32_t ngooddst;        /* GOODDST list                                             */
    uint32_t badsrc[FCGPU_MAX_ADDRS];
    uint32_t gooddst[FCGPU_MAX_ADDRS];
    uint32_t nbad6;           /* CheckIP6Header bad source list; default = {ff..ff}      */
    uint8_t  bad6[FCGPU_MAX_ADDRS][16];
    uint32_t process_eh;      /* CheckIP6Header PROCESS_EH: follow hop-by-hop, routing,
                                 fragment and AH extension headers (ip6_follow_eh,
                                 include/click/ip6address.hh:417-448)                    */
    uint32_t l4_mode;         /* FCGPU_L4_*                                               */
    uint32_t l4_checksum;     /* CheckUDPHeader/CheckTCPHeader CHECKSUM (reference default
                                 TRUE: checkudpheader.cc:54, checktcpheader.cc)          */
    uint32_t rewrite;         /* FCGPU_RW_* (IPv4 check modes)                            */
    uint32_t ttl_multicast;   /* DecIPTTL MULTICAST (default true: decrement multicast too) */
    uint32_t vlan_ethertype;  /* CHECK_AUTO tag protocol: 0x8100 (StripEtherVLANHeader, and
                                 VLANDecap's default) or VLANDecap ETHERTYPE (e.g. 0x88a8) */
} fcgpu_cfg;

/* Optional per-packet annotations (16 B), mirroring what the reference
 * elements leave on a valid packet. Offsets are relative to the frame start the
 * element received (the descriptor offset). */
typedef struct fcgpu_anno {
    uint32_t dst_ip;          /* DST_IP_ANNO (IPv4 valid) = raw ip_dst word             */
    uint16_t length;          /* packet length after Packet::take() trimming            */
    uint16_t vlan_tci;        /* VLAN_TCI_ANNO, raw network order (CHECK_AUTO)          */
    uint16_t nh;              /* network header offset (set_ip_header / set_ip6_header) */
    uint16_t th;              /* transport header offset (IPv6: after the extension
                                 headers when process_eh)                              */
    uint8_t  ip6_nxt;         /* IP6_NXT_ANNO (IPv6 valid)                              */
    uint8_t  ipver;           /* 4 or 6 for packets that reached a checker, else 0      */
    uint16_t reserved;
} fcgpu_anno;

/* Stable per-output partition (CLASSIFY_EACH_PACKET, packetbatch.hh:259-307),
 * selected by fcgpu_out.partition:
 *   FCGPU_PART_GLOBAL: the whole batch is one PacketBatch. perm[n] lists packet
 *       indices grouped by output in input order; output b occupies
 *       perm[port_start[b] .. port_start[b+1]). Three launches.
 *   FCGPU_PART_TILE: the batch is a sequence of FCGPU_TILE-packet PacketBatches
 *       (the element's input batches), each partitioned on its own, exactly as
 *       a ClassifyElement partitions every batch it receives. Tile t's entries
 *       are perm[t*FCGPU_TILE ...] (packet index) and/or tile_perm[t*FCGPU_TILE
 *       ...] (index within the tile, 1 byte), grouped by output;
 *       tile_count[t*(nports+1)+b] is the size of output b's run in tile t.
 *       One fused launch.                                                   */
#define FCGPU_PART_GLOBAL 0
#define FCGPU_PART_TILE   1
#define FCGPU_TILE        256

typedef struct fcgpu_out {
    uint16_t   *verdict;      /* [n] reason | (output port << 8); invalid -> port nports */
    uint32_t   *hash;         /* [n] AGGREGATE annotation (0 unless valid)               */
    fcgpu_anno *anno;         /* [n] optional annotations                                */
    uint32_t   *perm;         /* [n] packet indices grouped by output, input order kept  */
    uint32_t   *port_start;   /* GLOBAL: [nports+2] start of each output's run in perm   */
    uint16_t   *tile_count;   /* TILE: [ceil(n/FCGPU_TILE)][nports+1] run sizes          */
    uint32_t    partition;    /* FCGPU_PART_GLOBAL or FCGPU_PART_TILE                    */
    uint32_t    reserved;
    uint8_t    *tile_perm;    /* TILE: [n] index within the tile, grouped by output      */
    uint32_t   *flowid;       /* [n] flow ID from the context's flow table (fcgpu_flow_enable);
                                 FCGPU_FLOW_NONE for packets that reach no flow manager */
    uint32_t   *ip_rw;        /* [n] with cfg.rewrite: IP header bytes 8..11 after the rewrite
                                 (little-endian load: ttl | proto << 8 | checksum bytes << 16);
                                 for every packet that leaves with FCGPU_R_OK, rewritten
                                 or not (a rewritten word may be 0: compare it with the
                                 packet's bytes to see a change); 0 for the rest        */
} fcgpu_out;

typedef struct fcgpu_ctx fcgpu_ctx;

/* Counter vector layout returned by fcgpu_read_counters (uint64):
 *   [0] count (valid packets)         CheckIPHeader "count"
 *   [1] drops                         CheckIPHeader "drops"
 *   [2 .. 2+14) reason slots for reasons 0-5, 7, 8 ("drop_details") and
 *               9-14 (no classifier match, L4 checks, DecIPTTL / SetIPChecksum;
 *               not drops of the checker)
 *   [16 .. 16+nports+1) per-output packet counts, last = invalid list       */
#define FCGPU_CTR_COUNT   0
#define FCGPU_CTR_DROPS   1
#define FCGPU_CTR_REASON  2
#define FCGPU_CTR_PORT    16
#define FCGPU_NCOUNTERS   (FCGPU_CTR_PORT + FCGPU_MAX_PORTS + 1)
/* On the device the vector is kept in FCGPU_CTR_SHARDS replicas (tiles add to
 * replica tile % FCGPU_CTR_SHARDS) and summed on read, like per_thread<>
 * counters summed by PER_THREAD_SUM (include/click/sync.hh:56,384). */
#define FCGPU_CTR_SHARDS  64

int  fcgpu_abi_version(void);
int  fcgpu_device_count(void);
void fcgpu_default_cfg(fcgpu_cfg *cfg);

/* Open a context on HIP device `device` for batches of up to max_batch packets.
 * One context per (Click thread x stream); a context is not thread-safe. */
int  fcgpu_open(int device, uint32_t max_batch, fcgpu_ctx **out);
int  fcgpu_configure(fcgpu_ctx *ctx, const fcgpu_cfg *cfg);
void fcgpu_close(fcgpu_ctx *ctx);

/* Device-resident batch: arena, desc and every output pointer are device
 * memory. Asynchronous on `stream` (a hipStream_t; NULL = the HIP null stream,
 * as everywhere in HIP). Completion: synchronise that stream. */
int  fcgpu_process(fcgpu_ctx *ctx, const uint8_t *d_arena, const uint32_t *d_desc,
                   uint32_t n, const fcgpu_out *d_out, void *stream);

/* fcgpu_process for a batch whose size is known only on the device: the
 * first *d_count - base packets (at most n_max) of d_desc are processed, the
 * launch covers n_max. No host sync: what a received re-shard batch goes
 * through (fcgpu_exchange_unpack_fixed writes *d_count), in chunks of
 * max_batch (base = the chunk's first packet). Outputs are those of
 * fcgpu_process for the processed packets (per-tile counts of the tiles past
 * them are 0); a whole-batch partition (FCGPU_PART_GLOBAL with perm or
 * port_start) is refused. */
int  fcgpu_process_counted(fcgpu_ctx *ctx, const uint8_t *d_arena, const uint32_t *d_desc, uint32_t n_max,
                           const uint32_t *d_count, uint32_t base, const fcgpu_out *d_out, void *stream);

/* Several independent device-resident batches in one call -- e.g. the
 * batches of several rx queues, or a ring of batches a NIC filled: job k is
 * processed exactly as fcgpu_process(ctx, jobs[k].arena, jobs[k].desc,
 * jobs[k].n, &jobs[k].out, jobs[k].stream ? jobs[k].stream : stream), in
 * order, with one argument check and one device switch for the set. Jobs on
 * different streams run concurrently (their outputs must not overlap); that
 * is rejected when the context has a flow table or a job asks for a
 * whole-batch partition (both use context scratch). Every job is checked
 * before the first is launched.
 * Consecutive jobs of one stream whose outputs do not overlap share one
 * receive-kernel launch (up to 24 batches: the grid is their tiles end to
 * end; 8 with a flow table, whose new-flow passes follow in batch order; a
 * whole-batch partition adds one scan and one scatter launch for them all),
 * unless the context rewrites headers in place (FCGPU_RW_INPLACE: jobs may
 * share an arena) or a whole-batch partition comes without the caller's
 * verdicts or with a flow table; results are the same as one launch per job.
 * Sampled timing (fcgpu_set_timing) then counts batches: a fused launch is
 * timed when it covers a multiple of `every`, and fcgpu_read_timing reports
 * its batches as launches (time per batch = ms / launches). */
typedef struct fcgpu_job {
    const uint8_t  *arena;
    const uint32_t *desc;
    uint32_t        n;
    uint32_t        reserved;
    void           *stream;   /* hipStream_t or NULL (the call's stream)            */
    fcgpu_out       out;
} fcgpu_job;
int  fcgpu_process_jobs(fcgpu_ctx *ctx, const fcgpu_job *jobs, uint32_t njobs, void *stream);

/* Host-resident batch: frames[i] points at packet i's data (length lens[i]).
 * The first min(len, 128) bytes of every frame are gathered into pinned
 * staging, copied H2D, processed, and the requested outputs copied D2H into the
 * host pointers of h_out. Synchronous. Unless a whole-batch partition is asked
 * for (FCGPU_PART_GLOBAL with perm/port_start), the batch is pipelined in
 * chunks of 131,072 packets over three streams, so the gather of one chunk
 * overlaps the copies and kernel of the previous ones; results are identical
 * to one launch over the batch (chunks are whole 256-packet tiles). Outputs
 * are DMA'd straight into h_out arrays that are pinned (fcgpu_host_alloc),
 * otherwise through pinned staging. */
int  fcgpu_process_host(fcgpu_ctx *ctx, const uint8_t *const *frames,
                        const uint32_t *lens, uint32_t n, const fcgpu_out *h_out);

/* Host-resident batch whose frames already lie in one contiguous buffer
 * (e.g. pcap records read straight into pinned memory, include/fcpcap.h):
 * the span and the descriptors go to the device as two H2D copies -- no
 * per-packet gather -- then the kernels run and the requested outputs are
 * copied into the host pointers of h_out. Asynchronous: up to
 * FCGPU_SPAN_SLOTS submissions are in flight, each on its own stream (one
 * stream for all when a flow table is enabled, which needs batch order);
 * h_span, h_desc and h_out must stay valid until fcgpu_span_wait(slot).
 * Pinned buffers (fcgpu_host_alloc) make the copies true DMA. Every frame
 * starts inside the span (desc offsets < span_bytes: the descriptors are the
 * caller's and not checked per packet, as for fcgpu_process's arena) and the
 * span must be readable 128 bytes past every frame start (the context pads
 * its device copy; bytes past the span are never part of a verdict). */
#define FCGPU_SPAN_SLOTS 3
int  fcgpu_span_submit(fcgpu_ctx *ctx, uint32_t slot, const uint8_t *h_span, size_t span_bytes,
                       const uint32_t *h_desc, uint32_t n, const fcgpu_out *h_out);
int  fcgpu_span_wait(fcgpu_ctx *ctx, uint32_t slot);
/* Non-blocking: 1 if the slot's submission has completed (or none is in
 * flight), 0 if it is still running, < 0 on error. */
int  fcgpu_span_poll(fcgpu_ctx *ctx, uint32_t slot);

/* Block submissions: one H2D copy in, one D2H copy out per batch (instead of
 * one per array), for callers that stage into one pinned buffer -- the
 * GPUIPCheckClassify element. h_in holds the descriptors at desc_off and the
 * frames at frames_off (descriptor offsets are relative to frames_off); the
 * first in_bytes of h_in are copied, and the device copy is padded for the
 * header-window over-read. The requested outputs (FCGPU_OUT_* mask) come back
 * in h_out at the offsets fcgpu_block_layout_for() gives for (n, outputs,
 * partition) -- each array 256-B aligned, in the order of the mask bits.
 * Completion, slots and streams as fcgpu_span_submit. */
#define FCGPU_OUT_VERDICT    (1u << 0)
#define FCGPU_OUT_HASH       (1u << 1)
#define FCGPU_OUT_ANNO       (1u << 2)
#define FCGPU_OUT_PERM       (1u << 3)   /* GLOBAL: with port_start; TILE: packet indices */
#define FCGPU_OUT_PORT_START (1u << 4)   /* GLOBAL                                       */
#define FCGPU_OUT_TILE_COUNT (1u << 5)   /* TILE                                         */
#define FCGPU_OUT_TILE_PERM  (1u << 6)   /* TILE                                         */
#define FCGPU_OUT_FLOWID     (1u << 7)
#define FCGPU_OUT_IP_RW      (1u << 8)
/* Instead of FCGPU_OUT_ANNO, for the IPv4 check modes (CHECK_IP4 / MARK_IP4,
 * OFFSET < 256): 8-B annotations (fcgpu_anno8) at the layout's `anno`
 * offset -- half the bytes written back per packet. ipver is 4, vlan_tci and
 * ip6_nxt 0 for these modes; th = nh + thl. */
#define FCGPU_OUT_ANNO8      (1u << 9)
typedef struct fcgpu_anno8 {
    uint32_t dst_ip;          /* as fcgpu_anno                                            */
    uint16_t length;          /* as fcgpu_anno                                            */
    uint8_t  nh;              /* as fcgpu_anno (< 256)                                    */
    uint8_t  thl;             /* th - nh                                                  */
} fcgpu_anno8;
/* Not an output: this one submission goes through copies (H2D of h_in, D2H
 * of the results) whatever the span mode -- never zero-copy, never the shared
 * queue. What an element re-submits a failed batch with (SURVEY 8(b) Errors). */
#define FCGPU_SUBMIT_COPY    (1u << 31)
/* Not an output either: the block's descriptors are one uint32 per packet
 * (n x 4 B at a 4-B aligned desc_off) -- bits 0-15 the frame's offset from
 * frames_off in 8-B units (frames start on 8-B boundaries below 512 KiB),
 * bits 16-31 its length (< 65536) -- half the bytes a zero-copy batch reads
 * for them over PCIe. */
#define FCGPU_SUBMIT_DESC32  (1u << 30)
#define FCGPU_OUT_ABSENT     ((size_t)-1)
typedef struct fcgpu_block_layout {
    size_t verdict, hash, anno, perm, port_start, tile_count, tile_perm, flowid, ip_rw;  /* byte offsets */
    size_t bytes;                                                                       /* block size   */
} fcgpu_block_layout;
int  fcgpu_block_layout_for(const fcgpu_ctx *ctx, uint32_t n, uint32_t outputs, uint32_t partition,
                        fcgpu_block_layout *out);
int  fcgpu_span_submit_block(fcgpu_ctx *ctx, uint32_t slot, const void *h_in, size_t in_bytes,
                             size_t desc_off, size_t frames_off, uint32_t n, void *h_out, uint32_t outputs,
                             uint32_t partition);
/* Reserve every slot's device blocks (an in_bytes input block, a result block
 * for max_batch packets with these outputs) and streams now, on the calling
 * thread, instead of on the first submissions that need them. After it,
 * fcgpu_span_submit_block never allocates, frees or synchronises the device
 * -- not on its copy path, not for an FCGPU_SUBMIT_COPY re-submission while
 * other contexts' batches run on the device's shared queue -- and a block
 * larger than in_bytes is refused (FCGPU_ENOMEM). Without it the first
 * submission through copies sizes the blocks. Call it with no slot in flight
 * (FCGPU_EINVAL otherwise); again to grow the reservation. (Round 6: an
 * element's many threads must not grow device blocks while the shared queue
 * runs) */
int  fcgpu_span_reserve(fcgpu_ctx *ctx, size_t in_bytes, uint32_t outputs, uint32_t partition);

/* How span and block submissions reach the device (per context, default COPY):
 *   FCGPU_SPAN_COPY     -- one H2D copy of h_in and one D2H copy of the
 *                          results per batch, through the copy engine (the
 *                          device copy is padded for the header-window reads);
 *   FCGPU_SPAN_ZEROCOPY -- no copies: the kernels read the descriptors and
 *                          frames from h_in (fcgpu_span_submit: h_span,
 *                          h_desc) and write the results into h_out (the
 *                          h_out arrays) over PCIe, where they lie. All must
 *                          be page-locked (fcgpu_host_alloc, or
 *                          fcgpu_host_register / hipHostRegister), and the
 *                          frames readable 256 bytes past in_bytes /
 *                          span_bytes (the header-window over-read; those
 *                          bytes are never part of a verdict). The context
 *                          remembers each buffer address's device translation
 *                          until the next fcgpu_span_mode call, so a buffer
 *                          freed and replaced at the same address must be
 *                          page-locked as well. Many contexts
 *                          submitting small batches share one copy engine;
 *                          zero-copy batches only queue kernels.
 *   FCGPU_SPAN_AUTO     -- ZEROCOPY while at least 4 contexts of the process
 *                          are in AUTO mode on this device (one per element
 *                          thread), else COPY; decided at each submission.
 *                          Zero-copy block submissions of AUTO contexts then
 *                          share one queue per device: the 4th pending one, or
 *                          a wait/poll on one still pending, launches the
 *                          pending batches together (one kernel launch carries
 *                          several contexts' batches of one configuration, each
 *                          counted in its own context). Flow tables, whole-batch
 *                          partitions and in-place rewrites keep their own
 *                          launches. fcgpu_span_wait / fcgpu_span_poll of a slot
 *                          is how its batch is guaranteed to start.
 * Results are identical in every mode. Returns FCGPU_EINVAL for another mode
 * or while a slot is in flight. */
#define FCGPU_SPAN_COPY     0u
#define FCGPU_SPAN_ZEROCOPY 1u
#define FCGPU_SPAN_AUTO     2u
int  fcgpu_span_mode(fcgpu_ctx *ctx, uint32_t mode);
/* Fault injection (tests of the callers' error paths; process-wide, every
 * context): after `skip` events of kind `where` pass, the next `count` fail
 * as a HIP failure would, with FCGPU_ERUNTIME and a message:
 *   FCGPU_FAULT_SUBMIT -- fcgpu_span_submit / fcgpu_span_submit_block return
 *                         the error; nothing was queued, the slot stays free;
 *   FCGPU_FAULT_WAIT   -- fcgpu_span_submit / fcgpu_span_submit_block accept
 *                         the batch but nothing runs (an asynchronous launch
 *                         failure): its fcgpu_span_wait / fcgpu_span_poll
 *                         returns the error and frees the slot;
 *   FCGPU_FAULT_LAUNCH -- the next shared-queue launch (FCGPU_SPAN_AUTO) fails:
 *                         every batch it carried reports the error through its
 *                         owner's wait or poll;
 *   FCGPU_FAULT_ALLOC  -- a device or pinned allocation made after fcgpu_open
 *                         (scratch made on first use, span and staging blocks,
 *                         flow tables, programs) fails as out of memory: the
 *                         call returns FCGPU_ENOMEM or FCGPU_ERUNTIME and
 *                         leaves no partial state -- a group of buffers is made
 *                         whole or not at all, a flow table or program being
 *                         replaced is absent / the previous one -- so the next
 *                         call retries.
 * Events: submissions for SUBMIT and WAIT (an element's re-submission is
 * one), shared launches for LAUNCH, allocations for ALLOC. count 0 clears
 * the kind. Returns FCGPU_EINVAL for another kind. */
#define FCGPU_FAULT_SUBMIT 0u
#define FCGPU_FAULT_WAIT   1u
#define FCGPU_FAULT_LAUNCH 2u
#define FCGPU_FAULT_ALLOC  3u
int  fcgpu_inject_fault(uint32_t where, uint32_t skip, uint32_t count);

/* Host-only self-test of the launch guard every kernel launch passes (no
 * device needed): a set of malformed launches -- a partition output the
 * kernel stores through left null (tile_count under a tile partition, the
 * per-tile counts under a whole-batch one), null frames, descriptors or
 * counters, more workgroups than tiles, fused batches not end to end or too
 * many -- must all be refused. Returns how many were accepted (0 = all
 * refused), or -1 if a well-formed launch was refused. */
int  fcgpu_launch_guard_selftest(void);

/* 1 if the context's next block submission would be zero-copy (ZEROCOPY, or
 * AUTO with enough contexts), else 0 -- e.g. for an element that stages
 * smaller batches when its batches share the PCIe-read path with others. */
int  fcgpu_span_zerocopy_active(const fcgpu_ctx *ctx);

/* Decision programs. A program is the step list the
 * reference's own compiler produces and prints through the `program` handler
 * (IPFilter/IPClassifier: elements/ip/ipfilter.cc; Classifier:
 * elements/standard/classification.cc:978-991 and :1104-1140): each step loads
 * the 32-bit word at `offset`, masks it, compares with `value` and jumps to
 * `yes`/`no`; a jump > 0 is a step index, <= 0 is output -jump. A step whose
 * word is not entirely inside the packet takes `yes` if FCGPU_STEP_SHORT_YES
 * else `no` (length_checked_match, ipfilter.cc:1415-1474,
 * classification.cc:1146-1176).
 *   FCGPU_PROG_IPFILTER: offsets >= 512 address the transport header,
 *     >= 256 the network header, else the MAC header - 2 (ipfilter.hh:393-481).
 *   FCGPU_PROG_CLASSIFIER: offsets address the frame start
 *     (Classification::Wordwise::Program::match, classification.hh:372-392). */
#define FCGPU_PROG_IPFILTER   0
#define FCGPU_PROG_CLASSIFIER 1
#define FCGPU_STEP_SHORT_YES  1u
#define FCGPU_MAX_STEPS       8192

typedef struct fcgpu_step {
    int32_t  offset;
    uint32_t value;           /* bytes in packet order, read as a little-endian word */
    uint32_t mask;
    int32_t  yes;
    int32_t  no;
    uint32_t flags;           /* FCGPU_STEP_SHORT_YES */
} fcgpu_step;

/* Install a program for FCGPU_CLS_PROGRAM. output_everything >= 0 means the
 * program is empty and every packet goes to that output ("all->[N]"). */
int  fcgpu_set_program(fcgpu_ctx *ctx, uint32_t kind, const fcgpu_step *steps, uint32_t nsteps,
                       int32_t output_everything);
/* Programs compiled to code (enable != 0): the installed program, and every
 * program installed later, is also emitted as straight-line HIP (one block
 * per step with its offset, mask and value as immediates; a jump table as
 * compares over its runs) and compiled with hiprtc into the receive kernels
 * the context launches (~1-5 s per program and configuration, at this call /
 * fcgpu_set_program, or at the first launch of another configuration).
 * Results are identical to the interpreter's. A program with a cycle stays
 * interpreted (FCGPU_EINVAL here; fcgpu_set_program keeps it interpreted
 * silently). enable 0: back to the interpreter. */
int  fcgpu_program_jit(fcgpu_ctx *ctx, int enable);
/* 1 when the installed program runs as compiled code. */
int  fcgpu_program_jit_active(fcgpu_ctx *ctx);

/* The bucket -> output table of FCGPU_CLS_LB_TABLE: nbuckets entries, each
 * < the configured nports (checked here and at every submission). The folded
 * hash is < 65536, so a longer table's entries past 65535 are never read; they
 * are not kept. Synchronises the device before replacing a table. */
#define FCGPU_LB_TABLE_MAX (1u << 24)
int  fcgpu_set_lb_table(fcgpu_ctx *ctx, const uint8_t *table, uint32_t nbuckets);
/* LoadBalancer::build_hash_ring (include/click/loadbalancer.hh:170-189) over
 * the selector [0, nsel) (nsel <= FCGPU_MAX_PORTS): out[size] = the
 * constant_hash_agg ring, the table fcgpu_set_lb_table takes. Host-only (no
 * device, no context). */
int  fcgpu_lb_hash_ring(uint32_t nsel, uint32_t size, uint8_t *out);

/* Flow table: the IPFlow5ID flow classification of
 * FlowIPManagerHMP (elements/research/flowipmanagerhmp.cc:96-126; the
 * VirtualFlowManager family, include/click/flow/virtualflowmanager.hh) placed
 * after the IPv4 check (and the L4 check, if configured) and before the
 * classifier: every packet that passed the checks gets the ID of its
 * (saddr, daddr, sport, dport, proto) flow; a flow seen for the first time gets
 * the next ID (0, 1, 2, ... in packet order, persistent across batches: the
 * `_current.fetch_and_add(1)` of flowipmanagerhmp.cc:99-102 on one thread).
 * Non-first fragments key on ip_p alone: IPFlowID(p) returns before
 * assign() for them (lib/ipflowid.cc:34-38), so their addresses stay 0 and
 * their ports unset (defined as 0 here). IPv4 check modes only.
 *   max_flows: IDs 0 .. max_flows-1 (the table holds 2x that many slots, up to
 *     2^23 flows); a packet of a new flow beyond that gets FCGPU_FLOW_FULL (the
 *     manager kills it, virtualflowmanager.hh:262-266). 0 disables the table.
 * Batches are assigned IDs in the order the context receives them; a
 * fcgpu_process on a caller's stream is ordered after (and before) the
 * context's own span submissions, so mixing the two entry points is safe.
 * Each fcgpu_process with flow enabled adds a pass over the batch's new flows
 * after the receive kernel (one launch, three after a batch with many new
 * flows); fcgpu_process_host processes the batch in order on one stream.
 * The context's max_batch must be at most FCGPU_FLOW_MAX_BATCH. */
#define FCGPU_FLOW_NONE 0xffffffffu
#define FCGPU_FLOW_FULL 0xfffffffeu
#define FCGPU_MAX_FLOWS (1u << 23)
#define FCGPU_FLOW_MAX_BATCH (64u * ((1u << 14) + 64))
int  fcgpu_flow_enable(fcgpu_ctx *ctx, uint32_t max_flows);
/* Forget every flow (IDs restart at 0). */
int  fcgpu_flow_reset(fcgpu_ctx *ctx);
/* HMP: flow IDs assigned so far; IMP: flows in the table (the managers'
 * "count" handler, virtualflowmanager.hh:387-388). Synchronises the context's
 * device work. */
int  fcgpu_flow_count(fcgpu_ctx *ctx, uint32_t *count);

/* Flow managers (the VirtualFlowManager family). One table per
 * context, as the reference keeps one per thread (per_thread_oread<State>,
 * virtualflowmanager.hh:410); fcgpu_flow_enable(ctx, n) is the HMP manager.
 *   FCGPU_FLOW_MGR_HMP: FlowIPManagerHMP, IDs 0, 1, 2, ... (above); no timeout.
 *   FCGPU_FLOW_MGR_IMP: VirtualFlowManagerIMP over FlowManagerIMPState, the
 *     manager of FlowIPManager_CuckooPP / FlowIPManagerIMP
 *     (elements/flow/flowipmanager_cuckoopp.cc:57-121):
 *     - capacity is rounded up to a power of two (virtualflowmanager.hh:85);
 *       IDs come from a free-ID stack filled with 0 .. cap-1 (:113-115), popped
 *       from the top: cap-1, cap-2, ... A popped 0 means "full" (:264-268): a
 *       new flow when only 0 is left gets FCGPU_FLOW_FULL (the element kills
 *       it). (The reference then reads below its stack on the next pop; here
 *       the table stays full until IDs come back.)
 *     - timeout_s > 0 (TIMEOUT) with recycle_ms (RECYCLE_INTERVAL, 1 ..
 *       65535 ms): every flow with a packet in a batch is stamped with the
 *       batch's time (fcgpu_flow_set_time before the batch; :236-239,311-313);
 *       a new flow is scheduled on a timer wheel timeout_s * eps epochs ahead
 *       (eps = max(1, 1000 / recycle_ms); :72-74,293-296). Each
 *       fcgpu_flow_maintain is one maintainer run (:151-223): the IDs the
 *       previous run released go back onto the stack, then the wheel's current
 *       bucket is walked: a flow idle for old ms with old + recycle_ms >=
 *       timeout_s * 1000 is removed from the table and its ID released; others
 *       are rescheduled. The caller runs it every recycle_ms (the reference's
 *       maintain timer, :118-124,134-144), on the same clock.
 *       Memory: next_pow2(TE + 2) * cap * 4 B of wheel (TE = timeout epochs,
 *       at most 16382) and (cap / 1024) * (TE + 1) * 4 B of maintainer counts
 *       (at most 2^26 words); a second slot array the run rebuilds into.
 *   Times are ms on any clock that the caller uses consistently (32-bit,
 *   differences below 2^31 ms). */
#define FCGPU_FLOW_MGR_HMP 0u
#define FCGPU_FLOW_MGR_IMP 1u
typedef struct fcgpu_flow_config {
    uint32_t manager;       /* FCGPU_FLOW_MGR_* */
    uint32_t capacity;      /* HMP: max flows; IMP: CAPACITY (0 disables the table) */
    uint32_t timeout_s;     /* IMP: TIMEOUT in seconds, 0 = flows never expire */
    uint32_t recycle_ms;    /* IMP with timeout: RECYCLE_INTERVAL in ms (reference default 1000) */
} fcgpu_flow_config;
int  fcgpu_flow_configure(fcgpu_ctx *ctx, const fcgpu_flow_config *cfg);
/* The time stamp of the batches submitted after this call
 * (Timestamp::recent_steady() of push_batch, :227-230). */
int  fcgpu_flow_set_time(fcgpu_ctx *ctx, uint32_t now_ms);
/* One maintainer run at time now_ms, queued after the batches submitted
 * before it (on the context's own stream when it has one -- span submissions
 * -- else on `stream`, NULL = the null stream). No-op without timeouts. */
int  fcgpu_flow_maintain(fcgpu_ctx *ctx, uint32_t now_ms, void *stream);
typedef struct fcgpu_flow_stat {
    uint32_t manager, capacity;
    uint32_t count;         /* flows in the table ("count" handler) */
    uint32_t free_ids;      /* IDs the stack can still give ("count_fids", :390-391) */
    uint32_t pending;       /* IDs released by the last run, back on the stack at the next */
    uint32_t epochs;        /* maintainer runs so far (the wheel index) */
} fcgpu_flow_stat;
/* Synchronises the context's device work. */
int  fcgpu_flow_stats(fcgpu_ctx *ctx, fcgpu_flow_stat *st);

/* Host threads the context may use for the gather / copy-out loops of
 * fcgpu_process_host (the caller's thread included; default 1). */
int  fcgpu_set_host_threads(fcgpu_ctx *ctx, uint32_t nthreads);
/* Pinned host memory for fcgpu_process_host outputs (NULL on failure). */
void *fcgpu_host_alloc(size_t bytes);
void fcgpu_host_free(void *p);
/* Page-lock existing host memory for DMA (hipHostRegister; read-only mappings
 * such as an mmapped pcap are registered read-only). */
int  fcgpu_host_register(void *p, size_t bytes, int read_only);
int  fcgpu_host_unregister(void *p);

/* mbuf ingress: the batch FromDPDKDevice::_run_task gets
 * from rte_eth_rx_burst (elements/userlevel/fromdpdkdevice.cc:374-456) goes to
 * the GPU as the array of mbuf pointers itself -- no Packet objects, no host
 * copy of the frames. The packet-buffer pool (a DPDK mempool's memory: mbuf
 * headers and data rooms, < 4 GiB) is registered once per context (contexts
 * of other threads registering the same pool share one pinning, released
 * with the last of them); each call copies the
 * n pointers H2D, a kernel reads every mbuf's buf_addr / data_off / data_len
 * straight from host memory and builds the batch's descriptors, and k_rx
 * reads the frames' header windows from the pool over PCIe (zero copy).
 * Outputs go to device memory (d_out), as fcgpu_process. A pointer (or a
 * frame) outside the registered pool is never dereferenced: that packet is
 * processed as an empty frame (FCGPU_R_MINISCULE / not checked). Field
 * offsets are the caller's mbuf layout; FCGPU_MBUF_LAYOUT_DPDK is rte_mbuf's
 * (DPDK >= 20.11: buf_addr @0, data_off @16, data_len @40). Asynchronous on
 * `stream`; mbufs[] may be reused when the call returns. */
typedef struct fcgpu_mbuf_layout {
    uint32_t buf_addr;        /* offset of the void *buf_addr field          */
    uint32_t data_off;        /* offset of the uint16_t data_off field       */
    uint32_t data_len;        /* offset of the uint16_t data_len field       */
    uint32_t header_bytes;    /* bytes of the mbuf header read (>= every field end, <= 64) */
} fcgpu_mbuf_layout;
#define FCGPU_MBUF_LAYOUT_DPDK {0u, 16u, 40u, 64u}
int  fcgpu_pool_register(fcgpu_ctx *ctx, void *base, size_t bytes);
int  fcgpu_process_mbufs(fcgpu_ctx *ctx, void *const *mbufs, uint32_t n, const fcgpu_mbuf_layout *layout,
                         const fcgpu_out *d_out, void *stream);

int  fcgpu_read_counters(fcgpu_ctx *ctx, uint64_t *out, int n);
/* The device keeps the per-reason and per-output bins only; "count" and
 * "drops" are derived: drops = the reason slots of reasons 0-5, 7, 8 (the
 * checker's drops), count = all packets (sum of the output bins, invalid list
 * included) - drops. fcgpu_read_counters applies this; callers summing the
 * raw device replicas themselves (e.g. after an all-reduce) call this on the
 * summed FCGPU_NCOUNTERS vector. */
void fcgpu_counters_derive(uint64_t *vec);
int  fcgpu_reset_counters(fcgpu_ctx *ctx);
/* Device address of the context's uint64 counter replicas
 * (FCGPU_CTR_SHARDS x FCGPU_NCOUNTERS), for a cross-GPU all-reduce. */
int  fcgpu_counters_device(fcgpu_ctx *ctx, uint64_t **d_counters);
/* Make the context accumulate into caller-owned device memory
 * (FCGPU_CTR_SHARDS x FCGPU_NCOUNTERS uint64, initialised by the caller), e.g. a
 * tensor that is all-reduced over RCCL. NULL reverts to the context's own. */
int  fcgpu_use_counters(fcgpu_ctx *ctx, uint64_t *d_counters);

/* Per-kernel timing with HIP events on the launch stream (off by default).
 * fcgpu_set_timing(ctx, k): k > 0 brackets the k-th, 2k-th, ... launch of the
 * context after this call (1 = every launch) with start/stop events: the
 * event pair of hipExtLaunchKernelGGL for a one-batch launch, two stream
 * markers (hipEventRecord) around a fused launch of several batches (cheaper
 * on an idle queue; the interval adds the launch's dispatch latency). A fused
 * launch counts as its number of batches. The events are created by this
 * call, not on the launch path. 0 = off. (Each recorded event idles the queue for a few us,
 * so sparse sampling keeps the measured region representative.)
 * fcgpu_read_timing returns, per stage (0 = fused check/hash/classify,
 * 1 = count scan, 2 = partition scatter), the summed milliseconds and launches
 * since the last read, and resets them. Synchronises the context stream. */
int  fcgpu_set_timing(fcgpu_ctx *ctx, int every);
int  fcgpu_read_timing(fcgpu_ctx *ctx, double *ms, uint32_t *launches, int nstages);

/* Flow re-shard across GPUs (SURVEY 8(f) #1 over 8(e)). FastClick keeps one
 * flow table per core and relies on the NIC's RSS hash to send every packet
 * of a flow to one core (VirtualFlowManagerIMP::process,
 * include/click/flow/virtualflowmanager.hh:249-330; FlowIPManagerHMP,
 * elements/flow/flowipmanagerhmp.cc:101-117). When packets reach the GPUs
 * unsharded, each rank's device pass (fcgpu_process with FCGPU_CLS_LB_HASH
 * over nports = world outputs and FCGPU_PART_GLOBAL: perm + port_start) names
 * every packet's owner rank, and these calls build and read the buffers of
 * one all-to-all (RCCL over xGMI) that moves each packet to its owner:
 *
 *   fcgpu_exchange_plan   perm[0 .. port_start[world]) -- the packets that
 *       leave (output `world`, the invalid list, stays) -- gets one
 *       fcgpu_xmeta record each, in perm order; d_seg_bytes[d] = the bytes of
 *       owner d's segment of the send buffer. Each frame takes a 16-B aligned
 *       slot of (length + 15) & ~15 bytes (ABI 22; 4-B slots before), so every
 *       slot is written in whole aligned 16-B stores. Segments follow in owner
 *       order.
 *   fcgpu_exchange_pack   the frames into d_send (at least the sum of
 *       d_seg_bytes; nothing is written past send_cap; an owner whose
 *       d_seg_bytes exceeds 0xffffffff -- its records' 32-bit offsets cannot
 *       address it -- is not packed, so check the plan's sizes first): owner d's segment
 *       holds its packets in input order; slot bytes past a frame's length
 *       are zero. It reads the frames' arena offsets the plan left in the
 *       context: call it after fcgpu_exchange_plan of the same batch on the
 *       same context and stream, before the next plan.
 *   (the caller's all-to-all: records and segments; a receiver concatenates
 *    the segments it gets in source-rank order)
 *   fcgpu_exchange_unpack the received records -> descriptors into the
 *       received buffer: desc[2j] = src_displ[record.src_rank] + record.off,
 *       desc[2j+1] = record.length, where src_displ[r] is where source r's
 *       segment starts in that buffer (host array of `world` values). The
 *       offsets must fit in 32 bits; the receiver keeps the ABI's over-read
 *       slack (128 B past every frame start, 16 B past every frame end)
 *       readable after its buffer.
 * The frames keep their bytes and lengths exactly; the records carry each
 * packet's source (rank, index), so the receiver's order is (source rank,
 * source index). world <= FCGPU_MAX_PORTS; n <= the context's max_batch for
 * the plan. Asynchronous on `stream` (plan needs the context's scratch: one
 * plan at a time per context). */
typedef struct fcgpu_xmeta {
    uint32_t off;             /* the frame's slot within its owner's segment             */
    uint32_t length;          /* frame length                                            */
    uint32_t src_index;       /* index in the source rank's batch                        */
    uint32_t src_rank;        /* source rank (bytes 8..15 = src_rank << 32 | src_index)  */
} fcgpu_xmeta;
int  fcgpu_exchange_plan(fcgpu_ctx *ctx, const uint32_t *d_desc, const uint32_t *d_perm,
                         const uint32_t *d_port_start, uint32_t n, uint32_t world, uint32_t rank,
                         fcgpu_xmeta *d_meta, uint64_t *d_seg_bytes, void *stream);
int  fcgpu_exchange_pack(fcgpu_ctx *ctx, const uint8_t *d_arena, const uint32_t *d_port_start,
                         const fcgpu_xmeta *d_meta, const uint64_t *d_seg_bytes, uint32_t n, uint32_t world,
                         uint8_t *d_send, uint64_t send_cap, void *stream);
int  fcgpu_exchange_unpack(fcgpu_ctx *ctx, const fcgpu_xmeta *d_meta, uint32_t n, const uint64_t *src_displ,
                           uint32_t world, uint32_t *d_desc, void *stream);

/* The send side in one call, from the owner pass's verdicts instead of its
 * whole-batch partition: packet i leaves to owner d = d_verdict[i] >> 8 when
 * d < world (a k_rx pass with LB_MODE hash over `world` outputs; the invalid
 * list, port `world`, stays). Writes exactly what fcgpu_exchange_plan +
 * fcgpu_exchange_pack write for the stable partition of those owners (records
 * in owner order, input order within an owner; owner d's segment; slot
 * padding zero), plus d_seg_n[d], the packets of owner d. send_cap bounds the
 * send buffer as for fcgpu_exchange_pack (the sum of the leaving frames'
 * slots fits in send_cap whenever it is at least the arena's frame bytes +
 * 15 per packet), so no host sync is needed before the call. Every per-packet
 * load is in input order (three launches: per-tile owner counts and bytes,
 * their scan per owner, the records and frames per tile). The per-tile
 * counts are one scratch per context: builds on one context must be
 * serialised on one stream (as plan -> pack are). */
int  fcgpu_exchange_build(fcgpu_ctx *ctx, const uint8_t *d_arena, const uint32_t *d_desc,
                          const uint16_t *d_verdict, uint32_t n, uint32_t world, uint32_t rank,
                          fcgpu_xmeta *d_meta, uint32_t *d_seg_n, uint64_t *d_seg_bytes, uint8_t *d_send,
                          uint64_t send_cap, void *stream);

/* The fixed-capacity exchange: no host sync anywhere in a re-shard step.
 * Owner d's segment has room for seg_recs packets and seg_bytes frame bytes
 * (16-B slots): d_meta holds world x (seg_recs + 1) records -- segment d at
 * d (seg_recs + 1): a header (fcgpu_xseg) then its records, as
 * fcgpu_exchange_build writes them -- and d_send world x seg_bytes bytes,
 * segment d at d x seg_bytes (record offsets relative to it). Both go through
 * all-to-alls with equal splits (the split sizes never leave the device). An
 * owner whose packets do not fit gets its header alone, flags bit 0 set:
 * the receivers then process nothing for that step and the caller falls
 * back to the counted exchange (fcgpu_exchange_build) for it
 * (fastclick_amd.dist). world x seg_bytes must stay below 4 GiB. */
typedef struct fcgpu_xseg {
    uint32_t packets;         /* the owner's packets this step                          */
    uint32_t bytes_lo;        /* their slot bytes                                         */
    uint32_t bytes_hi;
    uint32_t flags;           /* bit 0: overflow -- more than the capacity, none sent     */
} fcgpu_xseg;
int  fcgpu_exchange_build_fixed(fcgpu_ctx *ctx, const uint8_t *d_arena, const uint32_t *d_desc,
                                const uint16_t *d_verdict, uint32_t n, uint32_t world, uint32_t rank,
                                uint32_t seg_recs, uint64_t seg_bytes, fcgpu_xmeta *d_meta, uint8_t *d_send,
                                void *stream);
/* The receive side after the equal-split all-to-alls: d_rmeta / the received
 * frames in the layout above, source s's segment at s. Writes the received
 * packets' descriptors (in source-rank order, then source order, as
 * fcgpu_exchange_unpack) into d_desc (room for world x seg_recs) and their
 * number into *d_count. If any segment overflowed, or *d_stall is already
 * non-zero (an earlier step stalled and is not repaired yet), *d_count = 0
 * and *d_stall = step when it was 0: the flow pass of this step and of every
 * later one processes nothing until the caller has replayed them, in order,
 * through the counted exchange and cleared *d_stall. step must be non-zero.
 * d_total (may be NULL): *d_total += the count, a running total of the
 * packets received that needs no host read per step. */
int  fcgpu_exchange_unpack_fixed(fcgpu_ctx *ctx, const fcgpu_xmeta *d_rmeta, uint32_t world, uint32_t seg_recs,
                                 uint64_t seg_bytes, uint32_t *d_desc, uint32_t *d_count, uint32_t *d_stall,
                                 uint64_t *d_total, uint32_t step, void *stream);

const char *fcgpu_last_error(fcgpu_ctx *ctx);   /* ctx may be NULL (open errors) */

#ifdef __cplusplus
}
#endif
#endif /* FASTCLICK_GPU_H */
