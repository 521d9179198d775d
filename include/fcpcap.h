/*
 * fcpcap.h -- pcap ingress for the MI355X receive path (libfcclick.so).
 *
 * The userlevel counterpart of FromDump (elements/userlevel/fromdump.cc)
 * without Packet objects: records are read straight from the file into a
 * caller-owned (pinned, fcgpu_host_alloc) buffer, record headers and all, and
 * described by (offset, captured length) pairs -- the arena + descriptor
 * batch libfcgpu consumes. A chunk goes to the device as one H2D copy
 * (fcgpu_span_submit), with no per-packet gather.
 *
 * Record semantics follow FromDump::read_packet (fromdump.cc:418-500) and its
 * file-header check (fromdump.cc:278-316): magic 0xA1B2C3D4 / 0xA1B23C4D
 * (nanosecond) / 0xA1B2CD34 (modified pcap: 8 extra header bytes) in either
 * byte order; major version 2; caplen and len swapped for minor versions < 3
 * (and = 3 when caplen > len); caplen > 65535 is a bad file; caplen > len is
 * cut to len (the rest skipped).
 */
#ifndef FCPCAP_H
#define FCPCAP_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct fcpcap fcpcap;

/* Open a pcap file. Returns 0, or -1 with the message in err. */
int  fcpcap_open(const char *path, fcpcap **out, char *err, size_t errcap);
/* The file header's link type (1 = Ethernet, 101/12/14 = raw IP) and snaplen. */
int  fcpcap_linktype(const fcpcap *r);
uint32_t fcpcap_snaplen(const fcpcap *r);
/* Fill buf (cap bytes) with whole records, up to max packets: desc[2i] is the
 * offset of packet i's data in buf, desc[2i+1] its captured length; wire[i]
 * (may be NULL) its original length, ts_ns[i] (may be NULL) its timestamp in
 * nanoseconds. A record that does not fit is kept for the next call. Returns
 * the packet count (0 at the end of the file), or -1 on a bad record (message
 * via fcpcap_error). *used = bytes of buf written. */
int  fcpcap_read(fcpcap *r, uint8_t *buf, size_t cap, uint32_t *desc, uint32_t *wire, uint64_t *ts_ns,
                 uint32_t max, size_t *used);
/* Zero-copy mode: map the whole file read-only (page cache pages; register
 * them with fcgpu_host_register so the H2D copies DMA straight from them). */
int  fcpcap_map(fcpcap *r, const uint8_t **base, size_t *bytes);
/* Index the next records of the mapped file (up to max packets / max_bytes):
 * the chunk is [base + *chunk_off, + *chunk_bytes); desc offsets are relative
 * to its start. Returns the count (0 at the end), -1 on a bad record header
 * (the records before it came with this call or the previous one). With
 * fcpcap_set_threads(T > 1) a chunk of >= 8 MiB is walked in up to T pieces
 * in parallel and stitched; the records are exactly the one-thread walk's.
 * Do not mix with fcpcap_read on one reader. */
int  fcpcap_index(fcpcap *r, uint32_t max, size_t max_bytes, size_t *chunk_off, size_t *chunk_bytes,
                  uint32_t *desc, uint32_t *wire, uint64_t *ts_ns);
const char *fcpcap_error(const fcpcap *r);
/* Threads fcpcap_read may use to copy file data into the buffer (parallel
 * pread() of >= 1 MiB pieces; default 1). */
int  fcpcap_set_threads(fcpcap *r, unsigned threads);
void fcpcap_close(fcpcap *r);

#ifdef __cplusplus
}
#endif
#endif
