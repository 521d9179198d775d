/*
 * fc_oracle.c -- TEST INFRASTRUCTURE ONLY (see fc_oracle.h).
 *
 * Plain-C restatement of the reference's receive-path semantics. Every function
 * names the reference lines it restates. This is the checker for the HIP path,
 * never a fallback for it.
 */
#include "fc_oracle.h"
#include <stdlib.h>
#include <string.h>

static inline uint32_t le32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
static inline uint16_t be16(const uint8_t *p) { return (uint16_t)((p[0] << 8) | p[1]); }
static inline uint16_t raw16(const uint8_t *p) { uint16_t v; memcpy(&v, p, 2); return v; }
static inline uint32_t rotl32(uint32_t v, unsigned r) {
    r &= 31;
    return r ? (v << r) | (v >> (32 - r)) : v;
}

/* lib/in_cksum.c:20-51: 32-bit accumulator over host-order 16-bit words, odd
 * trailing byte in the low byte, two folds, one's complement. */
uint16_t fco_in_cksum(const uint8_t *addr, int len)
{
    int nleft = len;
    uint32_t sum = 0;
    const uint8_t *w = addr;
    while (nleft > 1) {
        uint16_t x;
        memcpy(&x, w, 2);
        sum += x;
        w += 2;
        nleft -= 2;
    }
    if (nleft == 1)
        sum += (uint16_t)w[0];           /* *(uchar*)&answer = *w, little endian */
    sum = (sum & 0xffff) + (sum >> 16);
    sum += (sum >> 16);
    return (uint16_t)~sum;
}

/* click_in_cksum_pseudohdr_raw / _hard (lib/in_cksum.c:53-111) and the
 * dispatch of click_in_cksum_pseudohdr (include/clicknet/ip.h:156-163): with
 * IP options, the final destination of an SSRR/LSRR option replaces ip_dst. */
static uint16_t pseudohdr_raw(uint32_t csum, uint32_t src, uint32_t dst, int proto, int packet_len)
{
    csum = ~csum & 0xFFFF;
    csum += (src & 0xffff) + (src >> 16);
    csum += (dst & 0xffff) + (dst >> 16);
    csum += (uint32_t)(uint16_t)(((packet_len & 0xff) << 8) | ((packet_len >> 8) & 0xff)) + ((uint32_t)proto << 8);
    csum = (csum & 0xffff) + (csum >> 16);
    return (uint16_t)(~(csum + (csum >> 16)) & 0xFFFF);
}

uint16_t fco_in_cksum_pseudohdr(uint16_t data_csum, const uint8_t *iph, int packet_len)
{
    uint32_t src, dst;
    memcpy(&src, iph + 12, 4);
    memcpy(&dst, iph + 16, 4);
    const int hl = (iph[0] & 15) << 2;
    if (hl != 20) {
        const uint8_t *opt = iph + 20, *end = iph + hl;
        while (opt < end) {
            if (*opt == 1) { opt++; continue; }             /* IPOPT_NOP */
            if (*opt == 0) break;                           /* IPOPT_EOL */
            if (opt + 1 >= end || opt[1] < 2 || opt + opt[1] > end) break;
            if ((*opt == 137 || *opt == 131) && opt[1] >= 7) { /* IPOPT_SSRR, IPOPT_LSRR */
                memcpy(&dst, opt + opt[1] - 4, 4);
                break;
            }
            opt += opt[1];
        }
    }
    return pseudohdr_raw(data_csum, src, dst, iph[9], packet_len);
}

/* include/click/ipflowid.hh:153-164 with IPAddress::hashcode = raw s_addr
 * (include/click/ipaddress.hh:346-350); hashcode_t is 64-bit, consumers keep
 * the low 32 bits (elements/analysis/aggregatehash.cc:51). */
uint32_t fco_ipflowid_hash(uint32_t sx, uint16_t sport_net, uint32_t dx, uint16_t dport_net)
{
    uint32_t s = (uint16_t)((sport_net >> 8) | (sport_net << 8));
    uint32_t d = (uint16_t)((dport_net >> 8) | (dport_net << 8));
    return rotl32(sx, (s % 16) + 1) ^ rotl32(dx, 31 - (d % 16)) ^ ((d << 16) | s);
}

/* include/click/ip6address.hh:348-352: (data32[2] << 1) + data32[3]. */
static uint32_t ip6_addr_hash(const uint8_t a[16])
{
    return (le32(a + 8) << 1) + le32(a + 12);
}

/* include/click/ip6flowid.hh:220-230. ROT(v, 0) shifts a 32-bit value by 32
 * (UB); x86 masks the count and yields v, restated here as rotl32(v, 0) = v. */
uint32_t fco_ip6flowid_hash(const uint8_t src[16], uint16_t sport_net,
                            const uint8_t dst[16], uint16_t dport_net)
{
    uint32_t s = (uint16_t)((sport_net >> 8) | (sport_net << 8));
    uint32_t d = (uint16_t)((dport_net >> 8) | (dport_net << 8));
    return rotl32(ip6_addr_hash(src), s % 16) ^ rotl32(ip6_addr_hash(dst), 31 - d % 16)
        ^ ((d << 16) | s);
}

/* include/click/loadbalancer.hh:580-584 (direct_hash; direct_hash_agg at
 * :570-574 is the same on AGGREGATE_ANNO), identity selector. */
int fco_lb_hash_port(uint32_t h, int n)
{
    return (int)(((h >> 16) ^ (h & 65535)) % (uint32_t)n);
}

/* rte_hash_crc_4byte (DPDK rte_hash_crc.h, crc32c_sse42_u32 = _mm_crc32_u32(init,
 * data); crc32c_1word in software): CRC32-C, reflected polynomial 0x82F63B78, no
 * pre/post inversion. */
uint32_t fco_crc32c_u32(uint32_t data, uint32_t crc)
{
    crc ^= data;
    for (int k = 0; k < 32; k++)
        crc = (crc >> 1) ^ (0x82F63B78u & (0u - (crc & 1u)));
    return crc;
}

/* ipv4_hash_crc(&IPFlow5ID, sizeof, 0) (include/click/dpdk_glue.hh:13-27): proto,
 * saddr, daddr, then the ports word (the struct's third u32), folded as
 * direct_hash_crc does (include/click/loadbalancer.hh:563-569). */
int fco_lb_crc_port(uint32_t proto, uint32_t saddr, uint32_t daddr, uint32_t ports, int n)
{
    uint32_t c = fco_crc32c_u32(proto, 0);
    c = fco_crc32c_u32(saddr, c);
    c = fco_crc32c_u32(daddr, c);
    c = fco_crc32c_u32(ports, c);
    return (int)(((c >> 16) ^ (c & 65535)) % (uint32_t)n);
}

/* include/click/loadbalancer.hh:227-243 (hash_ip). */
int fco_hash_ip_port(const uint8_t *data, uint32_t len, int n)
{
    int o = 26, l = 8;
    if ((int)len < o + l)
        return 0;
    int d = 0;
    for (int i = o; i < o + l; i++)
        d += data[i];
    if (n == 2 || n == 4 || n == 8)
        return (d ^ (d >> 4)) & (n - 1);
    return d % n;
}

/* elements/standard/hashswitch.cc:50-66. */
int fco_hashswitch_port(const uint8_t *data, uint32_t len, int o, int l, int n)
{
    if ((int)len < o + l)
        return 0;
    int d = 0;
    for (int i = o; i < o + l; i++)
        d += data[i];
    if (n == 2 || n == 4 || n == 8)
        return (d ^ (d >> 4)) & (n - 1);
    return d % n;
}

/* LoadBalancer::build_hash_ring (include/click/loadbalancer.hh:170-189) over
 * the selector [0, nsel) (:519-524), with cantor (include/click/algorithm.hh:
 * 136-138): every server is placed at cantor(s, j) % size for j < fac, later
 * placements overwriting earlier ones; the empty buckets then take the last
 * server placed before them (selector[0] before the first). size = the
 * CST_BUCKETS keyword, or 100 per destination (:526-530). */
void fco_lb_hash_ring(uint32_t nsel, uint32_t size, uint32_t *ring)
{
    for (uint32_t i = 0; i < size; i++)
        ring[i] = 0xffffffffu;                 /* resize(size, -1) */
    const int fac = (int)((size - 1) / nsel) + 1;
    for (int j = 0; j < fac; j++)
        for (uint32_t i = 0; i < nsel; i++) {
            const unsigned a = i, b = (unsigned)j;
            const unsigned cantor = ((a + b) * (a + b + 1)) / 2 + b;
            ring[cantor % size] = i;
        }
    uint32_t cur = 0;
    for (uint32_t i = 0; i < size; i++) {
        if (ring[i] == 0xffffffffu)
            ring[i] = cur;
        else
            cur = ring[i];
    }
}

/* constant_hash_agg (include/click/loadbalancer.hh:585-589): the ring's entry
 * at ((h >> 16) ^ (h & 65535)) % _cst_hash.size(); fco_set_lb_table installs
 * the ring (global, as the program). */
static uint8_t *g_lbtab;
static uint32_t g_lbtab_n;
void fco_set_lb_table(const uint8_t *t, uint32_t n)
{
    free(g_lbtab);
    g_lbtab = (uint8_t *)malloc(n ? n : 1);
    if (n) memcpy(g_lbtab, t, n);
    g_lbtab_n = n;
}
int fco_lb_table_port(uint32_t h)
{
    if (!g_lbtab_n) return 0;
    return g_lbtab[((h >> 16) ^ (h & 65535)) % g_lbtab_n];
}

/* include/click/packetbatch.hh:259-307: stable partition into nbatches lists,
 * out-of-range outputs to the last list. */
void fco_classify_each_packet(int nbatches, const int *port, uint32_t n,
                              uint32_t *perm, uint32_t *start)
{
    uint32_t cnt[FCGPU_MAX_PORTS + 2];
    memset(cnt, 0, sizeof(cnt));
    for (uint32_t i = 0; i < n; i++) {
        int o = port[i];
        if (o < 0 || o >= nbatches) o = nbatches - 1;
        cnt[o]++;
    }
    uint32_t acc = 0;
    for (int b = 0; b < nbatches; b++) { start[b] = acc; acc += cnt[b]; }
    start[nbatches] = acc;
    if (!perm) return;
    uint32_t pos[FCGPU_MAX_PORTS + 2];
    memcpy(pos, start, sizeof(uint32_t) * (nbatches + 1));
    for (uint32_t i = 0; i < n; i++) {
        int o = port[i];
        if (o < 0 || o >= nbatches) o = nbatches - 1;
        perm[pos[o]++] = i;
    }
}

void fco_partition_tiles(int nbatches, const int *port, uint32_t n, uint32_t tile,
                         uint32_t *perm, uint16_t *tile_count)
{
    uint32_t start[FCGPU_MAX_PORTS + 2];
    for (uint32_t t0 = 0, t = 0; t0 < n; t0 += tile, ++t) {
        uint32_t m = n - t0 < tile ? n - t0 : tile;
        fco_classify_each_packet(nbatches, port + t0, m, perm + t0, start);
        for (uint32_t j = 0; j < m; ++j) perm[t0 + j] += t0;
        for (int b = 0; b < nbatches; ++b) tile_count[(size_t)t * nbatches + b] = (uint16_t)(start[b + 1] - start[b]);
    }
}

static int in_list(const uint32_t *l, uint32_t nl, uint32_t v)
{
    for (uint32_t i = 0; i < nl; i++)
        if (l[i] == v) return 1;
    return 0;
}

/* elements/ip/checkipheader.cc:163-226 (CheckIPHeader::valid) with
 * Packet::take (include/click/packet.hh:2189-2207), set_ip_header
 * (packet.hh:2493-2496) and set_dst_ip_anno. ip offset `o` from frame start. */
static int check_ip4(const fcgpu_cfg *c, const uint8_t *f, uint32_t len, uint32_t o,
                     fcgpu_anno *a)
{
    unsigned plen = len - o;
    if ((int)plen < 20)
        return FCGPU_R_MINISCULE;
    const uint8_t *ip = f + o;
    a->ipver = 4;
    if ((ip[0] >> 4) != 4)
        return FCGPU_R_BAD_VERSION;
    unsigned hlen = (unsigned)(ip[0] & 15) << 2;
    if (hlen < 20)
        return FCGPU_R_BAD_HLEN;
    unsigned L = be16(ip + 2);
    if (L > plen || L < hlen)
        return FCGPU_R_BAD_IP_LEN;
    if (c->checksum && fco_in_cksum(ip, (int)hlen) != 0)
        return FCGPU_R_BAD_CKSUM;
    uint32_t src = le32(ip + 12), dst = le32(ip + 16);
    if (in_list(c->badsrc, c->nbadsrc, src) && !in_list(c->gooddst, c->ngooddst, dst))
        return FCGPU_R_BAD_SADDR;
    a->nh = (uint16_t)o;
    a->th = (uint16_t)(o + hlen);
    a->length = (uint16_t)(plen > L ? len - (plen - L) : len);
    a->dst_ip = dst;
    return FCGPU_R_OK;
}

/* elements/ip6/checkip6header.cc:105-168; PROCESS_EH walks the extension
 * headers like ip6_follow_eh (include/click/ip6address.hh:417-448) up to the
 * untrimmed packet end: the last header visited gives IP6_NXT and the
 * transport header. */
static int check_ip6(const fcgpu_cfg *c, const uint8_t *f, uint32_t len, uint32_t o,
                     fcgpu_anno *a)
{
    unsigned plen = len - o;
    a->ipver = 6;
    if ((int)plen < 40)
        return FCGPU_R_BAD_IP6;
    const uint8_t *ip = f + o;
    if ((ip[0] >> 4) != 6)
        return FCGPU_R_BAD_IP6;
    unsigned pl6 = be16(ip + 4);
    if (pl6 > plen - 40)
        return FCGPU_R_BAD_IP6;
    for (uint32_t i = 0; i < c->nbad6; i++)
        if (memcmp(ip + 8, c->bad6[i], 16) == 0)
            return FCGPU_R_BAD_IP6;
    unsigned nxt = ip[6], tot = 40;
    if (c->process_eh) {
        unsigned eh = 40, t = nxt;
        while (eh < plen) {
            nxt = t;
            tot = eh;
            const unsigned en = ip[eh], el = ip[eh + 1];   /* eh->nxt, eh->len */
            if (t == 0 || t == 43)
                eh += el * 8 + 8;                  /* IP6_EH_HOPBYHOP, IP6_EH_ROUTING */
            else if (t == 51)
                eh += ((el + 2) * 4 + 7) / 8 * 8;  /* IP6_EH_AH: round_up((len+2)*4, 8) */
            else if (t == 44)
                eh += 8;                           /* IP6_EH_FRAGMENT */
            else
                break;
            t = en;
        }
    }
    a->nh = (uint16_t)o;
    a->th = (uint16_t)(o + tot);
    a->ip6_nxt = (uint8_t)nxt;
    a->length = (uint16_t)(pl6 < plen - tot ? len - (plen - tot - pl6) : len);
    return FCGPU_R_OK;
}

/* ---- decision programs (A11) ------------------------------------------- */
static struct {
    uint32_t kind, n;
    int32_t all;
    fcgpu_step *steps;
} g_prog = {0, 0, -1, NULL};

void fco_set_program(uint32_t kind, const fcgpu_step *steps, uint32_t nsteps, int32_t all)
{
    free(g_prog.steps);
    g_prog.steps = NULL;
    g_prog.kind = kind;
    g_prog.n = nsteps;
    g_prog.all = nsteps ? -1 : all;
    if (nsteps) {
        g_prog.steps = (fcgpu_step *)malloc(sizeof(fcgpu_step) * nsteps);
        memcpy(g_prog.steps, steps, sizeof(fcgpu_step) * nsteps);
    }
}

/* word at frame byte b; bytes before the frame start (MAC header - 2) are 0 */
static uint32_t prog_word(const uint8_t *f, int b)
{
    uint8_t w[4];
    for (int k = 0; k < 4; k++) w[k] = (b + k >= 0) ? f[b + k] : 0;
    return le32(w);
}

/* elements/ip/ipfilter.hh:393-481 + ipfilter.cc:1415-1474 (IPFilter), and
 * classification.hh:372-392 + classification.cc:1146-1176 (Classifier). The
 * reference skips length checks when the packet is at least the safe length,
 * where they always pass; here every step is checked. */
uint32_t fco_run_program(const uint8_t *f, const fcgpu_anno *a)
{
    if (g_prog.all >= 0) return (uint32_t)g_prog.all;
    int ipf = g_prog.kind == FCGPU_PROG_IPFILTER;
    int plen;
    if (ipf) {
        int nl = (int)a->length - (int)a->nh, nhl = (int)a->th - (int)a->nh;
        plen = nl > nhl ? nl + 512 - nhl : nl + 256;   /* ipfilter.hh:396-400 */
    } else {
        plen = (int)a->length;
    }
    int pos = 0;
    for (uint32_t it = 0; it <= g_prog.n; it++) {
        const fcgpu_step *st = &g_prog.steps[pos];
        int off = st->offset;
        int j;
        int ok = off + 4 <= plen;
        if (!ok && off < plen) {
            unsigned avail = (unsigned)(plen - off);
            const uint8_t *c = (const uint8_t *)&st->mask;
            ok = !(c[3] || (c[2] && avail <= 2) || (c[1] && avail == 1));
        }
        if (ok) {
            int b = !ipf ? off : off >= 512 ? (int)a->th + off - 512 : off >= 256 ? (int)a->nh + off - 256 : off - 2;
            uint32_t data = prog_word(f, b) & st->mask;
            j = data == (st->value & st->mask) ? st->yes : st->no;
        } else {
            j = (st->flags & FCGPU_STEP_SHORT_YES) ? st->yes : st->no;
        }
        if (j <= 0) return (j <= -32767) ? 0x7fff : (uint32_t)(-j);
        pos = j;
    }
    return 0x7fff;
}

/* CheckUDPHeader::simple_action (elements/tcpudp/checkudpheader.cc:96-121) /
 * CheckTCPHeader::simple_action (elements/tcpudp/checktcpheader.cc:96-123)
 * behind the IPv4 check. */
static int check_l4(const fcgpu_cfg *c, const uint8_t *f, const fcgpu_anno *a)
{
    const uint8_t *ip = f + a->nh, *th = f + a->th;
    const unsigned hl = (unsigned)(ip[0] & 15) << 2, proto = ip[9];
    unsigned len;
    int want;
    if (c->l4_mode == FCGPU_L4_UDP) {
        if (proto != 17)
            return FCGPU_R_L4_PROTO;
        len = be16(th + 4);
        if (len < 8 || a->length < len + hl + a->nh)
            return FCGPU_R_L4_LENGTH;
        want = c->l4_checksum && raw16(th + 6) != 0;
    } else {
        if (proto != 6)
            return FCGPU_R_L4_PROTO;
        len = be16(ip + 2) - hl;
        const unsigned toff = (unsigned)(th[12] >> 4) << 2;
        if (toff < 20 || len < toff || a->length < len + hl + a->nh)
            return FCGPU_R_L4_LENGTH;
        want = c->l4_checksum != 0;
    }
    if (want && fco_in_cksum_pseudohdr(fco_in_cksum(th, (int)len), ip, (int)len) != 0)
        return FCGPU_R_L4_CKSUM;
    return FCGPU_R_OK;
}

/* Header rewrites after the classifier, on a copy of IP header bytes 8..11.
 * DecIPTTL::simple_action (elements/ip/decipttl.cc:52-78) and
 * SetIPChecksum::simple_action (elements/ip/setipchecksum.cc:38-58). */
static void rewrite_ip4(const fcgpu_cfg *c, const uint8_t *f, fco_result *r)
{
    fcgpu_anno *a = &r->anno;
    const uint8_t *ip = f + a->nh;
    uint8_t b[4] = {ip[8], ip[9], ip[10], ip[11]};
    int changed = 0;
    if (c->rewrite & FCGPU_RW_DECTTL) {
        int mcast = (ip[16] & 0xf0) == 0xe0;          /* IPAddress::is_multicast */
        if (c->ttl_multicast || !mcast) {
            if (b[0] <= 1) {
                r->reason = FCGPU_R_TTL_EXPIRED;
                r->port = (uint8_t)c->nports;
                return;
            }
            b[0]--;
            unsigned long sum = (~(unsigned long)((b[2] << 8) | b[3]) & 0xFFFF) + 0xFEFF;
            uint16_t v = (uint16_t)(sum + (sum >> 16));   /* htons() takes a uint16_t */
            uint16_t ns = (uint16_t)~v;
            b[2] = (uint8_t)(ns >> 8);
            b[3] = (uint8_t)ns;
            changed = 1;
        }
    }
    if (c->rewrite & FCGPU_RW_SETCKSUM) {
        uint32_t plen = (uint32_t)a->length - a->nh, hl = (uint32_t)(ip[0] & 15) << 2;
        if (plen < 20 || hl < 20 || hl > plen) {
            r->reason = FCGPU_R_SETCKSUM_BAD;
            r->port = (uint8_t)c->nports;
            return;
        }
        uint8_t hdr[60];
        memcpy(hdr, ip, hl);
        memcpy(hdr + 8, b, 4);
        hdr[10] = hdr[11] = 0;
        uint16_t ck = fco_in_cksum(hdr, (int)hl);     /* stored as a host-order u16 */
        memcpy(b + 2, &ck, 2);
        changed = 1;
    }
    /* the bytes as the packet leaves, changed or not (fastclick_gpu.h ip_rw) */
    (void)changed;
    r->ip_rw = (uint32_t)b[0] | (uint32_t)b[1] << 8 | (uint32_t)b[2] << 16 | (uint32_t)b[3] << 24;
}

void fco_process_packet(const fcgpu_cfg *c, const uint8_t *f, uint32_t len, fco_result *r)
{
    memset(r, 0, sizeof(*r));
    fcgpu_anno *a = &r->anno;
    uint32_t o = (uint32_t)c->offset;
    int reason;
    int v6 = 0;
    if (c->check_mode == FCGPU_CHECK_AUTO) {
        /* elements/ethernet/stripethervlanheader.cc:48-61; with vlan_ethertype,
         * VLANDecap(ETHERTYPE) + Strip(14) (elements/ethernet/vlandecap.cc:49-70) */
        if (be16(f + o + 12) == (c->vlan_ethertype ? c->vlan_ethertype : 0x8100)) {
            a->vlan_tci = raw16(f + o + 14);
            o += 18;
        } else if (c->native_vlan >= 0) {
            uint16_t t = (uint16_t)c->native_vlan;
            a->vlan_tci = (uint16_t)((t >> 8) | (t << 8));
            o += 14;
        } else {
            r->reason = FCGPU_R_VLAN_REJECT;
            r->port = (uint8_t)c->nports;
            return;
        }
        a->nh = (uint16_t)o;   /* the pull() StripEtherVLANHeader did */
        /* version dispatch as Classifier(0/60%f0, -): needs one byte */
        v6 = ((int)(len - o) >= 1) && ((f[o] >> 4) == 6);
        reason = v6 ? check_ip6(c, f, len, o, a) : check_ip4(c, f, len, o, a);
    } else if (c->check_mode == FCGPU_MARK_IP6) {
        /* elements/ip6/markip6header.cc:43-48: set_ip6_header(data + o, 40) */
        a->nh = (uint16_t)o;
        a->th = (uint16_t)(o + 40);
        a->length = (uint16_t)len;
        a->ipver = 6;
        v6 = 1;
        reason = FCGPU_R_OK;
    } else if (c->check_mode == FCGPU_MARK_IP4) {
        /* elements/ip/markipheader.cc:43-48 */
        a->nh = (uint16_t)o;
        a->th = (uint16_t)(o + ((f[o] & 15) << 2));
        a->length = (uint16_t)len;
        a->ipver = 4;
        reason = FCGPU_R_OK;
    } else {
        reason = check_ip4(c, f, len, o, a);
    }
    if (reason == FCGPU_R_OK && c->l4_mode != FCGPU_L4_NONE && !v6)
        reason = check_l4(c, f, a);
    r->reason = (uint8_t)reason;
    if (reason != FCGPU_R_OK) {
        r->port = (uint8_t)c->nports;
        return;
    }
    uint32_t h = 0;
    if (c->hash_mode != FCGPU_HASH_NONE) {
        const uint8_t *nh = f + a->nh, *th = f + a->th;
        if (v6) {
            /* lib/ip6flowid.cc:29-50 */
            h = fco_ip6flowid_hash(nh + 8, raw16(th), nh + 24, raw16(th + 2));
        } else {
            /* lib/ipflowid.cc:29-46: non-first fragments leave the ID
             * uninitialised in the reference; restated as the zero flow. */
            int first = (be16(nh + 6) & 0x1fff) == 0;
            if (first)
                h = fco_ipflowid_hash(le32(nh + 12), raw16(th), le32(nh + 16), raw16(th + 2));
            if (c->hash_mode == FCGPU_HASH_FLOW5ID)
                h ^= nh[9];   /* include/click/ipflowid.hh:242-251 */
        }
    }
    r->hash = h;
    int port = 0;
    switch (c->classify) {
    case FCGPU_CLS_LB_HASH:    port = fco_lb_hash_port(h, (int)c->nports); break;
    case FCGPU_CLS_LB_CRC: {
        /* IPFlow5ID(p): a non-first fragment keeps zero addresses (and, here,
         * zero ports), lib/ipflowid.cc:34-38 */
        const uint8_t *nh = f + a->nh, *th = f + a->th;
        int first = (be16(nh + 6) & 0x1fff) == 0;
        port = fco_lb_crc_port(nh[9], first ? le32(nh + 12) : 0, first ? le32(nh + 16) : 0,
                               first ? le32(th) : 0, (int)c->nports);
        break;
    }
    case FCGPU_CLS_LB_TABLE:   port = fco_lb_table_port(h); break;
    case FCGPU_CLS_HASH_IP:    port = fco_hash_ip_port(f, a->length, (int)c->nports); break;
    case FCGPU_CLS_HASHSWITCH: port = fco_hashswitch_port(f, a->length, c->hs_offset,
                                                           c->hs_length, (int)c->nports); break;
    case FCGPU_CLS_PROGRAM: {
        uint32_t out = fco_run_program(f, a);
        if (out >= c->nports) { r->reason = FCGPU_R_NO_MATCH; port = (int)c->nports; }
        else port = (int)out;
        break;
    }
    default: port = 0;
    }
    r->port = (uint8_t)port;
    if (r->reason == FCGPU_R_OK && !v6 && (c->rewrite & (FCGPU_RW_DECTTL | FCGPU_RW_SETCKSUM)))
        rewrite_ip4(c, f, r);
}

static int reason_slot(int r) { return r < 6 ? r : r - 1; }

void fco_process_batch(const fcgpu_cfg *c, const uint8_t *arena, const uint32_t *desc,
                       uint32_t n, uint16_t *verdict, uint32_t *hash, fcgpu_anno *anno,
                       uint32_t *perm, uint32_t *port_start, uint64_t *ctr)
{
    fco_process_batch2(c, arena, desc, n, verdict, hash, anno, perm, port_start, NULL, NULL, ctr, NULL);
}

void fco_process_batch2(const fcgpu_cfg *c, const uint8_t *arena, const uint32_t *desc,
                        uint32_t n, uint16_t *verdict, uint32_t *hash, fcgpu_anno *anno,
                        uint32_t *perm, uint32_t *port_start, uint32_t *perm_tile,
                        uint16_t *tile_count, uint64_t *ctr, uint32_t *ip_rw)
{
    int nb = (int)c->nports + 1;
    int *port = (int *)malloc(sizeof(int) * (n ? n : 1));
    for (uint32_t i = 0; i < n; i++) {
        fco_result r;
        fco_process_packet(c, arena + desc[2 * i], desc[2 * i + 1], &r);
        if (verdict) verdict[i] = (uint16_t)(r.reason | (r.port << 8));
        if (hash) hash[i] = r.hash;
        if (anno) anno[i] = r.anno;
        if (ip_rw) ip_rw[i] = r.ip_rw;
        port[i] = r.port;
        if (ctr) {
            if (r.reason == FCGPU_R_OK) ctr[FCGPU_CTR_COUNT]++;
            else if (r.reason >= FCGPU_R_NO_MATCH) { ctr[FCGPU_CTR_COUNT]++; ctr[FCGPU_CTR_REASON + reason_slot(r.reason)]++; }
            else { ctr[FCGPU_CTR_DROPS]++; ctr[FCGPU_CTR_REASON + reason_slot(r.reason)]++; }
            ctr[FCGPU_CTR_PORT + r.port]++;
        }
    }
    if (perm || port_start) {
        uint32_t start[FCGPU_MAX_PORTS + 2];
        fco_classify_each_packet(nb, port, n, perm, start);
        if (port_start) memcpy(port_start, start, sizeof(uint32_t) * (nb + 1));
    }
    if (perm_tile && tile_count)
        fco_partition_tiles(nb, port, n, FCGPU_TILE, perm_tile, tile_count);
    free(port);
}

/* ---- Flow table: FlowIPManagerHMP::process (elements/research/flowipmanagerhmp.cc:96-126) ----
 * `_hash.find_create(IPFlow5ID(p), [] { return _current.fetch_and_add(1); })`
 * walked over the batch on one thread: a flow's ID is the number of distinct
 * flows seen before its first packet, kept across batches (no timeouts).
 * Keys: IPFlow5ID(p) (lib/ipflowid.cc:29-46,91-94) = saddr, sport, daddr,
 * dport, ip_p; equality on all five (include/click/ipflowid.hh:236-240). The
 * reference leaves the ports of a non-first fragment uninitialised; we use 0.
 * Beyond max_flows IDs a new flow gets FCGPU_FLOW_FULL (the IMP managers kill
 * such a packet, include/click/flow/virtualflowmanager.hh:262-266). */
typedef struct { uint32_t saddr, daddr, ports, proto, id, used; } fco_flow_ent;
struct fco_flowtab {
    fco_flow_ent *e;
    uint32_t cap, n, next, max_flows;
};

fco_flowtab *fco_flow_new(uint32_t max_flows)
{
    fco_flowtab *t = (fco_flowtab *)calloc(1, sizeof(*t));
    t->cap = 1024;
    t->e = (fco_flow_ent *)calloc(t->cap, sizeof(fco_flow_ent));
    t->max_flows = max_flows;
    return t;
}

void fco_flow_free(fco_flowtab *t)
{
    if (t) { free(t->e); free(t); }
}

uint32_t fco_flow_count(const fco_flowtab *t) { return t->next; }

static uint32_t fco_flow_h(uint32_t a, uint32_t b, uint32_t c, uint32_t d)
{
    uint32_t h = a * 0x9E3779B1u ^ (b * 0x85EBCA77u) ^ (c * 0xC2B2AE3Du) ^ d;
    h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13;
    return h;
}

static fco_flow_ent *fco_flow_slot(fco_flowtab *t, uint32_t s, uint32_t d, uint32_t p, uint32_t pr)
{
    uint32_t i = fco_flow_h(s, d, p, pr) & (t->cap - 1);
    while (t->e[i].used && !(t->e[i].saddr == s && t->e[i].daddr == d && t->e[i].ports == p && t->e[i].proto == pr))
        i = (i + 1) & (t->cap - 1);
    return &t->e[i];
}

static void fco_flow_grow(fco_flowtab *t)
{
    fco_flow_ent *old = t->e;
    uint32_t oc = t->cap;
    t->cap *= 2;
    t->e = (fco_flow_ent *)calloc(t->cap, sizeof(fco_flow_ent));
    for (uint32_t i = 0; i < oc; i++)
        if (old[i].used) *fco_flow_slot(t, old[i].saddr, old[i].daddr, old[i].ports, old[i].proto) = old[i];
    free(old);
}

/* Packet i's IPFlow5ID, or 0 when it has no flow. The manager sits after the
 * checks, before the classifier and the header rewrites: packets those drop
 * still have a flow. */
static int fco_flow_key(const uint8_t *arena, const uint32_t *desc, const uint16_t *verdict,
                        const fcgpu_anno *anno, uint32_t i, uint32_t k[4])
{
    uint32_t reason = verdict[i] & 0xff;
    if (anno[i].ipver != 4 || (reason != FCGPU_R_OK && reason != FCGPU_R_NO_MATCH &&
                               reason != FCGPU_R_TTL_EXPIRED && reason != FCGPU_R_SETCKSUM_BAD))
        return 0;
    const uint8_t *nh = arena + desc[2 * i] + anno[i].nh;
    const uint8_t *th = arena + desc[2 * i] + anno[i].th;
    /* IPFlow5ID(p) (lib/ipflowid.cc:29-46, :91-94): a non-first fragment
     * returns before assign(), so its addresses stay IPAddress() = 0
     * (ipaddress.hh:21-22) and its ports unset (defined here as 0);
     * only ip_p is filled in */
    k[0] = k[1] = k[2] = 0;
    k[3] = nh[9];
    if (((((uint32_t)nh[6] << 8) | nh[7]) & 0x1fff) == 0) {   /* IP_FIRSTFRAG */
        memcpy(&k[0], nh + 12, 4);
        memcpy(&k[1], nh + 16, 4);
        memcpy(&k[2], th, 4);
    }
    return 1;
}

void fco_flow_batch(fco_flowtab *t, const uint8_t *arena, const uint32_t *desc, uint32_t n,
                    const uint16_t *verdict, const fcgpu_anno *anno, uint32_t *flowid)
{
    for (uint32_t i = 0; i < n; i++) {
        flowid[i] = FCGPU_FLOW_NONE;
        uint32_t k[4];
        if (!fco_flow_key(arena, desc, verdict, anno, i, k))
            continue;
        const uint32_t s = k[0], d = k[1], p = k[2], pr = k[3];
        if (2 * (t->n + 1) > t->cap) fco_flow_grow(t);
        fco_flow_ent *e = fco_flow_slot(t, s, d, p, pr);
        if (!e->used) {
            if (t->next >= t->max_flows) { flowid[i] = FCGPU_FLOW_FULL; continue; }
            e->saddr = s; e->daddr = d; e->ports = p; e->proto = pr;
            e->id = t->next++;
            e->used = 1;
            t->n++;
        }
        flowid[i] = e->id;
    }
}

/* ---- Flow table with timeouts: VirtualFlowManagerIMP over a FlowManagerIMPState
 * (include/click/flow/virtualflowmanager.hh; FlowIPManager_CuckooPP,
 * elements/flow/flowipmanager_cuckoopp.cc:57-110, is its table) ----
 * Written the reference's way -- a LIFO free-ID stack, a timer wheel of
 * singly linked lists, a released list pushed back one maintainer run later
 * -- so that the device's array formulation is checked against the linked
 * one. Time is the caller's, in ms (Timestamp::recent_steady at push_batch and
 * at the maintainer run); only differences of at most 2^31 ms are meaningful.
 *
 *   stack: initialised by pushing 0 .. cap-1 (:113-115), pops from the top
 *     (:36-38); the reference treats a popped 0 as "table full" (:264-268) and
 *     then reads below the stack on the next pop -- here the table is full
 *     while only 0 is left (the same until that point; defined after it).
 *   process (:249-327): a hit refreshes lastseen; a new flow pops an ID, is
 *     inserted, and is scheduled TE epochs ahead (:293-296). lastseen = the
 *     batch's time for every flow with a packet in the batch (:236-239,311-313).
 *   maintainer (:151-223): push the IDs released by the previous run (:155-161,
 *     walking the list from its head), then run the wheel's current bucket
 *     (timerwheel.hh run_timers: from the bucket's head, LIFO): lastseen not in
 *     the past -> reschedule after TE; old + interval >= timeout -> remove the
 *     key and prepend the ID to the released list; else reschedule after
 *     (timeout - old) * eps / 1000 epochs. Then the wheel index advances. */
#define FCO_NIL 0xffffffffu
struct fco_imp {
    uint32_t cap, hmask, nb;
    uint32_t *stack; int64_t si;
    uint32_t (*key)[4];
    uint32_t *hhead, *hnext, *lastseen, *whead, *wnext, *qnext;
    uint8_t *live;
    uint32_t qhead, windex;
    uint32_t to_ms, ri_ms, eps, te;
    uint32_t count;
};

static uint32_t fco_next_pow2(uint32_t x)
{
    uint32_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

fco_imp *fco_imp_new(uint32_t capacity, uint32_t timeout_s, uint32_t recycle_ms)
{
    fco_imp *t = (fco_imp *)calloc(1, sizeof(*t));
    t->cap = fco_next_pow2(capacity ? capacity : 1);
    t->hmask = fco_next_pow2(2 * t->cap) - 1;
    t->stack = (uint32_t *)malloc(sizeof(uint32_t) * (t->cap + 1));
    t->si = -1;
    for (uint32_t i = 0; i < t->cap; i++) t->stack[++t->si] = i;
    t->key = (uint32_t (*)[4])calloc(t->cap, sizeof(uint32_t[4]));
    t->hhead = (uint32_t *)malloc(sizeof(uint32_t) * (t->hmask + 1));
    for (uint32_t i = 0; i <= t->hmask; i++) t->hhead[i] = FCO_NIL;
    t->hnext = (uint32_t *)calloc(t->cap, sizeof(uint32_t));
    t->lastseen = (uint32_t *)calloc(t->cap, sizeof(uint32_t));
    t->wnext = (uint32_t *)calloc(t->cap, sizeof(uint32_t));
    t->qnext = (uint32_t *)calloc(t->cap, sizeof(uint32_t));
    t->live = (uint8_t *)calloc(t->cap, 1);
    t->qhead = FCO_NIL;
    /* parse (:58-79) */
    t->ri_ms = recycle_ms;
    t->eps = recycle_ms ? 1000 / recycle_ms : 1;
    if (t->eps < 1) t->eps = 1;
    t->to_ms = timeout_s * 1000;
    t->te = timeout_s * t->eps;
    t->nb = t->te ? fco_next_pow2(t->te + 2) : 1;   /* TimerWheel::initialize */
    t->whead = (uint32_t *)malloc(sizeof(uint32_t) * t->nb);
    for (uint32_t i = 0; i < t->nb; i++) t->whead[i] = FCO_NIL;
    return t;
}

void fco_imp_free(fco_imp *t)
{
    if (!t) return;
    free(t->stack); free(t->key); free(t->hhead); free(t->hnext); free(t->lastseen);
    free(t->whead); free(t->wnext); free(t->qnext); free(t->live); free(t);
}

static uint32_t fco_imp_bucket(const fco_imp *t, const uint32_t k[4])
{
    return fco_flow_h(k[0], k[1], k[2], k[3]) & t->hmask;
}

static uint32_t fco_imp_find(const fco_imp *t, const uint32_t k[4])
{
    for (uint32_t id = t->hhead[fco_imp_bucket(t, k)]; id != FCO_NIL; id = t->hnext[id])
        if (!memcmp(t->key[id], k, 16)) return id;
    return FCO_NIL;
}

static void fco_imp_remove(fco_imp *t, uint32_t id)
{
    uint32_t *pp = &t->hhead[fco_imp_bucket(t, t->key[id])];
    while (*pp != id) pp = &t->hnext[*pp];
    *pp = t->hnext[id];
    t->live[id] = 0;
    t->count--;
}

/* TimerWheel::schedule_after: prepend to bucket (index + after) & mask */
static void fco_imp_schedule(fco_imp *t, uint32_t id, uint32_t after)
{
    const uint32_t b = (t->windex + after) & (t->nb - 1);
    t->wnext[id] = t->whead[b];
    t->whead[b] = id;
}

void fco_imp_batch(fco_imp *t, const uint8_t *arena, const uint32_t *desc, uint32_t n,
                   const uint16_t *verdict, const fcgpu_anno *anno, uint32_t now_ms, uint32_t *flowid)
{
    for (uint32_t i = 0; i < n; i++) {
        flowid[i] = FCGPU_FLOW_NONE;
        uint32_t k[4];
        if (!fco_flow_key(arena, desc, verdict, anno, i, k))
            continue;
        uint32_t id = fco_imp_find(t, k);
        if (id == FCO_NIL) {
            if (t->si <= 0) { flowid[i] = FCGPU_FLOW_FULL; continue; }   /* only ID 0 left */
            id = t->stack[t->si--];
            memcpy(t->key[id], k, 16);
            const uint32_t b = fco_imp_bucket(t, k);
            t->hnext[id] = t->hhead[b];
            t->hhead[b] = id;
            t->live[id] = 1;
            t->count++;
            if (t->te) fco_imp_schedule(t, id, t->te);
        }
        t->lastseen[id] = now_ms;
        flowid[i] = id;
    }
}

uint32_t fco_imp_maintain(fco_imp *t, uint32_t now_ms)
{
    if (!t->te) return 0;
    while (t->qhead != FCO_NIL) {               /* :155-161 */
        const uint32_t next = t->qnext[t->qhead];
        t->stack[++t->si] = t->qhead;
        t->qhead = next;
    }
    uint32_t removed = 0;
    const uint32_t cur = t->windex & (t->nb - 1);
    uint32_t f = t->whead[cur];
    while (f != FCO_NIL) {                      /* run_timers */
        const uint32_t next = t->wnext[f];
        const int32_t old = (int32_t)(now_ms - t->lastseen[f]);
        if (old <= 0) {
            fco_imp_schedule(t, f, t->te);      /* :174-180 */
        } else if ((uint32_t)old + t->ri_ms >= t->to_ms) {
            fco_imp_remove(t, f);               /* :185-205 */
            t->qnext[f] = t->qhead;
            t->qhead = f;
            removed++;
        } else {
            const uint32_t r = ((t->to_ms - (uint32_t)old) * t->eps) / 1000u;   /* :209-211 */
            fco_imp_schedule(t, f, r ? r : 1u);   /* timerwheel.hh:25: timeout > 0 */
        }
        f = next;
    }
    t->whead[cur] = FCO_NIL;
    t->windex++;
    return removed;
}

void fco_imp_stats(const fco_imp *t, uint32_t *count, uint32_t *free_ids, uint32_t *pending)
{
    uint32_t q = 0;
    for (uint32_t f = t->qhead; f != FCO_NIL; f = t->qnext[f]) q++;
    *count = t->count;
    *free_ids = t->si > 0 ? (uint32_t)t->si : 0;   /* IDs the stack can still give */
    *pending = q;
}
