// TEST INFRASTRUCTURE ONLY: reference harness (oracle/_ref/fcref).
//
// Compiled by oracle/ref/Makefile against the REFERENCE's own headers
// (/root/reference/include: IPFlowID, IP6FlowID, IPAddress, IP6Address are
// header-inline) and the reference's lib/in_cksum.c compiled from its source
// location. It evaluates those reference functions on binary records from stdin
// and writes the raw results to stdout, for tests/golden/gen_golden.py.
//
//   fcref cksum : records [u16 len][len bytes]      -> u16 click_in_cksum
//   fcref flow4 : records [4 saddr][2 sport][4 daddr][2 dport] (raw network
//                 order)                            -> u32 low32(IPFlowID::hashcode)
//   fcref flow6 : records [16 src][2 sport][16 dst][2 dport]
//                                                   -> u32 low32(IP6FlowID::hashcode)
#include <click/config.h>
#include <click/ipflowid.hh>
#include <click/ip6flowid.hh>
#include <clicknet/ip.h>
#include <stdio.h>
#include <string.h>
#include <vector>

static bool rd(void *p, size_t n) { return fread(p, 1, n, stdin) == n; }

int main(int argc, char **argv) {
    if (argc < 2) return 2;
    const char *mode = argv[1];
    if (!strcmp(mode, "cksum")) {
        uint16_t len;
        std::vector<unsigned char> buf;
        while (rd(&len, 2)) {
            buf.resize(len + 1);
            if (len && !rd(buf.data(), len)) return 3;
            uint16_t c = click_in_cksum(buf.data(), len);
            fwrite(&c, 2, 1, stdout);
        }
    } else if (!strcmp(mode, "flow4")) {
        unsigned char r[12];
        while (rd(r, 12)) {
            uint32_t s, d;
            uint16_t sp, dp;
            memcpy(&s, r, 4); memcpy(&sp, r + 4, 2); memcpy(&d, r + 6, 4); memcpy(&dp, r + 10, 2);
            IPFlowID f{IPAddress(s), sp, IPAddress(d), dp};
            uint32_t h = (uint32_t)f.hashcode();
            fwrite(&h, 4, 1, stdout);
        }
    } else if (!strcmp(mode, "flow6")) {
        unsigned char r[36];
        while (rd(r, 36)) {
            uint16_t sp, dp;
            memcpy(&sp, r + 16, 2); memcpy(&dp, r + 34, 2);
            IP6FlowID f(IP6Address(r), sp, IP6Address(r + 18), dp);
            uint32_t h = (uint32_t)f.hashcode();
            fwrite(&h, 4, 1, stdout);
        }
    } else {
        return 2;
    }
    return 0;
}
