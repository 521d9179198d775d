// pcap_reader.cc -- pcap ingress (include/fcpcap.h): FromDump's record parsing
// (elements/userlevel/fromdump.cc:278-316, 418-500) over read() straight into
// the caller's buffer; descriptors point at the packet bytes in place.
#include <algorithm>
#include <errno.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <string.h>
#include <unistd.h>

#include <string>
#include <thread>
#include <vector>

#include "../../../include/fcpcap.h"

namespace {
constexpr uint32_t kMagic = 0xA1B2C3D4u, kMagicNano = 0xA1B23C4Du, kMagicModified = 0xA1B2CD34u;
inline uint32_t sw32(uint32_t x) { return __builtin_bswap32(x); }
}  // namespace

struct fcpcap {
    int fd = -1;
    bool swapped = false, nano = false;
    uint32_t extra = 0;          // modified pcap: 8 header bytes after the regular 16
    int minor = 0, linktype = 0;
    uint32_t snaplen = 0;
    std::vector<uint8_t> carry;  // bytes read but not yet handed out (a partial record)
    bool eof = false;
    off_t fpos = 24;             // file offset of the next unread byte
    unsigned threads = 1;        // parallel pread() pieces per fill
    const uint8_t *map = nullptr;  // fcpcap_map: the whole file, read-only
    size_t map_bytes = 0;
    std::string err;
};

extern "C" {

int fcpcap_open(const char *path, fcpcap **out, char *err, size_t errcap) {
    auto fail = [&](const std::string &m) {
        if (err && errcap) snprintf(err, errcap, "%s", m.c_str());
        return -1;
    };
    if (!path || !out) return fail("null argument");
    int fd = open(path, O_RDONLY);
    if (fd < 0) return fail(std::string(path) + ": " + strerror(errno));
    uint32_t fh[6];
    ssize_t k = read(fd, fh, sizeof fh);
    if (k != (ssize_t)sizeof fh) {
        close(fd);
        return fail("not a tcpdump file (too short)");
    }
    fcpcap *r = new fcpcap;
    r->fd = fd;
    uint32_t magic = fh[0];
    if (magic != kMagic && magic != kMagicNano && magic != kMagicModified) {
        r->swapped = true;
        magic = sw32(magic);
    }
    if (magic != kMagic && magic != kMagicNano && magic != kMagicModified) {
        fcpcap_close(r);
        return fail("not a tcpdump file (bad magic number)");
    }
    r->extra = magic == kMagicModified ? 8 : 0;
    r->nano = magic == kMagicNano;
    uint32_t ver = r->swapped ? sw32(fh[1]) : fh[1];
    // version_major / version_minor are 16-bit fields in file order
    uint16_t vmaj, vmin;
    memcpy(&vmaj, reinterpret_cast<uint8_t *>(fh) + 4, 2);
    memcpy(&vmin, reinterpret_cast<uint8_t *>(fh) + 6, 2);
    if (r->swapped) {
        vmaj = __builtin_bswap16(vmaj);
        vmin = __builtin_bswap16(vmin);
    }
    (void)ver;
    if (vmaj != 2) {
        fcpcap_close(r);
        return fail("unknown major version " + std::to_string(vmaj));
    }
    r->minor = vmin;
    r->snaplen = r->swapped ? sw32(fh[4]) : fh[4];
    r->linktype = (int)(r->swapped ? sw32(fh[5]) : fh[5]);
    *out = r;
    return 0;
}

int fcpcap_linktype(const fcpcap *r) { return r ? r->linktype : -1; }
int fcpcap_set_threads(fcpcap *r, unsigned threads) {
    if (!r || threads < 1 || threads > 64) return -1;
    r->threads = threads;
    return 0;
}
uint32_t fcpcap_snaplen(const fcpcap *r) { return r ? r->snaplen : 0; }
const char *fcpcap_error(const fcpcap *r) { return r ? r->err.c_str() : "null reader"; }

void fcpcap_close(fcpcap *r) {
    if (!r) return;
    if (r->map) munmap(const_cast<uint8_t *>(r->map), r->map_bytes);
    if (r->fd >= 0) close(r->fd);
    delete r;
}

int fcpcap_map(fcpcap *r, const uint8_t **base, size_t *bytes) {
    if (!r || !base || !bytes) return -1;
    if (!r->map) {
        struct stat st;
        if (fstat(r->fd, &st) != 0) {
            r->err = std::string("fstat: ") + strerror(errno);
            return -1;
        }
        void *m = mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_SHARED | MAP_POPULATE, r->fd, 0);
        if (m == MAP_FAILED) {
            r->err = std::string("mmap: ") + strerror(errno);
            return -1;
        }
        r->map = static_cast<const uint8_t *>(m);
        r->map_bytes = (size_t)st.st_size;
    }
    *base = r->map;
    *bytes = r->map_bytes;
    return 0;
}

// One record header at pos of the mapped file, by FromDump::read_packet's
// rules (fromdump.cc:446-466, as fcpcap_read): 1 parsed, 0 the record does not
// fit in the file (a truncated final record), -1 a bad header.
namespace {
struct Rec {
    uint32_t len, caplen;
    size_t size;                 // header + captured bytes (+ bytes past len)
    uint64_t ts_ns;
};
inline int parse_rec(const fcpcap *r, size_t pos, Rec &o) {
    if (pos + 16 > r->map_bytes) return 0;
    uint32_t h[4];
    memcpy(h, r->map + pos, 16);
    if (r->swapped)
        for (auto &x : h) x = sw32(x);
    uint32_t len, caplen, skip = 0;
    if (r->minor > 3 || (r->minor == 3 && h[2] <= h[3])) {
        len = h[3];
        caplen = h[2];
    } else {
        len = h[2];
        caplen = h[3];
    }
    if (caplen > 65535) return -1;
    if (caplen > len) {
        skip = caplen - len;
        caplen = len;
    }
    o.len = len;
    o.caplen = caplen;
    o.size = (size_t)16 + r->extra + caplen + skip;
    o.ts_ns = (uint64_t)h[0] * 1000000000ull + (uint64_t)h[1] * (r->nano ? 1ull : 1000ull);
    if (pos + o.size > r->map_bytes) return 0;
    return 1;
}
// Could a record header start at pos? For the parallel walk's speculative
// starts only: a sub-second field in range and a sane length, for 16
// consecutive records (or to the end of the range). A wrong guess is caught
// when the walks are stitched.
inline bool plausible_chain(const fcpcap *r, size_t pos, size_t end) {
    for (int k = 0; k < 16 && pos < end; ++k) {
        Rec q;
        if (parse_rec(r, pos, q) != 1) return false;
        uint32_t frac;
        memcpy(&frac, r->map + pos + 4, 4);
        if (r->swapped) frac = sw32(frac);
        if (frac >= (r->nano ? 1000000000u : 1000000u) || q.len > (1u << 24)) return false;
        pos += q.size;
    }
    return true;
}
struct Walk {
    size_t from = 0, end = 0;    // first record start; the position after the walk's last record
    size_t bad = (size_t)-1;     // position of a bad header the walk stopped at
    std::vector<size_t> pos;     // record starts
    std::vector<Rec> rec;
};
// Records from `from` while their starts are below `stop` (and fit the file).
void walk(const fcpcap *r, size_t from, size_t stop, Walk &w) {
    w.from = from;
    w.pos.clear();
    w.rec.clear();
    w.bad = (size_t)-1;
    size_t pos = from;
    while (pos < stop) {
        Rec q;
        const int k = parse_rec(r, pos, q);
        if (k < 0) { w.bad = pos; break; }
        if (k == 0) break;
        w.pos.push_back(pos);
        w.rec.push_back(q);
        pos += q.size;
    }
    w.end = pos;
}
}  // namespace

int fcpcap_index(fcpcap *r, uint32_t max, size_t max_bytes, size_t *chunk_off, size_t *chunk_bytes, uint32_t *desc,
                 uint32_t *wire, uint64_t *ts_ns) {
    if (!r || !r->map || !chunk_off || !chunk_bytes || !desc) return -1;
    const uint32_t hdr = 16 + r->extra;
    const size_t start = (size_t)r->fpos;
    const size_t lim = std::min(r->map_bytes, start + max_bytes);   // record starts of this chunk lie below
    // the walk over [start, lim): in T pieces on T threads when the chunk is
    // large -- piece 0 from the exact start, the others from the first
    // plausible record header at or after their piece's start, each until
    // its records start in the next piece; stitched in order, a piece whose
    // guessed start is not where the walk before it ended is walked again
    // from there. The result is the sequential walk's, record for record.
    const size_t span = lim > start ? lim - start : 0;
    const unsigned T = (unsigned)std::max<size_t>(1, std::min<size_t>(r->threads, span >> 22));   // >= 4 MiB each
    std::vector<Walk> w(T);
    std::vector<size_t> b(T + 1);
    for (unsigned t = 0; t <= T; ++t) b[t] = start + span * t / T;
    auto piece = [&](unsigned t) {
        size_t from = b[t];
        if (t) {
            const size_t last = std::min(b[t + 1], b[t] + (size_t)hdr + 65535 * 2);
            while (from < last && !plausible_chain(r, from, lim)) ++from;
            if (from >= last) { w[t].from = (size_t)-1; return; }
        }
        walk(r, from, b[t + 1], w[t]);
    };
    if (T > 1) {
        std::vector<std::thread> th;
        for (unsigned t = 1; t < T; ++t) th.emplace_back(piece, t);
        piece(0);
        for (auto &x : th) x.join();
        for (unsigned t = 1; t < T; ++t)
            if (w[t].from != w[t - 1].end || w[t - 1].bad != (size_t)-1) {
                if (w[t - 1].bad != (size_t)-1) { w.resize(t); break; }   // the bad header ends the walk
                walk(r, w[t - 1].end, b[t + 1], w[t]);
            }
    } else {
        walk(r, start, lim, w[0]);
    }
    // the chunk: up to max records, the last ending within max_bytes of the start
    uint32_t n = 0;
    size_t pos = start;
    for (const Walk &x : w) {
        for (size_t k = 0; k < x.pos.size() && n < max; ++k) {
            const Rec &q = x.rec[k];
            if (x.pos[k] + q.size - start > max_bytes && n) goto done;
            desc[2 * n] = (uint32_t)(x.pos[k] + hdr - start);
            desc[2 * n + 1] = q.caplen;
            if (wire) wire[n] = q.len;
            if (ts_ns) ts_ns[n] = q.ts_ns;
            ++n;
            pos = x.pos[k] + q.size;
        }
        if (n >= max) break;
        if (x.bad != (size_t)-1) {
            // reached: the records before it leave now, and the next call
            // starts at the bad header and fails (FromDump stops there too)
            if (n) goto done;
            r->err = "bad packet header; giving up";
            return -1;
        }
    }
done:
    *chunk_off = start;
    *chunk_bytes = pos - start;
    r->fpos = (off_t)pos;
    return (int)n;
}

int fcpcap_read(fcpcap *r, uint8_t *buf, size_t cap, uint32_t *desc, uint32_t *wire, uint64_t *ts_ns,
                uint32_t max, size_t *used) {
    if (!r || !buf || !desc || !used) return -1;
    *used = 0;
    // the carried partial record first, then as much of the file as fits
    size_t have = r->carry.size() < cap ? r->carry.size() : cap;
    if (have) memcpy(buf, r->carry.data(), have);   // (an empty carry's data() may be null)
    r->carry.erase(r->carry.begin(), r->carry.begin() + have);
    if (!r->eof && have < cap && r->carry.empty()) {
        // the rest of the buffer from the file, as `threads` pread() pieces of
        // at least 1 MiB (the copy out of the page cache is the host-side cost
        // of this ingress); a short piece is the end of the file
        const size_t want = cap - have;
        const unsigned T = (unsigned)std::max<size_t>(1, std::min<size_t>(r->threads, want >> 20));
        std::vector<ssize_t> got(T, 0);
        std::vector<int> errs(T, 0);
        const size_t per = (want + T - 1) / T;
        auto piece = [&](unsigned t) {
            const size_t b = t * per, e = std::min(want, b + per);
            size_t done = 0;
            while (b + done < e) {
                ssize_t k = pread(r->fd, buf + have + b + done, e - b - done, r->fpos + (off_t)(b + done));
                if (k < 0) {
                    if (errno == EINTR) continue;
                    errs[t] = errno;
                    break;
                }
                if (k == 0) break;
                done += (size_t)k;
            }
            got[t] = (ssize_t)done;
        };
        std::vector<std::thread> th;
        for (unsigned t = 1; t < T; ++t) th.emplace_back(piece, t);
        piece(0);
        for (auto &x : th) x.join();
        size_t total = 0;
        for (unsigned t = 0; t < T; ++t) {
            if (errs[t]) {
                r->err = std::string("read: ") + strerror(errs[t]);
                return -1;
            }
            const size_t b = t * per, e = std::min(want, b + per);
            total += (size_t)got[t];
            if ((size_t)got[t] < e - b) {   // end of file inside this piece
                r->eof = true;
                break;
            }
        }
        r->fpos += (off_t)total;
        have += total;
    }
    const uint32_t hdr = 16 + r->extra;
    size_t pos = 0;
    uint32_t n = 0;
    while (n < max && pos + 16 <= have) {
        uint32_t h[4];
        memcpy(h, buf + pos, 16);
        if (r->swapped)
            for (auto &x : h) x = sw32(x);
        // FromDump::read_packet: caplen/len swapped before 2.3 (fromdump.cc:446-453)
        uint32_t len, caplen, skip = 0;
        if (r->minor > 3 || (r->minor == 3 && h[2] <= h[3])) {
            len = h[3];
            caplen = h[2];
        } else {
            len = h[2];
            caplen = h[3];
        }
        if (caplen > 65535) {   // fromdump.cc:460-462
            r->err = "bad packet header; giving up";
            return -1;
        }
        if (caplen > len) {     // fromdump.cc:463-466
            skip = caplen - len;
            caplen = len;
        }
        const size_t rec = (size_t)hdr + caplen + skip;
        if (pos + rec > have) break;
        desc[2 * n] = (uint32_t)(pos + hdr);
        desc[2 * n + 1] = caplen;
        if (wire) wire[n] = len;
        if (ts_ns) ts_ns[n] = (uint64_t)h[0] * 1000000000ull + (uint64_t)h[1] * (r->nano ? 1ull : 1000ull);
        ++n;
        pos += rec;
    }
    if (n == 0 && pos + 16 <= have && r->eof && have < cap) {
        // a record cut short by the end of the file: FromDump stops there
        have = pos;
    }
    // keep what was not handed out for the next call
    if (pos < have) r->carry.insert(r->carry.begin(), buf + pos, buf + have);
    if (n == 0 && !r->carry.empty() && (r->eof || have == cap)) {
        if (have == cap && pos == 0) {
            r->err = "record larger than the buffer";
            return -1;
        }
        if (r->eof) r->carry.clear();   // truncated final record
    }
    *used = pos;
    return (int)n;
}

}  // extern "C"
