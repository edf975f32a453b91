// fuzz_host.cpp — sanitizer run of the host-side code (built by tests/test_sanitizers.py with
// -fsanitize=address,undefined; no GPU):
//   - pkt_pcap_index (packet-rs_amd/csrc/pktgpu_host.cpp), the parser of UNTRUSTED capture files
//     (tests/pcap.rs:7-37 format), on valid, truncated, bit-flipped and length-corrupted captures,
//     with every cap from 0 to past the count; each result is checked against a second, minimal
//     walk of the same format written here;
//   - the metadata and checksum entry points of the same file, on every id and on short buffers;
//   - the CPU oracle (oracle/pkt_oracle.c: fast::parse, getters, slow::parse + to_vec, setters)
//     on random and mutated packets under every entry.
// Prints "fuzz OK <iterations>" and exits 0; any sanitizer report aborts with a nonzero status.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/pktgpu.h"
#include "../../oracle/pkt_oracle.h"

namespace {

uint64_t rng_state = 0x5EED5A11u;
uint64_t rnd() {  // splitmix64
    uint64_t z = (rng_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
uint32_t rnd_below(uint32_t n) { return n ? (uint32_t)(rnd() % n) : 0; }

void put32(std::vector<uint8_t>& b, uint32_t v) {
    for (int k = 0; k < 4; k++) b.push_back((uint8_t)(v >> (8 * k)));
}

// A capture of `nrec` records with random lengths (some 0, some large).
std::vector<uint8_t> make_pcap(uint32_t nrec) {
    static const uint8_t hdr[24] = {0xD4, 0xC3, 0xB2, 0xA1, 2, 0, 4, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0xFF, 0xFF, 0, 0, 1, 0, 0, 0};
    std::vector<uint8_t> b(hdr, hdr + 24);
    for (uint32_t r = 0; r < nrec; r++) {
        const uint32_t len = rnd_below(8) == 0 ? 0 : rnd_below(8) == 0 ? rnd_below(3000) : rnd_below(300);
        put32(b, (uint32_t)rnd());
        put32(b, rnd_below(1000000));
        put32(b, len);
        put32(b, len + rnd_below(4));
        for (uint32_t k = 0; k < len; k++) b.push_back((uint8_t)rnd());
    }
    return b;
}

// Minimal second walk of the format: returns the record count, or -1 on an error.
long ref_count(const std::vector<uint8_t>& b, std::vector<uint64_t>& offs, std::vector<uint32_t>& lens) {
    offs.clear();
    lens.clear();
    if (b.size() < 24 || b[0] != 0xD4 || b[1] != 0xC3 || b[2] != 0xB2 || b[3] != 0xA1) return -1;
    uint64_t o = 24;
    while (o + 16 <= b.size()) {
        uint32_t incl;
        std::memcpy(&incl, &b[o + 8], 4);
        if (o + 16 + (uint64_t)incl > b.size()) return -1;
        offs.push_back(o + 16);
        lens.push_back(incl);
        o += 16 + (uint64_t)incl;
    }
    return (long)offs.size();
}

int check_pcap(const std::vector<uint8_t>& b) {
    std::vector<uint64_t> ro;
    std::vector<uint32_t> rl;
    const long want = ref_count(b, ro, rl);
    // exact-size copy so ASan sees any read past the end
    uint8_t* buf = (uint8_t*)std::malloc(b.size() ? b.size() : 1);
    if (!b.empty()) std::memcpy(buf, b.data(), b.size());
    uint64_t n = 0;
    const int rc0 = pkt_pcap_index(buf, b.size(), nullptr, nullptr, 0, &n);
    int bad = 0;
    if (want < 0) {
        bad |= rc0 == PKT_SUCCESS;
    } else {
        bad |= rc0 != PKT_SUCCESS || n != (uint64_t)want;
        for (uint64_t cap : {(uint64_t)0, (uint64_t)1, n / 2, n, n + 3}) {
            std::vector<uint64_t> o(cap + 1, ~0ull);
            std::vector<uint32_t> l(cap + 1, ~0u);
            uint64_t m = 0;
            const int rc = pkt_pcap_index(buf, b.size(), o.data(), l.data(), cap, &m);
            bad |= rc != PKT_SUCCESS || m != n;
            for (uint64_t k = 0; k < cap && k < n; k++) bad |= o[k] != ro[k] || l[k] != rl[k];
            bad |= o[cap] != ~0ull || l[cap] != ~0u;  // nothing written past cap
        }
    }
    std::free(buf);
    return bad;
}

void fuzz_oracle(uint32_t iters) {
    pkt_out_t out;
    std::memset(&out, 0, sizeof(out));
    // one packet's worth of every column (slot columns: PKT_MAX_HDRS rows of one)
    static uint8_t cols[49][16 * PKT_MAX_HDRS];
    void** c = reinterpret_cast<void**>(&out);
    for (int k = 0; k < 49; k++) c[k] = cols[k];
    for (uint32_t it = 0; it < iters; it++) {
        const uint32_t len = rnd_below(200);
        uint8_t* p = (uint8_t*)std::malloc(len ? len : 1);
        for (uint32_t k = 0; k < len; k++) p[k] = (uint8_t)rnd();
        if (len >= 14 && rnd_below(2)) {  // steer toward real chains
            static const uint16_t et[] = {0x0800, 0x86DD, 0x8100, 0x8847, 0x0806, 0x0020};
            const uint16_t e = et[rnd_below(6)];
            p[12] = (uint8_t)(e >> 8);
            p[13] = (uint8_t)e;
        }
        const int entry = (int)rnd_below(PKT_ENTRY_COUNT);
        orc_parse_one(p, len, entry, &out, 0, 1);
        uint8_t vec[512];
        (void)orc_slow_parse_to_vec(p, len, entry, vec, sizeof(vec));
        if (len >= 20) {
            (void)orc_ipv4_checksum(p, 20);
            (void)pkt_ipv4_checksum_host(p, 20);
            (void)orc_bit_range(p, 8 * 20 - 1, rnd_below(8 * 20));
            orc_set_bit_range(p, 8 * 20 - 1, rnd_below(8 * 20), rnd());
        }
        std::free(p);
    }
}

}  // namespace

int main(int argc, char** argv) {
    const uint32_t iters = argc > 1 ? (uint32_t)std::atoi(argv[1]) : 2000;
    int bad = 0;
    // metadata over every id, including out-of-range ones
    for (int t = -2; t < PKT_HDR_COUNT + 2; t++) {
        (void)pkt_hdr_name(t);
        (void)pkt_hdr_size(t);
        const int nf = pkt_hdr_field_count(t);
        for (int k = -1; k <= nf; k++) {
            const char* name = nullptr;
            uint16_t s = 0, e = 0;
            (void)pkt_hdr_field(t, k, &name, &s, &e);
        }
    }
    for (int k = -2; k < PKT_ENTRY_COUNT + 2; k++) (void)pkt_entry_name(k);
    for (int k = -2; k < 5; k++) (void)pkt_status_name(k);
    for (size_t n = 0; n < 24; n++) {  // short checksum inputs
        uint8_t* h = (uint8_t*)std::malloc(n ? n : 1);
        std::memset(h, 0xAB, n);
        (void)pkt_ipv4_checksum_host(h, n);
        std::free(h);
    }
    // pcap indexer
    for (uint32_t it = 0; it < iters; it++) {
        std::vector<uint8_t> b = make_pcap(rnd_below(40));
        switch (rnd_below(5)) {
            case 0: break;                                              // valid
            case 1: b.resize(rnd_below((uint32_t)b.size() + 1)); break;  // truncated anywhere
            case 2:                                                     // bit flips
                for (int k = 0; k < 4 && !b.empty(); k++) b[rnd_below((uint32_t)b.size())] ^= (uint8_t)(1u << rnd_below(8));
                break;
            case 3:                                                     // a corrupted incl_len
                if (b.size() > 40) {
                    const uint32_t o = 24 + 8;
                    const uint32_t v = (uint32_t)rnd();
                    std::memcpy(&b[o], &v, 4);
                }
                break;
            default: b.push_back((uint8_t)rnd()); break;                // trailing partial header
        }
        bad |= check_pcap(b);
        if (bad) {
            std::fprintf(stderr, "pcap index mismatch at iteration %u\n", it);
            return 1;
        }
    }
    // null / degenerate arguments
    uint64_t n = 0;
    bad |= pkt_pcap_index(nullptr, 0, nullptr, nullptr, 0, &n) == PKT_SUCCESS;
    fuzz_oracle(iters * 10);
    std::printf("fuzz OK %u\n", iters);
    return bad;
}
