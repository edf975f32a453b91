// C++ end-to-end check of include/packet_rs_gpu.hpp on the GPU: parse the golden pcap
// (tests/golden/ref22.pcap) and print each packet's PacketSlice as
//   <index> <status> <name>@<off> ... | payload <off> <len> | to_vec_equal <0|1> | ttl <v>
// tests/test_cpp_mirror.py compares this with tests/golden/ref22_expected.json.
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iterator>
#include <vector>

#include "packet_rs_gpu.hpp"

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    std::ifstream f(argv[1], std::ios::binary);
    std::vector<uint8_t> buf((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    uint64_t n = 0;
    if (pkt_pcap_index(buf.data(), buf.size(), nullptr, nullptr, 0, &n) != PKT_SUCCESS) return 3;
    std::vector<uint64_t> offs(n);
    std::vector<uint32_t> lens(n);
    pkt_pcap_index(buf.data(), buf.size(), offs.data(), lens.data(), n, &n);
    uint8_t *d_slab;
    uint64_t* d_offs;
    uint32_t* d_lens;
    const size_t cap = (buf.size() + 255) / 256 * 256;
    packet_rs::gpu::hip_check(hipMalloc(&d_slab, cap), "hipMalloc");
    packet_rs::gpu::hip_check(hipMalloc(&d_offs, 8 * n), "hipMalloc");
    packet_rs::gpu::hip_check(hipMalloc(&d_lens, 4 * n), "hipMalloc");
    hipMemcpy(d_slab, buf.data(), buf.size(), hipMemcpyHostToDevice);
    hipMemcpy(d_offs, offs.data(), 8 * n, hipMemcpyHostToDevice);
    hipMemcpy(d_lens, lens.data(), 4 * n, hipMemcpyHostToDevice);
    pkt_batch_t b{};
    b.slab = d_slab;
    b.slab_len = buf.size();
    b.offsets = d_offs;
    b.lens = d_lens;
    b.n = n;
    packet_rs::gpu::Parser parser(0);
    auto res = parser.parse_chain(b);
    for (uint64_t i = 0; i < n; i++) {
        const uint8_t* pkt = buf.data() + offs[i];
        std::printf("%llu %s", (unsigned long long)i, pkt_status_name(res.status[i]));
        auto s = res.slice(i, pkt);
        for (const auto& h : s.hdrs) std::printf(" %s@%d", h.name(), (int)(h.as_slice() - pkt));
        auto v = s.to_vec();
        bool eq = v.size() == lens[i] && std::memcmp(v.data(), pkt, lens[i]) == 0;
        std::printf(" | payload %d %zu | len %zu | to_vec_equal %d", (int)(s.payload_ptr - pkt), s.payload_len,
                    s.len(), eq ? 1 : 0);
        try {
            std::printf(" | ttl %llu", (unsigned long long)s["IPv4"].field("ttl"));
        } catch (const std::out_of_range&) {
            std::printf(" | ttl -");
        }
        std::printf("\n");
    }
    // the same capture through Parser::parse_pcap (pkt_parse_pcap_host): identical chains and offsets
    std::vector<uint64_t> poffs;
    auto pres = parser.parse_pcap(buf.data(), buf.size(), poffs);
    bool same = pres.n == n && poffs == offs && pres.status == res.status && pres.n_hdrs == res.n_hdrs &&
                pres.payload_off == res.payload_off && pres.payload_len == res.payload_len;
    for (uint64_t i = 0; same && i < n; i++)
        for (int j = 0; j < res.n_hdrs[i]; j++)
            same = same && pres.hdr_type[(uint64_t)j * n + i] == res.hdr_type[(uint64_t)j * n + i] &&
                   pres.hdr_off[(uint64_t)j * n + i] == res.hdr_off[(uint64_t)j * n + i];
    std::fprintf(stderr, "parse_pcap_equal %d\n", same ? 1 : 0);
    hipFree(d_slab);
    hipFree(d_offs);
    hipFree(d_lens);
    return same ? 0 : 4;
}
