// packet_rs_gpu.hpp — C++ host mirror of packet_rs's decode API over the pktgpu C ABI.
//
// Shapes follow the reference so that C++ callers read like packet_rs users:
//   packet_rs::parser::fast::parse(&[u8]) -> PacketSlice      (src/parser/fast.rs:5)
//   PacketSlice::{payload, len, to_vec}, Index<&str>          (src/packet.rs:714-743, 61-67)
//   <Hdr>Slice::<field>() / bytes(msb, lsb) / name() / len()   (src/headers.rs:172-296)
// but work on whole batches: `Parser::parse` runs pkt_parse_batch on the GPU, `BatchResult`
// holds the host copy of the columns, and `BatchResult::slice(i, bytes)` rebuilds packet i's
// PacketSlice over the caller's bytes (zero-copy, like the reference's borrowed views).
// Header-only; link with libpktgpu.so and the HIP runtime.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "pktgpu.h"

namespace packet_rs {
namespace gpu {

inline void check(int rc, const pkt_ctx_t* ctx, const char* what) {
    if (rc != PKT_SUCCESS)
        throw std::runtime_error(std::string(what) + " failed (" + std::to_string(rc) + "): " +
                                 (ctx ? pkt_ctx_last_error(ctx) : ""));
}
inline void hip_check(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

// `<Hdr>Slice<'a>`: a header name plus a borrowed view of its bytes.
class HeaderSlice {
   public:
    HeaderSlice(int type, const uint8_t* p) : type_(type), p_(p) {}
    const char* name() const { return pkt_hdr_name(type_); }            // headers.rs:218-220
    size_t len() const { return (size_t)pkt_hdr_size(type_); }           // headers.rs:215-217
    int type() const { return type_; }
    const uint8_t* as_slice() const { return p_; }                       // headers.rs:221-223
    // headers.rs:253-263 (widths > 64: the release build's result, Q8)
    uint64_t bit_range(size_t msb, size_t lsb) const {
        uint64_t v = 0;
        for (size_t i = lsb; i <= msb; i++) v = (v << 1) | ((p_[i / 8] >> (7 - i % 8)) & 1u);
        const size_t sh = (64 - (msb - lsb + 1)) & 63;
        return v << sh >> sh;
    }
    // headers.rs:202-211
    std::vector<uint8_t> bytes(size_t msb, size_t lsb) const {
        std::vector<uint8_t> out;
        for (size_t i = lsb; i <= msb; i += 8) out.push_back((uint8_t)bit_range(i + 7, i));
        return out;
    }
    // `<Hdr>Slice::<field>()` by name, e.g. h.field("ttl")
    uint64_t field(const char* fname) const {
        for (int k = 0; k < pkt_hdr_field_count(type_); k++) {
            const char* nm;
            uint16_t s, e;
            pkt_hdr_field(type_, k, &nm, &s, &e);
            if (std::strcmp(nm, fname) == 0) return bit_range(e, s);
        }
        throw std::out_of_range(std::string(name()) + " has no field " + fname);
    }

   private:
    int type_;
    const uint8_t* p_;
};

// `PacketSlice<'a>` (lib.rs:136-140).
class PacketSlice {
   public:
    std::vector<HeaderSlice> hdrs;
    const uint8_t* payload_ptr = nullptr;
    size_t payload_len = 0;

    std::pair<const uint8_t*, size_t> payload() const { return {payload_ptr, payload_len}; }
    size_t len() const {  // packet.rs:741-743
        size_t s = payload_len;
        for (const auto& h : hdrs) s += h.len();
        return s;
    }
    std::vector<uint8_t> to_vec() const {  // packet.rs:733-740
        std::vector<uint8_t> v;
        for (const auto& h : hdrs) v.insert(v.end(), h.as_slice(), h.as_slice() + h.len());
        v.insert(v.end(), payload_ptr, payload_ptr + payload_len);
        return v;
    }
    // Index<&str>: the first header with that name (packet.rs:64-66); throws like unwrap().
    const HeaderSlice& operator[](const char* name) const {
        for (const auto& h : hdrs)
            if (std::strcmp(h.name(), name) == 0) return h;
        throw std::out_of_range(std::string("no header ") + name);
    }
};

// Host copy of the chain + field columns of one batch.
struct BatchResult {
    uint64_t n = 0;
    std::vector<uint8_t> status, n_hdrs, hdr_type;
    std::vector<uint16_t> hdr_off, payload_off, payload_len;
    std::vector<uint32_t> hdr_mask;

    // packet i's PacketSlice over its bytes `pkt` (the same bytes that were parsed).
    PacketSlice slice(uint64_t i, const uint8_t* pkt) const {
        if (status[i] != PKT_OK)
            throw std::runtime_error(std::string("packet ") + std::to_string(i) + ": " + pkt_status_name(status[i]));
        PacketSlice s;
        for (int j = 0; j < n_hdrs[i]; j++)
            s.hdrs.emplace_back(hdr_type[(uint64_t)j * n + i], pkt + hdr_off[(uint64_t)j * n + i]);
        s.payload_ptr = pkt + payload_off[i];
        s.payload_len = payload_len[i];
        return s;
    }
};

// A pkt_ctx plus device scratch for the chain columns.
struct DeviceFree {
    void operator()(void* p) const { (void)hipFree(p); }
};

class Parser {
   public:
    explicit Parser(int device = 0) { check(pkt_ctx_create(device, &ctx_), nullptr, "pkt_ctx_create"); }
    ~Parser() { pkt_ctx_destroy(ctx_); }
    Parser(const Parser&) = delete;
    Parser& operator=(const Parser&) = delete;
    pkt_ctx_t* ctx() { return ctx_; }

    // fast::parse_<entry> over a device batch; chain columns only, copied back to the host.
    BatchResult parse_chain(const pkt_batch_t& b, pkt_entry_t entry = PKT_ENTRY_PARSE, hipStream_t s = nullptr) {
        BatchResult r;
        r.n = b.n;
        if (b.n == 0) return r;
        const uint64_t n = b.n;
        void* d = nullptr;
        const size_t bytes = n * (1 + 1 + PKT_MAX_HDRS + 2 * PKT_MAX_HDRS + 2 + 2 + 4) + 64;
        hip_check(hipMalloc(&d, bytes), "hipMalloc");
        // freed on every exit, including a hip_check throw below
        std::unique_ptr<void, DeviceFree> guard(d);
        uint8_t* base = static_cast<uint8_t*>(d);
        pkt_out_t o;
        std::memset(&o, 0, sizeof(o));
        size_t off = 0;
        auto take = [&](size_t nb, size_t align) {
            off = (off + align - 1) / align * align;
            uint8_t* p = base + off;
            off += nb;
            return p;
        };
        o.hdr_mask = reinterpret_cast<uint32_t*>(take(4 * n, 4));
        o.hdr_off = reinterpret_cast<uint16_t*>(take(2 * n * PKT_MAX_HDRS, 2));
        o.payload_off = reinterpret_cast<uint16_t*>(take(2 * n, 2));
        o.payload_len = reinterpret_cast<uint16_t*>(take(2 * n, 2));
        o.status = take(n, 1);
        o.n_hdrs = take(n, 1);
        o.hdr_type = take(n * PKT_MAX_HDRS, 1);
        int rc = pkt_parse_batch(ctx_, &b, entry, &o, s);
        if (rc == PKT_SUCCESS) {
            r.status.resize(n); r.n_hdrs.resize(n); r.hdr_type.resize(n * PKT_MAX_HDRS);
            r.hdr_off.resize(n * PKT_MAX_HDRS); r.payload_off.resize(n); r.payload_len.resize(n);
            r.hdr_mask.resize(n);
            hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
            hip_check(hipMemcpy(r.status.data(), o.status, n, hipMemcpyDeviceToHost), "copy");
            hip_check(hipMemcpy(r.n_hdrs.data(), o.n_hdrs, n, hipMemcpyDeviceToHost), "copy");
            hip_check(hipMemcpy(r.hdr_type.data(), o.hdr_type, n * PKT_MAX_HDRS, hipMemcpyDeviceToHost), "copy");
            hip_check(hipMemcpy(r.hdr_off.data(), o.hdr_off, 2 * n * PKT_MAX_HDRS, hipMemcpyDeviceToHost), "copy");
            hip_check(hipMemcpy(r.payload_off.data(), o.payload_off, 2 * n, hipMemcpyDeviceToHost), "copy");
            hip_check(hipMemcpy(r.payload_len.data(), o.payload_len, 2 * n, hipMemcpyDeviceToHost), "copy");
            hip_check(hipMemcpy(r.hdr_mask.data(), o.hdr_mask, 4 * n, hipMemcpyDeviceToHost), "copy");
        }
        check(rc, ctx_, "pkt_parse_batch");
        return r;
    }

    // tests/pcap.rs:7-37 on the GPU: every record of a pcap capture in host memory through
    // fast::parse_<entry> (pkt_parse_pcap_host: copy in, device index, parse, chain columns back).
    // offsets[i] = record i's data offset in `file`, so BatchResult::slice(i, file + offsets[i]) is
    // its PacketSlice.  Throws like the reference's unwrap on a malformed capture.
    BatchResult parse_pcap(const uint8_t* file, size_t len, std::vector<uint64_t>& offsets,
                           pkt_entry_t entry = PKT_ENTRY_PARSE) {
        uint64_t n = 0;
        check(pkt_pcap_index(file, len, nullptr, nullptr, 0, &n), nullptr, "pkt_pcap_index (malformed capture)");
        BatchResult r;
        r.n = n;
        offsets.assign(n, 0);
        if (n == 0) return r;
        r.status.resize(n); r.n_hdrs.resize(n); r.hdr_type.resize(n * PKT_MAX_HDRS);
        r.hdr_off.resize(n * PKT_MAX_HDRS); r.payload_off.resize(n); r.payload_len.resize(n);
        r.hdr_mask.resize(n);
        std::vector<uint32_t> lens(n);
        pkt_out_t o;
        std::memset(&o, 0, sizeof(o));
        o.status = r.status.data();
        o.n_hdrs = r.n_hdrs.data();
        o.hdr_type = r.hdr_type.data();
        o.hdr_off = r.hdr_off.data();
        o.payload_off = r.payload_off.data();
        o.payload_len = r.payload_len.data();
        o.hdr_mask = r.hdr_mask.data();
        uint64_t m = 0;
        check(pkt_parse_pcap_host(ctx_, file, len, entry, &o, offsets.data(), lens.data(), n, &m), ctx_,
              "pkt_parse_pcap_host");
        return r;
    }

   private:
    pkt_ctx_t* ctx_ = nullptr;
};

}  // namespace gpu
}  // namespace packet_rs
