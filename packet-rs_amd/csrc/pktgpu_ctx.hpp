// pktgpu_ctx.hpp — the pkt_ctx behind the C ABI's opaque handle, shared by the kernel sources
// (pktgpu.hip: parse / extract / rewrite; pktgpu_pcap.hip: the device pcap indexer).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "../../include/pktgpu.h"

// Device buffers and streams of the host-memory pipeline (pkt_parse_host), grown on demand.
struct HostPipe {
    static constexpr int kSlots = 3;
    bool init = false;
    hipStream_t s[kSlots] = {};
    hipEvent_t ev[kSlots] = {};  // a slot's slot-row count has reached the host (pkt_chain_max_hdrs words)
    uint8_t* slab[kSlots] = {};
    uint64_t* offs[kSlots] = {};
    uint32_t* lens[kSlots] = {};
    uint8_t* out[kSlots] = {};
    uint64_t slab_cap = 0, pkt_cap = 0, out_cap = 0;  // bytes per slot (pkt_cap: offs and lens)
    // pkt_parse_pcap_host: the capture and its index on the device
    uint8_t* file = nullptr;
    uint64_t* ioffs = nullptr;
    uint32_t* ilens = nullptr;
    uint64_t file_cap = 0, idx_cap = 0;  // bytes; records
    // a capture indexed and parsed as its bytes arrive (pkt_parse_pcap_host's pieces, pkt_pcap_stream_*,
    // pktgpu.hip Ingest): a ring of kRing steps' carry words (the prefix's first uncounted record start,
    // its record count, the magic check) and n_hdrs maxima, and the events ordering the steps' streams
    static constexpr int kRing = 4;
    uint64_t* pcarry = nullptr;  // [kRing][4]
    uint32_t* pnh = nullptr;     // [kRing][256]: a step's n_hdrs maximum, spread
    static constexpr int kCopyRing = 8;
    hipEvent_t ev_copy[kCopyRing] = {};      // copy c has landed (slot c % kCopyRing)
    hipEvent_t ev_parsed = nullptr;          // the last step's records are parsed
    hipEvent_t ev_xdone[kRing] = {};         // step j's export has read its ring slot
    uint8_t* dcol = nullptr;     // the capture's columns on the device (the export's source)
    uint64_t dcol_cap = 0;       // bytes
};

// Per-region state of the device pcap indexer (pkt_pcap_index_device), grown on demand.
struct PcapScratch {
    void* buf = nullptr;   // the ticket, nb_cap scan-block states, then k_cap regions' words
    uint64_t bytes = 0;
    uint32_t k_cap = 0;    // regions the buffer holds (its layout is fixed by k_cap / nb_cap)
    uint32_t nb_cap = 0;   // scan-block states the buffer holds
    uint64_t* ctl = nullptr;      // pinned host words the indexer reads back (magic, total, error)
    uint64_t* ctl_dev = nullptr;  // the same words as the device addresses them (the kernel writes them)
    uint32_t epoch = 0;           // per call: block states of older calls are ignored, not cleared
    uint32_t scan_resident = 0;   // scan-kernel blocks resident at once (0 = not yet queried)
    bool scan64 = false;          // pkt_ctx_set_pcap_scan64: 64-bit scan compositions for every file
    // a capture queued by pkt_parse_pcap_async / pkt_parse_pcap_host_async whose outcome (the words
    // above) has not been taken yet: no other index call may reuse the scratch until it is
    bool pending = false;
    hipStream_t pending_stream = nullptr;
};

// Element size of each pkt_out_t column, in declaration order (slot columns: one slot; the
// ipv6 addresses: 16 raw bytes).
constexpr int kNumCols = 49;
constexpr uint8_t kColSize[kNumCols] = {1, 1, 1, 2, 2, 2, 4, 8, 8, 2, 1, 1, 2, 2, 1, 1, 1, 2, 2, 1, 2,
                                        1, 1, 2, 4, 4, 2, 1, 1, 4, 2, 1, 1, 16, 16, 2, 2, 4, 4, 1,
                                        1, 1, 2, 2, 2, 2, 2, 2, 2};
constexpr int kColHdrType = 2, kColHdrOff = 3;  // slot-major [PKT_MAX_HDRS][n]
constexpr int kColIpv6Src = 33, kColIpv6Dst = 34;  // 16 raw bytes per packet, 16-byte aligned
static_assert(kColSize[kColIpv6Src] == 16 && kColSize[kColIpv6Dst] == 16, "ipv6 address columns");
static_assert(sizeof(pkt_out_t) == kNumCols * sizeof(void*), "pkt_out_t layout");

// Bytes of column c for n packets.
inline uint64_t col_bytes(int c, uint64_t n) {
    return n * kColSize[c] * ((c == kColHdrType || c == kColHdrOff) ? PKT_MAX_HDRS : 1);
}

// Words of the slot-row reductions (pkt_chain_max_hdrs, the fused maximum of the parse kernels): one
// group of 256 words (kMaxSpread, pktgpu_device.hpp) per host-pipeline slot + one for the blocking
// calls, on the device and mirrored in pinned host memory; a group's maximum is the max of its words.
struct MaxScratch {
    static constexpr int kGroups = HostPipe::kSlots + 1;
    static constexpr int kSpread = 256;
    uint32_t* dev = nullptr;
    uint32_t* host = nullptr;
    uint32_t* dgroup(int g) const { return dev + g * kSpread; }
    uint32_t* hgroup(int g) const { return host + g * kSpread; }
    uint32_t host_max(int g) const {
        uint32_t m = 0;
        for (int k = 0; k < kSpread; k++) m = m > host[g * kSpread + k] ? m : host[g * kSpread + k];
        return m;
    }
};

struct pkt_ctx {
    int device;
    HostPipe hp;
    PcapScratch pc;
    MaxScratch mx;
    uint32_t window;  // 0 = auto
    int fast;         // register fast path for Ether/IPv4/UDP|TCP packets
    int staging;      // 0 = auto, 1 = per-lane windows, 2 = wave span (LDS-DMA)
    int walk;         // 0 = auto, 1 = waterfall, 2 = lockstep
    uint64_t host_piece = 0;  // pkt_parse_pcap_host: bytes of file per copied piece (0 = kHostPiece)
    // pkt_to_vec_batch: device words, nonzero = a chunk holds bytes of two records; a ring, one word
    // per call, so calls in flight on several streams do not share one; a word is reused only after
    // the call that last used it has passed its to_vec kernel (the call's stream waits on tv_ev[k])
    static constexpr uint32_t kTvFlags = 256;
    static constexpr uint32_t kTvSlotWords = 8;  // a slot: the flag, then end(0) and end(n - 1) (u64, words 2-5)
    uint32_t* tv_flag = nullptr;
    hipEvent_t tv_ev[kTvFlags] = {};
    uint32_t tv_next = 0;
    uint32_t tv_epoch = 0;  // the last call's mark (never 0: the words start zeroed)
    // pkt_to_vec_batch in a capture's layout: per 4 KiB window of the slab, the first record ending
    // past the window's start (one table per ctx; a call's stream waits on tv_win_ev, recorded after
    // the previous call's window kernel, before writing it)
    uint32_t* tv_win = nullptr;
    uint64_t tv_win_cap = 0;
    hipEvent_t tv_win_ev = nullptr;
    std::string err;
};

inline int fail(pkt_ctx* ctx, int code, const char* msg) {
    if (ctx) ctx->err = msg;
    return code;
}

inline int hip_fail(pkt_ctx* ctx, hipError_t e, const char* what) {
    if (ctx) ctx->err = std::string(what) + ": " + hipGetErrorString(e);
    return PKT_ERR_HIP;
}

// pkt_parse_batch that also leaves the batch's largest n_hdrs (its used slot rows, <= PKT_MAX_HDRS
// for a parsed packet) in pinned host memory: *rows_host is valid once `stream` has passed the call.
// The reduction is fused into the parse kernel.  Used by the multi-GPU gather (pktgpu_mgpu.cpp).
// *rows_host = the group of MaxScratch::kSpread pinned words whose maximum is the row count.
int pktgpu_parse_rows_async(pkt_ctx_t* ctx, const pkt_batch_t* b, int entry, const pkt_out_t* out, void* stream,
                            const uint32_t** rows_host);

// pkt_parse_batch with the record count taken on the device from *count_dev (blocks past it exit;
// NULL = b->n) and the slot columns strided by slot_stride (0 = b->n).  One launch: b->n <= 2^26 when
// count_dev is given.  Used by pkt_parse_pcap (pktgpu_pcap.hip).
int pktgpu_parse_counted(pkt_ctx_t* ctx, const pkt_batch_t* b, int entry, const pkt_out_t* out, void* stream,
                         const uint64_t* count_dev, uint64_t slot_stride = 0);

// The device pcap indexer's kernels queued on `stream` (no host wait; *count_dev = the device word
// holding the record count, 0 after an error), and its outcome once the stream has passed them
// (pktgpu_pcap.hip).  Used by pkt_parse_pcap_host_async (pktgpu.hip).
// partial / count_out: index buf[0, len) as the PREFIX of a capture still arriving (a record running past
// its end ends the index, no error) and write the record count to the device word count_out (NULL: the
// ctx's own word, returned in *count_dev either way).  pktgpu_pcap_reserve: scratch for a file of len bytes.
// r0 / carry_in / carry_out (segment mode): index only the regions [r0, ceil(len / region)) of the prefix,
// from the previous prefix's carry words (carry_in: its first uncounted record start, its record count, the
// magic check; r0 * region <= that prefix's end), writing this prefix's carry to carry_out (4 words, may be
// NULL; count_out = carry_out + 1 keeps the count there too).  pktgpu_pcap_region_bytes: the region size.
int pktgpu_pcap_launch(pkt_ctx_t* ctx, const uint8_t* buf, uint64_t len, uint64_t* offsets, uint32_t* lens,
                       uint64_t cap, hipStream_t s, const uint64_t** count_dev, bool partial = false,
                       uint64_t* count_out = nullptr, uint32_t r0 = 0, const uint64_t* carry_in = nullptr,
                       uint64_t* carry_out = nullptr);
uint32_t pktgpu_pcap_region_bytes();
constexpr int kPcapCarryWords = 4;  // [first uncounted record start, records, magic check, -]
int pktgpu_pcap_reserve(pkt_ctx_t* ctx, uint64_t len, hipStream_t s);
int pktgpu_pcap_finish(pkt_ctx_t* ctx, uint64_t* n_out);
int pktgpu_pcap_take(pkt_ctx_t* ctx, uint64_t* n_out);  // a queued capture's outcome (waits; clears pending)

// The merged gather's root-side repack (pktgpu_gather.hip): copy `bytes` from device address `src` to
// `dst` for every piece; piece p is served by blocks [first_block, first_block + pktgpu_repack_blocks(
// bytes)), the table sorted by first_block (used by pkt_mgpu_parse_gather, pktgpu_mgpu.cpp).
struct RepackPiece {
    uint64_t src, dst, bytes;
    uint32_t first_block, reserved;
};
uint32_t pktgpu_repack_blocks(uint64_t bytes);
hipError_t pktgpu_repack_launch(const RepackPiece* tab_dev, uint32_t np, uint32_t nblocks, hipStream_t s);

// The host paths' column export (pktgpu_gather.hip): column range y copies elements [*lo_dev (NULL: 0),
// min(*hi_dev, cap)) — or [lo_h, hi_h) when hi_dev is NULL — of `sz` bytes from device address src + lo *
// sz to the host column dst + lo * sz (device-mapped); a slot row (row != kExportNoRow) only below the
// largest of the 256 words at nhw (NULL: every row).
constexpr uint32_t kExportNoRow = 0xFFFFu;
constexpr int kExportMax = 80;   // 47 per-packet columns + 2 x 16 slot rows
constexpr int kExportParts = 32; // blocks per column range
struct ExportCol {
    uint64_t src, dst;
    uint32_t sz, row;
};
struct ExportArgs {
    ExportCol col[kExportMax];
    const uint64_t* lo_dev;  // NULL with hi_dev NULL: the host-known range [lo_h, hi_h)
    const uint64_t* hi_dev;
    const uint32_t* nhw;     // NULL: every slot row
    uint64_t lo_h, hi_h;
    uint64_t cap;
    uint32_t ncol;
};
hipError_t pktgpu_export_launch(const ExportArgs& a, hipStream_t s);
