// pktgpu_mgpu.cpp — packed output layout and the multi-GPU entry (pkt_mgpu_*) of the C ABI.
//
// One process drives several MI355X devices.  Every fast::parse_* is a pure function of one
// packet's bytes (reference src/parser/fast.rs:5-227), so a batch splits into contiguous shards
// with no exchange inside the parse; the only collective is the gather of the per-packet tuples
// to the root device: grouped ncclSend/ncclRecv (RCCL over xGMI) on one communicator per device
// from ncclCommInitAll.  A shard's tuples live in ONE packed buffer (pkt_out_packed), so the
// gather is one message per shard; the merged form sends each column (slot row) separately.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "pktgpu_ctx.hpp"

struct pkt_mgpu {
    static constexpr int kMaxStreams = 4;
    int ndev = 0;
    std::vector<int> dev;
    std::vector<pkt_ctx_t*> ctx;
    std::vector<hipStream_t> stream;  // each device's work stream (the gather runs on it)
    std::vector<ncclComm_t> comm;
    // pkt_mgpu_parse_steps: extra streams per device (joined back into `stream` after each call)
    // and one event per stream, created on first use
    std::vector<hipStream_t> xs;  // [ndev][kMaxStreams - 1]
    std::vector<hipEvent_t> xe;   // [ndev][kMaxStreams]
    bool xinit = false;           // xs / xe all created (set only after every creation succeeded)
    int root_copy = 1;            // the root's own pieces: 1 = hipMemcpyAsync, 0 = RCCL send/recv to itself
    int gather_rows = 0;          // slot rows parse_gather moves: 0 = each shard's largest n_hdrs (waits), 1..16 fixed
    // pkt_mgpu_set_gather_rows(k > 0): each shard's measured n_hdrs maximum of the last parse_gather (pinned
    // words), checked against k by pkt_mgpu_synchronize once the streams have passed it
    std::vector<const uint32_t*> rows_check;
    // pkt_mgpu_create_virtual: no communicators; repeated devices allowed; the gather's messages are device
    // copies on the sending shard's stream, ordered against the root's stream by one event per shard
    bool virt = false;
    std::vector<hipEvent_t> vev;
    // merge = 1: the root's staging area for the shards' packed buffers (the merge = 0 transfer) and
    // the repack table (pinned host copy, device copy; rp_ev = the last table upload has been read)
    int stage_dev = -1;
    uint8_t* stage = nullptr;
    uint64_t stage_cap = 0;
    RepackPiece* rp_host = nullptr;
    RepackPiece* rp_dev = nullptr;
    uint64_t rp_cap = 0;  // pieces
    hipEvent_t rp_ev = nullptr;
    std::string err;
};

namespace {

constexpr uint64_t kAlign = 256;
// Why the last pkt_mgpu_create on this thread failed (there is no handle to hold it):
// pkt_mgpu_last_error(NULL) returns it.
thread_local std::string g_create_err;
int create_fail(int code, const std::string& msg) {
    g_create_err = msg;
    return code;
}
inline uint64_t round_up(uint64_t x) { return (x + kAlign - 1) & ~(kAlign - 1); }

int mfail(pkt_mgpu* mg, int code, const std::string& msg) {
    if (mg) mg->err = msg;
    return code;
}
int mhip(pkt_mgpu* mg, hipError_t e, const char* what) {
    return mfail(mg, PKT_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}
int mnccl(pkt_mgpu* mg, ncclResult_t r, const char* what) {
    return mfail(mg, PKT_ERR_HIP, std::string(what) + ": " + ncclGetErrorString(r));
}

// Offset of column c inside a packed buffer of n packets: the selected per-packet columns in
// pkt_out_t order, then the slot columns hdr_type and hdr_off ([PKT_MAX_HDRS][n] each) last, so
// that a batch's used slot rows [0, rows) end the first piece of the buffer (packed_pieces).
uint64_t packed_layout(uint64_t mask, uint64_t n, uint64_t* off /* [kNumCols] or NULL */) {
    uint64_t o = 0;
    auto place = [&](int c) {
        if (!(mask >> c & 1)) return;
        if (off) off[c] = o;
        o += round_up(col_bytes(c, n));
    };
    for (int c = 0; c < kNumCols; c++)
        if (c != kColHdrType && c != kColHdrOff) place(c);
    place(kColHdrType);
    place(kColHdrOff);
    return o;
}

// The byte ranges of an n-packet packed buffer that hold every selected column with only the
// first `rows` slot rows (a PacketSlice holds exactly its headers, lib.rs:136-140): the head up to
// the end of hdr_type's used rows (or of hdr_off's when hdr_type is not selected), then hdr_off's
// used rows.  Returns the number of pieces (1 or 2).
int packed_pieces(uint64_t mask, uint64_t n, uint32_t rows, uint64_t off[2], uint64_t len[2]) {
    uint64_t co[kNumCols];
    const uint64_t total = packed_layout(mask, n, co);
    const bool t = mask >> kColHdrType & 1, h = mask >> kColHdrOff & 1;
    off[0] = off[1] = len[1] = 0;
    if (!t && !h) {
        len[0] = total;
        return 1;
    }
    if (t) {
        len[0] = co[kColHdrType] + (uint64_t)rows * n * kColSize[kColHdrType];
        if (!h) return 1;
        off[1] = co[kColHdrOff];
        len[1] = (uint64_t)rows * n * kColSize[kColHdrOff];
        return len[1] ? 2 : 1;
    }
    len[0] = co[kColHdrOff] + (uint64_t)rows * n * kColSize[kColHdrOff];
    return 1;
}

// The gather plan (pkt_gather_plan): one piece per message, in issue order.
//   merge = 0: shard i's packed buffer lands at the next 256-B boundary of recv, its used slot rows
//              only (packed_pieces: at most two messages per shard);
//   merge = 1: recv is ONE packed output of sum(n) packets (what pkt_parse_batch over the whole
//              batch writes): each column of shard i at its rows [lo_i, lo_i + n_i), one message per
//              column and per used slot row.
// Returns the receive-buffer size.
uint64_t gather_plan(uint64_t mask, int nd, const uint64_t* n, const uint32_t* rows, int merge,
                     std::vector<pkt_gather_piece_t>& out) {
    out.clear();
    uint64_t n_total = 0;
    for (int i = 0; i < nd; i++) n_total += n[i];
    if (merge) {
        uint64_t dof[kNumCols], lo = 0;
        packed_layout(mask, n_total, dof);
        for (int i = 0; i < nd; i++) {
            const uint64_t ni = n[i];
            const uint32_t r = rows ? rows[i] : PKT_MAX_HDRS;
            if (ni) {
                uint64_t so[kNumCols];
                packed_layout(mask, ni, so);
                for (int c = 0; c < kNumCols; c++) {
                    if (!(mask >> c & 1)) continue;
                    const uint64_t esz = kColSize[c];
                    if (c == kColHdrType || c == kColHdrOff) {
                        for (uint64_t j = 0; j < r; j++)
                            out.push_back({so[c] + j * ni * esz, dof[c] + (j * n_total + lo) * esz, ni * esz, i, 0});
                    } else {
                        out.push_back({so[c], dof[c] + lo * esz, ni * esz, i, 0});
                    }
                }
            }
            lo += ni;
        }
        return packed_layout(mask, n_total, nullptr);
    }
    uint64_t o = 0, need = 0;
    for (int i = 0; i < nd; i++) {
        o = round_up(need);
        if (n[i]) {
            uint64_t po[2], pl[2];
            const int np = packed_pieces(mask, n[i], rows ? rows[i] : PKT_MAX_HDRS, po, pl);
            for (int k = 0; k < np; k++)
                if (pl[k]) out.push_back({po[k], o + po[k], pl[k], i, 0});
        }
        need = o + packed_layout(mask, n[i], nullptr);
    }
    return need;
}

}  // namespace

extern "C" {

int pkt_out_packed(uint64_t mask, uint64_t n, void* base, pkt_out_t* out, uint64_t* bytes) {
    if (mask >> kNumCols) return PKT_ERR_INVALID_ARG;
    uint64_t off[kNumCols];
    const uint64_t total = packed_layout(mask, n, off);
    if (bytes) *bytes = total;
    if (out) {
        void** cols = reinterpret_cast<void**>(out);
        for (int c = 0; c < kNumCols; c++)
            cols[c] = (base && (mask >> c & 1)) ? static_cast<uint8_t*>(base) + off[c] : nullptr;
    }
    return PKT_SUCCESS;
}

int pkt_out_packed_pieces(uint64_t mask, uint64_t n, uint32_t rows, uint64_t* off, uint64_t* len, int* npieces) {
    if (mask >> kNumCols || rows > PKT_MAX_HDRS || !off || !len || !npieces) return PKT_ERR_INVALID_ARG;
    *npieces = packed_pieces(mask, n, rows, off, len);
    return PKT_SUCCESS;
}

uint64_t pkt_out_mask(const pkt_out_t* out) {
    if (!out) return 0;
    const void* const* cols = reinterpret_cast<const void* const*>(out);
    uint64_t m = 0;
    for (int c = 0; c < kNumCols; c++)
        if (cols[c]) m |= 1ull << c;
    return m;
}

int pkt_shard_range(uint64_t n, int nshards, int i, uint64_t* lo, uint64_t* hi) {
    if (nshards <= 0 || i < 0 || i >= nshards || !lo || !hi) return PKT_ERR_INVALID_ARG;
    const uint64_t base = n / (uint64_t)nshards, extra = n % (uint64_t)nshards;
    *lo = (uint64_t)i * base + std::min<uint64_t>((uint64_t)i, extra);
    *hi = *lo + base + ((uint64_t)i < extra ? 1 : 0);
    return PKT_SUCCESS;
}

namespace {
int mgpu_create(const int* devices, int ndev, bool virt, pkt_mgpu_t** out) {
    g_create_err.clear();
    if (!out || !devices || ndev <= 0) return create_fail(PKT_ERR_INVALID_ARG, "null argument or ndev <= 0");
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0) return create_fail(PKT_ERR_NO_DEVICE, "no HIP device");
    for (int i = 0; i < ndev; i++) {
        if (devices[i] < 0 || devices[i] >= count)
            return create_fail(PKT_ERR_INVALID_ARG, "device " + std::to_string(devices[i]) + " of " +
                                                        std::to_string(count) + " visible");
        for (int j = 0; j < i && !virt; j++)
            if (devices[j] == devices[i])  // one communicator per device
                return create_fail(PKT_ERR_INVALID_ARG, "device " + std::to_string(devices[i]) + " listed twice");
    }
    pkt_mgpu* mg = new pkt_mgpu();
    mg->ndev = ndev;
    mg->virt = virt;
    mg->dev.assign(devices, devices + ndev);
    mg->ctx.assign(ndev, nullptr);
    mg->stream.assign(ndev, nullptr);
    mg->comm.assign(ndev, nullptr);
    mg->vev.assign(virt ? ndev : 0, nullptr);
    mg->rows_check.assign(ndev, nullptr);
    int rc = PKT_SUCCESS;
    std::string why;
    for (int i = 0; i < ndev && rc == PKT_SUCCESS; i++) {
        rc = pkt_ctx_create(devices[i], &mg->ctx[i]);
        if (rc != PKT_SUCCESS) {
            why = "pkt_ctx_create(" + std::to_string(devices[i]) + ") failed";
            break;
        }
        hipError_t e = hipSetDevice(devices[i]);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&mg->stream[i], hipStreamNonBlocking);
        if (e == hipSuccess && virt) e = hipEventCreateWithFlags(&mg->vev[i], hipEventDisableTiming);
        if (e != hipSuccess) {
            rc = PKT_ERR_HIP;
            why = std::string("hipStreamCreate / hipEventCreate: ") + hipGetErrorString(e);
        }
    }
    if (rc == PKT_SUCCESS && !virt) {
        ncclResult_t r = ncclCommInitAll(mg->comm.data(), ndev, mg->dev.data());
        if (r != ncclSuccess) {
            for (auto& c : mg->comm) c = nullptr;
            rc = PKT_ERR_HIP;
            why = std::string("ncclCommInitAll: ") + ncclGetErrorString(r);
        }
    }
    if (rc != PKT_SUCCESS) {
        pkt_mgpu_destroy(mg);
        return create_fail(rc, why);
    }
    *out = mg;
    return PKT_SUCCESS;
}
}  // namespace

int pkt_mgpu_create(const int* devices, int ndev, pkt_mgpu_t** out) { return mgpu_create(devices, ndev, false, out); }

int pkt_mgpu_create_virtual(const int* devices, int ndev, pkt_mgpu_t** out) {
    return mgpu_create(devices, ndev, true, out);
}

int pkt_mgpu_is_virtual(const pkt_mgpu_t* mg) { return mg && mg->virt ? 1 : 0; }

int pkt_mgpu_destroy(pkt_mgpu_t* mg) {
    if (!mg) return PKT_SUCCESS;
    for (int i = 0; i < mg->ndev; i++) {
        (void)hipSetDevice(mg->dev[i]);
        if (mg->stream[i]) (void)hipStreamSynchronize(mg->stream[i]);
        for (size_t k = i * (pkt_mgpu::kMaxStreams - 1); k < mg->xs.size() && k < (i + 1) * (pkt_mgpu::kMaxStreams - 1ull); k++)
            if (mg->xs[k]) (void)hipStreamSynchronize(mg->xs[k]);
    }
    // the root's staging area and repack table (once: a virtual handle lists the device several times)
    if (mg->stage_dev != -1) {
        (void)hipSetDevice(mg->stage_dev);
        (void)hipDeviceSynchronize();
        (void)hipFree(mg->stage);
        (void)hipFree(mg->rp_dev);
        (void)hipHostFree(mg->rp_host);
        if (mg->rp_ev) (void)hipEventDestroy(mg->rp_ev);
    }
    for (int i = 0; i < mg->ndev; i++) {
        (void)hipSetDevice(mg->dev[i]);
        for (size_t k = i * (pkt_mgpu::kMaxStreams - 1); k < mg->xs.size() && k < (i + 1) * (pkt_mgpu::kMaxStreams - 1ull); k++)
            if (mg->xs[k]) (void)hipStreamDestroy(mg->xs[k]);
        for (size_t k = i * pkt_mgpu::kMaxStreams; k < mg->xe.size() && k < (i + 1) * (size_t)pkt_mgpu::kMaxStreams; k++)
            if (mg->xe[k]) (void)hipEventDestroy(mg->xe[k]);
        if (i < (int)mg->vev.size() && mg->vev[i]) (void)hipEventDestroy(mg->vev[i]);
        if (mg->comm[i]) (void)ncclCommDestroy(mg->comm[i]);
        if (mg->stream[i]) (void)hipStreamDestroy(mg->stream[i]);
        if (mg->ctx[i]) pkt_ctx_destroy(mg->ctx[i]);
    }
    delete mg;
    return PKT_SUCCESS;
}

int pkt_mgpu_ndev(const pkt_mgpu_t* mg) { return mg ? mg->ndev : 0; }
const char* pkt_mgpu_last_error(const pkt_mgpu_t* mg) { return mg ? mg->err.c_str() : g_create_err.c_str(); }
pkt_ctx_t* pkt_mgpu_ctx(pkt_mgpu_t* mg, int i) { return (mg && i >= 0 && i < mg->ndev) ? mg->ctx[i] : nullptr; }
void* pkt_mgpu_stream(pkt_mgpu_t* mg, int i) {
    return (mg && i >= 0 && i < mg->ndev) ? reinterpret_cast<void*>(mg->stream[i]) : nullptr;
}

int pkt_mgpu_parse(pkt_mgpu_t* mg, const pkt_batch_t* batches, int entry, uint64_t mask, void* const* shard_out) {
    if (!mg || !batches || !shard_out) return mfail(mg, PKT_ERR_INVALID_ARG, "null argument");
    if (mask >> kNumCols) return mfail(mg, PKT_ERR_INVALID_ARG, "bad column mask");
    for (int i = 0; i < mg->ndev; i++) {
        if (batches[i].n && !shard_out[i]) return mfail(mg, PKT_ERR_INVALID_ARG, "null shard output");
        pkt_out_t o;
        pkt_out_packed(mask, batches[i].n, shard_out[i], &o, nullptr);
        const int rc = pkt_parse_batch(mg->ctx[i], &batches[i], entry, &o, mg->stream[i]);
        if (rc != PKT_SUCCESS)
            return mfail(mg, rc, "shard " + std::to_string(i) + ": " + pkt_ctx_last_error(mg->ctx[i]));
    }
    return PKT_SUCCESS;
}

int pkt_mgpu_parse_steps(pkt_mgpu_t* mg, const pkt_batch_t* batches, int steps, int entry, uint64_t mask,
                         void* const* shard_out, int streams) {
    if (!mg || (steps > 0 && (!batches || !shard_out))) return mfail(mg, PKT_ERR_INVALID_ARG, "null argument");
    if (steps < 0 || streams < 1 || streams > pkt_mgpu::kMaxStreams)
        return mfail(mg, PKT_ERR_INVALID_ARG, "steps < 0 or streams not in 1..4");
    if (mask >> kNumCols) return mfail(mg, PKT_ERR_INVALID_ARG, "bad column mask");
    const int nd = mg->ndev, S = streams;
    for (int k = 0; k < steps * nd; k++)
        if (batches[k].n && !shard_out[k]) return mfail(mg, PKT_ERR_INVALID_ARG, "null shard output");
    if (!mg->xinit) {  // extra streams and the join events, once (all or nothing: retried after a failure)
        mg->xs.assign((size_t)nd * (pkt_mgpu::kMaxStreams - 1), nullptr);
        mg->xe.assign((size_t)nd * pkt_mgpu::kMaxStreams, nullptr);
        hipError_t e = hipSuccess;
        for (int i = 0; i < nd && e == hipSuccess; i++) {
            e = hipSetDevice(mg->dev[i]);
            for (int j = 0; j < pkt_mgpu::kMaxStreams - 1 && e == hipSuccess; j++)
                e = hipStreamCreateWithFlags(&mg->xs[i * (pkt_mgpu::kMaxStreams - 1) + j], hipStreamNonBlocking);
            for (int j = 0; j < pkt_mgpu::kMaxStreams && e == hipSuccess; j++)
                e = hipEventCreateWithFlags(&mg->xe[i * pkt_mgpu::kMaxStreams + j], hipEventDisableTiming);
        }
        if (e != hipSuccess) {
            for (int i = 0; i < nd; i++) {
                (void)hipSetDevice(mg->dev[i]);
                for (int j = 0; j < pkt_mgpu::kMaxStreams - 1; j++) {
                    hipStream_t& x = mg->xs[i * (pkt_mgpu::kMaxStreams - 1) + j];
                    if (x) (void)hipStreamDestroy(x);
                    x = nullptr;
                }
                for (int j = 0; j < pkt_mgpu::kMaxStreams; j++) {
                    hipEvent_t& v = mg->xe[i * pkt_mgpu::kMaxStreams + j];
                    if (v) (void)hipEventDestroy(v);
                    v = nullptr;
                }
            }
            mg->xs.clear();
            mg->xe.clear();
            return mhip(mg, e, "pkt_mgpu_parse_steps streams");
        }
        mg->xinit = true;
    }
    // One host thread per device issues that device's launches (one launch per step, round-robin
    // over S streams that first wait for the device's work stream and are joined back into it), so
    // the launch rate grows with the device count instead of serialising on one thread.
    std::vector<int> rc(nd, PKT_SUCCESS);
    std::vector<std::string> why(nd);
    auto issue = [&](int i) {
        hipError_t e = hipSetDevice(mg->dev[i]);
        hipStream_t st[pkt_mgpu::kMaxStreams];
        st[0] = mg->stream[i];
        for (int j = 1; j < S; j++) st[j] = mg->xs[i * (pkt_mgpu::kMaxStreams - 1) + j - 1];
        hipEvent_t* ev = &mg->xe[i * pkt_mgpu::kMaxStreams];
        if (e == hipSuccess && S > 1) e = hipEventRecord(ev[0], st[0]);
        for (int j = 1; j < S && e == hipSuccess; j++) e = hipStreamWaitEvent(st[j], ev[0], 0);
        if (e != hipSuccess) {
            rc[i] = PKT_ERR_HIP;
            why[i] = std::string("stream setup: ") + hipGetErrorString(e);
            return;
        }
        for (int k = 0; k < steps && rc[i] == PKT_SUCCESS; k++) {
            pkt_out_t o;
            pkt_out_packed(mask, batches[k * nd + i].n, shard_out[k * nd + i], &o, nullptr);
            rc[i] = pkt_parse_batch(mg->ctx[i], &batches[k * nd + i], entry, &o, st[k % S]);
            if (rc[i] != PKT_SUCCESS) why[i] = pkt_ctx_last_error(mg->ctx[i]);
        }
        for (int j = 1; j < S; j++) {  // join (also after a failed launch: the queued ones stay ordered)
            hipError_t ej = hipEventRecord(ev[j], st[j]);
            if (ej == hipSuccess) ej = hipStreamWaitEvent(st[0], ev[j], 0);
            if (ej != hipSuccess && rc[i] == PKT_SUCCESS) {
                rc[i] = PKT_ERR_HIP;
                why[i] = std::string("stream join: ") + hipGetErrorString(ej);
            }
        }
    };
    if (nd == 1) {
        issue(0);
    } else {
        std::vector<std::thread> th;
        th.reserve(nd);
        for (int i = 0; i < nd; i++) th.emplace_back(issue, i);
        for (auto& t : th) t.join();
    }
    for (int i = 0; i < nd; i++)
        if (rc[i] != PKT_SUCCESS) return mfail(mg, rc[i], "shard " + std::to_string(i) + ": " + why[i]);
    return PKT_SUCCESS;
}

int pkt_gather_plan(uint64_t mask, int nshards, const uint64_t* n, const uint32_t* rows, int merge,
                    pkt_gather_piece_t* pieces, uint64_t cap, uint64_t* npieces, uint64_t* recv_bytes) {
    if (mask >> kNumCols || nshards <= 0 || !n || (merge != 0 && merge != 1) || (cap && !pieces))
        return PKT_ERR_INVALID_ARG;
    if (rows)
        for (int i = 0; i < nshards; i++)
            if (rows[i] > PKT_MAX_HDRS) return PKT_ERR_INVALID_ARG;
    std::vector<pkt_gather_piece_t> v;
    const uint64_t rb = gather_plan(mask, nshards, n, rows, merge, v);
    for (uint64_t k = 0; k < v.size() && k < cap; k++) pieces[k] = v[k];
    if (npieces) *npieces = v.size();
    if (recv_bytes) *recv_bytes = rb;
    return PKT_SUCCESS;
}

size_t pkt_sizeof_gather_piece(void) { return sizeof(pkt_gather_piece_t); }

int pkt_mgpu_set_root_copy(pkt_mgpu_t* mg, int enable) {
    if (!mg || enable < 0 || enable > 1) return mfail(mg, PKT_ERR_INVALID_ARG, "bad argument");
    mg->root_copy = enable;
    return PKT_SUCCESS;
}

int pkt_mgpu_set_gather_rows(pkt_mgpu_t* mg, int rows) {
    if (!mg || rows < 0 || rows > PKT_MAX_HDRS) return mfail(mg, PKT_ERR_INVALID_ARG, "bad argument");
    mg->gather_rows = rows;
    return PKT_SUCCESS;
}

}  // extern "C"

namespace {
// The virtual handle's transport (pkt_mgpu_create_virtual): the pieces issue_plan would send by RCCL, as
// device copies on the sending shard's stream.  Like a grouped ncclSend/ncclRecv, shard i's copies start
// after the work queued so far on both shard i's stream and the root's stream (the root's event), and the
// root's stream waits for them (shard i's event) before anything queued on it later.
int issue_copies(pkt_mgpu* mg, int root, const void* const* send, void* recv, const std::vector<pkt_gather_piece_t>& plan) {
    const int nd = mg->ndev;
    std::vector<char> has(nd, 0);
    for (const pkt_gather_piece_t& p : plan)
        if (p.shard != root || !mg->root_copy) has[p.shard] = 1;
    hipError_t e = hipSetDevice(mg->dev[root]);
    if (e == hipSuccess) e = hipEventRecord(mg->vev[root], mg->stream[root]);
    if (e != hipSuccess) return mhip(mg, e, "hipEventRecord (virtual gather, root)");
    for (int i = 0; i < nd; i++) {
        if (!has[i]) continue;
        const bool own = i == root;  // the root's own pieces (root copy off): on the root's stream, in order
        if ((e = hipSetDevice(mg->dev[i])) != hipSuccess) return mhip(mg, e, "hipSetDevice (virtual gather)");
        if (!own && (e = hipStreamWaitEvent(mg->stream[i], mg->vev[root], 0)) != hipSuccess)
            return mhip(mg, e, "hipStreamWaitEvent (virtual gather)");
        for (const pkt_gather_piece_t& p : plan) {
            if (p.shard != i) continue;
            e = hipMemcpyAsync(static_cast<uint8_t*>(recv) + p.dst, static_cast<const uint8_t*>(send[i]) + p.src, p.bytes,
                               hipMemcpyDefault, mg->stream[i]);
            if (e != hipSuccess) return mhip(mg, e, "hipMemcpyAsync (virtual gather)");
        }
        if (own) continue;
        if ((e = hipEventRecord(mg->vev[i], mg->stream[i])) != hipSuccess) return mhip(mg, e, "hipEventRecord (virtual gather)");
        if ((e = hipSetDevice(mg->dev[root])) != hipSuccess) return mhip(mg, e, "hipSetDevice (virtual gather)");
        if ((e = hipStreamWaitEvent(mg->stream[root], mg->vev[i], 0)) != hipSuccess)
            return mhip(mg, e, "hipStreamWaitEvent (virtual gather, root)");
    }
    return PKT_SUCCESS;
}

// Issue a gather plan: each piece from shard p.shard's buffer send[p.shard] + p.src to recv + p.dst
// on the root.  The root's own pieces are device copies on the root stream (mg->root_copy) or RCCL
// send/recv to itself; every other piece is a grouped ncclSend (the shard's stream) / ncclRecv (the
// root's stream).
int issue_plan(pkt_mgpu* mg, int root, const void* const* send, void* recv, const std::vector<pkt_gather_piece_t>& plan) {
    if (mg->root_copy) {
        hipError_t e = hipSetDevice(mg->dev[root]);
        for (const pkt_gather_piece_t& p : plan)
            if (p.shard == root && e == hipSuccess)
                e = hipMemcpyAsync(static_cast<uint8_t*>(recv) + p.dst, static_cast<const uint8_t*>(send[root]) + p.src,
                                   p.bytes, hipMemcpyDeviceToDevice, mg->stream[root]);
        if (e != hipSuccess) return mhip(mg, e, "hipMemcpyAsync (root shard)");
    }
    if (mg->virt) return issue_copies(mg, root, send, recv, plan);
    ncclResult_t r = ncclGroupStart();
    if (r != ncclSuccess) return mnccl(mg, r, "ncclGroupStart");
    for (const pkt_gather_piece_t& p : plan) {
        const int i = p.shard;
        if (i == root && mg->root_copy) continue;
        r = ncclSend(static_cast<const uint8_t*>(send[i]) + p.src, p.bytes, ncclUint8, root, mg->comm[i], mg->stream[i]);
        if (r != ncclSuccess) break;
        r = ncclRecv(static_cast<uint8_t*>(recv) + p.dst, p.bytes, ncclUint8, i, mg->comm[root], mg->stream[root]);
        if (r != ncclSuccess) break;
    }
    const ncclResult_t r2 = ncclGroupEnd();
    if (r != ncclSuccess) return mnccl(mg, r, "ncclSend/ncclRecv");
    if (r2 != ncclSuccess) return mnccl(mg, r2, "ncclGroupEnd");
    return PKT_SUCCESS;
}

// The merged gather (merge = 1): the shards' packed buffers move as in merge = 0 (<= 2 messages per
// shard, their used slot rows only) into the root's staging area, then one repack kernel on the root
// stream places each piece of `pieces` (pkt_gather_plan's merge = 1 plan: source offset in the shard's
// packed buffer, destination offset in recv) — 16 messages instead of 248 for C2 at 8 x 2^21.  With
// the root copy on, the root's own pieces are repacked straight from its shard buffer (no staging).
int merged_gather(pkt_mgpu* mg, int root, const void* const* shard_out, void* recv, const std::vector<uint64_t>& n,
                  const std::vector<uint32_t>& rows, uint64_t mask, const std::vector<pkt_gather_piece_t>& pieces) {
    const int nd = mg->ndev;
    std::vector<pkt_gather_piece_t> msgs;
    const uint64_t stage_need = gather_plan(mask, nd, n.data(), rows.data(), 0, msgs);
    // each shard's packed buffer sits at stage + its merge = 0 offset (the same loop as gather_plan)
    std::vector<uint64_t> sofs(nd, 0);
    uint64_t need = 0;
    for (int i = 0; i < nd; i++) {
        sofs[i] = round_up(need);
        need = sofs[i] + packed_layout(mask, n[i], nullptr);
    }
    hipError_t e = hipSetDevice(mg->dev[root]);
    if (e != hipSuccess) return mhip(mg, e, "hipSetDevice (root)");
    if (mg->stage_dev != -1 && mg->stage_dev != mg->dev[root]) {  // a new root device: drop the old buffers
        (void)hipSetDevice(mg->stage_dev);
        (void)hipDeviceSynchronize();
        (void)hipFree(mg->stage);
        (void)hipFree(mg->rp_dev);
        (void)hipHostFree(mg->rp_host);
        if (mg->rp_ev) (void)hipEventDestroy(mg->rp_ev);
        mg->stage = nullptr;
        mg->rp_dev = mg->rp_host = nullptr;
        mg->rp_ev = nullptr;
        mg->stage_cap = mg->rp_cap = 0;
        if ((e = hipSetDevice(mg->dev[root])) != hipSuccess) return mhip(mg, e, "hipSetDevice (root)");
    }
    mg->stage_dev = mg->dev[root];
    if (!mg->rp_ev && (e = hipEventCreateWithFlags(&mg->rp_ev, hipEventDisableTiming)) != hipSuccess)
        return mhip(mg, e, "hipEventCreate (repack)");
    const bool staged_any = std::any_of(msgs.begin(), msgs.end(),
                                        [&](const pkt_gather_piece_t& p) { return p.shard != root || !mg->root_copy; });
    if (staged_any && stage_need > mg->stage_cap) {
        if ((e = hipStreamSynchronize(mg->stream[root])) != hipSuccess) return mhip(mg, e, "hipStreamSynchronize");
        (void)hipFree(mg->stage);
        mg->stage = nullptr;
        mg->stage_cap = 0;
        if ((e = hipMalloc(reinterpret_cast<void**>(&mg->stage), stage_need)) != hipSuccess)
            return mhip(mg, e, "hipMalloc (gather staging)");
        mg->stage_cap = stage_need;
    }
    if (pieces.size() > mg->rp_cap) {
        if ((e = hipEventSynchronize(mg->rp_ev)) != hipSuccess) return mhip(mg, e, "hipEventSynchronize");
        (void)hipFree(mg->rp_dev);
        (void)hipHostFree(mg->rp_host);
        mg->rp_dev = mg->rp_host = nullptr;
        mg->rp_cap = 0;
        const uint64_t cap = pieces.size() + 64;
        e = hipMalloc(reinterpret_cast<void**>(&mg->rp_dev), cap * sizeof(RepackPiece));
        if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void**>(&mg->rp_host), cap * sizeof(RepackPiece), hipHostMallocDefault);
        if (e != hipSuccess) return mhip(mg, e, "hipMalloc (repack table)");
        mg->rp_cap = cap;
    }
    // the transfer: the merge = 0 messages into the staging area, the root's own skipped with the
    // root copy on (repacked from its shard buffer below)
    std::vector<pkt_gather_piece_t> sent;
    for (const pkt_gather_piece_t& p : msgs)
        if (p.shard != root || !mg->root_copy) sent.push_back(p);
    if (!sent.empty()) {
        const int keep = mg->root_copy;
        mg->root_copy = 0;  // issue_plan: every listed piece by RCCL (the root's own only when listed)
        const int rc = issue_plan(mg, root, shard_out, mg->stage, sent);
        mg->root_copy = keep;
        if (rc != PKT_SUCCESS) return rc;
    }
    // the repack table: absolute device addresses, block ranges in table order
    if ((e = hipEventSynchronize(mg->rp_ev)) != hipSuccess) return mhip(mg, e, "hipEventSynchronize (repack table)");
    uint32_t blocks = 0;
    uint32_t np = 0;
    for (const pkt_gather_piece_t& p : pieces) {
        if (!p.bytes) continue;
        const bool direct = p.shard == root && mg->root_copy;
        const uint8_t* src = direct ? static_cast<const uint8_t*>(shard_out[root]) + p.src : mg->stage + sofs[p.shard] + p.src;
        mg->rp_host[np++] = RepackPiece{reinterpret_cast<uint64_t>(src), reinterpret_cast<uint64_t>(recv) + p.dst, p.bytes,
                                        blocks, 0u};
        blocks += pktgpu_repack_blocks(p.bytes);
    }
    if (!np) return PKT_SUCCESS;
    hipStream_t rs = mg->stream[root];
    if ((e = hipMemcpyAsync(mg->rp_dev, mg->rp_host, np * sizeof(RepackPiece), hipMemcpyHostToDevice, rs)) != hipSuccess)
        return mhip(mg, e, "hipMemcpyAsync (repack table)");
    if ((e = hipEventRecord(mg->rp_ev, rs)) != hipSuccess) return mhip(mg, e, "hipEventRecord (repack table)");
    if ((e = pktgpu_repack_launch(mg->rp_dev, np, blocks, rs)) != hipSuccess) return mhip(mg, e, "repack_kernel");
    return PKT_SUCCESS;
}
}  // namespace

extern "C" {

int pkt_mgpu_gather(pkt_mgpu_t* mg, int root, const void* const* send, const uint64_t* bytes, void* recv,
                    uint64_t recv_len, const uint64_t* recv_off) {
    if (!mg || !send || !bytes) return mfail(mg, PKT_ERR_INVALID_ARG, "null argument");
    if (root < 0 || root >= mg->ndev) return mfail(mg, PKT_ERR_INVALID_ARG, "bad root");
    std::vector<pkt_gather_piece_t> plan;
    uint64_t o = 0;
    for (int i = 0; i < mg->ndev; i++) {
        const uint64_t off = recv_off ? recv_off[i] : o;
        o = round_up(off + bytes[i]);
        if (bytes[i] && (!send[i] || !recv)) return mfail(mg, PKT_ERR_INVALID_ARG, "null buffer");
        if (off + bytes[i] > recv_len) return mfail(mg, PKT_ERR_INVALID_ARG, "recv buffer too small");
        if (bytes[i]) plan.push_back({0, off, bytes[i], i, 0});
    }
    return issue_plan(mg, root, send, recv, plan);
}

int pkt_mgpu_parse_gather(pkt_mgpu_t* mg, const pkt_batch_t* batches, int entry, uint64_t mask,
                          void* const* shard_out, int root, void* recv, uint64_t recv_len, int merge,
                          pkt_out_t* root_views) {
    if (!mg || !batches || !shard_out) return mfail(mg, PKT_ERR_INVALID_ARG, "null argument");
    if (root < 0 || root >= mg->ndev) return mfail(mg, PKT_ERR_INVALID_ARG, "bad root");
    if (merge != 0 && merge != 1) return mfail(mg, PKT_ERR_INVALID_ARG, "bad merge flag");
    if (mask >> kNumCols) return mfail(mg, PKT_ERR_INVALID_ARG, "bad column mask");
    const int nd = mg->ndev;
    // validate the receive buffer before anything is launched or any view is filled in
    std::vector<uint64_t> n(nd);
    uint64_t n_total = 0;
    for (int i = 0; i < nd; i++) {
        n[i] = batches[i].n;
        n_total += n[i];
        if (n[i] && !shard_out[i]) return mfail(mg, PKT_ERR_INVALID_ARG, "null shard output");
    }
    std::vector<pkt_gather_piece_t> plan;
    const uint64_t need = gather_plan(mask, nd, n.data(), nullptr, merge, plan);
    if (n_total && !recv) return mfail(mg, PKT_ERR_INVALID_ARG, "null recv");
    if (need > recv_len) return mfail(mg, PKT_ERR_INVALID_ARG, "recv buffer too small");
    // Parse every shard.  Slot rows to move per shard = its largest n_hdrs (rows past it hold
    // nothing, a PacketSlice holds exactly its headers): reduced inside the parse kernel and copied
    // to pinned host memory on the shard's stream; the host waits once per device, after every
    // shard's parse is queued.
    // with a fixed row count (pkt_mgpu_set_gather_rows) the host never waits: the count is still measured
    // (same fused reduction) and pkt_mgpu_synchronize checks it against the fixed rows
    const bool has_nh = mask >> 1 & 1;
    const bool nh = has_nh && mg->gather_rows == 0;
    const bool chk = has_nh && mg->gather_rows > 0;
    std::vector<uint32_t> rows(nd, mg->gather_rows ? (uint32_t)mg->gather_rows : PKT_MAX_HDRS);
    std::vector<const uint32_t*> rows_host(nd, nullptr);
    std::fill(mg->rows_check.begin(), mg->rows_check.end(), nullptr);
    for (int i = 0; i < nd; i++) {
        if (!n[i]) continue;
        pkt_out_t o;
        pkt_out_packed(mask, n[i], shard_out[i], &o, nullptr);
        const int rc = (nh || chk) ? pktgpu_parse_rows_async(mg->ctx[i], &batches[i], entry, &o, mg->stream[i], &rows_host[i])
                                   : pkt_parse_batch(mg->ctx[i], &batches[i], entry, &o, mg->stream[i]);
        if (rc != PKT_SUCCESS)
            return mfail(mg, rc, "shard " + std::to_string(i) + ": " + pkt_ctx_last_error(mg->ctx[i]));
        if (chk) mg->rows_check[i] = rows_host[i];
    }
    if (nh) {
        for (int i = 0; i < nd; i++) {
            if (!n[i]) continue;
            hipError_t e = hipSetDevice(mg->dev[i]);
            if (e == hipSuccess) e = hipStreamSynchronize(mg->stream[i]);
            if (e != hipSuccess) return mhip(mg, e, "hipStreamSynchronize (slot rows)");
            uint32_t m = 0;
            for (int k = 0; k < MaxScratch::kSpread; k++) m = std::max(m, rows_host[i][k]);
            rows[i] = std::min<uint32_t>(m, PKT_MAX_HDRS);
        }
    }
    if (nh || mg->gather_rows) gather_plan(mask, nd, n.data(), rows.data(), merge, plan);
    if (root_views) {
        if (merge) {
            pkt_out_packed(mask, n_total, recv, &root_views[0], nullptr);
        } else {
            uint64_t o = 0, end = 0;
            for (int i = 0; i < nd; i++) {
                o = round_up(end);
                pkt_out_packed(mask, n[i], static_cast<uint8_t*>(recv) + o, &root_views[i], nullptr);
                end = o + packed_layout(mask, n[i], nullptr);
            }
        }
    }
    if (!merge) return issue_plan(mg, root, shard_out, recv, plan);
    return merged_gather(mg, root, shard_out, recv, n, rows, mask, plan);
}

int pkt_mgpu_synchronize(pkt_mgpu_t* mg) {
    if (!mg) return PKT_ERR_INVALID_ARG;
    for (int i = 0; i < mg->ndev; i++) {
        hipError_t e = hipSetDevice(mg->dev[i]);
        if (e == hipSuccess) e = hipStreamSynchronize(mg->stream[i]);
        if (e != hipSuccess) return mhip(mg, e, "hipStreamSynchronize");
    }
    // the last parse_gather with fixed slot rows: did every packet fit them?
    for (int i = 0; i < mg->ndev; i++) {
        const uint32_t* w = mg->rows_check[i];
        if (!w) continue;
        uint32_t m = 0;
        for (int k = 0; k < MaxScratch::kSpread; k++) m = std::max(m, w[k]);
        if (m > (uint32_t)mg->gather_rows) {
            std::fill(mg->rows_check.begin(), mg->rows_check.end(), nullptr);
            return mfail(mg, PKT_ERR_GATHER_ROWS,
                         "shard " + std::to_string(i) + ": a packet has " + std::to_string(m) +
                             " headers, more than the gather's fixed " + std::to_string(mg->gather_rows) +
                             " slot rows (pkt_mgpu_set_gather_rows): hdr_type / hdr_off rows past them were not gathered");
        }
    }
    std::fill(mg->rows_check.begin(), mg->rows_check.end(), nullptr);
    return PKT_SUCCESS;
}

}  // extern "C"
