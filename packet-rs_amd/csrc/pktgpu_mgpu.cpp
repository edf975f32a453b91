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

// Merged gather plan: (source offset in the shard buffer, destination offset in the root
// buffer, bytes) of each message — one per column, one per slot row for slot columns.
struct Piece {
    uint64_t src, dst, bytes;
};
void merged_pieces(uint64_t mask, uint64_t n_i, uint64_t lo, uint64_t n_total, uint32_t rows,
                   std::vector<Piece>& out) {
    uint64_t so[kNumCols], dof[kNumCols];
    packed_layout(mask, n_i, so);
    packed_layout(mask, n_total, dof);
    out.clear();
    if (n_i == 0) return;
    for (int c = 0; c < kNumCols; c++) {
        if (!(mask >> c & 1)) continue;
        const uint64_t esz = kColSize[c];
        if (c == kColHdrType || c == kColHdrOff) {
            for (uint64_t j = 0; j < rows; j++)
                out.push_back({so[c] + j * n_i * esz, dof[c] + (j * n_total + lo) * esz, n_i * esz});
        } else {
            out.push_back({so[c], dof[c] + lo * esz, n_i * esz});
        }
    }
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

int pkt_mgpu_create(const int* devices, int ndev, pkt_mgpu_t** out) {
    g_create_err.clear();
    if (!out || !devices || ndev <= 0) return create_fail(PKT_ERR_INVALID_ARG, "null argument or ndev <= 0");
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0) return create_fail(PKT_ERR_NO_DEVICE, "no HIP device");
    for (int i = 0; i < ndev; i++) {
        if (devices[i] < 0 || devices[i] >= count)
            return create_fail(PKT_ERR_INVALID_ARG, "device " + std::to_string(devices[i]) + " of " +
                                                        std::to_string(count) + " visible");
        for (int j = 0; j < i; j++)
            if (devices[j] == devices[i])  // one communicator per device
                return create_fail(PKT_ERR_INVALID_ARG, "device " + std::to_string(devices[i]) + " listed twice");
    }
    pkt_mgpu* mg = new pkt_mgpu();
    mg->ndev = ndev;
    mg->dev.assign(devices, devices + ndev);
    mg->ctx.assign(ndev, nullptr);
    mg->stream.assign(ndev, nullptr);
    mg->comm.assign(ndev, nullptr);
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
        if (e != hipSuccess) {
            rc = PKT_ERR_HIP;
            why = std::string("hipStreamCreate: ") + hipGetErrorString(e);
        }
    }
    if (rc == PKT_SUCCESS) {
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

int pkt_mgpu_destroy(pkt_mgpu_t* mg) {
    if (!mg) return PKT_SUCCESS;
    for (int i = 0; i < mg->ndev; i++) {
        (void)hipSetDevice(mg->dev[i]);
        if (mg->stream[i]) (void)hipStreamSynchronize(mg->stream[i]);
        for (size_t k = i * (pkt_mgpu::kMaxStreams - 1); k < mg->xs.size() && k < (i + 1) * (pkt_mgpu::kMaxStreams - 1ull); k++)
            if (mg->xs[k]) {
                (void)hipStreamSynchronize(mg->xs[k]);
                (void)hipStreamDestroy(mg->xs[k]);
            }
        for (size_t k = i * pkt_mgpu::kMaxStreams; k < mg->xe.size() && k < (i + 1) * (size_t)pkt_mgpu::kMaxStreams; k++)
            if (mg->xe[k]) (void)hipEventDestroy(mg->xe[k]);
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
    if (mg->xs.empty()) {  // extra streams and the join events, once
        mg->xs.assign((size_t)nd * (pkt_mgpu::kMaxStreams - 1), nullptr);
        mg->xe.assign((size_t)nd * pkt_mgpu::kMaxStreams, nullptr);
        for (int i = 0; i < nd; i++) {
            hipError_t e = hipSetDevice(mg->dev[i]);
            for (int j = 0; j < pkt_mgpu::kMaxStreams - 1 && e == hipSuccess; j++)
                e = hipStreamCreateWithFlags(&mg->xs[i * (pkt_mgpu::kMaxStreams - 1) + j], hipStreamNonBlocking);
            for (int j = 0; j < pkt_mgpu::kMaxStreams && e == hipSuccess; j++)
                e = hipEventCreateWithFlags(&mg->xe[i * pkt_mgpu::kMaxStreams + j], hipEventDisableTiming);
            if (e != hipSuccess) return mhip(mg, e, "pkt_mgpu_parse_steps streams");
        }
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

int pkt_mgpu_gather(pkt_mgpu_t* mg, int root, const void* const* send, const uint64_t* bytes, void* recv,
                    uint64_t recv_len, const uint64_t* recv_off) {
    if (!mg || !send || !bytes) return mfail(mg, PKT_ERR_INVALID_ARG, "null argument");
    if (root < 0 || root >= mg->ndev) return mfail(mg, PKT_ERR_INVALID_ARG, "bad root");
    std::vector<uint64_t> off(mg->ndev);
    uint64_t o = 0;
    for (int i = 0; i < mg->ndev; i++) {
        off[i] = recv_off ? recv_off[i] : o;
        o = round_up(off[i] + bytes[i]);
        if (bytes[i] && (!send[i] || !recv)) return mfail(mg, PKT_ERR_INVALID_ARG, "null buffer");
        if (off[i] + bytes[i] > recv_len) return mfail(mg, PKT_ERR_INVALID_ARG, "recv buffer too small");
    }
    // the root's own shard: a device copy on the root stream (an RCCL send to itself moved it at
    // ~1 TB/s, bench c5 at N = 1)
    if (bytes[root]) {
        hipError_t e = hipSetDevice(mg->dev[root]);
        if (e == hipSuccess)
            e = hipMemcpyAsync(static_cast<uint8_t*>(recv) + off[root], send[root], bytes[root], hipMemcpyDeviceToDevice,
                               mg->stream[root]);
        if (e != hipSuccess) return mhip(mg, e, "hipMemcpyAsync (root shard)");
    }
    ncclResult_t r = ncclGroupStart();
    if (r != ncclSuccess) return mnccl(mg, r, "ncclGroupStart");
    for (int i = 0; i < mg->ndev && r == ncclSuccess; i++) {
        if (!bytes[i] || i == root) continue;
        r = ncclSend(send[i], bytes[i], ncclUint8, root, mg->comm[i], mg->stream[i]);
        if (r == ncclSuccess)
            r = ncclRecv(static_cast<uint8_t*>(recv) + off[i], bytes[i], ncclUint8, i, mg->comm[root],
                         mg->stream[root]);
    }
    const ncclResult_t r2 = ncclGroupEnd();
    if (r != ncclSuccess) return mnccl(mg, r, "ncclSend/ncclRecv");
    if (r2 != ncclSuccess) return mnccl(mg, r2, "ncclGroupEnd");
    return PKT_SUCCESS;
}

int pkt_mgpu_parse_gather(pkt_mgpu_t* mg, const pkt_batch_t* batches, int entry, uint64_t mask,
                          void* const* shard_out, int root, void* recv, uint64_t recv_len, int merge,
                          pkt_out_t* root_views) {
    if (!mg || !batches || !shard_out) return mfail(mg, PKT_ERR_INVALID_ARG, "null argument");
    if (root < 0 || root >= mg->ndev) return mfail(mg, PKT_ERR_INVALID_ARG, "bad root");
    if (merge != 0 && merge != 1) return mfail(mg, PKT_ERR_INVALID_ARG, "bad merge flag");
    const int nd = mg->ndev;
    // validate the receive buffer before anything is launched or any view is filled in
    uint64_t n_total = 0, need = 0;
    for (int i = 0; i < nd; i++) {
        n_total += batches[i].n;
        need = round_up(need) + packed_layout(mask, batches[i].n, nullptr);
    }
    if (merge) need = packed_layout(mask, n_total, nullptr);
    if (n_total && !recv) return mfail(mg, PKT_ERR_INVALID_ARG, "null recv");
    if (need > recv_len) return mfail(mg, PKT_ERR_INVALID_ARG, "recv buffer too small");
    int rc = pkt_mgpu_parse(mg, batches, entry, mask, shard_out);
    if (rc != PKT_SUCCESS) return rc;
    // Slot rows to move per shard: its largest n_hdrs (rows past it hold nothing), found on the
    // device after the parse (the shards' parses all run while the host waits for the first).
    std::vector<uint32_t> rows(nd, PKT_MAX_HDRS);
    if (mask >> 1 & 1) {  // n_hdrs is among the columns
        for (int i = 0; i < nd; i++) {
            if (!batches[i].n) continue;
            pkt_out_t o;
            pkt_out_packed(mask, batches[i].n, shard_out[i], &o, nullptr);
            rc = pkt_chain_max_hdrs(mg->ctx[i], o.n_hdrs, batches[i].n, &rows[i], mg->stream[i]);
            if (rc != PKT_SUCCESS)
                return mfail(mg, rc, "shard " + std::to_string(i) + ": " + pkt_ctx_last_error(mg->ctx[i]));
        }
    }
    std::vector<Piece> pieces;
    uint64_t lo = 0, o = 0;
    if (merge && root_views) pkt_out_packed(mask, n_total, recv, &root_views[0], nullptr);
    ncclResult_t r = ncclGroupStart();
    if (r != ncclSuccess) return mnccl(mg, r, "ncclGroupStart");
    for (int i = 0; i < nd && r == ncclSuccess; i++) {
        if (merge) {
            // each column (each used slot row) of the shard at its place in the whole batch's output
            merged_pieces(mask, batches[i].n, lo, n_total, rows[i], pieces);
            lo += batches[i].n;
        } else {
            // the shard's packed buffer at the next 256-B boundary of recv, used slot rows only
            pieces.clear();
            if (root_views) pkt_out_packed(mask, batches[i].n, static_cast<uint8_t*>(recv) + o, &root_views[i], nullptr);
            uint64_t po[2], pl[2];
            const int np = packed_pieces(mask, batches[i].n, rows[i], po, pl);
            for (int k = 0; k < np; k++)
                if (pl[k] && batches[i].n) pieces.push_back({po[k], o + po[k], pl[k]});
            o = round_up(o + packed_layout(mask, batches[i].n, nullptr));
        }
        if (i == root) {  // the root's own pieces: device copies on the root stream (not RCCL)
            hipError_t e = hipSetDevice(mg->dev[root]);
            for (const Piece& p : pieces)
                if (e == hipSuccess)
                    e = hipMemcpyAsync(static_cast<uint8_t*>(recv) + p.dst, static_cast<const uint8_t*>(shard_out[i]) + p.src,
                                       p.bytes, hipMemcpyDeviceToDevice, mg->stream[root]);
            if (e != hipSuccess) {
                (void)ncclGroupEnd();
                return mhip(mg, e, "hipMemcpyAsync (root shard)");
            }
            continue;
        }
        for (const Piece& p : pieces) {
            r = ncclSend(static_cast<const uint8_t*>(shard_out[i]) + p.src, p.bytes, ncclUint8, root, mg->comm[i],
                         mg->stream[i]);
            if (r != ncclSuccess) break;
            r = ncclRecv(static_cast<uint8_t*>(recv) + p.dst, p.bytes, ncclUint8, i, mg->comm[root], mg->stream[root]);
            if (r != ncclSuccess) break;
        }
    }
    const ncclResult_t r2 = ncclGroupEnd();
    if (r != ncclSuccess) return mnccl(mg, r, "ncclSend/ncclRecv");
    if (r2 != ncclSuccess) return mnccl(mg, r2, "ncclGroupEnd");
    return PKT_SUCCESS;
}

int pkt_mgpu_synchronize(pkt_mgpu_t* mg) {
    if (!mg) return PKT_ERR_INVALID_ARG;
    for (int i = 0; i < mg->ndev; i++) {
        hipError_t e = hipSetDevice(mg->dev[i]);
        if (e == hipSuccess) e = hipStreamSynchronize(mg->stream[i]);
        if (e != hipSuccess) return mhip(mg, e, "hipStreamSynchronize");
    }
    return PKT_SUCCESS;
}

}  // extern "C"
