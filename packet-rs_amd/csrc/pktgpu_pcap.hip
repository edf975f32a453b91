// pktgpu_pcap.hip — the device pcap indexer: pkt_pcap_index_device finds
// the record boundaries of a pcap file that is already in HBM and writes the (data offset,
// incl_len) pairs an indexed batch takes (pkt_batch_t.offsets / lens), so a capture copied to the
// device as-is goes to pkt_parse_batch without a host pass over it.
//
// Format: tests/pcap.rs:7-37 (24-byte global header with LE magic d4 c3 b2 a1, then records of a
// 16-byte header {ts_sec, ts_usec, incl_len, orig_len} + incl_len bytes).  Result and error
// behaviour are pkt_pcap_index's (pktgpu_host.cpp): records are taken while 16 header bytes
// remain; a record running past the end is an error; a shorter tail is ignored.
//
// The record chain is sequential (each header says where the next one starts), so the file is cut
// into 4 KiB regions, one wave each, and the chain is recovered by speculation plus a fix-up:
//   GUESS   a block stages 4 consecutive regions (16 KiB + 16 B) in LDS; each wave finds the
//           first offset of its region from which a chain of plausible record headers runs (64
//           offsets per step, one per lane; hops past the staged block read global memory), walks
//           the records from there and keeps (entry, exit, count, error) and the records' offsets
//           in the region (u16 list).  Region 0's entry is 24, by definition.
//   REPAIR  one thread per region compares its entry with the exit of the nearest non-empty
//           region to its left.  A region that disagrees while that neighbour agrees with its own
//           left is queued; the block's waves re-walk each queued region from that exit and chase
//           on into the following regions until an exit meets the next region's stored entry.
//           Every region left of the first disagreement is exact (region 0 is, and each agrees
//           with an exact left), so the first queued chase is exact and no round ends without
//           fixing at least that region; a round in which no region disagrees is the exact fixed
//           point — the true chain, whatever the guesses were.  A chase claims each region before
//           rewriting it (atomicMax of the round id on the region's owner word) and stops at a
//           region another chase already claimed this round, so a region's entry, exit, count,
//           error and list always come from ONE walk; the first queued chase cannot be stopped
//           (chases only move right and start at queued regions), which keeps the progress bound.
//   SCAN    exclusive prefix of the per-region counts (per 1024 regions; the last block to finish
//           scans the block totals).
//   EMIT    256 threads write 16 regions' records at their prefix: offset = pos + 16, incl_len =
//           next pos - pos - 16 (the last one from the region's exit); the file is not re-read.
// HBM traffic ≈ the file once + 2 B/record (the list) written and read + 12 B/record of output.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "pktgpu_ctx.hpp"

namespace {

#ifndef PKTGPU_PCAP_REGION
#define PKTGPU_PCAP_REGION 4096
#endif
constexpr uint32_t kRegion = PKTGPU_PCAP_REGION;  // bytes of record starts per region
static_assert(kRegion % 16 == 0 && kRegion / 16 <= 65536, "u16 record lists");
constexpr uint32_t kMaxRec = kRegion / 16;       // records per region (each >= 16 B apart)
constexpr int kWaves = 4;                         // waves per 256-thread block
constexpr uint32_t kBlockBytes = kWaves * kRegion;
constexpr uint32_t kScanBlock = 1024;             // regions per first-level scan block
constexpr uint32_t kEmitRegions = 16;             // regions per emit block
constexpr int kLookback = 64;                     // empty regions skipped when finding an entry
constexpr int kChaseMax = 256;                    // regions one repair chase may rewrite
#ifndef PKTGPU_PCAP_HOPS
#define PKTGPU_PCAP_HOPS 2, 2  // (min, max); 3, 4: 117 us per call, 2, 3: 112, 2, 2: 108 (profiles/ab/r02hops_*)
#endif
constexpr int kHops[2] = {PKTGPU_PCAP_HOPS};
constexpr int kMinHops = kHops[0], kMaxHops = kHops[1];  // guess chain length
constexpr uint32_t kTsSpan = 86400;               // guess: consecutive ts_sec within a day
constexpr uint32_t kPassSlots = 64;               // passes with their own control words
// Repair rounds per pass: 2.  With 1, the C4 capture's first pass always still finds a guess to fix
// and needs a second pass (one more read-back): 141 vs 111 us per call (round 3, same box).
constexpr uint32_t kRounds = 2;

// Control words (device, zeroed once per call): [0] magic is d4 c3 b2 a1; then per pass p (slot
// p % 64): [8 + 8s + 2r] regions that disagreed in round r, [9 + 8s + 2r] K - first such region
// (max; 0 = none), [12 + 8s] a region's walk hit a record running past the end, [13 + 8s] the
// record total, [14 + 8s] the scan's block ticket.
constexpr uint32_t kCtlWords = 8 + 8 * kPassSlots;

struct Scratch {
    uint64_t* entry;   // first record start >= region start (may lie past the region)
    uint64_t* exit;    // first record start >= region end, as walked from entry
    uint32_t* cnt;     // records starting in the region
    uint32_t* err;     // the walk met a record running past the end of the file
    uint32_t* pre;     // exclusive prefix of cnt within its scan block
    uint64_t* bpre;    // exclusive prefix of the scan blocks
    uint16_t* list;    // [region][kMaxRec] record offsets relative to the region base
    uint32_t* own;     // the last repair round whose chase rewrote the region (0 = none)
    uint64_t* ctl;     // control words above
};

__device__ __forceinline__ uint32_t lane_id() {
    return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}

// Order a wave's LDS writes before its other lanes' reads (no block barrier).
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint32_t ld32(const uint32_t* lw, uint32_t o) {
    // Little-endian u32 at any byte offset of the staged bytes (two dwords + v_alignbyte).
    return __builtin_amdgcn_alignbyte(lw[(o >> 2) + 1], lw[o >> 2], o & 3);
}

// A record header a real capture could hold: microseconds < 1e6, 0 < incl_len <= snaplen,
// incl_len <= orig_len <= 1 MiB, and the record ends inside the file.  Only a heuristic for the
// guess; the repair rounds make the result exact whatever it accepts.
struct RecHdr {
    uint32_t sec, usec, incl, orig;
};

__device__ __forceinline__ bool plausible(const RecHdr& h, uint64_t pos, uint64_t len, uint32_t snap) {
    return h.usec < 1000000u && h.incl != 0 && h.incl <= snap && h.incl <= h.orig && h.orig <= (1u << 20) &&
           pos + 16 + h.incl <= len;
}

__device__ __forceinline__ RecHdr hdr_lds(const uint32_t* lw, uint32_t o) {
    // five dwords in one go (ds_read2 x3, one wait), then v_alignbyte
    const uint32_t* q = lw + (o >> 2);
    const uint32_t sh = o & 3, d0 = q[0], d1 = q[1], d2 = q[2], d3 = q[3], d4 = q[4];
    return RecHdr{__builtin_amdgcn_alignbyte(d1, d0, sh), __builtin_amdgcn_alignbyte(d2, d1, sh),
                  __builtin_amdgcn_alignbyte(d3, d2, sh), __builtin_amdgcn_alignbyte(d4, d3, sh)};
}

// The same header read from global memory (past the staged bytes): aligned dwords below `len`
// only, then v_alignbyte.
__device__ __forceinline__ RecHdr hdr_global(const uint8_t* buf, uint64_t pos, uint64_t len) {
    const uint64_t a = pos & ~3ull;
    const uint32_t sh = (uint32_t)(pos & 3);
    uint32_t d[5];
#pragma unroll
    for (int i = 0; i < 5; i++) d[i] = a + 4 * i < len ? *reinterpret_cast<const uint32_t*>(buf + a + 4 * i) : 0u;
    return RecHdr{__builtin_amdgcn_alignbyte(d[1], d[0], sh), __builtin_amdgcn_alignbyte(d[2], d[1], sh),
                  __builtin_amdgcn_alignbyte(d[3], d[2], sh), __builtin_amdgcn_alignbyte(d[4], d[3], sh)};
}

// A guess candidate: plausible headers chained from `c` to the end of the region (at most
// kMaxHops checked) and at least kMinHops of them unless the file ends first; consecutive ts_sec
// within a day.  chain_local checks the hops inside the staged bytes with 32-bit offsets from
// LDS byte 0 (`lim` = file bytes from there, clamped to 32 bits) and returns 2 at the first hop
// past them ("needs global reads"); chain_global re-checks such a candidate reading those hops
// from global memory.  1 = plausible chain, 0 = not.
__device__ __forceinline__ bool plausible32(const RecHdr& h, uint32_t p, uint32_t lim, uint32_t snap) {
    // incl <= orig <= 1 MiB keeps p + 16 + incl far below 2^32 (p < 2^22 on every hop)
    // non-short-circuit: no branch between the loads and the verdict
    return (h.usec < 1000000u) & (h.incl != 0) & (h.incl <= snap) & (h.incl <= h.orig) & (h.orig <= (1u << 20)) &
           (p + 16 + h.incl <= lim);
}

__device__ __forceinline__ int chain_local(const uint32_t* lw, uint32_t c, uint32_t stop, uint32_t lend, uint32_t lim,
                                           uint32_t snap) {
    uint32_t p = c, prev = 0;
    for (int hops = 0; (p < stop || hops < kMinHops) && hops < kMaxHops; hops++) {
        if (p + 16 > lim) return 1;
        if (p >= lend) return 2;
        const RecHdr h = hdr_lds(lw, p);
        if (!plausible32(h, p, lim, snap) | ((hops != 0) & (h.sec - prev + kTsSpan > 2 * kTsSpan))) return 0;
        prev = h.sec;
        p += 16 + h.incl;
    }
    return 1;
}

__device__ __forceinline__ bool chain_global(const uint32_t* lw, const uint8_t* buf, uint64_t lbase, uint64_t lend,
                                             uint64_t c, uint64_t stop, uint64_t len, uint32_t snap) {
    uint64_t p = c;
    uint32_t prev = 0;
    for (int hops = 0; (p < stop || hops < kMinHops) && hops < kMaxHops; hops++) {
        if (p + 16 > len) return true;
        const RecHdr h = p < lend ? hdr_lds(lw, (uint32_t)(p - lbase)) : hdr_global(buf, p, len);
        if (!plausible(h, p, len, snap)) return false;
        if (hops && h.sec - prev + kTsSpan > 2 * kTsSpan) return false;
        prev = h.sec;
        p += 16 + (uint64_t)h.incl;
    }
    return true;
}

// The nearest region left of k that claims a record start (entry inside it), or region 0.
__device__ __forceinline__ uint32_t left_of(const Scratch& S, uint32_t k) {
    uint32_t j = k - 1;
    for (int s = 0; s < kLookback && j > 0 && S.entry[j] >= (uint64_t)(j + 1) * kRegion; s++) j--;
    return j;
}

// Stage file bytes [base, base + BYTES + 16) into LDS, zeros past the file's 16-byte-rounded end,
// plus 16 zero bytes of pad; NT threads, this one is `t`.  All loads are issued before the first
// LDS write (one memory latency per stage, not one per piece).
template <uint32_t BYTES, uint32_t NT>
__device__ __forceinline__ void stage(uint4* l4, const uint8_t* buf, uint64_t base, uint64_t len, uint32_t t) {
    constexpr uint32_t kPieces = BYTES / 16 + 2, kPer = (kPieces + NT - 1) / NT;
    uint4 v[kPer];
#pragma unroll
    for (uint32_t i = 0; i < kPer; i++) {
        const uint32_t q = t + i * NT;
        const uint64_t a = base + 16ull * q;
        v[i] = make_uint4(0, 0, 0, 0);
        if (q <= BYTES / 16 && a < len) v[i] = *reinterpret_cast<const uint4*>(buf + a);
    }
#pragma unroll
    for (uint32_t i = 0; i < kPer; i++)
        if (t + i * NT < kPieces) l4[t + i * NT] = v[i];
}

// Walk the records from `entry` while they start inside the region [base, base + kRegion) and
// 16 header bytes remain: pkt_pcap_index's loop restated per region.  Record i's offset in the
// region is kept by lane i in `rec` (a select per record, no branch, no LDS write); records 64..
// (regions of short records) go to `list` from lane 0.  The position lives in an SGPR
// (readfirstlane of each LDS read), so the loop's bounds checks are SALU compares and its branches
// uniform (round 3: guess kernel + 2 repair rounds + scan + emit 111-114 -> 101-102 us per
// 2^20-record call; the round-1 SGPR walk kept 64-bit positions and measured slower), with 32-bit
// offsets from lbase while the file's end is < 4 GiB past it; otherwise the 64-bit vector form.
__device__ __forceinline__ void walk(const uint32_t* lw, uint64_t lbase, uint16_t* list, uint64_t base,
                                     uint64_t entry, uint64_t len, uint64_t& exit, uint32_t& cnt, uint32_t& err,
                                     uint32_t& rec) {
    if (len - lbase <= 0xFFFFFFF0ull) {
        const uint32_t lane = lane_id();
        const uint32_t rb = (uint32_t)(base - lbase), rend = rb + kRegion, rlen = (uint32_t)(len - lbase);
        uint32_t p = __builtin_amdgcn_readfirstlane((uint32_t)(entry - lbase));
        uint32_t c = 0, e = 0, rv = 0;
        while (p < rend && p + 16 <= rlen) {
            const uint32_t incl = __builtin_amdgcn_readfirstlane(ld32(lw, p + 8));
            if (incl > rlen - p - 16) {  // pkt_pcap_index: record runs past the end
                e = 1;
                p = rlen;
                break;
            }
            rv = lane == c ? p - rb : rv;
            if (c >= 64u && lane == 0) list[c] = (uint16_t)(p - rb);
            c++;
            p += 16 + incl;
        }
        exit = lbase + p;
        cnt = c;
        err = e;
        rec = rv;
        return;
    }
    uint64_t pos = entry;
    cnt = 0;
    err = 0;
    rec = 0;
    const uint64_t end = base + kRegion;
    const uint32_t lane = lane_id();
    while (pos < end && pos + 16 <= len) {
        const uint32_t incl = ld32(lw, (uint32_t)(pos - lbase) + 8);
        if (pos + 16 + (uint64_t)incl > len) {  // pkt_pcap_index: record runs past the end
            err = 1;
            pos = len;
            break;
        }
        const uint32_t ro = (uint32_t)(pos - base);
        rec = lane == cnt ? ro : rec;
        if (__builtin_amdgcn_readfirstlane(cnt) >= 64u && lane == 0) list[cnt] = (uint16_t)ro;
        cnt++;
        pos += 16 + (uint64_t)incl;
    }
    exit = pos;
}

// Write a walked region back: the record offsets (lane i's register for record i < 64, the LDS
// list beyond) and the region's words.
__device__ __forceinline__ void store_region(const Scratch& S, uint32_t k, const uint16_t* list, uint32_t rec,
                                             uint64_t entry, uint64_t exit, uint32_t cnt, uint32_t err) {
    const uint32_t lane = lane_id();
    uint16_t* dst = S.list + (uint64_t)k * kMaxRec;
    if (lane < cnt) dst[lane] = (uint16_t)rec;
    for (uint32_t i = 64 + lane; i < cnt; i += 64) dst[i] = list[i];
    if (lane == 0) {
        S.entry[k] = entry;
        S.exit[k] = exit;
        S.cnt[k] = cnt;
        S.err[k] = err;
    }
}

// Diagnostic build only (-DPKTGPU_STAMPS=1): s_memtime stamps per guess wave — start, staged,
// entry found, walked, stored — to a debug buffer no other code reads (pkt_debug_pcap_stamps).
#ifndef PKTGPU_STAMPS
#define PKTGPU_STAMPS 0
#endif
#if PKTGPU_STAMPS
__device__ uint64_t* g_pcap_stamps;
#define PCAP_STAMP(k)                                                                         \
    do {                                                                                      \
        __builtin_amdgcn_sched_barrier(0);                                                    \
        uint64_t t_;                                                                          \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");            \
        __builtin_amdgcn_sched_barrier(0);                                                    \
        pst[k] = t_;                                                                          \
    } while (0)
#else
#define PCAP_STAMP(k) \
    do {              \
    } while (0)
#endif

// One region's guess (wave w of the block whose 4 regions are staged at lbase): its entry by the
// candidate scan, then its walk, stored to the region's words and list.
__device__ __forceinline__ void guess_region(const uint8_t* __restrict__ buf, uint64_t len, uint32_t K, const Scratch& S,
                                             const uint32_t* lw, uint16_t* list, uint64_t lbase, uint32_t k,
                                             uint64_t* pst) {
    (void)pst;
    const uint32_t lane = lane_id();
    const uint64_t lend = lbase + kBlockBytes;
    if (lane == 0) S.own[k] = 0;
    const uint64_t base = (uint64_t)k * kRegion;
    uint64_t entry = 24;
    if (k == 0) {
        if (lane == 0) S.ctl[0] = buf[0] == 0xD4 && buf[1] == 0xC3 && buf[2] == 0xB2 && buf[3] == 0xA1;
    } else {
        // snaplen (global header bytes 16..19) bounds a plausible incl_len
        uint32_t snap = *reinterpret_cast<const uint32_t*>(buf + 16);
        if (snap == 0 || snap > (1u << 30)) snap = 1u << 30;
        const uint64_t stop = len < base + kRegion ? len : base + kRegion;
        const uint32_t lim = len - lbase > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)(len - lbase);
        entry = base + kRegion;  // none found: guess "no record starts here"
        for (uint64_t c0 = base; c0 < stop; c0 += 64) {
            // The lowest candidate whose chain checks out inside the staged bytes wins; only when
            // there is none do the candidates whose chains leave them read global memory.
            const uint64_t c = c0 + lane;
            const int r = c < stop && c + 16 <= len
                              ? chain_local(lw, (uint32_t)(c - lbase), (uint32_t)(stop - lbase), kBlockBytes, lim, snap)
                              : 0;
            uint64_t m = __ballot(r == 1);
            if (!m) m = __ballot(r == 2 && chain_global(lw, buf, lbase, lend, c, stop, len, snap));
            if (m) {
                entry = c0 + (uint64_t)__builtin_ctzll(m);
                break;
            }
        }
    }
    PCAP_STAMP(2);
    uint64_t exit;
    uint32_t cnt, err, rec;
    walk(lw, lbase, list, base, entry, len, exit, cnt, err, rec);
    wave_lds_sync();
    PCAP_STAMP(3);
    store_region(S, k, list, rec, entry, exit, cnt, err);
#if PKTGPU_STAMPS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    PCAP_STAMP(4);
    if (lane == 0 && g_pcap_stamps) {
        uint32_t xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        for (int q = 0; q < 5; q++) g_pcap_stamps[(uint64_t)k * 8 + q] = pst[q];
        g_pcap_stamps[(uint64_t)k * 8 + 6] = xcc & 15u;  // s_memtime counts per XCD
    }
#endif
}

// One block stages 4 consecutive regions (16 KiB + 16 B) and each wave guesses one of them.  (A
// persistent form, each block looping over its tiles with the next tile's 16 KiB loaded into
// registers during the current tile's walks, measured slower: 83 vs 61 us per C4 call — the
// hardware already overlaps new blocks' staging with resident blocks' walks, round 3.)
__global__ __launch_bounds__(256) void pcap_guess_kernel(const uint8_t* __restrict__ buf, uint64_t len,
                                                         uint32_t K, Scratch S) {
    uint64_t pst[5] = {0, 0, 0, 0, 0};
    (void)pst;
    PCAP_STAMP(0);
    __shared__ uint4 lds[kBlockBytes / 16 + 2];
    __shared__ uint16_t lst[kWaves][kMaxRec];
    const uint32_t w = threadIdx.x / 64;
    const uint32_t k = blockIdx.x * kWaves + w;
    const uint64_t lbase = (uint64_t)blockIdx.x * kBlockBytes;
    stage<kBlockBytes, 256>(lds, buf, lbase, len, threadIdx.x);
    // the per-call zeroing the repair rounds rely on (no memset launches): control words 1.. here,
    // word 0 (the magic) and each region's owner word in guess_region
    if (blockIdx.x == 0)
        for (uint32_t c = 1 + threadIdx.x; c < kCtlWords; c += 256) S.ctl[c] = 0;
    __syncthreads();
    PCAP_STAMP(1);
    if (k < K) guess_region(buf, len, K, S, reinterpret_cast<const uint32_t*>(lds), lst[w], lbase, k, pst);
}

// One repair round (see the file header).  `slot` = this round's two control words.
__global__ __launch_bounds__(256) void pcap_repair_kernel(const uint8_t* __restrict__ buf, uint64_t len,
                                                          uint32_t K, Scratch S, uint32_t slot, uint32_t round) {
    __shared__ uint4 lds[kWaves][kRegion / 16 + 2];
    __shared__ uint16_t lst[kWaves][kMaxRec];
    __shared__ uint32_t qk[256];
    __shared__ uint64_t qe[256];
    __shared__ uint32_t qn;
    const uint32_t t = threadIdx.x, w = t / 64;
    if (t == 0) qn = 0;
    __syncthreads();
    const uint32_t k = blockIdx.x * 256 + t;
    if (k > 0 && k < K) {
        const uint32_t j = left_of(S, k);
        const uint64_t e = S.exit[j];
        if (e != S.entry[k]) {
            atomicAdd(reinterpret_cast<unsigned long long*>(&S.ctl[slot]), 1ull);
            atomicMax(reinterpret_cast<unsigned long long*>(&S.ctl[slot + 1]), (unsigned long long)(K - k));
            if ((j == 0 || S.exit[left_of(S, j)] == S.entry[j]) && e >= (uint64_t)k * kRegion) {
                const uint32_t q = atomicAdd(&qn, 1u);
                qk[q] = k;
                qe[q] = e;
            }
        }
    }
    __syncthreads();
    const uint32_t n = qn;
    const uint32_t* lw = reinterpret_cast<const uint32_t*>(lds[w]);
    for (uint32_t i = w; i < n; i += kWaves) {
        uint32_t r = qk[i];
        uint64_t e = qe[i];
        for (int step = 0; step < kChaseMax; step++) {
            // claim region r for this round; a region another chase claimed first is its alone
            uint32_t prev = 0;
            if (lane_id() == 0) prev = atomicMax(&S.own[r], round);
            if (__shfl(prev, 0, 64) >= round) break;
            const uint64_t base = (uint64_t)r * kRegion;
            wave_lds_sync();
            if (e < base + kRegion) stage<kRegion, 64>(lds[w], buf, base, len, lane_id());
            wave_lds_sync();
            uint64_t exit;
            uint32_t cnt, err, rec;
            walk(lw, base, lst[w], base, e, len, exit, cnt, err, rec);
            wave_lds_sync();
            store_region(S, r, lst[w], rec, e, exit, cnt, err);
            e = exit;
            if (++r >= K || e == S.entry[r] || e < (uint64_t)r * kRegion) break;
        }
    }
}

// Exclusive prefix of cnt within each block of kScanBlock regions (256 threads x 4), the block
// totals to bpre, and the OR of the regions' error flags.  The last block to finish (ticket in
// ctl[slot + 2]) then scans the block totals in place and writes the record total to
// ctl[slot + 1]; ctl[slot] collects the error flags.
__global__ __launch_bounds__(256) void pcap_scan_kernel(uint32_t K, uint32_t nb, Scratch S, uint32_t slot,
                                                        uint32_t pass_slot, uint64_t* host_ctl) {
    __shared__ uint64_t wsum[4];
    __shared__ uint64_t carry;
    __shared__ uint32_t last;
    const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
    const uint32_t k0 = blockIdx.x * kScanBlock + t * 4;
    uint32_t c[4], e = 0, s = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        c[i] = k0 + i < K ? S.cnt[k0 + i] : 0;
        e |= k0 + i < K ? S.err[k0 + i] : 0;
        s += c[i];
    }
    if (__ballot(e != 0) && lane == 0) atomicOr(reinterpret_cast<unsigned long long*>(&S.ctl[slot]), 1ull);
    uint32_t x = s;  // inclusive wave scan
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= (uint32_t)d) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    uint32_t wbase = 0;
    for (uint32_t i = 0; i < w; i++) wbase += (uint32_t)wsum[i];
    uint32_t run = wbase + x - s;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        if (k0 + i < K) S.pre[k0 + i] = run;
        run += c[i];
    }
    if (t == 255) S.bpre[blockIdx.x] = (uint64_t)wbase + x;
    __threadfence();
    __syncthreads();
    if (t == 0) last = atomicAdd(reinterpret_cast<unsigned long long*>(&S.ctl[slot + 2]), 1ull) == nb - 1;
    __syncthreads();
    if (!last) return;
    // Last block: exclusive scan of the block totals (read past L1: other blocks wrote them).
    __threadfence();
    if (t == 0) carry = 0;
    __syncthreads();
    for (uint32_t b0 = 0; b0 < nb; b0 += 256) {
        const uint32_t b = b0 + t;
        const uint64_t v = b < nb ? __hip_atomic_load(&S.bpre[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
        uint64_t y = v;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint64_t z = __shfl_up(y, d, 64);
            if (lane >= (uint32_t)d) y += z;
        }
        __syncthreads();
        if (lane == 63) wsum[w] = y;
        __syncthreads();
        uint64_t wb = carry;
        for (uint32_t i = 0; i < w; i++) wb += wsum[i];
        if (b < nb) S.bpre[b] = wb + y - v;
        __syncthreads();
        if (t == 255) carry = wb + y;
        __syncthreads();
    }
    if (t == 0) S.ctl[slot + 1] = carry;
    // The pass's verdict to the host's pinned words directly (no copy launch): the magic word and
    // the pass's 8 control words (the repair rounds' counts, this kernel's error flag and total).
    __syncthreads();
    if (t < 9) {
        const uint32_t wi = t == 0 ? 0u : pass_slot + t - 1;
        const uint64_t v = wi == slot + 1 ? carry : __hip_atomic_load(&S.ctl[wi], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&host_ctl[wi], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// 256 threads write the records of kEmitRegions consecutive regions, one record per thread per
// step, contiguous in the output (coalesced), at the regions' scanned prefix.
__global__ __launch_bounds__(256) void pcap_emit_kernel(uint32_t K, uint64_t cap, Scratch S,
                                                        uint64_t* __restrict__ offsets,
                                                        uint32_t* __restrict__ lens) {
    __shared__ uint32_t cpre[kEmitRegions + 1];
    const uint32_t k0 = blockIdx.x * kEmitRegions, t = threadIdx.x;
    if (t < 64) {  // the 16 counts in parallel, prefix by a lane scan
        const uint32_t c = t < kEmitRegions && k0 + t < K ? S.cnt[k0 + t] : 0;
        uint32_t x = c;
#pragma unroll
        for (uint32_t d = 1; d < kEmitRegions; d <<= 1) {
            const uint32_t y = __shfl_up(x, d, 64);
            if (t >= d) x += y;
        }
        if (t < kEmitRegions) cpre[t] = x - c;
        if (t == kEmitRegions - 1) cpre[kEmitRegions] = x;
    }
    __syncthreads();
    const uint64_t first = (uint64_t)S.pre[k0] + S.bpre[k0 / kScanBlock];
    const uint32_t total = cpre[kEmitRegions];
    for (uint32_t i = t; i < total; i += 256) {
        const uint64_t idx = first + i;
        if (idx >= cap) break;
        uint32_t r = 0;
#pragma unroll
        for (uint32_t b = kEmitRegions / 2; b; b >>= 1)
            if (cpre[r + b] <= i) r += b;
        const uint32_t k = k0 + r, li = i - cpre[r], c = cpre[r + 1] - cpre[r];
        const uint64_t base = (uint64_t)k * kRegion;
        const uint16_t* list = S.list + (uint64_t)k * kMaxRec;
        const uint64_t pos = base + list[li];
        const uint64_t next = li + 1 < c ? base + list[li + 1] : S.exit[k];
        offsets[idx] = pos + 16;
        lens[idx] = (uint32_t)(next - pos - 16);
    }
}

}  // namespace

extern "C" {
#if PKTGPU_STAMPS
// Diagnostic build only: where pcap_guess_kernel writes its per-wave stamps (8 u64 per region).
int pkt_debug_pcap_stamps(void* dev_buf) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_pcap_stamps), &dev_buf, sizeof(dev_buf)) == hipSuccess ? PKT_SUCCESS
                                                                                            : PKT_ERR_HIP;
}
#endif

int pkt_pcap_index_device(pkt_ctx_t* ctx, const uint8_t* buf, uint64_t len, uint64_t* offsets, uint32_t* lens,
                          uint64_t cap, uint64_t* n_out, void* stream) {
    if (!ctx || !buf || !n_out || (cap && (!offsets || !lens))) return fail(ctx, PKT_ERR_INVALID_ARG, "bad argument");
    *n_out = 0;
    if (len < 24) return fail(ctx, PKT_ERR_INVALID_ARG, "pcap shorter than its global header");
    if (reinterpret_cast<uintptr_t>(buf) & 15) return fail(ctx, PKT_ERR_INVALID_ARG, "pcap buffer not 16-byte aligned");
    const uint64_t K64 = (len + kRegion - 1) / kRegion;
    if (K64 > (1ull << 31)) return fail(ctx, PKT_ERR_INVALID_ARG, "pcap too large");
    const uint32_t K = (uint32_t)K64, nb = (K + kScanBlock - 1) / kScanBlock;
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail(ctx, e, "hipSetDevice");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);

    // Scratch: the control words, per-region words and record lists, the scan-block prefixes.
    const uint64_t need = 8ull * kCtlWords + (uint64_t)K * (8 + 8 + 4 + 4 + 4 + 4 + 2 * kMaxRec) + 8ull * nb + 64;
    PcapScratch& pc = ctx->pc;
    if (pc.bytes < need) {
        if (pc.buf) {
            (void)hipStreamSynchronize(s);
            (void)hipFree(pc.buf);
            pc.buf = nullptr;
            pc.bytes = 0;
        }
        e = hipMalloc(&pc.buf, need + need / 4);
        if (e != hipSuccess) return hip_fail(ctx, e, "hipMalloc (pcap index)");
        pc.bytes = need + need / 4;
    }
    if (!pc.ctl) {
        e = hipHostMalloc(reinterpret_cast<void**>(&pc.ctl), 8 * kCtlWords, hipHostMallocMapped);
        if (e == hipSuccess) e = hipHostGetDevicePointer(reinterpret_cast<void**>(&pc.ctl_dev), pc.ctl, 0);
        if (e != hipSuccess) return hip_fail(ctx, e, "hipHostMalloc (pcap index)");
    }
    Scratch S;
    char* p = static_cast<char*>(pc.buf);
    S.ctl = reinterpret_cast<uint64_t*>(p);
    p += 8ull * kCtlWords;
    S.entry = reinterpret_cast<uint64_t*>(p);
    p += 8ull * K;
    S.exit = reinterpret_cast<uint64_t*>(p);
    p += 8ull * K;
    S.bpre = reinterpret_cast<uint64_t*>(p);
    p += 8ull * nb;
    S.cnt = reinterpret_cast<uint32_t*>(p);
    p += 4ull * K;
    S.err = reinterpret_cast<uint32_t*>(p);
    p += 4ull * K;
    S.pre = reinterpret_cast<uint32_t*>(p);
    p += 4ull * K;
    S.own = reinterpret_cast<uint32_t*>(p);
    p += 4ull * K;
    S.list = reinterpret_cast<uint16_t*>(p);

    const dim3 blk(256);
    // (the guess kernel zeroes the control words and the owner words)
    hipLaunchKernelGGL(pcap_guess_kernel, dim3((K + kWaves - 1) / kWaves), blk, 0, s, buf, len, K, S);
    if ((e = hipGetLastError()) != hipSuccess) return hip_fail(ctx, e, "pcap guess launch");
    // Each pass: two repair rounds, then the scan and the emit on speculation, and ONE read-back.
    // When the second round found no region disagreeing, the state it saw was the fixed point and
    // the emitted index is final; otherwise the pass repeats (every round fixes at least the
    // first wrong region, so K passes always suffice).
    for (uint32_t pass = 0;; pass++) {
        if (pass > K) return fail(ctx, PKT_ERR_INVALID_ARG, "pcap index did not converge");
        const uint32_t slot = 8 + 8 * (pass % kPassSlots);
        if (pass && pass % kPassSlots == 0) {
            e = hipMemsetAsync(S.ctl + 8, 0, 8ull * (kCtlWords - 8), s);
            if (e != hipSuccess) return hip_fail(ctx, e, "hipMemset (pcap index)");
        }
        for (uint32_t r = 0; r < kRounds; r++)  // round ids 1, 2, 3, ... (owner words start at 0)
            hipLaunchKernelGGL(pcap_repair_kernel, dim3((K + 255) / 256), blk, 0, s, buf, len, K, S, slot + 2 * r,
                               kRounds * pass + r + 1);
        hipLaunchKernelGGL(pcap_scan_kernel, dim3(nb), blk, 0, s, K, nb, S, slot + 4, slot, pc.ctl_dev);
        if (cap)
            hipLaunchKernelGGL(pcap_emit_kernel, dim3((K + kEmitRegions - 1) / kEmitRegions), blk, 0, s, K, cap,
                               S, offsets, lens);
        if ((e = hipGetLastError()) != hipSuccess) return hip_fail(ctx, e, "pcap index launch");
        e = hipStreamSynchronize(s);
        if (e != hipSuccess) return hip_fail(ctx, e, "pcap index");
        if (!pc.ctl[0]) return fail(ctx, PKT_ERR_INVALID_ARG, "bad pcap magic");
        if (pc.ctl[slot + 2 * (kRounds - 1)] == 0) {
            if (pc.ctl[slot + 4]) return fail(ctx, PKT_ERR_INVALID_ARG, "pcap record runs past the end of the buffer");
            *n_out = pc.ctl[slot + 5];
            return PKT_SUCCESS;
        }
    }
}

}  // extern "C"
