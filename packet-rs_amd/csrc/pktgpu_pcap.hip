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
// The record chain is sequential (each header says where the next one starts): speculation per
// 4 KiB region, then an exact pass over the regions' states, then the output.  Three kernels, one
// host read-back (or none: pkt_parse_pcap's parse takes the count on the device):
//   GUESS (pcap_guess_kernel)  a block stages 4 consecutive regions (16 KiB) in LDS; each wave
//            finds the first offset of its region from which a chain of plausible record headers
//            runs (64 candidates per step, one per lane) — or "none" — and four lanes of wave 0 then
//            walk the block's four regions from their entries: per region entry, exit, count (+ error
//            bit) and the records' u16 offsets.  Region 0's entry is 24 by definition.  No block
//            waits for another.
//   SCAN (pcap_scan_kernel)  a block takes the next 256 regions (a ticket, so every lower block
//            is already running) and composes their states (combine() below: associative, and it
//            carries consistency — a region's state is exact iff its entry equals the exact exit of
//            the region before, "none" iff that exit lies past it, so a composition from offset 24
//            that is consistent at every seam IS exact).  Wrong guesses (a plausible-looking chain
//            inside a payload) show up as inconsistent seams: a region that disagrees with the
//            claiming region before it, while that one agrees with its own left, is re-walked from
//            its exit (stage the 4 KiB, walk: a few us, rare).  The block publishes its aggregate,
//            composes the published states of the blocks before it (256 per round trip, stopping at
//            the nearest exact one), fixes its own first seam against that exact exit if needed,
//            publishes its exact state and writes each region's exact record prefix.  The last
//            block writes the total and the error flag to pinned host words and the parse's count
//            to a device word.
//   EMIT (pcap_emit_wide_kernel)  32 regions per block, up to 4 records per thread per pass with their
//            list loads issued before the stores: offset = pos + 16, incl_len = next pos - pos - 16 (the
//            last one from the region's exit).
// Variants measured and rejected in rounds 3-5 (a dual-candidate guess, a branch-free chain check, a
// persistent prefetching guess kernel, walk priority, global record lists, record writes by the scan
// blocks, an emit co-scheduled in the scan grid, the 16-region emit) are kept out of this file as
// profiles/ab/r06_pcap_rejected_variants.patch, with their measurements under profiles/ab/.
// tests/test_pcap_model.py restates the composition and the fixes and checks them against the host
// indexer on captures built to defeat the guess.  HBM traffic ≈ the file once + 2 B/record of
// record lists written and read + 12 B/record of output.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <type_traits>

#include "pktgpu_ctx.hpp"

namespace {

constexpr uint32_t kRegion = 4096;  // bytes of record starts per region
static_assert(kRegion % 16 == 0 && kRegion / 16 <= 65536, "u16 record lists");
constexpr uint32_t kMaxRec = kRegion / 16;       // records per region (each >= 16 B apart)
constexpr int kWaves = 4;                         // waves (regions) per 256-thread block
constexpr int kMinHops = 2, kMaxHops = 2;         // guess chain length (3-4 hops measured slower)
constexpr uint32_t kTsSpan = 86400;               // guess: consecutive ts_sec within a day

// Host-visible words (pinned, written by the kernels).
enum : int { kHostMagic = 0, kHostTotal = 1, kHostErr = 2, kHostWords = 4 };

// A scan block's published states: its aggregate (a_*) once its own seams are consistent, its
// exact inclusive state (i_*) once it knows the exact exit before it.  EVERY field carries the call's
// 16-bit epoch in its top 16 bits (values: 48 bits — file positions and counts below 2^48): each field
// is written once per call, so a reader that sees the current epoch in every field of a state has that
// state's final values whatever order the fields became visible in — no ordering between data and flag
// is needed (round 3 published data, waited for the stores (s_waitcnt vmcnt(0)) and then a flag word,
// which relied on gfx950 behaviour outside the HIP memory model).  States of older calls carry older
// epochs, so the array needs no per-call reset (a full reset when the epoch wraps).
struct alignas(64) BlkDesc {
    uint64_t a_first, a_last, a_cnt, a_bits;
    uint64_t i_last, i_cnt, i_bits, pad;
};
constexpr uint32_t kEpochBits = 16;
constexpr uint64_t kValMask = (1ull << (64 - kEpochBits)) - 1;
__host__ __device__ constexpr uint64_t tagged(uint32_t epoch, uint64_t v) { return ((uint64_t)epoch << (64 - kEpochBits)) | v; }
__host__ __device__ constexpr uint32_t tag_of(uint64_t w) { return (uint32_t)(w >> (64 - kEpochBits)); }
enum : uint32_t { kBitNone = 1, kBitErr = 2, kBitBad = 4 };
// a region's count word: records | kCntErr (the walk met a record running past the end)
constexpr uint32_t kCntErr = 0x80000000u, kCntMask = 0x7FFFFFFFu;

constexpr uint32_t kScanRegions = 256;  // regions per scan block (one per thread)
// emit: regions per block and records per thread per pass (32 x 4: 75.3-75.8 us per call against
// 76.5-76.6 for 16 regions one record per step, profiles/ab/r05s_pcap_emit_wide.txt)
constexpr uint32_t kEmitRegions = 32, kEmitPer = 4;

struct Scratch {
    uint64_t* rentry;  // per region: the walk's entry (>= the region's end: no record starts in it)
    uint64_t* rexit;   // per region: exit (first record start >= the region's end, as walked)
    uint32_t* rcnt;    // per region: records, bit 31 = the walk met a record running past the end
    uint64_t* rpre;    // per region: records before it in the file (exact; the scan writes it)
    uint16_t* list;    // [region][kMaxRec] record offsets relative to the region base
    BlkDesc* blk;      // one per scan block
    uint32_t* ticket;  // the scan kernel's
    uint64_t* host;    // kHostWords pinned words (device address)
    uint64_t* dev;     // device words: [0] the record count for a parse that follows on the device (0 after
                       // an error), [1] the magic check (guess region 0)
    uint64_t* count_out;  // where the last scan block writes that count (dev + 0 unless the caller names a word)
    uint32_t epoch;
    // partial = 1: the buffer is a PREFIX of a capture still arriving (pkt_parse_pcap_host's pieces,
    // pkt_pcap_stream_*): a record running past its end ends the index without an error — the records
    // counted are those wholly inside it.  (The walks keep their error bit and the overrunning record's
    // start in the slot after the region's records; only the verdict ignores it.)
    uint32_t partial;
    // Segment mode (carry_in != NULL): the regions [r0, K) of the prefix buf[0, len) are indexed on from
    // the previous prefix's carry — the first record start it did not count (B) and the records it
    // counted (C), on the device — instead of the whole prefix from offset 24.  Every record starting
    // before region r0 other than B's was counted (r0 * kRegion <= the previous prefix's end), and the
    // record after B starts past that end, so B and its record decide region r0's exact entry and the
    // exact state before the segment.  carry_out (may be NULL): this prefix's carry for the next segment.
    uint32_t r0;
    const uint64_t* carry_in;  // [kCarryB], [kCarryC], [kCarryMagic]
    uint64_t* carry_out;
};
// A prefix's carry words (pcap_launch's carry_in / carry_out)
enum : int { kCarryB = 0, kCarryC = 1, kCarryMagic = 2, kCarryWords = 4 };

// The aggregate of a run of regions:
//   none (kBitNone): no region of the run claims a record start; consistent with a predecessor
//     exit e iff e >= last (the run's end), which it passes through;
//   otherwise: `first` = the entry of its first claiming region, `last` = the exit of its last,
//     `cnt` records, kBitBad if two of its regions disagree, kBitErr if a walk met a record
//     running past the end of the file.  Consistent with e iff e == first and not bad.
// combine(a, b) for a run a followed by run b is associative; none(0) is its identity.
// F: the type of positions and counts in the scan's compositions — uint32_t for files shorter than
// 4 GiB - 8 KiB (half the DPP moves and compare-selects per step: 74.4-75.1 vs 75.4-75.9 us per call,
// profiles/ab/r05ar_pcap_scan_32bit.txt), uint64_t beyond or when pkt_ctx_set_pcap_scan64 asks for it
// (the host picks, pcap_launch).
template <class F>
struct AggT {
    F first, last, cnt;
    uint32_t bits;
};
template <class F>
__device__ __forceinline__ AggT<F> mk_agg(uint64_t f, uint64_t l, uint64_t c, uint32_t b) {
    return AggT<F>{(F)f, (F)l, (F)c, b};
}
template <class F>
__device__ __forceinline__ AggT<F> agg_identity() { return AggT<F>{0, 0, 0, kBitNone}; }
// Without branches (selects; a "none" aggregate's first and cnt are 0): the scan steps, the
// cross-wave loops and the look-back compose with no exec-mask save / restore per combine.
template <class F>
__device__ __forceinline__ AggT<F> combine(const AggT<F>& a, const AggT<F>& b) {
    const bool an = (a.bits & kBitNone) != 0, bn = (b.bits & kBitNone) != 0;
    AggT<F> r;
    r.first = an ? b.first : a.first;
    r.last = an ? (bn ? (a.last > b.last ? a.last : b.last) : b.last) : (bn ? a.last : b.last);
    r.cnt = a.cnt + b.cnt;
    const uint32_t both = a.bits | b.bits | (a.last != b.first ? kBitBad : 0u);
    const uint32_t abad = a.bits | (a.last < b.last ? kBitBad : 0u);
    r.bits = an ? (bn ? kBitNone : b.bits) : (bn ? abad : both);
    return r;
}

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
// guess; the look-back makes the result exact whatever it accepts.
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

// Stage file bytes [base, base + BYTES + 16) into LDS, zeros past the file's 16-byte-rounded end;
// NT threads, this one is `t`.  All loads are issued before the first LDS write (one memory
// latency per stage, not one per piece).
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
// (regions of short records) go to `list` from lane 0.  32-bit offsets from the region base while
// the file's end is < 4 GiB past the staged bytes, otherwise the 64-bit form.  The position stays a
// vector value: a scalar walk (readfirstlane of each incl_len, SALU bounds checks) is slower, its
// per-hop chain VALU -> SGPR -> SALU -> VALU longer (111 vs 99 us per call), and the lean vector
// loop (one bound, no masks) beats the round-2 form 99 vs 102 us (profiles/ab/r03t_pcap_walk.txt).
__device__ __forceinline__ void walk(const uint32_t* lw, uint64_t lbase, uint16_t* list, uint64_t base,
                                     uint64_t entry, uint64_t len, uint64_t& exit, uint32_t& cnt, uint32_t& err,
                                     uint32_t& rec) {
    if (len - lbase <= 0xFFFFFFF0ull && entry - lbase <= 0xFFFFFFF0ull) {
        const uint32_t lane = lane_id();
        // q = the record's start relative to the region base (base < len: room >= 1); the walk goes
        // on while q < kRegion and 16 header bytes remain (q <= room - 16); incl_len = bytes
        // q + 8 .. q + 11 (v_alignbyte takes the shift's low two bits: no mask)
        const uint32_t rb = (uint32_t)(base - lbase), room = (uint32_t)(len - lbase) - rb;
        const uint32_t lim = room >= 16 ? (room - 15 < kRegion ? room - 15 : kRegion) : 0u;
        const uint32_t* lr = lw + (rb >> 2);
        uint32_t q = entry >= base ? (uint32_t)(entry - base) : kRegion;  // (entry >= base always)
        uint32_t c = 0, e = 0, rv = 0;
        while (q < lim) {
            const uint32_t k2 = (q >> 2) + 2;
            const uint32_t incl = __builtin_amdgcn_alignbyte(lr[k2 + 1], lr[k2], q);
            rv = lane == c ? q : rv;  // (an overrunning record's start too: slot c, not counted)
            if (c >= 64u && c < kMaxRec && lane == 0) list[c] = (uint16_t)q;
            if (incl > room - 16 - q) {  // pkt_pcap_index: record runs past the end
                e = 1;
                q = room;
                break;
            }
            c++;
            q += 16 + incl;
        }
        exit = base + q;
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
        const uint32_t ro = (uint32_t)(pos - base);
        rec = lane == cnt ? ro : rec;  // (an overrunning record's start too: slot cnt, not counted)
        if (__builtin_amdgcn_readfirstlane(cnt) >= 64u && cnt < kMaxRec && lane == 0) list[cnt] = (uint16_t)ro;
        if (pos + 16 + (uint64_t)incl > len) {  // pkt_pcap_index: record runs past the end
            err = 1;
            pos = len;
            break;
        }
        cnt++;
        pos += 16 + (uint64_t)incl;
    }
    exit = pos;
}

// Region k's guessed entry (the candidate scan of the staged tile at lbase); base + kRegion =
// "no record starts here".
template <uint32_t STAGED>
__device__ __forceinline__ uint64_t guess_entry(const uint8_t* __restrict__ buf, uint64_t len, const uint32_t* lw,
                                                uint64_t lbase, uint32_t k) {
    const uint32_t lane = lane_id();
    const uint64_t lend = lbase + STAGED;
    const uint64_t base = (uint64_t)k * kRegion;
    // snaplen (global header bytes 16..19) bounds a plausible incl_len
    uint32_t snap = *reinterpret_cast<const uint32_t*>(buf + 16);
    if (snap == 0 || snap > (1u << 30)) snap = 1u << 30;
    const uint64_t stop = len < base + kRegion ? len : base + kRegion;
    const uint32_t lim = len - lbase > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)(len - lbase);
    constexpr uint64_t kNoRun = ~0ull;
    uint64_t run = kNoRun;  // a run of verified candidates that reached the previous step's lane 63
    // One step of 64 candidates c0 + lane, r = chain_local's verdict for this lane's: true (and the entry
    // in `res`) when the step decides the region's entry.
    auto step = [&](int r, uint64_t c, uint64_t c0, uint64_t& res) -> bool {
        // The lowest candidate whose chain checks out inside the staged bytes wins; only when
        // there is none do the candidates whose chains leave them read global memory.
        uint64_t m = __ballot(r == 1);
        if (!m) m = __ballot(r == 2 && chain_global(lw, buf, lbase, lend, c, stop, len, snap));
        // The lowest verified candidate, moved to the LAST of the run of consecutive verified
        // candidates it starts: a record whose predecessor's payload ends in zero bytes verifies one
        // to three bytes early too (its fields shifted by whole bytes stay plausible), and the
        // scan's re-walk of such a wrong guess sets its critical path (pcap indexer).
        // A run that reaches lane 63 goes on into the next step (the bench capture's last 7 wrong
        // guesses were runs cut there, one byte early: profiles/ab/r05i_pcap_guess_runacross.txt).
        if (run != kNoRun && !(m & 1u)) {
            res = run;
            return true;
        }
        if (m) {
            const uint32_t f = run != kNoRun ? 0u : (uint32_t)__builtin_ctzll(m);
            const uint64_t rest = ~(m >> f);  // bit j clear iff candidate f + j verified (j < 64 - f)
            const uint32_t rl = rest ? (uint32_t)__builtin_ctzll(rest) : 64u;  // the run's length
            if (f + rl < 64u) {
                res = c0 + f + rl - 1u;
                return true;
            }
            run = c0 + 63;
        }
        return false;
    };
    uint64_t res = 0;
    for (uint64_t c0 = base; c0 < stop; c0 += 64) {
        const uint64_t c = c0 + lane;
        const int r = c < stop && c + 16 <= len
                          ? chain_local(lw, (uint32_t)(c - lbase), (uint32_t)(stop - lbase), STAGED, lim, snap)
                          : 0;
        if (step(r, c, c0, res)) return res;
    }
    return run != kNoRun ? run : base + kRegion;
}

// Tile states cross XCDs (each XCD has its own L2): every access is a device-scope relaxed atomic
// (performed at the device's coherence point); a state is valid when all its fields carry the call's
// epoch (BlkDesc), so no release/acquire fences are needed — on gfx950 they write back / invalidate
// the whole L2 at device scope (1.18 ms per call when round 3 tried them).  (A single-pass form that did the look-back per 16 KiB
// tile with a ticket per tile measured 160-436 us per 2^20-record call: 11.9K device-scope atomics
// on one word serialise, and exact states can only advance 64 tiles per round trip.)
template <class T>
__device__ __forceinline__ T ld_agent(const T* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class T>
__device__ __forceinline__ void st_agent(T* p, T v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Region k's aggregate from its (entry, exit, count|err) state; identity past the file.
template <class F>
__device__ __forceinline__ AggT<F> region_agg(uint32_t k, uint32_t K, uint64_t entry, uint64_t exit, uint32_t cw) {
    if (k >= K) return agg_identity<F>();
    const uint64_t end = ((uint64_t)k + 1) * kRegion;
    if (k != 0 && entry >= end) return mk_agg<F>(0, end, 0, kBitNone);
    return mk_agg<F>(entry, exit, cw & kCntMask, (cw & kCntErr) ? kBitErr : 0u);
}

// The walk of one region by ONE lane (pcap_guess_kernel): pkt_pcap_index's loop from `entry` while the
// record starts inside [base, base + kRegion) and 16 header bytes remain, each record's offset from the
// region base into lst[c].  32-bit positions relative to the staged bytes at lbase (the caller checks
// that the file's end lies < 4 GiB past them).
__device__ __forceinline__ void lane_walk(const uint32_t* lw, uint64_t lbase, uint16_t* lst, uint64_t base,
                                          uint64_t entry, uint64_t len, uint64_t& exit, uint32_t& cnt) {
    const uint32_t rb = (uint32_t)(base - lbase), room = (uint32_t)(len - lbase) - rb;
    const uint32_t lim = room >= 16 ? (room - 15 < kRegion ? room - 15 : kRegion) : 0u;
    const uint32_t* lr = lw + (rb >> 2);
    uint32_t q = entry >= base + kRegion ? kRegion : (uint32_t)(entry - base), c = 0, e = 0;
    while (q < lim) {
        const uint32_t k2 = (q >> 2) + 2;
        const uint32_t incl = __builtin_amdgcn_alignbyte(lr[k2 + 1], lr[k2], q);
        lst[c] = (uint16_t)q;  // (an overrunning record's start too: slot c, not counted)
        if (incl > room - 16 - q) {  // pkt_pcap_index: record runs past the end
            e = 1;
            q = room;
            break;
        }
        c++;
        q += 16 + incl;
    }
    exit = base + q;
    cnt = c | (e ? kCntErr : 0u);
}

// lane_walk without branches (files below 2 GiB): the walking lanes run a loop whose trip count is
// uniform (until no lane is active, two hops per test); a finished lane reads a safe LDS address and
// stores its would-be offset to a dummy slot (lst[kMaxRec]), so a hop is one ds_read2, the
// arithmetic and one ds_write with no exec-mask save/restore (the branchy loop above spent ~25
// scalar and vector instructions per hop on them, ~380 cycles per hop in the guess kernel's
// stamps: profiles/pcap/r04m_stamps.txt).  `valid` = the lane has a region to walk.

__device__ __forceinline__ void lane_walk2(const uint32_t* lw, uint64_t lbase, uint16_t* lst, uint64_t base, uint64_t entry,
                                           uint64_t len, bool valid, uint64_t& exit, uint32_t& cnt) {
    const uint32_t rb = (uint32_t)(base - lbase);
    const uint32_t room = valid ? (uint32_t)(len - lbase) - rb : 0u;  // < 2^31 (the caller checks)
    const uint32_t lim = room >= 16 ? (room - 15 < kRegion ? room - 15 : kRegion) : 0u;
    const uint8_t* lb = reinterpret_cast<const uint8_t*>(lw) + rb;
    // q walks freely (a finished lane's hops are never recorded; min(q, kRegion) keeps its reads
    // inside the staged bytes), qe holds the exit: the chain from one read to the next is a min,
    // an add3 and a min3
    uint32_t q = (!valid || entry >= base + kRegion) ? kRegion : (uint32_t)(entry - base), qe = q, c = 0, e = 0;
    bool act = q < lim;
    auto hop = [&]() {
        uint32_t incl;
        __builtin_memcpy(&incl, lb + __builtin_elementwise_min(q, kRegion) + 8, 4);  // unaligned LDS read
        const uint32_t t = q + 16 + __builtin_elementwise_min(incl, room);            // < 2^32
        const bool over = act & (t > room);  // pkt_pcap_index: record runs past the end
        const bool rec = act & !over;
        lst[act ? c : kMaxRec] = (uint16_t)q;  // (an overrunning record's start too: slot c, not counted)
        c += rec ? 1u : 0u;
        e |= over ? 1u : 0u;
        q = __builtin_elementwise_min(t, room);
        qe = act ? q : qe;
        act = rec & (q < lim);
    };
    while (__ballot(act)) {
        hop();
        hop();
    }
    exit = base + qe;
    cnt = c | (e ? kCntErr : 0u);
}

// GUESS (file header): one region per wave, a block stages 4 consecutive regions (16 KiB + 16 B).
// (One wave per 8 KiB tile walking its second region on from the first's exit — half the candidate
// scans — measured slower: 77 vs 63 us per 2^20-record call; the kernel is bound by each wave's
// chain of dependent LDS reads, and the 32-waves-per-CU cap is reached either way.)
// Round 4: after the four waves' candidate scans the block's four walks run on four LANES of wave 0
// (one region each, in parallel) instead of each on a whole wave: a walk is a serial chain of ~20
// dependent hops whose ~20 VALU instructions per hop a wave issued for all 64 lanes — two thirds of
// the kernel's VALU work (628 per wave, profiles/pcap/r03ad_pcap_guess_pmc.txt).
// Segment mode: the exact state before region r0 from the previous prefix's carry (B = its first
// uncounted record start, C = its records): `entry` = region r0's exact entry, (last, cnt, bits) = the
// exact state before it.  B inside region r0 (or later): its walk counts it.  B before region r0 (a
// record that spanned the previous prefix's end, so the record after it starts past that end): the
// record is counted here (rec_b: its index C, data at B + 16, incl_len b_incl) when it now ends inside
// the prefix; when its header or its bytes still run past the end, nothing of the segment starts a
// record (entry = last = len; kBitErr: the record runs past the end — an error unless partial).
struct SegStart {
    uint64_t entry, last, cnt;
    uint32_t bits;
    bool rec_b;
    uint64_t b;
    uint32_t b_incl;
};
__device__ __forceinline__ SegStart seg_start(const Scratch& S, const uint8_t* __restrict__ buf, uint64_t len) {
    const uint64_t base = (uint64_t)S.r0 * kRegion, B = S.carry_in[kCarryB], C = S.carry_in[kCarryC];
    SegStart r{B, B, C, 0u, false, B, 0u};
    if (B >= base) return r;
    r.entry = r.last = len;
    if (B + 16 > len) return r;
    const uint8_t* h = buf + B + 8;
    const uint32_t incl = (uint32_t)h[0] | ((uint32_t)h[1] << 8) | ((uint32_t)h[2] << 16) | ((uint32_t)h[3] << 24);
    if (B + 16 + (uint64_t)incl > len) {
        r.bits = kBitErr;
        return r;
    }
    r.entry = r.last = B + 16 + (uint64_t)incl;
    r.cnt = C + 1;
    r.rec_b = true;
    r.b_incl = incl;
    return r;
}

// Diagnostic build only (-DPKTGPU_STAMPS=1, read by scripts/pcap_stamps.py): per wave of the guess
// kernel, s_memrealtime at the start, after the staging barrier, after its candidate scan, after the
// walk barrier and after its stores drained, + XCC id and the entry's distance from the region
// base, written by lane 0 to a debug buffer nothing else reads (pkt_debug_pcap_stamps).
#ifndef PKTGPU_STAMPS
#define PKTGPU_STAMPS 0
#endif
#if PKTGPU_STAMPS
__device__ uint64_t* g_pcap_stamps;
#define PCAP_STAMP(k)                                                               \
    do {                                                                            \
        __builtin_amdgcn_sched_barrier(0);                                          \
        uint64_t t_;                                                                \
        asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); \
        __builtin_amdgcn_sched_barrier(0);                                          \
        st_[k] = t_;                                                                \
    } while (0)
#else
#define PCAP_STAMP(k) \
    do {              \
    } while (0)
#endif
__global__ __launch_bounds__(256) void pcap_guess_kernel(const uint8_t* __restrict__ buf, uint64_t len, uint32_t K,
                                                         Scratch S) {
    constexpr uint32_t kStaged = kWaves * kRegion;
    __shared__ uint4 lds[kStaged / 16 + 2];
    __shared__ uint16_t lst[kWaves][kMaxRec + 2];  // + the dummy slot of lane_walk2
    __shared__ uint64_t s_entry[kWaves], s_exit[kWaves];
    __shared__ uint32_t s_cnt[kWaves];
    const uint32_t t = threadIdx.x, w = t / 64, lane = t & 63;
    // (segment mode: the tiles start at region r0)
    const uint32_t k0 = S.r0 + blockIdx.x * kWaves;
    const uint64_t lbase = (uint64_t)k0 * kRegion;
    const bool seg = S.carry_in != nullptr;
#if PKTGPU_STAMPS
    uint64_t st_[5] = {0, 0, 0, 0, 0};
#endif
    PCAP_STAMP(0);
    if (blockIdx.x == 0 && t == 0 && S.carry_out) S.carry_out[kCarryB] = ~0ull;  // the scan's atomicMin target
    stage<kStaged, 256>(lds, buf, lbase, len, t);
    __syncthreads();
    PCAP_STAMP(1);
    const uint32_t k = k0 + w;
    const uint32_t* lw = reinterpret_cast<const uint32_t*>(lds);
    const uint64_t base = (uint64_t)k * kRegion;
    // region 0 starts at 24 by definition; a segment's first region is guessed like any other (the
    // scan fixes it against the carry: reading the carry here cost the kernel 34 VGPRs, 8 -> 6 waves
    // per SIMD, 50.9 -> 57.6 us per 2^20-record call)
    auto entry_of = [&]() -> uint64_t {
        if (k >= K) return base + kRegion;
        if (!seg && k == 0) return 24;
        return guess_entry<kStaged>(buf, len, lw, lbase, k);
    };
    if (len - lbase <= 0xFFFFFFF0ull) {
        // (lane_walk2 needs the file's end < 2 GiB past the staged bytes; lane_walk takes the rest)
        const bool w2 = len - lbase <= 0x7FFFFFF0ull;
        const uint64_t entry = entry_of();
        PCAP_STAMP(2);
        if (lane == 0) s_entry[w] = entry;
        __syncthreads();
        if (w == 0 && lane < (uint32_t)kWaves) {
            const uint32_t kk = k0 + lane;
            const uint64_t en = s_entry[lane];
            uint64_t ex = 0;
            uint32_t cw = 0;
            uint16_t* ll = lst[lane];
            if (w2)
                lane_walk2(lw, lbase, ll, (uint64_t)kk * kRegion, en, len, kk < K, ex, cw);
            else if (kk < K)
                lane_walk(lw, lbase, ll, (uint64_t)kk * kRegion, en, len, ex, cw);
            s_exit[lane] = ex;
            s_cnt[lane] = cw;
        }
        __syncthreads();
        PCAP_STAMP(3);
        if (k >= K) return;
        const uint32_t cw = s_cnt[w], cnt = cw & kCntMask;
        {
            // the records' offsets + an overrunning record's start (slot cnt)
            const uint32_t nl = cnt + ((cw & kCntErr) && cnt < kMaxRec ? 1u : 0u);
            uint16_t* dst = S.list + (uint64_t)k * kMaxRec;
            for (uint32_t i = lane; i < nl; i += 64) dst[i] = lst[w][i];
        }
        if (lane == 0) {
            S.rentry[k] = entry;
            S.rexit[k] = s_exit[w];
            S.rcnt[k] = cw;
            if (!seg && k == 0) {  // pkt_pcap_index rejects a bad magic whatever follows
                const uint64_t mg = buf[0] == 0xD4 && buf[1] == 0xC3 && buf[2] == 0xB2 && buf[3] == 0xA1;
                __hip_atomic_store(&S.host[kHostMagic], mg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                S.dev[1] = mg;
            }
        }
#if PKTGPU_STAMPS
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        PCAP_STAMP(4);
        if (lane == 0 && g_pcap_stamps) {
            uint32_t xcc;
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
            uint64_t* d = g_pcap_stamps + (uint64_t)(k - S.r0) * 8u;
            for (int q = 0; q < 5; q++) d[q] = st_[q];
            d[5] = xcc & 15u;
            d[6] = entry - base;
            d[7] = cw & kCntMask;
        }
#endif
        return;
    }
    if (k >= K) return;
    const uint64_t entry = entry_of();
    uint64_t exit;
    uint32_t cnt, err, rec;
    // (w = readfirstlane(t / 64), which lets the compiler see k as uniform and turn the walk into a
    // scalar loop — VALU per hop 20 -> 5, SALU 14 -> 17 — measured slower: 111 vs 102 us per call,
    // profiles/ab/r03n_pcap_uniform_wave.txt)
    // (the walk reading each incl_len by scalar-unit loads from L2 instead of LDS halves the VALU
    // instructions, 736 -> 374 per wave, but each hop then waits ~3x longer: 80 vs 63 us per call,
    // profiles/ab/r03i_pcap_uniform_walk.txt)
    uint16_t* dst = S.list + (uint64_t)k * kMaxRec;
    walk(lw, lbase, lst[w], base, entry, len, exit, cnt, err, rec);
    wave_lds_sync();
    const uint32_t nl = cnt + (err && cnt < kMaxRec ? 1u : 0u);  // + an overrunning record's start
    if (lane < nl) dst[lane] = (uint16_t)rec;
    for (uint32_t i = 64 + lane; i < nl; i += 64) dst[i] = lst[w][i];
    if (lane == 0) {
        S.rentry[k] = entry;
        S.rexit[k] = exit;
        S.rcnt[k] = cnt | (err ? kCntErr : 0u);
        if (!seg && k == 0) {  // pkt_pcap_index rejects a bad magic whatever follows
            const uint64_t mg = buf[0] == 0xD4 && buf[1] == 0xC3 && buf[2] == 0xB2 && buf[3] == 0xA1;
            __hip_atomic_store(&S.host[kHostMagic], mg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            S.dev[1] = mg;
        }
    }
}

// Block-wide exclusive composition of the threads' aggregates in thread order (all 256 threads).
// Also returns `idx`: the thread index of the nearest claiming (non-none) aggregate before t, or -1.
// The wave's inclusive scan by DPP moves: row_shr 1, 2, 4, 8 within each row of
// 16 lanes, then row_bcast 15 and 31 across rows — register moves, no LDS; a lane without a source
// takes the identity (update_dpp's `old`, bound_ctrl off), so every lane combines, without
// divergence.  (The __shfl_up form below — ds_bpermute round trips, each step under `lane >= d` —
// made the first block composition 2.8 us of every scan block, profiles/pcap/r04h2_stamps.txt.)
template <int CTRL, int ROWS>
__device__ __forceinline__ uint32_t dpp32(uint32_t old, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, CTRL, ROWS, 0xF, false);
}
template <int CTRL, int ROWS>
__device__ __forceinline__ uint64_t dpp64(uint64_t old, uint64_t v) {
    return ((uint64_t)dpp32<CTRL, ROWS>((uint32_t)(old >> 32), (uint32_t)(v >> 32)) << 32) |
           dpp32<CTRL, ROWS>((uint32_t)old, (uint32_t)v);
}
template <int CTRL, int ROWS, class F>
__device__ __forceinline__ F dppf(F old, F v) {
    if constexpr (sizeof(F) == 4) return dpp32<CTRL, ROWS>(old, v);
    else return dpp64<CTRL, ROWS>(old, v);
}
template <int CTRL, int ROWS, class F>
__device__ __forceinline__ void scan_step(AggT<F>& x, int32_t& ix) {
    AggT<F> y;
    y.first = dppf<CTRL, ROWS, F>(0, x.first);
    y.last = dppf<CTRL, ROWS, F>(0, x.last);
    y.cnt = dppf<CTRL, ROWS, F>(0, x.cnt);
    y.bits = dpp32<CTRL, ROWS>(kBitNone, x.bits);
    const int32_t iy = (int32_t)dpp32<CTRL, ROWS>(0xFFFFFFFFu, (uint32_t)ix);
    x = combine(y, x);
    ix = ix >= 0 ? ix : iy;
}

__device__ __forceinline__ uint64_t stamp_now() {
    uint64_t t_;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t_;
}

// (bx: diagnostic stamps — after the wave scans, after the first barrier — or NULL)
template <class F>
__device__ __forceinline__ AggT<F> block_exclusive(AggT<F> a, int32_t& idx, AggT<F>* wtot, int32_t* widx, AggT<F>& total,
                                               uint64_t* bx = nullptr) {
    const uint32_t t = threadIdx.x, w = t / 64, lane = t & 63;
    int32_t ix = (a.bits & kBitNone) ? -1 : (int32_t)t;
    AggT<F> x = a;
    scan_step<0x111, 0xF>(x, ix);  // row_shr:1
    scan_step<0x112, 0xF>(x, ix);  // row_shr:2
    scan_step<0x114, 0xF>(x, ix);  // row_shr:4
    scan_step<0x118, 0xF>(x, ix);  // row_shr:8
    scan_step<0x142, 0xA>(x, ix);  // row_bcast:15 into rows 1 and 3
    scan_step<0x143, 0xC>(x, ix);  // row_bcast:31 into rows 2 and 3
    if (PKTGPU_STAMPS && bx) bx[0] = stamp_now();
    if (lane == 63) {
        wtot[w] = x;
        widx[w] = ix;
    }
    __syncthreads();
    if (PKTGPU_STAMPS && bx) bx[1] = stamp_now();
    // the waves' totals in order, one running composition (its value before wave w is this wave's
    // prefix): four combines, no loop branch
    AggT<F> before = agg_identity<F>();
    int32_t ib = -1;
    AggT<F> run = agg_identity<F>();
    int32_t irun = -1;
#pragma unroll
    for (uint32_t q = 0; q < (uint32_t)kWaves; q++) {
        if (q == w) {
            before = run;
            ib = irun;
        }
        const int32_t iq = widx[q];
        run = combine(run, wtot[q]);
        irun = iq >= 0 ? iq : irun;
    }
    total = run;
    // exclusive: the wave prefix before this lane
    AggT<F> ex;  // wave_shr:1, lane 0 the identity
    ex.first = dppf<0x138, 0xF, F>(0, x.first);
    ex.last = dppf<0x138, 0xF, F>(0, x.last);
    ex.cnt = dppf<0x138, 0xF, F>(0, x.cnt);
    ex.bits = dpp32<0x138, 0xF>(kBitNone, x.bits);
    const int32_t iex = (int32_t)dpp32<0x138, 0xF>(0xFFFFFFFFu, (uint32_t)ix);
    idx = iex >= 0 ? iex : ib;
    __syncthreads();  // wtot / widx reusable
    return combine(before, ex);
}

// Does a region with aggregate r disagree with the run `pre` before it (pre claiming)?
template <class F>
__device__ __forceinline__ bool seam_bad(const AggT<F>& pre, const AggT<F>& r) {
    if (pre.bits & kBitNone) return false;
    return (r.bits & kBitNone) ? pre.last < r.last : pre.last != r.first;
}

// The look-back: a lane whose block has published nothing yet re-reads it after a short sleep, up to
// kSpinMax times, before the block-wide retry (78.1 vs 81.8-82.6 us per call without the spin,
// profiles/ab/r05m_pcap_lookback_spin.txt).
constexpr uint32_t kSpinMax = 4096;

// Scan kernel (file header: SCAN).  Thread t = region r0 + blk * 256 + t.  (cap, offsets, lens: where a
// segment's block 0 writes the record of the carry that spanned the previous prefix's end.)
template <class F>
__global__ __launch_bounds__(256) void pcap_scan_kernel(const uint8_t* __restrict__ buf, uint64_t len, uint32_t K,
                                                        uint32_t nb, int ticket, Scratch S, uint64_t cap,
                                                        uint64_t* __restrict__ offsets, uint32_t* __restrict__ lens) {
    using Agg = AggT<F>;
    __shared__ uint4 lds[kWaves][kRegion / 16 + 2];
    __shared__ uint16_t lst[kWaves][kMaxRec + 2];  // + the dummy slot of lane_walk2
    __shared__ uint64_t sen[kScanRegions], sex[kScanRegions];
    __shared__ uint32_t scw[kScanRegions];
    __shared__ uint32_t fq[kScanRegions];
    __shared__ uint64_t fe[kScanRegions];
    __shared__ uint8_t sbad[kScanRegions];
    __shared__ uint16_t sov[kScanRegions];  // a walk that met a record running past the end: its start
    __shared__ Agg wtot[kWaves];
    __shared__ int32_t widx[kWaves];
    __shared__ uint32_t s_blk, s_nf, s_retry, s_near;
    __shared__ Agg s_P;
    const uint32_t t = threadIdx.x, w = t / 64, lane = t & 63;
#if PKTGPU_STAMPS
    uint64_t st_[5] = {0, 0, 0, 0, 0};
    uint32_t n_fix = 0, n_wait = 0;
    uint64_t t_bx = 0;  // after the first block composition
    uint64_t bx[2] = {0, 0};
#endif
    PCAP_STAMP(0);
    // the block order: blockIdx when the device could hold the whole grid at once (the host checks
    // the occupancy; progress then rests on the dispatcher launching workgroups in blockIdx order, so
    // every lower block has been dispatched before this one — see pcap_launch), else a ticket (every
    // lower ticket's block is then already running)
    if (t == 0) s_blk = ticket ? atomicAdd(S.ticket, 1u) : blockIdx.x;
    __syncthreads();
    const uint32_t blk = s_blk;
    const bool seg = S.carry_in != nullptr;
    const uint32_t k = S.r0 + blk * kScanRegions + t;
    sov[t] = 0;
    if (k < K) {
        sen[t] = S.rentry[k];
        sex[t] = S.rexit[k];
        const uint32_t cw = S.rcnt[k];
        scw[t] = cw;
        if (cw & kCntErr) sov[t] = S.list[(uint64_t)k * kMaxRec + (cw & kCntMask)];
    } else {
        sen[t] = sex[t] = 0;
        scw[t] = 0;
    }
    __syncthreads();
    PCAP_STAMP(1);
    // Re-walk the queued regions fq[0, s_nf) from fe[]: one wave per region (stage its 4 KiB, walk),
    // the state to LDS and global memory.
    auto run_fixes = [&]() {
        const uint32_t nf = s_nf;
        for (uint32_t i = w; i < nf; i += kWaves) {
            const uint32_t r = fq[i], kk = S.r0 + blk * kScanRegions + r;
            const uint64_t base = (uint64_t)kk * kRegion, e = fe[i];
            wave_lds_sync();
            if (e < base + kRegion) stage<kRegion, 64>(lds[w], buf, base, len, lane);
            wave_lds_sync();
            if (len - base <= 0x7FFFFFF0ull) {  // wave-uniform
                // one lane walks (lane_walk2: the whole-wave walk below took ~9 us per fixed
                // region, on the scan's critical path: profiles/pcap/r04q_stamps_guess_scan.txt)
                uint64_t ex = 0;
                uint32_t cw = 0;
                if (lane == 0)
                    lane_walk2(reinterpret_cast<const uint32_t*>(lds[w]), base, lst[w], base, e, len, true, ex, cw);
                wave_lds_sync();
                cw = (uint32_t)__shfl((int)cw, 0, 64);
                ex = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(ex >> 32), 0, 64) << 32) |
                     (uint32_t)__shfl((int)(uint32_t)ex, 0, 64);
                const uint32_t cnt = cw & kCntMask;
                uint16_t* dst = S.list + (uint64_t)kk * kMaxRec;
                for (uint32_t j = lane; j < cnt; j += 64) dst[j] = lst[w][j];
                if (lane == 0) {
                    sov[r] = (cw & kCntErr) ? lst[w][cnt] : 0;
                    sen[r] = e;
                    sex[r] = ex;
                    scw[r] = cw;
                    S.rentry[kk] = e;
                    S.rexit[kk] = ex;
                    S.rcnt[kk] = cw;
                }
                continue;
            }
            uint64_t exit;
            uint32_t cnt, err, rec;
            walk(reinterpret_cast<const uint32_t*>(lds[w]), base, lst[w], base, e, len, exit, cnt, err, rec);
            wave_lds_sync();
            uint16_t* dst = S.list + (uint64_t)kk * kMaxRec;
            if (lane < cnt) dst[lane] = (uint16_t)rec;
            for (uint32_t j = 64 + lane; j < cnt; j += 64) dst[j] = lst[w][j];
            // an overrunning record's start: slot cnt (lane cnt's register below 64)
            const uint32_t ov = (uint32_t)__shfl((int)rec, (int)(cnt & 63u), 64);
            if (lane == 0) {
                const uint32_t cw = cnt | (err ? kCntErr : 0u);
                sov[r] = err ? (uint16_t)(cnt < 64 ? ov : lst[w][cnt]) : 0;
                sen[r] = e;
                sex[r] = exit;
                scw[r] = cw;
                S.rentry[kk] = e;
                S.rexit[kk] = exit;
                S.rcnt[kk] = cw;
            }
        }
        __syncthreads();
    };
    // ---- local fixes: a region that disagrees with the claiming region before it (in this block)
    // while that one agrees with its own left is re-walked from its exit; until no such region
    Agg total, pre_cur;  // pre_cur: the block-exclusive composition of the current states
    for (;;) {
        const Agg mine = region_agg<F>(k, K, sen[t], sex[t], scw[t]);
        int32_t j;
#if PKTGPU_STAMPS
        const Agg pre = block_exclusive(mine, j, wtot, widx, total, t_bx ? nullptr : bx);
#else
        const Agg pre = block_exclusive(mine, j, wtot, widx, total);
#endif
#if PKTGPU_STAMPS
        if (!t_bx) {
            __builtin_amdgcn_sched_barrier(0);
            asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_bx)::"memory");
            __builtin_amdgcn_sched_barrier(0);
        }
#endif
        pre_cur = pre;
        const bool bad = j >= 0 && seam_bad(pre, mine);
        sbad[t] = bad;
        // (an exit landing before this region's start means a "none" region between is wrong: that
        // one is fixed first, never this one from a position outside it)
        if (t == 0) s_nf = 0;
        __syncthreads();
        if (bad && !sbad[j] && pre.last >= (uint64_t)k * kRegion) {
            const uint32_t q = atomicAdd(&s_nf, 1u);
            fq[q] = t;
            fe[q] = pre.last;
        }
        __syncthreads();
        if (s_nf == 0) break;
#if PKTGPU_STAMPS
        n_fix += s_nf;
#endif
        run_fixes();
    }
    PCAP_STAMP(2);
    // ---- publish the aggregate; compose the blocks before (stopping at the nearest exact one)
    BlkDesc* my = S.blk + blk;
    if (t == 0) {
        st_agent(&my->a_first, tagged(S.epoch, total.first));
        st_agent(&my->a_last, tagged(S.epoch, total.last));
        st_agent(&my->a_cnt, tagged(S.epoch, total.cnt));
        st_agent(&my->a_bits, tagged(S.epoch, total.bits));
    }
    Agg P = agg_identity<F>();
    for (;;) {
        Agg acc = agg_identity<F>();
        bool exact = blk == 0;
        uint64_t il = 0, ic = 0;
        uint32_t ib = 0;
        if (t == 0) s_retry = 0;
        for (int64_t hi = blk; hi > 0 && !exact;) {
            // window [hi - 256, hi): lane l of wave v reads block hi - 1 - 64 v - l
            const int64_t jj = hi - 1 - (int64_t)t;
            uint32_t st = 0;  // 0 unpublished, 1 aggregate, 2 exact
            Agg a = agg_identity<F>();
            uint64_t xl = 0, xc = 0, xm = 0;
            // (a lane whose block has published nothing yet re-reads it after a short sleep, up to
            // kSpinMax times, instead of the whole window being re-read after a block-wide retry)
            for (uint32_t spin = 0; jj >= 0; spin++) {
                // all seven fields in one round trip; a state counts only with the epoch in every field
                const BlkDesc* d = S.blk + jj;
                const uint64_t il_ = ld_agent(&d->i_last), ic_ = ld_agent(&d->i_cnt), ib_ = ld_agent(&d->i_bits);
                const uint64_t af = ld_agent(&d->a_first), al = ld_agent(&d->a_last), ac = ld_agent(&d->a_cnt),
                               ab = ld_agent(&d->a_bits);
                const uint32_t ep = S.epoch;
                if (tag_of(il_) == ep && tag_of(ic_) == ep && tag_of(ib_) == ep) {
                    st = 2;
                    xl = il_ & kValMask;
                    xc = ic_ & kValMask;
                    xm = ib_ & kValMask;
                } else if (tag_of(af) == ep && tag_of(al) == ep && tag_of(ac) == ep && tag_of(ab) == ep) {
                    st = 1;
                    a = mk_agg<F>(af & kValMask, al & kValMask, ac & kValMask, (uint32_t)(ab & 15u));
                    // block 0's consistent aggregate IS its exact state (region 0 starts at 24 by
                    // definition; block 0 has no seam before it to fix): no wait for its exact
                    // state's publication, which a look-back's first read usually missed
                    // (one retry per block, ~2.5 us: profiles/pcap/r05k_stamps.txt)
                    // (not a segment's block 0: records before it are counted in the carry)
                    if (!seg && jj == 0 && !(a.bits & (kBitNone | kBitBad)) && a.first == 24) {
                        st = 2;
                        xl = a.last;
                        xc = a.cnt;
                        xm = a.bits & kBitErr;
                    }
                }
                if (st || spin >= kSpinMax) break;
                __builtin_amdgcn_s_sleep(1);
            }
            // the nearest exact block in the window (the smallest thread index with st == 2)
            if (t == 0) s_near = 256;
            __syncthreads();
            if (st == 2) atomicMin(&s_near, t);
            __syncthreads();
            const uint32_t near = s_near;
            if (jj >= 0 && t < near && st == 0) s_retry = 1;  // a nearer block has not published
            if (t >= near) a = agg_identity<F>();
            // compose the window's aggregates after the nearest exact block in block order: thread
            // order is reversed block order — within a wave lane 63 is the earliest, and wave 3 the
            // earliest wave
            Agg wr = agg_identity<F>();
            {
                Agg x = a;
#pragma unroll
                for (uint32_t dd = 1; dd < 64; dd <<= 1) {
                    Agg y;
                    y.first = __shfl_down(x.first, dd, 64);
                    y.last = __shfl_down(x.last, dd, 64);
                    y.cnt = __shfl_down(x.cnt, dd, 64);
                    y.bits = __shfl_down(x.bits, dd, 64);
                    if (lane + dd >= 64) y = agg_identity<F>();
                    x = combine(y, x);
                }
                if (lane == 0) wtot[w] = x;
                __syncthreads();
                for (int q = kWaves - 1; q >= 0; q--) wr = combine(wr, wtot[q]);
                __syncthreads();
            }
            acc = combine(wr, acc);
            if (near < 256) {
                exact = true;
                if (t == near) {
                    s_P = mk_agg<F>(0, xl, xc, (uint32_t)xm & kBitErr);
                }
                __syncthreads();
                il = s_P.last;
                ic = s_P.cnt;
                ib = s_P.bits;
                __syncthreads();
            }
            hi -= 256;
            if (s_retry) break;
        }
        __syncthreads();
        if (s_retry || !exact) {  // a block before has not published, or none is exact yet
#if PKTGPU_STAMPS
            n_wait++;
#endif
            __builtin_amdgcn_s_sleep(8);
            continue;
        }
        if (blk == 0) {
            P = agg_identity<F>();
            if (seg) {  // the exact state before region r0, from the carry
                const SegStart ss = seg_start(S, buf, len);
                P = mk_agg<F>(0, ss.last, ss.cnt, ss.bits);
                if (t == 0) {
                    if (ss.rec_b && ss.cnt - 1 < cap) {  // the spanning record, now whole
                        offsets[ss.cnt - 1] = ss.b + 16;
                        lens[ss.cnt - 1] = ss.b_incl;
                    }
                    // still not whole: it stays the next prefix's first uncounted record
                    if (!ss.rec_b && ss.b < (uint64_t)S.r0 * kRegion && S.carry_out)
                        atomicMin(reinterpret_cast<unsigned long long*>(&S.carry_out[kCarryB]), (unsigned long long)ss.b);
                }
            }
            break;
        }
        // P = the exact state before this block: (exit, count, error)
        if (acc.bits & kBitNone) {
            if (il >= acc.last) {
                P = mk_agg<F>(0, il, ic, ib | 0u);
                break;
            }
        } else if (!(acc.bits & kBitBad) && acc.first == il) {
            P = mk_agg<F>(0, acc.last, ic + acc.cnt, ib | (acc.bits & kBitErr));
            break;
        }
#if PKTGPU_STAMPS
        n_wait += 1u << 16;
#endif
        __builtin_amdgcn_s_sleep(8);  // an earlier block has not fixed its first seam yet
    }
    PCAP_STAMP(3);
    // ---- this block's seams against the exact exit before it: fix the first disagreeing region
    // from the exact state before it, until none disagrees (exact by induction)
    // (region 0 of a whole file has nothing before it; every other block, a segment's first included,
    // has the exact state P before it)
    const bool origin = blk == 0 && !seg;
    Agg exact_pre = origin ? agg_identity<F>() : mk_agg<F>(P.last, P.last, 0, 0);  // "claims" the exact exit
    // (the states have not changed since the local fixes' last composition: reuse it, and recompose
    // only after a fix below)
    for (bool fresh = true;; fresh = false) {
        const Agg mine = region_agg<F>(k, K, sen[t], sex[t], scw[t]);
        if (!fresh) {
            int32_t j;
            pre_cur = block_exclusive(mine, j, wtot, widx, total);
        }
        const Agg pre0 = pre_cur;
        const Agg pre = combine(exact_pre, pre0);
        const bool bad = seam_bad(pre, mine) && !(pre.bits & kBitBad) && pre.last >= (uint64_t)k * kRegion;
        if (t == 0) s_nf = 0;
        __syncthreads();
        if (bad) {  // exactly one region: the first disagreeing seam
            fq[0] = t;
            fe[0] = pre.last;
            s_nf = 1;
        }
        __syncthreads();
        if (s_nf == 0) break;
#if PKTGPU_STAMPS
        n_fix += s_nf;
#endif
        run_fixes();
    }
    // ---- the exact state after this block; each region's record prefix
    const Agg all = combine(origin ? agg_identity<F>() : mk_agg<F>(P.last, P.last, 0, 0), total);
    const uint64_t c_before = origin ? 0 : P.cnt;
    const uint32_t err_all = (P.bits | all.bits) & kBitErr;
    const uint64_t last = (all.bits & kBitNone) ? P.last : all.last;
    // the carry: the first record start this prefix does not count — the start of the record that runs
    // past its end, when the exact chain meets one (every region is now consistent, so a claiming region
    // whose walk met one is on the chain), else the chain's exit; the smallest candidate wins
    if (S.carry_out && k < K && (scw[t] & kCntErr) && !(sen[t] >= ((uint64_t)k + 1) * kRegion && k != 0))
        atomicMin(reinterpret_cast<unsigned long long*>(&S.carry_out[kCarryB]),
                  (unsigned long long)((uint64_t)k * kRegion + sov[t]));
    if (t == 0) {
        st_agent(&my->i_last, tagged(S.epoch, last));
        st_agent(&my->i_cnt, tagged(S.epoch, c_before + total.cnt));
        st_agent(&my->i_bits, tagged(S.epoch, err_all));
        if (blk == nb - 1) {
            // every block has taken its ticket by now (this one took the last): the next call's
            // tickets start at 0 without a memset launch on the call's critical path (4.7 us)
            if (ticket) st_agent(S.ticket, 0u);
            // the magic check of region 0 (a segment: the first prefix's, carried)
            const uint64_t magic = seg ? S.carry_in[kCarryMagic] : S.dev[1];
            // a record running past the end is an error of the whole capture only (not of a prefix)
            const bool err = err_all && !S.partial;
            __hip_atomic_store(&S.host[kHostTotal], c_before + total.cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&S.host[kHostMagic], magic, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            // the count a parse on the same stream reads (kernel boundary: no fence needed); 0 when
            // the call fails (bad magic, a record past the end), so that parse writes nothing
            *S.count_out = (magic && !err) ? c_before + total.cnt : 0;
            __hip_atomic_store(&S.host[kHostErr], (uint64_t)(err ? 1 : 0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            if (S.carry_out) {
                S.carry_out[kCarryMagic] = magic;
                atomicMin(reinterpret_cast<unsigned long long*>(&S.carry_out[kCarryB]), (unsigned long long)last);
            }
        }
    }
    // each region's exact record prefix (the emit kernel writes the records): the records of the
    // regions before it in the block are the exclusive composition's count
    if (k < K) S.rpre[k] = c_before + pre_cur.cnt;
#if PKTGPU_STAMPS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    PCAP_STAMP(4);
    if (t == 0 && g_pcap_stamps) {  // after the guess kernel's K rows: one row per scan block
        uint64_t* d = g_pcap_stamps + (uint64_t)K * 8u + blk * 16u;
        for (int q = 0; q < 5; q++) d[q] = st_[q];
        d[5] = n_fix;
        d[6] = n_wait;
        d[7] = t_bx;
        d[8] = bx[0];
        d[9] = bx[1];
    }
#endif
}

// Emit (file header: EMIT): NR consecutive regions per block; every thread takes up to PER records per
// pass and issues all their list loads before the first store, so a block waits one round trip for its
// region words and one for its lists instead of one per record step.  The records are contiguous in the
// output (coalesced stores), at the regions' exact prefix.
template <uint32_t NR, uint32_t PER>
__global__ __launch_bounds__(256) void pcap_emit_wide_kernel(uint32_t K, uint64_t cap, Scratch S,
                                                             uint64_t* __restrict__ offsets,
                                                             uint32_t* __restrict__ lens, const uint8_t* __restrict__ buf) {
    static_assert(NR >= 2 && NR <= 64 && (NR & (NR - 1)) == 0, "NR: a power of two <= 64");
    __shared__ uint32_t cpre[NR + 1];
    __shared__ uint64_t cex[NR];
    const uint32_t k0 = S.r0 + blockIdx.x * NR, t = threadIdx.x;
    const uint64_t first = S.rpre[k0];
    if (t < 64) {
        const bool in = t < NR && k0 + t < K;
        const uint32_t c = in ? (S.rcnt[k0 + t] & kCntMask) : 0;
        if (t < NR) cex[t] = in ? S.rexit[k0 + t] : 0;
        uint32_t x = c;
#pragma unroll
        for (uint32_t d = 1; d < NR; d <<= 1) {
            const uint32_t y = __shfl_up(x, d, 64);
            if (t >= d) x += y;
        }
        if (t < NR) cpre[t] = x - c;
        if (t == NR - 1) cpre[NR] = x;
    }
    __syncthreads();
    const uint32_t total = cpre[NR];
    for (uint32_t i0 = 0; i0 < total && first + i0 < cap; i0 += 256u * PER) {
        uint32_t rr[PER], li[PER], cc[PER], a[PER], b[PER];
#pragma unroll
        for (uint32_t u = 0; u < PER; u++) {
            const uint32_t i = i0 + u * 256u + t;
            uint32_t r = 0;
#pragma unroll
            for (uint32_t bb = NR / 2; bb; bb >>= 1)
                if (cpre[r + bb] <= i) r += bb;
            rr[u] = r;
            li[u] = i - cpre[r];
            cc[u] = cpre[r + 1] - cpre[r];
        }
#pragma unroll
        for (uint32_t u = 0; u < PER; u++) {
            const uint32_t i = i0 + u * 256u + t;
            a[u] = b[u] = 0;
            if (i < total) {
                const uint16_t* list = S.list + (uint64_t)(k0 + rr[u]) * kMaxRec;
                a[u] = list[li[u]];
                if (li[u] + 1 < cc[u]) b[u] = list[li[u] + 1];
            }
        }
#pragma unroll
        for (uint32_t u = 0; u < PER; u++) {
            const uint32_t i = i0 + u * 256u + t;
            const uint64_t idx = first + i;
            if (i >= total || idx >= cap) continue;
            const uint64_t base = (uint64_t)(k0 + rr[u]) * kRegion;
            const uint64_t pos = base + a[u];
            const bool last = li[u] + 1 == cc[u];
            const uint64_t next = last ? cex[rr[u]] : base + b[u];
            uint32_t incl = (uint32_t)(next - pos - 16);
            if (S.partial && last) {
                // a prefix of a capture: the walk that stopped at a record running past the prefix's end
                // set its region's exit to that end, not to the record's start — the region's last
                // counted record takes its incl_len from its own header (bytes pos + 8 .. pos + 11)
                const uint8_t* h = buf + pos + 8;
                incl = (uint32_t)h[0] | ((uint32_t)h[1] << 8) | ((uint32_t)h[2] << 16) | ((uint32_t)h[3] << 24);
            }
            offsets[idx] = pos + 16;
            lens[idx] = incl;
        }
    }
}


}  // namespace

// Queue the index of the pcap file `buf` on `s` (guess + scan kernels; the scan writes the records):
// no host synchronisation.  *count_dev = the device word a following parse may take its record count
// from (0 after an error).  pcap_finish reads the outcome once the stream is synchronised.
// The index scratch for K regions (grown on demand, after `s` has drained).
static hipError_t pcap_reserve(pkt_ctx_t* ctx, uint32_t K, hipStream_t s) {
    PcapScratch& pc = ctx->pc;
    if (K <= pc.k_cap) return hipSuccess;
    if (pc.buf) {
        (void)hipStreamSynchronize(s);
        (void)hipFree(pc.buf);
        pc.buf = nullptr;
        pc.bytes = 0;
        pc.k_cap = pc.nb_cap = 0;
    }
    const uint32_t kc = K + K / 4 + 64, nbc = (kc + kScanRegions - 1) / kScanRegions;
    const uint64_t bytes = 64 + (uint64_t)nbc * sizeof(BlkDesc) + (uint64_t)kc * (8 + 8 + 8 + 4 + 2 * kMaxRec);
    hipError_t e = hipMalloc(&pc.buf, bytes);
    if (e == hipSuccess) e = hipMemsetAsync(pc.buf, 0, bytes, s);
    if (e != hipSuccess) return e;
    pc.bytes = bytes;
    pc.k_cap = kc;
    pc.nb_cap = nbc;
    return hipSuccess;
}

int pktgpu_pcap_reserve(pkt_ctx_t* ctx, uint64_t len, hipStream_t s) {
    const uint64_t K64 = (len + kRegion - 1) / kRegion;
    if (K64 > (1ull << 31)) return fail(ctx, PKT_ERR_INVALID_ARG, "pcap too large");
    hipError_t e = hipSetDevice(ctx->device);
    if (e == hipSuccess) e = pcap_reserve(ctx, (uint32_t)K64, s);
    return e == hipSuccess ? PKT_SUCCESS : hip_fail(ctx, e, "hipMalloc (pcap index)");
}

// ev (measurement only, pkt_pcap_index_device_timed): 4 events recorded on `s` before the guess
// kernel and after each of the three kernels.
// partial / count_out (pkt_parse_pcap_host's pieces): index `buf[0, len)` as the prefix of a capture
// (Scratch.partial) and leave the record count in the device word count_out instead of the ctx's.
static int pcap_launch(pkt_ctx_t* ctx, const uint8_t* buf, uint64_t len, uint64_t* offsets, uint32_t* lens,
                       uint64_t cap, hipStream_t s, const uint64_t** count_dev, hipEvent_t* ev = nullptr,
                       bool partial = false, uint64_t* count_out = nullptr, uint32_t r0 = 0,
                       const uint64_t* carry_in = nullptr, uint64_t* carry_out = nullptr) {
    if (!ctx || !buf || (cap && (!offsets || !lens))) return fail(ctx, PKT_ERR_INVALID_ARG, "bad argument");
    if (len < 24) return fail(ctx, PKT_ERR_INVALID_ARG, "pcap shorter than its global header");
    if (reinterpret_cast<uintptr_t>(buf) & 15) return fail(ctx, PKT_ERR_INVALID_ARG, "pcap buffer not 16-byte aligned");
    if (ctx->pc.pending)
        return fail(ctx, PKT_ERR_INVALID_ARG, "a queued capture's outcome has not been taken on this ctx (pkt_parse_pcap_result)");
    const uint64_t K64 = (len + kRegion - 1) / kRegion;
    if (K64 > (1ull << 31) || len >= kValMask) return fail(ctx, PKT_ERR_INVALID_ARG, "pcap too large");
    const uint32_t K = (uint32_t)K64;
    if (r0 >= K || (r0 && !carry_in)) return fail(ctx, PKT_ERR_INVALID_ARG, "bad segment");
    const uint32_t KS = K - r0, nb = (KS + kScanRegions - 1) / kScanRegions;  // the segment's regions [r0, K)
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail(ctx, e, "hipSetDevice");

    // Scratch: the ticket, the scan blocks' states, per-region states, prefixes and record lists.
    // The layout is fixed by the ALLOCATED capacity (k_cap regions, nb_cap block states), not by
    // this call's K: the block-state array must never overlay an earlier call's per-region words
    // (file positions and prefixes a look-back could take for a state published in this epoch).
    PcapScratch& pc = ctx->pc;
    if ((e = pcap_reserve(ctx, K, s)) != hipSuccess) return hip_fail(ctx, e, "hipMalloc (pcap index)");
    if (!pc.ctl) {
        e = hipHostMalloc(reinterpret_cast<void**>(&pc.ctl), 8 * kHostWords, hipHostMallocMapped);
        if (e == hipSuccess) e = hipHostGetDevicePointer(reinterpret_cast<void**>(&pc.ctl_dev), pc.ctl, 0);
        if (e != hipSuccess) return hip_fail(ctx, e, "hipHostMalloc (pcap index)");
    }
    // a new epoch per call (block states of older calls are ignored, not cleared; the block-state
    // area only ever holds epoch-tagged states, reset in full on wrap)
    if (++pc.epoch >= (1u << kEpochBits)) {
        pc.epoch = 1;
        if ((e = hipMemsetAsync(pc.buf, 0, pc.bytes, s)) != hipSuccess) return hip_fail(ctx, e, "hipMemset (pcap index)");
    }
    Scratch S;
    char* p = static_cast<char*>(pc.buf);
    S.ticket = reinterpret_cast<uint32_t*>(p);
    S.blk = reinterpret_cast<BlkDesc*>(p + 64);
    p += 64 + (uint64_t)pc.nb_cap * sizeof(BlkDesc);
    S.rentry = reinterpret_cast<uint64_t*>(p);
    p += 8ull * pc.k_cap;
    S.rexit = reinterpret_cast<uint64_t*>(p);
    p += 8ull * pc.k_cap;
    S.rpre = reinterpret_cast<uint64_t*>(p);
    p += 8ull * pc.k_cap;
    S.rcnt = reinterpret_cast<uint32_t*>(p);
    p += 4ull * pc.k_cap;
    S.list = reinterpret_cast<uint16_t*>(p);
    S.host = pc.ctl_dev;
    S.dev = reinterpret_cast<uint64_t*>(static_cast<char*>(pc.buf) + 16);
    S.count_out = count_out ? count_out : S.dev;
    S.epoch = pc.epoch;
    S.partial = partial ? 1u : 0u;
    S.r0 = r0;
    S.carry_in = carry_in;
    S.carry_out = carry_out;
    for (int i = 0; i < kHostWords; i++) pc.ctl[i] = 0;
    const dim3 blk(256);
    if (ev && (e = hipEventRecord(ev[0], s)) != hipSuccess) return hip_fail(ctx, e, "hipEventRecord");
    const uint32_t ntiles = (KS + kWaves - 1) / kWaves;
    hipLaunchKernelGGL(pcap_guess_kernel, dim3(ntiles), blk, 0, s, buf, len, K, S);
    if (ev && (e = hipEventRecord(ev[1], s)) != hipSuccess) return hip_fail(ctx, e, "hipEventRecord");
    if (!pc.scan_resident) {  // scan blocks the device holds at once
        int per_cu = 0, cus = 0;
        // (the 64-bit build: at least the registers of the 32-bit one, so never more blocks)
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, pcap_scan_kernel<uint64_t>, 256, 0) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device) != hipSuccess)
            per_cu = cus = 0;
        pc.scan_resident = (uint32_t)std::max(1, per_cu * cus);
    }
    // (tickets serialise: 186 device-scope atomics on one word cost the last block ~2.4 us)
    // Forward progress of the blockIdx-ordered look-back: a running block waits only for blocks of
    // LOWER blockIdx, and the dispatcher launches a kernel's workgroups in blockIdx order, so every
    // such block has been dispatched (is resident or finished) — whatever else occupies the device,
    // e.g. the other ctx's capture of the async entries.  The occupancy test keeps the ticket for a
    // grid the device could not hold at once even alone.
    // 32-bit compositions while every position and count of the file fits (region ends included), unless
    // the ctx asks for the 64-bit ones (pkt_ctx_set_pcap_scan64: the form files past 4 GiB take)
    if (!pc.scan64 && len + 2ull * kRegion < (1ull << 32))
        hipLaunchKernelGGL(pcap_scan_kernel<uint32_t>, dim3(nb), blk, 0, s, buf, len, K, nb,
                           nb > pc.scan_resident ? 1 : 0, S, cap, offsets, lens);
    else
        hipLaunchKernelGGL(pcap_scan_kernel<uint64_t>, dim3(nb), blk, 0, s, buf, len, K, nb,
                           nb > pc.scan_resident ? 1 : 0, S, cap, offsets, lens);
    if (ev && (e = hipEventRecord(ev[2], s)) != hipSuccess) return hip_fail(ctx, e, "hipEventRecord");
    // (the records written by the scan blocks themselves, after their look-back, measured slower:
    // 36.9 vs 21.2 + 7.4 us per 2^20-record call — each of the 187 blocks walks its ~5.6K records with
    // a dependent global read per step, where the emit kernel's 3K blocks hide that latency, r04e)
    if (cap)
        hipLaunchKernelGGL((pcap_emit_wide_kernel<kEmitRegions, kEmitPer>), dim3((KS + kEmitRegions - 1) / kEmitRegions), blk,
                           0, s, K, cap, S, offsets, lens, buf);
    if (ev && (e = hipEventRecord(ev[3], s)) != hipSuccess) return hip_fail(ctx, e, "hipEventRecord");
    e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(ctx, e, "pcap index launch");
    if (count_dev) *count_dev = S.count_out;
    return PKT_SUCCESS;
}

// The outcome of the last pcap_launch (the stream has been synchronised).
static int pcap_finish(pkt_ctx_t* ctx, uint64_t* n_out) {
    const PcapScratch& pc = ctx->pc;
    if (!pc.ctl) return fail(ctx, PKT_ERR_INVALID_ARG, "no capture was indexed on this ctx");
    if (!pc.ctl[kHostMagic]) return fail(ctx, PKT_ERR_INVALID_ARG, "bad pcap magic");
    if (pc.ctl[kHostErr]) return fail(ctx, PKT_ERR_INVALID_ARG, "pcap record runs past the end of the buffer");
    *n_out = pc.ctl[kHostTotal];
    return PKT_SUCCESS;
}

int pktgpu_pcap_launch(pkt_ctx_t* ctx, const uint8_t* buf, uint64_t len, uint64_t* offsets, uint32_t* lens,
                       uint64_t cap, hipStream_t s, const uint64_t** count_dev, bool partial, uint64_t* count_out,
                       uint32_t r0, const uint64_t* carry_in, uint64_t* carry_out) {
    return pcap_launch(ctx, buf, len, offsets, lens, cap, s, count_dev, nullptr, partial, count_out, r0, carry_in,
                       carry_out);
}
uint32_t pktgpu_pcap_region_bytes() { return kRegion; }
int pktgpu_pcap_finish(pkt_ctx_t* ctx, uint64_t* n_out) { return pcap_finish(ctx, n_out); }

// The outcome of the capture queued on ctx (waits for it).
int pktgpu_pcap_take(pkt_ctx_t* ctx, uint64_t* n_out) {
    PcapScratch& pc = ctx->pc;
    if (!pc.pending) return fail(ctx, PKT_ERR_INVALID_ARG, "no capture queued on this ctx");
    const hipError_t e = hipStreamSynchronize(pc.pending_stream);
    pc.pending = false;
    pc.pending_stream = nullptr;
    if (e != hipSuccess) return hip_fail(ctx, e, "pkt_parse_pcap_result");
    return pcap_finish(ctx, n_out);
}

extern "C" {

#if PKTGPU_STAMPS
// Diagnostic build only: where the guess kernel writes its per-wave stamps (8 u64 per region).
int pkt_debug_pcap_stamps(void* dev_buf) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_pcap_stamps), &dev_buf, sizeof(dev_buf)) == hipSuccess ? PKT_SUCCESS
                                                                                            : PKT_ERR_HIP;
}
#endif

int pkt_pcap_index_device(pkt_ctx_t* ctx, const uint8_t* buf, uint64_t len, uint64_t* offsets, uint32_t* lens,
                          uint64_t cap, uint64_t* n_out, void* stream) {
    if (!ctx || !n_out) return fail(ctx, PKT_ERR_INVALID_ARG, "bad argument");
    *n_out = 0;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    int rc = pcap_launch(ctx, buf, len, offsets, lens, cap, s, nullptr);
    if (rc != PKT_SUCCESS) return rc;
    const hipError_t e = hipStreamSynchronize(s);
    if (e != hipSuccess) return hip_fail(ctx, e, "pcap index");
    return pcap_finish(ctx, n_out);
}

int pkt_pcap_index_device_timed(pkt_ctx_t* ctx, const uint8_t* buf, uint64_t len, uint64_t* offsets, uint32_t* lens,
                                uint64_t cap, uint64_t* n_out, void* stream, float* kernel_ms) {
    if (!ctx || !n_out || !kernel_ms) return fail(ctx, PKT_ERR_INVALID_ARG, "bad argument");
    *n_out = 0;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail(ctx, e, "hipSetDevice");
    hipEvent_t ev[4] = {};
    for (int k = 0; k < 4 && e == hipSuccess; k++) e = hipEventCreate(&ev[k]);
    int rc = e == hipSuccess ? pcap_launch(ctx, buf, len, offsets, lens, cap, s, nullptr, ev) : hip_fail(ctx, e, "hipEventCreate");
    if (rc == PKT_SUCCESS) {
        if ((e = hipStreamSynchronize(s)) != hipSuccess) rc = hip_fail(ctx, e, "pcap index");
        for (int k = 0; k < 3 && rc == PKT_SUCCESS; k++)
            if ((e = hipEventElapsedTime(&kernel_ms[k], ev[k], ev[k + 1])) != hipSuccess) rc = hip_fail(ctx, e, "hipEventElapsedTime");
        if (rc == PKT_SUCCESS) rc = pcap_finish(ctx, n_out);
    } else {
        (void)hipStreamSynchronize(s);
    }
    for (hipEvent_t x : ev)
        if (x) (void)hipEventDestroy(x);
    return rc;
}

// The index kernels and the counted parse, queued on `stream` (no host wait).
static int parse_pcap_queue(pkt_ctx_t* ctx, const uint8_t* buf, uint64_t len, int entry, const pkt_out_t* out,
                            uint64_t* offsets, uint32_t* lens, uint64_t cap, void* stream) {
    const uint64_t* count_dev = nullptr;
    int rc = pcap_launch(ctx, buf, len, offsets, lens, cap, reinterpret_cast<hipStream_t>(stream), &count_dev);
    if (rc != PKT_SUCCESS) return rc;
    pkt_batch_t b;
    b.slab = buf;
    b.slab_len = len;
    b.offsets = offsets;
    b.lens = lens;
    b.stride = 0;
    b.reserved = 0;
    b.n = cap;
    // one parse launch over cap records whose blocks past the device-produced count exit
    return pktgpu_parse_counted(ctx, &b, entry, out, stream, count_dev);
}

int pkt_parse_pcap_async(pkt_ctx_t* ctx, const uint8_t* buf, uint64_t len, int entry, const pkt_out_t* out,
                         uint64_t* offsets, uint32_t* lens, uint64_t cap, void* stream) {
    if (!ctx || !out || !cap || !offsets || !lens) return fail(ctx, PKT_ERR_INVALID_ARG, "bad argument");
    if (entry < 0 || entry >= PKT_ENTRY_COUNT) return fail(ctx, PKT_ERR_INVALID_ARG, "bad entry");
    if (cap > (1ull << 26)) return fail(ctx, PKT_ERR_INVALID_ARG, "pkt_parse_pcap_async: cap > 2^26 records");
    const int rc = parse_pcap_queue(ctx, buf, len, entry, out, offsets, lens, cap, stream);
    if (rc != PKT_SUCCESS) {
        (void)hipStreamSynchronize(reinterpret_cast<hipStream_t>(stream));  // nothing left in flight
        return rc;
    }
    ctx->pc.pending = true;
    ctx->pc.pending_stream = reinterpret_cast<hipStream_t>(stream);
    return PKT_SUCCESS;
}

int pkt_parse_pcap_result(pkt_ctx_t* ctx, uint64_t* n_out) {
    if (!ctx || !n_out) return fail(ctx, PKT_ERR_INVALID_ARG, "bad argument");
    *n_out = 0;
    return pktgpu_pcap_take(ctx, n_out);
}

int pkt_parse_pcap(pkt_ctx_t* ctx, const uint8_t* buf, uint64_t len, int entry, const pkt_out_t* out,
                   uint64_t* offsets, uint32_t* lens, uint64_t cap, uint64_t* n_out, void* stream) {
    if (!ctx || !out || !n_out || !cap || !offsets || !lens) return fail(ctx, PKT_ERR_INVALID_ARG, "bad argument");
    if (entry < 0 || entry >= PKT_ENTRY_COUNT) return fail(ctx, PKT_ERR_INVALID_ARG, "bad entry");
    *n_out = 0;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    int rc;
    if (cap <= (1ull << 26)) {
        // the host waits once, for the index and the parse together
        if ((rc = parse_pcap_queue(ctx, buf, len, entry, out, offsets, lens, cap, stream)) != PKT_SUCCESS) return rc;
        const hipError_t e = hipStreamSynchronize(s);
        if (e != hipSuccess) return hip_fail(ctx, e, "pkt_parse_pcap");
        return pcap_finish(ctx, n_out);
    }
    if ((rc = pcap_launch(ctx, buf, len, offsets, lens, cap, s, nullptr)) != PKT_SUCCESS) return rc;
    pkt_batch_t b;
    b.slab = buf;
    b.slab_len = len;
    b.offsets = offsets;
    b.lens = lens;
    b.stride = 0;
    b.reserved = 0;
    // batches over 2^26 records take several launches: the count first
    hipError_t e = hipStreamSynchronize(s);
    if (e != hipSuccess) return hip_fail(ctx, e, "pkt_parse_pcap");
    if ((rc = pcap_finish(ctx, n_out)) != PKT_SUCCESS) return rc;
    b.n = std::min(*n_out, cap);
    rc = pktgpu_parse_counted(ctx, &b, entry, out, stream, nullptr, cap);
    if (rc != PKT_SUCCESS) return rc;
    e = hipStreamSynchronize(s);
    return e == hipSuccess ? PKT_SUCCESS : hip_fail(ctx, e, "pkt_parse_pcap");
}

}  // extern "C"
