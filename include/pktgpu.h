/*
 * pktgpu.h — C ABI of the MI355X-native batched packet-header parser.
 *
 * This is the drop-in boundary for packet_rs 0.4.0's decode path:
 *   - the protocol walk `parser::fast::parse` and its 17 sub-entries
 *     (reference src/parser/fast.rs:5-227),
 *   - the `make_header!` MSB-first bit-field getters of the Slice headers
 *     (reference src/headers.rs:195-201 getters, 202-211 bytes(), 252-263 bit_range,
 *      field tables 529-827),
 *   - `Packet::ipv4_checksum` (reference src/packet.rs:93-107, incl. its carry-fold quirk).
 *
 * The reference is a Rust crate with no FFI of its own; these entry points are what a
 * Rust `extern "C"` block binds in place of calling
 * `fast::parse(&[u8]) -> PacketSlice` once per packet.  Everything here is plain C:
 * pointers, sizes and status codes.  No HIP, torch or C++ types cross the boundary
 * (streams are passed as `void*` = hipStream_t, 0 = the null stream).
 *
 * Errors: every function returns an int, 0 on success and a negative PKT_ERR_* code
 * otherwise.  Nothing panics or aborts across the ABI (the reference panics on short
 * input, fast.rs:6 and every `&arr[0..X::size()]`; here that is a per-packet
 * PKT_TRUNCATED status instead).
 */
#ifndef PKTGPU_H
#define PKTGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PKTGPU_ABI_VERSION 5

/* Maximum number of headers recorded per packet.  The reference recursion is unbounded
 * (fast.rs:53 VLAN stacks, :69 MPLS stacks, :89/:92/:104/:107 IP-in-IP, :168/:186/:219
 * tunnels back to Ethernet); chains longer than this report PKT_DEPTH_LIMIT. */
#define PKT_MAX_HDRS 16

/* Call-level return codes. */
#define PKT_SUCCESS            0
#define PKT_ERR_INVALID_ARG   -1
#define PKT_ERR_HIP           -2
#define PKT_ERR_NO_DEVICE     -3
#define PKT_ERR_UNSUPPORTED   -4
#define PKT_ERR_GATHER_ROWS   -5  /* pkt_mgpu_synchronize: a packet had more headers than the fixed gather rows */

/* Per-packet status (out->status). */
typedef enum pkt_status {
    PKT_OK          = 0, /* walk reached `accept` (fast.rs:223-227) */
    PKT_TRUNCATED   = 1, /* the reference would panic on a slice index (Q7) */
    PKT_DEPTH_LIMIT = 2  /* more than PKT_MAX_HDRS headers (build-only bound) */
} pkt_status_t;

/* Header type ids.  Names (pkt_hdr_name) are the reference's `Header::name()` strings,
 * i.e. the make_header! identifiers of headers.rs:529-827. */
typedef enum pkt_hdr_type {
    PKT_HDR_NONE               = 0,
    PKT_HDR_ETHER              = 1,  /* headers.rs:530-540  14 B */
    PKT_HDR_VLAN               = 2,  /* headers.rs:543-552   4 B */
    PKT_HDR_IPV4               = 3,  /* headers.rs:555-574  20 B */
    PKT_HDR_IPV6               = 4,  /* headers.rs:577-592  40 B */
    PKT_HDR_ICMP               = 5,  /* headers.rs:595-603   4 B */
    PKT_HDR_TCP                = 6,  /* headers.rs:606-622  20 B */
    PKT_HDR_UDP                = 7,  /* headers.rs:625-634   8 B */
    PKT_HDR_ARP                = 8,  /* headers.rs:637-653  28 B */
    PKT_HDR_VXLAN              = 9,  /* headers.rs:656-665   8 B */
    PKT_HDR_DOT3               = 10, /* headers.rs:668-678  14 B */
    PKT_HDR_LLC                = 11, /* headers.rs:681-689   3 B */
    PKT_HDR_SNAP               = 12, /* headers.rs:692-699   5 B */
    PKT_HDR_GRE                = 13, /* headers.rs:702-716   4 B */
    PKT_HDR_GRE_CHKSUM_OFFSET  = 14, /* headers.rs:719-726   4 B */
    PKT_HDR_GRE_SEQUENCE_NUM   = 15, /* headers.rs:729-735   4 B */
    PKT_HDR_GRE_KEY            = 16, /* headers.rs:738-744   4 B */
    PKT_HDR_ERSPAN2            = 17, /* headers.rs:747-760   8 B */
    PKT_HDR_ERSPAN3            = 18, /* headers.rs:763-782  12 B */
    PKT_HDR_ERSPAN_PLATFORM    = 19, /* headers.rs:785-792   8 B */
    PKT_HDR_STP                = 20, /* headers.rs:795-815  35 B (never produced by the walk) */
    PKT_HDR_MPLS               = 21, /* headers.rs:818-827   4 B */
    PKT_HDR_COUNT              = 22
} pkt_hdr_type_t;

/* Entry points: one per public function of parser::fast (fast.rs).  Parsing a batch with
 * entry E is `fast::parse_E(&pkt[..])` for every packet. */
typedef enum pkt_entry {
    PKT_ENTRY_PARSE     = 0,  /* fast::parse          fast.rs:5   (Dot3 if bytes 12..13 < 1500) */
    PKT_ENTRY_DOT3      = 1,  /* fast::parse_dot3     fast.rs:13  */
    PKT_ENTRY_LLC       = 2,  /* fast::parse_llc      fast.rs:19  */
    PKT_ENTRY_SNAP      = 3,  /* fast::parse_snap     fast.rs:29  */
    PKT_ENTRY_ETHERNET  = 4,  /* fast::parse_ethernet fast.rs:35  */
    PKT_ENTRY_VLAN      = 5,  /* fast::parse_vlan     fast.rs:49  */
    PKT_ENTRY_MPLS      = 6,  /* fast::parse_mpls     fast.rs:63  */
    PKT_ENTRY_MPLS_BOS  = 7,  /* fast::parse_mpls_bos fast.rs:74  */
    PKT_ENTRY_IPV4      = 8,  /* fast::parse_ipv4     fast.rs:84  */
    PKT_ENTRY_IPV6      = 9,  /* fast::parse_ipv6     fast.rs:99  */
    PKT_ENTRY_GRE       = 10, /* fast::parse_gre      fast.rs:114 */
    PKT_ENTRY_ERSPAN2   = 11, /* fast::parse_erspan2  fast.rs:166 */
    PKT_ENTRY_ERSPAN3   = 12, /* fast::parse_erspan3  fast.rs:172 */
    PKT_ENTRY_ARP       = 13, /* fast::parse_arp      fast.rs:193 */
    PKT_ENTRY_ICMP      = 14, /* fast::parse_icmp     fast.rs:198 */
    PKT_ENTRY_TCP       = 15, /* fast::parse_tcp      fast.rs:203 */
    PKT_ENTRY_UDP       = 16, /* fast::parse_udp      fast.rs:208 */
    PKT_ENTRY_VXLAN     = 17, /* fast::parse_vxlan    fast.rs:218 */
    PKT_ENTRY_COUNT     = 18
} pkt_entry_t;

/* A batch of packets resident in device memory (the caller owns every buffer).
 *  - Fixed-stride slab: offsets == NULL; packet i starts at slab + i*stride.  Its length is
 *    lens[i] when lens != NULL, else `stride`.
 *  - Indexed slab (e.g. a pcap file copied as-is): offsets[i] / lens[i] (both required)
 *    give each packet's byte range inside the slab.
 *  - A packet is the bytes of that range that lie inside [slab, slab + slab_len): its length
 *    is clamped to the slab end (a slot past the end is an empty packet) and to 65535 (the
 *    u16 offset/length columns).
 * The slab pointer must be 16-byte aligned; the kernels may read up to 15 bytes past a
 * packet's end but never past round_up(slab + slab_len, 16) (always inside a hipMalloc /
 * torch allocation, whose granularity is >= 256 B). */
typedef struct pkt_batch {
    const uint8_t  *slab;      /* device */
    uint64_t        slab_len;  /* bytes */
    const uint64_t *offsets;   /* device, [n] or NULL */
    const uint32_t *lens;      /* device, [n] or NULL */
    uint32_t        stride;    /* bytes between packets when offsets == NULL */
    uint32_t        reserved;
    uint64_t        n;         /* number of packets */
} pkt_batch_t;

/* Output columns (struct-of-arrays, device memory, caller-owned).  Every pointer may be
 * NULL: that column is then neither computed nor written (the reference's getters are
 * lazy, headers.rs:195-201 — a caller asks only for what it reads).
 *
 * Chain columns = PacketSlice (lib.rs:136-140, packet.rs:714-761):
 *   hdr_type/hdr_off are slot-major: slot j of packet i lives at [j*n + i]; slots
 *   j < n_hdrs[i] hold the chain; later slots are unspecified (not written for a parsed packet;
 *   a packet that fails may have written some before its failing header).  List order is the reference's `Vec::insert(0, ..)` order,
 *   i.e. wire order except GRE options (Q2: GRE, SeqNum, Key, ChksumOffset).
 *   hdr_off is the header's byte offset from the start of the packet (the Slice's
 *   pointer, headers.rs:187-192); payload_off/payload_len = PacketSlice::payload().
 *   On PKT_TRUNCATED / PKT_DEPTH_LIMIT no PacketSlice exists (the reference panics):
 *   n_hdrs = 0, hdr_mask = 0, payload_off = payload_len = 0 and every field column is 0.
 *
 * Field columns = the Slice getters of the FIRST header of that type in the list
 * (Packet's Index<&str> returns the first match, packet.rs:64-66 — Q11).  Values are the
 * reference's u64 getter results narrowed to the field's natural width; 0 when the packet
 * has no such header (check hdr_mask).  ipv6_src/dst are the 16 raw bytes that
 * `bytes(msb, lsb)` returns (headers.rs:202-211; the u64 getter is Q8).
 * ipv4_csum_calc = Packet::ipv4_checksum over that IPv4 header's 20 bytes (packet.rs:93-107). */
typedef struct pkt_out {
    /* chain */
    uint8_t  *status;          /* pkt_status_t */
    uint8_t  *n_hdrs;
    uint8_t  *hdr_type;        /* [PKT_MAX_HDRS][n] */
    uint16_t *hdr_off;         /* [PKT_MAX_HDRS][n] */
    uint16_t *payload_off;
    uint16_t *payload_len;
    uint32_t *hdr_mask;        /* bit t set iff a header of type t is in the list */
    /* Ether (headers.rs:530-540) */
    uint64_t *eth_dst;
    uint64_t *eth_src;
    uint16_t *eth_etype;
    /* Vlan (headers.rs:543-552) */
    uint8_t  *vlan_pcp;
    uint8_t  *vlan_cfi;
    uint16_t *vlan_vid;
    uint16_t *vlan_etype;
    /* IPv4 (headers.rs:555-574) */
    uint8_t  *ipv4_version;
    uint8_t  *ipv4_ihl;
    uint8_t  *ipv4_diffserv;
    uint16_t *ipv4_total_len;
    uint16_t *ipv4_identification;
    uint8_t  *ipv4_flags;
    uint16_t *ipv4_frag_startset;
    uint8_t  *ipv4_ttl;
    uint8_t  *ipv4_protocol;
    uint16_t *ipv4_header_checksum;
    uint32_t *ipv4_src;
    uint32_t *ipv4_dst;
    uint16_t *ipv4_csum_calc;  /* Packet::ipv4_checksum (packet.rs:93-107) */
    /* IPv6 (headers.rs:577-592) */
    uint8_t  *ipv6_version;
    uint8_t  *ipv6_traffic_class;
    uint32_t *ipv6_flow_label;
    uint16_t *ipv6_payload_len;
    uint8_t  *ipv6_next_hdr;
    uint8_t  *ipv6_hop_limit;
    uint8_t  *ipv6_src;        /* [n][16] */
    uint8_t  *ipv6_dst;        /* [n][16] */
    /* TCP (headers.rs:606-622) */
    uint16_t *tcp_src;
    uint16_t *tcp_dst;
    uint32_t *tcp_seq_no;
    uint32_t *tcp_ack_no;
    uint8_t  *tcp_data_startset;
    uint8_t  *tcp_res;
    uint8_t  *tcp_flags;
    uint16_t *tcp_window;
    uint16_t *tcp_checksum;
    uint16_t *tcp_urgent_ptr;
    /* UDP (headers.rs:625-634) */
    uint16_t *udp_src;
    uint16_t *udp_dst;
    uint16_t *udp_length;
    uint16_t *udp_checksum;
} pkt_out_t;

/* A field request for pkt_extract_fields: bits [start..=end] (MSB-first from the header's
 * first byte, the make_header! convention) of the `occurrence`-th header of `hdr_type`
 * in the chain (0 = first, as Packet's Index<&str>).  Any bit range is allowed, so a
 * user-defined make_header! field (lib.rs:81-103) is extracted the same way.  Widths
 * above 64 bits follow bit_range's release-build result (headers.rs:262, Q8). */
typedef struct pkt_field_spec {
    uint8_t  hdr_type;
    uint8_t  occurrence;
    uint16_t start;
    uint16_t end;
    uint16_t reserved;
} pkt_field_spec_t;

/* Chain columns produced by pkt_parse_batch, as input to pkt_extract_fields. */
typedef struct pkt_chain {
    const uint8_t  *n_hdrs;    /* [n] */
    const uint8_t  *hdr_type;  /* [PKT_MAX_HDRS][n] */
    const uint16_t *hdr_off;   /* [PKT_MAX_HDRS][n] */
} pkt_chain_t;

typedef struct pkt_ctx pkt_ctx_t;

/* ---- metadata (host only, no device needed) ---- */
int         pkt_abi_version(void);
/* sizeof the ABI structs, so a foreign binding (Rust/ctypes) can check its layout. */
size_t      pkt_sizeof_batch(void);
size_t      pkt_sizeof_out(void);
size_t      pkt_sizeof_field_spec(void);
/* Header::name() (headers.rs:218-220); NULL for an unknown id. */
const char *pkt_hdr_name(int hdr_type);
/* <Hdr>::size() (headers.rs:212-214); 0 for an unknown id. */
int         pkt_hdr_size(int hdr_type);
/* Field table of a header type (make_header! field list, headers.rs:529-827). */
int         pkt_hdr_field_count(int hdr_type);
int         pkt_hdr_field(int hdr_type, int idx, const char **name, uint16_t *start, uint16_t *end);
const char *pkt_status_name(int status);
const char *pkt_entry_name(int entry);   /* "parse", "parse_ethernet", ... */

/* ---- context ---- */
/* Binds to HIP device `device`.  No per-call allocation happens after creation. */
int         pkt_ctx_create(int device, pkt_ctx_t **ctx);
int         pkt_ctx_destroy(pkt_ctx_t *ctx);
const char *pkt_ctx_last_error(const pkt_ctx_t *ctx);
/* Tuning knob: packets staged per wave window (bytes of each packet copied to LDS).
 * 0 = automatic.  Values are rounded to a multiple of 16 and clamped to [16, 256]. */
int         pkt_ctx_set_window(pkt_ctx_t *ctx, uint32_t window_bytes);
/* Fast path (default on).  For entries PARSE and ETHERNET, a packet that starts on a 16-byte
 * boundary and whose first bytes read Ether / 0-2 x Vlan / IPv4 / UDP (dst != 4789) or TCP, long
 * enough for every header, has its chain decided by a few compares on the registers its bytes
 * were loaded into, so it skips the walk.  Results are identical to the walk's (the same fast.rs
 * path; the parity tests run with it forced on and off).  0 = off, 1 = on. */
int         pkt_ctx_set_fastpath(pkt_ctx_t *ctx, int enable);

/* Tuning knob: how packet bytes reach LDS.  0 = automatic (currently 1), 1 = per-lane windows of
 * pkt_ctx_set_window bytes (deeper headers read through L2), 2 = wave spans: each wave of 64
 * packets copies the contiguous byte range its packets occupy (up to 16 KiB; else per-lane
 * windows) into LDS by LDS-DMA and walks every header from there.  Results are identical in every
 * mode.  Any other value is PKT_ERR_INVALID_ARG. */
int         pkt_ctx_set_staging(pkt_ctx_t *ctx, int mode);

/* Tuning knob: walk schedule.  0 = automatic (lockstep for indexed batches, waterfall for fixed
 * stride), 1 = waterfall (each iteration advances the lanes in one state: one case per header
 * when a wave's packets share a layout), 2 = lockstep (every lane advances one header per
 * iteration: mixed chains in a wave cost their longest chain, not their number of distinct
 * states).  Results are identical in every mode. */
int         pkt_ctx_set_walk(pkt_ctx_t *ctx, int mode);

/* Tuning knob: bytes of file per copied piece of pkt_parse_pcap_host (pinned columns): 0 = the
 * default (16 MiB), else any value >= 4096; a capture is cut into at most 1024 pieces (larger pieces
 * for files past 1024 x the knob).  Results are identical for every value. */
int         pkt_ctx_set_host_piece(pkt_ctx_t *ctx, uint64_t bytes);

/* Tuning / test knob: 1 = the device pcap indexer composes its regions' states in 64-bit positions
 * and counts for every file (the form files of 4 GiB and more always take), 0 (default) = 32-bit ones
 * for files under 4 GiB.  Results are identical either way. */
int         pkt_ctx_set_pcap_scan64(pkt_ctx_t *ctx, int enable);

/* ---- the hot path ---- */
/* fast::parse_<entry> over every packet of `batch`, writing the requested columns of `out`.
 * Asynchronous on `stream`; returns after the launch.  `batch` and `out` may also point into pinned
 * host memory from pkt_host_alloc (mapped into the device): the kernel then reads and writes it
 * over the link directly — zero copy, still asynchronous (see pkt_parse_host for the blocking
 * form; pkt_ctx_set_staging(ctx, 2) suits host-resident indexed batches). */
int pkt_parse_batch(pkt_ctx_t *ctx, const pkt_batch_t *batch, int entry,
                    const pkt_out_t *out, void *stream);

/* `nbatch` independent batches: batches[k] -> outs[k], as nbatch pkt_parse_batch calls would write
 * them.  When the batches have the same n (<= 2^26), stride and layout (indexed or not, lens or not),
 * nbatch <= 16, and every batch's column pointers lie at one common byte distance from batch 0's (one
 * packed output buffer per batch, pkt_out_packed, qualifies), it is ONE launch whose grid covers every
 * batch's tiles, so the launch's ramp and drain are paid once; otherwise one launch per batch.
 * Asynchronous on `stream`. */
int pkt_parse_batches(pkt_ctx_t *ctx, const pkt_batch_t *batches, uint32_t nbatch, int entry,
                      const pkt_out_t *outs, void *stream);

/* ---- host-memory path ----
 * The reference's path starts and ends in host memory (a pcap file, a NIC ring).  One call moves
 * a HOST batch through the device: `batch` (slab, offsets, lens) and `out` (column pointers, the
 * pkt_out_t layout of pkt_parse_batch with slot columns strided by batch->n) are host memory.
 * The batch is cut into chunks of `chunk` packets (0 = 262144; 131072 with pinned columns)
 * pipelined over three streams of the ctx: the copy-in of chunk k+1 and the copy-out of chunk k-1
 * overlap the parse of chunk k.  Indexed chunks copy the byte span their records cover.  When the
 * slab, offsets, lens and every requested column are pinned memory from pkt_host_alloc, there are no
 * copies at all: one launch reads the slab and writes the columns over the link directly (zero copy;
 * `chunk` unused).  When only the columns are pinned, a chunk's columns go out by one kernel writing
 * them over the link in 16-byte chunks (else one copy per column).  Pageable buffers work, staged by
 * the runtime.  Blocks until every output is in host memory.  One host call at a time per ctx. */
int pkt_parse_host(pkt_ctx_t *ctx, const pkt_batch_t *batch, int entry, const pkt_out_t *out,
                   uint64_t chunk);
/* The capture path of tests/pcap.rs:7-37 end to end, host memory in and out: a pcap file in HOST
 * memory (`buf`, `len` bytes; pinned from pkt_host_alloc for the full link rate) is copied to the
 * device, indexed there (pkt_pcap_index_device: same records, count, cap behaviour and errors
 * as pkt_pcap_index) and parsed with `entry` (an indexed batch over the file in place); the requested
 * columns of `out` are HOST memory sized for `cap` records, slot columns strided by cap
 * ([PKT_MAX_HDRS][cap]).  Pinned columns are written by the parse kernel over the link directly; others
 * through the staged pipeline of pkt_parse_host.  offsets / lens (HOST, [cap], may be NULL) receive
 * the records' (data offset, incl_len).  *n_out = the record count (> cap: only the first cap are
 * parsed).  Blocking.  One host call at a time per ctx.
 * With pinned columns and a file longer than one piece (pkt_ctx_set_host_piece) the file is copied in
 * pieces and parsed while it arrives: once piece k has landed, the bytes it adds are indexed from the
 * previous piece's carry on the device (the first record it could not count and its record count —
 * pkt_pcap_stream_*'s steps; the file is indexed once, O(file), whatever the piece count; a record
 * running past a piece's end belongs to a later piece) and the records it completes are parsed, their
 * columns flowing out over the link while piece k + 1 flows in.  The last piece ends the file, indexed
 * with pkt_pcap_index's errors; on such an error the records of the earlier pieces may already be
 * written to `out`. */
int pkt_parse_pcap_host(pkt_ctx_t *ctx, const uint8_t *buf, uint64_t len, int entry, const pkt_out_t *out,
                        uint64_t *offsets, uint32_t *lens, uint64_t cap, uint64_t *n_out);
/* pkt_parse_pcap_host without the wait, for a stream of captures (cap <= 2^26, every column of `out`
 * in pinned memory from pkt_host_alloc, no index output): queues pkt_parse_pcap_host's pieces — the
 * copies in, the prefix indexes, the parses and the column exports — on the ctx's own streams and
 * returns; `buf` and `out` must stay untouched until pkt_parse_pcap_host_result, which waits for them
 * and gives the outcome as pkt_parse_pcap_host's (*n_out = the record count; on an error in the last
 * record the earlier pieces' records may be written).  One capture in flight per ctx (as
 * pkt_parse_pcap_async): two ctxs keep one capture's copy in flowing while the other's columns flow
 * out. */
int pkt_parse_pcap_host_async(pkt_ctx_t *ctx, const uint8_t *buf, uint64_t len, int entry, const pkt_out_t *out,
                              uint64_t cap);
int pkt_parse_pcap_host_result(pkt_ctx_t *ctx, uint64_t *n_out);
/* Pinned (page-locked) host memory for pkt_parse_host buffers. */
int pkt_host_alloc(pkt_ctx_t *ctx, uint64_t bytes, void **p);
int pkt_host_free(pkt_ctx_t *ctx, void *p);

/* Batched make_header! getter: for each spec s and packet i, values[s][i] = the field of
 * the chain's matching header (0 and found[s][i] = 0 when absent).  `values` and `found`
 * are HOST arrays of `nspec` DEVICE pointers, each to n elements; found may be NULL and
 * so may any found[s]. */
int pkt_extract_fields(pkt_ctx_t *ctx, const pkt_batch_t *batch, const pkt_chain_t *chain,
                       const pkt_field_spec_t *specs, uint32_t nspec,
                       uint64_t *const *values, uint8_t *const *found, void *stream);

/* PacketSlice::to_vec / Packet::to_vec (packet.rs:733-740, 385-392) of every parsed packet:
 * its header slices in LIST order, then its payload, written to dst + dst_offsets[i]
 * (dst_offsets == NULL: the input batch's own layout, i*stride or offsets[i]).  With two or
 * more GRE options the list order differs from wire order (Q2), so the bytes are reordered
 * exactly as the reference's round trip reorders them.  `parsed` holds the chain columns of a
 * pkt_parse_batch over the same batch (status, n_hdrs, hdr_type, hdr_off, payload_off,
 * payload_len are read; the rest is ignored).  out_len[i] = bytes written (0 and nothing
 * written for a packet whose status is not PKT_OK); out_len may be NULL.
 * In the input's own layout (dst_offsets == NULL) of an indexed batch whose records share no
 * 16-byte chunk of the slab (e.g. a capture, with its record headers between the packets), a
 * destination chunk that holds a packet's first or last bytes is read, merged and written back
 * whole: the dst bytes between records inside such a chunk are rewritten with their own values,
 * not atomically — no other stream may write them while the call runs. */
int pkt_to_vec_batch(pkt_ctx_t *ctx, const pkt_batch_t *batch, const pkt_out_t *parsed,
                     uint8_t *dst, uint64_t dst_len, const uint64_t *dst_offsets,
                     uint32_t *out_len, void *stream);

/* Batched header rewrite, in place in the slab (the slab of `batch` must be writable):
 * `<Hdr>::set_<field>(v)` (headers.rs:340-344 -> set_bit_range 315-324) for each spec, in spec
 * order, on the spec's header of every packet's chain.  The low (end-start+1) bits of
 * values[s][i] go to bits [start..=end] (bits of a field wider than 64 above the value's 64
 * bits become 0, as set_bit_range shifts the u64 right once per bit).  Packets whose chain lacks
 * the header are untouched.  `values` is a HOST array of nspec DEVICE pointers ([n] each).
 * The packets of one batch must not overlap: a packet's bytes may be stored back whole (with
 * their values unchanged outside the fields set), never bytes outside [offset, offset + len). */
int pkt_set_fields(pkt_ctx_t *ctx, const pkt_batch_t *batch, const pkt_chain_t *chain,
                   const pkt_field_spec_t *specs, uint32_t nspec, const uint64_t *const *values,
                   void *stream);

/* pkt_set_fields followed, in the same launch, by pkt_ipv4_update_checksum of the
 * `ipv4_occurrence`-th IPv4 header (< 0: no checksum refresh; nspec may then be 0 for a refresh
 * alone), as one pass over each packet's bytes.  The reference's update+clone loop
 * (tests/lib.rs:778-787) is setters only (set_etype; ipv4_occurrence < 0); the checksum refresh is
 * what the create_* builders do after setting IPv4 fields (utils.rs:233-236). */
int pkt_set_fields_csum(pkt_ctx_t *ctx, const pkt_batch_t *batch, const pkt_chain_t *chain,
                        const pkt_field_spec_t *specs, uint32_t nspec, const uint64_t *const *values,
                        int32_t ipv4_occurrence, void *stream);

/* `ipv4.set_header_checksum(Packet::ipv4_checksum(ipv4.to_vec()))` (utils.rs:233-236;
 * packet.rs:93-107 with the Q1 fold) on the `occurrence`-th IPv4 header of every packet, in
 * place.  Packets without that header are untouched. */
int pkt_ipv4_update_checksum(pkt_ctx_t *ctx, const pkt_batch_t *batch, const pkt_chain_t *chain,
                             uint32_t occurrence, void *stream);

/* Batched packet generation, clone step (`pkt.clone().to_vec()` of tests/lib.rs:770-776 for n
 * copies): writes the `len`-byte DEVICE packet `src` n times, at dst + i*stride, and zero-fills
 * the rest of each stride slot.  Follow with pkt_parse_batch (chain), pkt_set_fields and
 * pkt_ipv4_update_checksum to vary fields per packet (the update+clone workload, 778-787). */
int pkt_broadcast(pkt_ctx_t *ctx, const uint8_t *src, uint32_t len, uint64_t n, uint32_t stride,
                  uint8_t *dst, void *stream);

/* ---- batched packet generation: the pktgen loop (tests/lib.rs:756-788) ----
 * The reference builds a packet with a `utils::create_*` builder (utils.rs:7-876), clones it,
 * updates fields through the setters (headers.rs:340-344 -> set_bit_range 315-324) and serialises
 * it with to_vec, once per packet.  Here the builder's bytes are a TEMPLATE: pkt_gen_create parses
 * it once on the device (entry as for pkt_parse_batch) and places every generator field by its
 * (header, occurrence, bits) in the template's chain (Index<&str> semantics, packet.rs:64-66);
 * pkt_gen_run then writes n packets at dst + i*stride in one pass (the template, every field set
 * to its value for that packet, the listed IPv4 checksums refreshed with Packet::ipv4_checksum
 * (packet.rs:93-107) as the builders do, utils.rs:233-236; the rest of each stride slot zeroed).
 * A field gets the value's low (end-start+1) <= 64 bits, as set_bit_range does.  Packet i of a
 * run has global index g = first + i; the value of a field is
 *   PKT_GEN_VALUES  values[f][i]                   (a DEVICE array per field, given to pkt_gen_run)
 *   PKT_GEN_INC     base + step * (g % count)      (count 0: base + step * g; the reference's
 *                                                   update loop is base 0, step 1, count 0xFFFF)
 *   PKT_GEN_RANDOM  splitmix64(base + g)           (z = x + 0x9E3779B97F4A7C15;
 *                   z = (z ^ z>>30) * 0xBF58476D1CE4E5B9; z = (z ^ z>>27) * 0x94D049BB133111EB;
 *                   z ^ z>>31) — base is the seed.
 * Fields apply in order (a later field wins where two overlap); checksum refreshes come last. */
typedef enum pkt_gen_kind {
    PKT_GEN_VALUES = 0,
    PKT_GEN_INC    = 1,
    PKT_GEN_RANDOM = 2
} pkt_gen_kind_t;
typedef struct pkt_gen_field {
    pkt_field_spec_t field;  /* header type, occurrence, bits [start..=end], width 1..64 */
    uint32_t kind;           /* pkt_gen_kind_t */
    uint32_t reserved;
    uint64_t base;
    uint64_t step;
    uint64_t count;
} pkt_gen_field_t;
typedef struct pkt_gen pkt_gen_t;
size_t pkt_sizeof_gen_field(void);
/* `tpl` is HOST memory (len bytes, <= 65535); at most 32 fields.  ipv4_csum_mask bit k refreshes
 * the checksum of the template's k-th IPv4 header (at most 8).  Blocking (one template parse).
 * Fails with PKT_ERR_INVALID_ARG if the template does not parse to PKT_OK or lacks a named header. */
int pkt_gen_create(pkt_ctx_t *ctx, const uint8_t *tpl, uint32_t len, int entry,
                   const pkt_gen_field_t *fields, uint32_t nfields, uint32_t ipv4_csum_mask,
                   pkt_gen_t **gen);
/* Writes packets first .. first+n-1 to `dst` (device, 16-byte aligned, n*stride bytes; stride a
 * multiple of 16 and >= the template length).  `values` is a HOST array with one DEVICE pointer
 * ([n] uint64) per field, used by PKT_GEN_VALUES fields (may be NULL when there are none).
 * Asynchronous on `stream`. */
int pkt_gen_run(pkt_gen_t *gen, uint64_t first, uint64_t n, uint32_t stride,
                const uint64_t *const *values, uint8_t *dst, void *stream);
int pkt_gen_destroy(pkt_gen_t *gen);

/* Packet::ipv4_checksum (packet.rs:93-107) over n headers of 20 bytes at a fixed stride
 * in device memory: out[i] = checksum(hdrs + i*stride). */
int pkt_ipv4_checksum_batch(pkt_ctx_t *ctx, const uint8_t *hdrs, uint32_t stride, uint64_t n,
                            uint16_t *out, void *stream);

/* ---- host-side helpers ---- */
/* Index a pcap byte buffer in the tests/pcap.rs:7-37 format (LE magic d4 c3 b2 a1, 24-byte
 * global header, 16-byte record headers).  Writes up to `cap` record (data offset, incl_len)
 * pairs and the record count to *n_out (which can exceed cap: call again with a larger cap).
 * Returns PKT_ERR_INVALID_ARG on a bad magic or a record running past `len`. */
int pkt_pcap_index(const uint8_t *buf, uint64_t len, uint64_t *offsets, uint32_t *lens,
                   uint64_t cap, uint64_t *n_out);

/* pkt_pcap_index for a pcap file resident in DEVICE memory (`buf` 16-byte aligned, readable up to
 * round_up(len, 16)): same records, count, cap behaviour and errors, with `offsets` / `lens` in
 * device memory — ready for an indexed pkt_batch_t over the same buffer.  The sequential record
 * chain is recovered per 4 KiB region by a speculative guess plus exact fix-up rounds
 * (pktgpu_pcap.hip).  Blocking: returns once *n_out is known (work is ordered on `stream`). */
int pkt_pcap_index_device(pkt_ctx_t *ctx, const uint8_t *buf, uint64_t len, uint64_t *offsets,
                          uint32_t *lens, uint64_t cap, uint64_t *n_out, void *stream);
/* pkt_pcap_index_device with the index's three kernels timed by HIP events recorded between
 * them on `stream` (measurement): kernel_ms[0..2] = guess, scan, emit (emit ~0 when cap == 0). */
int pkt_pcap_index_device_timed(pkt_ctx_t *ctx, const uint8_t *buf, uint64_t len, uint64_t *offsets,
                                uint32_t *lens, uint64_t cap, uint64_t *n_out, void *stream,
                                float *kernel_ms);

/* The capture path of tests/pcap.rs:7-37 on a pcap file already in DEVICE memory, in one call:
 * pkt_pcap_index_device into offsets / lens (device, [cap], cap >= 1), then fast::parse_<entry> of
 * every record (an indexed batch over `buf` in place) into `out` (device columns sized for cap
 * records, slot columns strided by cap).  The parse takes the record count from the device (its
 * blocks past it exit), so the host waits once, for both; *n_out = the record count (> cap: only
 * the first cap records are indexed and parsed).  Errors as pkt_pcap_index_device (nothing is
 * parsed then).  Blocking. */
int pkt_parse_pcap(pkt_ctx_t *ctx, const uint8_t *buf, uint64_t len, int entry, const pkt_out_t *out,
                   uint64_t *offsets, uint32_t *lens, uint64_t cap, uint64_t *n_out, void *stream);

/* pkt_parse_pcap without the host wait, for a stream of captures: queues the index kernels and the
 * counted parse on `stream` (cap <= 2^26) and returns.  pkt_parse_pcap_result waits for them and
 * gives the outcome (the record count, or the errors of pkt_pcap_index_device; after an error
 * nothing was parsed).  The ctx's index scratch belongs to the queued capture until its result is
 * taken: one capture in flight per ctx (two in flight = two ctxs, e.g. one per stream); another
 * index call on the ctx before that fails with PKT_ERR_INVALID_ARG. */
int pkt_parse_pcap_async(pkt_ctx_t *ctx, const uint8_t *buf, uint64_t len, int entry, const pkt_out_t *out,
                         uint64_t *offsets, uint32_t *lens, uint64_t cap, void *stream);
int pkt_parse_pcap_result(pkt_ctx_t *ctx, uint64_t *n_out);

/* Packet::ipv4_checksum on the host (same arithmetic as the device kernel). */
uint16_t pkt_ipv4_checksum_host(const uint8_t *hdr, size_t len);

/* The largest n_hdrs[i] over n packets (`n_hdrs`: a device column from pkt_parse_batch): the slot
 * rows of hdr_type / hdr_off that hold data — a PacketSlice holds exactly its headers (lib.rs:136-140),
 * so a copy or gather of a batch's chain moves rows [0, *max_out) only.  Blocking (waits for
 * `stream`).  One such call at a time per ctx. */
int pkt_chain_max_hdrs(pkt_ctx_t *ctx, const uint8_t *n_hdrs, uint64_t n, uint32_t *max_out, void *stream);

/* PacketSlice of packet i of a parsed batch whose chain columns are in HOST memory (pkt_parse_host's
 * output, or device columns copied back): for k < *n_hdrs, types[k] / offs[k] = the k-th header of
 * the PacketSlice's list (its type id and its byte offset in the packet: the Slice the reference's
 * `insert` put at position k, lib.rs:136-140, packet.rs:724-726), and the payload is packet bytes
 * [*payload_off, *payload_off + *payload_len) (`set_payload`, packet.rs:728-731).  `out` must hold
 * status, n_hdrs, hdr_type, hdr_off, payload_off and payload_len (slot columns strided by n).  Returns
 * the packet's pkt_status_t (>= 0; on a status other than PKT_OK the reference panicked, there is no
 * PacketSlice, and *n_hdrs = *payload_off = *payload_len = 0), or PKT_ERR_INVALID_ARG.  Host only. */
int pkt_view(const pkt_out_t *out, uint64_t n, uint64_t i, uint8_t types[PKT_MAX_HDRS],
             uint16_t offs[PKT_MAX_HDRS], uint32_t *n_hdrs, uint16_t *payload_off, uint16_t *payload_len);

/* ---- packed output buffers (host only, no device needed) ----
 * A column mask selects pkt_out_t members: bit k = the k-th pointer of pkt_out_t (0 = status,
 * ..., 48 = udp_checksum).  The packed layout puts every selected column of an n-packet output in
 * one buffer, each column starting on a 256-byte boundary: the per-packet columns in pkt_out_t
 * order, then the slot columns hdr_type and hdr_off ([PKT_MAX_HDRS][n] each) last.  One buffer per
 * shard is what the multi-GPU gather moves; with only the used slot rows (pkt_out_packed_pieces)
 * that is at most two contiguous pieces. */
#define PKT_COL(k)      (1ull << (k))
#define PKT_COLS_ALL    ((1ull << 49) - 1)
#define PKT_COLS_CHAIN  0x7Full               /* status .. hdr_mask */
#define PKT_COLS_ETHER  (0x7ull << 7)
#define PKT_COLS_VLAN   (0xFull << 10)
#define PKT_COLS_IPV4   (0x1FFFull << 14)
#define PKT_COLS_IPV6   (0xFFull << 27)
#define PKT_COLS_TCP    (0x3FFull << 35)
#define PKT_COLS_UDP    (0xFull << 45)
/* Fills `out` with the selected columns' pointers inside `base` (NULL columns elsewhere; `base`
 * may be NULL to size only) and sets *bytes to the buffer size. */
int pkt_out_packed(uint64_t col_mask, uint64_t n, void *base, pkt_out_t *out, uint64_t *bytes);
/* The byte ranges of an n-packet packed buffer that hold every selected column with only the first
 * `rows` (<= PKT_MAX_HDRS) slot rows of hdr_type / hdr_off: piece k = [off[k], off[k] + len[k]),
 * k < *npieces (2 when both slot columns are selected: the head through hdr_type's used rows, then
 * hdr_off's used rows; else 1).  C2's chain + Ether/IPv4/UDP at rows = 3 is 69 B per packet. */
int pkt_out_packed_pieces(uint64_t col_mask, uint64_t n, uint32_t rows, uint64_t off[2], uint64_t len[2],
                          int *npieces);
/* The column mask of a pkt_out_t (bit k set iff its k-th pointer is non-NULL). */
uint64_t pkt_out_mask(const pkt_out_t *out);
/* [lo, hi) of shard i of n packets split into `nshards` contiguous blocks whose sizes differ by
 * at most one (the lower shards take the remainder). */
int pkt_shard_range(uint64_t n, int nshards, int i, uint64_t *lo, uint64_t *hi);

/* The gather plan of pkt_mgpu_parse_gather (host only): one piece per message — `bytes` bytes from
 * offset `src` of shard `shard`'s packed buffer to offset `dst` of the root's receive buffer — for
 * `nshards` shards of n[i] packets whose batches use rows[i] (<= PKT_MAX_HDRS; rows NULL = all 16)
 * slot rows.  merge = 0: shard i's packed buffer (its used slot rows only, pkt_out_packed_pieces) at
 * the next 256-byte boundary of recv; merge = 1: recv is ONE packed output of sum(n) packets (each
 * column of shard i at packets [lo_i, lo_i + n_i), one piece per column and per used slot row — the
 * pieces the root's repack places after the merge = 0 transfer, see pkt_mgpu_parse_gather).
 * Writes min(cap, count) pieces, *npieces = count, *recv_bytes = the receive buffer size. */
typedef struct pkt_gather_piece {
    uint64_t src;
    uint64_t dst;
    uint64_t bytes;
    int32_t  shard;
    uint32_t reserved;
} pkt_gather_piece_t;
size_t pkt_sizeof_gather_piece(void);
int pkt_gather_plan(uint64_t col_mask, int nshards, const uint64_t *n, const uint32_t *rows, int merge,
                    pkt_gather_piece_t *pieces, uint64_t cap, uint64_t *npieces, uint64_t *recv_bytes);

/* ---- a capture that arrives in pieces (a NIC ring drained into host memory, a file read as it grows) ----
 * The capture path of tests/pcap.rs:7-37 as a stream: bytes are pushed as they arrive and the device
 * indexes and parses the records they complete while later bytes are still in flight.  Each step
 * indexes only the new bytes: the device keeps the first record start a step could not count yet (a
 * record running past the bytes so far) and the record count, and the next step starts the device
 * indexer from them (no re-walk from offset 24: the whole capture is indexed once however many steps).
 * The records, counts and errors are pkt_pcap_index's over the whole capture.
 * open: a stream on `device` (its own ctx; pkt_pcap_stream_ctx gives it for the tuning knobs) for a
 * capture of at most max_bytes (one device buffer) and `cap` records (<= 2^26; more are counted, not
 * parsed); `out` = the requested columns for cap records (slot columns strided by cap), either all
 * device memory of `device` (the parse writes them) or all pinned host memory from pkt_host_alloc (each
 * step's columns are exported over the link while the next bytes copy in); step_bytes = new bytes that
 * start a step at a push (0 = 4 MiB).
 * push: append n bytes (host memory; the caller may reuse it when push returns).  Pushes under 1 MiB
 * are gathered in a pinned staging ring of the stream and copied in 1 MiB pieces (or earlier, when a
 * step is due), without a wait per push; larger ones are copied from `bytes` and waited for.
 * poll: a step over the bytes not yet indexed, then wait: *n_records = the records wholly inside the
 * bytes so far (a record running past them is not an error yet), their columns written; offsets / lens
 * (HOST, [cap], may be NULL) receive their (data offset, incl_len).
 * finish: the capture is complete: a last step, the tail taken as pkt_pcap_index takes it (a record
 * running past the end = PKT_ERR_INVALID_ARG; a partial record header is ignored), then as poll.
 * Errors name the call in pkt_pcap_stream_last_error; after one, every later call returns it. */
typedef struct pkt_pcap_stream pkt_pcap_stream_t;
int         pkt_pcap_stream_open(int device, uint64_t max_bytes, uint64_t cap, int entry, const pkt_out_t *out,
                                 uint64_t step_bytes, pkt_pcap_stream_t **st);
int         pkt_pcap_stream_push(pkt_pcap_stream_t *st, const uint8_t *bytes, uint64_t n);
int         pkt_pcap_stream_poll(pkt_pcap_stream_t *st, uint64_t *n_records, uint64_t *offsets, uint32_t *lens);
int         pkt_pcap_stream_finish(pkt_pcap_stream_t *st, uint64_t *n_records, uint64_t *offsets, uint32_t *lens);
pkt_ctx_t  *pkt_pcap_stream_ctx(pkt_pcap_stream_t *st);
const char *pkt_pcap_stream_last_error(const pkt_pcap_stream_t *st);
int         pkt_pcap_stream_close(pkt_pcap_stream_t *st);

/* ---- multi-GPU: one process drives several devices ----
 * Every fast::parse_* is a pure function of one packet (fast.rs:5-227), so a batch splits into
 * contiguous shards, one per device, with no exchange inside the parse.  The only collective is
 * the gather of the per-packet tuples to a root device over RCCL (xGMI): one grouped
 * ncclSend / ncclRecv per shard (ncclCommInitAll over the device list; one communicator per
 * device, owned by the handle).  Each device has its own pkt_ctx and work stream; every call
 * below is asynchronous on those streams and returns after the launches (pkt_mgpu_synchronize
 * waits).  One host thread at a time per handle. */
typedef struct pkt_mgpu pkt_mgpu_t;
/* `devices`: ndev distinct HIP device ids; index 0..ndev-1 into this list is the "shard" id. */
int         pkt_mgpu_create(const int *devices, int ndev, pkt_mgpu_t **mg);
/* TEST MODE (not a transport to measure): a handle whose device list may repeat a device (e.g. device 0
 * listed 8 times: 8 shards, each with its own ctx and streams) and which holds no RCCL communicator:
 * every gather message that pkt_mgpu_create's handle sends by ncclSend/ncclRecv is a hipMemcpyAsync on
 * the sending shard's stream, ordered after the root's queued work and before the root's later work by
 * events.  It runs the N-shard code paths (per-shard issuing threads, shard offsets, multi-shard gather
 * plans and repack) on a one-GPU box; every other call behaves as for pkt_mgpu_create's handle. */
int         pkt_mgpu_create_virtual(const int *devices, int ndev, pkt_mgpu_t **mg);
int         pkt_mgpu_is_virtual(const pkt_mgpu_t *mg);
int         pkt_mgpu_destroy(pkt_mgpu_t *mg);
int         pkt_mgpu_ndev(const pkt_mgpu_t *mg);
/* The handle's last error; pkt_mgpu_last_error(NULL) = why this thread's last pkt_mgpu_create failed. */
const char *pkt_mgpu_last_error(const pkt_mgpu_t *mg);
/* The per-device ctx (tuning knobs, other batched calls) and work stream (a hipStream_t). */
pkt_ctx_t  *pkt_mgpu_ctx(pkt_mgpu_t *mg, int shard);
void       *pkt_mgpu_stream(pkt_mgpu_t *mg, int shard);
/* Parse shard i: batches[i] (resident on devices[i]) -> the packed output buffer shard_out[i]
 * (device memory of devices[i], pkt_out_packed(col_mask, batches[i].n) bytes). */
int pkt_mgpu_parse(pkt_mgpu_t *mg, const pkt_batch_t *batches, int entry, uint64_t col_mask,
                   void *const *shard_out);
/* `steps` consecutive pkt_mgpu_parse calls in one: step k parses batches[k*ndev + i] into the packed
 * buffer shard_out[k*ndev + i] on device i.  One host thread per device issues its device's launches,
 * round-robin over `streams` (1..4) streams of that device which start after, and are joined back
 * into, its work stream (steps are independent: different inputs, different outputs), so the launch
 * rate scales with the device count.  Asynchronous: returns after the launches. */
int pkt_mgpu_parse_steps(pkt_mgpu_t *mg, const pkt_batch_t *batches, int steps, int entry, uint64_t col_mask,
                         void *const *shard_out, int streams);
/* How the root's own pieces move in pkt_mgpu_gather / pkt_mgpu_parse_gather: 1 (default) = device
 * copies on the root's stream (an RCCL send to itself moved ~1 TB/s, the copy ~2 TB/s), 0 = RCCL
 * ncclSend / ncclRecv to itself inside the group like every other shard. */
int pkt_mgpu_set_root_copy(pkt_mgpu_t *mg, int enable);
/* Slot rows pkt_mgpu_parse_gather moves per shard: 0 (default) = each shard's largest n_hdrs, reduced
 * inside its parse kernel — the host waits once per device for it before issuing the gather; 1..16 =
 * that many rows for every shard (the caller's bound, >= every packet's n_hdrs; 16 always holds), so the
 * parse and the gather are queued with no host wait at all.  The largest n_hdrs is still reduced (when
 * n_hdrs is among the columns) and the next pkt_mgpu_synchronize returns PKT_ERR_GATHER_ROWS if the last
 * parse_gather had a packet with more headers than the fixed rows (its rows past them are unspecified in
 * recv although its n_hdrs counts them). */
int pkt_mgpu_set_gather_rows(pkt_mgpu_t *mg, int rows);
/* Gather bytes[i] of send[i] (device memory of devices[i]) into `recv` on devices[root] at
 * recv_off[i] (recv_off NULL: consecutive blocks, each rounded up to 256 B), `recv_len` bytes.
 * Grouped ncclSend/ncclRecv from the other devices; the root's own block per pkt_mgpu_set_root_copy. */
int pkt_mgpu_gather(pkt_mgpu_t *mg, int root, const void *const *send, const uint64_t *bytes,
                    void *recv, uint64_t recv_len, const uint64_t *recv_off);
/* pkt_mgpu_parse, then the gather of pkt_gather_plan(col_mask, ndev, n, rows, merge) into `recv` on
 * the root (recv_len >= its recv_bytes with rows NULL), where rows[i] = pkt_mgpu_set_gather_rows' count,
 * or by default shard i's largest n_hdrs when n_hdrs is among the columns (reduced inside each shard's
 * parse kernel; the host waits once per device, after every parse is queued), else all 16.  merge = 0
 * sends the plan's pieces as they are (<= 2 per shard).  merge = 1 sends the same <= 2 messages per
 * shard into a staging area the handle keeps on the root, then one repack kernel on the root's stream
 * places the merge = 1 plan's pieces (with the root copy on, the root's own pieces straight from its
 * shard buffer).  root_views (host array of ndev pkt_out_t, may be NULL) receives the column pointers
 * of each shard's tuples inside `recv` (merge = 0), or root_views[0] the single view of the whole batch
 * (merge = 1: what pkt_parse_batch over the whole batch would write). */
int pkt_mgpu_parse_gather(pkt_mgpu_t *mg, const pkt_batch_t *batches, int entry, uint64_t col_mask,
                          void *const *shard_out, int root, void *recv, uint64_t recv_len,
                          int merge, pkt_out_t *root_views);
int pkt_mgpu_synchronize(pkt_mgpu_t *mg);

#ifdef __cplusplus
}
#endif

#endif /* PKTGPU_H */
