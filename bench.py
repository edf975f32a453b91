#!/usr/bin/env python3
"""Benchmark: device-resident batched parse of packet slabs on MI355X (BASELINE.json metric).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4]
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

A step = one parse of one batch of 2^20 packets per GPU (config C2 by default: 64-byte
Ether/IPv4/UDP, fixed stride) producing the chain + Ether/IPv4/UDP field tuple + recomputed IPv4
checksum.  Each step reads a different slab of a >= 1 GiB ring per GPU (and writes a different
output set), so the 256 MiB Infinity Cache cannot serve the working set.  Inputs are resident in
HBM before the timed region starts.

Multi-GPU = the library's own multi-device entry (include/pktgpu.h pkt_mgpu_*): ONE process drives
the N devices, the K steps go out through pkt_mgpu_parse_steps (one issuing host thread per device,
2 streams per device), weak scaling: every device parses its own 2^20-packet batch per step with no
exchange (fast::parse is a pure function of one packet, reference src/parser/fast.rs:5-12).  Under
torch.distributed.run rank 0 is that process and the other ranks wait at a CPU (gloo) barrier
without touching a GPU.  The "c5" record times the C5 config through pkt_mgpu_parse_gather: 2^24
packets in contiguous shards, parse and RCCL gather of the used tuple bytes to device 0 timed
separately.
At N = 1 the line also carries the other device-resident BASELINE configs ("c3", "c4": each with its own
roofline), the host-memory rate ("host": pinned zero-copy pkt_parse_host), the capture path ("pcap":
capture in HBM -> pkt_pcap_index_device -> parse, one step; "pcap.index": the index kernels alone) and
the capture in host memory ("host_pcap").

Prints ONE JSON line (see DESIGN.md "Measurement" for every field).
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "packet-rs_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
METRIC = "Gpkt/s + GB/s device-resident parse, 1M×64B Ether/IPv4/UDP, 1/2/4/8 MI355X"


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="c2", choices=["c2", "c3", "c4", "c5"],
                    help="c5 = 2^24 C2 packets in total, sharded over the ranks (strong scaling)")
    ap.add_argument("--total-packets", type=int, default=1 << 24, help="C5 total packets")
    ap.add_argument("--packets", type=int, default=1 << 20, help="packets per GPU per step")
    ap.add_argument("--ring-gib", type=float, default=1.0)
    ap.add_argument("--columns", default=None,
                    help="column groups; default per config: c2 chain,ether,ipv4,udp; "
                         "c3 chain,ether,vlan,ipv4,tcp,udp; c4 all")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-c5", action="store_true", help="skip the C5 record")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = every core this process may use")
    ap.add_argument("--fastpath", type=int, default=int(os.environ.get("PKTGPU_FASTPATH", "1")),
                    help="register fast path for Ether/IPv4/UDP|TCP (pkt_ctx_set_fastpath)")
    ap.add_argument("--staging", type=int, default=int(os.environ.get("PKTGPU_STAGING", "0")),
                    help="pkt_ctx_set_staging: 0 auto, 1 per-lane windows, 2 wave spans")
    ap.add_argument("--window", type=int, default=int(os.environ.get("PKTGPU_WINDOW", "0")),
                    help="pkt_ctx_set_window bytes (0 = auto)")
    ap.add_argument("--streams", type=int, default=2,
                    help="consecutive steps are issued round-robin on this many HIP streams per device")
    ap.add_argument("--no-extra", action="store_true", help="skip the host and pcap records (N = 1)")
    ap.add_argument("--virtual", action="store_true",
                    help="TEST MODE: --gpus N shards on device 0 (pkt_mgpu_create_virtual, device copies instead "
                         "of RCCL) to run the N-device code paths on one GPU; prints a line labelled as a smoke, "
                         "never a measurement or a scaling point")
    return ap.parse_args()


# ------------------------------------------------------------------------------ inputs
def make_input(cfg, n, seed):
    from pktgpu import gen
    if cfg in ("c2", "c5"):
        return gen.gen_c2(n, seed=seed).reshape(-1), 64, None, None
    if cfg == "c3":
        return gen.gen_c3(n, seed=seed).reshape(-1), 128, None, None
    buf, offs, lens = gen.gen_c4(n, seed=seed)
    return buf, None, offs, lens


def algorithmic_bytes(n, cols, n_slots, span):
    """read = sum over packets of ceil64(header span) — the 64-byte request granularity of the
    bytes the walk must see (span = offset of the payload, i.e. the end of the last header);
    written = bytes of the requested output columns (slot columns: the slots used)."""
    from pktgpu import schema
    span = np.maximum(span.astype(np.int64), 1)
    read = int(((span + 63) // 64 * 64).sum())
    written = schema.bytes_per_packet(cols, n_slots=n_slots) * n
    return read, written


def line_bytes(n, stride, offs, span):
    """Bytes of the distinct 128-byte lines (the HBM fetch granule on gfx950) that
    hold the packets' header bytes [start, start + span): what any kernel must read at least."""
    span = np.maximum(span.astype(np.int64), 1)
    start = offs.astype(np.int64) if offs is not None else np.arange(n, dtype=np.int64) * stride
    first, last = start // 128, (start + span - 1) // 128
    order = np.argsort(first, kind="stable")
    first, last = first[order], last[order]
    prev = np.concatenate(([np.int64(-1)], np.maximum.accumulate(last)[:-1]))
    return int(np.maximum(last - np.maximum(first, prev + 1) + 1, 0).sum()) * 128


# ------------------------------------------------------------------------------ CPU baseline
def host_cores():
    """Cores this process may run on: its affinity set, capped by a cgroup CPU quota if any."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    return (min(aff, quota) if quota else aff), aff, quota


def _timed(fn, budget_s, min_reps=2, max_reps=100000):
    reps, t0 = 0, time.perf_counter()
    while reps < min_reps or (time.perf_counter() - t0 < budget_s and reps < max_reps):
        fn()
        reps += 1
    return reps, time.perf_counter() - t0


def cpu_baseline(slab, stride, offs, lens, n, cols, threads):
    """The oracle (C restatement of packet_rs 0.4.0 with the reference's per-header allocation,
    front insert and per-bit getter loops; -O2) on the host cores, bounded samples of:
      (ii) the GPU's work: fast::parse + every requested getter + ipv4_checksum  -> `value`
      (i)  fast::parse alone (the PacketSlice: chain columns)
      (iii) C1: slow::parse(pkt).to_vec() round trip of 1024 x 64 B (tests/lib.rs:790-802)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle
    from pktgpu import gen, schema
    oracle.build()
    n = min(n, 1 << 20)  # bounded sample (c5 shards are up to 2^24 packets)
    if offs is not None:
        offs, lens = offs[:n], lens[:n]
    kw = dict(stride=stride, offsets=offs, lens=lens, nthreads=threads)
    r2, t2 = _timed(lambda: oracle.parse_batch(slab, n, columns=cols, **kw), 8.0, max_reps=400)
    chain = schema.columns_of(["chain"])
    r1, t1 = _timed(lambda: oracle.parse_batch(slab, n, columns=chain, **kw), 4.0, max_reps=400)
    c1 = gen.gen_c2(1024, seed=0x5EED0001)
    # one call = 256 passes over the 1024 packets (one thread per slice of a 256k-packet batch)
    c1_rep = np.tile(c1.reshape(-1), 256)
    r3, t3 = _timed(lambda: oracle.round_trip_batch(c1_rep, 1024 * 256, stride=64, slow=True,
                                                    nthreads=threads), 4.0)
    n1 = min(n, 1 << 18)
    _, ts = _timed(lambda: oracle.parse_batch(slab, n1, columns=cols, stride=stride,
                                              offsets=offs[:n1] if offs is not None else None,
                                              lens=lens[:n1] if lens is not None else None,
                                              nthreads=1), 0.0, min_reps=1)
    return {"value": round(r2 * n / t2 / 1e9, 6), "unit": "Gpkt/s", "cores": threads,
            "kind": "port",
            "sample": f"(ii) {r2} passes over the same {n}-packet slab ({r2 * n} packets, {t2:.1f} s), "
                      f"{threads} threads = every core this process may use; oracle/pkt_oracle.c -O2 "
                      f"(C restatement of packet_rs 0.4.0 fast::parse + getters + ipv4_checksum)",
            "variants": {
                "i_fast_parse_only": {"Gpkt/s": round(r1 * n / t1 / 1e9, 6), "cores": threads,
                                      "what": "fast::parse -> PacketSlice (chain columns), tests/lib.rs:804-817"},
                "ii_parse_getters_checksum": {"Gpkt/s": round(r2 * n / t2 / 1e9, 6), "cores": threads,
                                              "what": "the bench tuple: parse + every getter + ipv4_checksum"},
                "iii_c1_slow_parse_to_vec": {"Gpkt/s": round(r3 * 1024 * 256 / t3 / 1e9, 6), "cores": threads,
                                             "what": "C1: slow::parse(pkt).to_vec() of 1024 x 64 B, "
                                                     "tests/lib.rs:790-802"},
                "ii_single_thread": {"Gpkt/s": round(n1 / ts / 1e9, 6), "cores": 1}}}


# ------------------------------------------------------------------------------ GPU helpers
def packed_outputs(torch, dev, cols, n, count):
    """`count` output sets, each ONE packed buffer in the library's layout (pkt_out_packed), so a
    rank's tuples are one gatherable message."""
    from pktgpu import mgpu
    nb = mgpu.packed_bytes(cols, n)
    outs = []
    for _ in range(count):
        buf = torch.empty(max(1, nb), dtype=torch.uint8, device=dev)
        outs.append((buf, mgpu.packed_views(buf, cols, n)))
    return outs


def load_probe():
    import ctypes
    from pktgpu import _lib
    path = os.path.join(REPO, "packet-rs_amd", "lib", "libpktprobe.so")
    if not os.path.exists(path):
        return None
    L = ctypes.CDLL(path)
    L.pkt_probe_ceiling.restype = ctypes.c_int
    L.pkt_probe_ceiling.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                    ctypes.POINTER(_lib.PktOut), ctypes.c_void_p]
    L.pkt_probe_stream_copy.restype = ctypes.c_int
    L.pkt_probe_stream_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64,
                                        ctypes.c_uint64, ctypes.c_void_p]
    L.pkt_probe_ceiling_groups.restype = ctypes.c_int
    L.pkt_probe_ceiling_groups.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                           ctypes.POINTER(_lib.PktOut), ctypes.c_void_p]
    return L


def event_avg_ms(torch, stream, launch, reps):
    """Average duration of `reps` back-to-back launches on ONE stream, one HIP event pair on that
    stream (includes the dependent-launch boundary between them)."""
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(stream)
    for k in range(reps):
        launch(k, stream)
    b.record(stream)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


# ------------------------------------------------------------------------------ shared pieces
DEFAULT_COLS = {"c2": "chain,ether,ipv4,udp", "c3": "chain,ether,vlan,ipv4,tcp,udp", "c4": "all",
                "c5": "chain,ether,ipv4,udp"}
WORKLOAD = {"c2": "C2: 2^20 x 64 B Ether/IPv4/UDP fixed-stride slab per GPU",
            "c3": "C3: 2^20 x 128 B Ether/{0-2}xVlan/IPv4/TCP|UDP per GPU",
            "c4": "C4: 2^20-record pcap replay of the 22 reference templates per GPU"}


def roofline_phase(torch, P, cfg, use_probe, batches, ostructs, raw_slabs, ring, n, stride, entry, dev, slots, R,
                   copy_args=None):
    """The parse kernel in isolation on device 0 — R back-to-back launches on ONE stream between one
    event pair on that stream — alternated with the ceiling probe (same launch shape, same bytes, no
    parsing; the fixed-stride configs C2 and C3 with their default columns, `slots` header slot rows),
    a torch device copy of the slab and, for C2 (`copy_args` = (destination buffers, read bytes,
    written bytes)), the hand-written streaming copy of the parse's bytes in one launch per batch and
    in one launch over 16 batches (pkt_probe_stream_copy).  Median of 5 rounds each."""
    import ctypes
    rs = torch.cuda.Stream(dev)
    probe = load_probe() if use_probe else None

    def parse_launch(k, s):
        P.launch(batches[k % ring], entry, ostructs[k % ring], s)

    def probe_launch(k, s):
        if cfg == "c3":
            rc = probe.pkt_probe_ceiling_groups(ctypes.c_void_p(raw_slabs[k % ring].data_ptr()), n, stride, slots,
                                                ctypes.byref(ostructs[k % ring]), ctypes.c_void_p(s.cuda_stream))
        else:
            rc = probe.pkt_probe_ceiling(ctypes.c_void_p(raw_slabs[k % ring].data_ptr()), n, stride,
                                         ctypes.byref(ostructs[k % ring]), ctypes.c_void_p(s.cuda_stream))
        if rc != 0:
            raise RuntimeError(f"pkt_probe_ceiling failed ({rc})")

    copy_dst = torch.empty_like(raw_slabs[0])

    def copy_launch(k, s):
        with torch.cuda.stream(s):
            copy_dst.copy_(raw_slabs[k % ring])

    scopy = None
    if probe is not None and copy_args is not None:
        dsts, rb, wb = copy_args
        kb = min(16, ring)
        P8 = ctypes.POINTER(ctypes.c_uint8)

        def ptrs(bufs):
            return (P8 * len(bufs))(*[ctypes.cast(ctypes.c_void_p(b.data_ptr()), P8) for b in bufs])
        srcs_all = [ptrs([raw_slabs[r]]) for r in range(ring)]
        dsts_all = [ptrs([dsts[r]]) for r in range(ring)]
        srcs_k, dsts_k = ptrs(raw_slabs[:kb]), ptrs(dsts[:kb])

        def scopy_launch(k, s):
            rc = probe.pkt_probe_stream_copy(srcs_all[k % ring], dsts_all[k % ring], 1, rb, wb,
                                             ctypes.c_void_p(s.cuda_stream))
            if rc != 0:
                raise RuntimeError(f"pkt_probe_stream_copy failed ({rc})")

        def scopy_k_launch(k, s):
            rc = probe.pkt_probe_stream_copy(srcs_k, dsts_k, kb, rb, wb, ctypes.c_void_p(s.cuda_stream))
            if rc != 0:
                raise RuntimeError(f"pkt_probe_stream_copy failed ({rc})")
        scopy = {"one": [], "k": [], "kb": kb, "rb": rb, "wb": wb}

    kern, ceil_, copy_ = [], [], []
    for _ in range(5):
        kern.append(event_avg_ms(torch, rs, parse_launch, R))
        if probe is not None:
            ceil_.append(event_avg_ms(torch, rs, probe_launch, R))
        copy_.append(event_avg_ms(torch, rs, copy_launch, R))
        if scopy is not None:
            scopy["one"].append(event_avg_ms(torch, rs, scopy_launch, R))
            scopy["k"].append(event_avg_ms(torch, rs, scopy_k_launch, max(4, R // 4)))
    del copy_dst
    # the probes overwrote output sets: re-parse them so the outputs are real
    for r in range(ring):
        parse_launch(r, rs)
    torch.cuda.synchronize(dev)
    return kern, ceil_, copy_, scopy


def assemble(args, res, n, ndev, cols, read_b, write_b, kern, ceil_, copy_, R, slab_bytes, stride, offs_np, span,
             pipe_s, scopy=None):
    """The roofline / line-floor / traffic objects of the JSON line."""
    algo = read_b + write_b
    avg_kern_s = float(np.median(kern)) * 1e-3
    achieved = algo / avg_kern_s / 1e9
    res["roofline"] = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                       "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                       "frac_kind": "kernel: algorithmic bytes / isolated launch duration (HIP events, "
                                    "one stream) / 8 TB/s spec",
                       "kernel": "parse_kernel", "avg_kernel_us": round(avg_kern_s * 1e6, 3),
                       "read_only_frac": round(read_b / avg_kern_s / 1e9 / HBM_PEAK_GBS, 4),
                       "measured": f"device 0: median of 5 rounds of {R} back-to-back launches on one "
                                   f"stream, one HIP event pair per round",
                       "algorithmic_bytes_per_launch": algo,
                       "pipelined": {"streams": args.streams,
                                     "device_ms_per_step": round(pipe_s * 1e3, 5),
                                     "achieved": round(algo / pipe_s / 1e9, 2),
                                     "frac": round(algo / pipe_s / 1e9 / HBM_PEAK_GBS, 4),
                                     "frac_kind": "throughput: algorithmic bytes per step / device-0 time "
                                                  "per step of the timed region (HIP events) / 8 TB/s"}}
    if ceil_:
        cs = float(np.median(ceil_)) * 1e-3
        res["roofline"]["ceiling"] = {
            "kernel": "pkt_probe_ceiling (C2) / pkt_probe_ceiling_groups (C3), libpktprobe.so: same launch shape and bytes, no parsing",
            "avg_kernel_us": round(cs * 1e6, 3), "achieved": round(algo / cs / 1e9, 2),
            "frac_of_peak": round(algo / cs / 1e9 / HBM_PEAK_GBS, 4),
            "parse_frac_of_ceiling": round(cs / avg_kern_s, 4)}
    if scopy is not None:
        one_s = float(np.median(scopy["one"])) * 1e-3
        k_s = float(np.median(scopy["k"])) * 1e-3 / scopy["kb"]
        cb = scopy["rb"] + scopy["wb"]
        res["roofline"]["ceiling"]["stream_copy"] = {
            "kernel": "pkt_probe_stream_copy (libpktprobe.so): hand-written global_load_dwordx4 / "
                      "global_store_dwordx4 copy, 1 KiB contiguous per wave instruction, 4 loads in flight "
                      "per lane; the parse's read and written bytes, no parsing",
            "read_bytes": scopy["rb"], "written_bytes": scopy["wb"],
            "one_batch_per_launch": {"avg_kernel_us": round(one_s * 1e6, 3), "achieved": round(cb / one_s / 1e9, 2),
                                     "frac_of_peak": round(cb / one_s / 1e9 / HBM_PEAK_GBS, 4),
                                     "parse_frac_of_copy": round(one_s / avg_kern_s, 4)},
            f"{scopy['kb']}_batches_per_launch": {"us_per_batch": round(k_s * 1e6, 3),
                                                  "achieved": round(cb / k_s / 1e9, 2),
                                                  "frac_of_peak": round(cb / k_s / 1e9 / HBM_PEAK_GBS, 4)},
            "measured": f"median of 5 rounds, HIP events on one stream ({R} one-batch launches / "
                        f"{max(4, R // 4)} {scopy['kb']}-batch launches per round), same ring as the parse"}
    # the line-granular floor: distinct 128-B lines holding header bytes + the batch index read
    # + the columns written, priced at this box's measured copy rate
    idx_b = 12 * n if offs_np is not None else 0
    floor_b = line_bytes(n, stride, offs_np, span) + idx_b + write_b
    copy_gbs = 2 * slab_bytes / (float(np.median(copy_)) * 1e-3) / 1e9
    floor_s = floor_b / (copy_gbs * 1e9)
    res["roofline"]["line_floor"] = {
        "bytes_per_launch": floor_b, "read_lines": floor_b - idx_b - write_b, "index_read": idx_b,
        "written": write_b, "copy_rate_GBps": round(copy_gbs, 2),
        "copy": "torch copy_ of the slab over the same ring (read + write), HIP events, one stream",
        "floor_us_at_copy_rate": round(floor_s * 1e6, 3),
        "kernel_frac_of_floor": round(floor_s / avg_kern_s, 4),
        "pipelined_frac_of_floor": round(floor_s / pipe_s, 4)}
    # HBM traffic per launch from the committed rocprofv3 PMC passes of this config, if any
    tpath = os.path.join(REPO, "profiles", f"traffic_{args.config}.json")
    if os.path.exists(tpath) and args.columns == DEFAULT_COLS[args.config] and n == 1 << 20:
        t = json.load(open(tpath))
        res["roofline"]["traffic"] = t["traffic_bytes_per_launch"]
        res["roofline"]["traffic_source"] = {
            "measured_in_this_run": False,
            "file": f"profiles/traffic_{args.config}.json",
            "how": "rocprofv3 --pmc FETCH_SIZE (x2, gfx950) and WRITE_SIZE, separate passes of "
                   f"bench.py --config {args.config} (scripts/gpu.sh traffic={args.config})",
            "x2_check": "every memory-side read request of these launches is a 128-B line "
                        "(TCC_EA0_RDREQ_128B = TCC_EA0_RDREQ; FETCH_SIZE counts 64 B per request): "
                        "profiles/ab/r02calib_fetch_requests.txt",
            "run": t.get("label", "")}


def host_record(P, torch, cols, n=1 << 20, reps=5):
    """The host-memory path (north_star: the path starts and ends in host memory): a pinned C2
    batch and pinned columns through pkt_parse_host, which reads the slab and writes the columns
    over PCIe directly (zero copy, one launch); blocking per batch."""
    from pktgpu import gen
    slab = P.host_empty((n * 64,), np.uint8)
    slab[:] = gen.gen_c2(n, seed=0x5EED0004).reshape(-1)
    from pktgpu import schema
    out = {c: P.host_empty(schema.column_shape(c, n), schema.column_dtype(c)) for c in cols}
    P.parse_host(slab, stride=64, columns=cols, out=out)  # warm (code object, mapping)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        P.parse_host(slab, stride=64, columns=cols, out=out)
        ts.append(time.perf_counter() - t0)
    t = float(np.median(ts))
    used = int(out["n_hdrs"].max()) if "n_hdrs" in out else schema.MAX_HDRS
    written = schema.bytes_per_packet(cols, n_slots=used) * n
    return {"workload": "C2 2^20 x 64 B in pinned host memory -> pinned host columns (chain+ether+ipv4+udp)",
            "entry": "pkt_parse_host (zero copy: every buffer from pkt_host_alloc)",
            "ms_per_batch": round(t * 1e3, 4), "Gpkt/s": round(n / t / 1e9, 4),
            "link_GB/s": {"host_to_device": round(64 * n / t / 1e9, 2),
                          "device_to_host": round(written / t / 1e9, 2)},
            "reps": reps, "timing": "wall clock per blocking call, median"}


def pcap_record(P, torch, dev, n=1 << 20, reps=10):
    """The capture path of tests/pcap.rs:7-37 on the device as one step: a pcap file already in HBM
    -> pkt_parse_pcap (pkt_pcap_index_device's kernels, then pkt_parse_batch of every record, all
    columns, taking the record count from the device: one host synchronisation per step)."""
    from pktgpu import gen, schema
    buf, offs, lens = gen.gen_c4(n, seed=0x5EED0005)
    d_buf = torch.from_numpy(buf).to(dev)
    d_offs = torch.empty(n, dtype=torch.uint64, device=dev)
    d_lens = torch.empty(n, dtype=torch.uint32, device=dev)
    out = P.alloc(n, schema.COLUMN_NAMES)
    # the output descriptor (49 column pointers) built once, as a C / Rust caller keeps its pkt_out_t and
    # the headline's steps do (marshalling it from the dict costs ~15 us of Python per call)
    ostruct = P.out_struct(out)
    s = torch.cuda.current_stream(dev)
    cnt = [0]
    # the C ABI call with its arguments prebuilt (as the headline's steps are issued): the step times
    # pkt_parse_pcap, not the Python wrapper's argument checks and conversions
    cnt_c = ctypes.c_uint64()
    fn = P._L.pkt_parse_pcap
    args = (P._ctx, d_buf.data_ptr(), d_buf.numel(), schema.ENTRY_ID["parse"], ctypes.byref(ostruct),
            d_offs.data_ptr(), d_lens.data_ptr(), n, ctypes.byref(cnt_c), ctypes.c_void_p(s.cuda_stream))

    def step():
        rc = fn(*args)
        if rc != 0:
            raise RuntimeError(f"pkt_parse_pcap: {rc}")
        cnt[0] = cnt_c.value

    step()
    ok = cnt[0] == n and np.array_equal(d_offs.cpu().numpy(), offs)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        step()
        ts.append(time.perf_counter() - t0)
    t = float(np.median(ts))
    # the index alone, its three kernels timed by HIP events between them (pkt_pcap_index_device_timed)
    iw, ik = [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        ci, ms = P.pcap_index_device_timed(d_buf, d_offs, d_lens, stream=s)
        iw.append(time.perf_counter() - t0)
        ik.append(ms)
        ok = ok and ci == n
    ik = np.median(np.array(ik), axis=0)
    # the same blocking call without the timing events (pkt_pcap_index_device): what a caller pays
    cnt_u = ctypes.c_uint64()
    su = ctypes.c_void_p(s.cuda_stream)
    iu = []
    for _ in range(reps):
        t0 = time.perf_counter()
        rc = P._L.pkt_pcap_index_device(P._ctx, d_buf.data_ptr(), d_buf.numel(), d_offs.data_ptr(), d_lens.data_ptr(),
                                        n, ctypes.byref(cnt_u), su)
        iu.append(time.perf_counter() - t0)
        ok = ok and rc == 0 and cnt_u.value == n
    index = {"entry": "pkt_pcap_index_device_timed (blocking, cap = n: offsets and lens written)",
             "ms_per_call": round(float(np.median(iw)) * 1e3, 4),
             "ms_per_call_untimed": round(float(np.median(iu)) * 1e3, 4),
             "kernel_us": {"guess": round(float(ik[0]) * 1e3, 2), "scan": round(float(ik[1]) * 1e3, 2),
                           "emit": round(float(ik[2]) * 1e3, 2)},
             "kernels_us_total": round(float(ik.sum()) * 1e3, 2),
             "file_read_GB/s_guess": round(buf.size / (float(ik[0]) * 1e-3) / 1e9, 2),
             "timing": "wall clock per blocking call and HIP events recorded between the kernels on the "
                       "call's stream (the events themselves add ~10 us to the call and to the kernels' "
                       "spans: ms_per_call_untimed is pkt_pcap_index_device's, rocprof kernel averages in "
                       "profiles/pcap/), median of reps"}
    # a stream of captures: pkt_parse_pcap_async on two ctxs / two streams, one capture in flight on
    # each, so one capture's index kernels overlap the other's parse (the C2 value's 2-stream form)
    import pktgpu
    P2 = pktgpu.Parser(dev.index if dev.index is not None else 0)
    try:
        ps = [P, P2]
        ss = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
        out2 = P2.alloc(n, schema.COLUMN_NAMES)  # (held: the descriptor below points into it)
        outs = [ostruct, P2.out_struct(out2)]
        idx = [(d_offs, d_lens), (torch.empty_like(d_offs), torch.empty_like(d_lens))]
        for j in (0, 1):
            ss[j].wait_stream(torch.cuda.current_stream(dev))
        busy = [False, False]
        counts = []

        def queue(k):
            j = k % 2
            if busy[j]:
                ss[j].synchronize()
                counts.append(ps[j].pcap_result())
            ps[j].parse_pcap_async(d_buf, n, outs[j], idx[j][0], idx[j][1], stream=ss[j])
            busy[j] = True

        def drain():
            for j in (0, 1):
                if busy[j]:
                    ss[j].synchronize()
                    counts.append(ps[j].pcap_result())
                    busy[j] = False

        for k in range(4):
            queue(k)
        drain()
        counts.clear()
        K = 4 * reps
        t0 = time.perf_counter()
        for k in range(K):
            queue(k)
        drain()
        tp = (time.perf_counter() - t0) / K
        ok_p = len(counts) == K and all(c == n for c in counts) and \
            np.array_equal(idx[1][0].cpu().numpy(), offs)
    finally:
        P2.close()
    return {"workload": f"C4 capture: {n} records of the 22 reference templates, {buf.size} B pcap file in HBM",
            "step": "pkt_parse_pcap: pcap_guess_kernel + pcap_scan_kernel + pcap_emit_kernel (record boundaries, exact; written by the emit "
                    "kernel) + parse_kernel (all columns, record count read on the device); one blocking call",
            "ms_per_step": round(t * 1e3, 4), "Grecords/s": round(n / t / 1e9, 4),
            "file_GB/s": round(buf.size / t / 1e9, 2), "index_matches_host_indexer": bool(ok),
            "reps": reps, "timing": "wall clock per step, median", "index": index,
            "pipelined": {"ms_per_capture": round(tp * 1e3, 4), "Grecords/s": round(n / tp / 1e9, 4),
                          "file_GB/s": round(buf.size / tp / 1e9, 2), "captures": K, "counts_ok": bool(ok_p),
                          "form": "pkt_parse_pcap_async on 2 ctxs x 2 streams, one capture in flight per ctx, "
                                  "wall clock over all captures / captures"}}


def host_pcap_record(P, n=1 << 20, reps=5):
    """north_star's host-memory path for the capture config (tests/pcap.rs:7-37): the C4 capture in
    pinned host memory -> pkt_parse_pcap_host (copy in, device index, all-column parse, the kernel
    writing the pinned host columns over the link) -> pinned host columns; one blocking call."""
    from pktgpu import gen, schema
    buf, offs, lens = gen.gen_c4(n, seed=0x5EED0006)
    hb = P.host_empty((buf.size,), np.uint8)
    hb[:] = buf
    cols = list(schema.COLUMN_NAMES)
    out = {c: P.host_empty(schema.column_shape(c, n), schema.column_dtype(c)) for c in cols}
    m, _, _ = P.parse_pcap_host(hb, n, out=out, index=False)  # warm (buffers, code objects)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        m, _, _ = P.parse_pcap_host(hb, n, out=out, index=False)
        ts.append(time.perf_counter() - t0)
    t = float(np.median(ts))
    ok = m == n
    # the kernel writes every per-packet column and each packet's own n_hdrs slot entries (3 B each)
    written = schema.bytes_per_packet(cols, n_slots=0) * n + 3 * int(out["n_hdrs"].astype(np.int64).sum())
    # a stream of captures: pkt_parse_pcap_host_async on two ctxs, one capture in flight on each, so
    # one capture's file copy in overlaps the other's columns out (the link is full duplex)
    import pktgpu
    P2 = pktgpu.Parser(0)
    try:
        ps = [P, P2]
        outs = [out, {c: P2.host_empty(schema.column_shape(c, n), schema.column_dtype(c)) for c in cols}]
        busy = [False, False]
        counts = []

        def queue(k):
            j = k % 2
            if busy[j]:
                counts.append(ps[j].pcap_host_result())
            ps[j].parse_pcap_host_async(hb, n, outs[j])
            busy[j] = True

        def drain():
            for j in (0, 1):
                if busy[j]:
                    counts.append(ps[j].pcap_host_result())
                    busy[j] = False

        for k in range(2):
            queue(k)
        drain()
        counts.clear()
        K = 4 * reps
        t0 = time.perf_counter()
        for k in range(K):
            queue(k)
        drain()
        tp = (time.perf_counter() - t0) / K
        ok_p = len(counts) == K and all(c == n for c in counts)
    finally:
        P2.close()
    return {"workload": f"C4 capture: {n} records of the 22 reference templates, {buf.size} B pcap file "
                        f"in pinned host memory -> all {len(cols)} columns in pinned host memory",
            "entry": "pkt_parse_pcap_host (one blocking call: the file copied in 16 MiB pieces; once a piece has "
                     "landed, its prefix indexed on the device and the records it adds parsed into device columns, "
                     "exported to the pinned columns in 16-byte chunks while the next pieces copy in)",
            "ms_per_capture": round(t * 1e3, 4), "Grecords/s": round(n / t / 1e9, 4),
            "link_GB/s": {"host_to_device": round(buf.size / t / 1e9, 2),
                          "device_to_host": round(written / t / 1e9, 2)},
            "records": int(m), "count_ok": bool(ok), "reps": reps,
            "timing": "wall clock per blocking call, median",
            "pipelined": {"ms_per_capture": round(tp * 1e3, 4), "Grecords/s": round(n / tp / 1e9, 4),
                          "link_GB/s": {"host_to_device": round(buf.size / tp / 1e9, 2),
                                        "device_to_host": round(written / tp / 1e9, 2)},
                          "captures": K, "counts_ok": bool(ok_p),
                          "form": "pkt_parse_pcap_host_async on 2 ctxs, one capture in flight per ctx, "
                                  "wall clock over all captures / captures"}}


def pcap_stream_record(P, n=1 << 20, reps=3, pushes=(1 << 20, 64 << 10)):
    """north_star's "NIC ring buffer" form of the capture path (tests/pcap.rs:7-37 as bytes arrive):
    the C4 capture in pinned host memory pushed into pkt_pcap_stream_* in pieces of `push` bytes (each
    push returns with the caller's bytes reusable), 4 MiB steps, finish; device columns.  Wall clock
    from the first push to finish's return, median of reps; the record count is checked."""
    from pktgpu import gen
    from pktgpu.stream import PcapStream
    buf, _, _ = gen.gen_c4(n, seed=0x5EED0007)
    hb = P.host_empty((buf.size,), np.uint8)
    hb[:] = buf
    rows = {}
    ok = True
    for push in pushes:
        ts = []
        for r in range(reps + 1):  # (the first: warm)
            st = PcapStream(0, max_bytes=buf.size + 64, cap=n, columns="all")
            try:
                t0 = time.perf_counter()
                for p0 in range(0, buf.size, push):
                    st.push(hb[p0:p0 + push])
                c, _ = st.finish(index=False)
                if r:
                    ts.append(time.perf_counter() - t0)
                ok &= c == n
            finally:
                st.close()
        t = float(np.median(ts))
        rows[str(push)] = {"ms_per_capture": round(t * 1e3, 4), "Grecords/s": round(n / t / 1e9, 4),
                           "host_to_device_GB/s": round(buf.size / t / 1e9, 2)}
    return {"workload": f"C4 capture: {n} records, {buf.size} B in pinned host memory, pushed as it would arrive",
            "entry": "pkt_pcap_stream_open / _push (pieces of push_bytes; under 1 MiB through the stream's pinned "
                     "staging ring) / _finish, 4 MiB steps, all 49 columns into device memory",
            "by_push_bytes": rows, "count_ok": bool(ok), "reps": reps,
            "timing": "wall clock from the first push to finish's return, median"}


# ------------------------------------------------------------------------------ the library's multi-GPU entry
def run_mgpu(args, ndev):
    """One process, ndev devices through pkt_mgpu (the measured form for every N)."""
    import torch
    visible = torch.cuda.device_count()
    if visible < ndev and not args.virtual:
        print(f"bench.py: --gpus {ndev} but only {visible} device(s) visible", file=sys.stderr)
        sys.exit(2)
    import pktgpu
    from pktgpu import mgpu, schema
    torch.cuda.set_device(0)
    devices = [0] * ndev if args.virtual else list(range(ndev))
    MP = mgpu.MultiParser(devices, virtual=args.virtual)
    MP.set_knobs(fastpath=args.fastpath, staging=args.staging, window=args.window)
    default_cols = DEFAULT_COLS[args.config]
    if args.columns is None:
        args.columns = default_cols
    cols = pktgpu.resolve_columns("all" if args.columns == "all" else args.columns.split(","))
    entry = schema.ENTRY_ID["parse"]
    n = args.packets

    # ---------------- inputs: one seeded batch per device, replicated over a >= ring_gib ring
    per = []
    for i, d in enumerate(MP.torch_devices):
        slab_np, stride, offs_np, lens_np = make_input(args.config, n, seed=0x5EED0000 + 2 + i)
        ring = max(2, int(np.ceil(args.ring_gib * (1 << 30) / slab_np.size)))
        first = torch.from_numpy(slab_np).to(d)
        slabs = [first] + [first.clone() for _ in range(ring - 1)]
        offs = torch.from_numpy(offs_np).to(d) if offs_np is not None else None
        lens = torch.from_numpy(lens_np).to(d) if lens_np is not None else None
        outs = packed_outputs(torch, d, cols, n, ring)
        per.append(dict(slab_np=slab_np, stride=stride, offs_np=offs_np, lens_np=lens_np, ring=ring,
                        slabs=slabs, offs=offs, lens=lens, outs=outs))
    ring = per[0]["ring"]
    total_steps = args.warmup + args.steps
    plan = MP.steps_plan([[((pd["slabs"][k % ring], n, pd["stride"], pd["offs"], pd["lens"]), pd["outs"][k % ring][0])
                           for pd in per] for k in range(total_steps)])
    if args.warmup:
        MP.parse_steps(plan, entry, cols, first=0, count=args.warmup, streams=args.streams)
    MP.synchronize()

    # ---------------- timed region: K steps on every device, ONE foreign call (pkt_mgpu_parse_steps,
    # arguments prebuilt), all devices idle on both sides
    timed = MP.steps_call(plan, entry, cols, first=args.warmup, count=args.steps, streams=args.streams)
    t0 = time.perf_counter()
    timed()
    MP.synchronize()
    elapsed = time.perf_counter() - t0
    # the same K steps again with one event pair on device 0's work stream (the extra streams start
    # after it and are joined back into it): device 0's time per step, outside the timed region
    ext0 = MP.streams()[0]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(ext0)
    timed()
    e1.record(ext0)
    MP.synchronize()
    region_ms = e0.elapsed_time(e1)

    # ---------------- roofline sub-phase on device 0 (its own ctx, same buffers)
    P = pktgpu.Parser(0)
    P.set_fastpath(args.fastpath)
    P.set_staging(args.staging)
    P.set_window(args.window)
    p0 = per[0]
    batches0 = [P._batch(p0["slabs"][r], n, p0["stride"], p0["offs"], p0["lens"]) for r in range(ring)]
    ostructs0 = [P.out_struct(p0["outs"][r][1]) for r in range(ring)]
    o0 = p0["outs"][0][1]
    used_slots = int(o0["n_hdrs"].max().item()) if "n_hdrs" in o0 else 0
    R = min(max(args.steps, 20), 50)
    default_shape = args.columns == default_cols
    copy_args = None
    if args.config == "c2" and default_shape:  # the streaming-copy ceiling of the C2 bytes
        copy_args = ([p0["outs"][r][0] for r in range(ring)], p0["slab_np"].size,
                     schema.bytes_per_packet(cols, n_slots=max(used_slots, 1)) * n)
    kern, ceil_, copy_, scopy = roofline_phase(torch, P, args.config, args.config in ("c2", "c3", "c5") and default_shape,
                                               batches0, ostructs0, p0["slabs"], ring, n, p0["stride"], entry,
                                               MP.torch_devices[0], used_slots, R, copy_args)

    # ---------------- multi-batch launch (pkt_parse_batches): K ring batches in ONE launch, so the
    # launch's ramp and drain are paid once per K batches (same bytes per batch as `roofline`)
    batched = None
    kb = min(16, ring)
    if kb >= 2:
        rs = torch.cuda.Stream(MP.torch_devices[0])
        call = P.batches_call(batches0[:kb], ostructs0[:kb], entry, rs)
        bt = [event_avg_ms(torch, rs, lambda k, s: call(), max(4, min(R, 20))) for _ in range(5)]
        batched = {"entry": "pkt_parse_batches", "batches_per_launch": kb, "packets_per_batch": n,
                   "avg_launch_us": round(float(np.median(bt)) * 1e3, 3),
                   "us_per_batch": round(float(np.median(bt)) * 1e3 / kb, 3)}

    c5 = None
    if args.config == "c2" and not args.no_c5:
        # (after the headline's timed region: a failure here, e.g. RCCL on a new node, is recorded in
        # the line instead of losing it)
        try:
            c5 = run_c5_mgpu(args, torch, MP, per, cols, entry)
        except Exception as ex:  # noqa: BLE001
            c5 = {"workload": "C5", "error": f"{type(ex).__name__}: {ex}"}
            print(f"bench.py: C5 record failed: {ex}", file=sys.stderr)
            try:
                MP.synchronize()
            except Exception:  # noqa: BLE001
                pass

    span = o0["payload_off"].cpu().numpy() if "payload_off" in o0 else np.full(n, 64, np.int64)
    read_b, write_b = algorithmic_bytes(n, cols, max(used_slots, 1), span)
    algo = read_b + write_b
    slab_bytes = p0["slab_np"].size
    value = ndev * n * args.steps / elapsed / 1e9
    pipe_s = region_ms * 1e-3 / args.steps
    agg_gbs = algo * ndev * args.steps / elapsed / 1e9
    res = {
        "metric": METRIC,
        "value": round(value, 4),
        "unit": "Gpkt/s",
        "n_gpus": ndev,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seeded generator, pktgpu/gen.py)",
        "config": {
            "workload": WORKLOAD[args.config],
            "packets_per_gpu": n, "entry": "fast::parse", "columns": args.columns,
            "ring_slabs": ring, "ring_bytes": ring * slab_bytes, "parallelism": f"dp{ndev}",
            "launch": f"pkt_mgpu_parse_steps: one process, {ndev} device(s), one issuing host thread per "
                      f"device, {args.streams} streams per device",
            "staging": args.staging, "window": args.window,
        },
        "GB/s": {"algorithmic": round(agg_gbs, 2),
                 "slab": round(slab_bytes * ndev * args.steps / elapsed / 1e9, 2),
                 "algorithmic_bytes_per_pkt": {"read": read_b / n, "written": write_b / n},
                 "aggregate_frac_of_n_x_peak": round(agg_gbs / (ndev * HBM_PEAK_GBS), 4)},
    }
    assemble(args, res, n, ndev, cols, read_b, write_b, kern, ceil_, copy_, R, slab_bytes, p0["stride"],
             p0["offs_np"], span, pipe_s, scopy)
    if batched is not None:
        bs = batched["us_per_batch"] * 1e-6
        batched.update({"achieved": round(algo / bs / 1e9, 2), "frac": round(algo / bs / 1e9 / HBM_PEAK_GBS, 4),
                        "frac_kind": "algorithmic bytes of one batch / (one K-batch launch's duration / K), "
                                     "HIP events on one stream, median of 5 rounds / 8 TB/s; the headline "
                                     "`value` stays one launch per 2^20-packet batch"})
        res["roofline"]["batched"] = batched
    res["timing"] = {"wall_ms": round(elapsed * 1e3, 4), "device0_ms_same_steps_repeated": round(region_ms, 4),
                     "wall_minus_device_ms": round(elapsed * 1e3 - region_ms, 4),
                     "what": "wall = the timed region (one foreign call issuing K steps + synchronize); "
                             "device = the same K steps re-issued between one HIP event pair on device 0"}
    if c5 is not None:
        res["c5"] = c5
    if args.virtual:
        # a smoke of the N-shard code paths on one device: not the metric, not a scaling point
        res["metric"] = f"VIRTUAL SMOKE (not a measurement): {ndev} shards on device 0 through pkt_mgpu_create_virtual"
        res["n_gpus"] = 1
        res["virtual_shards"] = ndev
        res["scaling"] = None
        res["config"]["parallelism"] = f"virtual{ndev} on one GPU"
        res["config"]["launch"] += " (virtual handle: one physical device, gather messages by hipMemcpyAsync)"
    if ndev == 1 and not args.no_extra and args.config == "c2":
        # the other single-GPU BASELINE configs, device-resident, each with its own roofline
        for cfg in ("c3", "c4"):
            res[cfg] = config_record(args, torch, MP, P, cfg, entry)
    if ndev == 1 and not args.no_extra:
        res["host"] = host_record(P, torch, cols)
        res["pcap"] = pcap_record(P, torch, MP.torch_devices[0])
        res["host_pcap"] = host_pcap_record(P)
        res["pcap_stream"] = pcap_stream_record(P)
    if ndev == 1 and not args.no_cpu_baseline:
        cores, aff, quota = host_cores()
        threads = args.cpu_threads or cores
        res["cpu_baseline"] = cpu_baseline(p0["slab_np"], p0["stride"], p0["offs_np"], p0["lens_np"], n, cols, threads)
        res["cpu_baseline"]["host"] = {"affinity_cpus": aff, "cgroup_cpu_quota": quota,
                                       "os_cpu_count": os.cpu_count()}
    P.close()
    MP.close()
    return res


def config_record(args, torch, MP, P, cfg, entry):
    """A BASELINE config other than the headline's, device-resident on device 0 (N = 1 line): C3 (2^20 x
    128 B Ether/{0-2}xVlan/IPv4/TCP|UDP, fast.rs:49-62, 203-207) or C4 (2^20-record capture of the 22
    reference templates, fast.rs:5-227), with its default columns over its own >= ring_gib ring.  The
    same measurements as the headline: K pipelined steps through pkt_mgpu_parse_steps (wall clock and
    device-0 events), the isolated launch, the ceiling probe (C3) and the device copy of the slab (line
    floor), 16 batches per launch (pkt_parse_batches), and the committed PMC traffic of the config."""
    import pktgpu
    from pktgpu import schema
    cols_s = DEFAULT_COLS[cfg]
    cols = pktgpu.resolve_columns("all" if cols_s == "all" else cols_s.split(","))
    n = args.packets
    dev = MP.torch_devices[0]
    slab_np, stride, offs_np, lens_np = make_input(cfg, n, seed=0x5EED0000 + int(cfg[1:]))
    ring = max(2, int(np.ceil(args.ring_gib * (1 << 30) / slab_np.size)))
    first = torch.from_numpy(slab_np).to(dev)
    slabs = [first] + [first.clone() for _ in range(ring - 1)]
    offs = torch.from_numpy(offs_np).to(dev) if offs_np is not None else None
    lens = torch.from_numpy(lens_np).to(dev) if lens_np is not None else None
    outs = packed_outputs(torch, dev, cols, n, ring)
    K, W = args.steps, args.warmup
    plan = MP.steps_plan([[((slabs[k % ring], n, stride, offs, lens), outs[k % ring][0])] for k in range(W + K)])
    if W:
        MP.parse_steps(plan, entry, cols, first=0, count=W, streams=args.streams)
    MP.synchronize()
    timed = MP.steps_call(plan, entry, cols, first=W, count=K, streams=args.streams)
    t0 = time.perf_counter()
    timed()
    MP.synchronize()
    elapsed = time.perf_counter() - t0
    ext0 = MP.streams()[0]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(ext0)
    timed()
    e1.record(ext0)
    MP.synchronize()
    pipe_s = e0.elapsed_time(e1) * 1e-3 / K

    batches = [P._batch(slabs[r], n, stride, offs, lens) for r in range(ring)]
    ostructs = [P.out_struct(outs[r][1]) for r in range(ring)]
    o0 = outs[0][1]
    used_slots = int(o0["n_hdrs"].max().item())
    R = min(max(K, 20), 50)
    kern, ceil_, copy_, _ = roofline_phase(torch, P, cfg, cfg == "c3", batches, ostructs, slabs, ring, n, stride,
                                           entry, dev, used_slots, R)
    kb = min(16, ring)
    rs = torch.cuda.Stream(dev)
    call = P.batches_call(batches[:kb], ostructs[:kb], entry, rs)
    bt = [event_avg_ms(torch, rs, lambda k, s: call(), max(4, min(R, 20))) for _ in range(5)]
    span = o0["payload_off"].cpu().numpy()
    ok = int((o0["status"] == 0).sum().item())
    read_b, write_b = algorithmic_bytes(n, cols, max(used_slots, 1), span)
    algo = read_b + write_b
    rec = {"workload": WORKLOAD[cfg], "entry": "fast::parse", "columns": cols_s, "packets": n,
           "value": round(n * K / elapsed / 1e9, 4), "unit": "Gpkt/s", "steps": K, "warmup": W,
           "ms_per_step": round(elapsed / K * 1e3, 5), "ring_slabs": ring, "ring_bytes": ring * slab_np.size,
           "packets_status_ok": ok,
           "launch": f"pkt_mgpu_parse_steps on device 0, {args.streams} streams (the headline's step form)",
           "GB/s": {"algorithmic": round(algo * K / elapsed / 1e9, 2),
                    "slab": round(slab_np.size * K / elapsed / 1e9, 2),
                    "algorithmic_bytes_per_pkt": {"read": read_b / n, "written": write_b / n}}}
    sub = argparse.Namespace(**vars(args))
    sub.config, sub.columns = cfg, cols_s
    assemble(sub, rec, n, 1, cols, read_b, write_b, kern, ceil_, copy_, R, slab_np.size, stride, offs_np, span,
             pipe_s)
    bs = float(np.median(bt)) * 1e-3 / kb
    rec["roofline"]["kernel"] = "parse_kernel<6, 383u, 1> (lockstep walk, all columns)" if cfg == "c4" else \
        "parse_kernel<4, 111u, 0> (waterfall walk + fast path)"
    rec["roofline"]["batched"] = {"entry": "pkt_parse_batches", "batches_per_launch": kb, "packets_per_batch": n,
                                  "us_per_batch": round(bs * 1e6, 3), "achieved": round(algo / bs / 1e9, 2),
                                  "frac": round(algo / bs / 1e9 / HBM_PEAK_GBS, 4)}
    del slabs, outs, batches, ostructs, first
    torch.cuda.synchronize(dev)
    torch.cuda.empty_cache()
    return rec


def run_c5_mgpu(args, torch, MP, per, cols, entry):
    """C5: args.total_packets 64-B packets in contiguous shards over the devices (strong scaling):
    K parse steps through pkt_mgpu_parse_steps, then pkt_mgpu_parse_gather (merge = 0) to device 0,
    which moves each shard's packed tuples with only its used slot rows; parse and parse + gather
    timed separately (wall clock around each, devices idle on both sides)."""
    from pktgpu import dist as pdist, mgpu, schema
    nd = MP.ndev
    shards, outs = [], []
    ring = 2
    for i, pd in enumerate(per):
        lo, hi = pdist.shard_range(args.total_packets, nd, i)
        ni = hi - lo
        first = pd["slabs"][0]
        reps = -(-ni // (first.numel() // 64))
        base = first.repeat(reps)[:ni * 64].contiguous()
        slabs = [base] + [base.clone() for _ in range(ring - 1)]
        shards.append([(s, ni, 64, None, None) for s in slabs])
        outs.append([torch.empty(max(1, mgpu.packed_bytes(cols, ni)), dtype=torch.uint8, device=base.device)
                     for _ in range(ring)])
    K = max(4, min(args.steps, 20))
    plan = MP.steps_plan([[(shards[i][k % ring], outs[i][k % ring]) for i in range(nd)] for k in range(K + 2)])
    MP.parse_steps(plan, entry, cols, first=0, count=2, streams=args.streams)
    MP.synchronize()
    t0 = time.perf_counter()
    MP.parse_steps(plan, entry, cols, first=2, count=K, streams=args.streams)
    MP.synchronize()
    el = time.perf_counter() - t0
    rec = {"workload": f"C5: {args.total_packets} x 64 B Ether/IPv4/UDP, contiguous shards over {nd} GPU(s)",
           "scaling": "strong", "packets_per_gpu": [s[0][1] for s in shards], "steps": K,
           "ms_per_step": round(el / K * 1e3, 5), "Gpkt/s": round(args.total_packets * K / el / 1e9, 4)}
    # parse + gather (one step, blocking), and the parse alone the same way; the gather twice: every
    # piece through RCCL (pkt_mgpu_set_root_copy(0): the root's own shard by ncclSend/ncclRecv to
    # itself, so RCCL moves bytes at N = 1 too), and the root's own pieces by device copy (default)
    one = [shards[i][0] for i in range(nd)]
    recv = torch.empty(MP.recv_bytes(one, cols, False), dtype=torch.uint8, device=MP.torch_devices[0])
    sh_out = [outs[i][0] for i in range(nd)]

    recv_m = torch.empty(MP.recv_bytes(one, cols, True), dtype=torch.uint8, device=MP.torch_devices[0])

    def timed_gather(root_copy, merge=False, rows=0):
        MP.set_root_copy(root_copy)
        MP.set_gather_rows(rows)
        rb = recv_m if merge else recv
        MP.parse_gather(one, columns=cols, merge=merge, shard_out=sh_out, recv=rb)  # warm (RCCL channels)
        MP.synchronize()
        tp, tg = [], []
        for _ in range(9):
            t0 = time.perf_counter()
            MP.parse(one, columns=cols, shard_out=sh_out)
            MP.synchronize()
            tp.append(time.perf_counter() - t0)
            t0 = time.perf_counter()
            MP.parse_gather(one, columns=cols, merge=merge, shard_out=sh_out, recv=rb)
            MP.synchronize()
            tg.append(time.perf_counter() - t0)
        MP.set_root_copy(True)
        MP.set_gather_rows(0)
        return float(np.median(tp)), float(np.median(tg)), max(min(tg) - min(tp), 1e-9)

    parse_s, pg_s, gmin_s = timed_gather(False)
    parse_c, pg_c, _ = timed_gather(True)
    parse_m, pg_m, _ = timed_gather(False, merge=True)
    rows = int(max(int(o["n_hdrs"].max().item()) for o in
                   [mgpu.packed_views(sh_out[i], cols, one[i][1]) for i in range(nd)]))
    parse_q, pg_q, _ = timed_gather(False, rows=rows)  # the caller's row bound: no host wait
    plan, _ = mgpu.gather_plan(cols, [sh[1] for sh in one], [rows] * nd, False)
    plan_m, _ = mgpu.gather_plan(cols, [sh[1] for sh in one], [rows] * nd, True)
    moved = [sum(p[3] for p in plan if p[0] == i) for i in range(nd)]
    gather_s = max(pg_s - parse_s, 1e-9)
    gather_c = max(pg_c - parse_c, 1e-9)
    gather_m = max(pg_m - parse_m, 1e-9)
    rec["gather"] = {"entry": "pkt_mgpu_parse_gather (merge = 0, root = device 0, pkt_mgpu_set_root_copy(0): "
                              "every shard's pieces, the root's own included, by grouped ncclSend/ncclRecv)",
                     "parse_ms": round(parse_s * 1e3, 4), "parse_plus_gather_ms": round(pg_s * 1e3, 4),
                     "gather_ms": round(gather_s * 1e3, 4),
                     "gather_min_ms": round(gmin_s * 1e3, 4),
                     "bytes_per_pkt_moved": round(sum(moved) / args.total_packets, 2),
                     "slot_rows_moved": rows,
                     "bytes_into_root": sum(moved),
                     "bytes_from_other_devices": sum(moved) - moved[0],
                     "GB/s_into_root": round(sum(moved) / gather_s / 1e9, 2),
                     "rccl_messages": len(plan),
                     "backend": "RCCL (ncclCommInitAll, grouped ncclSend/ncclRecv over xGMI; at N = 1 the root's "
                                "send to itself)" if not MP.virtual else
                                "VIRTUAL handle: hipMemcpyAsync on one device in place of RCCL (test mode)",
                     "root_copy": {"gather_ms": round(gather_c * 1e3, 4),
                                   "parse_plus_gather_ms": round(pg_c * 1e3, 4),
                                   "what": "pkt_mgpu_set_root_copy(1), the default: the root's own pieces by "
                                           "hipMemcpyAsync on the root stream, the others by RCCL"},
                     "merged": {"gather_ms": round(gather_m * 1e3, 4), "parse_plus_gather_ms": round(pg_m * 1e3, 4),
                                "rccl_messages": len(plan), "repack_pieces": len(plan_m),
                                "rccl_messages_if_sent_per_column": len(plan_m),
                                "what": "merge = 1 (the whole batch's layout on the root), root copy off: the "
                                        "merge = 0 messages into the root's staging area, then one repack "
                                        "kernel placing every (shard, column / slot row) piece"},
                     "queued": {"parse_plus_gather_ms": round(pg_q * 1e3, 4), "rows": rows,
                                "what": "pkt_mgpu_set_gather_rows(rows): the caller's row bound, so parse and "
                                        "gather are queued with no host wait (root copy off, merge = 0)"},
                     "timing": "wall clock around each blocking call (+ synchronize), median of 9 "
                               "(min: gather_min_ms); gather = (parse + gather) - parse; the call's slot-row count "
                               "is reduced inside the parse kernel and read back once per device"}
    return rec


# ------------------------------------------------------------------------------ entry
def main():
    args = parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    ndev = world if world > 1 else args.gpus
    if args.virtual and world > 1:
        print("bench.py: --virtual runs in one process (no torch.distributed.run)", file=sys.stderr)
        sys.exit(2)
    if world > 1 and world != args.gpus and rank == 0:
        print(f"bench.py: WORLD_SIZE={world} overrides --gpus {args.gpus}", file=sys.stderr)
    dist = None
    if world > 1:
        # launched as one process per GPU: rank 0 drives all `world` devices through pkt_mgpu, the
        # other ranks wait here without touching a GPU (CPU barrier)
        import datetime
        import torch.distributed as dist
        dist.init_process_group("gloo", timeout=datetime.timedelta(minutes=30))
        if rank != 0:
            dist.barrier()
            dist.destroy_process_group()
            return
    try:
        res = run_mgpu(args, ndev)
    finally:
        if dist is not None:
            dist.barrier()
            dist.destroy_process_group()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
