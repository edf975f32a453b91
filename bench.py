#!/usr/bin/env python3
"""Benchmark: device-resident batched parse of packet slabs on MI355X (BASELINE.json metric).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4]
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

A step = one pkt_parse_batch launch over one batch of 2^20 packets (config C2 by default:
64-byte Ether/IPv4/UDP, fixed stride) producing the chain + Ether/IPv4/UDP field tuple +
recomputed IPv4 checksum.  Each step reads a different slab of a >= 1 GiB ring (and writes a
different output set), so the 256 MiB Infinity Cache cannot serve the working set.  Inputs are
resident in HBM before the timed region starts.

Multi-GPU, one process per GPU: under torch.distributed.run the ranks come from the environment;
`python bench.py --gpus N` (N > 1) starts the N ranks itself (one child per device, spawned before
anything touches the GPU) and fails if fewer than N devices are visible.  Every rank parses its
own 2^20-packet batch per step (weak scaling, no collective in the step).  A second record ("c5")
times the C5 config: 2^24 packets in total, split in contiguous shards over the ranks (strong
scaling), and the RCCL gather of the shards' packed tuple buffers to rank 0 — timed separately.

Prints ONE JSON line on rank 0 (see DESIGN.md "Measurement" for every field).
"""
import argparse
import json
import os
import socket
import subprocess
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
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend (nccl = RCCL)")
    ap.add_argument("--fastpath", type=int, default=int(os.environ.get("PKTGPU_FASTPATH", "1")),
                    help="register fast path for Ether/IPv4/UDP|TCP (pkt_ctx_set_fastpath)")
    ap.add_argument("--staging", type=int, default=int(os.environ.get("PKTGPU_STAGING", "0")),
                    help="pkt_ctx_set_staging: 0 auto, 1 per-lane windows, 2 wave spans")
    ap.add_argument("--window", type=int, default=int(os.environ.get("PKTGPU_WINDOW", "0")),
                    help="pkt_ctx_set_window bytes (0 = auto)")
    ap.add_argument("--streams", type=int, default=2,
                    help="consecutive steps are issued round-robin on this many HIP streams")
    return ap.parse_args()


# ------------------------------------------------------------------------------ rank launcher
def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(args):
    """`bench.py --gpus N` outside torch.distributed.run: start N rank processes, one per device.
    Nothing here touches the GPU (torch.cuda.device_count() does not initialise it), so the
    children start from a clean process."""
    import torch
    ndev = torch.cuda.device_count()
    if ndev == 0 or (args.backend == "nccl" and ndev < args.gpus):
        print(f"bench.py: --gpus {args.gpus} but only {ndev} device(s) visible", file=sys.stderr)
        return 2
    port = free_port()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 1
                for q in live:  # one rank failed: the others would wait forever in a collective
                    q.kill()
        time.sleep(0.05)
    return rc


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


def max_over_ranks(torch, dist, world, x, dev, backend):
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sync_barrier(torch, dist, world):
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()


def run_c5(args, torch, dist, P, world, rank, dev, cols, d_first, entry):
    """C5: args.total_packets 64-B packets split in contiguous shards over the ranks (strong
    scaling), timed like the main loop; then the RCCL gather of one step's packed shard tuples to
    rank 0 (dist.gather of each rank's single packed buffer), timed separately."""
    from pktgpu import dist as pdist
    lo, hi = pdist.shard_range(args.total_packets, world, rank)
    n5 = hi - lo
    # the shard: the rank's seeded C2 slab repeated (the parse cost depends only on the layout)
    reps = -(-n5 // (d_first.numel() // 64))
    base = d_first.repeat(reps)[:n5 * 64].contiguous()
    ring = max(2, int(np.ceil((1 << 30) / max(1, base.numel()))))
    slabs = [base] + [base.clone() for _ in range(ring - 1)]
    outs = packed_outputs(torch, dev, cols, n5, ring)
    batches = [P._batch(s, n5, 64, None, None) for s in slabs]
    ostr = [P.out_struct(o[1]) for o in outs]
    streams = [torch.cuda.Stream(dev) for _ in range(max(1, args.streams))]
    K = max(4, min(args.steps, 40))

    def step(k):
        P.launch(batches[k % ring], entry, ostr[k % ring], streams[k % len(streams)])

    for k in range(2 * ring):
        step(k)
    sync_barrier(torch, dist, world)
    t0 = time.perf_counter()
    for k in range(K):
        step(k)
    sync_barrier(torch, dist, world)
    el = max_over_ranks(torch, dist, world, time.perf_counter() - t0, dev, args.backend)
    rec = {"workload": f"C5: {args.total_packets} x 64 B Ether/IPv4/UDP, contiguous shards over {world} GPU(s)",
           "scaling": "strong", "packets_per_gpu": n5, "steps": K,
           "ms_per_step": round(el / K * 1e3, 5), "Gpkt/s": round(args.total_packets * K / el / 1e9, 4)}
    if world > 1:
        buf = outs[0][0] if args.backend == "nccl" else outs[0][0].cpu()
        nmax = pdist.shard_range(args.total_packets, world, 0)[1]  # shard 0 is the largest
        from pktgpu import mgpu
        cap = mgpu.packed_bytes(cols, nmax)
        if buf.numel() < cap:  # equal-size messages for dist.gather
            pad = torch.zeros(cap, dtype=torch.uint8, device=buf.device)
            pad[:buf.numel()] = buf
            buf = pad
        glist = [torch.empty_like(buf) for _ in range(world)] if rank == 0 else None
        dist.gather(buf, glist, dst=0)  # warm (communicator + channels)
        sync_barrier(torch, dist, world)
        G = 5
        tg = time.perf_counter()
        for _ in range(G):
            dist.gather(buf, glist, dst=0)
        sync_barrier(torch, dist, world)
        gs = max_over_ranks(torch, dist, world, (time.perf_counter() - tg) / G, dev, args.backend)
        into_root = buf.numel() * (world - 1)
        rec["gather"] = {"ms": round(gs * 1e3, 4), "bytes_into_root": into_root,
                         "GB/s_into_root": round(into_root / gs / 1e9, 2),
                         "message": "one packed tuple buffer per rank (pkt_out_packed layout)",
                         "backend": "nccl (RCCL over xGMI)" if args.backend == "nccl" else args.backend,
                         "parse_plus_gather_ms": round(el / K * 1e3 + gs * 1e3, 4)}
    return rec


# ------------------------------------------------------------------------------ one rank
def main():
    args = parse_args()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"bench.py: WORLD_SIZE={world} overrides --gpus {args.gpus}", file=sys.stderr)
    import torch
    import torch.distributed as dist
    ndev = torch.cuda.device_count()
    if ndev == 0:
        print("bench.py: no GPU visible", file=sys.stderr)
        sys.exit(2)
    if args.backend == "nccl" and ndev < world:
        print(f"bench.py: {world} ranks but only {ndev} device(s) visible", file=sys.stderr)
        sys.exit(2)
    gpu = local % ndev  # gloo rehearsal only: several ranks may share one device
    torch.cuda.set_device(gpu)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group(args.backend)
    dev = torch.device("cuda", gpu)

    import pktgpu
    from pktgpu import schema
    P = pktgpu.Parser(gpu)
    P.set_fastpath(args.fastpath)
    P.set_staging(args.staging)
    P.set_window(args.window)
    default_cols = {"c2": "chain,ether,ipv4,udp", "c3": "chain,ether,vlan,ipv4,tcp,udp",
                    "c4": "all", "c5": "chain,ether,ipv4,udp"}[args.config]
    if args.columns is None:
        args.columns = default_cols
    cols = pktgpu.resolve_columns("all" if args.columns == "all" else args.columns.split(","))
    n = args.packets
    if args.config == "c5":  # strong scaling: this rank's contiguous block of the global batch
        from pktgpu import dist as pdist
        lo, hi = pdist.shard_range(args.total_packets, world, rank)
        n = hi - lo

    # ---------------- input: one seeded batch per rank, replicated over a >= ring_gib ring
    slab_np, stride, offs_np, lens_np = make_input(args.config, n, seed=0x5EED0000 + 2 + rank)
    slab_bytes = slab_np.size
    ring = max(2, int(np.ceil(args.ring_gib * (1 << 30) / slab_bytes)))
    d_first = torch.from_numpy(slab_np).to(dev)
    slabs = [d_first] + [d_first.clone() for _ in range(ring - 1)]
    d_offs = torch.from_numpy(offs_np).to(dev) if offs_np is not None else None
    d_lens = torch.from_numpy(lens_np).to(dev) if lens_np is not None else None
    outs = packed_outputs(torch, dev, cols, n, ring)
    entry = schema.ENTRY_ID["parse"]
    batches = [P._batch(slabs[r], n, stride, d_offs, d_lens) for r in range(ring)]
    ostructs = [P.out_struct(outs[r][1]) for r in range(ring)]
    streams = [torch.cuda.Stream(dev) for _ in range(max(1, args.streams))]

    def step(k):
        P.launch(batches[k % ring], entry, ostructs[k % ring], streams[k % len(streams)])

    for k in range(args.warmup):
        step(k)
    sync_barrier(torch, dist, world)

    # ---------------- timed region: K steps round-robin over the streams (step k+1 may start
    # while step k drains).  One event pair brackets the region on stream 0, which joins the others.
    s0 = streams[0]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(s0)
    for s_ in streams[1:]:
        s_.wait_stream(s0)
    for k in range(args.steps):
        step(args.warmup + k)
    for s_ in streams[1:]:
        s0.wait_stream(s_)
    e1.record(s0)
    sync_barrier(torch, dist, world)
    elapsed = max_over_ranks(torch, dist, world, time.perf_counter() - t0, dev, args.backend)
    region_ms = e0.elapsed_time(e1)

    # ---------------- roofline sub-phase: the parse kernel in isolation — R back-to-back launches
    # on ONE stream between one event pair on that stream — alternated with the ceiling probe
    # (same launch shape, same bytes, no parsing; C2-shaped configs only).  Median of 5 rounds.
    R = min(args.steps, 50)
    rs = streams[0]
    probe = load_probe() if (args.config in ("c2", "c5") and args.columns == default_cols) else None

    def parse_launch(k, s):
        P.launch(batches[k % ring], entry, ostructs[k % ring], s)

    def probe_launch(k, s):
        import ctypes
        rc = probe.pkt_probe_ceiling(ctypes.c_void_p(slabs[k % ring].data_ptr()), n, stride,
                                     ctypes.byref(ostructs[k % ring]), ctypes.c_void_p(s.cuda_stream))
        if rc != 0:
            raise RuntimeError(f"pkt_probe_ceiling failed ({rc})")

    # the practical HBM rate of this box: a device copy of the slab (read + write), same ring
    copy_dst = torch.empty_like(d_first)

    def copy_launch(k, s):
        with torch.cuda.stream(s):
            copy_dst.copy_(slabs[k % ring])

    kern, ceil_, copy_ = [], [], []
    for _ in range(5):
        kern.append(event_avg_ms(torch, rs, parse_launch, R))
        if probe is not None:
            ceil_.append(event_avg_ms(torch, rs, probe_launch, R))
        copy_.append(event_avg_ms(torch, rs, copy_launch, R))
    del copy_dst
    # the probe overwrote output sets: re-parse them so the last step's columns are real
    for r in range(ring):
        parse_launch(r, rs)
    torch.cuda.synchronize()

    c5 = None
    if args.config == "c2" and not args.no_c5:
        c5 = run_c5(args, torch, dist, P, world, rank, dev, cols, d_first, entry)

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return

    o0 = outs[0][1]
    used_slots = int(o0["n_hdrs"].max().item()) if "n_hdrs" in o0 else 0
    span = o0["payload_off"].cpu().numpy() if "payload_off" in o0 else np.full(n, 64, np.int64)
    read_b, write_b = algorithmic_bytes(n, cols, max(used_slots, 1), span)
    algo = read_b + write_b
    avg_kern_s = float(np.median(kern)) * 1e-3
    achieved = algo / avg_kern_s / 1e9
    pkts_total = n * world * args.steps  # c5: = total_packets * steps (even shards)
    value = pkts_total / elapsed / 1e9
    pipe_s = region_ms * 1e-3 / args.steps
    agg_gbs = algo * world * args.steps / elapsed / 1e9
    res = {
        "metric": METRIC,
        "value": round(value, 4),
        "unit": "Gpkt/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 5),
        "higher_is_better": True,
        "scaling": "strong" if args.config == "c5" else "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seeded generator, pktgpu/gen.py)",
        "config": {
            "workload": {"c2": "C2: 2^20 x 64 B Ether/IPv4/UDP fixed-stride slab per GPU",
                         "c5": f"C5: {args.total_packets} x 64 B Ether/IPv4/UDP sharded over {world} GPU(s)",
                         "c3": "C3: 2^20 x 128 B Ether/{0-2}xVlan/IPv4/TCP|UDP per GPU",
                         "c4": "C4: 2^20-record pcap replay of the 22 reference templates per GPU"}[args.config],
            "packets_per_gpu": n, "entry": "fast::parse", "columns": args.columns,
            "ring_slabs": ring, "ring_bytes": ring * slab_bytes, "parallelism": f"dp{world}",
            "staging": args.staging, "window": args.window,
        },
        "GB/s": {"algorithmic": round(agg_gbs, 2),
                 "slab": round(slab_bytes * world * args.steps / elapsed / 1e9, 2),
                 "algorithmic_bytes_per_pkt": {"read": read_b / n, "written": write_b / n},
                 "aggregate_frac_of_n_x_peak": round(agg_gbs / (world * HBM_PEAK_GBS), 4)},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                     "frac_kind": "kernel: algorithmic bytes / isolated launch duration (HIP events, "
                                  "one stream) / 8 TB/s spec",
                     "kernel": "parse_kernel", "avg_kernel_us": round(avg_kern_s * 1e6, 3),
                     "read_only_frac": round(read_b / avg_kern_s / 1e9 / HBM_PEAK_GBS, 4),
                     "measured": f"median of 5 rounds of {R} back-to-back launches on one stream, one "
                                 f"HIP event pair per round",
                     "algorithmic_bytes_per_launch": algo,
                     # the timed region: K launches pipelined over `streams` streams
                     "pipelined": {"streams": len(streams),
                                   "device_ms_per_step": round(pipe_s * 1e3, 5),
                                   "achieved": round(algo / pipe_s / 1e9, 2),
                                   "frac": round(algo / pipe_s / 1e9 / HBM_PEAK_GBS, 4),
                                   "frac_kind": "throughput: algorithmic bytes per step / device time "
                                                "per step of the pipelined timed region / 8 TB/s"}},
    }
    if ceil_:
        cs = float(np.median(ceil_)) * 1e-3
        res["roofline"]["ceiling"] = {
            "kernel": "pkt_probe_ceiling (libpktprobe.so): same launch shape and bytes, no parsing",
            "avg_kernel_us": round(cs * 1e6, 3), "achieved": round(algo / cs / 1e9, 2),
            "frac_of_peak": round(algo / cs / 1e9 / HBM_PEAK_GBS, 4),
            "parse_frac_of_ceiling": round(cs / avg_kern_s, 4)}
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
    if os.path.exists(tpath) and args.columns == default_cols and n == 1 << 20:
        t = json.load(open(tpath))
        res["roofline"]["traffic"] = t["traffic_bytes_per_launch"]
        res["roofline"]["traffic_source"] = {
            "measured_in_this_run": False,
            "file": f"profiles/traffic_{args.config}.json",
            "how": "rocprofv3 --pmc FETCH_SIZE (x2, gfx950) and WRITE_SIZE, separate passes of "
                   "this bench command (scripts/gpu_round.sh)",
            "x2_check": "every memory-side read request of these launches is a 128-B line "
                        "(TCC_EA0_RDREQ_128B = TCC_EA0_RDREQ; FETCH_SIZE counts 64 B per request): "
                        "profiles/ab/r02calib_fetch_requests.txt",
            "run": t.get("label", "")}
    if c5 is not None:
        res["c5"] = c5
    if world == 1 and not args.no_cpu_baseline:
        cores, aff, quota = host_cores()
        threads = args.cpu_threads or cores
        res["cpu_baseline"] = cpu_baseline(slab_np, stride, offs_np, lens_np, n, cols, threads)
        res["cpu_baseline"]["host"] = {"affinity_cpus": aff, "cgroup_cpu_quota": quota,
                                       "os_cpu_count": os.cpu_count()}
    print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
