#!/usr/bin/env python3
"""Benchmark: device-resident batched parse of packet slabs on MI355X (BASELINE.json metric).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4]
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

A step = one pkt_parse_batch launch over one batch of 2^20 packets (config C2 by default:
64-byte Ether/IPv4/UDP, fixed stride) producing the chain + Ether/IPv4/UDP field tuple +
recomputed IPv4 checksum.  Each step reads a different slab of a >= 1 GiB ring (and writes a
different output set), so the 256 MiB Infinity Cache cannot serve the working set.  Inputs are
resident in HBM before the timed region starts.

Multi-GPU (one process per GPU): every rank parses its own batch (weak scaling, no collective
in the step); after the timed loop the per-packet tuples of one step are gathered to rank 0
with RCCL and timed separately ("gather" in the JSON line).

Prints ONE JSON line on rank 0 (see DESIGN.md "Measurement" for every field).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "packet-rs_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="c2", choices=["c2", "c3", "c4", "c5"],
                    help="c5 = 2^24 C2 packets in total, sharded over the ranks (strong scaling)")
    ap.add_argument("--total-packets", type=int, default=1 << 24, help="c5 only")
    ap.add_argument("--packets", type=int, default=1 << 20, help="packets per GPU per step")
    ap.add_argument("--ring-gib", type=float, default=1.0)
    ap.add_argument("--columns", default=None,
                    help="column groups; default per config: c2 chain,ether,ipv4,udp; "
                         "c3 chain,ether,vlan,ipv4,tcp,udp; c4 all")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=16)
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


def cpu_baseline(slab, stride, offs, lens, n, cols, threads):
    """The oracle (C restatement of packet_rs fast::parse + getters + ipv4_checksum, with the
    reference's per-header allocation and per-bit loops) on the host cores, bounded sample."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle
    oracle.build()
    n = min(n, 1 << 20)  # bounded sample (c5 shards are up to 2^24 packets)
    if offs is not None:
        offs, lens = offs[:n], lens[:n]
    # passes over the same slab until ~8 s of wall time (>= 2 passes): a bounded sample
    reps, t0 = 0, time.perf_counter()
    while reps < 2 or (time.perf_counter() - t0 < 8.0 and reps < 400):
        oracle.parse_batch(slab, n, stride=stride, offsets=offs, lens=lens, columns=cols,
                           nthreads=threads)
        reps += 1
    dt = time.perf_counter() - t0
    n1 = min(n, 1 << 19)
    t1 = time.perf_counter()
    oracle.parse_batch(slab, n1, stride=stride, offsets=offs[:n1] if offs is not None else None,
                       lens=lens[:n1] if lens is not None else None, columns=cols, nthreads=1)
    dt1 = time.perf_counter() - t1
    return {"value": round(reps * n / dt / 1e9, 6), "unit": "Gpkt/s", "cores": threads,
            "kind": "port",
            "sample": f"{reps} passes over the same {n}-packet slab ({reps * n} packets), "
                      f"{threads} threads, oracle/pkt_oracle.c -O2 (C restatement of packet_rs "
                      f"0.4.0 fast::parse + getters + ipv4_checksum)",
            "single_thread_gpkt_s": round(n1 / dt1 / 1e9, 6)}


def main():
    args = parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    ndev = torch.cuda.device_count()
    gpu = local % max(1, ndev)  # rehearsal only: several ranks may share one device (gloo)
    if world > 1:
        torch.cuda.set_device(gpu)
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group(args.backend)
    dev = torch.device("cuda", gpu)
    torch.cuda.set_device(dev)

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
        if args.total_packets % world:
            raise SystemExit("c5: --total-packets must divide evenly over the ranks (equal-size gather)")
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

    # output ring: every slot's columns are views of ONE contiguous buffer (gatherable)
    def alloc_packed():
        sizes, total = [], 0
        for c in cols:
            shp = schema.column_shape(c, n)
            nb = int(np.prod(shp)) * schema.column_dtype(c).itemsize
            sizes.append((c, shp, nb, total))
            total += (nb + 255) // 256 * 256
        buf = torch.empty(total, dtype=torch.uint8, device=dev)
        views = {}
        for c, shp, nb, o in sizes:
            views[c] = buf[o:o + nb].view(pktgpu._tdtype(schema.column_dtype(c))).view(shp)
        return buf, views

    outs = [alloc_packed() for _ in range(ring)]
    entry = schema.ENTRY_ID["parse"]
    batches, ostructs = [], []
    for r in range(ring):
        b = P._batch(slabs[r], n, stride, d_offs, d_lens)
        batches.append(b)
        ostructs.append(P.out_struct(outs[r][1]))
    streams = [torch.cuda.Stream(dev) for _ in range(max(1, args.streams))]

    def step(k):
        P.launch(batches[k % ring], entry, ostructs[k % ring], streams[k % len(streams)])

    for k in range(args.warmup):
        step(k)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()

    # ---------------- timed region: K steps round-robin over the streams (step k+1 may start
    # while step k drains).  No per-launch events here (each timing event costs the queue
    # several us); one event pair brackets the region on stream 0, which joins the others.
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
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    region_ms = e0.elapsed_time(e1)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if args.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # ---------------- roofline sub-phase: the kernel in isolation — R back-to-back launches on
    # ONE stream bracketed by one HIP event pair on that stream; avg launch duration =
    # elapsed / R (includes the ~1 us launch gaps; agrees with rocprofv3 --kernel-trace).
    R = min(args.steps, 50)
    rs = streams[0]
    f0, f1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    f0.record(rs)
    for k in range(R):
        P.launch(batches[k % ring], entry, ostructs[k % ring], rs)
    f1.record(rs)
    torch.cuda.synchronize()
    kern_ms = np.array([f0.elapsed_time(f1) / R])

    # ---------------- gather of one step's tuples to rank 0 (N > 1), timed separately
    gather = None
    if world > 1:
        buf = outs[0][0] if args.backend == "nccl" else outs[0][0].cpu()
        glist = [torch.empty_like(buf) for _ in range(world)] if rank == 0 else None
        dist.gather(buf, glist, dst=0)  # warm
        torch.cuda.synchronize()
        reps = 5
        dist.barrier()
        torch.cuda.synchronize()
        tg = time.perf_counter()
        for _ in range(reps):
            dist.gather(buf, glist, dst=0)
        torch.cuda.synchronize()
        dist.barrier()
        gms = (time.perf_counter() - tg) / reps * 1e3
        gbytes = buf.numel() * (world - 1)
        gather = {"ms": round(gms, 4), "bytes_into_root": gbytes,
                  "GB/s": round(gbytes / (gms * 1e-3) / 1e9, 2),
                  "backend": "nccl(RCCL)" if args.backend == "nccl" else args.backend,
                  "packets": n * world}

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return

    o0 = outs[(args.warmup + args.steps - 1) % ring][1]
    used_slots = int(o0["n_hdrs"].max().item()) if "n_hdrs" in o0 else 0
    if "payload_off" in o0:
        span = o0["payload_off"].cpu().numpy()
    else:
        span = np.full(n, 64, np.int64)
    read_b, write_b = algorithmic_bytes(n, cols, max(used_slots, 1), span)
    algo = read_b + write_b
    avg_kern_s = float(np.mean(kern_ms)) * 1e-3
    achieved = algo / avg_kern_s / 1e9
    pkts_total = n * world * args.steps  # c5: = total_packets * steps (even shards)
    value = pkts_total / elapsed / 1e9
    res = {
        "metric": "Gpkt/s + GB/s device-resident parse, 1M×64B Ether/IPv4/UDP, 1/2/4/8 MI355X",
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
        "GB/s": {"algorithmic": round(algo * world * args.steps / elapsed / 1e9, 2),
                 "slab": round(slab_bytes * world * args.steps / elapsed / 1e9, 2),
                 "algorithmic_bytes_per_pkt": {"read": read_b / n, "written": write_b / n}},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                     "kernel": "parse_kernel", "avg_kernel_us": round(avg_kern_s * 1e6, 3),
                     "read_only_frac": round(read_b / avg_kern_s / 1e9 / HBM_PEAK_GBS, 4),
                     "measured": f"{R} back-to-back launches on one stream, one HIP event pair",
                     # the timed region: K launches pipelined over `streams` streams
                     "pipelined": {"streams": len(streams),
                                   "device_ms_per_step": round(region_ms / args.steps, 5),
                                   "achieved": round(algo / (region_ms * 1e-3 / args.steps) / 1e9, 2),
                                   "frac": round(algo / (region_ms * 1e-3 / args.steps) / 1e9 / HBM_PEAK_GBS, 4)}},
    }
    # HBM traffic per launch from the committed rocprofv3 PMC passes of this config, if any
    tpath = os.path.join(REPO, "profiles", f"traffic_{args.config}.json")
    if os.path.exists(tpath) and args.columns == default_cols and n == 1 << 20:
        t = json.load(open(tpath))
        res["roofline"]["traffic"] = t["traffic_bytes_per_launch"]
        res["roofline"]["traffic_source"] = (f"profiles/traffic_{args.config}.json: rocprofv3 --pmc "
                                             f"FETCH_SIZE (x2, gfx950) + WRITE_SIZE, {t.get('label', '')}")
        res["roofline"]["algorithmic_bytes_per_launch"] = algo
    if gather is not None:
        res["gather"] = gather
    if world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(slab_np, stride, offs_np, lens_np, n, cols,
                                           min(args.cpu_threads, os.cpu_count() or 1))
    print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
