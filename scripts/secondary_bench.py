#!/usr/bin/env python3
"""Measurements of the §8(f) kernels beside the hot path: one JSON line per workload.

  pktgen_clone   tests/lib.rs:770-776  pkt.clone().to_vec() of test_tcp_packet (154 B), n times
  pktgen_update  tests/lib.rs:778-787  set_etype(i % 0xFFFF), clone, to_vec
  pktgen_new     tests/lib.rs:762-768  every builder argument of test_tcp_packet varied per packet
                 (MACs, IPs, tos, ttl, id, ports, seq, ack: splitmix64) + the IPv4 checksum refresh
  pktgen_values  the same fields from per-packet value arrays (8 B read per field per packet)
  to_vec_c2 / to_vec_c4   PacketSlice::to_vec of every parsed packet (tests/lib.rs:790-817), C2 slab
                 and C4 pcap replay, into the input's layout; to_vec_c4_packed: the C4 outputs
                 packed back to back (dst_offsets = prefix of the lengths)
  extract_c2     every field of Ether/IPv4/UDP (19 specs, one launch) over C2 (headers.rs:195-201)
  setfields_c2   4 setters + the IPv4 checksum refresh, in place over C2 (headers.rs:315-324)

Each line: kernel time per launch (HIP events over back-to-back launches on one stream, outputs
from a >= 1 GiB ring), Gpkt/s, algorithmic bytes per packet (what the kernel must read + write),
roofline frac vs 8 TB/s, and the CPU restatement (oracle/) on a bounded sample with every core this
process may use.  Parity of each workload's output is checked against the oracle on a sample.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "packet-rs_amd"), os.path.join(REPO, "oracle"), REPO]
import pktgpu  # noqa: E402
from pktgpu import gen, pktgen, schema  # noqa: E402

PEAK = 8000.0  # GB/s, MI355X HBM3E spec


def host_cores():
    aff = len(os.sched_getaffinity(0))
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            return min(aff, max(1, int(int(q) / int(per))))
    except (OSError, ValueError):
        pass
    return aff


def timed(fn, budget):
    reps, t0 = 0, time.perf_counter()
    while reps < 1 or time.perf_counter() - t0 < budget:
        fn()
        reps += 1
    return reps, time.perf_counter() - t0


def prepared_extract(P, slab, chain, specs):
    """pkt_extract_fields over a fixed-stride (64 B) slab with its arguments built once."""
    import ctypes
    b = P._batch(slab, None, 64, None, None)
    ch = P._chain(chain)
    k = len(specs)
    sp = (P._lib.PktFieldSpec * k)()
    for j, (t, occ, s0, e0) in enumerate(specs):
        sp[j] = P._lib.PktFieldSpec(schema.HDR_ID[t] if isinstance(t, str) else int(t), occ, s0, e0, 0)
    vals = [torch.empty(b.n, dtype=torch.uint64, device=slab.device) for _ in range(k)]
    found = [torch.empty(b.n, dtype=torch.uint8, device=slab.device) for _ in range(k)]
    vp = (ctypes.c_void_p * k)(*[v.data_ptr() for v in vals])
    fp = (ctypes.c_void_p * k)(*[f.data_ptr() for f in found])
    args = (P._ctx, ctypes.byref(b), ctypes.byref(ch), sp, k, vp, fp, P._stream(None))
    keep = (b, ch, sp, vals, found, vp, fp)

    def launch():
        assert P._L.pkt_extract_fields(*args) == 0 and keep
    return launch


def event_ms(launch, iters, warm=3):
    s = torch.cuda.current_stream()
    for k in range(warm):
        launch(k)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for k in range(iters):
        launch(k)
    b.record(s)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


_PROBE = []


def copy_ceiling(n, read_b, write_b, dev, it, kernel_ms):
    """The no-work ceiling of a workload's byte shape (as the C2 line's
    roofline.ceiling.stream_copy): libpktprobe's hand-written streaming copy reading read_b and writing
    write_b bytes per packet (16-byte global_load/store_dwordx4 by consecutive lanes, 1 KiB contiguous
    per wave instruction, 4 loads in flight per lane), one launch per batch over a >= 1 GiB ring, HIP
    events on one stream.  `kernel_frac_of_copy` = copy time / the workload's kernel time."""
    import ctypes
    from bench import load_probe
    if not _PROBE:
        _PROBE.append(load_probe())
    L = _PROBE[0]
    if L is None:
        return None
    rb, wb = (int(read_b * n) + 15) // 16 * 16, (int(write_b * n) + 15) // 16 * 16
    per = max(rb, wb, 16)
    ring = max(2, (1 << 30) // per + 1)
    srcs = [torch.empty(max(rb, 16), dtype=torch.uint8, device=dev) for _ in range(min(ring, 8))]
    dsts = [torch.empty(max(wb, 16), dtype=torch.uint8, device=dev) for _ in range(ring)]
    P8 = ctypes.POINTER(ctypes.c_uint8)
    sp = [(P8 * 1)(ctypes.cast(ctypes.c_void_p(t.data_ptr()), P8)) for t in srcs]
    dp = [(P8 * 1)(ctypes.cast(ctypes.c_void_p(t.data_ptr()), P8)) for t in dsts]
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    def launch(k):
        assert L.pkt_probe_stream_copy(sp[k % len(sp)], dp[k % ring], 1, rb, wb, st) == 0
    ms = min(event_ms(launch, it) for _ in range(3))
    del srcs, dsts
    torch.cuda.empty_cache()
    gbs = (rb + wb) / (ms * 1e-3) / 1e9
    return {"kernel": "pkt_probe_stream_copy (libpktprobe.so): the workload's read and written bytes, contiguous, "
                      "no work", "read_bytes": rb, "written_bytes": wb, "copy_us": round(ms * 1e3, 2),
            "copy_frac_of_peak": round(gbs / PEAK, 4), "kernel_frac_of_copy": round(ms / kernel_ms, 4),
            "measured": "min of 3 rounds of HIP events over back-to-back one-batch launches, same stream"}


def line(name, n, ms, read_b, write_b, cpu, extra=None):
    gbs = (read_b + write_b) * n / (ms * 1e-3) / 1e9
    d = {"workload": name, "packets": n, "kernel_us": round(ms * 1e3, 2), "Gpkt/s": round(n / (ms * 1e-3) / 1e9, 3),
         "algorithmic_bytes_per_pkt": {"read": read_b, "written": write_b},
         "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK, "unit": "GB/s",
                      "frac": round(gbs / PEAK, 4)},
         "cpu_baseline": cpu}
    if extra:
        d.update(extra)
    if CEILING[0]:
        c = copy_ceiling(n, read_b, write_b, torch.device("cuda", 0), 20, ms)
        if c is not None:
            d["roofline"]["ceiling"] = c
    print(json.dumps(d), flush=True)


CEILING = [True]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--cpu-budget", type=float, default=3.0)
    ap.add_argument("--only", default="")
    ap.add_argument("--no-ceiling", action="store_true", help="skip the streaming-copy ceiling of each line")
    args = ap.parse_args()
    CEILING[0] = not args.no_ceiling
    import oracle
    oracle.build()
    n, it = args.n, args.iters
    cores = host_cores()
    P = pktgpu.Parser(0)
    dev = P.torch_device
    only = set(args.only.split(",")) if args.only else None

    def want(name):
        return only is None or name in only

    # ---------------------------------------------------------------- pktgen
    tpl = pktgen.test_tcp_template()
    stride = 160
    ring = max(2, (1 << 30) // (n * stride) + 1)
    outs = [torch.empty(n * stride, dtype=torch.uint8, device=dev) for _ in range(ring)]
    cpu_n = 1 << 18
    cpu_out = np.zeros((cpu_n, stride), np.uint8)

    def cpu_loop(mode):
        r, t = timed(lambda: oracle.pktgen_loop(tpl, cpu_n, stride, mode, nthreads=cores, out=cpu_out), args.cpu_budget)
        return {"value": round(r * cpu_n / t / 1e9, 6), "unit": "Gpkt/s", "cores": cores, "kind": "port",
                "sample": f"{r} x {cpu_n} packets of oracle.pktgen_loop({mode}) (owned Packet: Box per header, "
                          f"Arc<Mutex> header bytes, Vec-grown to_vec), {cores} threads"}

    if want("pktgen_clone"):
        G = pktgen.Generator(P, tpl)
        ms = event_ms(lambda k: G.run(n, stride, dst=outs[k % ring]), it)
        got = G.run(4096, stride).cpu().numpy().reshape(4096, stride)
        ok = np.array_equal(got, oracle.pktgen_loop(tpl, 4096, stride, "clone"))
        line("pktgen_clone", n, ms, 0, stride, cpu_loop("clone"), {"parity_vs_oracle": bool(ok), "stride": stride})
    if want("pktgen_update"):
        G = pktgen.Generator(P, tpl, [pktgen.Field("Ether", "etype", kind="inc", count=0xFFFF)])
        ms = event_ms(lambda k: G.run(n, stride, dst=outs[k % ring]), it)
        got = G.run(70000, stride).cpu().numpy().reshape(70000, stride)
        ok = np.array_equal(got, oracle.pktgen_loop(tpl, 70000, stride, "update"))
        line("pktgen_update", n, ms, 0, stride, cpu_loop("update"), {"parity_vs_oracle": bool(ok), "stride": stride})
    names = [("Ether", "dst"), ("Ether", "src"), ("IPv4", "src"), ("IPv4", "dst"), ("IPv4", "diffserv"),
             ("IPv4", "ttl"), ("IPv4", "identification"), ("TCP", "src"), ("TCP", "dst"), ("TCP", "seq_no"),
             ("TCP", "ack_no")]
    for kind in ("random", "values"):
        name = "pktgen_new" if kind == "random" else "pktgen_values"
        if not want(name):
            continue
        fs = [pktgen.Field(h, f, kind=kind, base=1000 + j) for j, (h, f) in enumerate(names)]
        G = pktgen.Generator(P, tpl, fs, csum=[0])
        vals = {}
        if kind == "values":
            g = torch.Generator(device="cpu").manual_seed(5)
            vals = {j: torch.randint(0, 2**62, (n,), generator=g, dtype=torch.int64).to(torch.uint64).to(dev)
                    for j in range(len(fs))}
        ms = event_ms(lambda k: G.run(n, stride, values=vals, dst=outs[k % ring]), it)
        m = 8192
        got = G.run(m, stride, values=vals).cpu().numpy().reshape(m, stride)
        gi = np.arange(m, dtype=np.uint64)
        hv = [f.value(gi, vals[j][:m].cpu().numpy() if kind == "values" else None) for j, f in enumerate(fs)]
        slab = np.zeros((m, stride), np.uint8)
        slab[:, :len(tpl)] = np.frombuffer(tpl, np.uint8)
        slab = slab.reshape(-1)
        lens = np.full(m, len(tpl), np.uint32)
        chain = oracle.parse_batch(slab, m, stride=stride, lens=lens, columns=["status", "n_hdrs", "hdr_type", "hdr_off"])
        oracle.set_fields(slab, m, chain, [(f.hdr, 0, f.start, f.end) for f in fs], hv, stride=stride, lens=lens)
        oracle.ipv4_update_checksum(slab, m, chain, 0, stride=stride, lens=lens)
        ok = np.array_equal(got.reshape(-1), slab)
        line(name, n, ms, 8 * len(fs) if kind == "values" else 0, stride, None,
             {"parity_vs_oracle": bool(ok), "stride": stride, "fields": len(fs),
              "cpu_note": "the reference's 'new packet' loop runs the utils.rs builders (string parsing, "
                          "per-header allocation); no C restatement of the builders is timed"})
    del outs

    # ---------------------------------------------------------------- to_vec / extract / set_fields
    c2 = gen.gen_c2(n).reshape(-1)
    ring2 = max(2, (1 << 30) // c2.size + 1)
    slabs = [torch.from_numpy(c2).to(dev) for _ in range(min(ring2, 4))]
    chains = [P.parse(s, stride=64, columns=["chain"]) for s in slabs]
    torch.cuda.synchronize()
    if want("to_vec_c2"):
        dsts = [torch.empty_like(slabs[0]) for _ in range(ring2)]
        ms = event_ms(lambda k: P.to_vec(slabs[k % len(slabs)], chains[k % len(slabs)], stride=64,
                                         dst=dsts[k % ring2]), it)
        out, _ = P.to_vec(slabs[0], chains[0], stride=64)
        ok = np.array_equal(out.cpu().numpy(), c2)
        cpu_m = 1 << 18
        r, t = timed(lambda: oracle.round_trip_batch(c2[:cpu_m * 64], cpu_m, stride=64, slow=True, nthreads=cores),
                     args.cpu_budget)
        # read: the packet bytes + status/n_hdrs/3 slots (type+off)/payload_off/len; written: bytes + out_len
        line("to_vec_c2", n, ms, 64 + 1 + 1 + 3 * 3 + 4, 64 + 4,
             {"value": round(r * cpu_m / t / 1e9, 6), "unit": "Gpkt/s", "cores": cores, "kind": "port",
              "sample": f"{r} x {cpu_m} packets of oracle slow::parse(..).to_vec()"},
             {"parity_vs_oracle": bool(ok)})
        del dsts
    if want("to_vec_c4"):
        s4, o4, l4 = gen.gen_c4(n)
        d4, do4, dl4 = torch.from_numpy(s4).to(dev), torch.from_numpy(o4).to(dev), torch.from_numpy(l4).to(dev)
        ch4 = P.parse(d4, offsets=do4, lens=dl4, columns=["chain"])
        dsts = [torch.empty_like(d4) for _ in range(max(2, (1 << 30) // s4.size + 1))]
        ms = event_ms(lambda k: P.to_vec(d4, ch4, offsets=do4, lens=dl4, dst=dsts[k % len(dsts)]), it)
        out, ln = P.to_vec(d4, ch4, offsets=do4, lens=dl4)
        want_b, wl = oracle.round_trip_batch(s4, n, offsets=o4, lens=l4, slow=True, nthreads=cores)
        o = out.cpu().numpy()
        mask = np.zeros(s4.size, bool)
        for t_, L_ in zip(o4[:20000], wl[:20000]):
            mask[int(t_):int(t_) + int(L_)] = True
        ok = np.array_equal(ln.cpu().numpy(), wl) and np.array_equal(o[mask], want_b[mask])
        avg = float(l4.mean())
        nh = int(np.asarray(ch4["n_hdrs"].cpu().numpy(), np.int64).mean() + 0.5)
        cpu_m = 1 << 17
        r, t = timed(lambda: oracle.round_trip_batch(s4, cpu_m, offsets=o4[:cpu_m], lens=l4[:cpu_m], slow=True,
                                                     nthreads=cores), args.cpu_budget)
        line("to_vec_c4", n, ms, round(avg + 8 + 4 + 1 + 1 + 3 * nh + 4, 1), round(avg + 4, 1),
             {"value": round(r * cpu_m / t / 1e9, 6), "unit": "Gpkt/s", "cores": cores, "kind": "port",
              "sample": f"{r} x {cpu_m} records of oracle slow::parse(..).to_vec()"},
             {"parity_vs_oracle_first_20000": bool(ok), "avg_record_bytes": round(avg, 1)})
        # the same records packed back to back (dst_offsets = prefix of the lengths: each to_vec
        # output Vec in a contiguous packet buffer, no pcap record headers between them)
        po = np.zeros(n, np.uint64)
        po[1:] = np.cumsum(l4[:-1].astype(np.uint64))
        tot = int(po[-1]) + int(l4[-1])
        dpo = torch.from_numpy(po).to(dev)
        dstp = [torch.empty(((tot + 15) // 16) * 16, dtype=torch.uint8, device=dev)
                for _ in range(max(2, (1 << 30) // tot + 1))]
        ms = event_ms(lambda k: P.to_vec(d4, ch4, offsets=do4, lens=dl4, dst=dstp[k % len(dstp)], dst_offsets=dpo), it)
        outp, lnp = P.to_vec(d4, ch4, offsets=do4, lens=dl4, dst=dstp[0], dst_offsets=dpo)
        op = outp.cpu().numpy()
        okp = np.array_equal(lnp.cpu().numpy(), wl) and all(
            np.array_equal(op[int(po[j]):int(po[j]) + int(wl[j])], want_b[int(o4[j]):int(o4[j]) + int(wl[j])])
            for j in range(0, n, max(1, n // 20000)))
        line("to_vec_c4_packed", n, ms, round(avg + 8 + 8 + 4 + 1 + 1 + 3 * nh + 4, 1), round(avg + 4, 1),
             {"value": round(r * cpu_m / t / 1e9, 6), "unit": "Gpkt/s", "cores": cores, "kind": "port",
              "sample": f"{r} x {cpu_m} records of oracle slow::parse(..).to_vec()"},
             {"parity_vs_oracle_sampled": bool(okp), "avg_record_bytes": round(avg, 1),
              "dst": "packed: dst_offsets = prefix of the lengths"})
        del dstp
        del dsts, d4
    if want("extract_c2"):
        from pktgpu import fields as F
        specs = [(h, 0, s0, e0) for h in ("Ether", "IPv4", "UDP") for (s0, e0) in F.FIELDS[schema.HDR_ID[h]].values()]
        # ctypes arguments and output columns built once per ring slot: the Python wrapper's per-call
        # argument marshalling and 38 output allocations take longer than the kernel
        prep = [prepared_extract(P, slabs[r], chains[r], specs) for r in range(len(slabs))]
        ms = event_ms(lambda k: prep[k % len(prep)](), it)
        vals, found = P.extract_fields(slabs[0], chains[0], specs, stride=64)
        m = 1 << 16
        ch_h = {k: np.ascontiguousarray(v.cpu().numpy()[..., :m]) for k, v in chains[0].items()}
        spec_ids = [(schema.HDR_ID[h], o, s0, e0) for h, o, s0, e0 in specs]
        wv, _ = oracle.extract_fields(c2[:m * 64], m, ch_h, spec_ids, stride=64)
        ok = all(np.array_equal(vals[j].cpu().numpy()[:m], wv[j]) for j in range(len(specs)))
        r, t = timed(lambda: oracle.extract_fields(c2[:m * 64], m, ch_h, spec_ids, stride=64), args.cpu_budget)
        # read: 64 B window (the headers) + n_hdrs + 3 slots; written: 8 B value + 1 B found per spec
        line("extract_c2", n, ms, 64 + 1 + 9, 9 * len(specs),
             {"value": round(r * m / t / 1e9, 6), "unit": "Gpkt/s", "cores": 1, "kind": "port",
              "sample": f"{r} x {m} packets x {len(specs)} getters, oracle per-bit bit_range, 1 thread"},
             {"parity_vs_oracle": bool(ok), "specs": len(specs)})
    if want("setfields_c2"):
        fs = [("Ether", 0, 0, 47), ("IPv4", 0, 64, 71), ("IPv4", 0, 96, 127), ("UDP", 0, 0, 15)]
        g = torch.Generator(device="cpu").manual_seed(9)
        vals = [torch.randint(0, 2**62, (n,), generator=g, dtype=torch.int64).to(torch.uint64).to(dev) for _ in fs]

        def launch(k):
            s = slabs[k % len(slabs)]
            # setters + checksum refresh in one launch (pkt_set_fields_csum)
            P.set_fields(s, chains[k % len(slabs)], fs, vals, stride=64, ipv4_checksum=0)
        ms = event_ms(launch, it)
        m = 1 << 16
        s_cpu = c2[:m * 64].copy()
        ch_h = {k: np.ascontiguousarray(v.cpu().numpy()[..., :m]) for k, v in chains[0].items()}
        spec_ids = [(schema.HDR_ID[h], o, s0, e0) for h, o, s0, e0 in fs]
        vh = [v.cpu().numpy()[:m] for v in vals]
        oracle.set_fields(s_cpu, m, ch_h, spec_ids, vh, stride=64)
        oracle.ipv4_update_checksum(s_cpu, m, ch_h, 0, stride=64)
        ok = np.array_equal(slabs[0].cpu().numpy()[:m * 64], s_cpu)

        def cpu():
            s2 = c2[:m * 64].copy()
            oracle.set_fields(s2, m, ch_h, spec_ids, vh, stride=64)
            oracle.ipv4_update_checksum(s2, m, ch_h, 0, stride=64)
        r, t = timed(cpu, args.cpu_budget)
        # read: the 4 values + chain (n_hdrs + 3 slots) + the header lines touched; written: the fields
        line("setfields_c2 (+ipv4 checksum)", n, ms, 32 + 1 + 9 + 64, 64,
             {"value": round(r * m / t / 1e9, 6), "unit": "Gpkt/s", "cores": 1, "kind": "port",
              "sample": f"{r} x {m} packets x 4 setters + checksum, oracle per-bit set_bit_range, 1 thread"},
             {"parity_vs_oracle": bool(ok), "launches_per_step": 1})


if __name__ == "__main__":
    main()
