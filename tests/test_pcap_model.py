"""CPU model of the device pcap indexer's speculation + exact scan (pktgpu_pcap.hip): the same
regions, plausibility guess, per-region walk, state composition, local fix rounds, look-back
(from random earlier exact blocks: legal interleavings of the kernel's blocks) and fixes from the
exact exit, checked against the host indexer on captures built to make the guess wrong.  This pins
the algorithm's exactness claim without a GPU; tests/test_pcap_device.py checks the kernels themselves."""
import struct

import numpy as np

from pktgpu import gen

R = 4096


def u32(b, o):
    return struct.unpack_from("<I", b, o)[0] if o + 4 <= len(b) else int.from_bytes(
        (bytes(b[o:o + 4]) + b"\0\0\0\0")[:4], "little")


MIN_HOPS = 2  # kMinHops (pktgpu_pcap.hip)
MAX_HOPS = 2
ORIG_MAX = 1 << 20
TS_SPAN = 86400


def plausible(b, p, snap):
    usec, incl, orig = u32(b, p + 4), u32(b, p + 8), u32(b, p + 12)
    return (usec < 1000000 and incl != 0 and incl <= snap and incl <= orig and orig <= ORIG_MAX
            and p + 16 + incl <= len(b))


def chain_ok(b, c, stop, snap, lend=None):
    """Plausible headers from c to the region end (at most MAX_HOPS of them checked), and at
    least MIN_HOPS unless the file ends first; consecutive ts_sec within a day of each other.
    With `lend` (end of the block's staged bytes): 2 at the first hop past it."""
    p, hops, prev = c, 0, None
    while (p < stop or hops < MIN_HOPS) and hops < MAX_HOPS:
        if p + 16 > len(b):
            return 1
        if lend is not None and p >= lend:
            return 2
        if not plausible(b, p, snap):
            return 0
        sec = u32(b, p)
        if prev is not None and ((sec - prev + TS_SPAN) & 0xFFFFFFFF) > 2 * TS_SPAN:
            return 0
        prev = sec
        p += 16 + u32(b, p + 8)
        hops += 1
    return 1


def walk(b, base, entry, partial=False):
    """partial: `b` is a prefix of a capture (pkt_parse_pcap_host's pieces) — a record running past its
    end stops the walk like an error would, but is no error (the kernels drop the walk's error bit)."""
    pos, lst, err = entry, [], 0
    while pos < base + R and pos + 16 <= len(b):
        incl = u32(b, pos + 8)
        if pos + 16 + incl > len(b):
            return len(b), lst, 0 if partial else 1
        lst.append(pos)
        pos += 16 + incl
    return pos, lst, err


TILE = 4  # regions per guess block (staged together, pcap_guess_kernel)


def guess(b, k, snap):
    """First candidate of the region, 64 offsets per step: the lowest whose chain checks out in
    the tile's staged bytes (TILE regions + 16 B), else the lowest that checks out with reads past
    them, moved to the last of the run of consecutive verified candidates it starts, across steps
    (the run-last rule of guess_entry);
    none in the region -> "no record starts here"."""
    base = k * R
    stop = min(len(b), base + R)
    lend = (k // TILE + 1) * TILE * R
    run = None  # a run of verified candidates that reached the previous step's last lane
    for c0 in range(base, stop, 64):
        cs = [c for c in range(c0, min(c0 + 64, stop)) if c + 16 <= len(b)]
        rs = [chain_ok(b, c, stop, snap, lend) for c in cs]
        ok = {c for c, r in zip(cs, rs) if r == 1}
        if not ok:
            ok = {c for c, r in zip(cs, rs) if r == 2 and chain_ok(b, c, stop, snap) == 1}
        if run is not None and c0 not in ok:
            return run
        if ok:  # the last of the run of consecutive verified candidates (from the lowest, or continued)
            c = c0 if run is not None else min(ok)
            while c + 1 in ok:
                c += 1
            if c < c0 + 63:
                return c
            run = c
    return run if run is not None else base + R


B = 256  # regions per scan block (pcap_scan_kernel)


def combine(a, b):
    """The state composition of pktgpu_pcap.hip (run a, then run b).  An aggregate is ("none",
    end) — no region claims a record start, consistent with a predecessor exit >= end — or
    (first, last, cnt, err, bad)."""
    if a[0] == "none":
        return ("none", max(a[1], b[1])) if b[0] == "none" else b
    if b[0] == "none":
        return (a[0], a[1], a[2], a[3], a[4] or a[1] < b[1])
    return (a[0], b[1], a[2] + b[2], a[3] or b[3], a[4] or b[4] or a[1] != b[0])


IDENT = ("none", 0)


def region_agg(k, st):
    entry, (ex, lst, err) = st
    if k != 0 and entry >= (k + 1) * R:
        return ("none", (k + 1) * R)
    return (entry, ex, len(lst), bool(err), False)


def seam_bad(pre, r):
    if pre[0] == "none":
        return False
    return pre[1] < r[1] if r[0] == "none" else pre[1] != r[0]


def model_index(b, inject=None, order_seed=None, block=B, partial=False):
    """The three kernels restated: per-region guesses (`inject` {region: entry} overrides them:
    adversarial wrong guesses) and walks; per scan block of B regions the local fix rounds (a
    region disagreeing with the claiming region before it, while that one agrees with its own
    left, re-walks from its exit), the look-back — the block's exact prefix composed from the
    published aggregates back to a RANDOM earlier exact block (one legal interleaving per
    `order_seed`; the kernel stops at the nearest one) — and the fixes from the exact exit.
    `block` < B exercises many scan blocks on small captures.
    Asserts that every composition the kernel accepts gives the exact exit and count.  Returns
    (offsets, lens, regions re-walked)."""
    b = bytes(b)
    snap = u32(b, 16) or (1 << 30)
    K = (len(b) + R - 1) // R
    NB = (K + block - 1) // block
    rng = np.random.default_rng(order_seed if order_seed is not None else 0)
    st = []
    for k in range(K):  # the guess kernel: every region guesses its own entry
        e = 24 if k == 0 else (inject or {}).get(k, guess(b, k, snap))
        st.append((e, walk(b, k * R, e, partial)))
    fixed = 0

    def local_fixes(lo, hi):
        nonlocal fixed
        while True:
            pre, last_claim, bad = IDENT, -1, {}
            queue = []
            for k in range(lo, hi):
                r = region_agg(k, st[k])
                bad[k] = last_claim >= 0 and seam_bad(pre, r)
                if bad[k] and not bad[last_claim] and pre[1] >= k * R:
                    queue.append((k, pre[1]))
                if r[0] != "none":
                    last_claim = k
                pre = combine(pre, r)
            if not queue:
                return pre
            for k, e in queue:  # the waves of one round, from the states the round started with
                st[k] = (e, walk(b, k * R, e, partial))
                fixed += 1

    aggs = [local_fixes(q * block, min(K, (q + 1) * block)) for q in range(NB)]
    incl = []  # exact (exit, count, err) after each block
    for q in range(NB):
        lo, hi = q * block, min(K, (q + 1) * block)
        if q > 0:
            E, C, err = incl[q - 1]
            j = int(rng.integers(0, q))  # a look-back from exact block j through aggregates j+1..q-1
            acc = IDENT
            for x in range(j + 1, q):
                acc = combine(acc, aggs[x])
            e0, c0, r0 = incl[j]
            if acc[0] == "none":
                ok, got = e0 >= acc[1], (e0, c0, r0)
            else:
                ok, got = (not acc[4]) and acc[0] == e0, (acc[1], c0 + acc[2], r0 or acc[3])
            if ok:
                assert got == (E, C, err), (q, j)
            pre0 = (E, E, 0, False, False)
        else:
            E, C, err = 24, 0, False
            pre0 = IDENT
        while True:  # the first disagreeing seam against the exact exit, until none
            pre, todo = pre0, None
            for k in range(lo, hi):
                r = region_agg(k, st[k])
                if seam_bad(pre, r) and not pre[4]:
                    assert pre[1] >= k * R
                    todo = (k, pre[1])
                    break
                pre = combine(pre, r)
            if todo is None:
                break
            st[todo[0]] = (todo[1], walk(b, todo[0] * R, todo[1], partial))
            fixed += 1
        tot = IDENT
        for k in range(lo, hi):
            tot = combine(tot, region_agg(k, st[k]))
        aggs[q] = tot
        if tot[0] == "none":
            incl.append((E, C, err))
        else:
            incl.append((tot[1], C + tot[2], err or tot[3]))
    if incl[-1][2]:
        raise ValueError("truncated pcap record")
    offs, lens = [], []
    for k in range(K):
        _, (ex, lst, _) = st[k]
        for i, p in enumerate(lst):
            nxt = lst[i + 1] if i + 1 < len(lst) else ex
            offs.append(p + 16)
            # (partial: a walk stopped by a record past the prefix's end left the region's exit at
            # that end, so the emit reads the region's last incl_len from its header)
            lens.append(u32(b, p + 8) if partial and i + 1 == len(lst) else nxt - p - 16)
    assert len(offs) == incl[-1][1]
    return np.array(offs, np.uint64), np.array(lens, np.uint32), fixed


def records(pays, ts=None):
    out = bytearray(gen.PCAP_GLOBAL_HEADER)
    for i, p in enumerate(pays):
        sec, usec = ts[i] if ts else (0, 0)
        out += struct.pack("<IIII", sec, usec, len(p), len(p)) + bytes(p)
    return bytes(out)


def check(b, **kw):
    o1, l1 = gen.pcap_index_py(b)
    o2, l2, rounds = model_index(b, **kw)
    assert np.array_equal(o1, o2) and np.array_equal(l1, l2)
    return rounds


def test_model_c4_wrong_guesses_are_rare():
    for seed in (1, 2, 3):
        buf, _, _ = gen.gen_c4(4000, seed=seed)
        assert check(buf.tobytes(), order_seed=seed) <= 6


def test_model_fake_chains_and_large_records():
    rng = np.random.default_rng(3)
    pays = []
    for i in range(300):
        r = rng.random()
        if r < 0.5:
            inner = bytearray()
            for _ in range(int(rng.integers(1, 6))):
                L = int(rng.integers(1, 40))
                inner += struct.pack("<IIII", 1, 2, L, L) + rng.integers(0, 256, L, dtype=np.uint8).tobytes()
            pays.append(bytes(inner))
        elif r < 0.6:
            pays.append(bytes(int(rng.integers(4096, 30000))))
        elif r < 0.65:
            pays.append(b"")
        else:
            pays.append(rng.integers(0, 256, int(rng.integers(0, 3000)), dtype=np.uint8).tobytes())
    ts = [(0, int(rng.integers(0, 2 * 10**6))) for _ in pays]
    for order in range(4):
        print("regions re-walked", check(records(pays, ts), order_seed=order))


def test_model_errors_and_tails():
    good = records([b"\x01" * 60, b"\x02" * 70])
    for extra in range(16):
        check(good + b"\x07" * extra)
    try:
        model_index(good[:-3])
        raise AssertionError("expected an error")
    except ValueError:
        pass


def test_model_adjacent_wrong_guesses_any_chase_order():
    """Wrong guesses in regions a and a+2 (and runs of them), look-backs from random exact
    blocks: every composition that checks out is exact, and the fixes give the host indexer's
    result."""
    buf, _, _ = gen.gen_c4(3000, seed=11)
    b = buf.tobytes()
    K = (len(b) + R - 1) // R
    rng = np.random.default_rng(12)
    for trial in range(40):
        a = int(rng.integers(1, K - 6))
        bad = {a: a * R + int(rng.integers(0, R)), a + 2: (a + 2) * R + int(rng.integers(0, R))}
        if trial % 3 == 0:  # a run of wrong guesses
            for k in range(a + 3, min(K, a + 3 + int(rng.integers(1, 6)))):
                bad[k] = k * R + int(rng.integers(0, R))
        if trial % 4 == 1:  # a wrong guess pointing into the next region
            bad[a + 1] = (a + 2) * R + 17
        check(b, inject=bad, order_seed=trial, block=(5, 8, 256)[trial % 3])


def test_model_prefixes_of_a_capture():
    """pkt_parse_pcap_host's pieces: the index of a PREFIX of a capture (partial mode) is exactly the
    records wholly inside it — the full index's first m records, m = those whose data end lies within
    the prefix — for cuts inside record headers, inside record data and at record boundaries, with
    wrong guesses injected and look-backs in any order."""
    buf, _, _ = gen.gen_c4(2500, seed=21)
    b = buf.tobytes()
    o_full, l_full = gen.pcap_index_py(b)
    ends = o_full.astype(np.int64) + l_full.astype(np.int64)
    rng = np.random.default_rng(5)
    cuts = [24, 40, 4096, 4097] + [int(x) for x in rng.integers(24, len(b), 14)] + \
           [int(o_full[7]) - 16, int(o_full[7]) - 9, int(ends[100]), int(ends[100]) + 1, len(b)]
    for i, cut in enumerate(cuts):
        m = int((ends <= cut).sum())
        o, l, _ = model_index(b[:cut], order_seed=i, block=4, partial=True,
                              inject={3: 3 * R + 1} if cut > 5 * R else None)
        assert np.array_equal(o, o_full[:m]) and np.array_equal(l, l_full[:m]), (cut, m, len(o))


# ---------------------------------------------------------------------------- segment mode (round 6)
def walk_ovr(b, base, entry):
    """The round-6 walk: the error bit is kept in partial mode too (only the verdict ignores it) and the
    start of the record that runs past the end is kept (the slot after the region's records)."""
    pos, lst = entry, []
    while pos < base + R and pos + 16 <= len(b):
        incl = u32(b, pos + 8)
        if pos + 16 + incl > len(b):
            return len(b), lst, 1, pos
        lst.append(pos)
        pos += 16 + incl
    return pos, lst, 0, None


def seg_start(b, r0, carry):
    """pktgpu_pcap.hip seg_start: (entry of region r0, exact exit before it, count before it, err, the
    carried record (offset, incl) now counted or None, B kept as a carry candidate or None)."""
    B, C = carry
    base = r0 * R
    if B >= base:
        return B, B, C, False, None, None
    n = len(b)
    if B + 16 > n:
        return n, n, C, False, None, B
    incl = u32(b, B + 8)
    if B + 16 + incl > n:
        return n, n, C, True, None, B
    return B + 16 + incl, B + 16 + incl, C + 1, False, (B + 16, incl), None


def model_segment(b, r0, carry, partial, inject=None, order_seed=0, block=4):
    """One step of the incremental index: regions [r0, K) of the prefix `b`, the exact state before
    region r0 from `carry` = (B, C) of the previous step (None: the whole prefix from offset 24).
    Returns (new records [(offset, incl)], the new carry (B', C'), error)."""
    b = bytes(b)
    snap = u32(b, 16) or (1 << 30)
    K = (len(b) + R - 1) // R
    seg = carry is not None
    rng = np.random.default_rng(order_seed)
    st = {}
    for k in range(r0, K):  # the guess kernel guesses region r0 too (the scan fixes it against the carry)
        e = 24 if (not seg and k == 0) else (inject or {}).get(k, guess(b, k, snap))
        st[k] = (e, walk_ovr(b, k * R, e))

    def agg(k):
        e, (ex, lst, err, _) = st[k]
        if k != 0 and e >= (k + 1) * R:
            return ("none", (k + 1) * R)
        return (e, ex, len(lst), bool(err), False)

    ks = list(range(r0, K))
    blocks = [ks[i:i + block] for i in range(0, len(ks), block)]
    new = []
    cands = []
    if seg:
        e0, E, C, err0, rec_b, keepB = seg_start(b, r0, carry)
        if rec_b is not None:
            new.append(rec_b)
        if keepB is not None:
            cands.append(keepB)
    incl = []
    for q, ks_q in enumerate(blocks):
        if q == 0:
            if seg:
                pre0, cur = (E, E, 0, False, False), (E, C, err0)
            else:
                pre0, cur = IDENT, (24, 0, False)
        else:
            j = int(rng.integers(0, q))
            acc = IDENT
            for x in range(j + 1, q):
                t = IDENT
                for k in blocks[x]:
                    t = combine(t, agg(k))
                acc = combine(acc, t)
            cur = incl[q - 1]
            pre0 = (cur[0], cur[0], 0, False, False)
        while True:  # fix the first disagreeing seam against the exact state, until none
            pre, todo = pre0, None
            for k in ks_q:
                r = agg(k)
                if seam_bad(pre, r) and not pre[4]:
                    assert pre[1] >= k * R
                    todo = (k, pre[1])
                    break
                pre = combine(pre, r)
            if todo is None:
                break
            st[todo[0]] = (todo[1], walk_ovr(b, todo[0] * R, todo[1]))
        tot = IDENT
        for k in ks_q:
            r = agg(k)
            tot = combine(tot, r)
            e, (ex, lst, err, ovr) = st[k]
            if r[0] != "none" and err:  # a claiming region on the exact chain whose walk met an overrun
                cands.append(ovr)
        E_, C_, err_ = cur
        incl.append((E_, C_, err_) if tot[0] == "none" else (tot[1], C_ + tot[2], err_ or tot[3]))
    E_, C_, err_ = incl[-1]
    cands.append(E_)
    for k in ks:
        _, (ex, lst, _, _) = st[k]
        for i, p in enumerate(lst):
            nxt = lst[i + 1] if i + 1 < len(lst) else ex
            new.append((p + 16, u32(b, p + 8) if partial and i + 1 == len(lst) else nxt - p - 16))
    assert len(new) == C_ - (carry[1] if seg else 0)
    return new, (min(cands), C_), bool(err_) and not partial


def test_model_segments_continue_from_the_carry():
    """Round 6 (pktgpu_pcap.hip segment mode, pkt_pcap_stream_* / pkt_parse_pcap_host's pieces): a capture
    indexed step by step — each step only the regions from the one holding the previous step's end, from
    that step's carry (first uncounted record start, record count) — gives exactly the host indexer's
    records over the whole capture, for random step ends (inside record headers, inside data, at
    boundaries, one byte apart), long records spanning many steps, and wrong guesses injected into each
    step's first region; a poll after each step sees exactly the records wholly inside the bytes so far."""
    rng = np.random.default_rng(61)
    pays = []
    for i in range(700):
        r = rng.random()
        pays.append(bytes(int(rng.integers(5000, 14000))) if r < 0.08 else
                    rng.integers(0, 256, int(rng.integers(1, 400)), dtype=np.uint8).tobytes())
    caps = [records(pays, [(i, 0) for i in range(len(pays))]), gen.gen_c4(1500, seed=62)[0].tobytes()]
    for ci, b in enumerate(caps):
        o_full, l_full = gen.pcap_index_py(b)
        ends = o_full.astype(np.int64) + l_full.astype(np.int64)
        for trial in range(6):
            cuts = sorted(set(int(x) for x in rng.integers(24, len(b), 10 + 4 * trial)))
            cuts += [c + 1 for c in cuts[:3]]
            cuts = sorted(set(c for c in cuts if c < len(b))) + [len(b)]
            carry, prev, got = None, 0, []
            for si, cut in enumerate(cuts):
                K = (cut + R - 1) // R
                r0 = 0 if carry is None else min(prev // R, K - 1)
                inject = {r0: r0 * R + int(rng.integers(0, R))} if (trial % 2 and r0 > 0) else None
                new, carry, err = model_segment(b[:cut], r0, carry, cut < len(b), inject=inject,
                                                order_seed=trial * 100 + si, block=(2, 3, 5)[si % 3])
                assert not err
                got += new
                m = int((ends <= cut).sum())
                assert carry[1] == m, (ci, trial, cut, carry, m)
                assert [x[0] for x in got] == [int(v) for v in o_full[:m]], (ci, trial, cut)
                assert [x[1] for x in got] == [int(v) for v in l_full[:m]], (ci, trial, cut)
                prev = cut
    # the final step's verdict: a record running past the end of the capture is an error
    b = caps[1]
    _, carry, _ = model_segment(b[:len(b) // 2], 0, None, True)
    _, _, err = model_segment(b[:-3], min((len(b) // 2) // R, (len(b) - 3 + R - 1) // R - 1), carry, False)
    assert err
