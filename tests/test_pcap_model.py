"""CPU model of the device pcap indexer's speculation + fix-up (pktgpu_pcap.hip): the same
regions, plausibility guess, per-region walk and repair rounds (each round reading the state the
round started from — one legal interleaving of the kernel's waves), checked against the host
indexer on captures built to make the guess wrong.  This pins the algorithm's exactness claim
without a GPU; tests/test_pcap_device.py checks the kernels themselves."""
import struct

import numpy as np

from pktgpu import gen

R = 4096
LOOKBACK = 64


def u32(b, o):
    return struct.unpack_from("<I", b, o)[0] if o + 4 <= len(b) else int.from_bytes(
        (bytes(b[o:o + 4]) + b"\0\0\0\0")[:4], "little")


MIN_HOPS = 2  # PKTGPU_PCAP_HOPS (pktgpu_pcap.hip)
MAX_HOPS = 2
CHASE_MAX = 256
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


def walk(b, base, entry):
    pos, lst, err = entry, [], 0
    while pos < base + R and pos + 16 <= len(b):
        incl = u32(b, pos + 8)
        if pos + 16 + incl > len(b):
            return len(b), lst, 1
        lst.append(pos)
        pos += 16 + incl
    return pos, lst, err


def guess(b, k, snap):
    """First candidate of the region, 64 offsets per step: the lowest whose chain checks out in
    the block's staged bytes (4 regions + 16 B), else the lowest that checks out with reads past
    them; none in the region -> "no record starts here"."""
    base = k * R
    stop = min(len(b), base + R)
    lend = (k // 4 + 1) * 4 * R
    for c0 in range(base, stop, 64):
        cs = [c for c in range(c0, min(c0 + 64, stop)) if c + 16 <= len(b)]
        rs = [chain_ok(b, c, stop, snap, lend) for c in cs]
        for c, r in zip(cs, rs):
            if r == 1:
                return c
        for c, r in zip(cs, rs):
            if r == 2 and chain_ok(b, c, stop, snap) == 1:
                return c
    return base + R


def model_index(b, inject=None, order_seed=None):
    """`inject` {region: entry} overrides the guess (adversarial wrong guesses); `order_seed`
    runs each round's chases in a random order instead of queue order.  A chase claims every
    region it rewrites for the round and stops at one another chase claimed first (the owner
    words of pcap_repair_kernel), so each region's words come from one walk."""
    b = bytes(b)
    snap = u32(b, 16) or (1 << 30)
    K = (len(b) + R - 1) // R
    entry = [24 if k == 0 else guess(b, k, snap) for k in range(K)]
    for k, e in (inject or {}).items():
        if 0 < k < K:
            entry[k] = e
    rng = np.random.default_rng(order_seed) if order_seed is not None else None
    state = [walk(b, k * R, entry[k]) for k in range(K)]
    rounds = 0
    while True:
        rounds += 1
        assert rounds <= K + 1
        old_entry, old_state = list(entry), list(state)
        changed = 0
        def left(k):  # nearest region left of k that claims a record start (or region 0)
            j, s = k - 1, 0
            while s < LOOKBACK and j > 0 and old_entry[j] >= (j + 1) * R:
                j -= 1
                s += 1
            return j

        queue = []
        for k in range(1, K):
            j = left(k)
            e = old_state[j][0]
            if e == old_entry[k]:
                continue
            changed += 1
            # only a region whose left neighbour is settled (agrees with its own left) repairs,
            # and then chases on through the following regions until an exit meets a stored entry
            if (j == 0 or old_state[left(j)][0] == old_entry[j]) and e >= k * R:
                queue.append((k, e))
        if rng is not None:
            queue = [queue[i] for i in rng.permutation(len(queue))]
        owned = set()
        for k, e in queue:  # one interleaving of the chasing waves
            for _ in range(CHASE_MAX):
                if k in owned:  # claimed by another chase this round
                    break
                owned.add(k)
                entry[k] = e
                state[k] = walk(b, k * R, e)
                e = state[k][0]
                k += 1
                if k >= K or e == entry[k] or e < k * R:
                    break
        if not changed:
            break
    if any(st[2] for st in state):
        raise ValueError("truncated pcap record")
    offs, lens = [], []
    for k in range(K):
        ex, lst, _ = state[k]
        for i, p in enumerate(lst):
            nxt = lst[i + 1] if i + 1 < len(lst) else ex
            offs.append(p + 16)
            lens.append(nxt - p - 16)
    return np.array(offs, np.uint64), np.array(lens, np.uint32), rounds


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


def test_model_c4_isolated_wrong_guesses_cost_one_round():
    for seed in (1, 2, 3):
        buf, _, _ = gen.gen_c4(4000, seed=seed)
        assert check(buf.tobytes()) <= 2


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
    print("rounds", check(records(pays, ts)))


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
    """Wrong guesses in regions a and a+2 (and runs of them), chases in random orders: the
    ownership rule keeps every region consistent and the fixed point exact."""
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
        check(b, inject=bad, order_seed=trial)
