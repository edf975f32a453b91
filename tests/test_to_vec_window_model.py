"""CPU model of to_vec's window path (packet-rs_amd/csrc/pktgpu_rewrite.hip: tv_overlap_kernel's table,
tv_window_kernel's chunk -> record mapping), checked against the direct definition of
PacketSlice::to_vec into the input's own layout (reference src/packet.rs:733-740, 385-392): every
16-byte destination chunk holding bytes of a copied record is written exactly once, with exactly that
record's bytes [lo, hi) of it, and no other chunk is written.

The device kernels are restated step by step: the table (first[w] = the first record ending past byte
4096 w, written by the in-order pair whose interval [end(i-1), end(i)) holds the window start; the
windows before end(0) use record 0; those from end(n-1) on exit), and per window the batches of 64
records, the start map of the window's 256 chunks, s0 and rank - s0.  Layouts: pcap-like (16-byte
gaps), a long lead, records longer than a window, > 64 record starts in one window, records not copied
(not parsed, or gathered: Q2) between copied ones, and the out-of-order / shared-chunk batches the
overlap check must send to to_vec_kernel."""
import numpy as np
import pytest

WIN = 4096
CH = WIN // 16
MAX_WIN = 128


def overlap_pass(offs, lens, slab_len):
    """tv_overlap_kernel: (bad, first table, end(0), end(n-1))."""
    n = len(offs)
    nwin = (slab_len + WIN - 1) // WIN
    first = np.full(nwin, -1, np.int64)  # -1 = never written
    bad = False
    for i in range(n):
        o1, e1 = int(offs[i]), int(offs[i]) + int(lens[i])
        bad |= e1 > slab_len or int(lens[i]) == 0
        if i >= 1:
            o0, l0 = int(offs[i - 1]), int(lens[i - 1])
            e0 = o0 + l0
            pb = l0 == 0 or ((e0 - 1) >> 4) >= (o1 >> 4)
            bad |= pb
            if not pb:
                w0 = (e0 + WIN - 1) // WIN
                w1 = min((e1 + WIN - 1) // WIN, nwin)
                if w1 > w0 + MAX_WIN:
                    bad = True
                else:
                    first[w0:w1] = i
    return bad, first, int(offs[0]) + int(lens[0]), int(offs[-1]) + int(lens[-1]), nwin


def window_pass(offs, copy_len, mode, first, e0, en, nwin):
    """tv_window_kernel's chunk assignments: {chunk: (record, lo, hi)} (byte offsets in the chunk)."""
    n = len(offs)
    out = {}
    for w in range(nwin):
        wa, we = w * WIN, (w + 1) * WIN
        if wa >= en:
            continue
        i0 = 0 if wa < e0 else int(first[w])
        assert i0 >= 0, f"window {w} reads an unset table entry"
        while i0 < n:
            idx = np.arange(i0, min(i0 + 64, n))
            o = offs[idx].astype(np.int64)
            st = (o >= wa) & (o < we)
            smap = np.zeros(CH, bool)
            smap[(o[st] - wa) >> 4] = True
            s0 = 1 if (len(st) and st[0]) else 0
            run = np.cumsum(smap)  # starts at or below chunk g
            for g in range(CH):
                r = int(run[g]) - s0
                if 0 <= r < len(idx):
                    rec = int(idx[r])
                    if mode[rec] != 1:
                        continue
                    ca = wa + 16 * g
                    lo, hi = max(ca, int(offs[rec])), min(ca + 16, int(offs[rec]) + int(copy_len[rec]))
                    if lo < hi:
                        assert (ca // 16) not in out, f"chunk {ca // 16} written twice"
                        out[ca // 16] = (rec, lo - ca, hi - ca)
            # all 64 began before the window's end: the next 64 may too
            if not (len(idx) == 64 and int(offs[idx[-1]]) < we):
                break
            i0 += 64
    return out


def direct(offs, copy_len, mode):
    out = {}
    for i in range(len(offs)):
        if mode[i] != 1 or copy_len[i] == 0:
            continue
        a, z = int(offs[i]), int(offs[i]) + int(copy_len[i])
        for c in range(a // 16, (z - 1) // 16 + 1):
            ca = 16 * c
            out[c] = (i, max(a, ca) - ca, min(z, ca + 16) - ca)
    return out


def layout(rng, n, kind):
    if kind == "dense":  # many starts per window
        lens = rng.integers(1, 40, n)
    elif kind == "long":  # records longer than a window next to short ones
        lens = np.where(rng.random(n) < 0.1, rng.integers(4096, 30000, n), rng.integers(40, 1500, n))
    else:
        lens = rng.integers(42, 400, n)
    gaps = np.full(n, 16)
    gaps[0] = {"lead": 100_000}.get(kind, 24 + 16)
    offs = np.cumsum(gaps) + np.concatenate([[0], np.cumsum(lens)[:-1]])
    r = rng.random(n)
    mode = np.where(r < 0.05, 0, np.where(r < 0.08, 2, 1))  # not parsed / gathered (Q2) / copied
    copy_len = np.where(mode == 0, 0, np.maximum(1, (lens * np.where(rng.random(n) < 0.2, rng.random(n), 1.0)).astype(np.int64)))
    copy_len = np.minimum(copy_len, lens)
    slab_len = int(offs[-1] + lens[-1]) + int(rng.integers(0, 5000))
    return offs.astype(np.uint64), lens.astype(np.uint32), copy_len, mode, slab_len


@pytest.mark.parametrize("kind", ["pcap", "lead", "dense", "long"])
@pytest.mark.parametrize("seed", [1, 2])
def test_window_model_equals_direct(kind, seed):
    rng = np.random.default_rng(seed * 10 + len(kind))
    offs, lens, copy_len, mode, slab_len = layout(rng, 3000, kind)
    bad, first, e0, en, nwin = overlap_pass(offs, lens, slab_len)
    assert not bad
    got = window_pass(offs, copy_len, mode, first, e0, en, nwin)
    assert got == direct(offs, copy_len, mode)


def test_overlap_pass_sends_unfit_batches_to_to_vec_kernel():
    rng = np.random.default_rng(5)
    offs, lens, copy_len, mode, slab_len = layout(rng, 500, "pcap")
    assert not overlap_pass(offs, lens, slab_len)[0]
    shared = offs.copy()
    ends = offs.astype(np.int64) + lens.astype(np.int64)
    j = 1 + int(np.nonzero(ends[:-1] % 16)[0][0])
    shared[j] = np.uint64(ends[j - 1])  # record j back to back with j - 1: one 16-byte chunk holds both
    assert overlap_pass(shared, lens, slab_len)[0]
    swapped = offs.copy()
    swapped[[200, 201]] = swapped[[201, 200]]  # out of order
    assert overlap_pass(swapped, lens, slab_len)[0]
    past = lens.copy()
    past[-1] += slab_len  # past the slab's end
    assert overlap_pass(offs, past, slab_len)[0]
    empty = lens.copy()
    empty[-1] = 0  # an empty last record (its start may open a window past end(n-1)): to_vec_kernel
    assert overlap_pass(offs, empty, slab_len)[0]
    far = offs.copy()
    far[300:] += np.uint64(2 * MAX_WIN * WIN)  # a gap of more than 128 windows
    assert overlap_pass(far, lens, int(far[-1] + lens[-1]) + 1)[0]
