"""Batched header rewrite (§8(f) rank 3): `<Hdr>::set_<field>` = set_bit_range
(headers.rs:315-324) and the builders' checksum refresh (utils.rs:233-236), oracle vs reference
KATs on the CPU and HIP kernels vs oracle on the GPU."""
import json
import os

import numpy as np
import pytest

import oracle
from pktgpu import gen, schema

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
KAT = json.load(open(os.path.join(GOLD, "kat_reference.json")))
H = schema.HDR_ID


def test_set_bit_range_reference_kats():
    """headers.rs:882-927 test_header_set on the Tester header."""
    b = bytes(KAT["tester"]["bytes"])
    F = KAT["tester"]["fields"]
    steps = [("bit1", 0), ("bit2", 2), ("bit3", 3), ("bit4", 4), ("bit5", 5), ("bit6", 6),
             ("bit7", 7), ("bit8", 8), ("bit9", 9), ("bit10", 3), ("byte1", 1), ("byte1", 0xFF),
             ("byte2", 0xFFFF), ("byte3", 0xFFFFFF), ("byte8", 8), ("byte8", 0xFFFFFFFFFFFFFFFF)]
    for name, v in steps:
        s, e, _ = F[name]
        b = oracle.set_bit_range(b, e, s, v)
        assert oracle.bit_range(b, e, s) == v, name
    b = oracle.set_bit_range(b, 127, 66, 0xFFFFFFFF)  # byte4 (62 bits wide)
    assert oracle.bit_range(b, 127, 66) & 0xFFFFFFFF == 0xFFFFFFFF
    a = list(range(1, 17))
    for k, i in enumerate(range(192, 320, 8)):  # set_bytes(byte16) = set_bit_range per byte
        b = oracle.set_bit_range(b, i + 7, i, a[k])
    assert [oracle.bit_range(b, i + 7, i) for i in range(192, 320, 8)] == a


def test_set_bit_range_wide_field_zero_fills():
    """A field wider than 64 bits: the u64 is shifted right once per bit, so the bits above
    the value's 64 become 0 (headers.rs:318-323)."""
    b = oracle.set_bit_range(b"\xff" * 16, 127, 0, 0x0123456789ABCDEF)
    assert b == bytes(8) + (0x0123456789ABCDEF).to_bytes(8, "big")


def test_oracle_rewrite_then_checksum_verifies():
    n = 2000
    slab = gen.gen_c2(n, seed=5).reshape(-1).copy()
    ch = oracle.parse_batch(slab, n, stride=64, columns=["n_hdrs", "hdr_type", "hdr_off"])
    rng = np.random.default_rng(6)
    ttl = rng.integers(0, 256, n).astype(np.uint64)
    oracle.set_fields(slab, n, ch, [(H["IPv4"], 0, 64, 71)], [ttl], stride=64)
    oracle.ipv4_update_checksum(slab, n, ch, 0, stride=64)
    r = oracle.parse_batch(slab, n, stride=64)
    assert np.array_equal(r["ipv4_ttl"], ttl.astype(np.uint8))
    assert np.array_equal(r["ipv4_header_checksum"], r["ipv4_csum_calc"])


def _specs_and_values(n, rng):
    specs = [(H["IPv4"], 0, 64, 71), (H["IPv4"], 0, 96, 127), (H["Ether"], 0, 96, 111),
             (H["TCP"], 0, 104, 111), (H["UDP"], 0, 0, 15), (H["Vlan"], 0, 4, 15),
             (H["IPv4"], 1, 8, 15), (H["IPv6"], 0, 64, 191), (H["Vxlan"], 0, 32, 55),
             (H["IPv4"], 0, 48, 50), (H["MPLS"], 0, 23, 23), (H["ERSPAN3"], 0, 95, 95)]
    vals = [rng.integers(0, 2**63, n, dtype=np.uint64) * 2 + rng.integers(0, 2, n).astype(np.uint64)
            for _ in specs]
    return specs, vals


@pytest.mark.gpu
def test_gpu_set_fields_and_checksum_vs_oracle():
    torch = pytest.importorskip("torch")
    import pktgpu
    P = pktgpu.Parser(0)
    rng = np.random.default_rng(7)
    for kind in ("c2", "c3", "c4"):
        if kind == "c2":
            n = 40000
            slab = gen.gen_c2(n, seed=6).reshape(-1).copy()
            kw = dict(stride=64)
            dkw = dict(stride=64)
        elif kind == "c3":
            n = 40000
            slab = gen.gen_c3(n, seed=8).reshape(-1).copy()
            kw = dict(stride=128)
            dkw = dict(stride=128)
        else:
            slab, offs, lens = gen.gen_c4(30000, seed=9)
            slab = slab.copy()
            n = len(offs)
            kw = dict(offsets=offs, lens=lens)
            dkw = dict(offsets=torch.from_numpy(offs).cuda(), lens=torch.from_numpy(lens).cuda())
        ch = oracle.parse_batch(slab, n, columns=["n_hdrs", "hdr_type", "hdr_off"], **kw)
        specs, vals = _specs_and_values(n, rng)
        slab0 = slab.copy()
        ds = torch.from_numpy(slab.copy()).cuda()
        dch = {k: torch.from_numpy(np.ascontiguousarray(v)).cuda() for k, v in ch.items()}
        P.set_fields(ds, dch, specs, [torch.from_numpy(v).cuda() for v in vals], n=n, **dkw)
        P.ipv4_update_checksum(ds, dch, 0, n=n, **dkw)
        P.ipv4_update_checksum(ds, dch, 1, n=n, **dkw)
        torch.cuda.synchronize()
        oracle.set_fields(slab, n, ch, specs, vals, **kw)
        oracle.ipv4_update_checksum(slab, n, ch, 0, **kw)
        oracle.ipv4_update_checksum(slab, n, ch, 1, **kw)
        got = ds.cpu().numpy()
        assert np.array_equal(got, slab), kind
        # the fused form (setters + one checksum refresh in one launch) on the same inputs
        ds2 = torch.from_numpy(slab0).cuda()
        for occ in (0, 1):
            P.set_fields(ds2, dch, specs if occ == 0 else [], [torch.from_numpy(v).cuda() for v in vals] if occ == 0 else [],
                         n=n, ipv4_checksum=occ, **dkw)
        torch.cuda.synchronize()
        assert np.array_equal(ds2.cpu().numpy(), slab), kind + " fused"


@pytest.mark.gpu
def test_gpu_set_fields_csum_many_specs_vs_oracle():
    """pkt_set_fields_csum with more than 32 specs (ordered launches; the checksum refresh in the
    last one) and the inner IPv4 (occurrence 1) on a C4 pcap mix, vs the oracle's setters then
    Packet::ipv4_checksum."""
    torch = pytest.importorskip("torch")
    import pktgpu
    P = pktgpu.Parser(0)
    rng = np.random.default_rng(21)
    slab, offs, lens = gen.gen_c4(20000, seed=22)
    slab = slab.copy()
    n = len(offs)
    kw = dict(offsets=offs, lens=lens)
    dkw = dict(offsets=torch.from_numpy(offs).cuda(), lens=torch.from_numpy(lens).cuda())
    ch = oracle.parse_batch(slab, n, columns=["n_hdrs", "hdr_type", "hdr_off"], **kw)
    base, bvals = _specs_and_values(n, rng)
    specs = (base * 5)[:41]
    vals = (bvals * 5)[:41]
    ds = torch.from_numpy(slab.copy()).cuda()
    dch = {k: torch.from_numpy(np.ascontiguousarray(v)).cuda() for k, v in ch.items()}
    P.set_fields(ds, dch, specs, [torch.from_numpy(v).cuda() for v in vals], n=n, ipv4_checksum=1, **dkw)
    torch.cuda.synchronize()
    oracle.set_fields(slab, n, ch, specs, vals, **kw)
    oracle.ipv4_update_checksum(slab, n, ch, 1, **kw)
    assert np.array_equal(ds.cpu().numpy(), slab)


@pytest.mark.gpu
def test_gpu_extract_narrow_slots_vs_oracle():
    """Fixed-stride slabs of <= 64-byte slots take 4-chunk windows in extract / set_fields (a fifth
    chunk would be the next packet's): every Ether/IPv4/UDP getter on C2 at its 64-byte stride."""
    torch = pytest.importorskip("torch")
    import pktgpu
    from pktgpu import fields as F
    P = pktgpu.Parser(0)
    n = 30000
    slab = gen.gen_c2(n, seed=31).reshape(-1).copy()
    ch = oracle.parse_batch(slab, n, columns=["n_hdrs", "hdr_type", "hdr_off"], stride=64)
    specs = [(H[h], 0, s0, e0) for h in ("Ether", "IPv4", "UDP") for (s0, e0) in F.FIELDS[H[h]].values()]
    dch = {k: torch.from_numpy(np.ascontiguousarray(v)).cuda() for k, v in ch.items()}
    vals, found = P.extract_fields(torch.from_numpy(slab).cuda(), dch, specs, stride=64)
    torch.cuda.synchronize()
    ov, of = oracle.extract_fields(slab, n, ch, specs, stride=64)
    for k, sp in enumerate(specs):
        assert np.array_equal(vals[k].cpu().numpy(), ov[k]), sp
        assert np.array_equal(found[k].cpu().numpy(), of[k]), sp
