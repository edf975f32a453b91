"""Batched packet generation on the GPU (§8(f) rank 4: the reference's pktgen workload).

The reference builds packets one at a time (`utils::create_*_packet`, src/utils.rs:7-876) and its
perf test times new / clone / update+clone loops (tests/lib.rs:756-788).  Here the builder runs
once on the host to produce a TEMPLATE, and one device pass writes the whole batch
(`pkt_gen_create` / `pkt_gen_run`, include/pktgpu.h, kernel in csrc/pktgpu_gen.hip):

    clone         Generator(P, tpl).run(n)                         the template n times
    update+clone  Generator(P, tpl, [Field("Ether", "etype", kind="inc", count=0xFFFF)])
    new           Generator(P, tpl, [Field("IPv4", "src", kind="random", base=seed), ...],
                            csum=[0])                              builder args varied per packet,
                                                                   IPv4 checksum refreshed

A field is (header, field name or (start, end) bits, occurrence) as the make_header! tables name
it (headers.rs:529-827); its value per packet is an array, a counter or splitmix64.
"""
import ctypes

import numpy as np

from . import fields as _fields
from . import gen, schema

H = schema.HDR_ID
KINDS = {"values": 0, "inc": 1, "random": 2}


class Field:
    """One generator field: `hdr` (name or id), `field` (make_header! name or (start, end)),
    `occurrence` (0 = first such header, Index<&str> semantics), and how it varies:
    kind "values" (a uint64 device tensor per run), "inc" (base + step * (g % count), count 0 =
    no wrap) or "random" (splitmix64(base + g)); g = the packet's global index."""

    def __init__(self, hdr, field, occurrence=0, kind="values", base=0, step=1, count=0):
        self.hdr = H[hdr] if isinstance(hdr, str) else int(hdr)
        if isinstance(field, str):
            self.start, self.end = _fields.FIELDS[self.hdr][field]
        else:
            self.start, self.end = int(field[0]), int(field[1])
        self.occurrence = int(occurrence)
        self.kind = kind
        self.base, self.step, self.count = int(base), int(step), int(count)

    def value(self, g, values=None):
        """Host restatement of the per-packet value (numpy uint64 array for global indices g);
        used by the tests and the bench's CPU reference, never by the device path."""
        g = np.asarray(g, np.uint64)
        w = self.end - self.start + 1
        mask = np.uint64((1 << w) - 1) if w < 64 else np.uint64(2**64 - 1)
        with np.errstate(over="ignore"):
            if self.kind == "values":
                v = np.asarray(values, np.uint64)
            elif self.kind == "inc":
                k = g % np.uint64(self.count) if self.count else g
                v = np.uint64(self.base) + np.uint64(self.step) * k
            else:
                v = splitmix64(np.uint64(self.base) + g)
        return v & mask


def splitmix64(x):
    """splitmix64 as pkt_gen_run's PKT_GEN_RANDOM defines it (numpy, wrapping uint64)."""
    with np.errstate(over="ignore"):
        z = np.asarray(x, np.uint64) + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


class Generator:
    """A template plus its field engine, placed once on the device (pkt_gen_create)."""

    def __init__(self, parser, template, fields=(), csum=(), entry="parse"):
        from . import _lib
        self.P = parser
        self._L = parser._L
        self.template = bytes(template)
        self.fields = list(fields)
        arr = (_lib.PktGenField * max(1, len(self.fields)))()
        for i, f in enumerate(self.fields):
            arr[i] = _lib.PktGenField(_lib.PktFieldSpec(f.hdr, f.occurrence, f.start, f.end, 0),
                                      KINDS[f.kind], 0, f.base & (2**64 - 1), f.step & (2**64 - 1),
                                      f.count & (2**64 - 1))
        mask = 0
        for occ in csum:
            mask |= 1 << int(occ)
        e = schema.ENTRY_ID[entry] if isinstance(entry, str) else int(entry)
        h = ctypes.c_void_p()
        parser._check(self._L.pkt_gen_create(parser._ctx, self.template, len(self.template), e, arr,
                                             len(self.fields), mask, ctypes.byref(h)), "pkt_gen_create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            self._L.pkt_gen_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def default_stride(self):
        return (len(self.template) + 15) & ~15

    def run(self, n, stride=None, values=None, first=0, dst=None, stream=None):
        """Packets first .. first+n-1 -> flat uint8 device slab (n * stride bytes).  `values`:
        {field index: uint64 device tensor [n]} for the "values" fields."""
        import torch
        stride = stride or self.default_stride()
        if dst is None:
            dst = torch.empty(n * stride, dtype=torch.uint8, device=self.P.torch_device)
        # pkt_gen_run takes no length for dst or the value arrays: check them here (not with
        # assert, which python -O strips)
        if not (isinstance(dst, torch.Tensor) and dst.dtype == torch.uint8 and dst.is_cuda and
                dst.device == self.P.torch_device and dst.is_contiguous()):
            raise ValueError("dst must be a contiguous uint8 CUDA tensor on the parser's device")
        if dst.numel() < n * stride:
            raise ValueError(f"dst holds {dst.numel()} bytes, {n} packets at stride {stride} need {n * stride}")
        vp = (ctypes.c_void_p * max(1, len(self.fields)))()
        for i, f in enumerate(self.fields):
            t = (values or {}).get(i) if f.kind == "values" else None
            if t is not None:  # (a missing array is reported by pkt_gen_run)
                if not (isinstance(t, torch.Tensor) and t.dtype == torch.uint64 and t.is_cuda and
                        t.device == self.P.torch_device and t.is_contiguous()):
                    raise ValueError(f"values[{i}] must be a contiguous uint64 CUDA tensor on the parser's device")
                if t.numel() < n:
                    raise ValueError(f"values[{i}] holds {t.numel()} values, {n} packets need {n}")
                vp[i] = t.data_ptr()
        self.P._check(self._L.pkt_gen_run(self._h, int(first), int(n), int(stride), vp,
                                          ctypes.c_void_p(dst.data_ptr()), self.P._stream(stream)),
                      "pkt_gen_run")
        return dst


# ---------------------------------------------------------------- the reference's own templates
def test_tcp_template():
    """tests/lib.rs:711-714 `test_tcp_packet()` (the pktgen_perf_test packet): 154 bytes."""
    return gen.test_tcp_packet_with_payload(bytes(range(100))).to_vec()


def udp_template(payload_len=22):
    """create_udp_packet with the SURVEY §8(c) arguments: 14 + 20 + 8 header bytes + payload."""
    return gen.create_udp_packet("00:01:02:03:04:05", "00:06:07:08:09:0a", False, 10, 3, 5,
                                 "192.168.0.199", "192.168.0.1", 0, 64, 0, 0x4000, [], 1234, 9090,
                                 False, bytes(range(payload_len))).to_vec()


# (hdr, occurrence, start, end) of the fields gen_udp varies (headers.rs:530-634)
UDP_FIELDS = {
    "eth_dst": ("Ether", "dst"), "eth_src": ("Ether", "src"),
    "ipv4_diffserv": ("IPv4", "diffserv"), "ipv4_identification": ("IPv4", "identification"),
    "ipv4_ttl": ("IPv4", "ttl"), "ipv4_src": ("IPv4", "src"), "ipv4_dst": ("IPv4", "dst"),
    "udp_src": ("UDP", "src"), "udp_dst": ("UDP", "dst"),
}


def gen_udp(parser, n, fields, stride=64, template=None, stream=None):
    """n Ether/IPv4/UDP packets on the device in one pass: the template with every field in
    `fields` ({name in UDP_FIELDS: uint64 device tensor [n]}) set per packet and the IPv4
    checksum refreshed.  Returns the flat uint8 device slab.  The Generator of each (template,
    field set) is created once per parser and reused: pkt_gen_create parses the template and
    synchronises the device, which must stay off a generation loop."""
    tpl = bytes(template if template is not None else udp_template())
    names = tuple(fields)
    cache = parser.__dict__.setdefault("_gen_udp_cache", {})
    g = cache.get((tpl, names))
    if g is None:
        g = cache[(tpl, names)] = Generator(parser, tpl, [Field(*UDP_FIELDS[k]) for k in names], csum=[0])
    return g.run(n, stride, values={i: fields[k] for i, k in enumerate(names)}, stream=stream)
