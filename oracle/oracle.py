"""ctypes binding of the CPU oracle (TEST INFRASTRUCTURE ONLY).

Loads oracle/build/liboracle.so (built by `make -C oracle`) — the literal C restatement of
packet_rs's fast::parse / bit_range / ipv4_checksum (see pkt_oracle.c).  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
"""
import ctypes
import os
import subprocess
import sys

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_REPO = os.path.dirname(_HERE)
sys.path.insert(0, os.path.join(_REPO, "packet-rs_amd"))
from pktgpu import schema  # noqa: E402  (column layout shared with the product ABI)

LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")


def build(force=False):
    if force or not os.path.exists(LIB_PATH):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return LIB_PATH


class PktBatch(ctypes.Structure):
    _fields_ = [("slab", ctypes.c_void_p), ("slab_len", ctypes.c_uint64),
                ("offsets", ctypes.c_void_p), ("lens", ctypes.c_void_p),
                ("stride", ctypes.c_uint32), ("reserved", ctypes.c_uint32),
                ("n", ctypes.c_uint64)]


class PktOut(ctypes.Structure):
    _fields_ = [(c, ctypes.c_void_p) for c in schema.COLUMN_NAMES]


class PktChain(ctypes.Structure):
    _fields_ = [("n_hdrs", ctypes.c_void_p), ("hdr_type", ctypes.c_void_p),
                ("hdr_off", ctypes.c_void_p)]


class PktFieldSpec(ctypes.Structure):
    _fields_ = [("hdr_type", ctypes.c_uint8), ("occurrence", ctypes.c_uint8),
                ("start", ctypes.c_uint16), ("end", ctypes.c_uint16),
                ("reserved", ctypes.c_uint16)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(LIB_PATH)
        L.orc_bit_range.restype = ctypes.c_uint64
        L.orc_bit_range.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_size_t]
        L.orc_ipv4_checksum.restype = ctypes.c_uint16
        L.orc_ipv4_checksum.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
        L.orc_parse_batch.restype = ctypes.c_int
        L.orc_parse_batch.argtypes = [ctypes.POINTER(PktBatch), ctypes.c_int,
                                      ctypes.POINTER(PktOut), ctypes.c_int]
        L.orc_extract_fields.restype = ctypes.c_int
        L.orc_extract_fields.argtypes = [ctypes.POINTER(PktBatch), ctypes.POINTER(PktChain),
                                         ctypes.POINTER(PktFieldSpec), ctypes.c_uint32,
                                         ctypes.POINTER(ctypes.c_void_p),
                                         ctypes.POINTER(ctypes.c_void_p)]
        L.orc_slow_parse_to_vec.restype = ctypes.c_long
        L.orc_slow_parse_to_vec.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int,
                                            ctypes.c_char_p, ctypes.c_size_t]
        L.orc_hdr_name.restype = ctypes.c_char_p
        L.orc_hdr_field.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_char_p),
                                    ctypes.POINTER(ctypes.c_uint16), ctypes.POINTER(ctypes.c_uint16)]
        _lib = L
    return _lib


def bit_range(hdr_bytes, msb, lsb):
    return lib().orc_bit_range(bytes(hdr_bytes), msb, lsb)


def ipv4_checksum(v):
    return lib().orc_ipv4_checksum(bytes(v), len(v))


def field_table(hdr_type):
    L = lib()
    out = []
    name = ctypes.c_char_p()
    s, e = ctypes.c_uint16(), ctypes.c_uint16()
    for i in range(L.orc_hdr_field_count(hdr_type)):
        L.orc_hdr_field(hdr_type, i, ctypes.byref(name), ctypes.byref(s), ctypes.byref(e))
        out.append((name.value.decode(), s.value, e.value))
    return out


def _batch(slab, n, stride, offsets, lens):
    slab = np.ascontiguousarray(slab, dtype=np.uint8).reshape(-1)
    keep = [slab]
    b = PktBatch()
    b.slab = slab.ctypes.data
    b.slab_len = slab.size
    b.n = n
    b.stride = stride or 0
    if offsets is not None:
        offsets = np.ascontiguousarray(offsets, np.uint64)
        lens = np.ascontiguousarray(lens, np.uint32)
        keep += [offsets, lens]
        b.offsets = offsets.ctypes.data
        b.lens = lens.ctypes.data
    elif lens is not None:
        lens = np.ascontiguousarray(lens, np.uint32)
        keep.append(lens)
        b.lens = lens.ctypes.data
    return b, keep


def parse_batch(slab, n, stride=None, offsets=None, lens=None, entry=0, columns=None, nthreads=1):
    """Oracle fast::parse over a batch.  Returns {column: numpy array} in the pkt_out_t
    layout.  Slot columns are returned zero-filled beyond n_hdrs."""
    if isinstance(entry, str):
        entry = schema.ENTRY_ID[entry]
    columns = schema.COLUMN_NAMES if columns is None else list(columns)
    b, keep = _batch(slab, n, stride, offsets, lens)
    out = PktOut()
    res = {}
    for c in columns:
        a = np.zeros(schema.column_shape(c, n), schema.column_dtype(c))
        res[c] = a
        setattr(out, c, a.ctypes.data if a.size else None)
    rc = lib().orc_parse_batch(ctypes.byref(b), entry, ctypes.byref(out), nthreads)
    if rc != 0:
        raise RuntimeError(f"orc_parse_batch failed ({rc})")
    return res


def extract_fields(slab, n, chain, specs, stride=None, offsets=None, lens=None):
    """Oracle batched getter.  specs: list of (hdr_type, occurrence, start, end)."""
    b, keep = _batch(slab, n, stride, offsets, lens)
    ch = PktChain()
    nh = np.ascontiguousarray(chain["n_hdrs"], np.uint8)
    ht = np.ascontiguousarray(chain["hdr_type"], np.uint8)
    ho = np.ascontiguousarray(chain["hdr_off"], np.uint16)
    ch.n_hdrs, ch.hdr_type, ch.hdr_off = nh.ctypes.data, ht.ctypes.data, ho.ctypes.data
    sp = (PktFieldSpec * max(1, len(specs)))()
    for i, (t, occ, s, e) in enumerate(specs):
        sp[i] = PktFieldSpec(t, occ, s, e, 0)
    vals = [np.zeros(n, np.uint64) for _ in specs]
    found = [np.zeros(n, np.uint8) for _ in specs]
    vp = (ctypes.c_void_p * max(1, len(specs)))(*[v.ctypes.data for v in vals])
    fp = (ctypes.c_void_p * max(1, len(specs)))(*[f.ctypes.data for f in found])
    lib().orc_extract_fields(ctypes.byref(b), ctypes.byref(ch), sp, len(specs), vp, fp)
    return vals, found


def slow_parse_to_vec(pkt, entry=0):
    """slow::parse(pkt).to_vec() (config 1).  Returns bytes, or raises on a reference panic."""
    cap = len(pkt) + 64
    buf = ctypes.create_string_buffer(cap)
    k = lib().orc_slow_parse_to_vec(bytes(pkt), len(pkt), entry, buf, cap)
    if k < 0:
        raise ValueError(schema.STATUS_NAMES[-k])
    return buf.raw[:k]


def round_trip_batch(slab, n, stride=None, offsets=None, lens=None, entry=0, slow=True, nthreads=1,
                     dst=None):
    """Batched `parser::{slow,fast}::parse(pkt).to_vec()` (tests/lib.rs:790-817) written at each
    packet's own position; returns (dst, out_len)."""
    if isinstance(entry, str):
        entry = schema.ENTRY_ID[entry]
    b, keep = _batch(slab, n, stride, offsets, lens)
    flat = keep[0]
    if dst is None:
        dst = np.zeros(flat.size, np.uint8)
    out_len = np.zeros(n, np.uint32)
    L = lib()
    L.orc_round_trip_batch.restype = ctypes.c_int
    L.orc_round_trip_batch.argtypes = [ctypes.POINTER(PktBatch), ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                       ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int]
    rc = L.orc_round_trip_batch(ctypes.byref(b), entry, 1 if slow else 0, dst.ctypes.data, dst.size,
                                out_len.ctypes.data, nthreads)
    if rc != 0:
        raise RuntimeError(f"orc_round_trip_batch failed ({rc})")
    return dst, out_len


def set_bit_range(hdr, msb, lsb, value):
    """headers.rs:315-324 on a bytearray (returns a new bytes)."""
    a = (ctypes.c_uint8 * len(hdr)).from_buffer_copy(bytes(hdr))
    lib().orc_set_bit_range.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_uint64]
    lib().orc_set_bit_range(ctypes.addressof(a), msb, lsb, value)
    return bytes(a)


def _chain_struct(chain):
    ch = PktChain()
    nh = np.ascontiguousarray(chain["n_hdrs"], np.uint8)
    ht = np.ascontiguousarray(chain["hdr_type"], np.uint8)
    ho = np.ascontiguousarray(chain["hdr_off"], np.uint16)
    ch.n_hdrs, ch.hdr_type, ch.hdr_off = nh.ctypes.data, ht.ctypes.data, ho.ctypes.data
    return ch, (nh, ht, ho)


def set_fields(slab, n, chain, specs, values, stride=None, offsets=None, lens=None):
    """Oracle batched setters, in place on the numpy `slab` (must be writable, uint8)."""
    assert slab.flags.writeable and slab.dtype == np.uint8 and slab.flags.c_contiguous
    b, keep = _batch(slab, n, stride, offsets, lens)
    ch, keep2 = _chain_struct(chain)
    sp = (PktFieldSpec * max(1, len(specs)))()
    for i, (t, occ, s, e) in enumerate(specs):
        sp[i] = PktFieldSpec(t, occ, s, e, 0)
    vals = [np.ascontiguousarray(v, np.uint64) for v in values]
    vp = (ctypes.c_void_p * max(1, len(vals)))(*[v.ctypes.data for v in vals])
    L = lib()
    L.orc_set_fields.argtypes = [ctypes.POINTER(PktBatch), ctypes.POINTER(PktChain),
                                 ctypes.POINTER(PktFieldSpec), ctypes.c_uint32, ctypes.c_void_p]
    L.orc_set_fields(ctypes.byref(b), ctypes.byref(ch), sp, len(specs), vp)


def ipv4_update_checksum(slab, n, chain, occurrence=0, stride=None, offsets=None, lens=None):
    assert slab.flags.writeable and slab.dtype == np.uint8 and slab.flags.c_contiguous
    b, keep = _batch(slab, n, stride, offsets, lens)
    ch, keep2 = _chain_struct(chain)
    L = lib()
    L.orc_ipv4_update_checksum.argtypes = [ctypes.POINTER(PktBatch), ctypes.POINTER(PktChain), ctypes.c_uint32]
    L.orc_ipv4_update_checksum(ctypes.byref(b), ctypes.byref(ch), occurrence)


def pktgen_loop(tpl, cnt, stride, mode="clone", first=0, nthreads=1, out=None, entry=0):
    """tests/lib.rs:756-788 on the owned Packet model (clone / update+clone of a template; packet i
    at out[i - first]).  The bench's CPU baseline for the generator."""
    out = np.zeros((cnt, stride), np.uint8) if out is None else out
    L = lib()
    L.orc_pktgen_loop.restype = ctypes.c_int
    L.orc_pktgen_loop.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_uint64,
                                  ctypes.c_uint64, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    rc = L.orc_pktgen_loop(bytes(tpl), len(tpl), entry, {"clone": 0, "update": 1}[mode], first, cnt,
                           out.ctypes.data, stride, nthreads)
    if rc != 0:
        raise RuntimeError(f"orc_pktgen_loop failed ({rc})")
    return out
