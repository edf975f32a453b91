"""pktgpu — MI355X batched packet-header parser (Python host side).

Mirrors packet_rs's decode API for whole batches:

    fast::parse(&[u8]) -> PacketSlice            (src/parser/fast.rs:5)
    fast::parse_<hdr>(&[u8]) -> PacketSlice       (the 17 sub-entries, fast.rs:13-222)
    <Hdr>Slice::<field>() -> u64                  (make_header! getters, headers.rs:195-201)
    Packet::ipv4_checksum(&[u8]) -> u16           (src/packet.rs:93-107)

    >>> import torch, pktgpu
    >>> p = pktgpu.Parser(0)
    >>> res = p.parse(slab_u8_cuda, stride=64)              # every column
    >>> res = p.parse(slab, stride=64, columns=["chain", "ipv4", "udp"])
    >>> sl = pktgpu.packet_slice(res_host, i, packet_bytes) # PacketSlice-style view
    >>> sl.payload(), sl.to_vec(), sl["IPv4"].ttl()

All compute runs in the HIP kernels of lib/libpktgpu.so through its C ABI; torch only
provides device memory and the stream.  There is no CPU fallback.
"""
import ctypes

import numpy as np

from . import schema
from .schema import (ABI_VERSION, DEPTH_LIMIT, ENTRIES, ENTRY_ID, GROUPS, HDR_ID, HDR_NAMES,  # noqa: F401
                     HDR_SIZES, MAX_HDRS, OK, STATUS_NAMES, TRUNCATED)

__all__ = ["Parser", "packet_slice", "view", "PacketSlice", "HeaderSlice", "resolve_columns", "schema"]


def resolve_columns(columns):
    """"all" | list of column names and/or group names -> ordered column names."""
    if columns is None or columns == "all":
        return list(schema.COLUMN_NAMES)
    if isinstance(columns, str):
        columns = [columns]
    out = set()
    for c in columns:
        if c in schema.GROUPS:
            out.update(schema.columns_of([c]))
        elif c in schema.COLUMN_NAMES:
            out.add(c)
        else:
            raise ValueError(f"unknown column or group {c!r}")
    return [c for c in schema.COLUMN_NAMES if c in out]


def _torch():
    import torch  # noqa: F401  (must be loaded before libpktgpu: shared HIP runtime)
    return torch


_TORCH_DT = None


def _tdtype(np_dtype):
    torch = _torch()
    global _TORCH_DT
    if _TORCH_DT is None:
        _TORCH_DT = {np.dtype(np.uint8): torch.uint8, np.dtype(np.uint16): torch.uint16,
                     np.dtype(np.uint32): torch.uint32, np.dtype(np.uint64): torch.uint64}
    return _TORCH_DT[np.dtype(np_dtype)]


class Parser:
    """A pkt_ctx bound to one HIP device."""

    def __init__(self, device=0, window=0):
        torch = _torch()
        from . import _lib
        self._L = _lib.load()
        self._lib = _lib
        self.device = int(device)
        self.torch_device = torch.device("cuda", self.device)
        h = ctypes.c_void_p()
        rc = self._L.pkt_ctx_create(self.device, ctypes.byref(h))
        if rc != 0:
            raise RuntimeError(f"pkt_ctx_create({device}) failed: {rc}")
        self._ctx = h
        if window:
            self._L.pkt_ctx_set_window(self._ctx, window)

    def close(self):
        for g in self.__dict__.pop("_gen_udp_cache", {}).values():  # pktgen.gen_udp's generators
            g.close()
        for p in getattr(self, "_pinned", []):
            self._L.pkt_host_free(self._ctx, p)
        self._pinned = []
        if getattr(self, "_ctx", None):
            self._L.pkt_ctx_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_window(self, window_bytes):
        self._L.pkt_ctx_set_window(self._ctx, int(window_bytes))

    def set_fastpath(self, enable):
        """Walk-free fast path for aligned Ether/IPv4/UDP|TCP packets (pkt_ctx_set_fastpath)."""
        self._check(self._L.pkt_ctx_set_fastpath(self._ctx, int(bool(enable))), "pkt_ctx_set_fastpath")

    def set_staging(self, mode):
        """0 = auto, 1 = per-lane windows, 2 = wave spans (pkt_ctx_set_staging)."""
        self._check(self._L.pkt_ctx_set_staging(self._ctx, int(mode)), "pkt_ctx_set_staging")

    def set_walk(self, mode):
        """0 = auto, 1 = waterfall, 2 = lockstep (pkt_ctx_set_walk)."""
        self._check(self._L.pkt_ctx_set_walk(self._ctx, int(mode)), "pkt_ctx_set_walk")

    def set_pcap_scan64(self, enable):
        """pkt_ctx_set_pcap_scan64: the device pcap indexer's 64-bit compositions for every file."""
        self._check(self._L.pkt_ctx_set_pcap_scan64(self._ctx, int(bool(enable))), "pkt_ctx_set_pcap_scan64")

    def set_host_piece(self, nbytes):
        """pkt_ctx_set_host_piece: bytes per copied piece of parse_pcap_host (0 = 16 MiB)."""
        self._check(self._L.pkt_ctx_set_host_piece(self._ctx, int(nbytes)), "pkt_ctx_set_host_piece")

    def _check(self, rc, what):
        if rc != 0:
            msg = self._L.pkt_ctx_last_error(self._ctx)
            raise RuntimeError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")

    def _stream(self, stream):
        torch = _torch()
        if stream is None:
            stream = torch.cuda.current_stream(self.torch_device)
        return ctypes.c_void_p(stream.cuda_stream)

    def _batch(self, slab, n, stride, offsets, lens):
        torch = _torch()
        assert slab.dtype == torch.uint8 and slab.is_cuda and slab.is_contiguous()
        b = self._lib.PktBatch()
        b.slab = slab.data_ptr()
        b.slab_len = slab.numel()
        if offsets is not None:
            assert offsets.dtype == torch.uint64 and lens is not None and lens.dtype == torch.uint32
            b.offsets = offsets.data_ptr()
            b.lens = lens.data_ptr()
            n = offsets.numel() if n is None else n
        else:
            if lens is not None:
                assert lens.dtype == torch.uint32
                b.lens = lens.data_ptr()
            if n is None:
                n = slab.numel() // stride
        b.stride = stride or 0
        b.n = int(n)
        return b

    def alloc(self, n, columns="all"):
        """Device output columns for n packets (torch tensors, uninitialised)."""
        torch = _torch()
        res = {}
        for c in resolve_columns(columns):
            res[c] = torch.empty(schema.column_shape(c, n), dtype=_tdtype(schema.column_dtype(c)),
                                 device=self.torch_device)
        return res

    def out_struct(self, res):
        o = self._lib.PktOut()
        for c, t in res.items():
            setattr(o, c, t.data_ptr() if t.numel() else None)
        return o

    def parse(self, slab, stride=None, n=None, offsets=None, lens=None, entry="parse",
              columns="all", out=None, stream=None):
        """fast::parse_<entry> over every packet of the slab -> {column: device tensor}."""
        e = ENTRY_ID[entry] if isinstance(entry, str) else int(entry)
        b = self._batch(slab, n, stride, offsets, lens)
        res = out if out is not None else self.alloc(b.n, columns)
        o = self.out_struct(res)
        self._check(self._L.pkt_parse_batch(self._ctx, ctypes.byref(b), e, ctypes.byref(o),
                                            self._stream(stream)), "pkt_parse_batch")
        return res

    def parse_host(self, slab, stride=None, n=None, offsets=None, lens=None, entry="parse",
                   columns="all", out=None, chunk=0):
        """The host-memory path (pkt_parse_host): numpy slab/offsets/lens in host memory ->
        {column: numpy array} in host memory, pipelined through the device in chunks.
        `out` may hold preallocated (e.g. pinned, see host_empty) numpy columns."""
        e = ENTRY_ID[entry] if isinstance(entry, str) else int(entry)
        slab = np.ascontiguousarray(slab, np.uint8).reshape(-1)
        b = self._lib.PktBatch()
        b.slab = slab.ctypes.data
        b.slab_len = slab.size
        keep = [slab]
        if offsets is not None:
            offsets = np.ascontiguousarray(offsets, np.uint64)
            lens = np.ascontiguousarray(lens, np.uint32)
            keep += [offsets, lens]
            b.offsets, b.lens = offsets.ctypes.data, lens.ctypes.data
            n = offsets.size if n is None else n
        else:
            if lens is not None:
                lens = np.ascontiguousarray(lens, np.uint32)
                keep.append(lens)
                b.lens = lens.ctypes.data
            n = slab.size // stride if n is None else n
        b.stride = stride or 0
        b.n = int(n)
        if out is None:
            out = {c: np.zeros(schema.column_shape(c, b.n), schema.column_dtype(c))
                   for c in resolve_columns(columns)}
        o = self._lib.PktOut()
        for c, a in out.items():
            setattr(o, c, a.ctypes.data if a.size else None)
        self._check(self._L.pkt_parse_host(self._ctx, ctypes.byref(b), e, ctypes.byref(o), int(chunk)),
                    "pkt_parse_host")
        return out

    def parse_pcap(self, buf, cap=None, entry="parse", columns="all", out=None, offsets=None, lens=None,
                   stream=None):
        """pkt_parse_pcap: a pcap file in the uint8 device tensor `buf` -> (n records, {column: device
        tensor} sized for cap records (slot columns [16][cap]), offsets, lens), index and parse in one
        call with one host synchronisation.  cap=None: the file's size bounds the count (>= 16 B per
        record), which sizes the outputs.  `out` may also be a PktOut built once by out_struct() (it is
        then returned in place of the dict): the 49 column pointers are not marshalled per call."""
        torch = _torch()
        assert buf.dtype == torch.uint8 and buf.is_cuda and buf.is_contiguous()
        e = ENTRY_ID[entry] if isinstance(entry, str) else int(entry)
        if cap is None:
            cap = max(1, (buf.numel() - 24) // 16)
        res = out if out is not None else self.alloc(cap, columns)
        o = res if isinstance(res, self._lib.PktOut) else self.out_struct(res)
        offsets = offsets if offsets is not None else torch.empty(cap, dtype=torch.uint64, device=self.torch_device)
        lens = lens if lens is not None else torch.empty(cap, dtype=torch.uint32, device=self.torch_device)
        n = ctypes.c_uint64()
        self._check(self._L.pkt_parse_pcap(self._ctx, buf.data_ptr(), buf.numel(), e, ctypes.byref(o),
                                           offsets.data_ptr(), lens.data_ptr(), int(cap), ctypes.byref(n),
                                           self._stream(stream)), "pkt_parse_pcap")
        return n.value, res, offsets, lens

    def parse_pcap_async(self, buf, cap, out, offsets, lens, entry="parse", stream=None):
        """pkt_parse_pcap_async: queue the index and the parse of the capture in `buf` on `stream`
        (no host wait) into the caller's `out` / `offsets` / `lens` (sized for cap records).
        pcap_result() waits for it and returns the record count; one capture in flight per Parser."""
        torch = _torch()
        assert buf.dtype == torch.uint8 and buf.is_cuda and buf.is_contiguous()
        e = ENTRY_ID[entry] if isinstance(entry, str) else int(entry)
        o = out if isinstance(out, self._lib.PktOut) else self.out_struct(out)
        self._check(self._L.pkt_parse_pcap_async(self._ctx, buf.data_ptr(), buf.numel(), e, ctypes.byref(o),
                                                 offsets.data_ptr(), lens.data_ptr(), int(cap),
                                                 self._stream(stream)), "pkt_parse_pcap_async")

    def pcap_result(self):
        """pkt_parse_pcap_result: waits for the queued parse_pcap_async and returns its record
        count; raises on its errors."""
        n = ctypes.c_uint64()
        self._check(self._L.pkt_parse_pcap_result(self._ctx, ctypes.byref(n)), "pkt_parse_pcap_result")
        return n.value

    def parse_pcap_host_async(self, buf, cap, out, entry="parse"):
        """pkt_parse_pcap_host_async: queue copy-in, index and parse of the capture in pinned host
        memory `buf` (numpy uint8 from host_empty) into the pinned columns `out` ({column: numpy
        array from host_empty}, sized for cap records); pcap_host_result() waits and returns the
        record count.  One capture in flight per Parser."""
        e = ENTRY_ID[entry] if isinstance(entry, str) else int(entry)
        o = self._lib.PktOut()
        for c, v in out.items():
            setattr(o, c, v.ctypes.data if v.size else None)
        self._check(self._L.pkt_parse_pcap_host_async(self._ctx, buf.ctypes.data, buf.size, e, ctypes.byref(o),
                                                      int(cap)), "pkt_parse_pcap_host_async")

    def pcap_host_result(self):
        n = ctypes.c_uint64()
        self._check(self._L.pkt_parse_pcap_host_result(self._ctx, ctypes.byref(n)), "pkt_parse_pcap_host_result")
        return n.value

    def parse_pcap_host(self, buf, cap, entry="parse", columns="all", out=None, index=True):
        """pkt_parse_pcap_host: a pcap file in host memory (numpy uint8 / bytes; pinned via host_empty
        for the full link rate) -> (n records, {column: numpy array} sized for `cap` records, slot
        columns [16][cap], (offsets, lens) or None).  One blocking call: copy in, device index,
        parse, columns out."""
        e = ENTRY_ID[entry] if isinstance(entry, str) else int(entry)
        a = np.frombuffer(buf, np.uint8) if isinstance(buf, (bytes, bytearray)) else np.ascontiguousarray(buf, np.uint8)
        if out is None:
            out = {c: np.zeros(schema.column_shape(c, cap), schema.column_dtype(c)) for c in resolve_columns(columns)}
        o = self._lib.PktOut()
        for c, v in out.items():
            setattr(o, c, v.ctypes.data if v.size else None)
        offs = np.zeros(cap, np.uint64) if index else None
        lens = np.zeros(cap, np.uint32) if index else None
        n = ctypes.c_uint64()
        self._check(self._L.pkt_parse_pcap_host(self._ctx, a.ctypes.data, a.size, e, ctypes.byref(o),
                                                offs.ctypes.data if index else None,
                                                lens.ctypes.data if index else None, int(cap), ctypes.byref(n)),
                    "pkt_parse_pcap_host")
        m = min(n.value, cap)
        return n.value, out, ((offs[:m], lens[:m]) if index else None)

    def host_empty(self, shape, dtype):
        """A numpy array in pinned host memory (pkt_host_alloc), freed with the Parser."""
        dtype = np.dtype(dtype)
        nbytes = int(np.prod(shape)) * dtype.itemsize
        p = ctypes.c_void_p()
        self._check(self._L.pkt_host_alloc(self._ctx, max(1, nbytes), ctypes.byref(p)), "pkt_host_alloc")
        if not hasattr(self, "_pinned"):
            self._pinned = []
        self._pinned.append(p)
        buf = (ctypes.c_uint8 * max(1, nbytes)).from_address(p.value)
        return np.frombuffer(buf, dtype=np.uint8, count=nbytes).view(dtype).reshape(shape)

    def parse_batches(self, batches, outs, entry="parse", stream=None):
        """pkt_parse_batches: batches = [(slab, n, stride, offsets, lens)], outs = [{column: tensor}]
        -> outs.  One launch over every batch when they share size and layout and their outputs lie
        at one common distance (e.g. one packed buffer each, mgpu.packed_views); else one each."""
        e = ENTRY_ID[entry] if isinstance(entry, str) else int(entry)
        k = len(batches)
        barr = (self._lib.PktBatch * max(1, k))()
        oarr = (self._lib.PktOut * max(1, k))()
        for i, (bt, out) in enumerate(zip(batches, outs)):
            barr[i] = self._batch(*bt)
            oarr[i] = self.out_struct(out)
        self._check(self._L.pkt_parse_batches(self._ctx, barr, k, e, oarr, self._stream(stream)), "pkt_parse_batches")
        return outs

    def batches_call(self, batches, out_structs, entry=0, stream=None):
        """A zero-argument callable issuing one prebuilt pkt_parse_batches (bench loop)."""
        k = len(batches)
        barr = (self._lib.PktBatch * k)(*batches)
        oarr = (self._lib.PktOut * k)(*out_structs)
        f, ctx, s = self._L.pkt_parse_batches, self._ctx, self._stream(stream)

        def call():
            rc = f(ctx, barr, k, entry, oarr, s)
            if rc != 0:
                self._check(rc, "pkt_parse_batches")
        call.keep = (barr, oarr)
        return call

    def launch(self, batch_struct, entry, out_struct, stream=None):
        """Relaunch with prebuilt ctypes structs (no per-call Python allocation; bench loop)."""
        self._check(self._L.pkt_parse_batch(self._ctx, ctypes.byref(batch_struct), entry,
                                            ctypes.byref(out_struct), self._stream(stream)),
                    "pkt_parse_batch")

    def extract_fields(self, slab, chain, specs, stride=None, n=None, offsets=None, lens=None,
                       stream=None):
        """Batched getter: specs = [(hdr_type|name, occurrence, start, end)] -> (values, found)."""
        torch = _torch()
        b = self._batch(slab, n, stride, offsets, lens)
        ch = self._lib.PktChain()
        ch.n_hdrs = chain["n_hdrs"].data_ptr()
        ch.hdr_type = chain["hdr_type"].data_ptr()
        ch.hdr_off = chain["hdr_off"].data_ptr()
        k = len(specs)
        sp = (self._lib.PktFieldSpec * max(1, k))()
        for i, (t, occ, s, e) in enumerate(specs):
            t = HDR_ID[t] if isinstance(t, str) else int(t)
            sp[i] = self._lib.PktFieldSpec(t, occ, s, e, 0)
        vals = [torch.empty(b.n, dtype=torch.uint64, device=self.torch_device) for _ in range(k)]
        found = [torch.empty(b.n, dtype=torch.uint8, device=self.torch_device) for _ in range(k)]
        vp = (ctypes.c_void_p * max(1, k))(*[v.data_ptr() for v in vals])
        fp = (ctypes.c_void_p * max(1, k))(*[f.data_ptr() for f in found])
        self._check(self._L.pkt_extract_fields(self._ctx, ctypes.byref(b), ctypes.byref(ch), sp, k,
                                               vp, fp, self._stream(stream)), "pkt_extract_fields")
        return vals, found

    def to_vec(self, slab, parsed, stride=None, n=None, offsets=None, lens=None, dst=None,
               dst_offsets=None, stream=None):
        """PacketSlice::to_vec of every parsed packet into `dst` (default: a new buffer with
        the input's layout).  Returns (dst, out_len)."""
        torch = _torch()
        b = self._batch(slab, n, stride, offsets, lens)
        if dst is None:
            dst = torch.zeros_like(slab)
        out_len = torch.empty(b.n, dtype=torch.uint32, device=self.torch_device)
        o = self.out_struct(parsed)
        self._check(self._L.pkt_to_vec_batch(self._ctx, ctypes.byref(b), ctypes.byref(o),
                                             ctypes.c_void_p(dst.data_ptr()), dst.numel(),
                                             ctypes.c_void_p(dst_offsets.data_ptr() if dst_offsets is not None else 0),
                                             ctypes.c_void_p(out_len.data_ptr()), self._stream(stream)),
                    "pkt_to_vec_batch")
        return dst, out_len

    def _chain(self, chain):
        ch = self._lib.PktChain()
        ch.n_hdrs = chain["n_hdrs"].data_ptr()
        ch.hdr_type = chain["hdr_type"].data_ptr()
        ch.hdr_off = chain["hdr_off"].data_ptr()
        return ch

    def set_fields(self, slab, chain, specs, values, stride=None, n=None, offsets=None, lens=None,
                   stream=None, ipv4_checksum=None):
        """In-place batched `<Hdr>::set_<field>(v)`: specs = [(hdr_type|name, occurrence, start,
        end)], values = one uint64 device tensor per spec.  ipv4_checksum=occ also refreshes that
        IPv4 header's checksum after the setters, in the same launch (pkt_set_fields_csum)."""
        b = self._batch(slab, n, stride, offsets, lens)
        k = len(specs)
        sp = (self._lib.PktFieldSpec * max(1, k))()
        for i, (t, occ, s, e) in enumerate(specs):
            t = HDR_ID[t] if isinstance(t, str) else int(t)
            sp[i] = self._lib.PktFieldSpec(t, occ, s, e, 0)
        vp = (ctypes.c_void_p * max(1, k))(*[v.data_ptr() for v in values])
        if ipv4_checksum is None:
            self._check(self._L.pkt_set_fields(self._ctx, ctypes.byref(b), ctypes.byref(self._chain(chain)),
                                               sp, k, vp, self._stream(stream)), "pkt_set_fields")
        else:
            self._check(self._L.pkt_set_fields_csum(self._ctx, ctypes.byref(b), ctypes.byref(self._chain(chain)),
                                                    sp, k, vp, int(ipv4_checksum), self._stream(stream)),
                        "pkt_set_fields_csum")

    def ipv4_update_checksum(self, slab, chain, occurrence=0, stride=None, n=None, offsets=None,
                             lens=None, stream=None):
        """In-place: the occurrence-th IPv4 header's checksum := Packet::ipv4_checksum(header)."""
        b = self._batch(slab, n, stride, offsets, lens)
        self._check(self._L.pkt_ipv4_update_checksum(self._ctx, ctypes.byref(b),
                                                     ctypes.byref(self._chain(chain)), occurrence,
                                                     self._stream(stream)), "pkt_ipv4_update_checksum")

    def broadcast(self, src, n, stride, dst=None, stream=None):
        """n clones of the device packet `src` (uint8 tensor) at `stride` -> flat uint8 slab."""
        torch = _torch()
        if dst is None:
            dst = torch.empty(n * stride, dtype=torch.uint8, device=self.torch_device)
        self._check(self._L.pkt_broadcast(self._ctx, ctypes.c_void_p(src.data_ptr()), src.numel(), n,
                                          stride, ctypes.c_void_p(dst.data_ptr()), self._stream(stream)),
                    "pkt_broadcast")
        return dst

    def ipv4_checksum(self, hdrs, stride=20, n=None, stream=None):
        """Packet::ipv4_checksum over n 20-byte headers at a fixed stride (device u8 tensor)."""
        torch = _torch()
        n = hdrs.numel() // stride if n is None else n
        out = torch.empty(n, dtype=torch.uint16, device=self.torch_device)
        self._check(self._L.pkt_ipv4_checksum_batch(self._ctx, ctypes.c_void_p(hdrs.data_ptr()),
                                                    stride, n, ctypes.c_void_p(out.data_ptr()),
                                                    self._stream(stream)), "pkt_ipv4_checksum_batch")
        return out

    def pcap_index(self, buf, cap=None, stream=None):
        """pkt_pcap_index_device: (offsets uint64, lens uint32) device tensors of the records of a
        tests/pcap.rs-format file held in the uint8 device tensor `buf` (16-byte aligned).
        With cap=None the count is found first and exactly that many records are written."""
        torch = _torch()
        assert buf.dtype == torch.uint8 and buf.is_cuda and buf.is_contiguous()
        n = ctypes.c_uint64()
        s = self._stream(stream)
        if cap is None:
            self._check(self._L.pkt_pcap_index_device(self._ctx, buf.data_ptr(), buf.numel(), None, None,
                                                      0, ctypes.byref(n), s), "pkt_pcap_index_device")
            cap = n.value
        offs = torch.empty(cap, dtype=torch.uint64, device=self.torch_device)
        lens = torch.empty(cap, dtype=torch.uint32, device=self.torch_device)
        self._check(self._L.pkt_pcap_index_device(self._ctx, buf.data_ptr(), buf.numel(),
                                                  offs.data_ptr() if cap else None,
                                                  lens.data_ptr() if cap else None, cap,
                                                  ctypes.byref(n), s), "pkt_pcap_index_device")
        k = min(cap, n.value)
        return offs[:k], lens[:k], n.value

    def pcap_index_device_timed(self, buf, offsets, lens, stream=None):
        """pkt_pcap_index_device_timed into the caller's device `offsets` / `lens` (cap = their
        length): (record count, [guess, scan, emit] kernel ms from HIP events between them)."""
        n = ctypes.c_uint64()
        ms = (ctypes.c_float * 3)()
        self._check(self._L.pkt_pcap_index_device_timed(self._ctx, buf.data_ptr(), buf.numel(), offsets.data_ptr(),
                                                        lens.data_ptr(), offsets.numel(), ctypes.byref(n),
                                                        self._stream(stream), ms), "pkt_pcap_index_device_timed")
        return n.value, [ms[0], ms[1], ms[2]]


def pcap_index(buf):
    """(offsets uint64, lens uint32) of a tests/pcap.rs-format buffer, via the C ABI."""
    from . import _lib
    L = _lib.load()
    a = np.ascontiguousarray(np.frombuffer(buf, np.uint8) if isinstance(buf, (bytes, bytearray)) else buf)
    n = ctypes.c_uint64()
    rc = L.pkt_pcap_index(a.ctypes.data, a.size, None, None, 0, ctypes.byref(n))
    if rc != 0:
        raise ValueError("bad pcap")
    offs = np.zeros(n.value, np.uint64)
    lens = np.zeros(n.value, np.uint32)
    rc = L.pkt_pcap_index(a.ctypes.data, a.size, offs.ctypes.data, lens.ctypes.data, n.value,
                          ctypes.byref(n))
    if rc != 0:
        raise ValueError("bad pcap")
    return offs, lens


# ----------------------------------------------------------------- PacketSlice-style host views
class HeaderSlice:
    """A `<Hdr>Slice` (headers.rs:172-296): a name and a view of `len()` bytes of the packet.
    Field getters are generated from the header's make_header! table."""

    def __init__(self, hdr_type, data):
        self.hdr_type = hdr_type
        self._data = data

    def name(self):
        return HDR_NAMES[self.hdr_type]

    def len(self):
        return HDR_SIZES[self.hdr_type]

    def as_slice(self):
        return bytes(self._data[:self.len()])

    def bit_range(self, msb, lsb):
        """headers.rs:253-263 (release semantics for widths > 64, Q8)."""
        v = 0
        for i in range(lsb, msb + 1):
            v = (v << 1) | ((self._data[i // 8] >> (7 - i % 8)) & 1)
        w = msb - lsb + 1
        v &= (1 << 64) - 1
        sh = (64 - w) & 63
        return ((v << sh) & ((1 << 64) - 1)) >> sh

    def bytes(self, msb, lsb):
        return bytes(self.bit_range(i + 7, i) for i in range(lsb, msb + 1, 8))

    def __getattr__(self, field):
        from . import fields
        rng = fields.FIELDS.get(self.hdr_type, {}).get(field)
        if rng is None:
            raise AttributeError(field)
        return lambda: self.bit_range(rng[1], rng[0])


class PacketSlice:
    """packet_rs::PacketSlice (lib.rs:136-140, packet.rs:714-761) over one parsed packet."""

    def __init__(self, hdrs, payload):
        self.hdrs = hdrs
        self._payload = payload

    def payload(self):
        return self._payload

    def len(self):
        return sum(h.len() for h in self.hdrs) + len(self._payload)

    def to_vec(self):
        return b"".join(h.as_slice() for h in self.hdrs) + bytes(self._payload)

    def __getitem__(self, name):  # first match, like Packet's Index<&str> (packet.rs:64-66)
        for h in self.hdrs:
            if h.name() == name:
                return h
        raise KeyError(name)


def view(res, i):
    """pkt_view (the C ABI's PacketSlice of packet i) over host (numpy) chain columns:
    (status, [(hdr_type, offset)], payload_off, payload_len); no headers unless status is OK."""
    from . import _lib
    L = _lib.load()
    need = ("status", "n_hdrs", "hdr_type", "hdr_off", "payload_off", "payload_len")
    cols = {c: np.ascontiguousarray(res[c]) for c in need}
    n = cols["status"].shape[0]
    o = _lib.PktOut()
    for c in need:
        setattr(o, c, cols[c].ctypes.data)
    ty, of = (ctypes.c_uint8 * MAX_HDRS)(), (ctypes.c_uint16 * MAX_HDRS)()
    nh, po, pl = ctypes.c_uint32(), ctypes.c_uint16(), ctypes.c_uint16()
    rc = L.pkt_view(ctypes.byref(o), n, int(i), ty, of, ctypes.byref(nh), ctypes.byref(po), ctypes.byref(pl))
    if rc < 0:
        raise ValueError(f"pkt_view({i}) failed ({rc})")
    return rc, [(ty[k], of[k]) for k in range(nh.value)], po.value, pl.value


def packet_slice(res, i, pkt):
    """Build the PacketSlice of packet i from host (numpy) result columns and its bytes, through
    pkt_view (the same per-packet view a Rust caller builds its PacketSlice from)."""
    st, hl, po, pl = view(res, i)
    if st != OK:
        raise ValueError(f"packet {i}: {STATUS_NAMES[st]} (the reference panics)")
    pkt = bytes(pkt)
    hdrs = [HeaderSlice(t, memoryview(pkt)[o:]) for t, o in hl]
    return PacketSlice(hdrs, pkt[po:po + pl])
