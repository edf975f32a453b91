"""One process, several devices: the pkt_mgpu_* entry of the C ABI (include/pktgpu.h).

A batch splits into contiguous shards, one per device (every fast::parse_* is a pure function of
one packet, reference src/parser/fast.rs:5-227, so no exchange is needed inside the parse).  Each
shard's per-packet tuples are written into ONE packed device buffer (pkt_out_packed layout) and
gathered to the root device by grouped ncclSend/ncclRecv over RCCL — one message per shard, or
per column with merge=True (the root then holds exactly what one pkt_parse_batch over the whole
batch would write).

    >>> mp = MultiParser([0, 1, 2, 3, 4, 5, 6, 7])
    >>> shards = mp.shard_fixed(slab_host_u8, n, stride=64)     # one device slab per GPU
    >>> res = mp.parse_gather(shards, columns=["chain", "ipv4", "udp"], merge=True)
    >>> res["ipv4_src"]                                          # torch tensor on devices[0]
"""
import ctypes

import numpy as np

from . import _tdtype, _torch, resolve_columns, schema


def packed_views(buf, columns, n):
    """{column: torch view} of an n-packet packed output buffer (uint8 device tensor), using the
    library's own layout (pkt_out_packed)."""
    from . import _lib
    L = _lib.load()
    cols = resolve_columns(columns)
    mask = schema.column_mask(cols)
    o = _lib.PktOut()
    nb = ctypes.c_uint64()
    base = buf.data_ptr()
    rc = L.pkt_out_packed(mask, int(n), ctypes.c_void_p(base), ctypes.byref(o), ctypes.byref(nb))
    if rc != 0:
        raise ValueError("pkt_out_packed failed")
    if buf.numel() < nb.value:
        raise ValueError(f"packed buffer too small: {buf.numel()} < {nb.value}")
    views = {}
    for c in cols:
        off = getattr(o, c) - base
        shp = schema.column_shape(c, n)
        nbytes = int(np.prod(shp)) * schema.column_dtype(c).itemsize
        views[c] = buf[off:off + nbytes].view(_tdtype(schema.column_dtype(c))).view(shp)
    return views


def packed_bytes(columns, n):
    from . import _lib
    L = _lib.load()
    nb = ctypes.c_uint64()
    rc = L.pkt_out_packed(schema.column_mask(resolve_columns(columns)), int(n), None, None, ctypes.byref(nb))
    if rc != 0:
        raise ValueError("pkt_out_packed failed")
    return nb.value


def packed_pieces(columns, n, rows):
    """(offsets, lengths) of the byte ranges of an n-packet packed buffer holding every column with
    only the first `rows` slot rows (pkt_out_packed_pieces): what a copy or gather must move."""
    from . import _lib
    L = _lib.load()
    po, pl, npc = (ctypes.c_uint64 * 2)(), (ctypes.c_uint64 * 2)(), ctypes.c_int()
    if L.pkt_out_packed_pieces(schema.column_mask(resolve_columns(columns)), int(n), int(rows), po, pl,
                               ctypes.byref(npc)) != 0:
        raise ValueError("pkt_out_packed_pieces: bad arguments")
    return [po[k] for k in range(npc.value)], [pl[k] for k in range(npc.value)]


def gather_plan(columns, ns, rows=None, merge=False):
    """pkt_gather_plan: the messages of pkt_mgpu_parse_gather for shards of ns[i] packets with rows[i]
    used slot rows -> ([(shard, src, dst, bytes)], recv_bytes).  Host only."""
    from . import _lib
    L = _lib.load()
    nd = len(ns)
    n_arr = (ctypes.c_uint64 * nd)(*[int(x) for x in ns])
    r_arr = (ctypes.c_uint32 * nd)(*[int(x) for x in rows]) if rows is not None else None
    cnt, rb = ctypes.c_uint64(), ctypes.c_uint64()
    mask = schema.column_mask(resolve_columns(columns))
    if L.pkt_gather_plan(mask, nd, n_arr, r_arr, int(bool(merge)), None, 0, ctypes.byref(cnt), ctypes.byref(rb)) != 0:
        raise ValueError("pkt_gather_plan: bad arguments")
    arr = (_lib.PktGatherPiece * max(1, cnt.value))()
    if L.pkt_gather_plan(mask, nd, n_arr, r_arr, int(bool(merge)), arr, cnt.value, ctypes.byref(cnt),
                         ctypes.byref(rb)) != 0:
        raise ValueError("pkt_gather_plan: bad arguments")
    return [(p.shard, p.src, p.dst, p.bytes) for p in arr[:cnt.value]], rb.value


def shard_range(n, nshards, i):
    """The library's contiguous split (pkt_shard_range): [lo, hi) of shard i."""
    from . import _lib
    L = _lib.load()
    lo, hi = ctypes.c_uint64(), ctypes.c_uint64()
    if L.pkt_shard_range(int(n), int(nshards), int(i), ctypes.byref(lo), ctypes.byref(hi)) != 0:
        raise ValueError("pkt_shard_range: bad arguments")
    return lo.value, hi.value


class MultiParser:
    """A pkt_mgpu handle over a list of distinct HIP devices (one RCCL communicator each).

    virtual=True (TEST MODE, pkt_mgpu_create_virtual): the list may repeat a device — e.g. [0] * 8 is
    eight shards on one GPU, each with its own ctx and streams — and the gather's messages are device
    copies instead of RCCL, so the N-shard code paths run on a one-GPU box.  Not a measurement."""

    def __init__(self, devices, virtual=False):
        torch = _torch()
        from . import _lib
        self._lib = _lib
        self._L = _lib.load()
        self.devices = [int(d) for d in devices]
        self.virtual = bool(virtual)
        self.torch_devices = [torch.device("cuda", d) for d in self.devices]
        arr = (ctypes.c_int * len(self.devices))(*self.devices)
        h = ctypes.c_void_p()
        create = self._L.pkt_mgpu_create_virtual if self.virtual else self._L.pkt_mgpu_create
        rc = create(arr, len(self.devices), ctypes.byref(h))
        if rc != 0:
            msg = self._L.pkt_mgpu_last_error(None)
            raise RuntimeError(f"pkt_mgpu_create{'_virtual' if self.virtual else ''}({self.devices}) failed: {rc}: "
                               f"{msg.decode() if msg else ''}")
        self._mg = h

    @property
    def ndev(self):
        return len(self.devices)

    def close(self):
        if getattr(self, "_mg", None):
            self._L.pkt_mgpu_destroy(self._mg)
            self._mg = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc != 0:
            msg = self._L.pkt_mgpu_last_error(self._mg)
            raise RuntimeError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")

    def ctx(self, i):
        return self._L.pkt_mgpu_ctx(self._mg, i)

    def set_root_copy(self, enable):
        """pkt_mgpu_set_root_copy: the root's own pieces by device copy (True, default) or by RCCL
        send/recv to itself (False)."""
        self._check(self._L.pkt_mgpu_set_root_copy(self._mg, int(bool(enable))), "pkt_mgpu_set_root_copy")

    def set_gather_rows(self, rows):
        """pkt_mgpu_set_gather_rows: slot rows parse_gather moves per shard (0 = each shard's largest
        n_hdrs, measured in its parse: the host waits for it; 1..16 = fixed, no host wait)."""
        self._check(self._L.pkt_mgpu_set_gather_rows(self._mg, int(rows)), "pkt_mgpu_set_gather_rows")

    def synchronize(self):
        self._check(self._L.pkt_mgpu_synchronize(self._mg), "pkt_mgpu_synchronize")

    def streams(self):
        """The handle's per-device work streams (pkt_mgpu_stream) as torch ExternalStreams."""
        torch = _torch()
        if getattr(self, "_ext", None) is None:
            self._ext = [torch.cuda.ExternalStream(self._L.pkt_mgpu_stream(self._mg, i), device=d)
                         for i, d in enumerate(self.torch_devices)]
        return self._ext

    def _after_torch(self):
        """The library's streams are non-blocking streams of their own: make each wait for the work
        torch has queued on that device (e.g. a Generator.run slab, a non_blocking copy)."""
        torch = _torch()
        for d, ext in zip(self.torch_devices, self.streams()):
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(d))
            ext.wait_event(ev)

    def _before_torch(self, tensors):
        """Order torch's current streams after the library's work, and tell the caching allocator
        that every tensor the library touched is in use on the library's streams of its device (so
        it is not reused while a kernel, a copy or RCCL still reads or writes it)."""
        torch = _torch()
        ext = self.streams()
        by_dev = {}
        for d, e in zip(self.torch_devices, ext):
            ev = torch.cuda.Event()
            ev.record(e)
            torch.cuda.current_stream(d).wait_event(ev)
            by_dev.setdefault(d, []).append(e)
        for t in tensors:
            if t is not None and t.is_cuda and t.device in by_dev:
                for e in by_dev[t.device]:
                    t.record_stream(e)

    # ---------------------------------------------------------------- inputs
    def _bounds(self, n, bounds):
        """[lo, hi) of every shard: the library's even split, or the caller's `bounds` (ndev + 1
        non-decreasing record indices from 0 to n; uneven and empty shards allowed)."""
        if bounds is None:
            return [shard_range(n, self.ndev, i) for i in range(self.ndev)]
        b = [int(x) for x in bounds]
        if len(b) != self.ndev + 1 or b[0] != 0 or b[-1] != n or any(x > y for x, y in zip(b, b[1:])):
            raise ValueError(f"bounds must be {self.ndev + 1} non-decreasing indices from 0 to {n}")
        return list(zip(b[:-1], b[1:]))

    def shard_fixed(self, slab, n, stride, lens=None, bounds=None):
        """Copy the contiguous shards of a host fixed-stride slab (numpy uint8) to the devices:
        [(slab tensor, n_i, stride, None, lens tensor|None)]."""
        torch = _torch()
        slab = np.ascontiguousarray(slab, np.uint8).reshape(-1)
        out = []
        for i, (dev, (lo, hi)) in enumerate(zip(self.torch_devices, self._bounds(n, bounds))):
            s = torch.from_numpy(slab[lo * stride:hi * stride].copy()).to(dev) if hi > lo else \
                torch.zeros(16, dtype=torch.uint8, device=dev)
            ln = torch.from_numpy(np.ascontiguousarray(lens[lo:hi], np.uint32)).to(dev) if lens is not None else None
            out.append((s, hi - lo, stride, None, ln))
        return out

    def shard_indexed(self, buf, offsets, lens, bounds=None):
        """Shards of an indexed (pcap) batch by record index; each device gets the whole file
        and its records' (offsets, lens)."""
        torch = _torch()
        a = np.ascontiguousarray(np.frombuffer(buf, np.uint8) if isinstance(buf, (bytes, bytearray)) else buf)
        out = []
        for i, (dev, (lo, hi)) in enumerate(zip(self.torch_devices, self._bounds(len(offsets), bounds))):
            out.append((torch.from_numpy(a.copy()).to(dev), hi - lo, 0,
                        torch.from_numpy(np.ascontiguousarray(offsets[lo:hi], np.uint64)).to(dev),
                        torch.from_numpy(np.ascontiguousarray(lens[lo:hi], np.uint32)).to(dev)))
        return out

    def _batches(self, shards):
        arr = (self._lib.PktBatch * self.ndev)()
        for i, (slab, n, stride, offs, lens) in enumerate(shards):
            b = arr[i]
            b.slab = slab.data_ptr()
            b.slab_len = slab.numel()
            b.offsets = offs.data_ptr() if offs is not None else None
            b.lens = lens.data_ptr() if lens is not None else None
            b.stride = stride or 0
            b.n = int(n)
        return arr

    def set_knobs(self, fastpath=None, staging=None, window=None, walk=None):
        """pkt_ctx_set_* on every device's ctx."""
        for i in range(self.ndev):
            c = self.ctx(i)
            if fastpath is not None:
                self._check(self._L.pkt_ctx_set_fastpath(c, int(bool(fastpath))), "pkt_ctx_set_fastpath")
            if staging is not None:
                self._check(self._L.pkt_ctx_set_staging(c, int(staging)), "pkt_ctx_set_staging")
            if window is not None:
                self._check(self._L.pkt_ctx_set_window(c, int(window)), "pkt_ctx_set_window")
            if walk is not None:
                self._check(self._L.pkt_ctx_set_walk(c, int(walk)), "pkt_ctx_set_walk")

    def steps_plan(self, steps):
        """Prebuilt argument arrays of pkt_mgpu_parse_steps for `steps` steps: a list with, per
        step, one (shard tuple, packed output tensor) per device ->
        (PktBatch[steps * ndev], void*[steps * ndev]), step-major."""
        nd = self.ndev
        b = (self._lib.PktBatch * max(1, len(steps) * nd))()
        o = (ctypes.c_void_p * max(1, len(steps) * nd))()
        for k, per_dev in enumerate(steps):
            assert len(per_dev) == nd
            one = self._batches([sh for sh, _ in per_dev])
            for i, (_, out) in enumerate(per_dev):
                b[k * nd + i] = one[i]
                o[k * nd + i] = out.data_ptr()
        return b, o, len(steps)

    def steps_call(self, plan, entry="parse", columns="all", first=0, count=None, streams=2):
        """A zero-argument callable issuing steps [first, first + count) of a steps_plan through ONE
        pkt_mgpu_parse_steps call (one host thread per device issues that device's launches over
        `streams` streams), with every ctypes argument built here: calling it costs one foreign
        call (the bench's timed region).  Asynchronous on the handle's streams; no ordering with
        torch's streams (the caller owns every buffer)."""
        b, o, n = plan
        count = n - first if count is None else count
        assert 0 <= first and first + count <= n
        nd = self.ndev
        e = schema.ENTRY_ID[entry] if isinstance(entry, str) else int(entry)
        bp = ctypes.cast(ctypes.byref(b, first * nd * ctypes.sizeof(self._lib.PktBatch)),
                         ctypes.POINTER(self._lib.PktBatch))
        op = ctypes.cast(ctypes.byref(o, first * nd * ctypes.sizeof(ctypes.c_void_p)), ctypes.POINTER(ctypes.c_void_p))
        mask = ctypes.c_uint64(schema.column_mask(resolve_columns(columns)))
        f, mg, cnt, ent, st = self._L.pkt_mgpu_parse_steps, self._mg, ctypes.c_int(count), ctypes.c_int(e), ctypes.c_int(streams)

        def call():
            rc = f(mg, bp, cnt, ent, mask, op, st)
            if rc != 0:
                self._check(rc, "pkt_mgpu_parse_steps")
        call.keep = (plan, bp, op)  # the arrays the pointers point into
        return call

    def parse_steps(self, plan, entry="parse", columns="all", first=0, count=None, streams=2):
        """steps_call(...)() — build and issue in one go."""
        self.steps_call(plan, entry, columns, first, count, streams)()

    # ---------------------------------------------------------------- parse + gather
    def alloc_shard_outputs(self, shards, columns):
        torch = _torch()
        return [torch.empty(max(1, packed_bytes(columns, s[1])), dtype=torch.uint8, device=dev)
                for s, dev in zip(shards, self.torch_devices)]

    def parse(self, shards, entry="parse", columns="all", shard_out=None):
        """Parse every shard on its device -> [packed buffer per shard] (asynchronous)."""
        e = schema.ENTRY_ID[entry] if isinstance(entry, str) else int(entry)
        cols = resolve_columns(columns)
        if shard_out is None:
            shard_out = self.alloc_shard_outputs(shards, cols)
        ptrs = (ctypes.c_void_p * self.ndev)(*[b.data_ptr() for b in shard_out])
        self._after_torch()
        self._check(self._L.pkt_mgpu_parse(self._mg, self._batches(shards), e, schema.column_mask(cols), ptrs),
                    "pkt_mgpu_parse")
        self._before_torch(list(shard_out) + [t for sh in shards for t in (sh[0], sh[3], sh[4])])
        return shard_out

    def recv_bytes(self, shards, columns, merge):
        return gather_plan(columns, [s[1] for s in shards], None, merge)[1]

    def parse_gather(self, shards, entry="parse", columns="all", root=0, merge=False,
                     shard_out=None, recv=None):
        """Parse + RCCL gather into one device buffer on devices[root].  Returns (views, recv,
        shard_out): views = one {column: tensor} for merge=True (the whole batch), else one per
        shard.  Ordered like a torch op: the library's streams first wait for torch's current
        streams, torch's current streams then wait for the gather, and every tensor involved is
        marked in use on the library's streams (record_stream), so torch work may consume the
        results right away; synchronize() is needed only before host reads."""
        torch = _torch()
        e = schema.ENTRY_ID[entry] if isinstance(entry, str) else int(entry)
        cols = resolve_columns(columns)
        mask = schema.column_mask(cols)
        if shard_out is None:
            shard_out = self.alloc_shard_outputs(shards, cols)
        need = self.recv_bytes(shards, cols, merge)
        if recv is None:
            recv = torch.empty(max(1, need), dtype=torch.uint8, device=self.torch_devices[root])
        ptrs = (ctypes.c_void_p * self.ndev)(*[b.data_ptr() for b in shard_out])
        views = (self._lib.PktOut * self.ndev)()
        self._after_torch()
        self._check(self._L.pkt_mgpu_parse_gather(self._mg, self._batches(shards), e, mask, ptrs, root,
                                                  ctypes.c_void_p(recv.data_ptr()), recv.numel(),
                                                  1 if merge else 0, views), "pkt_mgpu_parse_gather")
        self._before_torch(list(shard_out) + [recv] + [t for sh in shards for t in (sh[0], sh[3], sh[4])])
        if merge:
            return packed_views(recv, cols, sum(s[1] for s in shards)), recv, shard_out
        out, o = [], 0
        for s in shards:
            nb = packed_bytes(cols, s[1])
            out.append(packed_views(recv[o:o + max(nb, 1)], cols, s[1]) if s[1] else {})
            o += (nb + 255) // 256 * 256
        return out, recv, shard_out
