"""A capture that arrives in pieces: pkt_pcap_stream_* of the C ABI (include/pktgpu.h).

The capture path of tests/pcap.rs:7-37 (reference) fed as bytes arrive — a NIC ring drained into host
memory, a file read while it grows.  Each push appends bytes on the device; the device indexes only the
new bytes (from the first record the previous step could not count, kept in device words) and parses
the records they complete into the stream's columns, while later bytes are still copying in.

    >>> st = PcapStream(0, max_bytes=1 << 30, cap=1 << 20, columns="all")          # device columns
    >>> for chunk in ring:                                                           # bytes / numpy u8
    ...     st.push(chunk)
    >>> n, (offs, lens) = st.finish()
    >>> st.out["ipv4_src"][:n]                                                       # torch tensor
"""
import ctypes

import numpy as np

from . import ENTRY_ID, Parser, _torch, resolve_columns, schema


class PcapStream:
    """pkt_pcap_stream_open(device, max_bytes, cap, entry, out, step_bytes).  `out`: None = device
    columns allocated here (torch tensors), "pinned" = pinned host columns (numpy arrays from
    pkt_host_alloc: each step's columns are exported over the link), or a dict of either kind."""

    def __init__(self, device=0, max_bytes=1 << 28, cap=1 << 20, columns="all", entry="parse", out=None,
                 step_bytes=0):
        from . import _lib
        self._lib = _lib
        self._L = _lib.load()
        self.cap = int(cap)
        self._keep = None
        cols = resolve_columns(columns)
        if out is None:
            torch = _torch()
            dev = torch.device("cuda", device)
            out = {c: torch.zeros(schema.column_shape(c, self.cap), dtype=_tdtype_of(c), device=dev) for c in cols}
        elif isinstance(out, str) and out == "pinned":
            self._keep = Parser(device)  # owns the pinned allocations
            out = {c: self._keep.host_empty(schema.column_shape(c, self.cap), schema.column_dtype(c)) for c in cols}
        self.out = out
        o = _lib.PktOut()
        for c, v in out.items():
            ptr = v.data_ptr() if hasattr(v, "data_ptr") else v.ctypes.data
            setattr(o, c, ptr if _size(v) else None)
        e = ENTRY_ID[entry] if isinstance(entry, str) else int(entry)
        h = ctypes.c_void_p()
        rc = self._L.pkt_pcap_stream_open(int(device), int(max_bytes), self.cap, e, ctypes.byref(o), int(step_bytes),
                                          ctypes.byref(h))
        if rc != 0:
            raise RuntimeError(f"pkt_pcap_stream_open failed ({rc})")
        self._st = h

    def _check(self, rc, what):
        if rc != 0:
            msg = self._L.pkt_pcap_stream_last_error(self._st)
            raise RuntimeError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")

    def ctx(self):
        return self._L.pkt_pcap_stream_ctx(self._st)

    def push(self, data):
        a = np.frombuffer(data, np.uint8) if isinstance(data, (bytes, bytearray, memoryview)) else \
            np.ascontiguousarray(data, np.uint8).reshape(-1)
        self._check(self._L.pkt_pcap_stream_push(self._st, a.ctypes.data if a.size else None, a.size),
                    "pkt_pcap_stream_push")

    def _counted(self, fn, what, index):
        n = ctypes.c_uint64()
        offs = np.zeros(self.cap, np.uint64) if index else None
        lens = np.zeros(self.cap, np.uint32) if index else None
        self._check(fn(self._st, ctypes.byref(n), offs.ctypes.data if index else None,
                       lens.ctypes.data if index else None), what)
        m = min(n.value, self.cap)
        return n.value, ((offs[:m], lens[:m]) if index else None)

    def poll(self, index=False):
        """Records wholly inside the bytes pushed so far (their columns written) -> (n, (offsets, lens))."""
        return self._counted(self._L.pkt_pcap_stream_poll, "pkt_pcap_stream_poll", index)

    def finish(self, index=True):
        """End of capture: the tail as pkt_pcap_index takes it -> (n, (offsets, lens))."""
        return self._counted(self._L.pkt_pcap_stream_finish, "pkt_pcap_stream_finish", index)

    def close(self):
        if getattr(self, "_st", None):
            self._L.pkt_pcap_stream_close(self._st)
            self._st = None
        if self._keep is not None:
            self._keep.close()
            self._keep = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _size(v):
    return v.numel() if hasattr(v, "numel") else v.size


def _tdtype_of(c):
    from . import _tdtype
    return _tdtype(schema.column_dtype(c))
