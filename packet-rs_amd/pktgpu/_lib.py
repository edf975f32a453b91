"""ctypes binding of lib/libpktgpu.so (the C ABI of include/pktgpu.h).

There is no fallback: if the library is missing or fails to load, importing raises.  Import
torch before this module so that the HIP runtime torch loaded (same soname,
libamdhip64.so.7) is the one the library binds to, and device pointers are shared.
"""
import ctypes
import os

from . import schema

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(_HERE)
# PKTGPU_LIB overrides the library path (A/B builds of the same ABI in one session).
LIB_PATH = os.environ.get("PKTGPU_LIB") or os.path.join(PKG_ROOT, "lib", "libpktgpu.so")


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


class PktGatherPiece(ctypes.Structure):
    _fields_ = [("src", ctypes.c_uint64), ("dst", ctypes.c_uint64), ("bytes", ctypes.c_uint64),
                ("shard", ctypes.c_int32), ("reserved", ctypes.c_uint32)]


class PktGenField(ctypes.Structure):
    _fields_ = [("field", PktFieldSpec), ("kind", ctypes.c_uint32), ("reserved", ctypes.c_uint32),
                ("base", ctypes.c_uint64), ("step", ctypes.c_uint64), ("count", ctypes.c_uint64)]


# Every function declared in include/pktgpu.h: name -> (restype, argtypes)
_P = ctypes.c_void_p
SIGNATURES = {
    "pkt_abi_version": (ctypes.c_int, []),
    "pkt_sizeof_batch": (ctypes.c_size_t, []),
    "pkt_sizeof_out": (ctypes.c_size_t, []),
    "pkt_sizeof_field_spec": (ctypes.c_size_t, []),
    "pkt_hdr_name": (ctypes.c_char_p, [ctypes.c_int]),
    "pkt_hdr_size": (ctypes.c_int, [ctypes.c_int]),
    "pkt_hdr_field_count": (ctypes.c_int, [ctypes.c_int]),
    "pkt_hdr_field": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_char_p),
                                     ctypes.POINTER(ctypes.c_uint16), ctypes.POINTER(ctypes.c_uint16)]),
    "pkt_status_name": (ctypes.c_char_p, [ctypes.c_int]),
    "pkt_entry_name": (ctypes.c_char_p, [ctypes.c_int]),
    "pkt_ctx_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(_P)]),
    "pkt_ctx_destroy": (ctypes.c_int, [_P]),
    "pkt_ctx_last_error": (ctypes.c_char_p, [_P]),
    "pkt_ctx_set_window": (ctypes.c_int, [_P, ctypes.c_uint32]),
    "pkt_ctx_set_fastpath": (ctypes.c_int, [_P, ctypes.c_int]),
    "pkt_ctx_set_staging": (ctypes.c_int, [_P, ctypes.c_int]),
    "pkt_ctx_set_walk": (ctypes.c_int, [_P, ctypes.c_int]),
    "pkt_ctx_set_host_piece": (ctypes.c_int, [_P, ctypes.c_uint64]),
    "pkt_ctx_set_pcap_scan64": (ctypes.c_int, [_P, ctypes.c_int]),
    "pkt_parse_batch": (ctypes.c_int, [_P, ctypes.POINTER(PktBatch), ctypes.c_int,
                                       ctypes.POINTER(PktOut), _P]),
    "pkt_parse_batches": (ctypes.c_int, [_P, ctypes.POINTER(PktBatch), ctypes.c_uint32, ctypes.c_int,
                                         ctypes.POINTER(PktOut), _P]),
    "pkt_parse_host": (ctypes.c_int, [_P, ctypes.POINTER(PktBatch), ctypes.c_int, ctypes.POINTER(PktOut),
                                      ctypes.c_uint64]),
    "pkt_parse_pcap_host": (ctypes.c_int, [_P, _P, ctypes.c_uint64, ctypes.c_int, ctypes.POINTER(PktOut),
                                           _P, _P, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]),
    "pkt_host_alloc": (ctypes.c_int, [_P, ctypes.c_uint64, ctypes.POINTER(_P)]),
    "pkt_host_free": (ctypes.c_int, [_P, _P]),
    "pkt_extract_fields": (ctypes.c_int, [_P, ctypes.POINTER(PktBatch), ctypes.POINTER(PktChain),
                                          ctypes.POINTER(PktFieldSpec), ctypes.c_uint32,
                                          ctypes.POINTER(_P), ctypes.POINTER(_P), _P]),
    "pkt_to_vec_batch": (ctypes.c_int, [_P, ctypes.POINTER(PktBatch), ctypes.POINTER(PktOut), _P,
                                        ctypes.c_uint64, _P, _P, _P]),
    "pkt_set_fields": (ctypes.c_int, [_P, ctypes.POINTER(PktBatch), ctypes.POINTER(PktChain),
                                      ctypes.POINTER(PktFieldSpec), ctypes.c_uint32,
                                      ctypes.POINTER(_P), _P]),
    "pkt_set_fields_csum": (ctypes.c_int, [_P, ctypes.POINTER(PktBatch), ctypes.POINTER(PktChain),
                                           ctypes.POINTER(PktFieldSpec), ctypes.c_uint32,
                                           ctypes.POINTER(_P), ctypes.c_int32, _P]),
    "pkt_ipv4_update_checksum": (ctypes.c_int, [_P, ctypes.POINTER(PktBatch), ctypes.POINTER(PktChain),
                                                ctypes.c_uint32, _P]),
    "pkt_broadcast": (ctypes.c_int, [_P, _P, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint32, _P, _P]),
    "pkt_sizeof_gen_field": (ctypes.c_size_t, []),
    "pkt_gen_create": (ctypes.c_int, [_P, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_int,
                                      ctypes.POINTER(PktGenField), ctypes.c_uint32, ctypes.c_uint32,
                                      ctypes.POINTER(_P)]),
    "pkt_gen_run": (ctypes.c_int, [_P, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                                   ctypes.POINTER(_P), _P, _P]),
    "pkt_gen_destroy": (ctypes.c_int, [_P]),
    "pkt_ipv4_checksum_batch": (ctypes.c_int, [_P, _P, ctypes.c_uint32, ctypes.c_uint64, _P, _P]),
    "pkt_pcap_index": (ctypes.c_int, [_P, ctypes.c_uint64, _P, _P, ctypes.c_uint64,
                                      ctypes.POINTER(ctypes.c_uint64)]),
    "pkt_pcap_index_device": (ctypes.c_int, [_P, _P, ctypes.c_uint64, _P, _P, ctypes.c_uint64,
                                             ctypes.POINTER(ctypes.c_uint64), _P]),
    "pkt_pcap_index_device_timed": (ctypes.c_int, [_P, _P, ctypes.c_uint64, _P, _P, ctypes.c_uint64,
                                                   ctypes.POINTER(ctypes.c_uint64), _P,
                                                   ctypes.POINTER(ctypes.c_float)]),
    "pkt_parse_pcap": (ctypes.c_int, [_P, _P, ctypes.c_uint64, ctypes.c_int, ctypes.POINTER(PktOut), _P, _P,
                                      ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64), _P]),
    "pkt_parse_pcap_host_async": (ctypes.c_int, [_P, _P, ctypes.c_uint64, ctypes.c_int, ctypes.POINTER(PktOut),
                                                 ctypes.c_uint64]),
    "pkt_parse_pcap_host_result": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_uint64)]),
    "pkt_parse_pcap_async": (ctypes.c_int, [_P, _P, ctypes.c_uint64, ctypes.c_int, ctypes.POINTER(PktOut), _P, _P,
                                            ctypes.c_uint64, _P]),
    "pkt_parse_pcap_result": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_uint64)]),
    "pkt_ipv4_checksum_host": (ctypes.c_uint16, [ctypes.c_char_p, ctypes.c_size_t]),
    # packed outputs + multi-GPU (pkt_mgpu_*)
    "pkt_out_packed": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_uint64, _P, ctypes.POINTER(PktOut),
                                      ctypes.POINTER(ctypes.c_uint64)]),
    "pkt_out_packed_pieces": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                                             ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                                             ctypes.POINTER(ctypes.c_int)]),
    "pkt_chain_max_hdrs": (ctypes.c_int, [_P, _P, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint32), _P]),
    "pkt_out_mask": (ctypes.c_uint64, [ctypes.POINTER(PktOut)]),
    "pkt_view": (ctypes.c_int, [ctypes.POINTER(PktOut), ctypes.c_uint64, ctypes.c_uint64,
                                ctypes.POINTER(ctypes.c_uint8), ctypes.POINTER(ctypes.c_uint16),
                                ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint16),
                                ctypes.POINTER(ctypes.c_uint16)]),
    "pkt_sizeof_gather_piece": (ctypes.c_size_t, []),
    "pkt_gather_plan": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64),
                                       ctypes.POINTER(ctypes.c_uint32), ctypes.c_int,
                                       ctypes.POINTER(PktGatherPiece), ctypes.c_uint64,
                                       ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]),
    "pkt_mgpu_set_root_copy": (ctypes.c_int, [_P, ctypes.c_int]),
    "pkt_mgpu_set_gather_rows": (ctypes.c_int, [_P, ctypes.c_int]),
    "pkt_shard_range": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                                       ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]),
    "pkt_pcap_stream_open": (ctypes.c_int, [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int,
                                            ctypes.POINTER(PktOut), ctypes.c_uint64, ctypes.POINTER(_P)]),
    "pkt_pcap_stream_push": (ctypes.c_int, [_P, _P, ctypes.c_uint64]),
    "pkt_pcap_stream_poll": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_uint64), _P, _P]),
    "pkt_pcap_stream_finish": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_uint64), _P, _P]),
    "pkt_pcap_stream_ctx": (_P, [_P]),
    "pkt_pcap_stream_last_error": (ctypes.c_char_p, [_P]),
    "pkt_pcap_stream_close": (ctypes.c_int, [_P]),
    "pkt_mgpu_create": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.POINTER(_P)]),
    "pkt_mgpu_create_virtual": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.POINTER(_P)]),
    "pkt_mgpu_is_virtual": (ctypes.c_int, [_P]),
    "pkt_mgpu_destroy": (ctypes.c_int, [_P]),
    "pkt_mgpu_ndev": (ctypes.c_int, [_P]),
    "pkt_mgpu_last_error": (ctypes.c_char_p, [_P]),
    "pkt_mgpu_ctx": (_P, [_P, ctypes.c_int]),
    "pkt_mgpu_stream": (_P, [_P, ctypes.c_int]),
    "pkt_mgpu_parse": (ctypes.c_int, [_P, ctypes.POINTER(PktBatch), ctypes.c_int, ctypes.c_uint64,
                                      ctypes.POINTER(_P)]),
    "pkt_mgpu_parse_steps": (ctypes.c_int, [_P, ctypes.POINTER(PktBatch), ctypes.c_int, ctypes.c_int,
                                            ctypes.c_uint64, ctypes.POINTER(_P), ctypes.c_int]),
    "pkt_mgpu_gather": (ctypes.c_int, [_P, ctypes.c_int, ctypes.POINTER(_P), ctypes.POINTER(ctypes.c_uint64),
                                       _P, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]),
    "pkt_mgpu_parse_gather": (ctypes.c_int, [_P, ctypes.POINTER(PktBatch), ctypes.c_int, ctypes.c_uint64,
                                             ctypes.POINTER(_P), ctypes.c_int, _P, ctypes.c_uint64,
                                             ctypes.c_int, ctypes.POINTER(PktOut)]),
    "pkt_mgpu_synchronize": (ctypes.c_int, [_P]),
}

_lib = None


def load():
    """Load libpktgpu.so and declare every prototype; raises if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: build it with `make -C packet-rs_amd` "
                          "(or __graft_entry__.build()); there is no CPU fallback")
    L = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    if L.pkt_abi_version() != schema.ABI_VERSION:
        raise ImportError("libpktgpu ABI version mismatch")
    if L.pkt_sizeof_out() != ctypes.sizeof(PktOut) or L.pkt_sizeof_batch() != ctypes.sizeof(PktBatch) \
            or L.pkt_sizeof_field_spec() != ctypes.sizeof(PktFieldSpec) \
            or L.pkt_sizeof_gen_field() != ctypes.sizeof(PktGenField) \
            or L.pkt_sizeof_gather_piece() != ctypes.sizeof(PktGatherPiece):
        raise ImportError("libpktgpu struct layout mismatch with pktgpu/_lib.py")
    _lib = L
    return L
