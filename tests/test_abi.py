"""CPU tests of the C-ABI library: it loads, exports every symbol include/pktgpu.h declares,
its struct layouts match the Python binding, and its host-side functions (metadata tables, the
pcap indexer, the host checksum) agree with the oracle.  No device call is made."""
import ctypes
import os
import re

import numpy as np
import pytest

import oracle
from pktgpu import _lib, gen, schema

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "pktgpu.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(pkt_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def L():
    return _lib.load()


def test_library_builds_and_loads(L):
    assert os.path.exists(_lib.LIB_PATH)
    assert L.pkt_abi_version() == schema.ABI_VERSION


def test_every_declared_symbol_is_exported(L):
    names = declared_functions()
    assert len(names) >= 50
    for n in names:
        assert hasattr(L, n), n
    assert set(names) == set(_lib.SIGNATURES), "pktgpu/_lib.py SIGNATURES out of sync with pktgpu.h"


def test_struct_layouts(L):
    assert L.pkt_sizeof_out() == ctypes.sizeof(_lib.PktOut) == 8 * len(schema.COLUMN_NAMES)
    assert L.pkt_sizeof_batch() == ctypes.sizeof(_lib.PktBatch)
    assert L.pkt_sizeof_field_spec() == ctypes.sizeof(_lib.PktFieldSpec) == 8
    assert L.pkt_sizeof_gen_field() == ctypes.sizeof(_lib.PktGenField) == 40


def test_metadata_tables_match_oracle(L):
    for t in range(1, len(schema.HDR_NAMES)):
        assert L.pkt_hdr_name(t).decode() == schema.HDR_NAMES[t]
        assert L.pkt_hdr_size(t) == schema.HDR_SIZES[t]
        mine = []
        for k in range(L.pkt_hdr_field_count(t)):
            nm, s, e = ctypes.c_char_p(), ctypes.c_uint16(), ctypes.c_uint16()
            assert L.pkt_hdr_field(t, k, ctypes.byref(nm), ctypes.byref(s), ctypes.byref(e)) == 0
            mine.append((nm.value.decode(), s.value, e.value))
        assert mine == oracle.field_table(t), schema.HDR_NAMES[t]
    assert L.pkt_hdr_name(0) is None and L.pkt_hdr_name(99) is None
    assert [L.pkt_entry_name(i).decode() for i in range(len(schema.ENTRIES))] == schema.ENTRIES
    assert [L.pkt_status_name(i).decode() for i in range(3)] == schema.STATUS_NAMES


def test_fields_module_in_sync():
    from pktgpu import fields
    for t in range(1, len(schema.HDR_NAMES)):
        assert [(n, s, e) for n, (s, e) in fields.FIELDS[t].items()] == oracle.field_table(t)


def test_pcap_index_matches_python():
    import pktgpu
    pc = open(os.path.join(REPO, "tests", "golden", "ref22.pcap"), "rb").read()
    o1, l1 = pktgpu.pcap_index(pc)
    o2, l2 = gen.pcap_index_py(pc)
    assert np.array_equal(o1, o2) and np.array_equal(l1, l2) and len(o1) == 22
    buf, offs, lens = gen.gen_c4(5000, seed=1)
    o3, l3 = pktgpu.pcap_index(buf)
    assert np.array_equal(o3, offs) and np.array_equal(l3, lens)
    with pytest.raises(ValueError):
        pktgpu.pcap_index(b"\x00" * 40)
    with pytest.raises(ValueError):
        pktgpu.pcap_index(pc[:-3])  # last record runs past the end


def test_host_checksum_matches_oracle(L):
    rng = np.random.default_rng(1)
    for _ in range(2000):
        h = rng.integers(0, 256, 20, dtype=np.uint8).tobytes()
        assert L.pkt_ipv4_checksum_host(h, 20) == oracle.ipv4_checksum(h)


def test_bytes_per_packet_schema():
    cols = schema.columns_of(["chain", "ether", "ipv4", "udp"])
    # chain: 1+1+3*(1+2)+2+2+4 = 19 at 3 slots; ether 18; ipv4 22+2; udp 8
    assert schema.bytes_per_packet(cols, n_slots=3) == 19 + 18 + 24 + 8
