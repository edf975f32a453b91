"""The Rust binding in INTEGRATION.md (what a packet_rs maintainer adds as src/gpu.rs to call the
library instead of fast::parse per packet, reference src/lib.rs:136-140, src/parser/fast.rs:5) must
match include/pktgpu.h exactly.  There is no cargo in this image, so this CPU test checks it
mechanically: every struct field (name, order, Rust type = C width + pointer levels + mutability)
and every function (name, argument names and types, return type)."""
import os
import re
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "scripts"))
import rust_binding as rb  # noqa: E402


def _rust_code():
    md = open(os.path.join(REPO, "INTEGRATION.md")).read()
    blocks = rb.RUST_BLOCK.findall(md)
    assert blocks, "no ```rust block in INTEGRATION.md"
    return blocks[0]


def test_every_struct_field_matches_the_header():
    code = _rust_code()
    hs, rs = rb.header_structs(), rb.rust_structs(code)
    assert set(hs) == set(rs), (sorted(hs), sorted(rs))
    for name, fields in hs.items():
        assert rs[name] == fields, name
    assert len(rs["PktOut"]) == 49
    assert "/* …" not in code and "..." not in code.split("extern")[0]


def test_every_function_matches_the_header():
    hf, rf = rb.header_functions(), rb.rust_functions(_rust_code())
    assert set(hf) == set(rf), (set(hf) ^ set(rf))
    for name, sig in hf.items():
        assert rf[name] == sig, name


def test_header_parser_sees_every_exported_prototype():
    """The parser must find exactly the functions the library's ctypes stub binds."""
    sys.path.insert(0, os.path.join(REPO, "packet-rs_amd"))
    from pktgpu import _lib
    assert set(rb.header_functions()) == set(_lib.SIGNATURES)


def test_c_type_mapping():
    assert rb.rust_of(*rb.c_type("const uint64_t *const *values")) == "*const *const u64"
    assert rb.rust_of(*rb.c_type("uint64_t *const *values")) == "*const *mut u64"
    assert rb.rust_of(*rb.c_type("void *const *shard_out")) == "*const *mut c_void"
    assert rb.rust_of(*rb.c_type("pkt_ctx_t **ctx")) == "*mut *mut PktCtx"
    assert rb.rust_of(*rb.c_type("uint64_t off[2]")) == "*mut u64"
    assert rb.rust_of(*rb.c_type("const char **name")) == "*mut *const c_char"
    assert rb.rust_of(*rb.c_type("uint32_t stride")) == "u32"


def test_packet_slice_adapter_builds_every_reference_slice_type():
    """the adapter `slices()` in INTEGRATION.md turns pkt_view's (type, offset) list into
    the reference's own PacketSlice (lib.rs:136-140) with `<Hdr>Slice::from(&arr[o..o + <Hdr>::size()])`
    + insert + set_payload (packet.rs:714-731).  Its match arms must map every header id of pktgpu.h to
    the Slice type of the make_header! invocation with that name (tests/golden/make_header_names.json,
    transcribed from headers.rs:529-827), and the adapter must call pkt_view."""
    import json
    sys.path.insert(0, os.path.join(REPO, "packet-rs_amd"))
    from pktgpu import schema
    code = _rust_code()
    body = code[code.index("pub fn slices<'a>"):]
    assert "pkt_view(" in body and "set_payload(" in body and "PacketSlice::new()" in body
    arms = re.findall(r"(\d+) => s\.insert\((\w+)Slice::from\(&arr\[o\.\.o \+ (\w+)::size\(\)\]\)\)", body)
    gold = [h["name"] for h in json.load(open(os.path.join(REPO, "tests", "golden", "make_header_names.json")))["headers"]]
    assert len(gold) == 21 and len(arms) == len(gold)
    for tid, slice_name, size_name in arms:
        t = int(tid)
        assert slice_name == size_name == schema.HDR_NAMES[t], (t, slice_name, size_name)
    assert [a[1] for a in arms] == gold
    # the list is inserted back to front (insert puts a header at position 0)
    assert "for k in (0..nh as usize).rev()" in body
