"""The C++ host mirror (include/packet_rs_gpu.hpp): it compiles against the C ABI here (CPU),
and on the GPU parses the golden pcap with the same chains as ref22_expected.json."""
import json
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "tests", "cpp", "test_packet_rs_gpu.cpp")
BIN = os.path.join(REPO, "tests", "cpp", "build", "test_packet_rs_gpu")
LIBDIR = os.path.join(REPO, "packet-rs_amd", "lib")


def build():
    os.makedirs(os.path.dirname(BIN), exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "-I", os.path.join(REPO, "include"), SRC,
                    "-L", LIBDIR, "-lpktgpu", f"-Wl,-rpath,{LIBDIR}", "-o", BIN], check=True)
    return BIN


def test_cpp_mirror_compiles():
    assert os.path.exists(build())


@pytest.mark.gpu
def test_cpp_mirror_on_gpu():
    b = BIN if os.path.exists(BIN) else build()
    r = subprocess.run([b, os.path.join(REPO, "tests", "golden", "ref22.pcap")], check=True,
                       capture_output=True, text=True, timeout=120)
    assert "parse_pcap_equal 1" in r.stderr  # Parser::parse_pcap (pkt_parse_pcap_host) == parse_chain
    out = r.stdout.strip().splitlines()
    exp = json.load(open(os.path.join(REPO, "tests", "golden", "ref22_expected.json")))
    assert len(out) == len(exp)
    for line, e in zip(out, exp):
        parts = line.split(" | ")
        head = parts[0].split()
        assert head[1] == e["status"]
        assert [h.split("@") for h in head[2:]] == [[n, str(o)] for n, o in e["hdrs"]]
        assert parts[1] == f"payload {e['payload_off']} {e['payload_len']}"
        assert parts[2] == f"len {e['len']}" and parts[3] == "to_vec_equal 1"
