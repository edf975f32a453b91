"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer (no GPU).

tests/cpp/fuzz_host.cpp drives the pcap indexer of the C ABI (packet-rs_amd/csrc/pktgpu_host.cpp —
the parser of untrusted capture files, tests/pcap.rs:7-37 format) over valid, truncated,
bit-flipped and length-corrupted captures with every cap, checking each result against a second
walk of the format, plus the metadata / checksum entry points and the CPU oracle
(oracle/pkt_oracle.c) on random packets under every entry.  Built here with g++/gcc
-fsanitize=address,undefined; any report fails the run.
"""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "tests", "cpp", "build")
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-O1", "-g"]


def build():
    if not shutil.which("g++") or not shutil.which("gcc"):
        pytest.skip("no host compiler")
    os.makedirs(OUT, exist_ok=True)
    obj = os.path.join(OUT, "pkt_oracle_asan.o")
    subprocess.run(["gcc", "-std=c11", *SAN, "-c", "-o", obj, os.path.join(REPO, "oracle", "pkt_oracle.c")],
                   check=True)
    exe = os.path.join(OUT, "fuzz_host_asan")
    subprocess.run(["g++", "-std=c++17", *SAN, "-static-libasan", "-o", exe,
                    os.path.join(REPO, "tests", "cpp", "fuzz_host.cpp"),
                    os.path.join(REPO, "packet-rs_amd", "csrc", "pktgpu_host.cpp"), obj, "-lpthread"], check=True)
    return exe


def test_host_code_under_asan_ubsan():
    exe = build()
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([exe, "3000"], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "fuzz OK 3000" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr
