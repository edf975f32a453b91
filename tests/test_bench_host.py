"""Host-side arithmetic of bench.py's roofline objects (no GPU): the line-granular floor."""
import importlib.util
import os

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_spec = importlib.util.spec_from_file_location("bench", os.path.join(REPO, "bench.py"))
bench = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(bench)


def brute_lines(starts, spans):
    lines = set()
    for s, n in zip(starts, spans):
        n = max(int(n), 1)
        lines.update(range(int(s) // 128, (int(s) + n - 1) // 128 + 1))
    return 128 * len(lines)


def test_line_bytes_fixed_stride():
    n = 1000
    # C2: 42-byte header spans at a 64-byte stride: two packets per line
    assert bench.line_bytes(n, 64, None, np.full(n, 42)) == 64 * n
    # C3: 128-byte slots, headers inside the slot: one line each
    assert bench.line_bytes(n, 128, None, np.full(n, 58)) == 128 * n
    # failed parses (span 0) still count the packet's first line
    assert bench.line_bytes(n, 128, None, np.zeros(n)) == 128 * n


def test_line_bytes_indexed_vs_brute_force():
    rng = np.random.default_rng(7)
    for _ in range(20):
        n = int(rng.integers(1, 300))
        lens = rng.integers(0, 400, n)
        gaps = rng.integers(0, 40, n)
        offs = np.cumsum(lens + gaps) - lens - gaps + 24
        span = np.minimum(lens, rng.integers(0, 200, n))
        perm = rng.permutation(n) if rng.integers(0, 2) else np.arange(n)  # any record order
        assert bench.line_bytes(n, None, offs[perm].astype(np.uint64), span[perm]) == brute_lines(offs, span)


def test_gpus_beyond_visible_devices_exits_nonzero():
    """`bench.py --gpus N` with fewer visible devices must fail.  This container has
    no GPU."""
    import subprocess
    import sys
    import pytest
    torch = pytest.importorskip("torch")
    if torch.cuda.device_count() >= 2:
        pytest.skip("two or more devices visible")
    for extra in ([],):
        r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "2",
                            "--warmup", "1", "--no-cpu-baseline"] + extra,
                           capture_output=True, text=True, timeout=300,
                           env=dict(os.environ, HIP_VISIBLE_DEVICES=os.environ.get("HIP_VISIBLE_DEVICES", "")))
        assert r.returncode != 0, (extra, r.stdout[-500:], r.stderr[-500:])
        assert "device" in r.stderr, r.stderr[-500:]
        assert not r.stdout.strip(), r.stdout[-500:]
