#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel stats.  Stops at the first step
# that crashes (signal / timeout); plain test failures (pytest exit 1) do not stop the bench.
# usage: scripts/gpu_round.sh TAG [bench args...]
set -u
TAG=${1:-r01}; shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
crashed() { case "$1" in 0|1) return 1;; *) return 0;; esac; }

echo "== build check" 
ls -la packet-rs_amd/lib oracle/build > "$OUT/ls.txt" 2>&1

if [ "${SKIP_TESTS:-0}" = "1" ]; then echo "== (tests skipped)"; else
echo "== pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/gpu_tests.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 "$OUT/gpu_tests.log"
if crashed $rc; then echo "pytest crashed ($rc), stopping"; exit $rc; fi

echo "== smoke"
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 "$OUT/smoke.log"
if crashed $rc; then exit $rc; fi
fi

echo "== bench"
timeout -k 10 300 python bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; cat "$OUT/bench.json"; tail -5 "$OUT/bench.err"
if [ $rc -ne 0 ]; then exit $rc; fi

echo "== rocprofv3 kernel trace (one stream: per-dispatch durations = the roofline phase)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o trace -- \
    python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-c5 --streams 1 "$@" > "$OUT/prof_bench.json" 2> "$OUT/prof.err"
rc=$?; echo "rocprof rc=$rc"; tail -2 "$OUT/prof.err"
if [ $rc -ne 0 ]; then exit $rc; fi
echo "== PMC traffic passes"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o pmc -- \
    python bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-c5 --streams 1 "$@" > /dev/null 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o pmc -- \
    python bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-c5 --streams 1 "$@" > /dev/null 2>&1 && \
python scripts/traffic.py "$OUT/pmc_fetch" "$OUT/pmc_write" "$OUT/traffic.json" parse_kernel "$TAG $*"
rc=$?; echo "pmc rc=$rc"
exit $rc
