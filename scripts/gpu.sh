#!/bin/bash
# The one GPU-box driver: runs the named steps in order under their own time limits and stops at
# the first step that crashes (signal, abort, time limit); a plain test failure (pytest rc 1) is
# reported and the later steps still run.  Everything lands in gpurun_out/TAG/.
#
#   scripts/gpu.sh TAG STEP [STEP ...]
#
# steps
#   tests              pytest -m gpu (the whole parity suite)
#   smoke              __graft_entry__.smoke()
#   bench[=ARGS]       python bench.py ARGS (default: the driver's --steps 20 --warmup 5)
#   prof[=CFG]         rocprofv3 --kernel-trace --stats of bench.py --config CFG (one stream)
#   traffic[=CFG]      FETCH_SIZE (x2, gfx950) and WRITE_SIZE passes of the same -> traffic.json
#   kbench=CFG:VARS:WINDOWS:STAGING   scripts/kbench.py, 1 and 2 streams, 3 rounds
#   anat=CFG           memory-side request anatomy by column set (scripts/gpu_c4anat.sh)
#   sq=CFG:VARS        SQ / LDS / TCC counter passes of kbench (scripts/pmc.sh + pmc_summary.py)
#   stamps             per-wave segment stamps (needs lib/variants/stamps.so: build_variant.sh stamps -DPKTGPU_STAMPS=1)
#   pcapab             pcap indexer variants lib/variants/*.so, interleaved (scripts/pcap_index_bench.py)
#   pcap               pcap indexer rate + rocprofv3 kernel stats of it
#   pcapstamps         guess-wave / scan-block segment stamps (lib/variants/stamps.so, scripts/pcap_stamps.py)
#   secondary          §8(f) kernels: scripts/secondary_bench.py + rocprofv3 kernel stats
#   host               host-memory path rates (scripts/hostpath_native.py, pinned and pageable)
#   hostab             pkt_parse_host pinned: export pipeline vs zero copy, C2 and C4, by chunk
#   hostpieces[=LIST]  pkt_parse_pcap_host by piece size + the link alone (scripts/pcap_host_pieces.py)
#   ab=CFGS:VARS       every lib/variants/*.so through kbench, interleaved (scripts/ab.sh)
#   abn=CFG:VARS:A,B   named builds (main = lib/libpktgpu.so, else lib/variants/NAME.so), kbench, 3 rounds
#   pcapn=A,B          named builds through scripts/pcap_index_bench.py, 3 interleaved rounds
#   secn=W1,W2:A,B     named builds through scripts/secondary_bench.py --only W1,W2, 3 interleaved rounds
set -u
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
crashed() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
run() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  echo "== $name"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -4 "$OUT/$name.log" | cut -c1-400
  if crashed $rc; then echo "step $name crashed ($rc): stopping"; exit $rc; fi
  return $rc
}
for step in "$@"; do
  key=${step%%=*}; arg=""; [ "$key" != "$step" ] && arg=${step#*=}
  case $key in
    tests) run tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider ;;
    smoke) run smoke 300 python -c 'import __graft_entry__ as g; g.smoke()' ;;
    bench) run bench${arg:+_$(echo $arg | tr -c 'a-z0-9' '_')} 600 python bench.py ${arg:---steps 20 --warmup 5} ;;
    prof)  c=${arg:-c2}
           run prof_$c 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$c" -o trace -- \
               python bench.py --config $c --steps 50 --warmup 5 --no-cpu-baseline --no-c5 --no-extra --streams 1 ;;
    traffic) c=${arg:-c2}
           run fetch_$c 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_$c" -o pmc -- \
               python bench.py --config $c --steps 20 --warmup 2 --no-cpu-baseline --no-c5 --no-extra --streams 1
           run write_$c 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_$c" -o pmc -- \
               python bench.py --config $c --steps 20 --warmup 2 --no-cpu-baseline --no-c5 --no-extra --streams 1
           run traffic_$c 60 python scripts/traffic.py "$OUT/pmc_fetch_$c" "$OUT/pmc_write_$c" "$OUT/traffic_$c.json" parse_kernel "$TAG $c" ;;
    kbench) IFS=: read -r c v w st <<< "$arg"
           run kbench_${c}_st${st:-0} 300 python scripts/kbench.py --config $c --variants "${v:-status;chain;all}" --windows ${w:-0} \
               --staging ${st:-0} --streams 1,2 --rounds ${KB_ROUNDS:-3} --iters 24 ;;
    anat)  run anat_${arg:-c4} 900 bash scripts/gpu_c4anat.sh ${TAG}_anat ;;
    sq)    IFS=: read -r c v w <<< "$arg"; n=sq_${c}_$(echo "${v:-all}${w:+_w$w}" | tr -c 'a-z0-9' '_')
           run $n 600 bash scripts/pmc.sh ${TAG}_$n "${v:-all}" $c "--windows ${w:-0}"
           python scripts/pmc_summary.py gpurun_out/${TAG}_$n > "$OUT/$n.txt"; cat "$OUT/$n.txt" ;;
    stamps) run stamps 600 bash -c 'export PKTGPU_LIB=packet-rs_amd/lib/variants/stamps.so;
               for s in "c4 all 64" "c4 all 128"; do
                 set -- $s; python scripts/stamps.py --config $1 --columns $2 --window $3 || exit $?; done' ;;
    pcapab) run pcapab 900 bash -c 'for rep in 1 2 3; do for v in packet-rs_amd/lib/variants/*.so; do
               PKTGPU_LIB=$v python scripts/pcap_index_bench.py --reps 20 | sed "s|^|$(basename $v) |" || exit $?; done; done' ;;
    pcapstamps) run pcapstamps 300 env PKTGPU_LIB=packet-rs_amd/lib/variants/stamps.so python scripts/pcap_stamps.py ;;
    pcap)  run pcap 300 python scripts/pcap_index_bench.py --reps 20
           run pcap_prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/pcap_prof" -o trace -- \
               python scripts/pcap_index_bench.py --reps 10 ;;
    secondary) run secondary 300 python scripts/secondary_bench.py
           run secondary_prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/secprof" -o trace -- \
               python scripts/secondary_bench.py --cpu-budget 0.2 ;;
    hostab) run hostab 600 bash -c 'for c in c2 c4; do for st in 0 2; do python scripts/hostpath_native.py --config $c --staging $st --chunks 65536,131072,262144,524288 || exit $?; done; done' ;;
    hostpieces) run hostpieces 300 python scripts/pcap_host_pieces.py ${arg:+--pieces $arg} ;;
    host)  run host 600 bash -c 'for c in c2 c4; do python scripts/hostpath_native.py --config $c --chunks 262144 || exit $?;
               python scripts/hostpath_native.py --config $c --pageable --chunks 131072,262144 || exit $?; done' ;;
    ab)    IFS=: read -r c v <<< "$arg"; run ab_${c:-c2} 900 bash scripts/ab.sh "${c:-c2}" "${v:-status;chain;all}" 2 ;;
    abn)   IFS=: read -r c v names <<< "$arg"; run abn_${c}_$(echo "${v:-all}" | tr -c 'a-z0-9' '_') 900 bash scripts/ab_named.sh "$c" "${v:-all}" 3 ${names//,/ } ;;
    secn)  IFS=: read -r only names <<< "$arg"; run secn_$(echo "$only" | tr -c 'a-z0-9' '_') 900 bash -c 'for rep in 1 2 3; do for name in '"${names//,/ }"'; do
               lib=packet-rs_amd/lib/variants/$name.so; [ "$name" = main ] && lib=packet-rs_amd/lib/libpktgpu.so
               PKTGPU_LIB=$lib timeout -k 10 300 python scripts/secondary_bench.py --only '"$only"' --cpu-budget 0.02 | sed "s|^|$name |" || exit $?; done; done' ;;
    pcapn) IFS=: read -r names <<< "$arg"; run pcapn 600 bash -c 'for rep in 1 2 3; do for name in '"${names//,/ }"'; do
               lib=packet-rs_amd/lib/variants/$name.so; [ "$name" = main ] && lib=packet-rs_amd/lib/libpktgpu.so
               PKTGPU_LIB=$lib timeout -k 10 120 python scripts/pcap_index_bench.py --reps 20 | sed "s|^|$name |" || exit $?; done; done' ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
