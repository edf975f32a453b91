#!/bin/bash
# Load cache-policy probe: time per launch and memory-side request sizes (scripts/probe_policy.hip).
set -u
OUT=gpurun_out/${1:-r03pol}; mkdir -p $OUT scripts/bin
export TMPDIR=/tmp
hipcc -O3 --offload-arch=gfx950 -o scripts/bin/probe_policy scripts/probe_policy.hip || exit 3
timeout -k 10 60 scripts/bin/probe_policy 16 > $OUT/time.txt 2>&1 || exit $?
cat $OUT/time.txt
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum \
  --output-format csv -d $OUT/pmc -o pmc -- scripts/bin/probe_policy 1 > $OUT/pmc.log 2>&1 || exit $?
python - $OUT <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
f = glob.glob(f"{d}/pmc/**/*counter_collection.csv", recursive=True)[0]
per = collections.defaultdict(lambda: collections.defaultdict(float)); name = {}
for r in csv.DictReader(open(f)):
    k = int(r["Dispatch_Id"]); per[k][r["Counter_Name"]] += float(r["Counter_Value"]); name[k] = r["Kernel_Name"]
pol = ["plain", "sc0", "nt", "sc0nt", "sc1", "sc1nt", "sc0sc1"]
for i, k in enumerate(sorted(per)):
    v = per[k]; w = 64 if i < 7 else 128
    print(f"width {w} {pol[i % 7]:7s} RDREQ {v['TCC_EA0_RDREQ_sum']/2**20:.3f}/item  32B {v['TCC_EA0_RDREQ_32B_sum']/2**20:.3f} 64B {v['TCC_EA0_RDREQ_64B_sum']/2**20:.3f} 128B {v['TCC_EA0_RDREQ_128B_sum']/2**20:.3f}")
PY
