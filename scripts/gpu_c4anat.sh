#!/bin/bash
# C4 request anatomy: L2 read/write requests and memory-side requests per parse launch, by column
# set and window width (what generates the reads beyond the windows' lines).
set -u
TAG=${1:-r03anat}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
P1="TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_READ_sum"
P2="TCC_HIT_sum TCC_MISS_sum TCC_WRITE_sum TCC_REQ_sum"
for w in ${WINDOWS:-64 0}; do for v in ${VARIANTS:-status all}; do
  for p in 1 2; do
    eval C=\$P$p
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C --output-format csv -d $OUT/w${w}_${v}_p$p -o pmc -- \
      python scripts/kbench.py --config c4 --variants $v --windows $w --streams 1 --rounds 1 --iters 8 > $OUT/kb_w${w}_$v.txt 2>&1 || exit $?
  done
done; done
python - $OUT <<'PY'
import csv, glob, sys, collections, statistics, os
d = sys.argv[1]
for w in [int(x) for x in os.environ.get("WINDOWS", "64 0").split()]:
    for v in os.environ.get("VARIANTS", "status all").split():
        vals = {}
        for p in (1, 2):
            f = glob.glob(f"{d}/w{w}_{v}_p{p}/**/*counter_collection.csv", recursive=True)[0]
            per = collections.defaultdict(lambda: collections.defaultdict(float))
            for r in csv.DictReader(open(f)):
                if "parse_kernel" in r["Kernel_Name"]:
                    per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
            for k in next(iter(per.values())):
                vals[k] = statistics.median(x[k] for x in per.values())
        print(f"w={w:3d} {v:6s} " + " ".join(f"{k.replace('_sum','')}={vals[k]/1e6:.3f}M" for k in sorted(vals)))
PY
