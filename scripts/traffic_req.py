#!/usr/bin/env python3
"""Per-launch L2 -> memory read bytes from the request-size counters (one rocprofv3 --pmc pass with
TCC_EA0_RDREQ_sum, TCC_EA0_RDREQ_32B_sum, TCC_EA0_RDREQ_64B_sum, TCC_EA0_RDREQ_128B_sum):
read bytes = 32 x RDREQ_32B + 64 x RDREQ_64B + 128 x RDREQ_128B (no FETCH_SIZE doubling needed).
usage: traffic_req.py PMC_DIR KERNEL_SUBSTRING [OUT_JSON LABEL]"""
import collections
import csv
import glob
import json
import statistics
import sys

d, kern = sys.argv[1], sys.argv[2]
f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
per = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f)):
    if kern in r["Kernel_Name"]:
        per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
names = ["TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum"]
med = {k: statistics.median(v[k] for v in per.values()) for k in names}
rd = 32 * med[names[1]] + 64 * med[names[2]] + 128 * med[names[3]]
res = {"kernel": kern, "dispatches": len(per), "requests_per_launch": med, "read_bytes": rd,
       "unsized_requests": med[names[0]] - med[names[1]] - med[names[2]] - med[names[3]],
       "how": "32*RDREQ_32B + 64*RDREQ_64B + 128*RDREQ_128B (TCC_EA0, summed over channels), median over dispatches",
       "label": sys.argv[4] if len(sys.argv) > 4 else ""}
print(json.dumps(res))
if len(sys.argv) > 3:
    json.dump(res, open(sys.argv[3], "w"), indent=1)
