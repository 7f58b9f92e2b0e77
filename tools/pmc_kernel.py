"""Mean of each PMC counter over the dispatches of one kernel in a rocprofv3 counter_collection.csv:
    python tools/pmc_kernel.py <dir> <kernel-substring>   (prints JSON; the CSV is not modified)"""
import csv
import glob
import json
import sys
from collections import defaultdict

d, name = sys.argv[1], sys.argv[2]
vals = defaultdict(list)
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if name in r.get("Kernel_Name", ""):
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(json.dumps({k: {"mean": sum(v) / len(v), "n": len(v)} for k, v in sorted(vals.items())}, indent=1))
