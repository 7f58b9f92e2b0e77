"""Summarise a tools/profile_round.sh output directory into one JSON object per kernel.

For every coalac kernel: dispatch count and mean duration (kernel trace, ns -> ms), mean FETCH_SIZE and
WRITE_SIZE per dispatch in bytes. FETCH_SIZE is reported raw AND doubled: on gfx950 it counts exactly
half of the bytes of wide (16 B/lane) coalesced streaming reads (MI355X_MICROARCH.md §HBM), which is
the access shape of k_scan / k_decode; rocprofv3 reports both counters in KB.

    python tools/pmc_summary.py gpurun_out/prof_r01
"""
import csv
import glob
import json
import os
import re
import sys


def rows(pattern):
    out = []
    for p in sorted(glob.glob(pattern, recursive=True)):
        with open(p, newline="") as f:
            out.extend(csv.DictReader(f))
    return out


def short(name):
    if name.startswith("_Z"):  # mangled (<length><name>): keep the kernel's base name
        m = re.search(r"N_\d(\d+)(k_\w+)", name)
        return m.group(2)[:int(m.group(1))] if m else name
    for tok in ("(anonymous namespace)::", "void ", "__global__ "):
        name = name.replace(tok, "")
    return name.split("(")[0].strip()


def main(d):
    res = {}
    for r in rows(os.path.join(d, "trace", "**", "*kernel_trace.csv")):
        k = short(r["Kernel_Name"])
        if not k.startswith("k_"):
            continue
        e = res.setdefault(k, {"dispatches": 0, "ns": 0})
        e["dispatches"] += 1
        e["ns"] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    for name, sub in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
        acc = {}
        for r in rows(os.path.join(d, sub, "**", "*counter_collection.csv")):
            if r.get("Counter_Name") != name:
                continue
            k = short(r["Kernel_Name"])
            if not k.startswith("k_"):
                continue
            a = acc.setdefault(k, {})
            key = r.get("Dispatch_Id") or r.get("Correlation_Id")
            a[key] = a.get(key, 0.0) + float(r["Counter_Value"])
        for k, per in acc.items():
            e = res.setdefault(k, {"dispatches": 0, "ns": 0})
            e[name + "_raw"] = round(sum(per.values()) / len(per), 3)
            e[name + "_bytes"] = round(1024.0 * sum(per.values()) / len(per))
    for k, e in res.items():
        if e["dispatches"]:
            e["mean_ms"] = round(e.pop("ns") / e["dispatches"] / 1e6, 5)
        else:
            e.pop("ns")
        if "FETCH_SIZE_bytes" in e:
            e["FETCH_SIZE_x2_bytes"] = 2 * e["FETCH_SIZE_bytes"]
    print(json.dumps(res, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(sys.argv[1])
