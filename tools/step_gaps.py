"""Per-step kernel sequence of a single-update config from a rocprofv3 kernel trace: for the last N steps (a step
= the run of codec kernels from one k_sample to the next), each kernel's start offset, duration and the idle gap
before it (µs), then the means — where the ~80 µs of one update's encode + decode go.

    python tools/step_gaps.py <dir with *kernel_trace.csv> [--steps 20]
"""
import argparse
import csv
import glob
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from timeline import CODEC, base_name  # noqa: E402

EXTRA = ("k_dense_minmax", "k_dense_seg", "k_dense_quant", "k_dense_deq")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--first", default="k_sample", help="kernel that opens a step")
    a = ap.parse_args()
    rows = []
    for f in glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = base_name(r.get("Kernel_Name", ""))
            if k in CODEC or k in EXTRA:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k))
    rows.sort()
    steps, cur = [], []
    for r in rows:
        if r[2] == a.first and cur:
            steps.append(cur)
            cur = []
        cur.append(r)
    if cur:
        steps.append(cur)
    steps = steps[-a.steps - 1:-1]  # (the last, maybe partial, run dropped)
    per = {}
    spans = []
    for st in steps:
        t0 = st[0][0]
        spans.append((st[-1][1] - t0) / 1e3)
        prev_end = None
        for i, (s, e, k) in enumerate(st):
            key = f"{i:02d} {k}"
            d = per.setdefault(key, {"start": [], "dur": [], "gap": []})
            d["start"].append((s - t0) / 1e3)
            d["dur"].append((e - s) / 1e3)
            d["gap"].append(0.0 if prev_end is None else (s - prev_end) / 1e3)
            prev_end = e
    print(f"{len(steps)} steps, span (first start -> last end) mean {statistics.mean(spans):.2f} us, "
          f"min {min(spans):.2f}")
    for key in sorted(per):
        d = per[key]
        print(f"  {key:20s} start {statistics.mean(d['start']):7.2f}  dur {statistics.mean(d['dur']):6.2f} "
              f"(min {min(d['dur']):6.2f})  gap before {statistics.mean(d['gap']):5.2f}")


if __name__ == "__main__":
    main()
