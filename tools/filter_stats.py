"""Reduce a rocprofv3 kernel_stats.csv to the codec's kernels (+ one summary row for everything else,
i.e. the torch kernels that synthesise the workload) with short names, for committing under profiles/.

    python tools/filter_stats.py IN.csv OUT.csv
"""
import csv
import sys


def main(src, dst):
    rows = list(csv.DictReader(open(src)))
    keep = [r for r in rows if "(anonymous namespace)::k_" in r["Name"] and "at::native" not in r["Name"]]
    other = [r for r in rows if r not in keep]
    with open(dst, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
        w.writeheader()
        for r in keep:
            r = dict(r)
            for tok in ("void (anonymous namespace)::", "((anonymous namespace)::Params)", "(anonymous namespace)::"):
                r["Name"] = r["Name"].replace(tok, "")
            w.writerow(r)
        tot = sum(int(r["TotalDurationNs"]) for r in other)
        calls = sum(int(r["Calls"]) for r in other)
        w.writerow({"Name": "(other: torch kernels of the synthetic workload setup, not timed by the bench)",
                    "Calls": calls, "TotalDurationNs": tot, "AverageNs": round(tot / max(calls, 1), 1)})


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
