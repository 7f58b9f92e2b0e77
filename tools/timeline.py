"""Summarise a rocprofv3 --kernel-trace CSV: how busy the HBM-streaming kernels keep the chip.

    python tools/timeline.py <dir with *kernel_trace.csv> [--last-frac 0.5]

Over the last `last-frac` of the codec's kernel trace (the timed steps; warm-up and setup kernels come
first): wall span, union of k_scan / k_decode intervals ("streaming busy"), union of all codec kernels,
the overlap of streaming kernels with each other (should be ~0: the lane pipeline serialises them),
and per-kernel mean duration.
"""
import argparse
import csv
import glob
import json
import os
import sys

CODEC = ("k_sample", "k_presel", "k_scan", "k_small", "k_ghist", "k_pick", "k_gwin", "k_select", "k_emit", "k_bounds",
         "k_decode", "k_decode_lds", "k_fill", "k_fillscatter", "k_scatter", "k_aggregate")
STREAMING = ("k_scan", "k_decode", "k_decode_lds")


def base_name(n):
    """'void (anonymous namespace)::k_scan<false, false>((anonymous namespace)::Params)' -> 'k_scan'"""
    n = n.replace("(anonymous namespace)::", "").replace("void ", "").strip().strip('"')
    return n.split("(")[0].split("<")[0].split("::")[-1].strip()


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--last-frac", type=float, default=0.5)
    ap.add_argument("--group", type=int, default=1,
                    help="streaming kernels launched this many at a time (bench --split): also report the mean "
                         "union interval (first start to last end) of each group of consecutive launches")
    ap.add_argument("--last-groups", type=int, default=0,
                    help="with --group: average only the last N groups (bench.py's joined roofline steps)")
    ap.add_argument("--dump", type=int, default=0, help="also print the last N kernels (start/end us, queue)")
    a = ap.parse_args()
    files = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        sys.exit(f"no kernel_trace.csv under {a.dir}")
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = base_name(r.get("Kernel_Name", ""))
                if k in CODEC:
                    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k,
                                 r.get("Queue_Id", r.get("Stream_Id", "?"))))
    rows.sort()
    all_rows = rows
    rows = rows[int(len(rows) * (1.0 - a.last_frac)):]
    t0, t1 = rows[0][0], max(r[1] for r in rows)
    span = t1 - t0
    st = [(s, e) for s, e, k, _ in rows if k in STREAMING]
    st_sum = sum(e - s for s, e in st)
    out = {
        "kernels": len(rows),
        "span_us": span / 1e3,
        "streaming_busy_us": union(st) / 1e3,
        "streaming_busy_frac": union(st) / span,
        "streaming_self_overlap_us": (st_sum - union(st)) / 1e3,
        "any_codec_busy_frac": union([(s, e) for s, e, _, _ in rows]) / span,
        "queues": sorted({q for *_, q in rows}),
        "mean_us": {},
    }
    for k in CODEC:
        d = [e - s for s, e, kk, _ in rows if kk == k]
        if d:
            out["mean_us"][k] = round(sum(d) / len(d) / 1e3, 2)
    if a.group > 1:
        out["group"] = a.group
        out["group_union_us"] = {}
        for k in STREAMING:
            # group over the whole trace (every step launches `group` of them), keep the last groups
            d = sorted((s, e) for s, e, kk, _ in all_rows if kk == k)
            spans = [max(e for _, e in d[i:i + a.group]) - d[i][0]
                     for i in range(0, len(d) - a.group + 1, a.group)]
            spans = spans[-a.last_groups:] if a.last_groups else spans[int(len(spans) * (1.0 - a.last_frac)):]
            if spans:
                out["group_union_us"][k] = round(sum(spans) / len(spans) / 1e3, 2)
    print(json.dumps(out, indent=1))
    if a.dump:
        tail = rows[-a.dump:]
        z = tail[0][0]
        for s_, e_, k, q in tail:
            print(f"{(s_ - z) / 1e3:9.1f} {(e_ - z) / 1e3:9.1f} {(e_ - s_) / 1e3:7.1f}  q{q}  {k}")


if __name__ == "__main__":
    main()
