"""Kernel timeline of the hooks' eager calls (rocprofv3 --kernel-trace of bench_hooks below): per call, each
kernel's start offset, duration and the gap before it, to see what a synchronised compression() /
decompression(model) spends beyond its kernels.

    rocprofv3 --kernel-trace -d DIR -o run --output-format csv -- python3 tools/hook_timeline.py run
    python3 tools/hook_timeline.py report DIR
"""
import csv
import glob
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run():
    import torch
    from coala_amd.compression import UpdateCodec
    from coala_amd.layouts import build_module
    dev = torch.device("cuda", 0)
    m = build_module("resnet50_tv", seed=1, device=dev)
    g = build_module("resnet50_tv", seed=2, device=dev)
    codec = UpdateCodec(0.01, 8, "delta")
    base = codec.snapshot(g)
    for _ in range(5):
        up = codec.encode_module(m, base=base)
        codec.decode_module(up, g, base=base)
    torch.cuda.synchronize()
    marks = []
    for _ in range(10):
        time.sleep(0.002)  # a gap in the trace between calls
        t0 = time.perf_counter()
        up = codec.encode_module(m, base=base)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        time.sleep(0.002)
        t2 = time.perf_counter()
        codec.decode_module(up, g, base=base)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        marks.append(((t1 - t0) * 1e3, (t3 - t2) * 1e3))
    print(json.dumps({"call_ms": marks}))


def report(d):
    rows = []
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    calls, cur = [], []
    for s, e, n in rows:  # a call = kernels separated by less than 1 ms
        if cur and s - cur[-1][1] > 1_000_000:
            calls.append(cur)
            cur = []
        cur.append((s, e, n))
    if cur:
        calls.append(cur)
    out = []
    for c in calls[-20:]:
        t0 = c[0][0]
        ks, prev = [], t0
        for s, e, n in c:
            short = n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:48]
            ks.append({"k": short, "start_us": round((s - t0) / 1e3, 2), "dur_us": round((e - s) / 1e3, 2),
                       "gap_us": round((s - prev) / 1e3, 2)})
            prev = e
        out.append({"span_us": round((c[-1][1] - t0) / 1e3, 2), "kernels": ks})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    run() if sys.argv[1] == "run" else report(sys.argv[2])
