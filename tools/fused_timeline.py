"""Timeline of one ONE_LAUNCH k_fused encode from its per-work-item timestamps (COALAC_FLAG_ITEM_STAMPS).

    python tools/fused_timeline.py [--layout resnet50_tv] [--clients 1] [--ratio 0.01] [--c5]

Prints per role: items, first start / last end (us from the first start), median / p90 / max duration,
median / max wait (start -> inputs ready); then a coarse activity chart (items running per 2 us bin).
Timestamps are the 100 MHz real-time counter (10 ns).
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

ROLES = ["SAMPLE", "SMALL", "SCAN", "GHIST", "GWIN", "SELECT", "EMIT"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layout", default="resnet50_tv")
    ap.add_argument("--clients", type=int, default=1)
    ap.add_argument("--ratio", type=float, default=0.01)
    ap.add_argument("--c5", action="store_true")
    ap.add_argument("--bin-us", type=float, default=2.0)
    a = ap.parse_args()
    import torch

    from coala_amd.compression import CodecPlan, SegmentTable, _lib
    from coala_amd.compression.plan import _ptr, _stream_handle
    from coala_amd.layouts import fp32_sizes
    from coala_amd.workload import c5_share, mixed_table, synth_batch

    dev = torch.device("cuda", 0)
    if a.c5:
        ids, names = c5_share(0)
        t = mixed_table(names, a.ratio)
    else:
        ids = None
        t = SegmentTable(fp32_sizes(a.layout), a.ratio, a.clients)
    plan = CodecPlan(None, a.ratio, 8, table=t)
    flat = synth_batch(t, dev, client_ids=ids)
    ws = plan.empty_workspace()
    enc = plan.empty_encoded()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    times = {}
    one = _lib.COALAC_FLAG_ONE_LAUNCH
    for flags, name in ((one, "plain"), (one | _lib.COALAC_FLAG_ITEM_STAMPS, "stamped")):
        for _ in range(5):
            plan.encode(flat, out=enc, workspace=ws, flags=flags)
        e0.record()
        for _ in range(10):
            plan.encode(flat, out=enc, workspace=ws, flags=flags)
        e1.record()
        torch.cuda.synchronize()
        times[name] = e0.elapsed_time(e1) / 10 * 1e3
    n = plan._lib.coalac_plan_query  # noqa: F841 (plan handle is valid)
    cap = 1 << 22
    items = (ctypes.c_uint32 * cap)()
    st = (ctypes.c_uint64 * (3 * cap))()
    cnt = plan._lib.coalac_debug_item_stamps(plan._h, _ptr(ws), _stream_handle(None), items, st, cap)
    _lib.check(min(cnt, 0), "coalac_debug_item_stamps")
    it = np.frombuffer(items, dtype=np.uint32, count=cnt)
    s = np.frombuffer(st, dtype=np.uint64, count=3 * cnt).reshape(cnt, 3).astype(np.int64)
    role = it >> 28
    t0 = s[:, 0].min()
    start = (s[:, 0] - t0) / 100.0
    ready = (np.where(s[:, 1] > 0, s[:, 1], s[:, 0]) - t0) / 100.0
    end = (s[:, 2] - t0) / 100.0
    out = {"config": vars(a), "items": int(cnt), "encode_us": times, "span_us": float(end.max()), "roles": {}}
    print(f"items {cnt}; encode {times['plain']:.1f} us (stamped {times['stamped']:.1f} us); "
          f"stamped span {end.max():.1f} us")
    for r, nm in enumerate(ROLES):
        m = role == r
        if not m.any():
            continue
        d = end[m] - start[m]
        w = ready[m] - start[m]
        row = {"n": int(m.sum()), "first_start": float(start[m].min()), "last_start": float(start[m].max()),
               "last_end": float(end[m].max()), "dur_med": float(np.median(d)), "dur_p90": float(np.percentile(d, 90)),
               "dur_max": float(d.max()), "wait_med": float(np.median(w)), "wait_max": float(w.max())}
        out["roles"][nm] = row
        print(f"{nm:7s} n={row['n']:6d} start {row['first_start']:7.1f}..{row['last_start']:7.1f} end<= "
              f"{row['last_end']:7.1f} dur med {row['dur_med']:6.1f} p90 {row['dur_p90']:6.1f} max "
              f"{row['dur_max']:6.1f} wait med {row['wait_med']:6.1f} max {row['wait_max']:6.1f}")
    nb = int(np.ceil(end.max() / a.bin_us)) + 1
    chart = {}
    for r, nm in enumerate(ROLES):
        m = role == r
        if not m.any():
            continue
        act = np.zeros(nb)
        for s0, e_ in zip(start[m], end[m]):
            act[int(s0 / a.bin_us):int(e_ / a.bin_us) + 1] += 1
        chart[nm] = act.astype(int).tolist()
    out["chart_bin_us"] = a.bin_us
    out["chart"] = chart
    for i in range(nb):
        print(f"{i * a.bin_us:6.1f} " + " ".join(f"{nm[:4]}={chart[nm][i]:5d}" for nm in chart))
    print(json.dumps(out), file=sys.stderr)


if __name__ == "__main__":
    main()
