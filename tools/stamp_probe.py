"""Per-block phase timestamps of one encode (COALAC_FLAG_STAMPS; 100 MHz real-time counter, 10 ns):
small segments (k_presel / k_small: slots 2-7), k_select blocks (slots 0, 1, 10-12) and k_emit blocks
(slots 13-14). Prints, per kernel role, when its blocks start (spread), how long each block runs (median /
p90 / max) and per-phase medians, in microseconds.

    python tools/stamp_probe.py [--layout resnet50_tv] [--clients 1]
"""
import argparse
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def stats(x):
    x = np.asarray(x, dtype=np.float64)
    if x.size == 0:
        return "-"
    return f"med {np.median(x):6.2f} p90 {np.percentile(x, 90):6.2f} max {x.max():6.2f}"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layout", default="resnet50_tv")
    ap.add_argument("--clients", type=int, default=1)
    ap.add_argument("--ratio", type=float, default=0.01)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import torch

    from coala_amd.compression import CodecPlan, SegmentTable, _lib
    from coala_amd.compression.plan import _ptr
    from coala_amd.layouts import fp32_sizes
    from coala_amd.workload import synth_batch

    dev = torch.device("cuda", 0)
    t = SegmentTable(fp32_sizes(a.layout), a.ratio, a.clients)
    plan = CodecPlan(None, a.ratio, 8, table=t, device=dev)
    flat = synth_batch(t, dev)
    ws = plan.empty_workspace()
    enc = plan.empty_encoded()
    nseg = t.n_segments
    n = t.segs[:, 1]
    small = np.nonzero(n <= 4096)[0]
    n_large = int((n > 4096).sum())
    F = _lib.COALAC_FLAG_STAMPS
    rows = []
    for mode in ("encode",):
        acc = []
        for r in range(a.reps):
            ws.zero_()
            plan.encode(flat, out=enc, workspace=ws, flags=F)
            torch.cuda.synchronize()
            buf = (ctypes.c_uint64 * (16 * nseg))()
            got = plan._lib.coalac_debug_stamps(plan._h, _ptr(ws), None, buf, 16 * nseg)
            acc.append(np.frombuffer(buf, dtype=np.uint64)[:got].reshape(-1, 16).astype(np.int64))
        st = acc[-1]
        print(f"== {mode} ({a.layout} x{a.clients}, last of {a.reps}) ==")
        # small segments
        S = st[small]
        S = S[S[:, 2] > 0]
        if len(S):
            t0 = S[:, 2].min()
            print(f"small blocks {len(S)}: start spread {(S[:, 2].max() - t0) / 100:.2f} us, last end "
                  f"{(S[:, 7].max() - t0) / 100:.2f} us; block {stats((S[:, 7] - S[:, 2]) / 100)}")
            names = ["load", "select", "scans", "minmax", "write"]
            for i, nm in enumerate(names):
                print(f"   {nm:7s} {stats((S[:, 3 + i] - S[:, 2 + i]) / 100)}")
            ns = n[small][st[small][:, 2] > 0]
            order = np.argsort(-(S[:, 7] - S[:, 2]))
            for j in list(order[:6]) + list(order[len(order) // 2:len(order) // 2 + 2]):
                b = S[j]
                print(f"   n={int(ns[j]):5d} start {(b[2] - t0) / 100:5.2f} " +
                      " ".join(f"{nm}={(b[3 + i] - b[2 + i]) / 100:5.2f}" for i, nm in enumerate(names)))
            by = {}
            for nn, d in zip(ns, (S[:, 7] - S[:, 2]) / 100):
                by.setdefault(int(nn), []).append(d)
            print("   by n:", " ".join(f"{k}:{np.median(v):.1f}({len(v)})" for k, v in sorted(by.items())))
        if mode == "encode":
            E = st[:, 13:15]
            E = E[E[:, 0] > 0]
            if len(E):
                t0 = E[:, 0].min()
                print(f"emit blocks {len(E)}: start spread {(E[:, 0].max() - t0) / 100:.2f} us, last end "
                      f"{(E[:, 1].max() - t0) / 100:.2f} us; block {stats((E[:, 1] - E[:, 0]) / 100)}")
            L = st[:n_large]
            L = L[L[:, 0] > 0]
            if len(L):
                t0 = L[:, 0].min()
                print(f"select blocks {len(L)}: start spread {(L[:, 0].max() - t0) / 100:.2f} us, last end "
                      f"{(L[:, 12].max() - t0) / 100:.2f} us; block {stats((L[:, 12] - L[:, 0]) / 100)}")
                for nm, i, j in (("groups", 0, 1), ("offsets", 10, 11), ("mn/scale", 11, 12)):
                    print(f"   {nm:8s} {stats((L[:, j] - L[:, i]) / 100)}")


if __name__ == "__main__":
    main()
