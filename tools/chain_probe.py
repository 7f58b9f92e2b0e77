"""Latency-chain probe for ONE update (or a small batch): runs, back to back on one stream,
  * R full encode + decode round trips (the kernel sequence),
  * R launches of each encode stage alone through the split-stage ABI (k_sample only, k_small only),
so that `rocprofv3 --kernel-trace --stats -- python3 tools/chain_probe.py` reports every kernel's mean
duration, k_sample and k_small separated from k_presel. Also prints the host-timed round trip.

    python tools/chain_probe.py [--layout resnet50_tv] [--clients 1] [--reps 200]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layout", default="resnet50_tv")
    ap.add_argument("--clients", type=int, default=1)
    ap.add_argument("--ratio", type=float, default=0.01)
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--stages", action="store_true", help="also launch k_sample / k_small alone")
    a = ap.parse_args()
    import torch

    from coala_amd.compression import CodecPlan, SegmentTable, _lib
    from coala_amd.layouts import fp32_sizes
    from coala_amd.workload import synth_batch

    dev = torch.device("cuda", 0)
    t = SegmentTable(fp32_sizes(a.layout), a.ratio, a.clients)
    plan = CodecPlan(None, a.ratio, 8, table=t, device=dev)
    flat = synth_batch(t, dev)
    ws, dws = plan.empty_workspace(), plan.empty_decode_workspace()
    enc = plan.empty_encoded()
    out = torch.empty(t.span, dtype=torch.float32, device=dev)
    for _ in range(10):
        plan.encode(flat, out=enc, workspace=ws)
        plan.decode(enc, out=out, workspace=dws)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        plan.encode(flat, out=enc, workspace=ws)
        plan.decode(enc, out=out, workspace=dws)
    torch.cuda.synchronize()
    rt = (time.perf_counter() - t0) / a.reps * 1e6
    print(f"{a.layout} x{a.clients}: round trip {rt:.1f} us ({4 * t.n_elements / rt / 1e3:.1f} GB/s of update)")
    if a.stages:
        nothing = [None] * 5
        for st in (_lib.COALAC_STAGE_SAMPLE, _lib.COALAC_STAGE_SMALL):
            for _ in range(a.reps):
                plan.encode(flat, out=enc, workspace=ws, sched=(nothing, nothing, st))
            torch.cuda.synchronize()


if __name__ == "__main__":
    main()
