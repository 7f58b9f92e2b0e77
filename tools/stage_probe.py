"""Probe: the real k_scan / k_decode launched back to back in isolation (split-stage ABI, one stage per
call), against the same kernels inside the encode+decode step. Separates the kernel's own speed from
its context (what ran before it). Default workload: 16 x resnet50_tv, ratio 0.01, 8 bits.

    python tools/stage_probe.py [--reps 10]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--reps", type=int, default=10)
    p.add_argument("--clients", type=int, default=16)
    a = p.parse_args()
    import torch

    from coala_amd.compression import CodecPlan
    from coala_amd.compression import _lib
    from coala_amd.layouts import fp32_sizes
    from coala_amd.workload import synth_batch

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    plan = CodecPlan(fp32_sizes("resnet50_tv"), 0.01, 8, clients=a.clients, device=dev)
    flat = synth_batch(plan.table, dev, client_ids=range(a.clients))
    ws, dws = plan.empty_workspace(), plan.empty_decode_workspace()
    enc, out = plan.empty_encoded(), plan.empty_flat()
    s = torch.cuda.current_stream()
    for _ in range(3):
        plan.encode(flat, out=enc, workspace=ws)
        plan.decode(enc, out=out, workspace=dws)
    torch.cuda.synchronize()
    nbytes = 4 * plan.table.span
    res = {}

    def time_it(name, fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        fn()
        torch.cuda.synchronize()
        e0.record(s)
        for _ in range(a.reps):
            fn()
        e1.record(s)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.reps
        res[name] = {"ms": round(ms, 4), "GBps_4N": round(nbytes / (ms * 1e-3) / 1e9, 1)}

    none5, none3 = [None] * 5, [None] * 3
    time_it("scan_only_b2b", lambda: plan.encode(flat, out=enc, workspace=ws,
                                                 sched=(none5, none5, _lib.COALAC_STAGE_SCAN)))
    time_it("decode_only_b2b", lambda: plan.decode(enc, out=out, workspace=dws,
                                                   sched=(none3, none3, _lib.COALAC_STAGE_DECODE)))
    time_it("bounds_only_b2b", lambda: plan.decode(enc, out=out, workspace=dws,
                                                   sched=(none3, none3, _lib.COALAC_STAGE_BOUNDS)))
    time_it("sample_only_b2b", lambda: plan.encode(flat, out=enc, workspace=ws,
                                                   sched=(none5, none5, _lib.COALAC_STAGE_SAMPLE)))
    time_it("select_emit_only_b2b", lambda: plan.encode(flat, out=enc, workspace=ws,
                                                        sched=(none5, none5, _lib.COALAC_STAGE_SELECT)))
    time_it("small_only_b2b", lambda: plan.encode(flat, out=enc, workspace=ws,
                                                  sched=(none5, none5, _lib.COALAC_STAGE_SMALL)))
    time_it("encode_b2b", lambda: plan.encode(flat, out=enc, workspace=ws))
    time_it("decode_b2b", lambda: plan.decode(enc, out=out, workspace=dws))
    time_it("step", lambda: (plan.encode(flat, out=enc, workspace=ws), plan.decode(enc, out=out, workspace=dws)))
    # scan then decode alternating (the step's streaming kernels only)
    time_it("scan_decode_alt", lambda: (
        plan.encode(flat, out=enc, workspace=ws, sched=(none5, none5, _lib.COALAC_STAGE_SCAN)),
        plan.decode(enc, out=out, workspace=dws, sched=(none3, none3, _lib.COALAC_STAGE_DECODE))))
    print(json.dumps(res, indent=1), flush=True)


if __name__ == "__main__":
    main()
