"""Cost of the raw-data path (one block per segment: exact select over the whole segment's input, per-unit counts,
re-read in k_emit) — what a segment pays when its sampled bracket misses or a unit overflows its record slots.
Times one encode (median of 20, HIP events on the launch stream) of
  * ResNet-50's largest segment alone (2,359,296 elements) and one whole ResNet-50 update (161 large segments),
  * on the sampled path and forced onto the raw-data path (COALAC_FLAG_FORCE_EXACT),
at ratios 0.01 and 0.1; prints one JSON line per case with the plan's fallback count.

    python tools/raw_path_cost.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from coala_amd.compression import CodecPlan
    from coala_amd.compression._lib import COALAC_FLAG_FORCE_EXACT
    from coala_amd.layouts import fp32_sizes
    from coala_amd.workload import synth_batch
    dev = torch.device("cuda:0")
    layouts = {"largest segment (2,359,296)": [2359296], "ResNet-50": fp32_sizes("resnet50_tv")}
    for ratio in (0.01, 0.1):
        for name, sizes in layouts.items():
            plan = CodecPlan(sizes, ratio, 8, device=dev)
            flat = synth_batch(plan.table, dev)
            ws = plan.empty_workspace()
            enc = plan.empty_encoded()
            row = {"case": name, "ratio": ratio}
            for label, flags in (("sampled", 0), ("raw_path", COALAC_FLAG_FORCE_EXACT)):
                for _ in range(3):
                    plan.encode(flat, out=enc, workspace=ws, flags=flags)
                ts = []
                for _ in range(20):
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record()
                    plan.encode(flat, out=enc, workspace=ws, flags=flags)
                    b.record()
                    b.synchronize()
                    ts.append(a.elapsed_time(b))
                ts.sort()
                row[label + "_ms"] = round(ts[len(ts) // 2], 4)
                row[label + "_fallbacks"] = plan.fallbacks(ws)
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
