"""Encode + decode time of one ResNet-50 update (ratio 0.01, 8 bits) for value distributions with heavy ties at a
NONZERO key — the raw-data path's territory: the §8(d) Gaussian, every |x| equal with random signs (a sign-SGD /
first-Adam-step delta), a Gaussian clipped at 1.5 sigma (value clipping: ~13 % of the elements at +-clip), and the
first-step delta in delta mode, where fp32 rounding of w -+ lr spreads the equal deltas over a few thousand ulps.
Prints ms per encode+decode (median of 20) and the plan's fallback count.

    python tools/tie_probe.py
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from coala_amd.compression import CodecPlan
    from coala_amd.layouts import fp32_sizes
    dev = torch.device("cuda:0")
    plan = CodecPlan(fp32_sizes("resnet50_tv"), 0.01, 8, device=dev)
    g = torch.Generator(device=dev).manual_seed(7)
    flat = plan.empty_flat()
    gauss = torch.randn(flat.numel(), generator=g, device=dev) * 1e-3
    cases = {
        "gaussian": gauss.clone(),
        "sign (all |x| equal)": torch.where(torch.rand(flat.numel(), generator=g, device=dev) < 0.5, -1e-3, 1e-3),
        "clipped at 1.5 sigma": gauss.clamp(-1.5e-3, 1.5e-3),
    }
    # delta mode: trained = fl(w - lr * sign), so x - w is lr only up to the rounding of w - lr (the deltas cluster
    # within a few thousand ulps of lr instead of tying exactly)
    w = torch.randn(flat.numel(), generator=g, device=dev) * 0.05
    adam = (w - torch.where(torch.rand(flat.numel(), generator=g, device=dev) < 0.5, -1e-3, 1e-3)).float()
    ws = plan.empty_workspace()
    enc = plan.empty_encoded()
    out = plan.empty_flat()
    cases["first-step delta (fl(w -+ lr) - w)"] = adam
    for name, x in cases.items():
        base = w if name.startswith("first-step") else None
        flat.copy_(x)
        ts = []
        for i in range(25):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            plan.encode(flat, base=base, out=enc, workspace=ws)
            plan.decode(enc, base=base, out=out)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        fb = plan.fallbacks(ws)
        ts = sorted(ts[5:])
        print(f"{name:24s} {1e3 * ts[len(ts) // 2]:8.3f} ms per encode+decode   fallbacks {fb}", flush=True)


if __name__ == "__main__":
    main()
