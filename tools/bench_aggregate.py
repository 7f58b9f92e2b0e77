"""Throughput of the fused server-side decode + FedAvg (coalac_aggregate).

C client updates of one layout (default 16 x ResNet-50, ratio 0.01, 8-bit, delta mode) are aggregated
into w_global + FedAvg(decoded deltas) in one launch (k_aggregate, with the payloads' per-unit starts: wire
v2), and — the "v1" line — from payloads without them (the starts computed on the device first,
CodecPlan.unit_starts, then k_aggregate). Reported: GB/s of fp32 update
aggregated (4 * N * C / t), the kernel's algorithmic HBM bytes (base read 4N + output write 4N + C payloads of
idx/code (5K) + mn/scale (8T) + the per-unit starts (4U)) against 8 TB/s, and the time of the unfused
reference flow on the same data: C x coalac_decode into dense modules + the restated weighted_sum /
torch.div on the GPU (strategies.py:6-29, 57-90).

    python tools/bench_aggregate.py [--clients 16] [--layout resnet50_tv] [--steps 20]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--clients", type=int, default=16)
    p.add_argument("--layout", default="resnet50_tv")
    p.add_argument("--ratio", type=float, default=0.01)
    p.add_argument("--bits", type=int, default=8)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    a = p.parse_args()
    import torch

    from coala_amd.compression import CodecPlan, Encoded
    from coala_amd.layouts import fp32_sizes
    from coala_amd.workload import synth_batch

    dev = torch.device("cuda", 0)
    sizes = fp32_sizes(a.layout)
    C = a.clients
    plan = CodecPlan(sizes, a.ratio, a.bits, clients=C, device=dev)
    one = CodecPlan(sizes, a.ratio, a.bits, clients=1, device=dev)
    base = synth_batch(one.table, dev, client_ids=[999])
    flat = synth_batch(plan.table, dev, client_ids=range(C))
    base_rep = base.repeat(C)
    enc = plan.encode(flat, base=base_rep)
    weights = [10 + 3 * i for i in range(C)]
    out = torch.empty(plan.table.span_per_client, dtype=torch.float32, device=dev)
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(a.steps)]
    for e in evs:
        for x in e:
            x.record()
    t0 = torch.cuda.Event(enable_timing=True)
    t1 = torch.cuda.Event(enable_timing=True)

    def timed(e_in):
        for _ in range(a.warmup):
            plan.aggregate(e_in, weights, base=base, out=out)
        torch.cuda.synchronize()
        t0.record()
        for i in range(a.steps):
            plan.aggregate(e_in, weights, base=base, out=out, events=evs[i])
        t1.record()
        torch.cuda.synchronize()
        return (t0.elapsed_time(t1) / a.steps, sum(e[0].elapsed_time(e[1]) for e in evs) / a.steps,
                sum(e[1].elapsed_time(e[2]) for e in evs) / a.steps)
    ms1, k_bounds1, k_agg1 = timed(Encoded(enc.idx, enc.vals, enc.mn, enc.scale))  # v1 payloads
    out_v1 = out.clone()
    ms, _, k_agg = timed(enc)  # wire v2: the per-unit starts ride with the payloads
    t = plan.table
    N1 = sum(sizes)
    K, T = t.total_k, t.n_segments
    vb = 4 if a.bits == 32 else 1
    alg_agg = 8 * N1 + (4 + vb) * K + 8 * T + 4 * t.n_units

    # unfused reference flow: decode every client into a dense buffer, then weighted_sum + div (GPU)
    S = t.span_per_client
    dense = torch.empty(C * S, dtype=torch.float32, device=dev)

    def unfused():
        plan.decode(enc, base=base_rep, out=dense)
        acc = dense[0:S].clone()
        acc *= weights[0]
        for i in range(1, C):
            acc += dense[i * S:(i + 1) * S] * weights[i]
        return torch.div(acc, sum(weights))

    for _ in range(a.warmup):
        unfused()
    torch.cuda.synchronize()
    t0.record()
    for _ in range(a.steps):
        ref = unfused()
    t1.record()
    torch.cuda.synchronize()
    ms_ref = t0.elapsed_time(t1) / a.steps
    same = all(torch.equal(out[o:o + n], ref[o:o + n]) and torch.equal(out_v1[o:o + n], ref[o:o + n])
               for o, n in zip(t.offsets, t.sizes))
    print(json.dumps({
        "metric": "fused decode+FedAvg GB/s of fp32 client updates", "clients": C, "layout": a.layout,
        "ratio": a.ratio, "bits": a.bits, "mode": "delta", "ms": round(ms, 4),
        "value": round(4.0 * N1 * C / (ms * 1e-3) / 1e9, 1), "unit": "GB/s",
        "k_aggregate_ms": round(k_agg, 4),
        "roofline": {"kernel": "k_aggregate", "alg_bytes": alg_agg,
                     "achieved_GBs": round(alg_agg / (k_agg * 1e-3) / 1e9, 1),
                     "frac": round(alg_agg / (k_agg * 1e-3) / 1e9 / 8000.0, 4)},
        "v1_payloads": {"ms": round(ms1, 4), "k_aggregate_ms": round(k_agg1, 4),
                        "starts": "computed on the device (CodecPlan.unit_starts) before the kernel"},
        "unfused_reference_flow_ms": round(ms_ref, 4), "speedup_vs_unfused": round(ms_ref / ms, 2),
        "bit_identical_to_unfused": bool(same)}), flush=True)


if __name__ == "__main__":
    main()
