"""Benchmark: device-resident encode+decode throughput of the MI355X update codec.

Metric (BASELINE.json): "encode+decode GB/s over fp32 weight updates (device-resident), 1/2/4/8 GPU".
Workload: C3 per GPU — 16 synthetic ResNet-50 (torchvision-equivalent layout, 267 fp32 tensors,
25,610,152 elements) client updates per GPU, top-k ratio 0.01, 8-bit codes, batched into one launch
sequence. One step = encode all 16 + decode all 16. Weak scaling: every rank does its own 16 clients
(clients are independent; no collective on the data path — torch.distributed only for the barrier and
the max-over-ranks of the elapsed time).

value = 4 * N * clients_total * steps / elapsed (GB/s of fp32 update processed, whole job).
roofline: the dominant kernel's algorithmic bytes per launch / its mean HIP-event duration, vs 8 TB/s.
cpu_baseline: the numpy oracle (oracle/codec_oracle.py) on a bounded sample of the same workload,
rank 0, N = 1 only.

    python bench.py [--gpus N] [--steps K] [--warmup W]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "encode+decode GB/s over fp32 weight updates (device-resident), 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md: 8.0 TB/s)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--layout", default="resnet50_tv")
    p.add_argument("--clients", type=int, default=16, help="client updates per GPU")
    p.add_argument("--ratio", type=float, default=0.01)
    p.add_argument("--bits", type=int, default=8)
    p.add_argument("--mode", choices=["weights", "delta"], default="weights")
    p.add_argument("--streams", type=int, default=1,
                   help="split each GPU's clients into this many sub-batches, one HIP stream each")
    p.add_argument("--flags", type=int, default=0, help="coalac encode flags (test hooks; 0 for the bench)")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline time budget")
    p.add_argument("--no-cpu-baseline", action="store_true")
    return p.parse_args()


def make_events(torch, n):
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(n)]
    for e in evs:  # torch creates the HIP event lazily on first record
        e.record()
    return evs


def pmc_traffic(kernel, a):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary of the default workload
    (profiles/rNN_pmc_summary.json, written by tools/profile_round.sh + tools/pmc_summary.py): FETCH_SIZE
    doubled (gfx950 reports half the bytes of wide coalesced streaming reads, MI355X_MICROARCH.md §HBM)
    + WRITE_SIZE. Only reported for the default configuration the summary was collected on."""
    import glob
    default = (a.layout, a.clients, a.ratio, a.bits, a.mode, a.streams) == ("resnet50_tv", 16, 0.01, 8, "weights", 1)
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_summary.json")))
    if not default or not files:
        return None, None
    with open(files[-1]) as f:
        d = json.load(f)
    for name, e in sorted(d.items()):
        if name.split("<")[0] == kernel and "FETCH_SIZE_x2_bytes" in e and "WRITE_SIZE_bytes" in e:
            return e["FETCH_SIZE_x2_bytes"] + e["WRITE_SIZE_bytes"], os.path.relpath(files[-1], ROOT)
    return None, None


def cpu_baseline(layout, ratio, bits, budget_s):
    """Oracle encode+decode of whole synthetic clients on the host, until ~budget_s elapsed."""
    import numpy as np

    from coala_amd.compression import SegmentTable
    from coala_amd.layouts import fp32_sizes
    from oracle import codec_oracle as O

    sizes = fp32_sizes(layout)
    t = SegmentTable(sizes, ratio, 1)
    segs = t.segs.astype(np.int64)
    N = sum(sizes)
    done, el = 0, 0.0
    while el < budget_s and done < 64:
        rng = np.random.default_rng(1234 + done)
        flat = np.zeros(t.span, np.float32)
        for off, n in zip(t.offsets, sizes):
            flat[off:off + n] = rng.standard_normal(n, dtype=np.float32) * np.float32(10 ** rng.uniform(-4, -2))
        t0 = time.perf_counter()
        idx, vals, mn, sc = O.encode(flat, segs, bits)
        O.decode(idx, vals, mn, sc, segs, bits, t.span)
        el += time.perf_counter() - t0
        done += 1
    return {"value": round(4.0 * N * done / el / 1e9, 4), "unit": "GB/s", "cores": 1, "kind": "port",
            "sample": f"{done} x {layout} client update(s) ({N} fp32 elements each), numpy oracle "
                      f"encode+decode, single thread, {el:.1f} s"}


def main():
    a = parse()
    import torch
    import torch.distributed as dist

    from coala_amd.compression import CodecPlan
    from coala_amd.compression.spec import SMALL_MAX
    from coala_amd.layouts import fp32_sizes
    from coala_amd.workload import synth_batch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world} (launch N>1 with torch.distributed.run)")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    sizes = fp32_sizes(a.layout)
    if a.clients % a.streams:
        raise SystemExit("--clients must be a multiple of --streams")
    per = a.clients // a.streams
    lanes = []  # one independent sub-batch per stream: plan, buffers, stream, events
    for si in range(a.streams):
        plan = CodecPlan(sizes, a.ratio, a.bits, clients=per, device=dev)
        ids = range(rank * a.clients + si * per, rank * a.clients + (si + 1) * per)
        flat = synth_batch(plan.table, dev, client_ids=ids)
        base = synth_batch(plan.table, dev, client_ids=[10_000 + i for i in ids]) if a.mode == "delta" else None
        lanes.append(dict(plan=plan, flat=flat, base=base, enc=plan.empty_encoded(), ws=plan.empty_workspace(),
                          out=plan.empty_flat(), dws=plan.empty_decode_workspace(),
                          stream=torch.cuda.current_stream() if a.streams == 1 else torch.cuda.Stream(dev)))
    from coala_amd.compression import SegmentTable
    t = SegmentTable(sizes, a.ratio, a.clients)
    torch.cuda.synchronize()

    def step(i=None):
        main = torch.cuda.current_stream()
        for L in lanes:
            if a.streams > 1:
                L["stream"].wait_stream(main)
            with torch.cuda.stream(L["stream"]):
                ev_e = None if i is None else L["ev_e"][i]
                ev_d = None if i is None else L["ev_d"][i]
                L["plan"].encode(L["flat"], base=L["base"], out=L["enc"], workspace=L["ws"], events=ev_e,
                                 flags=a.flags)
                L["plan"].decode(L["enc"], base=L["base"], out=L["out"], workspace=L["dws"], events=ev_d)
        if a.streams > 1:
            for L in lanes:
                main.wait_stream(L["stream"])

    for _ in range(a.warmup):
        step()
    fallbacks = sum(L["plan"].fallbacks(L["ws"], stream=L["stream"]) for L in lanes)
    for L in lanes:
        with torch.cuda.stream(L["stream"]):
            L["ev_e"] = [make_events(torch, 5) for _ in range(a.steps)]
            L["ev_d"] = [make_events(torch, 3) for _ in range(a.steps)]
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        x = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(x, op=dist.ReduceOp.MAX)
        el = x.item()

    # per-kernel mean durations (ms) from the HIP events recorded on each launch stream; with several
    # streams, kernels overlap and each duration includes the co-running work of the other streams
    def mean(pairs):
        return sum(s.elapsed_time(e) for s, e in pairs) / len(pairs)
    stages = {}
    for name, (which, i0, i1) in {"k_sample": ("ev_e", 0, 1), "k_scan": ("ev_e", 1, 2), "k_select": ("ev_e", 2, 3),
                                  "k_emit": ("ev_e", 3, 4), "k_bounds": ("ev_d", 0, 1),
                                  "k_decode": ("ev_d", 1, 2)}.items():
        stages[name] = mean([(e[i0], e[i1]) for L in lanes for e in L[which]])
    N, K, T = t.n_elements, t.total_k, t.n_segments
    delta = a.mode == "delta"
    vb = 4 if a.bits == 32 else 1
    large_elems = per * sum(n for n in sizes if n > SMALL_MAX)
    Np, Kp, Tp = N // a.streams, K // a.streams, T // a.streams  # per launch (one sub-batch)
    alg = {  # algorithmic HBM bytes per launch
        "k_scan": 4 * large_elems * (2 if delta else 1),
        "k_decode": 4 * Np * (2 if delta else 1) + (4 + vb) * Kp + 8 * Tp,
    }
    dom = max(alg, key=lambda k: stages[k])
    ach = alg[dom] / (stages[dom] * 1e-3) / 1e9
    traffic, traffic_src = pmc_traffic(dom, a)
    step_ms = el / a.steps * 1e3
    step_alg = t.algorithmic_bytes(a.bits, delta)
    value = 4.0 * N * world * a.steps / el / 1e9

    if rank == 0:
        res = {
            "metric": METRIC, "value": round(value, 2), "unit": "GB/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(step_ms, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": f"C3-per-GPU: {a.clients} x {a.layout} fp32 updates per GPU, top-k "
                                   f"{a.ratio}, {a.bits}-bit codes, {a.mode} mode, encode+decode batched",
                       "layout": a.layout, "clients_per_gpu": a.clients, "global_clients": a.clients * world,
                       "elements_per_client": sum(sizes), "segments_per_client": len(sizes),
                       "ratio": a.ratio, "bits": a.bits, "mode": a.mode, "streams_per_gpu": a.streams,
                       "parallelism": f"replicas{world}"},
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "traffic_source": traffic_src, "alg_bytes_per_launch": alg[dom]},
            "step_roofline": {"alg_bytes_per_step": step_alg,
                              "achieved_GBs": round(step_alg / (step_ms * 1e-3) / 1e9, 1),
                              "frac": round(step_alg / (step_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
            "stages_ms": {k: round(v, 4) for k, v in stages.items()},
            "sample_fallbacks": fallbacks,
        }
        if world == 1 and not a.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(a.layout, a.ratio, a.bits, a.cpu_seconds)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
