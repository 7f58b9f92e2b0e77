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
LANES = 1  # default pipeline lanes per GPU (2-3 lanes measured equal or slower: the latency-bound stages
           # of one lane slow the other lane's streaming kernel by as much as they overlap it)
SPLIT = 2  # sub-batches per step: two independent 8-client pipelines side by side fill the CUs the other
           # leaves idle in its latency-bound stages and launch tails (+11 % over one 16-client pipeline)
EVENT_EVERY = 4  # timing events on every 4th timed step (each recorded event adds a ~4 us dispatch gap)


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
    p.add_argument("--lanes", type=int, default=LANES,
                   help="pipeline lanes per GPU (coala_amd/compression/pipeline.py): the batch's segments "
                        "cut into this many contiguous ranges, one HIP stream each, streaming kernels "
                        "serialised across lanes")
    p.add_argument("--split", type=int, default=SPLIT,
                   help="the step's clients are cut into this many equal sub-batches, each an independent "
                        "pipeline (own plan, buffers, HIP stream) launched side by side")
    p.add_argument("--fork", action="store_true", help="keep the per-plan small-segment side streams with --split > 1")
    p.add_argument("--joined", action="store_true",
                   help="join the sub-batch streams with the caller's stream on entry/exit of every step")
    p.add_argument("--inflight", type=int, default=1,
                   help="independent pipelines (own plan, buffers and stream) taking the steps round-robin, so "
                        "consecutive batches overlap (each step still encodes + decodes its whole batch)")
    p.add_argument("--c-priority", type=int, default=-1, help="stream priority of the latency-stage streams")
    p.add_argument("--event-every", type=int, default=EVENT_EVERY,
                   help="record the per-kernel timing events on every Nth timed step (1 = every step)")
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
    default = (a.layout, a.clients, a.ratio, a.bits, a.mode, a.lanes, a.inflight, a.split) == \
        ("resnet50_tv", 16, 0.01, 8, "weights", LANES, 1, SPLIT)
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
    flats = []  # 4 distinct synthetic updates, cycled (generating one costs more than coding it)
    for c in range(4):
        rng = np.random.default_rng(1234 + c)
        flat = np.zeros(t.span, np.float32)
        for off, n in zip(t.offsets, sizes):
            flat[off:off + n] = rng.standard_normal(n, dtype=np.float32) * np.float32(10 ** rng.uniform(-4, -2))
        flats.append(flat)
    done, el = 0, 0.0
    while el < budget_s and done < 1000:
        flat = flats[done % len(flats)]
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

    from coala_amd.compression import LanePipeline, SegmentTable, SplitPipeline
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
    t = SegmentTable(sizes, a.ratio, a.clients)
    ids = range(rank * a.clients, (rank + 1) * a.clients)
    flat = synth_batch(t, dev, client_ids=ids)
    base = synth_batch(t, dev, client_ids=[10_000 + i for i in ids]) if a.mode == "delta" else None
    split = max(1, a.split)
    if a.lanes > 1 and split > 1:
        raise SystemExit("--lanes > 1 needs --split 1")
    # slots[j]: in-flight copy j of the step's pipeline with its own encoded / dense buffers
    slots = []
    for _ in range(max(1, a.inflight)):
        if a.lanes > 1:
            p = LanePipeline(t, a.bits, lanes=a.lanes, device=dev, flags=a.flags, c_priority=a.c_priority)
        else:
            p = SplitPipeline(t, a.bits, split=split, device=dev, flags=a.flags, fork=a.fork)
        slots.append((p, p.empty_encoded(), p.empty_flat()))
    pipes = [s[0] for s in slots]
    pipe = pipes[0]
    n_timed = pipe.n_lanes if a.lanes > 1 else 1  # timed intervals per streaming kernel and step
    torch.cuda.synchronize()

    def step(i=None, j=0):
        p, enc, out = slots[j % len(slots)]
        ee = ev_e[i] if i is not None else None
        de = ev_d[i] if i is not None else None
        if a.lanes > 1:
            # the pipeline's streaming stream as the current stream: back-to-back steps need no join hops
            with torch.cuda.stream(p.stream):
                p.roundtrip(flat, base=base, enc=enc, out=out, enc_events=ee, dec_events=de)
        else:
            # sub-batch streams ordered by themselves step after step (each slot's buffers are used by
            # its own streams only): no joins with the caller's stream inside the timed loop
            p.roundtrip(flat, base=base, enc=enc, out=out, enc_events=ee, dec_events=de, joined=a.joined)

    for w in range(max(a.warmup, len(slots))):
        step(j=w)
    fallbacks = sum(p.fallbacks() for p in pipes)
    # Timing events only at the streaming kernels' boundaries, and as few as possible: every recorded
    # event costs ~6 us of dispatch gap (rocprofv3 trace, profiles/). The streaming kernels run back to
    # back on one stream, so lane 0 records before and after its kernel and every later lane only
    # after; a lane's interval is [previous lane's end, its end]. The latency-bound stages are timed
    # by rocprofv3 (profiles/) instead.
    def lane_events(n):  # LanePipeline: per lane, [1] before lane 0's kernel, [2] after every lane's
        evs = []
        for li in range(pipe.n_lanes):
            ev = [None] * n
            ev[2] = make_events(torch, 1)[0]
            if li == 0:
                ev[1] = make_events(torch, 1)[0]
            evs.append(ev)
        return evs

    def part_events(n):  # SplitPipeline: per sub-batch, [1] / [2] around its kernel
        evs = []
        for _ in range(split):
            ev = [None] * n
            ev[1], ev[2] = make_events(torch, 2)
            evs.append(ev)
        return evs
    mk = lane_events if a.lanes > 1 else part_events
    every = max(1, a.event_every)
    timed_steps = [i for i in range(a.steps) if i % every == 0]
    ev_e = [mk(5) if i % every == 0 else None for i in range(a.steps)]
    ev_d = [mk(3) if i % every == 0 else None for i in range(a.steps)]
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        step(i, i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        x = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(x, op=dist.ReduceOp.MAX)
        el = x.item()

    # Per-kernel durations (ms, averaged over the event-carrying steps of the timed region, every
    # `--event-every`th one) from the HIP events recorded on each sub-batch's stream around its
    # streaming kernel. With --split S the S sub-batches' launches of a kernel run concurrently, so the
    # measured quantity is their union interval, first start to last end (events on different streams
    # of one device share a clock): the HBM phase the launch group occupies, against the bytes of all S
    # launches. With lanes (split 1) a lane's interval is [previous lane's end, its end] on the one
    # streaming stream; it can include co-running latency-bound kernels of other lanes.
    def union(pairs):
        ref = pairs[0][0]
        return max(ref.elapsed_time(e) for _, e in pairs) - min(ref.elapsed_time(s) for s, _ in pairs)
    stages = {}
    for name, which in {"k_scan": ev_e, "k_decode": ev_d}.items():
        per_step = []
        for i in timed_steps:
            evs = which[i]
            if a.lanes == 1:
                per_step.append(union([(e[1], e[2]) for e in evs]))
            else:
                per_step.extend((evs[li][1] if li == 0 else evs[li - 1][2]).elapsed_time(evs[li][2])
                                for li in range(pipe.n_lanes))
        stages[name] = sum(per_step) / len(per_step)
    N, K, T = t.n_elements, t.total_k, t.n_segments
    delta = a.mode == "delta"
    vb = 4 if a.bits == 32 else 1
    nl = n_timed  # timed intervals of each streaming kernel per step (a lane, or the split's union)
    segs = t.segs.astype("int64")
    large_elems = int(segs[segs[:, 1] > SMALL_MAX, 1].sum())
    alg = {  # algorithmic HBM bytes per timed interval
        "k_scan": 4 * large_elems * (2 if delta else 1) / nl,
        "k_decode": (4 * N * (2 if delta else 1) + (4 + vb) * K + 8 * T) / nl,
    }
    dom = max(alg, key=lambda k: stages[k])
    ach = alg[dom] / (stages[dom] * 1e-3) / 1e9
    traffic, traffic_src = pmc_traffic(dom, a)
    if traffic is not None:
        traffic *= split  # the summary is per dispatch; the timed interval holds `split` of them
    step_ms = el / a.steps * 1e3
    step_alg = t.algorithmic_bytes(a.bits, delta)
    value = 4.0 * N * world * a.steps / el / 1e9

    if rank == 0:
        res = {
            "metric": METRIC, "value": round(value, 2), "unit": "GB/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(step_ms, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": f"C3-per-GPU: {a.clients} x {a.layout} fp32 updates per GPU, top-k "
                                   f"{a.ratio}, {a.bits}-bit codes, {a.mode} mode, encode+decode batched "
                                   f"as {split} concurrent sub-batches",
                       "layout": a.layout, "clients_per_gpu": a.clients, "global_clients": a.clients * world,
                       "elements_per_client": sum(sizes), "segments_per_client": len(sizes),
                       "ratio": a.ratio, "bits": a.bits, "mode": a.mode, "lanes_per_gpu": pipe.n_lanes if a.lanes > 1 else 1,
                       "sub_batches_per_step": split, "inflight_steps": len(slots),
                       "parallelism": f"replicas{world}"},
            "roofline": {"bound": "hbm", "kernel": dom if split == 1 else f"{dom} x{split} concurrent launches (union interval)", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "traffic_source": traffic_src, "alg_bytes_per_launch": int(alg[dom])},
            "step_roofline": {"alg_bytes_per_step": step_alg,
                              "achieved_GBs": round(step_alg / (step_ms * 1e-3) / 1e9, 1),
                              "frac": round(step_alg / (step_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
            "stages_ms": {k: round(v, 4) for k, v in stages.items()},
            "stage_timing": f"HIP events on each sub-batch stream around k_scan / k_decode (union over the "
                            f"{split} sub-batches), {len(timed_steps)} of the {a.steps} timed steps",
            "sample_fallbacks": fallbacks,
        }
        if world == 1 and not a.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(a.layout, a.ratio, a.bits, a.cpu_seconds)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
