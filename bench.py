"""Benchmark: device-resident encode+decode throughput of the MI355X update codec.

Metric (BASELINE.json): "encode+decode GB/s over fp32 weight updates (device-resident), 1/2/4/8 GPU".
Headline workload (`value`): C3 per GPU — 16 synthetic ResNet-50 (torchvision-equivalent layout, 267 fp32
tensors, 25,610,152 elements) client updates per GPU, top-k ratio 0.01, 8-bit codes, batched. One step =
encode all 16 + decode all 16. Weak scaling: every rank does its own share (clients are independent; no
collective on the data path — torch.distributed only for the barrier and the max-over-ranks of the time).

`configs` extras, each timed the same way on the same GPU:
  C2      16 x ResNet-18 (CIFAR-10, 11,183,562 elements) per GPU
  C4      16 x ViT-B/16 (86,567,656 elements) per GPU (C4 is 128 clients on 8 GPUs)
  C5      one GPU's share of the heterogeneous splitFL round (256 clients, greedy-grouped over 8 GPUs:
          client-side models at cut 1/2/4 + feature tensors up to 8,388,608 elements), MixedTable
  single  ONE ResNet-50 update per step, steps serialised (north_star's "a 25.6 M-param fp32 update at
          1 GPU"; latency-bound)
  single_x2  ONE ResNet-50 update per step, two steps in flight on two streams (a server decoding
          concurrent uploads, one thread each: coala/server/service.py:71-111)
  single_x4  the same with four steps in flight (the reference's gRPC server runs up to 10 worker threads,
          coala/communication/grpc_wrapper.py:51)
  plugin  the hooks' own path per ResNet-50 client, delta mode: client compression() encoding the trained
          module's parameters in place + server decompression(model) into a new module on w_global
  C3_delta   the C3 share in delta mode (what the plugin runs by default: w_local - w_global on encode, + w_global
          fused into the decode; +8N bytes per client, SURVEY.md §8(d) "report these variants separately")
  C3_r0.001 / C3_r0.1  the C3 share at the other BASELINE.md top-k ratios
  C4_delta   the C4 share in delta mode
  C4_frozen  the C4 share in delta mode with the backbone frozen as FedPEFT does (application/FedPEFT/lora.py:64,
          main.py:62-67): every tensor but the classifier head is an exact-zero delta
  C3_signs   the C3 share in delta mode after one sign-like local step (signSGD, the first Adam step): trained =
          fl(w_global -+ lr), so every |delta| is lr up to the rounding of the subtraction — heavy near-ties at
          the k-th key (the tie mode of DESIGN.md §6e; the raw-data path's territory before it)
  download   the download direction: one ResNet-50 global model per step, dense 8-bit codes at
          ratio 1 (indices implied) — the server's compression() (coala/server/base.py:196) + one client's
          decode of it (coala/client/base.py:197-201); HBM bytes 10N + 32T
value = 4 * N * clients * steps / elapsed (GB/s of fp32 update processed, whole job).
roofline: the dominant kernel's algorithmic bytes per launch / its mean HIP-event duration, vs 8 TB/s.
cpu_baseline: the numpy oracle (oracle/codec_oracle.py) on a bounded sample of the same workload, on the
host's cores (a process pool, timed before the GPU is touched), plus its single-thread rate and the
reference's current boundary (identity pickle of the state, coala/protocol/codec.py:4-9); rank 0, N = 1.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C3] [--extras C2,C4,C5,single|none]
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
SPLIT = 2  # sub-batches per step: two independent pipelines side by side fill the CUs the other leaves
           # idle in its latency-bound stages and launch tails (+11 % over one 16-client pipeline)
ROOF_STEPS = 8  # joined steps after the timed region that carry the per-kernel timing events
CONFIGS = {  # name -> (layout | "c5", clients per GPU, sub-batches: the best of 1..4 on the box, DESIGN.md §7,
             #          options: ratio / mode / frozen override the command line's for that config)
    "C2": ("resnet18", 16, 3, {}),
    "C3": ("resnet50_tv", 16, SPLIT, {}),
    "C3_delta": ("resnet50_tv", 16, SPLIT, {"mode": "delta"}),
    "C3_r0.001": ("resnet50_tv", 16, SPLIT, {"ratio": 0.001}),
    "C3_r0.1": ("resnet50_tv", 16, SPLIT, {"ratio": 0.1}),
    "C4": ("vit_b16", 16, SPLIT, {}),
    "C4_delta": ("vit_b16", 16, SPLIT, {"mode": "delta"}),
    "C4_frozen": ("vit_b16", 16, SPLIT, {"mode": "delta", "frozen": True}),
    "C3_signs": ("resnet50_tv", 16, SPLIT, {"mode": "delta", "signs": True}),
    "C5": ("c5", None, 1, {}),  # one latency-bound plan (<= 8192 units): 0.116 ms vs 0.122 as 2 sub-batches
    "single": ("resnet50_tv", 1, "single", {}),
    "single_x2": ("resnet50_tv", 1, "single", {}),
    "single_x4": ("resnet50_tv", 1, "single", {}),
    "download": ("resnet50_tv", 1, "single", {"ratio": 1.0}),
}
# updates in flight per extra config: single_x2 = one update per step, consecutive steps on two streams (a
# server decodes concurrent uploads from one thread each, coala/server/service.py:71-111)
CONFIG_INFLIGHT = {"single_x2": 2, "single_x4": 4}
SINGLE_SPLIT = 1  # segment ranges of the single update run as this many concurrent sub-plans
DEFAULT_EXTRAS = "C2,C3_delta,C3_r0.001,C3_r0.1,C3_signs,C4,C4_delta,C4_frozen,C5,single,single_x2,single_x4,download,plugin"


def cfg_opts(cfg, a):
    """(ratio, mode, frozen) of a config: its own overrides, else the command line's."""
    o = CONFIGS[cfg][3]
    return o.get("ratio", a.ratio), o.get("mode", a.mode), bool(o.get("frozen", False))


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--config", default="C3", choices=sorted(CONFIGS), help="headline workload")
    p.add_argument("--extras", default=DEFAULT_EXTRAS, help="comma-separated extra configs, or 'none'")
    p.add_argument("--layout", default=None, help="override the headline layout (uniform configs)")
    p.add_argument("--clients", type=int, default=None, help="override client updates per GPU")
    p.add_argument("--ratio", type=float, default=0.01)
    p.add_argument("--bits", type=int, default=8)
    p.add_argument("--mode", choices=["weights", "delta"], default="weights")
    p.add_argument("--split", type=int, default=None,
                   help="the step's clients are cut into this many sub-batches (balanced by elements), each an "
                        "independent pipeline (own plan, buffers, HIP stream) launched side by side")
    p.add_argument("--fork", action="store_true", help="keep the per-plan small-segment side streams with --split > 1")
    p.add_argument("--joined", action="store_true",
                   help="join the sub-batch streams with the caller's stream on entry/exit of every step")
    p.add_argument("--inflight", type=int, default=1,
                   help="independent pipelines (own plan, buffers and stream) taking the steps round-robin, so "
                        "consecutive batches overlap (each step still encodes + decodes its whole batch)")
    p.add_argument("--roof-steps", type=int, default=ROOF_STEPS,
                   help="extra steps after the timed region, joined per step and carrying per-kernel HIP events, "
                        "that measure the streaming kernels' launch durations for the roofline")
    p.add_argument("--flags", type=int, default=0, help="coalac encode flags (test hooks; 0 for the bench)")
    p.add_argument("--extras-split", type=int, default=None, help="override the sub-batch count of the extras")
    p.add_argument("--single-split", type=int, default=SINGLE_SPLIT,
                   help="config 'single': the update's segments cut into this many ranges, each a sub-plan on its "
                        "own stream (their latency-bound phases overlap)")
    p.add_argument("--graph", choices=["auto", "on", "off"], default="auto",
                   help="replay each timed step as a captured hipGraph: auto = the latency-bound configs "
                        f"({', '.join(GRAPH_CONFIGS) if 'GRAPH_CONFIGS' in globals() else 'single, single_x2, C5'})")
    p.add_argument("--graph-steps", type=int, default=30,
                   help="at most this many timed steps captured in one graph (--graph; whole input rotations, the "
                        "count that needs the fewest launches): 1 / 4 / 10 steps per launch measured 0.0845 / 0.0803 / "
                        "0.0796 ms per single step (eager 0.080-0.083)")
    p.add_argument("--repeat-windows", type=int, default=5,
                   help="after the timed region, time the same K steps again this many times and report the min / "
                        "median / max ms per step beside the line (not part of value)")
    p.add_argument("--cpu-seconds", type=float, default=8.0, help="CPU baseline time budget per leg")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--launch-check", action="store_true",
                   help="test hook (CPU, no GPU): every rank joins a gloo group from the launcher's environment and "
                        "rank 0 prints the ranks' (RANK, LOCAL_RANK, WORLD_SIZE); tests/test_bench_launch.py")
    p.add_argument("--launch-check-fail", type=int, default=-1,
                   help="with --launch-check: this rank exits with code 3 before joining (the others block in the "
                        "rendezvous until the launcher stops them)")
    return p.parse_args()


# ----------------------------------------------------------------------------------------------------
# CPU baseline (rank 0, N = 1, BEFORE the GPU is initialised: the pool's workers are spawned children)
# ----------------------------------------------------------------------------------------------------
def _synth_np(sizes, offsets, span, seed):
    import numpy as np
    rng = np.random.default_rng(seed)
    flat = np.zeros(span, np.float32)
    for off, n in zip(offsets, sizes):
        flat[off:off + n] = rng.standard_normal(n, dtype=np.float32) * np.float32(10 ** rng.uniform(-4, -2))
    return flat


def _warm(_):
    from oracle import codec_oracle  # noqa: F401
    return os.getpid()


def _oracle_worker(args):
    """One pool worker: encode+decode whole synthetic clients with the oracle until `budget` seconds."""
    layout, ratio, bits, budget, seed = args
    from coala_amd.compression.spec import SegmentTable
    from coala_amd.layouts import fp32_sizes
    from oracle import codec_oracle as O
    sizes = fp32_sizes(layout)
    t = SegmentTable(sizes, ratio, 1)
    segs = t.segs.astype("int64")
    flats = [_synth_np(sizes, t.offsets, t.span, seed + j) for j in range(2)]
    done, el = 0, 0.0
    while el < budget and done < 1000:
        t0 = time.perf_counter()
        idx, vals, mn, sc = O.encode(flats[done % 2], segs, bits)
        O.decode(idx, vals, mn, sc, segs, bits, t.span)
        el += time.perf_counter() - t0
        done += 1
    return done, el


def host_cores():
    """(affinity cores, pool size). The pool is capped at the job's CPU share: OMP_NUM_THREADS, which the GPU
    box sets to 16 for a one-GPU job (its affinity mask shows the whole host, 256 cores); 16 without it."""
    aff = len(os.sched_getaffinity(0))
    cap = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or 16
    return aff, max(1, min(aff, cap))


def cpu_baseline(layout, ratio, bits, budget_s):
    import multiprocessing as mp
    import pickle

    import torch

    from coala_amd.layouts import build_module, fp32_sizes
    N = sum(fp32_sizes(layout))
    aff, W = host_cores()
    # single thread: one client stream in this process
    done1, el1 = _oracle_worker((layout, ratio, bits, budget_s, 1234))
    # W processes, each its own client stream (clients are independent)
    with mp.get_context("spawn").Pool(W) as pool:
        pool.map(_warm, range(W))  # spawn + import warm-up, not timed
        t0 = time.perf_counter()
        res = pool.map(_oracle_worker, [(layout, ratio, bits, budget_s, 5000 + 10 * w) for w in range(W)])
        wall = time.perf_counter() - t0
    doneW = sum(d for d, _ in res)
    # the reference's current boundary: codec.marshal(copy.deepcopy(model)) then codec.unmarshal
    # (coala/client/base.py:363, coala/protocol/codec.py:4-9) of a module with this layout, on the host
    import copy
    m = build_module(layout, seed=0)
    n_p, el_p = 0, 0.0
    while el_p < min(budget_s, 4.0) and n_p < 100:
        t0 = time.perf_counter()
        pickle.loads(pickle.dumps(copy.deepcopy(m)))
        el_p += time.perf_counter() - t0
        n_p += 1
    state_bytes = sum(t.numel() * t.element_size() for t in m.state_dict().values())
    return {"value": round(4.0 * N * doneW / wall / 1e9, 4), "unit": "GB/s", "cores": W, "kind": "port",
            "sample": f"{doneW} x {layout} client updates ({N} fp32 elements each) in {wall:.1f} s: numpy oracle "
                      f"encode+decode, {W} worker processes (one client stream each)",
            "host_cores_affinity": aff, "torch_threads": torch.get_num_threads(),
            "cores_note": f"pool capped at this job's CPU share (OMP_NUM_THREADS={os.environ.get('OMP_NUM_THREADS')}; "
                          f"{aff} cores in the affinity mask, which on the GPU box is the whole 8-GPU host)",
            "single_thread": {"value": round(4.0 * N * done1 / el1 / 1e9, 4), "unit": "GB/s", "cores": 1,
                              "sample": f"{done1} updates, {el1:.1f} s, one thread"},
            "reference_identity_pickle": {
                "value": round(state_bytes * n_p / el_p / 1e9, 4), "unit": "GB/s", "cores": 1,
                "sample": f"{n_p} x pickle.loads(pickle.dumps(copy.deepcopy(module))) of the {layout} state "
                          f"({state_bytes} B), {el_p:.1f} s — what coala/protocol/codec.py:4-9 does today"}}


# ----------------------------------------------------------------------------------------------------
# GPU workloads
# ----------------------------------------------------------------------------------------------------
def pmc_traffic(kernel, cfg, a, split, world=1):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary of the default workload
    (profiles/rNN_pmc_summary.json, written by tools/profile_round.sh + tools/pmc_summary.py): FETCH_SIZE
    doubled (gfx950 reports half the bytes of wide coalesced streaming reads, MI355X_MICROARCH.md §HBM)
    + WRITE_SIZE. Only reported for the configuration the summary was collected on: the default workload on
    ONE GPU (a multi-rank line gets null — its ranks were never profiled)."""
    import glob
    default = world == 1 and (cfg, a.layout, a.clients, a.ratio, a.bits, a.mode, a.inflight, split) == \
        ("C3", None, None, 0.01, 8, "weights", 1, SPLIT)
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_summary.json")))
    if not default or not files:
        return None, None
    names = {"k_decode": ("k_decode_lds", "k_decode")}.get(kernel, (kernel,))  # (the batch decode kernel)
    for path in reversed(files):  # the newest summary that holds the kernel
        with open(path) as f:
            d = json.load(f)
        for want in names:
            for name, e in sorted(d.items()):
                if name.split("<")[0] == want and "FETCH_SIZE_x2_bytes" in e and "WRITE_SIZE_bytes" in e:
                    return e["FETCH_SIZE_x2_bytes"] + e["WRITE_SIZE_bytes"], os.path.relpath(path, ROOT)
    return None, None


def large_elements(pipe):
    """Elements of the segments the pipeline's plans stream through k_scan (the others are encoded whole
    in k_presel; each plan's threshold follows its size, spec.small_limit)."""
    from coala_amd.compression.spec import small_limit
    tot = 0
    for q in pipe.parts:
        n = q["plan"].table.segs[:, 1].astype("int64")
        tot += int(n[n > small_limit(n)].sum())
    return tot


def make_events(torch, n):
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(n)]
    for e in evs:  # torch creates the HIP event lazily on first record
        e.record()
    return evs


def build_table(cfg, a, rank, headline):
    from coala_amd.compression import SegmentTable
    from coala_amd.layouts import fp32_sizes
    from coala_amd.workload import c5_share, mixed_table
    layout, clients, split, _ = CONFIGS[cfg]
    ratio = cfg_opts(cfg, a)[0]
    if split == "single":
        split = a.single_split
    elif not headline and a.extras_split is not None:
        split = a.extras_split
    if headline:
        layout = a.layout or layout
        clients = a.clients or clients
        split = a.split if a.split is not None else split
    if layout == "c5":
        ids, names = c5_share(rank)
        return mixed_table(names, ratio), ids, split, {"layouts": sorted(set(names)), "clients_per_gpu": len(ids),
                                                         "global_clients": 256, "grouping": "greedy LPT over 8 GPUs"}
    t = SegmentTable(fp32_sizes(layout), ratio, clients)
    ids = list(range(rank * clients, (rank + 1) * clients))
    _, mode, frozen = cfg_opts(cfg, a)
    return t, ids, split, {"layout": layout, "clients_per_gpu": clients, "elements_per_client": sum(t.sizes),
                           "segments_per_client": len(t.sizes), "ratio": ratio, "mode": mode,
                           **({"frozen": "every tensor but the classifier head an exact-zero delta"} if frozen else {}),
                           **({"signs": "trained = fl(w_global -+ 1e-3): every |delta| 1e-3 up to rounding"}
                              if CONFIGS[cfg][3].get("signs") else {})}


GRAPH_CONFIGS = ("single", "single_x2", "single_x4", "C5", "download")  # latency-bound plans: step time ~ host launch time
GRAPH_WARM_REPLAYS = 8  # untimed replays of each slot's whole-rotation graph right before the timed region


def use_graph(cfg, a):
    return a.graph == "on" or (a.graph == "auto" and cfg in GRAPH_CONFIGS)


# configs whose timed steps rotate over ROTATE distinct input / output buffer sets (one ResNet-50 update is
# 102 MB in + 102 MB out: a single set would stay resident in the 256 MB Infinity Cache, step after step)
ROTATE_CONFIGS = ("single", "single_x2", "single_x4", "download")
ROTATE = 3


def setup_workload(cfg, a, dev, rank, headline):
    """Buffers, pipelines and synthetic inputs of one config (nothing timed)."""
    import torch

    from coala_amd.compression import SplitPipeline
    from coala_amd.workload import freeze_segments, head_only, sign_step, synth_batch

    t, ids, split, desc = build_table(cfg, a, rank, headline)
    _, mode, frozen = cfg_opts(cfg, a)
    rot = ROTATE if cfg in ROTATE_CONFIGS else 1
    flats = [synth_batch(t, dev, client_ids=[1000 * r + i for i in ids]) for r in range(rot)]
    base = synth_batch(t, dev, client_ids=[10_000 + i for i in ids]) if mode == "delta" else None
    if frozen:  # trained = w_global + delta with the frozen tensors' deltas exactly zero
        for f in flats:
            freeze_segments(f, t, head_only(desc["layout"]))
            f.add_(base)
    if CONFIGS[cfg][3].get("signs"):  # trained = fl(w_global -+ lr): one sign-like step, lr = 1e-3
        for r, f in enumerate(flats):
            sign_step(f, base, 4242 + 17 * rank + r)
    split = max(1, split)
    inflight = max(1, a.inflight) if headline else CONFIG_INFLIGHT.get(cfg, 1)
    slots = []
    for j in range(inflight):  # slot j on its own pooled streams, so the slots' steps overlap
        p = SplitPipeline(t, a.bits, split=split, device=dev, flags=a.flags, fork=a.fork, stream_base=j * split)
        slots.append((p, [(p.empty_encoded(), p.empty_flat()) for _ in range(rot)]))
    torch.cuda.synchronize()
    return {"cfg": cfg, "headline": headline, "table": t, "desc": desc, "flats": flats, "base": base, "rot": rot,
            "mode": mode, "slots": slots, "split": slots[0][0].n_parts, "graphs": None, "graph_error": None}


def _step(W, i, joined, enc_events=None, dec_events=None):
    """Step i: slot i % inflight, buffer set (i // inflight) % rot. (Steps carrying timing events take the
    plain roundtrip: its kernel boundaries are the ones the events bracket.)"""
    p, bufs = W["slots"][i % len(W["slots"])]
    r = (i // len(W["slots"])) % W["rot"]
    enc, out = bufs[r]
    p.roundtrip(W["flats"][r], base=W["base"], enc=enc, out=out, enc_events=enc_events, dec_events=dec_events,
                joined=joined)


EXTRA_WARMUP = 20  # untimed steps before an extra config's timed region (the headline takes --warmup as given)


def warm_workload(W, a):
    import torch
    n = a.warmup if W["headline"] else max(a.warmup, EXTRA_WARMUP)
    for w in range(max(n, len(W["slots"]) * W["rot"])):
        _step(W, w, a.joined)
    torch.cuda.synchronize()
    W["fallbacks"] = sum(p.fallbacks() for p, _ in W["slots"])


def _graph_plan(W, a):
    """Per slot: how its share of the timed steps is replayed — whole-rotation graphs of gk steps, then single
    steps — with gk the multiple of the rotation (<= --graph-steps) that needs the fewest graph launches."""
    S, rot = len(W["slots"]), W["rot"]
    per = [a.steps // S + (1 if j < a.steps % S else 0) for j in range(S)]
    n = max(1, min(per))
    cands = [m * rot for m in range(1, max(1, a.graph_steps // rot) + 1)] or [rot]
    gk = min(cands, key=lambda g: (max(p // g + p % g for p in per), -g)) if n >= rot else rot
    return gk, per


def capture_graphs(W, a):
    """Latency-bound configs: each slot's steps captured as hipGraphs and replayed on the slot's first stream
    (the same kernels on the same buffers: one graph launch per gk steps instead of the per-call Python checks,
    ctypes calls and ~8 kernel launches per step, which take about as long as the ~80 us of GPU work of one
    update — a box with a slower host measured the eager single step at 0.138 ms for 0.080 ms of kernels).
    A one-part pipeline is captured on its own stream, unjoined (each join would add graph nodes: ~3.5 us per
    step); a pipeline of several sub-batches is captured on a stream of its own with the JOINED roundtrip, so
    every sub-batch stream forks from the capture and joins back into it (all parts land in the graph).
    Runs before any process group exists (no other thread makes HIP calls during the capture)."""
    import torch
    S = len(W["slots"])
    gk, per = _graph_plan(W, a)
    W["gk"], W["per_slot"] = gk, per

    def capture(steps_of_slot):  # buffer-set index per captured step
        gs = []
        for j, (p, _) in enumerate(W["slots"]):
            joined = p.n_parts > 1
            cap = torch.cuda.Stream(p.device) if joined else p.streams[0]
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=cap, capture_error_mode="thread_local"):
                for r in steps_of_slot:
                    _step(W, r * S + j, joined)
            gs.append((g, p.streams[0]))
        return gs
    try:
        torch.cuda.synchronize()
        W["graphs"] = {gk: capture(list(range(gk)))}
        for r in range(W["rot"]):  # single steps for the remainder, one per buffer set
            W["graphs"][(1, r)] = capture([r])
        torch.cuda.synchronize()
        for gs in W["graphs"].values():  # every captured graph once (a graph's first launch uploads it)
            for g, st in gs:
                with torch.cuda.stream(st):
                    g.replay()
        torch.cuda.synchronize()
    except RuntimeError as e:  # a runtime that cannot capture: time the eager steps instead (reported)
        W["graph_error"] = f"capture failed, eager steps: {e}"[:200]
        W["graphs"] = None
        torch.cuda.synchronize()


def time_workload(W, a, dev, world):
    import torch
    import torch.distributed as dist

    slots = W["slots"]
    pipes = [p for p, _ in slots]
    split, t, headline = W["split"], W["table"], W["headline"]
    graphs = W["graphs"]
    # The timed region carries no timing event (each recorded event costs a dispatch gap) and its sub-batch
    # streams are not joined per step, so consecutive steps overlap.
    def timed_region():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if graphs is None:
            for i in range(a.steps):
                _step(W, i, a.joined)
        else:  # per slot: its whole-rotation graphs, then its single steps; slots round-robin
            gk = W["gk"]
            ops = []
            for j, n in enumerate(W["per_slot"]):
                big = n // gk
                ops.append([graphs[gk][j]] * big + [graphs[(1, r % W["rot"])][j] for r in range(n - big * gk)])
            for q in range(max(len(o) for o in ops)):
                for o in ops:
                    if q < len(o):
                        g, st = o[q]
                        with torch.cuda.stream(st):
                            g.replay()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        return time.perf_counter() - t0
    if graphs is not None:
        # the graphs were captured (and replayed once) before the other configs ran: replay them again right before
        # the timed region, so their buffers are warm again (without this the first window measured a constant
        # ~0.05-0.1 ms above the repeat windows: C5 0.0911 vs 0.0866 ms per step, download 0.0791 vs 0.0735)
        for _ in range(GRAPH_WARM_REPLAYS):
            for g, st in graphs[W["gk"]]:
                with torch.cuda.stream(st):
                    g.replay()
        torch.cuda.synchronize()
    el = timed_region()
    rank_el = gather_elapsed(el, world, dev)
    el = max(rank_el)  # the job's time: the slowest rank
    # the same K steps timed again in a few more windows (not part of `value`): the spread a single short window
    # cannot show (box-to-box and run-to-run variance)
    rep_ms = sorted(timed_region() / a.steps * 1e3 for _ in range(a.repeat_windows))

    # Roofline steps (after the timed region, not part of `value`): per sub-batch, HIP events [1] / [2]
    # recorded on its own stream around its streaming kernels, each step joined with the caller's stream
    # so the sub-batches' launches of a kernel start together (unjoined, the streams drift apart and a
    # launch group's interval would hold other kernels).
    def part_events(n):
        evs = []
        for _ in range(split):
            ev = [None] * n
            ev[1], ev[2] = make_events(torch, 2)
            evs.append(ev)
        return evs
    timed_steps = list(range(max(1, a.roof_steps)))
    ev_e = [part_events(5) for _ in timed_steps]
    ev_d = [part_events(3) for _ in timed_steps]
    torch.cuda.synchronize()
    for i in timed_steps:
        _step(W, i, True, ev_e[i], ev_d[i])
    torch.cuda.synchronize()

    # Per-kernel durations (ms, averaged over the event-carrying steps) from HIP events on each
    # sub-batch's stream around its streaming kernel. With S sub-batches the S launches of a kernel run
    # concurrently, so the measured quantity is their union interval, first start to last end (events on
    # different streams of one device share a clock): the HBM phase the launch group occupies, against
    # the bytes of all S launches.
    def union(pairs):
        ref = pairs[0][0]
        return max(ref.elapsed_time(e) for _, e in pairs) - min(ref.elapsed_time(s) for s, _ in pairs)
    stages = {}
    for name, which in {"k_scan": ev_e, "k_decode": ev_d}.items():
        per = [union([(e[1], e[2]) for e in which[i]]) for i in timed_steps]
        stages[name] = sum(per) / len(per)
    N, K, T = t.n_elements, t.total_k, t.n_segments
    delta = W["mode"] == "delta"
    vb = 4 if a.bits == 32 else 1
    large_elems = large_elements(pipes[0])
    alg = {  # algorithmic HBM bytes per timed interval
        "k_scan": 4 * large_elems + (4 * N if delta else 0),
        "k_decode": 4 * N * (2 if delta else 1) + (4 + vb) * K + 8 * T,
    }
    dense = t.ratio >= 1.0
    if dense:  # the dense codec: k_dense_quant (read 4 B, write the code) / k_dense_deq (read the code, write 4 B)
        alg = {"k_scan": 4 * N * (2 if delta else 1) + vb * N, "k_decode": 4 * N * (2 if delta else 1) + vb * N + 8 * T}
    dom = max(alg, key=lambda k: stages[k])
    ach = alg[dom] / (stages[dom] * 1e-3) / 1e9
    step_ms = el / a.steps * 1e3
    step_alg = t.algorithmic_bytes(a.bits, delta)
    kname = {"k_scan": "k_dense_quant", "k_decode": "k_dense_deq"}[dom] if dense else dom
    res = {
        "value": round(4.0 * N * world * a.steps / el / 1e9, 2), "ms_per_step": round(step_ms, 4),
        "desc": W["desc"], "split": split, "inflight": len(slots), "rotation": W["rot"],
        "elements_per_gpu": N, "segments_per_gpu": T, "kept_per_gpu": K,
        "roofline": {"bound": "hbm", "kernel": kname if split == 1 else f"{kname} x{split} concurrent launches (union interval)",
                     "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                     "alg_bytes_per_launch": int(alg[dom])},
        "step_roofline": {"alg_bytes_per_step": step_alg, "achieved_GBs": round(step_alg / (step_ms * 1e-3) / 1e9, 1),
                          "frac": round(step_alg / (step_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
        "stages_ms": {({"k_scan": "k_dense_quant", "k_decode": "k_dense_deq"}[k] if dense else k): round(v, 4)
                      for k, v in stages.items()},
        "sample_fallbacks": W.get("fallbacks", 0),
        "graph": W["graph_error"] or (graphs is not None and f"{W['gk']} step(s) per graph launch"),
        "rank_ms_per_step": rank_spread(rank_el, a.steps),
        "repeat_windows": ({"windows": len(rep_ms), "steps_each": a.steps, "ms_per_step_min": round(rep_ms[0], 4),
                            "ms_per_step_median": round(rep_ms[len(rep_ms) // 2], 4),
                            "ms_per_step_max": round(rep_ms[-1], 4)} if rep_ms else None),
    }
    if headline:
        traffic, src = pmc_traffic(dom, W["cfg"], a, split, world)
        res["roofline"]["traffic"] = traffic * split if traffic is not None else None
        res["roofline"]["traffic_source"] = src
        res["stage_timing"] = (f"HIP events on each sub-batch stream around k_scan / k_decode, union over the "
                               f"{split} concurrent launches, mean of {len(timed_steps)} joined steps run after the "
                               f"timed region")
    return res


def gather_elapsed(el, world, device):
    """Every rank's elapsed seconds of the timed region, in rank order, on every rank (one all_gather; RCCL
    needs device tensors, gloo host ones). world == 1: [el]."""
    if world == 1:
        return [el]
    import torch
    import torch.distributed as dist
    if dist.get_backend() != "nccl":
        device = "cpu"
    x = torch.tensor([el], dtype=torch.float64, device=device)
    out = [torch.zeros_like(x) for _ in range(world)]
    dist.all_gather(out, x)
    return [float(t.item()) for t in out]


def rank_spread(rank_el, steps):
    """Per-rank ms per step of a multi-rank run (load imbalance shows as max / min > 1); None for one rank."""
    if len(rank_el) == 1:
        return None
    ms = [e / steps * 1e3 for e in rank_el]
    return {"min": round(min(ms), 4), "max": round(max(ms), 4), "per_rank": [round(m, 4) for m in ms]}


def box_probe(torch, dev):
    """This box's device-to-device copy rate (read + write bytes / time, torch's copy kernel on 1 GiB): a
    per-box yardstick beside the headline, since MI355X boxes of this pool differ by a few percent in
    streaming bandwidth (the headline's box-to-box spread tracks it). Taken after every timed region."""
    n = 1 << 28
    src = torch.empty(n, dtype=torch.float32, device=dev).fill_(1.0)
    dst = torch.empty_like(src)
    for _ in range(3):
        dst.copy_(src)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 20
    torch.cuda.synchronize(dev)
    e0.record()
    for _ in range(reps):
        dst.copy_(src)
    e1.record()
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / reps
    del src, dst
    return {"copy_GBps": round(2 * 4 * n / (ms * 1e-3) / 1e9, 1), "gpu": torch.cuda.get_device_name(dev)}


def release_workload(W):
    import torch
    for p, _ in W["slots"]:
        p.close()
    W.clear()
    torch.cuda.empty_cache()


def run_plugin(a, dev, steps):
    """Client compression() + server decompression(model) of one ResNet-50 client through the codec
    (UpdateCodec, as the mixins call it), on device-resident modules, delta mode. HBM bytes per client:
    encode reads the parameters and the w_global snapshot (8N) and writes 5K + 8T; decode reads those and
    the snapshot (4N) and writes the new module (4N): 16N + 10K + 16T."""
    import torch

    from coala_amd.compression import UpdateCodec
    from coala_amd.compression.codec import flatten_state
    from coala_amd.layouts import build_module
    m = build_module("resnet50_tv", seed=1, device=dev)
    g = build_module("resnet50_tv", seed=2, device=dev)
    codec = UpdateCodec(a.ratio, a.bits, "delta")
    base = codec.snapshot(g)
    state = m.state_dict()
    res = {}

    def per_call(fn, n):
        """Median and mean of n calls, each synchronised: the hooks return host objects, and about one call
        in twenty pays a Python garbage collection (tens of ms) that a mean would fold in."""
        ts, hs = [], []
        for _ in range(n):
            t0 = time.perf_counter()
            fn()
            hs.append((time.perf_counter() - t0) * 1e3)  # until the call returns: its host-side cost
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        ts.sort()
        hs.sort()
        host[0] = round(hs[len(hs) // 2], 4)
        return ts[len(ts) // 2], sum(ts) / len(ts)
    host = [None]
    for name, fn in (("in_place", lambda: codec.encode_module(m, base=base)),
                     ("flattened", lambda: codec.plan_for(
                         [e["n"] for e in base.entries if e["kind"] == "seg"], dev).encode(
                         flatten_state(state).flat, base=base.flat))):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        med, mean = per_call(fn, max(steps, 20))
        res[f"compression_{name}_ms"] = round(med, 4)
        res[f"compression_{name}_mean_ms"] = round(mean, 4)
        res[f"compression_{name}_host_ms"] = host[0]
    up = codec.encode_module(m, base=base)
    for _ in range(3):
        codec.decode_module(up, g, base=base)
    torch.cuda.synchronize()
    dec_ms, dec_mean = per_call(lambda: codec.decode_module(up, g, base=base), max(steps, 20))
    res["decompression_host_ms"] = host[0]
    N = sum(e["n"] for e in base.entries if e["kind"] == "seg")
    K, T = up.header["total_k"], up.header["n_segments"]
    alg = 16 * N + 10 * K + 16 * T
    ms = res["compression_in_place_ms"] + dec_ms
    # the fused server (codec_fused_aggregate): decompression(model) keeps the carrier, aggregate() decodes and
    # averages a round's uploads in one coalac_aggregate — per client, compression + 1/C of that call
    C = 16
    ups = [codec.encode_module(m, base=base) for _ in range(C)]
    wts = [10 + i for i in range(C)]
    for _ in range(3):
        codec.aggregate(ups, wts, g, base=base, mode="recip")
    torch.cuda.synchronize()
    agg_ms, _ = per_call(lambda: codec.aggregate(ups, wts, g, base=base, mode="recip"), max(steps, 20))
    fused_ms = res["compression_in_place_ms"] + agg_ms / C
    return {"value": round(4.0 * N / (ms * 1e-3) / 1e9, 2), "ms_per_client": round(ms, 4),
            **res, "decompression_ms": round(dec_ms, 4), "decompression_mean_ms": round(dec_mean, 4),
            "fused_server": {"value": round(4.0 * N / (fused_ms * 1e-3) / 1e9, 2), "ms_per_client": round(fused_ms, 4),
                             "aggregate_ms_per_round": round(agg_ms, 4), "clients_per_round": C,
                             "desc": "compression() + 1/C of the server's fused aggregate() of C uploads "
                                     "(UpdateCodec.aggregate: decode + FedAvg in one kernel, new module built once "
                                     "per round); decompression(model) passes the carrier through"},
            "timing": "median of per-call times (each call synchronised); means alongside; *_host_ms: median "
                      "time until the call returns (no wait inside it: its host-side cost)",
            "alg_bytes_per_client": alg,
            "step_roofline": {"achieved_GBs": round(alg / (ms * 1e-3) / 1e9, 1),
                              "frac": round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
            "desc": "UpdateCodec.encode_module(module, base) + decode_module(update, template, base): what "
                    "CompressionClientMixin.compression() / CompressionServerMixin.decompression() run, "
                    "host-side Python included; flattened = the round-1 path (torch.cat copy first)"}


def configs_summary(head, headline, results, plugin):
    """{config: [GB/s, ms per step, step roofline frac, dominant-kernel roofline frac]} for the headline and every
    extra (plugin: per client, its hooks' path; kernel frac null) — the line's last key."""
    out = {headline: [head["value"], head["ms_per_step"], head["step_roofline"]["frac"], head["roofline"]["frac"]]}
    for k, v in results.items():
        out[k] = [v["value"], v["ms_per_step"], v["step_roofline"]["frac"], v["roofline"]["frac"]]
    if plugin is not None:
        out["plugin"] = [plugin["value"], plugin["ms_per_client"], plugin["step_roofline"]["frac"], None]
    out["fields"] = "GB/s, ms_per_step, step_roofline_frac, kernel_roofline_frac"
    return out


def launch_ranks(a):
    """`--gpus N` (N > 1) without a launcher: start N rank processes of this script, one per GPU (RANK /
    LOCAL_RANK / WORLD_SIZE / MASTER_* in their environment, as torch.distributed.run sets them), before this
    process touches the GPU; rank 0 prints the JSON line. Mirrors the reference's own launcher, one
    process per GPU (examples/distributed_mp.py:77-84). Returns the exit code (the first failing rank's)."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(a.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.gpus), LOCAL_WORLD_SIZE=str(a.gpus),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        # rank 0's stdout through a pipe: only its JSON line reaches ours (the communication libraries print
        # status lines to stdout); everything else goes to stderr
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr, text=True))
    import threading

    def forward(pipe):
        for line in pipe:
            (sys.stdout if line.startswith('{"metric"') else sys.stderr).write(line)
            sys.stdout.flush()
    fwd = threading.Thread(target=forward, args=(procs[0].stdout,), daemon=True) if procs[0].stdout else None
    if fwd is not None:
        fwd.start()
    rc = 0
    try:
        pending = list(procs)
        while pending:
            for p in list(pending):
                code = p.poll()
                if code is None:
                    continue
                pending.remove(p)
                if code and not rc:
                    rc = code
                    for q in pending:  # one rank failed: the others would wait in a collective forever
                        q.terminate()
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
        if fwd is not None:
            fwd.join(timeout=10)
    return rc


def launch_check(a, world, rank, local):
    """--launch-check: the launcher's plumbing without a GPU — rendezvous over gloo on MASTER_ADDR / MASTER_PORT
    from the environment, gather every rank's (RANK, LOCAL_RANK, WORLD_SIZE) and print them from rank 0."""
    if rank == a.launch_check_fail:
        return 3
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mine = torch.tensor([rank, local, world], dtype=torch.int64)
    allr = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(allr, mine)
    times = gather_elapsed(0.01 * (rank + 1), world, "cpu")  # the timed region's per-rank gather, fake times
    if rank == 0:
        print(json.dumps({"metric": "launch-check", "ranks": [t.tolist() for t in allr],
                          "rank_ms_per_step": rank_spread(times, 1),
                          "master": [os.environ.get("MASTER_ADDR"), os.environ.get("MASTER_PORT")]}), flush=True)
    dist.destroy_process_group()
    return 0


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(a))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
    if a.launch_check:
        sys.exit(launch_check(a, world, rank, local))
    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        layout = a.layout or CONFIGS[a.config][0]
        cpu = cpu_baseline(layout if layout != "c5" else "resnet50_tv", a.ratio, a.bits, a.cpu_seconds)

    import torch
    import torch.distributed as dist
    # COALA_BENCH_DIST_BACKEND=gloo: a rehearsal of the N > 1 path with several ranks on fewer GPUs (ranks share
    # devices round-robin; RCCL refuses two ranks on one GPU). The driver's runs use RCCL, one rank per GPU.
    backend = os.environ.get("COALA_BENCH_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    order = [a.config] + ([] if a.extras == "none" else [c for c in a.extras.split(",") if c and c != a.config])
    # latency-bound configs: set up, warmed and captured as hipGraphs BEFORE the process group exists (with one
    # alive, RCCL's watchdog thread makes HIP calls while a capture runs); small buffers, kept until timed
    pre = {}
    for cfg in order:
        if cfg in CONFIGS and use_graph(cfg, a):
            W = setup_workload(cfg, a, dev, rank, headline=cfg == a.config)
            warm_workload(W, a)
            capture_graphs(W, a)
            pre[cfg] = W
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    results, plugin = {}, None
    for cfg in order:
        if cfg == "plugin":
            plugin = run_plugin(a, dev, a.steps)
            continue
        W = pre.pop(cfg, None)
        if W is None:
            W = setup_workload(cfg, a, dev, rank, headline=cfg == a.config)
            warm_workload(W, a)
        results[cfg] = time_workload(W, a, dev, world)
        release_workload(W)
    head = results.pop(a.config)
    box = box_probe(torch, dev) if rank == 0 else None

    if rank == 0:
        d = head["desc"]
        h_ratio, h_mode, _ = cfg_opts(a.config, a)  # (the headline config's own ratio / mode, else the command line's)
        res = {
            "metric": METRIC, "value": head["value"], "unit": "GB/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": head["ms_per_step"], "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": f"{a.config}-per-GPU: {d.get('clients_per_gpu')} x {d.get('layout', 'mixed')} "
                                   f"fp32 updates per GPU, top-k {h_ratio}, {a.bits}-bit codes, {h_mode} mode, "
                                   f"encode+decode batched as {head['split']} concurrent sub-batches",
                       **d, "global_clients": d.get("clients_per_gpu", 0) * world, "ratio": h_ratio, "bits": a.bits,
                       "mode": h_mode, "sub_batches_per_step": head["split"], "inflight_steps": head["inflight"],
                       "parallelism": f"replicas{world}"},
            "roofline": head["roofline"], "step_roofline": head["step_roofline"], "stages_ms": head["stages_ms"],
            "stage_timing": head["stage_timing"], "sample_fallbacks": head["sample_fallbacks"],
            "graph": head["graph"], "rank_ms_per_step": head["rank_ms_per_step"],
            "repeat_windows": head["repeat_windows"],
        }
        # cpu_baseline and box BEFORE the per-config details, and a compact summary of every config LAST: the driver
        # keeps only the tail of stdout, so every config's number must sit in the line's last ~2 KB
        if cpu is not None:
            res["cpu_baseline"] = cpu
        res["box"] = box
        res["configs"] = {k: {f: v[f] for f in ("value", "ms_per_step", "step_roofline", "roofline", "stages_ms",
                                                 "elements_per_gpu", "split", "graph", "sample_fallbacks",
                                                 "rank_ms_per_step", "repeat_windows")}
                          for k, v in results.items()}
        for v in res["configs"].values():  # (the roofline objects without their repeated constant fields)
            v["roofline"] = {f: v["roofline"][f] for f in ("kernel", "achieved", "frac")}
        if plugin is not None:
            res["configs"]["plugin"] = plugin
        res["configs_summary"] = configs_summary(head, a.config, results, plugin)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
