"""Lane pipeline: one batch of segments cut into L lanes (contiguous segment ranges, balanced by element
count), each a sub-plan, with the HBM-streaming kernels of every lane back to back on one stream and
the latency-bound kernels on one or two streams beside them.

Why: per batch, encode is k_sample → k_scan (one HBM read of the update) → k_ghist →
k_gwin → k_select → k_emit (+ k_small for the small segments), and decode is k_bounds → k_decode (one
HBM write of the dense output). k_scan / k_decode are HBM-bound; the rest are latency-bound (a block per
segment or group, tens of µs at a few CUs' worth of work). On one stream they serialise and HBM idles
for ~0.2 ms of the 0.87 ms step of 16 ResNet-50 updates. The split-stage ABI (coalac_encode_sched /
coalac_decode_sched, COALAC_STAGE_*) lets the host place stages on separate streams:

    S (streaming):  sample_0 scan_0 │ scan_1 … scan_{L-1} │ decode_0 … decode_{L-1}
    C (latency):    sample_i, small_i │ select_0 bounds_0 │ select_1 bounds_1 │ …   (lane i on C[i % nC])

scan_i waits for sample_i, select_i for scan_i, decode_i for bounds_i (events). HBM sees one read phase
then one write phase — mixed read/write traffic streams slower than either (tools/hbm_probe: copy
4.65 TB/s of traffic vs 6.15 read / 5.4 write) — and every latency-bound stage except sample_0 runs
under a streaming kernel. C streams get a higher priority so their few blocks are dispatched ahead of
the streaming kernel's backlog. Cross-queue waits cost ~15 µs when the waiting queue is idle, so the
schedule is arranged for each wait to be satisfied before the waiting queue reaches it; a caller that
submits batches back to back can make `pipe.stream` its current stream to drop the entry/exit joins.

Lanes are contiguous ranges of the segment table, so one client's update can be split as well as a
batch of many: every sub-plan keeps the absolute in/out offsets of its segments and writes the shared
idx / vals arrays and the dense output in place; mn / scale are indexed by segment, so a lane gets the
[s0, s1) slice of them. Results are bit-identical to a single plan over the whole table (tests/
test_gpu_pipeline.py) because segments are independent.
"""
import torch

from . import _lib
from .plan import CodecPlan, Encoded
from .spec import SegmentTable, small_limit

_IN_LAUNCH = _lib.COALAC_FLAG_ONE_LAUNCH | _lib.COALAC_FLAG_FRONT_LAUNCH  # encodes with in-launch waits


_STREAM_POOL = {}  # device index -> streams shared by every SplitPipeline of the process


def pooled_streams(device, n):
    """The first n streams of a per-device pool created once per process, in order. HIP binds a stream to
    one of its hardware queues (4 per process by default) when the stream is created, round-robin: two
    sub-batch streams created far apart can land on one queue and then run one after the other (a C2
    share as 3 sub-batches measured 1,707 vs 2,279 GB/s depending on which streams the process had made
    before). Pipelines that take their sub-batch streams from this pool always get the same consecutive,
    queue-distinct streams, whatever else the process created in between."""
    d = torch.device(device)
    key = d.index if d.index is not None else torch.cuda.current_device()
    pool = _STREAM_POOL.setdefault(key, [])
    with torch.cuda.device(key):
        while len(pool) < n:
            pool.append(torch.cuda.Stream(key))
    return pool[:n]


def split_lanes(sizes, lanes):
    """Cut segment sizes into <= `lanes` contiguous ranges [s0, s1) of about equal element count.

    Greedy prefix cut at the multiples of total/lanes; empty ranges are dropped, so fewer lanes come
    back when there are fewer segments than lanes.
    """
    sizes = [int(s) for s in sizes]
    lanes = max(1, int(lanes))
    total = sum(sizes)
    if not sizes:
        return []
    cuts, acc = [0], 0
    for i, n in enumerate(sizes):
        acc += n
        if len(cuts) < lanes and acc * lanes >= total * len(cuts) and i + 1 < len(sizes):
            cuts.append(i + 1)
    cuts.append(len(sizes))
    return [(a, b) for a, b in zip(cuts[:-1], cuts[1:]) if b > a]


def balanced_cuts(costs, parts):
    """Cut a client list into `parts` contiguous non-empty ranges of about equal total cost (element
    count): returns the cut points [0, ..., len(costs)]. Equal costs give equal client counts."""
    C = len(costs)
    parts = max(1, min(int(parts), C))
    pre = [0]
    for c in costs:
        pre.append(pre[-1] + int(c))
    total = pre[-1]
    cuts = [0]
    for g in range(1, parts):
        target = total * g / parts
        # first cut point whose prefix reaches the target, keeping every range non-empty
        j = max(cuts[-1] + 1, min(range(1, C), key=lambda i: abs(pre[i] - target)))
        cuts.append(min(j, C - (parts - g)))
    cuts.append(C)
    return cuts


class LanePipeline:
    """Encode / decode a SegmentTable's batch as L pipelined lanes on one GPU.

    The buffers are those of a single plan over the whole table (flat input fp32[span], Encoded with
    idx/vals[total_k] and mn/scale[n_segments], dense output fp32[span]). Every call is asynchronous
    with respect to the host and ordered with respect to the caller's current stream: the pipeline's
    streams wait for it on entry and it waits for them on exit. c_streams: latency-stage streams
    (default 1 for <= 2 lanes, else 2; with S and the caller's stream that stays within the 4
    hardware queues HIP gives a process by default). c_priority: their stream priority (lower =
    higher; torch clamps to the device's range).
    """

    def __init__(self, table: SegmentTable, bits=8, lanes=2, device=None, flags=0, c_streams=None, c_priority=-1):
        self.table = table
        self.bits = int(bits)
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None
                                   else torch.device(device).index or 0)
        self.ranges = split_lanes(table.segs[:, 1].tolist(), lanes)
        self.flags = int(flags)
        nc = c_streams if c_streams is not None else (1 if len(self.ranges) <= 2 else 2)
        self.lanes = []
        with torch.cuda.device(self.device):
            self.s_stream = torch.cuda.Stream(self.device)  # k_sample_0, every k_scan and k_decode
            self.c_streams = [torch.cuda.Stream(self.device, priority=c_priority) for _ in range(max(1, int(nc)))]
            for i, (s0, s1) in enumerate(self.ranges):
                plan = CodecPlan.from_segments(table.segs[s0:s1], self.bits, device=self.device)
                n = table.segs[s0:s1, 1]
                lim = small_limit(n)
                L = dict(s0=s0, s1=s1, plan=plan, ws=plan.empty_workspace(), dws=plan.empty_decode_workspace(),
                         c=self.c_streams[i % len(self.c_streams)],
                         n_small=int((n <= lim).sum()), n_large=int((n > lim).sum()))
                for name in ("sampled", "scanned", "bounded", "decoded"):
                    L[name] = torch.cuda.Event()
                    L[name].record(self.s_stream)  # torch creates the HIP event on first record
                self.lanes.append(L)

    @property
    def n_lanes(self):
        return len(self.lanes)

    @property
    def stream(self):
        """The streaming stream S: as the caller's current stream it makes back-to-back calls join-free."""
        return self.s_stream

    # -- buffers ----------------------------------------------------------------------------------
    def empty_flat(self):
        return torch.empty(self.table.span, dtype=torch.float32, device=self.device)

    def empty_encoded(self):
        d, vt = self.device, torch.float32 if self.bits == 32 else torch.uint8
        T, K = self.table.n_segments, self.table.total_k
        return Encoded(torch.empty(K, dtype=torch.int32, device=d), torch.empty(K, dtype=vt, device=d),
                       torch.empty(T, dtype=torch.float32, device=d), torch.empty(T, dtype=torch.float32, device=d))

    @staticmethod
    def _lane_view(enc, L):
        return Encoded(enc.idx, enc.vals, enc.mn[L["s0"]:L["s1"]], enc.scale[L["s0"]:L["s1"]])

    # -- scheduling -------------------------------------------------------------------------------
    def _streams(self):
        return [self.s_stream] + self.c_streams

    def _enter(self):
        cur = torch.cuda.current_stream(self.device)
        for s in self._streams():
            if s != cur:
                s.wait_stream(cur)

    def _leave(self):
        cur = torch.cuda.current_stream(self.device)
        for s in self._streams():
            if s != cur:
                cur.wait_stream(s)

    def _enc(self, L, flat, base, out, stream, stages, wait=None, record=None):
        L["plan"].encode(flat, base=base, out=self._lane_view(out, L), workspace=L["ws"], flags=self.flags,
                         stream=stream, sched=(wait or [None] * 5, record or [None] * 5, stages))

    def _dec(self, L, enc, base, out, stream, stages, wait=None, record=None):
        L["plan"].decode(self._lane_view(enc, L), base=base, out=out, workspace=L["dws"], stream=stream,
                         sched=(wait or [None] * 3, record or [None] * 3, stages))

    def _encode(self, flat, base, out, events, dense=None, free=False):
        S = self.s_stream
        for i, L in enumerate(self.lanes):  # samples of lanes 1.. (free: every lane) and the small segments on C
            if free:
                L["c"].wait_event(L["decoded"])  # the lane's previous decode read the idx / vals rewritten here
            if (i or free) and L["n_large"]:
                self._enc(L, flat, base, out, L["c"], _lib.COALAC_STAGE_SAMPLE,
                          record=[None, L["sampled"], None, None, None])
            if free and L["n_small"]:
                self._enc(L, flat, base, out, L["c"], _lib.COALAC_STAGE_SMALL)
        for L in self.lanes:
            if L["n_small"] and not free:
                self._enc(L, flat, base, out, L["c"], _lib.COALAC_STAGE_SMALL)
        for i, L in enumerate(self.lanes):  # the read phase: every k_scan back to back on S
            ev = events[i] if events is not None else [None] * 5
            stages = _lib.COALAC_STAGE_SCAN | (_lib.COALAC_STAGE_SAMPLE if i == 0 and not free else 0)
            wait = [None, L["sampled"] if (i or free) and L["n_large"] else None, None, None, None]
            rec = [None, ev[1], ev[2] if ev[2] is not None else L["scanned"], None, None]
            self._enc(L, flat, base, out, S, stages, wait=wait, record=rec)
            L["token"] = rec[2]
        for L in self.lanes:  # select + emit of lane i on C, under the scans of lanes > i
            self._enc(L, flat, base, out, L["c"], _lib.COALAC_STAGE_SELECT, wait=[None, None, L["token"], None, None])
            if dense is not None:  # roundtrip: lane i's decode bounds right after its emit
                self._dec(L, out, None, dense, L["c"], _lib.COALAC_STAGE_BOUNDS, record=[None, L["bounded"], None])

    def _decode(self, enc, base, out, events, bounds_done=False, free=False):
        S = self.s_stream
        if not bounds_done:
            for L in self.lanes:
                self._dec(L, enc, base, out, L["c"], _lib.COALAC_STAGE_BOUNDS, record=[None, L["bounded"], None])
        for i, L in enumerate(self.lanes):  # the write phase: every k_decode back to back on S
            ev = events[i] if events is not None else [None] * 3
            self._dec(L, enc, base, out, S, _lib.COALAC_STAGE_DECODE, wait=[None, L["bounded"], None],
                      record=[None, ev[1], ev[2]])
            if free:
                L["decoded"].record(S)

    def encode(self, flat, base=None, out=None, events=None):
        """Encode the whole batch (flat fp32[span]; base: delta mode) -> Encoded. events: optional
        per-lane lists of 5 recorded timing events; [1] / [2] are recorded around the lane's k_scan."""
        out = self.empty_encoded() if out is None else out
        if self.n_lanes == 1:
            return self._single_encode(flat, base, out, events)
        self._enter()
        self._encode(flat, base, out, events)
        self._leave()
        return out

    def decode(self, enc, base=None, out=None, events=None):
        """Decode the whole batch into the dense out (fp32[span]; + base, fused). events: optional
        per-lane lists of 3 recorded timing events; [1] / [2] are recorded around the lane's k_decode."""
        if out is None:
            out = self.empty_flat() if base is None else torch.empty_like(base)
        if self.n_lanes == 1:
            return self._single_decode(enc, base, out, events)
        self._enter()
        self._decode(enc, base, out, events)
        self._leave()
        return out

    def roundtrip(self, flat, base=None, enc=None, out=None, enc_events=None, dec_events=None, joined=True):
        """encode() then decode() of the same batch with no join in between: lane i's decode depends on
        lane i's encode only (bounds_i follows select_i on C), so the last lanes' select chains run
        under the first lanes' k_decode. Returns (Encoded, dense out).

        joined=False (back-to-back calls on the same buffers, e.g. the bench): no entry / exit joins with
        the caller's stream; every lane's sampler and small segments run on C once the lane's previous
        decode is done (it read what they overwrite), i.e. under the previous call's later decodes, so S
        runs scan_0 .. scan_{L-1} decode_0 .. decode_{L-1} back to back, call after call. The caller
        orders its own use of the results (e.g. synchronises, or waits on `self.stream` and the C streams)."""
        enc = self.empty_encoded() if enc is None else enc
        if out is None:
            out = self.empty_flat() if base is None else torch.empty_like(base)
        if self.n_lanes == 1:
            return self._single_encode(flat, base, enc, enc_events), self._single_decode(enc, base, out, dec_events)
        if joined:
            self._enter()
            self._encode(flat, base, enc, enc_events, dense=out)
            self._decode(enc, base, out, dec_events, bounds_done=True)
            self._leave()
        else:
            self._encode(flat, base, enc, enc_events, dense=out, free=True)
            self._decode(enc, base, out, dec_events, bounds_done=True, free=True)
        return enc, out

    # one lane: the plain whole-encode / whole-decode calls on the caller's stream (a split would only
    # add cross-queue hops; the plan forks its small segments to a side stream when that pays)
    def _single_encode(self, flat, base, out, events):
        L = self.lanes[0]
        L["plan"].encode(flat, base=base, out=self._lane_view(out, L), workspace=L["ws"], flags=self.flags,
                         events=None if events is None else events[0])
        return out

    def _single_decode(self, enc, base, out, events):
        L = self.lanes[0]
        L["plan"].decode(self._lane_view(enc, L), base=base, out=out, workspace=L["dws"],
                         events=None if events is None else events[0])
        return out

    def fallbacks(self):
        """Segments of the last encode whose sampled bracket missed (synchronises)."""
        torch.cuda.synchronize(self.device)
        return sum(L["plan"].fallbacks(L["ws"]) for L in self.lanes)

    def timeouts(self):
        """Bounded in-launch waits that gave up (one-launch / front-launch encodes only; the kernel
        sequence has none)."""
        if not self.flags & _IN_LAUNCH:
            return 0
        torch.cuda.synchronize(self.device)
        return sum(L["plan"].timeouts(L["ws"]) for L in self.lanes)

    @property
    def n_parts(self):
        return len(self.lanes)

    def close(self):
        for L in self.lanes:
            L["plan"].close()
        self.lanes = []


class SplitPipeline:
    """A batch of C client updates as S independent sub-batches of C / S clients, each with its own plan,
    workspaces and HIP stream, launched side by side.

    Why: one batch's launch sequence alternates HBM-bound kernels (k_scan, k_decode) with
    latency-bound ones (k_sample, the select chain, k_bounds) whose few blocks leave most CUs idle, and
    every kernel has a launch tail. Two sub-batches on two streams fill each other's idle phases and
    tails: 16 ResNet-50 updates run 11-14 % faster as 2 x 8 than as 1 x 16 (bench.py --split). Unlike
    LanePipeline's lanes, nothing is serialised across sub-batches; the hardware interleaves them.

    Sub-batches are contiguous client ranges. Every per-client quantity of a SegmentTable batch is
    client-major (input / dense output spans, idx / vals of total_k_per_client, mn / scale of the
    client's segments), so sub-batch g is an ordinary plan over its C_g clients working on views of the
    whole batch's buffers: results are bit-identical to a single plan's. (A plan over absolute segment
    rows, as LanePipeline uses, measured 2.5 % slower here.) Calls are asynchronous and ordered after /
    before the caller's current stream (the sub-batch streams wait for it on entry, it waits for them
    on exit), unless joined=False. Sub-batch g runs on the process-wide pooled stream g
    (pooled_streams): pipelines of one process share them, so their calls are ordered with each other
    per sub-batch index.
    """

    def __init__(self, table: SegmentTable, bits=8, split=2, device=None, flags=0, fork=False, stream_base=0):
        self.table = table
        self.bits = int(bits)
        self.flags = int(flags)
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None
                                   else torch.device(device).index or 0)
        C = max(1, int(table.clients))
        S = max(1, int(split))
        # several sub-batches already run side by side: no per-plan side stream for the small segments
        # (HIP maps streams onto 4 hardware queues; a side stream sharing one with the other sub-batch
        # would queue its k_small behind that sub-batch's kernels)
        self.fork_flag = _lib.COALAC_FLAG_NO_FORK if S > 1 and fork is False else 0
        self.parts = []
        with torch.cuda.device(self.device):
            if S <= C:  # client ranges: ordinary plans over views of the batch buffers
                cuts = balanced_cuts(table.client_elements(), S)
                so, ko, to = table.client_span_off, table.client_k_off, table.client_seg_off
                # stream_base: pipelines meant to run side by side (several batches in flight) take
                # disjoint pool ranges; by default every pipeline starts at pooled stream 0
                streams = pooled_streams(self.device, stream_base + len(cuts) - 1)[stream_base:]
                for c0, c1, st in zip(cuts[:-1], cuts[1:], streams):
                    plan = CodecPlan(None, table.ratio, self.bits, device=self.device, table=table.sub_table(c0, c1))
                    self.parts.append(dict(x=slice(so[c0], so[c1]), k=slice(ko[c0], ko[c1]), t=slice(to[c0], to[c1]),
                                           plan=plan, ws=plan.empty_workspace(), dws=plan.empty_decode_workspace(),
                                           stream=st))
            else:
                # fewer clients than sub-batches (e.g. ONE update): contiguous SEGMENT ranges balanced by
                # element count, each a plan over absolute segment rows that reads / writes the whole
                # buffers in place (its own segments only) — the ranges' latency-bound phases overlap
                ranges = split_lanes(table.segs[:, 1].tolist(), S)
                for (s0, s1), st in zip(ranges, pooled_streams(self.device, stream_base + len(ranges))[stream_base:]):
                    plan = CodecPlan.from_segments(table.segs[s0:s1], self.bits, device=self.device)
                    self.parts.append(dict(x=slice(None), k=slice(None), t=slice(s0, s1), plan=plan,
                                           ws=plan.empty_workspace(), dws=plan.empty_decode_workspace(),
                                           stream=st))

    @property
    def n_parts(self):
        return len(self.parts)

    @property
    def streams(self):
        return [P["stream"] for P in self.parts]

    def empty_flat(self):
        return torch.empty(self.table.span, dtype=torch.float32, device=self.device)

    def empty_encoded(self):
        d, vt = self.device, torch.float32 if self.bits == 32 else torch.uint8
        T, K = self.table.n_segments, self.table.total_k
        return Encoded(torch.empty(K, dtype=torch.int32, device=d), torch.empty(K, dtype=vt, device=d),
                       torch.empty(T, dtype=torch.float32, device=d), torch.empty(T, dtype=torch.float32, device=d))

    @staticmethod
    def _enc(enc, P):
        return Encoded(enc.idx[P["k"]], enc.vals[P["k"]], enc.mn[P["t"]], enc.scale[P["t"]])


    @staticmethod
    def _x(t, P):
        return None if t is None else t[P["x"]]

    def _run(self, fn, joined):
        cur = torch.cuda.current_stream(self.device)
        if joined:
            for P in self.parts:
                P["stream"].wait_stream(cur)
        for g, P in enumerate(self.parts):
            with torch.cuda.stream(P["stream"]):
                fn(g, P)
        if joined:
            for P in self.parts:
                cur.wait_stream(P["stream"])

    def _encode_part(self, g, P, flat, base, out, events):
        P["plan"].encode(self._x(flat, P), base=self._x(base, P), out=self._enc(out, P), workspace=P["ws"],
                         flags=self.flags | self.fork_flag, events=None if events is None else events[g])

    def _decode_part(self, g, P, enc, base, out, events):
        P["plan"].decode(self._enc(enc, P), base=self._x(base, P), out=self._x(out, P), workspace=P["dws"],
                         events=None if events is None else events[g])

    def encode(self, flat, base=None, out=None, events=None, joined=True):
        """Encode the batch -> Encoded. events: optional per-sub-batch lists of 5 timing events
        (coalac_encode_ev boundaries; [1] / [2] bracket k_scan). joined=False skips the entry/exit joins
        with the caller's stream (a caller that orders consecutive calls itself, e.g. the bench)."""
        out = self.empty_encoded() if out is None else out
        self._run(lambda g, P: self._encode_part(g, P, flat, base, out, events), joined)
        return out

    def decode(self, enc, base=None, out=None, events=None, joined=True):
        """Decode into the dense out (+ base, fused). events: per-sub-batch lists of 3 ([1] / [2] bracket
        k_decode)."""
        if out is None:
            out = self.empty_flat() if base is None else torch.empty_like(base)
        self._run(lambda g, P: self._decode_part(g, P, enc, base, out, events), joined)
        return out

    def roundtrip(self, flat, base=None, enc=None, out=None, enc_events=None, dec_events=None, joined=True):
        """encode() then decode() with one join each way: sub-batch g's decode follows its own encode on
        its stream only."""
        enc = self.empty_encoded() if enc is None else enc
        if out is None:
            out = self.empty_flat() if base is None else torch.empty_like(base)

        def both(g, P):
            self._encode_part(g, P, flat, base, enc, enc_events)
            self._decode_part(g, P, enc, base, out, dec_events)
        self._run(both, joined)
        return enc, out

    def fallbacks(self):
        torch.cuda.synchronize(self.device)
        return sum(P["plan"].fallbacks(P["ws"]) for P in self.parts)

    def timeouts(self):
        """Bounded in-launch waits that gave up (one-launch / front-launch encodes only)."""
        if not self.flags & _IN_LAUNCH:
            return 0
        torch.cuda.synchronize(self.device)
        return sum(P["plan"].timeouts(P["ws"]) for P in self.parts)

    def close(self):
        for P in self.parts:
            P["plan"].close()
        self.parts = []
