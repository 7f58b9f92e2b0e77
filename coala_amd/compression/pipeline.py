"""Batched pipelines over one GPU: SplitPipeline (a batch as independent sub-batches side by side).

Why: per batch, encode is k_sample -> k_scan (one HBM read of the update) -> k_ghist ->
k_gwin -> k_select -> k_emit (+ the small segments), and decode is k_bounds -> k_decode (one HBM write of
the dense output). k_scan / k_decode are HBM-bound; the rest are latency-bound (a block per segment or
group, tens of us at a few CUs' worth of work). Two sub-batches on two streams fill each other's
latency-bound phases and launch tails. (Round 2 also built a "lane" pipeline that put every streaming
kernel of a batch back to back on one stream and the latency-bound stages on another, ordered by the
split-stage ABI: it measured 8 % slower than free-running sub-batches and was removed in round 3.)
"""
import torch

from . import _lib
from .plan import CodecPlan, Encoded
from .spec import SegmentTable, units_of

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


class SplitPipeline:
    """A batch of C client updates as S independent sub-batches of C / S clients, each with its own plan,
    workspaces and HIP stream, launched side by side.

    Why: one batch's launch sequence alternates HBM-bound kernels (k_scan, k_decode) with
    latency-bound ones (k_sample, the select chain, k_bounds) whose few blocks leave most CUs idle, and
    every kernel has a launch tail. Two sub-batches on two streams fill each other's idle phases and
    tails: 16 ResNet-50 updates run 11-14 % faster as 2 x 8 than as 1 x 16 (bench.py --split). Nothing is
    serialised across sub-batches; the hardware interleaves them.

    Sub-batches are contiguous client ranges. Every per-client quantity of a SegmentTable batch is
    client-major (input / dense output spans, idx / vals of total_k_per_client, mn / scale of the
    client's segments), so sub-batch g is an ordinary plan over its C_g clients working on views of the
    whole batch's buffers: results are bit-identical to a single plan's. (A plan over absolute segment
    rows measured 2.5 % slower here.) Calls are asynchronous and ordered after /
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
                so, ko, to, uo = table.client_span_off, table.client_k_off, table.client_seg_off, table.client_unit_off
                # stream_base: pipelines meant to run side by side (several batches in flight) take
                # disjoint pool ranges; by default every pipeline starts at pooled stream 0
                streams = pooled_streams(self.device, stream_base + len(cuts) - 1)[stream_base:]
                for c0, c1, st in zip(cuts[:-1], cuts[1:], streams):
                    plan = CodecPlan(None, table.ratio, self.bits, device=self.device, table=table.sub_table(c0, c1))
                    self.parts.append(dict(x=slice(so[c0], so[c1]), k=slice(ko[c0], ko[c1]), t=slice(to[c0], to[c1]),
                                           u=slice(uo[c0], uo[c1]), plan=plan, ws=plan.empty_workspace(), stream=st))
            else:
                # fewer clients than sub-batches (e.g. ONE update): contiguous SEGMENT ranges balanced by
                # element count, each a plan over absolute segment rows that reads / writes the whole
                # buffers in place (its own segments only) — the ranges' latency-bound phases overlap
                ranges = split_lanes(table.segs[:, 1].tolist(), S)
                uo = [0]
                for n in table.segs[:, 1].tolist():
                    uo.append(uo[-1] + units_of(n))
                for (s0, s1), st in zip(ranges, pooled_streams(self.device, stream_base + len(ranges))[stream_base:]):
                    plan = CodecPlan.from_segments(table.segs[s0:s1], self.bits, device=self.device)
                    self.parts.append(dict(x=slice(None), k=slice(None), t=slice(s0, s1), u=slice(uo[s0], uo[s1]),
                                           plan=plan, ws=plan.empty_workspace(), stream=st))

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
        T, K, U = self.table.n_segments, self.table.total_k, self.table.n_units
        implied = all(P["plan"].implied_idx for P in self.parts)  # ratio 1: no idx / starts (dense codec)
        return Encoded(torch.empty(0 if implied else K, dtype=torch.int32, device=d), torch.empty(K, dtype=vt, device=d),
                       torch.empty(T, dtype=torch.float32, device=d), torch.empty(T, dtype=torch.float32, device=d),
                       None if implied else torch.empty(U, dtype=torch.int32, device=d))

    @staticmethod
    def _enc(enc, P):
        return Encoded(enc.idx[P["k"]] if enc.idx.numel() else enc.idx, enc.vals[P["k"]], enc.mn[P["t"]], enc.scale[P["t"]],
                       None if enc.ustart is None else enc.ustart[P["u"]])


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
        P["plan"].decode(self._enc(enc, P), base=self._x(base, P), out=self._x(out, P),
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

    def close(self):
        for P in self.parts:
            P["plan"].close()
        self.parts = []
