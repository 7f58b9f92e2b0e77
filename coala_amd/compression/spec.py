"""CodecSpec v1 host-side logic: kept-element counts and segment tables (no torch, no GPU).

The spec itself is SURVEY.md §8(a) rows a3/a4; the kernels implementing it are coala_amd/csrc/coalac.hip.
This module decides WHAT the kernels run on: one segment per fp32 state_dict entry, in the
state_dict's insertion order (the order coala/server/strategies.py:57-90 iterates), laid out in one
flat buffer with every segment start aligned to ALIGN elements (128 B), clients concatenated.
"""
import math
import os

import numpy as np

ALIGN = 32          # elements; 128-byte aligned segment starts (float4 loads need >= 4)
RAW_BITS = 32       # bits == 32: values stored as raw fp32 (lossless at ratio 1)
SMALL_MAX = 4096    # mirrors coalac.hip: the largest small-segment limit (one block, no sampling; COALAC_SMALL_MAX)
SMALL_MAX_BATCH = 1024     # mirrors coalac.hip: the default limit of batch plans
SMALL_MAX_LATENCY = 1024   # ... and of plans of <= LATENCY_PLAN_UNITS units (mirrors coalac.hip)
LATENCY_PLAN_UNITS = 8192
UNIT = 4096         # mirrors coalac.hip: elements per wave work unit
VALID_BITS = tuple(range(1, 9)) + (RAW_BITS,)


def small_limit(sizes):
    """The largest segment a plan over these segment sizes encodes whole in one block (coalac.hip
    coalac_plan_create): SMALL_MAX_LATENCY for latency-bound plans of <= LATENCY_PLAN_UNITS units, else
    SMALL_MAX_BATCH (COALAC_SMALL_MAX overrides, clamped to [1024, SMALL_MAX])."""
    units = sum((min(int(n), 1 << 31) + UNIT - 1) // UNIT for n in sizes)
    lim = SMALL_MAX_LATENCY if units <= LATENCY_PLAN_UNITS else SMALL_MAX_BATCH
    env = os.environ.get("COALAC_SMALL_MAX")
    if env:
        lim = min(max(int(env), 1024), SMALL_MAX)
    return lim


def k_for(n, ratio):
    """Kept elements of a segment of n elements: max(1, min(n, ceil(n * ratio))), 0 for n == 0.

    Computed in float64 on the host, as SURVEY.md §8(a) a3 specifies.
    """
    if not (ratio > 0.0):
        raise ValueError(f"ratio must be > 0, got {ratio}")
    n = int(n)
    if n <= 0:
        return 0
    return max(1, min(n, int(math.ceil(float(n) * float(ratio)))))


def align_up(x, a=ALIGN):
    return (int(x) + a - 1) // a * a


def units_of(n):
    """4096-element work units of a segment of n elements (0 for an empty one): the length of its stretch of the
    per-unit starts array (wire v2), in segment order (coalac.hip coalac_plan_create)."""
    return (int(n) + UNIT - 1) // UNIT


class SegmentTable:
    """Segment table of `clients` copies of one layout (list of fp32 segment sizes).

    segs: uint64 [clients * T, 4] rows (in_off, n, k, out_off) — the coalac_seg_t table.
    span_per_client: flat elements per client (aligned); total_k_per_client: kept entries per client.
    """

    def __init__(self, sizes, ratio, clients=1, align=ALIGN):
        self.sizes = [int(s) for s in sizes]
        self.ratio = float(ratio)
        self.clients = int(clients)
        if self.clients < 1:
            raise ValueError("clients must be >= 1")
        offs, ks, oofs = [], [], []
        off = oo = 0
        for n in self.sizes:
            offs.append(off)
            k = k_for(n, ratio)
            ks.append(k)
            oofs.append(oo)
            off = align_up(off + n, align)
            oo += k
        self.offsets = offs
        self.ks = ks
        self.out_offsets = oofs
        self.span_per_client = max(off, align)
        self.total_k_per_client = oo
        self.units_per_client = sum(units_of(n) for n in self.sizes)
        T = len(self.sizes)
        segs = np.zeros((self.clients * T, 4), dtype=np.uint64)
        for c in range(self.clients):
            for t in range(T):
                segs[c * T + t] = (c * self.span_per_client + offs[t], self.sizes[t], ks[t],
                                   c * self.total_k_per_client + oofs[t])
        self.segs = segs

    uniform = True  # clients are copies of one layout (fused aggregation needs this)

    @property
    def n_segments(self):
        return len(self.segs)

    @property
    def span(self):
        return self.clients * self.span_per_client

    @property
    def total_k(self):
        return self.clients * self.total_k_per_client

    @property
    def n_units(self):
        return self.clients * self.units_per_client

    @property
    def n_elements(self):
        return self.clients * sum(self.sizes)

    # per-client extents (client-major), as cumulative offsets of length clients + 1
    @property
    def client_span_off(self):
        return [c * self.span_per_client for c in range(self.clients + 1)]

    @property
    def client_k_off(self):
        return [c * self.total_k_per_client for c in range(self.clients + 1)]

    @property
    def client_seg_off(self):
        T = len(self.sizes)
        return [c * T for c in range(self.clients + 1)]

    @property
    def client_unit_off(self):
        return [c * self.units_per_client for c in range(self.clients + 1)]

    def client_sizes(self, c):
        return self.sizes

    def client_elements(self):
        return [sum(self.sizes)] * self.clients

    def sub_table(self, c0, c1):
        """Table of clients [c0, c1) with offsets relative to client c0's start."""
        return SegmentTable(self.sizes, self.ratio, c1 - c0)

    def algorithmic_bytes(self, bits=8, delta=False):
        return algorithmic_bytes(self.n_elements, self.total_k, self.n_segments, bits, delta, self.ratio >= 1.0)


def algorithmic_bytes(N, K, T, bits=8, delta=False, implied_idx=False):
    """HBM bytes an ideal encode+decode moves: 8N + 10K + 32T for 8-bit codes.

    Encode reads 4N, writes idx (4K) + codes (1K, or 4K raw) + mn/scale/k/off (16T); decode reads
    those and writes 4N. Delta mode adds a 4N base read on each side. implied_idx (ratio 1, the dense
    codec): no idx is written or read — 10N + 32T for 8-bit codes.
    """
    vb = 4 if bits == RAW_BITS else 1
    b = 8 * N + 2 * ((0 if implied_idx else 4) + vb) * K + 32 * T
    if delta:
        b += 8 * N
    return b


class MixedTable:
    """Segment table of clients with DIFFERENT layouts (splitFL client-side models of
    several architectures and cut layers next to feature tensors), laid out client-major in one flat
    buffer exactly like SegmentTable: every segment start ALIGN-aligned, each client's span a multiple
    of ALIGN, each client's kept entries contiguous.

    layouts: one list of fp32 segment sizes per client.
    """

    uniform = False

    def __init__(self, layouts, ratio, align=ALIGN):
        self.layouts = [[int(s) for s in sizes] for sizes in layouts]
        self.ratio = float(ratio)
        self.clients = len(self.layouts)
        if self.clients < 1:
            raise ValueError("a MixedTable needs at least one client")
        rows = []
        span_off, k_off, seg_off, unit_off = [0], [0], [0], [0]
        off = oo = uo = 0
        for sizes in self.layouts:
            c0 = off
            for n in sizes:
                k = k_for(n, ratio)
                rows.append((off, n, k, oo))
                off = align_up(off + n, align)
                oo += k
                uo += units_of(n)
            off = max(off, c0 + align)  # a client with no fp32 element still owns one aligned slot
            span_off.append(off)
            k_off.append(oo)
            seg_off.append(len(rows))
            unit_off.append(uo)
        self.segs = np.array(rows, dtype=np.uint64).reshape(-1, 4)
        self.client_span_off, self.client_k_off, self.client_seg_off = span_off, k_off, seg_off
        self.client_unit_off = unit_off

    @property
    def n_segments(self):
        return len(self.segs)

    @property
    def span(self):
        return self.client_span_off[-1]

    @property
    def total_k(self):
        return self.client_k_off[-1]

    @property
    def n_units(self):
        return self.client_unit_off[-1]

    @property
    def n_elements(self):
        return int(self.segs[:, 1].sum()) if len(self.segs) else 0

    def client_sizes(self, c):
        return self.layouts[c]

    def client_elements(self):
        return [sum(s) for s in self.layouts]

    def sub_table(self, c0, c1):
        return MixedTable(self.layouts[c0:c1], self.ratio)

    def algorithmic_bytes(self, bits=8, delta=False):
        return algorithmic_bytes(self.n_elements, self.total_k, self.n_segments, bits, delta)


class SubTable:
    """Explicit segment rows (in_off, n, k, out_off) with ABSOLUTE offsets, e.g. a contiguous slice of a
    SegmentTable (one lane of coala_amd/compression/pipeline.py). total_k / span are the buffer extents
    the rows need (max out_off + k, max in_off + n), not their sums."""

    clients = None  # not a copies-of-one-layout table: no fused aggregation over it
    uniform = False

    def __init__(self, segs):
        self.segs = np.ascontiguousarray(np.asarray(segs, dtype=np.uint64).reshape(-1, 4))

    @property
    def n_segments(self):
        return len(self.segs)

    @property
    def total_k(self):
        return int((self.segs[:, 3] + self.segs[:, 2]).max()) if len(self.segs) else 0

    @property
    def span(self):
        return int((self.segs[:, 0] + self.segs[:, 1]).max()) if len(self.segs) else 0

    @property
    def n_units(self):
        return sum(units_of(n) for n in self.segs[:, 1].tolist())

    @property
    def n_elements(self):
        return int(self.segs[:, 1].sum())
