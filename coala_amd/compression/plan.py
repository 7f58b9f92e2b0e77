"""Device-side codec plan: one segment table (a model layout × clients) bound to one GPU.

Thin typed wrapper over coalac_plan_create / coalac_encode / coalac_decode. Tensors are torch tensors
used purely as device memory; streams are torch's current HIP stream unless one is passed. Every
argument is checked against what the kernels assume (dtype, device, contiguity, length, 16-B
alignment) BEFORE a launch.
"""
import contextlib
import ctypes
from dataclasses import dataclass

import torch

from . import _lib
from .spec import RAW_BITS, UNIT, VALID_BITS, SegmentTable, SubTable


@dataclass
class Encoded:
    """Device buffers of one encode: idx int32[K], vals uint8[K] (fp32[K] when bits == 32),
    mn fp32[T], scale fp32[T], and (wire v2) ustart int32[U]: per 4096-element unit, the segment-relative
    index of its first kept entry — a decoder then needs no search of the idx lists (None: not available)."""
    idx: torch.Tensor
    vals: torch.Tensor
    mn: torch.Tensor
    scale: torch.Tensor
    ustart: torch.Tensor = None

    FIELDS = ("idx", "vals", "mn", "scale", "ustart")

    def to(self, device, non_blocking=False):
        return Encoded(*(None if t is None else t.to(device, non_blocking=non_blocking)
                         for t in (self.idx, self.vals, self.mn, self.scale, self.ustart)))


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _idx_ptr(t):
    """idx of an Encoded: NULL when it holds nothing (a dense plan's implied indices)."""
    return ctypes.c_void_p(t.data_ptr()) if t is not None and t.numel() else ctypes.c_void_p(0)


def _on(stream):
    """Allocation context for buffers a call creates itself: on the stream the kernels run on, so the
    caching allocator never hands their memory to other work before those kernels are done."""
    return torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()


_NULL_CTX = contextlib.nullcontext()


def _device_ctx(device):
    """torch.cuda.device(device), or nothing when it is already the current device (the common case: the
    context manager's exchange costs a few us per call on the hooks' path)."""
    return _NULL_CTX if torch.cuda.current_device() == device.index else torch.cuda.device(device)


def _stream_handle(stream):
    s = torch.cuda.current_stream() if stream is None else stream
    return ctypes.c_void_p(s.cuda_stream)


class CodecPlan:
    """Plan for `clients` copies of a layout given by fp32 segment sizes.

    Args:
        sizes: element count of every fp32 segment of ONE client, in state_dict order.
        ratio: top-k ratio in (0, 1].
        bits:  1..8 (uint8 codes) or 32 (raw fp32 values).
        clients: number of client updates batched into one launch sequence.
        device: CUDA/HIP device (default: current).
    """

    def __init__(self, sizes, ratio, bits=8, clients=1, device=None, table=None):
        if bits not in VALID_BITS:
            raise ValueError(f"bits must be one of {VALID_BITS}, got {bits}")
        self.table = SegmentTable(sizes, ratio, clients) if table is None else table
        self.bits = int(bits)
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None
                                   else torch.device(device).index or 0)
        self._lib = _lib.load()
        segs = self.table.segs
        arr = (_lib.SegDesc * len(segs))()
        for i, (a, b, c, d) in enumerate(segs.tolist()):
            arr[i] = _lib.SegDesc(a, b, c, d)
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _lib.check(self._lib.coalac_plan_create(arr, len(segs), self.bits, ctypes.byref(h)),
                       "coalac_plan_create")
        self._h = h
        ws, tk, span, nu = (ctypes.c_uint64() for _ in range(4))
        _lib.check(self._lib.coalac_plan_query(h, ctypes.byref(ws), ctypes.byref(tk), ctypes.byref(span),
                                               ctypes.byref(nu)), "coalac_plan_query")
        self.ws_bytes = ws.value
        self.total_k, self.span, self.n_units = tk.value, span.value, nu.value
        if self.total_k != self.table.total_k:
            raise _lib.CodecError(f"plan total_k {self.total_k} != table {self.table.total_k}")
        if self.n_units != self.table.n_units:
            raise _lib.CodecError(f"plan n_units {self.n_units} != table {self.table.n_units}")
        # every segment keeps all its elements: the library's dense codec (indices implied, never materialised
        # unless a caller passes a buffer for them); at ratio 1 (the wire's "dense" updates) the encoded buffers
        # carry no idx / starts by default
        segs = self.table.segs
        self.dense = bool(len(segs)) and bool((segs[:, 1] == segs[:, 2]).all())
        self.implied_idx = self.dense and getattr(self.table, "ratio", None) is not None and self.table.ratio >= 1.0

    @classmethod
    def from_segments(cls, segs, bits=8, device=None):
        """Plan over explicit coalac_seg_t rows (in_off, n, k, out_off), offsets absolute: e.g. a
        contiguous slice of a SegmentTable, whose results land in the buffers of the whole table
        (SplitPipeline's segment ranges of one update). mn / scale of such a plan are indexed by row of
        `segs`."""
        return cls(None, None, bits, device=device, table=SubTable(segs))

    # -- lifetime ---------------------------------------------------------------------------------
    def close(self):
        h, self._h = getattr(self, "_h", None), None
        if h is not None and h.value:
            with torch.cuda.device(self.device):
                self._lib.coalac_plan_destroy(h)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- buffers ----------------------------------------------------------------------------------
    @property
    def n_segments(self):
        return self.table.n_segments

    @property
    def vals_dtype(self):
        return torch.float32 if self.bits == RAW_BITS else torch.uint8

    def empty_flat(self):
        return torch.empty(self.span, dtype=torch.float32, device=self.device)

    def empty_encoded(self, with_idx=None):
        """The five output buffers of an encode as views of ONE allocation (16-byte aligned each). with_idx
        (default: not implied_idx): False leaves idx empty and ustart None (ratio 1: the indices are implied)."""
        if with_idx is None:
            with_idx = not self.implied_idx
        if not with_idx:
            vb = 4 if self.bits == RAW_BITS else 1
            T = self.n_segments
            buf = torch.empty((vb * self.total_k + 15) // 16 * 16 + 8 * T, dtype=torch.uint8, device=self.device)
            o = (vb * self.total_k + 15) // 16 * 16
            return Encoded(torch.empty(0, dtype=torch.int32, device=self.device), buf[:vb * self.total_k].view(self.vals_dtype),
                           buf[o:o + 4 * T].view(torch.float32), buf[o + 4 * T:o + 8 * T].view(torch.float32), None)
        geo = self.__dict__.get("_enc_geometry")
        if geo is None:
            K, T, U = self.total_k, self.n_segments, self.n_units
            vb = 4 if self.bits == RAW_BITS else 1
            views, o = [], 0
            dts = (torch.int32, self.vals_dtype, torch.float32, torch.float32, torch.int32)
            for nbytes, dt in zip((4 * K, vb * K, 4 * T, 4 * T, 4 * U), dts):
                views.append((o, nbytes, dt))
                o = (o + nbytes + 15) // 16 * 16
            geo = self._enc_geometry = (max(o, 16), tuple(views))
        buf = torch.empty(geo[0], dtype=torch.uint8, device=self.device)
        return Encoded(*[buf[a:a + n].view(dt) for a, n, dt in geo[1]])

    def empty_workspace(self):
        return torch.empty(self.ws_bytes, dtype=torch.uint8, device=self.device)

    # -- checks -----------------------------------------------------------------------------------
    def _check_flat(self, t, name, need=None):
        if t is None:
            return
        need = self.span if need is None else need
        if t.device != self.device or t.dtype != torch.float32 or not t.is_contiguous():
            raise ValueError(f"{name}: need a contiguous float32 tensor on {self.device}, got "
                             f"{t.dtype} on {t.device} (contiguous={t.is_contiguous()})")
        if t.numel() < need:
            raise ValueError(f"{name}: {t.numel()} elements < required {need}")
        if t.data_ptr() % 16:
            raise ValueError(f"{name}: storage must be 16-byte aligned")

    def _check_encoded(self, e):
        """Dtype, device, contiguity and length of every encoded buffer; returns the ustart pointer to pass (its
        length must be exactly the plan's unit count: a buffer of another layout is an error, not a hint)."""
        want = ((e.idx, torch.int32, 0 if self.dense and e.idx.numel() == 0 else self.total_k),
                (e.vals, self.vals_dtype, self.total_k),
                (e.mn, torch.float32, self.n_segments), (e.scale, torch.float32, self.n_segments))
        if e.ustart is not None:
            want += ((e.ustart, torch.int32, self.n_units),)
            if e.ustart.numel() != self.n_units:
                raise ValueError(f"encoded ustart: {e.ustart.numel()} entries, the plan has {self.n_units} units")
        for t, dt, n in want:
            if t.device != self.device or t.dtype != dt or not t.is_contiguous() or t.numel() < n:
                raise ValueError(f"encoded buffer mismatch: need {dt}[{n}] on {self.device}, got "
                                 f"{t.dtype}[{t.numel()}] on {t.device}")
        return _ptr(e.ustart)

    # -- codec ------------------------------------------------------------------------------------
    def encode(self, flat, base=None, out=None, workspace=None, flags=0, stream=None, events=None):
        """Encode flat (fp32[span]) [- base] -> Encoded. Asynchronous on `stream`.

        events: 5 timing events recorded at the kernel boundaries (coalac_encode_ev)."""
        self._check_flat(flat, "input")
        self._check_flat(base, "base")
        with _on(stream):
            out = self.empty_encoded() if out is None else out
            ws = self.empty_workspace() if workspace is None else workspace
        ust = self._check_encoded(out)
        if ws.device != self.device or ws.numel() * ws.element_size() < self.ws_bytes:
            raise ValueError(f"workspace: need {self.ws_bytes} bytes on {self.device}")
        args = (self._h, _ptr(flat), _ptr(base), _idx_ptr(out.idx), _ptr(out.vals), _ptr(out.mn),
                _ptr(out.scale), ust, _ptr(ws), ctypes.c_uint64(self.ws_bytes), ctypes.c_uint(flags),
                _stream_handle(stream))
        with torch.cuda.device(self.device):
            if events is None:
                rc = self._lib.coalac_encode(*args)
            else:
                rc = self._lib.coalac_encode_ev(*args, _event_array(events, 5))
        _lib.check(rc, "coalac_encode")
        return out

    def segment_pointers(self, tensors, checked=False, ptrs=None, stream=None):
        """Device array of the tensors' data pointers (one per segment), for encode_segments; cached per
        pointer tuple (a model's parameter storage does not move between rounds). checked: the caller has
        verified device, dtype, contiguity, alignment and sizes (UpdateCodec.encode); ptrs: their data
        pointers, if the caller has them. The array is marked as in use by `stream` (the launch stream), so
        an eviction from the cache never hands its memory to other work while a kernel still reads it."""
        segs = self.table.segs
        if len(tensors) != len(segs):
            raise ValueError(f"need {len(segs)} segment tensors, got {len(tensors)}")
        for i, t in enumerate(() if checked else tensors):
            if t.device != self.device or t.dtype != torch.float32 or not t.is_contiguous():
                raise ValueError(f"segment {i}: need a contiguous float32 tensor on {self.device}")
            if t.numel() != int(segs[i, 1]):
                raise ValueError(f"segment {i}: {t.numel()} elements, the plan says {int(segs[i, 1])}")
            if t.data_ptr() % 16:
                raise ValueError(f"segment {i}: storage must be 16-byte aligned")
        key = ptrs if ptrs is not None else tuple(t.data_ptr() for t in tensors)
        st = torch.cuda.current_stream(self.device) if stream is None else stream
        last = self.__dict__.get("_segptr_last")  # the same pointer tuple object on the same stream: no hashing
        if last is not None and last[0] is key and last[2] == st:
            return last[1]
        cache = self.__dict__.setdefault("_segptr_cache", {})
        d = cache.get(key)
        if d is None:
            if len(cache) >= 8:  # LRU-ish: drop the oldest entry (dicts keep insertion order)
                cache.pop(next(iter(cache)))
            with torch.cuda.stream(st):
                d = torch.tensor(key, dtype=torch.int64).to(self.device, non_blocking=False)
            cache[key] = (d, st)
        else:
            d, home = d
            if home != st:
                d.record_stream(st)
        self._segptr_last = (key, d, st)
        return d

    def encode_segments(self, tensors, base=None, out=None, workspace=None, flags=0, stream=None, checked=False,
                        ptrs=None, launch=None):
        """Encode with segment i read from tensors[i] itself (coalac_encode_segptr): e.g. a model's
        parameters, no flattening copy. base: flat fp32[span] (delta mode), as encode(). launch: the current
        stream when stream is None, if the caller already has it."""
        if launch is None:
            launch = torch.cuda.current_stream(self.device) if stream is None else stream
        ptrs = self.segment_pointers(tensors, checked=checked, ptrs=ptrs, stream=launch)
        self._check_flat(base, "base")
        mine = out is None  # (buffers this call allocates need no checking)
        with _on(stream):
            out = self.empty_encoded() if out is None else out
            ws = self.empty_workspace() if workspace is None else workspace
        ust = _ptr(out.ustart) if mine else self._check_encoded(out)
        if ws.device != self.device or ws.numel() * ws.element_size() < self.ws_bytes:
            raise ValueError(f"workspace: need {self.ws_bytes} bytes on {self.device}")
        with _device_ctx(self.device):
            rc = self._lib.coalac_encode_segptr(self._h, _ptr(ptrs), _ptr(base), _idx_ptr(out.idx), _ptr(out.vals),
                                                _ptr(out.mn), _ptr(out.scale), ust, _ptr(ws),
                                                ctypes.c_uint64(self.ws_bytes), ctypes.c_uint(flags),
                                                ctypes.c_void_p(launch.cuda_stream))
        _lib.check(rc, "coalac_encode_segptr")
        return out

    def unit_starts(self, idx, stream=None):
        """The per-unit starts (wire v2) of this plan's idx list, computed on the device for a payload that carries
        none (a version-1 blob, or an Encoded built without them): for unit j of segment s, the number of the
        segment's kept indices below j * 4096 — one searchsorted over the entries' global unit numbers, which are
        non-decreasing across the plan (segments in order, indices ascending). An unsorted (untrusted) list gives
        wrong but in-range starts; the decode kernels clamp them to their unit."""
        aux = self.__dict__.get("_starts_aux")
        if aux is None:
            segs = self.table.segs.astype("int64")
            n, k, oo = segs[:, 1], segs[:, 2], segs[:, 3]
            nu = (n + UNIT - 1) // UNIT
            ubase = torch.from_numpy((nu.cumsum() - nu).astype("int32"))
            kk, nnu = torch.from_numpy(k), torch.from_numpy(nu)
            first = torch.from_numpy((k.cumsum() - k).astype("int32"))  # each segment's first entry in the plan's list
            ents = None
            if not (oo == (k.cumsum() - k)).all():  # (a SubTable: the segments' entries sit at absolute offsets)
                ents = torch.cat([torch.arange(int(o), int(o) + int(c), dtype=torch.int64) for o, c in zip(oo, k)])
            aux = self._starts_aux = (torch.repeat_interleave(ubase, kk).to(self.device),
                                      torch.repeat_interleave(first, nnu).to(self.device),
                                      torch.arange(int(nu.sum()), dtype=torch.int32).to(self.device),
                                      None if ents is None else ents.to(self.device))
        ubase_rep, first_rep, units, ents = aux
        with _on(stream):
            own = idx[:self.total_k] if ents is None else idx[ents]
            gu = ubase_rep + torch.bitwise_right_shift(own, 12)
            return (torch.searchsorted(gu, units, out_int32=True) - first_rep).to(torch.int32)

    def _starts_for(self, enc, stream):
        """enc.ustart, or (no starts, a sparse plan) the device-computed ones."""
        if enc.ustart is not None or self.dense:
            return enc
        return Encoded(enc.idx, enc.vals, enc.mn, enc.scale, self.unit_starts(enc.idx, stream))

    def decode(self, enc, base=None, out=None, stream=None, events=None):
        """Decode Encoded -> dense flat fp32[span] (+ base, fused). Asynchronous on `stream`.

        enc.ustart: the wire v2 per-unit starts; without them (a v1 payload) they are computed on the device first
        (unit_starts). events: 3 timing events (coalac_decode_ev: [1] / [2] bracket the decode kernel)."""
        self._check_encoded(enc)
        enc = self._starts_for(enc, stream)
        ust = self._check_encoded(enc)
        self._check_flat(base, "base")
        with _on(stream):
            if out is None:
                out = self.empty_flat() if base is None else torch.empty_like(base)
        self._check_flat(out, "output")
        args = (self._h, _idx_ptr(enc.idx), _ptr(enc.vals), _ptr(enc.mn), _ptr(enc.scale), ust, _ptr(base), _ptr(out),
                _stream_handle(stream))
        with torch.cuda.device(self.device):
            if events is None:
                rc = self._lib.coalac_decode(*args)
            else:
                rc = self._lib.coalac_decode_ev(*args, _event_array(events, 3))
        _lib.check(rc, "coalac_decode")
        return out

    def aggregate(self, enc, weights, total=None, base=None, out=None, mode="recip", stream=None, events=None,
                  avg_mask=None):
        """Fused decode + FedAvg of the plan's `clients` updates (coalac_aggregate).

        enc: the batched Encoded of all clients (client-major, as encode() produces). weights: one
        number per client (FedAvg weights, e.g. sample counts); total: their sum (default
        sum(weights)). Returns out fp32[span_per_client] indexed like client 0's segments:
        base + decoded_i averaged exactly as coala/server/strategies.py:6-29,57-90 would on the decoded
        modules — mode "recip" reproduces torch on the GPU (division by a host scalar becomes a multiply
        by its fp32 reciprocal), "div" torch on the CPU, "sum" stops before the division (weighted_sum,
        strategies.py:57-90: what a multi-GPU server hands to reduce_models, distributed.py:42-57).
        avg_mask: one bool per segment of a client (None: all True); a False segment is not averaged but
        takes client 0's decoded value — aggregation_content "parameters" (strategies.py:32-54, 93-124).
        enc.ustart: the clients' per-unit starts, concatenated (computed on the device when absent).
        """
        self._check_encoded(enc)
        if not getattr(self.table, "uniform", False):
            raise ValueError("fused aggregation needs a plan over copies of one layout (a SegmentTable)")
        if self.dense and enc.idx.numel() == 0:  # (the aggregate kernel reads explicit indices: the implied ones and
            with _on(stream):                      # the implied starts, both made once per plan)
                enc = Encoded(self.implied_indices(), enc.vals, enc.mn, enc.scale,
                              self.implied_starts() if enc.ustart is None else enc.ustart)
        if enc.ustart is None:
            enc = Encoded(enc.idx, enc.vals, enc.mn, enc.scale, self.unit_starts(enc.idx, stream))
        ust = self._check_encoded(enc)
        C = self.table.clients
        if len(weights) != C:
            raise ValueError(f"need {C} weights, got {len(weights)}")
        modes = {"recip": _lib.COALAC_AGG_RECIP, "div": _lib.COALAC_AGG_DIV, "sum": _lib.COALAC_AGG_SUM}
        if mode not in modes:
            raise ValueError(f"mode must be one of {sorted(modes)}, got {mode!r}")
        n_out = self.table.span_per_client
        if base is not None:
            self._check_flat(base, "base", n_out)
        with _on(stream):
            out = torch.empty(n_out, dtype=torch.float32, device=self.device) if out is None else out
            w = torch.tensor([float(x) for x in weights], dtype=torch.float64).to(torch.float32).to(self.device)
            m = None
            if avg_mask is not None:
                if len(avg_mask) != len(self.table.sizes):
                    raise ValueError(f"avg_mask: need {len(self.table.sizes)} entries, got {len(avg_mask)}")
                m = torch.tensor([1 if x else 0 for x in avg_mask], dtype=torch.uint8).to(self.device)
        # (the kernel writes the segments' elements only: an output that ends with the last segment suffices,
        # e.g. a decoded module's buffer, which has no trailing alignment pad)
        self._check_flat(out, "output", self.table.offsets[-1] + self.table.sizes[-1] if self.table.sizes else 0)
        total = float(sum(weights)) if total is None else float(total)
        args = (self._h, C, _ptr(enc.idx), _ptr(enc.vals), _ptr(enc.mn), _ptr(enc.scale), ust, _ptr(w),
                ctypes.c_float(total), modes[mode], _ptr(m), _ptr(base), _ptr(out), _stream_handle(stream))
        with torch.cuda.device(self.device):
            if events is None:
                rc = self._lib.coalac_aggregate(*args)
            else:
                rc = self._lib.coalac_aggregate_ev(*args, _event_array(events, 3))
        _lib.check(rc, "coalac_aggregate")
        return out  # w / m were allocated on the launch stream: their memory is reused only after the kernel

    def implied_indices(self):
        """A dense plan's indices (0..n-1 per segment, every client) as a device int32 tensor, made once."""
        t = self.__dict__.get("_implied")
        if t is None:
            one = torch.cat([torch.arange(n, dtype=torch.int32) for n in self.table.segs[:, 1].tolist()])
            t = self._implied = one.to(self.device)
        return t

    def implied_starts(self):
        """A dense plan's per-unit starts (unit j of a segment starts at entry 4096 j: every element is kept), every
        client, as a device int32 tensor, made once (recomputed by a device searchsorted per call)."""
        t = self.__dict__.get("_implied_starts")
        if t is None:
            one = torch.cat([torch.arange(0, n, UNIT, dtype=torch.int32) for n in self.table.segs[:, 1].tolist()])
            t = self._implied_starts = one.to(self.device)
        return t

    def fallbacks(self, workspace, stream=None):
        """Segments of the last encode with this workspace whose sampled bracket missed (synchronises)."""
        c = ctypes.c_int()
        with torch.cuda.device(self.device):
            _lib.check(self._lib.coalac_workspace_fallbacks(self._h, _ptr(workspace), _stream_handle(stream),
                                                            ctypes.byref(c)), "coalac_workspace_fallbacks")
        return c.value


def _event_array(events, n):
    """torch.cuda.Event list -> void*[n] of hipEvent_t (events must have been recorded once or be
    created with enable_timing; torch creates the HIP event lazily on first record)."""
    arr = (ctypes.c_void_p * n)()
    for i, e in enumerate(events[:n]):
        if e is not None:
            arr[i] = ctypes.c_void_p(e.cuda_event)
    return arr
