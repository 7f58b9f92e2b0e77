"""Update codec over state_dicts: flatten -> HIP encode -> picklable carrier -> HIP decode -> module.

This is the host-side mirror of what COALA's empty compression package would provide
(/root/reference/coala/compression/__init__.py is 0 bytes). What the reference DOES pin, and this module
honours:
  * the carrier is whatever object the hook leaves in `self.model`; the reference deep-copies it and
    pickles it into UploadContent.data (/root/reference/coala/client/base.py:363,
    /root/reference/coala/protocol/codec.py:4-9), so CompressedUpdate pickles to a compact blob;
  * the server hands the decoded object to FedAvg, which iterates `state_dict()` of full modules
    including int64 `num_batches_tracked` buffers (/root/reference/coala/server/strategies.py:57-90),
    so decode returns a full nn.Module; non-fp32 entries travel raw (passthrough);
  * `calculate_model_size` calls `.parameters()` on whatever is in `self.model`
    (/root/reference/coala/client/base.py:155,474-487), so the carrier has a parameters() that reports
    its real payload size.
"""
import copy
import math
import sys
import threading
from collections import OrderedDict
from collections.abc import Mapping
from itertools import chain, repeat
from operator import attrgetter, is_, itemgetter

import ctypes

import numpy as np
import torch
from torch import nn

from . import _lib, wire
from .plan import CodecPlan, Encoded
from .spec import ALIGN, RAW_BITS, UNIT, VALID_BITS, SegmentTable, align_up, k_for

MODES = ("delta", "weights")


class HipBackend:
    """Default backend: hand-written HIP kernels behind the C ABI (coala_amd/csrc/coalac.hip)."""

    name = "hip"

    def default_device(self):
        return torch.device("cuda", torch.cuda.current_device())

    def runs_on(self, device):
        return torch.device(device).type == "cuda"

    def make_plan(self, sizes, ratio, bits, device, clients=1):
        if device.type != "cuda":
            raise RuntimeError(f"the HIP codec runs on GPU tensors only; got tensors on {device} "
                               "(there is no CPU fallback)")
        return CodecPlan(sizes, ratio, bits, clients=clients, device=device)

    def gather_scalars(self, ts, described=None):
        """One contiguous copy of the one-element tensors ts (one dtype, one GPU) in a single launch
        (coalac_gather), or None when they do not qualify (the caller then stacks them with torch).
        described: the _Described these tensors came from (their pointers; the checks run once per layout)."""
        t0 = ts[0]
        if described is not None and described.raw_ok is False:
            return None
        if t0.device.type != "cuda":
            return None
        dev, size = t0.device, t0.element_size()
        if size not in (1, 2, 4, 8):  # (coalac_gather copies 1/2/4/8-byte elements; complex128 is stacked)
            return None
        ptrs = tuple(map(_data_ptr, ts)) if described is None else described.raw_ptrs
        if described is None or described.raw_ok is None:
            ok = list(map(_get_device, ts)) == [dev.index] * len(ts) and not any(p % size for p in ptrs)
            if described is not None:
                described.raw_ok = ok
            if not ok:
                return None
        cache = self.__dict__.setdefault("_gather_ptrs", OrderedDict())
        d = cache.get(ptrs)
        if d is None:
            d = torch.tensor(ptrs, dtype=torch.int64).to(dev)
            cache[ptrs] = d
            while len(cache) > 16:
                cache.popitem(last=False)
        st = torch.cuda.current_stream(dev)
        d.record_stream(st)  # (an eviction from the cache never hands its memory to a kernel still reading it)
        out = torch.empty(len(ts), dtype=t0.dtype, device=dev)
        lib = _lib.load()
        _lib.check(lib.coalac_gather(ctypes.c_void_p(d.data_ptr()), len(ts), size, ctypes.c_void_p(out.data_ptr()),
                                     ctypes.c_void_p(st.cuda_stream)), "coalac_gather")
        return out


class FlatState:
    """A state_dict split into one aligned flat fp32 buffer (segments) plus raw passthrough entries."""

    def __init__(self, entries, flat, raw):
        self.entries = entries  # list of dicts: name, dtype, shape, kind, (seg, off, n) | ()
        self.flat = flat        # fp32 [span] on device (None if no fp32 entry)
        self.raw = raw          # OrderedDict name -> tensor
        self._on = {}           # device -> flat copy (a snapshot taken on one device, used on another)

    def flat_on(self, device):
        """The flat buffer on `device` (copied once per device and cached: the w_global snapshot of a
        round is immutable)."""
        if self.flat is None or self.flat.device == torch.device(device):
            return self.flat
        key = str(device)
        t = self._on.get(key)
        if t is None:
            t = self.flat.to(device)
            self._on[key] = t
        return t


def layout_of(state):
    """[(name, dtype str, shape)] of a state_dict — what must match between encoder and decoder."""
    return [(k, str(v.dtype).replace("torch.", ""), tuple(v.shape)) for k, v in state.items()]


_DTYPE_NAMES = {}


def _dtype_name(dt):
    n = _DTYPE_NAMES.get(dt)
    if n is None:
        n = _DTYPE_NAMES[dt] = str(dt).replace("torch.", "")
    return n


class _Layout:
    """The header entries of one state_dict layout (the (name, dtype, shape) sequence) and the names of its
    fp32 segments / raw passthrough entries. Built once per layout: a model's layout is fixed for a whole FL
    task, and the per-entry Python of building them was most of a ResNet-50 encode call's host time. The
    entries are shared by every header of that layout and never mutated."""

    def __init__(self, items):
        self.entries, self.seg_names, self.raw_names = [], [], []
        self.seg_idx, self.raw_idx = [], []
        off = seg = 0
        for i, (name, dt, shape) in enumerate(items):
            n = 1
            for d in shape:
                n *= d
            e = {"name": name, "dtype": _dtype_name(dt), "shape": list(shape)}
            if dt == torch.float32 and n > 0:
                e.update(kind="seg", seg=seg, off=off, n=n)
                self.seg_names.append(name)
                self.seg_idx.append(i)
                off = align_up(off + n)
                seg += 1
            else:
                e["kind"] = "raw"
                self.raw_names.append(name)
                self.raw_idx.append(i)
            self.entries.append(e)
        self.sizes = [e["n"] for e in self.entries if e["kind"] == "seg"]
        self.sizes_key = tuple(self.sizes)
        # the passthrough entries as one group when they are all scalars of one dtype (BatchNorm counters)
        raw_items = [items[i] for i in self.raw_idx]
        self.raw_scalars = (None if not raw_items or any(len(sh) for _, _, sh in raw_items)
                            or len({dt for _, dt, _ in raw_items}) != 1
                            else [(n, (), 1) for n, _, _ in raw_items])


_LAYOUTS = OrderedDict()
_LAYOUTS_LOCK = threading.Lock()


def _layout(state):
    return _layout_sig(tuple((k, v.dtype, v.shape) for k, v in state.items()))


def _layout_sig(sig):
    with _LAYOUTS_LOCK:
        L = _LAYOUTS.get(sig)
        if L is None:
            L = _LAYOUTS[sig] = _Layout(sig)
            while len(_LAYOUTS) > 16:
                _LAYOUTS.popitem(last=False)
    return L


_MOD_TABLES = itemgetter("_parameters", "_buffers", "_modules", "_non_persistent_buffers_set")


class _StateWalk:
    """The tensors of a module's state_dict, in state_dict order, without building the state_dict: the
    module tree walked once (pre-order, as Module.state_dict recurses), then per call each module's
    parameter and persistent-buffer tables read in place (no per-entry detach, no prefix strings, no
    state-dict hooks: the reference's models register none). Re-walked when a table's size changes, when a
    table object or a submodule is replaced (each module's children are compared by identity: a client that
    keeps one root module across rounds may swap `model.head`), or when the non-persistent buffer set changes.
    The per-call checks and the gather run as C-level maps over the modules' __dict__ tables (a Python loop
    over ResNet-50's 161 modules cost more than the encode's own launches)."""

    def __init__(self, module):
        self.mods, names = [], []
        srcs, keys = [], []  # per state entry: the table it lives in, its key
        self.parents, self.npbs = [], []  # (module, children) of the modules with children; (module, set) likewise
        self.hooked = False
        for prefix, m in module.named_modules(remove_duplicate=False):
            self.hooked = self.hooked or bool(m._state_dict_hooks or m._state_dict_pre_hooks)
            pn = tuple(k for k, v in m._parameters.items() if v is not None)
            bn = tuple(k for k, v in m._buffers.items() if v is not None and k not in m._non_persistent_buffers_set)
            self.mods.append(m)
            srcs.extend([m._parameters] * len(pn) + [m._buffers] * len(bn))
            keys.extend(pn + bn)
            if m._modules:
                self.parents.append((m, tuple(m._modules.values())))
            if m._non_persistent_buffers_set:
                self.npbs.append((m, frozenset(m._non_persistent_buffers_set)))
            p = prefix + "." if prefix else ""
            names.extend(p + k for k in pn + bn)
        self.dicts = [m.__dict__ for m in self.mods]
        self.tables = self._tables()           # every module's 4 table objects, flattened
        self.sizes = list(map(len, self.tables))
        self.kid_dicts = [m._modules for m, _ in self.parents]
        self.kids = [kids for _, kids in self.parents]
        self.srcs, self.keys = srcs, keys
        self.names = tuple(names)
        self.last = None  # _Described: the last describe_tensors of these tensors

    def _tables(self):
        return list(chain.from_iterable(map(_MOD_TABLES, self.dicts)))

    def tensors(self):
        """The tensors, or None when the tree changed since the walk (a table's size or object, a replaced or
        added submodule, the non-persistent buffer set): the caller walks again."""
        tables = self._tables()
        if list(map(len, tables)) != self.sizes or not all(map(is_, tables, self.tables)):
            return None
        if list(map(tuple, map(dict.values, self.kid_dicts))) != self.kids:  # (identity first: a swap is unequal)
            return None
        for m, npb in self.npbs:
            if m._non_persistent_buffers_set != npb:
                return None
        return list(map(dict.__getitem__, self.srcs, self.keys))


class _Described:
    """describe_tensors' result for one list of tensors: reused while the same tensor objects sit at the same
    storage (a dtype or shape change of a tensor in place moves its storage; a reshape of a parameter's .data
    that keeps its storage start is not looked for)."""

    __slots__ = ("tensors", "ptrs", "L", "seg_ptrs", "raw_ptrs", "raw_ok")

    def __init__(self, tensors, ptrs, L):
        self.tensors, self.ptrs, self.L = tensors, ptrs, L
        self.seg_ptrs = tuple(ptrs[i] for i in L.seg_idx)
        self.raw_ptrs = tuple(ptrs[i] for i in L.raw_idx)
        self.raw_ok = None  # the gather's own checks of the raw scalars, once


_WALKS = {}  # id(module) -> (weakref, _StateWalk)


def module_tensors(module):
    """(names, tensors) of module.state_dict() — the same names and tensor storage, in the same order — via a
    cached _StateWalk. A module tree with state-dict hooks takes state_dict() itself."""
    return _module_walk(module)[:2]


def _module_walk(module):
    """module_tensors' (names, tensors) and the walk (None when state_dict() was taken)."""
    if module._state_dict_hooks or module._state_dict_pre_hooks:
        st = module.state_dict()
        return tuple(st), list(st.values()), None
    hit = _WALKS.get(id(module))
    w = hit[1] if hit is not None and hit[0]() is module else None
    ts = w.tensors() if w is not None else None
    if ts is None:  # first call, another module at this id, or a table changed size: walk again
        import weakref
        w = _StateWalk(module)
        with _LAYOUTS_LOCK:
            _WALKS[id(module)] = (weakref.ref(module), w)
            if len(_WALKS) > 64:
                for k in [k for k, (r, _) in _WALKS.items() if r() is None]:
                    del _WALKS[k]
        ts = w.tensors()
    if w.hooked:
        st = module.state_dict()
        return tuple(st), list(st.values()), None
    return w.names, ts, w


_get_dtype, _get_shape = attrgetter("dtype"), attrgetter("shape")


def describe_tensors(names, tensors, walk=None, gather=None):
    """describe_state() over (names, tensors) in state_dict order (module_tensors). walk: the _StateWalk the
    tensors came from — the layout is then reused while the same tensor objects sit at the same storage (see
    _Described), instead of reading every tensor's dtype and shape. gather: a backend's one-launch copy of
    one-element tensors (HipBackend.gather_scalars) for the passthrough scalars."""
    d, segs = _layout_walk(names, tensors, walk)
    return d.L, segs, _raw_snapshot(d, tensors, gather)


def _layout_walk(names, tensors, walk):
    """(_Described, fp32 segment tensors) of the tensors: the layout part of describe_tensors."""
    ptrs = tuple(map(_data_ptr, tensors))
    d = walk.last if walk is not None else None
    if d is None or d.ptrs != ptrs or not all(map(is_, tensors, d.tensors)):
        dts, shs = list(map(_get_dtype, tensors)), list(map(_get_shape, tensors))
        d = _Described(tensors, ptrs, _layout_sig(tuple(zip(names, dts, shs))))
        if walk is not None:
            walk.last = d
    return d, list(map(tensors.__getitem__, d.L.seg_idx))


def _raw_snapshot(d, tensors, gather):
    """The passthrough entries' RawState: one gather launch for a group of scalars of one dtype."""
    L = d.L
    raw_ts = list(map(tensors.__getitem__, L.raw_idx))
    raw = None
    if L.raw_scalars is not None:
        flat = gather(raw_ts, d) if gather is not None else None
        if flat is not None:
            raw = RawState([(flat, L.raw_scalars)], L.raw_names)
        else:
            try:
                with torch.no_grad():  # one stack of the scalar counters: no per-entry checks
                    raw = RawState([(torch.stack(raw_ts), L.raw_scalars)], L.raw_names)
            except RuntimeError:  # (counters on several devices)
                raw = None
    if raw is None:
        raw = RawState.snapshot(list(zip(L.raw_names, raw_ts)))
    return raw


def describe_state(state):
    """state_dict -> (entries as flatten_state would write them, fp32 segment tensors in order, raw
    passthrough entries), WITHOUT copying the fp32 data: the zero-copy encode reads the tensors in place."""
    L, segs, raw = _describe(state)
    return L.entries, segs, raw


def _describe(state):
    L = _layout(state)
    segs = [state[n] for n in L.seg_names]  # read in place by the kernels (pointer, numel, dtype, contiguity)
    return L, segs, RawState.snapshot([(n, state[n]) for n in L.raw_names])


_data_ptr, _is_contig, _get_device = torch.Tensor.data_ptr, torch.Tensor.is_contiguous, torch.Tensor.get_device


_PACKED_HEADERS = OrderedDict()  # (layout entries id, fields, raw sizes) -> (entries, header JSON bytes)


def _to_host(*ts):
    """numpy copies of tensors, with ONE device-to-host transfer when they live on a GPU."""
    if not ts or ts[0].device.type == "cpu":
        return [t.numpy() for t in ts]
    parts = [t.contiguous().view(torch.uint8).reshape(-1) for t in ts]
    host = torch.cat(parts).cpu().numpy()
    out, o = [], 0
    for t, p in zip(ts, parts):
        n = p.numel()
        out.append(host[o:o + n].view(_NP_DTYPES[t.dtype]))
        o += n
    return out


_NP_DTYPES = {torch.float32: np.float32, torch.int32: np.int32, torch.uint8: np.uint8, torch.int64: np.int64}
# the dtypes a passthrough entry of a blob may name (a state_dict's non-fp32 or empty entries); a blob naming
# anything else is rejected rather than handed to getattr(torch, ...)
_RAW_DTYPES = {_dtype_name(d): d for d in (torch.float32, torch.float64, torch.float16, torch.bfloat16, torch.int64,
                                          torch.int32, torch.int16, torch.int8, torch.uint8, torch.bool,
                                          torch.complex64, torch.complex128)}


class RawState(Mapping):
    """The passthrough (non-fp32) entries of an update — BatchNorm's int64 num_batches_tracked and the like —
    held as ONE flat tensor per (dtype, device) with the entries' names and shapes, in state order. Taking
    the snapshot is one copy kernel per group (not one per entry); the per-entry tensors are views made on
    first access (one unbind / split call per group). A read-only mapping name -> tensor."""

    def __init__(self, groups, order):
        self._groups = groups    # [(flat, [(name, shape, numel)])]
        self._order = order      # names in state order
        self._views = None

    @classmethod
    def snapshot(cls, items):
        """Copies of (name, tensor) items taken now, grouped per (dtype, device)."""
        groups, index = [], {}
        for name, t in items:
            key = (t.dtype, t.device)
            g = index.get(key)
            if g is None:
                g = index[key] = []
                groups.append((key, g))
            g.append((name, t))
        out = []
        with torch.no_grad():
            for _, members in groups:
                ts = [t for _, t in members]
                if all(t.dim() == 0 for t in ts):
                    flat = torch.stack(ts)  # (one kernel: the usual case, scalar counters)
                else:
                    flat = torch.cat([t.reshape(-1) for t in ts])
                out.append((flat, [(n, tuple(t.shape), t.numel()) for n, t in members]))
        return cls(out, [n for n, _ in items])

    def _make_views(self, groups):
        views = {}
        for flat, members in groups:
            if all(len(shape) == 0 for _, shape, _ in members):
                views.update(zip((n for n, _, _ in members), flat.unbind()))
            else:
                for (n, shape, _), piece in zip(members, flat.split_with_sizes([m for _, _, m in members])):
                    views[n] = piece.view(shape)
        return views

    def __getitem__(self, name):
        if self._views is None:
            self._views = self._make_views(self._groups)
        return self._views[name]

    def __iter__(self):
        return iter(self._order)

    def __len__(self):
        return len(self._order)

    @property
    def nbytes(self):
        return sum(f.numel() * f.element_size() for f, _ in self._groups)

    @classmethod
    def from_entries(cls, entries, rawb):
        """From a blob's raw section: entries with "dtype", "shape", "off", "nbytes" (in state order). Runs of
        same-dtype entries stored back to back become one tensor (one copy of the bytes)."""
        groups, order, run = [], [], []

        def flush():
            if run:
                dt = _RAW_DTYPES.get(run[0]["dtype"])
                if dt is None:
                    raise ValueError(f"COALAQ1: unsupported raw entry dtype {run[0]['dtype']!r}")
                size = torch.empty(0, dtype=dt).element_size()
                members = []
                for e in run:  # every entry's byte count must match its own shape (not only the run's total)
                    m = int(np.prod(e["shape"], dtype=np.int64))
                    if m < 0 or int(e["nbytes"]) != m * size:
                        raise ValueError(f"COALAQ1: raw entry {e['name']!r}: {e['nbytes']} bytes for shape "
                                         f"{e['shape']} of {e['dtype']}")
                    members.append((e["name"], tuple(e["shape"]), m))
                lo, hi = run[0]["off"], run[-1]["off"] + run[-1]["nbytes"]
                if lo < 0 or hi > len(rawb):
                    raise ValueError("COALAQ1: raw entries past the end of the blob")
                buf = bytearray(rawb[lo:hi])
                flat = torch.frombuffer(buf, dtype=dt) if buf else torch.empty(0, dtype=dt)
                groups.append((flat, members))
                run.clear()
        for e in entries:
            if run and (e["dtype"] != run[-1]["dtype"] or e["off"] != run[-1]["off"] + run[-1]["nbytes"]):
                flush()
            run.append(e)
            order.append(e["name"])
        flush()
        return cls(groups, order)

    def entry_bytes(self):
        """{name: little-endian bytes} with one device-to-host copy per group."""
        out = {}
        for flat, members in self._groups:
            b = flat.detach().cpu().contiguous().view(torch.uint8).numpy().tobytes()
            per = flat.element_size()
            o = 0
            for n, _, m in members:
                out[n] = b[o:o + m * per]
                o += m * per
        return {n: out[n] for n in self._order}

    def fresh(self, device=None):
        """{name: tensor} with storage of its own (one copy per group, onto `device` if given): what a
        decode hands out, so decoded modules never alias the update or each other."""
        return self.fresh_groups(device)[1]

    def fresh_groups(self, device=None):
        """(the per-group flat copies, fresh()'s {name: view of them})."""
        groups = [(f.to(device, copy=True) if device is not None else f.clone(), m) for f, m in self._groups]
        views = self._make_views(groups)
        return [f for f, _ in groups], {n: views[n] for n in self._order}

    def signature(self):
        """What a copy into another RawState's group buffers needs to match: dtype, size and members per group."""
        return tuple((f.dtype, f.numel(), tuple(m)) for f, m in self._groups)


def _snapshot_raw(raw):
    """Copies of the passthrough entries taken now (RawState: one copy kernel per dtype / device)."""
    return RawState.snapshot(list(raw.items()))


def flatten_state(state, device=None):
    """state_dict -> FlatState with every fp32 entry at an ALIGN-aligned offset of one flat buffer.

    One torch.cat over the tensors and zero pads (a single device copy kernel), not one copy per entry.
    """
    entries, parts, raw = [], [], OrderedDict()
    off = seg = 0
    pad_src = None
    for name, t in state.items():
        e = {"name": name, "dtype": str(t.dtype).replace("torch.", ""), "shape": list(t.shape)}
        if t.dtype == torch.float32 and t.numel() > 0:
            if device is None:
                device = t.device
            n = t.numel()
            e.update(kind="seg", seg=seg, off=off, n=n)
            parts.append(t.detach().reshape(-1).to(device))
            pad = align_up(off + n) - (off + n)
            if pad:
                if pad_src is None:
                    pad_src = torch.zeros(ALIGN, dtype=torch.float32, device=device)
                parts.append(pad_src[:pad])
            off += n + pad
            seg += 1
        else:
            e.update(kind="raw")
            raw[name] = t.detach().clone()
        entries.append(e)
    flat = torch.cat(parts) if parts else None
    return FlatState(entries, flat, raw)


class CompressedUpdate:
    """Picklable carrier of one compressed client update (what `compression()` leaves in self.model).

    Holds the encoded buffers (device tensors right after encode; CPU tensors after unpickling) and the
    raw passthrough entries. Pickles to the COALAQ1 blob (wire.py).
    """

    def __init__(self, header, encoded, raw, blob=None):
        self.header = header
        self.encoded = encoded
        self.raw = raw
        # the packed COALAQ1 bytes, built on first pickle and shared by every deep copy: the reference
        # pickles copy.deepcopy(self.model) (client/base.py:363), so the payload is packed once
        self._blob = [blob]

    def __deepcopy__(self, memo):
        # The encoded payload is immutable after encode: a deep copy shares it (and the packed blob)
        # instead of a D2H + pack + unpack round trip through __getstate__/__setstate__.
        other = CompressedUpdate.__new__(CompressedUpdate)
        other.header = dict(self.header)  # (its "entries" list is shared and never mutated)
        other.encoded = self.encoded
        other.raw = self.raw
        other._blob = self._blob
        memo[id(self)] = other
        return other

    # -- size accounting (client/base.py:155, 474-487) -------------------------------------------
    @property
    def nbytes(self):
        h = self.header
        vb = 4 if h["bits"] == RAW_BITS else 1
        ib = 0 if h["ratio"] >= 1.0 else 4  # ratio 1: indices implied, not shipped (wire.py "dense")
        raw_b = self.raw.nbytes if isinstance(self.raw, RawState) else \
            sum(t.numel() * t.element_size() for t in self.raw.values())
        return 8 * h["n_segments"] + (ib + vb) * h["total_k"] + 4 * h.get("n_units", 0) + raw_b

    def parameters(self):
        """One meta tensor whose numel * 32 bit equals the payload size, so the reference's
        calculate_model_size reports the real upload size even without the plugin's override."""
        yield torch.empty(int(math.ceil(self.nbytes / 4)), device="meta")

    # -- wire -------------------------------------------------------------------------------------
    def to_bytes(self):
        if self._blob[0] is None:
            self._blob[0] = self._pack()
        return self._blob[0]

    def _pack(self):
        h = dict(self.header)
        raw = self.raw
        rawb = raw.entry_bytes() if isinstance(raw, RawState) else {
            n: (t.cpu().contiguous().reshape(-1).view(torch.uint8).numpy().tobytes() if t.numel() else b"")
            for n, t in raw.items()}
        # the header (with each raw entry's blob offset) depends on the layout and the raw byte counts only
        sizes = tuple(len(rawb[n]) for n in rawb)
        key = (id(h["entries"]), h["ratio"], h["bits"], h["mode"], h["n_segments"], h.get("total_k"),
               h.get("n_units"), sizes)
        hit = _PACKED_HEADERS.get(key)
        if hit is not None and hit[0] is h["entries"]:
            hjson = hit[1]
        else:
            raw_entries, pos = [], 0
            for e in h["entries"]:
                if e["kind"] == "raw":
                    nb = len(rawb[e["name"]])
                    e = dict(e, off=pos, nbytes=nb)
                    pos += nb
                raw_entries.append(e)
            h["entries"] = raw_entries
            if h["ratio"] >= 1.0:
                h["dense"] = True
            hjson = wire.encode_header(h)
            with _LAYOUTS_LOCK:
                _PACKED_HEADERS[key] = (self.header["entries"], hjson)
                while len(_PACKED_HEADERS) > 16:
                    _PACKED_HEADERS.popitem(last=False)
        enc = self.encoded
        v2 = "n_units" in h  # wire v2: the per-unit starts ride along
        arrs = _to_host(enc.mn, enc.scale, enc.idx, enc.vals, *((enc.ustart,) if v2 else ()))
        pack_h = {"dense": h["ratio"] >= 1.0}
        if v2:
            pack_h["n_units"] = h["n_units"]
        return wire.pack(pack_h, *arrs[:4], b"".join(rawb[e["name"]] for e in h["entries"] if e["kind"] == "raw"),
                         header_json=hjson, ustart=arrs[4] if v2 else None)

    def encoded_to(self, device, staging=None):
        """The encoded buffers on `device`. An unpickled update (the server side of a remote upload,
        coala/server/service.py:81-111) is moved with ONE host-to-device copy of the blob's mn / scale /
        idx / vals region through `staging` (a pinned host buffer: staging(nbytes) -> uint8 tensor), so
        the copy is asynchronous on the caller's stream; device tensors are typed views into it."""
        device = torch.device(device)
        blob = self._blob[0]
        if (staging is None or device.type != "cuda" or blob is None or self.header.get("dense")
                or self.encoded.idx.device == device):
            return self.encoded.to(device, non_blocking=True)
        _, sec = wire.sections(blob, self.header)
        lo = sec["mn"][0]
        last = sec["ustart"] if "ustart" in sec else sec["vals"]
        hi = last[0] + last[1]
        stage = staging(hi - lo)
        stage[:hi - lo].numpy()[:] = np.frombuffer(blob, dtype=np.uint8, count=hi - lo, offset=lo)
        dev = torch.empty(hi - lo, dtype=torch.uint8, device=device)
        dev.copy_(stage[:hi - lo], non_blocking=True)
        vdt = torch.float32 if self.header["bits"] == RAW_BITS else torch.uint8

        def view(name, dt):
            o, n = sec[name]
            return dev[o - lo:o - lo + n].view(dt)
        return Encoded(view("idx", torch.int32), view("vals", vdt), view("mn", torch.float32),
                       view("scale", torch.float32), view("ustart", torch.int32) if "ustart" in sec else None)

    @classmethod
    def from_bytes(cls, blob):
        h, mn, scale, idx, vals, rawb, ustart = wire.unpack(blob)
        validate(h, idx, ustart)
        raw = RawState.from_entries([e for e in h["entries"] if e["kind"] == "raw"], rawb)
        enc = Encoded(torch.from_numpy(idx.copy()), torch.from_numpy(vals.copy()),
                      torch.from_numpy(mn.copy()), torch.from_numpy(scale.copy()),
                      None if ustart is None else torch.from_numpy(ustart.copy()))
        return cls(h, enc, raw, blob=bytes(blob))

    def __getstate__(self):
        return {"blob": self.to_bytes()}

    def __setstate__(self, state):
        other = CompressedUpdate.from_bytes(state["blob"])
        self.__dict__.update(other.__dict__)

    @property
    def compression_ratio(self):
        """Dense fp32 (+ raw) bytes of the update / its payload bytes."""
        h = self.header
        dense = 4 * _dense_elements(h["entries"])
        dense += self.raw.nbytes if isinstance(self.raw, RawState) else \
            sum(t.numel() * t.element_size() for t in self.raw.values())
        return dense / max(1, self.nbytes)

    def __repr__(self):
        h = self.header
        return (f"CompressedUpdate(mode={h['mode']}, ratio={h['ratio']}, bits={h['bits']}, "
                f"segments={h['n_segments']}, kept={h['total_k']}, bytes={self.nbytes})")


_DENSE = OrderedDict()  # id(entries) -> (entries, fp32 elements)


def _dense_elements(entries):
    hit = _DENSE.get(id(entries))
    if hit is None or hit[0] is not entries:
        hit = (entries, sum(e["n"] for e in entries if e["kind"] == "seg"))
        with _LAYOUTS_LOCK:
            _DENSE[id(entries)] = hit
            while len(_DENSE) > 32:
                _DENSE.popitem(last=False)
    return hit[1]


_VALIDATED = OrderedDict()  # (id(entries), ratio, n_segments, total_k) -> (entries, ns_rep, first, units) of a layout


def validate(header, idx, ustart=None):
    """Check an (untrusted) blob's index lists: per fp32 segment, k = k_for(n, ratio) entries, strictly
    increasing, inside [0, n); and (wire v2) the per-unit starts: exactly the lower bounds of every unit's
    first element in its segment's list. The decode kernels are bounds-safe anyway; this turns a corrupt
    upload into an error instead of a silently wrong model. The header's structure is checked once per layout
    (headers of one layout share their entries list: wire._parse_header); the indices every call."""
    if header.get("bits") not in VALID_BITS or header.get("mode") not in MODES:
        raise ValueError("COALAQ1: bad bits/mode")
    entries = header["entries"]
    key = (id(entries), float(header["ratio"]), int(header["n_segments"]), int(header["total_k"]))
    hit = _VALIDATED.get(key)
    if hit is None or hit[0] is not entries:
        hit = (entries,) + _validate_layout(header)
        with _LAYOUTS_LOCK:
            _VALIDATED[key] = hit
            while len(_VALIDATED) > 32:
                _VALIDATED.popitem(last=False)
    _, ns_rep, first, units = hit
    if header.get("dense"):  # implied indices (0..n-1 per segment): nothing to check beyond the layout
        if idx.size != 0 or ustart is not None:
            raise ValueError("COALAQ1: a dense update carries no indices or starts")
        return
    if idx.size != int(header["total_k"]):
        raise ValueError("COALAQ1: kept-entry count mismatch")
    if ustart is not None and (units is None or int(header.get("n_units", -1)) != units[0].size
                               or ustart.size != units[0].size):
        raise ValueError("COALAQ1: per-unit start count mismatch")
    if ns_rep is None:
        return
    if idx.size and (int(idx.min()) < 0 or np.any(idx >= ns_rep)):
        raise ValueError("COALAQ1: index out of range")
    d = np.diff(idx, prepend=np.int32(-1))
    if np.any((d <= 0) & ~first):
        raise ValueError("COALAQ1: indices not strictly increasing")
    if ustart is not None:
        # every entry's global unit (non-decreasing, the indices being sorted per segment): a unit starts where
        # the first entry of that unit or a later one sits, relative to its segment's first entry
        unit_seg_out, unit_base_rep, arange_u = units
        gu = unit_base_rep + (idx >> 12)
        if not np.array_equal(np.searchsorted(gu, arange_u) - unit_seg_out, ustart):
            raise ValueError("COALAQ1: per-unit starts inconsistent with the indices")


def _validate_layout(header):
    segs = [e for e in header["entries"] if e["kind"] == "seg"]
    if len(segs) != int(header["n_segments"]):
        raise ValueError("COALAQ1: segment count mismatch")
    # the decoder slices its output with the offsets it derives itself (SegmentTable of the sizes); a
    # header whose own offsets / sizes disagree with that, or with the tensor shapes, is corrupt
    table = SegmentTable([e["n"] for e in segs], header["ratio"], 1) if segs else None
    for i, e in enumerate(segs):
        if int(e["seg"]) != i or int(e["n"]) != int(np.prod(e["shape"], dtype=np.int64)) or \
                int(e["off"]) != table.offsets[i]:
            raise ValueError(f"COALAQ1: segment entry {e.get('name')!r} has inconsistent seg/n/off/shape")
    ks = np.array([k_for(e["n"], header["ratio"]) for e in segs], dtype=np.int64)
    if int(ks.sum()) != int(header["total_k"]):
        raise ValueError("COALAQ1: kept-entry count mismatch")
    if not ks.size:
        return None, None, None
    ns = np.array([e["n"] for e in segs], dtype=np.int32)
    ns_rep = np.repeat(ns, ks)  # each entry's segment size
    first = np.zeros(int(ks.sum()), dtype=bool)  # each segment's first entry (no predecessor to compare)
    first[np.cumsum(ks)[:-1][ks[1:] > 0] if ks.size > 1 else []] = True
    first[0] = True
    # wire v2: per unit its segment's first entry; per entry its segment's first global unit
    nu = (ns.astype(np.int64) + UNIT - 1) // UNIT
    seg_out = np.concatenate([[0], np.cumsum(ks)[:-1]]).astype(np.int64)
    unit_base = np.concatenate([[0], np.cumsum(nu)[:-1]]).astype(np.int32)
    units = (np.repeat(seg_out, nu), np.repeat(unit_base, ks), np.arange(int(nu.sum()), dtype=np.int32))
    return ns_rep, first, units


class UpdateCodec:
    """Encode / decode model updates with CodecSpec v1.

    Args:
        ratio: top-k ratio per tensor, (0, 1].
        bits:  1..8 -> uint8 min/max codes; 32 -> raw fp32 values (lossless at ratio 1).
        mode:  "delta" encodes w_local - w_global (decode adds w_global back, fused in the kernel);
               "weights" encodes the weights themselves.
        backend: object with make_plan(sizes, ratio, bits, device); default HipBackend.
        recycle: decode_module / aggregate decode into a module this codec returned earlier once nothing
               outside the codec references it (_TreeRecipe.idle_skeleton); False builds a new module
               every call. release_pool() drops every pooled module.
    """

    def __init__(self, ratio=0.01, bits=8, mode="delta", backend=None, recycle=True):
        if not (0.0 < float(ratio) <= 1.0):
            raise ValueError(f"ratio must be in (0, 1], got {ratio}")
        if bits not in VALID_BITS:
            raise ValueError(f"bits must be one of {VALID_BITS}, got {bits}")
        if mode not in MODES:
            raise ValueError(f"mode must be one of {MODES}, got {mode}")
        self.ratio, self.bits, self.mode = float(ratio), int(bits), mode
        self.recycle = bool(recycle)
        self.backend = backend if backend is not None else HipBackend()
        self._plans = {}
        self._plan_fast = OrderedDict()  # (id(sizes), ratio, bits, clients) -> (sizes, device, plan)
        self._checked_ptrs = {}  # id(plan) -> the segment pointers of the last in-place encode that passed the checks
        self._ws = OrderedDict()
        self._lock = threading.Lock()
        self._tls = threading.local()

    def plan_for(self, sizes, device, ratio=None, bits=None, clients=1):
        # (per sizes OBJECT — a layout's cached tuple — no hash of a 161-entry tuple per hook call)
        fk = (id(sizes), ratio, bits, clients)
        hit = self._plan_fast.get(fk)
        if hit is not None and hit[0] is sizes and hit[1] == device:
            return hit[2]
        p = self._plan_for(sizes, device, ratio, bits, clients)
        with self._lock:
            self._plan_fast[fk] = (sizes, device, p)
            while len(self._plan_fast) > 32:
                self._plan_fast.popitem(last=False)
        return p

    def _plan_for(self, sizes, device, ratio, bits, clients):
        ratio = self.ratio if ratio is None else float(ratio)
        bits = self.bits if bits is None else int(bits)
        key = (tuple(sizes), ratio, bits, str(device), int(clients))
        with self._lock:
            p = self._plans.get(key)
            if p is None:
                p = self.backend.make_plan(list(sizes), ratio, bits, device, clients=clients)
                self._plans[key] = p
        return p

    @staticmethod
    def release_pool():
        """Drop every pooled decoded module (of every template): their storage is freed once their holders
        drop them too. For a server that ends training or changes its model; the pool also evicts trees
        unused for a while (_TreeRecipe.idle_skeleton) and is bounded by the device's memory."""
        release_decode_pool()

    # -- encode -----------------------------------------------------------------------------------
    def encode(self, state, base=None, device=None):
        """state_dict -> CompressedUpdate. `base` (delta mode): FlatState of w_global (same layout).
        `device`: where to flatten and encode (default: where the state lives if the backend runs there,
        else the backend's default device — a model trained on the CPU is encoded on the GPU)."""
        if device is None:
            device = self._device_for(state.values())
        L, segs, raw = _describe(state)
        return self._encode(L, segs, raw, base, device, lambda: state)

    def encode_module(self, module, base=None, device=None):
        """module -> CompressedUpdate of its state_dict (what CompressionClientMixin.compression() runs): the
        same result as encode(module.state_dict(), ...), with the state read through a cached walk of the
        module tree (module_tensors) instead of building the state_dict."""
        names, tensors, walk = _module_walk(module)
        if device is None:
            device = self._device_for(tensors)
        d, segs = _layout_walk(names, tensors, walk)
        gather = getattr(self.backend, "gather_scalars", None)
        # the passthrough snapshot is taken after the encode's launches (stream order: the same values), so
        # the GPU starts on the segments one gather launch earlier
        return self._encode(d.L, segs, lambda: _raw_snapshot(d, tensors, gather), base, device,
                            lambda: OrderedDict(zip(names, tensors)), d.seg_ptrs)

    def _encode(self, L, segs, raw, base, device, state_fn, ptrs=None):
        """raw: the RawState, or a function that takes it (called once the encode is enqueued)."""
        if self.mode == "delta" and base is None:
            raise ValueError("delta mode needs the global-model snapshot (base)")
        entries = L.entries
        sizes = L.sizes
        header = {"ratio": self.ratio, "bits": self.bits, "mode": self.mode, "n_segments": len(sizes),
                  "entries": entries}
        if not sizes:
            header["total_k"] = 0
            raw = raw() if callable(raw) else raw
            z = torch.zeros(0)
            return CompressedUpdate(header, Encoded(z.int(), z.to(torch.uint8), z, z), raw)
        device = torch.device(device)
        base_flat = None
        if self.mode == "delta":
            _check_same_layout(entries, base.entries)
            # the snapshot may have been taken where the global model arrived (the reference client's
            # set_model runs before pretrain moves the model to its device, client/base.py:138 vs :245)
            base_flat = base.flat_on(device)
        plan = self.plan_for(L.sizes_key, device)
        cur = torch.cuda.current_stream(device) if device.type == "cuda" else None  # (looked up once per call)
        ws = self._workspace(plan, cur)
        dev_index = device.index if device.type == "cuda" else -1  # (Tensor.get_device(): -1 on the CPU)
        in_place = getattr(plan, "encode_segments", None) is not None
        if in_place:  # every segment on the plan's device, contiguous, 16-B aligned (one pass per property)
            if ptrs is None:
                ptrs = tuple(map(_data_ptr, segs))
            # (the same storage as an encode that passed the checks: a model's parameters do not move between
            # rounds; contiguity is re-read every call — a parameter re-strided in place keeps its start,
            # `p.data = p.data.t()`, and would otherwise be read in storage order)
            last = self._checked_ptrs.get(id(plan))
            if (last is ptrs or last == ptrs) and not all(map(_is_contig, segs)):
                self._checked_ptrs.pop(id(plan), None)
                last = None
            if last is not ptrs and last != ptrs:
                in_place = (all(map(_is_contig, segs)) and list(map(_get_device, segs)) == [dev_index] * len(segs)
                            and not any(p & 15 for p in ptrs))
                if in_place:
                    self._checked_ptrs[id(plan)] = ptrs
        if in_place:  # read the parameters where they live: no flattening copy (+8 B/element of traffic)
            # (dtype and sizes hold by construction: the plan was made from this layout's segments)
            enc = plan.encode_segments(segs, base=base_flat, workspace=ws, checked=True, ptrs=ptrs, launch=cur)
        else:
            fs = flatten_state(state_fn(), device=device)
            enc = plan.encode(fs.flat, base=base_flat, workspace=ws)
        header["total_k"] = int(plan.table.total_k)
        if enc.ustart is not None and self.ratio < 1.0:  # wire v2 (a dense download implies its starts)
            header["n_units"] = int(plan.table.n_units)
        return CompressedUpdate(header, enc, raw() if callable(raw) else raw)

    def _thread_stream(self, device):
        """One HIP stream per (thread, device): concurrent decodes from several threads overlap on the GPU
        instead of queueing on one stream."""
        streams = getattr(self._tls, "streams", None)
        if streams is None:
            streams = self._tls.streams = {}
        key = str(device)
        s = streams.get(key)
        if s is None:
            s = streams[key] = torch.cuda.Stream(device)
        return s

    def _staging(self, nbytes):
        """This thread's pinned host staging buffer of at least nbytes (grown by doubling). Reused only once
        the copy out of it that the previous decode enqueued has completed (its event, _staged)."""
        ev = getattr(self._tls, "staging_event", None)
        if ev is not None:
            ev.synchronize()
            self._tls.staging_event = None
        buf = getattr(self._tls, "staging", None)
        if buf is None or buf.numel() < nbytes:
            buf = torch.empty(max(nbytes, 2 * (buf.numel() if buf is not None else 0), 1 << 20),
                              dtype=torch.uint8, pin_memory=True)
            self._tls.staging = buf
        self._tls.staging_used = True
        return buf

    def _staged(self, stream):
        """After encoded_to: if it staged through this thread's pinned buffer, mark the copy's completion."""
        if getattr(self._tls, "staging_used", False):
            self._tls.staging_used = False
            ev = torch.cuda.Event()
            ev.record(stream)
            self._tls.staging_event = ev

    WS_CACHE = 16  # encode workspaces kept per codec (one per plan and launch stream in use)

    def _workspace(self, plan, stream=None):
        """The encode workspace of `plan` for this thread and `stream` (default: the current one), reused across
        calls (kernels on
        one stream run in order, so consecutive encodes of one thread can share it). Keyed by thread too: two
        threads encoding on one stream (e.g. both on the default stream) interleave their launches, since the
        ctypes call releases the GIL, and one encode's select would read the other's scan results. A bounded
        LRU: an evicted workspace was allocated on its stream, whose later allocations are the only ones that
        can reuse it (stream-ordered)."""
        if not hasattr(plan, "empty_workspace"):
            return None
        if stream is None:
            stream = torch.cuda.current_stream(plan.device) if plan.device.type == "cuda" else None
        key = (id(plan), threading.get_ident(), None if stream is None else stream.cuda_stream)
        with self._lock:
            hit = self._ws.get(key)
            if hit is not None and hit[0] is plan:
                self._ws.move_to_end(key)
                return hit[1]
            ws = plan.empty_workspace()
            self._ws[key] = (plan, ws)
            self._ws.move_to_end(key)
            while len(self._ws) > self.WS_CACHE:
                self._ws.popitem(last=False)
        return ws

    def _device_for(self, tensors):
        for t in tensors:
            if t.dtype == torch.float32 and t.numel() > 0:
                runs = getattr(self.backend, "runs_on", None)
                return t.device if runs is None or runs(t.device) else self.backend.default_device()
        return None

    def snapshot(self, module_or_state, device=None):
        """FlatState of a model (the w_global snapshot for delta mode), flattened on `device` (default:
        where the codec will run: the state's own device if the backend runs there, else the backend's
        default device)."""
        state = module_or_state.state_dict() if isinstance(module_or_state, nn.Module) else module_or_state
        return flatten_state(state, device=device if device is not None else self._device_for(state.values()))

    # -- decode -----------------------------------------------------------------------------------
    def decode_state(self, update, base=None, device=None):
        """CompressedUpdate -> OrderedDict state (fp32 entries are views into one fresh flat buffer).

        On a GPU the decode runs on this thread's own stream (the remote server decodes from one thread per
        upload, coala/server/service.py:74), after a pinned H2D of a received payload; the caller's current
        stream waits for it (no host synchronisation), so the returned tensors are ready for any work the
        caller enqueues next."""
        return self._decode(update, base, device)[0]

    def _decode(self, update, base=None, device=None, into=None):
        """decode_state's work: (state, flat buffer, raw group buffers). `into` (a recycled skeleton, see
        decode_module): decode into its flat buffer and copy the passthrough entries into its raw buffers
        instead of allocating — state is then None."""
        h = update.header  # self-describing: decode with the blob's own ratio/bits/mode
        D = _decode_layout(h["entries"])
        flat = plan = None
        raw = update.raw
        if D.sizes:
            if device is None:
                device = self.backend.default_device()
            base_flat = None
            if h["mode"] == "delta":
                if base is None:
                    raise ValueError("delta-mode update needs the global model (base) to decode")
                _check_same_layout(h["entries"], base.entries)
                base_flat = base.flat_on(device)
            plan = self.plan_for(D.sizes, device, ratio=h["ratio"], bits=h["bits"])
            if device.type == "cuda":
                cur = torch.cuda.current_stream(device)
                side = self._thread_stream(device)
                side.wait_stream(cur)
                if into is not None:  # a recycled tree: after its previous holder's work (_reuse_after)
                    _reuse_after(into, side, cur)
                # (the caller's stream's pool)
                out = into.flat if into is not None else torch.empty(plan.span, dtype=torch.float32, device=device)
                with torch.cuda.stream(side):
                    enc = update.encoded_to(device, staging=self._staging)
                    self._staged(side)
                    flat = plan.decode(enc, base=base_flat, out=out, stream=side)
                    if into is not None:
                        for dst, (src, _) in zip(into.raws, raw._groups):
                            dst.copy_(src, non_blocking=True)
                cur.wait_stream(side)
            else:
                if into is not None:
                    _reuse_after(into, None, None)
                enc = update.encoded.to(device, non_blocking=True)
                flat = plan.decode(enc, base=base_flat, out=None if into is None else into.flat)
                if into is not None:
                    for dst, (src, _) in zip(into.raws, raw._groups):
                        dst.copy_(src)
        elif into is not None:
            for dst, (src, _) in zip(into.raws, raw._groups):
                dst.copy_(src)
        if into is not None:
            return None, flat, into.raws
        vals = [None] * len(D.names)
        if D.sizes:
            for pos, v in zip(D.seg_pos, _segment_views(flat, plan.table, h["entries"])):
                vals[pos] = v
        raws = None
        if D.raw:
            if isinstance(raw, RawState):
                raws, raw = raw.fresh_groups(device)
            else:
                raw = {n: (t.to(device) if device is not None else t).clone() for n, t in raw.items()}
            for pos, name in D.raw:
                vals[pos] = raw[name]
        return OrderedDict(zip(D.names, vals)), flat, raws

    def decode_module(self, update, template, base=None):
        """CompressedUpdate -> new nn.Module shaped like `template` holding the decoded state.

        No parameter data is copied: the new module's parameters/buffers are views into the decode
        output. `template` is never aliased. Decoded modules are RECYCLED: once nothing outside this codec
        references a module it returned — none of its submodules, parameters or buffers (the reference server
        drops a round's uploads when the next round's replace them in client_uploads, coala/server/base.py:
        377-381, 562-571) — a later call of the same layout decodes straight into that module's storage and
        returns it, instead of building a module tree again (the Python of ~130 modules and ~160 Parameters
        for a ResNet-50 was most of a decompression(model) call)."""
        D = _decode_layout(update.header["entries"])
        recipe = _recipe(template)
        device = self.backend.default_device() if D.sizes else None
        # (the root comes back taken under the pool lock: no other thread can be handed this tree)
        sk, root = recipe.idle_skeleton(D, update.raw, device) if self.recycle else (None, None)
        if sk is not None:
            self._decode(update, base, device, into=sk)
            recipe.refresh(sk)
            return root
        box = [None]
        box[0], flat, raws = self._decode(update, base, device)  # (the state lives in `box` only)
        return recipe.build_and_adopt(box, D, flat, raws, update.raw, device, adopt=self.recycle)

    # -- fused server-side aggregation ------------------------------------------------------------
    def aggregate(self, updates, weights, template, base=None, mode="recip", device=None, params_only=False):
        """Fused decode + FedAvg of several CompressedUpdates of one layout -> nn.Module (recycled from the
        decode pool once idle, as decode_module's are: a dropped earlier result is aggregated into).

        Equivalent to decode_module() of every update followed by the reference's
        strategies.federated_averaging(models, weights) (coala/server/strategies.py:6-29, 57-90), with
        the fp32 entries decoded and averaged in ONE kernel (coalac_aggregate) instead of C dense
        modules. mode "recip": torch-on-GPU division semantics (the decoded modules live on the GPU);
        "div": torch-on-CPU; "sum": strategies.weighted_sum (:57-90) — no division, the module a
        multi-GPU server passes to reduce_models (coala/distributed/distributed.py:42-57). Non-fp32
        entries (int64 BatchNorm counters) are combined with the same torch ops as the reference, on the
        output device. Weights follow federated_averaging / weighted_sum: empty or all-zero weights
        become 1 per update. params_only (aggregation_content "parameters", coala/server/base.py:588-591):
        only the template's parameters are averaged (federated_averaging_only_params /
        weighted_sum_only_params, strategies.py:32-54, 93-124); every buffer keeps update 0's decoded value,
        as the reference's deepcopy(models[0]) does.
        """
        if not updates:
            return None
        weights = list(weights) if weights is not None else []
        if not weights or sum(weights) == 0:
            weights = [1 for _ in updates]
        if len(weights) != len(updates):
            raise ValueError("one weight per update")
        total = sum(weights)
        h0 = updates[0].header
        for u in updates[1:]:
            h = u.header
            if (h["ratio"], h["bits"], h["mode"], h["entries"]) != (h0["ratio"], h0["bits"], h0["mode"], h0["entries"]):
                raise ValueError("fused aggregation needs updates of one layout / ratio / bits / mode")
        sizes = [e["n"] for e in h0["entries"] if e["kind"] == "seg"]
        device = self.backend.default_device() if device is None else torch.device(device)
        base_flat = None
        if h0["mode"] == "delta":
            if base is None:
                raise ValueError("delta-mode updates need the global model (base) to aggregate")
            _check_same_layout(h0["entries"], base.entries)
            base_flat = base.flat_on(device)
        state = OrderedDict()
        flat = None
        # the output module is recycled like decode_module's (the same pool: modules this codec returned that
        # nothing outside it references any more); not for params_only, whose buffers are update 0's values
        recipe = D = sk = root = None
        if self.recycle and not params_only and isinstance(updates[0].raw, RawState):
            D = _decode_layout(h0["entries"])
            recipe = _recipe(template)
            sk, root = recipe.idle_skeleton(D, updates[0].raw, device)  # (root taken under the pool lock)
            if sk is not None:
                cur = torch.cuda.current_stream(device) if device.type == "cuda" else None
                _reuse_after(sk, cur, cur)  # the kernel runs on the current stream
        if params_only:
            pnames = {n for n, _ in template.named_parameters(remove_duplicate=False)}
        accs = []
        raw_avg = _aggregate_raw(updates, weights, total, mode, device,
                                 keep=(lambda n: n not in pnames) if params_only else None, accs=accs)
        if raw_avg is None:  # (the passthrough entries are combined one by one below: nothing to recycle into)
            recipe = sk = root = None
        if sizes:
            C = len(updates)
            plan = self.plan_for(sizes, device, ratio=h0["ratio"], bits=h0["bits"], clients=C)
            encs = [u.encoded.to(device, non_blocking=True) for u in updates]
            batched = Encoded(*(torch.cat([getattr(e, f) for e in encs]) for f in ("idx", "vals", "mn", "scale")),
                              torch.cat([e.ustart for e in encs]) if all(e.ustart is not None for e in encs) else None)
            avg_mask = None
            if params_only:
                pnames = {n for n, _ in template.named_parameters(remove_duplicate=False)}
                avg_mask = [e["name"] in pnames for e in h0["entries"] if e["kind"] == "seg"]
            flat = plan.aggregate(batched, weights, total=total, base=base_flat, mode=mode, avg_mask=avg_mask,
                                  out=None if sk is None else sk.flat)
            if sk is not None and flat.data_ptr() != sk.flat.data_ptr():  # a backend that returns its own buffer
                sk = root = None
        if sk is not None:
            for dst, acc in zip(sk.raws, accs):
                dst.copy_(acc, non_blocking=True)
            recipe.refresh(sk)
            return root
        # the fp32 entries: one split of the output (_segment_views), not a slice + view per entry
        seg_views = iter(_segment_views(flat, plan.table, h0["entries"])) if sizes else None
        for e in h0["entries"]:
            if e["kind"] == "seg":
                state[e["name"]] = next(seg_views)
            elif raw_avg is not None:
                state[e["name"]] = raw_avg[e["name"]]
            elif params_only and e["name"] not in pnames:  # a buffer: update 0's (deepcopy(models[0]))
                state[e["name"]] = updates[0].raw[e["name"]].to(device).clone()
            else:  # restated weighted_sum (+ torch.div) on the raw entries
                acc = updates[0].raw[e["name"]].to(device).clone()
                acc *= weights[0]
                for i in range(1, len(updates)):
                    acc += updates[i].raw[e["name"]].to(device) * weights[i]
                state[e["name"]] = acc if mode == "sum" else torch.div(acc, total).to(acc.dtype)
        if recipe is not None:
            # no view of the output may outlive this frame beside the module's own: the pool's idle
            # fingerprint is taken inside build_and_adopt
            box = [state]
            del state, seg_views, raw_avg
            return recipe.build_and_adopt(box, D, flat, accs, updates[0].raw, device)
        return module_with_state(template, state)


def _aggregate_raw(updates, weights, total, mode, device, keep=None, accs=None):
    """The passthrough entries of several updates combined as the per-entry loop in UpdateCodec.aggregate
    does — acc = x_0 * w_0; acc += x_i * w_i in update order; then torch.div(acc, total) cast back (not in
    mode "sum"); entries for which keep(name) is true take update 0's value — but with the same elementwise
    ops on each dtype group's flat tensor at once (a BatchNorm model's 53 counters: 2 ops per update instead
    of 2 per update and counter). None when the updates' RawStates are not grouped alike. accs (a list):
    receives each dtype group's result buffer, the storage the returned entries view."""
    raws = [u.raw for u in updates]
    if not all(isinstance(r, RawState) for r in raws):
        return None
    g0 = raws[0]._groups
    sig = [(f.dtype, f.numel(), tuple(m)) for f, m in g0]
    if any([(f.dtype, f.numel(), tuple(m)) for f, m in r._groups] != sig for r in raws[1:]):
        return None
    out = {}
    int_weights = all(type(w) is int and -(1 << 62) < w < (1 << 62) for w in weights)
    for gi, (f0, members) in enumerate(g0):
        if int_weights and f0.dtype in (torch.int64, torch.int32) and len(raws) > 2:
            # integer entries, integer weights: two's-complement sums do not depend on their order, so the
            # update-order loop is one stacked product and sum (3 launches instead of 2 per update), cast back
            # to the entry dtype (the loop's in-place ops wrap the same way)
            X = torch.stack([r._groups[gi][0].to(device) for r in raws])
            W = torch.tensor(weights, dtype=torch.int64, device=device)
            acc = (X.to(torch.int64) * W[:, None]).sum(0).to(f0.dtype)
        else:
            acc = f0.to(device, copy=True)
            acc *= weights[0]
            for i in range(1, len(raws)):
                acc += raws[i]._groups[gi][0].to(device) * weights[i]
        if mode != "sum":
            acc = torch.div(acc, total).to(acc.dtype)
        if accs is not None:
            accs.append(acc)
        first = f0.to(device, copy=True) if keep is not None else None
        views = raws[0]._make_views([(acc, members)])
        firsts = raws[0]._make_views([(first, members)]) if first is not None else None
        for n, _, _ in members:
            out[n] = firsts[n] if keep is not None and keep(n) else views[n]
    return out


def _segment_views(flat, table, entries):
    """Views of the decoded flat buffer, one per fp32 segment (in segment order), shaped like the header's
    entries, at the decoder's own offsets (never the untrusted header's): ONE split of the buffer into
    segments and alignment pads, and a view only where a shape is not already the 1-D piece (a slice +
    view per entry cost ~3 us each, ~1 ms per ResNet-50 decode)."""
    split = table.__dict__.get("_split")
    if split is None:
        sizes, keep, prev = [], [], 0
        for off, n in zip(table.offsets, table.sizes):
            if off > prev:
                sizes.append(off - prev)
            keep.append(len(sizes))
            sizes.append(n)
            prev = off + n
        split = table.__dict__["_split"] = (sizes, keep, prev)
    sizes, keep, end = split
    pieces = flat[:end].split_with_sizes(sizes)
    seg_entries = [e for e in entries if e["kind"] == "seg"]
    out = []
    for j, e in zip(keep, seg_entries):
        t, shape = pieces[j], e["shape"]
        out.append(t if len(shape) == 1 else t.view(shape))
    return out


_PLAIN_TYPES = frozenset((bool, int, float, complex, str, bytes, type(None), torch.dtype, torch.device))
_CONTAINER_TYPES = frozenset((dict, OrderedDict, list, set))
_MODULE_TABLES = frozenset(("_parameters", "_buffers", "_modules"))
_TABLES3 = itemgetter("_parameters", "_buffers", "_modules")
_make_param = torch.Tensor._make_subclass


def _plain(v):
    """An attribute value a clone may share with the template: immutable and holding no tensor / module."""
    tv = type(v)
    if tv in _PLAIN_TYPES:
        return True
    if tv is tuple or tv is frozenset:
        return all(_plain(x) for x in v)
    return False


class _TreeRecipe:
    """How to rebuild a template's module tree around new tensors, classified once per template (the
    server's global model is one object for the whole task): the modules in pre-order (a submodule shared
    by several parents is cloned once, as copy.deepcopy would), and per module the attributes a clone
    shares (immutable plain values), gets as fresh empty containers (hook dicts, ...), deep-copies (any
    other object: non-empty containers, hook objects, unregistered modules — with a memo that maps the
    template's modules / parameters / buffers to the clone's, so bound hooks are rebound as deepcopy would)
    or clones (unregistered tensors), plus its parameter / buffer / child slots. A module whose attribute
    set, table sizes or special attribute types changed since is re-classified."""

    def __init__(self, template):
        self.pool, self.pool_lock = [], threading.Lock()
        self.tick = 0  # idle_skeleton calls so far (a pooled tree's last use is one of these)
        self.mods, self.prefixes, self.index = [], [], {}
        stack = [(template, "")]
        while stack:
            m, prefix = stack.pop()
            if id(m) in self.index:
                continue
            self.index[id(m)] = len(self.mods)
            self.mods.append(m)
            self.prefixes.append(prefix)
            stack.extend((c, prefix + n + ".") for n, c in reversed(list(m._modules.items())) if c is not None)
        self.info = [self.classify(m, p) for m, p in zip(self.mods, self.prefixes)]

    def classify(self, m, prefix):
        d = m.__dict__
        fresh, deep, tens = [], [], []
        for k, v in d.items():
            if k in _MODULE_TABLES or _plain(v):
                continue
            tv = type(v)
            if tv in _CONTAINER_TYPES and not v:
                fresh.append((k, tv))
            elif isinstance(v, torch.Tensor):
                tens.append((k, tv))
            else:
                deep.append((k, tv))
        params = tuple((n, prefix + n, p is None or p.requires_grad) for n, p in m._parameters.items())
        buffers = tuple((n, prefix + n) for n in m._buffers)
        children = tuple((n, None if c is None else self.index[id(c)]) for n, c in m._modules.items())
        sizes = (len(d), len(m._parameters), len(m._buffers), len(m._modules))
        return sizes, tuple(fresh), tuple(deep), tuple(tens), params, buffers, children

    def valid(self, i):
        """Cheap per-call check that module i still matches its classification: attribute / table sizes, its
        fresh containers still empty (a hook registered later must be deep-copied, not dropped) and the
        types of its deep-copied / cloned attributes."""
        m = self.mods[i]
        sizes, fresh, deep, tens = self.info[i][:4]
        d = m.__dict__
        if sizes != (len(d), len(m._parameters), len(m._buffers), len(m._modules)):
            return False
        g = self.getters[i]
        if g is not None and any(g(d)):
            return False
        return not (tens or deep) or all(type(d.get(k)) is tv for k, tv in tens + deep)

    def _getters(self):
        from operator import itemgetter
        self.getters = []
        for info in self.info:
            keys = [k for k, _ in info[1]]
            self.getters.append(None if not keys else itemgetter(*keys) if len(keys) > 1 else
                                (lambda d, k=keys[0]: (d[k],)))

    def _current(self):
        """Re-classify the template modules that changed since (attribute / table sizes, hooks registered, the
        types of special attributes); returns the per-module fast tables. A change also retires every pooled
        skeleton (they were built from the old classification)."""
        mods, info = self.mods, self.info
        if not hasattr(self, "getters"):
            self._getters()
        if self.__dict__.get("fast") is not None and self._unchanged():
            return self.fast
        stale = [i for i in range(len(mods)) if not self.valid(i)]
        if stale:
            for i in stale:
                info[i] = self.classify(mods[i], self.prefixes[i])
            self._getters()
            with self.pool_lock:
                self.pool.clear()
        fast = self.__dict__.get("fast")
        if fast is None or stale:
            fast = self.fast = [self._fast(x) for x in info]
            self.plain = [tuple(k for k in m.__dict__ if k not in _MODULE_TABLES and k not in set(f[5] + f[9] + f[10]))
                          for m, f in zip(mods, fast)]
            self._flat_tables()
        return fast

    def _flat_tables(self):
        """The per-call checks and the refresh as C-level maps over the whole tree (a Python loop over a
        ResNet-50's 132 modules and their ~1,600 hook containers cost more than the decode itself)."""
        dicts = self.t_dicts = [m.__dict__ for m in self.mods]
        self.t_dlens = list(map(len, dicts))
        self.t_tables = list(chain.from_iterable(map(_TABLES3, dicts)))
        self.t_sizes = list(map(len, self.t_tables))
        self.t_fresh = [d[k] for d, x in zip(dicts, self.info) for k, _ in x[1]]  # the template's empty containers
        self.t_typed = [(d, k, tv) for d, x in zip(dicts, self.info) for k, tv in x[3] + x[2]]
        self.p_src = [d for d, keys in zip(dicts, self.plain) for _ in keys]
        self.p_keys = [k for keys in self.plain for k in keys]
        self.p_mod = [i for i, keys in enumerate(self.plain) for _ in keys]
        self.special = [i for i, f in enumerate(self.fast) if f[9] or f[10]]

    def _unchanged(self):
        """Every template module as classified: __dict__ and table sizes, the same table objects, its fresh
        containers still empty (a hook registered later must be deep-copied), its special attributes' types."""
        dicts = self.t_dicts
        if list(map(len, dicts)) != self.t_dlens or any(self.t_fresh):
            return False
        tabs = list(chain.from_iterable(map(_TABLES3, dicts)))
        if not all(map(is_, tabs, self.t_tables)) or list(map(len, tabs)) != self.t_sizes:
            return False
        return all(type(d.get(k)) is tv for d, k, tv in self.t_typed)

    def tree_unchanged(self):
        """The template's module tree is still the one this recipe walked: every child slot holds the same
        module object (a replaced submodule — model.head = nn.Linear(...) — needs a new recipe)."""
        kids = self.__dict__.get("t_kids")
        if kids is None:
            self.t_kid_dicts = [m._modules for m in self.mods if m._modules]
            kids = self.t_kids = [tuple(d.values()) for d in self.t_kid_dicts]
        return list(map(tuple, map(dict.values, self.t_kid_dicts))) == kids

    def build(self, state):
        return self._build(state)[0]

    def _build(self, state):
        """The new module tree: the list of new module objects in recipe order (root first)."""
        mods = self.mods
        fast = self._current()
        new = [m.__class__.__new__(m.__class__) for m in mods]
        get = state.get
        deep_todo = []
        for i, m in enumerate(mods):
            pnames, pkeys, prgs, bnames, bkeys, fkeys, ftypes, cnames, cidx, tens, deep = fast[i]
            ts = list(map(get, pkeys))
            if any(map(is_, ts, repeat(None))):  # a parameter the state lacks (or a None slot): the template's, cloned
                src = m._parameters
                ts = [t if t is not None else (None if src[n] is None else src[n].detach().clone())
                      for n, t in zip(pnames, ts)]
                P = {n: None if t is None else _make_param(nn.Parameter, t, rg) for n, t, rg in zip(pnames, ts, prgs)}
            else:
                P = dict(zip(pnames, map(_make_param, repeat(nn.Parameter), ts, prgs)))
            B = dict(zip(bnames, map(get, bkeys)))
            if any(map(is_, B.values(), repeat(None))):
                srcb = m._buffers
                B = {n: (t if t is not None else (None if srcb[n] is None else srcb[n].clone())) for n, t in B.items()}
            d = m.__dict__.copy()  # plain attributes shared (read now: e.g. `training` follows the template)
            if fkeys:
                d.update(zip(fkeys, [tv() for tv in ftypes]))
            for k in tens:
                d[k] = d[k].clone()
            d["_parameters"] = P
            d["_buffers"] = B
            d["_modules"] = dict(zip(cnames, [None if j is None else new[j] for j in cidx]))
            new[i].__dict__.update(d)  # (a fresh object's dict: no Module.__setattr__ on the way)
            if deep:
                deep_todo.append((i, deep))
        if deep_todo:  # after every clone is filled in, so the memo maps every module / tensor
            memo = self._memo(new, state)
            for i, deep in deep_todo:
                nd = new[i].__dict__
                for k in deep:
                    nd[k] = copy.deepcopy(nd[k], memo)
        return new

    # -- recycling of decoded modules (UpdateCodec.decode_module) ------------------------------------------
    POOL_MAX = 64            # skeletons kept per template (a server needs two rounds' uploads: 2 x clients)
    POOL_BYTES = 16 << 30    # ... and at most this many bytes of decoded storage
    POOL_FRACTION = 8        # ... nor more than 1/8 of the device's memory
    EVICT_SLACK = 16         # a tree not handed out for 2 x pool size + this many calls is dropped from the pool

    def pool_limit(self, device):
        lim = self.__dict__.get("_pool_limit")
        if lim is None or lim[0] != device:
            total = None
            if device is not None and device.type == "cuda":
                total = torch.cuda.get_device_properties(device).total_memory
            lim = self._pool_limit = (device, self.POOL_BYTES if total is None else
                                      min(self.POOL_BYTES, total // self.POOL_FRACTION))
        return lim[1]

    def build_and_adopt(self, box, D, flat, raws, raw, device, adopt=True):
        """Build the module tree for the decoded state in box (a one-element list, emptied here: the caller
        keeps no reference to the state) and keep it in the pool as a skeleton for later decodes of the same
        layout (unless adopt is False). Returns the root module."""
        state = box.pop()
        new = self._build(state)
        del state
        root = new[0]
        if (not adopt or (flat is None and not raws) or not isinstance(raw, RawState)
                or len(self.pool) >= self.POOL_MAX):
            return root
        nbytes = (flat.numel() * 4 if flat is not None else 0) + sum(r.numel() * r.element_size() for r in raws or ())
        limit = self.pool_limit(device)
        stream = torch.cuda.current_stream(device) if device is not None and device.type == "cuda" else None
        with self.pool_lock:
            if sum(sk.nbytes for sk in self.pool) + nbytes > limit or len(self.pool) >= self.POOL_MAX:
                return root
            sk = _Skeleton(root, new, flat, list(raws or ()), D, raw.signature(), device, nbytes)
            sk.adopt(self)
            sk.stream, sk.last = stream, self.tick
            del new
            sk.base = sk.counts()
            sk.base[0][0] -= 1  # the root: this frame's `root` is the only transient reference
            self.pool.append(sk)
        return root

    def idle_skeleton(self, D, raw, device):
        """A pooled skeleton of this layout that nothing outside the pool references any more (every module,
        parameter and buffer object at its idle reference count, the decoded storage at its idle use count,
        every module's tables unchanged) and its root — (None, None) if there is none. The root is taken
        while the pool lock is held, so the moment a tree is chosen it is no longer idle for any other
        thread (the remote server decodes from one thread per upload, coala/server/service.py:74).
        Idle trees not handed out for a while (2 x the pool size + EVICT_SLACK calls: more than a round needs)
        are dropped from the pool; held ones stay."""
        if not self.pool or not isinstance(raw, RawState):
            return None, None
        self._current()
        sig = raw.signature()
        with self.pool_lock:
            self.tick += 1
            found = root = None
            for sk in self.pool:
                if sk.D is D and sk.device == device and sk.raw_sig == sig and sk.counts() == sk.base:
                    found, root = sk, sk.root
                    sk.generation += 1
                    sk.last = self.tick
                    break
            # only IDLE trees go: a tree still held (a server keeps round r's uploads until round r + 1 replaces them,
            # coala/server/base.py:377-381) becomes reusable when its holder lets go, however long that takes
            horizon = 2 * len(self.pool) + self.EVICT_SLACK
            if any(self.tick - sk.last > horizon for sk in self.pool):
                self.pool[:] = [sk for sk in self.pool
                                if self.tick - sk.last <= horizon or sk is found or sk.counts() != sk.base]
            return found, root

    def refresh(self, sk):
        """Bring a recycled tree's attributes in line with the template's CURRENT ones, as a fresh build would:
        plain attributes copied, hook containers emptied if a previous holder registered hooks, special
        attributes re-copied unless still equal."""
        memo = None
        list(map(dict.__setitem__, sk.p_dst, self.p_keys, map(dict.__getitem__, self.p_src, self.p_keys)))
        if any(sk.fresh):  # a previous holder registered hooks on the recycled tree: empty containers again
            for i, c in enumerate(sk.mods):
                nd, f = c.__dict__, self.fast[i]
                for k, tv in zip(f[5], f[6]):
                    if nd.get(k):
                        nd[k] = tv()
            sk.adopt(self)
        for i in self.special:
            m, c = self.mods[i], sk.mods[i]
            d, nd = m.__dict__, c.__dict__
            f = self.fast[i]
            for k in f[9]:
                nd[k] = d[k].clone()
            for k in f[10]:
                try:
                    same = bool(nd.get(k) == d[k])
                except Exception:
                    same = False
                if not same:
                    if memo is None:
                        memo = self._memo(sk.mods, {})
                    nd[k] = copy.deepcopy(d[k], memo)

    @staticmethod
    def _fast(x):
        _, fresh, deep, tens, params, buffers, children = x
        return (tuple(n for n, _, _ in params), tuple(k for _, k, _ in params), tuple(rg for _, _, rg in params),
                tuple(n for n, _ in buffers), tuple(k for _, k in buffers),
                tuple(k for k, _ in fresh), tuple(tv for _, tv in fresh),
                tuple(n for n, _ in children), tuple(j for _, j in children),
                tuple(k for k, _ in tens), tuple(k for k, _ in deep))

    def _memo(self, new, state=None):
        """deepcopy memo: template module / parameter / buffer -> its counterpart in the clone."""
        memo = {}
        for m, c in zip(self.mods, new):
            memo[id(m)] = c
        for m, c, p in zip(self.mods, new, self.prefixes):
            for name, t in m._parameters.items():
                if t is not None and name in c.__dict__.get("_parameters", {}):
                    memo[id(t)] = c._parameters[name]
            for name, t in m._buffers.items():
                if t is not None and name in c.__dict__.get("_buffers", {}):
                    memo[id(t)] = c._buffers[name]
        return memo


class _Skeleton:
    """A decoded module tree kept for reuse: its objects (modules, then their parameter / buffer tensors), the
    decoded storage they view (the flat fp32 decode output and the passthrough groups) and their idle
    reference counts."""

    __slots__ = ("root", "mods", "objs", "dicts", "dlens", "tables", "tsizes", "flat", "raws", "D", "raw_sig",
                 "device", "nbytes", "base", "generation", "p_dst", "fresh", "stream", "last")

    def __init__(self, root, mods, flat, raws, D, raw_sig, device, nbytes):
        self.root, self.mods = root, mods
        self.objs = list(mods)
        for c in mods:
            self.objs.extend(t for t in c._parameters.values() if t is not None)
            self.objs.extend(t for t in c._buffers.values() if t is not None)
        self.dicts = [c.__dict__ for c in mods]
        self.dlens = list(map(len, self.dicts))
        self.tables = list(chain.from_iterable(map(_TABLES3, self.dicts)))
        self.tsizes = list(map(len, self.tables))
        self.flat, self.raws, self.D, self.raw_sig, self.device, self.nbytes = flat, raws, D, raw_sig, device, nbytes
        self.generation = 0
        self.stream, self.last = None, 0

    def adopt(self, recipe):
        """The recipe's flat refresh tables for this tree: where each plain attribute goes, and the tree's own
        (empty) hook containers, checked in one pass per recycle."""
        self.p_dst = [self.dicts[i] for i in recipe.p_mod]
        self.fresh = [c.__dict__[k] for c, f in zip(self.mods, recipe.fast) for k in f[5]]

    def counts(self):
        """Idle fingerprint: every object's reference count, the decoded storage's use counts, and whether every
        module still has its attribute count and its very table objects at their sizes (an attribute added or a
        table replaced by a previous holder keeps the tree from being recycled)."""
        refs = list(map(sys.getrefcount, self.objs))
        store = [torch._C._storage_Use_Count(t.untyped_storage()._cdata) for t in [self.flat] + self.raws
                 if t is not None]
        tabs = list(chain.from_iterable(map(_TABLES3, self.dicts)))
        same = (list(map(len, self.dicts)) == self.dlens and all(map(is_, tabs, self.tables))
                and list(map(len, tabs)) == self.tsizes)
        return [refs, store, same]


_RECIPES = {}  # id(template) -> (weakref to it, recipe)
_RECIPES_LOCK = threading.Lock()


def _recipe(template):
    """The template's _TreeRecipe (one per template object: the server's global model, for a whole task)."""
    key = id(template)
    with _RECIPES_LOCK:
        hit = _RECIPES.get(key)
        if hit is None or hit[0]() is not template or not hit[1].tree_unchanged():
            import weakref
            hit = (weakref.ref(template), _TreeRecipe(template))
            _RECIPES[key] = hit
            if len(_RECIPES) > 32:
                for k in [k for k, (r, _) in _RECIPES.items() if r() is None]:
                    del _RECIPES[k]
    return hit[1]


def release_decode_pool():
    """Drop every template's pooled decoded modules (UpdateCodec.release_pool)."""
    with _RECIPES_LOCK:
        recipes = [r for _, r in _RECIPES.values()]
    for r in recipes:
        with r.pool_lock:
            r.pool.clear()


def _reuse_after(sk, stream, caller):
    """Order a recycled tree's rewrite after its previous holder's work and retire stale autograd state.
    `stream` (None on the CPU) is where the rewrite runs, `caller` the caller's current stream (the stream
    the module is handed out on). The host reference counts that made the tree idle do not see GPU work:
    the rewrite waits for everything enqueued so far on the stream the tree was last handed out on (where
    its holder's work ran, unless the holder moved it to another stream itself — torch's own contract for
    that is Tensor.record_stream, which a recycled tree cannot honour: pass recycle=False then). The decode
    kernel writes through raw pointers, so the storage's version counter is bumped here: an autograd graph
    that saved the previous values raises in backward instead of using the new ones."""
    if stream is not None and sk.stream is not None and sk.stream != stream and sk.stream != caller:
        stream.wait_stream(sk.stream)  # (the rewrite's stream already waits for the caller's)
    sk.stream = caller
    torch._C._increment_version([t for t in [sk.flat] + sk.raws if t is not None])


def module_with_state(template, state):
    """A new nn.Module shaped like `template` whose parameters / buffers ARE the tensors of `state`
    (views into the decode output: no parameter data is copied; `template` is never aliased).

    The module tree is rebuilt from a per-template recipe (_TreeRecipe) — new objects of the same classes,
    their __dict__ copied one level deep with fresh tables and hook dicts, other attributes deep-copied —
    instead of copy.deepcopy, whose generic recursion cost ~8 ms per ResNet-50 on the server's per-upload
    path. Tensors outside the state (non-persistent buffers, unregistered tensors) are cloned."""
    return _recipe(template).build(state)


_SAME_LAYOUT = OrderedDict()  # (id(a), id(b)) -> (a, b): pairs of entry lists already found equal


def _check_same_layout(entries, base_entries):
    key = (id(entries), id(base_entries))
    hit = _SAME_LAYOUT.get(key)
    if hit is not None and hit[0] is entries and hit[1] is base_entries:
        return
    a = [(e["name"], e["dtype"], tuple(e["shape"])) for e in entries]
    b = [(e["name"], e["dtype"], tuple(e["shape"])) for e in base_entries]
    if a != b:
        raise ValueError("update and base model have different state_dict layouts")
    with _LAYOUTS_LOCK:  # (the header entries are never mutated: the pair stays equal)
        _SAME_LAYOUT[key] = (entries, base_entries)
        while len(_SAME_LAYOUT) > 64:
            _SAME_LAYOUT.popitem(last=False)


class _DecodeLayout:
    """Per header-entries list: the state names, the fp32 segment sizes and where segments / raw entries sit."""

    def __init__(self, entries):
        self.names = tuple(e["name"] for e in entries)
        self.sizes = tuple(e["n"] for e in entries if e["kind"] == "seg")
        self.seg_pos = [i for i, e in enumerate(entries) if e["kind"] == "seg"]
        self.raw = [(i, e["name"]) for i, e in enumerate(entries) if e["kind"] != "seg"]


_DECODE_LAYOUTS = OrderedDict()  # id(entries) -> (entries, _DecodeLayout)


def _decode_layout(entries):
    hit = _DECODE_LAYOUTS.get(id(entries))
    if hit is not None and hit[0] is entries:
        return hit[1]
    D = _DecodeLayout(entries)
    with _LAYOUTS_LOCK:
        _DECODE_LAYOUTS[id(entries)] = (entries, D)
        while len(_DECODE_LAYOUTS) > 64:
            _DECODE_LAYOUTS.popitem(last=False)
    return D


def as_numpy(t):
    return t.detach().cpu().numpy() if isinstance(t, torch.Tensor) else np.asarray(t)
