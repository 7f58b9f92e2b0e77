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
import threading
from collections import OrderedDict

import numpy as np
import torch
from torch import nn

from . import wire
from .plan import CodecPlan, Encoded
from .spec import ALIGN, RAW_BITS, VALID_BITS, SegmentTable, align_up, k_for

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
        off = seg = 0
        for name, dt, shape in items:
            n = 1
            for d in shape:
                n *= d
            e = {"name": name, "dtype": _dtype_name(dt), "shape": list(shape)}
            if dt == torch.float32 and n > 0:
                e.update(kind="seg", seg=seg, off=off, n=n)
                self.seg_names.append(name)
                off = align_up(off + n)
                seg += 1
            else:
                e["kind"] = "raw"
                self.raw_names.append(name)
            self.entries.append(e)
        self.sizes = [e["n"] for e in self.entries if e["kind"] == "seg"]


_LAYOUTS = OrderedDict()
_LAYOUTS_LOCK = threading.Lock()


def _layout(state):
    sig = tuple((k, v.dtype, v.shape) for k, v in state.items())
    with _LAYOUTS_LOCK:
        L = _LAYOUTS.get(sig)
        if L is None:
            L = _LAYOUTS[sig] = _Layout(sig)
            while len(_LAYOUTS) > 16:
                _LAYOUTS.popitem(last=False)
    return L


def describe_state(state):
    """state_dict -> (entries as flatten_state would write them, fp32 segment tensors in order, raw
    passthrough entries), WITHOUT copying the fp32 data: the zero-copy encode reads the tensors in place."""
    L = _layout(state)
    segs = [state[n] for n in L.seg_names]  # read in place by the kernels (pointer, numel, dtype, contiguity)
    raw = OrderedDict((n, state[n].detach()) for n in L.raw_names)
    return L.entries, segs, _snapshot_raw(raw)


def _snapshot_raw(raw):
    """Copies of the passthrough entries (int64 BatchNorm counters, ...) taken now, batched per
    (dtype, device) into one copy kernel instead of one per entry."""
    out = OrderedDict()
    groups = {}
    for name, t in raw.items():
        groups.setdefault((t.dtype, t.device), []).append(name)
    for (dt, dev), names in groups.items():
        ts = [raw[n] for n in names]
        if dev.type != "cuda" or len(ts) == 1 or any(t.numel() == 0 for t in ts):  # CPU: a clone is cheaper
            for n, t in zip(names, ts):
                out[n] = t.clone()
            continue
        flat = torch.cat([t.reshape(-1) for t in ts])
        o = 0
        for n, t in zip(names, ts):
            out[n] = flat[o:o + t.numel()].view(t.shape)
            o += t.numel()
    return OrderedDict((n, out[n]) for n in raw)


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
        other.header = copy.deepcopy(self.header, memo)
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
        raw_b = sum(t.numel() * t.element_size() for t in self.raw.values())
        return 8 * h["n_segments"] + (ib + vb) * h["total_k"] + raw_b

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
        raw_entries, chunks, pos = [], [], 0
        for e in h["entries"]:
            if e["kind"] == "raw":
                b = self.raw[e["name"]].cpu().contiguous().reshape(-1).view(torch.uint8).numpy().tobytes() \
                    if self.raw[e["name"]].numel() else b""
                e = dict(e, off=pos, nbytes=len(b))
                chunks.append(b)
                pos += len(b)
            raw_entries.append(e)
        h["entries"] = raw_entries
        if h["ratio"] >= 1.0:
            h["dense"] = True
        enc = self.encoded
        return wire.pack(h, enc.mn.cpu().numpy(), enc.scale.cpu().numpy(), enc.idx.cpu().numpy(),
                         enc.vals.cpu().numpy(), b"".join(chunks))

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
        _, sec = wire.sections(blob)
        lo = sec["mn"][0]
        hi = sec["vals"][0] + sec["vals"][1]
        stage = staging(hi - lo)
        stage[:hi - lo].numpy()[:] = np.frombuffer(blob, dtype=np.uint8, count=hi - lo, offset=lo)
        dev = torch.empty(hi - lo, dtype=torch.uint8, device=device)
        dev.copy_(stage[:hi - lo], non_blocking=True)
        vdt = torch.float32 if self.header["bits"] == RAW_BITS else torch.uint8

        def view(name, dt):
            o, n = sec[name]
            return dev[o - lo:o - lo + n].view(dt)
        return Encoded(view("idx", torch.int32), view("vals", vdt), view("mn", torch.float32),
                       view("scale", torch.float32))

    @classmethod
    def from_bytes(cls, blob):
        h, mn, scale, idx, vals, rawb = wire.unpack(blob)
        validate(h, idx)
        raw = OrderedDict()
        for e in h["entries"]:
            if e["kind"] == "raw":
                dt = getattr(torch, e["dtype"])
                buf = bytearray(rawb[e["off"]:e["off"] + e["nbytes"]])
                t = torch.frombuffer(buf, dtype=dt) if buf else torch.empty(0, dtype=dt)
                raw[e["name"]] = t.reshape(e["shape"]).clone()
        enc = Encoded(torch.from_numpy(idx.copy()), torch.from_numpy(vals.copy()),
                      torch.from_numpy(mn.copy()), torch.from_numpy(scale.copy()))
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
        dense = 4 * sum(e["n"] for e in h["entries"] if e["kind"] == "seg")
        dense += sum(t.numel() * t.element_size() for t in self.raw.values())
        return dense / max(1, self.nbytes)

    def __repr__(self):
        h = self.header
        return (f"CompressedUpdate(mode={h['mode']}, ratio={h['ratio']}, bits={h['bits']}, "
                f"segments={h['n_segments']}, kept={h['total_k']}, bytes={self.nbytes})")


def validate(header, idx):
    """Check an (untrusted) blob's index lists: per fp32 segment, k = k_for(n, ratio) entries, strictly
    increasing, inside [0, n). The decode kernels are bounds-safe anyway; this turns a corrupt upload
    into an error instead of a silently wrong model."""
    if header.get("bits") not in VALID_BITS or header.get("mode") not in MODES:
        raise ValueError("COALAQ1: bad bits/mode")
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
    if int(ks.sum()) != int(header["total_k"]) or idx.size != int(header["total_k"]):
        raise ValueError("COALAQ1: kept-entry count mismatch")
    if not ks.size:
        return
    ns = np.array([e["n"] for e in segs], dtype=np.int64)
    seg_of = np.repeat(np.arange(ks.size), ks)
    i64 = idx.astype(np.int64)
    if np.any(i64 < 0) or np.any(i64 >= ns[seg_of]):
        raise ValueError("COALAQ1: index out of range")
    first = np.zeros(idx.size, dtype=bool)
    first[np.cumsum(ks)[:-1][ks[1:] > 0] if ks.size > 1 else []] = True
    first[0] = True
    d = np.diff(i64, prepend=-1)
    if np.any((d <= 0) & ~first):
        raise ValueError("COALAQ1: indices not strictly increasing")


class UpdateCodec:
    """Encode / decode model updates with CodecSpec v1.

    Args:
        ratio: top-k ratio per tensor, (0, 1].
        bits:  1..8 -> uint8 min/max codes; 32 -> raw fp32 values (lossless at ratio 1).
        mode:  "delta" encodes w_local - w_global (decode adds w_global back, fused in the kernel);
               "weights" encodes the weights themselves.
        backend: object with make_plan(sizes, ratio, bits, device); default HipBackend.
    """

    def __init__(self, ratio=0.01, bits=8, mode="delta", backend=None):
        if not (0.0 < float(ratio) <= 1.0):
            raise ValueError(f"ratio must be in (0, 1], got {ratio}")
        if bits not in VALID_BITS:
            raise ValueError(f"bits must be one of {VALID_BITS}, got {bits}")
        if mode not in MODES:
            raise ValueError(f"mode must be one of {MODES}, got {mode}")
        self.ratio, self.bits, self.mode = float(ratio), int(bits), mode
        self.backend = backend if backend is not None else HipBackend()
        self._plans = {}
        self._ws = {}
        self._lock = threading.Lock()
        self._tls = threading.local()

    def plan_for(self, sizes, device, ratio=None, bits=None, clients=1):
        ratio = self.ratio if ratio is None else float(ratio)
        bits = self.bits if bits is None else int(bits)
        key = (tuple(sizes), ratio, bits, str(device), int(clients))
        with self._lock:
            p = self._plans.get(key)
            if p is None:
                p = self.backend.make_plan(list(sizes), ratio, bits, device, clients=clients)
                self._plans[key] = p
        return p

    # -- encode -----------------------------------------------------------------------------------
    def encode(self, state, base=None, device=None):
        """state_dict -> CompressedUpdate. `base` (delta mode): FlatState of w_global (same layout).
        `device`: where to flatten and encode (default: where the state lives if the backend runs there,
        else the backend's default device — a model trained on the CPU is encoded on the GPU)."""
        if device is None:
            device = self._device_for(state)
        if self.mode == "delta" and base is None:
            raise ValueError("delta mode needs the global-model snapshot (base)")
        entries, segs, raw = describe_state(state)
        sizes = [e["n"] for e in entries if e["kind"] == "seg"]
        header = {"ratio": self.ratio, "bits": self.bits, "mode": self.mode, "n_segments": len(sizes),
                  "entries": entries}
        if not sizes:
            header["total_k"] = 0
            z = torch.zeros(0)
            return CompressedUpdate(header, Encoded(z.int(), z.to(torch.uint8), z, z), raw)
        device = torch.device(device)
        base_flat = None
        if self.mode == "delta":
            _check_same_layout(entries, base.entries)
            # the snapshot may have been taken where the global model arrived (the reference client's
            # set_model runs before pretrain moves the model to its device, client/base.py:138 vs :245)
            base_flat = base.flat_on(device)
        plan = self.plan_for(sizes, device)
        ws = self._workspace(plan)
        dev_index = device.index if device.type == "cuda" else -1  # (Tensor.get_device(): -1 on the CPU)
        in_place = getattr(plan, "encode_segments", None) is not None and all(
            t.get_device() == dev_index and t.is_contiguous() and t.data_ptr() % 16 == 0 for t in segs)
        if in_place:  # read the parameters where they live: no flattening copy (+8 B/element of traffic)
            # (dtype and sizes hold by construction: the plan was made from this layout's segments)
            enc = plan.encode_segments(segs, base=base_flat, workspace=ws, checked=True)
        else:
            fs = flatten_state(state, device=device)
            enc = plan.encode(fs.flat, base=base_flat, workspace=ws)
        header["total_k"] = int(plan.table.total_k)
        return CompressedUpdate(header, enc, raw)

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
        """This thread's pinned host staging buffer of at least nbytes (grown by doubling; reused once the
        thread's stream has finished with it, which decode_state waits for)."""
        buf = getattr(self._tls, "staging", None)
        if buf is None or buf.numel() < nbytes:
            buf = torch.empty(max(nbytes, 2 * (buf.numel() if buf is not None else 0), 1 << 20),
                              dtype=torch.uint8, pin_memory=True)
            self._tls.staging = buf
        return buf

    def _workspace(self, plan):
        """The encode workspace of `plan` for the calling thread and its current stream, reused across
        calls (kernels on one stream run in order, so consecutive encodes can share it)."""
        if not hasattr(plan, "empty_workspace"):
            return None
        stream = torch.cuda.current_stream(plan.device) if plan.device.type == "cuda" else None
        key = (id(plan), threading.get_ident(), None if stream is None else stream.cuda_stream)
        with self._lock:
            ws = self._ws.get(key)
            if ws is None:
                ws = plan.empty_workspace()
                self._ws[key] = ws
        return ws

    def _device_for(self, state):
        for t in state.values():
            if t.dtype == torch.float32 and t.numel() > 0:
                runs = getattr(self.backend, "runs_on", None)
                return t.device if runs is None or runs(t.device) else self.backend.default_device()
        return None

    def snapshot(self, module_or_state, device=None):
        """FlatState of a model (the w_global snapshot for delta mode), flattened on `device` (default:
        where the codec will run: the state's own device if the backend runs there, else the backend's
        default device)."""
        state = module_or_state.state_dict() if isinstance(module_or_state, nn.Module) else module_or_state
        return flatten_state(state, device=device if device is not None else self._device_for(state))

    # -- decode -----------------------------------------------------------------------------------
    def decode_state(self, update, base=None, device=None):
        """CompressedUpdate -> OrderedDict state (fp32 entries are views into one fresh flat buffer)."""
        h = update.header  # self-describing: decode with the blob's own ratio/bits/mode
        sizes = [e["n"] for e in h["entries"] if e["kind"] == "seg"]
        state = OrderedDict()
        flat = None
        if sizes:
            if device is None:
                device = self.backend.default_device()
            base_flat = None
            if h["mode"] == "delta":
                if base is None:
                    raise ValueError("delta-mode update needs the global model (base) to decode")
                _check_same_layout(h["entries"], base.entries)
                base_flat = base.flat_on(device)
            plan = self.plan_for(sizes, device, ratio=h["ratio"], bits=h["bits"])
            if device.type == "cuda":
                # this thread's own stream (the remote server decodes from one thread per upload,
                # coala/server/service.py:74): pinned H2D of the payload + decode, then wait for it
                side = self._thread_stream(device)
                side.wait_stream(torch.cuda.current_stream(device))
                out = torch.empty(plan.span, dtype=torch.float32, device=device)
                with torch.cuda.stream(side):
                    enc = update.encoded_to(device, staging=self._staging)
                    flat = plan.decode(enc, base=base_flat, out=out, stream=side)
                side.synchronize()
            else:
                enc = update.encoded.to(device, non_blocking=True)
                flat = plan.decode(enc, base=base_flat)
        views = _segment_views(flat, plan.table, h["entries"]) if sizes else None
        for e in h["entries"]:
            if e["kind"] == "seg":
                state[e["name"]] = views[e["seg"]]
            else:
                t = update.raw[e["name"]]
                state[e["name"]] = t.to(device) if device is not None else t
        return state

    def decode_module(self, update, template, base=None):
        """CompressedUpdate -> new nn.Module shaped like `template` holding the decoded state.

        No parameter data is copied: the new module's parameters/buffers are views into the decode
        output (deepcopy with a memo that pre-binds every tensor). `template` is never aliased.
        """
        state = self.decode_state(update, base=base)
        return module_with_state(template, state)


    # -- fused server-side aggregation ------------------------------------------------------------
    def aggregate(self, updates, weights, template, base=None, mode="recip", device=None):
        """Fused decode + FedAvg of several CompressedUpdates of one layout -> new nn.Module.

        Equivalent to decode_module() of every update followed by the reference's
        strategies.federated_averaging(models, weights) (coala/server/strategies.py:6-29, 57-90), with
        the fp32 entries decoded and averaged in ONE kernel (coalac_aggregate) instead of C dense
        modules. mode "recip": torch-on-GPU division semantics (the decoded modules live on the GPU);
        "div": torch-on-CPU; "sum": strategies.weighted_sum (:57-90) — no division, the module a
        multi-GPU server passes to reduce_models (coala/distributed/distributed.py:42-57). Non-fp32
        entries (int64 BatchNorm counters) are combined with the same torch ops as the reference, on the
        output device. Weights follow federated_averaging / weighted_sum: empty or all-zero weights
        become 1 per update.
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
        offs = None
        if sizes:
            C = len(updates)
            plan = self.plan_for(sizes, device, ratio=h0["ratio"], bits=h0["bits"], clients=C)
            encs = [u.encoded.to(device, non_blocking=True) for u in updates]
            batched = Encoded(*(torch.cat([getattr(e, f) for e in encs]) for f in ("idx", "vals", "mn", "scale")))
            flat = plan.aggregate(batched, weights, total=total, base=base_flat, mode=mode)
            offs = plan.table.offsets
        for e in h0["entries"]:
            if e["kind"] == "seg":
                o = offs[e["seg"]]
                state[e["name"]] = flat[o:o + e["n"]].view(e["shape"])
            else:  # restated weighted_sum (+ torch.div) on the raw entries
                acc = updates[0].raw[e["name"]].to(device).clone()
                acc *= weights[0]
                for i in range(1, len(updates)):
                    acc += updates[i].raw[e["name"]].to(device) * weights[i]
                state[e["name"]] = acc if mode == "sum" else torch.div(acc, total).to(acc.dtype)
        return module_with_state(template, state)


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


_PLAIN_TYPES = frozenset((bool, int, float, str, type(None), tuple))
_CONTAINER_TYPES = frozenset((dict, OrderedDict, list, set))
_MODULE_TABLES = frozenset(("_parameters", "_buffers", "_modules"))


def module_with_state(template, state):
    """A new nn.Module shaped like `template` whose parameters / buffers ARE the tensors of `state`
    (views into the decode output: no parameter data is copied; `template` is never aliased).

    The module tree is rebuilt directly (new objects of the same classes, their __dict__ copied one level
    deep, fresh parameter / buffer / submodule tables and hook dicts) instead of copy.deepcopy, whose
    generic recursion cost ~8 ms per ResNet-50 on the server's per-upload path. Tensors outside the state
    (non-persistent buffers, unregistered tensors) are cloned."""
    def shallow(v):  # a container one level deep; empty ones (most hook dicts) without copy.copy's reduce path
        if not v:
            try:
                return v.__class__()
            except TypeError:
                pass
        return copy.copy(v)

    def clone(mod, prefix):
        cls = mod.__class__
        new = cls.__new__(cls)
        d = {}
        for k, v in mod.__dict__.items():
            tv = type(v)
            if tv in _PLAIN_TYPES:  # most of a module's attributes: nothing to copy
                pass
            elif tv in _CONTAINER_TYPES:
                if k not in _MODULE_TABLES:
                    v = shallow(v)  # (the hook dicts included: the clone never shares them)
            elif isinstance(v, torch.Tensor):
                v = v.clone()
            elif isinstance(v, (list, dict, set)) and k not in _MODULE_TABLES:
                v = shallow(v)
            d[k] = v
        params = OrderedDict()
        for name, p in mod._parameters.items():
            if p is None:
                params[name] = None
                continue
            t = state.get(prefix + name)
            params[name] = nn.Parameter(t if t is not None else p.detach().clone(), requires_grad=p.requires_grad)
        buffers = OrderedDict()
        for name, b in mod._buffers.items():
            t = None if b is None else state.get(prefix + name)
            buffers[name] = None if b is None else (t if t is not None else b.clone())
        d["_parameters"], d["_buffers"] = params, buffers
        d["_modules"] = OrderedDict((name, None if c is None else clone(c, prefix + name + "."))
                                    for name, c in mod._modules.items())
        new.__dict__.update(d)
        return new
    return clone(template, "")


def _check_same_layout(entries, base_entries):
    a = [(e["name"], e["dtype"], tuple(e["shape"])) for e in entries]
    b = [(e["name"], e["dtype"], tuple(e["shape"])) for e in base_entries]
    if a != b:
        raise ValueError("update and base model have different state_dict layouts")


def as_numpy(t):
    return t.detach().cpu().numpy() if isinstance(t, torch.Tensor) else np.asarray(t)
