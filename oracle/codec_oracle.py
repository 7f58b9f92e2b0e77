"""CPU ORACLE for CodecSpec v1 — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module, and only as
the checker / the timed CPU baseline. The product path (coala_amd.*) never imports it.

PARITY STATUS: "parity unpinned" for top-k + quantise. The reference has no codec:
/root/reference/coala/compression/__init__.py is 0 bytes and the hooks it would implement are no-ops
(coala/client/base.py:203-205, :330-332; coala/server/base.py:347-349, :558-560). There are no reference
tests, golden vectors or fixtures for this path. This module restates the spec the
build defines in SURVEY.md §8(a) rows a3/a4 ("CodecSpec v1"), and is pinned by:
  * the reference's own behaviour where it exists (identity framing coala/protocol/codec.py:4-9, FedAvg
    coala/server/strategies.py:6-29/57-90 on decoded modules — tests/golden/fedavg.npz, hooks.json), and
  * an independent brute-force restatement (full stable sort; tests/test_oracle.py) plus the committed
    golden vectors tests/golden/codec_vectors.npz generated from it (tests/golden/make_codec_vectors.py).

CodecSpec v1 (per fp32 segment = one flattened tensor of n elements):
  k      = 0 if n == 0 else max(1, min(n, ceil(n * ratio)))   (ratio in float64, on the host)
  key(x) = uint32 bits of x with the sign bit cleared (monotone in |x|; NaN sorts above +inf;
           -0.0 and +0.0 share key 0)
  select = the k elements with the largest key; equal keys: the lower index wins.
  idx    = the selected indices, ascending, int32 (segment-relative)
  v      = x[idx]  (delta mode: x = in - base, fp32 subtraction first)
  bits == 32 ("raw"): values stored as fp32, mn = scale = 0.
  bits in 1..8: mn = NaN-ignoring min(v), mx = NaN-ignoring max(v), each then + 0.0f (canonical +0);
           L = 2^bits - 1; scale = 0 if mx == mn else (mx - mn) / L (fp32 ops);
           q = 0 if !(scale > 0) else { r = rint((v - mn) / scale) (half-to-even);
                                        q = 0 if !(r > 0) else min(r, L) }  -> uint8
  decode: xhat = mn + float(q) * scale  (fp32 multiply then fp32 add; never fused)
          dense out = 0 everywhere, xhat at idx; fused delta mode: out = base + dense (fp32 add, every
          element, so base -0.0 becomes +0.0 where nothing was selected).
  ustart (wire v2): per 4096-element unit of every segment (ceil(n / 4096) of them, in segment order), the
          index into the segment's idx list of the first kept entry at or after the unit's first element,
          i.e. the number of the segment's kept indices below unit * 4096 (a sorted-list lower bound).
"""
import math

import numpy as np

F32 = np.float32
SIGN_CLEAR = np.uint32(0x7FFFFFFF)
RAW_BITS = 32


def k_for(n, ratio):
    """Kept-element count of a segment."""
    if n <= 0:
        return 0
    return max(1, min(int(n), int(math.ceil(float(n) * float(ratio)))))


def keys(x):
    x = np.ascontiguousarray(x, dtype=F32)
    return x.view(np.uint32) & SIGN_CLEAR


def topk_indices(x, k):
    """Indices of the k largest keys, ties to the lower index, returned ascending (int32).

    O(n) with argpartition on a unique composite key = key * 2^32 + (2^32 - 1 - index).
    """
    n = x.size
    if k <= 0:
        return np.zeros(0, dtype=np.int32)
    if k >= n:
        return np.arange(n, dtype=np.int32)
    comp = (keys(x).astype(np.uint64) << np.uint64(32)) | (np.uint64(0xFFFFFFFF) - np.arange(n, dtype=np.uint64))
    part = np.argpartition(comp, n - k)[n - k:]
    return np.sort(part).astype(np.int32)


def topk_indices_bruteforce(x, k):
    """Independent restatement: full stable sort by descending key (used to pin topk_indices)."""
    order = np.argsort(-keys(x).astype(np.int64), kind="stable")
    return np.sort(order[:k]).astype(np.int32)


def _nanmin_canon(v):
    f = v[~np.isnan(v)]
    if f.size == 0:
        return F32(np.nan)
    return F32(F32(f.min()) + F32(0.0))


def _nanmax_canon(v):
    f = v[~np.isnan(v)]
    if f.size == 0:
        return F32(np.nan)
    return F32(F32(f.max()) + F32(0.0))


def quantize(v, bits):
    """fp32 values -> (codes uint8, mn fp32, scale fp32) exactly as CodecSpec v1."""
    v = np.ascontiguousarray(v, dtype=F32)
    if v.size == 0:
        return np.zeros(0, dtype=np.uint8), F32(0), F32(0)
    mn = _nanmin_canon(v)
    mx = _nanmax_canon(v)
    levels = F32((1 << bits) - 1)
    with np.errstate(all="ignore"):
        scale = F32(0) if mx == mn else F32(F32(mx - mn) / levels)
        if not (scale > 0):
            return np.zeros(v.size, dtype=np.uint8), mn, scale
        t = (v - mn) / scale          # float32 arrays: IEEE fp32 sub and div
        r = np.rint(t)                # half-to-even
        q = np.where(r > 0, np.minimum(r, levels), F32(0))   # NaN -> 0 (r > 0 is False)
        q = np.where(np.isnan(q), F32(0), q)
    return q.astype(np.uint8), mn, scale


def dequantize(q, mn, scale):
    with np.errstate(all="ignore"):
        p = q.astype(F32) * F32(scale)     # fp32 multiply
        return F32(mn) + p                  # fp32 add (no FMA)


def encode_segment(x, k, bits):
    """One segment -> (idx int32[k], vals uint8[k] | fp32[k], mn, scale)."""
    x = np.ascontiguousarray(x, dtype=F32)
    idx = topk_indices(x, k)
    v = x[idx]
    if bits == RAW_BITS:
        return idx, v.copy(), F32(0), F32(0)
    q, mn, scale = quantize(v, bits)
    return idx, q, mn, scale


def decode_segment(idx, vals, mn, scale, n, bits, base=None):
    dense = np.zeros(n, dtype=F32)
    if idx.size:
        dense[idx] = vals if bits == RAW_BITS else dequantize(vals, mn, scale)
    if base is not None:
        with np.errstate(all="ignore"):
            dense = np.ascontiguousarray(base, dtype=F32) + dense
    return dense


def encode(flat, segs, bits, base=None):
    """Batch encode over a flat fp32 buffer.

    segs: int array [T, 4] of (in_off, n, k, out_off). Returns idx[K], vals[K], mn[T], scale[T] with
    K = max(out_off + k).
    """
    segs = np.asarray(segs, dtype=np.int64).reshape(-1, 4)
    total = int((segs[:, 3] + segs[:, 2]).max()) if len(segs) else 0
    idx_out = np.zeros(total, dtype=np.int32)
    vals_out = np.zeros(total, dtype=F32 if bits == RAW_BITS else np.uint8)
    mn_out = np.zeros(len(segs), dtype=F32)
    sc_out = np.zeros(len(segs), dtype=F32)
    for s, (off, n, k, oo) in enumerate(segs):
        x = flat[off:off + n]
        if base is not None:
            with np.errstate(all="ignore"):
                x = x - base[off:off + n]
        idx, v, mn, sc = encode_segment(x, int(k), bits)
        idx_out[oo:oo + k] = idx
        vals_out[oo:oo + k] = v
        mn_out[s] = mn
        sc_out[s] = sc
    return idx_out, vals_out, mn_out, sc_out


def decode(idx, vals, mn, scale, segs, bits, span, base=None, out=None):
    """Inverse of encode into a dense flat buffer of `span` elements (positions outside segments: 0,
    or base in delta mode)."""
    segs = np.asarray(segs, dtype=np.int64).reshape(-1, 4)
    out = np.zeros(span, dtype=F32) if out is None else out
    for s, (off, n, k, oo) in enumerate(segs):
        b = None if base is None else base[off:off + n]
        out[off:off + n] = decode_segment(idx[oo:oo + k], vals[oo:oo + k], mn[s], scale[s], int(n), bits, b)
    return out


UNIT = 4096


def unit_starts(idx, segs):
    """The wire v2 per-unit starts of an encode (idx of encode(), same segs): int32[sum ceil(n / UNIT)]."""
    segs = np.asarray(segs, dtype=np.int64).reshape(-1, 4)
    parts = []
    for off, n, k, oo in segs:
        nu = (int(n) + UNIT - 1) // UNIT
        if nu:
            parts.append(np.searchsorted(idx[oo:oo + k], np.arange(nu, dtype=np.int64) * UNIT, side="left"))
    return np.concatenate(parts).astype(np.int32) if parts else np.zeros(0, dtype=np.int32)


AGG_DIV, AGG_RECIP, AGG_SUM = 0, 1, 2


def aggregate(idx, vals, mn, scale, segs, bits, clients, weights, total, mode, base=None, out_span=None,
              avg_mask=None):
    """Fused decode + FedAvg restated: decode every client (decode_segment, i.e. coalac_decode with the
    same base), then the reference's weighted average over the decoded fp32 entries, in client order:

        params = s_0 * w_0; params += s_i * w_i          coala/server/strategies.py:57-90 (weighted_sum)
        params = torch.div(params, total)                coala/server/strategies.py:6-29

    torch evaluates the division as params / total on the CPU (mode AGG_DIV) and as
    params * (1.0f / total) on a GPU, where a host scalar divisor becomes a reciprocal multiply (mode
    AGG_RECIP); AGG_SUM stops before the division (weighted_sum, strategies.py:57-90, the per-rank
    sum a multi-GPU server hands to reduce_models, distributed.py:42-57). weights / total are taken as fp32 (torch converts the Python scalars to the tensor's
    fp32 compute type). segs: [clients * T, 4] client-major copies of one layout; the output is
    indexed like client 0's segments (positions outside them: 0).

    avg_mask (one bool per segment of a client, None = all True): a False segment is not averaged; it
    keeps client 0's decoded value, as weighted_sum_only_params / federated_averaging_only_params keep
    models[0]'s buffers (coala/server/strategies.py:32-54, 93-124: deepcopy(models[0]), then only
    named_parameters() are summed and divided).
    """
    segs = np.asarray(segs, dtype=np.int64).reshape(-1, 4)
    T = len(segs) // clients
    w = np.asarray(weights, dtype=np.float64).astype(F32)
    tot = F32(total)
    span = int(max(segs[t, 0] + segs[t, 1] for t in range(T))) if out_span is None else out_span
    out = np.zeros(span, dtype=F32)
    with np.errstate(all="ignore"):
        for t in range(T):
            off0, n = int(segs[t, 0]), int(segs[t, 1])
            b = None if base is None else base[off0:off0 + n]
            if avg_mask is not None and not avg_mask[t]:
                off, n_, k, oo = (int(v) for v in segs[t])
                out[off0:off0 + n] = decode_segment(idx[oo:oo + k], vals[oo:oo + k], mn[t], scale[t], n, bits, b)
                continue
            acc = None
            for c in range(clients):
                off, n_, k, oo = (int(v) for v in segs[c * T + t])
                s = decode_segment(idx[oo:oo + k], vals[oo:oo + k], mn[c * T + t], scale[c * T + t], n, bits, b)
                term = s * w[c]
                acc = term if acc is None else acc + term
            if acc is None:
                continue
            if mode == AGG_SUM:
                out[off0:off0 + n] = acc
            else:
                out[off0:off0 + n] = acc / tot if mode == AGG_DIV else acc * (F32(1.0) / tot)
    return out
