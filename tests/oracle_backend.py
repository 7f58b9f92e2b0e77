"""Test-only codec backend that runs the CPU oracle behind the same plan interface as the HIP plan.

Used by CPU tests (C1 plumbing, gloo sharding) to exercise the plugin/host logic without a GPU. The
product never imports this (coala_amd has no CPU fallback); here the oracle is the checker.
"""
import numpy as np
import torch

from coala_amd.compression.plan import Encoded
from coala_amd.compression.spec import RAW_BITS, SegmentTable
from oracle import codec_oracle as O


class OraclePlan:
    def __init__(self, sizes, ratio, bits, clients=1):
        self.table = SegmentTable(sizes, ratio, clients)
        self.bits = bits

    def _idx(self, enc):
        """enc.idx, or a dense (ratio 1) update's implied indices (0..n-1 per segment)."""
        if enc.idx.numel() or not self.table.total_k:
            return enc.idx.numpy()
        return np.concatenate([np.arange(int(n), dtype=np.int32) for n in self.table.segs[:, 1]])

    def encode(self, flat, base=None, **_):
        x = flat.detach().cpu().numpy()
        b = None if base is None else base.detach().cpu().numpy()
        segs = self.table.segs.astype(np.int64)
        idx, vals, mn, sc = O.encode(x, segs, self.bits, base=b)
        if self.table.ratio >= 1.0:  # as the HIP plan: a dense update's indices stay implied
            return Encoded(torch.zeros(0, dtype=torch.int32), torch.from_numpy(vals), torch.from_numpy(mn),
                           torch.from_numpy(sc), None)
        return Encoded(torch.from_numpy(idx), torch.from_numpy(vals), torch.from_numpy(mn), torch.from_numpy(sc),
                       torch.from_numpy(O.unit_starts(idx, segs)))

    def decode(self, enc, base=None, out=None, **_):
        b = None if base is None else base.detach().cpu().numpy()
        res = np.zeros(self.table.span, dtype=np.float32) if b is None else b.copy()
        O.decode(self._idx(enc), enc.vals.numpy(), enc.mn.numpy(), enc.scale.numpy(),
                 self.table.segs.astype(np.int64), self.bits, self.table.span, base=b, out=res)
        if out is not None:  # (a recycled decoded module's storage: written in place, as the HIP plan does)
            out[:res.size].copy_(torch.from_numpy(res))
            return out
        return torch.from_numpy(res)

    def aggregate(self, enc, weights, total=None, base=None, mode="div", avg_mask=None, **_):
        total = float(sum(weights)) if total is None else float(total)
        b = None if base is None else base.detach().cpu().numpy()
        out = O.aggregate(self._idx(enc), enc.vals.numpy(), enc.mn.numpy(), enc.scale.numpy(),
                          self.table.segs.astype(np.int64), self.bits, self.table.clients, weights, total,
                          {"div": O.AGG_DIV, "recip": O.AGG_RECIP, "sum": O.AGG_SUM}[mode], base=b,
                          out_span=self.table.span_per_client, avg_mask=avg_mask)
        return torch.from_numpy(out)


class OracleBackend:
    name = "oracle"

    def default_device(self):
        return torch.device("cpu")

    def runs_on(self, device):
        return torch.device(device).type == "cpu"

    def make_plan(self, sizes, ratio, bits, device, clients=1):
        return OraclePlan(sizes, ratio, bits, clients)
