"""Full-size oracle parity at every BASELINE config's per-GPU share, through the bench's own pipelines.

The configs (BASELINE.json): C2 16 x ResNet-18 (179 M elements, 3 concurrent
sub-batches), C3 16 x ResNet-50 (410 M, 2 sub-batches; the headline), C4 16 x ViT-B/16 (1.385 G
elements, 338 k units: the uint32 unit / group indexing at its largest), C5 one GPU's share of the
heterogeneous splitFL round (MixedTable, one latency-bound plan), and the C3 share in delta mode, at the other
ratios, after a sign-like step (near-ties), and C4 with a frozen backbone (zero ties). Each
batch is synthesised on the GPU exactly as bench.py does (coala_amd/workload.py), encoded and decoded
with the SplitPipeline the bench times, and compared client by client with oracle/codec_oracle.py run
over a spawned process pool (tests/oracle_pool.py) on a shared-memory copy of the same batch.

Tolerance (the bar of test_gpu_parity.py): idx, codes, mn, scale and the per-unit starts (wire v2)
BIT-IDENTICAL; the dense output
bit-identical to the oracle's decode at every kept position and +0.0 (weights mode) / base + 0.0f (delta
mode) everywhere else inside the segments.
"""
import numpy as np
import pytest
import torch

from coala_amd.compression import SplitPipeline
from coala_amd.compression.spec import SegmentTable
from coala_amd.layouts import fp32_sizes
from coala_amd.workload import c5_share, freeze_segments, head_only, mixed_table, sign_step, synth_batch
from oracle import codec_oracle as O
from tests.oracle_pool import SharedBatch, oracle_clients

pytestmark = pytest.mark.gpu

# name -> (layout | "c5", clients, sub-batches, mode, ratio, trained): bench.py CONFIGS; trained: how the trained
# weights derive from the base in delta mode (None: synthesised independently)
CASES = {
    "C2": ("resnet18", 16, 3, "weights", 0.01, None),
    "C3": ("resnet50_tv", 16, 2, "weights", 0.01, None),
    "C4": ("vit_b16", 16, 2, "weights", 0.01, None),
    "C5": ("c5", None, 1, "weights", 0.01, None),
    "C3-delta": ("resnet50_tv", 16, 2, "delta", 0.01, None),
    "C3-r0.001": ("resnet50_tv", 16, 2, "weights", 0.001, None),
    "C3-r0.1": ("resnet50_tv", 16, 2, "weights", 0.1, None),
    # FedPEFT's frozen backbone (application/FedPEFT/lora.py:64): every tensor but the head an exact-zero delta
    "C4-frozen": ("vit_b16", 16, 2, "delta", 0.01, "frozen"),
    # one sign-like local step: trained = fl(w_global -+ 1e-3), near-ties at the k-th key (bench.py C3_signs)
    "C3-signs": ("resnet50_tv", 16, 2, "delta", 0.01, "signs"),
}


def _table(layout, clients, ratio):
    if layout == "c5":
        ids, names = c5_share(0)
        return mixed_table(names, ratio), ids
    return SegmentTable(fp32_sizes(layout), ratio, clients), list(range(clients))


def _to_shared(t):
    sb = SharedBatch(t.numel())
    torch.from_numpy(sb.array[:t.numel()]).copy_(t.view(-1))  # D2H into the shared pages
    return sb


@pytest.mark.parametrize("case", list(CASES))
def test_fullsize_share_bit_exact_vs_oracle(cuda, case):
    layout, clients, split, mode, ratio, trained = CASES[case]
    bits = 8
    table, ids = _table(layout, clients, ratio)
    flat = synth_batch(table, cuda, client_ids=ids)
    base = synth_batch(table, cuda, client_ids=[10_000 + i for i in ids]) if mode == "delta" else None
    if trained == "frozen":  # as bench.py's C4_frozen: trained = base + delta, the frozen tensors' deltas exactly zero
        freeze_segments(flat, table, head_only(layout))
        flat.add_(base)
    elif trained == "signs":  # as bench.py's C3_signs
        sign_step(flat, base, 4242)
    # host copies for the oracle (shared memory: the spawned workers map them, nothing is pickled)
    sb = _to_shared(flat)
    bb = _to_shared(base) if base is not None else None
    try:
        pipe = SplitPipeline(table, bits, split=split, device=cuda)
        assert pipe.n_parts == split
        enc = pipe.empty_encoded()
        out = torch.zeros(table.span, dtype=torch.float32, device=cuda)  # alignment pads stay 0
        pipe.roundtrip(flat, base=base, enc=enc, out=out)
        torch.cuda.synchronize()
        assert pipe.fallbacks() == 0
        g_idx, g_vals = enc.idx.cpu().numpy(), enc.vals.cpu().numpy()
        g_mn, g_sc = enc.mn.cpu().numpy().view(np.uint32), enc.scale.cpu().numpy().view(np.uint32)
        g_us = enc.ustart.cpu().numpy()

        so, ko, to, uo = table.client_span_off, table.client_k_off, table.client_seg_off, table.client_unit_off
        segs = table.segs.astype(np.int64)
        spans, csegs = [], []
        for c in range(table.clients):
            s = segs[to[c]:to[c + 1]].copy()
            s[:, 0] -= so[c]
            s[:, 3] -= ko[c]
            spans.append((so[c], so[c + 1] - so[c]))
            csegs.append(s)
        kept = torch.zeros(table.span, dtype=torch.bool, device=cuda)
        for c, (idx, vals, mn, sc, pos, xhat) in oracle_clients(sb, spans, csegs, bits, base=bb):
            k0, k1 = ko[c], ko[c + 1]
            np.testing.assert_array_equal(g_idx[k0:k1], idx, err_msg=f"{case} client {c}: idx")
            np.testing.assert_array_equal(g_vals[k0:k1], vals, err_msg=f"{case} client {c}: codes")
            np.testing.assert_array_equal(g_mn[to[c]:to[c + 1]], mn.view(np.uint32), err_msg=f"{case} client {c}: mn")
            np.testing.assert_array_equal(g_sc[to[c]:to[c + 1]], sc.view(np.uint32), err_msg=f"{case} client {c}: scale")
            np.testing.assert_array_equal(g_us[uo[c]:uo[c + 1]], O.unit_starts(idx, csegs[c]),
                                          err_msg=f"{case} client {c}: per-unit starts")
            p = torch.from_numpy(pos + so[c]).to(cuda)
            got = out[p].view(torch.int32)
            want = torch.from_numpy(xhat).to(cuda).view(torch.int32)
            bad = int((got != want).sum())
            assert bad == 0, f"{case} client {c}: {bad} decoded values differ from the oracle"
            kept[p] = True
        # everywhere else inside the segments: the background (0, or base + 0.0f in delta mode)
        if base is None:
            rest = out.view(torch.int32)[~kept]
            assert int((rest != 0).sum()) == 0, f"{case}: non-zero output outside the kept positions"
        else:
            inside = torch.zeros(table.span, dtype=torch.bool, device=cuda)
            for c in range(table.clients):
                for off, n, _, _ in segs[to[c]:to[c + 1]]:
                    inside[off:off + n] = True
            m = inside & ~kept
            want = (base + 0.0)[m].view(torch.int32)
            assert torch.equal(out[m].view(torch.int32), want), f"{case}: background differs from base + 0.0f"
        pipe.close()
    finally:
        sb.close()
        if bb is not None:
            bb.close()
