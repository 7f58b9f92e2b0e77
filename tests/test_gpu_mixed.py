"""C5 on the GPU: one GPU's share of the heterogeneous splitFL round — client-side
models of three architectures at cut 1/2/4 next to feature tensors up to 8,388,608 elements — encoded
and decoded in one batched launch sequence over a MixedTable, bit-exact against the CPU oracle.

Tolerance: bit-identical idx / codes / mn / scale / dense output (the same bar as test_gpu_parity.py).
"""
import numpy as np
import pytest
import torch

from coala_amd.compression import CodecPlan, SplitPipeline
from coala_amd.compression.spec import MixedTable
from coala_amd.layouts import fp32_sizes
from coala_amd.workload import c5_share, mixed_table, synth_batch
from oracle import codec_oracle as O

pytestmark = pytest.mark.gpu


def _oracle(table, flat, bits, base=None):
    segs = table.segs.astype(np.int64)
    idx, vals, mn, sc = O.encode(flat, segs, bits, base=base)
    dec = O.decode(idx, vals, mn, sc, segs, bits, table.span, base=base)
    return idx, vals, mn, sc, dec


def _check(table, enc, dec, ref):
    idx, vals, mn, sc, rdec = ref
    np.testing.assert_array_equal(enc.idx.cpu().numpy(), idx)
    np.testing.assert_array_equal(enc.vals.cpu().numpy().view(np.uint8), vals.view(np.uint8))
    np.testing.assert_array_equal(enc.mn.cpu().numpy().view(np.uint32), mn.view(np.uint32))
    np.testing.assert_array_equal(enc.scale.cpu().numpy().view(np.uint32), sc.view(np.uint32))
    got = dec.cpu().numpy()
    inside = np.zeros(table.span, bool)
    for off, n, k, oo in table.segs.astype(np.int64):
        inside[off:off + n] = True
    np.testing.assert_array_equal(got[inside].view(np.uint32), rdec[inside].view(np.uint32))


@pytest.mark.parametrize("ratio,bits", [(0.01, 8), (0.001, 4), (0.1, 32)])
def test_c5_share_bit_exact_vs_oracle(cuda, ratio, bits):
    ids, names = c5_share(0)
    assert "sfl_feature_256x32x32" in names  # an 8,388,608-element segment (2,048 units)
    table = mixed_table(names, ratio)
    plan = CodecPlan(None, ratio, bits, table=table)
    flat = synth_batch(table, cuda, client_ids=ids)
    ws = plan.empty_workspace()
    enc = plan.encode(flat, workspace=ws)
    dec = plan.decode(enc)
    torch.cuda.synchronize()
    _check(table, enc, dec, _oracle(table, flat.cpu().numpy(), bits))
    assert plan.fallbacks(ws) == 0


def test_c5_share_split_pipeline_equals_single_plan(cuda):
    """The bench's 2 concurrent sub-batches over a MixedTable (cut by element count) give the single
    plan's bytes."""
    ids, names = c5_share(3)
    table = mixed_table(names, 0.01)
    flat = synth_batch(table, cuda, client_ids=ids)
    plan = CodecPlan(None, 0.01, 8, table=table)
    e1 = plan.encode(flat)
    d1 = plan.decode(e1)
    pipe = SplitPipeline(table, 8, split=2, device=cuda)
    e2, d2 = pipe.roundtrip(flat)
    torch.cuda.synchronize()
    for f in ("idx", "vals", "mn", "scale"):
        assert torch.equal(getattr(e1, f), getattr(e2, f)), f
    assert _same_inside(table, d1, d2)  # the alignment pads between segments are never written


def _same_inside(table, a, b):
    for off, n, k, oo in table.segs.astype(np.int64):
        if not torch.equal(a[off:off + n].view(torch.int32), b[off:off + n].view(torch.int32)):
            return False
    return True


def test_c5_delta_mode_mixed(cuda):
    """Delta mode over a mixed batch (client-side models are trained against a global copy)."""
    names = ["resnet50_split_cut4", "sfl_feature_64x32x32", "simple_cnn_split_cut1", "resnet18_split_cut2"]
    table = MixedTable([fp32_sizes(n) for n in names], 0.01)
    flat = synth_batch(table, cuda, client_ids=range(4))
    base = synth_batch(table, cuda, client_ids=range(100, 104))
    plan = CodecPlan(None, 0.01, 8, table=table)
    enc = plan.encode(flat, base=base)
    dec = plan.decode(enc, base=base)
    torch.cuda.synchronize()
    _check(table, enc, dec, _oracle(table, flat.cpu().numpy(), 8, base=base.cpu().numpy()))
