"""The front-launch encode (COALAC_FLAG_FRONT_LAUNCH: samplers inside the scan launch) and the one-launch encode
(k_fused, COALAC_FLAG_ONE_LAUNCH), both opt-in, against the default kernel-sequence encode (SEQ): bit-identical outputs, no bounded wait ever giving up, control words re-initialised on
every call (the same workspace reused), and several plans in flight at once on separate streams.

Tolerance: bit-identical (the same bar as test_gpu_parity.py).
"""
import numpy as np
import pytest
import torch

from coala_amd.compression import CodecPlan, SegmentTable
from coala_amd.compression._lib import (COALAC_FLAG_FORCE_EXACT, COALAC_FLAG_GENERIC_SELECT, COALAC_FLAG_FRONT_LAUNCH,
                                        COALAC_FLAG_ONE_LAUNCH)
from coala_amd.layouts import fp32_sizes
from coala_amd.workload import c5_share, mixed_table, synth_batch

pytestmark = pytest.mark.gpu
SEQ = 0  # the default encode: the kernel sequence k_presel .. k_emit


def encode(plan, flat, base=None, flags=0, ws=None):
    ws = plan.empty_workspace() if ws is None else ws
    enc = plan.encode(flat, base=base, workspace=ws, flags=flags)
    torch.cuda.synchronize()
    return enc, ws


def same(a, b):
    return all(torch.equal(getattr(a, f), getattr(b, f)) for f in ("idx", "vals", "mn", "scale"))


@pytest.mark.parametrize("layout,clients,ratio,bits,delta", [
    ("resnet18", 2, 0.01, 8, False),
    ("resnet50_tv", 3, 0.01, 8, True),
    ("resnet50_tv", 1, 0.1, 4, False),
    ("resnet50_tv", 2, 0.001, 32, False),
    ("vit_b16", 1, 0.01, 8, False),
    ("lenet", 4, 0.05, 8, True),
])
@pytest.mark.parametrize("mode", [COALAC_FLAG_FRONT_LAUNCH, COALAC_FLAG_ONE_LAUNCH])
def test_fused_equals_multi_launch(cuda, layout, clients, ratio, bits, delta, mode):
    t = SegmentTable(fp32_sizes(layout), ratio, clients)
    plan = CodecPlan(None, ratio, bits, table=t)
    flat = synth_batch(t, cuda)
    base = synth_batch(t, cuda, client_ids=range(50, 50 + clients)) if delta else None
    e1, ws1 = encode(plan, flat, base, flags=mode)
    e2, _ = encode(plan, flat, base, flags=SEQ)
    assert plan.timeouts(ws1) == 0
    assert same(e1, e2)
    d1 = plan.decode(e1, base=base)
    d2 = plan.decode(e2, base=base)
    torch.cuda.synchronize()
    for off, n, k, oo in t.segs.astype(np.int64):
        assert torch.equal(d1[off:off + n].view(torch.int32), d2[off:off + n].view(torch.int32))


@pytest.mark.parametrize("mode", [COALAC_FLAG_FRONT_LAUNCH, COALAC_FLAG_ONE_LAUNCH])
def test_fused_c5_share_equals_multi_launch(cuda, mode):
    ids, names = c5_share(5)
    t = mixed_table(names, 0.01)
    plan = CodecPlan(None, 0.01, 8, table=t)
    flat = synth_batch(t, cuda, client_ids=ids)
    e1, ws = encode(plan, flat, flags=mode)
    e2, _ = encode(plan, flat, flags=SEQ)
    assert plan.timeouts(ws) == 0 and same(e1, e2)


@pytest.mark.parametrize("flags", [COALAC_FLAG_FORCE_EXACT | COALAC_FLAG_FRONT_LAUNCH,
                                   COALAC_FLAG_GENERIC_SELECT | COALAC_FLAG_FRONT_LAUNCH,
                                   COALAC_FLAG_FORCE_EXACT | COALAC_FLAG_ONE_LAUNCH,
                                   COALAC_FLAG_GENERIC_SELECT | COALAC_FLAG_ONE_LAUNCH])
def test_fused_exact_and_generic_paths(cuda, flags):
    t = SegmentTable(fp32_sizes("resnet18"), 0.01, 2)
    plan = CodecPlan(None, 0.01, 8, table=t)
    flat = synth_batch(t, cuda)
    e1, ws = encode(plan, flat, flags=flags)
    e2, _ = encode(plan, flat, flags=flags & ~(COALAC_FLAG_ONE_LAUNCH | COALAC_FLAG_FRONT_LAUNCH))
    assert plan.timeouts(ws) == 0 and same(e1, e2)


def test_fused_workspace_reuse_resets_control_words(cuda):
    """Back-to-back encodes of different inputs with ONE workspace: every call must start from zeroed
    hand-off words (a stale 'sampled' / 'selected' flag would let a phase run on the previous call's
    data)."""
    t = SegmentTable(fp32_sizes("resnet50_tv"), 0.01, 2)
    plan = CodecPlan(None, 0.01, 8, table=t)
    ws = plan.empty_workspace()
    flats = [synth_batch(t, cuda, client_ids=[2 * i, 2 * i + 1]) for i in range(3)]
    refs = [encode(plan, f, flags=SEQ)[0] for f in flats]
    outs = [plan.encode(f, workspace=ws, flags=m) for m in (COALAC_FLAG_FRONT_LAUNCH, COALAC_FLAG_ONE_LAUNCH) for f in flats]
    torch.cuda.synchronize()
    assert plan.timeouts(ws) == 0
    for i, o in enumerate(outs):  # enqueued back to back on one workspace, no sync in between
        assert same(o, refs[i % 3]), i


def test_fused_plans_concurrent_on_streams(cuda):
    """Four independent plans encoding at once on four streams (each k_fused only waits on its own
    blocks; launches of other plans interleave on the CUs)."""
    ts = [SegmentTable(fp32_sizes(n), 0.01, c) for n, c in
          (("resnet50_tv", 2), ("resnet18", 3), ("vit_b16", 1), ("lenet", 5))]
    plans = [CodecPlan(None, 0.01, 8, table=t) for t in ts]
    flats = [synth_batch(t, cuda, client_ids=range(10 * i, 10 * i + t.clients)) for i, t in enumerate(ts)]
    refs = [encode(p, f, flags=SEQ)[0] for p, f in zip(plans, flats)]
    streams = [torch.cuda.Stream() for _ in plans]
    wss = [p.empty_workspace() for p in plans]
    torch.cuda.synchronize()
    outs = []
    for i, (p, f, s, ws) in enumerate(zip(plans, flats, streams, wss)):
        with torch.cuda.stream(s):
            outs.append(p.encode(f, workspace=ws, stream=s, flags=COALAC_FLAG_ONE_LAUNCH if i % 2 else COALAC_FLAG_FRONT_LAUNCH))
    torch.cuda.synchronize()
    for p, ws, o, r in zip(plans, wss, outs, refs):
        assert p.timeouts(ws) == 0 and same(o, r)
