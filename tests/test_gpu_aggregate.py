"""GPU parity of the fused server-side decode + FedAvg (coalac_aggregate).

Bar: BIT-IDENTICAL to (a) the CPU oracle's restatement (oracle.codec_oracle.aggregate) in both division
modes and (b) what the reference flow computes on the GPU: decompress every upload (coalac_decode) and
run strategies.federated_averaging (coala/server/strategies.py:6-29, 57-90) on cuda tensors, i.e.
params *= w0; params += s_i * w_i; torch.div(params, total).
"""
import copy

import numpy as np
import pytest
import torch

from coala_amd.compression import CodecPlan, CompressionClientMixin, CompressionServerMixin, Encoded, UpdateCodec
from coala_amd.compression._lib import CodecError
from coala_amd.fl import LoopbackClient, LoopbackServer, federated_averaging
from coala_amd.layouts import build_module, fp32_sizes
from coala_amd.workload import synth_batch
from oracle import codec_oracle as O

pytestmark = pytest.mark.gpu


def setup(layout, ratio, bits, clients, delta, seed=0):
    sizes = fp32_sizes(layout)
    plan = CodecPlan(sizes, ratio, bits, clients=clients)
    dev = torch.device("cuda", 0)
    flat = synth_batch(plan.table, dev, client_ids=[seed * 100 + i for i in range(clients)])
    one = CodecPlan(sizes, ratio, bits, clients=1)
    base = synth_batch(one.table, dev, client_ids=[seed * 100 + 99]) if delta else None
    # every client's update is encoded against the same global model (base repeated per client)
    base_rep = base.repeat(clients) if delta else None
    enc = plan.encode(flat, base=base_rep)
    return plan, one, enc, base


@pytest.mark.parametrize("bits", [8, 32, 2])
@pytest.mark.parametrize("ratio", [0.01, 0.1])
@pytest.mark.parametrize("delta", [True, False])
def test_aggregate_matches_oracle_both_modes(cuda, bits, ratio, delta):
    C = 5
    plan, one, enc, base = setup("resnet18", ratio, bits, C, delta, seed=bits)
    weights = [17, 0, 5, 1000, 3]
    segs = plan.table.segs.astype(np.int64)
    h = [t.cpu().numpy() for t in (enc.idx, enc.vals, enc.mn, enc.scale)]
    b = None if base is None else base.cpu().numpy()
    v1 = Encoded(enc.idx, enc.vals, enc.mn, enc.scale)  # without the per-unit starts: computed on the device
    for mode, om in (("recip", O.AGG_RECIP), ("div", O.AGG_DIV)):
        ref = O.aggregate(*h, segs, bits, C, weights, sum(weights), om, base=b, out_span=plan.table.span_per_client)
        for e in (enc, v1):
            out = plan.aggregate(e, weights, base=base, mode=mode)
            torch.cuda.synchronize()
            g = out.cpu().numpy()
            for off, n in zip(plan.table.offsets, plan.table.sizes):
                np.testing.assert_array_equal(g[off:off + n].view(np.uint32), ref[off:off + n].view(np.uint32))


@pytest.mark.parametrize("bits", [8, 32])
@pytest.mark.parametrize("delta", [True, False])
def test_aggregate_dense_plan_matches_oracle(cuda, bits, delta):
    """A dense plan (ratio 1: every element kept, indices and starts implied — the download direction's codec):
    the fused aggregate from the implied indices and the plan's cached implied starts (made once, not per call) and
    from the device-computed starts, bit-identical to the oracle over the same implied indices."""
    C = 3
    plan, one, enc, base = setup("lenet", 1.0, bits, C, delta, seed=3 + bits)
    assert plan.dense and enc.idx.numel() == 0 and enc.ustart is None
    weights = [4, 1, 7]
    segs = plan.table.segs.astype(np.int64)
    idx = plan.implied_indices()
    h = [idx.cpu().numpy()] + [t.cpu().numpy() for t in (enc.vals, enc.mn, enc.scale)]
    b = None if base is None else base.cpu().numpy()
    starts = plan.implied_starts()
    assert starts is plan.implied_starts()  # cached
    np.testing.assert_array_equal(starts.cpu().numpy(), plan.unit_starts(idx).cpu().numpy())
    explicit = Encoded(idx, enc.vals, enc.mn, enc.scale)  # explicit indices, starts computed on the device
    for mode, om in (("recip", O.AGG_RECIP), ("div", O.AGG_DIV)):
        ref = O.aggregate(*h, segs, bits, C, weights, sum(weights), om, base=b, out_span=plan.table.span_per_client)
        for e in (enc, explicit):
            out = plan.aggregate(e, weights, base=base, mode=mode)
            torch.cuda.synchronize()
            g = out.cpu().numpy()
            for off, n in zip(plan.table.offsets, plan.table.sizes):
                np.testing.assert_array_equal(g[off:off + n].view(np.uint32), ref[off:off + n].view(np.uint32))


@pytest.mark.parametrize("delta", [True, False])
def test_aggregate_matches_torch_gpu_fedavg_on_decoded(cuda, delta):
    """The reference flow on the GPU: decode each client, then weighted_sum + torch.div on cuda."""
    C = 6
    plan, one, enc, base = setup("resnet50_tv", 0.01, 8, C, delta, seed=3)
    weights = [40, 12, 7, 0, 99, 1]
    S = plan.table.span_per_client
    dense = torch.empty(C * S, dtype=torch.float32, device="cuda")
    plan.decode(enc, base=None if base is None else base.repeat(C), out=dense)
    acc = dense[0:S].clone()
    acc *= weights[0]
    for i in range(1, C):
        acc += dense[i * S:(i + 1) * S] * weights[i]
    ref = torch.div(acc, sum(weights))
    out = plan.aggregate(enc, weights, base=base, mode="recip")
    torch.cuda.synchronize()
    for off, n in zip(plan.table.offsets, plan.table.sizes):
        assert torch.equal(out[off:off + n].view(torch.int32), ref[off:off + n].view(torch.int32))


@pytest.mark.parametrize("delta", [True, False])
@pytest.mark.parametrize("mode,om", [("recip", O.AGG_RECIP), ("sum", O.AGG_SUM)])
def test_aggregate_avg_mask_matches_oracle(cuda, delta, mode, om):
    """aggregation_content "parameters": segments outside the mask (the buffers) take client 0's decoded
    value, the others are averaged — against the oracle's restatement of federated_averaging_only_params /
    weighted_sum_only_params (coala/server/strategies.py:32-54, 93-124)."""
    C = 4
    plan, one, enc, base = setup("resnet18", 0.02, 8, C, delta, seed=6)
    rng = np.random.default_rng(3)
    mask = (rng.random(len(plan.table.sizes)) < 0.6).tolist()
    mask[0], mask[1] = True, False
    weights = [5, 9, 0, 2]
    segs = plan.table.segs.astype(np.int64)
    h = [t.cpu().numpy() for t in (enc.idx, enc.vals, enc.mn, enc.scale)]
    b = None if base is None else base.cpu().numpy()
    out = plan.aggregate(enc, weights, base=base, mode=mode, avg_mask=mask)
    torch.cuda.synchronize()
    ref = O.aggregate(*h, segs, 8, C, weights, sum(weights), om, base=b, out_span=plan.table.span_per_client,
                      avg_mask=mask)
    g = out.cpu().numpy()
    for off, n in zip(plan.table.offsets, plan.table.sizes):
        np.testing.assert_array_equal(g[off:off + n].view(np.uint32), ref[off:off + n].view(np.uint32))
    with pytest.raises(ValueError):
        plan.aggregate(enc, weights, base=base, mode=mode, avg_mask=mask[:-1])


def test_fused_params_only_server_end_to_end_on_gpu(cuda):
    """Mixin with the HIP backend, aggregation_content "parameters": fused == decompress-each +
    federated_averaging_only_params on the GPU (buffers from the first upload)."""
    dev = torch.device("cuda", 0)

    class Client(CompressionClientMixin, LoopbackClient):
        codec_ratio, codec_bits, codec_mode = 0.02, 8, "delta"

    class Plain(CompressionServerMixin, LoopbackServer):
        codec_ratio, codec_bits, codec_mode = 0.02, 8, "delta"

    class Fused(Plain):
        codec_fused_aggregate = True

    class Conf:
        class server:
            aggregation_strategy = "FedAvg"
            aggregation_content = "parameters"
        is_distributed = False

    g0 = build_module("resnet18", seed=4, device=dev)
    mk = lambda: [Client(f"c{i}", [11, 3, 30][i], device=dev, step_seed=i) for i in range(3)]
    plain, fused = Plain(copy.deepcopy(g0), mk()), Fused(copy.deepcopy(g0), mk())
    plain.conf = fused.conf = Conf
    for r in range(2):
        plain.round(r)
        fused.round(r)
        for (k, a), b in zip(plain.model.state_dict().items(), fused.model.state_dict().values()):
            assert a.dtype == b.dtype and torch.equal(a, b), k


def test_aggregate_single_client_equals_decode_scaled(cuda):
    plan, one, enc, base = setup("lenet", 0.05, 8, 1, True, seed=9)
    out = plan.aggregate(enc, [4], base=base, mode="div")
    dec = plan.decode(enc, base=base)
    ref = torch.div(dec * 4, 4)
    torch.cuda.synchronize()
    for off, n in zip(plan.table.offsets, plan.table.sizes):
        assert torch.equal(out[off:off + n], ref[off:off + n])


def test_aggregate_rejects_non_copy_layouts(cuda):
    import ctypes

    from coala_amd.compression import _lib
    plan = CodecPlan([5000, 300, 7000], 0.01, 8, clients=1)
    # 3 segments cannot be 2 copies of one layout: refused before any launch
    rc = plan._lib.coalac_aggregate(plan._h, 2, None, None, None, None, None, None, ctypes.c_float(1.0), 0, None,
                                    None, None, None)
    with pytest.raises(CodecError, match="copies"):
        _lib.check(rc, "coalac_aggregate")
    with pytest.raises(ValueError):
        plan.aggregate(plan.empty_encoded(), [1, 2])  # one weight per client


def test_fused_server_end_to_end_on_gpu(cuda):
    """Mixin with the HIP backend: fused aggregation == decompress-each + federated_averaging on the GPU."""
    dev = torch.device("cuda", 0)

    class Client(CompressionClientMixin, LoopbackClient):
        codec_ratio, codec_bits, codec_mode = 0.02, 8, "delta"

    class Plain(CompressionServerMixin, LoopbackServer):
        codec_ratio, codec_bits, codec_mode = 0.02, 8, "delta"

    class Fused(Plain):
        codec_fused_aggregate = True

    g0 = build_module("resnet18_split_cut4", seed=2, device=dev)
    mk = lambda: [Client(f"c{i}", [11, 3, 30, 6][i], device=dev, step_seed=i) for i in range(4)]
    plain, fused = Plain(copy.deepcopy(g0), mk()), Fused(copy.deepcopy(g0), mk())
    for r in range(2):
        plain.round(r)
        fused.round(r)
        for (k, a), b in zip(plain.model.state_dict().items(), fused.model.state_dict().values()):
            assert a.dtype == b.dtype and torch.equal(a, b), k
    assert federated_averaging is not None


@pytest.mark.parametrize("ratio", [0.01, 0.3])
@pytest.mark.parametrize("delta", [True, False])
@pytest.mark.parametrize("mode,om", [("recip", O.AGG_RECIP), ("div", O.AGG_DIV), ("sum", O.AGG_SUM)])
def test_aggregate_many_clients_matches_oracle(cuda, ratio, delta, mode, om):
    """More clients than one 16-client chunk of the aggregate kernel (37: two full chunks and a ragged one),
    ragged units (partial last units, a segment under one unit, n = 1), light (<= 64 kept entries per unit)
    and heavy (ratio 0.3: the one-client-at-a-time path) chunks, every division mode."""
    sizes = [1, 300, 5000, 8192, 12289, 70001]
    C = 37
    plan = CodecPlan(sizes, ratio, 8, clients=C)
    one = CodecPlan(sizes, ratio, 8, clients=1)
    dev = torch.device("cuda", 0)
    flat = synth_batch(plan.table, dev, client_ids=[500 + i for i in range(C)])
    base = synth_batch(one.table, dev, client_ids=[777]) if delta else None
    enc = plan.encode(flat, base=None if base is None else base.repeat(C))
    weights = [(7 * i) % 23 for i in range(C)]
    mask = [True, False, True, True, False, True]
    segs = plan.table.segs.astype(np.int64)
    h = [t.cpu().numpy() for t in (enc.idx, enc.vals, enc.mn, enc.scale)]
    b = None if base is None else base.cpu().numpy()
    for am in (None, mask):
        out = plan.aggregate(enc, weights, base=base, mode=mode, avg_mask=am)
        torch.cuda.synchronize()
        ref = O.aggregate(*h, segs, 8, C, weights, sum(weights), om, base=b, out_span=plan.table.span_per_client,
                          avg_mask=am)
        g = out.cpu().numpy()
        for off, n in zip(plan.table.offsets, plan.table.sizes):
            np.testing.assert_array_equal(g[off:off + n].view(np.uint32), ref[off:off + n].view(np.uint32))


@pytest.mark.parametrize("bits", [8, 32])
@pytest.mark.parametrize("ratio", [0.01, 0.3])
def test_aggregate_signed_zero_and_nan_base_matches_oracle(cuda, bits, ratio):
    """x_i = base + d_i where a base of -0.0 or NaN is not base + 0.0 bit for bit: those units take the
    kernel's generic path (base from global memory), the rest the tile path. Kept -0.0 values, a zero weight
    for the first client (x_0 * 0 = -0.0 for negative x_0) and NaN bases compared NaN-for-NaN."""
    sizes = [5000, 8192, 300, 4096]
    C = 3
    plan = CodecPlan(sizes, ratio, bits, clients=C)
    one = CodecPlan(sizes, ratio, bits, clients=1)
    dev = torch.device("cuda", 0)
    flat = synth_batch(plan.table, dev, client_ids=[40 + i for i in range(C)])
    S = plan.table.span_per_client
    for c in range(C):  # a mostly-zero third segment: -0.0 entries get kept
        o = c * S + int(plan.table.offsets[2])
        flat[o:o + 300] = -0.0
        flat[o + 7] = 0.5
    base = synth_batch(one.table, dev, client_ids=[91])
    base[int(plan.table.offsets[0]):int(plan.table.offsets[0]) + 5000:97] = -0.0
    base[int(plan.table.offsets[1]) + 3] = float("nan")
    base[int(plan.table.offsets[2]):int(plan.table.offsets[2]) + 300] = 0.0
    enc = plan.encode(flat)
    weights = [0, 3, 5]
    segs = plan.table.segs.astype(np.int64)
    h = [t.cpu().numpy() for t in (enc.idx, enc.vals, enc.mn, enc.scale)]
    b = base.cpu().numpy()
    for mode, om in (("recip", O.AGG_RECIP), ("sum", O.AGG_SUM)):
        out = plan.aggregate(enc, weights, base=base, mode=mode)
        torch.cuda.synchronize()
        ref = O.aggregate(*h, segs, bits, C, weights, sum(weights), om, base=b, out_span=S)
        g = out.cpu().numpy()
        for off, n in zip(plan.table.offsets, plan.table.sizes):
            gg, rr = g[off:off + n], ref[off:off + n]
            nan = np.isnan(rr)
            np.testing.assert_array_equal(np.isnan(gg), nan)
            np.testing.assert_array_equal(gg[~nan].view(np.uint32), rr[~nan].view(np.uint32))


@pytest.mark.parametrize("bits", [8, 32])
@pytest.mark.parametrize("ratio", [0.01, 0.3])
@pytest.mark.parametrize("delta", [True, False])
def test_aggregate_more_than_64_clients_matches_oracle(cuda, bits, ratio, delta):
    """70 clients: the kernel's second 64-client chunk (its metadata and entries loaded inside the client
    loop, not with the base rows), on the fast path (0.01) and the generic one (0.3), with and without an
    averaging mask."""
    sizes = [300, 5000, 4097, 8192]
    C = 70
    plan = CodecPlan(sizes, ratio, bits, clients=C)
    one = CodecPlan(sizes, ratio, bits, clients=1)
    dev = torch.device("cuda", 0)
    flat = synth_batch(plan.table, dev, client_ids=[900 + i for i in range(C)])
    base = synth_batch(one.table, dev, client_ids=[901]) if delta else None
    enc = plan.encode(flat, base=None if base is None else base.repeat(C))
    weights = [(5 * i + 3) % 17 for i in range(C)]
    segs = plan.table.segs.astype(np.int64)
    h = [t.cpu().numpy() for t in (enc.idx, enc.vals, enc.mn, enc.scale)]
    b = None if base is None else base.cpu().numpy()
    for mode, om, am in (("recip", O.AGG_RECIP, None), ("div", O.AGG_DIV, None),
                         ("sum", O.AGG_SUM, [True, False, True, False])):
        out = plan.aggregate(enc, weights, base=base, mode=mode, avg_mask=am)
        torch.cuda.synchronize()
        ref = O.aggregate(*h, segs, bits, C, weights, sum(weights), om, base=b, out_span=plan.table.span_per_client,
                          avg_mask=am)
        g = out.cpu().numpy()
        for off, n in zip(plan.table.offsets, plan.table.sizes):
            np.testing.assert_array_equal(g[off:off + n].view(np.uint32), ref[off:off + n].view(np.uint32))


def test_fused_aggregate_recycles_idle_output_modules(cuda):
    """UpdateCodec.aggregate returns modules from the decode pool once nothing else holds them: a dropped
    result is aggregated into again (the pool does not grow), a held one is never overwritten, and every
    result equals decompress-each + federated_averaging (coala/server/strategies.py:6-29) on the GPU."""
    from coala_amd.compression import UpdateCodec
    from coala_amd.compression.codec import _recipe
    from coala_amd.fl import federated_averaging as fedavg
    dev = torch.device("cuda", 0)
    codec = UpdateCodec(0.02, 8, "delta")
    g = build_module("resnet18", seed=5, device=dev)
    base = codec.snapshot(g)
    ms = [build_module("resnet18", seed=10 + i, device=dev) for i in range(4)]
    ups = [codec.encode_module(m, base=base) for m in ms]
    wts = [3, 9, 4, 7]
    pool = _recipe(g).pool

    def reference(us):
        return fedavg([codec.decode_module(u, g, base=base) for u in us], wts).state_dict()

    def same(mod, ref):
        for (k, a), b in zip(mod.state_dict().items(), ref.values()):
            assert a.dtype == b.dtype and torch.equal(a, b), k

    assert not pool  # (a fresh template: no decoded module to recycle yet)
    first = codec.aggregate(ups, wts, g, base=base, mode="recip")
    assert len(pool) == 1 and pool[0].root is first  # built, and kept in the pool
    ident = id(first)
    del first
    assert id(codec.aggregate(ups, wts, g, base=base, mode="recip")) == ident  # aggregated into, once dropped
    first = codec.aggregate(ups, wts, g, base=base, mode="recip")
    assert len(pool) == 1
    same(first, reference(ups))
    held = {k: v.clone() for k, v in first.state_dict().items()}
    del first
    n = len(pool)
    again = codec.aggregate(ups[::-1], wts, g, base=base, mode="recip")  # a different result
    assert len(pool) == n and any(sk.root is again for sk in pool)  # an idle pooled module, aggregated into
    same(again, reference(ups[::-1]))
    keep = again
    third = codec.aggregate(ups, wts, g, base=base, mode="recip")
    assert third is not keep
    same(third, reference(ups))
    same(keep, reference(ups[::-1]))  # the held result is untouched
    assert not all(torch.equal(a, b) for a, b in zip(held.values(), keep.state_dict().values()))
