"""GPU parity of the batched pipelines (coala_amd/compression/pipeline.py): SplitPipeline sub-batches
(client ranges, or segment ranges of one update) on their own streams, writing the whole batch's buffers.
Bar: bit-identical to the oracle (and so to a single plan), for every split, including a single client
cut into segment ranges and delta mode. Repeated and alternating unjoined steps check that no sub-batch
reads a buffer another step is still writing; graph capture must record every sub-batch."""
import numpy as np
import pytest
import torch

from coala_amd.compression import CodecPlan, SegmentTable, SplitPipeline
from coala_amd.compression._lib import CodecError
from coala_amd.layouts import fp32_sizes
from coala_amd.workload import synth_batch
from oracle import codec_oracle as O

pytestmark = pytest.mark.gpu


def oracle_roundtrip(table, flat, bits, base=None):
    segs = table.segs.astype(np.int64)
    idx, vals, mn, sc = O.encode(flat, segs, bits, base=base)
    dec = O.decode(idx, vals, mn, sc, segs, bits, table.span, base=base)
    return idx, vals, mn, sc, dec


def check(table, enc, dec, ref):
    idx, vals, mn, sc, rdec = ref
    np.testing.assert_array_equal(enc.idx.cpu().numpy(), idx)
    np.testing.assert_array_equal(enc.vals.cpu().numpy().view(np.uint8), vals.view(np.uint8))
    np.testing.assert_array_equal(enc.mn.cpu().numpy().view(np.uint32), mn.view(np.uint32))
    np.testing.assert_array_equal(enc.scale.cpu().numpy().view(np.uint32), sc.view(np.uint32))
    d = dec.cpu().numpy()
    for (off, n, k, oo) in table.segs.astype(np.int64):
        np.testing.assert_array_equal(d[off:off + n].view(np.uint32), rdec[off:off + n].view(np.uint32))


@pytest.mark.parametrize("bits", [4, 32])
def test_pipeline_single_client_split(cuda, bits):
    """One client's update cut into 3 segment ranges (idx / vals shared, mn / scale sliced)."""
    t = SegmentTable(fp32_sizes("vit_b16"), 0.02, 1)
    flat = synth_batch(t, cuda, client_ids=[9])
    pipe = SplitPipeline(t, bits, split=3, device=cuda)
    assert pipe.n_parts == 3
    enc = pipe.encode(flat)
    dec = pipe.decode(enc)
    torch.cuda.synchronize()
    check(t, enc, dec, oracle_roundtrip(t, flat.cpu().numpy(), bits))


def test_pipeline_repeated_steps_stable(cuda):
    """Five back-to-back encode+decode steps into the same buffers as 4 sub-batches: every step's result
    equals the first (a missing dependency would let decode read idx/vals mid-write)."""
    t = SegmentTable(fp32_sizes("resnet50_tv"), 0.01, 4)
    flat = synth_batch(t, cuda)
    pipe = SplitPipeline(t, 8, split=4, device=cuda)
    enc, out = pipe.empty_encoded(), pipe.empty_flat()
    out.zero_()  # decode writes segments only; the alignment pads keep what was there (the oracle: 0)
    pipe.roundtrip(flat, enc=enc, out=out)
    torch.cuda.synchronize()
    first = (enc.idx.clone(), enc.vals.clone(), out.clone())
    for _ in range(5):
        pipe.roundtrip(flat, enc=enc, out=out)
    torch.cuda.synchronize()
    assert torch.equal(first[0], enc.idx) and torch.equal(first[1], enc.vals) and torch.equal(first[2], out)
    # and against the oracle, client 0 only (seconds on the CPU)
    t1 = SegmentTable(fp32_sizes("resnet50_tv"), 0.01, 1)
    S, K = t1.span_per_client, t1.total_k_per_client
    idx, vals, mn, sc, rdec = oracle_roundtrip(t1, flat[:S].cpu().numpy(), 8)
    np.testing.assert_array_equal(enc.idx[:K].cpu().numpy(), idx)
    np.testing.assert_array_equal(enc.vals[:K].cpu().numpy(), vals)
    np.testing.assert_array_equal(out[:S].cpu().numpy().view(np.uint32), rdec.view(np.uint32))


@pytest.mark.parametrize("split", [1, 2, 3])
@pytest.mark.parametrize("delta", [False, True])
@pytest.mark.parametrize("fused", [False, True])
def test_split_pipeline_resnet18_x3(cuda, split, delta, fused):
    """SplitPipeline: client sub-batches on independent streams, results in the whole batch's buffers,
    bit-identical to the oracle (3 clients into 1 / 2 / 3 sub-batches: uneven cuts included)."""
    t = SegmentTable(fp32_sizes("resnet18"), 0.01, 3)
    flat = synth_batch(t, cuda, client_ids=[7, 8, 9])
    base = synth_batch(t, cuda, client_ids=[70, 80, 90]) if delta else None
    pipe = SplitPipeline(t, 8, split=split, device=cuda)
    assert pipe.n_parts == split
    if fused:
        enc, dec = pipe.roundtrip(flat, base=base)
    else:
        enc = pipe.encode(flat, base=base)
        dec = pipe.decode(enc, base=base)
    torch.cuda.synchronize()
    check(t, enc, dec, oracle_roundtrip(t, flat.cpu().numpy(), 8, None if base is None else base.cpu().numpy()))
    assert pipe.fallbacks() == 0


@pytest.mark.parametrize("split", [2, 3])
def test_split_pipeline_unjoined_alternating_inputs(cuda, split):
    """SplitPipeline.roundtrip(joined=False) back to back with TWO alternating inputs through one shared
    Encoded and two dense outputs: each step's encode overwrites idx / vals the previous step's decode
    read, so anything but stream order per sub-batch would mix the two inputs."""
    t = SegmentTable(fp32_sizes("resnet50_tv"), 0.01, 4)
    flats = [synth_batch(t, cuda, client_ids=range(4)), synth_batch(t, cuda, client_ids=range(10, 14))]
    pipe = SplitPipeline(t, 8, split=split, device=cuda)
    enc = pipe.empty_encoded()
    outs = [pipe.empty_flat().zero_(), pipe.empty_flat().zero_()]
    torch.cuda.synchronize()
    for i in range(6):
        pipe.roundtrip(flats[i % 2], enc=enc, out=outs[i % 2], joined=False)
    torch.cuda.synchronize()
    plan = CodecPlan(fp32_sizes("resnet50_tv"), 0.01, 8, clients=4, device=cuda)
    for j in range(2):
        e = plan.encode(flats[j])
        d = plan.decode(e, out=torch.zeros_like(outs[j]))
        torch.cuda.synchronize()
        assert torch.equal(d.view(torch.int32), outs[j].view(torch.int32)), j
    e1 = plan.encode(flats[1])  # the last step encoded flats[1]
    torch.cuda.synchronize()
    assert torch.equal(e1.idx, enc.idx) and torch.equal(e1.vals, enc.vals)


def test_split_pipeline_unjoined_steps_match_single_plan(cuda):
    """The bench's schedule: 6 back-to-back unjoined roundtrips of 16 ResNet-50 updates as 2 x 8 (plus
    the batch's small segments forked per sub-plan) equal one plan over the whole batch, bit for bit."""
    t = SegmentTable(fp32_sizes("resnet50_tv"), 0.01, 16)
    flat = synth_batch(t, cuda)
    pipe = SplitPipeline(t, 8, split=2, device=cuda)
    enc, out = pipe.empty_encoded(), pipe.empty_flat()
    out.zero_()
    for _ in range(6):
        pipe.roundtrip(flat, enc=enc, out=out, joined=False)
    torch.cuda.synchronize()
    plan = CodecPlan(fp32_sizes("resnet50_tv"), 0.01, 8, clients=16, device=cuda)
    e1 = plan.encode(flat)
    d1 = torch.zeros_like(out)
    plan.decode(e1, out=d1)
    torch.cuda.synchronize()
    assert torch.equal(enc.idx, e1.idx) and torch.equal(enc.vals, e1.vals)
    assert torch.equal(enc.mn, e1.mn) and torch.equal(enc.scale, e1.scale)
    assert torch.equal(out, d1)


@pytest.mark.parametrize("split", [2, 3, 4])
@pytest.mark.parametrize("delta", [False, True])
def test_split_pipeline_single_update_segment_ranges(cuda, split, delta):
    """One update into `split` segment ranges (SplitPipeline with fewer clients than sub-batches): each
    range a plan over absolute segment rows on its own stream, writing the shared buffers in place; the
    result is the oracle's, bit for bit, and equal to one plan over the whole update."""
    t = SegmentTable(fp32_sizes("resnet50_tv"), 0.01, 1)
    flat = synth_batch(t, cuda, client_ids=[3])
    base = synth_batch(t, cuda, client_ids=[30]) if delta else None
    pipe = SplitPipeline(t, 8, split=split, device=cuda)
    assert pipe.n_parts == split
    enc, dec = pipe.roundtrip(flat, base=base)
    torch.cuda.synchronize()
    check(t, enc, dec, oracle_roundtrip(t, flat.cpu().numpy(), 8, None if base is None else base.cpu().numpy()))
    assert pipe.fallbacks() == 0


def test_split_pipelines_share_pooled_streams(cuda):
    """Every SplitPipeline of a process takes sub-batch g's stream from one pool (pooled_streams): two
    pipelines over different tables share them, and their unjoined calls, interleaved, stay correct (the
    shared stream orders them) and equal single plans."""
    from coala_amd.compression.pipeline import pooled_streams
    ta = SegmentTable(fp32_sizes("resnet18"), 0.01, 4)
    tb = SegmentTable(fp32_sizes("lenet"), 0.05, 6)
    pa, pb = SplitPipeline(ta, 8, split=2, device=cuda), SplitPipeline(tb, 8, split=3, device=cuda)
    pool = pooled_streams(cuda, 3)
    assert pa.streams == pool[:2] and pb.streams == pool[:3]
    fa, fb = synth_batch(ta, cuda), synth_batch(tb, cuda, client_ids=range(20, 26))
    ea, oa = pa.empty_encoded(), pa.empty_flat().zero_()
    eb, ob = pb.empty_encoded(), pb.empty_flat().zero_()
    torch.cuda.synchronize()
    for _ in range(3):
        pa.roundtrip(fa, enc=ea, out=oa, joined=False)
        pb.roundtrip(fb, enc=eb, out=ob, joined=False)
    torch.cuda.synchronize()
    for t, f, e, o in ((ta, fa, ea, oa), (tb, fb, eb, ob)):
        plan = CodecPlan(None, t.ratio, 8, table=t, device=cuda)
        e1 = plan.encode(f)
        d1 = plan.decode(e1, out=torch.zeros_like(o))
        torch.cuda.synchronize()
        assert torch.equal(e1.idx, e.idx) and torch.equal(e1.vals, e.vals)
        assert torch.equal(d1.view(torch.int32), o.view(torch.int32))


def test_decode_without_starts_computes_them(cuda):
    """ABI 5: the sparse decode reads every unit's entry range from the per-unit starts (wire v2). A payload without
    them (a version-1 blob) has them computed on the device by the host (CodecPlan.unit_starts): equal to the
    encoder's own, and the decode equal to the one with the shipped starts — for a latency-bound plan, a batch plan
    and a plan over absolute segment rows (SplitPipeline's ranges of one update). The raw ABI refuses a NULL."""
    import ctypes

    from coala_amd.compression import Encoded, _lib
    for clients in (1, 4):
        t = SegmentTable(fp32_sizes("resnet50_tv"), 0.01, clients)
        flat = synth_batch(t, cuda, client_ids=range(clients))
        plan = CodecPlan(None, 0.01, 8, table=t, device=cuda)
        e2 = plan.encode(flat)
        e = Encoded(e2.idx, e2.vals, e2.mn, e2.scale)
        assert torch.equal(plan.unit_starts(e.idx), e2.ustart)
        ref = plan.decode(e2, out=torch.zeros_like(flat))
        out = plan.decode(e, out=torch.zeros_like(flat))
        torch.cuda.synchronize()
        assert torch.equal(out.view(torch.int32), ref.view(torch.int32))
        rc = plan._lib.coalac_decode(plan._h, ctypes.c_void_p(e.idx.data_ptr()), ctypes.c_void_p(e.vals.data_ptr()),
                                     ctypes.c_void_p(e.mn.data_ptr()), ctypes.c_void_p(e.scale.data_ptr()), None, None,
                                     ctypes.c_void_p(out.data_ptr()), None)
        with pytest.raises(CodecError, match="ustart"):
            _lib.check(rc, "coalac_decode")
    t1 = SegmentTable(fp32_sizes("resnet50_tv"), 0.01, 1)
    rows = t1.segs[100:180]
    sub = CodecPlan.from_segments(rows, 8, device=cuda)
    f1 = synth_batch(t1, cuda, client_ids=[9])
    full = CodecPlan(None, 0.01, 8, table=t1, device=cuda)
    ef = full.encode(f1)
    uo = [0]
    for n in t1.segs[:, 1].tolist():
        uo.append(uo[-1] + (int(n) + 4095) // 4096)
    assert torch.equal(sub.unit_starts(ef.idx), ef.ustart[uo[100]:uo[180]])


def test_split_pipelines_in_flight_on_disjoint_streams(cuda):
    """bench.py's single_x2: two single-update pipelines on disjoint pooled streams (stream_base), steps
    alternating between them unjoined, so consecutive updates overlap; each keeps its own buffers and the
    results equal a plain plan's, bit for bit."""
    from coala_amd.compression.pipeline import pooled_streams
    t = SegmentTable(fp32_sizes("resnet50_tv"), 0.01, 1)
    flats = [synth_batch(t, cuda, client_ids=[7]), synth_batch(t, cuda, client_ids=[8])]
    pipes = [SplitPipeline(t, 8, split=1, device=cuda, stream_base=j) for j in range(2)]
    assert pipes[0].streams == pooled_streams(cuda, 1) and pipes[1].streams == pooled_streams(cuda, 2)[1:]
    bufs = [(p.empty_encoded(), p.empty_flat().zero_()) for p in pipes]
    torch.cuda.synchronize()
    for i in range(6):
        pipes[i % 2].roundtrip(flats[i % 2], enc=bufs[i % 2][0], out=bufs[i % 2][1], joined=False)
    torch.cuda.synchronize()
    plan = CodecPlan(fp32_sizes("resnet50_tv"), 0.01, 8, clients=1, device=cuda)
    for j in range(2):
        e = plan.encode(flats[j])
        d = plan.decode(e, out=torch.zeros_like(flats[j]))
        torch.cuda.synchronize()
        assert torch.equal(e.idx, bufs[j][0].idx) and torch.equal(e.vals, bufs[j][0].vals), j
        assert torch.equal(d.view(torch.int32), bufs[j][1].view(torch.int32)), j


def test_single_update_roundtrip_graph_replay(cuda):
    """bench.py's latency-bound configs replay each step as a captured hipGraph: the captured roundtrip of
    one update (every kernel of the encode and the decode, launched through the C ABI on the capture
    stream) replayed on new input data in the same buffers gives exactly the eager result."""
    t = SegmentTable(fp32_sizes("resnet50_tv"), 0.01, 1)
    flat = synth_batch(t, cuda, client_ids=[21])
    pipe = SplitPipeline(t, 8, split=1, device=cuda)
    enc, out = pipe.empty_encoded(), pipe.empty_flat().zero_()
    pipe.roundtrip(flat, enc=enc, out=out, joined=False)  # warm-up (eager)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=pipe.streams[0]):
        pipe.roundtrip(flat, enc=enc, out=out, joined=False)
    torch.cuda.synchronize()
    flat.copy_(synth_batch(t, cuda, client_ids=[22]))  # new data, same buffers
    torch.cuda.synchronize()
    for _ in range(3):
        with torch.cuda.stream(pipe.streams[0]):
            g.replay()
    torch.cuda.synchronize()
    plan = CodecPlan(fp32_sizes("resnet50_tv"), 0.01, 8, clients=1, device=cuda)
    e = plan.encode(flat)
    d = plan.decode(e, out=torch.zeros_like(flat))
    torch.cuda.synchronize()
    assert torch.equal(e.idx, enc.idx) and torch.equal(e.vals, enc.vals)
    assert torch.equal(e.mn, enc.mn) and torch.equal(e.scale, enc.scale)
    assert torch.equal(d.view(torch.int32), out.view(torch.int32))


@pytest.mark.parametrize("split", [1, 2])
def test_split_pipeline_graph_capture_records_every_part(cuda, split):
    """bench.py captures its latency-bound steps as hipGraphs on a capture stream of its own with the
    pipeline's joined roundtrip, so every sub-batch stream forks from and joins back into the capture: a
    replay re-runs ALL parts (an unjoined capture on part 0's stream left parts 1.. out of the
    graph). Replayed on new data in the same buffers, the graph gives the eager result for split 1 and 2."""
    t = SegmentTable(fp32_sizes("resnet50_tv"), 0.01, 2)
    flat = synth_batch(t, cuda, client_ids=[31, 32])
    pipe = SplitPipeline(t, 8, split=split, device=cuda)
    assert pipe.n_parts == split
    enc, out = pipe.empty_encoded(), pipe.empty_flat().zero_()
    pipe.roundtrip(flat, enc=enc, out=out)  # warm-up (eager)
    torch.cuda.synchronize()
    cap = torch.cuda.Stream(cuda)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=cap):
        for _ in range(2):
            pipe.roundtrip(flat, enc=enc, out=out, joined=True)
    torch.cuda.synchronize()
    flat.copy_(synth_batch(t, cuda, client_ids=[41, 42]))
    enc.idx.zero_()
    out.zero_()
    torch.cuda.synchronize()
    with torch.cuda.stream(pipe.streams[0]):
        g.replay()
    torch.cuda.synchronize()
    plan = CodecPlan(None, 0.01, 8, table=t, device=cuda)
    e = plan.encode(flat)
    d = plan.decode(e, out=torch.zeros_like(flat))
    torch.cuda.synchronize()
    assert torch.equal(e.idx, enc.idx) and torch.equal(e.vals, enc.vals)
    assert torch.equal(d.view(torch.int32), out.view(torch.int32))
