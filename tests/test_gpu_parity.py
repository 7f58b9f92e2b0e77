"""GPU parity: HIP kernels (through the C ABI) vs the CPU oracle, bit-exact.

Tolerance (written here as the bar): indices, codes, mn, scale, the wire v2 per-unit starts and decoded values
must be BIT-IDENTICAL to oracle/codec_oracle.py (both follow the same fp32 op order with no FMA). The spec's
guaranteed bound, if a rounding-boundary case ever differed, would be one quantisation step;
we do not use it — any difference fails. Every decode runs twice: from the encoder's per-unit starts (wire v2)
and without them (a v1 payload: the host computes them on the device, CodecPlan.unit_starts).
"""
import numpy as np
import pytest
import torch

from coala_amd.compression import CodecPlan, Encoded, SegmentTable
from coala_amd.compression._lib import COALAC_FLAG_FORCE_EXACT, COALAC_FLAG_GENERIC_SELECT
from coala_amd.compression.spec import SMALL_MAX, SMALL_MAX_LATENCY, small_limit
from coala_amd.layouts import fp32_sizes
from coala_amd.workload import synth_batch
from oracle import codec_oracle as O

pytestmark = pytest.mark.gpu


def to_flat(table, xs):
    flat = np.zeros(table.span, dtype=np.float32)
    for c in range(table.clients):
        for t, (off, n) in enumerate(zip(table.offsets, table.sizes)):
            o = c * table.span_per_client + off
            flat[o:o + n] = xs[c][t]
    return flat


def run_both(sizes, ratio, bits, xs, bases=None, flags=0, clients=1, brackets=False):
    plan = CodecPlan(sizes, ratio, bits, clients=clients)
    table = plan.table
    flat = to_flat(table, xs)
    base = None if bases is None else to_flat(table, bases)
    d_flat = torch.from_numpy(flat).cuda()
    d_base = None if base is None else torch.from_numpy(base).cuda()
    ws = plan.empty_workspace()
    # (idx and starts asked for even at ratio 1, where a dense plan's are implied: the library writes them when
    # given buffers; the dense decode reads neither)
    enc = plan.encode(d_flat, base=d_base, workspace=ws, flags=flags, out=plan.empty_encoded(with_idx=True))
    dec = plan.decode(enc, base=d_base)
    dec_v1 = plan.decode(Encoded(enc.idx, enc.vals, enc.mn, enc.scale), base=d_base)  # no per-unit starts
    torch.cuda.synchronize()
    g = dict(idx=enc.idx.cpu().numpy(), vals=enc.vals.cpu().numpy(), mn=enc.mn.cpu().numpy(),
             scale=enc.scale.cpu().numpy(), ustart=enc.ustart.cpu().numpy(), dec=dec.cpu().numpy(),
             dec_v1=dec_v1.cpu().numpy(), fallbacks=plan.fallbacks(ws))
    if brackets:  # the sampled {T_lo, T_hi} of every large unit (coalac_debug_brackets)
        import ctypes
        nl = sum((int(n) + 4095) // 4096 for n in table.segs[:, 1] if n > small_limit(table.segs[:, 1]))
        lo, hi = (ctypes.c_uint32 * max(nl, 1))(), (ctypes.c_uint32 * max(nl, 1))()
        got = plan._lib.coalac_debug_brackets(plan._h, ctypes.c_void_p(ws.data_ptr()), None, lo, hi, nl)
        assert got == nl, (got, nl)
        g["tlo"], g["thi"] = np.frombuffer(lo, np.uint32)[:nl].copy(), np.frombuffer(hi, np.uint32)[:nl].copy()
    segs = table.segs.astype(np.int64)
    idx, vals, mn, sc = O.encode(flat, segs, bits, base=base)
    ref_dec = O.decode(idx, vals, mn, sc, segs, bits, table.span, base=base)
    r = dict(idx=idx, vals=vals, mn=mn, scale=sc, ustart=O.unit_starts(idx, segs), dec=ref_dec)
    return plan, g, r


def assert_same(plan, g, r):
    t = plan.table
    np.testing.assert_array_equal(g["idx"], r["idx"])
    np.testing.assert_array_equal(g["vals"].view(np.uint8), r["vals"].view(np.uint8))
    np.testing.assert_array_equal(g["mn"].view(np.uint32), r["mn"].view(np.uint32))
    np.testing.assert_array_equal(g["scale"].view(np.uint32), r["scale"].view(np.uint32))
    np.testing.assert_array_equal(g["ustart"], r["ustart"])
    for (off, n, k, oo) in t.segs.astype(np.int64):
        np.testing.assert_array_equal(g["dec"][off:off + n].view(np.uint32), r["dec"][off:off + n].view(np.uint32))
        np.testing.assert_array_equal(g["dec_v1"][off:off + n].view(np.uint32), r["dec"][off:off + n].view(np.uint32))


def gauss(rng, sizes, lo=-4, hi=-2):
    return [(rng.standard_normal(n) * 10 ** rng.uniform(lo, hi)).astype(np.float32) for n in sizes]


# -- edge cases ---------------------------------------------------------------------------------------
def edge_segments(rng):
    segs = []
    segs.append(np.array([3.0], np.float32))                                    # n = 1
    segs.append(np.array([-0.0, 0.0, -0.0, 0.0, 0.0], np.float32))              # signed zeros, all ties
    segs.append(np.full(37, 0.25, np.float32))                                  # constant -> scale 0
    segs.append(np.array([1, -1, 1, -1, 2, -2, 2, -2, 0.5], np.float32))        # equal magnitudes, signs
    segs.append(np.array([1e-40, -1e-41, 3e-39, 0, 1e-45, -1e-45], np.float32))  # denormals
    segs.append(np.array([np.inf, -1.0, 2.0, 0.5, -np.inf, 3.0], np.float32))   # infinities
    segs.append(np.array([np.nan, 1.0, -2.0, 0.25, 7.0, -7.0, np.nan], np.float32))  # NaN keys sort on top
    segs.append(np.zeros(SMALL_MAX, np.float32))                                # all zero, SMALL_MAX
    x = rng.standard_normal(SMALL_MAX + 1).astype(np.float32)                   # smallest large segment
    segs.append(x)
    segs.append(rng.standard_normal(SMALL_MAX_LATENCY).astype(np.float32))      # largest small, latency plans
    x = np.round(rng.standard_normal(SMALL_MAX_LATENCY + 1) * 2).astype(np.float32)  # smallest large there, ties
    segs.append(x)
    x = np.round(rng.standard_normal(50000) * 4).astype(np.float32) / 4         # heavy ties, large
    segs.append(x)
    segs.append(np.zeros(20000, np.float32))                                    # all-zero large
    x = rng.standard_normal(4096 * 3 + 5).astype(np.float32)                    # ragged tail unit
    segs.append(x)
    segs.append(rng.standard_normal(3).astype(np.float32))
    return segs


@pytest.mark.parametrize("small_max", [None, SMALL_MAX])
@pytest.mark.parametrize("flags", [0, COALAC_FLAG_GENERIC_SELECT])
@pytest.mark.parametrize("bits", [8, 4, 1, 32])
@pytest.mark.parametrize("ratio", [0.001, 0.01, 0.1, 0.5, 1.0])
def test_edge_cases(cuda, bits, ratio, flags, small_max, monkeypatch):
    """small_max None: the plan's own threshold (latency plan: segments of 1025..4096 elements take the
    sampled path); SMALL_MAX: forced, so those segments are encoded whole in one block."""
    if small_max is not None:
        monkeypatch.setenv("COALAC_SMALL_MAX", str(small_max))
    rng = np.random.default_rng(7)
    segs = edge_segments(rng)
    plan, g, r = run_both([s.size for s in segs], ratio, bits, [segs], flags=flags)
    assert_same(plan, g, r)


@pytest.mark.parametrize("flags", [0, COALAC_FLAG_FORCE_EXACT, COALAC_FLAG_GENERIC_SELECT])
@pytest.mark.parametrize("delta", [False, True])
def test_random_layout_resnet18(cuda, flags, delta):
    rng = np.random.default_rng(11)
    sizes = fp32_sizes("resnet18")
    xs = [gauss(rng, sizes)]
    bases = [gauss(rng, sizes, -2, -1)] if delta else None
    plan, g, r = run_both(sizes, 0.01, 8, xs, bases, flags)
    assert_same(plan, g, r)
    if flags == COALAC_FLAG_FORCE_EXACT:
        assert g["fallbacks"] == plan.table.n_segments - sum(1 for s in sizes if s <= small_limit(sizes))


@pytest.mark.parametrize("ratio", [0.001, 0.01, 0.1])
def test_batched_clients_resnet50_layout(cuda, ratio):
    rng = np.random.default_rng(int(ratio * 1e4))
    sizes = fp32_sizes("resnet50_tv")
    xs = [gauss(rng, sizes) for _ in range(2)]
    plan, g, r = run_both(sizes, ratio, 8, xs, clients=2)
    assert_same(plan, g, r)
    assert g["fallbacks"] == 0


@pytest.mark.parametrize("delta", [False, True])
def test_forked_small_segments_resnet50_x3(cuda, delta):
    """>= 16384 large units: the small segments are encoded by k_small on the plan's side stream,
    concurrently with k_sample / k_scan, and joined back before the encode returns."""
    rng = np.random.default_rng(33 + delta)
    sizes = fp32_sizes("resnet50_tv")
    xs = [gauss(rng, sizes) for _ in range(3)]
    bases = [gauss(rng, sizes) for _ in range(3)] if delta else None
    plan, g, r = run_both(sizes, 0.01, 8, xs, bases=bases, clients=3)
    assert plan.n_units - sum(1 for n in sizes if 0 < n <= small_limit(sizes * 3)) * 3 >= 16384
    assert_same(plan, g, r)


@pytest.mark.parametrize("name", ["lenet", "vit_b16", "resnet18_split_cut4", "simple_cnn_split_cut2"])
def test_layouts(cuda, name):
    rng = np.random.default_rng(3)
    sizes = fp32_sizes(name)
    plan, g, r = run_both(sizes, 0.01, 8, [gauss(rng, sizes)])
    assert_same(plan, g, r)


def _hash32(x):
    x = np.uint64(x) & np.uint64(0xFFFFFFFF)
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x7FEB352D)) & np.uint64(0xFFFFFFFF)
    x ^= x >> np.uint64(15)
    x = (x * np.uint64(0x846CA68B)) & np.uint64(0xFFFFFFFF)
    x ^= x >> np.uint64(16)
    return int(x)


def sampled_positions(n, seg_index):
    """Positions the sampler reads for a large segment (restates sample_thresholds in coalac.hip)."""
    R = max(64, min(512, n // 512)) & ~63
    stride = n // R
    room = stride - 16
    pos = np.zeros(n, bool)
    for run in range(R):
        h = _hash32(((run * 0x9E3779B9) & 0xFFFFFFFF) ^ (((seg_index + 1) * 0x85EBCA6B) & 0xFFFFFFFF))
        start = (run * stride + h % (room + 1)) & ~3
        pos[start:start + 16] = True
    return pos


def test_bracket_miss_forces_exact_reselection(cuda):
    """Adversarial input: the large values sit exactly where the sampler does not look, so the sampled
    bracket misses (count(A) > k) and the in-launch exact re-selection branch must produce the result."""
    n = 1 << 20
    rng = np.random.default_rng(5)
    x = (rng.standard_normal(n) * 1e-3).astype(np.float32)
    seen = sampled_positions(n, 0)
    unseen = np.flatnonzero(~seen)
    big = rng.choice(unseen, size=30000, replace=False)
    x[big] = (rng.standard_normal(big.size) * 10).astype(np.float32)
    plan, g, r = run_both([n], 0.01, 8, [[x]])
    assert g["fallbacks"] == 1
    assert_same(plan, g, r)


def test_raw_bits_idempotent(cuda):
    """bits = 32: decode(encode(x)) is x masked to its top-k, and re-encoding it is a fixed point."""
    sizes = fp32_sizes("resnet18")
    plan = CodecPlan(sizes, 0.05, 32, clients=2)
    flat = synth_batch(plan.table, cuda)
    e1 = plan.encode(flat)
    d1 = plan.decode(e1)
    e2 = plan.encode(d1)
    torch.cuda.synchronize()
    assert torch.equal(e1.idx, e2.idx) and torch.equal(e1.vals, e2.vals)


@pytest.mark.parametrize("starts", ["none", "garbage"])
@pytest.mark.parametrize("clients", [1, 3])
@pytest.mark.parametrize("kind", ["random", "reversed", "out_of_range", "duplicates"])
def test_decode_untrusted_idx_stays_in_bounds(cuda, kind, clients, starts):
    """A corrupt idx list or corrupt per-unit starts (the blob may be untrusted) can mis-decode but never write
    outside its segment: the decode kernels' unit ranges are clamped and every kept entry is bounds-checked
    against its unit. Sentinels after the span and in the alignment pads between segments must survive. clients
    3 makes a plan of > 8192 units (the batch decode), 1 a latency-bound one."""
    sizes = [5000, 70, 9000, 4096 * 3 + 5] + ([4096 * 4000] if clients == 3 else [])
    plan = CodecPlan(sizes, 0.1, 8, clients=clients)
    t = plan.table
    rng = np.random.default_rng(11)
    enc = plan.empty_encoded()
    K = plan.total_k
    if kind == "random":
        idx = rng.integers(0, 20000, K, dtype=np.int64)
    elif kind == "reversed":
        idx = np.concatenate([np.arange(k)[::-1] for k in t.ks] * clients)
    elif kind == "out_of_range":
        idx = rng.integers(-(2 ** 31), 2 ** 31 - 1, K, dtype=np.int64)
    else:
        idx = np.zeros(K, np.int64)
    enc.idx.copy_(torch.from_numpy(idx.astype(np.int32)))
    enc.vals.copy_(torch.from_numpy(rng.integers(0, 256, K, dtype=np.uint8)))
    enc.mn.fill_(1.0)
    enc.scale.fill_(0.5)
    if starts == "none":
        enc.ustart = None
    else:
        enc.ustart.copy_(torch.from_numpy(rng.integers(-(2 ** 31), 2 ** 31 - 1, plan.n_units, dtype=np.int64)
                                          .astype(np.int32)))
    sentinel = 12345.0
    out = torch.full((t.span + 1024,), sentinel, dtype=torch.float32, device="cuda")
    plan.decode(enc, out=out)
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    inside = np.zeros(o.size, bool)
    for (off, n, k, oo) in t.segs.astype(np.int64):
        inside[off:off + n] = True
        seg = o[off:off + n]
        assert np.all((seg == 0.0) | ((seg >= 1.0) & (seg <= 1.0 + 255 * 0.5)))
    assert np.all(o[~inside] == sentinel)


GOLD_NPZ = __import__("os").path.join(__import__("os").path.dirname(__file__), "golden", "codec_vectors.npz")


@pytest.mark.parametrize("bits", [1, 4, 8, 32])
@pytest.mark.parametrize("ratio", [0.001, 0.01, 0.3, 1.0])
def test_golden_vectors_bit_exact(cuda, ratio, bits):
    """Every committed golden case (tests/golden/codec_vectors.npz: ties, signed zeros, denormals, NaN / inf
    keys, constant segments, half-to-even rounding, n = 1, k = 1, k = n) × this ratio × bits, encoded as
    the segments of one batched plan: idx, codes, mn, scale and the dense decode equal the committed
    vectors bit for bit."""
    gold = np.load(GOLD_NPZ)
    names = sorted({k.split("/")[0] for k in gold.files})
    xs = [gold[f"{n}/x"] for n in names]
    plan = CodecPlan([x.size for x in xs], ratio, bits)
    t = plan.table
    flat = np.zeros(t.span, np.float32)
    for off, x in zip(t.offsets, xs):
        flat[off:off + x.size] = x
    enc = plan.encode(torch.from_numpy(flat).cuda(), out=plan.empty_encoded(with_idx=True))
    dec = plan.decode(enc).cpu().numpy()
    idx, vals = enc.idx.cpu().numpy(), enc.vals.cpu().numpy()
    mn, sc = enc.mn.cpu().numpy(), enc.scale.cpu().numpy()
    np.testing.assert_array_equal(enc.ustart.cpu().numpy(), O.unit_starts(idx, t.segs.astype(np.int64)))
    for s, (n, (off, _, k, oo)) in enumerate(zip(names, t.segs.astype(np.int64))):
        tag = f"{n}/r{ratio}/b{bits}"
        assert int(gold[f"{tag}/k"][0]) == k, tag
        np.testing.assert_array_equal(idx[oo:oo + k], gold[f"{tag}/idx"], err_msg=tag)
        np.testing.assert_array_equal(vals[oo:oo + k].view(np.uint8), gold[f"{tag}/vals"].view(np.uint8), err_msg=tag)
        np.testing.assert_array_equal(np.array([mn[s], sc[s]], np.float32).view(np.uint32),
                                      gold[f"{tag}/mn_scale"].view(np.uint32), err_msg=tag)
        np.testing.assert_array_equal(dec[off:off + xs[s].size].view(np.uint32), gold[f"{tag}/dec"].view(np.uint32),
                                      err_msg=tag)


@pytest.mark.parametrize("delta", [False, True])
def test_record_slot_overflow_takes_raw_path(cuda, monkeypatch, delta):
    """The candidate workspace is capped per unit (plan ccap); a unit that finds more candidates than its
    slots sends its segment to the raw-data path (exact k-th key of the raw segment, per-unit counts and
    the emit re-read from the raw data). Forced here with COALAC_CCAP=512 at ratio 0.3: bit-exact."""
    monkeypatch.setenv("COALAC_CCAP", "512")
    rng = np.random.default_rng(21 + delta)
    sizes = fp32_sizes("resnet18")
    xs = [gauss(rng, sizes)]
    bases = [gauss(rng, sizes, -2, -1)] if delta else None
    plan, g, r = run_both(sizes, 0.3, 8, xs, bases)
    assert_same(plan, g, r)
    assert g["fallbacks"] > 0


def test_workspace_is_capped(cuda):
    """16 ResNet-50 updates at ratio 0.01: the encode workspace is about 1 B per element (round 1: 8)."""
    sizes = fp32_sizes("resnet50_tv")
    plan = CodecPlan(sizes, 0.01, 8, clients=16)
    n = plan.table.n_elements
    assert plan.ws_bytes < 1.5 * n, plan.ws_bytes / n


@pytest.mark.parametrize("delta", [False, True])
def test_scan_stage_overflow_in_a_batch(cuda, delta):
    """k_scan stages a unit's first 512 candidate records per wave in LDS and stores the rest directly
    (coalac.hip scan_unit). One unit of a 2-client ResNet-50 batch plan (> 8192 units: the staged scan) gets
    450 large values on top of its ~300 ordinary candidates at ratio 0.05 (> 512, inside the plan's 896
    record slots, so no raw-path fallback): bit-exact against the oracle."""
    rng = np.random.default_rng(5 + delta)
    sizes = fp32_sizes("resnet50_tv")
    xs = [gauss(rng, sizes) for _ in range(2)]
    big = int(np.argmax(sizes))
    x = xs[0][big]
    lo = 5 * 4096
    pick = rng.choice(4096, 450, replace=False) + lo
    x[pick] = (rng.standard_normal(450) * 100.0 + 500.0).astype(np.float32)
    bases = [gauss(rng, sizes, -2, -1) for _ in range(2)] if delta else None
    plan, g, r = run_both(sizes, 0.05, 8, xs, bases, clients=2)
    assert plan.n_units > 8192  # a batch plan
    assert_same(plan, g, r)
    assert g["fallbacks"] == 0


def frozen_segments(rng, sizes, trained):
    """Delta-mode inputs of a frozen backbone (FedPEFT freezes every ViT parameter but the head and the LoRA
    adapters, /root/reference/application/FedPEFT/lora.py:64, main.py:62-67): the trained tensors move, every
    other one is exactly its base (an all-zero delta)."""
    bases = gauss(rng, sizes, -2, -1)
    xs = [b + d if i in trained else b.copy() for i, (b, d) in enumerate(zip(bases, gauss(rng, sizes)))]
    return xs, bases


@pytest.mark.parametrize("ratio", [0.001, 0.01, 0.1])
@pytest.mark.parametrize("clients", [1, 2])
def test_frozen_backbone_takes_the_zero_tie_path(cuda, ratio, clients):
    """An all-zero delta segment brackets at key 0: its zeros are counted, not recorded, and the k-th key is a
    zero with a tie quota over them (no raw-data fallback). ViT-B/16 with only the head trained: bit-exact,
    no fallback, in a latency-bound plan (1 client) and a batch plan (2 clients)."""
    rng = np.random.default_rng(77 + clients)
    sizes = fp32_sizes("vit_b16")
    trained = {len(sizes) - 2, len(sizes) - 1}  # fc.weight, fc.bias
    xs, bases = zip(*[frozen_segments(rng, sizes, trained) for _ in range(clients)])
    plan, g, r = run_both(sizes, ratio, 8, list(xs), list(bases), clients=clients)
    assert_same(plan, g, r)
    assert g["fallbacks"] == 0


@pytest.mark.parametrize("nnz_frac", [0.0, 0.002, 0.006, 0.05])
@pytest.mark.parametrize("bits", [8, 32])
def test_sparse_segments_zero_tie_path(cuda, nnz_frac, bits):
    """Weights-mode segments with fewer nonzeros than k (pruned tensors; +0 / -0 mixed) and with more: the k-th
    key is a zero exactly when nnz < k. Ragged last units, several segment sizes: bit-exact, no fallback."""
    rng = np.random.default_rng(int(nnz_frac * 1e4) + bits)
    sizes = [20000, 4096 * 7 + 3, 250000, 1 << 20, 1500]
    xs = []
    for n in sizes:
        x = np.where(rng.random(n) < 0.5, np.float32(0.0), np.float32(-0.0)).astype(np.float32)
        m = int(nnz_frac * n)
        pos = rng.choice(n, m, replace=False)
        x[pos] = (rng.standard_normal(m) * 1e-3).astype(np.float32)
        xs.append(x)
    plan, g, r = run_both(sizes, 0.01, bits, [xs])
    assert_same(plan, g, r)
    assert g["fallbacks"] == 0


def tie_segments(rng, sizes, case):
    """Segments whose k-th key (ratio 0.01 and 0.1) is one heavily repeated NONZERO key K."""
    xs = []
    c = np.float32(1e-3)
    for n in sizes:
        sgn = np.where(rng.random(n) < 0.5, -c, c).astype(np.float32)
        g = (rng.standard_normal(n) * 1e-3).astype(np.float32)
        if case == "sign":  # sign-SGD / first Adam step: every |x| equal
            x = sgn
        elif case == "clipped":  # value clipping at 1.5 sigma: ~13 % of the elements at +-clip
            x = np.clip(g, -1.5e-3, 1.5e-3).astype(np.float32)
        elif case == "outliers":  # 0.3 % larger values above a sea of equal |x| (the quota takes the first K-keys)
            x = sgn.copy()
            m = max(1, int(0.003 * n))
            pos = rng.choice(n, m, replace=False)
            x[pos] = (np.sign(rng.standard_normal(m)) * (2e-3 + np.abs(rng.standard_normal(m)) * 1e-3)).astype(np.float32)
        elif case == "half_zero":  # +-0 and equal |x| half each
            x = np.where(rng.random(n) < 0.5, np.float32(0.0), sgn).astype(np.float32)
            x[rng.random(n) < 0.25] = np.float32(-0.0)
        else:  # "grid": a 5-level quantised tensor (values in {0, +-c, +-2c}), the k-th key inside the top level
            x = (np.clip(np.round(g / 7e-4), -2, 2) * c).astype(np.float32)
        xs.append(x)
    return xs


@pytest.mark.parametrize("case", ["sign", "clipped", "outliers", "half_zero", "grid"])
@pytest.mark.parametrize("clients", [1, 2])
def test_heavy_ties_take_the_tie_path(cuda, case, clients):
    """A segment whose sampled keys around the k-th rank are all one key K > 0 (sign-like deltas, clipped values,
    quantised tensors) is encoded in tie mode: its K-keys counted per unit, not recorded, the k-th key K with a tie
    quota in index order, the first +K / -K kept ties in mn / scale (round 4: every unit overflowed its record slots and
    the segment took the one-block raw-data path, ~100x slower). ResNet-50: a latency-bound plan (1 client) and a batch
    plan (2 clients); ratios 0.01 and 0.1: bit-exact, no raw-path fallback."""
    rng = np.random.default_rng(sum(map(ord, case)) + clients)
    sizes = fp32_sizes("resnet50_tv")
    xs = [tie_segments(rng, sizes, case) for _ in range(clients)]
    for ratio in ((0.01, 0.1) if clients == 1 else (0.01,)):
        plan, g, r = run_both(sizes, ratio, 8, xs, clients=clients)
        assert_same(plan, g, r)
        assert g["fallbacks"] == 0, (case, ratio)


@pytest.mark.parametrize("bits", [1, 32])
def test_tie_mode_bits_and_delta(cuda, bits):
    """Tie mode at 1-bit codes and raw fp32 values, in delta mode: base = multiples of 2^-10, x = base +- 2^-10
    (exact in fp32, so every x - base is +-2^-10): bit-exact."""
    rng = np.random.default_rng(40 + bits)
    sizes = [4096 * 300 + 17, 250000, 1 << 20]
    q = np.float32(2.0 ** -10)
    bases = [[(rng.integers(-1000, 1000, n) * q).astype(np.float32) for n in sizes]]
    xs = [[(b + np.where(rng.random(b.size) < 0.5, -q, q)).astype(np.float32) for b in bases[0]]]
    plan, g, r = run_both(sizes, 0.01, bits, xs, bases)
    assert_same(plan, g, r)


@pytest.mark.parametrize("clients", [1, 2])
def test_tie_mode_nan_inf_and_denormal_ties(cuda, clients):
    """Large segments whose tie key is a NaN, +-inf or a denormal (all-NaN, NaN beside values, equal-magnitude
    infinities, a sea of one denormal with both signs): tie mode's K is then a non-finite or subnormal key, the kept
    +-K values enter mn / scale NaN-ignoring, as the oracle does. Bit-exact against the oracle."""
    rng = np.random.default_rng(3 + clients)
    n = 4096 * 5 + 7
    nan = np.float32(np.nan)
    segs = [
        np.full(n, nan, np.float32),
        np.where(rng.random(n) < 0.3, nan, rng.standard_normal(n).astype(np.float32)).astype(np.float32),
        np.where(rng.random(n) < 0.5, np.float32(np.inf), np.float32(-np.inf)).astype(np.float32),
        np.where(rng.random(n) < 0.5, np.float32(1e-40), np.float32(-1e-40)).astype(np.float32),
        (rng.standard_normal(n) * 1e-3).astype(np.float32),
    ]
    sizes = [x.size for x in segs]
    xs = [[x.copy() for x in segs] for _ in range(clients)]
    if clients == 2:  # a batch plan (> 8192 units): pad the layout with a large ordinary segment
        big = 4096 * 8200
        sizes.append(big)
        for c in range(clients):
            xs[c].append((rng.standard_normal(big) * 1e-3).astype(np.float32))
    for ratio in (0.01, 0.3):
        plan, g, r = run_both(sizes, ratio, 8, xs, clients=clients)
        assert_same(plan, g, r)


@pytest.mark.parametrize("plan_kind", ["latency", "batch"])
@pytest.mark.parametrize("delta", [False, True])
def test_near_tie_refinement(cuda, plan_kind, delta):
    """Near-tied values at the k-th key (tests/sampler_model.py near_tie_layout: 16 near-tied levels, a continuous band
    of near-ties, equal |x|, plain Gaussian — the neighbourhood of a sign-like update's k-th key), ratios 0.01 / 0.1:
    the sampler's concentrated-bin refinement ends in each of its outcomes (a split bracket, tie mode, a lower edge K
    seen too rarely for tie mode, no refinement; tests/test_sampler_model.py asserts they all occur). The kernel's
    bracket of every large segment equals the model's (tests/sampler_model.py restates sample_segment), the codec
    is bit-exact against the oracle, and exactly the segments the model predicts take the raw-data path. Delta mode: base = N(0, 1e-6) (x - base keeps the
    near-tie structure); batch: two clients + a 33.6 M-element segment (> 8192 units)."""
    from tests.sampler_model import bracket, ccap_for, near_tie_layout, takes_raw_path
    rng = np.random.default_rng(77)
    clients = 2 if plan_kind == "batch" else 1
    xs = [near_tie_layout(rng) for _ in range(clients)]
    if plan_kind == "batch":
        for c in range(clients):
            xs[c].append((rng.standard_normal(4096 * 8200) * 1e-3).astype(np.float32))
    sizes = [x.size for x in xs[0]]
    bases = None
    if delta:
        bases = [[(rng.standard_normal(n) * 1e-6).astype(np.float32) for n in sizes] for _ in range(clients)]
        xs = [[(x + b).astype(np.float32) for x, b in zip(xc, bc)] for xc, bc in zip(xs, bases)]
    T = len(sizes)
    outcomes = set()
    for ratio in (0.01, 0.1):
        plan, g, r = run_both(sizes, ratio, 8, xs, bases, clients=clients, brackets=True)
        assert_same(plan, g, r)
        lim = small_limit(plan.table.segs[:, 1])
        lu, raw = 0, 0
        for c in range(clients):
            for t in range(T):
                n = sizes[t]
                if n <= lim:
                    continue
                d = xs[c][t] if bases is None else (xs[c][t] - bases[c][t]).astype(np.float32)
                k = int(plan.table.segs[c * T + t, 2])
                tlo, thi, o = bracket(d, k, c * T + t)
                outcomes.add(o)
                assert (int(g["tlo"][lu]), int(g["thi"][lu])) == (tlo, thi), (ratio, c, t, n, o)
                raw += takes_raw_path(d, k, tlo, thi, ccap_for([ratio]))
                lu += (n + 4095) // 4096
        # the segments the model sends to the raw-data path (a split bracket of the 16-level input at ratio 0.1
        # holds more candidates than a unit's record slots), and no other
        assert g["fallbacks"] == raw, (ratio, g["fallbacks"], raw)
    assert {"split", "tie", "edge"} <= outcomes, outcomes


def test_tie_mode_sample_miss_takes_raw_path(cuda):
    """Tie mode is the sampler's call: equal |x| everywhere it looks, but 2 % larger values where it does not look
    put the k-th key above K (the records then hold more than k keys). The segment falls back to the raw-data path:
    one fallback, bit-exact."""
    n = 1 << 20
    rng = np.random.default_rng(9)
    x = np.where(rng.random(n) < 0.5, np.float32(-1e-3), np.float32(1e-3)).astype(np.float32)
    unseen = np.flatnonzero(~sampled_positions(n, 0))
    big = rng.choice(unseen, size=int(0.02 * n), replace=False)
    x[big] = (rng.standard_normal(big.size) * 1e-2).astype(np.float32)
    plan, g, r = run_both([n], 0.01, 8, [[x]])
    assert g["fallbacks"] == 1
    assert_same(plan, g, r)


@pytest.mark.parametrize("with_empty", [False, True])
@pytest.mark.parametrize("with_idx", [False, True])
@pytest.mark.parametrize("delta", [False, True])
@pytest.mark.parametrize("bits", [1, 8, 32])
def test_dense_plan_implied_indices(cuda, bits, delta, with_idx, with_empty):
    """Ratio 1 (the download direction's dense codec): min / max, quantise and dequantise streams with the
    indices implied — no idx / starts unless asked for. Ragged sizes put segments' codes at odd byte offsets
    (the byte-store / byte-load paths), NaN / inf / constant / signed-zero segments, a segment of 3 units + 5:
    bit-exact against the oracle, in a latency-bound and (2 x 20 MB) a batch plan. Without a 0-element segment
    the quantise waves reduce their segment's min / max themselves (round 6); with one, k_dense_seg runs."""
    rng = np.random.default_rng(bits * 2 + delta)
    segs = edge_segments(rng) + [gauss(rng, [4096 * 2100 + 3])[0]]
    if with_empty:
        segs = segs[:3] + [np.zeros(0, np.float32)] + segs[3:] + [np.zeros(0, np.float32)]
    sizes = [s.size for s in segs]
    for clients in (1, 2):
        plan = CodecPlan(sizes, 1.0, bits, clients=clients)
        assert plan.dense and plan.implied_idx
        t = plan.table
        xs = [segs] * clients
        flat = to_flat(t, xs)
        base = to_flat(t, [gauss(rng, sizes, -2, -1)] * clients) if delta else None
        d_flat = torch.from_numpy(flat).cuda()
        d_base = None if base is None else torch.from_numpy(base).cuda()
        out = plan.empty_encoded(with_idx=with_idx)
        assert (out.idx.numel() == 0 and out.ustart is None) != with_idx
        enc = plan.encode(d_flat, base=d_base, out=out)
        dec = plan.decode(enc, base=d_base).cpu().numpy()
        torch.cuda.synchronize()
        s64 = t.segs.astype(np.int64)
        idx, vals, mn, sc = O.encode(flat, s64, bits, base=base)
        ref = O.decode(idx, vals, mn, sc, s64, bits, t.span, base=base)
        np.testing.assert_array_equal(enc.vals.cpu().numpy().view(np.uint8), vals.view(np.uint8))
        np.testing.assert_array_equal(enc.mn.cpu().numpy().view(np.uint32), mn.view(np.uint32))
        np.testing.assert_array_equal(enc.scale.cpu().numpy().view(np.uint32), sc.view(np.uint32))
        if with_idx:
            np.testing.assert_array_equal(enc.idx.cpu().numpy(), idx)
            np.testing.assert_array_equal(enc.ustart.cpu().numpy(), O.unit_starts(idx, s64))
        for (off, n, k, oo) in s64:
            np.testing.assert_array_equal(dec[off:off + n].view(np.uint32), ref[off:off + n].view(np.uint32))


# -- the tie quota across units (round 6: a folded saturating subtract lost its clamp) -------------------------------
def tie_quota_segment(rng, n, k, tie_units, extra_kept_ties=0):
    """n distinct keys, except the k-th largest key T repeated once in each of `tie_units` (in that order), so the
    quota keeps only the first 1 + extra_kept_ties of them by index: every later tie unit must reserve no slot."""
    keys = np.unique(rng.integers(0x30000000, 0x3F000000, int(n * 1.05), dtype=np.int64))
    assert keys.size >= n
    keys = rng.permutation(keys[:n]).astype(np.uint32)
    order = np.argsort(-keys.astype(np.int64), kind="stable")
    kth = k - 1 - extra_kept_ties  # the key at this rank becomes T; the ranks above it up to k - 1 become ties too
    T = keys[order[kth]]
    extra = [int(p) for p in order[kth - extra_kept_ties:kth]]
    keys[extra] = T
    first = True
    for u in tie_units:
        lo, hi = u * 4096, min(n, u * 4096 + 4096)
        cand = lo + np.flatnonzero(keys[lo:hi] < T)
        q = int(cand[rng.integers(0, cand.size)])
        if first:  # move the original T element into the first tie unit
            p0 = int(order[kth])
            keys[p0], keys[q] = keys[q], keys[p0]
            first = False
        else:
            keys[q] = T
    sign = np.where(rng.random(n) < 0.5, 0x80000000, 0).astype(np.uint32)
    return (keys | sign).view(np.float32)


@pytest.mark.parametrize("clients", [1, 16])  # latency plan (k_select 512 threads), batch plan (256 threads)
@pytest.mark.parametrize("tie_units,extra", [((37, 222), 0), ((255, 256), 0), ((63, 64, 575), 1), ((0, 300, 301), 0),
                                             ((127, 128, 129, 511), 2)])
def test_tie_quota_across_units(cuda, clients, tie_units, extra):
    """One 576-unit segment (ResNet-50's largest) whose k-th key repeats in several units, only the first few of them
    kept, followed by a small segment that a reserved-but-unwritten slot would spill into. Bit-exact idx / starts /
    decode; the output offsets were off by one from the first unit after a skipped tie in round 6's first select
    finish."""
    sizes = [2359296, 512]
    ratio = 0.1
    k = int(np.ceil(sizes[0] * ratio))
    rng = np.random.default_rng(600 + sum(tie_units) + extra)
    xs = []
    for c in range(clients):
        xs.append([tie_quota_segment(rng, sizes[0], k, tie_units, extra),
                   rng.standard_normal(sizes[1]).astype(np.float32)])
    plan, g, r = run_both(sizes, ratio, 8, xs, clients=clients)
    assert_same(plan, g, r)
    assert g["fallbacks"] == 0


@pytest.mark.parametrize("bits", [4, 8])
def test_dense_quantise_near_code_boundaries(cuda, bits):
    """The dense quantise divides by the reciprocal with an FMA correction (round 6); the code must equal the
    oracle's IEEE (x - mn) / scale + rint wherever the quotient sits a few ulps off a half-integer or an integer,
    for scales of every mantissa shape (all ones, a power of two, random) and far-apart exponents."""
    rng = np.random.default_rng(40 + bits)
    levels = (1 << bits) - 1
    segs = []
    for mant in (0x7FFFFF, 0x0, 0x7FFF00, 0x3A5A5A, int(rng.integers(0, 1 << 23))):
        for e in (-100, -80, -20, -3, 0, 7, 60, 95):  # (-100, 95: outside [2^-90, 2^90], the division)
            sc = np.array([((127 + e) << 23) | mant], np.uint32).view(np.float32)[0]
            mn = np.float32(rng.standard_normal()) * np.float32(2.0 ** e)
            mx = np.float32(mn + np.float32(levels) * sc)
            sc = np.float32((mx - mn) / np.float32(levels))  # the scale the codec derives (CodecSpec v1)
            ks = rng.integers(0, levels, 6000).astype(np.float32)
            half = (ks + np.float32(0.5)) * sc
            whole = ks * sc
            base = np.where(rng.random(6000) < 0.5, half, whole).astype(np.float32)
            x = (mn + base).astype(np.float32)
            x = (x.view(np.int32) + rng.integers(-3, 4, 6000).astype(np.int32)).view(np.float32)
            x = np.clip(x, mn, mx).astype(np.float32)
            segs.append(np.concatenate([[mn, mx], x]).astype(np.float32))
    sizes = [s.size for s in segs]
    plan = CodecPlan(sizes, 1.0, bits)
    assert plan.dense
    t = plan.table
    flat = to_flat(t, [segs])
    enc = plan.encode(torch.from_numpy(flat).cuda())
    torch.cuda.synchronize()
    s64 = t.segs.astype(np.int64)
    idx, vals, mn, sc = O.encode(flat, s64, bits)
    np.testing.assert_array_equal(enc.mn.cpu().numpy().view(np.uint32), mn.view(np.uint32))
    np.testing.assert_array_equal(enc.scale.cpu().numpy().view(np.uint32), sc.view(np.uint32))
    np.testing.assert_array_equal(enc.vals.cpu().numpy().view(np.uint8), vals.view(np.uint8))
