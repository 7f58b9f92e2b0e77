"""CPU oracle: pinned against an independent brute-force restatement and the committed golden vectors."""
import math
import os

import numpy as np
import pytest

from oracle import codec_oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden", "codec_vectors.npz")


@pytest.mark.parametrize("n,ratio", [(1, 0.01), (7, 0.5), (100, 0.07), (1000, 0.001), (4097, 0.01), (10, 1.0)])
def test_k_for(n, ratio):
    k = O.k_for(n, ratio)
    assert k == max(1, min(n, math.ceil(n * ratio)))
    assert 1 <= k <= n


def test_k_for_zero_and_float64():
    assert O.k_for(0, 0.5) == 0
    assert O.k_for(100, 0.07) == 8  # 100 * 0.07 = 7.000000000000001 in float64 -> ceil = 8 (spec: float64)


@pytest.mark.parametrize("seed", range(6))
def test_topk_matches_bruteforce(seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 5000))
    x = (rng.standard_normal(n) * 10 ** rng.uniform(-6, 2)).astype(np.float32)
    x[rng.integers(0, n, n // 5)] = x[rng.integers(0, n)]          # ties
    x[rng.integers(0, n, n // 10)] *= -1                           # sign flips of equal magnitudes
    x[rng.integers(0, n, n // 20)] = 0.0
    for k in {1, max(1, n // 100), n // 2 or 1, n}:
        np.testing.assert_array_equal(O.topk_indices(x, k), O.topk_indices_bruteforce(x, k))


def test_tie_break_lower_index_and_signed_zero():
    x = np.array([1.0, -2.0, 2.0, -2.0, 0.0, -0.0], np.float32)
    assert O.topk_indices(x, 2).tolist() == [1, 2]
    assert O.topk_indices(x, 3).tolist() == [1, 2, 3]
    z = np.array([-0.0, 0.0, -0.0], np.float32)
    assert O.topk_indices(z, 2).tolist() == [0, 1]


def test_nan_sorts_above_inf():
    x = np.array([np.inf, 1.0, np.nan, -np.inf], np.float32)
    assert O.topk_indices(x, 1).tolist() == [2]
    assert O.topk_indices(x, 3).tolist() == [0, 2, 3]


def test_quantize_rules():
    q, mn, sc = O.quantize(np.array([0.0, 1.0, 0.5, 1.5], np.float32), 1)
    assert (mn, sc) == (0.0, 1.5)
    assert q.tolist() == [0, 1, 0, 1]          # 0.5/1.5 -> rint(0.333)=0; 1.0/1.5 -> rint(0.667) = 1
    q, mn, sc = O.quantize(np.full(5, 3.0, np.float32), 8)
    assert sc == 0.0 and q.tolist() == [0] * 5
    q, mn, sc = O.quantize(np.array([-0.0, -0.0], np.float32), 8)
    assert np.signbit(mn) == False  # canonical +0  # noqa: E712
    q, mn, sc = O.quantize(np.array([np.nan, 1.0, 3.0], np.float32), 8)
    assert mn == 1.0 and q[0] == 0
    # half-to-even at exact .5 steps
    v = np.array([0.0, 2.5, 3.5, 255.0], np.float32)
    q, mn, sc = O.quantize(v, 8)
    assert sc == 1.0 and q.tolist() == [0, 2, 4, 255]


def test_roundtrip_error_bound():
    rng = np.random.default_rng(1)
    x = (rng.standard_normal(20000) * 1e-3).astype(np.float32)
    for bits in (4, 8):
        k = O.k_for(x.size, 0.05)
        idx, q, mn, sc = O.encode_segment(x, k, bits)
        d = O.decode_segment(idx, q, mn, sc, x.size, bits)
        assert np.all(d[np.setdiff1d(np.arange(x.size), idx)] == 0)
        bound = sc / 2 + 2 * np.finfo(np.float32).eps * np.abs(x[idx]).max()
        assert np.abs(d[idx] - x[idx]).max() <= bound


def test_raw_bits_lossless_at_ratio_one():
    rng = np.random.default_rng(2)
    x = rng.standard_normal(777).astype(np.float32)
    idx, v, mn, sc = O.encode_segment(x, x.size, 32)
    np.testing.assert_array_equal(O.decode_segment(idx, v, mn, sc, x.size, 32), x)


def test_batch_encode_decode_segments_and_delta():
    rng = np.random.default_rng(3)
    sizes = [5, 300, 64]
    offs, oo, segs = [0, 32, 352], 0, []
    for n, off in zip(sizes, offs):
        k = O.k_for(n, 0.1)
        segs.append((off, n, k, oo))
        oo += k
    flat = rng.standard_normal(416).astype(np.float32)
    base = rng.standard_normal(416).astype(np.float32)
    idx, vals, mn, sc = O.encode(flat, segs, 8, base=base)
    out = O.decode(idx, vals, mn, sc, segs, 8, 416, base=base)
    for (off, n, k, o) in segs:
        d = (flat[off:off + n] - base[off:off + n]).astype(np.float32)
        i2, v2, m2, s2 = O.encode_segment(d, k, 8)
        np.testing.assert_array_equal(idx[o:o + k], i2)
        ref = base[off:off + n] + O.decode_segment(i2, v2, m2, s2, n, 8)
        np.testing.assert_array_equal(out[off:off + n].view(np.uint32), ref.view(np.uint32))


def test_golden_vectors_reproduce():
    """The oracle reproduces every committed golden vector bit for bit."""
    g = np.load(GOLD)
    names = sorted({k.split("/")[0] for k in g.files})
    checked = 0
    for name in names:
        x = g[f"{name}/x"]
        for ratio in (0.001, 0.01, 0.3, 1.0):
            for bits in (1, 4, 8, 32):
                tag = f"{name}/r{ratio}/b{bits}"
                k = int(g[f"{tag}/k"][0])
                assert k == O.k_for(x.size, ratio)
                idx, vals, mn, sc = O.encode_segment(x, k, bits)
                np.testing.assert_array_equal(idx, g[f"{tag}/idx"])
                np.testing.assert_array_equal(vals.view(np.uint8), g[f"{tag}/vals"].view(np.uint8))
                np.testing.assert_array_equal(np.array([mn, sc], np.float32).view(np.uint32),
                                              g[f"{tag}/mn_scale"].view(np.uint32))
                dec = O.decode_segment(idx, vals, mn, sc, x.size, bits)
                np.testing.assert_array_equal(dec.view(np.uint32), g[f"{tag}/dec"].view(np.uint32))
                checked += 1
    assert checked == len(names) * 16
