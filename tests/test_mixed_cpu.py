"""C5 host logic on CPU: mixed-layout segment tables, the seeded splitFL round and its greedy split over
GPUs, and oracle round trips over a mixed table (the layouts come from
application/splitFL/models/*_split.py and the feature shapes from application/splitFL/client/
base_sfl.py:249-257)."""
import numpy as np
import pytest

from coala_amd.compression.pipeline import balanced_cuts
from coala_amd.compression.spec import ALIGN, MixedTable, SegmentTable, k_for
from coala_amd.layouts import FEATURES, fp32_sizes
from coala_amd.workload import C5_CHOICES, C5_CLIENTS, C5_GPUS, c5_draw, c5_groups, c5_share, mixed_table
from oracle import codec_oracle as O


def test_mixed_table_equals_segment_table_for_one_layout():
    sizes = fp32_sizes("resnet18_split_cut4")
    a = SegmentTable(sizes, 0.01, 3)
    b = MixedTable([sizes] * 3, 0.01)
    assert np.array_equal(a.segs, b.segs)
    assert (a.span, a.total_k, a.n_segments, a.n_elements) == (b.span, b.total_k, b.n_segments, b.n_elements)
    assert a.client_span_off == b.client_span_off and a.client_k_off == b.client_k_off
    assert a.client_seg_off == b.client_seg_off


def test_mixed_table_layout_rules():
    layouts = [[5, 4097, 3], [8388608], [], [1, 1]]
    t = MixedTable(layouts, 0.01)
    segs = t.segs.astype(np.int64)
    assert np.all(segs[:, 0] % ALIGN == 0)
    assert [int(x) for x in segs[:, 2]] == [k_for(n, 0.01) for n in (5, 4097, 3, 8388608, 1, 1)]
    # client-major: every client's segments inside [span_off[c], span_off[c+1]), kept entries contiguous
    for c in range(4):
        rows = segs[t.client_seg_off[c]:t.client_seg_off[c + 1]]
        assert np.all(rows[:, 0] >= t.client_span_off[c])
        assert np.all(rows[:, 0] + rows[:, 1] <= t.client_span_off[c + 1])
        assert int(rows[:, 2].sum()) == t.client_k_off[c + 1] - t.client_k_off[c]
    assert t.client_span_off[3] - t.client_span_off[2] == ALIGN  # an empty client still owns a slot
    sub = t.sub_table(1, 3)
    assert sub.clients == 2 and sub.span == t.client_span_off[3] - t.client_span_off[1]


def test_balanced_cuts():
    assert balanced_cuts([1] * 16, 2) == [0, 8, 16]
    assert balanced_cuts([1] * 5, 8) == [0, 1, 2, 3, 4, 5]
    cuts = balanced_cuts([100, 1, 1, 1, 100, 1], 2)
    assert cuts[0] == 0 and cuts[-1] == 6 and 0 < cuts[1] < 6
    for costs in ([3, 9, 1, 7, 2], [10] * 7, [1, 2, 3, 4, 5, 6, 7, 8]):
        for p in (1, 2, 3):
            c = balanced_cuts(costs, p)
            assert c[0] == 0 and c[-1] == len(costs) and all(b > a for a, b in zip(c, c[1:]))


def test_c5_round_is_seeded_and_partitioned():
    names = c5_draw()
    assert len(names) == C5_CLIENTS and set(names) <= set(C5_CHOICES)
    assert names == c5_draw()  # seeded
    groups = c5_groups(names)
    assert sorted(i for g in groups for i in g) == list(range(C5_CLIENTS))
    loads = [sum(sum(fp32_sizes(names[i])) for i in g) for g in groups]
    biggest = max(sum(fp32_sizes(n)) for n in C5_CHOICES)
    assert max(loads) - min(loads) <= biggest
    ids, nm = c5_share(0)
    assert ids == sorted(groups[0]) and "sfl_feature_256x32x32" in nm
    assert c5_share(C5_GPUS) == c5_share(0)  # weak scaling past 8 ranks repeats the shares


def test_feature_layouts():
    for name, shape in FEATURES.items():
        assert fp32_sizes(name) == [int(np.prod(shape))]
    assert fp32_sizes("sfl_feature_256x32x32") == [8388608]


@pytest.mark.parametrize("bits", [8, 32])
def test_oracle_round_trip_on_mixed_table(bits):
    names = ["simple_cnn_split_cut1", "resnet18_split_cut2", "sfl_feature_128x16x16", "resnet50_split_cut1"]
    t = mixed_table(names, 0.01)
    rng = np.random.default_rng(0)
    flat = np.zeros(t.span, np.float32)
    segs = t.segs.astype(np.int64)
    for off, n, k, oo in segs:
        flat[off:off + n] = rng.standard_normal(n) * 10 ** rng.uniform(-4, -2)
    idx, vals, mn, sc = O.encode(flat, segs, bits)
    dec = O.decode(idx, vals, mn, sc, segs, bits, t.span)
    for s, (off, n, k, oo) in enumerate(segs):
        sel = idx[oo:oo + k]
        assert np.all(np.diff(sel) > 0)
        d = dec[off:off + n]
        assert np.count_nonzero(d) <= k
        if bits == 32:
            np.testing.assert_array_equal(d[sel], flat[off:off + n][sel])
