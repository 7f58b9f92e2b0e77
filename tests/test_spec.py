"""Host-side CodecSpec v1 logic and the reference-model layouts (no GPU)."""
import numpy as np
import pytest

from coala_amd.compression import spec
from coala_amd.compression.spec import ALIGN, SegmentTable, k_for
from coala_amd.layouts import SPLITFL, build_module, fp32_sizes, load, names
from oracle import codec_oracle as O


def test_k_for_matches_oracle():
    rng = np.random.default_rng(0)
    for _ in range(500):
        n = int(rng.integers(0, 10 ** 7))
        r = float(rng.choice([0.001, 0.01, 0.1, 0.07, 0.3333, 1.0]))
        assert k_for(n, r) == O.k_for(n, r)
    with pytest.raises(ValueError):
        k_for(10, 0.0)


def test_segment_table_layout():
    t = SegmentTable([5, 100, 33, 1], 0.1, clients=3)
    assert t.n_segments == 12 and t.clients == 3
    segs = t.segs.astype(np.int64)
    assert np.all(segs[:, 0] % ALIGN == 0)                 # aligned starts (float4 needs 4)
    ends = segs[:, 0] + segs[:, 1]
    assert np.all(ends[:-1] <= segs[1:, 0])               # no overlap, increasing
    assert np.all(segs[1:, 3] == segs[:-1, 3] + segs[:-1, 2])  # contiguous outputs
    assert t.total_k == int(segs[-1, 3] + segs[-1, 2])
    assert t.span == 3 * t.span_per_client
    assert t.algorithmic_bytes(8) == 8 * t.n_elements + 10 * t.total_k + 32 * t.n_segments


# element counts SURVEY.md §8(a)/(d) quotes for the reference models
EXPECTED = {"lenet": (8, 6603710), "resnet18": (102, 11183562), "resnet50_tv": (267, 25610152),
            "vit_b16": (200, 86567656)}


@pytest.mark.parametrize("name", sorted(EXPECTED))
def test_layouts_match_survey(name):
    sizes = fp32_sizes(name)
    assert (len(sizes), sum(sizes)) == EXPECTED[name]
    assert load(name)["n_float32_elements"] == sum(sizes)


def test_splitfl_layouts():
    want = {"resnet18_split_cut1": 1856, "resnet18_split_cut2": 75840, "resnet18_split_cut4": 379968,
            "resnet50_split_cut1": 1856, "resnet50_split_cut2": 76864, "resnet50_split_cut4": 217664,
            "simple_cnn_split_cut1": 896, "simple_cnn_split_cut2": 19392, "simple_cnn_split_cut4": 121920}
    assert set(SPLITFL) <= set(names())
    for k, v in want.items():
        assert sum(fp32_sizes(k)) == v


def test_build_module_layout_order():
    m = build_module("resnet18")
    ref = [(e["name"], tuple(e["shape"]), e["dtype"]) for e in load("resnet18")["entries"]]
    got = [(k, tuple(v.shape), str(v.dtype).replace("torch.", "")) for k, v in m.state_dict().items()]
    assert got == ref


def test_constants_mirror_kernel():
    src = open(__import__("coala_amd._build", fromlist=["SRC"]).SRC).read()
    assert f"constexpr uint32_t SMALL_MAX = {spec.SMALL_MAX};" in src
    assert f"constexpr uint32_t SMALL_MAX_LATENCY = {spec.SMALL_MAX_LATENCY};" in src
    assert f"constexpr uint32_t SMALL_MAX_BATCH = {spec.SMALL_MAX_BATCH};" in src
    assert f"constexpr uint32_t LATENCY_PLAN_UNITS = {spec.LATENCY_PLAN_UNITS};" in src
    assert f"constexpr uint32_t UNIT = {spec.UNIT};" in src


@pytest.mark.parametrize("lanes", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("name,clients", [("resnet50_tv", 16), ("resnet50_tv", 1), ("vit_b16", 2), ("lenet", 1)])
def test_split_lanes_contiguous_balanced(name, clients, lanes):
    """Lane ranges tile [0, T) in order, never empty, and (with many segments) each lane holds about
    1/L of the elements."""
    from coala_amd.compression import split_lanes
    t = SegmentTable(fp32_sizes(name), 0.01, clients)
    sizes = t.segs[:, 1].astype(np.int64)
    r = split_lanes(sizes.tolist(), lanes)
    assert r[0][0] == 0 and r[-1][1] == len(sizes)
    assert all(a < b for a, b in r) and all(r[i][1] == r[i + 1][0] for i in range(len(r) - 1))
    assert len(r) <= lanes
    if len(sizes) >= 16 * lanes and max(sizes) * lanes * 4 <= sizes.sum():
        assert len(r) == lanes
        share = np.array([sizes[a:b].sum() for a, b in r]) / sizes.sum()
        assert share.max() <= 1.0 / lanes + max(sizes) / sizes.sum() + 1e-9


def test_subtable_extents():
    from coala_amd.compression import SubTable
    t = SegmentTable([10, 5000, 70], 0.1, 2)
    sub = SubTable(t.segs[2:5])
    assert sub.n_segments == 3
    assert sub.total_k == int(t.segs[4, 3] + t.segs[4, 2])
    assert sub.span == int(t.segs[4, 0] + t.segs[4, 1])
    assert sub.n_elements == int(t.segs[2:5, 1].sum())


def test_small_limit_follows_plan_size(monkeypatch):
    """spec.small_limit mirrors coalac_plan_create: latency-bound plans (<= LATENCY_PLAN_UNITS units)
    encode segments of up to SMALL_MAX_LATENCY elements whole, bigger plans up to SMALL_MAX_BATCH; the
    COALAC_SMALL_MAX override is clamped to [1024, SMALL_MAX]."""
    monkeypatch.delenv("COALAC_SMALL_MAX", raising=False)
    one = fp32_sizes("resnet50_tv")
    assert spec.small_limit(one) == spec.SMALL_MAX_LATENCY
    assert spec.small_limit(one * 2) == spec.SMALL_MAX_BATCH
    units = spec.LATENCY_PLAN_UNITS
    assert spec.small_limit([spec.UNIT] * units) == spec.SMALL_MAX_LATENCY
    assert spec.small_limit([spec.UNIT] * (units + 1)) == spec.SMALL_MAX_BATCH
    monkeypatch.setenv("COALAC_SMALL_MAX", "4096")
    assert spec.small_limit(one) == 4096
    monkeypatch.setenv("COALAC_SMALL_MAX", "10")
    assert spec.small_limit(one) == 1024
