"""module_with_state (the server decompression's module rebuild) keeps copy.deepcopy's semantics where a
template holds more than plain values: hooks bound to the template are rebound to the clone,
tensors inside container attributes are copied, unregistered submodules are deep-copied, and plain
attributes follow the template's CURRENT values (the recipe is cached per template). Also: the cached
state walk (module_tensors) returns exactly state_dict()'s names and storage, and follows changes."""
import copy

import pytest

import torch
from torch import nn

from coala_amd.compression.codec import module_tensors, module_with_state


class Block(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv = nn.Conv2d(2, 3, 3)
        self.bn = nn.BatchNorm2d(3)
        self.calls = []
        self.register_forward_hook(self._record)
        self.extra = [torch.ones(3), 5]
        self.table = {"w": torch.zeros(2)}
        self.__dict__["aux"] = nn.Linear(2, 2)  # an unregistered module attribute

    def _record(self, mod, inp, out):
        self.calls.append(out.shape)

    def forward(self, x):
        return self.bn(self.conv(x))


class Net(nn.Module):
    def __init__(self):
        super().__init__()
        self.b1 = Block()
        self.shared = nn.Linear(4, 4)
        self.b2 = nn.Sequential(self.shared, nn.ReLU(), self.shared)  # shared submodule
        self.register_buffer("scratch", torch.zeros(2), persistent=False)


def _new_state(m):
    return {k: torch.randn_like(v) if v.is_floating_point() else v.clone() for k, v in m.state_dict().items()}


def test_clone_has_the_state_and_no_aliasing():
    m = Net()
    st = _new_state(m)
    c = module_with_state(m, st)
    cs = c.state_dict()
    assert list(cs) == list(m.state_dict())
    for k, v in st.items():  # (a shared submodule is cloned once, from its first name: "shared.")
        if not k.startswith("b2."):
            assert cs[k].data_ptr() == v.data_ptr()
    assert all(isinstance(p, nn.Parameter) for p in c.parameters())
    assert c.b2[0] is c.b2[2] is c.shared and c.shared is not m.shared  # sharing kept, template not aliased
    assert c.scratch is not m.scratch and torch.equal(c.scratch, m.scratch)  # non-persistent: cloned


def test_hooks_rebound_and_containers_copied_like_deepcopy():
    m = Net()
    c = module_with_state(m, _new_state(m))
    ref = copy.deepcopy(m)
    x = torch.randn(1, 2, 5, 5)
    c.b1(x)
    assert len(c.b1.calls) == 1 and m.b1.calls == []  # the clone's hook records on the clone
    ref.b1(x)
    assert len(ref.b1.calls) == 1
    assert c.b1.extra is not m.b1.extra and c.b1.extra[0] is not m.b1.extra[0] and c.b1.extra[1] == 5
    assert torch.equal(c.b1.extra[0], m.b1.extra[0])
    assert c.b1.table["w"] is not m.b1.table["w"]
    assert c.b1.aux is not m.b1.aux and torch.equal(c.b1.aux.weight, m.b1.aux.weight)
    # a hook registered on the template after the first clone is carried by the next clone
    seen = []
    m.b2.register_forward_hook(lambda mod, i, o: seen.append(1))
    c2 = module_with_state(m, _new_state(m))
    c2.b2(torch.randn(1, 4))
    assert seen == [1]


def test_plain_attributes_follow_the_template():
    m = Net()
    module_with_state(m, _new_state(m))
    m.eval()
    c = module_with_state(m, _new_state(m))
    assert not c.training and not c.b1.bn.training
    m.train()
    assert module_with_state(m, _new_state(m)).b1.bn.training


def test_module_tensors_matches_state_dict_and_follows_changes():
    m = Net()
    names, ts = module_tensors(m)
    st = m.state_dict()
    assert names == tuple(st) and [t.data_ptr() for t in ts] == [v.data_ptr() for v in st.values()]
    m.b1.register_buffer("extra_buf", torch.ones(1))
    names2, ts2 = module_tensors(m)
    assert names2 == tuple(m.state_dict()) and "b1.extra_buf" in names2
    m.b1.conv.weight = nn.Parameter(torch.zeros(3, 2, 3, 3))  # replaced parameter: same table size
    _, ts3 = module_tensors(m)
    assert any(t is m.b1.conv.weight for t in ts3)
    # a replaced submodule (same table sizes everywhere): the walk must return the NEW module's tensors
    m.shared = nn.Linear(4, 4)
    names4, ts4 = module_tensors(m)
    st4 = m.state_dict()
    assert names4 == tuple(st4) and [t.data_ptr() for t in ts4] == [v.data_ptr() for v in st4.values()]
    # a replaced grandchild, and a buffer turned non-persistent
    m.b1.bn = nn.BatchNorm2d(3)
    names5, ts5 = module_tensors(m)
    assert [t.data_ptr() for t in ts5] == [v.data_ptr() for v in m.state_dict().values()]
    m.b1._non_persistent_buffers_set.add("extra_buf")
    names6, _ = module_tensors(m)
    assert names6 == tuple(m.state_dict()) and "b1.extra_buf" not in names6


# -- recycled decoded modules (UpdateCodec.decode_module) ------------------------------------------------------
def _codec_round(seed_global=0):
    from coala_amd.compression import UpdateCodec
    from coala_amd.layouts import build_module
    from tests.oracle_backend import OracleBackend
    codec = UpdateCodec(0.05, 8, "delta", OracleBackend())
    g = build_module("resnet18_split_cut2", seed=seed_global)
    base = codec.snapshot(g)
    ups = [codec.encode(build_module("resnet18_split_cut2", seed=10 + i).state_dict(), base=base) for i in range(3)]
    fresh = [{k: v.clone() for k, v in codec.decode_state(u, base=base).items()} for u in ups]
    return codec, g, base, ups, fresh


def _equal_state(m, st):
    ms = m.state_dict()
    return list(ms) == list(st) and all(torch.equal(ms[k], st[k]) for k in st)


def test_decoded_modules_are_recycled_once_released():
    """A decoded module nothing else references is reused by the next decode of the layout: same object, the
    NEW update's values, parameters still Parameters; while it is referenced (the module, a submodule, a
    parameter, or a state_dict view of its storage) a new tree is built instead."""
    codec, g, base, ups, fresh = _codec_round()
    m = codec.decode_module(ups[0], g, base=base)
    assert _equal_state(m, fresh[0])
    first = id(m)
    del m
    m = codec.decode_module(ups[1], g, base=base)
    assert id(m) == first and _equal_state(m, fresh[1])
    assert all(isinstance(p, nn.Parameter) for p in m.parameters())
    # held: every way of holding on to a piece of it keeps it from being recycled (a fresh template each time:
    # its pool then holds this one tree only)
    for hold in (lambda x: x, lambda x: next(iter(x.children())), lambda x: next(x.parameters()),
                 lambda x: x.state_dict(), lambda x: list(x.parameters())[-1].detach()[:1]):
        codec, g, base, ups, fresh = _codec_round(seed_global=1)
        m = codec.decode_module(ups[0], g, base=base)
        mid = id(m)
        kept = hold(m)
        del m
        other = codec.decode_module(ups[1], g, base=base)
        assert id(other) != mid and _equal_state(other, fresh[1])
        del other
        kept = None  # released: now the first tree is idle again (and so is the second)
        ids = {id(codec.decode_module(ups[2], g, base=base)) for _ in range(2)}
        assert mid in ids


def test_recycled_module_follows_the_template_and_drops_foreign_hooks():
    codec, g, base, ups, fresh = _codec_round()
    m = codec.decode_module(ups[0], g, base=base)
    seen = []
    m.register_forward_hook(lambda *a: seen.append(1))  # the previous holder's hook
    m.train()
    first = id(m)
    del m
    g.eval()
    m = codec.decode_module(ups[1], g, base=base)
    assert id(m) == first
    assert not m.training and all(not c.training for c in m.modules())
    assert not m._forward_hooks  # a fresh build would not carry the previous holder's hook
    g.train()


def test_recycling_survives_a_template_change():
    """A template whose structure changed (a new buffer) retires the pooled trees: the next decode builds a
    module with the new structure."""
    codec, g, base, ups, fresh = _codec_round()
    m = codec.decode_module(ups[0], g, base=base)
    del m
    g.register_buffer("extra_note", torch.ones(2), persistent=False)
    m = codec.decode_module(ups[1], g, base=base)
    assert torch.equal(m.extra_note, torch.ones(2)) and m.extra_note is not g.extra_note
    assert _equal_state(m, fresh[1])


def test_layout_reused_only_while_tensors_and_storage_are_unchanged():
    """describe_tensors keeps the layout of the last call while the same tensor objects sit at the same storage;
    a parameter whose .data is swapped for another shape (new storage) or a replaced parameter object is seen."""
    from coala_amd.compression.codec import _module_walk, describe_tensors
    m = Net()
    names, ts, w = _module_walk(m)
    L1 = describe_tensors(names, ts, w)[0]
    names, ts, w = _module_walk(m)
    assert describe_tensors(names, ts, w)[0] is L1
    with torch.no_grad():
        m.shared.weight.data = torch.randn(2, 8)  # same element count, new storage and shape
    names, ts, w = _module_walk(m)
    L2 = describe_tensors(names, ts, w)[0]
    shapes = {e["name"]: tuple(e["shape"]) for e in L2.entries}
    assert L2 is not L1 and shapes["shared.weight"] == (2, 8)
    m.b1.conv.bias = nn.Parameter(torch.zeros(3))  # a replaced parameter object
    names, ts, w = _module_walk(m)
    L3, segs, _ = describe_tensors(names, ts, w)
    assert any(t is m.b1.conv.bias for t in segs)
    assert [e["name"] for e in L3.entries] == list(m.state_dict())


def test_recycling_checks_attributes_tables_and_template_children():
    """A tree a previous holder gave a new attribute is not recycled; hooks registered on a recycled tree are
    dropped; a template whose submodule was replaced gets a new recipe (the decoded module follows the new
    child's attributes)."""
    codec, g, base, ups, fresh = _codec_round()
    m = codec.decode_module(ups[0], g, base=base)
    first = id(m)
    list(m.modules())[1].note = "held"  # an attribute a fresh build would not have
    del m
    m = codec.decode_module(ups[1], g, base=base)
    assert id(m) != first and not hasattr(list(m.modules())[1], "note") and _equal_state(m, fresh[1])
    second = id(m)
    list(m.modules())[2].register_forward_hook(lambda *a: None)
    del m
    m = codec.decode_module(ups[2], g, base=base)
    assert id(m) == second and not list(m.modules())[2]._forward_hooks and _equal_state(m, fresh[2])
    del m
    name, child = next(iter(g.named_children()))
    new_child = copy.deepcopy(child)
    new_child.tag = 7
    setattr(g, name, new_child)
    m = codec.decode_module(ups[1], g, base=base)
    got = getattr(m, name)
    assert got is not new_child and got is not child and got.tag == 7 and _equal_state(m, fresh[1])


def test_recycler_hands_one_idle_module_to_one_thread_only(monkeypatch):
    """Two upload threads (the remote server runs decompression in one thread per upload,
    coala/server/service.py:74) that both find the same idle pooled tree must not both decode into it: a
    barrier injected right after idle_skeleton returns forces both threads through the window between the
    idle check and the caller taking the tree."""
    import threading
    from coala_amd.compression.codec import _TreeRecipe
    codec, g, base, ups, fresh = _codec_round(seed_global=3)
    m = codec.decode_module(ups[0], g, base=base)
    del m  # one idle tree in the pool
    orig = _TreeRecipe.idle_skeleton
    barrier = threading.Barrier(2, timeout=30)

    def forced(self, *a, **kw):
        res = orig(self, *a, **kw)
        barrier.wait()  # both threads have checked idleness before either decodes
        return res
    monkeypatch.setattr(_TreeRecipe, "idle_skeleton", forced)
    out, errs = [None, None], []

    def run(i):
        try:
            out[i] = codec.decode_module(ups[1 + i], g, base=base)
        except Exception as e:  # pragma: no cover - reported below
            errs.append(e)
    ts = [threading.Thread(target=run, args=(i,)) for i in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs
    assert out[0] is not out[1]
    assert _equal_state(out[0], fresh[1]) and _equal_state(out[1], fresh[2])


def test_recycled_storage_bumps_the_version_counter():
    """A live autograd graph that saved a decoded parameter keeps its tree out of reuse (the saved tensor holds
    the parameter object); a recycled tree's storage, written through raw pointers, has its version counter
    bumped, so anything that still saved it raises in backward instead of using the new values."""
    codec, g, base, ups, fresh = _codec_round(seed_global=4)
    m = codec.decode_module(ups[0], g, base=base)
    p = next(m.parameters())
    loss = (p * p).sum()  # saves p for backward
    first = id(m)
    del m, p
    m = codec.decode_module(ups[1], g, base=base)
    assert id(m) != first and _equal_state(m, fresh[1])
    loss.backward()  # the saved values were never overwritten
    del loss, m
    m = codec.decode_module(ups[2], g, base=base)  # one of the two idle trees
    ids = set()
    for i in range(3):  # the same tree again and again: its version moves every time
        vs = next(m.parameters())._version
        mid = id(m)
        del m
        m = codec.decode_module(ups[i], g, base=base)
        if id(m) == mid:
            ids.add(mid)
            assert next(m.parameters())._version > vs
    assert ids


def test_recycling_with_more_clients_per_round_than_half_the_pool():
    """A server with more uploads per round than POOL_MAX / 2: each round's decoded module of client
    j replaces client j's module of the previous round (coala/server/base.py:377-381), so the trees of round r stay held
    while round r + 1 decodes. From the third round on every decode reuses a pooled tree (none is evicted while held,
    none built anew beyond the pool's capacity), and every module holds its own update."""
    from coala_amd.compression.codec import _TreeRecipe, _recipe
    codec, g, base, ups, fresh = _codec_round(seed_global=7)
    C = _TreeRecipe.POOL_MAX // 2 + 8
    held, seen, built = {}, set(), []
    for rnd in range(4):
        new_ids = 0
        for j in range(C):
            m = codec.decode_module(ups[j % 3], g, base=base)
            new_ids += id(m) not in seen
            seen.add(id(m))
            held[j] = m  # replaces client j's module of the previous round
            del m
        built.append(new_ids)
    assert built[0] == C and built[2] == 0 and built[3] == 0, built
    assert len(_recipe(g).pool) <= C + 1
    assert all(_equal_state(held[j], fresh[j % 3]) for j in range(C))


def test_pool_release_eviction_and_opt_out():
    """release_pool() empties the pool; trees not handed out for a while are evicted; recycle=False never
    pools or reuses a module."""
    from coala_amd.compression import UpdateCodec
    from coala_amd.compression.codec import _TreeRecipe, _recipe
    from tests.oracle_backend import OracleBackend
    codec, g, base, ups, fresh = _codec_round(seed_global=5)
    ms = [codec.decode_module(u, g, base=base) for u in ups]
    rec = _recipe(g)
    assert len(rec.pool) == 3
    codec.release_pool()
    assert not rec.pool
    # eviction: with the pool of 3, trees 1 and 2 stay HELD while tree 0 is reused again and again: kept past the
    # horizon (a held tree becomes reusable when its holder lets go); released, they are idle and stale: dropped
    ms = [codec.decode_module(u, g, base=base) for u in ups]
    keep = ms[1:]
    del ms
    horizon = 2 * 3 + _TreeRecipe.EVICT_SLACK
    for i in range(horizon + 3):
        m = codec.decode_module(ups[i % 3], g, base=base)
        del m
    assert len(rec.pool) == 3  # held trees are not evicted
    assert all(_equal_state(k, fresh[1 + j]) for j, k in enumerate(keep))  # (nor overwritten)
    keep = None
    for i in range(2):
        m = codec.decode_module(ups[i % 3], g, base=base)
        del m
    assert len(rec.pool) == 1  # idle and not handed out for longer than the horizon: dropped
    # opt-out
    off = UpdateCodec(0.05, 8, "delta", OracleBackend(), recycle=False)
    codec.release_pool()
    a = off.decode_module(ups[0], g, base=base)
    b = off.decode_module(ups[1], g, base=base)
    assert not rec.pool and a is not b
    assert _equal_state(a, fresh[0]) and _equal_state(b, fresh[1])
