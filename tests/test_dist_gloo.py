"""Multi-process path on CPU (world_size 2, gloo): each rank encodes+decodes only its own clients —
the codec needs no collective — and the union over ranks equals the serial result.
Heterogeneous C5-style clients (splitFL layouts) are balanced with the reference's greedy grouping."""
import hashlib
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from coala_amd.sharding import contiguous_groups, greedy_groups, split_sizes

LAYOUTS = ["resnet18_split_cut2", "simple_cnn_split_cut4", "resnet50_split_cut2", "simple_cnn_split_cut1",
           "resnet18_split_cut1", "simple_cnn_split_cut2", "resnet50_split_cut1"]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def client_digest(cid):
    from coala_amd.compression import UpdateCodec
    from coala_amd.layouts import build_module
    from tests.oracle_backend import OracleBackend

    name = LAYOUTS[cid % len(LAYOUTS)]
    g = build_module(name, seed=100)
    w = build_module(name, seed=200 + cid)
    codec = UpdateCodec(0.01, 8, "delta", backend=OracleBackend())
    up = codec.encode(w.state_dict(), base=codec.snapshot(g))
    st = codec.decode_state(up, base=codec.snapshot(g))
    h = hashlib.sha256(up.to_bytes())
    for t in st.values():
        h.update(t.contiguous().reshape(-1).view(torch.uint8).numpy().tobytes())
    return cid, h.hexdigest()


def client_cost(cid):
    from coala_amd.layouts import fp32_sizes
    return sum(fp32_sizes(LAYOUTS[cid % len(LAYOUTS)]))


def _worker(rank, world, port, n_clients, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    groups = greedy_groups([client_cost(c) for c in range(n_clients)], world)
    mine = [client_digest(c) for c in groups[rank]]
    allr = [None] * world
    dist.all_gather_object(allr, mine)
    if rank == 0:
        q.put(sorted(x for part in allr for x in part))
    dist.destroy_process_group()


def test_split_sizes_match_reference_randomize_grouping():
    assert split_sizes(10, 4) == [2, 2, 3, 3]
    assert split_sizes(64, 4) == [16] * 4
    assert [len(g) for g in contiguous_groups(range(7), 3)] == [2, 2, 3]
    gs = contiguous_groups(range(20), 3, shuffle_seed=1)
    assert sorted(x for g in gs for x in g) == list(range(20))


def test_greedy_groups_balance():
    costs = [10, 9, 8, 7, 6, 5, 4, 3, 2, 1]
    gs = greedy_groups(costs, 3)
    loads = sorted(sum(costs[i] for i in g) for g in gs)
    assert sorted(i for g in gs for i in g) == list(range(10))
    assert loads[-1] - loads[0] <= max(costs)


@pytest.mark.timeout(300)
def test_two_rank_gloo_sharded_equals_serial():
    n_clients, world = 7, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_clients, q)) for r in range(world)]
    [p.start() for p in procs]
    got = q.get(timeout=240)
    [p.join(timeout=60) for p in procs]
    assert all(p.exitcode == 0 for p in procs)
    serial = sorted(client_digest(c) for c in range(n_clients))
    assert got == serial


def _fused_sum_worker(rank, world, port, q, content="all"):
    """Each rank aggregates its own uploads; the fused path (one coalac_aggregate in "sum" mode, then
    reduce_models) must equal the reference's distributed branch on decoded modules (server/base.py:
    594-598: weighted_sum, then reduce_models = all_reduce + div, distributed.py:42-57)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from coala_amd.compression import CompressionServerMixin, UpdateCodec
    from coala_amd.fl import LoopbackServer, weighted_sum
    from coala_amd.fl.distributed import reduce_models
    from coala_amd.layouts import build_module
    from tests.oracle_backend import OracleBackend

    class Conf:
        class server:
            aggregation_strategy = "FedAvg"
            aggregation_content = content
        is_distributed = True
        device = "cpu"

    class Fused(CompressionServerMixin, LoopbackServer):
        codec_ratio, codec_bits, codec_mode, codec_backend = 0.05, 8, "delta", OracleBackend()
        codec_fused_aggregate = True

    name = "resnet18_split_cut4"
    g = build_module(name, seed=1)
    codec = UpdateCodec(0.05, 8, "delta", backend=OracleBackend())
    base = codec.snapshot(g)
    ups, weights = [], []
    for i in range(3):
        cid = rank * 3 + i
        w = build_module(name, seed=50 + cid)
        for b in w.buffers():
            if b.dtype == torch.int64:
                b.fill_(cid + 2)
        ups.append(codec.encode(w.state_dict(), base=base))
        weights.append([4, 0, 9, 1, 6, 2][cid])
    s = Fused(g, [])
    s.conf = Conf
    fused = s.aggregate(list(ups), list(weights))
    dec = [codec.decode_module(u, g, base=base) for u in ups]
    if content == "parameters":  # server/base.py:588-591: the *_only_params pair (distributed.py:60-74)
        from coala_amd.fl.distributed import reduce_models_only_params
        from coala_amd.fl.strategies import weighted_sum_only_params
        ref, tot = weighted_sum_only_params(dec, list(weights))
        reduce_models_only_params(ref, torch.tensor(tot))
    else:
        ref, tot = weighted_sum(dec, list(weights))
        reduce_models(ref, torch.tensor(tot))
    same = all(a.dtype == b.dtype and torch.equal(a, b)
               for a, b in zip(ref.state_dict().values(), fused.state_dict().values()))
    res = [None] * world
    dist.all_gather_object(res, same)
    if rank == 0:
        q.put(res)
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("content", ["all", "parameters"])
def test_two_rank_gloo_fused_weighted_sum_equals_reference_reduce(content):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fused_sum_worker, args=(r, world, port, q, content)) for r in range(world)]
    [p.start() for p in procs]
    got = q.get(timeout=240)
    [p.join(timeout=60) for p in procs]
    assert all(p.exitcode == 0 for p in procs)
    assert got == [True, True]
