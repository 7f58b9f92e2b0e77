"""Plugin surface end to end on CPU (C1 plumbing): the hook mixins inside the loopback FL loop, with the
CPU oracle injected as the codec backend (the product has no CPU path; here the oracle is the checker).

Pinned against the reference: hook order and upload framing (tests/golden/hooks.json, captured from
coala/client/base.py:123-159,353-383) and FedAvg (tests/golden/fedavg.npz, from
coala/server/strategies.py:6-29,57-90).
"""
import copy
import json
import os
import pickle
import threading

import numpy as np
import pytest
import torch
from torch import nn

from coala_amd.compression import CompressedUpdate, CompressionClientMixin, CompressionServerMixin, UpdateCodec
from coala_amd.fl import LoopbackClient, LoopbackServer, federated_averaging, marshal, unmarshal, weighted_sum
from coala_amd.layouts import build_module
from oracle import codec_oracle as O
from tests.oracle_backend import OracleBackend

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def make_classes(ratio, bits, mode):
    class Client(CompressionClientMixin, LoopbackClient):
        codec_ratio, codec_bits, codec_mode, codec_backend = ratio, bits, mode, OracleBackend()

    class Server(CompressionServerMixin, LoopbackServer):
        codec_ratio, codec_bits, codec_mode, codec_backend = ratio, bits, mode, OracleBackend()

    return Client, Server


def test_hook_order_and_framing_match_reference():
    gold = json.load(open(os.path.join(GOLD, "hooks.json")))
    Client, _ = make_classes(0.01, 8, "delta")
    c = Client("c0", datasize=gold["data_size"])
    req = c.run_train(build_module("lenet", seed=1), round_id=gold["round_id"], task_id=gold["task_id"])
    assert c.trace == gold["hook_order"]
    assert req.content.type == gold["DATA_TYPE_PARAMS"] == gold["content_type"]
    assert req.content.data_size == gold["data_size"]
    up = unmarshal(req.content.data)
    assert isinstance(up, CompressedUpdate)
    # after upload the client holds its trained module again (next round's set_model needs it)
    assert isinstance(c.model, nn.Module)
    # real payload size is tracked, not params x 32 bit (client/base.py:155, 474-487)
    nominal = sum(p.numel() for p in c.model.parameters()) * 32 / 8 / 2 ** 20
    assert c.upload_sizes[-1] < nominal / 15


def _tiny_from_npz(arrs, prefix):
    root = nn.Module()
    for key in [k for k in arrs.files if k.startswith(prefix + "/")]:
        path = key[len(prefix) + 1:].split(".")
        mod = root
        for p in path[:-1]:
            if not hasattr(mod, p):
                mod.add_module(p, nn.Module())
            mod = getattr(mod, p)
        t = torch.from_numpy(arrs[key].copy())
        if t.dtype == torch.float32 and path[-1] not in ("running_mean", "running_var"):
            mod.register_parameter(path[-1], nn.Parameter(t))
        else:
            mod.register_buffer(path[-1], t)
    return root


def test_fedavg_restatement_matches_reference_fixture():
    a = np.load(os.path.join(GOLD, "fedavg.npz"))
    models = [_tiny_from_npz(a, f"in{i}") for i in range(3)]
    w = a["weights"].tolist()
    avg = federated_averaging([copy.deepcopy(m) for m in models], w)
    for k, v in avg.state_dict().items():
        ref = a[f"avg/{k}"]
        assert v.dtype == torch.from_numpy(ref).dtype, k
        np.testing.assert_array_equal(v.numpy(), ref)
    s, tot = weighted_sum([copy.deepcopy(m) for m in models], w)
    assert tot == int(a["total"][0])
    for k, v in s.state_dict().items():
        np.testing.assert_array_equal(v.numpy(), a[f"sum/{k}"])


def test_lossless_mode_aggregates_identically_to_uncompressed():
    """ratio 1, raw fp32 values, weights mode: compression on/off must give bit-identical FedAvg."""
    Client, Server = make_classes(1.0, 32, "weights")
    g0 = build_module("resnet18_split_cut4", seed=3)
    plain = LoopbackServer(copy.deepcopy(g0), [LoopbackClient(f"c{i}", 10 + i, step_seed=i) for i in range(3)])
    comp = Server(copy.deepcopy(g0), [Client(f"c{i}", 10 + i, step_seed=i) for i in range(3)])
    for r in range(2):
        plain.round(r)
        comp.round(r)
    for (k, a), (k2, b) in zip(plain.model.state_dict().items(), comp.model.state_dict().items()):
        assert k == k2 and a.dtype == b.dtype
        assert torch.equal(a, b), k


def test_c1_plumbing_lenet_four_clients_delta_mode():
    """C1: LeNet (FEMNIST model), 4 loopback clients, delta mode, ratio 0.01, 8-bit codes."""
    Client, Server = make_classes(0.01, 8, "delta")
    g0 = build_module("lenet", seed=5)
    clients = [Client(f"c{i}", 20 + i, step_seed=i) for i in range(4)]
    server = Server(copy.deepcopy(g0), clients)
    server.round(0)
    # independent check: every decoded upload equals w_global + oracle(decode(encode(delta)))
    for c in clients:
        up = server.uploaded[c.cid]
        trained = c.model.state_dict()
        for (name, w), g in zip(up.state_dict().items(), g0.state_dict().values()):
            if w.dtype != torch.float32:
                assert torch.equal(w, trained[name])
                continue
            d = (trained[name] - g).reshape(-1).numpy()
            k = O.k_for(d.size, 0.01)
            idx, q, mn, sc = O.encode_segment(d, k, 8)
            ref = g.reshape(-1).numpy() + O.decode_segment(idx, q, mn, sc, d.size, 8)
            np.testing.assert_array_equal(w.reshape(-1).numpy().view(np.uint32), ref.view(np.uint32))
    ref_avg = federated_averaging(list(server.uploaded.values()), list(server.weights.values()))
    for a, b in zip(ref_avg.state_dict().values(), server.model.state_dict().values()):
        assert torch.equal(a.to(b.dtype), b)


def test_server_passes_through_non_carriers_and_none_model_client():
    _, Server = make_classes(0.01, 8, "delta")
    s = Server(build_module("lenet"), [])
    feat = {"content": [torch.zeros(2, 3), torch.ones(2)], "name": ["f", "y"]}  # splitFL payload
    assert s.decompression(feat) is feat
    m = build_module("lenet")
    assert s.decompression(m) is m
    Client, _ = make_classes(0.01, 8, "delta")
    c = Client("c", 1)
    c.model = None           # application/MAS pattern: decompression() before any model exists
    c.decompression()
    c.compression()
    assert c.model is None


def test_server_decode_is_thread_safe_and_never_aliases_global():
    """Remote servers decode from one thread per upload (server/service.py:74)."""
    Client, Server = make_classes(0.05, 8, "delta")
    g0 = build_module("simple_cnn_split_cut4", seed=9)
    ups = []
    for i in range(6):
        c = Client(f"c{i}", 1, step_seed=i)
        ups.append(pickle.loads(c.run_train(g0, 0).content.data))
    s = Server(copy.deepcopy(g0), [])
    seq = [s.decompression(u) for u in ups]
    out = [None] * len(ups)

    def work(i):
        out[i] = s.decompression(ups[i])
    ts = [threading.Thread(target=work, args=(i,)) for i in range(len(ups))]
    [t.start() for t in ts]
    [t.join() for t in ts]
    gptrs = {t.data_ptr() for t in s.model.state_dict().values()}
    for a, b in zip(seq, out):
        for x, y in zip(a.state_dict().values(), b.state_dict().values()):
            assert torch.equal(x, y)
            assert y.data_ptr() not in gptrs


def test_codec_rejects_mismatched_layouts_and_bad_args():
    with pytest.raises(ValueError):
        UpdateCodec(ratio=0.0)
    with pytest.raises(ValueError):
        UpdateCodec(bits=9)
    with pytest.raises(ValueError):
        UpdateCodec(mode="sparse")
    codec = UpdateCodec(0.1, 8, "delta", backend=OracleBackend())
    a = build_module("lenet")
    b = build_module("simple_cnn_split_cut1")
    with pytest.raises(ValueError):
        codec.encode(a.state_dict(), base=codec.snapshot(b))


@pytest.mark.parametrize("mode,bits,strategy", [("delta", 8, "FedAvg"), ("weights", 4, "FedAvg"),
                                                 ("delta", 32, "equal")])
def test_fused_aggregation_matches_decode_then_fedavg(mode, bits, strategy):
    """codec_fused_aggregate: decode + FedAvg of all uploads in one call must leave the global model
    bit-identical to decompressing every upload and running the reference federated_averaging
    (here on the CPU: mode "div"), including int64 BatchNorm counters, over two rounds."""
    Client, Server = make_classes(0.05, bits, mode)

    class Fused(Server):
        codec_fused_aggregate = True

    class Conf:
        class server:
            aggregation_strategy = strategy
            aggregation_content = "all"
        is_distributed = False

    g0 = build_module("resnet18_split_cut4", seed=7)
    mk = lambda: [Client(f"c{i}", [13, 0, 7][i] if strategy == "FedAvg" else 5, step_seed=i) for i in range(3)]
    plain, fused = Server(copy.deepcopy(g0), mk()), Fused(copy.deepcopy(g0), mk())
    fused.conf = plain.conf = Conf
    if strategy == "equal":  # the reference's EQUAL_AVERAGE branch (server/base.py:584-585)
        plain.aggregate = lambda models, weights: federated_averaging(models, [1 for _ in models])
    for r in range(2):
        plain.round(r)
        fused.round(r)
        assert all(isinstance(m, CompressedUpdate) for m in fused.uploaded.values())
        for (k, a), (k2, b) in zip(plain.model.state_dict().items(), fused.model.state_dict().items()):
            assert k == k2 and a.dtype == b.dtype, k
            assert torch.equal(a, b), k


def test_fused_aggregation_zero_weights_and_oracle_modes():
    """Weights summing to 0 become 1 per update (strategies.py:21-22); the two division modes of the
    oracle restate torch's CPU (a / b) and GPU (a * (1 / b)) scalar division."""
    codec = UpdateCodec(0.1, 8, "weights", backend=OracleBackend())
    ms = [build_module("simple_cnn_split_cut2", seed=s) for s in range(3)]
    ups = [codec.encode(m.state_dict()) for m in ms]
    agg = codec.aggregate(ups, [0, 0, 0], ms[0], mode="div")
    dec = [codec.decode_module(u, ms[0]) for u in ups]
    ref = federated_averaging(dec, [0, 0, 0])
    for a, b in zip(ref.state_dict().values(), agg.state_dict().values()):
        assert torch.equal(a, b)
    x = np.float32([1.0, 3.0, 10.0])
    tot = np.float32(3.0)
    assert np.array_equal(x / tot, torch.div(torch.from_numpy(x), 3).numpy())
    r = x * (np.float32(1.0) / tot)
    assert not np.array_equal(r, x / tot)  # 10 * (1/3) != 10 / 3 in fp32: the modes really differ


def test_params_only_restatement_matches_reference_fixture():
    """federated_averaging_only_params / weighted_sum_only_params restated (coala_amd/fl/strategies.py)
    against the reference's own outputs (tests/golden/fedavg_params.npz, made by make_golden.py from
    coala/server/strategies.py:32-54, 93-124): parameters averaged, buffers left as models[0]'s."""
    from coala_amd.fl.strategies import federated_averaging_only_params, weighted_sum_only_params
    a = np.load(os.path.join(GOLD, "fedavg_params.npz"))
    models = [_tiny_from_npz(a, f"in{i}") for i in range(3)]
    w = a["weights"].tolist()
    avg = federated_averaging_only_params([copy.deepcopy(m) for m in models], w)
    for k, v in avg.state_dict().items():
        np.testing.assert_array_equal(v.detach().numpy(), a[f"avg/{k}"], err_msg=k)
    for tag, ww, tot_key in (("sum", w, "total"), ("sum0", [0, 0, 0], "total0")):
        s, tot = weighted_sum_only_params([copy.deepcopy(m) for m in models], ww)
        assert tot == int(a[tot_key][0])
        for k, v in s.state_dict().items():
            np.testing.assert_array_equal(v.detach().numpy(), a[f"{tag}/{k}"], err_msg=f"{tag}/{k}")
    assert np.array_equal(a["avg/bn.running_mean"], a["in0/bn.running_mean"])  # buffers: models[0]'s


@pytest.mark.parametrize("mode,bits", [("delta", 8), ("weights", 32)])
def test_fused_params_only_aggregation_matches_decode_then_fedavg_only_params(mode, bits):
    """aggregation_content "parameters" stays fused: the server's global model after two rounds is
    bit-identical to decompressing every upload and running federated_averaging_only_params (buffers —
    fp32 running stats and int64 counters — from the first upload)."""
    Client, Server = make_classes(0.05, bits, mode)

    class Fused(Server):
        codec_fused_aggregate = True

    class Conf:
        class server:
            aggregation_strategy = "FedAvg"
            aggregation_content = "parameters"
        is_distributed = False

    g0 = build_module("resnet18_split_cut4", seed=9)
    mk = lambda: [Client(f"c{i}", [13, 4, 7][i], step_seed=i) for i in range(3)]
    plain, fused = Server(copy.deepcopy(g0), mk()), Fused(copy.deepcopy(g0), mk())
    fused.conf = plain.conf = Conf
    for r in range(2):
        plain.round(r)
        fused.round(r)
        assert all(isinstance(m, CompressedUpdate) for m in fused.uploaded.values())
        for (k, a), (k2, b) in zip(plain.model.state_dict().items(), fused.model.state_dict().items()):
            assert k == k2 and a.dtype == b.dtype, k
            assert torch.equal(a, b), k
