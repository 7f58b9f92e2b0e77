"""GPU parity of the download direction through the C ABI: the server's compressed
global model (weights mode, dense ratio 1 and sparse ratios) decoded by the HIP kernels is bit-identical
to the CPU oracle's per-tensor restatement, survives the pickle that remote distribution does
(server/base.py:397), and a full loopback round with compressed download + delta uploads decodes every
upload against exactly the base the client encoded it against."""
import copy
import pickle

import numpy as np
import pytest
import torch
from torch import nn

from coala_amd.compression import CompressedModel, CompressionClientMixin, CompressionServerMixin, \
    UpdateCodec, compress_model
from coala_amd.fl import LoopbackClient, LoopbackServer
from coala_amd.layouts import build_module
from oracle import codec_oracle as O

pytestmark = pytest.mark.gpu


def oracle_roundtrip(state, ratio, bits):
    out = {}
    for name, w in state.items():
        w = w.detach().cpu()
        if w.dtype != torch.float32 or w.numel() == 0:
            out[name] = w
            continue
        x = w.reshape(-1).numpy()
        idx, q, mn, sc = O.encode_segment(x, O.k_for(x.size, ratio), bits)
        out[name] = torch.from_numpy(O.decode_segment(idx, q, mn, sc, x.size, bits)).view(w.shape)
    return out


def assert_state_bits_equal(got, ref):
    assert list(got) == list(ref)
    for k in got:
        a, b = got[k].detach().cpu(), ref[k]
        assert a.dtype == b.dtype and a.shape == b.shape, k
        if a.dtype == torch.float32:
            np.testing.assert_array_equal(a.numpy().view(np.uint32), b.numpy().view(np.uint32), err_msg=k)
        else:
            assert torch.equal(a, b), k


@pytest.mark.parametrize("layout,ratio,bits", [("resnet18", 1.0, 8), ("resnet18", 1.0, 4),
                                               ("vit_b16", 1.0, 8), ("resnet18", 0.1, 8),
                                               ("lenet", 1.0, 32)])
def test_compressed_global_model_matches_oracle(cuda, layout, ratio, bits):
    g = build_module(layout, seed=11)
    cm = compress_model(g, UpdateCodec(ratio, bits, "weights"))
    ref = oracle_roundtrip(g.state_dict(), ratio, bits)
    assert_state_bits_equal(cm.state_dict(), ref)
    back = pickle.loads(pickle.dumps(cm))          # remote distribution: marshal / unmarshal
    assert_state_bits_equal(back.state_dict(), ref)
    m = back.materialize()
    assert isinstance(m, nn.Module) and not isinstance(m, CompressedModel)
    assert_state_bits_equal(m.state_dict(), ref)


def test_compressed_download_round_on_gpu(cuda):
    dev = torch.device("cuda", 0)

    class Client(CompressionClientMixin, LoopbackClient):
        codec_ratio, codec_bits, codec_mode = 0.02, 8, "delta"

    class Server(CompressionServerMixin, LoopbackServer):
        codec_ratio, codec_bits, codec_mode = 0.02, 8, "delta"
        codec_download = True

    g0 = build_module("resnet18_split_cut4", seed=5, device=dev)
    clients = [Client(f"c{i}", 4 + i, device=dev, step_seed=i) for i in range(3)]
    server = Server(copy.deepcopy(g0), clients, remote=True)
    for r in range(2):
        recon = oracle_roundtrip(server.model.state_dict(), 1.0, 8)
        server.round(r)
        assert not isinstance(server.model, CompressedModel)
        for c in clients:
            base = c._codec_base
            got = {e["name"]: base.flat[e["off"]:e["off"] + e["n"]].view(e["shape"])
                   for e in base.entries if e["kind"] == "seg"}
            assert_state_bits_equal(got, {k: recon[k] for k in got})
            up = server.uploaded[c.cid].state_dict()
            trained = c.model.state_dict()
            for name, w in up.items():
                if w.dtype != torch.float32:
                    continue
                d = (trained[name].cpu() - recon[name]).reshape(-1).numpy()
                idx, q, mn, sc = O.encode_segment(d, O.k_for(d.size, 0.02), 8)
                ref = recon[name].reshape(-1).numpy() + O.decode_segment(idx, q, mn, sc, d.size, 8)
                np.testing.assert_array_equal(w.detach().cpu().reshape(-1).numpy().view(np.uint32),
                                              ref.view(np.uint32), err_msg=name)
    fp32 = sum(t.numel() * 4 for t in g0.state_dict().values())
    assert max(server.download_sizes) < fp32 / 3
