"""The plugin mixins on the GPU with the reference's device placement:

  * the server's global model stays on the CPU (coala/server/base.py keeps self.model there until
    test_in_server, :280; set_model(load_dict=True) loads into it, :571);
  * the client snapshots w_global in decompression() right after set_model (client/base.py:138-141),
    BEFORE pretrain moves the model to the training device (:245), so the snapshot starts on the CPU;
  * compression() then encodes the trained GPU state (client/base.py:144-153).

The HIP codec must run on the GPU in all three places, and every decoded upload must equal the oracle
backend's (w_global + decode(encode(delta))) bit for bit.
"""
import copy

import numpy as np
import pytest
import torch

from coala_amd.compression import CompressedUpdate, CompressionClientMixin, CompressionServerMixin
from coala_amd.fl import LoopbackClient, LoopbackServer
from coala_amd.layouts import build_module
from tests.oracle_backend import OracleBackend

pytestmark = pytest.mark.gpu


def classes(backend, device):
    class Client(CompressionClientMixin, LoopbackClient):
        codec_ratio, codec_bits, codec_mode, codec_backend = 0.01, 8, "delta", backend

        def __init__(self, *a, **k):
            super().__init__(*a, device=device, **k)

    class Server(CompressionServerMixin, LoopbackServer):
        codec_ratio, codec_bits, codec_mode, codec_backend = 0.01, 8, "delta", backend

    return Client, Server


@pytest.mark.parametrize("layout", ["lenet", "resnet18"])
def test_cpu_global_gpu_training_delta_mode(cuda, layout):
    g0 = build_module(layout, seed=4)  # on the CPU, like the reference server's global model
    Cg, Sg = classes(None, "cuda")      # default backend: the HIP codec
    Co, So = classes(OracleBackend(), "cpu")
    hip = Sg(copy.deepcopy(g0), [Cg(f"c{i}", 10 + i, step_seed=i) for i in range(3)])
    ora = So(copy.deepcopy(g0), [Co(f"c{i}", 10 + i, step_seed=i) for i in range(3)])
    for r in range(2):
        hip.distribution_to_train(r)
        ora.distribution_to_train(r)
        for cid in hip.uploaded:
            a, b = hip.uploaded[cid].state_dict(), ora.uploaded[cid].state_dict()
            for (k, x), (k2, y) in zip(a.items(), b.items()):
                assert k == k2 and x.dtype == y.dtype
                assert x.device.type == "cuda"
                xc = x.cpu()
                if x.dtype == torch.float32:
                    np.testing.assert_array_equal(xc.numpy().view(np.uint32), y.numpy().view(np.uint32), err_msg=k)
                else:
                    assert torch.equal(xc, y), k
        hip.aggregation()
        ora.aggregation()
        assert all(t.device.type == "cpu" for t in hip.model.state_dict().values())
        # the two global models differ only by torch's GPU-vs-CPU scalar division inside FedAvg
        for x, y in zip(hip.model.state_dict().values(), ora.model.state_dict().values()):
            if x.dtype == torch.float32:
                assert torch.allclose(x, y, rtol=1e-6, atol=1e-9)
        ora.model.load_state_dict(hip.model.state_dict())  # next round starts from the same global


def test_carrier_deepcopy_then_marshal_on_gpu(cuda):
    """construct_upload_request's codec.marshal(copy.deepcopy(self.model)) (client/base.py:363) on a
    GPU carrier: the deep copy shares the device payload; the pickle is one pack."""
    import pickle
    Cg, _ = classes(None, "cuda")
    c = Cg("c0", 3)
    g = build_module("resnet18_split_cut4", seed=1)
    req = c.run_train(g, 0)
    up = pickle.loads(req.content.data)
    assert isinstance(up, CompressedUpdate) and up.encoded.idx.device.type == "cpu"
    assert len(req.content.data) < up.nbytes + 16384


@pytest.mark.parametrize("mode", ["delta", "weights"])
def test_encode_in_place_from_parameters_equals_flat_encode(cuda, mode):
    """compression() reads the parameters in place (coalac_encode_segptr: one device pointer per tensor,
    no flattening copy); the result equals the flat-buffer encode bit for bit, and a state with a
    misaligned tensor (a view at an odd offset) falls back to the flattened path with the same bytes."""
    from coala_amd.compression import UpdateCodec, flatten_state
    m = build_module("resnet18", seed=3, device="cuda")
    g = build_module("resnet18", seed=4, device="cuda")
    codec = UpdateCodec(0.01, 8, mode)
    base = codec.snapshot(g) if mode == "delta" else None
    up = codec.encode(m.state_dict(), base=base)
    fs = flatten_state(m.state_dict())
    plan = codec.plan_for([e["n"] for e in fs.entries if e["kind"] == "seg"], fs.flat.device)
    ref = plan.encode(fs.flat, base=None if base is None else base.flat)
    torch.cuda.synchronize()
    for f in ("idx", "vals", "mn", "scale"):
        assert torch.equal(getattr(up.encoded, f), getattr(ref, f)), f
    # misaligned tensor: a 4-byte-offset view
    st = dict(m.state_dict())
    name = next(k for k, v in st.items() if v.dtype == torch.float32 and v.numel() > 5000)
    buf = torch.empty(st[name].numel() + 1, device="cuda")
    view = buf[1:].view(st[name].shape)
    view.copy_(st[name])
    assert view.data_ptr() % 16 != 0
    st[name] = view
    up2 = codec.encode(st, base=base)
    torch.cuda.synchronize()
    for f in ("idx", "vals", "mn", "scale"):
        assert torch.equal(getattr(up2.encoded, f), getattr(ref, f)), f


def test_encode_module_snapshots_counters_in_one_launch(cuda):
    """compression() through encode_module: the passthrough int64 counters are snapshotted by coalac_gather (one
    launch over a cached pointer array) — the same values as state_dict(), taken at encode time (a later change
    of the live counters does not reach the carrier), and the fp32 payload equals encode(state_dict())."""
    from coala_amd.compression import UpdateCodec
    from coala_amd.compression.codec import HipBackend
    m = build_module("resnet50_tv", seed=5, device="cuda")
    with torch.no_grad():
        for i, (k, v) in enumerate((k, v) for k, v in m.state_dict().items() if v.dtype == torch.int64):
            v.fill_(1000 + i)
    codec = UpdateCodec(0.01, 8, "weights")
    up = codec.encode_module(m)
    ref = codec.encode(m.state_dict())
    torch.cuda.synchronize()
    raw_names = [k for k, v in m.state_dict().items() if v.dtype == torch.int64]
    assert len(raw_names) == 53
    for k in raw_names:
        assert up.raw[k].item() == m.state_dict()[k].item() == ref.raw[k].item()
    for f in ("idx", "vals", "mn", "scale", "ustart"):
        assert torch.equal(getattr(up.encoded, f), getattr(ref.encoded, f)), f
    before = {k: up.raw[k].item() for k in raw_names}
    with torch.no_grad():
        for k in raw_names:
            m.state_dict()[k].add_(7)
    torch.cuda.synchronize()
    assert {k: up.raw[k].item() for k in raw_names} == before
    # the gather itself, against torch.stack, on scalars of every element size
    for dt in (torch.int64, torch.int32, torch.int16, torch.uint8):
        ts = [torch.tensor((i * 3 + 1) % 251, dtype=dt, device="cuda") for i in range(300)]
        got = HipBackend().gather_scalars(ts)
        assert got is not None and torch.equal(got, torch.stack(ts)), dt
