"""The plugin boundary pinned by the REAL reference client (tests/golden/plugin_run_train.npz).

tests/golden/make_golden.py mixed CompressionClientMixin into the reference's own BaseClient and drove its
run_train (/root/reference/coala/client/base.py:123-159: set_model, decompression, train, compression,
calculate_model_size, upload -> construct_upload_request, codec.marshal(copy.deepcopy(self.model)) :363)
for 3 clients of the reference simple_cnn (channels=16), with the CPU oracle as codec backend, and ran the
reference's strategies.federated_averaging (server/strategies.py:6-29) on the decoded uploads.

Here the loopback harness (coala_amd/fl/loop.py, the restated run_train) reproduces, from the committed
global model and the fixture's deterministic training step:
  * the exact UploadContent.data bytes, data_size and type of every upload (CPU oracle backend, and on
    the GPU the HIP backend: same bytes);
  * the decoded uploads (sha256 of the decoded state) and the reference FedAvg of them, bit for bit —
    both the restated decode-then-FedAvg and the fused aggregate kernel in CPU-division mode.
"""
import copy
import hashlib
import os

import numpy as np
import pytest
import torch
from torch import nn

from coala_amd.compression import CompressionClientMixin, CompressionServerMixin, UpdateCodec
from coala_amd.fl import LoopbackClient, federated_averaging, unmarshal
from tests.oracle_backend import OracleBackend

GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "plugin_run_train.npz"))
SIZES = GOLD["weights"].tolist()
RATIO, BITS, NOISE_SEED, NOISE = 0.05, 8, 1000, 1e-3  # tests/golden/make_golden.py PLUGIN_*


def global_model():
    root = nn.Module()
    for key in [k for k in GOLD.files if k.startswith("global/")]:
        path = key[len("global/"):].split(".")
        mod = root
        for p in path[:-1]:
            if not hasattr(mod, p):
                mod.add_module(p, nn.Module())
            mod = getattr(mod, p)
        mod.register_parameter(path[-1], nn.Parameter(torch.from_numpy(GOLD[key].copy())))
    return root


def make_client_class(backend, device):
    class Client(CompressionClientMixin, LoopbackClient):
        codec_ratio, codec_bits, codec_mode, codec_backend = RATIO, BITS, "delta", backend

        def train(self, round_id):  # make_golden.plugin_train_step, restated
            self.model.to(self.device)
            g = torch.Generator().manual_seed(NOISE_SEED + int(self.cid[1:]))
            with torch.no_grad():
                for p in self.model.parameters():
                    p.add_((torch.randn(p.shape, generator=g) * NOISE).to(p.device))

    return lambda i: Client(f"c{i}", SIZES[i], device=device)


def digest(state):
    h = hashlib.sha256()
    for t in state.values():
        h.update(t.detach().cpu().contiguous().reshape(-1).view(torch.uint8).numpy().tobytes())
    return h.digest()


def run(backend, device):
    g0 = global_model()
    mk = make_client_class(backend, device)
    reqs = [mk(i).run_train(g0, 0, task_id="task0") for i in range(len(SIZES))]
    for i, req in enumerate(reqs):
        gold = GOLD[f"upload_bytes/{i}"].tobytes()
        assert req.content.data == gold, f"upload {i}: {len(req.content.data)} B vs reference {len(gold)} B"
        assert req.content.data_size == int(GOLD[f"data_size/{i}"][0])
        assert req.content.type == int(GOLD[f"content_type/{i}"][0])

    class Server(CompressionServerMixin):
        codec_ratio, codec_bits, codec_mode, codec_backend = RATIO, BITS, "delta", backend

    srv = Server()
    srv.model = g0
    ups = [unmarshal(r.content.data) for r in reqs]
    dec = [srv.decompression(u) for u in ups]
    for i, m in enumerate(dec):
        assert digest(m.state_dict()) == GOLD[f"decoded_sha256/{i}"].tobytes(), f"decoded upload {i}"
    cpu = [copy.deepcopy(m).cpu() for m in dec]
    avg = federated_averaging(cpu, list(SIZES))
    fused = UpdateCodec(RATIO, BITS, "delta", backend).aggregate(
        ups, list(SIZES), g0, base=srv._global_snapshot(), mode="div")
    for (k, v), (k2, w) in zip(avg.state_dict().items(), fused.state_dict().items()):
        ref = GOLD[f"avg/{k}"]
        np.testing.assert_array_equal(v.numpy().view(np.uint32), ref.view(np.uint32), err_msg=k)
        np.testing.assert_array_equal(w.cpu().numpy().view(np.uint32), ref.view(np.uint32), err_msg=k)


def test_reference_run_train_fixture_oracle():
    run(OracleBackend(), "cpu")


def test_fixture_upload_size_is_payload():
    up = unmarshal(GOLD["upload_bytes/0"].tobytes())
    assert float(GOLD["upload_size_mb/0"][0]) == up.nbytes * 8 / (8 * 1024 * 1024)


@pytest.mark.gpu
def test_reference_run_train_fixture_hip(cuda):
    run(None, "cuda")
