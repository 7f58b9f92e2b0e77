"""splitFL cut-layer feature uploads through the plugin (the C5 feature tensors).

The reference's splitFL client serialises `{"content": [feature.detach().cpu(), label], "name": [...]}`
in marshal_data("feature_label") (application/splitFL/client/base_sfl.py:248-257) and its server reads
it back with decompression(codec.unmarshal(data)) (application/splitFL/server/base_sfl.py:207-209). The
reference splitFL client cannot be imported on the GPU box (no /root/reference there), so `SFLClient` below
restates that marshal_data as the mixin's parent; tests/golden/splitfl_features.npz, written in the build
container by the REAL BaseSFLClient.marshal_data (plain, and with the mixin: tests/golden/make_golden.py
make_splitfl_fixture), pins the restatement's dict layout and the mixin's exact upload bytes. Bar: the
server-side decoded feature equals the oracle's decode of the same tensor bit for bit (CPU: oracle backend;
GPU: the HIP codec), labels unchanged, model uploads and uncompressed runs untouched.
"""
import os
import copy
import pickle

import numpy as np
import pytest
import torch

from coala_amd.compression import CompressedUpdate, CompressionClientMixin, CompressionServerMixin
from coala_amd.compression.plugin import DATA_TYPE_FEATURE
from coala_amd.compression.spec import SegmentTable
from oracle import codec_oracle as O
from tests.oracle_backend import OracleBackend

FEATURE_SHAPES = [(32, 64, 32, 32), (32, 256, 32, 32), (32, 128, 16, 16)]  # C5's feature tensors


class SFLClient:
    """Restates application/splitFL/client/base_sfl.py:248-257 (marshal_data) for the tests."""

    def __init__(self, feature, label):
        self.feature, self.label, self.model = feature, label, None

    def marshal_data(self, content):
        if content == "model":
            return pickle.dumps(copy.deepcopy(self.model)), 0
        d = {"content": [copy.deepcopy(self.feature.detach().cpu()), copy.deepcopy(self.label)],
             "name": ["feature", "label"]}
        return pickle.dumps(d), DATA_TYPE_FEATURE


class SFLServer:
    def decompression(self, model):
        return model


def classes(backend, ratio=0.01, bits=8, on=True):
    class Client(CompressionClientMixin, SFLClient):
        codec_features, codec_ratio, codec_bits, codec_backend = on, ratio, bits, backend

    class Server(CompressionServerMixin, SFLServer):
        codec_ratio, codec_bits, codec_backend = ratio, bits, backend

    return Client, Server


def synth_feature(shape, device, seed=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.relu(torch.randn(shape, generator=g))  # activations after ReLU: half zeros
    return x.to(device)


def oracle_dense(x, ratio, bits):
    n = x.numel()
    t = SegmentTable([n], ratio, 1)
    segs = t.segs.astype(np.int64)
    flat = np.zeros(t.span, np.float32)
    flat[:n] = x.detach().cpu().reshape(-1).numpy()
    idx, vals, mn, sc = O.encode(flat, segs, bits)
    return O.decode(idx, vals, mn, sc, segs, bits, t.span)[:n].reshape(x.shape)


def roundtrip(Client, Server, feature, label):
    c = Client(feature, label)
    data, typ = c.marshal_data("feature_label")
    got = Server().decompression(pickle.loads(data))  # server/base_sfl.py:207
    return data, typ, got


@pytest.mark.parametrize("shape", [(4, 8, 8, 8), (3, 5, 7)])
def test_feature_upload_cpu_oracle(shape):
    Client, Server = classes(OracleBackend())
    x, lab = synth_feature(shape, "cpu", 1), torch.arange(shape[0])
    data, typ, got = roundtrip(Client, Server, x, lab)
    assert typ == DATA_TYPE_FEATURE
    sent = pickle.loads(data)
    assert isinstance(sent["content"][0], CompressedUpdate) and sent["name"] == ["feature", "label"]
    f, l2 = got["content"]
    assert tuple(f.shape) == shape and torch.equal(l2, lab)
    np.testing.assert_array_equal(f.cpu().numpy().view(np.uint32), oracle_dense(x, 0.01, 8).view(np.uint32))
    assert got is not sent and isinstance(sent["content"][0], CompressedUpdate)  # the received dict is kept


def test_feature_upload_off_and_model_pass_through():
    x, lab = synth_feature((2, 3, 4, 4), "cpu"), torch.tensor([1, 0])
    Client, Server = classes(OracleBackend(), on=False)
    data, typ, got = roundtrip(Client, Server, x, lab)
    ref, rtyp = SFLClient(x, lab).marshal_data("feature_label")
    a, b = pickle.loads(data), pickle.loads(ref)  # (pickled storage keys differ between calls)
    assert typ == rtyp and a["name"] == b["name"] and all(torch.equal(u, v) for u, v in zip(a["content"], b["content"]))
    assert torch.equal(got["content"][0], x)
    Client, Server = classes(OracleBackend())
    c = Client(x, lab)
    c.model = torch.nn.Linear(2, 2)
    data, typ = c.marshal_data("model")
    assert typ == 0 and isinstance(pickle.loads(data), torch.nn.Linear)
    plain = {"content": [x, lab], "name": ["feature", "label"]}
    assert Server().decompression(plain) is plain  # nothing compressed: unchanged


@pytest.mark.gpu
@pytest.mark.parametrize("shape", FEATURE_SHAPES)
def test_feature_upload_gpu(cuda, shape):
    """The C5 feature tensors (up to 8,388,608 elements) on the training device: encoded in place by the
    HIP codec, decoded on the server's GPU, bit-exact vs the oracle; the upload is ~40x smaller than the
    reference's dense pickle."""
    from coala_amd.compression.codec import HipBackend
    Client, Server = classes(HipBackend())
    x, lab = synth_feature(shape, cuda, 2), torch.randint(0, 10, (shape[0],))
    data, typ, got = roundtrip(Client, Server, x, lab)
    f, l2 = got["content"]
    assert f.device.type == "cuda" and tuple(f.shape) == shape and torch.equal(l2, lab)
    np.testing.assert_array_equal(f.cpu().numpy().view(np.uint32), oracle_dense(x, 0.01, 8).view(np.uint32))
    dense, _ = SFLClient(x, lab).marshal_data("feature_label")
    assert len(data) * 30 < len(dense)


GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "splitfl_features.npz")
SFL_RATIO, SFL_BITS = 0.05, 8  # make_golden.py make_splitfl_fixture


def _fixture():
    z = np.load(GOLDEN)  # data arrays only (allow_pickle stays False)
    return {k: z[k] for k in z.files}


def test_restated_marshal_data_matches_reference_client():
    """The restated SFLClient.marshal_data builds what the reference's BaseSFLClient.marshal_data built for
    the fixture's feature: the same data type, the same name list, the same feature and label tensors."""
    z = _fixture()
    x, lab = torch.from_numpy(z["feature"]), torch.from_numpy(z["label"])
    data, typ = SFLClient(x, lab).marshal_data("feature_label")
    d = pickle.loads(data)  # (our own bytes)
    assert typ == int(z["plain/type"][0]) == DATA_TYPE_FEATURE
    assert d["name"] == [str(v) for v in z["plain/names"]]
    assert torch.equal(d["content"][0], x) and torch.equal(d["content"][1], lab)


def _mixin_upload(backend, device):
    z = _fixture()
    Client, _ = classes(backend, ratio=SFL_RATIO, bits=SFL_BITS)
    x, lab = torch.from_numpy(z["feature"]).to(device), torch.from_numpy(z["label"])
    data, typ = Client(x, lab).marshal_data("feature_label")
    d = pickle.loads(data)  # (our own bytes)
    assert typ == int(z["mixed/type"][0])
    assert d["name"] == [str(v) for v in z["mixed/names"]] and torch.equal(d["content"][1], lab)
    assert isinstance(d["content"][0], CompressedUpdate)
    return z, d["content"][0].to_bytes()


def test_mixin_feature_upload_bytes_match_reference_client_cpu():
    """CompressionClientMixin on the restated client (oracle backend) writes the upload the mixin wrote on top
    of the REAL reference BaseSFLClient for the fixture: same type and dict layout, the encoded feature byte
    for byte (the whole pickle differs only in the label storage's address key)."""
    z, blob = _mixin_upload(OracleBackend(), "cpu")
    assert blob == z["mixed/carrier"].tobytes()


@pytest.mark.gpu
def test_mixin_feature_upload_bytes_match_reference_client_gpu(cuda):
    """The same upload encoded on the GPU by the HIP codec: the identical bytes."""
    from coala_amd.compression.codec import HipBackend
    z, blob = _mixin_upload(HipBackend(), cuda)
    assert blob == z["mixed/carrier"].tobytes()
