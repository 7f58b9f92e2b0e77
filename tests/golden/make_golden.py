"""Generate the committed golden fixtures under tests/golden/ and coala_amd/layouts/.

Run in the build container (NOT on the GPU box — /root/reference does not exist there):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

What it pins, and from where (SURVEY.md §8(c) "What reference imports pin"):

1. Tensor layouts (name, shape, dtype of every state_dict entry, in insertion order) of the reference
   models the benchmarks synthesise updates for:
     lenet            /root/reference/coala/models/lenet.py:7-25            (C1, num_classes=62)
     resnet18         /root/reference/coala/models/resnet18.py:62-90        (C2, CIFAR-10)
     resnet50_tv      /root/reference/coala/models/resnet50.py:72-107       (C3; num_classes=1000 with a
                      7x7 stride-2 stem = the torchvision-equivalent layout SURVEY §8(a) a1 counts)
     vit_b16          /root/reference/application/FedPEFT/base_vit.py:346   (C4, ViT('B_16'), 224 px)
     splitFL client-side models at cut 1/2/4
                      /root/reference/application/splitFL/models/{resnet18,resnet50,simple_cnn}_split.py (C5)
2. FedAvg of decoded models: reference `strategies.federated_averaging` / `weighted_sum`
   (/root/reference/coala/server/strategies.py:6-29,57-90) on small seeded modules incl. an int64
   BatchNorm `num_batches_tracked` buffer -> fedavg.npz.
3. Hook order + upload framing of `BaseClient.run_train` (/root/reference/coala/client/base.py:123-159,
   353-383): a recording subclass drives the real method -> hooks.json.
4. Identity round trip of `codec.marshal/unmarshal` (/root/reference/coala/protocol/codec.py:4-9).
5. The plugin inside the REAL reference client (plugin_run_train.npz): CompressionClientMixin mixed into
   the reference's BaseClient (/root/reference/coala/client/base.py:123-159), driven by its own run_train
   for 3 clients of the reference simple_cnn (/root/reference/coala/models/simple_cnn.py, channels=16),
   with the CPU oracle as the codec backend: the UploadContent.data bytes the reference produces (the
   pickled carrier: codec.marshal(copy.deepcopy(self.model)), base.py:363), data_size / type, the
   tracked upload size, and the reference's strategies.federated_averaging (server/strategies.py:6-29)
   of the decoded uploads. tests/test_reference_fixture.py reproduces all of it with the HIP backend.
6. splitFL feature uploads through the REAL reference BaseSFLClient.marshal_data
   (/root/reference/application/splitFL/client/base_sfl.py:248-257), plain and with the mixin
   (splitfl_features.npz); tests/test_splitfl_features.py reproduces both.

The reference is imported read-only with a namespace stub for `coala` (its __init__ needs omegaconf,
which is not installed). No reference source is copied; only data is written.
"""
import copy
import json
import os
import sys
import types
from types import SimpleNamespace

import numpy as np
import torch
from torch import nn

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
LAYOUT_DIR = os.path.join(REPO, "coala_amd", "layouts")


def _stub_coala():
    pkg = types.ModuleType("coala")
    pkg.__path__ = [os.path.join(REF, "coala")]
    sys.modules["coala"] = pkg
    # coala/server/__init__.py imports server/base.py (omegaconf, torchvision): bypass it too
    srv = types.ModuleType("coala.server")
    srv.__path__ = [os.path.join(REF, "coala", "server")]
    sys.modules["coala.server"] = srv


def _layout(model):
    out = []
    for name, t in model.state_dict().items():
        out.append({"name": name, "shape": list(t.shape), "dtype": str(t.dtype).replace("torch.", "")})
    return out


def _save_layout(key, model, source):
    entries = _layout(model)
    n_f32 = sum(int(np.prod(e["shape"])) for e in entries if e["dtype"] == "float32")
    doc = {"model": key, "source": source, "n_entries": len(entries),
           "n_float32_entries": sum(e["dtype"] == "float32" for e in entries),
           "n_float32_elements": n_f32, "entries": entries}
    with open(os.path.join(LAYOUT_DIR, key + ".json"), "w") as f:
        json.dump(doc, f, indent=0)
    print(f"layout {key}: {doc['n_entries']} entries, {doc['n_float32_entries']} fp32, {n_f32} elems")
    return doc


def make_layouts():
    os.makedirs(LAYOUT_DIR, exist_ok=True)
    from coala.models import lenet, resnet18, resnet50
    _save_layout("lenet", lenet.Model(num_classes=62), "coala/models/lenet.py:7-25 Model(num_classes=62)")
    _save_layout("resnet18", resnet18.Model(num_classes=10), "coala/models/resnet18.py:62-90 Model(num_classes=10)")
    m = resnet50.Model(num_classes=1000)
    m.conv1 = nn.Conv2d(3, 64, kernel_size=7, stride=2, padding=3, bias=False)  # torchvision stem
    _save_layout("resnet50_tv", m, "coala/models/resnet50.py:72-107 Model(num_classes=1000) + 7x7/2 stem")

    sys.path.insert(0, os.path.join(REF, "application", "FedPEFT"))
    import base_vit
    vit = base_vit.ViT("B_16", pretrained=False, image_size=224, num_classes=1000)
    _save_layout("vit_b16", vit, "application/FedPEFT/base_vit.py:346 ViT('B_16', pretrained=False, 224, 1000)")
    sys.path.pop(0)

    sys.path.insert(0, os.path.join(REF, "application", "splitFL"))
    import importlib
    for mod in ("resnet18_split", "resnet50_split", "simple_cnn_split"):
        lib = importlib.import_module("models." + mod)
        for cut in (1, 2, 4):
            model = lib.Model()
            model.split(cut)
            client = model.client_cloud_copy[0]
            _save_layout(f"{mod}_cut{cut}", client,
                         f"application/splitFL/models/{mod}.py Model().split({cut}) client side")
    sys.path.pop(0)


class _Tiny(nn.Module):
    """Small module with conv + BN (int64 num_batches_tracked) + linear, for the FedAvg fixture."""

    def __init__(self):
        super().__init__()
        self.conv = nn.Conv2d(2, 3, 3)
        self.bn = nn.BatchNorm2d(3)
        self.fc = nn.Linear(5, 4)


def _seeded_tiny(seed):
    torch.manual_seed(seed)
    m = _Tiny()
    with torch.no_grad():
        for name, t in m.state_dict().items():
            if t.dtype == torch.float32:
                t.copy_(torch.randn(t.shape) * 0.1)
            else:
                t.fill_(seed % 7 + 1)
    return m


def make_fedavg():
    from coala.server import strategies
    models = [_seeded_tiny(s) for s in (11, 12, 13)]
    weights = [3, 5, 2]
    avg = strategies.federated_averaging([copy.deepcopy(m) for m in models], list(weights))
    wsum, total = strategies.weighted_sum([copy.deepcopy(m) for m in models], list(weights))
    arrays = {}
    for i, m in enumerate(models):
        for k, v in m.state_dict().items():
            arrays[f"in{i}/{k}"] = v.numpy()
    for k, v in avg.state_dict().items():
        arrays[f"avg/{k}"] = v.numpy()
    for k, v in wsum.state_dict().items():
        arrays[f"sum/{k}"] = v.numpy()
    arrays["weights"] = np.array(weights, dtype=np.int64)
    arrays["total"] = np.array([total], dtype=np.int64)
    np.savez(os.path.join(HERE, "fedavg.npz"), **arrays)
    print("fedavg.npz:", len(arrays), "arrays; avg dtypes",
          sorted({str(v.dtype) for v in avg.state_dict().values()}))


def make_fedavg_params():
    """aggregation_content "parameters" (coala/server/base.py:588-591): the reference's
    federated_averaging_only_params / weighted_sum_only_params (coala/server/strategies.py:32-54, 93-124) on
    the fedavg.npz inputs, plus the zero-weights case of weighted_sum_only_params."""
    from coala.server import strategies
    models = [_seeded_tiny(s) for s in (11, 12, 13)]
    weights = [3, 5, 2]
    avg = strategies.federated_averaging_only_params([copy.deepcopy(m) for m in models], list(weights))
    wsum, total = strategies.weighted_sum_only_params([copy.deepcopy(m) for m in models], list(weights))
    wzero, tz = strategies.weighted_sum_only_params([copy.deepcopy(m) for m in models], [0, 0, 0])
    arrays = {}
    for i, m in enumerate(models):
        for k, v in m.state_dict().items():
            arrays[f"in{i}/{k}"] = v.numpy()
    for tag, mod in (("avg", avg), ("sum", wsum), ("sum0", wzero)):
        for k, v in mod.state_dict().items():
            arrays[f"{tag}/{k}"] = v.detach().numpy()
    arrays["weights"] = np.array(weights, dtype=np.int64)
    arrays["total"] = np.array([total], dtype=np.int64)
    arrays["total0"] = np.array([tz], dtype=np.int64)
    np.savez(os.path.join(HERE, "fedavg_params.npz"), **arrays)
    print("fedavg_params.npz:", len(arrays), "arrays")


def make_hooks():
    from coala.client.base import BaseClient
    from coala.pb import common_pb2 as common_pb
    from coala.protocol import codec

    calls = []

    class _Data:
        def size(self, cid):
            return 37

    class Recording(BaseClient):
        def decompression(self):
            calls.append(["decompression", self.model is not None])

        def pre_train(self):
            calls.append(["pre_train", True])

        def train(self, conf, device="cpu"):
            calls.append(["train", True])
            with torch.no_grad():
                for p in self.model.parameters():
                    p.add_(0.5)

        def post_train(self):
            calls.append(["post_train", True])

        def compression(self):
            calls.append(["compression", self.model is not None])

        def encryption(self):
            calls.append(["encryption", True])

        def post_upload(self):
            calls.append(["post_upload", True])

    conf = SimpleNamespace(track=False, local_test=False, task_id="task0", round_id=3)
    client = Recording("c0", conf, _Data(), None, "cpu")
    model = _seeded_tiny(21)
    req = client.run_train(model, conf)
    content = req.content
    uploaded = codec.unmarshal(content.data)
    same = all(torch.equal(a, b) for a, b in zip(uploaded.state_dict().values(),
                                                 client.model.state_dict().values()))
    doc = {
        "source": "coala/client/base.py:123-159 (run_train), :353-383 (construct_upload_request)",
        "hook_order": [c[0] for c in calls],
        "model_present_at_hook": {c[0]: c[1] for c in calls},
        "task_id": req.task_id, "round_id": req.round_id, "client_id": req.client_id,
        "content_type": int(content.type),
        "DATA_TYPE_PARAMS": int(common_pb.DATA_TYPE_PARAMS),
        "DATA_TYPE_PERFORMANCE": int(common_pb.DATA_TYPE_PERFORMANCE),
        "DATA_TYPE_FEATURE": int(common_pb.DATA_TYPE_FEATURE),
        "data_size": int(content.data_size),
        "upload_is_trained_model": bool(same),
        "upload_type": type(uploaded).__name__,
        "upload_size_mb": client.calculate_model_size(client.model),
    }
    with open(os.path.join(HERE, "hooks.json"), "w") as f:
        json.dump(doc, f, indent=1)
    print("hooks.json:", doc["hook_order"], "type", doc["content_type"], "size", doc["data_size"])

    # identity round trip of the reference's own framing (codec.py:4-9)
    m = _seeded_tiny(5)
    back = codec.unmarshal(codec.marshal(copy.deepcopy(m)))
    assert all(torch.equal(a, b) for a, b in zip(m.state_dict().values(), back.state_dict().values()))


PLUGIN_SIZES = [13, 7, 21]   # client sample counts (FedAvg weights)
PLUGIN_SEED, PLUGIN_NOISE_SEED, PLUGIN_NOISE = 7, 1000, 1e-3
PLUGIN_RATIO, PLUGIN_BITS = 0.05, 8


def plugin_train_step(model, cid_index):
    """The deterministic local 'training' of the fixture (also restated by tests/test_reference_fixture.py):
    every parameter += N(0, 1) * 1e-3 drawn from a CPU generator seeded 1000 + client index."""
    g = torch.Generator().manual_seed(PLUGIN_NOISE_SEED + cid_index)
    with torch.no_grad():
        for p in model.parameters():
            p.add_((torch.randn(p.shape, generator=g) * PLUGIN_NOISE).to(p.device))


def make_plugin_fixture():
    import hashlib

    sys.path.insert(0, REPO)
    from coala.client.base import BaseClient
    from coala.models import simple_cnn
    from coala.protocol import codec
    from coala.server import strategies

    from coala_amd.compression import CompressionClientMixin, UpdateCodec
    from tests.oracle_backend import OracleBackend

    class _Data:
        def size(self, cid):
            return PLUGIN_SIZES[int(cid[1:])]

    class Client(CompressionClientMixin, BaseClient):
        codec_ratio, codec_bits, codec_mode, codec_backend = PLUGIN_RATIO, PLUGIN_BITS, "delta", OracleBackend()

        def train(self, conf, device="cpu"):
            plugin_train_step(self.model, int(self.cid[1:]))

    torch.manual_seed(PLUGIN_SEED)
    g0 = simple_cnn.Model(channels=16, num_classes=10)
    conf = SimpleNamespace(track=False, local_test=False, task_id="task0", round_id=0)
    arrays = {f"global/{k}": v.numpy() for k, v in g0.state_dict().items()}
    ups, weights = [], []
    for i in range(len(PLUGIN_SIZES)):
        c = Client(f"c{i}", conf, _Data(), None, "cpu")
        req = c.run_train(g0, conf)
        data = req.content.data
        arrays[f"upload_bytes/{i}"] = np.frombuffer(data, dtype=np.uint8).copy()
        arrays[f"data_size/{i}"] = np.array([req.content.data_size], np.int64)
        arrays[f"content_type/{i}"] = np.array([int(req.content.type)], np.int64)
        arrays[f"upload_size_mb/{i}"] = np.array([c.calculate_model_size(codec.unmarshal(data))], np.float64)
        ups.append(codec.unmarshal(data))
        weights.append(req.content.data_size)
    # server side: w_global + decode(delta) per upload (oracle), then the reference FedAvg on the CPU
    oc = UpdateCodec(PLUGIN_RATIO, PLUGIN_BITS, "delta", OracleBackend())
    base = oc.snapshot(g0)
    dec = [oc.decode_module(u, g0, base=base) for u in ups]
    for i, m in enumerate(dec):
        h = hashlib.sha256()
        for t in m.state_dict().values():
            h.update(t.contiguous().reshape(-1).view(torch.uint8).numpy().tobytes())
        arrays[f"decoded_sha256/{i}"] = np.frombuffer(h.digest(), dtype=np.uint8).copy()
    avg = strategies.federated_averaging([copy.deepcopy(m) for m in dec], list(weights))
    for k, v in avg.state_dict().items():
        arrays[f"avg/{k}"] = v.numpy()
    arrays["weights"] = np.array(weights, np.int64)
    np.savez_compressed(os.path.join(HERE, "plugin_run_train.npz"), **arrays)
    print("plugin_run_train.npz:", len(arrays), "arrays; upload bytes",
          [int(arrays[f"upload_bytes/{i}"].size) for i in range(len(PLUGIN_SIZES))])


SFL_FEATURE_SHAPE, SFL_SEED, SFL_RATIO, SFL_BITS = (3, 8, 6, 6), 11, 0.05, 8


def sfl_feature():
    """The fixture's cut-layer activation (also restated by tests/test_splitfl_features.py)."""
    g = torch.Generator().manual_seed(SFL_SEED)
    return torch.relu(torch.randn(SFL_FEATURE_SHAPE, generator=g)), torch.tensor([4, 0, 9])


def make_splitfl_fixture():
    """splitFL feature upload through the REAL reference client (splitfl_features.npz): the reference's own
    BaseSFLClient.marshal_data("feature_label") (application/splitFL/client/base_sfl.py:248-257), plain and with
    CompressionClientMixin mixed in (oracle backend). base_sfl.py imports coala.datasets.dataset_util for its
    training data wrapper only; that module (torchvision) is absent here, so a placeholder module stands in for
    it — marshal_data does not touch it. Pinned: the plain upload's dict layout (names, feature, label) and data
    type, and the mixin's upload: its dict layout and the exact bytes of the encoded feature (the carrier's
    COALAQ1 blob); tests/test_splitfl_features.py reproduces both."""
    import importlib.util
    import pickle

    sys.path.insert(0, REPO)
    ds = types.ModuleType("coala.datasets")
    ds.__path__ = []
    du = types.ModuleType("coala.datasets.dataset_util")
    du.TransformDataset = object
    sys.modules.setdefault("coala.datasets", ds)
    sys.modules.setdefault("coala.datasets.dataset_util", du)
    spec = importlib.util.spec_from_file_location(
        "_ref_base_sfl", os.path.join(REF, "application", "splitFL", "client", "base_sfl.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    from coala_amd.compression import CompressionClientMixin
    from tests.oracle_backend import OracleBackend

    class Mixed(CompressionClientMixin, mod.BaseSFLClient):
        codec_features, codec_ratio, codec_bits, codec_backend = True, SFL_RATIO, SFL_BITS, OracleBackend()

    x, lab = sfl_feature()
    arrays = {"feature": x.numpy(), "label": lab.numpy()}
    for key, cls in (("plain", mod.BaseSFLClient), ("mixed", Mixed)):
        c = cls.__new__(cls)  # marshal_data reads feature / label only (no dataset, no config)
        c.feature, c.label, c.model = x.clone(), lab.clone(), None
        data, typ = c.marshal_data("feature_label")
        arrays[f"{key}/type"] = np.array([int(typ)], np.int64)
        d = pickle.loads(data)  # (bytes this script just wrote)
        arrays[f"{key}/names"] = np.array(d["name"])
        assert torch.equal(d["content"][1], lab)
        if key == "mixed":  # the carrier's COALAQ1 blob (the label's pickle embeds a storage address)
            arrays["mixed/carrier"] = np.frombuffer(d["content"][0].to_bytes(), dtype=np.uint8).copy()
    np.savez_compressed(os.path.join(HERE, "splitfl_features.npz"), **arrays)
    print("splitfl_features.npz:", {k: v.shape for k, v in arrays.items()})


if __name__ == "__main__":
    if not os.environ.get("PYTHONDONTWRITEBYTECODE"):
        sys.exit("run with PYTHONDONTWRITEBYTECODE=1 so nothing is written into /root/reference")
    sys.dont_write_bytecode = True
    _stub_coala()
    parts = {"layouts": make_layouts, "fedavg": make_fedavg, "fedavg_params": make_fedavg_params,
             "hooks": make_hooks, "plugin": make_plugin_fixture, "splitfl": make_splitfl_fixture}
    for name in (sys.argv[1:] or list(parts)):  # e.g. `make_golden.py fedavg_params`: that fixture only
        parts[name]()
