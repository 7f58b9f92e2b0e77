"""Loopback client/server with the reference's hook order and upload framing.

LoopbackClient.run_train mirrors /root/reference/coala/client/base.py:123-159 (set_model :191-201,
download size :139, decompression :141, pre_train/train/post_train :143-145, compression :153, upload
size :155, encryption :157, upload :159 -> construct_upload_request :353-383 with
codec.marshal(deepcopy(model)) and DATA_TYPE_PARAMS = 0). track() records into `metrics` the way the
reference's ClientMetric does (known names as keys, the rest under "extra": tracking/metric.py:64-73). LoopbackServer.round mirrors distribution_to_train_locally
(/root/reference/coala/server/base.py:363-381: decompression(codec.unmarshal(data)) per client) and
aggregation (:562-571 -> strategies.federated_averaging). The hook order is checked against
tests/golden/hooks.json, captured from the reference itself.
"""
import copy
import pickle
from dataclasses import dataclass, field

import torch

from .strategies import federated_averaging, federated_averaging_only_params

DATA_TYPE_PARAMS = 0  # coala/pb common.proto DataType (tests/golden/hooks.json)


def marshal(obj):      # coala/protocol/codec.py:4-5
    return pickle.dumps(obj)


def unmarshal(data):   # coala/protocol/codec.py:8-9
    return pickle.loads(data)


@dataclass
class UploadContent:
    data: bytes
    type: int
    data_size: int


@dataclass
class UploadRequest:
    task_id: str
    round_id: int
    client_id: str
    content: UploadContent
    trace: list = field(default_factory=list)


class LoopbackClient:
    """Client whose local 'training' is a deterministic synthetic step (no datasets offline)."""

    def __init__(self, cid, datasize, device="cpu", step_seed=0, step_scale=1e-3):
        self.cid = cid
        self._datasize = datasize
        self.device = device
        self.model = None
        self.step_seed = step_seed
        self.step_scale = step_scale
        self.trace = []
        self.upload_sizes = []
        self.download_sizes = []
        self.metrics = {"extra": {}}

    # hook points (no-ops, as in the reference)
    def decompression(self):
        pass

    def pre_train(self):
        pass

    def post_train(self):
        pass

    def compression(self):
        pass

    def encryption(self):
        pass

    def post_upload(self):
        pass

    def set_model(self, model):  # client/base.py:191-201
        if self.model is not None:
            self.model.load_state_dict(model.state_dict())
        else:
            self.model = copy.deepcopy(model)

    def train(self, round_id):
        g = torch.Generator(device="cpu")
        g.manual_seed(self.step_seed * 1000 + round_id)
        self.model.to(self.device)
        with torch.no_grad():
            for p in self.model.parameters():
                p.add_((torch.randn(p.shape, generator=g) * self.step_scale).to(p.device))
            for name, b in self.model.named_buffers():
                if b.dtype == torch.int64:
                    b.add_(1)

    def calculate_model_size(self, model, param_size=32):
        return sum(p.numel() for p in model.parameters()) * param_size / (8 * 1024 * 1024)

    KNOWN_METRICS = ("train_download_size", "train_upload_size", "train_time", "train_metric")

    def track(self, metric_name, value):  # client/base.py:447-457 -> ClientMetric.add (metric.py:64-73)
        if metric_name in self.KNOWN_METRICS:
            self.metrics[metric_name] = value
        else:
            self.metrics["extra"][metric_name] = value

    def _t(self, name):
        self.trace.append(name)

    def run_train(self, model, round_id, task_id="task"):
        self.set_model(model)
        self.download_sizes.append(self.calculate_model_size(model))
        self.track("train_download_size", self.download_sizes[-1])
        self._t("decompression"); self.decompression()
        self._t("pre_train"); self.pre_train()
        self._t("train"); self.train(round_id)
        self._t("post_train"); self.post_train()
        self._t("compression"); self.compression()
        self.upload_sizes.append(self.calculate_model_size(self.model))
        self.track("train_upload_size", self.upload_sizes[-1])
        self._t("encryption"); self.encryption()
        data = marshal(copy.deepcopy(self.model))
        req = UploadRequest(task_id, round_id, self.cid, UploadContent(data, DATA_TYPE_PARAMS, self._datasize))
        self._t("post_upload"); self.post_upload()
        return req


class LoopbackServer:
    """remote=True distributes the way remote training does: `codec.marshal(self.model)` per client
    (server/base.py:397) and the client unpickles it (client/service.py), instead of handing the object
    over as local training does (server/base.py:373)."""

    def __init__(self, model, clients, remote=False):
        self.model = model
        self.clients = clients
        self.remote = remote
        self.uploaded = {}
        self.weights = {}
        self.download_sizes = []

    def compression(self):
        pass

    def decompression(self, model):
        return model

    def round(self, round_id):  # server/base.py:190-201: compression -> distribution -> aggregation
        self.compression()
        self.distribution_to_train(round_id)
        self.aggregation()
        return self.model

    def distribution_to_train(self, round_id):  # server/base.py:363-381 (local) / :383-410 (remote)
        self.uploaded, self.weights = {}, {}
        for c in self.clients:
            if self.remote:
                data = marshal(self.model)
                self.download_sizes.append(len(data))
                sent = unmarshal(data)
            else:
                sent = self.model
            req = c.run_train(sent, round_id)
            model = self.decompression(unmarshal(req.content.data))
            self.uploaded[c.cid] = model
            self.weights[c.cid] = req.content.data_size

    def aggregation(self):  # server/base.py:562-571
        agg = self.aggregate(list(self.uploaded.values()), list(self.weights.values()))
        self.model.load_state_dict(agg.state_dict())  # set_model(load_dict=True), server/base.py:571

    def aggregate(self, models, weights):  # server/base.py:573-601, non-distributed branch
        server = getattr(getattr(self, "conf", None), "server", None)
        if getattr(server, "aggregation_content", "all") == "parameters":  # base.py:588-591
            return federated_averaging_only_params(models, weights)
        return federated_averaging(models, weights)
