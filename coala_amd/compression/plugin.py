"""COALA compression plugin surface: client/server hook mixins with the reference's exact signatures.

The reference exposes compression only as no-op hooks that users override in subclasses
(/root/reference/docs/en/tutorials/customize_server_and_client.md:57-58,72-73,168-169):

    BaseClient.decompression(self) -> None          coala/client/base.py:203-205   (called :141)
    BaseClient.compression(self) -> None            coala/client/base.py:330-332   (called :153)
    BaseServer.compression(self) -> None            coala/server/base.py:347-349   (called :196)
    BaseServer.decompression(self, model) -> model  coala/server/base.py:558-560   (called :376,
                                                    server/service.py:106,125)
    plus BaseServer.aggregation() / aggregation_test() (server/base.py:562-571, test path :265-267), which
    the server mixin wraps to put the real global model back after a compressed download.

Usage (drop-in, nothing else in COALA changes):

    from coala.client import BaseClient
    from coala_amd.compression import CompressionClientMixin, CompressionServerMixin
    class Client(CompressionClientMixin, BaseClient): pass
    class Server(CompressionServerMixin, BaseServer): pass
    coala.register_client(Client); coala.register_server(Server)   # coordinator.py:519-536

Behaviour:
  * client decompression(): runs right after set_model (base.py:138,141) — snapshots w_global for delta
    mode; tolerates self.model being None (application/MAS/fl_client.py:23-26 pattern).
  * client compression(): encodes the trained model (still on the training device, base.py:144-153) and
    leaves a CompressedUpdate carrier in self.model, which construct_upload_request deep-copies and
    pickles into UploadContent.data (base.py:363). post_upload() puts the trained module back so the
    next round's set_model (base.py:197-201) works.
  * calculate_model_size(): reports the real payload size for a carrier (base.py:155, 474-487).
  * server decompression(model): CompressedUpdate -> a NEW nn.Module (never aliases self.model, which
    aggregation overwrites, base.py:571) built on the pre-aggregation global model (delta mode: w_global
    + decoded delta, fused in the decode kernel); anything else (plain modules, splitFL feature dicts,
    server/service.py:124-131) passes through unchanged. Safe to call from several threads
    (server/service.py:74 spawns one per upload).
  * splitFL cut-layer features (opt-in, `codec_features = True`): the splitFL client uploads its
    features as `{"content": [feature, label], "name": [...]}` through marshal_data("feature_label")
    (application/splitFL/client/base_sfl.py:248-257) and the server reads them back through
    decompression(codec.unmarshal(data)) (application/splitFL/server/base_sfl.py:207-209). With the flag,
    the client mixin's marshal_data encodes the feature tensor on its training device (weights mode, no
    dense .cpu() copy) into a CompressedUpdate that stands where the tensor stood, and the server mixin's
    decompression decodes it back to a dense tensor of the same shape; labels and other entries travel
    unchanged. Without the flag (default) the dict passes through exactly as before.
  * download direction (opt-in, `codec_download = True`): server compression()
    encodes the global model once per round into a CompressedModel (download.py) that stands where the
    global module stood during distribution; aggregation() restores the real module first. Client
    decompression() turns a received CompressedModel into a real module (later rounds decode inside
    set_model's load_state_dict). Delta-mode uploads are decoded against the server's reconstruction of
    its own download, which is bit-identical to what the clients decoded.
"""
import copy
import pickle
import threading

from torch import nn

from .codec import CompressedUpdate, UpdateCodec
from .download import CompressedModel, compress_model

DATA_TYPE_FEATURE = 2  # coala/pb/common.proto: DataType.DATA_TYPE_FEATURE (protos/coala/pb/common.proto:26)
FEATURE_CONTENT = "feature_label"  # application/splitFL/client/base_sfl.py:252


def _marshal(obj):
    """The reference's codec.marshal (coala/protocol/codec.py:4-5) when COALA is installed, else its
    restatement (pickle.dumps)."""
    try:
        from coala.protocol.codec import marshal
    except ImportError:
        marshal = pickle.dumps
    return marshal(obj)


def _data_type_feature():
    try:
        from coala.pb import common_pb2
        return common_pb2.DATA_TYPE_FEATURE
    except ImportError:
        return DATA_TYPE_FEATURE

EQUAL_AVERAGE = "equal"                     # coala/server/base.py:37
TRAIN_UPLOAD_COMPRESSION_RATIO = "train_upload_compression_ratio"  # tracked next to metric.TRAIN_UPLOAD_SIZE
AGGREGATION_CONTENT_PARAMS = "parameters"   # coala/server/base.py:40


def _bit_to_megabyte(bits):
    # same conversion as the reference tracker (coala/tracking/evaluation.py:16-17)
    return bits / (8 * 1024 * 1024)


class _CodecOwner:
    codec_ratio = 0.01
    codec_bits = 8
    codec_mode = "delta"
    codec_backend = None
    codec_recycle = True  # decoded modules are reused once released (UpdateCodec recycle; False: never)

    def _codec(self):
        c = self.__dict__.get("_update_codec")
        if c is None:
            c = UpdateCodec(self.codec_ratio, self.codec_bits, self.codec_mode, self.codec_backend,
                            recycle=self.codec_recycle)
            self.__dict__["_update_codec"] = c
        return c


class CompressionClientMixin(_CodecOwner):
    """Mix in before coala's BaseClient: `class Client(CompressionClientMixin, BaseClient)`."""

    codec_features = False        # splitFL: compress the uploaded cut-layer features as well
    codec_feature_ratio = None    # their top-k ratio (None: codec_ratio)
    codec_feature_bits = None     # their code width (None: codec_bits)

    def _feature_codec(self):
        c = self.__dict__.get("_feature_update_codec")
        if c is None:
            ratio = self.codec_feature_ratio if self.codec_feature_ratio is not None else self.codec_ratio
            bits = self.codec_feature_bits if self.codec_feature_bits is not None else self.codec_bits
            c = UpdateCodec(ratio, bits, "weights", self.codec_backend)
            self.__dict__["_feature_update_codec"] = c
        return c

    def marshal_data(self, content):
        """splitFL's upload serialiser (application/splitFL/client/base_sfl.py:248-257) with the feature
        tensor encoded: the same dict, the same DATA_TYPE_FEATURE, a CompressedUpdate where the dense
        `feature.detach().cpu()` was. Model uploads ("model") and uncompressed runs go to the parent."""
        feature = getattr(self, "feature", None)
        parent = getattr(super(), "marshal_data", None)
        if content != FEATURE_CONTENT or not self.codec_features or feature is None:
            if parent is None:
                raise AttributeError("marshal_data: no parent implementation (not a splitFL client)")
            return parent(content)
        carrier = self._feature_codec().encode({"feature": feature.detach()})
        customize_dict = {"content": [carrier, copy.deepcopy(self.label)], "name": ["feature", "label"]}
        return _marshal(customize_dict), _data_type_feature()

    def set_model(self, model):
        # a compressed download decodes with this client's codec backend (inside the reference's
        # set_model: load_state_dict(model.state_dict()), client/base.py:197-201)
        if isinstance(model, CompressedModel):
            model.bind(self._codec().backend)
        parent = getattr(super(), "set_model", None)
        if parent is not None:
            return parent(model)
        self.model = model

    def decompression(self):
        if getattr(self, "model", None) is None:
            return
        if isinstance(self.model, CompressedModel):  # compressed download, first round (set_model deepcopy)
            self.model = self.model.materialize()
        if isinstance(self.model, nn.Module) and self._codec().mode == "delta":
            self._codec_base = self._codec().snapshot(self.model)

    def compression(self):
        model = getattr(self, "model", None)
        if model is None or not isinstance(model, nn.Module):
            return
        codec = self._codec()
        base = getattr(self, "_codec_base", None) if codec.mode == "delta" else None
        update = codec.encode_module(model, base=base)
        self._codec_trained_model = model
        self.model = update
        # §8(f) 3: the compression ratio next to TRAIN_UPLOAD_SIZE (client/base.py:155); an unknown
        # metric name lands in the tracker's "extra" dict (coala/tracking/metric.py:64-73)
        track = getattr(self, "track", None)
        if track is not None and getattr(getattr(self, "conf", None), "track", True):
            track(TRAIN_UPLOAD_COMPRESSION_RATIO, update.compression_ratio)

    def post_upload(self):
        trained = self.__dict__.pop("_codec_trained_model", None)
        if trained is not None:
            self.model = trained
        parent = getattr(super(), "post_upload", None)
        if parent is not None:
            parent()

    def calculate_model_size(self, model, param_size=32):
        # real payload sizes for the carriers: the upload (client/base.py:155) and a compressed
        # download (TRAIN/TEST_DOWNLOAD_SIZE, client/base.py:139, :178)
        if isinstance(model, (CompressedUpdate, CompressedModel)):
            return _bit_to_megabyte(model.nbytes * 8)
        parent = getattr(super(), "calculate_model_size", None)
        if parent is not None:
            return parent(model, param_size)
        return _bit_to_megabyte(sum(p.numel() for p in model.parameters()) * param_size)


def reduce_models(params_only=False):
    """The reference's reduce_models / reduce_models_only_params (coala/distributed/distributed.py:42-57,
    60-74) when COALA is installed, else their restatements (coala_amd/fl/distributed.py)."""
    name = "reduce_models_only_params" if params_only else "reduce_models"
    try:
        from coala.distributed import distributed as mod
    except ImportError:
        from ..fl import distributed as mod
    return getattr(mod, name)


class CompressionServerMixin(_CodecOwner):
    """Mix in before coala's BaseServer: `class Server(CompressionServerMixin, BaseServer)`."""

    codec_download = False        # compress the distributed global model (download direction)
    codec_download_ratio = 1.0    # dense: indices implied (wire.py "dense")
    codec_download_bits = 8

    def _download_codec(self):
        c = self.__dict__.get("_download_update_codec")
        if c is None:
            c = UpdateCodec(self.codec_download_ratio, self.codec_download_bits, "weights", self.codec_backend)
            self.__dict__["_download_update_codec"] = c
        return c

    def _real_global(self):
        """The global nn.Module, also while a CompressedModel stands in for it during distribution."""
        g = self.__dict__.get("_codec_global")
        return g if g is not None else self.model

    @staticmethod
    def _stamp(module, state):
        # storage address + version counter (state_dict() returns fresh detached views each call, which
        # share the parameter's storage and version counter)
        return (id(module), tuple((t.data_ptr(), t._version) for t in state.values()))

    def _restore_global(self):
        g = self.__dict__.pop("_codec_global", None)
        if g is not None:
            self.model = g

    def compression(self):
        if not self.codec_download:
            parent = getattr(super(), "compression", None)
            return parent() if parent is not None else None
        self._restore_global()
        g = self.model
        carrier = compress_model(g, self._download_codec())
        # what every client will decode: base of their delta-mode uploads (kept until the global changes)
        recon = self._codec().snapshot(carrier.decoded_state())
        self.__dict__["_codec_recon"] = (self._stamp(g, g.state_dict()), recon)
        self.__dict__["_codec_global"] = g
        self.model = carrier

    def aggregation(self):
        self._restore_global()
        parent = getattr(super(), "aggregation", None)
        return parent() if parent is not None else None

    def aggregation_test(self):
        self._restore_global()
        parent = getattr(super(), "aggregation_test", None)
        return parent() if parent is not None else None

    def _global_snapshot(self):
        """Flat fp32 copy of the global model the clients started from: the reconstruction of the
        compressed download when there was one, else the global model itself (rebuilt only when its
        tensors changed)."""
        lock = self.__dict__.setdefault("_codec_lock", threading.Lock())
        with lock:
            g = self._real_global()
            state = g.state_dict()
            stamp = self._stamp(g, state)
            recon = self.__dict__.get("_codec_recon")
            if recon is not None and recon[0] == stamp:
                return recon[1]
            snap = self.__dict__.get("_codec_snapshot")
            if snap is None or snap[0] != stamp:
                snap = (stamp, self._codec().snapshot(state))
                self.__dict__["_codec_snapshot"] = snap
            return snap[1]

    codec_fused_aggregate = False

    def _decode_upload(self, model):
        base = self._global_snapshot() if model.header["mode"] == "delta" else None
        return self._codec().decode_module(model, self._real_global(), base=base)

    def decompression(self, model):
        if isinstance(model, CompressedUpdate):
            if self.codec_fused_aggregate:
                return model  # decoded together with the other uploads in aggregate()
            return self._decode_upload(model)
        if isinstance(model, dict) and isinstance(model.get("content"), list):
            return self._decode_features(model)
        return model

    def _decode_features(self, upload):
        """A splitFL feature upload (application/splitFL/server/base_sfl.py:207-209): every CompressedUpdate
        in "content" (the client mixin's encoded features) back to a dense tensor of its shape on the
        codec's device; everything else unchanged. A new dict; the received one is not modified."""
        content = upload["content"]
        if not any(isinstance(c, CompressedUpdate) for c in content):
            return upload
        codec = self._codec()
        out = dict(upload)
        out["content"] = [self._decode_feature(codec, c) if isinstance(c, CompressedUpdate) else c for c in content]
        return out

    @staticmethod
    def _decode_feature(codec, carrier):
        entries = carrier.header["entries"]
        if carrier.header["mode"] != "weights" or len(entries) != 1:
            raise ValueError("a splitFL feature carrier holds one tensor in weights mode")
        return codec.decode_state(carrier)[entries[0]["name"]]

    def aggregate(self, models, weights):
        """server/base.py:573-601 with the fused decode: FedAvg in one kernel (single process), or in a
        multi-GPU run the per-rank weighted sum in one kernel followed by the reference's reduce_models
        (:595-598), exactly the two calls the reference makes on decoded modules."""
        conf = getattr(self, "conf", None)
        server_conf = getattr(conf, "server", None)
        distributed = bool(getattr(conf, "is_distributed", False))
        params_only = getattr(server_conf, "aggregation_content", "all") == AGGREGATION_CONTENT_PARAMS
        fusable = self.codec_fused_aggregate and models and all(isinstance(m, CompressedUpdate) for m in models)
        if fusable:
            if getattr(server_conf, "aggregation_strategy", None) == EQUAL_AVERAGE:
                weights = [1 for _ in models]
            h0 = models[0].header
            if all(m.header["entries"] == h0["entries"] and
                   (m.header["ratio"], m.header["bits"], m.header["mode"]) == (h0["ratio"], h0["bits"], h0["mode"])
                   for m in models):
                base = self._global_snapshot() if h0["mode"] == "delta" else None
                codec = self._codec()
                dev = codec.backend.default_device()
                if distributed:
                    import torch
                    import torch.distributed as dist
                    dist.barrier()
                    sample_sum = sum(weights)  # weighted_sum returns the caller's sum (0 stays 0)
                    model = codec.aggregate(models, weights, self._real_global(), base=base, mode="sum", device=dev,
                                            params_only=params_only)
                    reduce_models(params_only)(model, torch.tensor(sample_sum).to(getattr(conf, "device", dev)))
                    return model
                mode = "div" if dev.type == "cpu" else "recip"  # torch's division semantics on that device
                return codec.aggregate(models, weights, self._real_global(), base=base, mode=mode, device=dev,
                                       params_only=params_only)
        models = [self._decode_upload(m) if isinstance(m, CompressedUpdate) else m for m in models]
        parent = getattr(super(), "aggregate", None)
        if parent is not None:
            return parent(models, weights)
        from ..fl.strategies import federated_averaging, federated_averaging_only_params
        return (federated_averaging_only_params if params_only else federated_averaging)(models, weights)
