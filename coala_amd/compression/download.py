"""Download direction: the server compresses the global model once per round, clients
decode it.

The reference calls `BaseServer.compression()` right before distribution (coala/server/base.py:196 in
train(), :265 in test_in_client()) and `BaseClient.decompression()` right after `set_model`
(coala/client/base.py:138-141; docstring :204: "when the model is compressed in the server"). Remote
distribution pickles `self.model` once per selected client (`codec.marshal(self.model)`,
server/base.py:397); local distribution hands `self.model` to `client.run_train` (:373).

So the carrier the server distributes has to stand where the global nn.Module stood:

  * `CompressedModel` is an nn.Module holding a weight-less skeleton of the architecture (parameters and
    persistent buffers on the meta device) plus a weights-mode `CompressedUpdate`. Its `state_dict()`
    decodes (HIP kernels) into a fresh state, so the reference client's `set_model`
    (`self.model.load_state_dict(model.state_dict())`, client/base.py:197-201) just works; the first-round
    path (`copy.deepcopy(model)`) leaves a carrier in the client, which the client mixin's
    `decompression()` turns into a real module.
  * It pickles to the skeleton plus the COALAQ1 blob, serialised once and cached: the per-client
    `codec.marshal(self.model)` of remote distribution (server/base.py:397) re-sends bytes instead of
    re-encoding (the "hoisting" of §8(f) 2).
  * Default download codec: ratio 1, 8 bits — dense per-tensor min/max codes with the index list implied
    (wire.py "dense"), ≈ 4x smaller than fp32. bits 32 at ratio 1 is lossless.
  * The server keeps the real global module for aggregation and testing, and decodes its own carrier
    once: the reconstruction clients see is bit-identical (same kernels, same spec), so delta-mode
    uploads are decoded against exactly the base the client encoded them against.
"""
import copy
import pickle
from collections import OrderedDict

import torch
from torch import nn

from .codec import CompressedUpdate, UpdateCodec, module_with_state


def skeleton_of(module):
    """Deep copy of `module` whose state_dict tensors are meta tensors (shape/dtype only). Tensors that
    are not in the state_dict (non-persistent buffers) are copied for real: they never travel otherwise."""
    state = module.state_dict(keep_vars=True)
    memo = {}
    for t in state.values():
        if isinstance(t, nn.Parameter):
            memo[id(t)] = nn.Parameter(torch.empty(t.shape, dtype=t.dtype, device="meta"),
                                       requires_grad=t.requires_grad)
        elif isinstance(t, torch.Tensor):
            memo[id(t)] = torch.empty(t.shape, dtype=t.dtype, device="meta")
    return copy.deepcopy(module, memo)


def _rebuild(skeleton_bytes, blob):
    skel = pickle.loads(skeleton_bytes)  # the reference unpickles the whole model here (protocol/codec.py:8-9)
    return CompressedModel(skel, CompressedUpdate.from_bytes(blob), blob=blob, skeleton_bytes=skeleton_bytes)


class CompressedModel(nn.Module):
    """A compressed global model that stands in for the nn.Module the server distributes.

    Args:
        skeleton: the architecture with meta-device state (skeleton_of()).
        update:   weights-mode CompressedUpdate of the full state.
        codec:    decoder (its backend decides the device; default: the HIP codec on the current GPU).
    """

    def __init__(self, skeleton, update, codec=None, blob=None, skeleton_bytes=None):
        super().__init__()
        if update.header["mode"] != "weights":
            raise ValueError("a distributed model is coded in weights mode")
        self.__dict__["_skeleton"] = skeleton   # kept out of nn.Module bookkeeping (never trained)
        self.__dict__["_update"] = update
        self.__dict__["_codec"] = codec
        self.__dict__["_blob"] = blob
        self.__dict__["_skeleton_bytes"] = skeleton_bytes

    @property
    def update(self):
        return self._update

    @property
    def nbytes(self):
        return self._update.nbytes

    def bind(self, backend):
        """Decode with `backend` (the receiving side's codec backend; default: the HIP codec)."""
        h = self._update.header
        self.__dict__["_codec"] = UpdateCodec(h["ratio"], h["bits"], "weights", backend)
        return self

    def _decoder(self):
        c = self._codec
        if c is None:
            h = self._update.header
            c = UpdateCodec(h["ratio"], h["bits"], "weights")
            self.__dict__["_codec"] = c
        return c

    def decoded_state(self):
        """Decode into a fresh OrderedDict (fp32 entries: views into one flat buffer)."""
        return self._decoder().decode_state(self._update)

    def state_dict(self, *args, destination=None, prefix="", keep_vars=False):
        state = self.decoded_state()
        out = OrderedDict() if destination is None else destination
        for k, v in state.items():
            out[prefix + k] = v
        return out

    def materialize(self):
        """A real nn.Module (the skeleton's architecture) holding the decoded state."""
        return module_with_state(self._skeleton, self.decoded_state())

    def forward(self, *args, **kwargs):
        raise RuntimeError("CompressedModel is a transport carrier: call materialize() (the client mixin's "
                           "decompression() does) before using it as a model")

    # -- transport --------------------------------------------------------------------------------
    def __reduce__(self):
        if self._blob is None:
            self.__dict__["_blob"] = self._update.to_bytes()
        if self._skeleton_bytes is None:
            self.__dict__["_skeleton_bytes"] = pickle.dumps(self._skeleton)
        return (_rebuild, (self._skeleton_bytes, self._blob))

    def __deepcopy__(self, memo):
        # client set_model's first-round copy.deepcopy(model) (client/base.py:201): share the immutable
        # encoded payload and skeleton, keep the decoder
        return CompressedModel(self._skeleton, self._update, codec=self._codec, blob=self._blob,
                               skeleton_bytes=self._skeleton_bytes)

    def __repr__(self):
        return f"CompressedModel({self._skeleton.__class__.__name__}, {self._update!r})"


def compress_model(module, codec):
    """Global nn.Module -> CompressedModel (weights mode, `codec`'s ratio/bits)."""
    if codec.mode != "weights":
        raise ValueError("download codec must be in weights mode")
    update = codec.encode(module.state_dict(), device=codec.backend.default_device())
    return CompressedModel(skeleton_of(module), update, codec=codec)
