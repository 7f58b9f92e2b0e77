"""Loopback federated-learning harness: the minimum of COALA's client/server loop the codec needs,
restated (not imported: the reference cannot travel to the GPU box) so the plugin can be exercised
end to end. Semantics are pinned against the reference by tests/golden/{hooks.json,fedavg.npz}."""
from .loop import LoopbackClient, LoopbackServer, marshal, unmarshal
from .strategies import federated_averaging, weighted_sum

__all__ = ["LoopbackClient", "LoopbackServer", "marshal", "unmarshal", "federated_averaging", "weighted_sum"]
