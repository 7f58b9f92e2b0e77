"""Tensor layouts of the reference models the benchmarks synthesise updates for.

The JSON files are fixtures captured from the reference model definitions by
tests/golden/make_golden.py (see its docstring for the source file:line of each); no reference code is
needed at run time.
"""
import json
import os

_DIR = os.path.dirname(os.path.abspath(__file__))

SPLITFL = [f"{m}_cut{c}" for m in ("resnet18_split", "resnet50_split", "simple_cnn_split") for c in (1, 2, 4)]

# splitFL feature uploads: the client-side activations a splitFL client sends every
# step as {"content": [feature, label], "name": [...]} (application/splitFL/client/base_sfl.py:249-257),
# batch 32; one fp32 tensor each (the int64 label rides raw)
FEATURES = {"sfl_feature_64x32x32": [32, 64, 32, 32],
            "sfl_feature_256x32x32": [32, 256, 32, 32],
            "sfl_feature_128x16x16": [32, 128, 16, 16]}


def names():
    return sorted(f[:-5] for f in os.listdir(_DIR) if f.endswith(".json")) + sorted(FEATURES)


def load(name):
    if name in FEATURES:
        shape = FEATURES[name]
        n = 1
        for d in shape:
            n *= d
        return {"model": name, "source": "application/splitFL/client/base_sfl.py:249-257 feature upload",
                "n_entries": 1, "n_float32_entries": 1, "n_float32_elements": n,
                "entries": [{"name": "feature", "shape": list(shape), "dtype": "float32"}]}
    with open(os.path.join(_DIR, name + ".json")) as f:
        return json.load(f)


def fp32_sizes(name):
    """Element counts of the fp32 entries, in state_dict order (= the codec's segments)."""
    out = []
    for e in load(name)["entries"]:
        if e["dtype"] == "float32":
            n = 1
            for d in e["shape"]:
                n *= d
            out.append(n)
    return out


def build_module(name, seed=0, device="cpu"):
    """An nn.Module whose state_dict has exactly the layout of reference model `name` (same names,
    shapes, dtypes, order): fp32 weights as Parameters, BatchNorm running stats and int64 counters as
    buffers. Values are seeded random (no checkpoints offline)."""
    import torch
    from torch import nn

    g = torch.Generator().manual_seed(seed)
    root = nn.Module()
    for e in load(name)["entries"]:
        path = e["name"].split(".")
        mod = root
        for p in path[:-1]:
            if not hasattr(mod, p):
                mod.add_module(p, nn.Module())
            mod = getattr(mod, p)
        dt = getattr(torch, e["dtype"])
        leaf = path[-1]
        if dt == torch.float32:
            t = torch.randn(e["shape"], generator=g) * 0.05
            if leaf in ("running_mean", "running_var"):
                mod.register_buffer(leaf, t.abs() if leaf == "running_var" else t)
            else:
                mod.register_parameter(leaf, nn.Parameter(t))
        else:
            mod.register_buffer(leaf, torch.zeros(e["shape"], dtype=dt))
    return root.to(device)
