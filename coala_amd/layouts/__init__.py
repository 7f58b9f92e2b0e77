"""Tensor layouts of the reference models the benchmarks synthesise updates for.

The JSON files are fixtures captured from the reference model definitions by
tests/golden/make_golden.py (see its docstring for the source file:line of each); no reference code is
needed at run time.
"""
import json
import os

_DIR = os.path.dirname(os.path.abspath(__file__))

SPLITFL = [f"{m}_cut{c}" for m in ("resnet18_split", "resnet50_split", "simple_cnn_split") for c in (1, 2, 4)]


def names():
    return sorted(f[:-5] for f in os.listdir(_DIR) if f.endswith(".json"))


def load(name):
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
