"""Per-call host timing of the hooks' decode path on the GPU (diagnostics for bench.py's 'plugin' extra):
decode_module with the previous result kept alive (as a server's uploaded_models dict keeps them) vs
discarded at once, and decode_state alone; per-call times show where the variance comes from."""
import sys
import time

import torch

sys.path.insert(0, ".")
from coala_amd.compression import UpdateCodec  # noqa: E402
from coala_amd.layouts import build_module  # noqa: E402

dev = torch.device("cuda", 0)
m = build_module("resnet50_tv", seed=1, device=dev)
g = build_module("resnet50_tv", seed=2, device=dev)
codec = UpdateCodec(0.01, 8, "delta")
base = codec.snapshot(g)
up = codec.encode(m.state_dict(), base=base)
for _ in range(3):
    codec.decode_module(up, g, base=base)
torch.cuda.synchronize()


def per_call(fn, n=20):
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ts.append((time.perf_counter() - t0) * 1e3)
    return " ".join(f"{t:.2f}" for t in ts)


keep = []
print("keep   ", per_call(lambda: keep.append(codec.decode_module(up, g, base=base))), flush=True)
keep.clear()
print("discard", per_call(lambda: codec.decode_module(up, g, base=base)), flush=True)
print("state  ", per_call(lambda: codec.decode_state(up, base=base)), flush=True)
print("encode ", per_call(lambda: codec.encode(m.state_dict(), base=base)), flush=True)
