"""Host-path breakdown of the hooks on the GPU (one ResNet-50 client, delta mode): UpdateCodec.encode_module
of the trained module in place (client compression()) and decode_module into a new module on w_global
(server decompression(model)), as bench.py's 'plugin' extra runs them. Prints the median per-call time of
each host step (each call synchronised, like the bench), then cProfile's top functions by own time.

    python tools/plugin_profile.py [steps]
"""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from coala_amd.compression import UpdateCodec  # noqa: E402
from coala_amd.compression import codec as C  # noqa: E402
from coala_amd.layouts import build_module  # noqa: E402


def med(fn, n, sync=True):
    """sync True: until the GPU is done; False: the call alone; "host": until the call returns, then the GPU
    drained outside the timing (the host cost of a call that enqueues work)."""
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        if sync is True:
            torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
        if sync == "host":
            torch.cuda.synchronize()
    ts.sort()
    return ts[len(ts) // 2]


def main(steps=50):
    dev = torch.device("cuda", 0)
    m = build_module("resnet50_tv", seed=1, device=dev)
    g = build_module("resnet50_tv", seed=2, device=dev)
    codec = UpdateCodec(0.01, 8, "delta")
    base = codec.snapshot(g)
    for _ in range(5):
        up = codec.encode_module(m, base=base)
        codec.decode_module(up, g, base=base)
    torch.cuda.synchronize()
    names, ts, walk = C._module_walk(m)
    d, segs = C._layout_walk(names, ts, walk)
    L, ptrs = d.L, d.seg_ptrs
    plan = codec.plan_for(L.sizes_key, dev)
    ws = codec._workspace(plan)
    st = codec.decode_state(up, base=base)
    rows = [
        ("compression: encode_module (total)", lambda: codec.encode_module(m, base=base), True),
        ("  module_tensors", lambda: C.module_tensors(m), False),
        ("  describe_tensors (layout + raw snapshot)", lambda: C.describe_tensors(names, ts), False),
        ("  state_dict() (what round 2 walked)", lambda: m.state_dict(), False),
        ("  host: encode_module returns", lambda: codec.encode_module(m, base=base), "host"),
        ("  host: _module_walk", lambda: C._module_walk(m), "host"),
        ("  host: _layout_walk", lambda: C._layout_walk(names, ts, walk), "host"),
        ("  host: _raw_snapshot (gather launch)", lambda: C._raw_snapshot(d, ts, codec.backend.gather_scalars),
         "host"),
        ("  host: plan.encode_segments", lambda: plan.encode_segments(segs, base=base.flat, workspace=ws,
                                                                      checked=True, ptrs=ptrs), "host"),
        ("  host: empty_encoded", lambda: plan.empty_encoded(), "host"),
        ("decompression: decode_module (total)", lambda: codec.decode_module(up, g, base=base), True),
        ("  decode_state", lambda: codec.decode_state(up, base=base), True),
        ("  module_with_state", lambda: C.module_with_state(g, st), False),
        ("empty sync", lambda: None, True),
    ]
    for name, fn, sync in rows:
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        print(f"{name:48s} {med(fn, steps, sync):.4f} ms (median of {steps})", flush=True)
    import gc
    import pickle
    blob = pickle.dumps(up)
    up_r = pickle.loads(blob)
    for name, fn in (("pickle.dumps (fresh pack)", lambda: pickle.dumps(C.CompressedUpdate(up.header, up.encoded, up.raw))),
                     ("pickle.loads", lambda: pickle.loads(blob)),
                     ("decode_module of the unpickled update", lambda: codec.decode_module(up_r, g, base=base))):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        print(f"{name:48s} {med(fn, steps):.4f} ms (median of {steps})", flush=True)
    for gc_on in (True, False):  # the mean vs the median: Python's cyclic GC passes triggered by allocations
        (gc.enable if gc_on else gc.disable)()
        ts = []
        for _ in range(200):
            t0 = time.perf_counter()
            codec.decode_module(up, g, base=base)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        ts.sort()
        print(f"decode_module x200, gc {'on ' if gc_on else 'off'}: median {ts[100]:.3f} mean {sum(ts) / 200:.3f} "
              f"max {ts[-1]:.3f} ms", flush=True)
    gc.enable()
    for name, fn in (("encode_module", lambda: codec.encode_module(m, base=base)),
                     ("decode_module", lambda: codec.decode_module(up, g, base=base)),
                     ("decode_module (unpickled)", lambda: codec.decode_module(up_r, g, base=base))):
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize()
        pr.disable()
        print(f"---- {name}")
        pstats.Stats(pr).sort_stats("tottime").print_stats(14)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 50)
