"""cProfile of the hooks' host path on the GPU (one ResNet-50 client, delta mode): UpdateCodec.encode of
the trained state in place (client compression()) and decode_module into a new module on w_global (server
decompression(model)), as bench.py's 'plugin' extra runs them. Prints the top host functions by own time.

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
from coala_amd.layouts import build_module  # noqa: E402


def main(steps=50):
    dev = torch.device("cuda", 0)
    m = build_module("resnet50_tv", seed=1, device=dev)
    g = build_module("resnet50_tv", seed=2, device=dev)
    codec = UpdateCodec(0.01, 8, "delta")
    base = codec.snapshot(g)
    state = m.state_dict()
    for _ in range(5):
        up = codec.encode(state, base=base)
        codec.decode_module(up, g, base=base)
    torch.cuda.synchronize()
    for name, fn in (("encode", lambda: codec.encode(state, base=base)),
                     ("decode_module", lambda: codec.decode_module(up, g, base=base))):
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize()
        print(f"{name}: {(time.perf_counter() - t0) / steps * 1e3:.3f} ms per call", flush=True)
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize()
        pr.disable()
        st = pstats.Stats(pr)
        st.sort_stats("tottime").print_stats(18)
        st.sort_stats("cumulative").print_stats(18)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 50)
