"""Where the fused server aggregate() call spends its host time: 16 ResNet-50 delta uploads through
UpdateCodec.aggregate (the codec_fused_aggregate server path). Prints the median call time and a cProfile."""
import cProfile
import io
import pstats
import time

import torch

from coala_amd.compression import UpdateCodec
from coala_amd.layouts import build_module


def main(C=16, n=30):
    dev = torch.device("cuda", 0)
    m = build_module("resnet50_tv", seed=1, device=dev)
    g = build_module("resnet50_tv", seed=2, device=dev)
    codec = UpdateCodec(0.01, 8, "delta")
    base = codec.snapshot(g)
    ups = [codec.encode_module(m, base=base) for _ in range(C)]
    wts = [10 + i for i in range(C)]
    call = lambda: codec.aggregate(ups, wts, g, base=base, mode="recip")
    for _ in range(3):
        call()
    torch.cuda.synchronize()
    ts, hs = [], []
    for _ in range(n):
        t0 = time.perf_counter()
        call()
        hs.append(time.perf_counter() - t0)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    hs.sort()
    print(f"aggregate of {C}: median {ts[n // 2] * 1e3:.4f} ms, host until return {hs[n // 2] * 1e3:.4f} ms")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(n):
        call()
    torch.cuda.synchronize()
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(25)
    print(s.getvalue())


if __name__ == "__main__":
    main()
