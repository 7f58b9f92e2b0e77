"""Host cost of one ResNet-50 in-place encode: the direct launch sequence (coalac_encode_segptr, 6 kernels)
against a replay of the same sequence captured as a graph (torch.cuda.CUDAGraph over the ctypes call).
Prints median host microseconds until the call returns, and the synchronised per-call time."""
import json
import time

import torch

from coala_amd.compression import UpdateCodec
from coala_amd.layouts import build_module


def med(xs):
    xs = sorted(xs)
    return round(xs[len(xs) // 2] * 1e6, 2)


def main():
    dev = torch.device("cuda", 0)
    m = build_module("resnet50_tv", seed=1, device=dev)
    g = build_module("resnet50_tv", seed=2, device=dev)
    codec = UpdateCodec(0.01, 8, "delta")
    base = codec.snapshot(g)
    up = codec.encode_module(m, base=base)
    torch.cuda.synchronize()
    from coala_amd.compression.codec import _layout_walk, _module_walk
    names, tensors, walk = _module_walk(m)
    d, segs = _layout_walk(names, tensors, walk)
    plan = codec.plan_for(d.L.sizes_key, dev)
    ws = codec._workspace(plan)
    bflat = base.flat_on(dev)
    out = plan.empty_encoded()
    res = {}

    def timeit(fn, n=200):
        hs, ts = [], []
        for _ in range(n):
            t0 = time.perf_counter()
            fn()
            hs.append(time.perf_counter() - t0)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        return med(hs), med(ts)

    for _ in range(5):
        plan.encode_segments(segs, base=bflat, out=out, workspace=ws, checked=True, ptrs=d.seg_ptrs)
    torch.cuda.synchronize()
    res["direct_fixed_out_us"] = timeit(lambda: plan.encode_segments(segs, base=bflat, out=out, workspace=ws,
                                                                      checked=True, ptrs=d.seg_ptrs))
    res["direct_new_out_us"] = timeit(lambda: plan.encode_segments(segs, base=bflat, workspace=ws, checked=True,
                                                                    ptrs=d.seg_ptrs))
    res["empty_encoded_us"] = timeit(plan.empty_encoded)
    cap = torch.cuda.Stream(dev)
    cap.wait_stream(torch.cuda.current_stream(dev))
    ws2 = plan.empty_workspace()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, stream=cap, capture_error_mode="thread_local"):
        plan.encode_segments(segs, base=bflat, out=out, workspace=ws2, checked=True, ptrs=d.seg_ptrs)
    torch.cuda.synchronize()
    for _ in range(5):
        gr.replay()
    torch.cuda.synchronize()
    res["graph_replay_us"] = timeit(gr.replay)
    ref = [t.clone() for t in (out.idx, out.vals, out.mn, out.scale)]
    plan.encode_segments(segs, base=bflat, out=out, workspace=ws, checked=True, ptrs=d.seg_ptrs)
    torch.cuda.synchronize()
    res["graph_equals_direct"] = all(torch.equal(a, b) for a, b in zip(ref, (out.idx, out.vals, out.mn, out.scale)))
    res["encode_module_us"] = timeit(lambda: codec.encode_module(m, base=base))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
