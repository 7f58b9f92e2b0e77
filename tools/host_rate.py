"""Host-inclusive encode+decode rate (SURVEY.md §8(d) "Host-inclusive rate").

The serialised update starts and ends in host memory (UploadContent.data). One step here:
  client side: pinned H2D of the 4N-byte update -> encode -> D2H of the payload (idx, codes, mn, scale)
  server side: H2D of the payload -> decode -> D2H of the dense 4N-byte update
all on one stream, timed with the host clock around K steps after warmup. Reported as GB/s of fp32
update (4N per client per step), next to the device-resident rate of the same batch.

    python tools/host_rate.py [--clients 1 16] [--steps 10]

Then the hooks' own bytes-to-bytes path (run_hooks): compression() -> pickle -> unpickle -> decompression()
-> D2H of the decoded state.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(clients, steps, warmup, layout, ratio, bits):
    import torch

    from coala_amd.compression import CodecPlan
    from coala_amd.layouts import fp32_sizes
    from coala_amd.workload import synth_batch

    dev = torch.device("cuda", 0)
    plan = CodecPlan(fp32_sizes(layout), ratio, bits, clients=clients, device=dev)
    flat_d = synth_batch(plan.table, dev, client_ids=range(clients))
    flat_h = flat_d.cpu().pin_memory()
    out_h = torch.empty_like(flat_h).pin_memory()
    enc_d, ws = plan.empty_encoded(), plan.empty_workspace()
    out_d = torch.empty_like(flat_d)
    enc_h = [torch.empty_like(t, device="cpu").pin_memory() for t in (enc_d.idx, enc_d.vals, enc_d.mn, enc_d.scale)]
    enc_r = plan.empty_encoded()  # server-side device copy of the received payload
    in_d = torch.empty_like(flat_d)

    def device_step():
        plan.encode(in_d, out=enc_d, workspace=ws)
        plan.decode(enc_d, out=out_d)

    def host_step():
        in_d.copy_(flat_h, non_blocking=True)
        plan.encode(in_d, out=enc_d, workspace=ws)
        for h, d in zip(enc_h, (enc_d.idx, enc_d.vals, enc_d.mn, enc_d.scale)):
            h.copy_(d, non_blocking=True)
        for h, d in zip(enc_h, (enc_r.idx, enc_r.vals, enc_r.mn, enc_r.scale)):
            d.copy_(h, non_blocking=True)
        plan.decode(enc_r, out=out_d)
        out_h.copy_(out_d, non_blocking=True)

    res = {}
    in_d.copy_(flat_d)
    for name, fn in (("device_resident", device_step), ("host_inclusive", host_step)):
        for _ in range(warmup):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        res[name] = {"GBps": round(4.0 * plan.table.n_elements * steps / el / 1e9, 2),
                     "ms_per_step": round(el / steps * 1e3, 4)}
    payload = sum(t.numel() * t.element_size() for t in enc_h)
    ok = torch.equal(out_h.to(dev), out_d)
    res.update(clients=clients, layout=layout, ratio=ratio, bits=bits, update_bytes=4 * plan.table.n_elements,
               payload_bytes=payload, pcie_bytes_per_step=2 * 4 * plan.table.span + 2 * payload,
               roundtrip_consistent=bool(ok))
    return res


def run_hooks(steps, warmup, layout, ratio, bits, mode="delta"):
    """The hooks' own path, bytes to bytes: client compression() of the trained module on the
    GPU (UpdateCodec.encode_module, in place) -> pickle.dumps of the carrier (the D2H of the payload + the
    COALAQ1 pack, what codec.marshal does at coala/client/base.py:363) -> pickle.loads on the server
    (coala/server/service.py:83) -> decompression(model) (UpdateCodec.decode_module: one pinned H2D of the
    payload + decode into a new module on w_global) -> D2H of the decoded dense state (one copy of its flat
    storage). Per client, serial, wall clock."""
    import pickle

    import torch

    from coala_amd.compression import UpdateCodec
    from coala_amd.layouts import build_module

    dev = torch.device("cuda", 0)
    m = build_module(layout, seed=1, device=dev)
    g = build_module(layout, seed=2, device=dev)
    codec = UpdateCodec(ratio, bits, mode)
    base = codec.snapshot(g) if mode == "delta" else None
    N = sum(p.numel() for p in m.state_dict().values() if p.dtype == torch.float32)
    host = None
    parts = {"encode_module": 0.0, "pickle_dumps": 0.0, "pickle_loads": 0.0, "decode_module": 0.0, "d2h_state": 0.0}

    def step(acc):
        nonlocal host
        t = [time.perf_counter()]
        up = codec.encode_module(m, base=base)
        t.append(time.perf_counter())
        blob = pickle.dumps(up)
        t.append(time.perf_counter())
        up2 = pickle.loads(blob)
        t.append(time.perf_counter())
        mod = codec.decode_module(up2, g, base=base)
        torch.cuda.synchronize()
        t.append(time.perf_counter())
        w = next(iter(mod.parameters()))
        st = w.untyped_storage()
        if host is None or host.numel() < st.nbytes():
            host = torch.empty(st.nbytes(), dtype=torch.uint8, pin_memory=True)
        src = torch.empty(0, dtype=torch.uint8, device=dev).set_(st)
        host[:st.nbytes()].copy_(src)
        t.append(time.perf_counter())
        if acc:
            for k, a, b in zip(parts, t[:-1], t[1:]):
                parts[k] += b - a
        return len(blob)

    for _ in range(warmup):
        step(False)
    nb = 0
    t0 = time.perf_counter()
    for _ in range(steps):
        nb = step(True)
    el = time.perf_counter() - t0
    return {"path": "hooks, bytes to bytes", "layout": layout, "mode": mode, "ratio": ratio, "bits": bits,
            "GBps": round(4.0 * N * steps / el / 1e9, 2), "ms_per_client": round(el / steps * 1e3, 4),
            "blob_bytes": nb, "update_bytes": 4 * N,
            "ms_parts": {k: round(v / steps * 1e3, 4) for k, v in parts.items()}}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--clients", type=int, nargs="+", default=[1, 16])
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--layout", default="resnet50_tv")
    p.add_argument("--ratio", type=float, default=0.01)
    p.add_argument("--bits", type=int, default=8)
    a = p.parse_args()
    for c in a.clients:
        print(json.dumps(run(c, a.steps, a.warmup, a.layout, a.ratio, a.bits)), flush=True)
    for mode in ("delta", "weights"):
        print(json.dumps(run_hooks(max(a.steps, 20), a.warmup, a.layout, a.ratio, a.bits, mode)), flush=True)


if __name__ == "__main__":
    main()
