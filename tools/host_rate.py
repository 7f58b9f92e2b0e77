"""Host-inclusive encode+decode rate (SURVEY.md §8(d) "Host-inclusive rate").

The serialised update starts and ends in host memory (UploadContent.data). One step here:
  client side: pinned H2D of the 4N-byte update -> encode -> D2H of the payload (idx, codes, mn, scale)
  server side: H2D of the payload -> decode -> D2H of the dense 4N-byte update
all on one stream, timed with the host clock around K steps after warmup. Reported as GB/s of fp32
update (4N per client per step), next to the device-resident rate of the same batch.

    python tools/host_rate.py [--clients 1 16] [--steps 10]
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
    enc_d, ws, dws = plan.empty_encoded(), plan.empty_workspace(), plan.empty_decode_workspace()
    out_d = torch.empty_like(flat_d)
    enc_h = [torch.empty_like(t, device="cpu").pin_memory() for t in (enc_d.idx, enc_d.vals, enc_d.mn, enc_d.scale)]
    enc_r = plan.empty_encoded()  # server-side device copy of the received payload
    in_d = torch.empty_like(flat_d)

    def device_step():
        plan.encode(in_d, out=enc_d, workspace=ws)
        plan.decode(enc_d, out=out_d, workspace=dws)

    def host_step():
        in_d.copy_(flat_h, non_blocking=True)
        plan.encode(in_d, out=enc_d, workspace=ws)
        for h, d in zip(enc_h, (enc_d.idx, enc_d.vals, enc_d.mn, enc_d.scale)):
            h.copy_(d, non_blocking=True)
        for h, d in zip(enc_h, (enc_r.idx, enc_r.vals, enc_r.mn, enc_r.scale)):
            d.copy_(h, non_blocking=True)
        plan.decode(enc_r, out=out_d, workspace=dws)
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


if __name__ == "__main__":
    main()
