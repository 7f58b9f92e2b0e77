"""Probe: step time of the default bench workload eager vs hipGraph-replayed, with and without timing
events, at 16 clients and 1 client per GPU. Prints one JSON line per variant.

    python tools/graph_probe.py [--clients 16] [--steps 20]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--clients", type=int, nargs="+", default=[16, 1])
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--lanes", type=int, default=1)
    a = p.parse_args()
    import torch

    from coala_amd.compression import LanePipeline, SegmentTable
    from coala_amd.layouts import fp32_sizes
    from coala_amd.workload import synth_batch

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    for C in a.clients:
        t = SegmentTable(fp32_sizes("resnet50_tv"), 0.01, C)
        flat = synth_batch(t, dev, client_ids=range(C))
        pipe = LanePipeline(t, 8, lanes=a.lanes, device=dev)
        enc, out = pipe.empty_encoded(), pipe.empty_flat()
        s = pipe.stream

        def run(evs=None):
            with torch.cuda.stream(s):
                pipe.roundtrip(flat, enc=enc, out=out,
                               enc_events=None if evs is None else [evs[0]],
                               dec_events=None if evs is None else [evs[1]])

        def ev_pair(external=False):
            kw = {"enable_timing": True}
            if external:
                kw["external"] = True
            e = [None, torch.cuda.Event(**kw), torch.cuda.Event(**kw), None, None]
            d = [None, torch.cuda.Event(**kw), torch.cuda.Event(**kw)]
            for x in (e[1], e[2], d[1], d[2]):  # torch creates the HIP event on first record
                x.record()
            return e, d

        for _ in range(3):
            run()
        torch.cuda.synchronize()
        ref_idx = enc.idx.clone()
        ref_out = out.clone()
        res = {"clients": C, "bytes": 4 * t.n_elements}

        def timed(fn, K):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(K):
                fn(i)
            torch.cuda.synchronize()
            return (time.perf_counter() - t0) / K * 1e3

        res["eager_noev_ms"] = timed(lambda i: run(), a.steps)
        evs = [ev_pair() for _ in range(a.steps)]
        res["eager_ev_ms"] = timed(lambda i: run(evs[i]), a.steps)
        res["eager_ev_scan_ms"] = sum(e[0][1].elapsed_time(e[0][2]) for e in evs) / a.steps
        res["eager_ev_decode_ms"] = sum(e[1][1].elapsed_time(e[1][2]) for e in evs) / a.steps
        # graph without events
        try:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.stream(s):
                torch.cuda.synchronize()
                with torch.cuda.graph(g, stream=s):
                    pipe.roundtrip(flat, enc=enc, out=out)
            torch.cuda.synchronize()
            enc.idx.zero_()
            out.zero_()
            g.replay()
            torch.cuda.synchronize()
            res["graph_equal"] = bool(torch.equal(enc.idx, ref_idx) and torch.equal(out, ref_out))
            res["graph_noev_ms"] = timed(lambda i: g.replay(), a.steps)
        except Exception as e:  # noqa: BLE001
            res["graph_noev_err"] = repr(e)[:300]
        # graph with external timing events captured inside
        try:
            ge = torch.cuda.CUDAGraph()
            gev = ev_pair(external=True)
            torch.cuda.synchronize()  # the events exist before capture
            with torch.cuda.graph(ge, stream=s):
                pipe.roundtrip(flat, enc=enc, out=out, enc_events=[gev[0]], dec_events=[gev[1]])
            torch.cuda.synchronize()
            scan, dec = [], []

            def rep(i):
                ge.replay()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(a.steps):
                ge.replay()
                torch.cuda.synchronize()
                scan.append(gev[0][1].elapsed_time(gev[0][2]))
                dec.append(gev[1][1].elapsed_time(gev[1][2]))
            res["graph_ev_synced_ms"] = (time.perf_counter() - t0) / a.steps * 1e3
            res["graph_ev_ms"] = timed(rep, a.steps)
            res["graph_ev_scan_ms"] = sum(scan) / len(scan)
            res["graph_ev_decode_ms"] = sum(dec) / len(dec)
        except Exception as e:  # noqa: BLE001
            res["graph_ev_err"] = repr(e)[:300]
        for k in list(res):
            if k.endswith("_ms") and "scan" not in k and "decode" not in k:
                res[k.replace("_ms", "_GBs")] = round(res["bytes"] / (res[k] * 1e-3) / 1e9, 1)
        print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in res.items()}), flush=True)
        pipe.close()
        del flat, enc, out


if __name__ == "__main__":
    main()
