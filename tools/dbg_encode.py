"""Debug: encode a batch (layout, ratio, clients, delta) on the GPU and compare every segment with the oracle;
print the first mismatching segments (n, k, unit count, the first differing entries)."""
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from coala_amd.compression import CodecPlan
from coala_amd.layouts import fp32_sizes
from coala_amd.workload import synth_batch
from oracle import codec_oracle as O

layout, ratio, clients, delta = sys.argv[1], float(sys.argv[2]), int(sys.argv[3]), sys.argv[4] == "1"
sizes = fp32_sizes(layout)
plan = CodecPlan(sizes, ratio, 8, clients=clients)
dev = torch.device("cuda", 0)
flat = synth_batch(plan.table, dev, client_ids=[800 + i for i in range(clients)])
one = CodecPlan(sizes, ratio, 8, clients=1)
base = synth_batch(one.table, dev, client_ids=[899]).repeat(clients) if delta else None
ws = plan.empty_workspace()
fill = os.environ.get("FILL")  # poison the workspace first: a read of a word this encode never wrote shows up
if fill == "ff":
    ws.fill_(255)
elif fill == "rand":
    ws.copy_(torch.randint(0, 256, ws.shape, dtype=torch.uint8, device=dev))
f0 = flat.clone(); b0 = None if base is None else base.clone()
enc = plan.encode(flat, base=base, workspace=ws)
torch.cuda.synchronize()
print('input changed', bool((flat != f0).any()), None if base is None else bool((base != b0).any()))
torch.cuda.synchronize()
print("fallbacks", plan.fallbacks(ws))
g = [t.cpu().numpy() for t in (enc.idx, enc.vals, enc.mn, enc.scale)]
segs = plan.table.segs.astype(np.int64)
idx, vals, mn, sc = O.encode(flat.cpu().numpy(), segs, 8, base=None if base is None else base.cpu().numpy())
bad = 0
for s, (off, n, k, oo) in enumerate(segs):
    a, b = g[0][oo:oo + k], idx[oo:oo + k]
    if not np.array_equal(a, b) or not np.array_equal(g[1][oo:oo + k], vals[oo:oo + k]):
        d = np.flatnonzero(a != b)
        print(f"seg {s}: n={n} k={k} units={(n + 4095) // 4096} first diffs at {d[:5].tolist()} gpu={a[d[:5]].tolist()} "
              f"ref={b[d[:5]].tolist()} n_diff={d.size}")
        bad += 1
        if bad > 12:
            break
print("bad segments", bad, "of", len(segs))
if os.environ.get("DUMP"):  # instrumented variants: tlo = per-unit counts (above | equal << 16), thi = output offset
    import ctypes
    nl = plan._n_lunits if hasattr(plan, "_n_lunits") else sum((int(n) + 4095) // 4096 for n in segs[:, 1] if n > 4096)
    lo, hi = (ctypes.c_uint32 * nl)(), (ctypes.c_uint32 * nl)()
    got = plan._lib.coalac_debug_brackets(plan._h, ctypes.c_void_p(ws.data_ptr()), None, lo, hi, nl)
    lo, hi = np.frombuffer(lo, np.uint32)[:got], np.frombuffer(hi, np.uint32)[:got]
    s = int(os.environ["DUMP"])
    u0 = int(os.environ.get("DUMPU", "250"))
    # large segments in table order (segs with n > small limit), their unit ranges
    from coala_amd.compression.spec import small_limit
    lim = small_limit(segs[:, 1])
    lb = 0
    for i, (off, n, k, oo) in enumerate(segs):
        if n > lim:
            if i == s:
                break
            lb += (int(n) + 4095) // 4096
    keys = (flat.cpu().numpy() - (0 if base is None else base.cpu().numpy())).view(np.uint32) & 0x7FFFFFFF
    off, n, k, oo = segs[s]
    sk = np.sort(keys[off:off + n])[::-1]
    T = sk[k - 1]
    print("lb", lb, "T", T, "rt", int((sk[:k] == T).sum()))
    nu = (int(n) + 4095) // 4096
    xs = keys[off:off + n]
    rg = np.array([int((xs[u * 4096:u * 4096 + 4096] > T).sum()) for u in range(nu)])
    re = np.array([int((xs[u * 4096:u * 4096 + 4096] == T).sum()) for u in range(nu)])
    rt = int((sk[:k] == T).sum())
    pe = np.concatenate([[0], np.cumsum(re)])[:-1]
    rso = np.concatenate([[0], np.cumsum(rg)])[:-1] + np.minimum(rt, pe)
    gg, ge_, gso = lo[lb:lb + nu] & 0xFFFF, lo[lb:lb + nu] >> 16, hi[lb:lb + nu]
    bad = np.flatnonzero((gg != rg) | (ge_ != re) | (gso != rso))
    print("units with mismatching g/e/so:", bad[:20].tolist())
    if os.environ.get("RT"):  # vi: tlo = rt, thi = min(rt, ex_e)
        print("rt values", np.unique(lo[lb:lb + nu]).tolist(), "min(rt, ex_e) at 215..225", hi[lb + 215:lb + 226].tolist())
    if os.environ.get("PREFIX"):  # vh: tlo = tie prefix, thi = above prefix
        pg = np.concatenate([[0], np.cumsum(rg)])[:-1]
        bp = np.flatnonzero((lo[lb:lb + nu] != pe) | (hi[lb:lb + nu] != pg))
        print("prefix mismatches", bp[:20].tolist())
        for u in bp[:8]:
            print(u, "gpu ex_e ex_g", lo[lb + u], hi[lb + u], "ref", pe[u], pg[u])
    for u in bad[:6]:
        print(u, "gpu", gg[u], ge_[u], gso[u], "ref", rg[u], re[u], rso[u])
    tp = np.flatnonzero(keys[off:off + n] == T)
    print("tie positions", tp.tolist()[:10], "units", (tp // 4096).tolist()[:10])
    p0 = int(os.environ.get("DUMPP", "105380"))
    print("gpu", g[0][oo + p0:oo + p0 + 12].tolist())
    print("ref", idx[oo + p0:oo + p0 + 12].tolist())
