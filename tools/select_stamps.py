"""Diagnostics: per-phase timing of k_select blocks (COALAC_FLAG_STAMPS), 1 ResNet-50 client."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from coala_amd.compression import CodecPlan  # noqa: E402
from coala_amd.compression._lib import COALAC_FLAG_STAMPS  # noqa: E402
from coala_amd.layouts import fp32_sizes  # noqa: E402
from coala_amd.workload import synth_batch  # noqa: E402

clients = int(sys.argv[1]) if len(sys.argv) > 1 else 1
signs = len(sys.argv) > 2 and sys.argv[2] == "signs"  # C3_signs data: delta mode after one sign-like step
sizes = fp32_sizes("resnet50_tv")
plan = CodecPlan(sizes, 0.01, 8, clients=clients)
flat = synth_batch(plan.table, torch.device("cuda", 0))
base = None
if signs:
    from coala_amd.workload import sign_step  # noqa: E402
    base = synth_batch(plan.table, torch.device("cuda", 0), client_ids=[10_000 + i for i in range(clients)])
    sign_step(flat, base, 4242)
ws = plan.empty_workspace()
enc = plan.empty_encoded()
for _ in range(3):
    plan.encode(flat, base=base, out=enc, workspace=ws, flags=COALAC_FLAG_STAMPS)
torch.cuda.synchronize()
nseg = plan.n_segments
buf = (ctypes.c_uint64 * (16 * nseg))()
n = plan._lib.coalac_debug_stamps(plan._h, ctypes.c_void_p(ws.data_ptr()), None, buf, 16 * nseg)
st = np.frombuffer(buf, dtype=np.uint64)[:n].reshape(-1, 16).astype(np.int64)
large = [s for s in sizes if s > 4096] * clients
rows = []
for b in range(len(large)):
    r = st[b]
    if r[0] == 0:
        continue
    d = {f"p{i}": round((r[i] - r[0]) * 0.01, 2) for i in range(16) if r[i] > 0}
    rows.append((large[b], d))
rows.sort(key=lambda x: -x[1].get("p12", 0))
for n_el, d in rows[:6]:
    print(json.dumps({"n": n_el, "us_since_start": d}))
t0 = min(r[0] for r in st if r[0] > 0)
print(json.dumps({"block_start_spread_us": round((max(r[0] for r in st if r[0] > 0) - t0) * 0.01, 2),
                  "last_end_us": round((max(r[12] for r in st if r[12] > 0) - t0) * 0.01, 2)}))
