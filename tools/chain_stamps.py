"""Diagnostics: where one update's select chain spends its time (COALAC_FLAG_STAMPS phase stamps, 100 MHz real-time
counter, coalac.hip STAMP slots): per large segment the sampler (16 start, 17 keys reduced, 18 bracket picked, 19 end),
the band histogram (20 / 21, the segment's last group block), the window pass (22 start, 23 segment histogram picked,
24 end) and the segment select (0 start, 1 window resolved, 10 exact key, 11 unit offsets, 12 end), in us since the
first sampler block started. Prints the largest segments and, per slot, the earliest / latest stamp over segments.

    python tools/chain_stamps.py [layout] [clients]
"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from coala_amd.compression import CodecPlan  # noqa: E402
from coala_amd.compression._lib import COALAC_FLAG_STAMPS  # noqa: E402
from coala_amd.compression.spec import small_limit  # noqa: E402
from coala_amd.layouts import fp32_sizes  # noqa: E402
from coala_amd.workload import synth_batch  # noqa: E402

NSTAMP = 32
layout = sys.argv[1] if len(sys.argv) > 1 else "resnet50_tv"
clients = int(sys.argv[2]) if len(sys.argv) > 2 else 1
sizes = fp32_sizes(layout)
plan = CodecPlan(sizes, 0.01, 8, clients=clients)
flats = [synth_batch(plan.table, torch.device("cuda", 0), client_ids=[100 * r + c for c in range(clients)])
         for r in range(3)]  # rotated inputs (one set would sit in the Infinity Cache)
ws = plan.empty_workspace()
enc = plan.empty_encoded()
for r in range(6):
    plan.encode(flats[r % 3], out=enc, workspace=ws, flags=COALAC_FLAG_STAMPS)
torch.cuda.synchronize()
nseg = plan.n_segments
buf = (ctypes.c_uint64 * (NSTAMP * nseg))()
n = plan._lib.coalac_debug_stamps(plan._h, ctypes.c_void_p(ws.data_ptr()), None, buf, NSTAMP * nseg)
st = np.frombuffer(buf, dtype=np.uint64)[:n].reshape(-1, NSTAMP).astype(np.int64)
lim = small_limit(sizes * clients)
large = [s for s in sizes * clients if s > lim]
rows = st[:len(large)]
t0 = rows[:, 16][rows[:, 16] > 0].min()
slots = {"sample": (16, 17, 18, 19), "ghist": (20, 21), "gwin": (22, 23, 24), "select": (0, 1, 10, 11, 12)}


def us(v):
    return round((int(v) - int(t0)) * 0.01, 2) if v > 0 else None


order = np.argsort(-np.array(large))
for i in order[:5]:
    print(json.dumps({"n": int(large[i]), **{k: [us(rows[i, j]) for j in v] for k, v in slots.items()}}))
summary = {}
for k, v in slots.items():
    for j in v:
        col = rows[:, j][rows[:, j] > 0]
        if col.size:
            summary[f"{k}[{j}]"] = [us(col.min()), us(col.max())]
print(json.dumps({"first..last per slot (us)": summary}))
