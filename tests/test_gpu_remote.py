"""Remote-mode wire path on the GPU: the gRPC server decodes every upload in its own
thread (coala/server/service.py:71-111: Upload -> Thread(_handle_upload) -> codec.unmarshal ->
decompression). Each decoding thread gets its own HIP stream and pinned staging buffer, and moves the
blob's payload to the GPU in one asynchronous copy.

Checked: 8 uploads decoded by 8 concurrent threads are bit-identical to the serial decodes; the pinned,
one-copy transfer equals the plain per-tensor transfer; the decoded modules never alias the global model.
"""
import copy
import pickle
import threading
import time

import numpy as np
import pytest
import torch

from coala_amd.compression import CompressionServerMixin, UpdateCodec
from coala_amd.layouts import build_module

pytestmark = pytest.mark.gpu


class Server(CompressionServerMixin):
    codec_ratio, codec_bits, codec_mode = 0.01, 8, "delta"


def uploads(n, layout="resnet18"):
    g = build_module(layout, seed=0)  # the server's global model: on the CPU, as in the reference
    codec = UpdateCodec(0.01, 8, "delta")
    base = codec.snapshot(g)
    blobs = []
    for i in range(n):
        w = build_module(layout, seed=100 + i, device="cuda")
        blobs.append(pickle.dumps(codec.encode(w.state_dict(), base=base)))  # UploadContent.data
    return g, blobs


def states(mods):
    return [{k: v.detach().cpu().clone() for k, v in m.state_dict().items()} for m in mods]


def test_pinned_one_copy_transfer_equals_plain(cuda):
    g, blobs = uploads(1)
    up = pickle.loads(blobs[0])
    codec = UpdateCodec(0.01, 8, "delta")
    a = up.encoded_to(cuda, staging=codec._staging)
    b = up.encoded.to(cuda)
    torch.cuda.synchronize()
    for f in ("idx", "vals", "mn", "scale"):
        assert torch.equal(getattr(a, f), getattr(b, f)), f


def test_concurrent_decodes_match_serial(cuda):
    g, blobs = uploads(8)
    srv = Server()
    srv.model = g
    t0 = time.perf_counter()
    serial = states([srv.decompression(pickle.loads(b)) for b in blobs])
    t_serial = time.perf_counter() - t0
    out = [None] * len(blobs)
    gate = threading.Barrier(len(blobs))

    def handle(i):  # server/service.py: _handle_upload -> codec.unmarshal -> decompression
        up = pickle.loads(blobs[i])
        gate.wait()
        out[i] = srv.decompression(up)

    ts = [threading.Thread(target=handle, args=(i,)) for i in range(len(blobs))]
    t0 = time.perf_counter()
    [t.start() for t in ts]
    [t.join() for t in ts]
    t_conc = time.perf_counter() - t0
    conc = states(out)
    gptrs = {t.data_ptr() for t in g.state_dict().values()}
    for i, (a, b) in enumerate(zip(serial, conc)):
        for k in a:
            assert torch.equal(a[k], b[k]), (i, k)
    for m in out:
        assert not any(t.data_ptr() in gptrs for t in m.state_dict().values())
    print(f"8 decodes: serial {t_serial * 1e3:.1f} ms, 8 threads {t_conc * 1e3:.1f} ms")
