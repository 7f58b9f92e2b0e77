"""Remote-mode wire path on the GPU: the gRPC server decodes every upload in its own
thread (coala/server/service.py:71-111: Upload -> Thread(_handle_upload) :74 -> codec.unmarshal :83 ->
decompression :106). Each decoding thread gets its own HIP stream and pinned staging buffer, and moves the
blob's payload to the GPU in one asynchronous copy.

Checked against the CPU ORACLE (tests/oracle_backend.py), not only against the HIP path itself: 8 uploads
decoded by 8 concurrent threads are bit-identical to the oracle's decode of the same blobs (and to the serial
HIP decodes); the fused server (decompression(model) keeps the carrier, aggregate() decodes + averages in one
kernel) fed by 8 concurrent threads equals the oracle's FedAvg; the uploads themselves equal the oracle's
encode of the same trained states byte for byte; two client threads encoding on ONE stream equal serial
encodes (per-thread workspaces); the pinned one-copy transfer equals the plain per-tensor transfer;
decoded modules never alias the global model.
"""
import pickle
import threading
import time

import numpy as np
import pytest
import torch

from coala_amd.compression import CompressionServerMixin, UpdateCodec
from coala_amd.layouts import build_module
from tests.oracle_backend import OracleBackend

pytestmark = pytest.mark.gpu

N_UP = 8


class Server(CompressionServerMixin):
    codec_ratio, codec_bits, codec_mode = 0.01, 8, "delta"


class FusedServer(Server):
    codec_fused_aggregate = True


def trained(n, layout="resnet18"):
    return [build_module(layout, seed=100 + i, device="cuda") for i in range(n)]


def uploads(n, layout="resnet18"):
    g = build_module(layout, seed=0)  # the server's global model: on the CPU, as in the reference
    codec = UpdateCodec(0.01, 8, "delta")
    base = codec.snapshot(g)
    ws = trained(n, layout)
    blobs = [pickle.dumps(codec.encode(w.state_dict(), base=base)) for w in ws]  # UploadContent.data
    return g, ws, blobs


def states(mods):
    return [{k: v.detach().cpu().clone() for k, v in m.state_dict().items()} for m in mods]


def assert_state_equal(a, b, what):
    assert list(a) == list(b), what
    for k in a:
        x, y = a[k].cpu(), b[k].cpu()
        assert x.dtype == y.dtype and x.shape == y.shape, (what, k)
        if x.dtype == torch.float32:
            assert torch.equal(x.view(torch.int32), y.view(torch.int32)), (what, k)
        else:
            assert torch.equal(x, y), (what, k)


@pytest.fixture(scope="module")
def remote_round(cuda):
    g, ws, blobs = uploads(N_UP)
    oc = UpdateCodec(0.01, 8, "delta", backend=OracleBackend())
    obase = oc.snapshot(g)
    oracle_dec = states([oc.decode_module(pickle.loads(b), g, base=obase) for b in blobs])
    return g, ws, blobs, oc, obase, oracle_dec


def test_uploads_equal_oracle_encode(remote_round):
    """The HIP upload bytes are the oracle's upload bytes for the same trained states."""
    g, ws, blobs, oc, obase, _ = remote_round
    for i, (w, b) in enumerate(zip(ws, blobs)):
        st = {k: v.detach().cpu() for k, v in w.state_dict().items()}
        assert pickle.dumps(oc.encode(st, base=obase)) == b, i


def test_pinned_one_copy_transfer_equals_plain(remote_round, cuda):
    blobs = remote_round[2]
    up = pickle.loads(blobs[0])
    codec = UpdateCodec(0.01, 8, "delta")
    a = up.encoded_to(cuda, staging=codec._staging)
    b = up.encoded.to(cuda)
    torch.cuda.synchronize()
    for f in ("idx", "vals", "mn", "scale"):
        assert torch.equal(getattr(a, f), getattr(b, f)), f


def _threaded(n, fn):
    out = [None] * n
    gate = threading.Barrier(n)
    errs = []

    def run(i):
        try:
            gate.wait()
            out[i] = fn(i)
        except BaseException as e:  # (re-raised in the main thread)
            errs.append(e)
    ts = [threading.Thread(target=run, args=(i,)) for i in range(n)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    if errs:
        raise errs[0]
    return out


def test_concurrent_decodes_match_oracle(remote_round):
    g, _, blobs, _, _, oracle_dec = remote_round
    srv = Server()
    srv.model = g
    t0 = time.perf_counter()
    serial = states([srv.decompression(pickle.loads(b)) for b in blobs])
    t_serial = time.perf_counter() - t0
    t0 = time.perf_counter()
    # server/service.py: _handle_upload -> codec.unmarshal -> decompression, one thread per upload
    out = _threaded(len(blobs), lambda i: srv.decompression(pickle.loads(blobs[i])))
    torch.cuda.synchronize()
    t_conc = time.perf_counter() - t0
    conc = states(out)
    gptrs = {t.data_ptr() for t in g.state_dict().values()}
    for i in range(len(blobs)):
        assert_state_equal(conc[i], oracle_dec[i], f"thread decode {i} vs oracle")
        assert_state_equal(serial[i], oracle_dec[i], f"serial decode {i} vs oracle")
    for m in out:
        assert not any(t.data_ptr() in gptrs for t in m.state_dict().values())
    print(f"{len(blobs)} decodes: serial {t_serial * 1e3:.1f} ms, {len(blobs)} threads {t_conc * 1e3:.1f} ms")


def test_concurrent_fused_server_matches_oracle_fedavg(remote_round):
    """codec_fused_aggregate: uploads arrive on 8 threads (decompression keeps the carrier), then ONE fused
    decode + FedAvg kernel; equal to the oracle's FedAvg of the same blobs (torch-on-GPU division)."""
    g, _, blobs, oc, obase, _ = remote_round
    srv = FusedServer()
    srv.model = g
    carriers = _threaded(len(blobs), lambda i: srv.decompression(pickle.loads(blobs[i])))
    weights = [10 + 3 * i for i in range(len(blobs))]
    got = srv.aggregate(carriers, weights)
    torch.cuda.synchronize()
    ref = oc.aggregate([pickle.loads(b) for b in blobs], weights, g, base=obase, mode="recip")
    assert_state_equal(states([got])[0], states([ref])[0], "fused aggregate vs oracle")


def test_two_threads_encode_on_one_stream(cuda):
    """Two client threads encoding with ONE codec (one plan) on the same (default) stream: each gets its own
    workspace, so the interleaved launches cannot mix scan and select results."""
    g = build_module("resnet18", seed=0, device="cuda")
    codec = UpdateCodec(0.01, 8, "delta")
    base = codec.snapshot(g)
    ws = trained(2)
    serial = [pickle.dumps(codec.encode_module(w, base=base)) for w in ws]
    for _ in range(3):
        conc = _threaded(2, lambda i: codec.encode_module(ws[i], base=base))
        torch.cuda.synchronize()
        assert [pickle.dumps(u) for u in conc] == serial
