"""Oracle over a spawned process pool, for the full-size parity tests (TEST INFRASTRUCTURE ONLY).

The per-GPU shares of the BASELINE configs (C2 16 x ResNet-18, C3 16 x ResNet-50, C4 16 x ViT-B/16:
179 M / 410 M / 1.385 G elements) are checked client by client with oracle/codec_oracle.py. One client
is one task: a spawned worker attaches the shared-memory copy of the batch the GPU encoded, runs the
oracle's encode + decode on its client's span, and returns the encoded arrays plus the decoded values
at the kept positions (the only non-zero positions of the oracle's dense output, which the worker
checks). Workers import numpy and the oracle only: no torch, no GPU.
"""
import os
from multiprocessing import get_context, shared_memory

import numpy as np


def pool_size():
    """Worker processes: the box's CPU share (OMP_NUM_THREADS, 16 per GPU there), at most the affinity."""
    aff = len(os.sched_getaffinity(0))
    cap = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or 16
    return max(1, min(aff, cap, 16))


def _client_task(args):
    name, nbytes, x0, span, segs, bits, base_name = args
    from oracle import codec_oracle as O
    shm = shared_memory.SharedMemory(name=name)
    bshm = shared_memory.SharedMemory(name=base_name) if base_name else None
    try:
        flat = np.ndarray((nbytes // 4,), dtype=np.float32, buffer=shm.buf)[x0:x0 + span]
        base = None if bshm is None else np.ndarray((nbytes // 4,), dtype=np.float32, buffer=bshm.buf)[x0:x0 + span]
        idx, vals, mn, sc = O.encode(flat, segs, bits, base=base)
        dense = O.decode(idx, vals, mn, sc, segs, bits, span, base=base)
        ks = segs[:, 2]
        pos = np.repeat(segs[:, 0], ks) + idx.astype(np.int64)  # client-relative positions of the kept entries
        kept = dense[pos].copy()
        if base is None:  # the oracle's dense output is zero everywhere else
            nz = int(np.count_nonzero(dense.view(np.uint32)))
            assert nz == int(np.count_nonzero(kept.view(np.uint32))), "oracle dense output has stray non-zeros"
        del flat, base, dense
        return idx, vals, mn, sc, pos, kept
    finally:
        shm.close()
        if bshm is not None:
            bshm.close()


class SharedBatch:
    """A host copy of a flat fp32 batch in POSIX shared memory (unlinked on close)."""

    def __init__(self, n_elements):
        self.nbytes = max(4, 4 * int(n_elements))
        self.shm = shared_memory.SharedMemory(create=True, size=self.nbytes)
        self.array = np.ndarray((self.nbytes // 4,), dtype=np.float32, buffer=self.shm.buf)

    @property
    def name(self):
        return self.shm.name

    def close(self):
        self.array = None
        self.shm.close()
        self.shm.unlink()


def oracle_clients(batch, client_spans, client_segs, bits, base=None, workers=None):
    """Oracle results of every client, computed in a spawned pool. client_spans: [(x0, span)] per client
    (flat element ranges), client_segs: int64 [T_c, 4] rows (in_off, n, k, out_off) RELATIVE to the
    client's x0 and k-offset. Returns an iterator of (client index, result) in client order."""
    tasks = [(batch.name, batch.nbytes, x0, span, segs, bits, None if base is None else base.name)
             for (x0, span), segs in zip(client_spans, client_segs)]
    W = min(workers or pool_size(), len(tasks))
    with get_context("spawn").Pool(W) as pool:
        for i, r in enumerate(pool.imap(_client_task, tasks)):
            yield i, r
