"""Synthetic client updates with the reference models' exact layouts (SURVEY.md §8(d) "Values / seeds").

Per client c (seed 1234 + c), per fp32 tensor t: delta ~ N(0, sigma_t^2) with sigma_t = 10^U(-4,-2);
then 0.5 % of positions are set to exact zeros and 0.5 % are overwritten with +/- the magnitude of another
random element (ties and sign flips of equal magnitude — tie-break stress). No datasets, no checkpoints:
the offline box has neither, and the codec's cost does not depend on trained values beyond their
magnitude distribution.
"""
import torch

from .compression.spec import SegmentTable
from .layouts import fp32_sizes, load


def fill_client(flat, table, client_id, seed_base=1234, zero_frac=0.005, tie_frac=0.005):
    """Write client `client_id`'s synthetic update into flat[0:table.span_per_client]."""
    g = torch.Generator(device=flat.device)
    g.manual_seed(seed_base + int(client_id))
    T = len(table.sizes)
    sig = torch.pow(10.0, torch.rand(T, generator=g, device=flat.device, dtype=torch.float64) * 2.0 - 4.0)
    sig = sig.tolist()
    for t, (off, n) in enumerate(zip(table.offsets, table.sizes)):
        seg = flat[off:off + n]
        seg.normal_(0.0, sig[t], generator=g)
    span = table.span_per_client
    N = sum(table.sizes)
    m0, m1 = int(zero_frac * N), int(tie_frac * N)
    if m0:
        zi = torch.randint(0, span, (m0,), generator=g, device=flat.device)
        flat[:span].index_fill_(0, zi, 0.0)
    if m1:
        # distinct targets: index_copy_ with a repeated index keeps whichever write lands last on the GPU, so
        # the data (and a test's k-th key) would change from run to run
        ti = torch.unique(torch.randint(0, span, (m1,), generator=g, device=flat.device))
        tj = torch.randint(0, span, (m1,), generator=g, device=flat.device)[:ti.numel()]
        sgn = torch.randint(0, 2, (m1,), generator=g, device=flat.device)[:ti.numel()].to(torch.float32) * 2.0 - 1.0
        flat[:span].index_copy_(0, ti, flat[:span][tj].abs() * sgn)
    return flat


def synth_batch(table, device, client_ids=None, seed_base=1234):
    """Flat fp32 buffer [table.span] holding table.clients synthetic updates back to back (a SegmentTable
    of copies of one layout, or a MixedTable of per-client layouts)."""
    ids = list(range(table.clients)) if client_ids is None else list(client_ids)
    flat = torch.zeros(table.span, dtype=torch.float32, device=device)
    so = table.client_span_off
    for c, cid in enumerate(ids):
        single = SegmentTable(table.client_sizes(c), table.ratio, 1)
        fill_client(flat[so[c]:so[c + 1]], single, cid, seed_base)
    return flat


def head_only(layout):
    """Indices (in fp32-segment order) of the tensors a FedPEFT client trains with its backbone frozen: the
    classifier head. The reference freezes every ViT parameter (application/FedPEFT/lora.py:64, and
    main.py:62-67 for linear probing) and trains the new head (plus, with LoRA, adapter tensors that the
    plain ViT-B/16 layout does not hold)."""
    names = [e["name"] for e in load(layout)["entries"] if e["dtype"] == "float32" and _numel(e["shape"]) > 0]
    return [i for i, n in enumerate(names) if n.startswith(("fc.", "head."))]


def _numel(shape):
    n = 1
    for d in shape:
        n *= d
    return n


def sign_step(flat, base, seed, lr=1e-3):
    """trained = fl(w_global -+ lr) in place of `flat`: one sign-like local step (signSGD, the first Adam step), so
    every |delta| is lr up to the rounding of the subtraction — heavy near-ties at the k-th key (bench.py C3_signs)."""
    import torch
    g = torch.Generator(device=flat.device).manual_seed(seed)
    flat.copy_(base + torch.where(torch.rand(flat.numel(), generator=g, device=flat.device) < 0.5, -lr, lr))
    return flat


def freeze_segments(flat, table, trained):
    """Zero every fp32 segment of every client except the `trained` ones (segment indices of one client's
    layout): the delta of a frozen tensor is exactly zero."""
    keep = set(trained)
    so = table.client_span_off
    for c in range(table.clients):
        sizes = table.client_sizes(c)
        single = SegmentTable(sizes, table.ratio, 1)
        for t, (off, n) in enumerate(zip(single.offsets, sizes)):
            if t not in keep:
                flat[so[c] + off:so[c] + off + n].zero_()
    return flat


# C5: 256 splitFL clients on 8 GPUs; each client draws (seeded) one of the client-side
# models at cut 1/2/4 or one of the three feature-tensor uploads
C5_CHOICES = [f"{m}_cut{c}" for m in ("resnet18_split", "resnet50_split", "simple_cnn_split") for c in (1, 2, 4)] + \
    ["sfl_feature_64x32x32", "sfl_feature_256x32x32", "sfl_feature_128x16x16"]
C5_CLIENTS, C5_GPUS, C5_SEED = 256, 8, 2024


def c5_draw(n_clients=C5_CLIENTS, seed=C5_SEED):
    """Layout name of every client of the C5 round (seeded, uniform over C5_CHOICES)."""
    import numpy as np
    rng = np.random.default_rng(seed)
    return [C5_CHOICES[i] for i in rng.integers(0, len(C5_CHOICES), n_clients)]


def c5_groups(names, world=C5_GPUS):
    """Clients -> GPUs by the reference's greedy grouping (LPT on the update size; coala_amd/sharding.py,
    restating coala/distributed/distributed.py:192-217)."""
    from .sharding import greedy_groups
    return greedy_groups([sum(fp32_sizes(n)) for n in names], world)


def c5_share(rank, n_clients=C5_CLIENTS, gpus=C5_GPUS, seed=C5_SEED):
    """(client ids, layout names) of GPU `rank % gpus`'s share of the C5 round, in client-id order."""
    names = c5_draw(n_clients, seed)
    ids = sorted(c5_groups(names, gpus)[rank % gpus])
    return ids, [names[i] for i in ids]


def mixed_table(names, ratio):
    from .compression.spec import MixedTable
    return MixedTable([fp32_sizes(n) for n in names], ratio)


def layout_table(name, ratio, clients=1):
    return SegmentTable(fp32_sizes(name), ratio, clients)


def describe(name):
    d = load(name)
    return {k: d[k] for k in ("model", "n_entries", "n_float32_entries", "n_float32_elements")}
