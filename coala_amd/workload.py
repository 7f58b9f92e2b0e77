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
        ti = torch.randint(0, span, (m1,), generator=g, device=flat.device)
        tj = torch.randint(0, span, (m1,), generator=g, device=flat.device)
        sgn = torch.randint(0, 2, (m1,), generator=g, device=flat.device).to(torch.float32) * 2.0 - 1.0
        flat[:span].index_copy_(0, ti, flat[:span][tj].abs() * sgn)
    return flat


def synth_batch(table, device, client_ids=None, seed_base=1234):
    """Flat fp32 buffer [table.span] holding table.clients synthetic updates back to back."""
    ids = list(range(table.clients)) if client_ids is None else list(client_ids)
    flat = torch.zeros(table.span, dtype=torch.float32, device=device)
    S = table.span_per_client
    single = SegmentTable(table.sizes, table.ratio, 1)
    for c, cid in enumerate(ids):
        fill_client(flat[c * S:(c + 1) * S], single, cid, seed_base)
    return flat


def layout_table(name, ratio, clients=1):
    return SegmentTable(fp32_sizes(name), ratio, clients)


def describe(name):
    d = load(name)
    return {k: d[k] for k in ("model", "n_entries", "n_float32_entries", "n_float32_elements")}
