"""Client -> rank sharding for multi-GPU runs (one process per GPU; no collective on the codec path).

Restates the reference's grouping (/root/reference/coala/distributed/distributed.py:142-217): clients
are independent units, so a rank simply encodes/decodes its own group. `split_sizes` reproduces
randomize_grouping's group sizes (:165-189: the first world - r groups get n // world, the last r get
one more); `greedy_groups` is greedy_grouping's LPT (:192-217) with the per-client cost being the
update's element count (the codec's work) instead of a profiled round time.
"""
import numpy as np


def split_sizes(n, world):
    base, extra = divmod(n, world)
    return [base] * (world - extra) + [base + 1] * extra


def contiguous_groups(items, world, shuffle_seed=None):
    """randomize_grouping: optional np.random shuffle (seeded as the reference does), then split."""
    items = list(items)
    if shuffle_seed is not None:
        np.random.seed(shuffle_seed)
        np.random.shuffle(items)
    out, pos = [], 0
    for s in split_sizes(len(items), world):
        out.append(items[pos:pos + s])
        pos += s
    return out


def greedy_groups(costs, world):
    """greedy_grouping over item indices: largest cost first (ties: larger index first, as the
    reference sorts (time, index) in reverse), each to the currently least-loaded group."""
    order = sorted(((c, i) for i, c in enumerate(costs)), reverse=True)
    groups = [[i] for (_, i) in order[:world]]
    load = [c for (c, _) in order[:world]]
    while len(groups) < world:
        groups.append([])
        load.append(0)
    for c, i in order[world:]:
        j = int(np.argmin(load))
        groups[j].append(i)
        load[j] += c
    return groups
