"""The sampler model (tests/sampler_model.py) on the near-tie inputs of test_gpu_parity.py::test_near_tie_refinement:
every outcome of the sampler's concentrated-bin refinement — no refinement, a split bracket, a heavy tie (tie mode) and
a lower edge K seen too rarely for tie mode — occurs among them at ratios 0.01 and 0.1, so the GPU test (which compares
the kernel's brackets with this model and the codec with the oracle, bit for bit) covers both refinement branches
(the split bracket and K below the tie threshold were never checked bit-exact)."""
import math

import numpy as np

from tests.sampler_model import bracket, near_tie_layout


def test_near_tie_inputs_cover_every_refinement_outcome():
    seen = set()
    for clients in (1, 2):
        rng = np.random.default_rng(77)
        xs = [near_tie_layout(rng) for _ in range(clients)]
        T = len(xs[0])
        for ratio in (0.01, 0.1):
            for c in range(clients):
                for t, x in enumerate(xs[c]):
                    k = max(1, min(x.size, math.ceil(x.size * ratio)))
                    seen.add(bracket(x, k, c * T + t)[2])
    assert seen == {"none", "split", "tie", "edge"}, seen


def test_model_tie_flag_and_bracket_order():
    """Sanity of the model itself: a tie-mode bracket carries the flag and T_lo <= T_hi (keys) otherwise."""
    rng = np.random.default_rng(1)
    x = (rng.standard_normal(1 << 16) * 1e-3).astype(np.float32)
    tlo, thi, o = bracket(x, 655, 0)
    assert o == "none" and tlo <= thi
    x = np.where(rng.random(1 << 16) < 0.5, np.float32(-1e-3), np.float32(1e-3)).astype(np.float32)
    tlo, thi, o = bracket(x, 655, 0)
    assert o == "tie" and tlo & 0x80000000 and (tlo & 0x7FFFFFFF) == thi
