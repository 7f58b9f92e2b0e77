"""Generate tests/golden/codec_vectors.npz: small CodecSpec v1 input/output vectors from the CPU oracle.

The reference has no codec, so these vectors are NOT reference outputs ("parity unpinned", SURVEY.md
§8(c)); they freeze the spec's behaviour on the edge cases it defines (ties, signed zeros, denormals,
NaN/inf keys, constant segments, k = 1, k = n, n = 1, all bit widths) so that any later change to the
oracle or the kernels is caught. The GPU tests compare the HIP path against them bit for bit.

    python tests/golden/make_codec_vectors.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import codec_oracle as O  # noqa: E402

CASES = {
    "n1": np.array([3.0], np.float32),
    "signed_zeros": np.array([-0.0, 0.0, -0.0, 0.0, 0.0, -0.0], np.float32),
    "constant": np.full(37, 0.25, np.float32),
    "equal_magnitudes": np.array([1, -1, 1, -1, 2, -2, 2, -2, 0.5], np.float32),
    "denormals": np.array([1e-40, -1e-41, 3e-39, 0, 1e-45, -1e-45, 2e-38], np.float32),
    "infinities": np.array([np.inf, -1.0, 2.0, 0.5, -np.inf, 3.0], np.float32),
    "nan_keys": np.array([np.nan, 1.0, -2.0, 0.25, 7.0, -7.0, -np.nan], np.float32),
    "half_even": np.array([0.0, 1.0, 0.5, 1.5, 2.5, 3.5, 255.0, 127.5, 128.5], np.float32),
}


def build():
    rng = np.random.default_rng(20251015)
    cases = dict(CASES)
    cases["gauss_1000"] = (rng.standard_normal(1000) * 1e-3).astype(np.float32)
    cases["quarter_ties_5000"] = (np.round(rng.standard_normal(5000) * 4) / 4).astype(np.float32)
    cases["gauss_9000"] = (rng.standard_normal(9000) * 1e-2).astype(np.float32)
    out = {}
    for name, x in cases.items():
        out[f"{name}/x"] = x
        for ratio in (0.001, 0.01, 0.3, 1.0):
            k = O.k_for(x.size, ratio)
            for bits in (1, 4, 8, 32):
                idx, vals, mn, sc = O.encode_segment(x, k, bits)
                dec = O.decode_segment(idx, vals, mn, sc, x.size, bits)
                tag = f"{name}/r{ratio}/b{bits}"
                out[f"{tag}/k"] = np.array([k], np.int64)
                out[f"{tag}/idx"] = idx
                out[f"{tag}/vals"] = vals
                out[f"{tag}/mn_scale"] = np.array([mn, sc], np.float32)
                out[f"{tag}/dec"] = dec
    return out


if __name__ == "__main__":
    vec = build()
    np.savez_compressed(os.path.join(HERE, "codec_vectors.npz"), **vec)
    print(len(vec), "arrays")
