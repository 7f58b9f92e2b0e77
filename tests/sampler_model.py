"""Test-side restatement of the encoder's sampled bracket (coala_amd/csrc/coalac.hip `sample_segment`), so tests can
say which branch of the sampler a segment takes and compare the kernel's bracket {T_lo, T_hi} with this model
(coalac_debug_brackets). Integer arithmetic on uint32 keys, as the kernel does; the margin in float64 as the kernel
does. Test infrastructure only (never imported by the product path).

Outcomes of the concentrated-bin refinement (coalac.hip sample_segment, the `tie` block):
  "none"  the sampled keys are not concentrated where the bracket lies: bracket = bin edges of one histogram pass
  "split" both bracket ranks shared a bin and parted in a refinement pass: bracket = their sub-bins' outward edges
  "tie"   the refinement reached single keys and the lower rank's key K repeats (both ranks on K, or K seen
          >= max(8, margin / 4) times): tie mode, T_lo = K | TIE_FLAG
  "edge"  the refinement reached single keys but K repeats fewer times: T_lo = K (the lower edge itself)
"""
import math

import numpy as np

KEY_MAX = 0x7FFFFFFF
TIE_FLAG = 0x80000000
SAMPLE_MAX = 8192
HIST_BINS = 2048


def _hash32(x):
    x &= 0xFFFFFFFF
    x ^= x >> 16
    x = (x * 0x7FEB352D) & 0xFFFFFFFF
    x ^= x >> 15
    x = (x * 0x846CA68B) & 0xFFFFFFFF
    x ^= x >> 16
    return x


def sample_keys(x, seg_index):
    """The keys the sampler reads: R runs of 16 elements, one per stratum, jittered by a hash of (run, segment)."""
    n = x.size
    R = max(64, min(SAMPLE_MAX // 16, n // 512)) & ~63
    stride = n // R
    room = stride - 16
    keys = np.empty(R * 16, np.uint32)
    bits = x.view(np.uint32) & np.uint32(KEY_MAX)
    for run in range(R):
        h = _hash32(((run * 0x9E3779B9) & 0xFFFFFFFF) ^ (((seg_index + 1) * 0x85EBCA6B) & 0xFFFFFFFF))
        start = (run * stride + h % (room + 1)) & ~3
        keys[run * 16:run * 16 + 16] = bits[start:start + 16]
    return keys.astype(np.int64)


def _band_shift(lo, hi, bits=11):
    w = hi - lo
    if w == 0:
        return 0
    bl = int(w).bit_length()
    return bl - bits if bl > bits else 0


def _pick(hist, r):
    """Bin of the r-th largest key (1-based) and the rank inside it; (None, 0) for r == 0 (hist_pick2)."""
    if r == 0:
        return None, 0
    above = 0
    for b in range(len(hist) - 1, -1, -1):
        if above + hist[b] >= r:
            return b, r - above
        above += int(hist[b])
    return None, 0


def bracket(x, k, seg_index):
    """(T_lo, T_hi, outcome) the sampler computes for a large segment x (float32) keeping k of its elements."""
    n = x.size
    kk = sample_keys(x, seg_index)
    m = kk.size
    p = k / n
    se = p * m
    d = 6.0 * math.sqrt(se) + 8.0
    rlo, rhi = math.ceil(se + d), math.floor(se - d)
    kmin, kmax = int(kk.min()), int(kk.max())
    shift = _band_shift(kmin, kmax)
    hist = np.bincount((kk - kmin) >> shift, minlength=HIST_BINS)
    r1 = int(rlo) if rlo < m else 0
    r2 = int(rhi) if rhi >= 1 else 1
    blo, qlo = _pick(hist, r1)
    bhi, qhi = _pick(hist, r2)
    tlo, thi = 0, KEY_MAX
    if rlo < m:
        tlo = kmin + (blo << shift)
    if rhi >= 1:
        thi = min(kmin + ((bhi + 1) << shift) - 1, kmax)
    outcome = "none"
    mw = (int(rlo) - r2) if rlo < m else 0
    if rlo < m and (blo == bhi or hist[blo] >= mw):
        two = blo == bhi
        base, ck, sft = kmin + (blo << shift), int(hist[blo]), shift
        split = False
        while sft > 0:
            ns = sft - 11 if sft > 11 else 0
            top = base + (1 << sft) - 1
            sel = kk[(kk >= base) & (kk <= top)]
            h2 = np.bincount((sel - base) >> ns, minlength=HIST_BINS)
            b1, q1 = _pick(h2, qlo)
            b2, q2 = _pick(h2, qhi if two else 0)
            if two and b1 != b2:
                tlo = base + (b1 << ns)
                if rhi >= 1:
                    thi = min(base + ((b2 + 1) << ns) - 1, kmax)
                split = True
                outcome = "split"
                break
            qlo, qhi = q1, q2
            ck = int(h2[b1])
            base += b1 << ns
            sft = ns
        if not split:
            if base != 0 and (two or ck >= max(8, mw // 4)):
                outcome = "tie"
                tlo = base | TIE_FLAG
                if two:
                    thi = base
            else:
                outcome = "edge"
                tlo = base
                if two and rhi >= 1:
                    thi = base
    return tlo, thi, outcome


def near_tie_segment(rng, kind, n, lr=1e-3):
    """Near-tied values around lr (the k-th key's neighbourhood of a sign-like update) with 5 % wide outliers that
    stretch the sampled key range (coarse first histogram: the refinement runs):
      "levels"  16 near-tied magnitudes 8 ulps apart ({tie, split} by ratio and size)
      "band"    a continuous band of near-ties, lr (1 + U(0, 1e-4)) ({edge, split} by ratio and size)
      "sign"    every |x| = lr (tie)
      "gauss"   N(0, lr^2), no near-ties (no refinement)"""
    lr = np.float32(lr)
    sgn = np.where(rng.random(n) < 0.5, -1, 1).astype(np.float32)
    if kind == "levels":
        lv = (lr * (1 + np.arange(16) * 1e-6)).astype(np.float32)
        x = (sgn * lv[rng.integers(0, 16, n)]).astype(np.float32)
    elif kind == "band":
        x = (sgn * (lr * (1 + rng.random(n) * 1e-4))).astype(np.float32)
    elif kind == "sign":
        x = (sgn * lr).astype(np.float32)
    else:
        return (rng.standard_normal(n) * lr).astype(np.float32)
    if kind != "sign":
        o = rng.random(n) < 0.05
        x[o] = (rng.standard_normal(int(o.sum())) * 1e-3).astype(np.float32)
    return x


NEAR_TIE_SIZES = (1 << 20, 300000, 65536, 5000)
NEAR_TIE_KINDS = ("levels", "band", "sign", "gauss")


def near_tie_layout(rng):
    """One client's segments: every kind at every size."""
    return [near_tie_segment(rng, kind, n) for kind in NEAR_TIE_KINDS for n in NEAR_TIE_SIZES]


def ccap_for(ratios):
    """Record slots per large unit of a plan whose large segments keep at most max(ratios) (coalac_plan_create)."""
    r = max(ratios)
    c = int(math.ceil((4096 * min(1.0, 2.0 * r + 0.05) + 256.0) / 64.0)) * 64
    return max(512, min(4096, c))


def takes_raw_path(x, k, tlo, thi, ccap):
    """Whether the segment falls back to the raw-data path with this bracket: a unit with more candidate records than
    its ccap slots (candidates: keys >= T_lo, or in tie mode the keys above K), or a bracket that misses the k-th key
    (segment_pick / select_fallback)."""
    keys = (x.view(np.uint32) & np.uint32(KEY_MAX)).astype(np.int64)
    if tlo == 0 or tlo & TIE_FLAG:
        K = tlo & KEY_MAX
        cand = keys > K
        sc, sz, sa = int(cand.sum()), int((keys == K).sum()), int((keys > thi).sum())
        ok = (sc < k <= sc + sz) or (sa < k <= sc)
    else:
        cand = keys >= tlo
        sa, sc = int((keys > thi).sum()), int(cand.sum())
        ok = sa < k <= sc
    per_unit = np.add.reduceat(cand.astype(np.int64), np.arange(0, x.size, 4096))
    return (not ok) or bool((per_unit > ccap).any())
