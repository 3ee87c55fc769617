"""Known-answer tests that pin the parts of the oracle the reference holds no vectors for.

* Otsu (``cv2.threshold(..., THRESH_OTSU)``, opencv-python unpinned, absent here): the
  sequential fp64 restatement is checked against an exact-rational evaluation of the same
  recurrence on histograms without exact ties, and on hand-computed cases.
* Percentile (legacy mask): the oracle calls NumPy itself; the integer-histogram restatement
  that the GPU uses is checked against ``np.percentile`` (including n > 2**24, where NumPy's
  float32 virtual index rounds).
* Gray code: encoder/decoder round trip over every code of 10-12 bits.
"""
from fractions import Fraction

import numpy as np
import pytest

from oracle import sl_oracle as O

EPS = Fraction(float(np.finfo(np.float32).eps))


def otsu_exact(h):
    """Same recurrence as OpenCV, evaluated in exact rationals; returns (argmax, tie)."""
    n = sum(h)
    mu = Fraction(sum(i * c for i, c in enumerate(h)), n)
    mu1, q1 = Fraction(0), Fraction(0)
    sig = []
    for i in range(256):
        p = Fraction(h[i], n)
        mu1 *= q1
        q1 += p
        q2 = 1 - q1
        if min(q1, q2) < EPS or max(q1, q2) > 1 - EPS:
            continue
        mu1 = (mu1 + i * p) / q1
        mu2 = (mu - q1 * mu1) / q2
        sig.append((q1 * q2 * (mu1 - mu2) ** 2, i))
    if not sig:
        return 0, False
    best = max(s for s, _ in sig)
    if best <= 0:
        return 0, False
    idx = [i for s, i in sig if s == best]
    return idx[0], len(idx) > 1


def test_otsu_two_level_and_constant():
    h = [0] * 256
    h[0], h[255] = 50, 50
    assert O.otsu_from_hist(h) == 0.0
    h = [0] * 256
    h[37] = 1000
    assert O.otsu_from_hist(h) == 0.0          # single bin: every bin skipped
    img = np.array([[10, 10, 200, 200], [10, 12, 198, 200]], np.uint8)
    t = O.otsu_threshold(img)
    assert 12 <= t < 198


def test_otsu_hand_computed():
    # h = {1: 2, 3: 1, 6: 1}: n=4, mu=11/4.  i=1: q1=1/2, mu1=1, mu2=9/2, sigma=49/16;
    # i=2: same state (plateau, no update); i=3: q1=3/4, mu1=5/3, mu2=6, sigma=169/48 > 49/16
    # -> threshold 3 (cv2 returns the bin index)
    h = [0] * 256
    h[1], h[3], h[6] = 2, 1, 1
    assert otsu_exact(h)[0] == 3                # bins 4, 5 tie exactly (plateau): first wins
    assert O.otsu_from_hist(h) == 3.0


@pytest.mark.parametrize("seed", range(40))
def test_otsu_matches_exact_rational(seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(500, 50000))
    a = rng.normal(rng.uniform(10, 80), rng.uniform(3, 20), n // 2)
    b = rng.normal(rng.uniform(120, 230), rng.uniform(3, 30), n - n // 2)
    u = np.arange(256).repeat(int(rng.integers(1, 4)))        # dense: no empty-bin plateaus
    img = np.clip(np.round(np.concatenate([a, b, u])), 0, 255).astype(np.uint8)
    h = np.bincount(img, minlength=256).tolist()
    want, tie = otsu_exact(h)
    if tie:
        pytest.skip("exact tie")
    assert O.otsu_threshold(img) == float(want)


def percentile_from_hist(h, n):
    """Float32 restatement used by the GPU stats kernel (slgpu.hip:percentile95_from_hist)."""
    cum = np.cumsum(h)

    def kth(k):
        return int(np.searchsorted(cum, k, side="right"))

    q = np.float32(95) / np.float32(100)
    vi = np.float32(np.float32(n - 1) * q)
    prev = np.floor(vi)
    nxt = np.float32(prev + np.float32(1))
    gamma = np.float32(vi - prev)
    pi, ni = int(prev), int(nxt)
    if vi >= np.float32(n - 1):
        pi = ni = n - 1
    a, b = np.float32(kth(pi)), np.float32(kth(ni))
    d = np.float32(b - a)
    r = np.float32(a + np.float32(d * gamma))
    if gamma >= np.float32(0.5):
        r = np.float32(b - np.float32(d * np.float32(np.float32(1) - gamma)))
    return r


@pytest.mark.parametrize("n", [4, 5, 17, 1000, 20001, 1 << 20, (1 << 24) + 12345, 24_000_000])
def test_percentile_restatement_matches_numpy(n):
    rng = np.random.default_rng(n)
    img = rng.integers(0, 40, size=n).astype(np.uint8)
    img[rng.integers(0, n, size=max(1, n // 50))] = rng.integers(40, 256)
    h = np.bincount(img, minlength=256)
    want = np.percentile(img.astype(np.float32), 95)
    got = percentile_from_hist(h, n)
    assert want.dtype == np.float32
    assert np.float32(got).tobytes() == np.float32(want).tobytes()


@pytest.mark.parametrize("bits", [10, 11, 12])
def test_gray_code_round_trip(bits):
    n = 1 << bits
    seq = O.gray_code_frames(n, 4)
    col_frames = seq[2: 2 + 2 * bits]
    g = np.zeros(n, np.int32)
    for b in range(bits):
        p, i = col_frames[2 * b][0], col_frames[2 * b + 1][0]
        g |= (p > i).astype(np.int32) << (bits - 1 - b)
    assert np.array_equal(O._gray_to_binary(g), np.arange(n))


# ---- Otsu cases where an OpenCV build other than the C path could diverge.
# The restatement is OpenCV's C getThreshVal_Otsu_8u; opencv-python wheels may dispatch to
# IPP's ippiComputeThreshold_Otsu, whose agreement is unpinned here.  These fix what the C
# recurrence returns (the GPU's otsu_wave / otsu_from_parts follow it, tests/test_gpu_parity.py).
def _hist(pairs):
    h = [0] * 256
    for v, c in pairs:
        h[v] += c
    return h


def cross_tie(h):
    """Exact-rational maxima of sigma at thresholds with DIFFERENT class splits (q1), i.e. a
    real tie, not a plateau of empty bins (which the strict '>' resolves to its first bin)."""
    n = sum(h)
    mu = Fraction(sum(i * c for i, c in enumerate(h)), n)
    mu1, q1, sig = Fraction(0), Fraction(0), []
    for i in range(256):
        p = Fraction(h[i], n)
        mu1 *= q1
        q1 += p
        q2 = 1 - q1
        if min(q1, q2) < EPS or max(q1, q2) > 1 - EPS:
            continue
        mu1 = (mu1 + i * p) / q1
        mu2 = (mu - q1 * mu1) / q2
        sig.append((q1 * q2 * (mu1 - mu2) ** 2, q1))
    if not sig:
        return False
    best = max(s for s, _ in sig)
    return len({q for s, q in sig if s == best}) > 1


OTSU_CASES = {
    # name: (histogram, value the C recurrence returns, exact-rational tie across splits?)
    "single_bin_0": (_hist([(0, 1000)]), 0.0, False),        # every bin skipped (q1 or q2 ~ 0)
    "single_bin_255": (_hist([(255, 1000)]), 0.0, False),
    "single_bin_128": (_hist([(128, 7)]), 0.0, False),
    "two_bins_0_255": (_hist([(0, 3), (255, 1)]), 0.0, False),   # plateau 0..254: first bin
    "symmetric_4": (_hist([(10, 5), (20, 5), (30, 5), (40, 5)]), 20.0, False),
    # {0, 100, 200} x 1: splitting after 0 or after 100 gives sigma = (2/9) * 150^2 exactly; in
    # sequential fp64 the second split's sigma rounds higher, so the C path returns 100 where
    # exact arithmetic (and any differently-ordered implementation) may return 0
    "exact_tie_3bins": (_hist([(0, 1), (100, 1), (200, 1)]), 100.0, True),
    "exact_tie_scaled": (_hist([(20, 333), (90, 333), (160, 333)]), 90.0, True),
}


@pytest.mark.parametrize("name", sorted(OTSU_CASES))
def test_otsu_edge_and_tie_cases(name):
    h, want, tie = OTSU_CASES[name]
    assert O.otsu_from_hist(h) == want
    assert cross_tie(h) == tie
    if not tie:
        assert float(otsu_exact(h)[0]) == want
