"""The Otsu tail's speculative quotient (csrc/slgpu.hip: mu1_run<true>), restated with exactly
rounded fp64 arithmetic: m = fma(a, y, a * (fma(-q, y, 1) * y)) with y = RN(1/q) must be a
faithful a / q, RN(a / q) in practice, and the kernel's check RN(m + fma(-q, m, a) * y) must
always land on RN(a / q) (Markstein), so a miss is always caught and rerun exactly.  The chain
is OpenCV's getThreshVal_Otsu_8u mu1 recurrence (oracle/sl_oracle.py:otsu_from_hist) over the
unskipped run [lo, hi], which must be contiguous."""
from fractions import Fraction

import numpy as np
import pytest


def _fma(a, b, c):
    return float(Fraction(a) * Fraction(b) + Fraction(c))   # int / int true division: RN


def _chain(h):
    n = int(h.sum())
    scale = 1.0 / n
    eps = float(np.finfo(np.float32).eps)
    p = [float(x) * scale for x in h]
    ip = [i * p[i] for i in range(256)]
    q1, q1r = 0.0, []
    for i in range(256):
        q1 = q1 + p[i]
        q1r.append(q1)
    ok = [not (min(q, 1.0 - q) < eps or max(q, 1.0 - q) > 1.0 - eps) for q in q1r]
    run = [i for i in range(256) if ok[i]]
    if not run:
        return 0, 0
    lo, hi = run[0], run[-1]
    assert len(run) == hi - lo + 1                         # one contiguous run of unskipped bins
    mu1 = q_prev = 0.0
    misses = caught = 0
    for i in range(lo, hi + 1):
        a = mu1 * q_prev + ip[i]
        q = q1r[i]
        y = 1.0 / q
        m = _fma(a, y, a * (_fma(-q, y, 1.0) * y))
        exact = float(Fraction(a) / Fraction(q))
        assert abs(Fraction(m) - Fraction(a) / Fraction(q)) < abs(Fraction(np.spacing(exact)))   # faithful
        mc = _fma(_fma(-q, m, a), y, m)
        assert mc == exact
        misses += m != exact
        caught += mc != m
        mu1, q_prev = exact, q
    assert misses == caught
    return misses, caught


@pytest.mark.parametrize("seed", range(4))
def test_speculative_quotient_chain(seed):
    rng = np.random.default_rng(seed)
    hists = [rng.integers(0, 5000, 256), rng.poisson(rng.uniform(0, 3e4, 256)),
             np.bincount(rng.integers(0, 256, int(rng.integers(1000, 2_000_000))), minlength=256)]
    h = np.zeros(256, np.int64)
    h[rng.choice(256, 9, replace=False)] = rng.integers(1, 10 ** 6, 9)
    hists.append(h)
    for h in hists:
        _chain(np.asarray(h, np.int64))
