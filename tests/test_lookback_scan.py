"""The lone-view scan of csrc/slgpu.hip ``lookback_scan``, restated lane by lane in NumPy.

One wave reads the look-back words of up to 1024 tiles, 8 consecutive tiles per lane and 512
per block.  A word holds a tile's aggregate, or its inclusive prefix when the tile's own walk (or
tile 0) got there first.  The wave writes every tile's inclusive prefix.  The restatement
follows the kernel's order of operations: the lane-local segmented sums, the Hillis-Steele
segmented scan of the lane totals, the exclusive shift with the block carry, and the fix-up
pass.  It is checked against the sequential prefix sums for random mixes of aggregate and
inclusive words, tile counts that are not multiples of 8 or 512, and every tile as the scanner.
The GPU suite runs the kernel itself (``tests/test_gpu_instances.py``).
"""
import numpy as np
import pytest

PER = 8          # kScanPer
LANES = 64


def scan_restated(agg_words, inc_flags, tile):
    """Mirror of lookback_scan after the ticket: returns (inclusive prefix per tile as
    published or already held, the scanner's own inclusive prefix)."""
    tiles = len(agg_words)
    out = np.array(agg_words, dtype=np.uint64)
    carry, mine = np.uint64(0), None
    for c0 in range(0, tiles, LANES * PER):
        i0 = c0 + PER * np.arange(LANES)
        w = np.zeros((LANES, PER), np.uint64)
        inc = np.zeros((LANES, PER), bool)
        for k in range(PER):
            ok = i0 + k < tiles
            w[ok, k] = np.asarray(agg_words, np.uint64)[i0[ok] + k]
            inc[ok, k] = np.asarray(inc_flags)[i0[ok] + k]
        x = np.zeros(LANES, np.uint64)
        f = np.zeros(LANES, bool)
        for k in range(PER):
            x = np.where(inc[:, k], w[:, k], x + w[:, k])
            f = f | inc[:, k]
        sx, sf = x.copy(), f.copy()
        o = 1
        while o < LANES:
            xo = np.concatenate([np.zeros(o, np.uint64), sx[:-o]])     # __shfl_up: values before the step
            fo = np.concatenate([np.zeros(o, bool), sf[:-o]])
            upd = (np.arange(LANES) >= o) & ~sf
            sx = np.where(upd, sx + xo, sx)
            sf = np.where(upd, fo, sf)
            o <<= 1
        ex = np.concatenate([[np.uint64(0)], sx[:-1]])
        ef = np.concatenate([[False], sf[:-1]])
        ex = ex + np.where(ef, np.uint64(0), carry)
        x = ex.copy()
        for k in range(PER):
            x = np.where(inc[:, k], w[:, k], x + w[:, k])
            for lane in range(LANES):
                i = int(i0[lane]) + k
                if i < tiles:
                    if not inc[lane, k]:
                        out[i] = x[lane]
                    if i == tile:
                        mine = x[lane]
        carry = x[LANES - 1]
    return out, mine


@pytest.mark.parametrize("tiles", [1, 2, 7, 8, 9, 63, 64, 65, 507, 511, 512, 513, 1000, 1024])
def test_scan_equals_sequential_prefix(tiles):
    rng = np.random.default_rng(tiles)
    for trial in range(6):
        agg = rng.integers(0, 4097, tiles).astype(np.uint64)
        incl = np.cumsum(agg).astype(np.uint64)
        # which words already hold inclusive prefixes: none, a few, many, all (tile 0 always)
        p_inc = [0.0, 0.02, 0.3, 1.0, 0.1, 0.6][trial]
        inc = rng.random(tiles) < p_inc
        inc[0] = True
        words = np.where(inc, incl, agg)
        for tile in sorted({0, tiles - 1, tiles // 2, int(rng.integers(0, tiles))}):
            out, mine = scan_restated(words, inc, tile)
            assert np.array_equal(out, incl), (tiles, trial)
            assert mine == incl[tile]
            assert int(mine) - int(agg[tile]) == int(incl[tile] - agg[tile])      # the exclusive prefix
