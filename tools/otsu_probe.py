#!/usr/bin/env python
"""Write the Otsu histograms tools/otsu_probe.hip times: white and clip(white - black) of a few
rendered C2 views (server/processing.py:63-72), uint32 [2 * views][256], to argv[1]."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from structured_light_for_3d_model_replication_amd import synth  # noqa: E402

rig = synth.default_rig(1920, 1080, 1920, 1080)
hs = []
for i in range(3):
    v = synth.render_view(rig, 50.0 * i, seed=i, n_present=2)
    w = v.frames[0].astype(np.int32)
    b = v.frames[1].astype(np.int32)
    hs.append(np.bincount(w.ravel(), minlength=256))
    hs.append(np.bincount(np.clip(w - b, 0, 255).ravel(), minlength=256))
# + shapes the C2 captures do not have (the probe checks every threshold against the host loop):
# narrow, sparse, one or two bins, flat, heavy tails, the full-1080p pixel count and small counts
rng = np.random.default_rng(7)
for k in range(40):
    h = np.zeros(256, np.int64)
    kind = k % 8
    if kind == 0:
        h[rng.integers(0, 256)] = 2073600
    elif kind == 1:
        a, b = sorted(rng.integers(0, 256, 2))
        h[a] += 1000000
        h[b] += 1073600
    elif kind == 2:
        h[:] = 8100
    elif kind == 3:
        lo = int(rng.integers(0, 200))
        h[lo:lo + int(rng.integers(2, 56))] = rng.integers(1, 50000, 1)[0]
    elif kind == 4:
        h[rng.integers(0, 256, 30)] += rng.integers(1, 100000, 30)
    elif kind == 5:
        h = (rng.pareto(1.5, 256) * 1000).astype(np.int64)
    elif kind == 6:
        h = rng.integers(0, 3, 256)
    else:
        x = np.arange(256)
        h = (30000 * np.exp(-0.5 * ((x - rng.integers(0, 256)) / rng.uniform(2, 40)) ** 2)).astype(np.int64)
    if h.sum() == 0:
        h[0] = 1
    hs.append(h)
np.stack(hs).astype(np.uint32).tofile(sys.argv[1] if len(sys.argv) > 1 else "/tmp/otsu_hists.bin")
