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
np.stack(hs).astype(np.uint32).tofile(sys.argv[1] if len(sys.argv) > 1 else "/tmp/otsu_hists.bin")
