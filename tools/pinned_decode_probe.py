#!/usr/bin/env python
"""Host PNG decode (slg_png_gray8_decode) into pinned vs pageable memory, one thread, the same
1080p capture frames (PIL-written, as tools/e2e_files.py writes them): whether the destination
being page-locked host memory slows the decoder, whose un-filter reads back the previous output
row.  Prints one JSON line.   python tools/pinned_decode_probe.py [--frames 44] [--reps 3]"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=44)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import numpy as np
    import torch
    from PIL import Image
    from structured_light_for_3d_model_replication_amd import _native as N, synth
    rig = synth.default_rig(1920, 1080, 1920, 1080)
    v = synth.render_view(rig, 30.0, seed=3, n_present=a.frames)
    d = tempfile.mkdtemp()
    paths = []
    for i, f in enumerate(v.frames[: a.frames]):
        p = os.path.join(d, f"{i:02d}.png")
        Image.fromarray(np.asarray(f)).save(p)
        paths.append(os.fsencode(p))
    L = N.lib()
    W, H = 1920, 1080
    n = W * H
    pinned = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    pageable = np.empty(n, np.uint8)
    res = {}
    for rep in range(a.reps):
        for name, ptr in (("pinned", pinned.data_ptr()), ("pageable", pageable.ctypes.data)):
            t = time.perf_counter()
            for p in paths:
                rc = L.slg_png_gray8_decode(p, ctypes.c_void_p(ptr), n, W, H)
                assert rc == 0, rc
            res.setdefault(name, []).append(round((time.perf_counter() - t) / len(paths) * 1e3, 3))
    assert np.array_equal(pinned.numpy(), pageable)
    print(json.dumps({"ms_per_frame": res, "frames": len(paths),
                      "mb_per_frame_png": round(sum(os.path.getsize(p) for p in paths) / len(paths) / 1e6, 3)}))


if __name__ == "__main__":
    main()
