#!/usr/bin/env python
"""Device PNG decode throughput (slg_png_decode_device): a rendered C2 capture's 44 PNG frames
(PIL, as the tests write them), decoded in one launch as 1, 4 and 16 views' worth of frames.
Prints one JSON line: ms per launch and per view, against the host decoder (slg_png_gray8_decode
on 16 threads).  Run under rocprofv3 --kernel-trace --stats to split inflate from un-filter."""
from __future__ import annotations

import ctypes
import json
import os
import sys
import tempfile
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    from structured_light_for_3d_model_replication_amd import _native as N, synth
    L = N.lib()
    rig = synth.default_rig(1920, 1080, 1920, 1080)
    v = synth.render_view(rig, 0.0, seed=0, n_present=44)
    out = {}
    with tempfile.TemporaryDirectory() as tmp:
        paths = synth.write_capture(v, tmp)
        zs, infos = [], []
        for p in paths:
            cap = os.path.getsize(p) + 8
            buf = np.zeros(cap + 256, np.uint8)
            info = (ctypes.c_int32 * 4)()
            assert L.slg_png_zstream(os.fsencode(p), buf.ctypes.data_as(ctypes.c_void_p), cap, info) == 0
            zs.append(torch.from_numpy(buf).cuda())
            infos.append(tuple(info))
        W, H, C = infos[0][:3]
        raw_b = int(L.slg_png_raw_bytes(W, H, C))
        out["zbytes_per_frame"] = int(np.mean([i[3] for i in infos]))
        for views in (1, 4, 16):
            n = views * len(paths)
            raw = torch.empty(n * raw_b, dtype=torch.uint8, device="cuda")
            frames = torch.empty((n, H * W), dtype=torch.uint8, device="cuda")
            descs = (N.PngFrame * n)()
            for k in range(n):
                j = k % len(paths)
                descs[k] = N.PngFrame(z=zs[j].data_ptr(), zlen=infos[j][3], raw=raw.data_ptr() + k * raw_b,
                                      out=frames[k].data_ptr(), out_pitch=W, width=W, height=H, channels=C, reserved=0)
            d = torch.frombuffer(bytearray(ctypes.string_at(ctypes.addressof(descs), ctypes.sizeof(descs))),
                                 dtype=torch.uint8).cuda()
            status = torch.zeros(2 * n, dtype=torch.int32, device="cuda")
            s = torch.cuda.current_stream()
            times = []
            for rep in range(3):
                torch.cuda.synchronize()
                t = time.perf_counter()
                N.check(L.slg_png_decode_device(ctypes.c_void_p(d.data_ptr()), n, ctypes.c_void_p(status.data_ptr()),
                                                ctypes.c_void_p(s.cuda_stream)))
                torch.cuda.synchronize()
                times.append(time.perf_counter() - t)
            ok = bool((status.view(-1, 2)[:, 0] == 0).all().item())
            same = bool(torch.equal(frames[0].cpu(), torch.from_numpy(v.frames[0].reshape(-1))))
            out[f"views_{views}"] = {"frames": n, "ms_per_launch": round(1e3 * min(times), 2),
                                     "ms_per_view": round(1e3 * min(times) / views, 2), "status_ok": ok, "frame0_ok": same}
            print(json.dumps(out), file=sys.stderr, flush=True)
        # host decoder on 16 threads, one view
        bufs = np.zeros((len(paths), H * W), np.uint8)

        def one(k):
            return L.slg_png_gray8_decode(os.fsencode(paths[k]), bufs[k].ctypes.data_as(ctypes.c_void_p), H * W, W, H)
        with ThreadPoolExecutor(16) as ex:
            t = time.perf_counter()
            list(ex.map(one, range(len(paths))))
            out["host_16_threads_ms_per_view"] = round(1e3 * (time.perf_counter() - t), 2)
        t = time.perf_counter()
        one(0)
        out["host_1_thread_ms_per_frame"] = round(1e3 * (time.perf_counter() - t), 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
