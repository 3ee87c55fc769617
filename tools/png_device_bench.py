#!/usr/bin/env python
"""Device PNG decode throughput (slg_png_decode_device): a rendered C2 capture's 44 PNG frames
(PIL, as the tests write them), decoded in one launch as 1, 4 and 16 views' worth of frames.
Prints one JSON line: ms per launch and per view, against the host decoder (slg_png_gray8_decode
on 16 threads).  Run under rocprofv3 --kernel-trace --stats to split inflate from un-filter.
--libs a.so,b.so: one subprocess per library (SLG_LIB), alternating, --rounds times."""
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
            if hasattr(L, "slg_png_prof_read"):          # PNG_PROF build: counters of the last launch
                pfv = (ctypes.c_uint64 * 16)()
                L.slg_png_prof_read(pfv, 1)
                torch.cuda.synchronize()
                N.check(L.slg_png_decode_device(ctypes.c_void_p(d.data_ptr()), n, ctypes.c_void_p(status.data_ptr()),
                                                ctypes.c_void_p(s.cuda_stream)))
                torch.cuda.synchronize()
                L.slg_png_prof_read(pfv, 1)
                names = ["total", "build", "header", "copy", "flush", "lit", "match", "match_bytes", "blocks",
                         "slow", "symbols"]
                per = {k: pfv[i] / n for i, k in enumerate(names)}
                for k in ("total", "build", "header", "copy", "flush"):
                    per[k + "_ms"] = round(per.pop(k) * 1e-5, 3)    # 100 MHz ticks per stream -> ms
                per = {k: (round(v, 1) if not k.endswith("_ms") else v) for k, v in per.items()}
                per["ns_per_symbol_total"] = round(per["total_ms"] * 1e6 / max(per["symbols"], 1), 1)
                out[f"prof_views_{views}"] = per
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


def ab():
    import subprocess
    i = sys.argv.index("--libs") + 1                  # comma- or space-separated (tools/gpu.sh py=)
    libs = []
    while i < len(sys.argv) and not sys.argv[i].startswith("--"):
        libs += [x for x in sys.argv[i].split(",") if x]
        i += 1
    rounds = int(sys.argv[sys.argv.index("--rounds") + 1]) if "--rounds" in sys.argv else 2
    res = {lib: [] for lib in libs}
    for r in range(rounds):
        for lib in libs:
            env = dict(os.environ, SLG_LIB=lib)
            out = subprocess.run([sys.executable, os.path.abspath(__file__)], env=env, capture_output=True, text=True,
                                 timeout=600)
            if out.returncode != 0:
                print(out.stderr[-3000:], file=sys.stderr)
                raise SystemExit(f"{lib} failed")
            d = json.loads(out.stdout.strip().splitlines()[-1])
            res[lib].append(d)
            print(f"[png-ab] round {r} {lib}: " + json.dumps({k: d[k] for k in d if k.startswith(("views_16", "prof_views_16"))}), flush=True)
    print(json.dumps({lib: min(x["views_16"]["ms_per_view"] for x in v) for lib, v in res.items()}), flush=True)


if __name__ == "__main__":
    ab() if "--libs" in sys.argv else main()
