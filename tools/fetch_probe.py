#!/usr/bin/env python
"""Write the mask file tools/fetch_probe.hip reads: the valid mask of a rendered C2 view (bench.py's
view 0: 1920x1080, 11 + 10 bits, Otsu), decoded by the product's maps path on the GPU, one byte
per pixel.  Usage: python tools/fetch_probe.py <out.bin>"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from structured_light_for_3d_model_replication_amd import engine as E, synth
    rig = synth.default_rig(1920, 1080, 1920, 1080)
    v = synth.render_view(rig, view_deg=0.0, seed=0, n_present=44)
    dev = E.DeviceFrames(list(v.frames), v.texture)
    _, _, mask = E.Reconstructor(1080, 1920).decode(dev, E.DecodeConfig(1920, 1080, 11, 10, "otsu"))
    m = mask.cpu().numpy().astype("uint8")
    m.tofile(sys.argv[1])
    print(f"mask: {int(m.sum())} valid of {m.size} px -> {sys.argv[1]}")


if __name__ == "__main__":
    main()
