"""Drop-in for the reconstruction half of ``server/sl_system.py`` (class ``SLSystem``).

* ``generate_cloud(scan_dir, calib_file)`` — the legacy single-view pipeline
  (``server/sl_system.py:491-702``): percentile/dynamic-range mask, every code bit, column-only
  triangulation, inline ASCII PLY.  Runs the same HIP kernels as ``ProcessingLogic`` with
  ``variant='slsystem'``.
* ``generate_patterns()`` — the Gray-code encoder (``server/sl_system.py:44-86``).
* ``calibration_tables(...)`` — the table geometry of ``calibrate_final`` (``:355-423``) for
  given intrinsics/extrinsics (the OpenCV solvers themselves are out of scope).

Projector window, capture and OpenCV calibration methods are hardware I/O and out of scope.
"""
from __future__ import annotations

import os

import numpy as np

from . import calibration
from . import engine as E
from . import ply as PLY
from . import processing as PR

SCREEN_WIDTH = 1920      # server/config.py:16
SCREEN_HEIGHT = 1080     # server/config.py:18
PROJ_VALUE = 200         # server/config.py:20
D_SAMPLE_PROJ = 1        # server/config.py:22


class SLSystem:
    def __init__(self):
        self.window_name = "Projector"

    def generate_patterns(self):
        """``[[col bit planes], [row bit planes]]`` of 0/1 uint8 images (sl_system.py:44-86):
        bit ``b`` (MSB first) of the binary-reflected Gray code of each column / row."""
        width, height = SCREEN_WIDTH // D_SAMPLE_PROJ, SCREEN_HEIGHT // D_SAMPLE_PROJ
        n_cols = int(np.ceil(np.log2(width)))
        n_rows = int(np.ceil(np.log2(height)))
        c = np.arange(width)
        r = np.arange(height)
        gc, gr = c ^ (c >> 1), r ^ (r >> 1)
        cols = [np.broadcast_to(((gc >> (n_cols - 1 - b)) & 1).astype(np.uint8)[None, :],
                                (height, width)).copy() for b in range(n_cols)]
        rows = [np.broadcast_to(((gr >> (n_rows - 1 - b)) & 1).astype(np.uint8)[:, None],
                                (height, width)).copy() for b in range(n_rows)]
        return [cols, rows]

    @staticmethod
    def calibration_tables(K1, K2, R, T, cam_size, dist=None):
        """Tables ``calibrate_final`` saves, for the configured projector size."""
        return calibration.build_tables(K1, K2, R, T, cam_size, (SCREEN_WIDTH, SCREEN_HEIGHT), dist)

    def generate_cloud(self, scan_dir, calib_file):
        """Decode + triangulate one scan folder and write ``<scan_dir>/<name>.ply``."""
        if not os.path.exists(calib_file):
            raise FileNotFoundError(f"Calibration file not found at {calib_file}")
        print(f"[Process] Processing {scan_dir} using {calib_file}...")
        import scipy.io
        data = scipy.io.loadmat(calib_file)
        if 'Oc' not in data:
            raise ValueError("Calibration file missing 'Oc'.")
        calib_data = {"Nc": data["Nc"], "Oc": data["Oc"], "wPlaneCol": data["wPlaneCol"],
                      "wPlaneRow": data["wPlaneRow"], "cam_K": data["cam_K"]}

        files = FR_discover(scan_dir)
        if len(files) < 4:
            raise ValueError("Not enough images in folder to decode.")
        cfg = E.DecodeConfig(1920, 1080, variant="slsystem")
        imgs, tex = PR.FR.load_frames(files, texture=True)
        dev = E.DeviceFrames(imgs, tex)
        # the reference's two steps (sl_system.py:666-669): maps (slg_decode), then the cloud
        # from the maps (slg_triangulate); the legacy path is not throughput-critical, and the
        # maps give the valid-pixel count the reference prints (sl_system.py:610)
        eng = PR._engine(dev.height, dev.width)
        print("Decoding Columns...")
        print("Decoding Rows...")
        col, row, mask = eng.decode(dev, cfg)
        print("Reconstructing 3D points...")
        print(f"Processing {int(mask.sum().item())} valid pixels...")
        dc = PR._device_calib(calib_data, dev.height, dev.width)
        P, C = eng.triangulate(col, row, mask, dev.texture_bgr(), dc, row_mode=0, xyz_f64=True).result()
        points, colors = P.cpu().numpy(), C.cpu().numpy()

        ply_name = os.path.basename(scan_dir) + ".ply"
        out_path = os.path.join(scan_dir, ply_name)
        print(f"Saving {len(points)} points to {out_path}...")
        PLY.write_ascii(out_path, points, colors)
        print(f"[Success] Generated {out_path}")


def FR_discover(scan_dir):
    """``generate_cloud``'s discovery order: ``*.png`` first, then ``*.bmp`` (sl_system.py:518-520)."""
    return PR.FR.discover(scan_dir, order=("png", "bmp"))
