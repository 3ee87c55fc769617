"""CPU tests of the host side: ABI exports, frame discovery/ingest, PLY bytes, calibration
tables, NEP-50 threshold semantics, decode planning and the synthetic renderer."""
import os
import re
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT, load_calibs
from oracle import sl_oracle as O

PKG = "structured_light_for_3d_model_replication_amd"


def header_exports():
    txt = open(os.path.join(ROOT, "include", "slgpu.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int32_t|int64_t|const char \*)\s*\*?(slg_\w+)\(", txt, re.M)))


def test_library_loads_and_exports_every_header_symbol():
    from structured_light_for_3d_model_replication_amd import build
    build.build_native()
    code = (
        "import ctypes, json, sys\n"
        f"import {PKG}._native as N\n"
        "L = N.lib()\n"
        f"names = {header_exports()!r}\n"
        "missing = [n for n in names if not hasattr(L, n)]\n"
        "print(json.dumps({'missing': missing, 'v': L.slg_version(), 'hip': N.loaded_hip_runtimes(),"
        " 'ws': L.slg_workspace_bytes(1920*1080)}))\n")
    out = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, check=True)
    import json
    r = json.loads(out.stdout.strip().splitlines()[-1])
    assert len(header_exports()) >= 9
    assert r["missing"] == [] and r["v"] == 2
    assert len(r["hip"]) == 1, r["hip"]          # one HIP runtime (torch's) in the process
    assert r["ws"] > 1920 * 1080 * 27


def test_capture_limits_rejected_before_any_launch():
    """The kernels address frames and texture with 32-bit buffer offsets (include/slgpu.h): a
    frame stack of 4 GiB or more, or an image of 1.43e9 pixels or more, is refused by the C ABI's
    argument check, before anything touches the GPU (fake, never dereferenced pointers)."""
    code = (
        "import ctypes, json\n"
        f"import {PKG}._native as N\n"
        "L = N.lib()\n"
        "dp = N.DecodeParams(proj_cols=1920, proj_rows=1080, n_sets_col=11, n_sets_row=11)\n"
        "out = {}\n"
        "for tag, h, w, stride, nf in (('stack', 1080, 1920, 1 << 29, 8), ('pixels', 40000, 40000, 1600000000, 4),\n"
        "                              ('ok_stack', 1080, 1920, 1 << 29, 7)):\n"
        "    cap = N.Capture(frames=4096, frame_stride=stride, n_frames=nf, height=h, width=w, texture=4096)\n"
        "    rc = L.slg_decode_stats(ctypes.byref(cap), ctypes.byref(dp), None, None)\n"
        "    out[tag] = [rc, L.slg_last_error().decode()]\n"
        "print(json.dumps(out))\n")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, check=True)
    import json
    res = json.loads(r.stdout.strip().splitlines()[-1])
    from structured_light_for_3d_model_replication_amd import _native as N
    assert res["stack"][0] == N.SLG_ERR_UNSUPPORTED and "4 GiB" in res["stack"][1]
    assert res["pixels"][0] == N.SLG_ERR_UNSUPPORTED and "1.43e9" in res["pixels"][1]
    # 7 x 512 MiB passes the capture check and stops at the NULL workspace instead
    assert res["ok_stack"][0] == N.SLG_ERR_INVALID and "NULL" in res["ok_stack"][1]


def test_every_fused_kernel_instance_is_in_the_code_object():
    """The fused kernel's instance table (``slg_kernel_table``, what pick_main can launch) is
    complete in the production build, and the library's own reading of its gfx950 code object
    agrees with llvm-readelf on the unbundled code objects (a missing instance would abort the
    HIP runtime at launch; the library now refuses it instead)."""
    code = (
        "import json\n"
        f"import {PKG}._native as N\n"
        "print(json.dumps(N.kernel_table()))\n")
    out = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, check=True)
    import json
    table = json.loads(out.stdout.strip().splitlines()[-1])
    assert len(table) == 42, len(table)       # 24 generic + 16 plan + 2 profiling instances
    assert all(table.values()), [k for k, v in table.items() if not v]
    llvm = "/opt/rocm/lib/llvm/bin"
    if not os.path.exists(os.path.join(llvm, "llvm-readelf")):
        pytest.skip("no llvm-readelf")
    import tempfile
    lib = os.path.join(ROOT, PKG, "libslgpu.so")
    with tempfile.TemporaryDirectory() as td:
        import shutil
        copy = os.path.join(td, "lib.so")           # (the unbundled files land beside the input)
        shutil.copy(lib, copy)
        subprocess.run([os.path.join(llvm, "llvm-objdump"), "--offloading", copy], cwd=td, capture_output=True,
                       check=True)
        syms = set()
        for f in os.listdir(td):
            if "gfx950" in f:
                r = subprocess.run([os.path.join(llvm, "llvm-readelf"), "--symbols", "-W", os.path.join(td, f)],
                                   capture_output=True, text=True, check=True)
                syms.update(line.split()[-1] for line in r.stdout.splitlines() if "main3_kernel" in line)
    assert set(table) <= syms, sorted(set(table) - syms)[:3]


def test_build_id_follows_source_content(tmp_path):
    """Build provenance: the library embeds the digest of its sources + flags; a content-only
    source change (mtime kept) makes needs_build() true, and the digest of the sources present
    is what _native.lib() demands of the product library."""
    import shutil
    from structured_light_for_3d_model_replication_amd import build as B
    from structured_light_for_3d_model_replication_amd import _native as N
    B.build_native()
    assert B.built_digest() == B.source_digest()
    assert not B.needs_build()
    assert N.lib().slg_build_id().decode() == B.BUILD_ID_PREFIX.decode() + B.source_digest()
    copies = []
    for p in B.SRCS:
        q = tmp_path / os.path.basename(p)
        shutil.copy2(p, q)
        copies.append(str(q))
    st = os.stat(copies[2])
    data = open(copies[2], "rb").read()
    with open(copies[2], "wb") as f:                 # same length, one byte changed, mtime restored
        f.write(data[:-2] + bytes([data[-2] ^ 1]) + data[-1:])
    os.utime(copies[2], ns=(st.st_atime_ns, st.st_mtime_ns))
    assert B.source_digest(copies) != B.source_digest()
    old = B.SRCS
    try:
        B.SRCS = copies
        assert B.needs_build()
    finally:
        B.SRCS = old
    assert not B.needs_build()


def test_ab_library_must_be_in_tree(tmp_path):
    """SLG_LIB (A/B builds) only accepts libraries inside the in-tree A/B build directories."""
    env = dict(os.environ, SLG_LIB=str(tmp_path / "x.so"))
    r = subprocess.run([sys.executable, "-c", f"import {PKG}._native"], cwd=ROOT, env=env, capture_output=True,
                       text=True)
    assert r.returncode != 0 and "A/B libraries must live in" in r.stderr


def test_exports_match_ctypes_table():
    from structured_light_for_3d_model_replication_amd import _native as N
    assert sorted(N.EXPORTS) == header_exports()


def test_ctypes_struct_layout_matches_header(tmp_path):
    """Every ctypes structure has the C compiler's size and field offsets for include/slgpu.h."""
    from structured_light_for_3d_model_replication_amd import _native as N
    import ctypes
    structs = {"slg_capture": N.Capture, "slg_decode_params": N.DecodeParams, "slg_calib": N.Calib,
               "slg_tri_params": N.TriParams, "slg_maps": N.Maps, "slg_cloud": N.Cloud,
               "slg_png_frame": N.PngFrame}
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{ROOT}/include/slgpu.h"', 'int main(void) {']
    for cname, cls in structs.items():
        lines.append(f'  printf("{cname} size %zu\\n", sizeof({cname}));')
        for f, _ in cls._fields_:
            lines.append(f'  printf("{cname} {f} %zu\\n", offsetof({cname}, {f}));')
    lines.append("  return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines) + "\n")
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c99", "-o", str(exe), str(src)], check=True)
    want = {}
    for line in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.splitlines():
        name, field, val = line.split()
        want[(name, field)] = int(val)
    for cname, cls in structs.items():
        assert ctypes.sizeof(cls) == want[(cname, "size")], cname
        for f, _ in cls._fields_:
            assert getattr(cls, f).offset == want[(cname, f)], (cname, f)


def test_discovery_orders(tmp_path):
    from structured_light_for_3d_model_replication_amd import frames as FR
    from PIL import Image
    for name in ("02.png", "01.png", "01.bmp", "02.bmp"):
        Image.fromarray(np.zeros((4, 4), np.uint8)).save(tmp_path / name)
    proc = FR.discover(str(tmp_path))                        # processing.py:52-54: bmp first
    sl = FR.discover(str(tmp_path), order=("png", "bmp"))    # sl_system.py:518-520: png first
    assert [os.path.basename(p) for p in proc] == ["01.bmp", "02.bmp"]
    assert [os.path.basename(p) for p in sl] == ["01.png", "02.png"]
    assert FR.discover(["b", "a"]) == ["b", "a"]              # lists are used as given


def test_gray_png_bmp_are_identity(tmp_path):
    from structured_light_for_3d_model_replication_amd import frames as FR
    from PIL import Image
    a = np.random.default_rng(0).integers(0, 256, (13, 17)).astype(np.uint8)
    for ext in ("png", "bmp"):
        p = str(tmp_path / f"x.{ext}")
        Image.fromarray(a, mode="L").save(p)
        assert np.array_equal(FR.imread_gray(p), a)
        bgr = FR.imread_bgr(p)
        assert bgr.shape == (13, 17, 3) and np.array_equal(bgr[..., 1], a)
    with pytest.raises(AttributeError):
        FR.imread_gray(str(tmp_path / "missing.png"))


def test_gray16_png_keeps_the_high_byte(tmp_path):
    """A 16-bit grayscale PNG read as cv2.imread(f, 0) / cv2.imread(f): OpenCV asks libpng for
    8-bit samples (png_set_strip_16), which keeps each sample's high byte -- v >> 8, not a
    rounded v / 257.  The values straddle every rounding boundary of the two."""
    from structured_light_for_3d_model_replication_amd import frames as FR
    from PIL import Image
    hi = np.arange(256, dtype=np.uint16).reshape(16, 16)
    a = (hi << 8) | np.array([0, 127, 128, 255], np.uint16)[np.arange(256).reshape(16, 16) % 4]
    p = str(tmp_path / "g16.png")
    Image.fromarray(a.astype(np.uint16)).save(p)
    assert Image.open(p).mode.startswith("I;16")              # really a 16-bit gray file
    assert np.array_equal(FR.imread_gray(p), hi.astype(np.uint8))
    assert np.array_equal(FR.imread_bgr(p), np.repeat(hi.astype(np.uint8)[..., None], 3, -1))


def test_needed_frames_matches_reference_reads():
    from structured_light_for_3d_model_replication_amd import processing as PR, engine as E
    cfg = E.DecodeConfig(1920, 1080, 3, 2)
    need = PR._needed_frames(46, cfg)
    assert need == [0, 1, 2, 3, 4, 5, 6, 7, 24, 25, 26, 27]
    need = PR._needed_frames(9, E.DecodeConfig(1920, 1080, 11, 11))
    assert need == [0, 1, 2, 3, 4, 5, 6, 7]                  # pair (8, 9) missing


def test_weak_scalar_follows_numpy_comparison():
    from structured_light_for_3d_model_replication_amd.engine import weak_scalar
    img = np.arange(256, dtype=np.float32)
    for thr in (40, 30.5, 7.25, 16777217, 0.1, np.float64(30.1), np.float32(12.7), np.int64(9)):
        want = img > thr
        got = img.astype(np.float64) > weak_scalar(thr)
        assert np.array_equal(want, got), thr


def test_ply_bytes_match_reference_writer(tmp_path):
    from structured_light_for_3d_model_replication_amd import ply
    rng = np.random.default_rng(3)
    P = rng.normal(0, 300, (500, 3))
    P[:9] = [[-0.0, 0.0, 1e-9], [0.00005, 0.00015, -0.00005], [1.23445, 2.5, -2.5],
             [1e6, -1e6, 123.45675], [0.12345, 0.98765, 5e-5],
             [0.03125, -0.03125, 2.25e-4],            # exact ties -> round half to even
             [5e-324, -5e-324, 1e20], [9.3e14, -9.3e14, 1e-300],
             [np.nan, np.inf, -np.inf]]
    C = rng.integers(0, 256, (500, 3)).astype(np.uint8)
    f = tmp_path / "a.ply"
    ply.write_ascii(str(f), P, C)
    assert f.read_bytes() == O.ply_bytes(P, C)
    ply.write_ascii(str(f), np.zeros((0, 3)), np.zeros((0, 3), np.uint8))
    assert f.read_bytes() == O.ply_bytes(np.zeros((0, 3)), np.zeros((0, 3), np.uint8))
    big = rng.uniform(-2e3, 2e3, (50000, 3))
    cb = rng.integers(0, 256, (50000, 3)).astype(np.uint8)
    for th in (1, 3, 8):                       # chunking across threads keeps the order
        ply.write_ascii(str(f), big, cb, threads=th)
        assert f.read_bytes() == O.ply_bytes(big, cb)


def test_calibration_tables_match_reference_calibrate_final():
    from structured_light_for_3d_model_replication_amd import synth
    ref = load_calibs()["rig"]
    mine = synth.default_rig(96, 64, 1920, 1080).tables()
    assert np.array_equal(mine["Nc"], ref["Nc"])           # bitwise: pinhole rays
    for k in ("wPlaneCol", "wPlaneRow"):                     # bitwise: stripe planes
        assert mine[k].shape == ref[k].shape
        assert np.array_equal(mine[k], ref[k]), (k, np.abs(mine[k] - ref[k]).max())
    assert np.array_equal(mine["Oc"], ref["Oc"]) and np.array_equal(mine["cam_K"], ref["cam_K"])


def test_fast_stripe_planes_within_4_ulps():
    """The opt-in batched plane generator against the bit-exact per-plane
    loop: <= 4 ulps everywhere (it is not the default: the loop matches calibrate_final bitwise)."""
    from structured_light_for_3d_model_replication_amd import calibration, synth
    rig = synth.default_rig(1920, 1080, 1920, 1080)
    exact = calibration.stripe_planes(rig.K2, rig.R, rig.T, 1920, 1080)
    fast = calibration.stripe_planes_fast(rig.K2, rig.R, rig.T, 1920, 1080)
    for a, b in zip(exact, fast):
        assert a.shape == b.shape
        assert np.all(np.abs(a - b) <= 4 * np.spacing(np.abs(a)))


def test_mat_round_trip(tmp_path):
    from structured_light_for_3d_model_replication_amd import calibration, synth
    t = synth.default_rig(32, 16, 1920, 1080).tables()
    p = str(tmp_path / "c.mat")
    calibration.save_mat(p, t)
    back = calibration.load_mat(p)
    for k in calibration.CALIB_KEYS:
        assert np.array_equal(back[k], t[k]), k


def test_synth_is_deterministic_and_decodes_to_ground_truth():
    from structured_light_for_3d_model_replication_amd import synth
    rig = synth.default_rig(80, 60, 1920, 1080)
    a = synth.render_view(rig, 15.0, seed=5)
    b = synth.render_view(rig, 15.0, seed=5)
    assert np.array_equal(a.frames, b.frames) and np.array_equal(a.texture, b.texture)
    col, row, mask = O.decode_processing(list(a.frames), thresh_mode="otsu")
    lit = a.lit & mask
    assert lit.sum() > 0.3 * lit.size
    assert np.array_equal(col[lit], a.proj_col[lit]) and np.array_equal(row[lit], a.proj_row[lit])


def test_generate_patterns_is_gray_code():
    from structured_light_for_3d_model_replication_amd.sl_system import SLSystem
    P = SLSystem().generate_patterns()
    assert len(P[0]) == 11 and len(P[1]) == 11
    seq = O.gray_code_frames(1920, 1080, 1)
    for b in range(11):
        assert np.array_equal(P[0][b], seq[2 + 2 * b])
        assert np.array_equal(P[1][b], seq[24 + 2 * b])


def test_run_view_folders_pipeline(tmp_path):
    """Batch-mode folder loop (processing.py:314-334) as read / reconstruct / write stages:
    every folder processed once and in order, errors isolated per folder and per stage,
    image-less folders skipped, a folder counted only after its PLY is written."""
    import threading
    from structured_light_for_3d_model_replication_amd import processing as PR
    names = ["a", "b_readfail", "c", "empty", "d_gpufail", "e_writefail", "f"]
    for n in names:
        (tmp_path / n).mkdir()
        if n != "empty":
            (tmp_path / n / "00.png").write_bytes(b"x")
    folders = [str(tmp_path / n) for n in names]
    main = threading.get_ident()
    seen = {"read": [], "rec": [], "write": []}

    def read(f):
        assert threading.get_ident() != main
        seen["read"].append(os.path.basename(f))
        if f.endswith("readfail"):
            raise ValueError("Not enough images (got 3, need at least 4).")
        return os.path.basename(f).upper()

    def rec(f, get_host):
        assert threading.get_ident() == main
        seen["rec"].append(os.path.basename(f))
        logs.append(f"-> Decoding {os.path.basename(f)}")     # the stage logs before the read resolves
        host = get_host()
        assert host == os.path.basename(f).upper()
        if f.endswith("gpufail"):
            raise RuntimeError("kernel failed")
        return host

    def write(f, res):
        assert threading.get_ident() != main
        seen["write"].append(res)
        if f.endswith("writefail"):
            raise OSError("disk full")
        return os.path.basename(f) + ".ply"

    logs = []
    ok = PR.run_view_folders(folders, logs.append, rec, read=read, write=write)
    assert ok == 3
    assert seen["read"] == [n for n in names if n != "empty"]
    assert seen["rec"] == ["a", "b_readfail", "c", "d_gpufail", "e_writefail", "f"]
    assert seen["write"] == ["A", "C", "E_WRITEFAIL", "F"]
    # reference order (processing.py:322-330): a folder's progress line, then its error
    assert [s.strip() for s in logs] == [
        "-> Decoding a",
        "-> Decoding b_readfail",
        "✔ Saved: a.ply",
        "❌ Error in b_readfail: Not enough images (got 3, need at least 4).",
        "-> Decoding c",
        "Skipping empty (No images found).",
        "-> Decoding d_gpufail",
        "✔ Saved: c.ply",
        "❌ Error in d_gpufail: kernel failed",
        "-> Decoding e_writefail",
        "-> Decoding f",
        "❌ Error in e_writefail: disk full",
        "✔ Saved: f.ply",
    ]


def _png_bytes(img, filters, interlace=0, depth=8, ctype=0, corrupt=False):
    """A PNG written by hand with the given per-row filter types (PNG spec §9 filters)."""
    import struct
    import zlib
    h, w = img.shape
    raw = bytearray()
    prev = np.zeros(w, np.int32)
    for y in range(h):
        cur = img[y].astype(np.int32)
        left = np.concatenate([[0], cur[:-1]])
        ul = np.concatenate([[0], prev[:-1]])
        f = filters[y % len(filters)]
        if f == 0:
            pred = np.zeros(w, np.int32)
        elif f == 1:
            pred = left
        elif f == 2:
            pred = prev
        elif f == 3:
            pred = (left + prev) >> 1
        else:
            p = left + prev - ul
            pa, pb, pc = abs(p - left), abs(p - prev), abs(p - ul)
            pred = np.where((pa <= pb) & (pa <= pc), left, np.where(pb <= pc, prev, ul))
        raw += bytes([f]) + ((cur - pred) & 255).astype(np.uint8).tobytes()
        prev = cur

    def chunk(t, d):
        crc = zlib.crc32(t + d) ^ (1 if corrupt and t == b"IDAT" else 0)
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", crc & 0xffffffff)
    ihdr = struct.pack(">IIBBBBB", w, h, depth, ctype, 0, 0, interlace)
    return (b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", ihdr) + chunk(b"tEXt", b"k\x00v")
            + chunk(b"IDAT", zlib.compress(bytes(raw))[:20]) + chunk(b"IDAT", zlib.compress(bytes(raw))[20:])
            + chunk(b"IEND", b""))


def test_png_gray8_fast_path_matches_general_decoder(tmp_path):
    """Native PNG ingest (slg_png_gray8_*): every row filter, split IDATs, ancillary chunks;
    identical to the general (PIL) decoder; other formats and corrupt files fall back."""
    from PIL import Image
    from structured_light_for_3d_model_replication_amd import build, frames as FR
    build.build_native()
    rng = np.random.default_rng(5)
    for (h, w) in ((23, 37), (1, 1), (64, 5)):
        img = rng.integers(0, 256, (h, w), dtype=np.uint8)
        img[: h // 2] = np.clip(img[: h // 2] // 8 + np.arange(w) * 3, 0, 255)   # some smooth rows
        for filters in ((0,), (1,), (2,), (3,), (4,), (4, 3, 2, 1, 0)):
            p = tmp_path / f"f{h}_{w}_{''.join(map(str, filters))}.png"
            p.write_bytes(_png_bytes(img, filters))
            fast = FR._png_gray8(str(p))
            assert fast is not None and np.array_equal(fast, img)
            assert np.array_equal(np.asarray(Image.open(p)), img)
            assert np.array_equal(FR.imread_gray(str(p)), img)
            assert np.array_equal(FR.imread_bgr(str(p)), np.repeat(img[..., None], 3, -1))
    # PIL-written capture frames (synthetic renderer's writer)
    a = rng.integers(0, 256, (40, 60), dtype=np.uint8)
    Image.fromarray(a).save(tmp_path / "pil.png")
    assert np.array_equal(FR._png_gray8(str(tmp_path / "pil.png")), a)
    # not handled here: colour, 16-bit, interlaced, corrupt -> general decoder
    Image.fromarray(np.stack([a] * 3, -1)).save(tmp_path / "rgb.png")
    Image.fromarray(a.astype(np.uint16) * 257).save(tmp_path / "g16.png")
    (tmp_path / "il.png").write_bytes(_png_bytes(a, (0,), interlace=1))
    (tmp_path / "bad.png").write_bytes(_png_bytes(a, (1,), corrupt=True))
    (tmp_path / "trunc.png").write_bytes(_png_bytes(a, (1,))[:-30])
    for n in ("rgb", "g16", "il", "bad", "trunc"):
        assert FR._png_gray8(str(tmp_path / f"{n}.png")) is None, n
    assert FR._png_gray8(str(tmp_path / "missing.png")) is None
    assert np.array_equal(FR.imread_gray(str(tmp_path / "rgb.png")),
                          FR._to_gray(Image.open(tmp_path / "rgb.png"), "rgb.png"))
    with pytest.raises(AttributeError):
        FR.imread_gray(str(tmp_path / "missing.png"))


def test_read_capture_native_png_matches_general_decoder(tmp_path, monkeypatch):
    """Frame ingest of a capture folder (processing.py:49-60,98-99,124): the native gray PNG fast
    path (texture replicated from frame 0's gray decode) equals the general decoder
    (slg_png_read, pinned to libpng) exactly."""
    from structured_light_for_3d_model_replication_amd import build, synth, engine as E
    from structured_light_for_3d_model_replication_amd import processing as PR, frames as FR
    build.build_native()
    rig = synth.default_rig(96, 64, 1920, 1080)
    v = synth.render_view(rig, 40.0, seed=3, n_present=20)
    synth.write_capture(v, str(tmp_path / "cap"))
    cfg = E.DecodeConfig(1920, 1080, 11, 11, "otsu")
    stack, tex = PR.read_capture(str(tmp_path / "cap"), cfg)
    monkeypatch.setattr(FR, "_png_gray8", lambda p: None)        # every frame the general way
    monkeypatch.setattr(FR, "_is_png_gray8", lambda p: False)
    stack2, tex2 = PR.read_capture(str(tmp_path / "cap"), cfg)
    assert np.array_equal(tex, tex2) and tex.shape == (64, 96, 3) and tex.dtype == np.uint8
    assert all((a is None and b is None) or np.array_equal(a, b) for a, b in zip(stack, stack2))
    assert np.array_equal(stack[0], v.frames[0])
    monkeypatch.setenv("SLG_DECODE_THREADS", "3")
    assert FR.decode_threads() == 3
