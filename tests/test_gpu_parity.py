"""GPU parity: the HIP path (through the C ABI) against the reference's golden vectors and the
oracle.  Integer/byte outputs (maps, mask, colours, order, counts) must be bit-exact; XYZ
must be bit-exact in the float64 mode and within 1e-4 relative (north star) in float32 mode.
"""
import os

import numpy as np
import pytest

from conftest import decode_kwargs, expected_cloud, golden_cases, load_calibs, load_case
from oracle import sl_oracle as O

pytestmark = pytest.mark.gpu

XYZ32_RTOL = 1e-4     # BASELINE.json north_star: XYZ within 1e-4 relative (fp32 vs float64)


@pytest.fixture(scope="module")
def mods():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a ROCm device")
    from structured_light_for_3d_model_replication_amd import engine as E, processing as PR, _native as N
    N.lib()
    return E, PR, N


def _cfg(E, p):
    if p["variant"] == "slsystem":
        return E.DecodeConfig(1920, 1080, variant="slsystem")
    kw = decode_kwargs(p)
    return E.DecodeConfig(kw.get("n_cols", 1920), kw.get("n_rows", 1080), kw.get("n_sets_col", 11),
                          kw.get("n_sets_row", 11), kw.get("thresh_mode", "otsu"),
                          kw.get("shadow_val", 40), kw.get("contrast_val", 10))


def _xyz32_close(got, want):
    got = np.asarray(got, np.float64)
    scale = np.maximum(np.abs(want), 1e-3)
    assert np.all(np.abs(got - want) <= XYZ32_RTOL * scale)


@pytest.mark.parametrize("name", golden_cases())
def test_decode_maps_bit_exact(name, mods):
    E, PR, N = mods
    z = load_case(name)
    dev = E.DeviceFrames(list(z["frames"]), z["texture"])
    eng = E.Reconstructor(dev.height, dev.width)
    cfg = _cfg(E, z["params"])
    if "error" in z:
        with pytest.raises(IndexError):
            eng.decode(dev, cfg)
        return
    col, row, mask = eng.decode(dev, cfg)
    shape = (dev.height, dev.width)
    assert np.array_equal(col.reshape(shape).cpu().numpy(), z["col"])
    assert np.array_equal(row.reshape(shape).cpu().numpy(), z["row"])
    assert np.array_equal(mask.reshape(shape).cpu().numpy().astype(bool), z["mask"])


@pytest.mark.parametrize("name", golden_cases())
@pytest.mark.parametrize("fused", [False, True])
def test_cloud_bit_exact_f64(name, fused, mods):
    E, PR, N = mods
    z = load_case(name)
    if "error" in z:
        pytest.skip("reference raises")
    import torch
    cal = load_calibs()[z["params"]["calib"]]
    dev = E.DeviceFrames(list(z["frames"]), z["texture"])
    eng = E.Reconstructor(dev.height, dev.width)
    dc = E.DeviceCalib(cal, dev.height, dev.width)
    cfg = _cfg(E, z["params"])
    for rm in (0, 1, 2):
        if f"P{rm}" not in z:
            continue
        if fused:
            out = eng.reconstruct(dev, cfg, dc, row_mode=rm, xyz_f64=True)
        else:
            t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).reshape(-1).astype(dt)).cuda()
            out = eng.triangulate(t(z["col"], np.int32), t(z["row"], np.int32),
                                  t(z["mask"], np.uint8), dev.texture, dc, row_mode=rm, xyz_f64=True)
        P, C = out.result()
        P, C = P.cpu().numpy(), C.cpu().numpy()
        Pw, Cw = expected_cloud(z, cal, rm)
        assert P.shape == Pw.shape, (rm, P.shape, Pw.shape)
        assert np.array_equal(P, Pw), f"row_mode {rm}: max |d| {np.abs(P - Pw).max()}"
        assert np.array_equal(C, Cw), f"row_mode {rm} colours"
        assert eng.error_flags() & 1 == 0


@pytest.mark.parametrize("name", ["proc_otsu_full", "proc_c2style", "proc_odd_geometry", "sl_full",
                                  "proc_oc_table", "proc_oc_krays", "proc_oc_raw"])
def test_cloud_f32_within_tolerance(name, mods):
    E, PR, N = mods
    z = load_case(name)
    cal = load_calibs()[z["params"]["calib"]]
    dev = E.DeviceFrames(list(z["frames"]), z["texture"])
    eng = E.Reconstructor(dev.height, dev.width)
    dc = E.DeviceCalib(cal, dev.height, dev.width)
    for rm in (0, 1, 2):
        if f"P{rm}" not in z:
            continue
        P, C = eng.reconstruct(dev, _cfg(E, z["params"]), dc, row_mode=rm, xyz_f64=False).result()
        assert P.dtype.itemsize == 4
        assert len(P) == len(z[f"P{rm}"])
        _xyz32_close(P.cpu().numpy(), z[f"P{rm}"])
        assert np.array_equal(C.cpu().numpy(), z[f"C{rm}"])


@pytest.mark.parametrize("name", ["proc_c2style", "proc_odd_geometry", "proc_manual_sets"])
def test_lookback_helper_path_bit_exact(name, mods, monkeypatch):
    """Force the look-back to compute unpublished predecessors itself (the progress guarantee
    used when tiles are dispatched out of order); results must not change."""
    E, PR, N = mods
    z = load_case(name)
    cal = load_calibs()[z["params"]["calib"]]
    dev = E.DeviceFrames(list(z["frames"]), z["texture"])
    eng = E.Reconstructor(dev.height, dev.width)
    dc = E.DeviceCalib(cal, dev.height, dev.width)
    monkeypatch.setenv("SLG_HELP_AFTER", "0")
    for rm in (0, 1, 2):
        P, C = eng.reconstruct(dev, _cfg(E, z["params"]), dc, row_mode=rm, xyz_f64=True).result()
        assert np.array_equal(P.cpu().numpy(), z[f"P{rm}"]) and np.array_equal(C.cpu().numpy(), z[f"C{rm}"])


def test_ray_table_paths_agree(mods):
    """Nc gathered from the table == recomputed pinhole rays (bitwise), and the table is
    detected as the pinhole one."""
    E, PR, N = mods
    z = load_case("proc_otsu_full")
    cal = load_calibs()["rig"]
    dev = E.DeviceFrames(list(z["frames"]), z["texture"])
    eng = E.Reconstructor(dev.height, dev.width)
    d_pin = E.DeviceCalib(cal, dev.height, dev.width)
    d_tab = E.DeviceCalib(cal, dev.height, dev.width, keep_table=True)
    assert d_pin.table_is_pinhole and d_pin.ray_mode == N.RAYS_PINHOLE
    assert d_tab.ray_mode == N.RAYS_TABLE
    cfg = _cfg(E, z["params"])
    a = eng.reconstruct(dev, cfg, d_pin, 1).result()[0].cpu().numpy()
    b = eng.reconstruct(dev, cfg, d_tab, 1).result()[0].cpu().numpy()
    assert np.array_equal(a, b) and np.array_equal(a, z["P1"])
    # a perturbed table is not the pinhole one and must be gathered
    cal2 = dict(cal)
    cal2["Nc"] = cal["Nc"].copy()
    cal2["Nc"][0, 7] = np.nextafter(cal2["Nc"][0, 7], 1.0)
    d2 = E.DeviceCalib(cal2, dev.height, dev.width)
    assert not d2.table_is_pinhole and d2.ray_mode == N.RAYS_TABLE


def test_dropin_file_api_matches_oracle(tmp_path, mods):
    """ProcessingLogic._gray_decode on PNG files + _reconstruct_point_cloud, vs the oracle."""
    E, PR, N = mods
    from structured_light_for_3d_model_replication_amd import synth
    rig = synth.default_rig(160, 120, 1920, 1080)
    v = synth.render_view(rig, 33.0, seed=3)
    files = synth.write_capture(v, str(tmp_path / "scan"))
    cal = rig.tables()
    col, row, mask, tex = PR.ProcessingLogic._gray_decode(str(tmp_path / "scan"), n_sets_col=10, n_sets_row=9)
    oc, orow, om = O.decode_processing(list(v.frames), n_sets_col=10, n_sets_row=9)
    assert np.array_equal(col, oc) and np.array_equal(row, orow) and np.array_equal(mask, om)
    assert tex.shape == (120, 160, 3) and np.array_equal(tex[..., 0], v.frames[0])
    for rm in (0, 1, 2):
        P, C = PR.ProcessingLogic._reconstruct_point_cloud(col, row, mask, tex, cal, row_mode=rm)
        Po, Co = O.reconstruct_processing(oc, orow, om, tex, cal, row_mode=rm)
        assert P.dtype == np.float64 and np.array_equal(P, Po) and np.array_equal(C, Co)
    assert PR.ProcessingLogic._reconstruct_point_cloud(col, row, mask, tex, cal, row_mode=3) is None
    with pytest.raises(ValueError, match="Not enough images"):
        PR.ProcessingLogic._gray_decode(files[:3])


def test_process_multi_ply_batch(tmp_path, mods):
    """Batch mode end to end: one PLY per view folder, byte-identical to the oracle's writer,
    a bad folder is reported and skipped (processing.py:319-334)."""
    E, PR, N = mods
    from structured_light_for_3d_model_replication_amd import synth, calibration
    rig = synth.default_rig(128, 96, 1920, 1080)
    calibration.save_mat(str(tmp_path / "calib.mat"), rig.tables())
    root = tmp_path / "obj"
    views = {}
    for k, ang in enumerate((0.0, 90.0)):
        v = synth.render_view(rig, ang, seed=100 + k)
        d = root / f"obj_{int(ang)}deg_scan"
        synth.write_capture(v, str(d))
        views[d] = v
    bad = root / "bad_scan"
    synth.write_capture(synth.render_view(rig, 0.0, seed=9, n_present=3), str(bad))
    (root / "empty").mkdir()
    logs = []
    PR.ProcessingLogic.process_multi_ply(str(tmp_path / "calib.mat"), str(root), "batch",
                                         log_callback=logs.append, n_sets_col=11, n_sets_row=10)
    cal = calibration.load_mat(str(tmp_path / "calib.mat"))
    for d, v in views.items():
        c, r, m = O.decode_processing(list(v.frames), n_sets_col=11, n_sets_row=10)
        tex = np.repeat(v.frames[0][..., None], 3, -1)
        P, C = O.reconstruct_processing(c, r, m, tex, cal, row_mode=1)
        assert (d / f"{d.name}.ply").read_bytes() == O.ply_bytes(P, C)
    assert any("Error in bad_scan" in s and "Not enough images" in s for s in logs)
    # the reference logs a folder's progress line before its error (processing.py:322-330)
    i_dec = next(i for i, s in enumerate(logs) if "Decoding folder 'bad_scan'" in s)
    i_err = next(i for i, s in enumerate(logs) if "Error in bad_scan" in s)
    assert i_dec < i_err
    assert any("Skipping empty" in s for s in logs)
    assert logs[-1].startswith("=== Batch Complete: 2/4 succeeded")


def test_sharded_batch_single_process(tmp_path, mods):
    """The multi-GPU batch entry (``distributed.process_batch_sharded``) with no process group:
    the same read / GPU / write pipeline as batch mode, PLY bytes equal to the oracle's, a
    bad folder isolated, the job-wide summary line last."""
    E, PR, N = mods
    from structured_light_for_3d_model_replication_amd import synth, calibration, distributed as D
    rig = synth.default_rig(160, 120, 1920, 1080)
    calibration.save_mat(str(tmp_path / "calib.mat"), rig.tables())
    root = tmp_path / "obj"
    views = {}
    for k, ang in enumerate((0.0, 120.0, 240.0)):
        v = synth.render_view(rig, ang, seed=200 + k)
        d = root / f"v{k}"
        synth.write_capture(v, str(d))
        views[d] = v
    synth.write_capture(synth.render_view(rig, 0.0, seed=9, n_present=3), str(root / "bad"))
    logs = []
    ok = D.process_batch_sharded(str(tmp_path / "calib.mat"), str(root), log_callback=logs.append,
                                 n_sets_col=11, n_sets_row=11, row_mode=1)
    assert ok == 3
    cal = calibration.load_mat(str(tmp_path / "calib.mat"))
    for d, v in views.items():
        c, r, m = O.decode_processing(list(v.frames), n_sets_col=11, n_sets_row=11)
        tex = np.repeat(v.frames[0][..., None], 3, -1)
        P, C = O.reconstruct_processing(c, r, m, tex, cal, row_mode=1)
        assert (d / f"{d.name}.ply").read_bytes() == O.ply_bytes(P, C)
    assert any("Error in bad" in s and "Not enough images" in s for s in logs)
    assert logs[-1] == "=== Batch Complete: 3/4 succeeded ==="


def test_generate_cloud_legacy(tmp_path, mods, capsys):
    E, PR, N = mods
    from structured_light_for_3d_model_replication_amd import synth, calibration
    from structured_light_for_3d_model_replication_amd.sl_system import SLSystem
    rig = synth.default_rig(120, 80, 1920, 1080)
    calibration.save_mat(str(tmp_path / "c.mat"), rig.tables())
    v = synth.render_view(rig, 45.0, seed=4)
    synth.write_capture(v, str(tmp_path / "scanA"))
    SLSystem().generate_cloud(str(tmp_path / "scanA"), str(tmp_path / "c.mat"))
    cal = calibration.load_mat(str(tmp_path / "c.mat"))
    c, r, m = O.decode_slsystem(list(v.frames))
    P, C = O.reconstruct_slsystem(c, r, m, np.repeat(v.frames[0][..., None], 3, -1), cal)
    assert (tmp_path / "scanA" / "scanA.ply").read_bytes() == O.ply_bytes(P, C)
    with pytest.raises(FileNotFoundError):
        SLSystem().generate_cloud(str(tmp_path / "scanA"), str(tmp_path / "nope.mat"))


@pytest.mark.parametrize("cam,proj,nsets,thresh", [
    ((1920, 1080), (1920, 1080), (11, 10), "otsu"),      # C2
    ((1280, 720), (1024, 1080), (10, 11), "otsu"),       # C1 geometry
    ((1921, 1079), (1920, 1080), (8, 7), "manual"),      # ragged size, coarse codes
])
def test_full_size_parity(cam, proj, nsets, thresh, mods):
    """BASELINE-size views: maps + f64 cloud equal the oracle, and decoded codes equal the
    renderer's ground truth on lit, valid pixels (size-independent property)."""
    E, PR, N = mods
    from structured_light_for_3d_model_replication_amd import synth
    rig = synth.default_rig(*cam, *proj)
    n_present = 44 if proj == (1920, 1080) and nsets == (11, 10) else (22 if proj[0] == 1024 else None)
    v = synth.render_view(rig, 10.0, seed=7, n_present=n_present)
    cal = rig.tables()
    kw = dict(n_cols=proj[0], n_rows=proj[1], n_sets_col=nsets[0], n_sets_row=nsets[1], thresh_mode=thresh)
    dev = E.DeviceFrames(list(v.frames), v.texture)
    eng = E.Reconstructor(dev.height, dev.width)
    cfg = E.DecodeConfig(proj[0], proj[1], nsets[0], nsets[1], thresh)
    col, row, mask = eng.decode(dev, cfg)
    oc, orow, om = O.decode_processing(list(v.frames), **kw)
    shape = (cam[1], cam[0])
    col, row, mask = (col.reshape(shape).cpu().numpy(), row.reshape(shape).cpu().numpy(),
                      mask.reshape(shape).cpu().numpy().astype(bool))
    assert np.array_equal(col, oc) and np.array_equal(row, orow) and np.array_equal(mask, om)
    if nsets == (11, 10) or nsets == (10, 11):
        lit = v.lit & mask
        assert np.array_equal(col[lit], v.proj_col[lit])
    dc = E.DeviceCalib(cal, dev.height, dev.width)
    rm = 1 if proj[0] == 1920 else 0
    P, C = eng.reconstruct(dev, cfg, dc, rm, xyz_f64=True).result()
    Po, Co = O.reconstruct_processing(oc, orow, om, v.texture, cal, row_mode=rm)
    assert np.array_equal(P.cpu().numpy(), Po) and np.array_equal(C.cpu().numpy(), Co)
    assert eng.error_flags() & 1 == 0


@pytest.mark.parametrize("rm", [0, 2])
def test_full_size_row_modes(rm, mods):
    """C2 geometry at full size in row_mode 0 and 2 (the col + row clouds; row planes nearly
    parallel to the rays, the ill-conditioned case): the fused path and the maps-in
    triangulation both equal the oracle bit for bit in f64, and within XYZ32_RTOL in f32."""
    E, PR, N = mods
    import torch
    from structured_light_for_3d_model_replication_amd import synth
    rig = synth.default_rig(1920, 1080, 1920, 1080)
    v = synth.render_view(rig, 200.0, seed=21, n_present=44)
    cal = rig.tables()
    dev = E.DeviceFrames(list(v.frames), v.texture)
    eng = E.Reconstructor(dev.height, dev.width)
    cfg = E.DecodeConfig(1920, 1080, 11, 10, "otsu")
    dc = E.DeviceCalib(cal, dev.height, dev.width)
    oc, orow, om = O.decode_processing(list(v.frames), n_sets_col=11, n_sets_row=10)
    Po, Co = O.reconstruct_processing(oc, orow, om, v.texture, cal, row_mode=rm)
    assert len(Po) > 500_000
    P, C = eng.reconstruct(dev, cfg, dc, rm, xyz_f64=True).result()
    assert np.array_equal(P.cpu().numpy(), Po) and np.array_equal(C.cpu().numpy(), Co)
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dt).ravel()).cuda()
    P, C = eng.triangulate(t(oc, np.int32), t(orow, np.int32), t(om, np.uint8), dev.texture, dc,
                           row_mode=rm, xyz_f64=True).result()
    assert np.array_equal(P.cpu().numpy(), Po) and np.array_equal(C.cpu().numpy(), Co)
    P, C = eng.reconstruct(dev, cfg, dc, rm, xyz_f64=False).result()
    assert len(P) == len(Po) and np.array_equal(C.cpu().numpy(), Co)
    _xyz32_close(P.cpu().numpy(), Po)


def test_c4_full_size_parity(mods):
    """BASELINE configs[3] (C4): 6000x4000 capture, projector 3840x2160 (12 + 12 bits, 50
    frames), Otsu, row_mode 1.  Maps and the f64 cloud equal the oracle bit for bit, the f32
    cloud is within XYZ32_RTOL, and the decoded codes equal the renderer's ground truth on lit,
    valid pixels (size-independent property)."""
    E, PR, N = mods
    from structured_light_for_3d_model_replication_amd import synth
    rig = synth.default_rig(6000, 4000, 3840, 2160)
    v = synth.render_view(rig, 30.0, seed=11)
    assert v.frames.shape == (50, 4000, 6000)
    cal = rig.tables()
    dev = E.DeviceFrames(list(v.frames), v.texture)
    eng = E.Reconstructor(dev.height, dev.width)
    cfg = E.DecodeConfig(3840, 2160, 12, 12, "otsu")
    col, row, mask = eng.decode(dev, cfg)
    oc, orow, om = O.decode_processing(list(v.frames), n_cols=3840, n_rows=2160, n_sets_col=12, n_sets_row=12)
    shape = (4000, 6000)
    col, row, mask = (col.reshape(shape).cpu().numpy(), row.reshape(shape).cpu().numpy(),
                      mask.reshape(shape).cpu().numpy().astype(bool))
    assert np.array_equal(col, oc) and np.array_equal(row, orow) and np.array_equal(mask, om)
    lit = v.lit & mask
    assert lit.sum() > 1_000_000
    assert np.array_equal(col[lit], v.proj_col[lit]) and np.array_equal(row[lit], v.proj_row[lit])
    dc = E.DeviceCalib(cal, dev.height, dev.width)
    Po, Co = O.reconstruct_processing(oc, orow, om, v.texture, cal, row_mode=1)
    P, C = eng.reconstruct(dev, cfg, dc, 1, xyz_f64=True).result()
    assert np.array_equal(P.cpu().numpy(), Po) and np.array_equal(C.cpu().numpy(), Co)
    P, C = eng.reconstruct(dev, cfg, dc, 1, xyz_f64=False).result()
    assert len(P) == len(Po) and np.array_equal(C.cpu().numpy(), Co)
    _xyz32_close(P.cpu().numpy(), Po)
    assert eng.error_flags() & 1 == 0


def test_percentile_thresholds_large(mods):
    """Legacy mask thresholds at 6000x4000 (n > 2**24: NumPy's float32 index rounding)."""
    E, PR, N = mods
    import torch
    H, W = 4000, 6000
    g = torch.Generator().manual_seed(1)
    black = torch.randint(0, 30, (H, W), generator=g, dtype=torch.uint8)
    white = torch.clamp(black.int() + torch.randint(0, 200, (H, W), generator=g), 0, 255).to(torch.uint8)
    frames = torch.stack([white, black, white, black]).cuda()
    dev = E.DeviceFrames(frames)
    eng = E.Reconstructor(H, W)
    col, row, mask = eng.decode(dev, E.DecodeConfig(variant="slsystem"))
    want = O.mask_percentile(white.numpy(), black.numpy())
    assert np.array_equal(mask.reshape(H, W).cpu().numpy().astype(bool), want)
    ts, tc = eng.thresholds()
    nf = np.percentile(black.numpy().astype(np.float32), 95)
    assert np.float32(ts) == np.float32(nf * 1.5)


def test_repeated_calls_and_streams(mods):
    """Workspace re-arming across calls and concurrent streams with separate engines."""
    E, PR, N = mods
    import torch
    z = load_case("proc_c2style")
    cal = load_calibs()["rig"]
    dev = E.DeviceFrames(list(z["frames"]), z["texture"])
    engs = [E.Reconstructor(dev.height, dev.width) for _ in range(2)]
    dc = E.DeviceCalib(cal, dev.height, dev.width)
    cfg = _cfg(E, z["params"])
    streams = [torch.cuda.Stream() for _ in range(2)]
    outs = []
    for it in range(6):
        k = it % 2
        with torch.cuda.stream(streams[k]):
            outs.append(engs[k].reconstruct(dev, cfg, dc, 1, xyz_f64=True))
    torch.cuda.synchronize()
    for o in outs:
        P, C = o.result()
        assert np.array_equal(P.cpu().numpy(), z["P1"]) and np.array_equal(C.cpu().numpy(), z["C1"])


def test_batch_api_matches_single_view(mods):
    """slg_reconstruct_batch (one batched stats launch + back-to-back fused kernels) gives
    every view's cloud bit-exactly, including a batch larger than one stats launch (16)."""
    E, PR, N = mods
    import torch
    names = ["proc_otsu_full", "proc_c2style", "proc_missing_odd", "proc_flat_ties", "proc_manual_float"]
    cal = load_calibs()["rig"]
    zs = [load_case(n) for n in names]
    H, W = zs[0]["mask"].shape
    dc = E.DeviceCalib(cal, H, W)
    for reps in (1, 4):                                   # 5 and 20 views
        seq = zs * reps
        eng = E.BatchReconstructor(H, W, len(seq))
        frames = [E.DeviceFrames(list(z["frames"]), z["texture"]) for z in seq]
        # one decode config per batch: run the Otsu ones together, manual separately
        for cfg_name in ("otsu",):
            idx = [k for k, z in enumerate(seq) if z["params"].get("thresh_mode", "otsu") == cfg_name
                   and z["params"].get("n_sets_col", 11) == 11 and z["params"].get("n_sets_row", 11) == 11]
            fr = [frames[k] for k in idx]
            outs = [E.Cloud(H * W, 1, True) for _ in idx]
            eng.run(eng.prepare(fr, E.DecodeConfig(1920, 1080, 11, 11, "otsu"), dc, outs, row_mode=1))
            torch.cuda.synchronize()
            for k, o in zip(idx, outs):
                P, C = o.result()
                assert np.array_equal(P.cpu().numpy(), seq[k]["P1"]), names[k % len(names)]
                assert np.array_equal(C.cpu().numpy(), seq[k]["C1"])


def test_batch_pipelined_matches_golden(mods):
    """BatchReconstructor.run_pipelined: stats of batch k+1 on a side stream while batch k's
    fused launch runs (alternating workspace slots); ragged batches, views with different
    frame counts in one launch, and a batch spanning two launches (> 16 views)."""
    E, PR, N = mods
    import torch
    names = ["proc_otsu_full", "proc_c2style", "proc_missing_odd", "proc_flat_ties", "proc_manual_float"]
    cal = load_calibs()["rig"]
    zs = [load_case(n) for n in names]
    H, W = zs[0]["mask"].shape
    dc = E.DeviceCalib(cal, H, W)
    cfg = E.DecodeConfig(1920, 1080, 11, 11, "otsu")
    seq = [z for z in zs * 6 if z["params"].get("thresh_mode", "otsu") == "otsu"
           and z["params"].get("n_sets_col", 11) == 11 and z["params"].get("n_sets_row", 11) == 11]
    assert len({z["frames"].shape[0] for z in seq}) > 1        # mixed frame counts per launch
    frames = [E.DeviceFrames(list(z["frames"]), z["texture"]) for z in seq]
    assert len(seq) == 18
    for mode, sizes in (("overlap", [7, 7, 4]), ("overlap", [18]), ("fused", [7, 7, 4]),
                        ("fused", [5, 6, 4, 3]), ("fused", [3, 4, 6, 5]), ("fused", [18])):
        eng = E.BatchReconstructor(H, W, max(sizes), slots=2)
        outs, batches, j = [], [], 0
        for n in sizes:
            o = [E.Cloud(H * W, 1, True) for _ in range(n)]
            batches.append(eng.prepare(frames[j:j + n], cfg, dc, o, row_mode=1, slot=len(batches) % 2))
            outs += o
            j += n
        s_main, s_stats = torch.cuda.Stream(), torch.cuda.Stream()
        eng.run_pipelined(batches, s_main, s_stats, mode=mode)
        torch.cuda.synchronize()
        for z, o in zip(seq[:j], outs):
            P, C = o.result()
            assert np.array_equal(P.cpu().numpy(), z["P1"]) and np.array_equal(C.cpu().numpy(), z["C1"]), (mode, sizes)


@pytest.mark.parametrize("hw", [(1080, 1920), (999, 1001), (37, 53)])
def test_partial_histograms_match_frame_stats(mods, hw):
    """Otsu thresholds from the per-tile partial histograms a fused launch computes for the
    batch after next (slg_decode_triangulate_batch_next + slg_decode_stats_partials_batch)
    equal those of the regular stats pass over the frames -- the histogram and the Otsu
    search are exact, so the (float) thresholds are compared bit for bit.  Pixel counts that
    are not multiples of 2048 exercise the zero padding of the last tile."""
    E, PR, N = mods
    import torch
    H, W = hw
    rng = np.random.default_rng(H * 7 + W)
    nv = 3
    frames = []
    for v in range(nv):
        white = np.clip(rng.normal(120 + 30 * v, 60, (H, W)), 0, 255).astype(np.uint8)
        white[: H // 3] = rng.integers(0, 12, (H // 3, W), dtype=np.uint8)        # dark background
        black = np.clip(white.astype(np.int16) - rng.integers(0, 90, (H, W)), 0, 255).astype(np.uint8)
        pats = [rng.integers(0, 256, (H, W), dtype=np.uint8) for _ in range(4)]
        tex = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
        frames.append(E.DeviceFrames([white, black] + pats, tex))
    cfg = E.DecodeConfig(1920, 1080, 1, 1, "otsu")
    from structured_light_for_3d_model_replication_amd import synth
    dc = E.DeviceCalib(synth.default_rig(W, H, 1920, 1080).tables(), H, W)
    eng = E.BatchReconstructor(H, W, nv, slots=1)
    outs = [E.Cloud(H * W, 1, False) for _ in range(nv)]
    pb = eng.prepare(frames, cfg, dc, outs, row_mode=1, slot=0)
    eng.stats(pb)
    torch.cuda.synchronize()
    fields = lambda v: torch.cat([eng.header(0, v)[3088:3096], eng.header(0, v)[3104:3120]])   # smin cmin thr_s thr_c
    want = [fields(v).clone() for v in range(nv)]
    ref = [(int(np.frombuffer(w.cpu().numpy().tobytes()[:4], np.int32)[0])) for w in want]
    eng.main_next(pb, pb)                            # carry the same captures as "batch after next"
    for v in range(nv):                              # poison the thresholds the partials must restore
        eng.header(0, v)[3088:3120] = 0x55
    eng.stats_partials(pb)
    torch.cuda.synchronize()
    for v in range(nv):
        assert torch.equal(fields(v), want[v]), (v, ref[v])
    assert any(r > 0 for r in ref)
    # the same thresholds from the finishing workgroups of a later fused launch on one stream
    # (slg_decode_triangulate_batch_carry): slot 1 runs its own batch and finishes slot 0's
    eng2 = E.BatchReconstructor(H, W, nv, slots=2)
    pb0 = eng2.prepare(frames, cfg, dc, outs, row_mode=1, slot=0)
    outs1 = [E.Cloud(H * W, 1, False) for _ in range(nv)]
    pb1 = eng2.prepare(frames, cfg, dc, outs1, row_mode=1, slot=1)
    eng2.stats(pb0)
    eng2.stats(pb1)
    eng2.main_carry(pb0, pb0, None)                  # carries slot 0's own captures
    for v in range(nv):
        eng2.header(0, v)[3088:3120] = 0x55
    eng2.main_carry(pb1, None, pb0)                  # finishes slot 0 at the front of its grid
    torch.cuda.synchronize()
    fields2 = lambda v: torch.cat([eng2.header(0, v)[3088:3096], eng2.header(0, v)[3104:3120]])
    for v in range(nv):
        assert torch.equal(fields2(v), want[v]), v
    eng2.main(pb0)                                   # the finished slot is armed: its launch works
    torch.cuda.synchronize()
    for o, o1 in zip(outs, outs1):
        assert torch.equal(o.result()[0], o1.result()[0])


@pytest.mark.parametrize("name,shape", [("single_bin_0", (25, 40)), ("single_bin_255", (25, 40)),
                                        ("exact_tie_scaled", (27, 37))])
def test_otsu_edge_and_tie_thresholds(name, shape, mods):
    """The GPU Otsu (stats pass) on the KAT histograms of tests/test_oracle_kat.py: a single
    non-empty bin at 0 / 255, and an exact sigma tie between two splits that sequential fp64
    resolves to the second (OpenCV's C getThreshVal_Otsu_8u order)."""
    E, PR, N = mods
    import torch
    from test_oracle_kat import OTSU_CASES
    h, want, _ = OTSU_CASES[name]
    vals = np.repeat(np.arange(256), h).astype(np.uint8)
    assert vals.size == shape[0] * shape[1]
    white = np.random.default_rng(5).permutation(vals).reshape(shape)
    black = np.zeros(shape, np.uint8)
    frames = torch.from_numpy(np.stack([white, black, white, black])).cuda()
    dev = E.DeviceFrames(frames)
    eng = E.Reconstructor(*shape)
    eng.stats(dev, E.DecodeConfig(1920, 1080, 11, 11, "otsu"))
    torch.cuda.synchronize()
    ts, tc = eng.thresholds()
    assert (ts, tc) == (want, want) == (O.otsu_threshold(white), O.otsu_threshold(white))


def _otsu_images(kind, rng, shape):
    """white / black captures whose white and clip(white - black) histograms have `kind`'s shape."""
    n = shape[0] * shape[1]
    if kind == "dense":
        w = rng.integers(0, 256, n)
    elif kind == "gaps":                              # 17 occupied levels, the rest empty
        w = rng.choice(rng.choice(256, 17, replace=False), n)
    elif kind == "spikes":                            # three spikes and a thin scatter
        w = rng.choice([12, 140, 251], n, p=[0.5, 0.3, 0.2])
        k = rng.random(n) < 0.01
        w[k] = rng.integers(0, 256, int(k.sum()))
    elif kind == "narrow":                            # 11 adjacent levels
        w = rng.integers(100, 111, n)
    elif kind == "one_off":                           # one pixel off a constant image
        w = np.zeros(n, np.int64)
        w[rng.integers(n)] = 1
    else:                                             # "extremes": 0 and 255 only
        w = np.where(rng.random(n) < 0.37, 255, 0)
    b = np.clip(w - rng.integers(0, 60, n), 0, 255)
    return w.astype(np.uint8).reshape(shape), b.astype(np.uint8).reshape(shape)


@pytest.mark.parametrize("kind", ["dense", "gaps", "spikes", "narrow", "one_off", "extremes"])
def test_otsu_histogram_shapes(kind, mods):
    """The stats pass's Otsu (one-view launch, and a 3-view batched launch) against the oracle's
    OpenCV getThreshVal_Otsu_8u restatement, on white and clip(white - black), for histograms
    with empty bins, spikes, a narrow occupied range and near-constant images: the mu1 chain's
    branch-free run over the unskipped bins must reproduce the sequential fp64 loop exactly."""
    E, PR, N = mods
    import torch
    rng = np.random.default_rng(["dense", "gaps", "spikes", "narrow", "one_off", "extremes"].index(kind) + 40)
    shape = (83, 129)
    cfg = E.DecodeConfig(1920, 1080, 1, 1, "otsu")
    caps = [_otsu_images(kind, rng, shape) for _ in range(3)]
    want = [(O.otsu_threshold(w), O.otsu_threshold(np.clip(w.astype(np.int16) - b, 0, 255).astype(np.uint8)))
            for w, b in caps]
    eng = E.Reconstructor(*shape)
    devs = [E.DeviceFrames(torch.from_numpy(np.stack([w, b] * 3)).cuda()) for w, b in caps]
    for dev, wt in zip(devs, want):
        eng.stats(dev, cfg)
        torch.cuda.synchronize()
        assert eng.thresholds() == wt
    from structured_light_for_3d_model_replication_amd import synth
    dc = E.DeviceCalib(synth.default_rig(shape[1], shape[0], 1920, 1080).tables(), *shape)
    beng = E.BatchReconstructor(*shape, 3, slots=1)
    pb = beng.prepare(devs, cfg, dc, [E.Cloud(shape[0] * shape[1], 1, False) for _ in range(3)], row_mode=1, slot=0)
    beng.stats(pb)
    torch.cuda.synchronize()
    for v, wt in enumerate(want):
        thr = np.frombuffer(beng.header(0, v)[3104:3120].cpu().numpy().tobytes(), np.float64)
        assert tuple(thr) == wt, v


@pytest.mark.parametrize("rm", [0, 1])
@pytest.mark.parametrize("nsets", [(11, 10), (11, 11), (10, 9)])
def test_mask_first_extremes(nsets, rm, mods):
    """The fused launch reads pattern frames only in lanes holding a valid pixel (mask first):
    views with no valid pixel, every pixel valid, 5-pixel valid stripes (lanes partly valid, odd
    width so lanes straddle rows) and 2 % scattered valid pixels, in one batch, against the oracle
    (f64 bit-exact).  Row mode 1 with 11+10 and 11+11 pairs runs the plan-specialised instances,
    10+9 and row mode 0 (every valid pixel kept: random codes fail the epipolar test) the generic
    one."""
    E, PR, N = mods
    import torch
    from structured_light_for_3d_model_replication_amd import synth
    H, W = 128, 203
    rig = synth.default_rig(W, H, 1920, 1080)
    cal = rig.tables()
    nf = 2 + 2 * (nsets[0] + nsets[1])
    rng = np.random.default_rng(7 + nsets[1])
    xs = np.arange(W)[None, :].repeat(H, 0)
    lit = {"dark": np.zeros((H, W), bool), "full": np.ones((H, W), bool),
           "stripes": (xs // 5) % 2 == 0, "sparse": rng.random((H, W)) < 0.02}
    views = {}
    for name, m in lit.items():
        fr = rng.integers(0, 256, size=(nf, H, W), dtype=np.uint8)
        fr[0] = np.where(m, 200, 5)
        fr[1] = 5
        views[name] = fr
    cfg = E.DecodeConfig(1920, 1080, nsets[0], nsets[1], "manual", 40, 10)
    dc = E.DeviceCalib(cal, H, W)
    names = list(views)
    frames = [E.DeviceFrames(list(views[n]), np.repeat(views[n][0][..., None], 3, -1)) for n in names]
    eng = E.BatchReconstructor(H, W, len(names))
    outs = [E.Cloud(H * W, rm, True) for _ in names]
    eng.run(eng.prepare(frames, cfg, dc, outs, row_mode=rm))
    torch.cuda.synchronize()
    for n, o in zip(names, outs):
        c, r, m = O.decode_processing(list(views[n]), n_sets_col=nsets[0], n_sets_row=nsets[1],
                                      thresh_mode="manual", shadow_val=40, contrast_val=10)
        Po, Co = O.reconstruct_processing(c, r, m, np.repeat(views[n][0][..., None], 3, -1), cal, row_mode=rm)
        P, C = o.result()
        assert P.shape[0] == Po.shape[0], (n, P.shape[0], Po.shape[0])
        assert np.array_equal(P.cpu().numpy(), Po), n
        assert np.array_equal(C.cpu().numpy(), Co), n
        if n == "dark":
            assert P.shape[0] == 0
        if n == "full":
            assert P.shape[0] > 0


def test_device_ply_body_matches_host_formatter(tmp_path, mods):
    """slg_ply_format (the batch pipeline's PLY bodies, formatted on the GPU) is byte-identical to
    the host writer and the oracle's ``_save_ply`` bytes, on random clouds and the values where
    exact rounding matters: binary ties at the 5th decimal (±0.03125, 2.5e-5 is not a tie), -0.0
    and negatives that round to zero, subnormals, the largest magnitudes of the fast path; NaN,
    inf and |x| >= 9.2e14 are left to the host (body() returns None)."""
    E, PR, N = mods
    import torch
    from structured_light_for_3d_model_replication_amd import ply as PLY
    rng = np.random.default_rng(3)
    special = np.array([0.0, -0.0, 0.03125, -0.03125, 0.09375, 1e-5, -1e-5, 4.9999e-5, 5e-5, -5e-5, 2.5e-5,
                        5e-324, -5e-324, 2.2250738585072014e-308, 123456.78905, 9.1999999e14, -9.1999999e14,
                        1.00005, 0.99995, 2.00015, 1e-4, 0.5e-4, 1.5e-4, 2.5e-4, 3.5e-4])
    pts = np.concatenate([rng.normal(0, 500, (200_000, 3)), rng.uniform(-1e9, 1e9, (1000, 3)),
                          np.resize(special, (len(special) * 3,)).reshape(-1, 3)])
    cols = rng.integers(0, 256, (len(pts), 3), dtype=np.uint8)
    fmt = PLY.DeviceFormatter()
    for n in (0, 1, 1023, 1024, 1025, len(pts)):
        P, C = pts[:n], cols[:n]
        body = fmt.body(torch.from_numpy(P).cuda(), torch.from_numpy(C).cuda())
        assert body is not None
        got = PLY.header(n) + body.cpu().numpy().tobytes()
        path = tmp_path / f"h{n}.ply"
        PLY.write_ascii(path, P, C)
        assert got == path.read_bytes(), n
        if n <= 1025:
            assert got == O.ply_bytes(P, C), n
    for bad in (np.nan, np.inf, -np.inf, 9.2e14, -1e300):
        P = pts[:5].copy()
        P[3, 1] = bad
        assert fmt.body(torch.from_numpy(P).cuda(), torch.from_numpy(cols[:5]).cuda()) is None, bad


@pytest.mark.parametrize("name", ["proc_otsu_full", "proc_c2style", "proc_odd_geometry", "sl_full"])
def test_gray_texture_mode_matches_materialised(name, mods):
    """GRAY texture mode (slg_capture.texture NULL: the colour of a point is frame 0 replicated,
    taken from the white bytes the kernel reads anyway) == the same capture with that texture
    stored and read, bitwise, for every row mode, f64 and f32, one-view and batched launches
    (ragged 101x37 geometry: the tail tile's guarded path)."""
    E, PR, N = mods
    z = load_case(name)
    cal = load_calibs()[z["params"]["calib"]]
    frames = list(z["frames"])
    tex = np.repeat(np.asarray(frames[0])[..., None], 3, axis=-1)
    stored = E.DeviceFrames(frames, tex)
    gray = E.DeviceFrames(frames, E.GRAY)
    assert gray.texture is None and gray.capture().texture in (0, None)
    assert np.array_equal(gray.texture_bgr().cpu().numpy(), stored.texture.cpu().numpy())
    eng = E.Reconstructor(stored.height, stored.width)
    dc = E.DeviceCalib(cal, stored.height, stored.width)
    cfg = _cfg(E, z["params"])
    for rm in (0, 1, 2):
        for f64 in (True, False):
            a = [t.cpu().numpy() for t in eng.reconstruct(stored, cfg, dc, row_mode=rm, xyz_f64=f64).result()]
            b = [t.cpu().numpy() for t in eng.reconstruct(gray, cfg, dc, row_mode=rm, xyz_f64=f64).result()]
            assert len(a[0]) > 0 and np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]), (rm, f64)
    beng = E.BatchReconstructor(stored.height, stored.width, 3)
    clouds = {k: [E.Cloud(stored.n_px, 1, True) for _ in range(3)] for k in ("s", "g")}
    outs = {}
    for k, views in (("s", [stored, gray, stored]), ("g", [gray, gray, gray])):
        pb = beng.prepare(views, cfg, dc, clouds[k], 1)
        beng.run(pb)
        outs[k] = [[t.cpu().numpy() for t in c.result()] for c in clouds[k]]
    for (pa, ca), (pg, cg) in zip(outs["s"], outs["g"]):
        assert np.array_equal(pa, pg) and np.array_equal(ca, cg)


@pytest.mark.parametrize("misalign", ["stride", "base"])
def test_unaligned_frame_stack_takes_the_8_byte_loads(misalign, mods):
    """Two-axis decodes read frame pairs with paired 16-byte loads when the stack is 16-byte
    aligned (DeviceFrames always is); a caller's stack with an 8-byte stride remainder or an
    8-byte base offset (what include/slgpu.h allows) takes the 8-byte loads.  Both must give the
    golden cloud, the maps path too."""
    E, PR, N = mods
    import ctypes
    import torch
    z = load_case("proc_c2style")
    cal = load_calibs()["rig"]
    ref = E.DeviceFrames(list(z["frames"]), z["texture"])
    F, n = ref.n_frames, ref.n_px
    stride = (n + 7) // 8 * 8
    if misalign == "stride" and stride % 16 == 0:
        stride += 8                                   # an 8-byte remainder either way
    off = 8 if misalign == "base" else 0
    buf = torch.zeros(off + max(F, 2) * stride + 64, dtype=torch.uint8, device=ref.data.device)
    stack = buf[off: off + max(F, 2) * stride].view(max(F, 2), stride)
    stack[:F, :n].copy_(ref.data[:F, :n])
    odd = E.DeviceFrames.allocate(F, ref.height, ref.width)
    odd.data, odd.stride, odd.texture = stack, stride, ref.texture
    assert (odd.data.data_ptr() % 16 != 0) == (misalign == "base") and (stride % 16 != 0) == (misalign == "stride")
    dc = E.DeviceCalib(cal, ref.height, ref.width)
    cfg = _cfg(E, z["params"])
    eng = E.Reconstructor(ref.height, ref.width)
    for rm in (1, 2):
        P, C = eng.reconstruct(odd, cfg, dc, rm, xyz_f64=True).result()
        want = expected_cloud(z, cal, rm)
        assert np.array_equal(P.cpu().numpy(), want[0]) and np.array_equal(C.cpu().numpy(), want[1]), rm
    col, row, mask = eng.decode(odd, cfg)
    c2, r2, m2 = eng.decode(ref, cfg)
    assert torch.equal(col, c2) and torch.equal(row, r2) and torch.equal(mask, m2)
