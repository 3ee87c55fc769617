"""Every fused-kernel instance the library can launch runs and matches the oracle.

``slg_kernel_table`` lists the instances ``pick_main`` chooses from (csrc/slgpu.hip
``kMain3Table``): the generic ones per (source, row_mode, XYZ type, ray source) and the
plan-specialised ones per pair-count plan (C2 11+10, 1080p 11+11, C4 12+12, C1 10+0; each
also in a gray-capture form).  The two SLG_DBG profiling instances are left out.  Each case below is a
small synthetic view (a ragged 320x200 camera: the tail tile's guarded path) whose decode
parameters select one instance.  Its row planes are shifted so that row_mode 1 rejects about two
points in three.  ``slg_last_kernel`` names the instance each launch picked, so
the test checks which instance produced each cloud.  f64 clouds must equal the oracle
(``server/processing.py:127-234`` restated) bit for bit; f32 ones must be within XYZ32_RTOL,
with colours and point order exact.
"""
import numpy as np
import pytest

from oracle import sl_oracle as O

XYZ32_RTOL = 1e-4     # BASELINE.json north_star: XYZ within 1e-4 relative (fp32 vs float64)
CAM = (320, 200)
GRAY_BIT = 0x100      # csrc/slgpu.hip kPlanGray

# plan key -> (projector, n_sets, n_present, row_mode): the pair counts that select the plan
PLANS = {
    0xBA: ((1920, 1080), (11, 10), 44, 1),     # C2
    0xBB: ((1920, 1080), (11, 11), None, 1),   # 1080p, 11 + 11
    0xCC: ((3840, 2160), (12, 12), None, 1),   # C4
    0xA0: ((1024, 1080), (10, 11), 22, 0),     # C1: column pairs only
}
GENERIC = ((1920, 1080), (8, 7), None)         # pair counts no plan instance has


def symbol(rm, x64, src, rays, plan, prof=False):
    """Itanium name of main3_kernel<RM, X, S, R, P, PL> (csrc/slgpu.hip main3_symbol)."""
    li = lambda v: f"Li{v}E"
    return ("_ZN12_GLOBAL__N_112main3_kernelI" + li(rm) + li(x64) + li(src) + li(rays) +
            ("Lb1E" if prof else "Lb0E") + li(plan) + "EEvNS_11Main3ParamsE")


def cases():
    """(id, src, row_mode, x64, rays, plan, gray) for every product instance."""
    out = []
    for src in (0, 1):
        for rm in (0, 1, 2):
            for x64 in (0, 1):
                for rays in (0, 1):
                    out.append((f"generic-src{src}-rm{rm}-{'f64' if x64 else 'f32'}-{'pin' if rays else 'tab'}",
                                src, rm, x64, rays, 0, False))
    for plan, (_, _, _, rm) in PLANS.items():
        for gray in (False, True):
            for x64 in (0, 1):
                out.append((f"plan{plan:X}-{'gray' if gray else 'bgr'}-{'f64' if x64 else 'f32'}",
                            1, rm, x64, 1, plan, gray))
    return out


CASES = cases()


def test_cases_cover_the_instance_table():
    """The cases name every non-profiling instance of the library's table, once (no GPU call:
    slg_kernel_table reads the library file)."""
    from structured_light_for_3d_model_replication_amd import _native as N
    table = {s for s in N.kernel_table() if "Lb0E" in s}
    want = [symbol(rm, x64, src, rays, plan | (GRAY_BIT if gray else 0)) for _, src, rm, x64, rays, plan, gray in CASES]
    assert len(want) == len(set(want)) == len(table) == 40
    assert set(want) == table


_views = {}


def _view(proj, nsets, n_present):
    key = (proj, nsets, n_present)
    if key not in _views:
        from structured_light_for_3d_model_replication_amd import synth
        rig = synth.default_rig(*CAM, *proj)
        v = synth.render_view(rig, 20.0, seed=5, n_present=n_present)
        kw = dict(n_cols=proj[0], n_rows=proj[1], n_sets_col=nsets[0], n_sets_row=nsets[1], thresh_mode="otsu")
        maps = O.decode_processing(list(v.frames), **kw)
        # The renderer's rig puts every decoded row within the 2 mm epipolar tolerance.  Shifting
        # two rows in three of the row planes by 3 mm makes row_mode 1 reject points too.
        cal = rig.tables()
        rows = cal["wPlaneRow"].copy()
        rows[3] += 3.0 * (np.arange(rows.shape[1]) % 3 - 1)
        cal["wPlaneRow"] = rows
        _views[key] = (v, cal, maps)
    return _views[key]


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_every_fused_instance_matches_oracle(case):
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a ROCm device")
    from structured_light_for_3d_model_replication_amd import engine as E, _native as N
    _, src, rm, x64, rays, plan, gray = case
    proj, nsets, n_present = (PLANS[plan][:3] if plan else GENERIC)
    v, cal, (oc, orow, om) = _view(proj, nsets, n_present)
    frames = list(v.frames)
    tex = np.repeat(np.asarray(frames[0])[..., None], 3, axis=-1) if gray else v.texture
    dev = E.DeviceFrames(frames, E.GRAY if gray else tex)
    H, W = dev.height, dev.width
    dc = E.DeviceCalib(cal, H, W, keep_table=not rays)
    assert dc.ray_mode == (N.RAYS_PINHOLE if rays else N.RAYS_TABLE)
    eng = E.Reconstructor(H, W)
    if src == 1:
        cfg = E.DecodeConfig(proj[0], proj[1], nsets[0], nsets[1], "otsu")
        out = eng.reconstruct(dev, cfg, dc, row_mode=rm, xyz_f64=bool(x64))
    else:
        t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dt).ravel()).cuda()
        out = eng.triangulate(t(oc, np.int32), t(orow, np.int32), t(om, np.uint8), dev.texture, dc,
                              row_mode=rm, xyz_f64=bool(x64))
    assert N.last_kernel() == symbol(rm, x64, src, rays, plan | (GRAY_BIT if gray else 0))
    P, C = (t.cpu().numpy() for t in out.result())
    Po, Co = O.reconstruct_processing(oc, orow, om, tex, cal, row_mode=rm)
    assert len(Po) > 1000 and P.shape == Po.shape, (P.shape, Po.shape)
    if rm == 1:
        assert len(Po) < 0.6 * om.sum()                  # the epipolar test rejected points
    assert np.array_equal(C, Co)
    if x64:
        assert np.array_equal(P, Po), f"max |d| {np.abs(P - Po).max()}"
    else:
        scale = np.maximum(np.abs(Po), 1e-3)
        assert np.all(np.abs(P.astype(np.float64) - Po) <= XYZ32_RTOL * scale)
    assert eng.error_flags() & 1 == 0


@pytest.mark.gpu
def test_lone_view_scan_repeatable():
    """A lone view's launch takes its tile offsets from the last-arriving tile's scan
    (csrc/slgpu.hip lookback_scan) or from the look-back walks, whichever lands first at each
    tile; a launch of two views always walks.  Forty one-view calls on a 1080p C2 view must each
    equal the two-view launch bit for bit, row_mode 1 and 2."""
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a ROCm device")
    from structured_light_for_3d_model_replication_amd import engine as E, synth
    rig = synth.default_rig(1920, 1080, 1920, 1080)
    v = synth.render_view(rig, 40.0, seed=9, n_present=44)
    dev = E.DeviceFrames(list(v.frames), v.texture)
    dc = E.DeviceCalib(rig.tables(), dev.height, dev.width)
    cfg = E.DecodeConfig(1920, 1080, 11, 10, "otsu")
    eng = E.Reconstructor(dev.height, dev.width)
    beng = E.BatchReconstructor(dev.height, dev.width, 2)
    for rm in (1, 2):
        clouds = [E.Cloud(dev.n_px, rm, False) for _ in range(2)]
        beng.run(beng.prepare([dev, dev], cfg, dc, clouds, rm))
        want = [t.clone() for t in clouds[0].result()]
        assert len(want[0]) > 500_000
        out = E.Cloud(dev.n_px, rm, False)
        for _ in range(40):
            eng.reconstruct(dev, cfg, dc, rm, out=out)
            got = out.result()
            assert torch.equal(got[0], want[0]) and torch.equal(got[1], want[1]), rm
        assert eng.error_flags() & 1 == 0
