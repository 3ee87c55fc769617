"""GPU parity at the BASELINE configurations' full sizes and at the benchmark's exact launch shape
(VERDICT r1 "next" #1).  Every check goes through the C ABI and compares with the oracle
(tests only):

* C2 bench shape: ``BatchReconstructor.run_pipelined(mode="fused")`` over 36 full-size 1920x1080
  views, 12 per main3 launch, 2 workspace slots, batch k carrying batch k+2's Otsu histograms
  (per-tile partials -> parts_kernel), issued in two pieces (the stream continuation bench.py
  uses).  Every view's count equals the oracle's; f32 clouds within the north-star tolerance
  and f64 clouds bit-exact on a subset; the 1013-tile look-back chains are full length.
* C3: the 36-view turntable job at 1080p with 11 + 11 bits through the sharded path's pieces
  (12-view batches, the C-ABI RCCL gatherv at world size 1): every view's count and a subset of
  clouds (f64, bit for bit) against the oracle, gathered layout checked.
* C5 geometry: a 3840x2160 view, projector 1920x1080, 11 + 11 bits, row_mode 1 -- maps, f64
  cloud bit-exact, f32 within tolerance, codes equal the renderer's ground truth; and a 2-view
  batch of them.
"""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from oracle import sl_oracle as O

pytestmark = pytest.mark.gpu

XYZ32_RTOL = 1e-4     # BASELINE.json north_star: XYZ within 1e-4 relative (fp32 vs float64)
N_VIEWS = 36


def _xyz32_close(got, want):
    got = np.asarray(got, np.float64)
    scale = np.maximum(np.abs(want), 1e-3)
    assert np.all(np.abs(got - want) <= XYZ32_RTOL * scale)


@pytest.fixture(scope="module")
def mods():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a ROCm device")
    from structured_light_for_3d_model_replication_amd import engine as E, _native as N
    N.lib()
    return E, N


@pytest.fixture(scope="module")
def scan():
    """36 rendered 1080p turntable views (10 degree steps, 46 frames each) + their calibration."""
    from structured_light_for_3d_model_replication_amd import synth
    rig = synth.default_rig(1920, 1080, 1920, 1080)
    with ThreadPoolExecutor(8) as ex:
        views = list(ex.map(lambda i: synth.render_view(rig, 10.0 * i, seed=500 + i), range(N_VIEWS)))
    return rig.tables(), views


def _oracle_all(cal, views, nsets, row_mode=1):
    def one(v):
        c, r, m = O.decode_processing(list(v.frames), n_sets_col=nsets[0], n_sets_row=nsets[1])
        return O.reconstruct_processing(c, r, m, v.texture, cal, row_mode=row_mode)
    with ThreadPoolExecutor(8) as ex:
        return list(ex.map(one, views))


def test_c2_bench_launch_shape(mods, scan):
    """The benchmark's exact shape: 12 C2 views per fused launch, two slots, carried histograms;
    every view's count, colours and XYZ (f64 bit for bit, f32 within the north-star tolerance)."""
    E, N = mods
    import torch
    cal, views = scan
    want = _oracle_all(cal, views, (11, 10))
    dev = [E.DeviceFrames(list(v.frames), v.texture) for v in views]
    dcal = E.DeviceCalib(cal, 1080, 1920)
    cfg = E.DecodeConfig(1920, 1080, 11, 10, "otsu")
    for f64 in (False, True):
        eng = E.BatchReconstructor(1080, 1920, 12, slots=2)
        clouds = [E.Cloud(1920 * 1080, 1, f64) for _ in range(N_VIEWS)]
        batches = [eng.prepare(dev[12 * b:12 * b + 12], cfg, dcal, clouds[12 * b:12 * b + 12], 1, 2.0, slot=b % 2)
                   for b in range(3)]
        s_main, s_stats = torch.cuda.Stream(), torch.cuda.Stream()
        eng.run_pipelined(batches, s_main, s_stats, mode="fused", start=0, stop=1)   # bench: warmup ...
        eng.run_pipelined(batches, s_main, s_stats, mode="fused", start=1, stop=3)   # ... then timed steps
        torch.cuda.synchronize()
        for k, (c, (Po, Co)) in enumerate(zip(clouds, want)):
            P, C = c.result()
            assert P.shape[0] == Po.shape[0], (f64, k, P.shape[0], Po.shape[0])
            P, C = P.cpu().numpy(), C.cpu().numpy()          # every view, both output types
            assert np.array_equal(C, Co), (f64, k)
            if f64:
                assert np.array_equal(P, Po), k
            else:
                _xyz32_close(P, Po)
        assert all(eng.header(s, v)[3084:3088].cpu().numpy()[0] & 1 == 0 for s in range(2) for v in range(12))
    assert min(len(w[0]) for w in want) > 500_000


@pytest.mark.parametrize("bv", [6, 16])
def test_c2_two_stream_pipeline(mods, scan, bv):
    """bench.py --pipeline fused2: batch k on stream k % 2 (launches overlap), launch k carrying
    batch k+4's histograms and finishing batch k+2's thresholds, 4 slots; bv-view batches over
    the 36 views taken cyclically (16: the bench's launch, 7 batches so launches carry and
    finish at that width too), issued in two pieces.  Every view's count, colours and XYZ against
    the oracle."""
    E, N = mods
    import torch
    cal, views = scan
    want = _oracle_all(cal, views, (11, 10))
    dev = [E.DeviceFrames(list(v.frames), v.texture) for v in views]
    dcal = E.DeviceCalib(cal, 1080, 1920)
    cfg = E.DecodeConfig(1920, 1080, 11, 10, "otsu")
    eng = E.BatchReconstructor(1080, 1920, bv, slots=4)
    nb = max(6, (N_VIEWS + bv - 1) // bv) if bv < 16 else 7
    idx = [(bv * b + k) % N_VIEWS for b in range(nb) for k in range(bv)]
    clouds = [E.Cloud(1920 * 1080, 1, False) for _ in idx]
    batches = [eng.prepare([dev[i] for i in idx[bv * b:bv * b + bv]], cfg, dcal, clouds[bv * b:bv * b + bv], 1, 2.0,
                           slot=b % 4) for b in range(nb)]
    s0, s1 = torch.cuda.Stream(), torch.cuda.Stream()
    eng.run_pipelined(batches, s0, s1, mode="fused2", start=0, stop=nb // 2)
    torch.cuda.synchronize()
    eng.run_pipelined(batches, s0, s1, mode="fused2", start=nb // 2, stop=nb)
    torch.cuda.synchronize()
    for k, (c, i) in enumerate(zip(clouds, idx)):
        Po, Co = want[i]
        P, C = c.result()
        assert P.shape[0] == Po.shape[0], (k, P.shape[0], Po.shape[0])
        assert np.array_equal(C.cpu().numpy(), Co), k
        _xyz32_close(P.cpu().numpy(), Po)
    assert all(eng.header(s, v)[3084:3088].cpu().numpy()[0] & 1 == 0 for s in range(4) for v in range(bv))


def test_c3_sharded_job(mods, scan):
    """C3: 36 views, 11 + 11 bits, 12-view batches, then the C-ABI RCCL gatherv (world 1)."""
    E, N = mods
    import torch
    from structured_light_for_3d_model_replication_amd import distributed as D
    cal, views = scan
    want = _oracle_all(cal, views, (11, 11))
    dev = [E.DeviceFrames(list(v.frames), v.texture) for v in views]
    dcal = E.DeviceCalib(cal, 1080, 1920)
    cfg = E.DecodeConfig(1920, 1080, 11, 11, "otsu")
    lo, hi = D.shard_range(N_VIEWS, 0, 1)
    assert (lo, hi) == (0, N_VIEWS)
    eng = E.BatchReconstructor(1080, 1920, 12, slots=3)
    clouds = [E.Cloud(1920 * 1080, 1, True) for _ in range(N_VIEWS)]
    s = torch.cuda.Stream()
    for b in range(3):
        eng.run(eng.prepare(dev[12 * b:12 * b + 12], cfg, dcal, clouds[12 * b:12 * b + 12], 1, 2.0, slot=b), stream=s)
    s.synchronize()
    parts = []
    for c, (Po, _) in zip(clouds, want):
        P, C = c.result()
        assert P.shape[0] == Po.shape[0]
        parts.append((P, C))
    g = D.RcclCloudGather()
    try:
        got = g.gather(parts, N_VIEWS, root=0, stream=s)
        s.synchronize()
    finally:
        g.close()
    assert len(got) == N_VIEWS
    rx, rb = g.last_buffers
    assert rx.shape[0] == sum(len(w[0]) for w in want)
    for k in range(N_VIEWS):                         # every gathered view, bit for bit (f64)
        assert np.array_equal(got[k][0].cpu().numpy(), want[k][0]), k
        assert np.array_equal(got[k][1].cpu().numpy(), want[k][1]), k


def test_c5_full_size(mods):
    """C5 geometry: 3840x2160 camera, projector 1920x1080, 11 + 11 bits (46 frames), row_mode 1."""
    E, N = mods
    import torch
    from structured_light_for_3d_model_replication_amd import synth
    rig = synth.default_rig(3840, 2160, 1920, 1080)
    cal = rig.tables()
    vs = [synth.render_view(rig, a, seed=31 + i) for i, a in enumerate((15.0, 195.0))]
    assert vs[0].frames.shape == (46, 2160, 3840)
    cfg = E.DecodeConfig(1920, 1080, 11, 11, "otsu")
    dcal = E.DeviceCalib(cal, 2160, 3840)
    dev = [E.DeviceFrames(list(v.frames), v.texture) for v in vs]
    eng = E.Reconstructor(2160, 3840)
    v = vs[0]
    col, row, mask = eng.decode(dev[0], cfg)
    oc, orow, om = O.decode_processing(list(v.frames), n_sets_col=11, n_sets_row=11)
    shape = (2160, 3840)
    col, row, mask = (col.reshape(shape).cpu().numpy(), row.reshape(shape).cpu().numpy(),
                      mask.reshape(shape).cpu().numpy().astype(bool))
    assert np.array_equal(col, oc) and np.array_equal(row, orow) and np.array_equal(mask, om)
    lit = v.lit & mask
    assert lit.sum() > 1_000_000
    assert np.array_equal(col[lit], v.proj_col[lit]) and np.array_equal(row[lit], v.proj_row[lit])
    Po, Co = O.reconstruct_processing(oc, orow, om, v.texture, cal, row_mode=1)
    P, C = eng.reconstruct(dev[0], cfg, dcal, 1, xyz_f64=True).result()
    assert np.array_equal(P.cpu().numpy(), Po) and np.array_equal(C.cpu().numpy(), Co)
    P, C = eng.reconstruct(dev[0], cfg, dcal, 1, xyz_f64=False).result()
    assert len(P) == len(Po) and np.array_equal(C.cpu().numpy(), Co)
    _xyz32_close(P.cpu().numpy(), Po)
    assert eng.error_flags() & 1 == 0
    # the 2-view batch of the bench's c5 shape (stats + one fused launch, f32)
    beng = E.BatchReconstructor(2160, 3840, 2)
    outs = [E.Cloud(2160 * 3840, 1, False) for _ in vs]
    beng.run(beng.prepare(dev, cfg, dcal, outs, 1, 2.0))
    torch.cuda.synchronize()
    Po2, Co2 = _oracle_all(cal, vs[1:], (11, 11))[0]
    for o, (Pw, Cw) in zip(outs, [(Po, Co), (Po2, Co2)]):
        P, C = o.result()
        assert len(P) == len(Pw) and np.array_equal(C.cpu().numpy(), Cw)
        _xyz32_close(P.cpu().numpy(), Pw)


def test_c5_resident_job(mods):
    """BASELINE configs[4] reduced to 2 objects x 4 views (bench.py --config c5job's code path,
    jobs.ResidentJob): 3840x2160 views, each an HBM copy of one of 2 captures per object, one
    fused launch per view on the two-stream carried pipeline (4 primed + 4 carried groups), the
    clouds packed in one arena by capacity hints.  Every view's count and colours equal the
    oracle's, XYZ within the north-star tolerance; a view given too small a hint is reported as
    overflowed and its successor as damaged (the stores stay inside the arena); the default
    device-reserved arena (no sizing pass), one too small for the job, and row_mode 2."""
    E, N = mods
    import torch
    from structured_light_for_3d_model_replication_amd import jobs as J, synth
    H, W = 2160, 3840
    rig = synth.default_rig(W, H, 1920, 1080)
    cal = rig.tables()
    keys = [(o, k) for o in range(2) for k in range(2)]
    with ThreadPoolExecutor(4) as ex:
        caps = list(ex.map(lambda ok: synth.render_view(rig, synth.job_view_angle(ok[0], 2 * ok[1], 4),
                                                        seed=1000 * ok[0] + ok[1]), keys))
    want = _oracle_all(cal, caps, (11, 11))
    cfg = E.DecodeConfig(1920, 1080, 11, 11, "otsu")
    dcal = E.DeviceCalib(cal, H, W)
    sources = [E.DeviceFrames(list(v.frames), v.texture) for v in caps]
    plan = [2 * o + a * 2 // 4 for o in range(2) for a in range(4)]       # source of job view j
    views = J.stage_copies(sources, plan)
    del sources
    hints = [len(want[p][0]) for p in plan]
    job = J.ResidentJob(views, cfg, dcal, batch=1, capacity_hints=hints)
    s0, s1 = torch.cuda.Stream(), torch.cuda.Stream()
    for _ in range(2):                                  # a job re-run rewrites the same clouds
        job.run(s0, s1)
    torch.cuda.synchronize()
    counts = job.host_counts()
    assert counts == hints and job.overflowed(counts) == []
    assert len(job.batches) == 8 and job.xyz.shape[0] == sum(hints) + H * W
    for j, p in enumerate(plan):
        x, b = job.cloud(j, counts)
        assert np.array_equal(b.cpu().numpy(), want[p][1]), j
        _xyz32_close(x.cpu().numpy(), want[p][0])
    small = list(hints)
    small[2] -= 1000                                    # view 2 cannot fit: flagged, not faulted
    job2 = J.ResidentJob(views[:4], cfg, dcal, batch=2, capacity_hints=small[:4])
    job2.run(s0, s1)
    torch.cuda.synchronize()
    assert job2.overflowed() == [2]
    assert job2.damaged() == [2, 3]                     # view 3's region begins inside view 2's overflow
    # refusal: a damaged view's arena slice is never handed out
    for j in (2, 3):
        with pytest.raises(J.DamagedViewError):
            job2.cloud(j)
    # recovery: the damaged views re-run into clouds of their own, equal to the oracle's
    assert job2.recover() == [2, 3]
    for j in range(4):
        x, b = job2.cloud(j)
        assert np.array_equal(b.cpu().numpy(), want[plan[j]][1]), j
        _xyz32_close(x.cpu().numpy(), want[plan[j]][0])
    # the default: a device-reserved arena -- each view's region reserved by the kernel that
    # finishes its thresholds, min(#white >= smin, #(white - black) >= cmin) points (an upper
    # bound of its count), no sizing pass, nothing can overflow
    job3 = J.ResidentJob(views, cfg, dcal, batch=2)
    assert job3.hints_source == "device_reserved"
    for _ in range(2):                                  # every run reserves afresh
        job3.run(s0, s1)
    torch.cuda.synchronize()
    counts3, offs3 = job3.host_counts(), job3.host_offsets()
    assert counts3 == hints and job3.damaged(counts3) == [] and min(offs3) >= 0
    spans = sorted((o, o + n) for o, n in zip(offs3, counts3))
    assert all(a[1] <= b[0] for a, b in zip(spans, spans[1:])) and spans[-1][1] <= job3.arena_points
    for j, p in enumerate(plan):
        x, b = job3.cloud(j, counts3)
        assert np.array_equal(b.cpu().numpy(), want[p][1]), j
        _xyz32_close(x.cpu().numpy(), want[p][0])
    # an arena with room for about two views: the others are refused (they store nothing), named
    # by overflowed(), refused by cloud() and recovered by recover()
    job4 = J.ResidentJob(views[:4], cfg, dcal, batch=2, arena_points=2 * max(hints) + 1000)
    job4.run(s0, s1)
    torch.cuda.synchronize()
    refused = job4.overflowed()
    assert 1 <= len(refused) <= 3 and job4.damaged() == refused
    for j in refused:
        with pytest.raises(J.DamagedViewError):
            job4.cloud(j)
    assert job4.recover() == refused
    for j in range(4):
        x, b = job4.cloud(j)
        assert np.array_equal(b.cpu().numpy(), want[plan[j]][1]), j
        _xyz32_close(x.cpu().numpy(), want[plan[j]][0])
    # row_mode 2 (server/processing.py:209-234: column cloud then row cloud): reserved at twice
    # the bound, every view equal to the oracle's concatenated clouds, f64 bit for bit
    want2 = _oracle_all(cal, caps, (11, 11), row_mode=2)
    job5 = J.ResidentJob(views[:4], cfg, dcal, batch=2, row_mode=2, xyz_f64=True)
    job5.run(s0, s1)
    torch.cuda.synchronize()
    assert job5.damaged() == []
    for j in range(4):
        x, b = job5.cloud(j)
        assert np.array_equal(b.cpu().numpy(), want2[plan[j]][1]), j
        assert np.array_equal(x.cpu().numpy(), want2[plan[j]][0]), j


def test_valid_bounds_match_histogram_counts(mods, scan):
    """``BatchReconstructor.valid_bounds`` (the resident jobs' device sizing): per view
    min(#(white > ts), #((white - black) > tc)) with the Otsu thresholds of
    server/processing.py:63-72, exactly; >= the valid pixels; 20 views in groups of 16 + 4."""
    E, N = mods
    cal, views = scan
    vs = views[:20]
    cfg = E.DecodeConfig(1920, 1080, 11, 11, "otsu")
    eng = E.BatchReconstructor(1080, 1920, 16, slots=1)
    got = eng.valid_bounds([E.DeviceFrames(list(v.frames), v.texture) for v in vs], cfg).tolist()
    for v, g in zip(vs, got):
        w = v.frames[0].astype(np.float32)
        b = v.frames[1].astype(np.float32)
        ts = O.otsu_threshold(w.astype(np.uint8))
        tc = O.otsu_threshold(np.clip(w - b, 0, 255).astype(np.uint8))
        want = min(int(np.count_nonzero(w > ts)), int(np.count_nonzero((w - b) > tc)))
        assert g == want
        assert g >= int(np.count_nonzero(O.mask_processing(v.frames[0], v.frames[1])))




def test_concurrent_stats_thresholds(mods, scan):
    """The stats tickets run without release / acquire fences (agent-scope atomics only, the
    hardware assumption documented at stats_kernel): four engines' 16-view stats launches on four
    streams at once, eight rounds, every view's Otsu thresholds (white, clip(white - black)) equal
    to the oracle's (server/processing.py:63-72)."""
    E, N = mods
    import ctypes
    import torch
    cal, views = scan
    cfg = E.DecodeConfig(1920, 1080, 11, 11, "otsu")
    dp = cfg.struct()
    want = []
    for v in views:
        w = v.frames[0]
        b = v.frames[1].astype(np.float32)
        want.append((O.otsu_threshold(w), O.otsu_threshold(np.clip(w.astype(np.float32) - b, 0, 255).astype(np.uint8))))
    dev = [E.DeviceFrames(list(v.frames[:2]) + [None] * 2, "gray", n_frames=4) for v in views]
    engs = [E.BatchReconstructor(1080, 1920, 16, slots=1) for _ in range(4)]
    streams = [torch.cuda.Stream() for _ in range(4)]
    groups = [[(9 * e + k) % len(views) for k in range(16)] for e in range(4)]
    torch.cuda.synchronize()
    for rnd in range(8):
        for eng, g, s in zip(engs, groups, streams):
            caps = (N.Capture * 16)(*[dev[j].capture() for j in g])
            N.check(N.lib().slg_decode_stats_batch(caps, 16, ctypes.byref(dp), eng._ws(0), eng.ws_stride,
                                                   E._stream(s)))
        torch.cuda.synchronize()
        for eng, g in zip(engs, groups):
            for k, j in enumerate(g):
                hdr = eng.header(0, k).cpu().numpy()
                thr = np.frombuffer(hdr[3104:3120].tobytes(), np.float64)
                assert (thr[0], thr[1]) == (float(want[j][0]), float(want[j][1])), (rnd, j)
