"""GPU: one view split over bands of rows (bands.py; SURVEY §8(e) "single huge view"), through the
C ABI (``slg_decode_histograms`` -> the exchange -> ``slg_thresholds_from_histograms`` ->
``slg_decode_triangulate`` per band).  The ranks are simulated in one process: every band's
histograms are counted first and their sum / max handed to each band as the all-reduce would.
The reassembled cloud must equal the unsplit view's bit for bit (f64 and f32 XYZ, BGR, order),
for Otsu, manual and percentile thresholds, row_mode 0 / 1 / 2, pinhole and table rays, bands of
one row and image widths that are not a multiple of 8; the unsplit view is itself checked against
the oracle (tests only)."""
import numpy as np
import pytest

from oracle import sl_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mods():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a ROCm device")
    from structured_light_for_3d_model_replication_amd import bands as B, engine as E, _native as N
    N.lib()
    return B, E


def _scene(w, h, pw, ph, seed):
    from structured_light_for_3d_model_replication_amd import synth
    rig = synth.default_rig(w, h, pw, ph)
    return rig.tables(), synth.render_view(rig, 35.0, seed=seed)


def _banded(B, E, frames, calib, cfg, row_mode, f64, bounds):
    import torch
    H, W = frames.height, frames.width
    brs = [B.BandReconstructor(H, W, r0, r1) for r0, r1 in bounds]
    bfs = [B.band_frames(frames, r0, r1) for r0, r1 in bounds]
    bcs = [B.band_calib(calib, r0, r1) for r0, r1 in bounds]
    # the exchange, simulated: every band's histograms first, then their sum / max (manual
    # thresholds: no exchange)
    total = None
    if cfg.thresh_mode != "manual" or cfg.variant == "slsystem":
        hs = torch.stack([br.engine.histograms(bf, cfg).clone() for br, bf in zip(brs, bfs)])
        total = torch.cat([hs[:, :512].sum(0, dtype=torch.int32), hs[:, 512:].amax(0)])

    def exchange(h):
        h.copy_(total)

    parts, cols, ths = [], [], []
    for br, bf, bc in zip(brs, bfs, bcs):
        out, ncol = br.run(bf, cfg, bc, row_mode, 2.0, f64, exchange=exchange)
        parts.append(out.result())
        cols.append(ncol)
        ths.append(br.engine.thresholds())
    xyz, bgr = B.assemble(parts, cols, row_mode)
    return xyz, bgr, ths, total


CFGS = [("otsu", "processing"), ("manual", "processing"), ("otsu", "slsystem")]


@pytest.mark.parametrize("geom", ["c2", "ragged"])
def test_banded_view_equals_unsplit(mods, geom):
    B, E = mods
    import torch
    if geom == "c2":
        W, H, PW, PH, nsets = 1920, 1080, 1920, 1080, (11, 10)
        bounds = [(0, 300), (300, 301), (301, 777), (777, 1080)]
    else:
        W, H, PW, PH, nsets = 101, 37, 128, 64, (7, 6)
        bounds = [(0, 12), (12, 24), (24, 37)]
    cal, v = _scene(W, H, PW, PH, 11)
    frames = E.DeviceFrames(list(v.frames), v.texture)
    checked_oracle = False
    for rays in ("pinhole", "table"):
        calib = E.DeviceCalib(cal, H, W, keep_table=rays == "table")
        assert (calib.rays is None) == (rays == "pinhole")
        for thresh, variant in CFGS:
            cfg = E.DecodeConfig(PW, PH, nsets[0], nsets[1], thresh, variant=variant)
            for row_mode in ((0,) if variant == "slsystem" else (0, 1, 2)):
                for f64 in (True, False):
                    eng = E.Reconstructor(H, W)
                    wx, wb = eng.reconstruct(frames, cfg, calib, row_mode, 2.0, xyz_f64=f64).result()
                    gx, gb, ths, total = _banded(B, E, frames, calib, cfg, row_mode, f64, bounds)
                    tag = (rays, thresh, variant, row_mode, f64)
                    assert gx.shape == wx.shape and torch.equal(gx, wx), tag
                    assert torch.equal(gb, wb), tag
                    assert all(t == eng.thresholds() for t in ths), tag
                    assert wx.shape[0] > 100, tag
                    if thresh == "otsu" and variant == "processing":
                        w8, b8 = np.asarray(v.frames[0]), np.asarray(v.frames[1])
                        assert np.array_equal(total[:256].cpu().numpy(), np.bincount(w8.ravel(), minlength=256))
                        d = np.clip(w8.astype(np.int32) - b8.astype(np.int32), 0, 255)
                        assert np.array_equal(total[256:512].cpu().numpy(), np.bincount(d.ravel(), minlength=256))
                    if f64 and not checked_oracle and thresh == "otsu" and variant == "processing" and row_mode == 1:
                        c, r, m = O.decode_processing(list(v.frames), PW, PH, nsets[0], nsets[1])
                        P, C = O.reconstruct_processing(c, r, m, v.texture, cal, row_mode=1)
                        assert np.array_equal(gx.cpu().numpy(), P) and np.array_equal(gb.cpu().numpy(), C)
                        checked_oracle = True
    assert checked_oracle


def test_banded_percentile_max_code(mods):
    """The percentile rule's exchange: black's histogram summed, max(white - black) + 256 maxed."""
    B, E = mods
    import torch
    cal, v = _scene(101, 37, 128, 64, 3)
    frames = E.DeviceFrames(list(v.frames), v.texture)
    cfg = E.DecodeConfig(128, 64, 7, 6, "otsu", variant="slsystem")
    hs = []
    for r0, r1 in [(0, 5), (5, 37)]:
        br = B.BandReconstructor(37, 101, r0, r1)
        hs.append(br.engine.histograms(B.band_frames(frames, r0, r1), cfg).clone())
    w8, b8 = np.asarray(v.frames[0]).astype(np.int32), np.asarray(v.frames[1]).astype(np.int32)
    tot = hs[0][:256] + hs[1][:256]
    assert np.array_equal(tot.cpu().numpy(), np.bincount(b8.ravel().astype(np.int64), minlength=256))
    assert int(torch.maximum(hs[0][512], hs[1][512])) == int((w8 - b8).max()) + 256


def _rank_main(rank, world, port, q):
    """One rank of the two-process split on the one GPU (gloo: the exchange and the gather go
    through host memory; two RCCL ranks cannot share a device)."""
    import os
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from structured_light_for_3d_model_replication_amd import bands as B, engine as E
        cal, v = _scene(333, 211, 256, 128, 5)
        H, W = 211, 333
        r0, r1 = B.band_rows(H, rank, world)
        full = E.DeviceFrames(list(v.frames), v.texture)
        calib = E.DeviceCalib(cal, H, W)
        cfg = E.DecodeConfig(256, 128, 8, 7, "otsu")
        out = {}
        for row_mode in (1, 2):
            br = B.BandReconstructor(H, W, r0, r1)
            c, ncol = br.run(B.band_frames(full, r0, r1), cfg, B.band_calib(calib, r0, r1), row_mode, 2.0, True)
            x, b = c.result()
            got = B.gather_banded(x.cpu(), b.cpu(), ncol, row_mode, dst=0)
            if rank == 0:
                wx, wb = E.Reconstructor(H, W).reconstruct(full, cfg, calib, row_mode, 2.0, xyz_f64=True).result()
                out[row_mode] = bool(torch.equal(got[0], wx.cpu()) and torch.equal(got[1], wb.cpu()) and len(wx) > 100)
        q.put((rank, out))
    except BaseException as e:  # report instead of hanging the parent on q.get
        q.put((rank, f"EXC {type(e).__name__}: {e}"))
        raise
    finally:
        dist.destroy_process_group()


def test_two_process_band_split_on_one_gpu(mods):
    """The exchange and the gather through torch.distributed with real kernels: two processes,
    one band each, the gathered cloud equal to the unsplit view's (row_mode 1 and 2)."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=200) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res[0] == {1: True, 2: True} and res[1] == {}, res
    assert all(p.exitcode == 0 for p in procs)
