#!/usr/bin/env python
"""Benchmark: decoded+triangulated Mpoints/s of the structured-light hot path on MI355X.

Workload (BASELINE.json configs[1], "C2"): 1920x1080 views, 11 column + 10 row Gray-code bits
with inverses + white/black (44 frames), Otsu mask, row_mode 1 (epipolar filter, tol 2.0),
fp32 XYZ + BGR out, inputs resident in HBM.  A STEP is one batch of B views (default 16, the
most one launch takes; 2.6 % less time per view than 12, profiles/r3k) through the whole path:
ONE fused decode/triangulate/compaction launch over the batch, plus its Otsu thresholds.  Default ``--pipeline fused2``: batch k's launch runs on stream k % 2, counts batch
k+4's histograms (per-tile partials: no separate pass over its white/black frames) and, with
workgroups at the front of its grid, turns batch k+2's partials into thresholds; every
dependency stays on one stream, so launch k+1 fills the GPU while launch k's last workgroups
drain (BatchReconstructor.run_pipelined; ``fused`` is the same on one stream with distance 2).
The pipeline runs continuously from the priming stats passes (outside any timing) through the
W warmup steps into the K timed steps, so every timed step is a steady-state step whatever K
is.  Steps rotate over a pool of distinct rendered turntable views (views x copies HBM buffers,
> 256 MiB Infinity Cache), so frames stream from HBM and a carried batch is never the batch
being decoded.  One HIP event pair brackets the timed region (both streams join it), so
``roofline.kernel_avg_us`` is the step period: with overlapping launches a launch's own
duration is longer than the period at which they complete.

``--config c3``: the 36-view turntable scan (BASELINE configs[2]) as ONE job, views sharded
across the ranks (strong scaling): every rank decodes its block, the clouds are gathered to rank
0 through the C-ABI RCCL gatherv (``slg_gather_*``), the timed region includes it.
``--config c5job``: BASELINE configs[4], 8 objects x 72 views at 4K resident in HBM, one job per
step (bench_c5job.py).  ``--config c4band``: ONE C4 view split over the ranks by bands of rows,
one histogram all-reduce per view (bench_c4band.py, strong scaling).  ``--config c4|c5``: the larger single-GPU geometries.  For N>1 on the default config each rank
runs its own stream of views (weak scaling, no data-path collective); value = all ranks' points /
max-over-ranks time.

Prints ONE JSON line on stdout (rank 0).  Diagnostics go to stderr.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "decoded+triangulated Mpoints/sec (1 GPU & 8-GPU node); % of HBM roofline"
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec (6.3 measured copy)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# Workloads (BASELINE.json configs / SURVEY §8(d)).  c2 is the metric's configuration and the
# default; the others run on request (--config).  A fused2 launch k decodes batch k and carries
# batch k+4's histograms; with D distinct batches in the pool (views x copies / batch) those are
# the frames of batch (k+4) mod D.  D = 6 (c2, c4, c5) makes them the batch decoded two launches
# earlier on the same stream, GBs of traffic ago: cold HBM reads.  (D = 2 or 4 would make them
# the batch this launch decodes, read twice through the caches; c2's earlier D = 3 made them the
# batch the other stream decodes at the same time: 1.7 % faster, profiles/r4ab.)  c2: D = 6 too.
CONFIGS = {
    # c1: the reference GUI's legacy single-view call, _gray_decode(files, n_cols=1024, n_rows=1080)
    # with the default n_sets (col bits clamp to Bc = 10), row frames absent, row_mode 0
    # (server/processing.py:28,80-84,174-182)
    "c1": dict(cam=(1280, 720), proj=(1024, 1080), nsets=(11, 11), n_present=22, views=12, copies=8, batch=16,
               row_mode=0,
               text="C1: 1280x720 view, projector 1024 wide, 10 col Gray bits + inverses + white/black (22 frames), "
                    "row frames absent"),
    "c2": dict(cam=(1920, 1080), proj=(1920, 1080), nsets=(11, 10), n_present=44, views=12, copies=8, batch=16,
               text="C2: 1920x1080 view, 11 col + 10 row Gray bits + inverses + white/black (44 frames)"),
    "c3": dict(cam=(1920, 1080), proj=(1920, 1080), nsets=(11, 11), n_present=None, views=36, copies=1, batch=12,
               text="C3: 36-view 360-degree turntable scan at 1920x1080, 11 col + 11 row Gray bits + "
                    "inverses + white/black (46 frames), views sharded over the ranks, clouds gathered to rank 0"),
    "c4": dict(cam=(6000, 4000), proj=(3840, 2160), nsets=(12, 12), n_present=None, views=2, copies=6, batch=2,
               text="C4: 6000x4000 view, projector 3840x2160, 12 col + 12 row Gray bits + inverses + "
                    "white/black (50 frames)"),
    "c4band": dict(cam=(6000, 4000), proj=(3840, 2160), nsets=(12, 12), n_present=None, views=1, copies=1, batch=1,
                   text="C4 split: ONE 6000x4000 view, projector 3840x2160, 12 col + 12 row Gray bits + inverses + "
                        "white/black (50 frames), split over the ranks by bands of rows"),
    "c5": dict(cam=(3840, 2160), proj=(1920, 1080), nsets=(11, 11), n_present=None, views=4, copies=6, batch=4,
               text="C5: 3840x2160 view, projector 1920x1080, 11 col + 11 row Gray bits + inverses + "
                    "white/black (46 frames)"),
    "c5job": dict(cam=(3840, 2160), proj=(1920, 1080), nsets=(11, 11), n_present=None, views=576, copies=1, batch=4,
                  text="C5 job: 8 objects x 72 views at 3840x2160, projector 1920x1080, 11 col + 11 row Gray bits "
                       "+ inverses + white/black (46 frames), all views resident in HBM, one job per step, "
                       "views sharded over the ranks"),
}
REF_CALIBRATION_OF = {"c5job": "c5", "c4band": "c4"}     # workloads timed by tools/ref_vs_port.py under another name


def row_mode_of(wl) -> int:
    return int(wl.get("row_mode", 1))


# main3's decode-plan instances (csrc/slgpu.hip SLG_PLAN_*): (row_mode, (col pairs << 4) | row pairs)
PLAN_INSTANCES = {(1, 0xBA), (1, 0xBB), (1, 0xCC), (0, 0xA0)}


def plan_key(wl) -> int:
    """(used column pairs << 4) | used row pairs present, as fused_batch computes it (row_mode 0:
    no row pairs)."""
    from structured_light_for_3d_model_replication_amd import synth
    (PW, PH), (nc, nr) = wl["proj"], wl["nsets"]
    bc, br = synth.n_bits(PW), synth.n_bits(PH)
    present = wl["n_present"] if wl["n_present"] is not None else synth.frame_slots(PW, PH)
    cp = max(0, min(min(nc, bc), (present - 2) // 2))
    rp = 0 if row_mode_of(wl) == 0 else max(0, min(min(nr, br), (present - 2 - 2 * bc) // 2))
    return (cp << 4) | rp


def frames_used(wl) -> int:
    """Frames the decode reads per view: white + black + the used (pattern, inverse) pairs that
    are present ((2 + 2 (nc + nr)) per pixel; C1 has no row frames)."""
    from structured_light_for_3d_model_replication_amd import synth
    (PW, PH), (nc, nr) = wl["proj"], wl["nsets"]
    bc, br = synth.n_bits(PW), synth.n_bits(PH)
    used = 2 + 2 * (min(nc, bc) + min(nr, br))
    row_first = 2 + 2 * bc                     # row bit planes start here whatever nc is
    present = wl["n_present"] if wl["n_present"] is not None else synth.frame_slots(PW, PH)
    if present <= row_first:                   # no row frame present: only the column pairs count
        return min(present, 2 + 2 * min(nc, bc))
    return min(used, 2 + 2 * min(nc, bc) + (present - row_first))


# ----------------------------------------------------------------------------- CPU baseline
_CPU_JOB = None     # (views, calib, proj, nsets): inherited by the forked workers, never pickled
MAX_CPU_WORKERS = 64        # host-memory bound of the pool (~1 GB per C2 worker, ~4 at 4K)


def _cpu_worker(args):
    """One host process: the reference's operation sequence (oracle/sl_refseq.py) over views
    until `seconds` elapse -> (points, views, s)."""
    os.environ["OMP_NUM_THREADS"] = "1"
    from oracle import sl_refseq as R
    seconds, first = args
    views, cal, proj, nsets, row_mode = _CPU_JOB
    (PW, PH), (nc, nr) = proj, nsets
    done, pts, t0 = 0, 0, time.perf_counter()
    while True:
        v = views[(first + done) % len(views)]
        col, row, mask, tex = R.gray_decode(list(v.frames), v.texture, n_cols=PW, n_rows=PH, n_sets_col=nc,
                                            n_sets_row=nr)
        P, _ = R.reconstruct(col, row, mask, tex, cal, row_mode=row_mode)
        pts += len(P)
        done += 1
        if time.perf_counter() - t0 >= seconds:
            break
    return pts, done, time.perf_counter() - t0


def ref_over_port(config: str):
    """The committed calibration of the port against the reference itself for this workload
    (tools/ref_vs_port.py -> profiles/r4_ref_vs_port.json, build container): reference time /
    port time on the same views, or None."""
    p = os.path.join(ROOT, "profiles", "r4_ref_vs_port.json")
    try:
        with open(p) as f:
            c = json.load(f)["configs"].get(REF_CALIBRATION_OF.get(config, config))
    except (OSError, ValueError, KeyError):
        return None
    return None if c is None else {"ref_over_port": c["ref_over_port"], "ref_over_oracle": c["ref_over_oracle"],
                                   "median_s": c["median_s"], "views": c["views"],
                                   "source": "profiles/r4_ref_vs_port.json (tools/ref_vs_port.py)"}


def _cpu_model():
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name:"):
                return line.split(":", 1)[1].strip()
    except (OSError, subprocess.SubprocessError):
        pass
    return platform.processor() or "unknown"


def cpu_quota():
    """The cgroup CPU quota (frames.cpu_quota; None when unlimited)."""
    from structured_light_for_3d_model_replication_amd.frames import cpu_quota as q
    return q()


def _pool_rate(workers, seconds):
    import multiprocessing as mp
    with mp.get_context("fork").Pool(workers) as pool:
        res = pool.map(_cpu_worker, [(seconds, w) for w in range(workers)])
    return sum(r[0] for r in res), sum(r[1] for r in res), max(r[2] for r in res)


def cpu_baseline(views, cal, seconds, wl, config: str):
    """The reference CPU path on this host: ``oracle/sl_refseq.py``, the reference's own NumPy
    operation sequence (``server/processing.py:49-234``: boolean-scatter bit planes, the
    ``while np.any`` Gray loop, ``Nc[:, idx]`` gather, full-width temporaries; frames in memory,
    no PNG decode; ``Nc`` Fortran-ordered as ``scipy.io.loadmat`` hands it over), timed (i) in one
    process and (ii) on a process pool with one stream of views per worker on every CPU the lease
    owns -- the affinity mask, capped by the cgroup CPU quota when one is set and by
    ``MAX_CPU_WORKERS`` (more processes than the quota only time-share it: ``oversubscribed_2x``
    measures that, with twice as many workers for half the time).  ``ref_over_port``: the
    committed reference/port time ratio measured in the build container, where the reference
    exists (tools/ref_vs_port.py).  Runs on rank 0 BEFORE the GPU is touched (fork-safe), at
    every N.  ``value`` is the pool figure, the stronger baseline."""
    global _CPU_JOB
    import numpy as np
    cal = dict(cal, Nc=np.asfortranarray(cal["Nc"]))
    _CPU_JOB = (views, cal, wl["proj"], wl["nsets"], row_mode_of(wl))
    nsets = wl["nsets"]
    one = _cpu_worker((seconds, 0))
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    quota = cpu_quota()
    workers = max(1, min(avail, quota or avail, MAX_CPU_WORKERS))
    pts, n_views, wall = _pool_rate(workers, seconds)
    over = None
    if quota is not None and quota < avail and 2 * workers <= MAX_CPU_WORKERS:
        p2, v2, w2 = _pool_rate(min(avail, 2 * workers), seconds / 2)
        over = {"workers": min(avail, 2 * workers), "value": round(p2 / w2 / 1e6, 4), "views": v2,
                "what": "2x the quota in worker processes, ~half the time: the quota, not the process "
                        "count, bounds the host"}
    tag = wl["text"].split(":")[0]
    # the bit counts actually decoded: clamped to the projector's bits, row pairs only if present
    from structured_light_for_3d_model_replication_amd import synth
    bc, br = synth.n_bits(wl["proj"][0]), synth.n_bits(wl["proj"][1])
    dc = min(nsets[0], bc)
    dr = (frames_used(wl) - 2 - 2 * dc) // 2
    return {"value": round(pts / wall / 1e6, 4), "unit": "Mpoints/s", "cores": workers, "kind": "port",
            "sample": f"{n_views} {tag} views ({wl['cam'][0]}x{wl['cam'][1]}, {dc}+{dr} bits decoded, Otsu, "
                      f"row_mode {row_mode_of(wl)}) on {workers} worker processes x ~{seconds:.0f} s, frames in memory",
            "what": "oracle/sl_refseq.py: the reference's NumPy operation sequence for server/processing.py:49-234 "
                    "(in-memory frames, no PNG decode), one view stream per process",
            "ref_calibration": ref_over_port(config),
            "single_process_value": round(one[0] / one[2] / 1e6, 4),
            "single_process_sample": f"{one[1]} views in {one[2]:.1f} s, 1 process",
            "host_cpus": os.cpu_count(), "cpus_available": avail, "cpu_quota": quota,
            "oversubscribed_2x": over, "cpu_model": _cpu_model(), "numpy": np.__version__}


def rank0_cpu_baseline(args, rank: int, views, cal, wl):
    """``cpu_baseline`` on rank 0 at every N (the other ranks wait at the rendezvous meanwhile),
    None elsewhere or with ``--no-cpu-baseline``.  Must run before this process touches the GPU."""
    if rank != 0 or args.no_cpu_baseline:
        return None
    t = time.perf_counter()
    cpu = cpu_baseline(views, cal, args.cpu_seconds, wl, args.config)
    log(f"[rank 0] cpu baseline {cpu['value']} Mpts/s on {cpu['cores']} processes "
        f"({cpu['single_process_value']} on 1) in {time.perf_counter() - t:.1f}s")
    return cpu


def cpu_baseline_only(args, rank: int, world: int, cpu) -> None:
    """``--cpu-baseline-only``: the JSON line with the CPU baseline and no GPU part (any host;
    the ranks still rendezvous over gloo so a spawned run behaves as the GPU one does)."""
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "Mpoints/s", "n_gpus": world,
                          "config": {"workload": CONFIGS[args.config]["text"]}, "cpu_baseline": cpu}),
              file=getattr(args, "result_out", None) or RESULT_OUT, flush=True)


def load_traffic_per_view(config: str = "c2"):
    """The committed rocprofv3 PMC summary of the fused kernel on this config's bench shape
    (profiles/pmc_main_kernel.json for C2, pmc_main_kernel_<config>.json otherwise: HBM bytes
    per view, reads from the gfx950 request-size counters as calibrated by
    tools/fetch_probe.hip, writes from WRITE_SIZE), or None."""
    name = "pmc_main_kernel.json" if config == "c2" else f"pmc_main_kernel_{config}.json"
    p = os.path.join(ROOT, "profiles", name)
    if not os.path.exists(p):
        return None
    try:
        with open(p) as f:
            d = json.load(f)
        return d if d.get("hbm_bytes_per_view") else None
    except (OSError, ValueError):
        return None


def segments_holding(mask, stride: int, frame_idx, block: int = 64) -> int:
    """Aligned ``block``-byte pieces (64-B segments, 128-B lines) of the given frames (frame f at
    byte f * stride of the stack) that hold a valid pixel, summed over the frames: the pattern
    bytes a mask-first decode must read at that granularity.  A lane's 8-byte load never straddles
    one (lanes start at multiples of 8 px, stride % 16 == 0).  `mask` is a flat torch bool tensor
    of the view's pixels."""
    import torch
    shift = block.bit_length() - 1
    idx = torch.nonzero(mask.reshape(-1)).reshape(-1).to(torch.int64)
    total = 0
    for f in frame_idx:
        total += int(torch.unique((idx + f * stride) >> shift).numel())
    return total


def texture_lines_holding(mask, block: int = 128) -> int:
    """``block``-byte pieces of the [n_px][3] texture that main3 reads: 24 bytes per 8-pixel lane
    holding a valid pixel (mask first)."""
    import torch
    m = mask.reshape(-1)
    n = m.numel()
    pad = (-n) % 8
    if pad:
        m = torch.cat([m, torch.zeros(pad, dtype=m.dtype, device=m.device)])
    lanes = torch.nonzero(m.reshape(-1, 8).any(1)).reshape(-1).to(torch.int64)
    shift = block.bit_length() - 1
    return int(torch.unique(torch.cat([(24 * lanes) >> shift, (24 * lanes + 23) >> shift])).numel())


def _view_mask(frames, cfg, H, W, dev):
    from structured_light_for_3d_model_replication_amd import engine as E
    rec = _view_mask.__dict__.setdefault("rec", {}).get((H, W))
    if rec is None:
        rec = _view_mask.rec[(H, W)] = E.Reconstructor(H, W, device=dev)
    return rec.decode(frames, cfg)[2] != 0


def mask_first_segments(frames, cfg, H, W, dev, block: int = 64) -> int:
    """`segments_holding` of one device view's pattern frames, its mask from the maps path."""
    mask = _view_mask(frames, cfg, H, W, dev)
    n = min(frames.n_frames, 2 + 2 * (cfg.n_sets_col + cfg.n_sets_row))   # frames the plan reads
    if frames.stride % block == 0:       # every frame's pieces line up: one count per frame
        return (n - 2) * segments_holding(mask, frames.stride, [0], block)
    return segments_holding(mask, frames.stride, range(2, n), block)


def read_model(frames, cfg, H, W, dev, carried: bool = True, texture: bool = True) -> dict:
    """The HBM bytes one view's fused launch reads, piece by piece, at the 128-byte request size
    rocprofv3 shows for every main3 read (profiles/r4c/pmc_calibration.json: RDREQ_128B ~ all
    requests; tools/fetch_probe.hip's mask-gated 8 B/lane reads fetch exactly the 128-B lines
    holding a requested byte): white + black of every pixel, each pattern frame's lines holding a
    valid pixel, the texture lines of valid lanes, and -- in the steady-state pipeline -- the
    carried batch's white + black (Otsu partials)."""
    mask = _view_mask(frames, cfg, H, W, dev)
    n_px = H * W
    dense = 2 * ((n_px + 127) // 128) * 128
    out = {"white_black": dense,
           "pattern_lines128": 128 * mask_first_segments(frames, cfg, H, W, dev, 128),
           "texture_lines128": 128 * texture_lines_holding(mask, 128) if texture else 0,
           "carried_white_black": dense if carried else 0}
    out["total"] = sum(out.values())
    return out


RESULT_OUT = sys.stdout          # main() points it at the original stdout


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_mode(gpus: int, env) -> str:
    """How this invocation runs (decided before any GPU call):
    ``"spawn"`` -- ``--gpus N > 1`` and no launcher: start N rank processes here;
    ``"rank"``  -- a launcher (torchrun) set WORLD_SIZE and it equals ``--gpus``;
    ``"single"`` -- one process, N = 1.
    A WORLD_SIZE that disagrees with ``--gpus`` raises SystemExit (non-zero): a silent
    one-rank measurement labelled N GPUs is never produced."""
    if gpus < 1:
        raise SystemExit(f"--gpus must be >= 1 (got {gpus})")
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != gpus:
            raise SystemExit(f"WORLD_SIZE={ws} disagrees with --gpus {gpus}")
        return "rank" if gpus > 1 else "single"
    return "spawn" if gpus > 1 else "single"


def spawn_ranks(n: int, argv, script: str | None = None) -> int:
    """Run ``bench.py`` as ``n`` rank processes on this node (one per GPU, LOCAL_RANK = RANK),
    rendezvous on 127.0.0.1.  The parent never touches the GPU; rank 0's stdout (the JSON line)
    is this process's stdout, the other ranks' stdout goes to stderr.  Returns the first
    non-zero exit code, or 0."""
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, script or os.path.abspath(__file__), *argv], env=env,
                                      stdout=None if r == 0 else sys.stderr))
    rc = 0
    for p in procs:
        code = p.wait()
        if code and not rc:
            rc = code
            for q in procs:              # one rank failed: the others would wait at a barrier
                if q.poll() is None:
                    q.terminate()
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100, help="timed steps (one fused batch launch each)")
    ap.add_argument("--warmup", type=int, default=6)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="c2",
                    help="workload (default c2, the metric's configuration)")
    ap.add_argument("--views", type=int, default=None, help="distinct rendered views")
    ap.add_argument("--copies", type=int, default=None, help="device copies of each view in the pool")
    ap.add_argument("--batch", type=int, default=None, help="views per fused launch (<= 16)")
    ap.add_argument("--xyz", choices=["f32", "f64"], default="f32")
    ap.add_argument("--gray-texture", action="store_true",
                    help="gray captures (the reference scanner's 8-bit gray PNGs): the texture is frame 0 "
                         "replicated, run in GRAY texture mode (no texture reads); default: a colour texture")
    ap.add_argument("--objects", type=int, default=8, help="c5job: objects in the job")
    ap.add_argument("--views-per-object", type=int, default=72, help="c5job: turntable views per object")
    ap.add_argument("--distinct", type=int, default=1, help="c5job: rendered captures per object")
    ap.add_argument("--pipeline", choices=["serial", "overlap", "fused", "fused2"], default="fused2",
                    help="serial: stats + fused launch per batch on one stream; overlap: the next "
                         "batch's stats on a side stream during this batch's fused launch; fused: "
                         "batch k's fused launch computes batch k+2's histograms; fused2: the same on two "
                         "streams (batch k on stream k %% 2, carrying batch k+4), launches overlap")
    ap.add_argument("--settle-ms", type=float, default=60.0,
                    help="untimed launches (ms of GPU time) before the warmup, for the clocks to ramp")
    ap.add_argument("--kernel-events", choices=["launch", "region"], default="region",
                    help="HIP events per fused launch, or one pair around the timed region")
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-baseline-only", action="store_true",
                    help="print the JSON line with the CPU baseline alone (no GPU is touched)")
    ap.add_argument("--no-verify", action="store_true")
    args = ap.parse_args()
    mode = launch_mode(args.gpus, os.environ)
    if mode == "spawn":
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    # stdout carries exactly ONE line, the JSON result: runtime banners that native libraries
    # print to fd 1 (RCCL's version block, gloo's peer lines) go to stderr with the logs
    global RESULT_OUT
    RESULT_OUT = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)
    wl = CONFIGS[args.config]
    for k in ("views", "copies", "batch"):
        if getattr(args, k) is None:
            setattr(args, k, wl[k])
    args.result_out = RESULT_OUT         # (bench_c3 imports this file as module "bench")
    if args.gray_texture and args.config in ("c3", "c5job", "c4band"):
        raise SystemExit("--gray-texture applies to the single-view configs (c2, c4, c5)")
    if args.config == "c3":
        import bench_c3
        return bench_c3.main(args, wl)
    if args.config == "c5job":
        import bench_c5job
        return bench_c5job.main(args, wl)
    if args.config == "c4band":
        import bench_c4band
        return bench_c4band.main(args, wl)

    import numpy as np
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))

    from structured_light_for_3d_model_replication_amd import synth

    (W, H), (PW, PH), (NC, NR) = wl["cam"], wl["proj"], wl["nsets"]
    rig = synth.default_rig(W, H, PW, PH)
    cal = rig.tables()
    t = time.perf_counter()
    views = [synth.render_view(rig, view_deg=(rank * args.views + i) * 360.0 / (world * args.views),
                               seed=1000 * rank + i, n_present=wl["n_present"]) for i in range(args.views)]
    log(f"[rank {rank}] rendered {len(views)} views in {time.perf_counter() - t:.1f}s")
    cpu = rank0_cpu_baseline(args, rank, views, cal, wl)          # before the GPU is touched
    if args.cpu_baseline_only:
        return cpu_baseline_only(args, rank, world, cpu)

    # Rehearsal knobs for the multi-rank path on a one-GPU box (never set by the driver):
    # SLG_BENCH_DEVICE pins every rank to one device, SLG_BENCH_BACKEND=gloo replaces RCCL.
    if os.environ.get("SLG_BENCH_DEVICE"):
        local = int(os.environ["SLG_BENCH_DEVICE"])
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        backend = os.environ.get("SLG_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    from structured_light_for_3d_model_replication_amd import engine as E

    cfg = E.DecodeConfig(PW, PH, NC, NR, "otsu")
    row_mode, tol, f64 = row_mode_of(wl), 2.0, args.xyz == "f64"
    # Device pool: every rendered view uploaded `copies` times (distinct HBM buffers), so a batch
    # never shares frames with the batch before or after next -- e.g. the histograms a fused
    # launch computes for batch k+2 are cold HBM reads, as in a real turntable stream.
    if args.gray_texture:                             # cv2.imread(files[0]) of a gray PNG capture
        for v in views:
            v.texture = np.repeat(np.asarray(v.frames[0])[..., None], 3, axis=-1)
    dframes = [E.DeviceFrames(list(v.frames), E.GRAY if args.gray_texture else v.texture, device=dev)
               for _ in range(args.copies) for v in views]
    P = len(dframes)
    dcal = E.DeviceCalib(cal, H, W, device=dev)
    B = max(1, min(args.batch, E.MAX_VIEWS_PER_LAUNCH, P))
    s_main = torch.cuda.Stream(device=dev)
    s_stats = torch.cuda.Stream(device=dev)
    NSL = 4 if args.pipeline == "fused2" else 2      # workspace / cloud slots (batch k on slot k % NSL)
    beng = E.BatchReconstructor(H, W, B, device=dev, slots=NSL)
    clouds = [[E.Cloud(H * W, row_mode, f64, device=dev) for _ in range(B)] for _ in range(NSL)]
    preps = {}

    def prep(start, slot):
        """Batch of B consecutive pool views from `start` on workspace/cloud slot `slot`."""
        key = (start % P, slot)
        if key not in preps:
            fr = [dframes[(start + k) % P] for k in range(B)]
            preps[key] = beng.prepare(fr, cfg, dcal, clouds[slot], row_mode, tol, slot=slot)
        return preps[key]

    # Reference counts: every pool view once through the plain (non-pipelined) batch path.
    pts = []
    for v0 in range(0, P, B):
        pb = prep(v0, 0)
        beng.run(pb, stream=s_main)
        s_main.synchronize()
        pts += [int(clouds[0][k].count.item()) for k in range(B)]
    pts = pts[:P]
    seg_frames = [mask_first_segments(dframes[v], cfg, H, W, dev) for v in range(P)]
    models = [read_model(dframes[v], cfg, H, W, dev, carried=args.pipeline in ("fused", "fused2"),
                         texture=not args.gray_texture) for v in range(P)]

    K, Wm = args.steps, args.warmup
    # the whole run as ONE batch stream: warmup + timed + 2 look-ahead batches whose thresholds
    # the last timed launches prepare (carried histograms), as every other step does
    batches = [prep(b * B, b % NSL) for b in range(Wm + K + NSL)]
    # HIP events on the launch stream: one pair per fused launch ("launch": kernel time alone),
    # or one pair around the timed region ("region": launches + the gaps between them)
    n_ev = K if args.kernel_events == "launch" else 1
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n_ev)]
    for a, b in ev:                                  # materialise the HIP events
        a.record(s_main)
        b.record(s_main)
    torch.cuda.synchronize()
    frame_b = frames_used(wl) * H * W
    out_b = 30 if f64 else 18            # 3 B texture read + 12|24 B XYZ + 3 B BGR per point
    if args.gray_texture:
        out_b -= 3                       # GRAY mode: the colour comes from the white frame, no texture read

    def pool_views(b):
        return [(b * B + k) % P for k in range(B)]

    total_pts = sum(pts[v] for b in range(Wm, Wm + K) for v in pool_views(b))
    # algorithmic bytes: SURVEY §8(d)'s (every frame byte once + 18 B per point), and beside it
    # the mask-first decode's own (white + black of every pixel, each pattern frame's 64-byte
    # segments that hold a valid pixel, 18 B per point)
    wb_b = 2 * H * W
    bytes_alg = sum(wb_b + 64 * seg_frames[v] + out_b * pts[v] for b in range(Wm, Wm + K) for v in pool_views(b))
    bytes_dense = sum(frame_b + out_b * pts[v] for b in range(Wm, Wm + K) for v in pool_views(b))

    def run_range(lo, hi, events=None):
        if args.pipeline in ("overlap", "fused", "fused2"):
            beng.run_pipelined(batches, s_main, s_stats, events=events, mode=args.pipeline, start=lo, stop=hi)
        else:
            for k in range(lo, hi):
                beng.run(batches[k], events=None if events is None else events[k - lo], stream=s_main)

    # settle: the GPU's clocks ramp under load; the same launches, untimed, for args.settle_ms
    # of GPU time before the pipeline starts (then the cold start, warmup and timed steps)
    settle = max(0, int(round(args.settle_ms / 0.35)))
    if settle:
        sb = [prep(b * B, b % NSL) for b in range(settle + NSL)]
        if args.pipeline in ("overlap", "fused", "fused2"):
            beng.run_pipelined(sb, s_main, s_stats, mode=args.pipeline, start=0, stop=settle)
        else:
            for k in range(settle):
                beng.run(sb[k], stream=s_main)
    # cold start: the priming stats passes + the first launch, alone (not part of the metric)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run_range(0, min(1, Wm))
    torch.cuda.synchronize()
    cold_ms = (time.perf_counter() - t0) * 1e3
    run_range(min(1, Wm), Wm)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if args.kernel_events == "launch":
        run_range(Wm, Wm + K, events=[(a.cuda_event, b.cuda_event) for a, b in ev])
    else:
        ev[0][0].record(s_main)
        if args.pipeline == "fused2":
            s_stats.wait_event(ev[0][0])              # the second stream starts there too
        run_range(Wm, Wm + K)
        if args.pipeline == "fused2":
            s_main.wait_stream(s_stats)
        ev[0][1].record(s_main)
    t_enq = time.perf_counter() - t0              # host time to enqueue the K steps
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    kern_ms = sum(a.elapsed_time(b) for a, b in ev)
    helper_runs = sum(int(np.frombuffer(beng.header(s, k)[3084:3088].cpu().numpy().tobytes(), np.uint32)[0] & 2 != 0)
                      for s in range(NSL) for k in range(B))

    # ---- verification, outside the timed region: the last timed batch's clouds (nothing wrote
    # its slot after it) against the plain batch path (bitwise) and one view against the oracle
    verify = None
    if not args.no_verify:
        last = Wm + K - 1
        slot = last % NSL
        got = [(int(c.count.item()), c.xyz[: int(c.count.item())].clone(), c.bgr[: int(c.count.item())].clone())
               for c in clouds[slot]]
        ref_b = prep(last * B, slot)
        beng.stats(ref_b, stream=s_main)
        beng.main(ref_b, stream=s_main)
        s_main.synchronize()
        same = all(g[0] == int(c.count.item()) and torch.equal(g[1], c.xyz[: g[0]]) and torch.equal(g[2], c.bgr[: g[0]])
                   for g, c in zip(got, clouds[slot]))
        counts_ok = [g[0] for g in got] == [pts[v] for v in pool_views(last)]
        from oracle import sl_oracle as O
        v0 = pool_views(last)[0]
        vw = views[v0 % len(views)]
        oc, orow, om = O.decode_processing(list(vw.frames), n_cols=PW, n_rows=PH, n_sets_col=NC, n_sets_row=NR)
        Po, Co = O.reconstruct_processing(oc, orow, om, vw.texture, cal, row_mode=row_mode)
        xg = got[0][1].double().cpu().numpy()
        rel = float(np.max(np.abs(xg - Po) / np.maximum(np.abs(Po), 1e-3))) if len(Po) == len(xg) else None
        oracle_ok = (len(Po) == got[0][0] and np.array_equal(got[0][2].cpu().numpy(), Co)
                     and rel is not None and rel <= (0.0 if f64 else 1e-4))
        checksum = float(sum(g[1].double().sum().item() for g in got))
        verify = {"batch": last, "views": B, "pipelined_equals_plain_bitwise": bool(same),
                  "counts_equal_reference_pass": bool(counts_ok), "oracle_view": int(v0),
                  "oracle_count_and_colours_equal": bool(len(Po) == got[0][0]), "oracle_xyz_max_rel": rel,
                  "oracle_ok": bool(oracle_ok), "xyz_checksum": checksum}
        if not (same and counts_ok and oracle_ok):
            log(f"[rank {rank}] VERIFY FAILED: {verify}")
    bad = torch.tensor([0.0 if verify is None or (verify["pipelined_equals_plain_bitwise"] and verify["oracle_ok"]
                                                  and verify["counts_equal_reference_pass"]) else 1.0],
                       dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(bad, op=dist.ReduceOp.MAX)
    verify_failed = bool(bad.item())

    stats = torch.tensor([dt, float(total_pts), kern_ms, bytes_alg, bytes_dense], dtype=torch.float64, device=dev)
    if world > 1:
        tmax = stats[:1].clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        sums = stats[1:].clone()
        dist.all_reduce(sums, op=dist.ReduceOp.SUM)
        dt_max = float(tmax.item())
        all_pts, kern_sum, bytes_sum, dense_sum = (float(x) for x in sums.tolist())
    else:
        dt_max, all_pts, kern_sum, bytes_sum, dense_sum = dt, float(total_pts), kern_ms, bytes_alg, bytes_dense

    if rank == 0:
        launches = K * world
        kern_avg_s = kern_sum / launches / 1e3
        achieved = dense_sum / launches / kern_avg_s / 1e9          # SURVEY 8(d)'s algorithmic bytes
        mf_achieved = bytes_sum / launches / kern_avg_s / 1e9       # the mask-first decode's own bytes
        # the committed PMC summary of this instance: pmc_main_kernel[_<config>][_f64].json
        pkey = args.config if not f64 else ("f64" if args.config == "c2" else f"{args.config}_f64")
        pmc = load_traffic_per_view(pkey) if args.config in ("c1", "c2", "c4", "c5") else None
        pmc_name = "pmc_main_kernel.json" if pkey == "c2" else f"pmc_main_kernel_{pkey}.json"
        traffic_view = pmc["hbm_bytes_per_view"] if pmc else None
        n_pts_mean = float(np.mean(pts))
        model = {k: round(float(np.mean([m[k] for m in models]))) for k in models[0]}
        xyz_b = 24 if f64 else 12
        model["writes"] = round((xyz_b + 3) * n_pts_mean + 1024 * ((H * W + 4095) // 4096))   # cloud + Otsu partials
        model["total_with_writes"] = model["total"] + model["writes"]
        traffic_model = {"per_view": model,
                         "what": "bytes the fused launch must move per view (pool average) at the 128-B read "
                                 "request size the PMC counters show: white + black, pattern-frame lines holding a "
                                 "valid pixel, texture lines of valid lanes, the carried batch's white + black; "
                                 f"writes {xyz_b + 3} B per point ({xyz_b} B XYZ + 3 B BGR) + 1 KB of Otsu partials "
                                 "per tile"}
        if pmc:
            traffic_model["measured_per_view"] = {"reads": pmc.get("fetch_bytes_per_view"),
                                                  "writes": pmc.get("write_bytes_per_view"),
                                                  "source": pmc.get("tag")}
            traffic_model["measured_over_model"] = round(traffic_view / model["total_with_writes"], 4)
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                # committed PMC bytes (profiles/pmc_main_kernel*.json) are per view of this config
                "traffic": round(traffic_view * B) if traffic_view else None,
                "traffic_source": (f"profiles/{pmc_name} (rocprofv3 per launch: reads 128 x RDREQ_128B + "
                                   "64 x RDREQ_64B + 32 x RDREQ_32B, = FETCH_SIZE x 2 since all reads are 128-B "
                                   "requests, calibrated on known byte counts in profiles/r4c; writes WRITE_SIZE)")
                if traffic_view else None,
                "traffic_model": traffic_model,
                "kernel": (f"main3_kernel<{row_mode},{int(f64)},1,1,false,PLAN=0x{(0x100 if args.gray_texture else 0) | plan_key(wl):X}> "
                           f"(fused decode+triangulate+"
                           f"compaction, decode-plan instance, {B} views per launch)"
                           if (row_mode, plan_key(wl)) in PLAN_INSTANCES else
                           f"main3_kernel<{row_mode},{int(f64)},1,1> (fused decode+triangulate+compaction, {B} views per launch)"),
                "kernel_avg_us": round(kern_avg_s * 1e6, 2),
                "kernel_time": ("HIP events around each fused launch on its stream" if args.kernel_events == "launch"
                                else "HIP events around the timed region (both launch streams joined) / steps: "
                                     "the step period, gaps included"),
                "alg_bytes_per_launch": round(dense_sum / launches),
                "alg_bytes": (f"SURVEY 8(d): (2 + 2(nc+nr)) B per pixel (every frame once; {frames_used(wl)} frames) "
                              f"+ {out_b} B per point "
                              f"(3 B texture read, {24 if f64 else 12} B XYZ, 3 B BGR written)" if not args.gray_texture else
                              f"SURVEY 8(d) without the texture read: (2 + 2(nc+nr)) B per pixel + {out_b} B per point "
                              f"({24 if f64 else 12} B XYZ, 3 B BGR written; a gray capture's colour is its white frame)"),
                # the kernel reads a pattern frame only where a lane holds a valid pixel (SLG_MASK_FIRST),
                # so it moves fewer bytes than SURVEY's figure: the same time over the bytes it needs
                "mask_first": {"alg_bytes_per_launch": round(bytes_sum / launches),
                               "achieved": round(mf_achieved, 1), "frac": round(mf_achieved / HBM_PEAK_GBS, 4),
                               "what": "white + black of every pixel, each pattern frame's 64-B segments that hold "
                                       f"a valid pixel, {out_b} B per point"}}
        out = {
            "metric": METRIC,
            # a run whose clouds failed verification (any rank) measured nothing valid: no value,
            # non-zero exit (as bench_c5job)
            "value": None if verify_failed else round(all_pts / dt_max / 1e6, 2),
            "unit": "Mpoints/s",
            "n_gpus": world,
            "steps": K,
            "warmup": Wm,
            "ms_per_step": round(dt_max / K * 1e3, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": f"{wl['text']}, Otsu, row_mode {row_mode}"
                                   + (" tol 2.0" if row_mode == 1 else "") + f", XYZ {args.xyz} + BGR out"
                                   + (", gray capture (texture = frame 0, GRAY mode)" if args.gray_texture else ""),
                       "step": f"one batch of {B} views: one fused launch + its thresholds (steady-state pipeline)",
                       "us_per_view": round(dt_max / (K * B) * 1e6, 3),
                       "cold_start_ms": round(cold_ms, 3),
                       "settle_launches": settle,
                       "kernel_events": args.kernel_events,
                       "views_per_rank": len(views), "device_pool": P, "points_per_view": int(np.mean(pts)),
                       "batch_views": B,
                       "stats_pipeline": args.pipeline,
                       "lookback_helper_runs": helper_runs,
                       "host_enqueue_ms_per_step": round(t_enq / K * 1e3, 4),
                       "decode": "u8 compares, int32 codes; triangulation f64",
                       "parallelism": f"view-sharded x{world}"},
            "roofline": roof,
            "cpu_baseline": cpu,
            "verify": verify,
        }
        print(json.dumps(out), file=RESULT_OUT, flush=True)
    if world > 1:
        dist.destroy_process_group()
    if verify_failed:
        sys.exit(1)


if __name__ == "__main__":
    main()
