"""CPU tests of bench.py's launch handling: ``--gpus N`` runs N rank processes itself when no
launcher set WORLD_SIZE, a launcher's WORLD_SIZE must agree with ``--gpus``, and rank 0's
stdout is the only stdout (the driver parses one JSON line)."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_launch_mode_rules():
    assert bench.launch_mode(1, {}) == "single"
    assert bench.launch_mode(4, {}) == "spawn"
    assert bench.launch_mode(8, {"WORLD_SIZE": "8"}) == "rank"
    assert bench.launch_mode(1, {"WORLD_SIZE": "1"}) == "single"
    for gpus, env in ((2, {"WORLD_SIZE": "1"}), (1, {"WORLD_SIZE": "8"}), (0, {})):
        with pytest.raises(SystemExit):
            bench.launch_mode(gpus, env)


def test_world_size_mismatch_exits_nonzero():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "disagrees" in r.stderr and r.stdout == ""


def test_spawn_ranks_env_and_stdout(tmp_path):
    """Two ranks through a gloo rendezvous on 127.0.0.1: each sees RANK/LOCAL_RANK/WORLD_SIZE,
    an all-reduce crosses the ranks, only rank 0's line reaches stdout."""
    script = tmp_path / "rank.py"
    script.write_text(
        "import json, os, sys, torch, torch.distributed as dist\n"
        "dist.init_process_group('gloo')\n"
        "t = torch.tensor([float(os.environ['RANK']) + 1.0]); dist.all_reduce(t)\n"
        "print(json.dumps({'rank': int(os.environ['RANK']), 'local': int(os.environ['LOCAL_RANK']),\n"
        "                  'world': dist.get_world_size(), 'sum': float(t.item()), 'argv': sys.argv[1:]}))\n"
        "dist.destroy_process_group()\n")
    code = (f"import sys; sys.path.insert(0, {ROOT!r}); import bench\n"
            f"sys.exit(bench.spawn_ranks(2, ['--gpus', '2'], script={str(script)!r}))\n")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr
    # (gloo prints its peer banner on fd 1; bench.py moves such banners to stderr itself)
    lines = [json.loads(l) for l in r.stdout.strip().splitlines() if l.startswith("{")]
    assert lines == [{"rank": 0, "local": 0, "world": 2, "sum": 3.0, "argv": ["--gpus", "2"]}]
    assert '"rank": 1' in r.stderr


@pytest.mark.parametrize("config", ["c2", "c3"])
def test_spawned_two_rank_line_carries_cpu_baseline(config):
    """``bench.py --gpus 2`` (self-spawned ranks, the driver's N>1 lines): rank 0 times the
    reference CPU path before touching the GPU, so the N>1 line carries ``cpu_baseline`` too
    (``--cpu-baseline-only`` stops there; no GPU is needed)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--config", config,
                        "--views", "1" if config == "c2" else "2", "--cpu-seconds", "0.2", "--cpu-baseline-only"],
                       env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(l) for l in r.stdout.strip().splitlines() if l.startswith("{")]
    assert len(lines) == 1 and lines[0]["n_gpus"] == 2
    cpu = lines[0]["cpu_baseline"]
    assert cpu is not None and cpu["value"] > 0 and cpu["kind"] == "port" and cpu["cores"] >= 1
    assert "sl_refseq" in cpu["what"]


def test_spawn_ranks_propagates_failure(tmp_path):
    script = tmp_path / "fail.py"
    script.write_text("import os, sys\nsys.exit(3 if os.environ['RANK'] == '1' else 0)\n")
    assert bench.spawn_ranks(2, [], script=str(script)) == 3


def test_mask_first_segments_count():
    """bench.segments_holding (the mask-first algorithmic bytes): 64-byte segments of each frame
    that hold a valid pixel, checked against a brute-force count, with frames at offsets that
    are and are not multiples of 64."""
    import numpy as np
    import torch
    rng = np.random.default_rng(5)
    n_px = 5000
    mask = rng.random(n_px) < 0.05
    mask[:70] = True                                   # a run across a segment boundary
    for stride, frames in ((5056, [0, 2, 3]), (5008, [0, 1, 2, 5])):
        want = 0
        for f in frames:
            segs = set(((f * stride + np.nonzero(mask)[0]) >> 6).tolist())
            want += len(segs)
        assert bench.segments_holding(torch.from_numpy(mask), stride, frames) == want
    assert bench.segments_holding(torch.zeros(n_px, dtype=torch.bool), 5056, [0, 1]) == 0
