"""The final cloud gather of a sharded scan (north star: RCCL only for the final
point-cloud gather).  CPU: the C-ABI plan ``slg_gatherv_plan`` (offsets, which peers are
received from, argument checks) and the host plan of ``RcclCloudGather`` (dtype agreement across
ranks, padding slots dropped).  GPU: the C-ABI RCCL path with an empty root at world size 1, and
at world size 2 (two processes, one GPU each) when the box has two GPUs -- skipped on a one-GPU
box, which cannot host two RCCL ranks.  The reference has no collective (serial batch loop,
server/processing.py:319-330)."""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from conftest import ROOT

PKG = "structured_light_for_3d_model_replication_amd"


def _plan(n_ranks, rank, root, send_bytes, recv_bytes):
    from structured_light_for_3d_model_replication_amd import _native as N
    L = N.lib()
    rb = (ctypes.c_int64 * n_ranks)(*recv_bytes) if recv_bytes is not None else None
    off = (ctypes.c_int64 * (n_ranks + 1))()
    frm = (ctypes.c_int32 * max(1, n_ranks))()
    ops = L.slg_gatherv_plan(n_ranks, rank, root, send_bytes, rb, off, frm)
    return ops, list(off), list(frm), L.slg_last_error().decode()


def test_gatherv_plan_root_offsets_and_peers():
    ops, off, frm, _ = _plan(4, 1, 1, 30, [12, 30, 0, 7])
    assert ops == 2 and off == [0, 12, 42, 42, 49] and frm == [1, 0, 0, 1]
    ops, off, frm, _ = _plan(3, 0, 0, 0, [0, 0, 0])            # empty job: nothing moves
    assert ops == 0 and off == [0, 0, 0, 0] and frm == [0, 0, 0]
    ops, off, frm, _ = _plan(1, 0, 0, 5, [5])                   # world 1: the root's own copy only
    assert ops == 0 and off == [0, 5]


def test_gatherv_plan_senders():
    assert _plan(4, 2, 0, 9, None)[:1] == (1,)
    ops, _, frm, _ = _plan(4, 3, 0, 0, None)                    # zero-byte peers send nothing
    assert ops == 0 and frm[0] == 0


@pytest.mark.parametrize("args,msg", [
    ((2, 0, 0, 4, [5, 1]), "recv_bytes[root]"),
    ((2, 0, 0, 4, [4, -1]), "negative"),
    ((2, 0, 0, 4, None), "root needs"),
    ((2, 0, 2, 4, [4, 0]), "bad gatherv"),
    ((0, 0, 0, 0, None), "bad gatherv"),
    ((2, 1, 0, -1, None), "bad gatherv"),
])
def test_gatherv_plan_rejects(args, msg):
    ops, _, _, err = _plan(*args)
    assert ops < 0 and msg in err


def test_gather_plan_agrees_dtype_and_drops_padding():
    from structured_light_for_3d_model_replication_amd import distributed as D
    # root holds no views, its peers hold float64 clouds: the root sizes for 8-byte XYZ
    dt, counts = D.gather_plan([[-1, -1, 0], [100003, 1, 8], [0, -1, 8]], 2)
    assert dt == torch.float64 and counts == [[], [100003, 1], [0]]
    dt, counts = D.gather_plan([[-1, 0], [-1, 0]], 1)           # nobody holds anything
    assert dt == torch.float32 and counts == [[], []]
    dt, _ = D.gather_plan([[-1, 0], [-1, 0]], 1, torch.float64)
    assert dt == torch.float64
    with pytest.raises(ValueError):
        D.gather_plan([[5, 4], [6, 8]], 1)
    with pytest.raises(ValueError):
        D.gather_plan([[5, 4], [-1, 0]], 1, torch.float64)


def test_local_gather_row_flags_bad_arguments():
    """Invalid arguments on one rank become a flag in its count row (no local raise before the
    collective); the plan then raises on every rank alike."""
    from structured_light_for_3d_model_replication_amd import distributed as D
    f32 = (torch.zeros((3, 3), dtype=torch.float32), torch.zeros((3, 3), dtype=torch.uint8))
    f64 = (torch.zeros((2, 3), dtype=torch.float64), torch.zeros((2, 3), dtype=torch.uint8))
    assert D.local_gather_row([f32, f32], 3) == [3, 3, -1, 4]
    assert D.local_gather_row([], 2) == [-1, -1, 0]
    for clouds, dt in (([f32, f32, f32], None),     # more views than n_per_rank
                       ([f32, f64], None),          # mixed widths
                       ([f32], torch.float64)):     # not of the agreed dtype
        row = D.local_gather_row(clouds, 2, dt)
        assert row[2] == D.BAD_SLOT
        table = [row, D.local_gather_row([f64], 2)]
        with pytest.raises(ValueError, match="rank"):
            D.gather_plan(table, 2)


def _gloo_bad_rank_worker(rank, world, port, q):
    import torch.distributed as dist
    from structured_light_for_3d_model_replication_amd import distributed as D
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        x = (torch.zeros((4, 3), dtype=torch.float32), torch.zeros((4, 3), dtype=torch.uint8))
        clouds = [x, x, x] if rank == 1 else [x]          # rank 1 passes too many views
        row = torch.tensor(D.local_gather_row(clouds, 2), dtype=torch.int64)
        rows = [torch.empty_like(row) for _ in range(world)]
        dist.all_gather(rows, row)                         # every rank reaches the collective
        try:
            D.gather_plan([r.tolist() for r in rows], 2)
            q.put((rank, "no error"))
        except ValueError as e:
            q.put((rank, "ValueError" if "[1]" in str(e) else str(e)))
    finally:
        dist.destroy_process_group()


def test_gather_bad_rank_raises_on_every_rank_gloo():
    """World size 2 over gloo: rank 1's invalid arguments make BOTH ranks raise after the counts
    all-gather -- none is left waiting in the collective."""
    import multiprocessing as mp
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gloo_bad_rank_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs)
    assert sorted(q.get(timeout=5) for _ in range(2)) == [(0, "ValueError"), (1, "ValueError")]


# ------------------------------------------------------------------------------------- GPU
def _rank_clouds(rank, case, f64):
    """Deterministic ragged clouds per (rank, case): list of (xyz, bgr) numpy arrays."""
    sizes = {("root_empty", 0): [], ("root_empty", 1): [100003, 1, 0],
             ("ragged", 0): [7, 0, 65536], ("ragged", 1): [1]}[(case, rank)]
    rng = np.random.default_rng(1000 * rank + len(case))
    dt = np.float64 if f64 else np.float32
    return [(rng.standard_normal((n, 3)).astype(dt) * 500, rng.integers(0, 256, (n, 3), dtype=np.uint8)) for n in sizes]


def _run_case(case, f64, world, rank, device):
    from structured_light_for_3d_model_replication_amd import distributed as D
    mine = _rank_clouds(rank, case, f64)
    parts = [(torch.from_numpy(x).to(device), torch.from_numpy(b).to(device)) for x, b in mine]
    g = D.RcclCloudGather(device=device)
    s = torch.cuda.Stream(device=device)
    try:
        got = g.gather(parts, 3, root=0, stream=s, xyz_dtype=torch.float64 if f64 else None)
        s.synchronize()
    finally:
        g.close()
    if rank != 0:
        assert got is None
        return
    want = [c for r in range(world) for c in _rank_clouds(r, case, f64)]
    assert len(got) == len(want)
    for (gx, gb), (wx, wb) in zip(got, want):
        assert np.array_equal(gx.cpu().numpy(), wx) and np.array_equal(gb.cpu().numpy(), wb)
    rx, _ = g.last_buffers
    assert rx.dtype == (torch.float64 if f64 else torch.float32)
    assert rx.shape[0] == sum(len(w[0]) for w in want)


@pytest.mark.gpu
def test_rccl_gather_world1_empty_root():
    """World size 1 through the C ABI: an empty root with an explicit dtype, then ragged views."""
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a ROCm device")
    dev = torch.device("cuda", 0)
    _run_case("root_empty", True, 1, 0, dev)
    _run_case("ragged", False, 1, 0, dev)


WORKER = r'''
import os, sys
sys.path.insert(0, {root!r}); sys.path.insert(0, os.path.join({root!r}, "tests"))
import torch, torch.distributed as dist
rank = int(os.environ["RANK"])
torch.cuda.set_device(rank)
dev = torch.device("cuda", rank)
dist.init_process_group("nccl", device_id=dev)
import test_gather as T
for case, f64 in (("root_empty", True), ("ragged", False), ("ragged", True)):
    T._run_case(case, f64, 2, rank, dev)
dist.barrier()
dist.destroy_process_group()
print("RANK_OK", rank)
'''


@pytest.mark.gpu
def test_rccl_gather_world2_point_to_point(tmp_path):
    """Two ranks, one GPU each: ncclSend/ncclRecv move ragged clouds (an empty root with float64
    peers, a zero-point view, a 65536-point view) to rank 0, bit for bit."""
    if torch.cuda.device_count() < 2:
        pytest.skip("needs 2 GPUs (this box has %d): two RCCL ranks cannot share one GPU" % torch.cuda.device_count())
    script = tmp_path / "worker.py"
    script.write_text(WORKER.format(root=ROOT))
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = [subprocess.Popen([sys.executable, str(script)], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                              env=dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r),
                                       MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port)))
             for r in range(2)]
    outs = [p.communicate(timeout=100)[0] for p in procs]
    for r, (p, o) in enumerate(zip(procs, outs)):
        assert p.returncode == 0 and f"RANK_OK {r}" in o, o[-3000:]
