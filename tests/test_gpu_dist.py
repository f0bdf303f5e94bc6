"""The multi-GPU exchange on the GPU, on a one-GPU box:

- libsurfcomm's RCCL communicator with one rank: surfhip_allgather of a slab
  packed by surfhip_pack_slab_cap from real detect_batch output (and the
  overflow flag of a slab beyond its capacity);
- two ranks (gloo control plane, both on cuda:0): each detects its shard on
  the GPU, packs the PRODUCT slab format at a fixed capacity, all-gathers;
  every rank then holds every frame's result, equal to the oracle;
- bench.py's world > 1 loop itself, launched by torch.distributed.run with 2
  ranks and the host-staged gloo exchange (RCCL refuses two ranks on one GPU).
"""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import REPO, assert_points_equal
from test_gpu_parity import compare_frame, gpu_run

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_comm_single_rank_allgather(surf):
    """In the test process (no torch: one HIP runtime, /opt/rocm's) libsurfcomm
    resolves /opt/rocm's RCCL; under torch it binds torch's bundled copy."""
    w, h, n = 640, 480, 3
    frames = surf.synth_frames(n, w, h, first=11)
    param = surf.make_param(4, 4.0, upright=True)
    ref = gpu_run(surf, param, frames, w, h, max_pts=4096)
    det = surf.Detector(param, w, h, max_batch=n, max_pts=4096)
    pitch = frames.shape[2]
    fb = surf.DeviceBuffer(frames.nbytes)
    fb.upload(frames)
    pb = surf.DeviceBuffer(48 * n * 4096)
    db = surf.DeviceBuffer(4 * n * 4096 * 64)
    cb = surf.DeviceBuffer(4 * n)
    det.detect_batch(fb.ptr, n, pitch, h * pitch, pb.ptr, db.ptr, cb.ptr)
    used = det.slab_bytes(n, int(ref["counts"].sum()))
    cap = surf.align_up(used + 1000, 256)
    send = surf.DeviceBuffer(cap)
    recv = surf.DeviceBuffer(cap)
    det.pack_slab_cap(pb.ptr, db.ptr, cb.ptr, n, send.ptr, cap)
    comm = surf.Comm(1, 0, surf.comm_unique_id())
    comm.allgather(send.ptr, cap, recv.ptr)
    tot = surf.DeviceBuffer(16)
    tot.upload(np.array([5, -7], np.int64))
    comm.allreduce_sum_i64(tot.ptr, 2)
    surf.synchronize()
    assert tot.download(np.int64, 2).tolist() == [5, -7]
    g = recv.download(np.uint8, cap)
    assert g.tobytes() == send.download(np.uint8, cap).tobytes()
    assert surf.slab_flags(g) == 0
    c, pts, desc = surf.parse_slab(g)
    np.testing.assert_array_equal(c, ref["counts"])
    o = 0
    for f in range(n):
        assert_points_equal(pts[o:o + c[f]], ref["pts"][f])
        assert desc[o:o + c[f]].tobytes() == ref["desc"][f].tobytes()
        o += c[f]
    # a capacity below the batch's slab: header + counts + overflow flag only
    small = surf.DeviceBuffer(4096)
    det.pack_slab_cap(pb.ptr, db.ptr, cb.ptr, n, small.ptr, 4096)
    surf.synchronize()
    s = small.download(np.uint8, 4096)
    assert surf.slab_flags(s) & surf.SLAB_OVERFLOW
    np.testing.assert_array_equal(s[16:16 + 4 * n].view(np.int32), ref["counts"])
    comm.close()
    det.close()


def _worker(rank, world, port, n_frames, w, h, q):
    sys.path.insert(0, HERE)
    import torch
    import torch.distributed as dist
    from conftest import load_surf_amd

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    surf = load_surf_amd()
    surf.set_device(0)
    start, count = surf.dist.shard_range(n_frames, world, rank)
    frames = surf.synth_frames(count, w, h, first=start)
    pitch = frames.shape[2]
    param = surf.make_param(4, 4.0, upright=True)
    max_pts = 4096
    det = surf.Detector(param, w, h, max_batch=count, max_pts=max_pts)
    fb = surf.DeviceBuffer(frames.nbytes)
    fb.upload(frames)
    pb = surf.DeviceBuffer(48 * count * max_pts)
    db = surf.DeviceBuffer(4 * count * max_pts * 64)
    cb = surf.DeviceBuffer(4 * count)
    det.detect_batch(fb.ptr, count, pitch, h * pitch, pb.ptr, db.ptr, cb.ptr)
    cap = 1 << 21                                   # fixed per-rank capacity, agreed up front
    slab = surf.DeviceBuffer(cap)
    det.pack_slab_cap(pb.ptr, db.ptr, cb.ptr, count, slab.ptr, cap)
    surf.synchronize()
    buf = torch.from_numpy(slab.download(np.uint8, cap))
    out, _ = surf.dist.allgather_slabs(dist, torch, buf, cap, world)
    per_rank = surf.dist.split_gathered(out.numpy(), world, cap, surf.parse_slab)
    flags = [surf.slab_flags(out.numpy()[r * cap:(r + 1) * cap]) for r in range(world)]
    q.put((rank, flags, np.concatenate([c for c, _, _ in per_rank]).tolist(),
           np.concatenate([p for _, p, _ in per_rank]).tobytes(),
           np.concatenate([d for _, _, d in per_rank]).tobytes()))
    det.close()
    dist.barrier()
    dist.destroy_process_group()


def test_two_ranks_product_slabs_gloo(surf, orc):
    import multiprocessing as mp                    # not torch's: the test process stays torch-free

    world, n_frames, w, h = 2, 5, 640, 480
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_frames, w, h, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    try:
        results = [q.get(timeout=150) for _ in range(world)]
    finally:
        for pr in procs:
            pr.join(timeout=60)
            if pr.is_alive():
                pr.kill()
    assert all(pr.exitcode == 0 for pr in procs)
    frames = surf.synth_frames(n_frames, w, h)
    op = orc.make_param(4, 4.0, upright=True)
    ref = [orc.detect(op, frames[f], w, h, max_pts=4096) for f in range(n_frames)]
    for rank, flags, c, pb, db in results:
        assert flags == [0] * world, rank
        assert c == [len(r[0]) for r in ref], rank
        pts = np.frombuffer(pb, surf.POINT_DTYPE)
        desc = np.frombuffer(db, np.float32).reshape(len(pts), -1)
        o = 0
        for f in range(n_frames):
            compare_frame(pts[o:o + c[f]], desc[o:o + c[f]], ref[f][0], ref[f][1], True)
            o += c[f]


def test_bench_world2_loop_gloo_rehearsal():
    """bench.py's N > 1 loop (fixed slab capacity agreed once, pack_slab_cap
    into the gather buffer, comm stream + events, post-run slab checks) with
    two ranks on one GPU."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(REPO, "bench.py"), "--gpus", "2", "--exchange", "gloo", "--batch", "8",
           "--steps", "4", "--warmup", "2", "--no-cpu", "--no-profile"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(line) == 1, r.stdout
    d = json.loads(line[0])
    assert d["n_gpus"] == 2 and d["value"] > 0
    ex = d["exchange"]
    assert ex["backend"] == "gloo" and ex["keypoints_gathered_per_step"] == d["keypoints_per_step"] > 0


@pytest.mark.parametrize("gather", ["full", "points"])
def test_bench_spawns_its_ranks(gather):
    """`python bench.py --gpus 2` with no launcher starts its own two rank
    processes (before touching the GPU) and prints ONE line with n_gpus 2 and
    the exchange's bytes and time per step."""
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--exchange", "gloo", "--gather", gather,
           "--batch", "8", "--steps", "4", "--warmup", "2", "--no-cpu"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=REPO, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(line) == 1, r.stdout
    d = json.loads(line[0])
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["steps"] == 4
    ex = d["exchange"]
    assert ex["mode"] == gather and ex["keypoints_gathered_per_step"] == d["keypoints_per_step"] > 0
    per_kp = 48 + (4 * 64 if gather == "full" else 0)
    assert ex["payload_bytes_per_step"] == ex["keypoints_gathered_per_step"] * per_kp
    assert ex["allgather_ms_per_step"] > 0 and ex["gathered_bytes_per_step"] == 2 * ex["slab_cap_bytes"]


def test_bench_single_gpu_exchange_probe():
    """N = 1: the line carries a 1-rank RCCL all-gather of the real slab."""
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--batch", "8", "--steps", "3",
                        "--warmup", "1", "--no-cpu"], capture_output=True, text=True, timeout=240, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), r.stdout      # RCCL's banner goes to stderr
    d = json.loads(lines[0])
    ex = d["exchange"]
    assert "error" not in ex, ex
    assert ex["full"]["bytes_equal"] and ex["points"]["bytes_equal"]
    assert ex["full"]["slab_bytes"] > ex["points"]["slab_bytes"] > 0


def test_bench_exchange_proxy():
    """N = 1 with --exchange-proxy 8: the step re-timed with
    the HBM traffic an 8-rank all-gather lands on this GPU, (8-1) x slab
    bytes per step beside compute, in both gather modes."""
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--batch", "16", "--steps", "4",
                        "--warmup", "1", "--no-cpu", "--no-exchange-probe", "--no-stream-peak", "--exchange-proxy", "8"],
                       capture_output=True, text=True, timeout=240, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    px = json.loads(lines[0])["exchange_proxy"]
    assert px["nranks"] == 8 and px["base_ms_per_step"] > 0
    for mode in ("full", "points"):
        m = px[mode]
        assert m["received_bytes_per_step"] >= 7 * m["slab_bytes"]
        for at in ("pack", "describe"):          # copy issued after the pack / at the next describe
            assert m[at]["ms_per_step"] > 0 and m[at]["copy_ms"] > 0, m
    assert px["full"]["slab_bytes"] > px["points"]["slab_bytes"]


_UNDER_TORCH = r"""
import importlib.util, sys
import torch
spec = importlib.util.spec_from_file_location("surf_amd", sys.argv[1] + "/cuda-surf_amd/__init__.py",
                                              submodule_search_locations=[sys.argv[1] + "/cuda-surf_amd"])
surf = importlib.util.module_from_spec(spec); sys.modules["surf_amd"] = surf; spec.loader.exec_module(surf)
dev = torch.device("cuda", 0)
s = torch.cuda.Stream(dev)
comm = surf.Comm(1, 0, surf.comm_unique_id())
src = torch.arange(1 << 20, dtype=torch.int32, device=dev).view(torch.uint8)
dst = torch.zeros_like(src)
comm.allgather(src.data_ptr(), src.numel(), dst.data_ptr(), s.cuda_stream)
s.synchronize()
assert torch.equal(src, dst)
comm.close()
print("UNDER_TORCH_OK")
"""


def test_comm_under_torch():
    """bench.py's arrangement: torch loaded first, so libsurfcomm binds the
    RCCL and HIP runtime torch bundles (one copy of each in the process)."""
    r = subprocess.run([sys.executable, "-c", _UNDER_TORCH, REPO], capture_output=True, text=True, timeout=180)
    assert r.returncode == 0 and "UNDER_TORCH_OK" in r.stdout, r.stderr[-3000:]
