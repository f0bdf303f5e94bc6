"""Multi-process (gloo, world_size 2 and 8, CPU) test of the frame sharding and the
single all-gather of compacted result slabs.  Each rank runs
the CPU oracle on its contiguous shard of a synthetic batch, packs the
results in the libsurfhip slab format, and all-gathers; every rank must then
hold exactly the concatenation of the per-frame single-process results.
World 8 with 11 frames rehearses config #4's layout (one rank per GPU of a
node) with a batch that 8 does not divide: shards of 1 and 2 frames."""
from __future__ import annotations

import os
import socket
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n_frames, w, h, q):
    sys.path.insert(0, HERE)
    import torch
    import torch.distributed as dist
    from conftest import load_oracle, load_surf_amd

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    surf = load_surf_amd()
    orc = load_oracle()
    start, count = surf.dist.shard_range(n_frames, world, rank)
    frames = surf.synth_frames(count, w, h, first=start)
    p = orc.make_param(4, 4.0, upright=True)
    counts, pts, descs = [], [], []
    for f in range(count):
        pt, d, _ = orc.detect(p, frames[f], w, h)
        counts.append(len(pt))
        pts.append(pt)
        descs.append(d)
    assert count >= 1
    slab = surf.build_slab(np.array(counts, np.int32), np.concatenate(pts), np.concatenate(descs))
    cap = surf.dist.agree_slab_size(dist, torch, len(slab), "cpu")
    buf = torch.zeros(cap, dtype=torch.uint8)
    buf[:len(slab)] = torch.from_numpy(slab)
    out, _ = surf.dist.allgather_slabs(dist, torch, buf, cap, world)
    per_rank = surf.dist.split_gathered(out.numpy(), world, cap, surf.parse_slab)
    allc = np.concatenate([c for c, _, _ in per_rank])
    allp = np.concatenate([pp for _, pp, _ in per_rank])
    alld = np.concatenate([dd for _, _, dd in per_rank])
    q.put((rank, allc.tolist(), allp.tobytes(), alld.tobytes()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n_frames", [(2, 4), (2, 3), (8, 11)])
def test_shard_and_allgather_gloo(world, n_frames):
    torch = pytest.importorskip("torch")
    import torch.multiprocessing as mp
    from conftest import load_oracle, load_surf_amd

    w, h = 160, 120
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_frames, w, h, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    results = [q.get(timeout=300) for _ in range(world)]
    assert sorted(r[0] for r in results) == list(range(world))
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    # single-process reference: all frames in order
    surf = load_surf_amd()
    orc = load_oracle()
    frames = surf.synth_frames(n_frames, w, h)
    p = orc.make_param(4, 4.0, upright=True)
    ref = [orc.detect(p, frames[f], w, h) for f in range(n_frames)]
    ref_c = [len(r[0]) for r in ref]
    ref_p = np.concatenate([r[0] for r in ref]).tobytes()
    ref_d = np.concatenate([r[1] for r in ref]).tobytes()
    for rank, c, pb, db in results:
        assert c == ref_c, rank
        assert pb == ref_p, rank
        assert db == ref_d, rank
