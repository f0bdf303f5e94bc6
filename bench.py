#!/usr/bin/env python3
"""bench.py -- SURF detect+describe throughput on MI355X.

Metric (BASELINE.json): 1080p frames/sec (detect+describe); keypoints/s is
reported beside it.  Workload (config #3, the HBM-bound Hessian roofline run):
a batch of 256 synthetic 1920x1080 u8 frames per GPU, 4 octaves, 64-D upright
descriptors, thresh=4, sampling 2, init mask 9 (main.cpp:187-204), resident
in HBM before the timed region.  One step = the whole hot path over one batch:
integral -> Hessian (all octaves) -> NMS + interpolation -> canonical sort ->
descriptors.

Multi-GPU (config #4 at N = 8): one process per GPU.  Under
torch.distributed.run the ranks come from RANK/LOCAL_RANK/WORLD_SIZE (which
must equal --gpus); a plain `python bench.py --gpus N` starts the N rank
processes itself before anything touches the GPU.  Each rank processes its
own 256 frames (weak scaling) and the compacted result slab of every rank is
all-gathered over xGMI through libsurfcomm's surfhip_allgather (RCCL, the
C-ABI data path; --gather full = SurfPoints + descriptors, points = SurfPoints
only, descriptors stay sharded) into a per-rank capacity agreed once before
the timed region; the gather of batch i overlaps the compute of batch i+1 on
a comm stream.  The control plane (barriers, the capacity agreement, the
RCCL id broadcast, the max-over-ranks time) runs over a gloo group, so each
process holds exactly one RCCL communicator.  The run fails (exit 3, no
JSON) if any frame hit max_pts, the candidate capacity overflowed, or a slab
exceeded its capacity.

Rank 0 prints ONE JSON line (the driver's contract), with a `roofline` object
for the Hessian stage (HIP events on the detector's stream; algorithmic
bytes = integral image read once + valid responses written), an `exchange`
object (all-gather bytes and time per step; at N = 1 a 1-rank RCCL
all-gather of the real slab) and a `cpu_baseline` object (the oracle/ CPU
restatement on a bounded sample of the same frames, rank 0 at N = 1 only).
"""
from __future__ import annotations

import argparse
import importlib.util
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
METRIC = "1080p frames/sec (detect+describe) at 1/2/4/8 MI355X; keypoints/sec"   # BASELINE.json


def load_surf():
    pkg = os.path.join(REPO, "cuda-surf_amd")
    spec = importlib.util.spec_from_file_location("surf_amd", os.path.join(pkg, "__init__.py"),
                                                  submodule_search_locations=[pkg])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["surf_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


# ----------------------------------------------------------- rank launcher

def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(args) -> int | None:
    """`--gpus N` without a launcher: start N rank processes (fresh
    interpreters, so no process that touched the GPU ever execs) and return
    the job's exit code; None when this process is itself a rank.  Runs
    before torch is imported."""
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None:
        if int(env_world) != args.gpus:
            print(f"bench.py: --gpus {args.gpus} disagrees with WORLD_SIZE={env_world}", file=sys.stderr,
                  flush=True)
            sys.exit(2)
        return None
    if args.gpus <= 1:
        return None
    n = args.gpus
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc, live, kill_at = 0, list(procs), None
    while live:
        for p in list(live):
            r = p.poll()
            if r is None:
                continue
            live.remove(p)
            if r != 0 and rc == 0:
                rc = r if r > 0 else 128 - r
                for q in live:                     # a lost rank would leave the others in a collective
                    q.terminate()
                kill_at = time.time() + 20
        if kill_at is not None and time.time() > kill_at:
            for q in live:
                q.kill()
            kill_at = None
        time.sleep(0.1)
    return rc


# ------------------------------------------------------------ CPU baseline

def cpu_share() -> tuple[int, dict]:
    """Threads for the CPU baseline: the CPUs this job may use (affinity,
    capped by a cgroup CPU quota and by the job's OMP_NUM_THREADS share),
    plus what the host has."""
    host = os.cpu_count() or 1
    try:
        visible = len(os.sched_getaffinity(0))
    except AttributeError:
        visible = host
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    omp = int(omp) if omp and omp.isdigit() else None
    share = visible
    for lim in (quota, omp):
        if lim:
            share = min(share, lim)
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return share, {"host_cpus": host, "affinity_cpus": visible, "cgroup_cpu_quota": quota,
                   "omp_num_threads": omp, "cpu_model": model}


def cpu_baseline(frames, w, h, args):
    """The oracle (a scalar C restatement of the reference) on a bounded sample:
    passes over chunks of the same frames until about --cpu-seconds of wall
    time, one frame per thread, on every CPU this job may use."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle  # test infrastructure: the baseline only, never the measured path
    chunk = min(args.cpu_frames, frames.shape[0])
    share, host = cpu_share()
    threads = args.cpu_threads or share
    p = oracle.make_param(args.octaves, args.thresh, False, 9, 2, bool(args.upright), bool(args.extend), 4)
    secs, pts, n, start = 0.0, 0, 0, 0
    while secs < args.cpu_seconds or n == 0:
        sub = frames[start:start + chunk]
        s, k = oracle.bench_frames(p, sub, w, h, args.max_pts, threads)
        secs += s
        pts += k
        n += sub.shape[0]
        start = (start + chunk) % frames.shape[0]
    out = {"value": round(n / secs, 3), "unit": "frames/s", "cores": threads, "kind": "port",
           "sample": f"{n} frames ({chunk}-frame chunks cycling over the {frames.shape[0]} synthetic {w}x{h} "
                     f"frames of the GPU batch), detect+describe, one frame per thread, {threads} threads "
                     f"(the job's CPU share), {pts} keypoints, {secs:.2f} s wall; the herbertbay CPU SURF "
                     f"named by BASELINE is not available offline, the oracle port stands in for it"}
    out.update(host)
    return out


def pmc_traffic(args):
    """Per-batch HBM bytes of the Hessian stage from the committed rocprofv3
    --pmc passes of this build (profiles/hessian_pmc.json, FETCH_SIZE +
    WRITE_SIZE, gfx950-corrected; tools/profile_round.sh + tools/summarize_profiles.py), with the
    profile's tag -- (bytes, tag) or (None, None).  A PMC pass cannot run
    inside this process (rocprofv3 wraps the whole program), so the figure is
    labelled with the run it came from."""
    path = args.pmc_json or os.path.join(REPO, "profiles", "hessian_pmc.json")
    try:
        with open(path) as fh:
            d = json.load(fh)
        if d.get("config") == f"{args.batch}x{args.width}x{args.height}x{args.octaves}":
            return float(d["bytes_per_launch"]), d.get("tag")
    except (OSError, ValueError, KeyError):
        pass
    return None, None


def hessian_profile(args, kernels: str):
    """The committed kernel-trace + SQ-counter summary of this config's
    Hessian stage (profiles/hessian_profile.json, one entry per config key
    "BxWxHxOct[r|u][x]", written by tools/hessian_profile.py from the
    rocprofv3 runs of tools/profile_round.sh): the sum of the stage kernels'
    rocprof AVERAGE durations (the judge's rule), the bound the counters
    show, and the profile's tag -- or None when there is no entry for this
    config or its kernels are not the ones this build launches."""
    path = os.path.join(REPO, "profiles", "hessian_profile.json")
    try:
        with open(path) as fh:
            d = json.load(fh)
    except (OSError, ValueError):
        return None
    e = d.get(profile_key(args))
    if not e:
        return None
    import re
    names = sorted(set(re.findall(r"k_\w+", kernels)))
    if sorted(e.get("kernels_avg_ns", {})) != names:
        return None
    return e


def profile_key(args) -> str:
    return (f"{args.batch}x{args.width}x{args.height}x{args.octaves}"
            f"{'u' if args.upright else 'r'}{'x' if args.extend else ''}")


def config_name(args, world) -> str:
    """BASELINE.json config this run is (configs[1..4] = #2..#5)."""
    hd = (args.width, args.height) == (1920, 1080) and args.octaves == 4 and args.upright and not args.extend
    if hd and args.batch == 1 and world == 1:
        return "config#2"
    if hd and args.batch == 256:
        return "config#4" if world == 8 else ("config#3" if world == 1 else f"config#3/#4 at {world} GPUs")
    if ((args.width, args.height) == (3840, 2160) and args.octaves == 5 and not args.upright and args.extend
            and args.batch == 64):
        return "config#5" if world == 8 else f"config#5 per-rank shard at {world} GPU(s)"
    return "custom"


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256, help="frames per GPU per step")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--octaves", type=int, default=4)
    ap.add_argument("--upright", type=int, default=1)
    ap.add_argument("--extend", type=int, default=0)
    ap.add_argument("--thresh", type=float, default=4.0)
    ap.add_argument("--max-pts", type=int, default=0,
                    help="keypoint cap per frame (default 65,536 up to 1080p, 262,144 above; SURVEY 8d)")
    ap.add_argument("--exchange", choices=("rccl", "gloo"), default="rccl",
                    help="world > 1: slab all-gather through libsurfcomm (RCCL), or host-staged over gloo "
                         "(a rehearsal that runs several ranks on one GPU)")
    ap.add_argument("--gather", choices=("full", "points"), default="full",
                    help="world > 1: all-gather SurfPoints + descriptors, or SurfPoints only "
                         "(descriptors stay on the rank that computed them)")
    ap.add_argument("--gather-at", choices=("pack", "describe"), default="pack",
                    help="N > 1: issue batch i's all-gather right after its pack, or after batch i+1's "
                         "describe starts (beside the latency-bound stage)")
    ap.add_argument("--slab-headroom", type=float, default=1.10,
                    help="fixed per-rank slab capacity = max over ranks of the warm-up slab x this")
    ap.add_argument("--no-exchange-probe", action="store_true",
                    help="N = 1: skip the 1-rank RCCL all-gather of the real slab")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="compute each batch's integral beside its own Hessian instead of beside the previous "
                         "batch's describe (surfhip_detect_batch_next)")
    ap.add_argument("--exchange-proxy", type=int, default=0, metavar="N",
                    help="N = 1 only: after the timed region, time the step again with the HBM traffic an N-rank "
                         "all-gather would put on this GPU each step ((N-1) x slab bytes copied D2D on a comm "
                         "stream beside compute), for --gather full and points (SURVEY 8e; DESIGN.md 5)")
    ap.add_argument("--cpu-frames", type=int, default=128, help="frames per CPU baseline chunk")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline wall-time budget")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-stream-peak", action="store_true", help="skip the measured HBM stream rates")
    ap.add_argument("--no-profile", action="store_true", help="no HIP events in the timed region")
    ap.add_argument("--pmc-json", default=None)
    ap.add_argument("--hessian-only", action="store_true",
                    help="time only the Hessian stage (for rocprofv3 --pmc passes)")
    ap.add_argument("--with-integral", action="store_true",
                    help="with --hessian-only: run the integral before every Hessian launch")
    args = ap.parse_args()
    if args.max_pts <= 0:
        args.max_pts = 65536 if args.width * args.height <= 1920 * 1088 else 262144
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")

    rc = spawn_ranks(args)              # before torch: the launcher never touches the GPU
    if rc is not None:
        sys.exit(rc)
    run_rank(args)


def run_rank(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # torch first: its HIP runtime is the one copy in this process
    import torch
    import torch.distributed as dist

    ndev = torch.cuda.device_count()
    if world > 1 and args.exchange == "rccl" and ndev < world:
        print(f"bench.py rank {rank}: --exchange rccl needs one GPU per rank ({world} ranks, {ndev} GPUs); "
              f"--exchange gloo rehearses several ranks on one GPU", file=sys.stderr, flush=True)
        sys.exit(2)
    # one process per GPU; with --exchange gloo several ranks may share a GPU
    gpu = local % max(1, ndev) if world > 1 else 0
    dev = torch.device("cuda", gpu)
    torch.cuda.set_device(dev)
    if world > 1:
        # control plane only (barriers, capacity agreement, id broadcast, max
        # time): gloo on host tensors; the data path is libsurfcomm's RCCL
        dist.init_process_group("gloo")
    surf = load_surf()
    surf.set_device(dev.index)

    def allreduce_max(v, dtype=torch.int64):
        t = torch.tensor([v], dtype=dtype)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return t.item()

    W, H, B = args.width, args.height, args.batch
    pitch = surf.align_up(W, 128)
    t0 = time.time()
    first, _ = surf.dist.shard_range(world * B, world, rank)   # rank r: frames [r*B, (r+1)*B)
    frames = surf.synth_frames(B, W, H, pitch, first=first)
    gen_s = time.time() - t0
    d_frames = torch.from_numpy(frames).to(dev)
    param = surf.make_param(args.octaves, args.thresh, False, 9, 2, bool(args.upright), bool(args.extend), 4)
    nf = param.nfeatures
    stream = torch.cuda.current_stream(dev)
    det = surf.Detector(param, W, H, max_batch=B, max_pts=args.max_pts, stream=stream.cuda_stream)
    d_pts = torch.empty(B * args.max_pts * 48, dtype=torch.uint8, device=dev)
    d_desc = torch.empty(B * args.max_pts * nf, dtype=torch.float32, device=dev)
    d_cnt = torch.zeros(B, dtype=torch.int32, device=dev)
    profile = not args.no_profile
    # the timed loop runs unprofiled (the detector then overlaps the integral
    # with the u8 Hessian kernels on a side stream); stage times come from a
    # separate serial pass afterwards
    det.set_profiling(False)

    def run_batch():
        if args.hessian_only:
            if args.with_integral:
                det.run_integral(d_frames.data_ptr(), B, pitch, H * pitch)
            det.run_hessian(B)
        elif args.no_pipeline:
            det.detect_batch(d_frames.data_ptr(), B, pitch, H * pitch, d_pts.data_ptr(), d_desc.data_ptr(),
                             d_cnt.data_ptr())
        else:
            # the next step's batch is the same resident frames: its integral
            # is computed beside this batch's describe (one integral per step,
            # as in the serial arrangement)
            det.detect_batch_next(d_frames.data_ptr(), B, pitch, H * pitch, d_pts.data_ptr(), d_desc.data_ptr(),
                                  d_cnt.data_ptr(), d_frames.data_ptr(), B, pitch, H * pitch)

    if args.hessian_only:
        det.run_integral(d_frames.data_ptr(), B, pitch, H * pitch)

    # multi-GPU exchange: every rank packs its compacted slab
    # straight into its own section of a gather buffer of a FIXED per-rank
    # capacity (agreed once, below) and the sections are all-gathered through
    # the C-ABI (libsurfcomm, surfhip_allgather over RCCL) on a comm stream: no
    # host synchronisation per step; gather(i) overlaps compute(i+1), two
    # buffers alternate.
    exchange = world > 1 and not args.hessian_only
    desc_ptr_for_slab = d_desc.data_ptr() if args.gather == "full" else None
    comm = comm_stream = None
    cap = 0
    gathered, ev_packed, ev_gathered = [None, None], [None, None], [None, None]
    ag_events = []                                      # (start, end) on the comm stream, timed steps
    if exchange:
        for i in range(args.warmup):                  # the detector's steady state sizes the slab
            run_batch()
        used = det.slab_bytes(B, det.batch_total(B), desc=args.gather == "full")
        cap = int(allreduce_max(used))                 # once, outside the timed region
        cap = surf.align_up(int(cap * args.slab_headroom) + 64, 256)
        for k in range(2):
            gathered[k] = torch.empty(world * cap, dtype=torch.uint8, device=dev)
            ev_packed[k] = torch.cuda.Event()
            ev_gathered[k] = torch.cuda.Event()
        comm_stream = torch.cuda.Stream(dev)
        if args.exchange == "rccl":
            uid = torch.zeros(surf.COMM_ID_BYTES, dtype=torch.uint8)
            if rank == 0:
                uid[:] = torch.frombuffer(bytearray(surf.comm_unique_id()), dtype=torch.uint8)
            dist.broadcast(uid, 0)
            with _StdoutToStderr():
                comm = surf.Comm(world, rank, bytes(uid.numpy().tobytes()))

    nstep = 0                                          # buffer i & 1 across warmup and timed steps
    timing = [False]

    # --gather-at describe: batch i's all-gather is issued after batch i+1's
    # describe-start event (surfhip_detector_set_describe_event), so its HBM
    # writes land beside the latency-bound describe rather than the next
    # batch's Hessian and NMS; the last batch's goes out after the loop,
    # inside the timed region
    ev_desc = None
    pending = [None]

    def pack(i):
        k = i & 1
        mine = gathered[k].data_ptr() + rank * cap
        if i >= 2:
            stream.wait_event(ev_gathered[k])         # gather(i-2) has read this buffer
        # pack before the next detect_batch reuses the detector's scratch and status
        det.pack_slab_cap(d_pts.data_ptr(), desc_ptr_for_slab, d_cnt.data_ptr(), B, mine, cap)
        ev_packed[k].record(stream)

    def gather(i):
        k = i & 1
        mine = gathered[k].data_ptr() + rank * cap
        comm_stream.wait_event(ev_packed[k])
        if ev_desc is not None:
            surf.stream_wait_event(comm_stream.cuda_stream, ev_desc)
        ev = None
        if timing[0]:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record(comm_stream)
        if comm is not None:
            comm.allgather(mine, cap, gathered[k].data_ptr(), comm_stream.cuda_stream)
        else:                                         # --exchange gloo: host-staged rehearsal
            with torch.cuda.stream(comm_stream):
                chunks = list(gathered[k].view(world, cap).cpu().unbind(0))
                dist.all_gather(chunks, chunks[rank].clone())
                gathered[k].copy_(torch.cat(chunks).to(dev))
        if ev is not None:
            ev[1].record(comm_stream)
            ag_events.append(ev)
        ev_gathered[k].record(comm_stream)

    if exchange and args.gather_at == "describe":
        ev_desc = surf.event_create()
        det.set_describe_event(ev_desc)

    def step():
        nonlocal nstep
        run_batch()
        if exchange:
            if ev_desc is not None:
                if pending[0] is not None:
                    gather(pending[0])                # the previous batch, beside this one's describe
                pack(nstep)
                pending[0] = nstep
            else:
                pack(nstep)
                gather(nstep)
        nstep += 1

    def flush():
        if pending[0] is not None:
            gather(pending[0])
            pending[0] = None

    for i in range(args.warmup):
        step()
    if ev_desc is not None:
        # the warm-up's last gather goes out here, outside the timed region
        # (the first timed step's describe event would otherwise order it)
        flush()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)

    timing[0] = True
    t_start = time.perf_counter()
    for i in range(args.steps):
        step()
    flush()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t_start
    timing[0] = False
    if world > 1:
        elapsed = float(allreduce_max(elapsed, torch.float64))
    # The roofline's launch time: the same pipelined steps again (after the
    # timed region, so its HIP events cannot perturb `value` -- three event
    # records per step cost a latency-bound 1-frame step ~0.1 ms), each
    # Hessian stage bracketed from its fork to the end of its last kernel on
    # either stream
    hess_instep = []
    if not args.hessian_only:
        det.time_hessian(True)
        for i in range(min(args.steps, 32)):
            run_batch()
        torch.cuda.synchronize(dev)
        hess_instep = det.hessian_times()
        det.time_hessian(False)

    # no truncation anywhere: a frame at max_pts, a candidate-capacity
    # overflow or a slab beyond the agreed capacity invalidates the run.  The
    # counts, the truncation flag and the slab flags are read from the last
    # step: every step processes the same frames and the pipeline is
    # deterministic (tests/test_gpu_parity.py), so they are the same in every
    # step (round 4 kept a running max of the counts with a torch kernel in
    # each timed step; it is not needed)
    counts = d_cnt.cpu().numpy()
    counts_max = counts
    problems = []
    if not args.hessian_only:
        if det.truncated():
            problems.append("candidate capacity overflow (surfhip_detector_status)")
        if (counts_max >= args.max_pts).any():
            problems.append(f"{int((counts_max >= args.max_pts).sum())} frames reached max_pts {args.max_pts}")
    exchanged = None
    if exchange:
        last = (nstep - 1) & 1
        g = gathered[last].cpu().numpy().reshape(world, cap)
        totals = []
        for r in range(world):
            fl = surf.slab_flags(g[r])
            if fl:
                problems.append(f"rank {r} slab flags {fl}")
                continue
            c, pts, desc = surf.parse_slab(g[r])
            want_nf = nf if args.gather == "full" else 0
            got_nf = 0 if desc is None else desc.shape[1]
            if len(c) != B or got_nf != want_nf or len(pts) != int(c.sum()):
                problems.append(f"rank {r} slab malformed")
            totals.append(int(c.sum()))
        c0, _, _ = surf.parse_slab(g[rank])
        if not np.array_equal(c0, counts):
            problems.append(f"rank {rank}: gathered counts differ from detect_batch's")
        ag_ms = [a.elapsed_time(b) for a, b in ag_events]
        ag_mean = float(np.mean(ag_ms)) if ag_ms else None
        if world > 1 and ag_mean is not None:
            ag_mean = float(allreduce_max(ag_mean, torch.float64))
        payload = int(sum(totals)) * (48 + (4 * nf if args.gather == "full" else 0))
        exchanged = {"backend": args.exchange, "mode": args.gather, "slab_cap_bytes": cap,
                     "gathered_bytes_per_step": world * cap,
                     "received_bytes_per_rank_per_step": (world - 1) * cap,
                     "payload_bytes_per_step": payload,
                     "keypoints_gathered_per_step": sum(totals),
                     "allgather_ms_per_step": None if ag_mean is None else round(ag_mean, 4),
                     "allgather_busbw_GBps": (None if not ag_mean else
                                              round((world - 1) * cap / (ag_mean * 1e-3) / 1e9, 1)),
                     "overlap": ("gather(i) on a comm stream after batch i+1's describe starts"
                                 if ev_desc is not None else "gather(i) on a comm stream beside compute(i+1)")}
    if world > 1:
        bad = allreduce_max(len(problems))
        if int(bad) and not problems:
            problems.append("another rank reported truncation")
    if problems:
        print(f"bench.py rank {rank}: INVALID RUN: " + "; ".join(problems), file=sys.stderr, flush=True)
        sys.exit(3)
    kp_per_batch = int(counts.sum())
    if world > 1:
        kt = torch.tensor([kp_per_batch], dtype=torch.int64)
        dist.all_reduce(kt)
        kp_total_batch = int(kt.item())
    else:
        kp_total_batch = kp_per_batch

    stage_acc = {}
    # per-stage times: a short serial pass with HIP events between the stages
    nprof = min(args.steps, 3)
    if profile and not args.hessian_only:
        det.set_profiling(True)
        for i in range(nprof):
            run_batch()
            for k, v in det.stage_times().items():
                stage_acc[k] = stage_acc.get(k, 0.0) + v
        det.set_profiling(False)
        torch.cuda.synchronize(dev)
    # the Hessian stage alone (events on the detector's stream; all its
    # kernels in series, nothing beside them), after one integral of the same
    # frames: the serial figure, reported next to the in-step one
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    if not args.hessian_only:
        det.run_integral(d_frames.data_ptr(), B, pitch, H * pitch)
    ev0.record(stream)
    for _ in range(args.steps):
        det.run_hessian(B)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    hess_serial_ms = ev0.elapsed_time(ev1) / args.steps
    hess_ms = float(np.mean(hess_instep)) if hess_instep else hess_serial_ms

    # N = 1: what this rank's exchange would move -- a 1-rank RCCL all-gather
    # (libsurfcomm) of the real slab, both modes, after the timed region
    probe = None
    if world == 1 and not args.hessian_only and not args.no_exchange_probe:
        with _StdoutToStderr():
            probe = exchange_probe(surf, torch, det, dev, stream, d_pts, d_desc, d_cnt, B, nf)

    proxy = None
    if world == 1 and args.exchange_proxy > 1 and not args.hessian_only:
        proxy = exchange_proxy(surf, torch, det, dev, stream, run_batch, d_pts, d_desc, d_cnt, B, args.exchange_proxy,
                               args.steps, 1e3 * elapsed / args.steps)

    peaks = None
    if rank == 0 and not args.no_stream_peak:
        peaks = stream_peaks(surf, torch, dev, stream)

    frames_total = world * B * args.steps
    value = frames_total / elapsed
    result = None
    if rank == 0:
        hb = det.hessian_bytes_per_frame() * B
        achieved = hb / (hess_ms * 1e-3) / 1e9
        traffic, traffic_tag = pmc_traffic(args)
        kern = det.hessian_kernels()
        hp = hessian_profile(args, kern)
        cfg_name = config_name(args, world)
        result = {
            "metric": METRIC if (W, H) == (1920, 1080) else f"{W}x{H} frames/sec (detect+describe)",
            "value": round(value, 2),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8/i32/f32",
            "data": f"synthetic (seeded Gaussian-blob {W}x{H} frames, resident in HBM)",
            "config": {"workload": f"{cfg_name}: batch {B} x {W}x{H} per GPU, {args.octaves} octaves, "
                                   f"{nf}-D {'upright' if args.upright else 'rotated'} descriptors, thresh {args.thresh}"
                                   + (f", RCCL all-gather of compacted SurfPoint{'+descriptor' if args.gather == 'full' else ''} slabs"
                                      if world > 1 else ""),
                       "frames_per_gpu_per_step": B, "width": W, "height": H, "octaves": args.octaves,
                       "nfeatures": nf, "upright": bool(args.upright), "parallelism": f"frames sharded x{world}"},
            "keypoints_per_s": round(kp_total_batch * args.steps / elapsed, 1),
            "keypoints_per_frame": round(kp_total_batch / (world * B), 1),
            "keypoints_per_step": kp_total_batch,
            "stage_ms_per_step_serial": {k: round(v / nprof, 4) for k, v in stage_acc.items()},
            "roofline": {"kernel": "Hessian stage, all octaves: " + kern + ", per batch",
                         # what the committed SQ / PMC counters of this config
                         # say limits the stage (tools/hessian_profile.py);
                         # `frac` is priced against the HBM peak either way,
                         # as SURVEY 8(d) defines it
                         "bound": hp["bound"] if hp else None,
                         "bound_evidence": hp.get("bound_evidence") if hp else None,
                         "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4),
                         # the in-repo stream kernels' measured rates beside
                         # the spec: `frac_measured` prices the stage against
                         # the copy rate (read + write, the stage's mix)
                         "peak_measured": peaks,
                         "frac_measured": (round(achieved / peaks["copy_GBps"], 4) if peaks else None),
                         # the stage's algorithmic reads and writes each at
                         # the measured read / write rate: the time HBM needs
                         # for this byte mix, and the stage's fraction of it
                         **mix_floor(peaks, hb, W, H, B, "writing the integral image" in kern, hess_ms),
                         # the same bytes over the sum of the stage kernels'
                         # rocprof average durations in the committed trace
                         "launch_ms_profile": round(hp["stage_ms"], 4) if hp else None,
                         "frac_profile": (round(hb / (hp["stage_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                                          if hp else None),
                         "profile": hp["tag"] if hp else None,
                         "traffic": traffic, "traffic_profile": traffic_tag,
                         # the counter bytes (what the kernels really move) over the same time
                         "frac_traffic": (None if not traffic else
                                          round(traffic / (hess_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)),
                         "algorithmic_bytes_per_launch": hb,
                         "algorithmic_bytes_def": (
                             "per frame: u8 frame read + integral image written + valid responses written "
                             "(the stage writes the integral image; before round 5 it was a separate pass beside "
                             "NMS and the definition was integral read + responses)"
                             if "writing the integral image" in kern else
                             "per frame: integral image read once + valid responses written (SURVEY 8d)"),
                         "launch_ms": round(hess_ms, 4),
                         "launch_ms_source": ("in-step: HIP events from the Hessian's fork to the end of its "
                                              "last kernel on either stream, in "
                                              f"{len(hess_instep)} pipelined steps run after the timed region, "
                                              + ("k_hess_w writing the batch's integral image, the next "
                                                 "batch's row-sum pass beside describe"
                                                 if "writing the integral image" in kern else
                                                 "the batch's own integral beside them" if args.no_pipeline else
                                                 "the next batch's integral beside the NMS stage instead")
                                              if hess_instep else "serial"),
                         "launch_ms_serial": round(hess_serial_ms, 4),
                         #  the integral the stage writes also
                         # needs k_ii_rowseg's row sums (1,296 of 1,920 columns
                         # read), which run outside the bracket beside the
                         # previous describe: their serial time, and the
                         # fraction with it added to the stage
                         **(rowseg_terms(stage_acc, nprof, hb, hess_ms)
                            if "writing the integral image" in kern else {})},
            "gen_s": round(gen_s, 2),
            "device": _device_info(surf, dev.index),
        }
        if exchanged is not None:
            result["exchange"] = exchanged
        elif probe is not None:
            result["exchange"] = probe
        if proxy is not None:
            result["exchange_proxy"] = proxy
        if world == 1 and not args.no_cpu and not args.hessian_only:
            result["cpu_baseline"] = cpu_baseline(frames, W, H, args)
        else:
            result["cpu_baseline"] = None
        print(json.dumps(result), flush=True)
    if ev_desc is not None:
        det.set_describe_event(None)
        surf.event_destroy(ev_desc)
    det.close()
    if comm is not None:
        comm.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


class _StdoutToStderr:
    """RCCL prints its version banner on fd 1 when a communicator comes up;
    the bench's stdout carries only the JSON line, so fd 1 points at fd 2
    while libsurfcomm runs."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)
        return self

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)
        return False


def mix_floor(peaks, hb, W, H, B, fused, hess_ms):
    """HBM time of the Hessian stage's algorithmic bytes at the measured
    stream rates: reads (the u8 frames when the stage writes the integral
    image, else the integral image) at the read rate, writes (responses, and
    the integral image when fused) at the write rate."""
    if not peaks:
        return {"floor_ms_measured": None, "frac_floor": None}
    rd = (W * H if fused else (W + 1) * (H + 1) * 4) * B
    wr = hb - rd
    floor = rd / (peaks["read_GBps"] * 1e6) + wr / (peaks["write_GBps"] * 1e6)
    return {"floor_bytes": {"read": rd, "write": wr}, "floor_ms_measured": round(floor, 4),
            "frac_floor": round(floor / hess_ms, 4)}


def rowseg_terms(stage_acc, nprof, hb, hess_ms):
    rs = stage_acc.get("integral")
    if not rs:
        return {"rowseg_ms_serial": None, "frac_with_rowseg": None}
    rs_ms = rs / nprof
    return {"rowseg_ms_serial": round(rs_ms, 4),
            "frac_with_rowseg": round(hb / ((hess_ms + rs_ms) * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}


def _device_info(surf, index):
    try:
        name, cus = surf.device_name(index)
        return {"name": name, "cus": cus}
    except Exception as e:                                  # informational only
        return {"error": str(e)}


def stream_peaks(surf, torch, dev, stream, nbytes=2 << 30, reps=10):
    """Measured HBM stream rates: the in-repo
    16-B-per-lane streaming kernels (surfhip_stream_run) over 2-GiB buffers
    (8x the 256-MB memory-side cache), each timed over `reps` back-to-back
    launches with HIP events on the bench stream after two warm-up launches.
    GB/s = HBM bytes the kernel moves (copy: read + write) / time."""
    src = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    dst = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    src.fill_(1)
    out = {"kernel": "surfhip_stream_run (cuda-surf_amd/csrc/surfhip_stream.hip)", "buffer_bytes": nbytes}
    for mode in ("copy", "read", "write"):
        s_ptr = src.data_ptr() if mode != "write" else None
        d_ptr = dst.data_ptr() if mode != "read" else None
        for _ in range(2):
            surf.stream_run(mode, s_ptr, d_ptr, nbytes, stream.cuda_stream)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        moved = 0
        for _ in range(reps):
            moved += surf.stream_run(mode, s_ptr, d_ptr, nbytes, stream.cuda_stream)
        e1.record(stream)
        torch.cuda.synchronize(dev)
        ms = e0.elapsed_time(e1)
        out[f"{mode}_GBps"] = round(moved / (ms * 1e-3) / 1e9, 1)
    del src, dst
    torch.cuda.empty_cache()
    return out


def exchange_proxy(surf, torch, det, dev, stream, run_batch, d_pts, d_desc, d_cnt, B, nranks, steps, base_ms):
    """Single-GPU proxy of the N-rank exchange's cost to the step: each step
    packs its slab (as the N > 1 loop does) and a comm stream then writes
    (N-1) x slab bytes into a receive buffer by a D2D copy -- the bytes an
    all-gather lands in this GPU's HBM -- beside the next batch's compute.
    Two issue points: `pack` (the copy follows the pack at once, so it runs
    beside the next batch's row sums, Hessian and NMS) and `describe` (the
    comm stream waits for the next batch's describe-start event,
    surfhip_detector_set_describe_event: the copy runs beside the
    latency-bound describe, which leaves HBM idle).  xGMI link time is not in
    it (DESIGN.md 5 models that); what it measures is the HBM and CU
    contention the received slabs cost the pipeline."""
    out = {"nranks": nranks, "base_ms_per_step": round(base_ms, 4),
           "note": "D2D copy of (N-1) x slab bytes per step on a comm stream, event-ordered after the pack "
                   "(at: pack) or after the next batch's describe start (at: describe); the xGMI transfer "
                   "itself is modelled in DESIGN.md 5"}
    total = det.batch_total(B)
    cs = torch.cuda.Stream(dev)
    ev_desc = surf.event_create()
    for mode in ("full", "points"):
        used = det.slab_bytes(B, total, desc=mode == "full")
        cap = (int(used * 1.10) + 64 + 255) // 256 * 256
        slab = [torch.empty(cap, dtype=torch.uint8, device=dev) for _ in range(2)]
        src = torch.empty((nranks - 1) * cap, dtype=torch.uint8, device=dev)
        dst = [torch.empty((nranks - 1) * cap, dtype=torch.uint8, device=dev) for _ in range(2)]
        src.fill_(1)
        res = {"slab_bytes": used, "received_bytes_per_step": (nranks - 1) * cap}
        for at in ("pack", "describe"):
            packed = [torch.cuda.Event() for _ in range(2)]
            landed = [torch.cuda.Event() for _ in range(2)]
            cev = []
            pending = [None]
            det.set_describe_event(ev_desc if at == "describe" else None)

            def copy(k, timed):
                cs.wait_event(packed[k])
                if at == "describe":
                    surf.stream_wait_event(cs.cuda_stream, ev_desc)
                with torch.cuda.stream(cs):
                    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) if timed else None
                    if ev:
                        ev[0].record(cs)
                    dst[k].copy_(src, non_blocking=True)
                    if ev:
                        ev[1].record(cs)
                        cev.append(ev)
                landed[k].record(cs)

            def one(i, timed):
                k = i & 1
                run_batch()
                if at == "describe" and pending[0] is not None:
                    copy(pending[0], timed)          # batch i-1's slab, beside batch i's describe
                if i >= 2:
                    stream.wait_event(landed[k])
                det.pack_slab_cap(d_pts.data_ptr(), d_desc.data_ptr() if mode == "full" else None,
                                  d_cnt.data_ptr(), B, slab[k].data_ptr(), cap)
                packed[k].record(stream)
                if at == "pack":
                    copy(k, timed)
                else:
                    pending[0] = k

            for i in range(3):
                one(i, False)
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for i in range(steps):
                one(3 + i, True)
            if at == "describe":                 # the last batch's slab, inside the timed region
                copy(pending[0], True)
            torch.cuda.synchronize(dev)
            ms = 1e3 * (time.perf_counter() - t0) / steps
            cms = float(np.mean([a.elapsed_time(b) for a, b in cev]))
            res[at] = {"ms_per_step": round(ms, 4), "copy_ms": round(cms, 4), "slowdown": round(ms / base_ms, 4)}
        det.set_describe_event(None)
        out[mode] = res
        del slab, src, dst
    surf.event_destroy(ev_desc)
    return out


def exchange_probe(surf, torch, det, dev, stream, d_pts, d_desc, d_cnt, B, nf, reps=5):
    """Time a 1-rank RCCL all-gather (libsurfcomm) of this batch's slab in
    both modes.  With one rank RCCL copies the section locally, so this is
    the launch + copy floor of the exchange, not an xGMI rate."""
    out = {"backend": "rccl (1 rank)", "note": "N = 1: the exchange is not in the timed step; the slab this "
           "rank would contribute, all-gathered by a 1-rank RCCL communicator after the timed region"}
    try:
        uid = surf.comm_unique_id()
        comm = surf.Comm(1, 0, uid)
    except Exception as e:            # the probe is informational; the bench line stands without it
        out["error"] = str(e)[:200]
        return out
    try:
        total = det.batch_total(B)
        cs = torch.cuda.Stream(dev)
        for mode in ("full", "points"):
            used = det.slab_bytes(B, total, desc=mode == "full")
            cap = surf.align_up(used + 64, 256)
            send = torch.empty(cap, dtype=torch.uint8, device=dev)
            recv = torch.empty(cap, dtype=torch.uint8, device=dev)
            det.pack_slab_cap(d_pts.data_ptr(), d_desc.data_ptr() if mode == "full" else None, d_cnt.data_ptr(),
                              B, send.data_ptr(), cap)
            torch.cuda.synchronize(dev)
            comm.allgather(send.data_ptr(), cap, recv.data_ptr(), cs.cuda_stream)     # warm
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(cs)
            for _ in range(reps):
                comm.allgather(send.data_ptr(), cap, recv.data_ptr(), cs.cuda_stream)
            e1.record(cs)
            torch.cuda.synchronize(dev)
            ms = e0.elapsed_time(e1) / reps
            ok = bool(torch.equal(send, recv))
            out[mode] = {"slab_bytes": used, "allgather_ms": round(ms, 4), "bytes_equal": ok}
        out["keypoints"] = total
    finally:
        comm.close()
    return out


if __name__ == "__main__":
    main()
