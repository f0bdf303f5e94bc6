"""Experiment: N detectors on N streams, batches dealt round-robin, vs one
detector (sustained frames/s of detect+describe on resident frames)."""
import os, sys, time
import torch
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import __graft_entry__ as g
surf = g._load_pkg()
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
surf.set_device(0)
W, H, B, MP = 1920, 1080, int(os.environ.get("B", "256")), 16384
pitch = surf.align_up(W, 128)
frames = torch.from_numpy(surf.synth_frames(B, W, H, pitch, first=0)).to(dev)
param = surf.make_param(4, 4.0, False, 9, 2, True, False, 4)
for ns in (1, 2, 3):
    streams = [torch.cuda.Stream(dev) for _ in range(ns)]
    dets = [surf.Detector(param, W, H, max_batch=B, max_pts=MP, stream=s.cuda_stream) for s in streams]
    pts = [torch.empty(B * MP * 48, dtype=torch.uint8, device=dev) for _ in range(ns)]
    dsc = [torch.empty(B * MP * 64, dtype=torch.float32, device=dev) for _ in range(ns)]
    cnt = [torch.zeros(B, dtype=torch.int32, device=dev) for _ in range(ns)]
    def step(i):
        k = i % ns
        dets[k].detect_batch(frames.data_ptr(), B, pitch, H * pitch, pts[k].data_ptr(), dsc[k].data_ptr(), cnt[k].data_ptr())
    for i in range(3 * ns):
        step(i)
    torch.cuda.synchronize()
    K = 24
    t = time.perf_counter()
    for i in range(K):
        step(i)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    print(f"streams {ns}: {K * B / dt:.0f} frames/s, {dt / K * 1e3:.3f} ms per batch", flush=True)
    for d in dets:
        d.close()
    del pts, dsc, cnt
    torch.cuda.empty_cache()
