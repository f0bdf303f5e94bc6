#!/usr/bin/env python3
"""Time surfhip_match (Surfor::match) on one GPU: n x n points, nf-D
descriptors, caller-provided scratch, HIP events via torch on the null
stream.  Prints one JSON line per case.

    python tools/match_bench.py [--n 3000] [--iters 50]
"""
from __future__ import annotations

import argparse
import importlib.util
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load_surf():
    pkg = os.path.join(REPO, "cuda-surf_amd")
    spec = importlib.util.spec_from_file_location("surf_amd", os.path.join(pkg, "__init__.py"),
                                                  submodule_search_locations=[pkg])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["surf_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=3000)
    ap.add_argument("--iters", type=int, default=50)
    args = ap.parse_args()
    import torch
    surf = load_surf()
    for nf in (64, 128):
        for flags in (0, 1):
            n = args.n
            rng = np.random.default_rng(nf)
            f = rng.standard_normal((2, n, nf)).astype(np.float32)
            f /= np.linalg.norm(f, axis=2, keepdims=True)
            ft = torch.from_numpy(f).cuda()
            pts = torch.zeros((2, n, 48), dtype=torch.uint8, device="cuda")
            scratch = torch.empty(max(surf.match_scratch_bytes(n, n, flags), 4), dtype=torch.uint8, device="cuda")
            args_ = (pts[0].data_ptr(), pts[1].data_ptr(), ft[0].data_ptr(), ft[1].data_ptr(), n, n, nf, flags,
                     scratch.data_ptr())
            for _ in range(3):
                surf.match_points(*args_)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                surf.match_points(*args_)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / args.iters
            fma = n * (n if flags else 32 * (n // 32)) * nf
            print(json.dumps({"case": f"match {n}x{n} nf={nf} full_tail={flags}", "ms": round(ms, 4),
                              "pairs_per_s": round(n * n / ms * 1e3, 1),
                              "fp32_tflops": round(2 * fma / ms / 1e9, 2)}), flush=True)


if __name__ == "__main__":
    main()
