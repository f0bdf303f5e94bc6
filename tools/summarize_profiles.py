#!/usr/bin/env python3
"""Turn the rocprofv3 outputs of tools/profile_round.sh (gpurun_out/prof_<tag>_*)
into the committed summaries under profiles/:

  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary
  profiles/<tag>_pmc.csv            per-kernel mean FETCH_SIZE / WRITE_SIZE (KB)
  profiles/<tag>_bench.json         the bench line of the profiled run
  profiles/hessian_pmc.json         Hessian per-launch HBM bytes read by bench.py
  profiles/<tag>_stage_bytes.csv    every kernel of the full pipeline: HBM bytes
                                    per launch (FETCH x 2, WRITE) and its trace
                                    time (when the fetchall/writeall passes ran)

HBM bytes follow MI355X_MICROARCH.md "HBM": FETCH_SIZE and WRITE_SIZE are in
KiB; on gfx950 FETCH_SIZE reads 1/2 of the bytes of a wide coalesced
stream, so traffic = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.  (The Hessian's
reads are dword gathers, an uncalibrated width: the raw counters are kept.)

    python tools/summarize_profiles.py r01 [--batch 256 --width 1920 --height 1080 --octaves 4]
"""
from __future__ import annotations

import argparse
import collections
import csv
import json
import os
import shutil

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--src", default=os.path.join(REPO, "gpurun_out"))
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--octaves", type=int, default=4)
    args = ap.parse_args()
    t = args.tag
    prof = os.path.join(REPO, "profiles")
    os.makedirs(prof, exist_ok=True)
    kt = os.path.join(args.src, f"prof_{t}_kt", "run_kernel_stats.csv")
    shutil.copy(kt, os.path.join(prof, f"{t}_kernel_stats.csv"))
    bench = os.path.join(args.src, f"prof_{t}_kt.json")
    if os.path.exists(bench):
        shutil.copy(bench, os.path.join(prof, f"{t}_bench_profiled.json"))
    rows = collections.defaultdict(list)
    for which in ("fetch", "write"):
        path = os.path.join(args.src, f"prof_{t}_{which}", "run_counter_collection.csv")
        for r in csv.DictReader(open(path)):
            rows[(r["Kernel_Name"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    kernels = sorted({k for k, _ in rows})
    sq_path = os.path.join(args.src, f"prof_{t}_sq", "run_counter_collection.csv")
    if os.path.exists(sq_path):
        sq = collections.defaultdict(list)
        for r in csv.DictReader(open(sq_path)):
            sq[(r["Kernel_Name"], r["Counter_Name"])].append(float(r["Counter_Value"]))
        with open(os.path.join(prof, f"{t}_sq.txt"), "w") as fh:
            fh.write(f"# rocprofv3 --pmc SQ counters (one pass), tools/profile_round.sh {t}; "
                     "mean per launch\n")
            for (k, c) in sorted(x for x in sq if not x[0].startswith("__amd_rocclr")):
                v = sq[(k, c)]
                fh.write(f"{k:28s} {c:24s} {sum(v) / len(v):18.1f}\n")
    with open(os.path.join(prof, f"{t}_pmc.csv"), "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["kernel", "launches", "FETCH_SIZE_KiB_mean", "WRITE_SIZE_KiB_mean",
                    "hbm_bytes_mean (2*FETCH+WRITE)*1024"])
        for k in kernels:
            f = rows.get((k, "FETCH_SIZE"), [0.0])
            wr = rows.get((k, "WRITE_SIZE"), [0.0])
            fm, wm = sum(f) / len(f), sum(wr) / len(wr)
            w.writerow([k, len(f), round(fm, 2), round(wm, 2), int((2 * fm + wm) * 1024)])
    # the Hessian stage = every launch whose name starts with k_hess (octave 0
    # ring, octave 1 ring, gather kernel for octaves >= 2): per-batch sums
    hk = [k for k in kernels if k.startswith("k_hess")]
    fm = sum(sum(rows[(k, "FETCH_SIZE")]) / len(rows[(k, "FETCH_SIZE")]) for k in hk)
    wm = sum(sum(rows[(k, "WRITE_SIZE")]) / len(rows[(k, "WRITE_SIZE")]) for k in hk)
    out = {"config": f"{args.batch}x{args.width}x{args.height}x{args.octaves}", "tag": t,
           "kernel": "+".join(hk), "fetch_kib": fm, "write_kib": wm,
           "bytes_per_launch": (2 * fm + wm) * 1024,
           "note": "rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE in separate passes over "
                   "`bench.py --hessian-only`; traffic = (2*FETCH_SIZE + WRITE_SIZE) KiB (gfx950 "
                   "correction), summed over the Hessian stage's kernels per batch"}
    with open(os.path.join(prof, "hessian_pmc.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))
    stage_bytes(args, prof, kt)


def stage_bytes(args, prof, kt):
    t = args.tag
    fa = os.path.join(args.src, f"prof_{t}_fetchall", "run_counter_collection.csv")
    wa = os.path.join(args.src, f"prof_{t}_writeall", "run_counter_collection.csv")
    if not (os.path.exists(fa) and os.path.exists(wa)):
        return
    rows = collections.defaultdict(list)
    for path in (fa, wa):
        for r in csv.DictReader(open(path)):
            if r["Kernel_Name"].startswith("__amd_rocclr"):
                continue
            rows[(r["Kernel_Name"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    avg_ms = {}
    for r in csv.DictReader(open(kt)):
        avg_ms[r["Name"]] = float(r["AverageNs"]) / 1e6
    kernels = sorted({k for k, _ in rows}, key=lambda k: -avg_ms.get(k, 0.0))
    with open(os.path.join(prof, f"{t}_stage_bytes.csv"), "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["kernel", "trace_avg_ms", "fetch_bytes (2*FETCH_SIZE)", "write_bytes (WRITE_SIZE)",
                    "hbm_bytes", "GBps_at_trace_avg"])
        for k in kernels:
            f = rows.get((k, "FETCH_SIZE"), [0.0])
            wr = rows.get((k, "WRITE_SIZE"), [0.0])
            fb = 2 * 1024 * sum(f) / len(f)
            wb = 1024 * sum(wr) / len(wr)
            ms = avg_ms.get(k)
            w.writerow([k[:90], None if ms is None else round(ms, 4), int(fb), int(wb), int(fb + wb),
                        None if not ms else round((fb + wb) / (ms * 1e-3) / 1e9, 1)])
    print(f"wrote profiles/{t}_stage_bytes.csv")


if __name__ == "__main__":
    main()
