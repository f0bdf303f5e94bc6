#!/usr/bin/env python3
"""Per-config summary of the Hessian stage from one profile_round.sh run,
merged into profiles/hessian_profile.json (read by bench.py's roofline):

  kernels_avg_ns   rocprofv3 --kernel-trace --stats AVERAGE duration of each of
                   the stage's kernels (the names bench.py's line gives in
                   roofline.kernel), from gpurun_out/prof_<tag>_kt
  stage_ms         their sum: the stage's time by the rocprof-average rule
  counters         per-launch means of the SQ pass (prof_<tag>_sq) and the
                   FETCH_SIZE / WRITE_SIZE passes (prof_<tag>_fetch / _write),
                   summed over the stage's kernels
  bound            what the counters say limits the stage, and the evidence:
                     hbm_util   (2 x FETCH_SIZE + WRITE_SIZE) KiB / stage_ms / 8 TB/s
                                (the gfx950 FETCH correction, MI355X_MICROARCH.md HBM)
                     valu_util  SQ_INSTS_VALU x 3 cycles / (1,024 SIMDs x 2.4 GHz x
                                stage_ms): a wave64 VALU instruction costs 2-2.7
                                cycles plain, 4.3 packed (measured),
                                the Hessian's mix is about half each
                     lds_util   SQ_INSTS_LDS x 2 cycles / (256 CUs x 2.4 GHz x stage_ms)
                     wait_frac  SQ_WAIT_ANY / SQ_WAVE_CYCLES
                   bound = "hbm" / "valu-issue" / "lds" when that utilisation
                   is >= 0.6, else "latency" (waves waiting, no unit busy)

    python tools/hessian_profile.py <tag> [bench args: --batch B --width W ...]
"""
from __future__ import annotations

import argparse
import collections
import csv
import json
import os
import re

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PEAK = 8000e9
SIMDS, CUS, CLK = 1024, 256, 2.4e9


def kernel_avgs(path):
    out = {}
    for r in csv.DictReader(open(path)):
        out[r["Name"]] = float(r["AverageNs"])
    return out


def counter_means(path):
    d = collections.defaultdict(list)
    if not os.path.exists(path):
        return {}
    for r in csv.DictReader(open(path)):
        d[(r["Kernel_Name"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in d.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--src", default=os.path.join(REPO, "gpurun_out"))
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--octaves", type=int, default=4)
    ap.add_argument("--upright", type=int, default=1)
    ap.add_argument("--extend", type=int, default=0)
    args = ap.parse_args()
    t = args.tag
    key = (f"{args.batch}x{args.width}x{args.height}x{args.octaves}"
           f"{'u' if args.upright else 'r'}{'x' if args.extend else ''}")
    line = None
    with open(os.path.join(args.src, f"prof_{t}_kt.json")) as fh:
        for ln in fh:
            if ln.startswith("{"):
                line = json.loads(ln)
    names = sorted(set(re.findall(r"k_\w+", line["roofline"]["kernel"])))
    avgs = kernel_avgs(os.path.join(args.src, f"prof_{t}_kt", "run_kernel_stats.csv"))
    kav = {k: avgs[k] for k in names}
    stage_ns = sum(kav.values())
    cnt = {}
    for which in ("sq", "fetch", "write"):
        cnt.update(counter_means(os.path.join(args.src, f"prof_{t}_{which}", "run_counter_collection.csv")))
    tot = collections.defaultdict(float)
    for (k, c), v in cnt.items():
        if k in names:
            tot[c] += v
    sec = stage_ns * 1e-9
    ev = {}
    if "FETCH_SIZE" in tot and "WRITE_SIZE" in tot:
        ev["hbm_util"] = round((2 * tot["FETCH_SIZE"] + tot["WRITE_SIZE"]) * 1024 / sec / PEAK, 3)
        ev["hbm_bytes_per_launch"] = int((2 * tot["FETCH_SIZE"] + tot["WRITE_SIZE"]) * 1024)
    if "SQ_INSTS_VALU" in tot:
        ev["valu_util"] = round(tot["SQ_INSTS_VALU"] * 3 / (SIMDS * CLK * sec), 3)
        ev["valu_insts_per_launch"] = int(tot["SQ_INSTS_VALU"])
    if "SQ_INSTS_LDS" in tot:
        ev["lds_util"] = round(tot["SQ_INSTS_LDS"] * 2 / (CUS * CLK * sec), 3)
    if tot.get("SQ_WAVE_CYCLES"):
        ev["wait_frac"] = round(tot["SQ_WAIT_ANY"] / tot["SQ_WAVE_CYCLES"], 3)
    units = {"hbm": ev.get("hbm_util", 0), "valu-issue": ev.get("valu_util", 0), "lds": ev.get("lds_util", 0)}
    top = max(units, key=units.get)
    bound = top if units[top] >= 0.6 else "latency"
    entry = {"tag": t, "kernels_avg_ns": kav, "stage_ms": stage_ns * 1e-6, "bound": bound,
             "bound_evidence": ev,
             "counters_per_launch": {c: v for c, v in sorted(tot.items())},
             "source": f"rocprofv3 --kernel-trace --stats (averages) + --pmc SQ / FETCH_SIZE / WRITE_SIZE "
                       f"passes, tools/profile_round.sh {t}"}
    path = os.path.join(REPO, "profiles", "hessian_profile.json")
    d = {}
    if os.path.exists(path):
        d = json.load(open(path))
    d[key] = entry
    with open(path, "w") as fh:
        json.dump(d, fh, indent=1, sort_keys=True)
    print(key, json.dumps(entry, indent=1))


if __name__ == "__main__":
    main()
