#!/usr/bin/env python3
"""Per-kernel min / median / mean (us) from a rocprofv3 kernel-trace CSV.
    python tools/kstats.py gpurun_out/<dir>/run_kernel_trace.csv [substr ...]"""
import csv
import statistics
import sys
from collections import defaultdict

d = defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    if len(sys.argv) > 2 and not any(k in n for k in sys.argv[2:]):
        continue
    d[n[:48]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for n, v in sorted(d.items(), key=lambda x: -sum(x[1])):
    print(f"{n:48s} n {len(v):3d} min {min(v):9.1f} med {statistics.median(v):9.1f} mean {statistics.mean(v):9.1f} us")
