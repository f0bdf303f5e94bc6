#!/bin/bash
# Quick per-kernel timing of the bench workload: rocprofv3 kernel trace + stats.
#   bash tools/ktrace.sh <tag> [bench args...]
set -u
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d gpurun_out/kt_$TAG -o run -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu "$@" > gpurun_out/kt_$TAG.json 2> gpurun_out/kt_$TAG.err || exit $?
python3 - "$TAG" <<'PY'
import csv, sys
tag = sys.argv[1]
for r in csv.DictReader(open(f"gpurun_out/kt_{tag}/run_kernel_stats.csv")):
    print(f"{r['Name'][:44]:44s} calls {r['Calls']:>4s}  avg {float(r['AverageNs'])/1e3:10.1f} us  {float(r['Percentage']):6.2f} %")
PY
