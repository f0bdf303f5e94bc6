#!/bin/bash
# SQ counter passes (one rocprofv3 run each) over a short full-pipeline bench,
# averaged per kernel whose name contains <kernel-substr>.
#   bash tools/pmc_kern.sh <tag> <kernel-substr> "<counters pass 1>" ["<pass 2>" ...] [-- bench args]
set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=$1; K=$2; shift 2
PASSES=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do PASSES+=("$1"); shift; done
[ $# -gt 0 ] && shift
i=0
for C in "${PASSES[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C -T -f csv -d gpurun_out/pmc_${TAG}_$i -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu --no-profile "$@" > gpurun_out/pmc_${TAG}_$i.json 2> gpurun_out/pmc_${TAG}_$i.err || { tail -5 gpurun_out/pmc_${TAG}_$i.err; exit 1; }
  python3 - "gpurun_out/pmc_${TAG}_$i/run_counter_collection.csv" "$K" <<'PY'
import csv, sys, collections
d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if sys.argv[2] in r["Kernel_Name"]:
        d[(r["Kernel_Name"][:40], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(d.items()):
    print(f"{k:40s} {c:28s} {sum(v)/len(v):16.1f}")
PY
done
echo PMC_DONE
