#!/bin/bash
# One rocprofv3 --pmc pass over the bench (counters given as args, one pass).
#   bash tools/pmc.sh <tag> "CNT1 CNT2 ..." [bench args...]
set -u
TAG=$1; CNTS=$2; shift 2
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --pmc $CNTS -T -f csv -d gpurun_out/pmc_$TAG -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu --no-profile "$@" > gpurun_out/pmc_$TAG.json 2> gpurun_out/pmc_$TAG.err || exit $?
python3 - "$TAG" <<'PY'
import csv, sys, collections
tag = sys.argv[1]
d = collections.defaultdict(list)
for r in csv.DictReader(open(f"gpurun_out/pmc_{tag}/run_counter_collection.csv")):
    d[(r["Kernel_Name"][:30], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(d.items()):
    print(f"{k:30s} {c:24s} {sum(v)/len(v):16.1f}")
PY
