#!/bin/bash
# SQ counter passes over the Hessian stage for one SURFHIP_V0_SPLIT value
#   bash tools/exp_pmc.sh <split> "<counters pass 1>" ["<counters pass 2>" ...]
set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
v=$1; shift
i=0
for C in "$@"; do
  i=$((i+1))
  SURFHIP_V0_SPLIT=$v timeout -s KILL 120 rocprofv3 --pmc $C -T -f csv -d gpurun_out/pmc_exp${v}_$i -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu --no-profile --hessian-only > gpurun_out/pmc_exp${v}_$i.json 2> gpurun_out/pmc_exp${v}_$i.err || { tail -5 gpurun_out/pmc_exp${v}_$i.err; exit 1; }
  python3 - "gpurun_out/pmc_exp${v}_$i/run_counter_collection.csv" <<'PY'
import csv, sys, collections
d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if 'k_hess' in r["Kernel_Name"]:
        d[(r["Kernel_Name"][:24], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(d.items()):
    print(f"{k:24s} {c:28s} {sum(v)/len(v):16.1f}")
PY
done
echo PMC_DONE
