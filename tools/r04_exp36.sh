#!/bin/bash
# k_sort: how much of it is the bitonic network (diag/nosort: network skipped, wrong order)
set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
O=gpurun_out
for v in nosort default; do
  if [ $v = default ]; then EV=(); else EV=(SURFHIP_LIB_DIR=cuda-surf_amd/diag/$v); fi
  env "${EV[@]}" timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -f csv -d $O/e36_$v -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu --no-profile > $O/e36_$v.json 2> $O/e36_$v.err || { tail -5 $O/e36_$v.err; exit 1; }
  python3 - $O/e36_$v/run_kernel_stats.csv $v <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if r["Name"].startswith(("k_sort", "k_offsets", "k_worklist")):
        print(sys.argv[2], r["Name"][:30], r["Calls"], round(float(r["AverageNs"]) / 1000, 1), "us")
PY
done
echo EXP36_DONE
