#!/bin/bash
# Kernel-trace each diagnostic build (tools/diag_build.sh) over a short bench
# and print the average duration of kernels matching <pattern>.
#   bash tools/diag_run.sh <pattern> <variant>... [-- bench args]
set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
PAT=$1; shift
VS=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do VS+=("$1"); shift; done
[ $# -gt 0 ] && shift
for v in "${VS[@]}"; do
  LD=cuda-surf_amd/diag/$v; [ "$v" = default ] && LD=cuda-surf_amd
  SURFHIP_LIB_DIR=$LD timeout -k 10 120 rocprofv3 --kernel-trace --stats -T -f csv -d gpurun_out/dg_$v -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu --no-profile "$@" > gpurun_out/dg_$v.json 2> gpurun_out/dg_$v.err || { tail -5 gpurun_out/dg_$v.err; exit 1; }
  python3 - "gpurun_out/dg_$v/run_kernel_stats.csv" "$PAT" "$v" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if sys.argv[2] in r["Name"]:
        print(f"{sys.argv[3]:10s} {r['Name'][:60]:60s} calls {int(r['Calls']):4d} avg {float(r['AverageNs'])/1e3:9.1f} us")
PY
done
echo DIAG_DONE
