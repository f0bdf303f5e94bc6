#!/bin/bash
# k_hess_v0 experiment variants (SURFHIP_V0_SPLIT), kernel trace of the Hessian stage each
set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in "$@"; do
  SURFHIP_V0_SPLIT=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats -T -f csv -d gpurun_out/kt_exp$v -o run -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu --hessian-only > gpurun_out/kt_exp$v.json 2> gpurun_out/kt_exp$v.err || { tail -5 gpurun_out/kt_exp$v.err; exit 1; }
  python3 - "$v" <<'PY'
import csv, sys
v = sys.argv[1]
for r in csv.DictReader(open(f"gpurun_out/kt_exp{v}/run_kernel_stats.csv")):
    if r['Name'].startswith('void surfhip::k_hess') or 'k_hess' in r['Name']:
        print(f"exp{v} {r['Name'][:60]:60s} calls {r['Calls']:>4s} avg {float(r['AverageNs'])/1e3:9.1f} us min {float(r['MinNs'])/1e3:9.1f}")
PY
done
echo EXP_DONE
