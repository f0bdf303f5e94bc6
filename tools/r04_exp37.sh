#!/bin/bash
# k_sort: bitonic passes of distance <= 64 in registers (diag/sortreg) vs HEAD
set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
O=gpurun_out
SURFHIP_LIB_DIR=cuda-surf_amd/diag/sortreg timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/e37_pytest.log 2>&1 || { tail -40 $O/e37_pytest.log; exit 1; }
tail -2 $O/e37_pytest.log
for v in sortreg default; do
  if [ $v = default ]; then EV=(); else EV=(SURFHIP_LIB_DIR=cuda-surf_amd/diag/$v); fi
  env "${EV[@]}" timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -f csv -d $O/e37_$v -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu --no-profile > $O/e37_$v.json 2> $O/e37_$v.err || { tail -5 $O/e37_$v.err; exit 1; }
  python3 - $O/e37_$v/run_kernel_stats.csv $v <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if r["Name"].startswith(("k_sort",)):
        print(sys.argv[2], r["Name"][:30], r["Calls"], round(float(r["AverageNs"]) / 1000, 1), "us")
PY
done
bench() {  # tag env
  local tag=$1 ev=$2; shift 2
  if [ "$ev" = "-" ]; then EV=(); else EV=($ev); fi
  env "${EV[@]}" timeout -k 10 120 python3 bench.py --steps 30 --warmup 3 --no-cpu "$@" > $O/x_$tag.json 2> $O/x_$tag.err || { tail -5 $O/x_$tag.err; return 1; }
  python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]);s=d['stage_ms_per_step_serial'];print(sys.argv[2], d['value'], d['ms_per_step'], 'sort', s.get('sort'))" $O/x_$tag.json "$tag"
}
bench s_new_a SURFHIP_LIB_DIR=cuda-surf_amd/diag/sortreg || exit 1
bench s_old_a - || exit 1
bench s_new_b SURFHIP_LIB_DIR=cuda-surf_amd/diag/sortreg || exit 1
bench s_old_b - || exit 1
echo EXP37_DONE
