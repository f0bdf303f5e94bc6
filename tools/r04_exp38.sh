#!/bin/bash
# k_offsets / k_scan_top: parallel 1,024-entry scans instead of one thread's loop (diag/scan) vs HEAD
set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
O=gpurun_out
SURFHIP_LIB_DIR=cuda-surf_amd/diag/scan timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/e38_pytest.log 2>&1 || { tail -40 $O/e38_pytest.log; exit 1; }
tail -2 $O/e38_pytest.log
for v in scan default; do
  if [ $v = default ]; then EV=(); else EV=(SURFHIP_LIB_DIR=cuda-surf_amd/diag/$v); fi
  env "${EV[@]}" timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -f csv -d $O/e38_$v -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu --no-profile > $O/e38_$v.json 2> $O/e38_$v.err || { tail -5 $O/e38_$v.err; exit 1; }
  python3 - $O/e38_$v/run_kernel_stats.csv $v <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if r["Name"].startswith(("k_scan", "k_offsets")):
        print(sys.argv[2], r["Name"][:30], r["Calls"], round(float(r["AverageNs"]) / 1000, 1), "us")
PY
done
b1() {  # tag env
  local tag=$1 ev=$2
  if [ "$ev" = "-" ]; then EV=(); else EV=($ev); fi
  env "${EV[@]}" timeout -k 10 120 python3 bench.py --batch 1 --steps 400 --warmup 20 --no-cpu > $O/y_$tag.json 2> $O/y_$tag.err || { tail -5 $O/y_$tag.err; return 1; }
  python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]);print(sys.argv[2], d['value'], d['ms_per_step'], d.get('stage_ms_per_step_serial'))" $O/y_$tag.json "$tag"
}
b1 q_new_a SURFHIP_LIB_DIR=cuda-surf_amd/diag/scan || exit 1
b1 q_old_a - || exit 1
b1 q_new_b SURFHIP_LIB_DIR=cuda-surf_amd/diag/scan || exit 1
b1 q_old_b - || exit 1
echo EXP38_DONE
