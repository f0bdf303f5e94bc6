#!/bin/bash
# Whole-step A/B of environment settings (no profiler): bench.py's value per setting.
#   bash tools/env_ab.sh "VAR=a" "VAR=b" ...   ("-" = no extra variable)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
i=0
for e in "$@"; do
  i=$((i + 1))
  if [ "$e" = "-" ]; then EV=(); else EV=("$e"); fi
  env "${EV[@]}" timeout -k 10 120 python3 bench.py --steps 30 --warmup 3 --no-cpu --no-profile \
    > gpurun_out/envab_$i.json 2> gpurun_out/envab_$i.err || { tail -5 gpurun_out/envab_$i.err; exit 1; }
  python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]);print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/envab_$i.json "$e"
done
