#!/bin/bash
# Whole-step A/B of library builds (no profiler): bench.py's value per build.
#   bash tools/lib_ab.sh <variant>...   (default = cuda-surf_amd, else cuda-surf_amd/diag/<variant>)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in "$@"; do
  LD=cuda-surf_amd/diag/$v; [ "$v" = default ] && LD=cuda-surf_amd
  SURFHIP_LIB_DIR=$LD timeout -k 10 120 python3 bench.py --steps 30 --warmup 3 --no-cpu --no-profile \
    > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { tail -5 gpurun_out/ab_$v.err; exit 1; }
  python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]);print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/ab_$v.json $v
done
