#!/bin/bash
# Interleaved A/B of libsurfhip builds on the GPU box (no profiler): bench.py
# per variant, PAIRS rounds of A B [C ...], one JSON line each into
# gpurun_out/ab_<tag>_<variant>_<round>.json and a summary line per run:
# value, ms/step, the Hessian stage (in-step events and serial), describe.
#   bash tools/ab.sh <tag> "<variant> <variant> ..." [pairs] [bench args...]
# variant: "default" (cuda-surf_amd/) or a diag build name (cuda-surf_amd/diag/<name>,
# tools/diag_build.sh); an "env:NAME=VAL[,NAME=VAL]" variant runs the default build with that env.
set -u
TAG=$1; VARS=$2; PAIRS=${3:-2}; shift 3 2>/dev/null || shift $#
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
O=gpurun_out
for r in $(seq 1 $PAIRS); do
  for v in $VARS; do
    EV=(); LD=cuda-surf_amd
    case $v in
      default) ;;
      env:*) IFS=, read -ra EV <<< "${v#env:}" ;;
      *) LD=cuda-surf_amd/diag/$v ;;
    esac
    n=$(echo "$v" | tr -c 'A-Za-z0-9_\n' '_')
    env SURFHIP_LIB_DIR=$LD "${EV[@]}" timeout -k 10 180 python3 bench.py --steps 30 --warmup 3 --no-cpu \
        --no-exchange-probe --no-stream-peak "$@" > $O/ab_${TAG}_${n}_$r.json 2> $O/ab_${TAG}_${n}_$r.err \
        || { tail -5 $O/ab_${TAG}_${n}_$r.err; exit 1; }
    python3 - $O/ab_${TAG}_${n}_$r.json "$v" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][0])
s, rf = d["stage_ms_per_step_serial"], d["roofline"]
print(f"{sys.argv[2]:28s} {d['value']:10.1f} fr/s {d['ms_per_step']:7.4f} ms  hess {rf['launch_ms']:.4f} "
      f"(serial {rf['launch_ms_serial']:.4f})  desc {s.get('describe', 0):.4f}  nms {s.get('nms', 0):.4f}")
PY
  done
done
echo AB_DONE
