#!/bin/bash
# config #2 latency: u2 vs ur describe, standalone
set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
O=gpurun_out
for t in u2a ura u2b urb; do
  case $t in ur*) E="SURFHIP_DESC_UR=1";; *) E="SURFHIP_X=1";; esac
  env $E timeout -k 10 120 python3 bench.py --batch 1 --steps 200 --warmup 20 --no-cpu > $O/c2_$t.json 2> $O/c2_$t.err || { tail -5 $O/c2_$t.err; exit 1; }
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[0]);print(sys.argv[2],d['ms_per_step'],d['stage_ms_per_step_serial'])" $O/c2_$t.json $t
done
echo EXP13_DONE
