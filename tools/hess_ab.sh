#!/bin/bash
# Hessian-stage A/B on the GPU box: bench --hessian-only under each given
# environment setting (one JSON line each), then one SQ counter pass.
#   bash tools/hess_ab.sh <tag> "ENV1=..;ENV2=.." "counter list" [env for the pmc pass]
set -u
TAG=$1; ENVS=$2; CNTS=${3:-}; PENV=${4:-}
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
O=gpurun_out
IFS=';' read -ra ES <<< "$ENVS"
for e in "${ES[@]}"; do
    env $e timeout -k 10 120 python3 bench.py --hessian-only --steps 20 --no-cpu > $O/${TAG}_ab.json 2> $O/${TAG}_ab.err || { tail -5 $O/${TAG}_ab.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$O/${TAG}_ab.json').read().strip().splitlines()[-1]); print('$e', d['roofline']['launch_ms'], d['roofline']['kernel'])"
done
if [ -n "$CNTS" ]; then
    export $PENV
    bash tools/pmc.sh ${TAG}_pmc "$CNTS" --hessian-only | grep -E "k_hess" || exit 1
fi
echo AB_DONE
