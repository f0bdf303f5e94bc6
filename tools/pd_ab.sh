# time the Hessian stage of diag builds under each SURFHIP_P0 value
#   bash tools/pd_ab.sh "variants" "P0 values"
set -u
for v in $1; do
  LD=cuda-surf_amd/diag/$v; [ "$v" = default ] && LD=cuda-surf_amd
  for e in $2; do
    env SURFHIP_LIB_DIR=$LD SURFHIP_P0=$e timeout -k 10 120 python3 bench.py --hessian-only --steps 20 --no-cpu > gpurun_out/pd_ab.json 2> gpurun_out/pd_ab.err || { tail -5 gpurun_out/pd_ab.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/pd_ab.json').read().strip().splitlines()[-1]); print('$v P0=$e', d['roofline']['launch_ms'])"
  done
done
