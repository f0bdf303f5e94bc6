#!/bin/bash
# integral band height (fill waves per round): 32 (default) vs 24 vs 16; integral parity at 24
set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
O=gpurun_out
SURFHIP_II_BAND=24 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
   -k "integral or config3_batch256_vs_oracle" > $O/e17_pytest.log 2>&1 || { tail -40 $O/e17_pytest.log; exit 1; }
tail -2 $O/e17_pytest.log
bench() {  # tag env args...
  local tag=$1 ev=$2; shift 2
  if [ "$ev" = "-" ]; then EV=(); else EV=($ev); fi
  env "${EV[@]}" timeout -k 10 120 python3 bench.py --steps 30 --warmup 3 --no-cpu "$@" > $O/x_$tag.json 2> $O/x_$tag.err || { tail -5 $O/x_$tag.err; return 1; }
  python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]);s=d['stage_ms_per_step_serial'];print(sys.argv[2], d['value'], d['ms_per_step'], 'integral', s.get('integral'), 'nms', s.get('nms'), 'desc', s.get('describe'))" $O/x_$tag.json "$tag"
}
bench b32a - || exit 1
bench b24a SURFHIP_II_BAND=24 || exit 1
bench b16a SURFHIP_II_BAND=16 || exit 1
bench b32b - || exit 1
bench b24b SURFHIP_II_BAND=24 || exit 1
bench b16b SURFHIP_II_BAND=16 || exit 1
echo EXP17_DONE
