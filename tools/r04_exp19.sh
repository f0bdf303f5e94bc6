#!/bin/bash
# chunked Hessian + NMS scan (SURFHIP_HN_CHUNK): parity at 64, step A/B at 0 / 128 / 64 / 32
set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
O=gpurun_out
SURFHIP_HN_CHUNK=64 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
   -k "config3 or detect_batch_next or batch_equals" > $O/e19_pytest.log 2>&1 || { tail -40 $O/e19_pytest.log; exit 1; }
tail -2 $O/e19_pytest.log
bench() {  # tag env args...
  local tag=$1 ev=$2; shift 2
  if [ "$ev" = "-" ]; then EV=(); else EV=($ev); fi
  env "${EV[@]}" timeout -k 10 120 python3 bench.py --steps 30 --warmup 3 --no-cpu "$@" > $O/x_$tag.json 2> $O/x_$tag.err || { tail -5 $O/x_$tag.err; return 1; }
  python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]);r=d['roofline'];print(sys.argv[2], d['value'], d['ms_per_step'], 'hess_in', r['launch_ms'])" $O/x_$tag.json "$tag"
}
bench c0a - || exit 1
bench c128 SURFHIP_HN_CHUNK=128 || exit 1
bench c64 SURFHIP_HN_CHUNK=64 || exit 1
bench c32 SURFHIP_HN_CHUNK=32 || exit 1
bench c0b - || exit 1
bench c64b SURFHIP_HN_CHUNK=64 || exit 1
echo EXP19_DONE
