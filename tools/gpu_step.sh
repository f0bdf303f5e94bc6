set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
bash tools/profile_round.sh r01b > gpurun_out/prof_r01b.log 2>&1 || { tail -20 gpurun_out/prof_r01b.log; exit 1; }
tail -2 gpurun_out/prof_r01b.log
timeout -k 10 300 python3 bench.py > gpurun_out/r01b_bench.json 2> gpurun_out/r01b_bench.err || { tail gpurun_out/r01b_bench.err; exit 1; }
cat gpurun_out/r01b_bench.json
