#!/bin/bash
# Round-2 first GPU pass: GPU parity suite, default bench line, counter list,
# one SQ pass over the Hessian stage.  Each GPU step has its own limit.
set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > $O/r02a_pytest.log 2>&1 || { tail -30 $O/r02a_pytest.log; exit 1; }
tail -2 $O/r02a_pytest.log
timeout -k 10 300 python3 bench.py --no-cpu > $O/r02a_bench.json 2> $O/r02a_bench.err || { tail -20 $O/r02a_bench.err; exit 1; }
cat $O/r02a_bench.json
timeout -s KILL 60 rocprofv3 -L > $O/r02a_counters.txt 2>&1 || echo "counter list failed"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU \
    -T -f csv -d $O/pmc_r02a_sq1 -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-profile --hessian-only \
    > $O/pmc_r02a_sq1.json 2> $O/pmc_r02a_sq1.err || { tail -5 $O/pmc_r02a_sq1.err; exit 1; }
echo DIAG_DONE
