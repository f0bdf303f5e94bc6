set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in default nowpe; do
LD=cuda-surf_amd/diag/$v; [ "$v" = default ] && LD=cuda-surf_amd
SURFHIP_LIB_DIR=$LD timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "describe or upright or golden or reference or synthetic" > gpurun_out/e20_$v.log 2>&1 || { tail -30 gpurun_out/e20_$v.log; exit 1; }
tail -1 gpurun_out/e20_$v.log
done
bash tools/diag_run.sh k_describe default nowpe prev default nowpe prev > /dev/null
for v in default nowpe prev; do echo $v; python3 tools/kstats.py gpurun_out/dg_$v/run_kernel_trace.csv k_describe; done
