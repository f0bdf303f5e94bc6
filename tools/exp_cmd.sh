set -u
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "hessian" > gpurun_out/p0n_pytest.log 2>&1; tail -2 gpurun_out/p0n_pytest.log
bash tools/hess_ab.sh p0n "SURFHIP_P0=93;SURFHIP_P0=94;SURFHIP_P0=95;SURFHIP_P0=0;SURFHIP_P0=93;SURFHIP_P0=94"
