# A/B of two library builds: describe tests on the new one, then k_describe timing
set -u
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "describe or golden or batch or config or surfor" > gpurun_out/ab_pytest.log 2>&1; tail -2 gpurun_out/ab_pytest.log
bash tools/diag_run.sh k_describe base default base default
