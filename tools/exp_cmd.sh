timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "window_sizes or match_random or golden or surfor" > gpurun_out/wsz_pytest.log 2>&1; tail -3 gpurun_out/wsz_pytest.log
bash tools/pd_ab.sh "default prio1 prio2 prio0" "93"
