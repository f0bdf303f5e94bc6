# rotated-descriptor parity + config #5 timing
set -u
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "rot or config or window or doubled or gather_plan or golden or detect_describe" > gpurun_out/rot_pytest.log 2>&1; tail -3 gpurun_out/rot_pytest.log
bash tools/diag_run.sh k_describe default -- --width 3840 --height 2160 --octaves 5 --upright 0 --extend 1 --batch 64 --max-pts 262144
