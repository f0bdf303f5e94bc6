# config #2 and #5 bench lines of this build
set -u
timeout -k 10 300 python3 bench.py --batch 1 --steps 200 --warmup 20 --no-cpu > gpurun_out/c2_bench.json 2> gpurun_out/c2_bench.err || { tail -5 gpurun_out/c2_bench.err; exit 1; }
tail -1 gpurun_out/c2_bench.json
timeout -k 10 300 python3 bench.py --width 3840 --height 2160 --octaves 5 --upright 0 --extend 1 --batch 64 --max-pts 262144 --steps 10 --warmup 2 --no-cpu > gpurun_out/c5_bench.json 2> gpurun_out/c5_bench.err || { tail -5 gpurun_out/c5_bench.err; exit 1; }
tail -1 gpurun_out/c5_bench.json
