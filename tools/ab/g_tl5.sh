# kernel trace (timestamps) of config-5 steps, for tools/timeline.py
set -o pipefail
export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl6 -o run -- python3 bench.py --config power --steps 4 --warmup 2 --cpu-seconds 0 --no-h2d > gpurun_out/tl6.log 2>&1 || exit 1
F=$(find gpurun_out/tl6 -name "*kernel_trace.csv" | head -1)
python3 tools/timeline.py $F k_join_window 300 > gpurun_out/tl6_step.txt && cat gpurun_out/tl6_step.txt
