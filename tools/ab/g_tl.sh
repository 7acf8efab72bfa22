# kernel trace (timestamps) of a few mesh steps, for tools/timeline.py
set -o pipefail
export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl4 -o run -- python3 bench.py --steps 4 --warmup 2 --cpu-seconds 0 --no-h2d > gpurun_out/tl4.log 2>&1 || exit 1
F=$(find gpurun_out/tl4 -name "*kernel_trace.csv" | head -1)
python3 tools/timeline.py $F > gpurun_out/tl4_step.txt && head -60 gpurun_out/tl4_step.txt
