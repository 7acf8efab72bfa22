# kernel trace of config 5 steps for tools/timeline.py (K3 beside the settle)
set -o pipefail
export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tlp -o run -- python3 bench.py --config power --steps 6 --warmup 2 --cpu-seconds 0 --no-h2d > gpurun_out/tlp.log 2>&1 || exit 1
F=$(find gpurun_out/tlp -name "*kernel_trace.csv" | head -1)
python3 tools/timeline.py $F k_join_window 60 > gpurun_out/tlp_step.txt && cat gpurun_out/tlp_step.txt
