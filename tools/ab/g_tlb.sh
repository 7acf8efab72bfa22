# kernel trace of Bookinfo steps (10^6 spans) for tools/timeline.py
set -o pipefail
export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tlb -o run -- python3 bench.py --config bookinfo --steps 30 --warmup 10 --cpu-seconds 0 --no-h2d > gpurun_out/tlb.log 2>&1 || exit 1
F=$(find gpurun_out/tlb -name "*kernel_trace.csv" | head -1)
python3 tools/timeline.py $F k_join_chain 40 > gpurun_out/tlb_step.txt && cat gpurun_out/tlb_step.txt
