#!/bin/bash
# One GPU measurement cycle (run on the box via gpurun): parity tests, a
# rocprofv3 kernel trace of the mesh bench, then plain benches.  Every GPU
# step has its own time limit and the script stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-x}
timeout -k 10 500 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 > gpurun_out/t_$TAG.log 2>&1
echo "tests exit $?" >> gpurun_out/t_$TAG.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o mesh -- python3 bench.py --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/prof_$TAG.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 > gpurun_out/bench_mesh_$TAG.json 2>gpurun_out/bench_mesh_$TAG.err || exit 1
timeout -k 10 200 python bench.py --config bookinfo --steps 20 --warmup 5 --cpu-seconds 0 > gpurun_out/bench_book_$TAG.json 2>gpurun_out/bench_book_$TAG.err || exit 1
echo DONE
