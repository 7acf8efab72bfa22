#!/bin/bash
# One GPU measurement cycle (run on the box via gpurun): parity tests, a
# rocprofv3 kernel trace of the mesh bench, two PMC passes (FETCH_SIZE,
# WRITE_SIZE: one pass each) for HBM traffic, then plain benches.  Every GPU
# step has its own time limit and the script stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-x}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1
rc=$?
echo "tests exit $rc" >> gpurun_out/t_$TAG.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o mesh -- python3 bench.py --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/prof_$TAG.log 2>&1 || exit 1
KR="k4_chain|k_join_window|k3_produce|k3_reduce|k_cert_split|k_cert_check"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KR" -d gpurun_out/pmcf_$TAG -o pmc -- python3 bench.py --steps 2 --warmup 1 --cpu-seconds 0 > gpurun_out/pmcf_$TAG.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KR" -d gpurun_out/pmcw_$TAG -o pmc -- python3 bench.py --steps 2 --warmup 1 --cpu-seconds 0 > gpurun_out/pmcw_$TAG.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds ${CPU_SECONDS:-0} > gpurun_out/bench_mesh_$TAG.json 2>gpurun_out/bench_mesh_$TAG.err || exit 1
timeout -k 10 200 python bench.py --config bookinfo --steps 20 --warmup 5 --cpu-seconds 0 > gpurun_out/bench_book_$TAG.json 2>gpurun_out/bench_book_$TAG.err || exit 1
timeout -k 10 300 python bench.py --config power --steps 10 --warmup 3 --cpu-seconds 0 > gpurun_out/bench_power_$TAG.json 2>gpurun_out/bench_power_$TAG.err || exit 1
echo DONE
