#!/bin/bash
# Bench lines of configs 2/3/5 again on another box (host-side gaps vary by
# box; the kernels do not).  usage: tools/r03_rebench.sh TAG
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 python -u bench.py --config bookinfo --steps 200 --warmup 50 > $O/bench_book.json 2> $O/bench_book.err || exit 1
timeout -k 10 300 python -u bench.py --config power --steps 10 --warmup 3 > $O/bench_power.json 2> $O/bench_power.err || exit 1
timeout -k 10 300 python -u bench.py > $O/bench_mesh.json 2> $O/bench_mesh.err || exit 1
echo REBENCH_DONE
