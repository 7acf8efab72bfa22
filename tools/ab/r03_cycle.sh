#!/bin/bash
# Round-3 GPU cycle (run on the box via gpurun): all GPU tests, then the
# default bench lines of configs 3/2/5.  Every GPU step has its own limit;
# stop at the first failure.  usage: tools/r03_cycle.sh TAG [pytest -k expr]
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-x}
O=gpurun_out/$TAG
mkdir -p $O
if [ -n "$2" ]; then K=(-k "$2"); else K=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 240 --timeout-method thread "${K[@]}" > $O/tests.log 2>&1
rc=$?; echo "tests exit $rc" >> $O/tests.log; [ $rc -eq 0 ] || exit 1
[ -n "$NOBENCH" ] && exit 0
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-seconds 0 > $O/bench_mesh.json 2> $O/bench_mesh.err || exit 1
timeout -k 10 300 python -u bench.py --config bookinfo --steps 20 --warmup 5 --cpu-seconds 0 > $O/bench_book.json 2> $O/bench_book.err || exit 1
timeout -k 10 300 python -u bench.py --config power --steps 10 --warmup 3 --cpu-seconds 0 > $O/bench_power.json 2> $O/bench_power.err || exit 1
echo CYCLE_DONE
