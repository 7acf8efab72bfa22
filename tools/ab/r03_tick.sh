#!/bin/bash
# GPU tests, then the production-tick latency (tools/bench_tick.py) and its
# kernel trace.  usage: tools/r03_tick.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-tick}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests exit $rc" >> $O/tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/bench_tick.py > $O/tick.json 2> $O/tick.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o tick -- python3 tools/bench_tick.py --ticks 50 > $O/tick_prof.json 2> $O/tick_prof.err || exit 1
timeout -k 10 300 python -u bench.py --config bookinfo --steps 20 --warmup 5 --cpu-seconds 0 > $O/bench_book.json 2> $O/bench_book.err || exit 1
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-seconds 0 > $O/bench_mesh.json 2> $O/bench_mesh.err || exit 1
timeout -k 10 300 python -u bench.py --config power --steps 10 --warmup 3 --cpu-seconds 0 > $O/bench_power.json 2> $O/bench_power.err || exit 1
echo TICK_DONE
