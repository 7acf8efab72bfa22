#!/bin/bash
# Round-5 measurement, part 2: configs 2 and 5, the tick latency, the 2-rank
# gloo rehearsal and 1e9 spans on one GPU.  usage: tools/r05_measure2.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-m}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u bench.py --config bookinfo --steps 200 --warmup 50 > $O/bench_book.json 2> $O/bench_book.err || exit 1
timeout -k 10 300 python -u bench.py --config power --steps 10 --warmup 3 > $O/bench_power.json 2> $O/bench_power.err || exit 1
timeout -k 10 300 python -u tools/bench_tick.py > $O/tick.json 2> $O/tick.err || exit 1
bash tools/rehearse_multi.sh 2 --spans 2e7 > $O/rehearse2.json 2> $O/rehearse2.err || exit 1
timeout -k 10 300 python -u bench.py --spans 1e9 --steps 5 --warmup 2 --cpu-seconds 0 > $O/bench_mesh1B.json 2> $O/bench_mesh1B.err || exit 1
timeout -k 10 300 python tools/bench_guard.py > $O/guard_cost.json 2> $O/guard_cost.err || exit 1
echo MEASURE2_DONE
