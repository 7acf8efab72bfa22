#!/bin/bash
# Round-end measurement (run on the box via gpurun): every GPU test, the
# rocprofv3 kernel trace of the default bench, the stamped PMC traffic of
# this build, then the bench lines of configs 2/3/5 with their CPU baselines,
# the production-tick latency, a 2-rank rehearsal of the multi-GPU bench over
# gloo, and 1e9 spans on one GPU (last: the heaviest).  Every GPU step has its own limit; stop at the
# first failure.  usage: tools/final_cycle.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-final}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests exit $rc" >> $O/tests.log; [ $rc -eq 0 ] || exit 1
# (optional A/B of a variant build on config 5 before the measurements: FINAL_AB=<variant>)
if [ -n "$FINAL_AB" ]; then
  for rep in 1 2; do
    timeout -k 10 300 python -u bench.py --config power --steps 10 --warmup 3 --cpu-seconds 0 --no-h2d > $O/ab_power_def_$rep.json 2> $O/ab_power_def_$rep.err || exit 1
    KMZ_LIB_VARIANT=$FINAL_AB timeout -k 10 300 python -u bench.py --config power --steps 10 --warmup 3 --cpu-seconds 0 --no-h2d > $O/ab_power_${FINAL_AB}_$rep.json 2> $O/ab_power_${FINAL_AB}_$rep.err || exit 1
  done
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o mesh -- python3 bench.py --steps 5 --warmup 2 --cpu-seconds 0 > $O/prof.log 2>&1 || exit 1
bash tools/traffic.sh $TAG > $O/traffic.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > $O/bench_mesh.json 2> $O/bench_mesh.err || exit 1
timeout -k 10 300 python -u bench.py --config bookinfo --steps 200 --warmup 50 > $O/bench_book.json 2> $O/bench_book.err || exit 1
timeout -k 10 300 python -u bench.py --config power --steps 10 --warmup 3 > $O/bench_power.json 2> $O/bench_power.err || exit 1
timeout -k 10 300 python -u tools/bench_tick.py > $O/tick.json 2> $O/tick.err || exit 1
bash tools/rehearse_multi.sh 2 --spans 2e7 > $O/rehearse2.json 2> $O/rehearse2.err || exit 1
timeout -k 10 300 python -u bench.py --spans 1e9 --steps 5 --warmup 2 --cpu-seconds 0 > $O/bench_mesh1B.json 2> $O/bench_mesh1B.err || exit 1
echo FINAL_DONE
