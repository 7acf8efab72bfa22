#!/bin/bash
# service tail: its GPU tests, then config 5 bench lines, the default build
# vs a variant (tools/variant.sh), twice.  usage: tools/r03_tail.sh TAG VARIANT
set -o pipefail
export TMPDIR=/tmp
TAG=$1; V=$2
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_tail.py tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  -k "tail or messy_batches_vs or headline_config5" > $O/tests.log 2>&1
rc=$?; echo "tests exit $rc" >> $O/tests.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  unset KMZ_LIB_VARIANT
  timeout -k 10 300 python -u bench.py --config power --steps 10 --warmup 3 --cpu-seconds 0 --no-h2d > $O/power_def_$rep.json 2> $O/power_def_$rep.err || exit 1
  KMZ_LIB_VARIANT=$V timeout -k 10 300 python -u bench.py --config power --steps 10 --warmup 3 --cpu-seconds 0 --no-h2d > $O/power_${V}_$rep.json 2> $O/power_${V}_$rep.err || exit 1
done
echo TAIL_DONE
