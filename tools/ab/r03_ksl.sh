#!/bin/bash
# lockstep k_key_slice (variant ksl): config 5 default vs variant twice, then
# the variant's direct-enumeration parity tests.  usage: tools/r03_ksl.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-ksl}
O=gpurun_out/$TAG
mkdir -p $O
for rep in 1 2; do
  unset KMZ_LIB_VARIANT
  timeout -k 10 300 python -u bench.py --config power --steps 10 --warmup 3 --cpu-seconds 0 --no-h2d > $O/power_def_$rep.json 2> $O/power_def_$rep.err || exit 1
  KMZ_LIB_VARIANT=ksl timeout -k 10 300 python -u bench.py --config power --steps 10 --warmup 3 --cpu-seconds 0 --no-h2d > $O/power_ksl_$rep.json 2> $O/power_ksl_$rep.err || exit 1
done
KMZ_LIB_VARIANT=ksl timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_tail.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  -k "direct or compact or key_staging or headline_config5 or power" > $O/tests.log 2>&1
rc=$?; echo "tests exit $rc" >> $O/tests.log; [ $rc -eq 0 ] || exit 1
echo KSL_DONE
