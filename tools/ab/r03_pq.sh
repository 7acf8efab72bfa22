#!/bin/bash
# certificate pass-2 chunk (KMZ_CERT_PQ) A/B on the mesh: default vs variant
# twice, then the variant's certificate tests.  usage: tools/r03_pq.sh TAG VARIANT
set -o pipefail
export TMPDIR=/tmp
TAG=$1; V=$2
O=gpurun_out/$TAG
mkdir -p $O
for rep in 1 2; do
  unset KMZ_LIB_VARIANT
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-h2d > $O/mesh_def_$rep.json 2> $O/mesh_def_$rep.err || exit 1
  KMZ_LIB_VARIANT=$V timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-h2d > $O/mesh_${V}_$rep.json 2> $O/mesh_${V}_$rep.err || exit 1
done
KMZ_LIB_VARIANT=$V timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_guard.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  -k "repeat or cert or wide or window_join or synthetic_vs_c_oracle" > $O/tests.log 2>&1
rc=$?; echo "tests exit $rc" >> $O/tests.log; [ $rc -eq 0 ] || exit 1
echo PQ_DONE
