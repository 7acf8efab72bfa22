#!/bin/bash
# XCD-aware tile order (KMZ_XCD=1 variant build): the mesh bench default vs
# variant twice, then the variant's parity tests.  usage: tools/r03_xcd.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-xcd}
O=gpurun_out/$TAG
mkdir -p $O
for rep in 1 2; do
  unset KMZ_LIB_VARIANT
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-h2d > $O/mesh_def_$rep.json 2> $O/mesh_def_$rep.err || exit 1
  KMZ_LIB_VARIANT=xcd timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-h2d > $O/mesh_xcd_$rep.json 2> $O/mesh_xcd_$rep.err || exit 1
done
KMZ_LIB_VARIANT=xcd timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests exit $rc" >> $O/tests.log; [ $rc -eq 0 ] || exit 1
echo XCD_DONE
