#!/bin/bash
# every GPU test, then the mesh bench (balanced vs fixed-slice K3 reduce) and
# 10^9 spans on one GPU (the certificate's 2^8 pass-1 bins).  usage: tools/r03_cert.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-cert}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests exit $rc" >> $O/tests.log; [ $rc -eq 0 ] || exit 1
b() {  # name, ablate, bench args...
  local name=$1 ab=$2; shift 2
  KMZ_ABLATE=$ab timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-h2d "$@" \
    > $O/$name.json 2> $O/$name.err || exit 1
}
b mesh 0
b mesh_k3fixed 16384
b power 0 --config power
b power_k3fixed 16384 --config power
b mesh1B 0 --spans 1e9 --steps 5 --warmup 2
echo CERT_DONE
