#!/bin/bash
# K3 partition sums split over workgroups, certificate 2^8 bins at 5e8 / 1e9
# spans (default vs KMZ_ABLATE2 bit 7), tick latency.  usage: tools/r03_k3b.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-k3b}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  -k "k3 or wide or synthetic_vs_c_oracle or shard_generation" > $O/tests.log 2>&1
rc=$?; echo "tests exit $rc" >> $O/tests.log; [ $rc -eq 0 ] || exit 1
b() {  # name, ablate, ablate2, bench args...
  local name=$1 ab=$2 ab2=$3; shift 3
  KMZ_ABLATE=$ab KMZ_ABLATE2=$ab2 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-h2d "$@" \
    > $O/$name.json 2> $O/$name.err || exit 1
}
b mesh 0 0
b mesh_k3fixed 16384 0
b power 0 0 --config power
b mesh5e8 0 0 --spans 5e8 --steps 5 --warmup 2
b mesh5e8_narrow 0 128 --spans 5e8 --steps 5 --warmup 2
b mesh1B_narrow 0 128 --spans 1e9 --steps 5 --warmup 2
timeout -k 10 300 python -u tools/bench_tick.py > $O/tick.json 2> $O/tick.err || exit 1
echo K3B_DONE
