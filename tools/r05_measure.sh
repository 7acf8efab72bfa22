#!/bin/bash
# Round-5 measurement, part 1 (on the box via gpurun): rocprofv3 kernel trace
# + stats of the default bench, the stamped PMC traffic of this build, the
# default bench line.  usage: tools/r05_measure.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-m}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o mesh -- python3 bench.py --steps 5 --warmup 2 --cpu-seconds 0 > $O/prof.log 2>&1 || exit 1
bash tools/traffic.sh $TAG > $O/traffic.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > $O/bench_mesh.json 2> $O/bench_mesh.err || exit 1
echo MEASURE1_DONE
