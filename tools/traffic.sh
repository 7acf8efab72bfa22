#!/bin/bash
# PMC traffic of the current build on the mesh bench (run on the box via
# gpurun): FETCH_SIZE and WRITE_SIZE passes, one each, then the stamped
# summary gpurun_out/traffic_<TAG>.json (copy it to profiles/ to be quoted).
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-x}
ARGS="--steps 2 --warmup 1 --cpu-seconds 0"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/trf_$TAG/fetch -o run -- python3 bench.py $ARGS > gpurun_out/trf_$TAG.fetch.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/trf_$TAG/write -o run -- python3 bench.py $ARGS > gpurun_out/trf_$TAG.write.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d gpurun_out/trf_$TAG/tcc -o run -- python3 bench.py $ARGS > gpurun_out/trf_$TAG.tcc.log 2>&1 || exit 1
N=$(python3 -c "import json;print(json.loads([l for l in open('gpurun_out/trf_$TAG.fetch.log') if l.startswith('{')][-1])['config']['spans_per_gpu'])")
python3 tools/pmc_traffic.py gpurun_out/trf_$TAG/fetch gpurun_out/trf_$TAG/write 3 $N gpurun_out/traffic_$TAG.json gpurun_out/trf_$TAG/tcc > /dev/null || exit 1
echo TRAFFIC_DONE
