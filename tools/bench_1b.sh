#!/bin/bash
# config 4's whole batch (10^9 mesh spans) on one GPU: bench line + its stderr
export TMPDIR=/tmp
TAG=${1:-r04}
timeout -k 10 400 python -u bench.py --spans 1e9 --steps 5 --warmup 2 --cpu-seconds 0 --no-h2d > gpurun_out/${TAG}_1b.json 2> gpurun_out/${TAG}_1b.err || exit 1
python3 -c "
import json;d=json.load(open('gpurun_out/${TAG}_1b.json'));k=d['roofline']['kernels']
print('1e9', d['ms_per_step'], {x: k[x]['ms_per_step'] for x in k if k[x]['ms_per_step'] > 0.04})"
