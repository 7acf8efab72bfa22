#!/bin/bash
# tail parity tests, then the config-5 bench (host phase times on stderr)
export TMPDIR=/tmp
TAG=${1:-r04}
timeout -k 10 400 python -u -m pytest tests/test_tail.py tests/test_dist_engine.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tailtests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tailtests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tailtests.log
for rep in 1 2; do
  KMZ_BENCH_TRACE=1 timeout -k 10 300 python bench.py --config power --steps 10 --warmup 3 --cpu-seconds 0 --no-h2d > gpurun_out/${TAG}_power_$rep.json 2> gpurun_out/${TAG}_power_$rep.err || exit 1
  python3 -c "
import json;d=json.load(open('gpurun_out/${TAG}_power_$rep.json'));k=d['roofline']['kernels']
print('power', d['ms_per_step'], {x: k[x]['ms_per_step'] for x in k if k[x]['ms_per_step'] > 0.04})"
  grep phase gpurun_out/${TAG}_power_$rep.err
done
