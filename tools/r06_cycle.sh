#!/bin/bash
# Round-6 full cycle on the box: the GPU suite, then the default bench lines
# of configs 3 / 5 / 2 (A/B against k4_tile8 on the mesh), then the tick.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-c}
D=gpurun_out/r06$TAG
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  > $D/tests.log 2>&1
rc=$?
tail -3 $D/tests.log
[ $rc -eq 0 ] || exit 1
bash tools/ab/ab_env.sh ${TAG}m "--steps 10 --warmup 3" 2 t9=base t8=base:KMZ_ABLATE2=4194304 || exit 1
python3 tools/ab/abread.py gpurun_out/ab_${TAG}m
bash tools/ab/ab_env.sh ${TAG}p "--config power --steps 10 --warmup 3" 2 t9=base || exit 1
python3 tools/ab/abread.py gpurun_out/ab_${TAG}p
bash tools/ab/ab_env.sh ${TAG}b "--config bookinfo --steps 200 --warmup 50" 2 graph=base direct=base:KMZ_HIPGRAPH=0 || exit 1
python3 tools/ab/abread.py gpurun_out/ab_${TAG}b
timeout -k 10 300 python -u tools/bench_tick.py > $D/tick.json 2> $D/tick.err || exit 1
python3 -c "
import json
d=json.load(open('$D/tick.json'))
for c,v in d['configs'].items():
    print(c, v.get('spans'), {k:(x['run_fetch_us_median'], x['tick_us_median']) for k,x in v.items() if isinstance(x,dict)})
"
echo CYCLE_DONE
