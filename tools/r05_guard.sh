#!/bin/bash
# The guard's GPU tests, its cost (tools/bench_guard.py), the 2-rank
# rehearsal of bench.py's multi-rank path and one mesh bench line, on the box.
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/${1:-g2}
mkdir -p $D
timeout -k 10 700 python -u -m pytest tests/test_gpu_guard.py tests/test_dist_engine.py -x -v --timeout 200 --timeout-method thread > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -3 $D/tests.log
timeout -k 10 400 python -u tools/bench_guard.py > $D/guard_cost.json 2> $D/guard_cost.err || { tail -20 $D/guard_cost.err; exit 1; }
cat $D/guard_cost.json
bash tools/rehearse_multi.sh 2 --spans 2e7 > $D/rehearse2.json 2> $D/rehearse2.err || { tail -20 $D/rehearse2.err; exit 1; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 0 > $D/bench_mesh.json 2> $D/bench_mesh.err || { tail -20 $D/bench_mesh.err; exit 1; }
python3 -c "import json;d=json.loads(open('$D/bench_mesh.json').read().strip().splitlines()[-1]);print('mesh',d['ms_per_step'],d['value'])"
echo GUARD_DONE
