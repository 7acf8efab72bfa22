# run graphs with the live timing events (KMZ_HIPGRAPH=1) against direct launches: Bookinfo, a 4e6-span mesh
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/graph2
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "graph or small or book" > gpurun_out/graph2/tests.log 2>&1 || { tail -30 gpurun_out/graph2/tests.log; exit 1; }
tail -1 gpurun_out/graph2/tests.log
bash tools/ab/ab_env.sh graph2b "--config bookinfo --steps 200 --warmup 50 --no-h2d" 3 direct=base graph=base:KMZ_HIPGRAPH=1 || exit 1
bash tools/ab/ab_env.sh graph2m "--spans 4e6 --steps 100 --warmup 20 --no-h2d" 2 direct=base graph=base:KMZ_HIPGRAPH=1 || exit 1
python3 tools/ab/abread.py gpurun_out/ab_graph2b
python3 tools/ab/abread.py gpurun_out/ab_graph2m
grep -h '"graph' gpurun_out/ab_graph2b/graph_1.json | head -0
python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/ab_graph2b/graph_1.json') if l.startswith('{')][-1])
print(d['roofline'].get('kernel'), d['roofline'].get('achieved'), d['roofline'].get('frac'))
"
