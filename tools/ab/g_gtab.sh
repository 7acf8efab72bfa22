# the kept gather table's GPU test, then a short default bench line (stamped traffic found?)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/gtab
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "gather_table or sig_collision" --timeout 120 --timeout-method thread > gpurun_out/gtab/tests.log 2>&1 || { tail -40 gpurun_out/gtab/tests.log; exit 1; }
tail -3 gpurun_out/gtab/tests.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-seconds 0 > gpurun_out/gtab/bench.json 2> gpurun_out/gtab/bench.err || exit 1
python3 -c "import json;d=json.loads(open('gpurun_out/gtab/bench.json').read().splitlines()[-1]);r=d['roofline'];print(d['ms_per_step'],r['frac'],r['traffic'],r['traffic_lower'],r['traffic_source'])"
