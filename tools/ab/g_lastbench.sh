# the default bench line of the committed build (the stamped traffic must be found)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/lastbench
timeout -k 10 400 python -u bench.py > gpurun_out/lastbench/bench.json 2> gpurun_out/lastbench/bench.err || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/lastbench/smoke.log 2>&1 || exit 1
python3 -c "import json;d=json.loads(open('gpurun_out/lastbench/bench.json').read().splitlines()[-1]);r=d['roofline'];print(d['value'],d['ms_per_step'],r['frac'],r['traffic'],r['traffic_lower'],r['l2_hit_rate'],r['traffic_source'],d['cpu_baseline']['value'])"
tail -1 gpurun_out/lastbench/smoke.log
