# ticks with the side stream from 2^18 spans, and the Bookinfo bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/tick2
timeout -k 10 300 python -u tools/bench_tick.py > gpurun_out/tick2/tick.json 2> gpurun_out/tick2/tick.err || exit 1
python3 -c "
import json
d=json.load(open('gpurun_out/tick2/tick.json'))
for c,v in d['configs'].items():
    print(c, v.get('spans'), {k:(x['tick_us_median'], x['run_fetch_us_median']) for k,x in v.items() if isinstance(x,dict)})
"
bash tools/ab/ab_env.sh book18 "--config bookinfo --steps 200 --warmup 50 --no-h2d" 2 base=base || exit 1
python3 tools/ab/abread.py gpurun_out/ab_book18
