# per-tick latency of the f2 build (libkmz_f2.so) against HEAD, alternated on one box
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/tickab
for i in 1 2; do
  KMZ_LIB_VARIANT=f2 timeout -k 10 200 python -u tools/bench_tick.py > gpurun_out/tickab/old_$i.json 2> gpurun_out/tickab/old_$i.err || exit 1
  timeout -k 10 200 python -u tools/bench_tick.py > gpurun_out/tickab/new_$i.json 2> gpurun_out/tickab/new_$i.err || exit 1
done
python3 - <<'P'
import json
for n in ['old_1','new_1','old_2','new_2']:
    t=json.load(open(f'gpurun_out/tickab/{n}.json'))
    print(n, {c:(v['default']['run_fetch_us_median'],v['default']['tick_us_median'],v['serial']['tick_us_median']) for c,v in t['configs'].items()})
P
