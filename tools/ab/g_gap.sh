# the step's leading gap: host phases (KMZ_BENCH_TRACE), and the step without the fetch / with a sync fetch
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/gap
KMZ_BENCH_TRACE=1 timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 0 --no-h2d > gpurun_out/gap/trace.json 2> gpurun_out/gap/trace.err || exit 1
grep -E "step ms|phase ms" gpurun_out/gap/trace.err
for a in "--no-fetch" "--fetch sync" ""; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 0 --no-h2d $a > gpurun_out/gap/b.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads([l for l in open('gpurun_out/gap/b.json') if l.startswith('{')][-1]);print('$a', d['ms_per_step'])"
done
