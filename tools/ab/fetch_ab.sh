# A/B: bench.py --fetch sync vs pipelined (kmz_fetch_begin/_end), mesh; then config 5
mkdir -p gpurun_out/fab
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "pipelined_fetch or bookinfo" > gpurun_out/fab/t.log 2>&1 || exit 1
tail -2 gpurun_out/fab/t.log
for m in sync pipelined sync pipelined; do
  KMZ_BENCH_TRACE=1 timeout -k 10 200 python bench.py --cpu-seconds 0 --no-h2d --steps 30 --fetch $m \
    > gpurun_out/fab/$m.json 2> gpurun_out/fab/$m.err || exit 1
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/fab/$m.json | head -1
  grep "step ms" gpurun_out/fab/$m.err | cut -c1-200
done
timeout -k 10 200 python bench.py --cpu-seconds 0 --no-h2d --config power > gpurun_out/fab/power.json \
  2> gpurun_out/fab/power.err || exit 1
grep -o '"ms_per_step": [0-9.]*' gpurun_out/fab/power.json
