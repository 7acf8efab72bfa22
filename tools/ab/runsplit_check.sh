# kmz_run_begin/_end: every GPU test, then config 5 (tail host finish beside the next run) and the mesh
export TMPDIR=/tmp
O=gpurun_out/rsc
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 1
for c in power power mesh; do
  KMZ_BENCH_TRACE=1 timeout -k 10 300 python -u bench.py --config $c --cpu-seconds 0 --no-h2d > $O/$c.json 2> $O/$c.err || exit 1
  grep -o '"ms_per_step": [0-9.]*' $O/$c.json | head -1
  grep "phase ms" $O/$c.err
done
echo RSC_DONE
