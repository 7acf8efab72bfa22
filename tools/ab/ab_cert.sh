set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/abc
timeout -k 10 300 python -u -m pytest tests/test_gpu_guard.py tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -k "guard or repeat or synthetic_vs_c or headline or window_join or messy_batches_vs_oracle" > gpurun_out/abc/tests.log 2>&1 || exit 1
for sp in 1e8 1e9; do
for v in base pb0 pb3; do
  [ "$v" = base ] && vv="" || vv=$v
  KMZ_LIB_VARIANT=$vv timeout -k 10 300 python bench.py --spans $sp --steps 5 --warmup 2 --cpu-seconds 0 --no-h2d > gpurun_out/abc/ab_${v}_$sp.json 2>gpurun_out/abc/ab_${v}_$sp.err || { echo "$v $sp failed"; exit 1; }
done; done
echo AB_DONE
