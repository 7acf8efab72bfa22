# k3_combine_bal with its item loop unrolled (base) against HEAD (old); rocprof of the combine
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/comb
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "k3 or stats or reduce or group" > gpurun_out/comb/tests.log 2>&1 || { tail -40 gpurun_out/comb/tests.log; exit 1; }
tail -2 gpurun_out/comb/tests.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/comb/prof -o new -- python3 bench.py --steps 5 --warmup 2 --cpu-seconds 0 --no-h2d > gpurun_out/comb/prof_new.log 2>&1 || exit 1
KMZ_LIB_VARIANT=old timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/comb/prof -o old -- python3 bench.py --steps 5 --warmup 2 --cpu-seconds 0 --no-h2d > gpurun_out/comb/prof_old.log 2>&1 || exit 1
grep -h "combine\|k3_first\|k3_reduce" gpurun_out/comb/prof/*stats.csv | cut -c1-160
bash tools/ab/ab_env.sh comb "--steps 20 --warmup 3 --no-h2d" 2 new=base old=old || exit 1
python3 tools/ab/abread.py gpurun_out/ab_comb
