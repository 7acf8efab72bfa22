# full GPU suite on the new join, then config 5 and Bookinfo against the old build
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/fp8c
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/fp8c/tests.log 2>&1 || { tail -40 gpurun_out/fp8c/tests.log; exit 1; }
tail -2 gpurun_out/fp8c/tests.log
bash tools/ab/ab_env.sh fp8c5 "--config power --steps 20 --warmup 3" 2 fp8=base old=old || exit 1
bash tools/ab/ab_env.sh fp8cb "--config bookinfo --steps 200 --warmup 50" 2 fp8=base old=old || exit 1
python3 tools/ab/abread.py gpurun_out/ab_fp8c5
python3 tools/ab/abread.py gpurun_out/ab_fp8cb
