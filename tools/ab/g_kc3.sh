# config 5: key cache of 4096 32-bit residuals (base) against 2048 whole keys (old)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/kc3
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/kc3/tests.log 2>&1 || { tail -40 gpurun_out/kc3/tests.log; exit 1; }
tail -2 gpurun_out/kc3/tests.log
bash tools/ab/ab_env.sh kc3 "--config power --steps 20 --warmup 3" 2 r32=base k64=old || exit 1
python3 tools/ab/abread.py gpurun_out/ab_kc3
