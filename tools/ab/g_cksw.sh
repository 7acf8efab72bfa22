# k_cert_check with swizzled bucket slots (base) against HEAD (old)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/cksw
timeout -k 10 600 python -u -m pytest tests/test_gpu_guard.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/cksw/tests.log 2>&1 || { tail -40 gpurun_out/cksw/tests.log; exit 1; }
tail -2 gpurun_out/cksw/tests.log
bash tools/ab/ab_env.sh cksw "--steps 20 --warmup 3 --no-h2d" 2 sw=base old=old || exit 1
python3 tools/ab/abread.py gpurun_out/ab_cksw
