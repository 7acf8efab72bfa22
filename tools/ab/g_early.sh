set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/e1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/e1/tests.log 2>&1 || { tail -40 gpurun_out/e1/tests.log; exit 1; }
tail -3 gpurun_out/e1/tests.log
bash tools/ab/ab_env.sh early "--steps 20 --warmup 3" 3 early=base old=base:KMZ_ABLATE2=8192 || exit 1
python3 tools/ab/abread.py gpurun_out/ab_early
