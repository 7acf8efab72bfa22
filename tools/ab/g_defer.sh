# config 5: certificate beside the settle (default) against between join and walk (KMZ_ABLATE2 bit 15)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/defer
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/defer/tests.log 2>&1 || { tail -40 gpurun_out/defer/tests.log; exit 1; }
tail -2 gpurun_out/defer/tests.log
bash tools/ab/ab_env.sh defer "--config power --steps 20 --warmup 3" 2 defer=base main=base:KMZ_ABLATE2=32768 || exit 1
python3 tools/ab/abread.py gpurun_out/ab_defer
