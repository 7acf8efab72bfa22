# join at 46 KB (base), + k3_produce beside the join (bit 19), against HEAD (old)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/k3p
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/k3p/tests.log 2>&1 || { tail -40 gpurun_out/k3p/tests.log; exit 1; }
KMZ_ABLATE2=524288 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/k3p/tests19.log 2>&1 || { tail -40 gpurun_out/k3p/tests19.log; exit 1; }
tail -1 gpurun_out/k3p/tests.log; tail -1 gpurun_out/k3p/tests19.log
bash tools/ab/ab_env.sh k3p "--steps 20 --warmup 3 --no-h2d" 2 base=base split=base:KMZ_ABLATE2=524288 old=old || exit 1
python3 tools/ab/abread.py gpurun_out/ab_k3p
