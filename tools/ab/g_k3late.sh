# K3 after the walk on the main stream (KMZ_ABLATE2 bit 18) against beside the join
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/k3late
KMZ_ABLATE2=262144 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/k3late/tests.log 2>&1 || { tail -40 gpurun_out/k3late/tests.log; exit 1; }
tail -2 gpurun_out/k3late/tests.log
bash tools/ab/ab_env.sh k3late "--steps 20 --warmup 3" 2 side=base late=base:KMZ_ABLATE2=262144 || exit 1
python3 tools/ab/abread.py gpurun_out/ab_k3late
