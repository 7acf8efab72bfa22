# K3 after the walk as the default on the chain-tile path: full suite, then the three configs against bit 18
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/k3late2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/k3late2/tests.log 2>&1 || { tail -40 gpurun_out/k3late2/tests.log; exit 1; }
tail -2 gpurun_out/k3late2/tests.log
bash tools/ab/ab_env.sh k3l2 "--steps 20 --warmup 3" 2 late=base side=base:KMZ_ABLATE2=262144 || exit 1
bash tools/ab/ab_env.sh k3l2p "--config power --steps 20 --warmup 3" 1 late=base side=base:KMZ_ABLATE2=262144 || exit 1
python3 tools/ab/abread.py gpurun_out/ab_k3l2
python3 tools/ab/abread.py gpurun_out/ab_k3l2p
