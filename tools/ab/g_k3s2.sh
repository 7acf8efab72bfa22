# K3 beside config 5's settle as the default: the GPU suite, then A/B against beside the join (KMZ_ABLATE2 bit 21)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/k3s2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/k3s2/tests.log 2>&1 || { tail -40 gpurun_out/k3s2/tests.log; exit 1; }
tail -1 gpurun_out/k3s2/tests.log
bash tools/ab/ab_env.sh k3s2 "--config power --steps 20 --warmup 3 --no-h2d" 3 new=base old=base:KMZ_ABLATE2=2097152 || exit 1
bash tools/ab/ab_env.sh k3s2m "--steps 20 --warmup 3 --no-h2d" 1 new=base old=base:KMZ_ABLATE2=2097152 || exit 1
python3 tools/ab/abread.py gpurun_out/ab_k3s2
python3 tools/ab/abread.py gpurun_out/ab_k3s2m
