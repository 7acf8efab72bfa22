# K3 between the join and the walk on the main stream (KMZ_ABLATE2 bit 17) against beside the join
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/k3mid
KMZ_ABLATE2=131072 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/k3mid/tests.log 2>&1 || { tail -40 gpurun_out/k3mid/tests.log; exit 1; }
tail -2 gpurun_out/k3mid/tests.log
bash tools/ab/ab_env.sh k3mid "--steps 20 --warmup 3" 2 side=base mid=base:KMZ_ABLATE2=131072 || exit 1
bash tools/ab/ab_env.sh k3mid5 "--config power --steps 20 --warmup 3" 2 side=base mid=base:KMZ_ABLATE2=131072 || exit 1
python3 tools/ab/abread.py gpurun_out/ab_k3mid
python3 tools/ab/abread.py gpurun_out/ab_k3mid5
