# config 5: K3 beside the direct walk (KMZ_ABLATE2 bit 19) against beside the join
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/k3walk
KMZ_ABLATE2=524288 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "power or config5 or direct or tail" > gpurun_out/k3walk/tests.log 2>&1 || { tail -40 gpurun_out/k3walk/tests.log; exit 1; }
tail -2 gpurun_out/k3walk/tests.log
bash tools/ab/ab_env.sh k3walk "--config power --steps 20 --warmup 3" 2 join=base walk=base:KMZ_ABLATE2=524288 || exit 1
python3 tools/ab/abread.py gpurun_out/ab_k3walk
