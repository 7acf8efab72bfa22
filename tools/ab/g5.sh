set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu > gpurun_out/t_parity5.log 2>&1 || exit 1
tools/ab/ab_env.sh w8 "--steps 10 --warmup 3" 2 old=base:KMZ_ABLATE2=1024 w8=base w7=w7 w6=w6
