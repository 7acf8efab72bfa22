# fewer launches per run / fetch (base) against HEAD (old): the GPU suite, Bookinfo, mesh
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/launch
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/launch/tests.log 2>&1 || { tail -40 gpurun_out/launch/tests.log; exit 1; }
tail -1 gpurun_out/launch/tests.log
bash tools/ab/ab_env.sh launchb "--config bookinfo --steps 200 --warmup 50 --no-h2d" 3 new=base old=old || exit 1
bash tools/ab/ab_env.sh launchm "--steps 20 --warmup 3 --no-h2d" 2 new=base old=old || exit 1
python3 tools/ab/abread.py gpurun_out/ab_launchb
python3 tools/ab/abread.py gpurun_out/ab_launchm
