# the walk's gather table kept across runs (base) against HEAD (old): the GPU suite, Bookinfo, config 5
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/etab
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/etab/tests.log 2>&1 || { tail -40 gpurun_out/etab/tests.log; exit 1; }
tail -1 gpurun_out/etab/tests.log
bash tools/ab/ab_env.sh etabb "--config bookinfo --steps 200 --warmup 50 --no-h2d" 3 new=base old=old || exit 1
bash tools/ab/ab_env.sh etabp "--config power --steps 20 --warmup 3 --no-h2d" 2 new=base old=old || exit 1
python3 tools/ab/abread.py gpurun_out/ab_etabb
python3 tools/ab/abread.py gpurun_out/ab_etabp
