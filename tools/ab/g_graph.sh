# hipGraph replay of the run (KMZ_HIPGRAPH=1) against direct launches, mesh / Bookinfo / config 5
set -o pipefail
export TMPDIR=/tmp
bash tools/ab/ab_env.sh graphm "--steps 20 --warmup 3 --no-h2d" 2 direct=base graph=base:KMZ_HIPGRAPH=1 || exit 1
bash tools/ab/ab_env.sh graphb "--config bookinfo --steps 200 --warmup 50 --no-h2d" 2 direct=base graph=base:KMZ_HIPGRAPH=1 || exit 1
bash tools/ab/ab_env.sh graphp "--config power --steps 10 --warmup 3 --no-h2d" 1 direct=base graph=base:KMZ_HIPGRAPH=1 || exit 1
for d in graphm graphb graphp; do python3 tools/ab/abread.py gpurun_out/ab_$d; done
