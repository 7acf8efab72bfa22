# k4_tile8 tile geometry: 960 spans x 2 walkers (base) against 1440 x 3 and 1920 x 4
set -o pipefail
export TMPDIR=/tmp
bash tools/ab/ab_env.sh t8 "--steps 20 --warmup 3 --no-h2d" 2 base=base t1440=t1440 t1920=t1920 t1920w5=t1920w6 || exit 1
python3 tools/ab/abread.py gpurun_out/ab_t8
