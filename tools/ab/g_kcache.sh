# config 5: the direct walk's key cache 1024 (base) against 2048 / 512
set -o pipefail
export TMPDIR=/tmp
bash tools/ab/ab_env.sh kcache "--config power --steps 10 --warmup 3 --no-h2d" 2 k1024=base k2048=kc2k k512=kc512 || exit 1
python3 tools/ab/abread.py gpurun_out/ab_kcache
