# compile-knob sweep on the end-of-round arrangement (mesh)
set -o pipefail
export TMPDIR=/tmp
bash tools/ab/ab_env.sh sweep "--steps 20 --warmup 3 --no-h2d" 2 base=base pq4=pq4 cct512=cct512 k3u2=k3u2 k3u8=k3u8 tw6=tw6 || exit 1
python3 tools/ab/abread.py gpurun_out/ab_sweep
