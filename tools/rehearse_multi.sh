#!/bin/bash
# Rehearsal of bench.py's multi-rank path (sharding, table digest, the three
# merge collectives on device tensors, the union of edge keys) on a one-GPU
# box: N ranks on cuda:0 over gloo.  usage: tools/rehearse_multi.sh N [bench args]
export TMPDIR=/tmp
N=${1:-2}; shift
KMZ_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus $N --steps 3 --warmup 1 --cpu-seconds 0 --no-h2d "$@"
