#!/bin/bash
# diagnostic of the config-5 shard/whole group partials + the tail / service-sum tests
mkdir -p gpurun_out/diag
step() {  # name, command...: stop the script after a GPU fault, abort or time limit
  local name=$1; shift
  timeout -k 10 "$@" > gpurun_out/diag/$name.txt 2>&1
  local rc=$?
  echo "$name rc=$rc"
  case $rc in 124|134|137|139) echo "stopping after $name"; exit $rc;; esac
  return 0
}
step base 120 python -u tools/diag_shard.py
KMZ_ABLATE=8192 step nograph 120 python -u tools/diag_shard.py
KMZ_LIB_VARIANT=s0 step s0 120 python -u tools/diag_shard.py
step tests 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_tail.py \
  "tests/test_gpu_parity.py::test_shard_generation_and_index_map"
tail -5 gpurun_out/diag/tests.txt
