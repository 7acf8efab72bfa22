#!/bin/bash
# Build an A/B variant of the engine into kmamiz_amd/libkmz_<name>.so with
# extra defines (diagnostic; selected at run time by KMZ_LIB_VARIANT=<name>).
# usage: tools/variant.sh NAME -DKNOB=VALUE ...
set -e
NAME=$1; shift
D=build/var_$NAME
mkdir -p $D
HIPFLAGS="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=off $*"
objs=""
for f in kmamiz_amd/csrc/*.hip; do
  o=$D/$(basename $f .hip).o
  /opt/rocm/bin/hipcc $HIPFLAGS -c $f -o $o &
  objs="$objs $o"
done
g++ -O3 -std=c++17 -fPIC -Wall -pthread -c kmamiz_amd/csrc/kmz_ingest.cpp -o $D/kmz_ingest.o &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -pthread -o kmamiz_amd/libkmz_$NAME.so $objs $D/kmz_ingest.o
echo built kmamiz_amd/libkmz_$NAME.so
