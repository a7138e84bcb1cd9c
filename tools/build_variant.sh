#!/bin/bash
# Timing-experiment build: tools/build_variant.sh NAME "-DMACRO ..." -> libopenpose_hip.NAME.so
# (loaded with OP_LIB_VARIANT=NAME; never the product library)
set -e
NAME=$1; DEFS=$2
SRC=$(cd "$(dirname "$0")/../chainer_realtime_multi-person_pose_estimation_amd/csrc" && pwd)
OUT=/tmp/opvar_$NAME; mkdir -p $OUT
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wno-unused-value -Wno-unused-result -I$SRC/../../include $DEFS"
objs=""
for f in $SRC/*.hip; do
  b=$(basename $f .hip); /opt/rocm/bin/hipcc $FLAGS -c $f -o $OUT/$b.o & objs="$objs $OUT/$b.o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $SRC/../libopenpose_hip.$NAME.so $objs -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo built $SRC/../libopenpose_hip.$NAME.so
