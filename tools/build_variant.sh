#!/bin/bash
# Timing-experiment build: tools/build_variant.sh NAME "-DMACRO ..." -> libopenpose_hip.NAME.so
# (the product Makefile, per-object scheduler flags included, plus DEFS; loaded with
# OP_LIB_VARIANT=NAME; never the product library)
set -e
NAME=$1; DEFS=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=chainer_realtime_multi-person_pose_estimation_amd
W=/tmp/opvar_$NAME; rm -rf $W; mkdir -p $W/$PKG/csrc $W/include
cp $ROOT/$PKG/csrc/*.hip $ROOT/$PKG/csrc/*.hpp $ROOT/$PKG/csrc/*.cpp $ROOT/$PKG/csrc/Makefile $W/$PKG/csrc/
cp $ROOT/include/*.h $W/include/
make -s -j8 -C $W/$PKG/csrc DEFS="$DEFS"
cp $W/$PKG/libopenpose_hip.so $ROOT/$PKG/libopenpose_hip.$NAME.so
echo built $ROOT/$PKG/libopenpose_hip.$NAME.so with $DEFS
