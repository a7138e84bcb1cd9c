#!/bin/bash
# A/B aid: build the working tree's library with per-object Makefile flags as
# libopenpose_hip.NAME.so (loaded with OP_LIB_VARIANT=NAME; never the product library).
# usage: tools/build_flags.sh NAME 'FLAGS_conv_head=-mllvm -amdgpu-sched-strategy=max-ilp' ...
set -e
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=chainer_realtime_multi-person_pose_estimation_amd
W=/tmp/opflags_$NAME; rm -rf $W; mkdir -p $W/$PKG/csrc $W/include
cp $ROOT/$PKG/csrc/*.hip $ROOT/$PKG/csrc/*.hpp $ROOT/$PKG/csrc/*.cpp $ROOT/$PKG/csrc/Makefile $W/$PKG/csrc/
cp $ROOT/include/*.h $W/include/
make -s -j8 -C $W/$PKG/csrc "$@"
cp $W/$PKG/libopenpose_hip.so $ROOT/$PKG/libopenpose_hip.$NAME.so
echo built $ROOT/$PKG/libopenpose_hip.$NAME.so
