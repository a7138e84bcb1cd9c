#!/bin/bash
# A/B aid: build the library of git revision REV as libopenpose_hip.NAME.so next to the product one
# (loaded with OP_LIB_VARIANT=NAME by _lib.py / tools/ab_lib.py; never the product library).
# usage: tools/build_rev.sh REV NAME
set -e
REV=$1; NAME=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=chainer_realtime_multi-person_pose_estimation_amd
W=/tmp/oprev_$NAME; rm -rf $W; mkdir -p $W/$PKG/csrc $W/include
git -C $ROOT archive $REV $PKG/csrc include | tar -x -C $W
make -s -j8 -C $W/$PKG/csrc
cp $W/$PKG/libopenpose_hip.so $ROOT/$PKG/libopenpose_hip.$NAME.so
echo built $ROOT/$PKG/libopenpose_hip.$NAME.so from $REV
