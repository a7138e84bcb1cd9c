#!/bin/bash
# Fabric read bytes by request size: one PMC pass of TCC_EA0_RDREQ_{32B,64B,128B} + TCC_EA0_RDREQ
# (4 TCC counters, kernel trace only, nothing else) over the FETCH calibration micro-benchmark (known
# byte counts) and over the default bench per spec; summarised per kernel by tools/tcc_bytes.py.
# FETCH_SIZE's formula counts 128-B requests through TCC_BUBBLE, which stays 0 here, so FETCH_SIZE
# tallies a 128-B request at 64 B; these counters give the bytes directly.
# usage: tools/gpu_tcc_bytes.sh TAG [spec...]   (spec: base, a library variant, or NAME=VALUE[,NAME=VALUE])
set -o pipefail
TAG=$1; shift
O=$GRAFT_REPO_ROOT/gpurun_out/tcc_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
C="TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum"
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/calib -o run -- \
  $GRAFT_REPO_ROOT/tools/micro/fetch_calib > $O/calib.log 2>&1 || exit $?
for spec in "${@:-base}"; do
  (
    if [ "$spec" != base ]; then
      case "$spec" in
        *=*) for kv in ${spec//,/ }; do export "$kv"; done ;;
        *) export OP_LIB_VARIANT=$spec ;;
      esac
    fi
    timeout -s KILL 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/$spec -o run -- \
      python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-variants --no-profile \
      > $O/$spec.log 2>&1
  ) || exit $?
done
python3 $GRAFT_REPO_ROOT/tools/tcc_bytes.py $O > $O/summary.txt
