#!/bin/bash
# FETCH_SIZE calibration pass (tools/micro/fetch_calib.hip), one PMC counter, kernel trace only
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/fetch_calib; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 $GRAFT_REPO_ROOT/tools/micro/fetch_calib > $O/plain.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch -o run -- $GRAFT_REPO_ROOT/tools/micro/fetch_calib > $O/fetch.log 2>&1
