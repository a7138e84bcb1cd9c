#!/bin/bash
# Round 4: the tests named in $SEL first (verbose), then (FULL=1) the whole GPU suite, then one
# bench line (BENCH=1, extra args in $BARGS).   usage: SEL="tests/x.py -k y" tools/gpu_r04_check.sh TAG
set -o pipefail
TAG=${1:-r04}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $O
if [ -n "$SEL" ]; then
  timeout -k 10 900 python -u -m pytest -v -s --timeout 600 --timeout-method thread $SEL > $O/sel.log 2>&1 || exit $?
fi
if [ -n "$FULL" ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/suite.log 2>&1 || exit $?
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 600 python -u bench.py $BARGS > $O/bench.log 2>&1 || exit $?
fi
echo done
