#!/bin/bash
# Round-end evidence on the final tree: smoke, the whole GPU suite, the bench lines (default
# headline with its side lines, C5 720p, C4 multi-scale), then the rocprofv3 evidence set
# (kernel-trace stats, FETCH_SIZE / WRITE_SIZE, SQ, clock / MFMA busy, fabric reads by request
# size), each PMC pass a run of its own.   usage: tools/gpu_final.sh TAG
set -o pipefail
TAG=${1:-r04z}
O=$GRAFT_REPO_ROOT/gpurun_out/final_$TAG; mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/suite.log 2>&1 || exit $?
bash tools/gpu_lines.sh $TAG || exit $?
bash tools/gpu_evidence.sh $TAG || exit $?
bash tools/gpu_tcc_bytes.sh $TAG || exit $?
echo done
