#!/bin/bash
# Round evidence for the default bench workload: rocprofv3 kernel-trace stats + FETCH_SIZE /
# WRITE_SIZE passes (tools/profile.sh), one SQ pass and one clock / MFMA-busy pass, each a run of its
# own (no PMC pass is combined with a trace domain).   usage: tools/gpu_evidence.sh TAG
set -o pipefail
TAG=$1
bash tools/profile.sh $TAG || exit $?
bash tools/sq_counters.sh $TAG || exit $?
bash tools/clk_counters.sh $TAG --no-variants || exit $?
