#!/bin/bash
# Round-end evidence on the final tree (round 6): first the rocprofv3 kernel-trace stats + FETCH_SIZE
# / WRITE_SIZE passes of the three bench lines (headline 368x368 x 232, C5 720p x 64, C4 multi-scale
# 720p x 16), summarised into profiles/<round>/ ON THE BOX so that the bench lines run after them cite
# this tree's sets (bench.py committed_traffic); then smoke, the whole GPU suite, the bench lines, the
# SQ and clock / MFMA-busy passes and the fabric reads by request size -- each PMC pass a run of its
# own, each step under its own time limit, the first failure ending the call.
#   usage: tools/gpu_round_end.sh TAG [PART]   (e.g. r06z; copies land in gpurun_out/final_TAG/)
#   PART: all (default); prof = the PMC sets, smoke and the bench lines; rest = the suite and the SQ /
#   clock / TCC passes (two calls that each fit gpurun's time limit)
set -o pipefail
TAG=$1; PART=${2:-all}; R=${TAG:0:3}
O=$GRAFT_REPO_ROOT/gpurun_out/final_$TAG; mkdir -p $O
cd $GRAFT_REPO_ROOT
if [ "$PART" != rest ]; then
for spec in "${TAG}_m4_b232|" "${TAG}_c5_m4_b64|--frame 720x1280" "${TAG}_c4_m4_b16|--precise --frame 720x1280"; do
  nm=${spec%%|*}; args=${spec#*|}
  echo "[$(date +%T)] profile $nm $args"
  bash tools/profile.sh $nm $args || exit $?
  python3 tools/summarize_profile.py gpurun_out/prof_$nm $R/$nm > /dev/null || exit $?
  cp profiles/$R/$nm.md profiles/$R/${nm}_traffic.json $O/ || exit $?
done
echo "[$(date +%T)] smoke"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
echo "[$(date +%T)] lines"
bash tools/gpu_lines.sh $TAG || exit $?
cp gpurun_out/lines_$TAG/*.log gpurun_out/lines_$TAG/lines.jsonl $O/ || exit $?
fi
if [ "$PART" != prof ]; then
echo "[$(date +%T)] suite"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/suite.log 2>&1 || exit $?
tail -2 $O/suite.log
echo "[$(date +%T)] sq / clk / tcc"
bash tools/sq_counters.sh $TAG || exit $?
bash tools/clk_counters.sh $TAG --no-variants || exit $?
bash tools/gpu_tcc_bytes.sh $TAG || exit $?
fi
echo done
