#!/bin/bash
# One parameterised GPU-box runner (replaces round 4's single-use gpu_r04*.sh launchers):
#   tools/gpu_run.sh TAG STEP [STEP ...]
# Steps run in order, each under its own time limit; the first failure ends the call (no GPU step
# runs after a fault, an abort or a time limit).  Output: gpurun_out/run_TAG/.
#   smoke              __graft_entry__.smoke()
#   suite[:EXPR]       the GPU test suite (pytest -m gpu), optionally -k EXPR
#   file:PATH[:EXPR]   one test file (-m gpu), optionally -k EXPR
#   bench[:ARGS]       one bench line (ARGS: bench.py arguments, commas for spaces)
#   lines              the default bench line (with its side lines) + --no-side-lines variants off
#   c4prof             rocprofv3 kernel-trace stats of the C4 line
#   evidence           tools/gpu_evidence.sh (kernel stats, FETCH/WRITE, SQ, clock passes)
#   tcc                tools/gpu_tcc_bytes.sh (fabric reads by request size)
#   prof:NAME[:ARGS]   tools/profile.sh NAME ARGS (kernel stats + FETCH/WRITE passes of one bench line,
#                      e.g. prof:r06a_c5_m4_b64:--frame,720x1280 -> gpurun_out/prof_NAME)
#   ablib:ARGS         tools/ab_lib.py ARGS (interleaved A/B of library variants; commas for spaces)
#   abenv:TAG:A:B[:N]  tools/gpu_ab_env.sh (interleaved A/B of env settings on the default bench)
#   abb1:TAG:A:B[:N]   tools/gpu_ab_b1.sh (the same on the one-frame line)
set -o pipefail
TAG=$1; shift
O=$GRAFT_REPO_ROOT/gpurun_out/run_$TAG; mkdir -p $O
cd $GRAFT_REPO_ROOT
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
n=0
for step in "$@"; do
  n=$((n + 1))
  kind=${step%%:*}; arg=${step#*:}; [ "$arg" = "$step" ] && arg=""
  log=$O/$(printf %02d $n)_$kind.log
  echo "[$(date +%T)] step $n: $step -> $log"
  case $kind in
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $log 2>&1 ;;
    suite) if [ -n "$arg" ]; then timeout -k 10 900 $PYT tests -m gpu -k "$arg" > $log 2>&1
           else timeout -k 10 900 $PYT tests -m gpu > $log 2>&1; fi ;;
    file) f=${arg%%:*}; k=${arg#*:}; [ "$k" = "$arg" ] && k=""
          if [ -n "$k" ]; then timeout -k 10 900 $PYT $f -m gpu -k "$k" > $log 2>&1
          else timeout -k 10 900 $PYT $f -m gpu > $log 2>&1; fi ;;
    bench) timeout -k 10 600 python -u bench.py ${arg//,/ } > $log 2>&1 ;;
    lines) timeout -k 10 600 python -u bench.py > $log 2>&1 ;;
    c4prof) (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
             -d $O/c4prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --precise --frame 720x1280 --steps 3 --warmup 1 \
             --no-variants --no-profile) > $log 2>&1 ;;
    evidence) bash tools/gpu_evidence.sh $TAG > $log 2>&1 ;;
    tcc) bash tools/gpu_tcc_bytes.sh $TAG > $log 2>&1 ;;
    prof) nm=${arg%%:*}; pa=${arg#*:}; [ "$pa" = "$arg" ] && pa=""
          bash tools/profile.sh $nm ${pa//,/ } > $log 2>&1 ;;
    ablib) timeout -k 10 1100 python3 -u tools/ab_lib.py ${arg//,/ } > $log 2>&1 ;;
    abenv) IFS=: read -r t a b r <<< "$arg"; bash tools/gpu_ab_env.sh $t "$a" "$b" ${r:-2} > $log 2>&1 ;;
    abb1) IFS=: read -r t a b r <<< "$arg"; bash tools/gpu_ab_b1.sh $t "$a" "$b" ${r:-3} > $log 2>&1 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  rc=$?
  echo "[$(date +%T)] step $n rc=$rc"; tail -3 $log
  [ $rc -ne 0 ] && exit $rc
done
echo done
