#!/bin/bash
# Submit one gpurun call, re-submitting ONLY while the pool reports no free box / slot or an
# infrastructure event (nothing ran, nothing charged); any run of the command itself ends it.
#   tools/gpurun_when_free.sh OUTFILE TIMEOUT 'command'
OUT=$1; TO=$2; CMD=$3
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout $TO -- "$CMD" > $OUT 2>&1
  rc=$?
  if grep -q "no free box\|slot(s) on this pod are busy\|backing off\|stopped responding while being prepared\|taken away by the GPU service" $OUT && ! grep -q "^\[gpurun\] merged" $OUT; then
    sleep 150
    continue
  fi
  exit $rc
done
exit 3
