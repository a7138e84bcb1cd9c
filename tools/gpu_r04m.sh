#!/bin/bash
# Round 4: 7x7 time decomposition probes on the headline (timing-only builds, wrong maps):
# nohalo = the halo loaded for the first chunk only (chunk-boundary drain + halo traffic),
# nopad = the zero padding pair of the odd 49th tap skipped, nobar = no per-tap-pair barrier.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r04m; mkdir -p $O
timeout -k 10 900 python3 -u tools/ab_lib.py 3 base nohalo nopad nobar > $O/ab_probes.log 2>&1 || exit $?
echo done
