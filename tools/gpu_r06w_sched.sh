# Scheduler A/B, second set: post-RA scheduler off for the 7x7 (m16iinp) and the 3x3 conv_m16r
# (rnopost), AMDGPU register-pressure trackers for conv_m16r (rtr); 5 interleaved rounds.
set -o pipefail
O=gpurun_out/r06w; mkdir -p $O
timeout -k 10 600 python3 -u tools/ab_lib.py 5 base m16iinp rnopost rtr > $O/ab_headline.log 2>&1
