"""Power-limit probe: the same staged batch with random weights vs all-zero weights (MFMA operands
all zero -> far less switching energy); per-class ms from the bench's HIP-event profile.
usage: python tools/power_probe.py [rounds]"""
import importlib
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
PKG = "chainer_realtime_multi-person_pose_estimation_amd"
L = importlib.import_module(PKG + "._lib")
W = importlib.import_module(PKG + ".weights")

B = 38
lim = L.OpLimits()
lim.max_batch = B
ctx = L.Context(0, None, lim)
rw = W.random_weights(0)
zw = {k: (np.zeros_like(a), np.zeros_like(b)) for k, (a, b) in rw.items()}
frames = np.random.default_rng(1).integers(0, 256, (B, 368, 368, 3), dtype=np.uint8)
ctx.stage_frames(frames)
for r in range(int(sys.argv[1]) if len(sys.argv) > 1 else 2):
    for name, w in (("random", rw), ("zero", zw)):
        ctx.set_weights(w)
        for _ in range(3):
            ctx.run_staged()
        ctx.synchronize()
        ctx.profile_classes(list(ctx.PROFILE_CLASSES))
        ctx.profile(True)
        ctx.profile_reset()
        for _ in range(5):
            ctx.run_staged()
        ctx.synchronize()
        p = ctx.profile_read()
        ctx.profile(False)
        print(r, name, {k: round(v[0] / 5, 3) for k, v in p.items()}, flush=True)
