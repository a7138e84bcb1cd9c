"""Writes the averaged detect_precise maps of one seeded 1280x720 frame to <out>.npz (GPU).
Run once with OP_CUBIC_FLAT=1 (flat-index first map resize) and once without, then compare:
  python tools/cubic_ab_maps.py a.npz; OP_CUBIC_FLAT=1 python tools/cubic_ab_maps.py b.npz
  python tools/cubic_ab_maps.py --compare a.npz b.npz
"""
import importlib
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
PKG = "chainer_realtime_multi-person_pose_estimation_amd"

if sys.argv[1] == "--compare":
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    same = all(np.array_equal(a[k], b[k]) for k in ("pafs", "heat"))
    print("maps bit-identical:", same, "max|d| paf %.3g heat %.3g" % (
        float(np.abs(a["pafs"] - b["pafs"]).max()), float(np.abs(a["heat"] - b["heat"]).max())))
    sys.exit(0 if same else 1)
lib = importlib.import_module(PKG + "._lib")
W = importlib.import_module(PKG + ".weights").random_weights(seed=0)
rng = np.random.default_rng(7)
img = np.clip(128 + 40 * rng.standard_normal((720, 1280, 3)), 0, 255).astype(np.uint8)
lim = lib.OpLimits()
lim.max_peaks_per_joint = 2048
c = lib.Context(0, None, lim)
c.set_weights(W)
c.set_batch_invariant(True)
try:
    _, _, _, pafs, heat = c.detect_precise(img, return_maps=True)
except IndexError as e:
    pafs, heat = e.maps
np.savez(sys.argv[1], pafs=pafs, heat=heat)
print("wrote", sys.argv[1], pafs.shape, heat.shape)
