"""Interleaved A/B of conv kernel families in ONE process (the bench workload, staged frames,
batch 42): per round and family, wall ms of 5 steps and the per-class HIP-event ms of 2 more.
usage: python tools/ab_algo.py ROUNDS ALGO ALGO ..."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = "chainer_realtime_multi-person_pose_estimation_amd"
import importlib  # noqa: E402

L = importlib.import_module(PKG + "._lib")
Wm = importlib.import_module(PKG + ".weights")

rounds = int(sys.argv[1])
algos = [int(a) for a in sys.argv[2:]]
B = 42
limits = L.OpLimits()
limits.max_batch = B
ctx = L.Context(0, None, limits)
ctx.set_weights(Wm.random_weights(seed=0))
ctx.stage_frames(np.random.default_rng(1).integers(0, 256, (B, 368, 368, 3), dtype=np.uint8))
res = {a: {"wall": [], "cls": []} for a in algos}
for a in algos:  # warm every family once
    ctx.set_conv_algo(a)
    ctx.run_staged()
    ctx.synchronize()
for r in range(rounds):
    for a in algos:
        ctx.set_conv_algo(a)
        ctx.profile(False)
        ctx.run_staged()
        ctx.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            ctx.run_staged()
        ctx.synchronize()
        res[a]["wall"].append((time.perf_counter() - t0) * 1e3 / 5)
        ctx.profile_classes(list(ctx.PROFILE_CLASSES))
        ctx.profile(True)
        ctx.profile_reset()
        for _ in range(2):
            ctx.run_staged()
        ctx.synchronize()
        p = ctx.profile_read()
        ctx.profile(False)
        res[a]["cls"].append({k: v[0] / 2 for k, v in p.items()})
    print("round", r, {a: round(res[a]["wall"][-1], 3) for a in algos}, flush=True)
for a in algos:
    w = np.array(res[a]["wall"])
    cls = {k: np.median([c[k] for c in res[a]["cls"]]) for k in res[a]["cls"][0]}
    print("algo %d: wall ms/step median %.3f min %.3f | %s" % (
        a, np.median(w), w.min(), " ".join("%s %.3f" % (k, v) for k, v in cls.items())))
ctx.close()
