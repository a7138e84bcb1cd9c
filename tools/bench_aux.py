"""Measurements of the SURVEY §8 f3 / f4 rows (not the headline; bench.py is): one JSON line each.

  python tools/bench_aux.py [--crops 12] [--train-batch 10] [--iters 5] [--no-cpu]

f3: FaceNet / HandNet detectors on random-weight crops of demo-like sizes: one op_cpm_detect per
    crop (the reference's per-person calls, demo.py:38-56) vs one op_cpm_detect_batch; effective
    TF/s = the 368x368 CPM forward's algorithmic FLOPs x crops / wall time (f32-accurate bf16x3
    arithmetic; peak 2500/3 TF/s), next to the oracle (oracle/cpm.py, NumPy) on the host cores.
f4: one training iteration (op_train_step: forward + compute_loss + backward + Adam, every layer
    trainable) at batch B, 368x368, exact f32 on v_mfma_f32_32x32x2_f32 (peak 157.3 TF/s);
    algorithmic FLOPs = forward + input gradients (all but conv1_1) + weight gradients.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
PKG = "chainer_realtime_multi-person_pose_estimation_amd"


def layer_res(name, size=368):
    for p, d in (("conv1_", 1), ("conv2_", 2), ("conv3_", 4)):
        if name.startswith(p):
            return size // d
    return size // 8


def cpm_flops(table, size=368):
    return sum(2.0 * ci * co * k * k * layer_res(n, size) ** 2 for n, ci, co, k in table)


def bench_cpm(L, W, arch, n_crops, reps, cpu):
    from importlib import import_module
    thr = {"facenet": 0.1, "handnet": 0.1}[arch]
    c = L.CpmContext(arch, 0)
    w = W.random_weights(seed=3, arch=arch)
    c.set_weights(w)
    rng = np.random.default_rng(0)
    sizes = [(int(s), int(s * r)) for s, r in zip(rng.integers(90, 260, n_crops), rng.uniform(0.8, 1.2, n_crops))]
    crops = [rng.integers(0, 256, (h, ww, 3), dtype=np.uint8) for h, ww in sizes]
    flips = [arch == "handnet" and i % 2 == 1 for i in range(n_crops)]
    for im, f in zip(crops, flips):  # warm-up: every single-call geometry
        c.detect(im, thr, flip_maps=f)
    t0 = time.perf_counter()
    for _ in range(reps):
        for im, f in zip(crops, flips):
            c.detect(im, thr, flip_maps=f)
    t_single = (time.perf_counter() - t0) / reps
    c.detect_batch(crops, thr, flip_maps=flips)
    t0 = time.perf_counter()
    for _ in range(reps):
        c.detect_batch(crops, thr, flip_maps=flips)
    t_batch = (time.perf_counter() - t0) / reps
    fl = cpm_flops(c.table)
    out = {"row": "f3 %s detector" % arch, "crops": n_crops, "crop_sizes": sizes,
           "ms_per_crop_single_calls": round(t_single / n_crops * 1e3, 3),
           "ms_per_crop_batched": round(t_batch / n_crops * 1e3, 3),
           "crops_per_s_batched": round(n_crops / t_batch, 1),
           "gflop_per_crop": round(fl / 1e9, 2),
           "effective_tflops_batched": round(fl * n_crops / t_batch / 1e12, 1),
           "peak_tflops": round(2500.0 / 3, 1), "dtype": "bf16x3 (f32-accurate)"}
    if cpu:
        OC = import_module("oracle.cpm")
        t0 = time.perf_counter()
        OC.detect(w, arch, crops[0], hand_type="left" if flips[0] else "right")
        dt = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": round(1.0 / dt, 3), "unit": "crops/s", "kind": "port",
                               "sample": "1 crop %dx%d: oracle/cpm.py (NumPy im2col+sgemm forward, resize, "
                                         "gaussian, peaks)" % sizes[0]}
    c.close()
    return out


def bench_train(L, W, n, iters):
    T = __import__(PKG + ".train", fromlist=["train"])
    ctx = L.TrainContext(n, 368, 368, 0)
    ctx.set_weights(W.random_weights(seed=0))
    ctx.set_hyper(1e-4)
    rng = np.random.default_rng(0)
    imgs, paf, heat, ign = T.synthetic_batch(rng, n, 368, 368)
    x = T.preprocess(imgs)
    ctx.step(x, paf, heat, ign)  # warm-up
    t0 = time.perf_counter()
    for _ in range(iters):
        ctx.step(x, paf, heat, ign)
    dt = (time.perf_counter() - t0) / iters
    fwd = L.forward_flops(368, 368) * n
    c11 = 2.0 * 3 * 64 * 9 * 368 * 368 * n  # conv1_1 has no input gradient
    fl = fwd + (fwd - c11) + fwd
    ctx.close()
    return {"row": "f4 training iteration", "batch": n, "size": "368x368", "ms_per_iteration": round(dt * 1e3, 2),
            "frames_per_s": round(n / dt, 1), "tflop_per_iteration": round(fl / 1e12, 2),
            "effective_tflops": round(fl / dt / 1e12, 1), "peak_tflops": 157.3,
            "dtype": "f32 (v_mfma_f32_32x32x2_f32 + VALU weight gradients)", "layers": "all trainable"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--crops", type=int, default=12)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--train-batch", type=int, default=10)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--only", choices=["cpm", "train"], default=None)
    args = ap.parse_args()
    from importlib import import_module
    L = import_module(PKG + "._lib")
    W = import_module(PKG + ".weights")
    if args.only in (None, "cpm"):
        for arch in ("facenet", "handnet"):
            print(json.dumps(bench_cpm(L, W, arch, args.crops, args.reps, not args.no_cpu)), flush=True)
    if args.only in (None, "train"):
        print(json.dumps(bench_train(L, W, args.train_batch, args.iters)), flush=True)


if __name__ == "__main__":
    main()
