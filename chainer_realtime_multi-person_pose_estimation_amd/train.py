"""Training of CocoPoseNet on the MI355X path: train_coco_pose_estimation.py.

``Updater`` mirrors the reference's ``Updater.update_core`` (:90-126) on one device: every
iteration runs ``preprocess`` (:76-82, host), then forward + ``compute_loss`` (:41-73) + backward +
``GradientScaling(1/4)`` on conv1_1 .. conv4_4_CPM (:25-38, :213-217) + ``optimizers.Adam`` (:210)
in one call into the HIP library (op_train_step, exact f32).  The schedule is the reference's: the
VGG layers conv1_1 .. conv4_2 start frozen (:219-225) and are enabled at iteration 2000 (:95-100);
alpha 1e-4, then 1e-5 from 100k and 1e-6 from 200k iterations (:102-105).  All of it (Adam's
hyperparameters, the hook's layers and scale, the frozen layers, the re-enable and the alpha at
each schedule edge) is pinned to the reference's own script run under recording stubs
(tests/golden/make_golden_train_host.py -> tests/golden/train/host_schedule.json).

The COCO data pipeline (coco_data_loader.py, pycocotools, getData.sh) needs the dataset and the
network: ``synthetic_batch`` stands in with seeded images and COCO-like maps of random skeletons
(Gaussian heat peaks + unit-vector PAFs on the limbs, the reference's label formulas restated).

    python -m chainer_realtime_multi-person_pose_estimation_amd.train --batchsize 4 --iteration 10
"""
import argparse
import json
import os
import sys
import time

import numpy as np

from . import _lib
from . import weights as _weights
from .constants import params

VGG_FROZEN = ["conv1_1", "conv1_2", "conv2_1", "conv2_2", "conv3_1", "conv3_2", "conv3_3", "conv3_4", "conv4_1",
              "conv4_2"]
GRAD_SCALED = VGG_FROZEN + ["conv4_3_CPM", "conv4_4_CPM"]


def preprocess(imgs):
    """train_coco_pose_estimation.py:76-82: (n, h, w, 3) uint8 BGR -> (n, 3, h, w) f32, x/255 - 0.5."""
    x = np.asarray(imgs).astype("f")
    x /= 255
    x -= 0.5
    return np.ascontiguousarray(x.transpose(0, 3, 1, 2))


class GradientScaling(object):
    """train_coco_pose_estimation.py:25-38: multiplies the gradients of ``layer_names`` by ``scale``
    (in f32, ``grad *= scale``) before the optimizer's update.  Registered with
    ``Updater.add_hook`` (the reference's ``optimizer.add_hook``, :213-217); on the device the scale
    is applied inside op_train_step (op_train_set_grad_scale)."""

    name = "GradientScaling"

    def __init__(self, layer_names, scale):
        self.layer_names = layer_names
        self.scale = scale

    def __call__(self, updater):
        for layer_name in self.layer_names:
            updater.ctx.set_grad_scale(updater.names.index(layer_name), self.scale)


def alpha_at(iteration, alpha):
    """update_core's learning-rate schedule (:102-105): the optimizer's alpha before the update of
    ``iteration``, given the alpha in force before it (the reference only ever lowers it)."""
    if 100000 <= iteration < 200000:
        return 1e-5
    if 200000 <= iteration:
        return 1e-6
    return alpha


class Updater(object):
    """One device, one batch shape (n, h, w).  ``update(batch)`` = Updater.update_core (:90-126).

    Set up like the reference's ``__main__`` (:208-225) for ``posenet``: ``optimizers.Adam(alpha=1e-4,
    beta1=0.9, beta2=0.999, eps=1e-8)``, ``GradientScaling(conv1_1 .. conv4_4_CPM, 1/4)`` and, unless
    resuming, conv1_1 .. conv4_2 frozen (re-enabled at iteration 2000).  ``ctx`` (tests) replaces the
    device context: anything with set_weights / set_hyper / enable / set_grad_scale / step / get."""

    def __init__(self, n, h=368, w=368, model=None, device=0, alpha=1e-4, beta1=0.9, beta2=0.999, eps=1e-8,
                 resume=False, ctx=None):
        self.ctx = ctx if ctx is not None else _lib.TrainContext(n, h, w, device)
        self.names = [t[0] for t in self.ctx.table]
        self.iteration = 0
        self.alpha, self.beta1, self.beta2, self.eps = alpha, beta1, beta2, eps
        self.hooks = []
        self.ctx.set_weights(model if model is not None else _weights.random_weights(0))
        self.ctx.set_hyper(alpha, beta1, beta2, eps)
        self.add_hook(GradientScaling(GRAD_SCALED, 1 / 4))
        if not resume:
            for name in VGG_FROZEN:
                self.disable_update(name)

    def add_hook(self, hook):
        self.hooks.append(hook)
        hook(self)

    def enable_update(self, name):
        self.ctx.enable(self.names.index(name), True)

    def disable_update(self, name):
        self.ctx.enable(self.names.index(name), False)

    def update(self, batch):
        """batch = (imgs (n,h,w,3) u8, pafs (n,38,h/8,w/8), heatmaps (n,19,h/8,w/8), ignore_mask (n,h/8,w/8)).
        Returns (loss, paf_loss_log, heatmap_loss_log) as compute_loss does."""
        if self.iteration == 2000:
            for name in VGG_FROZEN:
                self.enable_update(name)
        self.alpha = alpha_at(self.iteration, self.alpha)
        self.ctx.set_hyper(self.alpha, self.beta1, self.beta2, self.eps)
        imgs, pafs, heatmaps, ignore_mask = batch
        losses = self.ctx.step(preprocess(imgs), pafs, heatmaps, ignore_mask)
        self.iteration += 1
        paf_log = [float(v) for v in losses[0::2]]
        heat_log = [float(v) for v in losses[1::2]]
        return sum(paf_log) + sum(heat_log), paf_log, heat_log

    def weights(self):
        return self.ctx.get()

    def grads(self):
        return self.ctx.get(grads=True)


def synthetic_batch(rng, n, h, w, people=3):
    """Seeded stand-in for CocoDataLoader (coco_data_loader.py:216-268 label formulas): heat maps are
    max-combined Gaussians exp(-d^2 / 2 sigma^2) (sigma 7 px at the input scale) with the background
    channel 1 - max, PAFs the unit limb vector within 8 px of the limb (averaged over people)."""
    h8, w8 = h // 8, w // 8
    imgs = rng.integers(0, 256, (n, h, w, 3), dtype=np.uint8)
    heat = np.zeros((n, 19, h8, w8), np.float32)
    paf = np.zeros((n, 38, h8, w8), np.float32)
    yy, xx = np.mgrid[0:h8, 0:w8].astype(np.float32) * 8 + 3.5
    for f in range(n):
        cnt = np.zeros((19, h8, w8), np.float32)
        for _ in range(people):
            c = rng.uniform([0.2 * w, 0.2 * h], [0.8 * w, 0.8 * h])
            joints = c + rng.normal(0, 0.12 * min(h, w), (18, 2))
            for j, (x, y) in enumerate(joints):
                heat[f, j] = np.maximum(heat[f, j], np.exp(-((xx - x) ** 2 + (yy - y) ** 2) / (2 * 7.0 ** 2)))
            for li, (a, b) in enumerate(params["limbs_point"]):
                v = joints[b] - joints[a]
                ln = np.linalg.norm(v)
                if ln < 1e-3:
                    continue
                u = v / ln
                px, py = xx - joints[a][0], yy - joints[a][1]
                along = px * u[0] + py * u[1]
                across = np.abs(px * u[1] - py * u[0])
                m = (along >= 0) & (along <= ln) & (across <= 8.0)
                paf[f, 2 * li][m] += u[0]
                paf[f, 2 * li + 1][m] += u[1]
                cnt[li][m] += 1
        for li in range(19):
            nz = cnt[li] > 0
            paf[f, 2 * li][nz] /= cnt[li][nz]
            paf[f, 2 * li + 1][nz] /= cnt[li][nz]
        heat[f, 18] = 1.0 - heat[f, :18].max(axis=0)
    ignore = (rng.random((n, h8, w8)) < 0.02).astype(np.uint8)
    return imgs, paf, heat, ignore


def main(argv=None):
    ap = argparse.ArgumentParser(description="Train pose estimation (MI355X, synthetic data)")
    ap.add_argument("--arch", "-a", choices=["posenet"], default="posenet")
    ap.add_argument("--batchsize", "-B", type=int, default=10)
    ap.add_argument("--iteration", "-i", type=int, default=10)
    ap.add_argument("--insize", type=int, default=368)
    ap.add_argument("--gpu", "-g", type=int, default=-1, help="HIP device (negative: device 0; no CPU path)")
    ap.add_argument("--initmodel", help="initialise the model from a Chainer npz")
    ap.add_argument("--resume", action="store_true", help="do not freeze the VGG layers")
    ap.add_argument("--out", "-o", default="result/test")
    ap.add_argument("--seed", type=int, default=0)
    args = ap.parse_args(argv)
    model = _weights.load_npz(args.initmodel) if args.initmodel else _weights.random_weights(args.seed)
    up = Updater(args.batchsize, args.insize, args.insize, model=model, device=max(args.gpu, 0), resume=args.resume)
    rng = np.random.default_rng(args.seed)
    os.makedirs(args.out, exist_ok=True)
    log = []
    for it in range(args.iteration):
        batch = synthetic_batch(rng, args.batchsize, args.insize, args.insize)
        t0 = time.perf_counter()
        loss, pl, hl = up.update(batch)
        dt = time.perf_counter() - t0
        log.append({"iteration": up.iteration, "main/loss": loss, "main/paf": sum(pl), "main/heat": sum(hl),
                    "elapsed_s": dt})
        print("iter %d loss %.6f paf %.6f heat %.6f (%.1f ms)" % (up.iteration, loss, sum(pl), sum(hl), dt * 1e3),
              flush=True)
    with open(os.path.join(args.out, "log"), "w") as f:
        json.dump(log, f, indent=1)
    _weights.save_npz(os.path.join(args.out, "model_iter_%d.npz" % up.iteration), up.weights())
    return 0


if __name__ == "__main__":
    sys.exit(main())
