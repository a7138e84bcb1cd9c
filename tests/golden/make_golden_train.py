"""Generate the TRAINING-LOSS golden fixtures by running the REFERENCE's own ``compute_loss``.

Run in the build container only (it needs /root/reference, absent on the GPU box):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_train.py

``/root/reference/train_coco_pose_estimation.py`` is imported with empty stub modules for the
absent cv2 / pycocotools / chainer (and for the reference's own ``entity`` / ``models`` /
``coco_data_loader``, which only its ``__main__`` block uses), and its UNMODIFIED
``compute_loss`` (train_coco_pose_estimation.py:41-73) runs on:

* ``pafs_ys`` / ``heatmaps_ys``: the six stage outputs of the reference's own CocoPoseNet
  (``tests/golden/forward/posenet_<case>.npz``, made by make_golden_forward.py from
  models/CocoPoseNet.py with seed-0 random weights and the fixture's seeded input), wrapped in a
  Variable stand-in (``.data``, ``.shape``);
* ``pafs_t`` / ``heatmaps_t`` / ``ignore_mask``: seeded targets at the network map size and a
  seeded boolean ignore mask (about 20 % of pixels) -- the shapes the reference's data loader
  feeds (coco_data_loader.py; the maps are at insize/8, so the ``F.resize_images`` branch at
  :57-61 is not taken, as in training).

Chainer stand-ins on this path (Chainer is absent, so these are restatements: parity unpinned at
these two ops only): ``F.mean_squared_error`` = Chainer's ``MeanSquaredError.forward_cpu``
(``diff = x0 - x1`` in f32, ``diff.ravel().dot(diff) / diff.size`` cast to f32) and
``cuda.to_cpu`` = identity.  The mask replacement (:63-64: masked target pixels take the
prediction's value, so they contribute 0) and the per-stage loop are the reference's own code.

Output: tests/golden/train/loss_<case>.npz (data only, no code).
"""
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
CASES = ("posenet_2x48x48", "posenet_1x64x80")


class Variable(object):
    """chainer.Variable stand-in: what compute_loss touches (.data, .shape, + for the total)."""

    def __init__(self, data):
        self.data = data
        self.shape = data.shape

    def __add__(self, other):
        o = other.data if isinstance(other, Variable) else other
        return Variable(np.asarray(self.data + o, dtype=np.float32))

    __radd__ = __add__


def mean_squared_error(x0, x1):
    """Chainer MeanSquaredError.forward_cpu: f32 diff, ravel, dot / size, f32 result."""
    a = x0.data if isinstance(x0, Variable) else x0
    b = x1.data if isinstance(x1, Variable) else x1
    diff = (a - b).ravel()
    return Variable(np.array(diff.dot(diff) / diff.size, dtype=diff.dtype))


def install_stubs():
    names = ["cv2", "pycocotools", "pycocotools.coco", "chainer", "chainer.cuda", "chainer.training",
             "chainer.training.extensions", "chainer.reporter", "chainer.function", "chainer.serializers",
             "chainer.optimizers", "chainer.functions", "entity", "coco_data_loader", "models",
             "models.CocoPoseNet"]
    for n in names:
        sys.modules[n] = types.ModuleType(n)
    m = sys.modules
    m["pycocotools.coco"].COCO = object
    ch = m["chainer"]
    for sub in ("cuda", "training", "reporter", "function", "serializers", "optimizers", "functions"):
        setattr(ch, sub, m["chainer." + sub])
    ch.cuda.to_cpu = lambda a: a
    ch.cuda.get_array_module = lambda *a: np
    ch.training.StandardUpdater = object
    ch.training.extensions = m["chainer.training.extensions"]
    ch.training.extensions.Evaluator = object
    ch.functions.mean_squared_error = mean_squared_error

    def resize_images(*a, **k):
        raise AssertionError("targets are at the network map size: F.resize_images is not on this path")

    ch.functions.resize_images = resize_images
    m["entity"].params = {"archs": {}}
    m["coco_data_loader"].CocoDataLoader = object
    m["models"].CocoPoseNet = m["models.CocoPoseNet"]
    sys.path.insert(0, REF)


def targets(case, paf_shape, heat_shape):
    seed = sum(ord(ch) for ch in case)
    rng = np.random.default_rng(seed)
    pafs_t = rng.uniform(-1, 1, paf_shape).astype(np.float32)
    heat_t = rng.uniform(0, 1, heat_shape).astype(np.float32)
    ignore = rng.random((paf_shape[0],) + paf_shape[2:]) < 0.2
    return seed, pafs_t, heat_t, ignore


def main():
    install_stubs()
    import importlib
    train = importlib.import_module("train_coco_pose_estimation")
    for case in CASES:
        d = dict(np.load(os.path.join(HERE, "forward", case + ".npz")))
        pys = [Variable(p) for p in d["paf_stages"]]
        hys = [Variable(h) for h in d["heat_stages"]]
        seed, pt, ht, ig = targets(case, d["paf_stages"].shape[1:], d["heat_stages"].shape[1:])
        total, paf_log, heat_log = train.compute_loss(None, pys, hys, pt, ht, ig)
        out = os.path.join(HERE, "train", "loss_%s.npz" % case)
        np.savez(out, target_seed=np.int64(seed), pafs_t=pt, heatmaps_t=ht, ignore_mask=ig.astype(np.uint8),
                 paf_loss=np.array(paf_log, np.float64), heat_loss=np.array(heat_log, np.float64),
                 total_loss=np.float64(total.data))
        print(case, "paf", np.array(paf_log), "heat", np.array(heat_log), "total", float(total.data))


if __name__ == "__main__":
    main()
