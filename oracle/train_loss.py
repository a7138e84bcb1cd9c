"""ORACLE — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

NumPy restatement of ``compute_loss`` (train_coco_pose_estimation.py:41-73) for targets at the
network map size (the training case: the ``F.resize_images`` branch at :57-61 is not taken):
per stage, masked target pixels take the prediction's value (:63-64), then
``F.mean_squared_error`` as Chainer's ``MeanSquaredError.forward_cpu`` (f32 diff, ravel,
``dot / size``, f32).  Pinned by tests/golden/train/ (the reference's own compute_loss, run by
tests/golden/make_golden_train.py).
"""
import numpy as np


def _mse(y, t):
    diff = (y - t).ravel()
    return np.float32(diff.dot(diff) / diff.size)


def compute_loss(pafs_ys, heatmaps_ys, pafs_t, heatmaps_t, ignore_mask):
    """(paf_loss[6], heat_loss[6]) as float64 lists of the f32 per-stage losses."""
    m = np.asarray(ignore_mask).astype(bool)
    paf_m = np.repeat(m[:, None], pafs_t.shape[1], axis=1)
    heat_m = np.repeat(m[:, None], heatmaps_t.shape[1], axis=1)
    paf_log, heat_log = [], []
    for py, hy in zip(pafs_ys, heatmaps_ys):
        tp = np.where(paf_m, py, pafs_t).astype(np.float32)
        th = np.where(heat_m, hy, heatmaps_t).astype(np.float32)
        paf_log.append(float(_mse(py, tp)))
        heat_log.append(float(_mse(hy, th)))
    return paf_log, heat_log
