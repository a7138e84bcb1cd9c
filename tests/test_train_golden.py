"""f4 (training step) pinned to the reference: tests/golden/train/ holds the per-stage losses of
the reference's own compute_loss (train_coco_pose_estimation.py:41-73, run unmodified by
tests/golden/make_golden_train.py) on the six stage outputs of the reference's own CocoPoseNet
(tests/golden/forward/).  Here the oracle restatement must reproduce them bit for bit; the GPU
training step is compared with them in tests/test_gpu_train.py."""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import train_loss

CASES = ("posenet_2x48x48", "posenet_1x64x80")


def load_train_case(case):
    g = dict(np.load(os.path.join(GOLDEN, "train", "loss_%s.npz" % case)))
    f = dict(np.load(os.path.join(GOLDEN, "forward", case + ".npz")))
    return g, f


@pytest.mark.parametrize("case", CASES)
def test_oracle_compute_loss_is_the_reference(case):
    g, f = load_train_case(case)
    paf, heat = train_loss.compute_loss(f["paf_stages"], f["heat_stages"], g["pafs_t"], g["heatmaps_t"],
                                        g["ignore_mask"])
    assert np.array_equal(np.array(paf), g["paf_loss"]) and np.array_equal(np.array(heat), g["heat_loss"])
    assert 0.05 < g["ignore_mask"].mean() < 0.35  # the mask is live: masked pixels are excluded


def test_mask_replacement_changes_the_loss():
    """The mask matters (a no-op mask would make the golden insensitive to :63-64)."""
    g, f = load_train_case(CASES[0])
    paf, _ = train_loss.compute_loss(f["paf_stages"], f["heat_stages"], g["pafs_t"], g["heatmaps_t"],
                                     np.zeros_like(g["ignore_mask"]))
    assert not np.array_equal(np.array(paf), g["paf_loss"])
