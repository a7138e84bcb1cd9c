"""Training host side, CPU: preprocess (train_coco_pose_estimation.py:80-86), the
synthetic stand-in batches, and that the library exports the training ABI."""
import numpy as np

from conftest import pkg_module


def test_preprocess_matches_reference_formula():
    T = pkg_module("train")
    imgs = np.random.default_rng(0).integers(0, 256, (2, 16, 24, 3), dtype=np.uint8)
    x = imgs.astype("f")
    x /= 255
    x -= 0.5
    ref = x.transpose(0, 3, 1, 2)
    got = T.preprocess(imgs)
    assert got.dtype == np.float32 and got.shape == (2, 3, 16, 24) and np.array_equal(got, ref)


def test_synthetic_batch_shapes_and_ranges():
    T = pkg_module("train")
    imgs, paf, heat, ign = T.synthetic_batch(np.random.default_rng(1), 2, 64, 48)
    assert imgs.shape == (2, 64, 48, 3) and paf.shape == (2, 38, 8, 6) and heat.shape == (2, 19, 8, 6)
    assert ign.shape == (2, 8, 6) and ign.dtype == np.uint8
    assert heat.min() >= 0 and heat.max() <= 1 + 1e-6 and np.abs(paf).max() <= 1 + 1e-5
    assert np.allclose(heat[:, 18], 1 - heat[:, :18].max(axis=1))
    assert set(T.GRAD_SCALED) >= set(T.VGG_FROZEN) and len(T.GRAD_SCALED) == 12
