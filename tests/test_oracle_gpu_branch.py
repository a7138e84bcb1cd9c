"""The oracle's restatement of the reference's GPU-branch peaks (pose_detector.py:38-44, 111-132),
checked on the CPU: the kernel against its formula, the zero-padded filter against SciPy's
correlate (mode 'constant'), and the >= NMS against the strict CPU branch on a plateau.

Parity unpinned against the reference itself: its GPU branch needs CUDA + cuDNN (absent here), so no
fixture of it exists; these checks pin the restatement to the reference's formulas."""
import numpy as np
import pytest
from scipy import ndimage

from oracle import postproc as P


def test_kernel_is_the_reference_formula():
    k = P.create_gaussian_kernel(P.PARAMS["gaussian_sigma"], P.PARAMS["ksize"])
    assert k.dtype == np.float32 and k.shape == (17, 17)
    s = 2.5
    d2 = (np.arange(17)[None, :] - 8) ** 2 + (np.arange(17)[:, None] - 8) ** 2
    assert np.array_equal(k, (np.exp(-0.5 * d2 / s ** 2) / (2 * np.pi * s ** 2)).astype("f"))
    assert abs(float(k.astype(np.float64).sum()) - 1.0) > 1e-4  # not normalised (truncated at 3.2 sigma)
    assert np.array_equal(k, k.T) and np.array_equal(k, k[::-1])


@pytest.mark.parametrize("shape", [(3, 40, 56), (2, 17, 23), (1, 9, 9)])
def test_filter_is_zero_padded_correlation(shape):
    rng = np.random.default_rng(shape[1])
    h = rng.random(shape, dtype=np.float32)
    got = P.gpu_branch_filter(h)
    k = P.create_gaussian_kernel(2.5, 17).astype(np.float64)
    want = np.stack([ndimage.correlate(h[j].astype(np.float64), k, mode="constant", cval=0.0) for j in range(shape[0])])
    assert np.allclose(got, want.astype(np.float32), rtol=2e-7, atol=1e-9)


def test_ge_nms_keeps_plateau_peaks_the_cpu_branch_drops():
    """Two equal neighbouring maxima: the GPU branch (>=) reports both, the CPU branch (>) neither."""
    heat = np.zeros((19, 40, 40), np.float32)
    heat[0, 20, 20] = heat[0, 20, 21] = 5.0  # symmetric pair: equal filtered values at (20,20), (20,21)
    g = P.compute_peaks_gpu_branch(heat)
    assert g.shape == (2, 5)
    assert [tuple(r[:3]) for r in g] == [(0.0, 20.0, 20.0), (0.0, 21.0, 20.0)]
    assert np.array_equal(g[:, 4], [0, 1]) and g[0, 3] == g[1, 3]
    c = P.compute_peaks_from_heatmaps(heat)
    assert len(c) == 0


def test_peak_rows_order_and_ids():
    rng = np.random.default_rng(5)
    heat = np.zeros((19, 48, 64), np.float32)
    for j in range(18):
        for _ in range(3):
            heat[j, rng.integers(0, 48), rng.integers(0, 64)] = rng.uniform(1, 3)
    g = P.compute_peaks_gpu_branch(heat)
    assert g.dtype == np.float64 and g.shape[1] == 5
    key = g[:, 0] * 1e6 + g[:, 2] * 1e3 + g[:, 1]  # (joint, y, x) order of np.nonzero
    assert np.all(np.diff(key) > 0)
    assert np.array_equal(g[:, 4], np.arange(len(g)))
    assert np.all(g[:, 3] > 0.05)


def _separable_like_the_device(h, sigma=2.5, ksize=17):
    """The device's arithmetic for the GPU branch (postproc.hip heat_fused<.., G>): the 1-D factor
    g(d) = exp(-d^2 / 2 s^2) / sqrt(2 pi s^2) (host_pack.hpp gpu_branch_taps), a vertical then a
    horizontal pass in f64 over zero-padded f32 maps, rounded to f32 after each pass."""
    r = ksize // 2
    d = np.arange(-r, r + 1, dtype=np.float64)
    g = np.exp(-0.5 * d * d / (sigma * sigma)) / np.sqrt(2.0 * np.pi * sigma * sigma)
    J, H, W = h.shape
    p = np.zeros((J, H + 2 * r, W), np.float64)
    p[:, r:r + H] = h
    v = sum(g[k] * p[:, k:k + H] for k in range(ksize)).astype(np.float32)
    q = np.zeros((J, H, W + 2 * r), np.float64)
    q[:, :, r:r + W] = v
    return sum(g[k] * q[:, :, k:k + W] for k in range(ksize)).astype(np.float32)


def test_device_arithmetic_within_rounding_of_the_restatement():
    """The separable f64 / f32-between-passes form the device runs stays within a few f32 ulp of the
    oracle's exact 2-D sum on the golden maps (upsampled like the single-scale path)."""
    from conftest import golden_cases, load_golden
    from oracle import cvresize
    for case in golden_cases():
        d = load_golden(case)
        mw, mh = cvresize.compute_optimal_size(int(d["orig_h"]), int(d["orig_w"]), 320)
        heat = P.resize_images(d["heat_low"], mh, mw)[:-1]
        a = P.gpu_branch_filter(heat).astype(np.float64)
        b = _separable_like_the_device(heat).astype(np.float64)
        scale = max(float(np.abs(a).max()), 1e-30)
        assert float(np.abs(a - b).max()) <= 3e-7 * scale, case
        # ... and finds the same peaks
        want = P.compute_peaks_gpu_branch(np.concatenate([heat, heat[:1]]))
        nb = np.zeros((4,) + b.shape, np.float32)
        bf = b.astype(np.float32)
        nb[0][:, 1:, :] = bf[:, :-1, :]
        nb[1][:, :-1, :] = bf[:, 1:, :]
        nb[2][:, :, 1:] = bf[:, :, :-1]
        nb[3][:, :, :-1] = bf[:, :, 1:]
        got = np.argwhere((bf > np.float32(0.05)) & np.all(bf[None] >= nb, axis=0))
        assert np.array_equal(got[:, [0, 2, 1]].astype(np.float64), want[:, :3].reshape(-1, 3)), case
