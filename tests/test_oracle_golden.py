"""The CPU oracle against the reference's own outputs (tests/golden/, made by make_golden.py)."""
import numpy as np
import pytest
from scipy.ndimage import gaussian_filter

from conftest import GOLDEN, golden_cases, load_golden
from oracle import postproc as P


@pytest.mark.parametrize("case", golden_cases())
def test_oracle_matches_reference(case):
    d = load_golden(case)
    mh, mw = int(d["map_h"]), int(d["map_w"])
    pafs = P.resize_images(d["paf_low"], mh, mw)
    heat = P.resize_images(d["heat_low"], mh, mw)
    peaks = P.compute_peaks_from_heatmaps(heat)
    assert np.array_equal(np.asarray(peaks).reshape(-1, 5), d["all_peaks"])
    if int(d["status"]) == 1:
        assert len(peaks) == 0
        poses, scores = P.postprocess(d["paf_low"], d["heat_low"], int(d["orig_h"]), int(d["orig_w"]))
        assert poses.shape == (0, 18, 3) and scores.shape == (0,)
        return
    conns = P.compute_connections(pafs, peaks, mw)
    assert np.array_equal(np.concatenate(conns), d["conn"])
    assert np.array_equal(np.cumsum([0] + [len(c) for c in conns]), d["conn_off"])
    if int(d["status"]) == 4:
        with pytest.raises(IndexError):
            P.grouping_key_points(conns, peaks)
        return
    subsets = P.grouping_key_points(conns, peaks)
    assert np.array_equal(subsets, d["subsets"])
    poses, scores = P.postprocess(d["paf_low"], d["heat_low"], int(d["orig_h"]), int(d["orig_w"]))
    assert tuple(np.asarray(poses).shape) == tuple(d["poses_shape"])
    assert np.array_equal(np.asarray(poses, np.float64).reshape(d["poses"].shape), d["poses"])
    assert np.array_equal(scores, d["scores"])


def test_gaussian_bit_exact_vs_scipy():
    g = np.load(GOLDEN + "/gauss_scipy.npz")
    for i in range(len(g["up"])):
        assert np.array_equal(P.gaussian_filter(g["up"][i]), g["g"][i])
        # and against SciPy live, on an odd-sized map with the reflect boundary in play
    rng = np.random.default_rng(3)
    m = rng.standard_normal((37, 53)).astype(np.float32)
    assert np.array_equal(P.gaussian_filter(m), gaussian_filter(m, sigma=2.5))


def test_gaussian_weights_match_scipy():
    from scipy.ndimage._filters import _gaussian_kernel1d
    assert np.array_equal(P.gaussian_weights(2.5), _gaussian_kernel1d(2.5, 0, 10)[::-1])


def test_numpy_dot_and_sum_contract():
    """The line-integral arithmetic the oracle fixes (fma(px,ux, py*uy); pairwise sum) is what
    NumPy does on this host for the reference's np.dot / .sum() calls (pose_detector.py:149-151)."""
    from fractions import Fraction
    rng = np.random.default_rng(1)
    for _ in range(200):
        p = rng.standard_normal((10, 2)).astype(np.float32)
        v = rng.integers(-300, 300, 2).astype(np.float64)
        n = np.linalg.norm(v)
        if n == 0:
            continue
        u = v / n
        d = np.dot(p, u)
        for k in range(10):
            exact = Fraction(float(p[k, 0])) * Fraction(u[0]) + Fraction(float(p[k, 1]) * u[1])
            assert d[k] == float(exact)
        s = ((d[0] + d[1]) + (d[2] + d[3])) + ((d[4] + d[5]) + (d[6] + d[7]))
        assert d.sum() == (s + d[8]) + d[9]


def test_grouping_indexerror_like_reference():
    """pose_detector.py:197 raises IndexError when a connection touches 3 subsets."""
    d = load_golden("grouping_indexerror")
    off = d["conn_off"]
    conns = [d["conn"][off[l]:off[l + 1]] for l in range(19)]
    with pytest.raises(IndexError):
        P.grouping_key_points(conns, d["all_peaks"])
