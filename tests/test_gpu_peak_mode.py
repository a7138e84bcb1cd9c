"""GPU-branch peak semantics (op_set_peak_mode, include/openpose_hip.h) against the oracle's
restatement of the reference's GPU branch (pose_detector.py:38-44, 111-132; oracle/postproc.py
compute_peaks_gpu_branch).

Parity unpinned against the reference itself (its GPU branch needs CUDA + cuDNN, so no fixture of
it exists).  The device filter is separable f64 with one f32 rounding between the passes; the oracle
is the exact 2-D sum rounded once.  Tolerance: peak sets and poses exact (no peak decision of the
inputs lies within 5e-7 of a tie relative to the map maximum, asserted below), scores within 1e-6
relative."""
import numpy as np
import pytest

from conftest import golden_cases, load_golden, people_image
from oracle import postproc as P

pytestmark = pytest.mark.gpu
SCORE_RTOL = 1e-6


@pytest.fixture(scope="module")
def gctx(lib, rand_weights):
    c = lib.Context(0)
    c.set_weights(rand_weights)
    c.set_peak_mode("gpu", 17)
    yield c
    c.close()


def _decision_margin(heat_low, orig_h, orig_w):
    """Relative room a rounding difference has before one peak decision flips: for a peak, its
    smallest gap to the threshold or a neighbour; for any other pixel, its largest failing gap (all
    of them must flip to make it a peak).  Neighbours outside the map count as 0."""
    from oracle import cvresize
    mw, mh = cvresize.compute_optimal_size(orig_h, orig_w, 320)
    f = P.gpu_branch_filter(P.resize_images(heat_low, mh, mw)[:-1]).astype(np.float64)
    pad = np.pad(f, ((0, 0), (1, 1), (1, 1)))
    g = [f - np.float64(np.float32(0.05))]
    for dy, dx in ((0, 1), (2, 1), (1, 0), (1, 2)):
        g.append(f - pad[:, dy:dy + f.shape[1], dx:dx + f.shape[2]])
    g = np.stack(g)
    peak = (g[0] > 0) & np.all(g[1:] >= 0, axis=0)
    m_peak = np.where(peak, np.abs(g).min(axis=0), np.inf)
    fail = np.where(np.concatenate([(g[0] <= 0)[None], g[1:] < 0]), np.abs(g), 0.0)
    m_non = np.where(~peak, fail.max(axis=0), np.inf)
    return min(float(m_peak.min()), float(m_non.min())) / max(float(f.max()), 1e-30)


@pytest.mark.parametrize("case", golden_cases())
def test_gpu_branch_postprocess_vs_oracle(gctx, case):
    d = load_golden(case)
    oh, ow = int(d["orig_h"]), int(d["orig_w"])
    poses, scores, res = gctx.postprocess(d["paf_low"], d["heat_low"], oh, ow)
    want_p, want_s, dbg = P.postprocess(d["paf_low"], d["heat_low"], oh, ow, return_debug=True, branch="gpu")
    # no decision within ~7 f32 ulp of a tie (the golden maps' closest is 7.5e-7, noise_crowd), where
    # the device's two-pass rounding (~1e-7) could flip it
    assert _decision_margin(d["heat_low"], oh, ow) > 5e-7
    assert res.n_peaks == len(dbg["all_peaks"])
    assert res.n_persons == len(want_s)
    if len(want_s):
        assert np.array_equal(poses.reshape(np.asarray(want_p).shape), np.asarray(want_p, np.float64))
        assert np.allclose(scores, want_s, rtol=SCORE_RTOL, atol=0)


def test_peak_mode_round_trip_restores_cpu_branch(lib, rand_weights):
    """Switching to the GPU branch and back gives the reference's CPU-branch golden bit for bit."""
    c = lib.Context(0)
    try:
        c.set_weights(rand_weights)
        d = load_golden("six_people")
        args = (d["paf_low"], d["heat_low"], int(d["orig_h"]), int(d["orig_w"]))
        c.set_peak_mode("gpu")
        _, sg, _ = c.postprocess(*args)
        c.set_peak_mode("cpu")
        p, s, _ = c.postprocess(*args)
        assert np.array_equal(p.reshape(d["poses"].shape), d["poses"]) and np.array_equal(s, d["scores"])
        assert not np.array_equal(sg, s)  # the unnormalised kernel gives other scores
        with pytest.raises(Exception):
            c.set_peak_mode("gpu", 16)  # even ksize
        with pytest.raises(Exception):
            c.set_peak_mode("gpu", 35)  # radius past the tiled kernel's 16
    finally:
        c.close()


@pytest.mark.parametrize("graph", [False, True])
def test_gpu_branch_staged_batch_equals_single(gctx, graph):
    """The batched path (staged maps, eager and hipGraph) gives each frame the single-frame result."""
    cases = ["six_people", "noise_crowd"]
    ds = [load_golden(c) for c in cases]
    oh, ow = int(ds[0]["orig_h"]), int(ds[0]["orig_w"])
    ds = [d for d in ds if (int(d["orig_h"]), int(d["orig_w"])) == (oh, ow) and d["heat_low"].shape == ds[0]["heat_low"].shape]
    maps = np.stack([np.concatenate([d["paf_low"], d["heat_low"]]) for d in ds])
    single = [gctx.postprocess(d["paf_low"], d["heat_low"], oh, ow) for d in ds]
    gctx.stage_frames(np.zeros((len(ds), oh, ow, 3), np.uint8))
    gctx.stage_maps(maps)
    gctx.use_staged_maps(True)
    try:
        for _ in range(2):
            gctx.run_staged(graph=graph)
            gctx.synchronize()
            for i in range(len(ds)):
                p, s, r = gctx.fetch_result(i)
                assert r.n_peaks == single[i][2].n_peaks
                assert np.array_equal(p, single[i][0]) and np.array_equal(s, single[i][1])
    finally:
        gctx.use_staged_maps(False)


def _near_ties(heat_low, orig_h, orig_w, eps=1e-6):
    """Peak decisions within eps (relative to the map maximum) of a tie: the pixels whose decision
    a rounding difference of that size could flip (see _decision_margin)."""
    from oracle import cvresize
    mw, mh = cvresize.compute_optimal_size(orig_h, orig_w, 320)
    f = P.gpu_branch_filter(P.resize_images(heat_low, mh, mw)[:-1]).astype(np.float64)
    pad = np.pad(f, ((0, 0), (1, 1), (1, 1)))
    g = [f - np.float64(np.float32(0.05))]
    for dy, dx in ((0, 1), (2, 1), (1, 0), (1, 2)):
        g.append(f - pad[:, dy:dy + f.shape[1], dx:dx + f.shape[2]])
    g = np.stack(g)
    peak = (g[0] > 0) & np.all(g[1:] >= 0, axis=0)
    m = np.where(peak, np.abs(g).min(axis=0),
                 np.where(np.concatenate([(g[0] <= 0)[None], g[1:] < 0]), np.abs(g), 0.0).max(axis=0))
    return int((m < eps * max(float(f.max()), 1e-30)).sum())


def test_pose_detector_gpu_branch(pkg, rand_weights):
    """PoseDetector(peak_branch='gpu')(img) runs the GPU-branch post-process: equal bit for bit to the
    context's GPU-branch post-process of the same device forward, different from the CPU branch, and
    its peak count within the near-tie decisions of the oracle's (the random network's noise maps
    hold decisions within 1e-7 of a tie, so peaks are compared by count here; the golden cases
    above compare them exactly)."""
    det = pkg.PoseDetector("posenet", model=rand_weights, device=0, peak_branch="gpu")
    img = people_image()
    x = det._ctx.preprocess(img, 368, 368)
    paf, heat = det._ctx.forward(x)
    poses, scores = det(img)
    p2, s2, r2 = det._ctx.postprocess(paf[0], heat[0], img.shape[0], img.shape[1])
    assert np.array_equal(np.asarray(poses, np.float64).reshape(p2.shape), p2) and np.array_equal(scores, s2)
    _, _, dbg = P.postprocess(paf[0], heat[0], img.shape[0], img.shape[1], return_debug=True, branch="gpu")
    _, _, dbg_cpu = P.postprocess(paf[0], heat[0], img.shape[0], img.shape[1], return_debug=True)
    ties = _near_ties(heat[0], img.shape[0], img.shape[1])
    print("GPU-branch peaks: device %d, oracle %d (CPU branch %d), near-tie decisions %d" % (
        r2.n_peaks, len(dbg["all_peaks"]), len(dbg_cpu["all_peaks"]), ties))
    assert abs(r2.n_peaks - len(dbg["all_peaks"])) <= ties
    assert len(dbg["all_peaks"]) != len(dbg_cpu["all_peaks"]) or not np.array_equal(dbg["all_peaks"], dbg_cpu["all_peaks"])


def test_precise_mode_keeps_the_cpu_branch(lib, rand_weights_small):
    """detect_precise takes the CPU branch whatever the peak mode (the reference's precise heatmaps
    are NumPy arrays: pose_detector.py:470-475)."""
    rng = np.random.default_rng(11)
    img = rng.integers(0, 256, (96, 128, 3), dtype=np.uint8)
    out = []
    for mode in ("cpu", "gpu"):
        c = lib.Context(0)
        try:
            c.set_weights(rand_weights_small)
            c.set_peak_mode(mode)
            p, s, r = c.detect_precise(img)
            out.append((p, s, r.n_peaks))
        finally:
            c.close()
    assert out[0][2] == out[1][2]
    assert np.array_equal(out[0][0], out[1][0]) and np.array_equal(out[0][1], out[1][1])
