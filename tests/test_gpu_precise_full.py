"""Config C4 at its real size (BASELINE configs[3]): detect_precise
(pose_detector.py:433-482) on 1280x720 frames with the reference's four inference scales
(entity.py:72: 0.5 / 1.0 / 1.5 / 2.0 -> network inputs 184x328, 368x656, 552x984, 736x1312),
through the C ABI, against the oracle:

* the averaged full-resolution maps within the north star's 1e-3 of oracle/precise.py (four oracle
  forwards, ~40 s of host BLAS);
* the full-resolution post-process (img_len = orig_w, :474-482) on the GPU's own maps bit-exact with
  the oracle's (peaks / connections / grouping on 1280x720 maps);
* a loaded full-resolution post-process: COCO-like 20-person maps at 1280x720 staged in place of the
  averaged maps (op_stage_maps at the frame size), bit-exact with the oracle -- the workload the
  C4 bench line runs.
"""
import numpy as np
import pytest

from conftest import load_golden, pkg_module
from oracle import postproc as P
from oracle import precise as PR

pytestmark = pytest.mark.gpu
FWD_TOL = 1e-3  # north star: PAF / heatmap values within 1e-3 (fp32)
H, W = 720, 1280


def _crowd_frame(seed):
    """A seeded 1280x720 BGR frame with smooth structure (a noise frame at every scale would be a
    weak test of the cubic resizes): low-frequency colour fields plus noise."""
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:H, 0:W].astype(np.float32)
    img = np.zeros((H, W, 3), np.float32)
    for c in range(3):
        for _ in range(4):
            fx, fy, ph = rng.uniform(0.002, 0.03), rng.uniform(0.002, 0.03), rng.uniform(0, 6.28)
            img[:, :, c] += 40 * np.sin(fx * xx + fy * yy + ph)
    img += 128 + rng.normal(0, 12, img.shape)
    return np.clip(img, 0, 255).astype(np.uint8)


def _weights(rand_weights):
    """The seeded random CocoPoseNet with the last stage's biases lowered (fewer noise peaks on the
    maps of a random network, as test_gpu_parity's staged precise test)."""
    Wt = {k: (w, b.copy()) for k, (w, b) in rand_weights.items()}
    for k in ("Mconv7_stage6_L1", "Mconv7_stage6_L2"):
        Wt[k] = (Wt[k][0], Wt[k][1] - np.float32(0.3))
    return Wt


def test_scale_sizes_720p():
    sizes = PR.scale_sizes(H, W, P.PARAMS)
    assert [(pw, ph) for _, _, pw, ph in sizes] == [(328, 184), (656, 368), (984, 552), (1312, 736)]


def test_detect_precise_1280x720_vs_oracle(lib, rand_weights):
    Wt = _weights(rand_weights)
    limits = lib.OpLimits()
    limits.max_peaks_per_joint = 2048
    c = lib.Context(0, None, limits)
    try:
        c.set_weights(Wt)
        c.set_batch_invariant(True)  # the lone frame and the staged pair then sum in one order
        img = _crowd_frame(7)
        try:
            poses, scores, res, pafs, heat = c.detect_precise(img, return_maps=True)
            raised = None
        except IndexError as e:  # then the oracle raises on these maps too (checked below)
            pafs, heat = e.maps
            raised = IndexError
        want_paf, want_heat = PR.precise_maps(Wt, img, P.PARAMS)
        assert pafs.shape == (38, H, W) and heat.shape == (19, H, W)
        err = max(float(np.abs(pafs - want_paf).max()), float(np.abs(heat - want_heat).max()))
        print("C4 1280x720: max|gpu-oracle| averaged maps = %.3g" % err)
        assert err <= FWD_TOL
        # the full-resolution post-process of the GPU's own maps == the oracle's, bit for bit
        if raised is IndexError:
            with pytest.raises(IndexError):
                PR.postprocess_full(pafs, heat, W, P.PARAMS)
        else:
            wp, ws = PR.postprocess_full(pafs, heat, W, P.PARAMS)
            assert res.n_peaks == len(P.compute_peaks_from_heatmaps(heat, P.PARAMS))
            assert np.array_equal(poses.reshape(wp.shape), wp) and np.array_equal(scores, ws)
        # the staged batch path gives the same frame the same maps and result
        c.stage_frames(np.stack([img, img[::-1].copy()]))
        try:
            c.run_staged_precise()
            c.synchronize()
            sp, sh = c.fetch_maps(0, 1)
            assert np.array_equal(sp[0], pafs) and np.array_equal(sh[0], heat)
            if raised is None:
                p0, s0, _ = c.fetch_result(0)
                assert np.array_equal(p0, poses) and np.array_equal(s0, scores)
        except IndexError:
            assert raised is IndexError
    finally:
        c.close()


def _loaded_full_maps(ctx):
    """COCO-like 20-person maps at 1280x720: the reference-generated 46x82 maps of the twenty_720p
    golden, upsampled on the device (F.resize_images) to the frame size."""
    d = load_golden("twenty_720p")
    assert (int(d["orig_h"]), int(d["orig_w"])) == (H, W)
    low = np.concatenate([d["paf_low"], d["heat_low"]])
    return ctx.resize_images(low, H, W)


def test_loaded_full_resolution_postprocess(lib, rand_weights):
    c = lib.Context(0)
    try:
        c.set_weights(rand_weights)
        maps = _loaded_full_maps(c)
        assert maps.shape == (57, H, W)
        wp, ws = PR.postprocess_full(maps[:38], maps[38:], W, P.PARAMS)
        assert len(wp) >= 15  # the maps are loaded: most of the 20 people come out
        frames = np.zeros((2, H, W, 3), np.uint8)
        c.stage_frames(frames)
        c.stage_maps(np.stack([maps, maps]))
        c.use_staged_maps(True)
        c.run_staged_precise()
        c.synchronize()
        for i in range(2):
            p, s, r = c.fetch_result(i)
            assert r.status == 0 and r.map_w == W and r.map_h == H
            assert np.array_equal(p.reshape(wp.shape), wp) and np.array_equal(s, ws)
        # the averaged network maps are still computed (only the post-process input is replaced)
        sp, sh = c.fetch_maps(0, 1)
        assert sp.shape == (1, 38, H, W) and np.isfinite(sp).all() and np.abs(sh).max() > 0
        c.use_staged_maps(False)
    finally:
        c.close()


@pytest.mark.parametrize("shape,n", [((H, W), 3), ((481, 643), 2), ((96, 128), 2)])
def test_fused_map_resize_equals_two_pass(lib, rand_weights, shape, n, monkeypatch):
    """Round 4 experiment (opt-in, OP_CUBIC_FUSED=1; the default is the two-pass path, which measured
    faster): detect_precise's two cubic map resizes per scale and the scale mean as one fused pass
    (precise.hip resize_cubic_fused_mean: the padded-size maps never reach HBM).  It restates the
    two-pass kernels' f32 operations in their order, so the averaged maps of a staged batch are
    BIT-IDENTICAL with the two-pass path (held to the oracle above).  96x128 frames upsample their
    scale-2 crop ~7.7x in the second resize: the fused tile then exceeds LDS and the two-pass path
    runs (census)."""
    Wt = _weights(rand_weights)
    limits = lib.OpLimits()
    limits.max_peaks_per_joint = 2048
    c = lib.Context(0, None, limits)
    h, w = shape
    try:
        c.set_weights(Wt)
        c.set_batch_invariant(True)
        frames = np.stack([_crowd_frame(11 + i)[:h, :w] for i in range(n)])
        out = {}
        for fused in ("1", "0"):
            monkeypatch.setenv("OP_CUBIC_FUSED", fused)
            c.stage_frames(frames)
            lib.conv_census(reset=True)
            try:
                c.run_staged_precise()
            except IndexError:
                pass
            c.synchronize()
            cen = lib.conv_census(reset=True)
            out[fused] = (c.fetch_maps(0, n), cen)
        (p1, h1), cen1 = out["1"]
        (p0, h0), cen0 = out["0"]
        assert cen0["cubic_two_pass"] == 1 and cen0["cubic_fused"] == 0
        if shape == (96, 128):
            assert cen1["cubic_two_pass"] == 1 and cen1["cubic_fused"] == 0
        else:
            assert cen1["cubic_fused"] == 1 and cen1["cubic_two_pass"] == 0
        assert p1.shape == (n, 38, h, w) and h1.shape == (n, 19, h, w)
        assert np.array_equal(p1, p0) and np.array_equal(h1, h0)
    finally:
        c.close()


@pytest.mark.parametrize("shape,n", [((H, W), 3), ((481, 643), 2), ((96, 128), 2)])
def test_row_block_map_resize_equals_per_frame(lib, rand_weights, shape, n, monkeypatch):
    """Round 4: the two-pass path's second resize (every scale's crop cubic-resized to the frame
    size, summed in scale order, divided by the scale count) as one launch for the batch with blocks
    of 8 output rows that make each source row's horizontal sums once
    (precise.hip resize_cubic_f32_planar_mean_rows, the default) and its form with each scale's
    source tile staged in LDS (_tile, OP_CUBIC_TILE=1) are BIT-IDENTICAL to the per-frame form
    (OP_CUBIC_ROWS=0, resize_cubic_f32_planar_mean, held to the oracle above); the census shows
    which ran."""
    Wt = _weights(rand_weights)
    limits = lib.OpLimits()
    limits.max_peaks_per_joint = 2048
    c = lib.Context(0, None, limits)
    h, w = shape
    try:
        c.set_weights(Wt)
        c.set_batch_invariant(True)
        frames = np.stack([_crowd_frame(21 + i)[:h, :w] for i in range(n)])
        out = {}
        for rows in ("tile", "1", "0"):  # tile: the LDS-staged form (OP_CUBIC_TILE=1)
            monkeypatch.setenv("OP_CUBIC_ROWS", "0" if rows == "0" else "1")
            monkeypatch.setenv("OP_CUBIC_TILE", "1" if rows == "tile" else "0")
            c.stage_frames(frames)
            lib.conv_census(reset=True)
            try:
                c.run_staged_precise()
            except IndexError:
                pass
            c.synchronize()
            cen = lib.conv_census(reset=True)
            out[rows] = (c.fetch_maps(0, n), cen)
        (p1, h1), cen1 = out["1"]
        (p0, h0), cen0 = out["0"]
        (pt, ht), cent = out["tile"]
        assert cent["cubic_two_pass"] == 1 and cent["cubic_rows"] == 1
        assert np.array_equal(pt, p0) and np.array_equal(ht, h0)
        assert cen1["cubic_two_pass"] == 1 and cen1["cubic_rows"] == 1
        assert cen0["cubic_two_pass"] == 1 and cen0["cubic_rows"] == 0
        assert p1.shape == (n, 38, h, w) and h1.shape == (n, 19, h, w)
        assert np.isfinite(p1).all() and np.isfinite(h1).all()
        assert np.array_equal(p1, p0) and np.array_equal(h1, h0)
    finally:
        c.close()
