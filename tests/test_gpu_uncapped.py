"""The post-process has no caps, like the reference (pose_detector.py:75-250): frames over the
batched buffers' limits (512 peaks per joint by default, 2048 subsets in the LDS grouping, int16
peak ids) are re-run alone with buffers sized from their own counts, and give the reference's
answer (the oracle, itself pinned to the reference's goldens) through every entry point."""
import numpy as np
import pytest

from oracle import postproc as P

pytestmark = pytest.mark.gpu


def _lattice_heat(h, w, step, seed, joints=18):
    """(19, h, w) heat maps with an isolated jittered bump every `step` pixels (offset per joint):
    far more peaks per joint than the batched cap."""
    rng = np.random.default_rng(seed)
    heat = np.zeros((joints + 1, h, w), np.float32)
    for j in range(joints):
        oy, ox = (j % 3), (j // 3) % 3
        ys, xs = np.meshgrid(np.arange(oy + 2, h - 2, step), np.arange(ox + 2, w - 2, step), indexing="ij")
        heat[j, ys, xs] = 3.0 + 0.03 * rng.random(ys.shape).astype(np.float32)
    return heat


@pytest.mark.parametrize("h,w,step", [(200, 200, 6), (300, 320, 6)])
def test_compute_peaks_over_cap(ctx, h, w, step):
    """1089 / 2650 peaks per joint (> 512; the second also > the 2048 LDS sort): bit-exact peaks."""
    heat = _lattice_heat(h, w, step, seed=h)
    want = P.compute_peaks_from_heatmaps(heat, P.PARAMS)
    per_joint = np.bincount(want[:, 0].astype(int), minlength=18)
    assert per_joint.max() > 512
    got = ctx.compute_peaks(heat)
    assert got.shape == want.shape and np.array_equal(got, want)


def _crowded_low_maps(seed):
    """46x46 network maps whose 320x320 upsample has ~529 peaks per joint (a bump every second
    low-res pixel) and a uniform PAF field: hundreds of candidates per limb pair."""
    rng = np.random.default_rng(seed)
    heat = np.zeros((19, 46, 46), np.float32)
    for j in range(18):
        oy, ox = j % 2, (j // 2) % 2
        heat[j, oy::2, ox::2] = 0.5 + 0.1 * rng.random(heat[j, oy::2, ox::2].shape)
    paf = np.full((38, 46, 46), 0.3, np.float32) + 0.05 * rng.random((38, 46, 46)).astype(np.float32)
    return paf, heat


def _oracle_post(paf, heat, oh, ow):
    try:
        return P.postprocess(paf, heat, oh, ow, P.PARAMS)
    except IndexError:
        return IndexError


def test_postprocess_over_cap_single_and_staged(ctx):
    paf, heat = _crowded_low_maps(3)
    want = _oracle_post(paf, heat, 368, 368)
    # the oracle's peaks: over the cap
    mh, mw = 320, 320
    n = P.compute_peaks_from_heatmaps(P.resize_images(heat, mh, mw), P.PARAMS)
    assert np.bincount(n[:, 0].astype(int), minlength=18).max() > 512
    if want is IndexError:
        with pytest.raises(IndexError):
            ctx.postprocess(paf, heat, 368, 368)
    else:
        p, s, r = ctx.postprocess(paf, heat, 368, 368)
        assert r.n_peaks == len(n)
        assert np.array_equal(p.reshape(want[0].shape), want[0]) and np.array_equal(s, want[1])
    # staged batch: frame 1 over the cap between two ordinary frames
    from conftest import load_golden
    d = load_golden("six_people")
    ok = np.concatenate([d["paf_low"], d["heat_low"]])
    assert ok.shape[1:] == (46, 46)
    oh, ow = int(d["orig_h"]), int(d["orig_w"])
    want = _oracle_post(paf, heat, oh, ow)  # the staged frames have the golden's size
    maps = np.stack([ok, np.concatenate([paf, heat]), ok])
    ctx.stage_frames(np.zeros((3, oh, ow, 3), np.uint8))
    ctx.stage_maps(maps)
    ctx.use_staged_maps(True)
    try:
        ctx.run_staged()
        ctx.synchronize()
        for i in (0, 2):
            p, s, r = ctx.fetch_result(i)
            assert np.array_equal(p.reshape(d["poses"].shape), d["poses"]) and np.array_equal(s, d["scores"])
        if want is IndexError:
            with pytest.raises(IndexError):
                ctx.fetch_result(1)
        else:
            p, s, r = ctx.fetch_result(1)
            assert r.status == 0 and np.array_equal(p.reshape(want[0].shape), want[0])
            allr = ctx.fetch_results(0, 3, cap=4)  # cap smaller than the persons: grown by the wrapper
            assert np.array_equal(allr[1][0].reshape(want[0].shape), want[0])
            assert np.array_equal(allr[0][0].reshape(d["poses"].shape), d["poses"])
        # a second graph-replayed run gives the same (re-run uncapped at fetch time again)
        ctx.run_staged(graph=True)
        ctx.synchronize()
        if want is not IndexError:
            p, s, r = ctx.fetch_result(1)
            assert np.array_equal(p.reshape(want[0].shape), want[0]) and np.array_equal(s, want[1])
    finally:
        ctx.use_staged_maps(False)


def test_grouping_over_lds_subsets_and_int16_ids(ctx):
    """2100 full skeletons: 2100 peaks per joint (ids up to 37799 > int16), 2100 subsets (> the 2048
    LDS rows), 2100 persons (> the wrapper's first 2048-row array)."""
    K = 2100
    rng = np.random.default_rng(5)
    peaks = []
    for j in range(18):
        for k in range(K):
            peaks.append([j, rng.integers(0, 300), rng.integers(0, 300), 0.5 + 0.5 * rng.random(), 0])
    peaks = np.array(peaks, np.float64)
    peaks[:, 3] = peaks[:, 3].astype(np.float32)  # peak scores are f32 map values in the reference
    peaks[:, 4] = np.arange(len(peaks))
    conns = []
    for l, (ja, jb) in enumerate(P.PARAMS["limbs_point"]):
        c = np.stack([ja * K + np.arange(K), jb * K + np.arange(K), 0.5 + 0.4 * rng.random(K)], 1).astype(np.float64)
        conns.append(c)
    want = P.grouping_key_points(conns, peaks, P.PARAMS)
    assert len(want) == K
    got = ctx.grouping(conns, peaks)
    assert got.shape == want.shape and np.array_equal(got, want)


def _tie_maps(step):
    """46x46 maps with a lattice of equal bumps (one every `step` low-res pixels per joint) and an
    exactly constant PAF field: candidate scores depend only on the pair's displacement, so the
    limbs have thousands of candidates (more than limb_greedy's 4096-slot sorted batch) with long
    runs of equal scores, resolved by enumeration order (pose_detector.py:172, stable sort)."""
    heat = np.zeros((19, 46, 46), np.float32)
    for j in range(18):
        oy, ox = j % step, (j // step) % step
        heat[j, oy::step, ox::step] = 0.8
    paf = np.full((38, 46, 46), 0.3, np.float32)
    return paf, heat


@pytest.mark.parametrize("step", [3, 4])
def test_greedy_ties_and_batches_vs_oracle(ctx, step):
    """Round 3's limb_greedy (threshold batches sorted in LDS, one wave walking them) on tie-heavy
    candidate lists: bit-exact with the oracle, alone and as one frame of a staged batch."""
    paf, heat = _tie_maps(step)
    want = _oracle_post(paf, heat, 368, 368)
    if want is IndexError:
        with pytest.raises(IndexError):
            ctx.postprocess(paf, heat, 368, 368)
        return
    p, s, r = ctx.postprocess(paf, heat, 368, 368)
    assert np.array_equal(p.reshape(want[0].shape), want[0]) and np.array_equal(s, want[1])
    ctx.stage_frames(np.zeros((2, 368, 368, 3), np.uint8))
    ctx.stage_maps(np.stack([np.concatenate([paf, heat])] * 2))
    ctx.use_staged_maps(True)
    try:
        ctx.run_staged()
        ctx.synchronize()
        for i in range(2):
            p, s, r = ctx.fetch_result(i)
            assert np.array_equal(p.reshape(want[0].shape), want[0]) and np.array_equal(s, want[1]), i
    finally:
        ctx.use_staged_maps(False)
