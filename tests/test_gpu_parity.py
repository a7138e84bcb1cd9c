"""Parity of the HIP path (through the C ABI) with the CPU oracle and the reference goldens.

Bit-exact for the integer/index work and the post-process (which restates f64/f32 NumPy/SciPy
arithmetic exactly); the fp32 forward is held to |gpu - oracle| <= 1e-3 (north star) on maps
of O(1) magnitude."""
import os

import numpy as np
import pytest

from conftest import golden_cases, load_golden, people_image, pkg_module
from oracle import cvresize, postproc as P
from oracle import forward as F

pytestmark = pytest.mark.gpu
FWD_TOL = 1e-3


@pytest.mark.parametrize("shape", [(584, 584), (480, 640), (642, 482), (37, 53), (720, 1280)])
def test_preprocess_bit_exact(ctx, shape):
    rng = np.random.default_rng(shape[0])
    img = rng.integers(0, 256, shape + (3,), dtype=np.uint8)
    w, h = cvresize.compute_optimal_size(shape[0], shape[1], 368)
    got = ctx.preprocess(img, w, h)
    want = cvresize.preprocess(cvresize.resize_linear_u8(img, w, h))
    assert np.array_equal(got, want)


def test_preprocess_people_png(ctx):
    img = people_image()
    got = ctx.preprocess(img, 368, 368)
    assert np.array_equal(got, cvresize.preprocess(cvresize.resize_linear_u8(img, 368, 368)))


@pytest.mark.parametrize("src,dst", [((46, 46), (320, 320)), ((46, 82), (320, 576)), ((62, 46), (432, 320)),
                                     ((5, 7), (40, 13))])
def test_resize_images_bit_exact(ctx, src, dst):
    rng = np.random.default_rng(7)
    x = rng.standard_normal((5,) + src).astype(np.float32)
    assert np.array_equal(ctx.resize_images(x, *dst), P.resize_images(x, *dst))


@pytest.mark.parametrize("case", golden_cases())
def test_peaks_connections_grouping_vs_reference(ctx, case):
    d = load_golden(case)
    mh, mw = int(d["map_h"]), int(d["map_w"])
    heat = P.resize_images(d["heat_low"], mh, mw)
    peaks = ctx.compute_peaks(heat)
    assert np.array_equal(peaks.reshape(-1, 5), d["all_peaks"])
    if int(d["status"]) == 1:
        return
    pafs = P.resize_images(d["paf_low"], mh, mw)
    conns = ctx.compute_connections(pafs, peaks, mw)
    assert np.array_equal(np.concatenate(conns), d["conn"])
    subsets = ctx.grouping(conns, peaks)
    assert np.array_equal(subsets, d["subsets"])


@pytest.mark.parametrize("case", golden_cases())
def test_postprocess_from_network_maps_vs_reference(ctx, case):
    d = load_golden(case)
    poses, scores, res = ctx.postprocess(d["paf_low"], d["heat_low"], int(d["orig_h"]), int(d["orig_w"]))
    assert res.n_peaks == len(d["all_peaks"])
    if int(d["status"]) == 1:
        assert res.n_persons == 0
        return
    assert res.n_persons == int(d["poses_shape"][0])
    assert np.array_equal(poses.reshape(d["poses"].shape), d["poses"])
    assert np.array_equal(scores, d["scores"])


@pytest.mark.parametrize("sigma", [1.5, 4.0])
def test_peaks_nondefault_sigma_vs_oracle(lib, sigma):
    """gaussian_sigma != 2.5 runs the run-time-radius heat kernel (radius 6 and 16 = kMaxR); the
    default radius 10 has its own register-blocked instantiation, covered by the goldens."""
    params = dict(P.PARAMS, gaussian_sigma=sigma)
    c = lib.Context(0, lib.params_from_dict(params), lib.OpLimits())
    try:
        for case in golden_cases()[:3]:
            d = load_golden(case)
            mh, mw = int(d["map_h"]), int(d["map_w"])
            heat = P.resize_images(d["heat_low"], mh, mw)
            want = P.compute_peaks_from_heatmaps(heat, params)
            assert np.array_equal(c.compute_peaks(heat).reshape(-1, 5), want.reshape(-1, 5))
            try:  # fused upsample + filter from the low-res maps: same peak count
                _, _, res = c.postprocess(d["paf_low"], d["heat_low"], int(d["orig_h"]), int(d["orig_w"]))
            except IndexError:  # the grouping quirk may fire on other peaks; the count is not reported then
                continue
            assert res.n_peaks == len(want)
    finally:
        c.close()


def test_grouping_indexerror(ctx):
    d = load_golden("grouping_indexerror")
    off = d["conn_off"]
    with pytest.raises(IndexError):
        ctx.grouping([d["conn"][off[l]:off[l + 1]] for l in range(19)], d["all_peaks"])


def _fwd_check(ctx, weights, x):
    paf, heat = ctx.forward(x)
    opaf, oheat = F.cocoposenet_forward(weights, x)
    err = max(float(np.abs(paf - opaf).max()), float(np.abs(heat - oheat).max()))
    mag = max(float(np.abs(opaf).max()), float(np.abs(oheat).max()))
    print("forward %s: max|gpu-oracle| = %.3g (max|map| = %.3g)" % (x.shape, err, mag))
    assert err <= FWD_TOL
    return paf, heat


@pytest.fixture(params=["bf16x3", "fp32"])
def precision_ctx(request, ctx):
    ctx.set_precision(request.param)
    yield ctx
    ctx.set_precision("bf16x3")


@pytest.mark.parametrize("shape", [(1, 3, 64, 80), (2, 3, 48, 48), (3, 3, 40, 56)])
def test_forward_small_vs_oracle(precision_ctx, rand_weights, shape):
    rng = np.random.default_rng(11)
    x = rng.uniform(-0.5, 0.5, shape).astype(np.float32)
    _fwd_check(precision_ctx, rand_weights, x)


def test_forward_368_vs_oracle(precision_ctx, rand_weights):
    x = cvresize.preprocess(cvresize.resize_linear_u8(people_image(), 368, 368))
    _fwd_check(precision_ctx, rand_weights, x)


@pytest.mark.parametrize("shape", [(1, 3, 184, 328), (1, 3, 368, 656), (2, 3, 552, 984), (1, 3, 736, 1312)])
def test_forward_wide_vs_oracle(ctx, rand_weights, shape):
    """The multi-scale path's wide maps (82 / 123 / 164 columns): the 7x7 raster kernel with the
    tight halo pitch and with frame-aligned tiles (conv_big.hip raster_tiling(wide))."""
    rng = np.random.default_rng(shape[2])
    x = rng.uniform(-0.5, 0.5, shape).astype(np.float32)
    _fwd_check(ctx, rand_weights, x)


@pytest.mark.parametrize("algo", [0, 3])
def test_conv_algos_agree(ctx, algo):
    """Every bf16x3 kernel family computes the same forward (batch 2 at 368x368 and 720p-shaped
    656x368) as the default family, within the 3xBF16 rounding (the default is held to the oracle
    by test_forward_*_vs_oracle)."""
    rng = np.random.default_rng(algo)
    for shape in ((2, 3, 368, 368), (1, 3, 368, 656)):
        x = rng.uniform(-0.5, 0.5, shape).astype(np.float32)
        ctx.set_conv_algo(4)
        p4, h4 = ctx.forward(x)
        ctx.set_conv_algo(algo)
        try:
            pa, ha = ctx.forward(x)
        finally:
            ctx.set_conv_algo(4)
        err = max(float(np.abs(p4 - pa).max()), float(np.abs(h4 - ha).max()))
        assert err <= FWD_TOL, (algo, shape, err)


def test_forward_7x7_tile_sizes_agree(ctx):
    """The 7x7 raster kernel picks its tile size by how many workgroups a launch gets (batch 16 at
    368x368: 320-px tiles; one frame: 128-px tiles), which leaves a pixel's accumulation order
    alone (exact in batch-invariant mode); by default launches that fill few CUs also split their
    input chunks over workgroups (7x7 and 3x3, f32 partials summed by conv_m16_splitk_reduce), so
    a frame's maps agree between batch 16 and batch 1 up to that f32 re-association."""
    rng = np.random.default_rng(16)
    x = rng.uniform(-0.5, 0.5, (16, 3, 368, 368)).astype(np.float32)
    ctx.set_batch_invariant(True)  # tile sizes alone do not change a pixel's accumulation order
    try:
        pi, hi = ctx.forward(x)
        for i in (0, 15):
            p1, h1 = ctx.forward(x[i:i + 1])
            assert np.array_equal(pi[i], p1[0]) and np.array_equal(hi[i], h1[0])
    finally:
        ctx.set_batch_invariant(False)
    pb, hb = ctx.forward(x)  # default: split-K where a launch fills few CUs
    for i in (0, 7, 15):
        p1, h1 = ctx.forward(x[i:i + 1])
        err = max(float(np.abs(pb[i] - p1[0]).max()), float(np.abs(hb[i] - h1[0]).max()))
        mag = max(1.0, float(np.abs(pb[i]).max()), float(np.abs(hb[i]).max()))
        assert err <= 1e-4 * mag, (i, err, mag)  # 10x inside the 1e-3 parity tolerance


def test_forward_precisions_agree(ctx, rand_weights):
    """bf16x3 vs exact-f32 MFMA on a 720p-shaped input (656x368), batch 2."""
    rng = np.random.default_rng(2)
    x = rng.uniform(-0.5, 0.5, (2, 3, 368, 656)).astype(np.float32)
    ctx.set_precision("fp32")
    p32, h32 = ctx.forward(x)
    ctx.set_precision("bf16x3")
    p16, h16 = ctx.forward(x)
    err = max(float(np.abs(p32 - p16).max()), float(np.abs(h32 - h16).max()))
    print("bf16x3 vs fp32 at 656x368: %.3g" % err)
    assert err <= FWD_TOL


@pytest.mark.parametrize("prec", ["fp32", "bf16x3"])
def test_fused_heads_equal_two_launches(ctx, prec, monkeypatch):
    """Each branch's closing 1x1 pair (conv5_4 + conv5_5, Mconv6 + Mconv7; CocoPoseNet.py:162-165,
    181-184) runs as one launch with the intermediate on chip (fp32: conv.hip conv_head_f32; bf16x3:
    conv_head.hip).  The fp32 kernel contracts both layers in the two-launch kernel's order, so every
    stage's maps are BIT-IDENTICAL with OP_HEAD_FUSED=0; the bf16x3 kernel re-splits the
    intermediate on chip and is held to 1e-4 x the map magnitude."""
    rng = np.random.default_rng(21)
    x = rng.uniform(-0.5, 0.5, (2, 3, 184, 248)).astype(np.float32)
    ctx.set_precision(prec)
    try:
        fused = ctx.forward(x)
        monkeypatch.setenv("OP_HEAD_FUSED", "0")
        plain = ctx.forward(x)
        monkeypatch.delenv("OP_HEAD_FUSED")
    finally:
        ctx.set_precision("bf16x3")
    for a, b in zip(fused, plain):
        if prec == "fp32":
            assert np.array_equal(a, b), float(np.abs(a - b).max())
        else:
            assert float(np.abs(a - b).max()) <= 1e-4 * max(1.0, float(np.abs(b).max()))


@pytest.mark.parametrize("n,pl", [(1, 3), (3, 1), (3, 2), (3, 3)])
def test_head_lds_layouts_bit_identical(ctx, n, pl, monkeypatch):
    """conv_head.hip keeps its input (X) and intermediate (T) tiles in LDS either as pixel rows
    (round 5) or as channel-group planes (round 6: no bank conflicts); OP_HEAD_PLANAR (Mconv6+7) /
    OP_HEAD_PLANAR1 (conv5_4+5) = bit 0 X planar, bit 1 T planar.  Only the LDS addresses differ, so
    every stage's maps are BIT-IDENTICAL; 46 x 62 maps leave a partial last 64-pixel tile, and both
    the chunk-planar (stages 2-6) and [pixel][channels] (stage 1) head inputs are read."""
    rng = np.random.default_rng(22)
    x = rng.uniform(-0.5, 0.5, (n, 3, 184, 248)).astype(np.float32)
    ctx.set_precision("bf16x3")
    outs = []
    for v in (pl, 0):
        monkeypatch.setenv("OP_HEAD_PLANAR", str(v))
        monkeypatch.setenv("OP_HEAD_PLANAR1", str(v))
        outs.append(ctx.forward(x))
    for a, b in zip(*outs):
        assert np.array_equal(a, b), float(np.abs(a - b).max())


def test_detect_equals_stagewise_oracle_composition(pkg, rand_weights):
    """PoseDetector(img) == oracle post-process of the GPU forward of the GPU-preprocessed image."""
    det = pkg.PoseDetector("posenet", model=rand_weights, device=0)
    img = people_image()
    x = det._ctx.preprocess(img, 368, 368)
    paf, heat = det._ctx.forward(x)
    want_p, want_s = P.postprocess(paf[0], heat[0], img.shape[0], img.shape[1])
    poses, scores = det(img)
    assert np.asarray(poses).shape == np.asarray(want_p).shape
    assert np.array_equal(np.asarray(poses, np.float64), np.asarray(want_p, np.float64))
    assert np.array_equal(scores, want_s)


@pytest.mark.parametrize("prec", ["bf16x3", "fp32"])
def test_staged_batch_matches_single_and_graph(ctx, prec):
    """A staged batch (eager and hipGraph replay) gives each frame exactly the result of a
    single-frame detect in batch-invariant mode (op_set_batch_invariant: no split-K for the lone
    frame's 7x7 launches)."""
    ctx.set_precision(prec)
    ctx.set_batch_invariant(True)

    rng = np.random.default_rng(3)
    frames = rng.integers(0, 256, (3, 300, 420, 3), dtype=np.uint8)
    single = [ctx.detect(f) for f in frames]
    ctx.stage_frames(frames)
    for graph in (False, True, True):
        ctx.run_staged(graph=graph)
        ctx.synchronize()
        for i in range(3):
            p, s, r = ctx.fetch_result(i)
            assert r.n_peaks == single[i][2].n_peaks
            assert np.array_equal(p, single[i][0]) and np.array_equal(s, single[i][1])
        for i, (p, s, r) in enumerate(ctx.fetch_results(0, 3, cap=2048)):
            assert r.n_peaks == single[i][2].n_peaks and r.status == 0
            assert np.array_equal(p, single[i][0]) and np.array_equal(s, single[i][1])
    ctx.set_precision("bf16x3")
    ctx.set_batch_invariant(False)


def test_graph_replay_follows_batch_invariant_switch(ctx):
    """A hipGraph captured for one staged frame in the default mode (its small launches split K)
    is not replayed after op_set_batch_invariant(1): the replay equals the eager batch-invariant
    run bit for bit, and switching back restores the split-K replay (graph key)."""
    frame = np.random.default_rng(21).integers(0, 256, (1, 368, 368, 3), dtype=np.uint8)
    ctx.stage_frames(frame)
    ctx.set_batch_invariant(False)
    ctx.run_staged(graph=True)
    ctx.synchronize()
    split_maps = ctx.fetch_maps(0, 1)
    try:
        ctx.set_batch_invariant(True)
        ctx.run_staged(graph=True)
        ctx.synchronize()
        g = ctx.fetch_maps(0, 1)
        ctx.run_staged(graph=False)
        ctx.synchronize()
        e = ctx.fetch_maps(0, 1)
        assert np.array_equal(g[0], e[0]) and np.array_equal(g[1], e[1])
    finally:
        ctx.set_batch_invariant(False)
    ctx.run_staged(graph=True)
    ctx.synchronize()
    back = ctx.fetch_maps(0, 1)
    assert np.array_equal(back[0], split_maps[0]) and np.array_equal(back[1], split_maps[1])
    # split-K and invariant sums differ only by f32 re-association
    assert np.abs(split_maps[0] - e[0]).max() <= 1e-4 and np.abs(split_maps[1] - e[1]).max() <= 1e-4


def test_step_graph_touches_device_memory_only(ctx):
    """Regression for the round-1 replay fault: the captured step graph holds kernels and
    device-side memsets / copies only -- no node reads or writes host memory, so no replay can write
    through a host pointer whose pages were since freed.  Results are fetched after each replay into
    freshly allocated (pageable, immediately dropped) NumPy arrays of varying capacity, and every
    replay still equals the eager run."""
    frames = np.random.default_rng(23).integers(0, 256, (4, 368, 368, 3), dtype=np.uint8)
    ctx.stage_frames(frames)
    ctx.run_staged(graph=False)
    ctx.synchronize()
    want = [(p.copy(), s.copy()) for p, s, _ in ctx.fetch_results(0, 4, cap=2048)]
    ctx.run_staged(graph=True)
    ctx.synchronize()
    info = ctx.graph_info()
    assert info["host_nodes"] == 0, info
    assert info["kernels"] >= 50 and info["nodes"] >= info["kernels"] + info["memsets"] + info["memcpys"], info
    for it in range(12):
        ctx.run_staged(graph=True)
        ctx.synchronize()
        got = ctx.fetch_results(0, 4, cap=(16, 2048, 64)[it % 3])
        for (p, s, r), (wp, ws) in zip(got, want):
            assert r.status == 0 and np.array_equal(p, wp) and np.array_equal(s, ws)
        del got
        junk = [np.empty((it + 1) * 1_000_003, np.uint8) for _ in range(3)]  # churn the host heap
        del junk


def test_fetch_maps_equals_forward_of_preprocessed_frames(ctx):
    """op_fetch_maps after op_run_staged = op_forward of the op_preprocess'ed frames (the staged
    path resamples the input inside its first conv kernel)."""
    frames = np.random.default_rng(22).integers(0, 256, (2, 300, 420, 3), dtype=np.uint8)
    ctx.set_batch_invariant(True)
    try:
        ctx.stage_frames(frames)
        ctx.run_staged()
        ctx.synchronize()
        pafs, heat = ctx.fetch_maps(0, 2)
        x = np.concatenate([ctx.preprocess(f, 520, 368) for f in frames])  # compute_optimal_size: 520 x 368
        wp, wh = ctx.forward(x)
    finally:
        ctx.set_batch_invariant(False)
    assert pafs.shape == (2, 38, 46, 65) and heat.shape == (2, 19, 46, 65)
    err = max(float(np.abs(pafs - wp).max()), float(np.abs(heat - wh).max()))
    assert err <= 1e-5, err


@pytest.mark.parametrize("graph", [False, True])
def test_async_uploads_equal_staged_frames(ctx, lib, graph):
    """op_upload_frames (pinned host -> 2-slot device ring on the copy stream, overlapped with the
    previous run) gives each run exactly the maps and results of op_stage_frames of the same frames,
    over alternating ring slots and a shape change."""
    rng = np.random.default_rng(23)
    batches = [rng.integers(0, 256, (2, 240, 320, 3), dtype=np.uint8) for _ in range(3)]
    batches.append(rng.integers(0, 256, (3, 200, 256, 3), dtype=np.uint8))
    want = []
    for b in batches:
        ctx.stage_frames(b)
        ctx.run_staged(graph=graph)
        ctx.synchronize()
        want.append((ctx.fetch_maps(0, len(b)), ctx.fetch_results(0, len(b))))
    pinned = [lib.PinnedFrames(*b.shape[:3]) for b in batches]
    for p, b in zip(pinned, batches):
        p.array[...] = b
    try:
        ctx.upload_frames(pinned[0].array)
        for k in range(len(batches)):
            ctx.run_staged(graph=graph)
            if k + 1 < len(batches):
                ctx.upload_frames(pinned[k + 1].array)  # overlaps run k
            ctx.synchronize()
            maps, res = ctx.fetch_maps(0, len(batches[k])), ctx.fetch_results(0, len(batches[k]))
            (wm, wr) = want[k]
            assert np.array_equal(maps[0], wm[0]) and np.array_equal(maps[1], wm[1]), k
            for (p, sc, r), (wp, ws, wr_) in zip(res, wr):
                assert r.n_peaks == wr_.n_peaks and np.array_equal(p, wp) and np.array_equal(sc, ws)
    finally:
        for p in pinned:
            p.close()


def test_one_pinned_buffer_rewritten_after_upload_wait(ctx, lib):
    """The op_upload_frames contract (include/openpose_hip.h): the host buffer may be rewritten
    once op_upload_wait returns, even while the run consuming the copy is still in flight -- so a
    caller can recycle ONE pinned buffer.  Each run still sees exactly its own frames."""
    rng = np.random.default_rng(29)
    batches = [rng.integers(0, 256, (2, 240, 320, 3), dtype=np.uint8) for _ in range(3)]
    want = []
    for b in batches:
        ctx.stage_frames(b)
        ctx.run_staged()
        ctx.synchronize()
        want.append(ctx.fetch_maps(0, len(b)))
    pinned = lib.PinnedFrames(2, 240, 320)
    try:
        got = []
        for b in batches:
            pinned.array[...] = b
            ctx.upload_frames(pinned.array)
            ctx.run_staged()
            ctx.upload_wait()
            pinned.array[...] = 255 - b  # the run may still be executing; its copy has landed
            ctx.synchronize()
            got.append(ctx.fetch_maps(0, len(b)))
        for k, (g, w) in enumerate(zip(got, want)):
            assert np.array_equal(g[0], w[0]) and np.array_equal(g[1], w[1]), k
    finally:
        pinned.close()


def test_staged_synthetic_maps_match_reference(ctx):
    d = load_golden("six_people")
    maps = np.concatenate([d["paf_low"], d["heat_low"]])[None].repeat(2, axis=0)
    frames = np.zeros((2, int(d["orig_h"]), int(d["orig_w"]), 3), np.uint8)
    ctx.stage_frames(frames)
    ctx.stage_maps(maps)
    ctx.use_staged_maps(True)
    try:
        ctx.run_staged()
        ctx.synchronize()
        for i in range(2):
            p, s, r = ctx.fetch_result(i)
            assert np.array_equal(p.reshape(d["poses"].shape), d["poses"]) and np.array_equal(s, d["scores"])
    finally:
        ctx.use_staged_maps(False)


# ---- multi-scale path: detect_precise (pose_detector.py:433-482) ----
from oracle import precise as PR  # noqa: E402


@pytest.mark.parametrize("h,w,oh,ow,cn", [(720, 1280, 184, 328, 3), (50, 70, 37, 91, 3), (17, 23, 61, 45, 1),
                                          (368, 368, 736, 736, 3)])
def test_resize_cubic_u8_bit_exact(ctx, h, w, oh, ow, cn):
    rng = np.random.default_rng(h + w)
    img = rng.integers(0, 256, (h, w, cn), dtype=np.uint8)
    assert np.array_equal(ctx.resize_cubic(img, ow, oh), PR.resize_cubic_u8(img, ow, oh))


@pytest.mark.parametrize("h,w,oh,ow,cn", [(46, 82, 368, 656, 38), (23, 41, 184, 328, 19), (45, 81, 720, 1280, 19),
                                          (7, 5, 13, 11, 3)])
def test_resize_cubic_f32_bit_exact(ctx, h, w, oh, ow, cn):
    rng = np.random.default_rng(h * w)
    x = rng.standard_normal((h, w, cn)).astype(np.float32)
    assert np.array_equal(ctx.resize_cubic(x, ow, oh), PR.resize_cubic_f32(x, ow, oh))


@pytest.mark.parametrize("prec", ["bf16x3", "fp32"])
def test_detect_precise_vs_oracle(lib, rand_weights_small, prec):
    params = dict(P.PARAMS, inference_img_size=32)
    limits = lib.OpLimits()
    limits.max_peaks_per_joint = 2048
    c = lib.Context(0, lib.params_from_dict(params), limits)
    try:
        c.set_precision(prec)
        c.set_weights(rand_weights_small)
        img = np.random.default_rng(5).integers(0, 256, (40, 56, 3), dtype=np.uint8)
        try:
            poses, scores, res, pafs, heat = c.detect_precise(img, return_maps=True)
            raised = False
        except IndexError as e:  # then the reference raises on these maps too (checked below)
            pafs, heat = e.maps
            raised = True
        want_paf, want_heat = PR.precise_maps(rand_weights_small, img, params)
        assert pafs.shape == want_paf.shape and heat.shape == want_heat.shape
        assert np.abs(pafs - want_paf).max() <= FWD_TOL and np.abs(heat - want_heat).max() <= FWD_TOL
        # the post-process on the GPU's own maps is bit-exact with the oracle's
        if raised:
            with pytest.raises(IndexError):
                PR.postprocess_full(pafs, heat, img.shape[1], params)
        else:
            wp, ws = PR.postprocess_full(pafs, heat, img.shape[1], params)
            assert res.n_peaks == len(P.compute_peaks_from_heatmaps(heat, params))
            assert np.array_equal(poses.reshape(wp.shape), wp) and np.array_equal(scores, ws)
    finally:
        c.close()


def test_staged_precise_batch_equals_per_frame(lib, rand_weights):
    """op_run_staged_precise (all staged frames batched per scale) == op_detect_precise per frame:
    poses, scores and status identical, incl. frames whose noise maps exceed the batched caps (re-run
    uncapped) or raise the reference's IndexError (pose_detector.py:197).  Any other exception (a HIP
    failure surfaces as RuntimeError) fails the test: it is never compared as an outcome."""
    W = {k: (w, b.copy()) for k, (w, b) in rand_weights.items()}
    for k in ("Mconv7_stage6_L1", "Mconv7_stage6_L2"):  # fewer noise peaks on the random maps
        W[k] = (W[k][0], W[k][1] - np.float32(0.3))
    limits = lib.OpLimits()
    limits.max_batch = 3
    c = lib.Context(0, None, limits)
    try:
        c.set_weights(W)
        frames = np.random.default_rng(9).integers(0, 256, (3, 72, 104, 3), dtype=np.uint8)
        single = []
        for f in frames:
            try:
                single.append((0,) + tuple(c.detect_precise(f)[:2]))
            except IndexError:
                single.append(("IndexError",))
        c.stage_frames(frames)
        c.run_staged_precise()
        for i in range(3):
            try:
                p, s_, r = c.fetch_result(i)
                got = (0, p, s_)
                assert r.map_w == 104 and r.map_h == 72
            except IndexError:
                got = ("IndexError",)
            assert got[0] == single[i][0]
            if got[0] == 0:
                assert np.array_equal(got[1], single[i][1]) and np.array_equal(got[2], single[i][2])
    finally:
        c.close()


def test_pose_detector_precise_mode(pkg, rand_weights):
    """PoseDetector(precise=True) == the oracle's full-resolution post-process of the GPU's averaged
    maps; where the oracle raises the reference's IndexError (pose_detector.py:197), so must the
    detector.  No other exception is accepted."""
    from oracle import precise as PR
    det = pkg.PoseDetector("posenet", model=rand_weights, precise=True)
    img = np.random.default_rng(6).integers(0, 256, (96, 128, 3), dtype=np.uint8)
    try:
        _, _, _, pafs, heat = det._ctx.detect_precise(img, return_maps=True)
    except IndexError as e:
        pafs, heat = e.maps
    assert pafs.shape == (38, 96, 128) and heat.shape == (19, 96, 128)
    try:
        want_p, want_s = PR.postprocess_full(pafs, heat, 128, P.PARAMS)
    except IndexError:
        with pytest.raises(IndexError):
            det(img)
        return
    poses, scores = det(img)
    assert np.array_equal(det.pafs, pafs) and np.array_equal(det.heatmaps, heat)
    assert np.asarray(poses).shape == np.asarray(want_p).shape
    assert np.array_equal(np.asarray(poses, np.float64), np.asarray(want_p, np.float64))
    assert np.array_equal(scores, want_s)


def test_cli_writes_result_png(tmp_path, rand_weights):
    """pose_detector.py:555-579: npz weights + image -> result image."""
    from PIL import Image
    W = pkg_module("weights")
    D = pkg_module("draw")
    wpath = str(tmp_path / "w.npz")
    W.save_npz(wpath, rand_weights)
    ipath = str(tmp_path / "in.png")
    Image.fromarray(people_image()[:, :, ::-1]).save(ipath)
    out = str(tmp_path / "result.png")
    assert D.main(["posenet", wpath, "--img", ipath, "--out", out]) == 0
    res = np.asarray(Image.open(out))
    assert res.shape == people_image().shape


def test_cli_on_person_png_draws_the_detected_poses(tmp_path, pkg, rand_weights):
    """C1 (BASELINE configs[0]): the CLI on data/person.png (RGBA 584x584, README.md:16;
    pose_detector.py:555-579).  The written image must be exactly draw_person_pose of the poses the
    detector returns for cv2.imread's BGR view of the file, and pixels no pose touches unchanged."""
    from PIL import Image
    W = pkg_module("weights")
    D = pkg_module("draw")
    wpath = str(tmp_path / "w.npz")
    W.save_npz(wpath, rand_weights)
    ipath = os.path.join(os.path.dirname(__file__), "golden", "person.png")
    out = str(tmp_path / "result.png")
    img = D.read_bgr(ipath)
    det = pkg.PoseDetector("posenet", model=rand_weights)
    try:
        assert D.main(["posenet", wpath, "--img", ipath, "--out", out]) == 0
    except IndexError:
        # only acceptable where the reference raises too: the oracle post-process of these maps
        x = det._ctx.preprocess(img, 368, 368)
        paf, heat = det._ctx.forward(x)
        with pytest.raises(IndexError):
            P.postprocess(paf[0], heat[0], img.shape[0], img.shape[1])
        pytest.skip("random weights: the reference's grouping raises IndexError on these maps too (checked)")
    poses, _ = det(img)
    want = D.draw_person_pose(img, poses)
    got = D.read_bgr(out)
    assert got.shape == (584, 584, 3)
    assert np.array_equal(got, want)


def test_profile_counts_every_7x7_launch_with_joined_events(ctx, lib):
    """bench.py's roofline timing: Mconv1..Mconv5 of a stage share one event pair (prof_join), yet
    the class still counts 25 launches and the algorithmic FLOPs of all of them per forward."""
    ctx.stage_frames(np.zeros((2, 368, 368, 3), np.uint8))  # net 368 x 368, maps 46 x 46
    ctx.profile_classes(["conv7x7"])
    ctx.profile(True)
    ctx.profile_reset()
    try:
        for _ in range(2):
            ctx.run_staged()
        ctx.synchronize()
        ms, n, fl, by = ctx.profile_read()["conv7x7"]
    finally:
        ctx.profile(False)
    assert n == 2 * 25 and ms > 0.0
    # 2 runs x 2 frames x 5 stages x 2 branches x 2 FLOP x 49 taps x 128 outputs x (185 + 4 x 128) inputs x 46^2
    assert fl == 2 * 2 * 5 * 2 * 2 * 49 * 128 * (185 + 4 * 128) * 46 * 46
