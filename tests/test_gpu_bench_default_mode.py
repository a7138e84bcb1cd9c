"""Parity at the kernels the C4 and C5 bench lines run in the DEFAULT mode.

bench.py never calls set_batch_invariant: launches that leave CUs idle split their input chunks
over several workgroups (f32 partials + conv_m16_splitk_reduce, a batch-dependent re-association).
test_gpu_bench_configs.py holds C4's 16-frame and C5's 64-frame batches to single-frame runs in
batch-invariant mode (split-K off); here the same batches run exactly as the bench runs them:

* C4 (bench.py --precise --frame 720x1280: 16 frames of 1280x720 through run_staged_precise,
  pose_detector.py:433-482): op_conv_census shows the split-K 7x7 launches that ran (the cost model
  splits some of the per-scale launches); frames 0, 8 and 15 are held to the CPU
  oracle's detect_precise maps (oracle/precise.py: cv2 CUBIC restatement, the reference network,
  the scale mean) at the north star's 1e-3; every frame's full-resolution post-process == the
  oracle post-process of that frame's GPU maps, bit for bit; a second run gives the same bits
  (the split-K reduce sums in a fixed order).
* C5 (bench.py --frame 720x1280: 64 frames, single scale, pose_detector.py:484-517): the census
  proves no split-K launch ran in the default mode (so the batch-invariant evidence carries over:
  the default-mode maps are asserted bit-identical to the invariant-mode ones, which
  test_c5_stream_batch_of_64_720p_frames holds to single frames); frames 0 / 31 / 63 <= 1e-3 vs the
  oracle; their post-process == the oracle post-process of the GPU maps.
* One 368x368 frame (the batch-1 line): the pooled 3x3 launches split K
  (conv_m16_splitk_reduce_pool: census 3x3_pool with 3x3_splitk) -- their maps close to the
  unsplit (batch-invariant) run (REL_SPLIT, relative to the map scale), and a replayed hipGraph == eager.
"""
import numpy as np
import pytest

from conftest import pkg_module
from oracle import cvresize
from oracle import forward as F
from oracle import postproc as P
from oracle import precise as PR
from test_forward_golden import case_weights
from test_gpu_precise_full import _crowd_frame, _weights

pytestmark = pytest.mark.gpu
TOL = 1e-3  # north star: PAF / heatmap values within 1e-3 (fp32)
H, W = 720, 1280
C4_N = 16  # bench.py --precise default batch
C5_N = 64  # bench.py --frame 720x1280 default batch
# split vs unsplit channel sums of the pooled 3x3 launches, seen at the network output after ~85
# more layers: each split activation is stored as bf16 hi + bf16 lo (~16 significant bits), so a
# last-bit change of an f32 sum can move the stored value by ~2^-16 relative
REL_SPLIT = 1e-4


@pytest.fixture(scope="module")
def lib():
    return pkg_module("_lib")


def _result(fetch):
    try:
        return fetch()
    except IndexError:  # the reference's grouping quirk (pose_detector.py:197)
        return IndexError


def _max_err(a, b):
    return float(np.abs(np.float64(a) - np.float64(b)).max())


@pytest.fixture(scope="module")
def c4_run(lib):
    """16 1280x720 frames through run_staged_precise with the bench's own context settings
    (OpLimits with max_batch = 16, bf16x3, NO batch-invariant switch), run twice."""
    frames = np.stack([_crowd_frame(300 + i) for i in range(C4_N)])
    Wt = _weights(case_weights("posenet", 0))
    limits = lib.OpLimits()
    limits.max_batch = C4_N
    c = lib.Context(0, None, limits)
    try:
        c.set_weights(Wt)
        c.stage_frames(frames)
        lib.conv_census(reset=True)
        try:
            c.run_staged_precise()
        except IndexError:
            pass
        c.synchronize()
        cen = lib.conv_census(reset=True)
        paf, heat = c.fetch_maps(0, C4_N)
        res = [_result(lambda i=i: c.fetch_result(i)) for i in range(C4_N)]
        try:
            c.run_staged_precise()
        except IndexError:
            pass
        c.synchronize()
        paf2, heat2 = c.fetch_maps(0, C4_N)
        same = np.array_equal(paf, paf2) and np.array_equal(heat, heat2)
        del paf2, heat2
    finally:
        c.close()
    return {"frames": frames, "W": Wt, "census": cen, "paf": paf, "heat": heat, "res": res, "repeat_same": same}


def test_c4_default_mode_census_runs_split_k(c4_run):
    cen = c4_run["census"]
    print("C4 default-mode census:", cen)
    assert cen["7x7_splitk"] > 0, cen  # the bench's split-K 7x7 launches are what is tested here
    assert sum(cen["npx"].values()) == 4 * 25, cen  # 4 scales x 5 stages x Mconv1..5
    assert c4_run["repeat_same"]  # the reduce sums the partials in a fixed order


@pytest.mark.parametrize("i", [0, C4_N // 2, C4_N - 1])
def test_c4_default_mode_maps_vs_oracle(c4_run, i):
    want_paf, want_heat = PR.precise_maps(c4_run["W"], c4_run["frames"][i], P.PARAMS)
    e = max(_max_err(c4_run["paf"][i], want_paf), _max_err(c4_run["heat"][i], want_heat))
    print("C4 default mode frame %d: max|gpu-oracle| averaged maps = %.3g" % (i, e))
    assert e <= TOL, (i, e)


@pytest.mark.parametrize("i", range(C4_N))
def test_c4_default_mode_postprocess_bit_exact(c4_run, i):
    """pose_detector.py:474-482 on frame i's own GPU maps: the oracle's peaks / connections /
    grouping at 1280x720 == the GPU post-process of the staged batch (big mode for frames past the
    batched caps)."""
    paf, heat = c4_run["paf"][i], c4_run["heat"][i]
    got = c4_run["res"][i]
    try:
        wp, ws = PR.postprocess_full(paf, heat, W, P.PARAMS)
    except IndexError:
        assert got is IndexError, i
        return
    assert got is not IndexError, i
    poses, scores, r = got
    assert r.status == 0 and r.map_w == W and r.map_h == H
    assert r.n_peaks == len(P.compute_peaks_from_heatmaps(heat, P.PARAMS))
    assert np.array_equal(np.asarray(poses).reshape(wp.shape), wp) and np.array_equal(scores, ws), i


@pytest.fixture(scope="module")
def c5_run(lib):
    """64 u8 1280x720 frames through upload -> run_staged, default mode and batch-invariant mode."""
    rng = np.random.default_rng(7200)
    frames = rng.integers(0, 256, (C5_N, H, W, 3), dtype=np.uint8)
    Wt = _weights(case_weights("posenet", 0))
    limits = lib.OpLimits()
    limits.max_batch = C5_N
    c = lib.Context(0, None, limits)
    out = {"frames": frames, "W": Wt}
    try:
        c.set_weights(Wt)
        pinned = lib.PinnedFrames(C5_N, H, W)
        try:
            pinned.array[:] = frames
            for inv in (False, True):
                c.set_batch_invariant(inv)
                c.upload_frames(pinned.array)
                lib.conv_census(reset=True)
                c.run_staged()
                c.synchronize()
                out["census", inv] = lib.conv_census(reset=True)
                out["maps", inv] = c.fetch_maps(0, C5_N)
                if not inv:
                    out["res"] = [_result(lambda i=i: c.fetch_result(i)) for i in (0, 31, C5_N - 1)]
        finally:
            c.set_batch_invariant(False)
            pinned.close()
    finally:
        c.close()
    return out


def test_c5_default_mode_no_split_k_and_equals_invariant(c5_run):
    cen = c5_run["census", False]
    print("C5 default-mode census:", cen)
    assert cen["npx"] == {10: 25}, cen
    assert cen["7x7_splitk"] == 0 and cen["3x3_splitk"] == 0, cen  # the bench's own launches
    (p, h), (pi, hi) = c5_run["maps", False], c5_run["maps", True]
    assert np.array_equal(p, pi) and np.array_equal(h, hi)


@pytest.mark.parametrize("k,i", [(0, 0), (1, 31), (2, C5_N - 1)])
def test_c5_default_mode_vs_oracle(c5_run, k, i):
    net_w, net_h = cvresize.compute_optimal_size(H, W, 368)
    x = cvresize.preprocess(cvresize.resize_linear_u8(c5_run["frames"][i], net_w, net_h))
    opaf, oheat = F.cocoposenet_forward(c5_run["W"], x)
    paf, heat = c5_run["maps", False]
    e = max(_max_err(paf[i], opaf[0]), _max_err(heat[i], oheat[0]))
    print("C5 default mode frame %d vs oracle: %.3g" % (i, e))
    assert e <= TOL, (i, e)
    # the post-process (pose_detector.py:501-517) of this frame's GPU maps, bit for bit
    got = c5_run["res"][k]
    try:
        wp, ws = P.postprocess(paf[i], heat[i], H, W)
    except IndexError:
        assert got is IndexError
        return
    poses, scores, r = got
    assert np.array_equal(np.asarray(poses).reshape(wp.shape), wp) and np.array_equal(scores, ws), i


def test_one_frame_pooled_split_k(lib, rand_weights):
    """Advisor r04: one 368x368 frame's pooled 3x3 launches (conv2_2, conv3_4) split K in the default
    mode through conv_m16_splitk_reduce_pool.  Census: 3x3_pool and 3x3_splitk launches ran; the
    maps stay within REL_SPLIT (relative to the map's largest magnitude) of the unsplit batch-invariant
    run -- the two differ only by the f32 re-association of the channel sums -- and a replayed
    hipGraph of the staged step gives the eager bits."""
    rng = np.random.default_rng(55)
    frame = rng.integers(0, 256, (1, 368, 368, 3), dtype=np.uint8)
    c = lib.Context(0)
    try:
        c.set_weights(rand_weights)
        c.stage_frames(frame)
        lib.conv_census(reset=True)
        c.run_staged()
        c.synchronize()
        cen = lib.conv_census(reset=True)
        print("one frame census:", cen)
        assert cen["3x3_pool"] >= 1 and cen["3x3_splitk"] >= 1, cen
        eager = c.fetch_maps(0, 1)
        c.run_staged(graph=True)
        c.synchronize()
        c.run_staged(graph=True)
        c.synchronize()
        graph = c.fetch_maps(0, 1)
        assert np.array_equal(graph[0], eager[0]) and np.array_equal(graph[1], eager[1])
        c.set_batch_invariant(True)
        try:
            lib.conv_census(reset=True)  # (the graph captures above counted their launches)
            c.run_staged()
            c.synchronize()
            cen_i = lib.conv_census(reset=True)
            inv = c.fetch_maps(0, 1)
        finally:
            c.set_batch_invariant(False)
        assert cen_i["3x3_splitk"] == 0 and cen_i["7x7_splitk"] == 0, cen_i
        for a, b in zip(eager, inv):
            scale = max(float(np.abs(b).max()), 1e-6)
            rel = _max_err(a, b) / scale
            print("pooled split-K vs unsplit: rel %.3g (scale %.3g)" % (rel, scale))
            assert rel <= REL_SPLIT, rel
    finally:
        c.close()
