"""Parity at the configurations the bench itself runs (VERDICT r02 "next" item 1).

The 7x7 stage kernel picks its raster-tile size per launch shape (conv_big.hip cost model): one
frame -> NPX 2, 16 frames -> 5, 38, 114 and 232 frames -> NPX 10 (640-px tiles; 232 frames = six
full rounds per launch), 57 frames -> NPX 8.  The headline (bench.py, 232 frames of 368x368 per step
since round 3's last A/B; 114 before) and
the C4 line (16 frames of 1280x720) therefore run instantiations that batch <= 16 tests never reach.
Here, at those exact batches:

* every frame's maps are compared BIT-EXACT with a single-frame run of the same frame: tile size
  and batch position must not change any pixel's accumulation order (batch-invariant mode only
  turns split-K off, which launches this large never use -- asserted below by comparing the
  default mode's maps with the invariant ones);
* frames at the start, the end and the middle of the batch (raster tiles cross every frame border
  but frame 0's start, so the middle frame's first and last pixels sit in tiles shared with its
  neighbours) are held to the reference-network fixture `posenet_1x368x368` (made by running the
  reference's own models/CocoPoseNet.py:132-262, tests/golden/make_golden_forward.py) at the north
  star's 1e-3, and on the bench's own u8 path to the CPU oracle at 1e-3;
* op_conv_census proves which 7x7 instantiation ran.
"""
import numpy as np
import pytest

from conftest import pkg_module
from oracle import cvresize
from oracle import forward as F
from test_forward_golden import case_weights, load_case

pytestmark = pytest.mark.gpu
TOL = 1e-3
SIDE = 368


@pytest.fixture(scope="module")
def lib():
    return pkg_module("_lib")


@pytest.fixture(scope="module")
def bctx(lib):
    c = lib.Context(0)
    c.set_weights(case_weights("posenet", 0))
    yield c
    c.close()


def _census_npx(lib):
    return lib.conv_census(reset=True)


def _max_err(a, b):
    return float(np.abs(np.float64(a) - np.float64(b)).max())


@pytest.mark.parametrize("n,npx", [(38, 10), (57, 8), (114, 10), (232, 10)])
def test_forward_at_bench_batches_vs_fixture_and_single_frames(lib, bctx, n, npx):
    """Both kernel sets at the bench's batches: conv algo 5 (conv_m16 raster tap pairs with NPX-block
    tiles, conv_m16k) and the default 4 (large 3x3 launches on the register-weight kernel
    conv_m16r).  Every frame of both == that frame alone, bit for bit; the fixture frames <= 1e-3
    from the reference network's own output."""
    _, d = load_case("posenet_1x368x368")
    xf = d["x"][0]
    rng = np.random.default_rng(n)
    x = rng.uniform(-0.5, 0.5, (n, 3, SIDE, SIDE)).astype(np.float32)
    mid = n // 2
    fixture_at = (0, mid, n - 1)
    for i in fixture_at:
        x[i] = xf
    bctx.set_batch_invariant(True)
    try:
        bctx.set_conv_algo(5)
        try:
            _census_npx(lib)
            paf, heat = bctx.forward(x)
            cen = _census_npx(lib)
        finally:
            bctx.set_conv_algo(4)
        # every 7x7 launch of this batch ran the NPX instantiation the cost model picks for it
        assert set(cen["npx"]) == {npx}, cen
        assert cen["npx"][npx] == 5 * 5 and cen["7x7_splitk"] == 0, cen  # 5 stages x Mconv1..5
        for i in fixture_at:
            e = max(_max_err(paf[i], d["paf"][0]), _max_err(heat[i], d["heat"][0]))
            print("batch %d frame %d vs reference fixture: %.3g" % (n, i, e))
            assert e <= TOL, (n, i, e)
        # frames holding the same input agree bit for bit wherever they sit in the batch
        for i in fixture_at[1:]:
            assert np.array_equal(paf[i], paf[0]) and np.array_equal(heat[i], heat[0]), i
        # the default kernels (the register-weight 3x3 on the large launches): the same bits
        _census_npx(lib)
        paf4, heat4 = bctx.forward(x)
        cen4 = _census_npx(lib)
        print("batch %d default kernels:" % n, cen4)
        assert cen4["npx"] == {npx: 25}, cen4
        if n >= 57:
            assert cen4["3x3_r128"] + cen4["3x3_r_pool"] >= 8, cen4
        assert np.array_equal(paf4, paf) and np.array_equal(heat4, heat)
        # every frame == the same frame run alone (NPX 2 tiles, one frame per launch)
        for i in range(n):
            p1, h1 = bctx.forward(x[i:i + 1])
            assert np.array_equal(paf[i], p1[0]) and np.array_equal(heat[i], h1[0]), (n, i)
    finally:
        bctx.set_batch_invariant(False)
    # the default mode (what bench.py runs) gives the same bits at this batch: no split-K here
    _census_npx(lib)
    paf_d, heat_d = bctx.forward(x)
    cen = _census_npx(lib)
    assert cen["7x7_splitk"] == 0, cen
    assert np.array_equal(paf_d, paf) and np.array_equal(heat_d, heat)


@pytest.mark.parametrize("n", [114, 232])
def test_staged_u8_path_at_the_headline_batch(lib, bctx, n):
    """bench.py's own path and batch: n u8 368x368 frames (232: the headline's batch; 114: round 3's
    earlier one) through upload -> run_staged (fused cv2-LINEAR resize + preprocess inside the conv1
    pair, 92 convs, post-process)."""
    rng = np.random.default_rng(n)
    frames = rng.integers(0, 256, (n, SIDE, SIDE, 3), dtype=np.uint8)
    bctx.set_batch_invariant(True)
    try:
        pinned = lib.PinnedFrames(n, SIDE, SIDE)
        try:
            pinned.array[:] = frames
            bctx.upload_frames(pinned.array)
            _census_npx(lib)
            bctx.run_staged()
            bctx.synchronize()
            cen = _census_npx(lib)
            paf, heat = bctx.fetch_maps(0, n)
        finally:
            pinned.close()
        assert set(cen["npx"]) == {10} and cen["npx"][10] == 25, cen
        assert cen["conv1_pair"] == 1 and cen["3x3_splitk"] == 0, cen
        # the register-weight 3x3 kernel runs the large 3x3 launches of this batch (bit-identical to
        # conv_m16k, which the single-frame runs below take: asserted by the per-frame comparison)
        assert cen["3x3_r256"] + cen["3x3_r128"] + cen["3x3_r_pool"] >= 8, cen
        assert paf.shape == (n, 38, 46, 46) and heat.shape == (n, 19, 46, 46)
        # a border-spanning frame in the middle, and the two ends, against the CPU oracle
        W = case_weights("posenet", 0)
        for i in (0, n // 2, n - 1):
            x = cvresize.preprocess(cvresize.resize_linear_u8(frames[i], SIDE, SIDE))
            opaf, oheat = F.cocoposenet_forward(W, x)
            e = max(_max_err(paf[i], opaf[0]), _max_err(heat[i], oheat[0]))
            print("staged batch %d frame %d vs oracle: %.3g" % (n, i, e))
            assert e <= TOL, (i, e)
        # each frame == that frame staged alone
        for i in range(n):
            bctx.stage_frames(frames[i:i + 1])
            bctx.run_staged()
            bctx.synchronize()
            p1, h1 = bctx.fetch_maps(0, 1)
            assert np.array_equal(paf[i], p1[0]) and np.array_equal(heat[i], h1[0]), i
    finally:
        bctx.set_batch_invariant(False)


def test_c5_stream_batch_of_64_720p_frames(lib, bctx):
    """C5's own bench configuration (bench.py --frame 720x1280: 64 u8 1280x720 frames per step,
    single scale, net 656x368, maps 82x46 -> 576x320): upload -> run_staged.  The 7x7 launches run
    NPX 10 batch-raster tiles on the 82-column maps (3772 px per frame: tiles cross frame borders
    mid-row; conv_big.hip raster_tiling), which no single frame and no 368x368 batch reaches.

    * op_conv_census: every 7x7 launch is conv_m16_bf16x3<7, 10> on batch rasters (not
      frame-aligned), no split-K;
    * every frame == that frame staged alone, bit for bit;
    * frames 0, 31 (its first rows share a tile with frame 30's last: the tile starts at pixel
      116480 = frame 30 row 40 col 40) and 63 <= 1e-3 vs the CPU oracle on the same u8 path
      (cv2-LINEAR resize, preprocess, the reference network's forward, models/CocoPoseNet.py:132-262);
    * with the reference-generated twenty_720p maps staged for all 64 frames (what the bench's
      post-process reads), every frame's 576x320 post-process == the golden poses and scores bit for
      bit (pose_detector.py:484-517)."""
    from conftest import load_golden
    n, H, Wd = 64, 720, 1280
    net_w, net_h = cvresize.compute_optimal_size(H, Wd, SIDE)
    assert (net_w, net_h) == (656, 368)
    rng = np.random.default_rng(720)
    frames = rng.integers(0, 256, (n, H, Wd, 3), dtype=np.uint8)
    bctx.set_batch_invariant(True)
    try:
        pinned = lib.PinnedFrames(n, H, Wd)
        try:
            pinned.array[:] = frames
            bctx.upload_frames(pinned.array)
            _census_npx(lib)
            bctx.run_staged()
            bctx.synchronize()
            cen = _census_npx(lib)
            paf, heat = bctx.fetch_maps(0, n)
        finally:
            pinned.close()
        print("C5 batch 64 census:", cen)
        assert cen["npx"] == {10: 25} and cen["7x7_splitk"] == 0, cen
        assert cen["7x7_frame_aligned"] == 0, cen  # batch rasters: tiles cross frame borders
        assert cen["7x7_planar"] == 25, cen
        assert paf.shape == (n, 38, 46, 82) and heat.shape == (n, 19, 46, 82)
        W = case_weights("posenet", 0)
        for i in (0, 31, n - 1):
            x = cvresize.preprocess(cvresize.resize_linear_u8(frames[i], net_w, net_h))
            opaf, oheat = F.cocoposenet_forward(W, x)
            e = max(_max_err(paf[i], opaf[0]), _max_err(heat[i], oheat[0]))
            print("C5 batch frame %d vs oracle: %.3g" % (i, e))
            assert e <= TOL, (i, e)
        for i in range(n):
            bctx.stage_frames(frames[i:i + 1])
            _census_npx(lib)
            bctx.run_staged()
            bctx.synchronize()
            assert 10 not in _census_npx(lib)["npx"]  # the lone frame runs other tiles
            p1, h1 = bctx.fetch_maps(0, 1)
            assert np.array_equal(paf[i], p1[0]) and np.array_equal(heat[i], h1[0]), i
    finally:
        bctx.set_batch_invariant(False)
    # the bench's post-process input: the twenty_720p maps staged for every frame of the batch
    d = load_golden("twenty_720p")
    assert (int(d["orig_h"]), int(d["orig_w"])) == (H, Wd) and (int(d["map_h"]), int(d["map_w"])) == (320, 576)
    maps = np.ascontiguousarray(np.concatenate([d["paf_low"], d["heat_low"]])[None].repeat(n, axis=0))
    bctx.stage_frames(frames)
    bctx.stage_maps(maps)
    bctx.use_staged_maps(True)
    try:
        bctx.run_staged()
        bctx.synchronize()
        res = bctx.fetch_results(0, n)
    finally:
        bctx.use_staged_maps(False)
    assert len(res) == n
    for i, (p, s, r) in enumerate(res):
        assert r.map_w == 576 and r.map_h == 320 and r.n_peaks == len(d["all_peaks"]), i
        assert np.array_equal(np.asarray(p).reshape(d["poses"].shape), d["poses"]), i
        assert np.array_equal(s, d["scores"]), i


@pytest.mark.parametrize("n", [1, 16])
def test_precise_side_stream_bit_identical(lib, monkeypatch, n):
    """Round 6: detect_precise runs the scales whose padded input is at most a
    quarter of the largest's (0.5 and 1.0 at 1280x720) on a second stream, concurrent with the large
    ones; each scale has its own arena, d_pmid region and split-K workspace, so the averaged maps
    are bit-identical to every scale on the compute stream (OP_PRECISE_STREAMS=1), in the default
    (split-K) mode the C4 bench line runs, for the bench's 16 frames and one frame; the census
    counts the runs that forked."""
    from test_gpu_precise_full import _crowd_frame, _weights
    frames = np.stack([_crowd_frame(300 + i) for i in range(n)])
    c = lib.Context(0)
    try:
        c.set_weights(_weights(case_weights("posenet", 0)))
        out = {}
        for streams in ("1", "2", "2b"):
            monkeypatch.setenv("OP_PRECISE_STREAMS", streams[0])
            c.stage_frames(frames)
            _census_npx(lib)
            try:
                c.run_staged_precise()
            except IndexError:
                pass
            c.synchronize()
            cen = _census_npx(lib)
            assert cen["precise_side"] == (0 if streams == "1" else 1), (streams, cen)
            out[streams] = c.fetch_maps(0, n)
        monkeypatch.delenv("OP_PRECISE_STREAMS")
        for k in ("2", "2b"):
            for a, b in zip(out["1"], out[k]):
                assert np.array_equal(a, b), (k, float(np.abs(a - b).max()))
    finally:
        c.close()


def test_precise_staged_batch_of_16_equals_single_frames(lib):
    """The C4 line's batch (bench.py --precise: 16 frames of 1280x720, 4 scales): the per-scale
    batched forwards run NPX 8 / 10 tiles that one frame never reaches; every frame's averaged maps
    and poses == detect_precise of that frame alone (which test_gpu_precise_full.py holds to the
    oracle at 1280x720 on frame 0's image)."""
    from test_gpu_precise_full import _crowd_frame, _weights
    n, H, W = 16, 720, 1280
    frames = np.stack([_crowd_frame(7)] + [_crowd_frame(100 + i) for i in range(n - 1)])
    limits = lib.OpLimits()
    limits.max_peaks_per_joint = 2048
    c = lib.Context(0, None, limits)
    try:
        c.set_weights(_weights(case_weights("posenet", 0)))
        c.set_batch_invariant(True)
        c.stage_frames(frames)
        _census_npx(lib)
        c.run_staged_precise()
        c.synchronize()
        cen = _census_npx(lib)
        print("C4 batch 16 7x7 tiles:", cen["npx"])
        assert max(cen["npx"]) >= 8, cen  # the large tiles a lone frame never uses
        paf, heat = c.fetch_maps(0, n)
        assert paf.shape == (n, 38, H, W)

        def result(fetch):
            try:
                return fetch()
            except IndexError:  # the reference's grouping quirk (pose_detector.py:197)
                return IndexError

        got = [result(lambda i=i: c.fetch_result(i)) for i in range(n)]
        for i in range(n):
            try:
                poses, scores, res, p1, h1 = c.detect_precise(frames[i], return_maps=True)
                single = (poses, scores)
            except IndexError as e:
                p1, h1 = e.maps
                single = IndexError
            assert np.array_equal(paf[i], p1) and np.array_equal(heat[i], h1), i
            if single is IndexError or got[i] is IndexError:
                assert single is got[i], i
            else:
                assert np.array_equal(got[i][0], single[0]) and np.array_equal(got[i][1], single[1]), i
    finally:
        c.close()


@pytest.mark.parametrize("n", [1, 38])
def test_planar_stage_layout_is_bit_identical(lib, bctx, n):
    """op_set_stage_layout: the 7x7 stage tensors of stages 2-6 in the chunk-planar layout (the
    default; conv_m16 halo loads as contiguous runs) or [row][col][channels] -- the same kernels
    and accumulation order, so the maps agree bit for bit; the census shows which layout ran."""
    rng = np.random.default_rng(500 + n)
    x = rng.uniform(-0.5, 0.5, (n, 3, SIDE, SIDE)).astype(np.float32)
    out = {}
    for planar in (1, 0):
        bctx.set_stage_layout(planar)
        try:
            _census_npx(lib)
            out[planar] = bctx.forward(x)
            cen = _census_npx(lib)
        finally:
            bctx.set_stage_layout(1)
        assert cen["7x7_planar"] == (25 if planar else 0), (planar, cen)
    assert np.array_equal(out[1][0], out[0][0]) and np.array_equal(out[1][1], out[0][1])


@pytest.mark.parametrize("n", [1, 38, 232])
def test_staggered_halves_bit_identical(lib, bctx, monkeypatch, n):
    """Round 5: the 7x7 kernel's staggered halves (waves 0-3 meet the ring barrier at a pair's start,
    waves 4-7 in its middle; OP_M16_STAG=0 restores one barrier per pair for all 8 waves) move only
    when each wave waits, not what it accumulates: the maps are bit-identical at 38 and the
    headline's 232 frames and at one frame (split-K tiles on the deep 12-tap ring); the census shows
    which ring ran."""
    rng = np.random.default_rng(900 + n)
    x = rng.uniform(-0.5, 0.5, (n, 3, SIDE, SIDE)).astype(np.float32)
    monkeypatch.setenv("OP_M16Q", "0")  # one frame: conv_m16's split-K tiles, not conv_m16q
    out = {}
    for stag in ("1", "0"):
        monkeypatch.setenv("OP_M16_STAG", stag)
        _census_npx(lib)
        out[stag] = bctx.forward(x)
        cen = _census_npx(lib)
        print("n %d OP_M16_STAG=%s census:" % (n, stag), cen)
        if stag == "1":
            assert cen["7x7_stag"] == 25, cen  # one frame: the deep 12-tap ring, staggered too
        else:
            assert cen["7x7_stag"] == 0 and cen["7x7_plain_ring"] == 25, cen
    monkeypatch.delenv("OP_M16_STAG")
    for a, b in zip(out["1"], out["0"]):
        assert np.array_equal(a, b), float(np.abs(a - b).max())


@pytest.mark.parametrize("n", [38, 232])
def test_circular_halo_bit_identical(lib, bctx, monkeypatch, n):
    """Round 6: the staggered 7x7 kernel with circular halo planes (conv_m16.hip CIRC: tiles of one
    frame stream the next chunk's halo in the background instead of draining at every chunk
    boundary; OP_M16_CIRC=0 keeps the drain) changes where a chunk's halo sits in LDS and when it is
    loaded, not what any MFMA reads: the maps are bit-identical to the drained kernel at 38 frames
    and at the headline's 232, and the census shows the circular kernel ran every 7x7 launch."""
    rng = np.random.default_rng(700 + n)
    x = rng.uniform(-0.5, 0.5, (n, 3, SIDE, SIDE)).astype(np.float32)
    out = {}
    for circ in ("1", "0"):
        monkeypatch.setenv("OP_M16_CIRC", circ)
        _census_npx(lib)
        out[circ] = bctx.forward(x)
        cen = _census_npx(lib)
        print("n %d OP_M16_CIRC=%s census:" % (n, circ), cen)
        assert cen["7x7_stag"] == 25, cen
        assert cen["7x7_circ"] == (25 if circ == "1" else 0), cen
    monkeypatch.delenv("OP_M16_CIRC")
    for a, b in zip(out["1"], out["0"]):
        assert np.array_equal(a, b), float(np.abs(a - b).max())


@pytest.mark.parametrize("n", [38, 232])
def test_linear_halo_sources_bit_identical(lib, bctx, monkeypatch, n):
    """Round 6: the staggered 7x7 kernel with linear halo sources (conv_m16.hip LIN: on chunk-planar
    input with the tight pitch a halo slot's source pixel is one linear index; OP_M16_LIN=0 keeps the
    row / column cursor), with the halo trimmed to a tile's own rows (OP_M16_TRIM) and as a
    persistent grid (PERS, OP_M16_PERS) loads the same pixels into the slots the MFMAs read: the maps
    are bit-identical at 38 frames and at the headline's 232, and the census shows LIN ran every 7x7
    launch."""
    rng = np.random.default_rng(500 + n)
    x = rng.uniform(-0.5, 0.5, (n, 3, SIDE, SIDE)).astype(np.float32)
    out = {}
    # trim: only a tile's own halo rows loaded; pers: a persistent grid of one workgroup per CU
    for lin, trim, pers in (("1", "1", "1"), ("1", "1", "0"), ("1", "0", "0"), ("0", "0", "0")):
        monkeypatch.setenv("OP_M16_LIN", lin)
        monkeypatch.setenv("OP_M16_TRIM", trim)
        monkeypatch.setenv("OP_M16_PERS", pers)
        _census_npx(lib)
        out[lin + trim + pers] = bctx.forward(x)
        cen = _census_npx(lib)
        print("n %d OP_M16_LIN=%s OP_M16_TRIM=%s OP_M16_PERS=%s census:" % (n, lin, trim, pers), cen)
        assert cen["7x7_stag"] == 25, cen
        assert cen["7x7_lin"] == (25 if lin == "1" else 0), cen
        if pers == "1" and n == 232:  # launches of more than one round (38 frames: 252 workgroups)
            assert cen["7x7_pers"] == 25, cen
    for k in ("OP_M16_LIN", "OP_M16_TRIM", "OP_M16_PERS"):
        monkeypatch.delenv(k)
    for k in ("111", "110", "100"):
        for a, b in zip(out[k], out["000"]):
            assert np.array_equal(a, b), (k, float(np.abs(a - b).max()))


def test_staggered_halves_precise_720p(lib, monkeypatch):
    """The staggered 7x7 halves on the multi-scale path's wide maps (41- to 164-column maps, halo
    planes up to 32 KiB, frame-aligned and tight-pitch raster tiles): 2 frames of 1280x720 through
    run_staged_precise give bit-identical averaged maps with OP_M16_STAG=1 and 0."""
    from test_gpu_precise_full import _crowd_frame, _weights
    frames = np.stack([_crowd_frame(41), _crowd_frame(42)])
    monkeypatch.setenv("OP_M16Q", "0")  # the smallest scale's launch (<= 4800 px) stays on conv_m16
    c = lib.Context(0)
    try:
        c.set_weights(_weights(case_weights("posenet", 0)))
        out = {}
        for stag in ("1", "0", "circ0"):  # circ0: staggered, the circular halo off (round 6)
            monkeypatch.setenv("OP_M16_STAG", "1" if stag == "circ0" else stag)
            monkeypatch.setenv("OP_M16_CIRC", "0" if stag == "circ0" else "1")
            c.stage_frames(frames)
            _census_npx(lib)
            try:
                c.run_staged_precise()
            except IndexError:
                pass
            c.synchronize()
            cen = _census_npx(lib)
            if stag == "1":  # the launches whose halo planes fit 28 KiB (and every deep-ring launch)
                assert cen["7x7_stag"] > 0 and cen["7x7_circ"] > 0, cen
            elif stag == "circ0":
                assert cen["7x7_stag"] > 0 and cen["7x7_circ"] == 0, cen
            else:
                assert cen["7x7_stag"] == 0 and cen["7x7_plain_ring"] == 4 * 25, cen
            out[stag] = c.fetch_maps(0, 2)
        monkeypatch.delenv("OP_M16_STAG")
        monkeypatch.delenv("OP_M16_CIRC")
        # round 6: linear halo sources, trimmed halos and the persistent grid on these wide maps too
        # (frame-aligned tiles on the unstaggered ring included)
        for k, v in (("OP_M16_LIN", "1"), ("OP_M16_TRIM", "1"), ("OP_M16_PERS", "1")):
            monkeypatch.setenv(k, v)
        c.stage_frames(frames)
        _census_npx(lib)
        try:
            c.run_staged_precise()
        except IndexError:
            pass
        c.synchronize()
        cen = _census_npx(lib)
        assert cen["7x7_lin"] > 0, cen  # (2 frames: every launch within one round, so no PERS grid)
        out["lin"] = c.fetch_maps(0, 2)
        for k in ("OP_M16_LIN", "OP_M16_TRIM", "OP_M16_PERS"):
            monkeypatch.delenv(k)
        for other in ("0", "circ0", "lin"):
            for a, b in zip(out["1"], out[other]):
                assert np.array_equal(a, b), (other, float(np.abs(a - b).max()))
    finally:
        c.close()
