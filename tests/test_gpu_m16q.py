"""The small-launch 7x7 kernel conv_m16q_bf16x3 (round 5, VERDICT r04 item 4: batch-1 latency;
csrc/conv_m16q.hip): one 368x368 frame's Mconv1..5 (46 x 46 maps, models/CocoPoseNet.py:167-260)
split K over (chunk pair, tap range) across 4-wave workgroups, f32 partials summed in split order
by conv_m16_splitk_reduce.  It runs only where split-K is allowed (never in batch-invariant mode)
on launches of <= 4800 pixels.

* census: every 7x7 launch of a one-frame forward is conv_m16q (slot 7x7_q), none of conv_m16's
  raster instantiations, and none in batch-invariant mode;
* the reference-network fixture posenet_1x368x368 (made by running the reference's own
  models/CocoPoseNet.py, tests/golden/make_golden_forward.py) at the north star's 1e-3, for every
  instantiated tile height (2 / 4 / 8 rows), tap-range count (2 / 3 / 4) and prefetch (2 / 4);
* the maps differ from conv_m16's split-K run (OP_M16Q=0) only by the re-association of the f32
  channel sums (REL, relative to the map scale: the bf16 hi/lo storage of ~40 later layers);
* two frames in one launch (4232 pixels) vs each frame alone (within REL: the small 3x3
  launches' split-K factors depend on the batch); a replayed hipGraph == eager;
* a non-square map (23 x 25: partial column and row tiles) vs the CPU oracle.
"""
import numpy as np
import pytest

from conftest import pkg_module
from oracle import forward as F
from test_forward_golden import case_weights, load_case

pytestmark = pytest.mark.gpu
TOL = 1e-3
REL = 1e-4


@pytest.fixture(scope="module")
def lib():
    return pkg_module("_lib")


@pytest.fixture(scope="module")
def qctx(lib):
    c = lib.Context(0)
    c.set_weights(case_weights("posenet", 0))
    yield c
    c.close()


def _max_err(a, b):
    return float(np.abs(np.float64(a) - np.float64(b)).max())


def _fixture():
    _, d = load_case("posenet_1x368x368")
    return d["x"][:1].astype(np.float32), d["paf"][0], d["heat"][0]


@pytest.mark.parametrize("tr,nth,pf,iwg", [("4", "2", "2", "1"), ("4", "2", "2", "0"), ("2", "2", "2", "1"),
                                           ("8", "2", "2", "1"), ("4", "3", "2", "1"), ("4", "4", "2", "1"),
                                           ("4", "2", "4", "1")])
def test_one_frame_vs_reference_fixture(lib, qctx, monkeypatch, tr, nth, pf, iwg):
    """Every instantiation, incl. round 6's opt-in in-workgroup tap ranges (TR 4, 2 tap ranges in one
    8-wave workgroup, iwg 1; measured slower, OP_M16Q_IWG=1) and the default one workgroup per (chunk
    pair, tap range) (iwg 0)."""
    monkeypatch.setenv("OP_M16Q_TR", tr)
    monkeypatch.setenv("OP_M16Q_NTH", nth)
    monkeypatch.setenv("OP_M16Q_PF", pf)
    monkeypatch.setenv("OP_M16Q_IWG", iwg)
    x, want_paf, want_heat = _fixture()
    lib.conv_census(reset=True)
    paf, heat = qctx.forward(x)
    cen = lib.conv_census(reset=True)
    print("TR %s NTH %s census:" % (tr, nth), cen)
    assert cen["7x7_q"] == 25 and cen["npx"] == {}, cen  # 5 stages x Mconv1..5, all on conv_m16q
    # the in-workgroup sum is instantiated for TR 4, 2 tap ranges, prefetch 2; with 3 or 4 tap ranges
    # asked for, Mconv1 (6 chunk pairs: 18 / 24 splits > kMaxSplitK) falls back to 2 and takes it
    iwg_n = 25 if (tr, nth, pf, iwg) == ("4", "2", "2", "1") else 5 if (tr, pf, iwg) == ("4", "2", "1") else 0
    assert cen["7x7_q_iwg"] == iwg_n, cen
    e = max(_max_err(paf[0], want_paf), _max_err(heat[0], want_heat))
    print("TR %s NTH %s vs reference fixture: %.3g" % (tr, nth, e))
    assert e <= TOL, e


def test_b_prefetch_bit_identical(lib, qctx, monkeypatch):
    """Round 6 (OP_M16Q_BPF=1): the B fragments read one tap ahead into two register sets change when
    each LDS read is issued, not the MFMAs or their order: the one-frame maps are bit-identical to
    the default kernel's, within TOL of the reference fixture, and the census shows it ran every
    7x7 launch."""
    x, want_paf, want_heat = _fixture()
    out = {}
    for bpf in ("1", "0"):
        monkeypatch.setenv("OP_M16Q_BPF", bpf)
        lib.conv_census(reset=True)
        out[bpf] = qctx.forward(x)
        cen = lib.conv_census(reset=True)
        assert cen["7x7_q"] == 25 and cen["7x7_q_bpf"] == (25 if bpf == "1" else 0), cen
    for a, b in zip(out["1"], out["0"]):
        assert np.array_equal(a, b), _max_err(a, b)
    assert max(_max_err(out["1"][0][0], want_paf), _max_err(out["1"][1][0], want_heat)) <= TOL


def test_vs_conv_m16_split_k_and_invariant_mode(lib, qctx, monkeypatch):
    x, _, _ = _fixture()
    lib.conv_census(reset=True)
    q = qctx.forward(x)
    monkeypatch.setenv("OP_M16Q", "0")
    m = qctx.forward(x)
    cen = lib.conv_census(reset=True)
    assert cen["7x7_q"] == 25 and sum(cen["npx"].values()) == 25, cen  # 25 each way
    monkeypatch.delenv("OP_M16Q")
    for a, b in zip(q, m):
        rel = _max_err(a, b) / max(float(np.abs(b).max()), 1e-6)
        print("conv_m16q vs conv_m16 split-K: rel %.3g" % rel)
        assert rel <= REL, rel
    qctx.set_batch_invariant(True)
    try:
        lib.conv_census(reset=True)
        qctx.forward(x)
        cen = lib.conv_census(reset=True)
    finally:
        qctx.set_batch_invariant(False)
    assert cen["7x7_q"] == 0 and cen["7x7_splitk"] == 0, cen


def test_two_frames_vs_each_frame_alone(lib, qctx):
    """Two frames per launch (4232 pixels): conv_m16q's per-frame tiles and split order do not
    depend on the batch, but the small 3x3 launches' split-K factors do (conv_m16k), so each
    frame is held to its single-frame run within REL."""
    rng = np.random.default_rng(46)
    x = rng.uniform(-0.5, 0.5, (2, 3, 368, 368)).astype(np.float32)
    lib.conv_census(reset=True)
    paf, heat = qctx.forward(x)
    cen = lib.conv_census(reset=True)
    assert cen["7x7_q"] == 25, cen  # 2 x 2116 pixels per launch, still conv_m16q
    for i in range(2):
        p1, h1 = qctx.forward(x[i:i + 1])
        for a, b in ((paf[i], p1[0]), (heat[i], h1[0])):
            rel = _max_err(a, b) / max(float(np.abs(b).max()), 1e-6)
            assert rel <= REL, (i, rel)


def test_staged_graph_replay_equals_eager(lib, qctx):
    rng = np.random.default_rng(47)
    frame = rng.integers(0, 256, (1, 368, 368, 3), dtype=np.uint8)
    qctx.stage_frames(frame)
    lib.conv_census(reset=True)
    qctx.run_staged()
    qctx.synchronize()
    assert lib.conv_census(reset=True)["7x7_q"] == 25
    eager = qctx.fetch_maps(0, 1)
    for _ in range(2):
        qctx.run_staged(graph=True)
        qctx.synchronize()
    graph = qctx.fetch_maps(0, 1)
    assert np.array_equal(graph[0], eager[0]) and np.array_equal(graph[1], eager[1])


def test_partial_tiles_vs_oracle(lib, qctx):
    rng = np.random.default_rng(48)
    x = rng.uniform(-0.5, 0.5, (1, 3, 184, 200)).astype(np.float32)  # maps 23 x 25
    lib.conv_census(reset=True)
    paf, heat = qctx.forward(x)
    assert lib.conv_census(reset=True)["7x7_q"] == 25
    opaf, oheat = F.cocoposenet_forward(case_weights("posenet", 0), x)
    e = max(_max_err(paf, opaf), _max_err(heat, oheat))
    print("23 x 25 maps vs oracle: %.3g" % e)
    assert e <= TOL, e


def test_in_workgroup_tap_ranges_vs_split_tap_ranges(lib, qctx, monkeypatch):
    """Round 6: the two tap ranges of a chunk pair summed in LDS inside one workgroup (IWG, the
    default; split K = chunk pairs) vs round 5's separate workgroups per tap range (split K = chunk
    pairs x 2): the same products, the f32 sums re-associated, so within REL; deterministic."""
    x, _, _ = _fixture()
    out = {}
    for iwg in ("1", "0", "1"):
        monkeypatch.setenv("OP_M16Q_IWG", iwg)
        lib.conv_census(reset=True)
        r = qctx.forward(x)
        cen = lib.conv_census(reset=True)
        assert cen["7x7_q_iwg"] == (25 if iwg == "1" else 0), cen
        if iwg in out:
            for a, b in zip(r, out[iwg]):
                assert np.array_equal(a, b)  # run to run: the same bits
        out[iwg] = r
    monkeypatch.delenv("OP_M16Q_IWG")
    for a, b in zip(out["1"], out["0"]):
        rel = _max_err(a, b) / max(float(np.abs(b).max()), 1e-6)
        print("conv_m16q in-workgroup vs split tap ranges: rel %.3g" % rel)
        assert rel <= REL, rel
