"""The whole-depth register-weight 7x7 experiment conv_m16w_bf16x3 (round 5, VERDICT r04 item 3;
csrc/conv_m16w.hip, opt-in OP_M16W=1): weights streamed from L2 into registers, a double-buffered
LDS halo of each chunk pair, one barrier per pair.  Held to the reference-network fixture
posenet_1x368x368 (tests/golden/make_golden_forward.py runs the reference's models/CocoPoseNet.py)
at the north star's 1e-3 for both tile heights, at one frame and inside a 38-frame batch (fixture
frames at both ends and the middle), on the default chunk-planar stage tensors and the plain ones."""
import numpy as np
import pytest

from conftest import pkg_module
from test_forward_golden import case_weights, load_case

pytestmark = pytest.mark.gpu
TOL = 1e-3


@pytest.fixture(scope="module")
def lib():
    return pkg_module("_lib")


@pytest.fixture(scope="module")
def wctx(lib):
    c = lib.Context(0)
    c.set_weights(case_weights("posenet", 0))
    yield c
    c.close()


@pytest.mark.parametrize("n,tr,planar", [(1, "4", 1), (1, "8", 0), (38, "4", 1), (38, "8", 1)])
def test_vs_reference_fixture(lib, wctx, monkeypatch, n, tr, planar):
    _, d = load_case("posenet_1x368x368")
    rng = np.random.default_rng(38 + n)
    x = rng.uniform(-0.5, 0.5, (n, 3, 368, 368)).astype(np.float32)
    at = sorted({0, n // 2, n - 1})
    for i in at:
        x[i] = d["x"][0]
    monkeypatch.setenv("OP_M16W", "1")
    monkeypatch.setenv("OP_M16W_TR", tr)
    wctx.set_stage_layout(planar)
    try:
        lib.conv_census(reset=True)
        paf, heat = wctx.forward(x)
        cen = lib.conv_census(reset=True)
    finally:
        wctx.set_stage_layout(1)
    assert cen["npx"] == {} and cen["7x7_q"] == 0, cen  # no 7x7 launch on conv_m16 / conv_m16q
    for i in at:
        e = max(float(np.abs(paf[i] - d["paf"][0]).max()), float(np.abs(heat[i] - d["heat"][0]).max()))
        print("n %d TR %s planar %d frame %d vs reference fixture: %.3g" % (n, tr, planar, i, e))
        assert e <= TOL, (i, e)
