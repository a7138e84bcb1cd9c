"""The HIP forward (through the C ABI) against fixtures made by running the REFERENCE's own
models/CocoPoseNet.py / FaceNet.py / HandNet.py __init__ + __call__ (make_golden_forward.py).

Tolerance: the north star's 1e-3 absolute on the maps (BASELINE.json), in both conv precisions
(bf16x3 and exact f32); every one of the six stage outputs for the cases that store them."""
import numpy as np
import pytest

from conftest import pkg_module
from test_forward_golden import CASES, case_weights, load_case

pytestmark = pytest.mark.gpu
TOL = 1e-3
POSE = [c for c in CASES if c.startswith("posenet")]


@pytest.fixture(scope="module")
def pose_ctx():
    lib = pkg_module("_lib")
    c = lib.Context(0)
    c.set_weights(case_weights("posenet", 0))
    yield c
    c.close()


@pytest.mark.parametrize("prec", ["bf16x3", "fp32"])
@pytest.mark.parametrize("name", POSE)
def test_forward_vs_reference_fixture(pose_ctx, name, prec):
    _, d = load_case(name)
    assert int(d["weight_seed"]) == 0
    pose_ctx.set_precision(prec)
    try:
        paf, heat = pose_ctx.forward(d["x"])
    finally:
        pose_ctx.set_precision("bf16x3")
    err = max(float(np.abs(paf - d["paf"]).max()), float(np.abs(heat - d["heat"]).max()))
    assert err <= TOL, (name, prec, err)


@pytest.mark.parametrize("prec", ["bf16x3", "fp32"])
@pytest.mark.parametrize("name", POSE)
def test_forward_every_stage_vs_reference_fixture(pose_ctx, name, prec):
    """op_forward_stages: the six (paf, heat) pairs CocoPoseNet.__call__ returns."""
    _, d = load_case(name)
    pose_ctx.set_precision(prec)
    try:
        pafs, heats = pose_ctx.forward_stages(d["x"])
        last_paf, last_heat = pose_ctx.forward(d["x"])
    finally:
        pose_ctx.set_precision("bf16x3")
    np.testing.assert_array_equal(pafs[-1], last_paf)
    np.testing.assert_array_equal(heats[-1], last_heat)
    if "paf_stages" in d:
        for s in range(6):
            e = max(float(np.abs(pafs[s] - d["paf_stages"][s]).max()),
                    float(np.abs(heats[s] - d["heat_stages"][s]).max()))
            assert e <= TOL, (name, prec, s + 1, e)
    sums = np.array([[np.float64(p).sum(), np.float64(h).sum(), np.abs(np.float64(p)).sum(),
                      np.abs(np.float64(h)).sum()] for p, h in zip(pafs, heats)])
    n_el = np.array([pafs[0].size, heats[0].size] * 2, np.float64)
    # per-stage means within the tolerance (a wiring error moves these by O(0.1))
    assert float(np.abs((sums - d["stage_sums"]) / n_el).max()) <= TOL, name


@pytest.mark.parametrize("name", [c for c in CASES if not c.startswith("posenet")])
def test_cpm_forward_vs_reference_fixture(name):
    arch, d = load_case(name)
    lib = pkg_module("_lib")
    c = lib.CpmContext(arch, 0)
    try:
        c.set_weights(case_weights(arch, int(d["weight_seed"])))
        maps = c.forward(d["x"])
    finally:
        c.close()
    err = float(np.abs(maps - d["maps"]).max())
    assert err <= TOL, (name, err)
