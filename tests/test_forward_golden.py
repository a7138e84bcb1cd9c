"""The forward oracle against fixtures made by running the REFERENCE's own network definitions
(models/CocoPoseNet.py:23-262, models/FaceNet.py, models/HandNet.py) under op stubs
(tests/golden/make_golden_forward.py).  This pins the oracle's wiring -- layer table, ReLU
placement, pools, the concat order, all six stage outputs -- to the reference; the GPU tests then
compare the HIP path with the same fixtures (tests/test_gpu_forward_golden.py)."""
import glob
import os

import numpy as np
import pytest

from conftest import GOLDEN, pkg_module

FWD = os.path.join(GOLDEN, "forward")
CASES = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(FWD, "*.npz")))
_WCACHE = {}


def load_case(name):
    d = dict(np.load(os.path.join(FWD, name + ".npz")))
    arch = name.split("_")[0]
    if "x" not in d:
        n, h, w = (int(v) for v in name.split("_")[1].split("x"))
        d["x"] = np.random.default_rng(int(d["x_seed"])).uniform(-0.5, 0.5, (n, 3, h, w)).astype(np.float32)
        assert float(np.float64(d["x"]).sum()) == float(d["x_sum"]), "input generator changed"
    return arch, d


def case_weights(arch, seed):
    if (arch, seed) not in _WCACHE:
        _WCACHE[arch, seed] = pkg_module("weights").random_weights(seed=seed, arch=arch)
    return _WCACHE[arch, seed]


def test_fixture_set_complete():
    assert {"posenet_1x64x80", "posenet_2x48x48", "posenet_1x184x328", "posenet_1x368x368",
            "facenet_1x64x64", "handnet_1x64x64"} <= set(CASES)


@pytest.mark.parametrize("name", CASES)
def test_layer_table_is_reference(name):
    """nets.py tables (and the HIP library's own op_layer_info table) == the reference's
    Convolution2D declarations: names, order, Ci, Co, ksize, pad = ksize // 2."""
    arch, d = load_case(name)
    nets = pkg_module("nets")
    ref = [(str(n), int(s[0]), int(s[1]), int(s[2])) for n, s in zip(d["layer_names"], d["layer_shape"])]
    assert ref == [tuple(t) for t in nets.layers(arch)]
    assert all(int(s[3]) == int(s[2]) // 2 for s in d["layer_shape"])
    if arch == "posenet":
        from oracle import forward as F
        assert ref == [tuple(t) for t in F.LAYERS]
        assert ref == [tuple(t) for t in pkg_module("_lib").layer_table()]
    else:
        assert ref == [tuple(t) for t in pkg_module("_lib").cpm_layer_table(arch)]


@pytest.mark.parametrize("name", CASES)
def test_weights_generator_unchanged(name):
    arch, d = load_case(name)
    w = case_weights(arch, int(d["weight_seed"]))
    got = np.array([float(np.float64(w[n][0]).sum()) + float(np.float64(w[n][1]).sum()) for n in d["layer_names"]])
    np.testing.assert_array_equal(got, d["weights_checksum"])


def test_reference_trace_shape():
    """The reference's own call sequence: 92 convs / 3 pools / 5 concats of (38, 19, 128)."""
    _, d = load_case("posenet_1x64x80")
    ops = list(d["trace_op"])
    assert ops.count("conv") == 92 and ops.count("pool") == 3
    cats = [a for o, a in zip(d["trace_op"], d["trace_arg"]) if o == "concat"]
    assert cats == ["38,19,128"] * 5
    # no ReLU directly after conv5_5_CPM_L* / Mconv7_* (CocoPoseNet.py:158,163,...)
    convs = [(i, a) for i, (o, a) in enumerate(zip(d["trace_op"], d["trace_arg"])) if o == "conv"]
    for i, a in convs:
        nxt = d["trace_op"][i + 1] if i + 1 < len(ops) else ""
        last = a.startswith("conv5_5") or a.startswith("Mconv7")
        assert (nxt == "relu") != last, a


@pytest.mark.parametrize("name", [c for c in CASES if c.startswith("posenet")])
def test_oracle_forward_matches_reference_wiring(name):
    """oracle.forward.cocoposenet_forward == the reference's own CocoPoseNet.__call__ (same ops,
    so equal to f32 rounding of identical operation sequences: bit-exact)."""
    from oracle import forward as F
    arch, d = load_case(name)
    w = case_weights(arch, int(d["weight_seed"]))
    pafs, heats = F.cocoposenet_forward(w, d["x"], all_stages=True)
    np.testing.assert_array_equal(pafs[-1], d["paf"])
    np.testing.assert_array_equal(heats[-1], d["heat"])
    if "paf_stages" in d:
        np.testing.assert_array_equal(np.stack(pafs), d["paf_stages"])
        np.testing.assert_array_equal(np.stack(heats), d["heat_stages"])
    sums = np.array([[np.float64(p).sum(), np.float64(h).sum(), np.abs(np.float64(p)).sum(),
                      np.abs(np.float64(h)).sum()] for p, h in zip(pafs, heats)])
    np.testing.assert_array_equal(sums, d["stage_sums"])


@pytest.mark.parametrize("name", [c for c in CASES if not c.startswith("posenet")])
def test_oracle_cpm_matches_reference_wiring(name):
    from oracle import cpm
    arch, d = load_case(name)
    w = case_weights(arch, int(d["weight_seed"]))
    maps = cpm.cpm_forward(w, d["x"], all_stages=True)
    np.testing.assert_array_equal(maps[-1], d["maps"])
    np.testing.assert_array_equal(np.stack(maps), d["map_stages"])
