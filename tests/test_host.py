"""Host-side logic: sizes, constants, weight files, frame sharding, oracle pre-processing."""
import numpy as np
import pytest

from conftest import PKG_NAME, pkg_module
from oracle import cvresize


@pytest.mark.parametrize("hw,img_size,expect", [((584, 584), 368, (368, 368)), ((480, 480), 320, (320, 320)),
                                                ((720, 1280), 368, (656, 368)), ((720, 1280), 320, (576, 320)),
                                                ((642, 482), 368, (368, 496)), ((642, 482), 320, (320, 432))])
def test_compute_optimal_size(hw, img_size, expect):
    assert cvresize.compute_optimal_size(hw[0], hw[1], img_size) == expect
    PD = pkg_module("pose_detector").PoseDetector
    assert PD.compute_optimal_size(None, np.zeros(hw + (3,)), img_size) == expect


def test_joint_type_and_params(pkg):
    assert len(pkg.JointType) == 18 and pkg.JointType.LeftEar == 17 and pkg.JointType.Neck == 1
    assert len(pkg.params["limbs_point"]) == 19
    from oracle.postproc import PARAMS
    for k, v in PARAMS.items():
        if k == "limbs_point":
            assert [[int(a), int(b)] for a, b in pkg.params[k]] == v
        else:
            assert pkg.params[k] == v, k


def test_weights_npz_roundtrip(tmp_path, rand_weights):
    W = pkg_module("weights")
    p = str(tmp_path / "w.npz")
    W.save_npz(p, rand_weights)
    back = W.load_npz(p)
    assert set(back) == set(rand_weights)
    for k in ("conv1_1", "Mconv7_stage6_L2"):
        np.testing.assert_array_equal(back[k][0], rand_weights[k][0])
    # prefixed keys (e.g. a Classifier's 'predictor/') are accepted
    flat = {"predictor/" + k + "/W": v[0] for k, v in rand_weights.items()}
    flat.update({"predictor/" + k + "/b": v[1] for k, v in rand_weights.items()})
    np.savez(p, **flat)
    assert np.array_equal(W.load_npz(p)["conv4_2"][1], rand_weights["conv4_2"][1])


def test_random_weights_shapes(rand_weights, lib):
    for name, ci, co, k in lib.layer_table():
        W, b = rand_weights[name]
        assert W.shape == (co, ci, k, k) and b.shape == (co,) and W.dtype == np.float32


def test_pad_image_matches_reference_semantics():
    PD = pkg_module("pose_detector").PoseDetector
    img = np.arange(5 * 7 * 3, dtype=np.uint8).reshape(5, 7, 3)
    out, pad = PD.pad_image(None, img, 8, (104, 117, 123))
    assert out.shape == (8, 8, 3) and pad == [3, 1]
    assert np.array_equal(out[:5, :7], img) and tuple(out[7, 7]) == (104, 117, 123)


def test_resize_linear_identity_and_constant():
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, (40, 60, 3), dtype=np.uint8)
    assert np.array_equal(cvresize.resize_linear_u8(img, 60, 40), img)
    c = np.full((33, 47, 3), 200, np.uint8)
    assert np.all(cvresize.resize_linear_u8(c, 91, 20) == 200)


def test_frame_sharding_and_records():
    F = pkg_module("frames")
    assert F.shard(10, 1, 4) == [1, 5, 9]
    all_ids = sorted(sum((F.shard(13, r, 3) for r in range(3)), []))
    assert all_ids == list(range(13))
    poses = np.arange(2 * 18 * 3, dtype=np.float64).reshape(2, 18, 3)
    rec = F.pack_records([(7, 0, 30, poses, np.array([1.5, 2.5])), (8, 0, 0, np.zeros((0, 18, 3)), np.zeros(0))], 4)
    back = F.unpack_records(rec, 4)
    fid, st, npk, p, s = back[0]
    assert (fid, st, npk) == (7, 0, 30) and np.array_equal(p, poses) and np.array_equal(s, [1.5, 2.5])
    assert back[1][3].shape == (0, 18, 3)
