"""Face / hand detectors, CPU side: the oracle's peak step and the host crop helpers
against fixtures made by the reference's own code (tests/golden/make_golden_cpm.py), the FaceNet /
HandNet forward restatement against an independent float64 convolution, and the drawing helpers.
"""
import hashlib
import os

import numpy as np
import pytest

from conftest import GOLDEN, pkg_module

from oracle import cpm as OC

CPM = os.path.join(GOLDEN, "cpm")


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _golden_kps(d):
    return [None if not f else [int(k[0]), int(k[1]), np.float32(k[2])] for k, f in zip(d["keypoints"], d["found"])]


@pytest.mark.parametrize("case,thresh_key", [("face_peaks", "face_heatmap_peak_thresh"),
                                             ("hand_peaks", "hand_heatmap_peak_thresh"),
                                             ("hand_peaks_wide", "hand_heatmap_peak_thresh")])
def test_oracle_peaks_match_reference(case, thresh_key):
    d = np.load(os.path.join(CPM, case + ".npz"))
    heat = d["heat_f16"].astype(np.float32)
    got = OC.compute_peaks_from_heatmaps(heat, OC.PARAMS[thresh_key])
    exp = _golden_kps(d)
    assert len(got) == len(exp) == heat.shape[0] - 1
    for g, e in zip(got, exp):
        assert (g is None) == (e is None)
        if g is not None:
            assert g[0] == e[0] and g[1] == e[1] and np.float32(g[2]) == e[2]
    # the np.where quirk is in the fixtures: two equal maxima -> [y1, y0]; constant map -> [0, 0]
    h, w = heat.shape[1:]
    assert exp[1][:2] == [3 * h // 4, h // 4] and exp[2][:2] == [0, 0]


def _bare_pose_detector():
    PD = pkg_module("pose_detector").PoseDetector
    return object.__new__(PD)  # host-side crop helpers only (no device context)


def test_pose_detector_crops_match_reference():
    from PIL import Image
    d = np.load(os.path.join(CPM, "crops.npz"))
    img = np.ascontiguousarray(np.asarray(Image.open(os.path.join(GOLDEN, "people.png")).convert("RGB"))[:, :, ::-1])
    pd = _bare_pose_detector()
    keys = sorted({k[:k.index("_", 3)] for k in d.keys() if k.startswith("s")})
    assert len(keys) == 14
    for key in keys:
        pose = d[key + "_pose"].copy()
        u = pd.get_unit_length(pose)
        assert u == float(d[key + "_unit"])
        if key + "_face_err" in d:
            with pytest.raises(ValueError):
                pd.crop_face(img, pose.copy(), u)
        else:
            fimg, fbox = pd.crop_face(img, pose.copy(), u)
            assert (fbox is None) == (d[key + "_face_bbox"].size == 0)
            if fbox is not None:
                assert list(fbox) == list(d[key + "_face_bbox"]) and _sha(fimg) == str(d[key + "_face_sha"])
        if key + "_hands_err" in d:
            with pytest.raises(ValueError):
                pd.crop_hands(img, pose.copy(), u)
        else:
            hands = pd.crop_hands(img, pose.copy(), u)
            for side in ("left", "right"):
                hb = d["%s_%s_bbox" % (key, side)]
                assert (hands[side] is None) == (hb.size == 0)
                if hands[side] is not None:
                    assert list(hands[side]["bbox"]) == list(hb)
                    assert _sha(hands[side]["img"]) == str(d["%s_%s_sha" % (key, side)])
        assert str(d[key + "_person_err"]) == "NameError"
        with pytest.raises(NameError):
            pd.crop_person(img, pose.copy(), u)


def test_face_crop_face_matches_reference():
    from PIL import Image
    crop_face = pkg_module("face_detector").crop_face
    d = np.load(os.path.join(CPM, "crops.npz"))
    img = np.ascontiguousarray(np.asarray(Image.open(os.path.join(GOLDEN, "people.png")).convert("RGB"))[:, :, ::-1])
    for i in range(4):
        fimg, lt = crop_face(img, tuple(int(v) for v in d["rect%d" % i]))
        assert list(lt) == list(d["rect%d_lt" % i])
        assert list(fimg.shape) == list(d["rect%d_shape" % i]) and _sha(fimg) == str(d["rect%d_sha" % i])


@pytest.mark.parametrize("arch", ["facenet", "handnet"])
def test_oracle_cpm_forward_vs_float64_torch(arch):
    """oracle/cpm.py (Chainer CPU restatement) against an independent float64 torch composition."""
    torch = pytest.importorskip("torch")
    W = pkg_module("weights").random_weights(seed=3, arch=arch)
    rng = np.random.default_rng(0)
    x = (rng.random((1, 3, 32, 40), dtype=np.float32) - 0.5).astype(np.float32)
    got = OC.cpm_forward(W, x)
    tf = torch.nn.functional

    def conv(name, h, act=True):
        w, b = W[name]
        y = tf.conv2d(h, torch.from_numpy(w).double(), torch.from_numpy(b).double(), padding=w.shape[2] // 2)
        return torch.relu(y) if act else y

    h = torch.from_numpy(x).double()
    for blk in (("conv1_1", "conv1_2"), ("conv2_1", "conv2_2"), ("conv3_1", "conv3_2", "conv3_3", "conv3_4")):
        for n in blk:
            h = conv(n, h)
        h = tf.max_pool2d(h, 2)
    for n in ("conv4_1", "conv4_2", "conv4_3", "conv4_4", "conv5_1", "conv5_2", "conv5_3_CPM"):
        h = conv(n, h)
    feat = h
    h = conv("conv6_2_CPM", conv("conv6_1_CPM", h), act=False)
    for s in range(2, 7):
        h = torch.cat((h, feat), 1)
        for i in range(1, 7):
            h = conv("Mconv%d_stage%d" % (i, s), h)
        h = conv("Mconv7_stage%d" % s, h, act=False)
    ref = h.numpy()
    assert got.shape == ref.shape == (1, OC.N_MAPS[arch], 4, 5)
    assert np.abs(got - ref).max() <= 1e-4 * max(1.0, np.abs(ref).max())


def test_draw_keypoints_paint():
    fd, hd = pkg_module("face_detector"), pkg_module("hand_detector")
    img = np.zeros((60, 60, 3), np.uint8)
    kps = [None] * 70
    kps[0], kps[1] = [10, 10, np.float32(0.5)], [30, 12, np.float32(0.4)]
    out = fd.draw_face_keypoints(img, kps, (5, 5))
    assert out[15, 15].tolist() == [255, 255, 0] and out[16, 25].tolist() == [255, 255, 0] and not img.any()
    hk = [None] * 21
    hk[0], hk[5] = [20, 20, np.float32(0.9)], [40, 20, np.float32(0.9)]
    out = hd.draw_hand_keypoints(img, hk, (0, 0))
    # the wrist (0) starts every finger: the last finger (colour 4) paints it last, as the reference
    assert out[20, 20].tolist() == [255, 0, 255] and out[20, 30].tolist() == [0, 255, 255]
