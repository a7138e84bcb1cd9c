"""Face / hand detectors on the GPU, through the C ABI (op_cpm_*): the peak step
bit-exact against the reference's own outputs, the FaceNet / HandNet forward within the north
star's 1e-3 of the oracle, and the whole detector equal to the oracle composition fed with the
device forward's maps."""
import os

import numpy as np
import pytest

from conftest import GOLDEN, pkg_module
from oracle import cpm as OC
from oracle import cvresize, postproc as P

pytestmark = pytest.mark.gpu
FWD_TOL = 1e-3
CPM = os.path.join(GOLDEN, "cpm")


@pytest.fixture(scope="module", params=["facenet", "handnet"])
def cpm(request):
    lib = pkg_module("_lib")
    W = pkg_module("weights").random_weights(seed=4, arch=request.param)
    c = lib.CpmContext(request.param, 0)
    c.set_weights(W)
    yield request.param, c, W
    c.close()


def _same(got, exp):
    assert len(got) == len(exp)
    for i, (g, e) in enumerate(zip(got, exp)):
        assert (g is None) == (e is None), i
        if g is not None:
            assert g[0] == e[0] and g[1] == e[1] and np.float32(g[2]) == np.float32(e[2]), (i, g, e)


@pytest.mark.parametrize("case", ["face_peaks", "hand_peaks", "hand_peaks_wide"])
def test_cpm_peaks_bit_exact_vs_reference(cpm, case):
    _, c, _ = cpm
    d = np.load(os.path.join(CPM, case + ".npz"))
    heat = d["heat_f16"].astype(np.float32)
    exp = [None if not f else [int(k[0]), int(k[1]), np.float32(k[2])] for k, f in zip(d["keypoints"], d["found"])]
    _same(c.peaks(heat, 0.1), exp)
    # the left-hand readout: peaks of the x-mirrored maps
    _same(c.peaks(heat, 0.1, flip=True), OC.compute_peaks_from_heatmaps(np.ascontiguousarray(heat[:, :, ::-1]), 0.1))


@pytest.mark.parametrize("shape", [(1, 3, 368, 368), (2, 3, 64, 96)])
def test_cpm_forward_vs_oracle(cpm, shape):
    arch, c, W = cpm
    rng = np.random.default_rng(5)
    x = rng.uniform(-0.5, 0.5, shape).astype(np.float32)
    got = c.forward(x)
    ref = OC.cpm_forward(W, x)
    err = float(np.abs(got - ref).max())
    print("%s forward %s: max|gpu-oracle| = %.3g (max|map| = %.3g)" % (arch, shape, err, np.abs(ref).max()))
    assert got.shape == ref.shape and err <= FWD_TOL


@pytest.mark.parametrize("hw,hand_type", [((96, 80), "right"), ((61, 75), "left")])
def test_cpm_detect_equals_oracle_composition(cpm, hw, hand_type):
    """detect == oracle resize + peaks of the device forward on the oracle's preprocessed input
    (so the preprocess (/256), the map upsample and the peak step are each held exactly)."""
    arch, c, _ = cpm
    h, w = hw
    img = np.random.default_rng(h * w).integers(0, 256, (h, w, 3), dtype=np.uint8)
    left = arch == "handnet" and hand_type == "left"
    src = np.ascontiguousarray(img[:, ::-1]) if left else img
    x = OC.preprocess(cvresize.resize_linear_u8(src, 368, 368))
    low = c.forward(x)[0]
    heat = P.resize_images(low, h, w)
    if left:
        heat = np.ascontiguousarray(heat[:, :, ::-1])
    # a threshold the random-weight maps cross, so keypoints are found
    thr = float(np.float32(np.median(heat.max(axis=(1, 2)))))
    exp = OC.compute_peaks_from_heatmaps(heat, thr)
    got = c.detect(src, thr, flip_maps=left)
    assert sum(k is not None for k in exp) > 0
    _same(got, exp)


def _close(got, exp):
    """Same keypoints; confidences equal up to f32 re-association (a single crop's 7x7 launches
    split their input chunks over workgroups, a batch's do not)."""
    assert len(got) == len(exp)
    for i, (g, e) in enumerate(zip(got, exp)):
        assert (g is None) == (e is None), i
        if g is not None:
            assert g[0] == e[0] and g[1] == e[1] and abs(float(g[2]) - float(e[2])) <= 1e-4 * max(1.0, abs(float(e[2]))), (i, g, e)


def test_cpm_detect_batch_equals_single_calls(cpm):
    """op_cpm_detect_batch over crops of mixed sizes (and mixed left/right readouts) == one
    op_cpm_detect per crop: the same keypoints, confidences up to f32 re-association."""
    arch, c, _ = cpm
    rng = np.random.default_rng(11)
    sizes = [(96, 80), (61, 75), (300, 210), (40, 33), (368, 368)]
    crops = [rng.integers(0, 256, (h, w, 3), dtype=np.uint8) for h, w in sizes]
    flips = [arch == "handnet" and i % 2 == 1 for i in range(len(crops))]
    for thr in (-10.0, 0.05):
        single = [c.detect(im, thr, flip_maps=f) for im, f in zip(crops, flips)]
        batch = c.detect_batch(crops, thr, flip_maps=flips)
        assert len(batch) == len(single)
        for g, e in zip(batch, single):
            _close(g, e)
    assert c.detect_batch([], 0.1) == []
    with pytest.raises(ValueError):
        c.detect_batch([crops[0], crops[1][:1]], 0.1)  # a 1-row crop: rejected like op_cpm_detect
    # batch-invariant mode: no split-K, so the batch equals the single calls bit for bit
    c.set_batch_invariant(True)
    try:
        single = [c.detect(im, 0.05, flip_maps=f) for im, f in zip(crops, flips)]
        for g, e in zip(c.detect_batch(crops, 0.05, flip_maps=flips), single):
            _same(g, e)
    finally:
        c.set_batch_invariant(False)


def test_cpm_detect_strided_crop_views(cpm):
    """Crops that are views into a larger image (row stride > 3 * width) are uploaded row by row:
    the same result as a packed copy (op_cpm_detect / op_cpm_detect_batch row_stride)."""
    arch, c, _ = cpm
    big = np.random.default_rng(12).integers(0, 256, (200, 300, 3), dtype=np.uint8)
    views = [big[10:110, 20:97], big[50:190, 150:299], big[:41, :33]]
    for v in views:
        assert v.strides[0] == 900 and not v.flags.c_contiguous
        _same(c.detect(v, 0.05), c.detect(np.ascontiguousarray(v), 0.05))
    got = c.detect_batch(views, 0.05)
    exp = c.detect_batch([np.ascontiguousarray(v) for v in views], 0.05)
    for g, e in zip(got, exp):
        _same(g, e)


def test_face_and_hand_detector_api():
    fd = pkg_module("face_detector").FaceDetector("facenet", None, model=pkg_module("weights").random_weights(1, arch="facenet"))
    hd = pkg_module("hand_detector").HandDetector("handnet", None, model=pkg_module("weights").random_weights(1, arch="handnet"))
    img = np.random.default_rng(0).integers(0, 256, (120, 100, 3), dtype=np.uint8)
    fk = fd(img)
    hk_r, hk_l = hd(img, hand_type="right"), hd(img, hand_type="left")
    assert len(fk) == 70 and len(hk_r) == 21 and len(hk_l) == 21
    for k in fk + hk_r + hk_l:
        assert k is None or (isinstance(k[0], int) and isinstance(k[1], int) and isinstance(k[2], np.float32))
    with pytest.raises(ValueError):
        pkg_module("face_detector").FaceDetector("handnet", None)


def test_demo_on_golden_poses(tmp_path):
    """demo.py's flow (pose -> face / hand crops -> detectors -> drawing) on people.png with the
    six-person golden poses standing in for the random-weight pose detector's (empty) output."""
    from conftest import load_golden, people_image
    demo = pkg_module("demo")
    W = pkg_module("weights")
    pd = pkg_module("pose_detector").PoseDetector("posenet", model=W.random_weights(0))
    poses = load_golden("six_people")["poses"]

    class Pose(object):
        def __call__(self, img):
            return poses.copy(), np.ones(len(poses))

        def __getattr__(self, name):
            return getattr(pd, name)

    fd = pkg_module("face_detector").FaceDetector("facenet", model=W.random_weights(2, arch="facenet"))
    hd = pkg_module("hand_detector").HandDetector("handnet", model=W.random_weights(2, arch="handnet"))
    # batch-invariant mode: the batched crops and the per-crop calls sum in the same order, so the
    # drawn images are equal by construction, not by the absence of near-ties
    fd._ctx.set_batch_invariant(True)
    hd._ctx.set_batch_invariant(True)
    img = people_image()
    log = []
    out = demo.run(img, Pose(), fd, hd, log=log.append)
    assert out.shape == img.shape and out.dtype == np.uint8 and (out != img).any()
    assert log.count("Estimating face keypoints...") == len(poses)
    # the batched detectors draw the same image as the reference's one call per crop
    seq = demo.add_weighted(img, 0.6, pkg_module("draw").draw_person_pose(img, poses), 0.4, 0)
    for pose in poses:
        unit = pd.get_unit_length(pose)
        face, bbox = pd.crop_face(img, pose, unit)
        if face is not None:
            seq = pkg_module("face_detector").draw_face_keypoints(seq, fd(face), (bbox[0], bbox[1]))
            demo.draw_rectangle(seq, (bbox[0], bbox[1]), (bbox[2], bbox[3]), (255, 255, 255))
        hands = pd.crop_hands(img, pose, unit)
        for side in ("left", "right"):
            if hands[side] is not None:
                bbox = hands[side]["bbox"]
                seq = pkg_module("hand_detector").draw_hand_keypoints(seq, hd(hands[side]["img"], hand_type=side),
                                                                      (bbox[0], bbox[1]))
                demo.draw_rectangle(seq, (bbox[0], bbox[1]), (bbox[2], bbox[3]), (255, 255, 255))
    assert np.array_equal(out, seq)
    # the CLI with seeded random weights (no persons: the pose blend only)
    dst = tmp_path / "result.png"
    src = os.path.join(GOLDEN, "people.png")
    assert demo.main(["--img", src, "--random-weights", "--out", str(dst)]) == 0 and dst.exists()
