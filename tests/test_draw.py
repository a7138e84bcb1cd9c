"""draw_person_pose (pose_detector.py:520-553): colours, skipped limbs, undetected joints."""
import numpy as np
import pytest

from conftest import pkg_module


def test_empty_poses_return_the_image():
    D = pkg_module("draw")
    img = np.zeros((10, 10, 3), np.uint8)
    assert D.draw_person_pose(img, np.empty((0, 18, 3))) is img


def test_joints_and_limbs_drawn_in_reference_colours():
    D = pkg_module("draw")
    img = np.zeros((80, 80, 3), np.uint8)
    pose = np.zeros((1, 18, 3))
    pose[0, 1] = (20, 20, 2)   # neck
    pose[0, 8] = (20, 60, 2)   # right waist: limb 0 (1 -> 8), colour LIMB_COLORS[0]
    pose[0, 2] = (60, 20, 2)   # right shoulder
    pose[0, 16] = (60, 60, 2)  # right ear: limb 9 (2 -> 16) is never drawn
    out = D.draw_person_pose(img, pose)
    assert out is not img and img.sum() == 0
    assert tuple(out[40, 20]) == tuple(D.LIMB_COLORS[0])       # middle of limb 0
    assert tuple(out[40, 60]) == (0, 0, 0)                       # limb 9 skipped
    assert tuple(out[20, 20]) == tuple(D.JOINT_COLORS[1])      # neck disc over the limb
    assert tuple(out[60, 60]) == tuple(D.JOINT_COLORS[16])
    assert tuple(out[20, 40]) == tuple(D.LIMB_COLORS[6])       # limb 6 (1 -> 2)
    assert tuple(out[23, 20]) == tuple(D.JOINT_COLORS[1]) and tuple(out[24, 20]) == tuple(D.LIMB_COLORS[0])


def test_undetected_joint_breaks_its_limbs():
    D = pkg_module("draw")
    img = np.zeros((50, 50, 3), np.uint8)
    pose = np.zeros((1, 18, 3))
    pose[0, 1] = (10, 10, 2)
    pose[0, 8] = (10, 40, 0)  # not detected
    out = D.draw_person_pose(img, pose)
    assert tuple(out[25, 10]) == (0, 0, 0)


def _draw_cases():
    import json
    import os
    with open(os.path.join(os.path.dirname(__file__), "golden", "draw_calls.json")) as f:
        return json.load(f)


DRAW_CASES = _draw_cases()


@pytest.mark.parametrize("case", sorted(DRAW_CASES))
def test_draw_call_sequence_equals_the_reference(case):
    """The reference's own draw_person_pose (pose_detector.py:520-553), run unmodified under a
    recording cv2 stub (tests/golden/make_golden_draw.py), made exactly these cv2.line /
    cv2.circle calls -- same order, endpoints, colours, thickness, radius, on a copy of the input;
    the package's draw_person_pose must make the identical sequence (the rasteriser behind the
    calls stays unpinned: OpenCV is absent)."""
    D = pkg_module("draw")
    c = DRAW_CASES[case]
    img = np.zeros((c["h"], c["w"], 3), np.uint8)
    calls = []

    class Recorder(D.Raster):
        def line(self, canvas, pt1, pt2, color, thickness):
            calls.append({"op": "line", "pt1": [int(v) for v in pt1], "pt2": [int(v) for v in pt2],
                          "color": [float(v) for v in color], "thickness": int(thickness), "canvas": canvas})
            super().line(canvas, pt1, pt2, color, thickness)

        def circle(self, canvas, center, radius, color, thickness):
            calls.append({"op": "circle", "center": [int(v) for v in center], "radius": int(radius),
                          "color": [float(v) for v in color], "thickness": int(thickness), "canvas": canvas})
            super().circle(canvas, center, radius, color, thickness)

    res = D.draw_person_pose(img, np.asarray(c["poses"], np.float64).reshape(-1, 18, 3), raster=Recorder())
    assert (res is img) == c["returns_input"]
    for k in calls:
        k["canvas"] = "returned" if k["canvas"] is res else ("input" if k["canvas"] is img else "other")
    assert calls == c["calls"]
    if not c["returns_input"]:
        assert img.sum() == 0  # the input is never drawn on


def test_read_bgr_drops_alpha_like_imread_color():
    """C1's input, data/person.png (584x584 RGBA, README.md:16): cv2.imread(path) with the default
    IMREAD_COLOR (pose_detector.py:571) returns the colour channels as BGR and ignores alpha (no
    compositing); read_bgr must give the same array."""
    import os
    from PIL import Image
    D = pkg_module("draw")
    path = os.path.join(os.path.dirname(__file__), "golden", "person.png")
    raw = np.asarray(Image.open(path))
    assert raw.shape == (584, 584, 4)  # RGBA on disk (opaque alpha)
    img = D.read_bgr(path)
    assert img.shape == (584, 584, 3) and img.dtype == np.uint8 and img.flags.c_contiguous
    assert np.array_equal(img, raw[:, :, 2::-1])
