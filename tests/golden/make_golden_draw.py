"""Record the REFERENCE's own draw_person_pose call sequence.

Run in the build container only (it needs /root/reference):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_draw.py

OpenCV is absent, so the rasteriser itself stays unpinned; what this pins is everything
draw_person_pose (/root/reference/pose_detector.py:520-553) decides: which limbs are drawn (both
joints detected, the ear-shoulder limbs 9 and 13 skipped), in which order, with which endpoints
(``poses.round().astype('i')``: NumPy half-to-even), colours, thickness and radius, that the canvas
is a copy, and that no pose leaves the input untouched.  The reference module is imported unmodified
with the stub modules of make_golden.py; its ``cv2`` stub gets ``line`` / ``circle`` functions that
record their arguments instead of drawing.

Writes tests/golden/draw_calls.json: per case the input poses and the ordered call list.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import install_stubs  # noqa: E402

CASES = ["six_people", "neckless_merge", "portrait_four", "twenty_720p", "one_person"]


def _pt(p):
    return [int(v) for v in p]


def _color(c):
    return [float(v) for v in c]


def main():
    install_stubs()
    cv2 = sys.modules["cv2"]
    calls = []

    def line(img, pt1, pt2, color, thickness=1, *rest):
        calls.append({"op": "line", "img": id(img), "pt1": _pt(pt1), "pt2": _pt(pt2), "color": _color(color),
                      "thickness": int(thickness), "extra": len(rest)})

    def circle(img, center, radius, color, thickness=1, *rest):
        calls.append({"op": "circle", "img": id(img), "center": _pt(center), "radius": int(radius),
                      "color": _color(color), "thickness": int(thickness), "extra": len(rest)})

    cv2.line = line
    cv2.circle = circle
    import pose_detector  # the reference, from /root/reference
    out = {}
    inputs = {}
    for name in CASES:
        d = np.load(os.path.join(HERE, name + ".npz"))
        inputs[name] = (np.asarray(d["poses"], np.float64), int(d["orig_h"]), int(d["orig_w"]))
    # rounding and visibility edge cases: half-integer coordinates (half-to-even), a person with
    # only some joints, joints at the image border
    rng = np.random.default_rng(553)
    edge = np.zeros((3, 18, 3))
    edge[0, :, :2] = rng.integers(0, 60, (18, 2)) + 0.5
    edge[0, :, 2] = 2
    edge[1, :, :2] = rng.uniform(0, 63, (18, 2))
    edge[1, ::3, 2] = 2
    edge[1, 1, 2] = 2
    edge[2, :, :2] = rng.choice([0.0, 63.0, 0.49, 62.51], (18, 2))
    edge[2, :, 2] = 2
    edge[2, 5, :] = 0
    inputs["edge_rounding"] = (edge, 64, 64)
    inputs["no_pose"] = (np.empty((0, 18, 3)), 16, 16)
    for name, (poses, h, w) in inputs.items():
        img = np.zeros((h, w, 3), np.uint8)
        del calls[:]
        res = pose_detector.draw_person_pose(img, poses)
        returned_input = res is img
        rec = []
        for raw in calls:
            c = dict(raw)
            assert c.pop("extra") == 0
            # which array the call draws on: the returned canvas (a copy of the input), or the input
            c["canvas"] = "returned" if raw["img"] == id(res) else ("input" if raw["img"] == id(img) else "other")
            del c["img"]
            rec.append(c)
        out[name] = {"poses": np.asarray(poses, np.float64).tolist(), "h": h, "w": w,
                     "returns_input": bool(returned_input), "calls": rec}
        print("%-16s persons=%2d calls=%4d returns_input=%s" % (name, len(poses), len(rec), returned_input))
    with open(os.path.join(HERE, "draw_calls.json"), "w") as f:
        json.dump(out, f, separators=(",", ":"))


if __name__ == "__main__":
    main()
