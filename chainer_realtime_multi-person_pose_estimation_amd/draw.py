"""Rendering and CLI of the reference (pose_detector.py:520-579), SURVEY §8 row f1.

``draw_person_pose`` follows the reference: limbs in ``params['limbs_point']`` order with its 19
colours, the ear-shoulder limbs 9 and 13 skipped, a limb drawn only when both joints are
detected, 2-px lines, then filled radius-3 joint discs, on ``pose.round().astype('i')`` coordinates.
OpenCV's rasteriser (``cv2.line`` / ``cv2.circle``) is not installed here; lines are the pixels
within 1 px of the segment and discs the pixels within radius 3, so edge pixels can differ from
OpenCV's (rendering parity unpinned).  Host-side: drawing is not on the measured path.
"""
import argparse

import numpy as np

from .constants import params

LIMB_COLORS = [
    [0, 255, 0], [0, 255, 85], [0, 255, 170], [0, 255, 255], [0, 170, 255], [0, 85, 255], [255, 0, 0],
    [255, 85, 0], [255, 170, 0], [255, 255, 0], [255, 0, 85], [170, 255, 0], [85, 255, 0], [170, 0, 255],
    [0, 0, 255], [0, 0, 255], [255, 0, 255], [170, 0, 255], [255, 0, 170]]
JOINT_COLORS = [
    [255, 0, 0], [255, 85, 0], [255, 170, 0], [255, 255, 0], [170, 255, 0], [85, 255, 0], [0, 255, 0],
    [0, 255, 85], [0, 255, 170], [0, 255, 255], [0, 170, 255], [0, 85, 255], [0, 0, 255], [85, 0, 255],
    [170, 0, 255], [255, 0, 255], [255, 0, 170], [255, 0, 85]]


def _paint(canvas, mask, y0, x0, color):
    h, w = canvas.shape[:2]
    ys, xs = np.nonzero(mask)
    ys, xs = ys + y0, xs + x0
    keep = (ys >= 0) & (ys < h) & (xs >= 0) & (xs < w)
    canvas[ys[keep], xs[keep]] = np.asarray(color, np.float64).round().astype(canvas.dtype)


def draw_line(canvas, p0, p1, color, thickness=2):
    (x0, y0), (x1, y1) = p0, p1
    r = thickness / 2.0
    lx, hx = int(np.floor(min(x0, x1) - r)), int(np.ceil(max(x0, x1) + r))
    ly, hy = int(np.floor(min(y0, y1) - r)), int(np.ceil(max(y0, y1) + r))
    yy, xx = np.mgrid[ly:hy + 1, lx:hx + 1]
    dx, dy = x1 - x0, y1 - y0
    n2 = float(dx * dx + dy * dy)
    t = np.clip(((xx - x0) * dx + (yy - y0) * dy) / n2, 0.0, 1.0) if n2 > 0 else np.zeros(xx.shape)
    d2 = (xx - (x0 + t * dx)) ** 2 + (yy - (y0 + t * dy)) ** 2
    _paint(canvas, d2 <= r * r, ly, lx, color)


def draw_disc(canvas, center, radius, color):
    x, y = center
    yy, xx = np.mgrid[-radius:radius + 1, -radius:radius + 1]
    _paint(canvas, xx * xx + yy * yy <= radius * radius, y - radius, x - radius, color)


class Raster(object):
    """The two OpenCV primitives draw_person_pose uses, with cv2's argument order:
    ``line(img, pt1, pt2, color, thickness)`` and ``circle(img, center, radius, color, thickness)``
    (thickness -1 = filled).  The default draws with the approximations above; tests pass a
    recording subclass to compare the call sequence with the reference's own
    (tests/golden/draw_calls.json, made by running pose_detector.py:520-553 under a recording cv2)."""

    def line(self, img, pt1, pt2, color, thickness):
        draw_line(img, pt1, pt2, color, thickness)

    def circle(self, img, center, radius, color, thickness):
        if thickness >= 0:
            raise ValueError("draw.Raster.circle: only filled discs (thickness -1) are drawn")
        draw_disc(img, center, radius, color)


def draw_person_pose(orig_img, poses, raster=None):
    """pose_detector.py:520-553 (``raster``: the cv2 stand-in, default Raster())."""
    if len(poses) == 0:
        return orig_img
    cv = raster if raster is not None else Raster()
    canvas = orig_img.copy()
    poses_i = np.asarray(poses).round().astype("i")
    for pose in poses_i:  # limbs
        for i, (limb, color) in enumerate(zip(params["limbs_point"], LIMB_COLORS)):
            if i in (9, 13):  # ear-shoulder connections are not drawn
                continue
            ind = np.array([int(j) for j in limb])
            if np.all(pose[ind][:, 2] != 0):
                (a, b) = pose[ind][:, :2]
                cv.line(canvas, tuple(a), tuple(b), color, 2)
    for pose in poses_i:  # joints
        for (x, y, v), color in zip(pose, JOINT_COLORS):
            if v != 0:
                cv.circle(canvas, (x, y), 3, color, -1)
    return canvas


def read_bgr(path):
    from PIL import Image
    return np.ascontiguousarray(np.asarray(Image.open(path).convert("RGB"))[:, :, ::-1])


def write_bgr(path, img):
    from PIL import Image
    Image.fromarray(np.ascontiguousarray(np.asarray(img, np.uint8)[:, :, ::-1])).save(path)


def main(argv=None):
    """pose_detector.py:555-579: python -m chainer_realtime_multi-person_pose_estimation_amd ARCH WEIGHTS --img IMG."""
    from .pose_detector import PoseDetector
    ap = argparse.ArgumentParser(description="Pose detector")
    ap.add_argument("arch", choices=list(params["archs"].keys()), default="posenet", help="Model architecture")
    ap.add_argument("weights", help="weights file path (Chainer npz)")
    ap.add_argument("--img", "-i", default=None, help="image file path")
    ap.add_argument("--gpu", "-g", type=int, default=-1, help="HIP device (negative: device 0; no CPU path)")
    ap.add_argument("--precise", action="store_true", help="do precise inference")
    ap.add_argument("--out", default="result.png", help="output image path")
    args = ap.parse_args(argv)
    det = PoseDetector(args.arch, args.weights, device=args.gpu, precise=args.precise)
    img = read_bgr(args.img)
    poses, _ = det(img)
    img = draw_person_pose(img, poses)
    print("Saving result into %s..." % args.out)
    write_bgr(args.out, img)
    return 0
