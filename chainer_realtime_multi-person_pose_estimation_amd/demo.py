"""demo.py of the reference (demo.py:1-60): pose, then per person the face and both hands.

    python -m chainer_realtime_multi-person_pose_estimation_amd.demo --img IMG [--gpu G]

Loads models/coco_posenet.npz, models/handnet.npz and models/facenet.npz (the reference's fixed
paths; ``--models DIR`` changes the directory, ``--random-weights`` uses seeded random weights for
a plumbing run without trained weights), runs PoseDetector on the image, blends the skeletons in
(``cv2.addWeighted(img, 0.6, pose, 0.4, 0)``), then for every person crops the face and the hands
(PoseDetector.get_unit_length / crop_face / crop_hands), runs FaceDetector / HandDetector on the
crops and draws their keypoints and white crop rectangles; writes result.png.
"""
import argparse
import os
import sys

import numpy as np

from . import weights as _weights
from .draw import draw_line, draw_person_pose, read_bgr, write_bgr
from .face_detector import FaceDetector, draw_face_keypoints
from .hand_detector import HandDetector, draw_hand_keypoints
from .pose_detector import PoseDetector


def add_weighted(a, wa, b, wb, gamma=0.0):
    """cv2.addWeighted on uint8: saturate(round(a*wa + b*wb + gamma))."""
    v = a.astype(np.float64) * wa + b.astype(np.float64) * wb + gamma
    return np.clip(np.rint(v), 0, 255).astype(np.uint8)


def draw_rectangle(img, p0, p1, color):
    """cv2.rectangle(img, p0, p1, color, 1): the four 1-px edges."""
    (x0, y0), (x1, y1) = p0, p1
    for a, b in (((x0, y0), (x1, y0)), ((x1, y0), (x1, y1)), ((x1, y1), (x0, y1)), ((x0, y1), (x0, y0))):
        draw_line(img, a, b, color, 1)


def run(img, pose_detector, face_detector, hand_detector, log=print):
    """demo.py:20-56.  The crops of every person are detected in two batched forwards (faces,
    hands: ``detect_batch``) and drawn in the reference's per-person order, so the image is the
    same as with one detector call per crop."""
    log("Estimating pose...")
    person_pose_array, _ = pose_detector(img)
    res_img = add_weighted(img, 0.6, draw_person_pose(img, person_pose_array), 0.4, 0)
    faces, hands = [], []
    for person_pose in person_pose_array:
        unit_length = pose_detector.get_unit_length(person_pose)
        faces.append(pose_detector.crop_face(img, person_pose, unit_length))
        hands.append(pose_detector.crop_hands(img, person_pose, unit_length))
    face_crops = [f[0] for f in faces if f[0] is not None]
    hand_crops = [(h[side]["img"], side) for h in hands for side in ("left", "right") if h[side] is not None]
    face_kps = iter(face_detector.detect_batch(face_crops) if face_crops else [])
    hand_kps = iter(hand_detector.detect_batch([c for c, _ in hand_crops], [s for _, s in hand_crops])
                    if hand_crops else [])
    for (cropped_face_img, bbox), person_hands in zip(faces, hands):
        log("Estimating face keypoints...")
        if cropped_face_img is not None:
            res_img = draw_face_keypoints(res_img, next(face_kps), (bbox[0], bbox[1]))
            draw_rectangle(res_img, (bbox[0], bbox[1]), (bbox[2], bbox[3]), (255, 255, 255))
        log("Estimating hands keypoints...")
        for side in ("left", "right"):
            if person_hands[side] is not None:
                bbox = person_hands[side]["bbox"]
                res_img = draw_hand_keypoints(res_img, next(hand_kps), (bbox[0], bbox[1]))
                draw_rectangle(res_img, (bbox[0], bbox[1]), (bbox[2], bbox[3]), (255, 255, 255))
    return res_img


def main(argv=None):
    ap = argparse.ArgumentParser(description="Pose detector")
    ap.add_argument("--img", help="image file path")
    ap.add_argument("--gpu", "-g", type=int, default=-1, help="HIP device (negative: device 0; no CPU path)")
    ap.add_argument("--models", default="models", help="directory of coco_posenet.npz / handnet.npz / facenet.npz")
    ap.add_argument("--random-weights", action="store_true", help="seeded random weights (plumbing run)")
    ap.add_argument("--out", default="result.png")
    args = ap.parse_args(argv)
    if args.random_weights:
        pd = PoseDetector("posenet", model=_weights.random_weights(0), device=args.gpu)
        hd = HandDetector("handnet", model=_weights.random_weights(0, arch="handnet"), device=args.gpu)
        fd = FaceDetector("facenet", model=_weights.random_weights(0, arch="facenet"), device=args.gpu)
    else:
        pd = PoseDetector("posenet", os.path.join(args.models, "coco_posenet.npz"), device=args.gpu)
        hd = HandDetector("handnet", os.path.join(args.models, "handnet.npz"), device=args.gpu)
        fd = FaceDetector("facenet", os.path.join(args.models, "facenet.npz"), device=args.gpu)
    img = read_bgr(args.img)
    res_img = run(img, pd, fd, hd)
    print("Saving result into %s..." % args.out)
    write_bgr(args.out, res_img)
    return 0


if __name__ == "__main__":
    sys.exit(main())
