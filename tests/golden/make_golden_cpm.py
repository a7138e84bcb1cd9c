"""Golden fixtures for the face / hand detectors and PoseDetector's crop helpers,
generated from the REFERENCE's own code.

Run in the build container only (needs /root/reference, absent on the GPU box):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_cpm.py

* Imports /root/reference/face_detector.py, hand_detector.py and pose_detector.py with the
  same empty stub modules as make_golden.py (cv2 / chainer are absent; nothing of theirs runs on
  these paths) and calls, unmodified:
    FaceDetector.compute_peaks_from_heatmaps / HandDetector.compute_peaks_from_heatmaps (CPU
      branch: scipy gaussian_filter, global max, np.where argmax; face_detector.py:58-84,
      hand_detector.py:68-94),
    face_detector.crop_face(img, rect) (face_detector.py:104-118),
    PoseDetector.get_unit_length / crop_face / crop_hands / crop_person (pose_detector.py:266-425).
* Heat-map inputs are synthetic smooth blobs, stored as float16 (every value is f16-exact, so the
  f32 maps the reference saw are reproduced exactly), plus planes that hit the np.where quirk:
  two equal maxima ([coords[1], coords[0]] is then [y1, y0]) and a constant plane.
* Crops are taken from tests/golden/people.png (BGR via PIL, as make_golden.py) and recorded as
  shape + SHA-256 of the bytes; bboxes and unit lengths are stored as numbers.

Writes tests/golden/cpm/*.npz (inputs + expected outputs, no code).
"""
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, REPO)
from make_golden import install_stubs  # noqa: E402

OUT = os.path.join(HERE, "cpm")


def blobs(rng, c, h, w, amp_hi=0.7):
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float64)
    m = np.zeros((c, h, w))
    for k in range(c):
        for _ in range(rng.integers(1, 3)):
            cy, cx = rng.uniform(0, h - 1), rng.uniform(0, w - 1)
            s = rng.uniform(1.5, 5.0)
            m[k] += rng.uniform(0.0, amp_hi) * np.exp(-((yy - cy) ** 2 + (xx - cx) ** 2) / (2 * s * s))
        m[k] += rng.normal(0, 0.01, (h, w))
    return m.astype(np.float16)


def quirk_planes(m):
    """Plane 1: two equal interior spikes (equal filtered maxima); plane 2: constant 0.5."""
    c, h, w = m.shape
    m[1] = 0
    m[1, h // 4, w // 4] = 8.0
    m[1, 3 * h // 4, 3 * w // 4] = 8.0
    m[2] = 0.5
    return m


def keypoints_array(kps):
    """list of [x, y, conf] | None -> (K, 3) f64 with NaN rows for None."""
    out = np.full((len(kps), 3), np.nan)
    for i, k in enumerate(kps):
        if k is not None:
            out[i] = [float(k[0]), float(k[1]), float(k[2])]
    return out


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main():
    install_stubs()
    import chainer
    chainer.using_config = lambda *a, **k: None
    import face_detector
    import hand_detector
    import pose_detector
    from PIL import Image
    os.makedirs(OUT, exist_ok=True)
    rng = np.random.default_rng(2024)

    fd = object.__new__(face_detector.FaceDetector)
    hd = object.__new__(hand_detector.HandDetector)
    for name, det, c, h, w in (("face_peaks", fd, 71, 40, 36), ("hand_peaks", hd, 22, 56, 48),
                               ("hand_peaks_wide", hd, 22, 30, 70)):
        m16 = quirk_planes(blobs(rng, c, h, w))
        heat = m16.astype(np.float32)
        kps = det.compute_peaks_from_heatmaps(heat)
        np.savez_compressed(os.path.join(OUT, name + ".npz"), heat_f16=m16, keypoints=keypoints_array(kps),
                            found=np.array([k is not None for k in kps]))
        print(name, sum(k is not None for k in kps), "of", len(kps), kps[1], kps[2])

    # crops on people.png with the six-person golden poses (in 480x480 image coordinates)
    img = np.ascontiguousarray(np.asarray(Image.open(os.path.join(HERE, "people.png")).convert("RGB"))[:, :, ::-1])
    poses = np.load(os.path.join(HERE, "six_people.npz"))["poses"]
    sets = [poses]
    p2 = poses.copy()
    p2[0, [0, 4, 7]] = 0  # no nose, no hands: the None branches
    p2[1, [3, 6]] = 0      # hands without elbows
    p2[2, :, :2] += 300    # partly outside the image: padded crops
    sets.append(p2)
    pd = pose_detector.PoseDetector(model=object())
    rec = {}
    for si, ps in enumerate(sets):
        for pi, pose in enumerate(ps):
            key = "s%d_p%d" % (si, pi)
            u = pd.get_unit_length(pose)
            rec[key + "_pose"] = pose
            rec[key + "_unit"] = np.float64(u)
            try:
                fimg, fbox = pd.crop_face(img, pose.copy(), u)
                rec[key + "_face_bbox"] = np.array(fbox if fbox is not None else [], np.int64)
                rec[key + "_face_sha"] = np.array(sha(fimg) if fimg is not None else "")
                rec[key + "_face_shape"] = np.array(fimg.shape if fimg is not None else [], np.int64)
            except Exception as e:  # noqa: BLE001  (record the reference's own failure)
                rec[key + "_face_err"] = np.array(type(e).__name__)
            try:
                hands = pd.crop_hands(img, pose.copy(), u)
                for side in ("left", "right"):
                    hnd = hands[side]
                    rec[key + "_%s_bbox" % side] = np.array(hnd["bbox"] if hnd else [], np.int64)
                    rec[key + "_%s_sha" % side] = np.array(sha(hnd["img"]) if hnd else "")
                    rec[key + "_%s_shape" % side] = np.array(hnd["img"].shape if hnd else [], np.int64)
            except Exception as e:  # noqa: BLE001
                rec[key + "_hands_err"] = np.array(type(e).__name__)
            try:
                cimg, cbox = pd.crop_person(img, pose.copy(), u)
                rec[key + "_person_bbox"] = np.array(cbox, np.int64)
                rec[key + "_person_sha"] = np.array(sha(cimg))
            except Exception as e:  # noqa: BLE001  (record the reference's own failure)
                rec[key + "_person_err"] = np.array(type(e).__name__)
    rects = [(100, 80, 60, 70), (0, 0, 50, 40), (440, 430, 60, 60), (10, 200, 30, 90)]
    for i, r in enumerate(rects):
        fimg, lt = face_detector.crop_face(img, r)
        rec["rect%d" % i] = np.array(r, np.int64)
        rec["rect%d_lt" % i] = np.array(lt, np.int64)
        rec["rect%d_sha" % i] = np.array(sha(fimg))
        rec["rect%d_shape" % i] = np.array(fimg.shape, np.int64)
    np.savez_compressed(os.path.join(OUT, "crops.npz"), **rec)
    print("crops", len(rec))


if __name__ == "__main__":
    main()
