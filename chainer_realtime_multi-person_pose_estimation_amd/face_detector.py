"""``FaceDetector`` — drop-in for face_detector.py:12-84, MI355X only.

``FaceDetector(arch, weights_file, model=None, device=-1)`` builds a FaceNet replica on the HIP
device (op_cpm_* in include/openpose_hip.h); ``__call__(face_img, fast_mode=False)`` runs the whole
detector there — cv2 LINEAR resize to 368x368 + ``x/256 - 0.5`` (face_detector.py:32-33), the
FaceNet forward on the CocoPoseNet conv kernels, ``F.resize_images`` to the crop size, SciPy
Gaussian (sigma 2.5) and the per-map argmax with the reference's ``np.where`` quirk — and returns
the reference's list: ``[x, y, conf]`` (ints, np.float32) or ``None`` per keypoint (70 of them).
``crop_face`` / ``draw_face_keypoints`` are the reference's host helpers (:86-118).  There is no
CPU path: ``device=-1`` selects HIP device 0.
"""
import numpy as np

from . import _lib
from . import weights as _weights
from .constants import params
from .draw import draw_disc, draw_line


class FaceDetector(object):
    def __init__(self, arch=None, weights_file=None, model=None, device=-1):
        arch = arch or "facenet"
        if arch != "facenet":
            raise ValueError("FaceDetector needs arch 'facenet', got %r" % (arch,))
        print("Loading FaceNet...")
        self.device = 0 if device is None or device < 0 else int(device)
        self._ctx = _lib.CpmContext("facenet", self.device)
        if model is not None:
            w = model
        elif weights_file:
            w = _weights.load_npz(weights_file, arch="facenet")
        else:
            w = _weights.random_weights(0, arch="facenet")
        self._ctx.set_weights(w)

    def create_gaussian_kernel(self, sigma=1, ksize=5):
        """face_detector.py:44-54 (the reference's GPU-branch kernel; kept for API parity)."""
        center = int(ksize / 2)
        d2 = (np.arange(ksize)[None, :] - center) ** 2 + (np.arange(ksize)[:, None] - center) ** 2
        return (np.exp(-d2 / (2 * sigma ** 2)) / (sigma ** 2 * 2 * np.pi)).astype(np.float32)[None, None]

    def compute_peaks_from_heatmaps(self, heatmaps):
        """face_detector.py:56-84 (CPU-branch semantics) on the device."""
        return self._ctx.peaks(heatmaps, params["face_heatmap_peak_thresh"])

    def __call__(self, face_img, fast_mode=False):
        return self._ctx.detect(face_img, params["face_heatmap_peak_thresh"])

    def detect_batch(self, face_imgs):
        """``__call__`` over many crops in one batched forward (op_cpm_detect_batch)."""
        return self._ctx.detect_batch(face_imgs, params["face_heatmap_peak_thresh"])


def draw_face_keypoints(orig_img, face_keypoints, left_top):
    """face_detector.py:86-102: radius-2 discs and 1-px lines in (255, 255, 0) (BGR)."""
    img = orig_img.copy()
    left, top = left_top
    for kp in face_keypoints:
        if kp:
            x, y, _ = kp
            draw_disc(img, (int(x + left), int(y + top)), 2, (255, 255, 0))
    for a, b in params["face_line_indices"]:
        ka, kb = face_keypoints[a], face_keypoints[b]
        if ka and kb:
            draw_line(img, (ka[0] + left, ka[1] + top), (kb[0] + left, kb[1] + top), (255, 255, 0), 1)
    return img


def crop_face(img, rect):
    """Restates face_detector.py:104-118: the (x, y, w, h) rect scaled by face_crop_scale about its
    centre, clipped to [0, W-1) x [0, H-1) like the reference (its right/bottom bound is W-1 / H-1,
    exclusive), copied into the top-left corner of a zero square whose side is the longer clipped
    edge.  -> (square crop, (left, top))."""
    h, w = img.shape[:2]
    s = params["face_crop_scale"]
    cx, cy = rect[0] + rect[2] / 2, rect[1] + rect[3] / 2
    half_w, half_h = rect[2] * s / 2, rect[3] * s / 2
    x0, x1 = max(0, int(cx - half_w)), min(w - 1, int(cx + half_w))
    y0, y1 = max(0, int(cy - half_h)), min(h - 1, int(cy + half_h))
    window = img[y0:y1, x0:x1]
    side = max(window.shape[:2])
    square = np.zeros((side, side, window.shape[2]), np.uint8)
    square[:window.shape[0], :window.shape[1]] = window
    return square, (x0, y0)


def main(argv=None):
    """face_detector.py:120-136: python -m ....face_detector facenet WEIGHTS --img IMG."""
    import argparse
    from .draw import read_bgr, write_bgr
    ap = argparse.ArgumentParser(description="Face detector")
    ap.add_argument("arch", choices=list(params["archs"].keys()), default="facenet", help="Model architecture")
    ap.add_argument("weights", help="weights file path")
    ap.add_argument("--img", help="image file path")
    ap.add_argument("--gpu", "-g", type=int, default=-1, help="HIP device (negative: device 0; no CPU path)")
    ap.add_argument("--out", default="result.png", help="output image path")
    args = ap.parse_args(argv)
    det = FaceDetector(args.arch, args.weights, device=args.gpu)
    img = read_bgr(args.img)
    kps = det(img)
    img = draw_face_keypoints(img, kps, (0, 0))
    print("Saving result into %s..." % args.out)
    write_bgr(args.out, img)
    return 0


if __name__ == "__main__":
    import sys
    sys.exit(main())
