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
    """face_detector.py:104-118: rect (x, y, w, h) scaled by face_crop_scale around its centre,
    clipped to the image, zero-padded to a square; returns (padded_face, (crop_left, crop_top))."""
    orig_img_h, orig_img_w, _ = img.shape
    crop_center_x = rect[0] + rect[2] / 2
    crop_center_y = rect[1] + rect[3] / 2
    crop_width = rect[2] * params["face_crop_scale"]
    crop_height = rect[3] * params["face_crop_scale"]
    crop_left = max(0, int(crop_center_x - crop_width / 2))
    crop_top = max(0, int(crop_center_y - crop_height / 2))
    crop_right = min(orig_img_w - 1, int(crop_center_x + crop_width / 2))
    crop_bottom = min(orig_img_h - 1, int(crop_center_y + crop_height / 2))
    cropped_face = img[crop_top:crop_bottom, crop_left:crop_right]
    max_edge_len = np.max(cropped_face.shape[:-1])
    padded_face = np.zeros((max_edge_len, max_edge_len, cropped_face.shape[-1]), dtype=np.uint8)
    padded_face[0:cropped_face.shape[0], 0:cropped_face.shape[1]] = cropped_face
    return padded_face, (crop_left, crop_top)


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
