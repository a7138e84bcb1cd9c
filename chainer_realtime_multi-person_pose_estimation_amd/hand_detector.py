"""``HandDetector`` — drop-in for hand_detector.py:12-94, MI355X only.

As ``FaceDetector`` with HandNet (22 maps -> 21 keypoints).  ``hand_type="left"`` mirrors the
crop before the network (the host copy ``cv2.flip(hand_img, 1)`` of hand_detector.py:30-31) and
reads the upsampled maps mirrored before the peaks (hand_detector.py:47-48), on the device.
"""
import numpy as np

from . import _lib
from . import weights as _weights
from .constants import params
from .draw import draw_disc, draw_line

FINGER_COLORS = [(0, 0, 255), (0, 255, 255), (0, 255, 0), (255, 0, 0), (255, 0, 255)]


class HandDetector(object):
    def __init__(self, arch=None, weights_file=None, model=None, device=-1):
        arch = arch or "handnet"
        if arch != "handnet":
            raise ValueError("HandDetector needs arch 'handnet', got %r" % (arch,))
        print("Loading HandNet...")
        self.device = 0 if device is None or device < 0 else int(device)
        self._ctx = _lib.CpmContext("handnet", self.device)
        if model is not None:
            w = model
        elif weights_file:
            w = _weights.load_npz(weights_file, arch="handnet")
        else:
            w = _weights.random_weights(0, arch="handnet")
        self._ctx.set_weights(w)

    def create_gaussian_kernel(self, sigma=1, ksize=5):
        """hand_detector.py:54-64 (the reference's GPU-branch kernel; kept for API parity)."""
        center = int(ksize / 2)
        d2 = (np.arange(ksize)[None, :] - center) ** 2 + (np.arange(ksize)[:, None] - center) ** 2
        return (np.exp(-d2 / (2 * sigma ** 2)) / (sigma ** 2 * 2 * np.pi)).astype(np.float32)[None, None]

    def compute_peaks_from_heatmaps(self, heatmaps):
        """hand_detector.py:66-94 (CPU-branch semantics) on the device."""
        return self._ctx.peaks(heatmaps, params["hand_heatmap_peak_thresh"])

    def __call__(self, hand_img, fast_mode=False, hand_type="right"):
        left = hand_type == "left"
        if left:
            hand_img = np.ascontiguousarray(np.asarray(hand_img)[:, ::-1])
        return self._ctx.detect(hand_img, params["hand_heatmap_peak_thresh"], flip_maps=left)

    def detect_batch(self, hand_imgs, hand_types):
        """``__call__`` over many crops in one batched forward (op_cpm_detect_batch): the same
        keypoints as one call per crop, for demo.py's every-person loop."""
        lefts = [t == "left" for t in hand_types]
        imgs = [np.ascontiguousarray(np.asarray(im)[:, ::-1]) if lf else im for im, lf in zip(hand_imgs, lefts)]
        return self._ctx.detect_batch(imgs, params["hand_heatmap_peak_thresh"], flip_maps=lefts)


def draw_hand_keypoints(orig_img, hand_keypoints, left_top):
    """hand_detector.py:96-116: per finger, radius-3 discs on both ends and a 1-px line."""
    img = orig_img.copy()
    left, top = left_top
    for i, finger in enumerate(params["fingers_indices"]):
        for a, b in finger:
            ka, kb = hand_keypoints[a], hand_keypoints[b]
            if ka:
                draw_disc(img, (int(ka[0] + left), int(ka[1] + top)), 3, FINGER_COLORS[i])
            if kb:
                draw_disc(img, (int(kb[0] + left), int(kb[1] + top)), 3, FINGER_COLORS[i])
            if ka and kb:
                draw_line(img, (ka[0] + left, ka[1] + top), (kb[0] + left, kb[1] + top), FINGER_COLORS[i], 1)
    return img


def main(argv=None):
    """hand_detector.py:118-139: python -m ....hand_detector handnet WEIGHTS --img IMG."""
    import argparse
    from .draw import read_bgr, write_bgr
    ap = argparse.ArgumentParser(description="Hand detector")
    ap.add_argument("arch", choices=list(params["archs"].keys()), default="handnet", help="Model architecture")
    ap.add_argument("weights", help="weights file path")
    ap.add_argument("--img", help="image file path")
    ap.add_argument("--gpu", "-g", type=int, default=-1, help="HIP device (negative: device 0; no CPU path)")
    ap.add_argument("--out", default="result.png", help="output image path")
    args = ap.parse_args(argv)
    det = HandDetector(args.arch, args.weights, device=args.gpu)
    img = read_bgr(args.img)
    kps = det(img, hand_type="right")
    img = draw_hand_keypoints(img, kps, (0, 0))
    print("Saving result into %s..." % args.out)
    write_bgr(args.out, img)
    return 0


if __name__ == "__main__":
    import sys
    sys.exit(main())
