"""ORACLE — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Host-side pre-processing restatements for ``PoseDetector.__call__`` (pose_detector.py:484-494):

* ``compute_optimal_size`` — pose_detector.py:57-73 (np.round = half-to-even).
* ``resize_linear_u8`` — ``cv2.resize(img, (w, h))`` default INTER_LINEAR on uint8
  (pose_detector.py:493).  OpenCV is not installed, so this is a restatement of OpenCV's
  fixed-point path ("parity unpinned"): 11-bit coefficients ``saturate_cast<short>(c*2048)``,
  horizontal pass in int32, vertical pass as OpenCV's SIMD body computes it
  (``((H0>>4)*b0 >> 16) + ((H1>>4)*b1 >> 16) + 2 >> 2``).  OpenCV's scalar tail and its
  IPP / exact-2x-downscale INTER_AREA shortcuts can differ from this by 1 LSB.
* ``preprocess`` — pose_detector.py:426-431: f32 ``x/255 - 0.5``, HWC -> (1,3,H,W), BGR kept.
"""
import numpy as np


def compute_optimal_size(orig_img_h, orig_img_w, img_size, stride=8):
    aspect = orig_img_h / orig_img_w
    if orig_img_h < orig_img_w:
        img_h = img_size
        img_w = int(np.round(img_size / aspect))
        surplus = img_w % stride
        if surplus != 0:
            img_w += stride - surplus
    else:
        img_w = img_size
        img_h = int(np.round(img_size * aspect))
        surplus = img_h % stride
        if surplus != 0:
            img_h += stride - surplus
    return img_w, img_h


def _coeffs(dsize, ssize, clamp):
    inv_scale = float(dsize) / float(ssize)
    scale = 1.0 / inv_scale
    d = np.arange(dsize, dtype=np.float64)
    f = ((d + 0.5) * scale - 0.5).astype(np.float32)
    s = np.floor(f).astype(np.int64)
    f = (f - s.astype(np.float32)).astype(np.float32)
    if clamp:
        lo = s < 0
        f[lo] = 0.0
        s[lo] = 0
        hi = s >= ssize - 1
        f[hi] = 0.0
        s[hi] = ssize - 1
    c0 = np.rint((np.float32(1.0) - f) * np.float32(2048.0)).astype(np.int64)
    c1 = np.rint(f * np.float32(2048.0)).astype(np.int64)
    c0 = np.clip(c0, -32768, 32767)
    c1 = np.clip(c1, -32768, 32767)
    return s, c0, c1


def resize_linear_u8(img, out_w, out_h):
    """cv2.resize(img, (out_w, out_h)) INTER_LINEAR, uint8 HxWxC (restated)."""
    img = np.asarray(img)
    sh, sw = img.shape[:2]
    sx, a0, a1 = _coeffs(out_w, sw, True)
    x1 = np.minimum(sx + 1, sw - 1)
    sy, b0, b1 = _coeffs(out_h, sh, False)
    src = img.astype(np.int64)
    hres = src[:, sx, :] * a0[None, :, None] + src[:, x1, :] * a1[None, :, None]  # (sh, out_w, C)
    r0 = np.clip(sy, 0, sh - 1)
    r1 = np.clip(sy + 1, 0, sh - 1)
    t0 = ((hres[r0] >> 4) * b0[:, None, None]) >> 16
    t1 = ((hres[r1] >> 4) * b1[:, None, None]) >> 16
    out = (t0 + t1 + 2) >> 2
    return np.clip(out, 0, 255).astype(np.uint8)


def preprocess(img):
    x = img.astype("f")
    x /= 255
    x -= 0.5
    return x.transpose(2, 0, 1)[None]
