"""ORACLE — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Multi-scale inference ``PoseDetector.detect_precise`` (pose_detector.py:433-482) + ``pad_image``
(:46-55) on the oracle forward, with ``cv2.resize(INTER_CUBIC)`` restated in oracle/cvcubic.c
("parity unpinned": OpenCV is not installed; see the header of cvcubic.c for the restated path).
"""
import ctypes
import math

import numpy as np

from . import cvresize
from . import forward as _fwd
from . import postproc as _pp

_READY = False


def _lib():
    global _READY
    L = _pp._lib()
    if not _READY:
        P = ctypes.c_void_p
        L.orc_resize_cubic_u8.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int64, P,
                                          ctypes.c_int, ctypes.c_int]
        L.orc_resize_cubic_f32.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int64, P,
                                           ctypes.c_int, ctypes.c_int]
        _READY = True
    return L


def resize_cubic_u8(img, out_w, out_h):
    """cv2.resize(img, (out_w, out_h), interpolation=cv2.INTER_CUBIC), uint8 H x W x C."""
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape[:2]
    cn = 1 if img.ndim == 2 else img.shape[2]
    out = np.empty((out_h, out_w, cn), np.uint8)
    _lib().orc_resize_cubic_u8(img.ctypes.data, h, w, cn, w * cn, out.ctypes.data, out_h, out_w)
    return out if img.ndim == 3 else out[:, :, 0]


def resize_cubic_f32(img, out_w, out_h):
    """cv2.resize(img, (out_w, out_h), interpolation=cv2.INTER_CUBIC), float32 H x W x C."""
    img = np.ascontiguousarray(img, np.float32)
    h, w = img.shape[:2]
    cn = 1 if img.ndim == 2 else img.shape[2]
    out = np.empty((out_h, out_w, cn), np.float32)
    _lib().orc_resize_cubic_f32(img.ctypes.data, h, w, cn, w * cn, out.ctypes.data, out_h, out_w)
    return out if img.ndim == 3 else out[:, :, 0]


def pad_image(img, stride, pad_value):
    """pose_detector.py:46-55."""
    h, w, _ = img.shape
    pad = [0] * 2
    pad[0] = (stride - (h % stride)) % stride
    pad[1] = (stride - (w % stride)) % stride
    img_padded = np.zeros((h + pad[0], w + pad[1], 3), "uint8") + pad_value
    img_padded[:h, :w, :] = img.copy()
    return img_padded, pad


def scale_sizes(orig_h, orig_w, params):
    """[(resized_w, resized_h, padded_w, padded_h)] per inference scale (pose_detector.py:442-445)."""
    out = []
    for scale in params["inference_scales"]:
        multiplier = scale * params["inference_img_size"] / min(orig_h, orig_w)
        rw, rh = math.ceil(orig_w * multiplier), math.ceil(orig_h * multiplier)
        pw = rw + (params["downscale"] - rw % params["downscale"]) % params["downscale"]
        ph = rh + (params["downscale"] - rh % params["downscale"]) % params["downscale"]
        out.append((rw, rh, pw, ph))
    return out


def scale_maps(paf, heat, rw, rh, pw, ph, orig_w, orig_h, downscale=8):
    """One scale's contribution (pose_detector.py:459-467): network maps (38|19, ph/8, pw/8) ->
    (orig_h, orig_w, 38|19) after the cubic resize to the padded size, the crop and the cubic
    resize to the original size."""
    tmp_paf = resize_cubic_f32(paf.transpose(1, 2, 0), pw, ph)[:rh, :rw, :]
    out_paf = resize_cubic_f32(tmp_paf, orig_w, orig_h)
    tmp_heat = resize_cubic_f32(heat.transpose(1, 2, 0), heat.shape[2] * downscale, heat.shape[1] * downscale)
    tmp_heat = tmp_heat[:rh, :rw, :]
    out_heat = resize_cubic_f32(tmp_heat, orig_w, orig_h)
    return out_paf, out_heat


def precise_maps(weights, orig_img, params=_pp.PARAMS, forward=None):
    """Averaged full-resolution maps of detect_precise: pafs (38, H, W), heatmaps (19, H, W) f32.
    ``forward(x) -> (paf (38,h,w), heat (19,h,w))`` defaults to the oracle forward."""
    orig_h, orig_w = orig_img.shape[:2]
    pafs_sum = 0
    heatmaps_sum = 0
    for rw, rh, pw, ph in scale_sizes(orig_h, orig_w, params):
        img = resize_cubic_u8(orig_img, rw, rh)
        padded, pad = pad_image(img, params["downscale"], (104, 117, 123))
        assert padded.shape[:2] == (ph, pw)
        x = cvresize.preprocess(padded)
        if forward is None:
            paf, heat = _fwd.cocoposenet_forward(weights, x)
            paf, heat = paf[0], heat[0]
        else:
            paf, heat = forward(x)
        p, hm = scale_maps(paf, heat, rw, rh, pw, ph, orig_w, orig_h, params["downscale"])
        pafs_sum += p
        heatmaps_sum += hm
    n = len(params["inference_scales"])
    return (pafs_sum / n).transpose(2, 0, 1), (heatmaps_sum / n).transpose(2, 0, 1)


def postprocess_full(pafs, heatmaps, orig_w, params=_pp.PARAMS):
    """pose_detector.py:474-482: peaks / connections / grouping at the original resolution."""
    all_peaks = _pp.compute_peaks_from_heatmaps(heatmaps, params)
    if len(all_peaks) == 0:
        return np.empty((0, _pp.N_JOINTS, 3)), np.empty(0)
    all_connections = _pp.compute_connections(pafs, all_peaks, orig_w, params)
    subsets = _pp.grouping_key_points(all_connections, all_peaks, params)
    poses = _pp.subsets_to_pose_array(subsets, all_peaks)
    scores = subsets[:, -2]
    return poses, scores


def detect_precise(weights, orig_img, params=_pp.PARAMS):
    pafs, heatmaps = precise_maps(weights, orig_img, params)
    return postprocess_full(pafs, heatmaps, orig_img.shape[1], params)
