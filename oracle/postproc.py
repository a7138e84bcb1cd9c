"""ORACLE — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Python faces of the plain-C post-process restatement in oracle/postproc.c, named after the
reference methods they restate (pose_detector.py:75-265, 484-517) with the same argument
meaning, return types and empty-result shapes.
"""
import ctypes
import os

import numpy as np

from . import cvresize
from . import forward as _fwd

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

# entity.py:70-105 (inference params), restated so the oracle stays independent of the product.
PARAMS = {
    "inference_img_size": 368,
    "inference_scales": [0.5, 1, 1.5, 2],
    "heatmap_size": 320,
    "gaussian_sigma": 2.5,
    "ksize": 17,
    "n_integ_points": 10,
    "n_integ_points_thresh": 8,
    "heatmap_peak_thresh": 0.05,
    "inner_product_thresh": 0.05,
    "limb_length_ratio": 1.0,
    "length_penalty_value": 1,
    "n_subset_limbs_thresh": 3,
    "subset_score_thresh": 0.2,
    "limbs_point": [[1, 8], [8, 9], [9, 10], [1, 11], [11, 12], [12, 13], [1, 2], [2, 3],
                    [3, 4], [2, 16], [1, 5], [5, 6], [6, 7], [5, 17], [1, 0], [0, 14],
                    [0, 15], [14, 16], [15, 17]],
    "downscale": 8,
}
N_JOINTS = 18


class _OrcParams(ctypes.Structure):
    _fields_ = [("n_integ_points", ctypes.c_int32), ("n_integ_points_thresh", ctypes.c_int32),
                ("inner_product_thresh", ctypes.c_double), ("limb_length_ratio", ctypes.c_double),
                ("length_penalty_value", ctypes.c_double), ("n_subset_limbs_thresh", ctypes.c_int32),
                ("subset_score_thresh", ctypes.c_double)]


def _lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liborc.so")
        if not os.path.exists(path):
            import subprocess
            subprocess.check_call(["make", "-s", "-C", _HERE])
        L = ctypes.CDLL(path)
        P = ctypes.c_void_p
        L.orc_resize_align_corners.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, P]
        L.orc_gaussian_weights.argtypes = [ctypes.c_double, ctypes.c_double, P, ctypes.c_int]
        L.orc_gaussian_weights.restype = ctypes.c_int
        L.orc_gaussian_filter.argtypes = [P, P, P, ctypes.c_int, ctypes.c_int, P, ctypes.c_int]
        L.orc_find_peaks.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float, P, ctypes.c_long]
        L.orc_find_peaks.restype = ctypes.c_long
        L.orc_candidate_connections.argtypes = [P, P, ctypes.c_int, ctypes.c_int, P, ctypes.c_int, P, ctypes.c_int,
                                                ctypes.c_double, P, P, ctypes.c_long]
        L.orc_candidate_connections.restype = ctypes.c_long
        L.orc_connections.argtypes = [P, ctypes.c_int, ctypes.c_int, P, ctypes.c_long, P, ctypes.c_int,
                                      ctypes.c_double, P, P, ctypes.c_long, P]
        L.orc_connections.restype = ctypes.c_int
        L.orc_grouping.argtypes = [P, P, P, ctypes.c_int, P, P, P, ctypes.c_long, P]
        L.orc_grouping.restype = ctypes.c_int
        _LIB = L
    return _LIB


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _params_struct(params):
    return _OrcParams(int(params["n_integ_points"]), int(params["n_integ_points_thresh"]),
                      float(params["inner_product_thresh"]), float(params["limb_length_ratio"]),
                      float(params["length_penalty_value"]), int(params["n_subset_limbs_thresh"]),
                      float(params["subset_score_thresh"]))


def resize_images(x, out_h, out_w):
    """Chainer<=6 F.resize_images on (C,H,W) f32 -> (C,out_h,out_w) f32 (pose_detector.py:501-502)."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    C, H, W = x.shape
    y = np.empty((C, out_h, out_w), np.float32)
    _lib().orc_resize_align_corners(_ptr(x), C, H, W, out_h, out_w, _ptr(y))
    return y


def gaussian_weights(sigma=2.5, truncate=4.0):
    w = np.zeros(64, np.float64)
    r = _lib().orc_gaussian_weights(float(sigma), float(truncate), _ptr(w), 64)
    return w[:2 * r + 1].copy()


def gaussian_filter(m, sigma=2.5):
    """scipy.ndimage.gaussian_filter(m, sigma) on a 2-D f32 map (pose_detector.py:86)."""
    m = np.ascontiguousarray(m, dtype=np.float32)
    H, W = m.shape
    w = gaussian_weights(sigma)
    out = np.empty_like(m)
    tmp = np.empty_like(m)
    _lib().orc_gaussian_filter(_ptr(m), _ptr(out), _ptr(tmp), H, W, _ptr(w), len(w) // 2)
    return out


def compute_peaks_from_heatmaps(heatmaps, params=PARAMS):
    """pose_detector.py:75-110 (CPU branch).  heatmaps (19,H,W); the last channel is dropped."""
    heatmaps = np.ascontiguousarray(heatmaps[:-1], dtype=np.float32)
    J, H, W = heatmaps.shape
    filt = np.stack([gaussian_filter(heatmaps[j], params["gaussian_sigma"]) for j in range(J)])
    cap = J * H * W
    out = np.empty((max(cap, 1), 5), np.float64)
    n = _lib().orc_find_peaks(_ptr(filt), J, H, W, float(np.float32(params["heatmap_peak_thresh"])), _ptr(out), cap)
    if n == 0:
        return np.array([])
    return out[:n].copy()


def create_gaussian_kernel(sigma=1, ksize=5):
    """pose_detector.py:38-44: the GPU branch's ksize x ksize kernel, exp(-d^2 / 2 sigma^2) /
    (2 pi sigma^2) in f64, NOT normalised, stored as f32."""
    center = int(ksize / 2)
    grid_x = np.tile(np.arange(ksize), (ksize, 1))
    grid_y = grid_x.transpose().copy()
    grid_d2 = (grid_x - center) ** 2 + (grid_y - center) ** 2
    return (1 / (sigma ** 2 * 2 * np.pi) * np.exp(-0.5 * grid_d2 / sigma ** 2)).astype("f")


def gpu_branch_filter(heatmaps, params=PARAMS):
    """pose_detector.py:112-113: F.convolution_2d(heatmaps[:, None], kernel, stride 1, pad ksize // 2)
    of the (J, H, W) f32 maps, zero padding.  The reference runs it as a cuDNN f32 convolution whose
    accumulation order is not specified; restated here as the exact sum (f64 over the f32 kernel)
    rounded once to f32, so a correct device result lies within a few f32 ulp of it."""
    h = np.asarray(heatmaps, np.float32)
    k = create_gaussian_kernel(params["gaussian_sigma"], params["ksize"]).astype(np.float64)
    ks = k.shape[0]
    r = ks // 2
    J, H, W = h.shape
    pad = np.zeros((J, H + 2 * r, W + 2 * r), np.float64)
    pad[:, r:r + H, r:r + W] = h
    acc = np.zeros((J, H, W), np.float64)
    for dy in range(ks):
        for dx in range(ks):
            acc += k[dy, dx] * pad[:, dy:dy + H, dx:dx + W]
    return acc.astype(np.float32)


def compute_peaks_gpu_branch(heatmaps, params=PARAMS):
    """pose_detector.py:75-79, 111-132 (GPU branch): the background channel dropped, the filter
    above, a peak where value > heatmap_peak_thresh and >= each of its 4 neighbours (0 outside the
    map); rows [joint, x, y, score, id] f64 in (joint, y, x) order, ids consecutive."""
    f = gpu_branch_filter(np.asarray(heatmaps)[:-1], params)
    nb = np.zeros((4,) + f.shape, np.float32)
    nb[0][:, 1:, :] = f[:, :-1, :]
    nb[1][:, :-1, :] = f[:, 1:, :]
    nb[2][:, :, 1:] = f[:, :, :-1]
    nb[3][:, :, :-1] = f[:, :, 1:]
    binary = (f > np.float32(params["heatmap_peak_thresh"])) & np.all(f[None] >= nb, axis=0)
    c, y, x = np.nonzero(binary)
    all_peaks = np.vstack((c, x, y, f[c, y, x])).transpose()
    return np.hstack((all_peaks, np.arange(len(all_peaks)).reshape(-1, 1)))


def compute_candidate_connections(paf, cand_a, cand_b, img_len, params=PARAMS):
    """pose_detector.py:135-159: list of [id_a, id_b, score] sorted by score desc."""
    paf = np.ascontiguousarray(paf, dtype=np.float32)
    ca = np.ascontiguousarray(cand_a, dtype=np.float64)
    cb = np.ascontiguousarray(cand_b, dtype=np.float64)
    _, H, W = paf.shape
    cap = max(len(ca) * len(cb), 1)
    out = np.empty((cap, 3), np.float64)
    prm = _params_struct(params)
    k = _lib().orc_candidate_connections(_ptr(paf[0]), _ptr(paf[1]), H, W, _ptr(ca), len(ca), _ptr(cb), len(cb),
                                         float(img_len), ctypes.byref(prm), _ptr(out), cap)
    return [[int(r[0]), int(r[1]), float(r[2])] for r in out[:k]]


def compute_connections(pafs, all_peaks, img_len, params=PARAMS):
    """pose_detector.py:161-181: list of 19 (K_l, 3) f64 arrays."""
    pafs = np.ascontiguousarray(pafs, dtype=np.float32)
    peaks = np.ascontiguousarray(all_peaks, dtype=np.float64).reshape(-1, 5)
    _, H, W = pafs.shape
    limbs = np.ascontiguousarray(np.array(params["limbs_point"], dtype=np.int32))
    L = len(limbs)
    cap = max(len(peaks) * L, 1)
    out = np.empty((cap, 3), np.float64)
    off = np.zeros(L + 1, np.int64)
    prm = _params_struct(params)
    st = _lib().orc_connections(_ptr(pafs), H, W, _ptr(peaks), len(peaks), _ptr(limbs), L, float(img_len),
                                ctypes.byref(prm), _ptr(out), cap, _ptr(off))
    if st != 0:
        raise RuntimeError("oracle compute_connections capacity")
    return [out[off[l]:off[l + 1]].copy().reshape(-1, 3) for l in range(L)]


def grouping_key_points(all_connections, candidate_peaks, params=PARAMS):
    """pose_detector.py:183-250: (S, 20) f64 subsets (IndexError where the reference raises it)."""
    L = len(all_connections)
    conn = np.ascontiguousarray(np.concatenate([np.asarray(c, np.float64).reshape(-1, 3) for c in all_connections]))
    off = np.zeros(L + 1, np.int64)
    off[1:] = np.cumsum([len(np.asarray(c).reshape(-1, 3)) for c in all_connections])
    limbs = np.ascontiguousarray(np.array(params["limbs_point"], dtype=np.int32))
    peaks = np.ascontiguousarray(candidate_peaks, dtype=np.float64).reshape(-1, 5)
    cap = max(len(conn), 1)
    subsets = np.empty((cap, 20), np.float64)
    n = ctypes.c_long(0)
    prm = _params_struct(params)
    st = _lib().orc_grouping(_ptr(conn), _ptr(off), _ptr(limbs), L, _ptr(peaks), ctypes.byref(prm),
                             _ptr(subsets), cap, ctypes.byref(n))
    if st == 4:
        raise IndexError("list assignment index out of range")
    if st != 0:
        raise RuntimeError("oracle grouping capacity")
    return subsets[:n.value].copy()


def subsets_to_pose_array(subsets, all_peaks):
    """pose_detector.py:252-265."""
    person_pose_array = []
    for subset in subsets:
        joints = []
        for joint_index in subset[:18].astype("i"):
            if joint_index >= 0:
                joint = all_peaks[joint_index][1:3].tolist()
                joint.append(2)
                joints.append(joint)
            else:
                joints.append([0, 0, 0])
        person_pose_array.append(np.array(joints))
    return np.array(person_pose_array)


def postprocess(paf_low, heat_low, orig_h, orig_w, params=PARAMS, return_debug=False, branch="cpu"):
    """pose_detector.py:501-517 from the last-stage network maps (38,h,w) and (19,h,w); branch 'gpu':
    the peaks of a detector built with device >= 0 (compute_peaks_gpu_branch)."""
    map_w, map_h = cvresize.compute_optimal_size(orig_h, orig_w, params["heatmap_size"])
    pafs = resize_images(paf_low, map_h, map_w)
    heatmaps = resize_images(heat_low, map_h, map_w)
    if branch == "gpu":
        all_peaks = compute_peaks_gpu_branch(heatmaps, params)
    else:
        all_peaks = compute_peaks_from_heatmaps(heatmaps, params)
    if len(all_peaks) == 0:
        res = (np.empty((0, N_JOINTS, 3)), np.empty(0))
        return (res + ({"all_peaks": all_peaks, "connections": None, "subsets": None},)) if return_debug else res
    all_connections = compute_connections(pafs, all_peaks, map_w, params)
    subsets = grouping_key_points(all_connections, all_peaks, params)
    dbg = {"all_peaks": all_peaks.copy(), "connections": all_connections, "subsets": subsets}
    all_peaks[:, 1] *= orig_w / map_w
    all_peaks[:, 2] *= orig_h / map_h
    poses = subsets_to_pose_array(subsets, all_peaks)
    scores = subsets[:, -2]
    return (poses, scores, dbg) if return_debug else (poses, scores)


def detect(weights, orig_img, params=PARAMS):
    """pose_detector.py:484-517 (single scale) on a BGR uint8 image with the oracle forward."""
    h, w = orig_img.shape[:2]
    in_w, in_h = cvresize.compute_optimal_size(h, w, params["inference_img_size"])
    x = cvresize.preprocess(cvresize.resize_linear_u8(orig_img, in_w, in_h))
    paf, heat = _fwd.cocoposenet_forward(weights, x)
    return postprocess(paf[0], heat[0], h, w, params)
