"""ORACLE — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

CPU restatement of the face / hand detectors:
  * ``cpm_forward`` — FaceNet / HandNet ``__call__`` (models/FaceNet.py:78-161,
    models/HandNet.py:78-161) on Chainer's CPU primitives (oracle/forward.py): VGG conv1-conv5
    with three 2x2 pools, conv5_3_CPM, stage 1 = conv6_1_CPM (ReLU) + conv6_2_CPM, stages 2-6 on
    concat((heatmaps, feature_map)) = Mconv1-5 7x7 + Mconv6 1x1 (ReLU) + Mconv7 1x1.  Chainer is
    absent: parity unpinned at that boundary (same restatement as the CocoPoseNet forward).
  * ``compute_peaks_from_heatmaps`` — face_detector.py:58-84 / hand_detector.py:68-94 CPU
    branch: per map but the last, scipy gaussian_filter (oracle/postproc.c restatement, bit-exact),
    global max, and ``np.where(heatmap == max)`` flattened -> ``[coords[1], coords[0], max]``
    (with several maxima that is [y1, y0], the reference's own quirk).  Pinned by
    tests/golden/cpm/*_peaks.npz (the reference's own function).
  * ``detect`` — FaceDetector.__call__ (face_detector.py:29-42) / HandDetector.__call__
    (hand_detector.py:29-53): cv2 LINEAR resize to 368x368 (oracle/cvresize.py, unpinned),
    ``x / 256 - 0.5``, forward, F.resize_images to the crop size, optional horizontal flips for a
    left hand, peaks.
"""
import numpy as np

from . import cvresize
from . import forward as F
from . import postproc as P

PARAMS = {"face_inference_img_size": 368, "face_heatmap_peak_thresh": 0.1,
          "hand_inference_img_size": 368, "hand_heatmap_peak_thresh": 0.1, "gaussian_sigma": 2.5}
N_MAPS = {"facenet": 71, "handnet": 22}


def cpm_forward(weights, x, all_stages=False):
    """weights: {name: (W, b)} of FaceNet or HandNet; x (N,3,H,W) f32 -> last-stage maps (N,C,H/8,W/8)."""
    def conv(name, h, act=True):
        W, b = weights[name]
        y = F.convolution_2d(h, W, b, W.shape[2] // 2)
        return F.relu(y) if act else y

    h = conv("conv1_1", x)
    h = conv("conv1_2", h)
    h = F.max_pooling_2d(h)
    h = conv("conv2_1", h)
    h = conv("conv2_2", h)
    h = F.max_pooling_2d(h)
    for n in ("conv3_1", "conv3_2", "conv3_3", "conv3_4"):
        h = conv(n, h)
    h = F.max_pooling_2d(h)
    for n in ("conv4_1", "conv4_2", "conv4_3", "conv4_4", "conv5_1", "conv5_2", "conv5_3_CPM"):
        h = conv(n, h)
    feature_map = h
    h = conv("conv6_1_CPM", h)
    h = conv("conv6_2_CPM", h, act=False)
    maps = [h]
    for s in range(2, 7):
        h = np.concatenate((h, feature_map), axis=1)
        for i in range(1, 7):
            h = conv("Mconv%d_stage%d" % (i, s), h)
        h = conv("Mconv7_stage%d" % s, h, act=False)
        maps.append(h)
    return maps if all_stages else maps[-1]


def preprocess(img):
    """np.array(resized[None], f32).transpose(0, 3, 1, 2) / 256 - 0.5 (face_detector.py:33)."""
    x = np.array(img[np.newaxis], dtype=np.float32).transpose(0, 3, 1, 2) / 256 - 0.5
    return np.ascontiguousarray(x.astype(np.float32))


def compute_peaks_from_heatmaps(heatmaps, thresh, sigma=2.5):
    """list of [x, y, max] or None per map but the last."""
    keypoints = []
    for i in range(heatmaps.shape[0] - 1):
        heatmap = P.gaussian_filter(heatmaps[i], sigma)
        max_value = heatmap.max()
        if max_value > thresh:
            coords = np.array(np.where(heatmap == max_value)).flatten().tolist()
            keypoints.append([coords[1], coords[0], max_value])
        else:
            keypoints.append(None)
    return keypoints


def detect(weights, arch, img, hand_type="right", return_maps=False):
    if arch == "handnet" and hand_type == "left":
        img = np.ascontiguousarray(img[:, ::-1])
    h, w = img.shape[:2]
    size = PARAMS["face_inference_img_size" if arch == "facenet" else "hand_inference_img_size"]
    x = preprocess(cvresize.resize_linear_u8(img, size, size))
    low = cpm_forward(weights, x)[0]
    heat = P.resize_images(low, h, w)
    if arch == "handnet" and hand_type == "left":
        heat = np.ascontiguousarray(heat[:, :, ::-1])
    thresh = PARAMS["face_heatmap_peak_thresh" if arch == "facenet" else "hand_heatmap_peak_thresh"]
    kps = compute_peaks_from_heatmaps(heat, thresh)
    return (kps, low, heat) if return_maps else kps
