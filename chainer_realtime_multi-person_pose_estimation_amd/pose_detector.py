"""``PoseDetector`` — drop-in for the reference's detector (pose_detector.py:15-517), MI355X only.

Same constructor and call signature, same return types and empty-result shapes.  Each method
named after a reference method runs that step through the HIP library (C ABI in
include/openpose_hip.h); ``__call__`` runs the whole path on the device in one call
(resize + normalise, 92 convs, upsample, Gaussian + NMS, line integrals, greedy assignment,
grouping) and only the final poses come back to the host.

There is no CPU path: ``device=-1`` (the reference's CPU default) selects HIP device 0.
"""
import numpy as np

from . import _lib
from . import weights as _weights
from .constants import JointType, params


class PoseDetector(object):
    """PoseDetector(arch=None, weights_file=None, model=None, device=-1, precise=False)

    arch: 'posenet' (the CocoPoseNet path; entity.py:50-54).
    weights_file: Chainer npz written by serializers.save_npz (pose_detector.py:26).
    model: instead of a file, a {layer: (W, b)} dict (e.g. weights.random_weights()); like the
           reference's ``model=`` it skips loading from disk.
    device: HIP device ordinal (negative -> 0).
    precise: multi-scale inference (pose_detector.py:433-482).
    precision: 'bf16x3' (default; 3xBF16-split products with f32 accumulation, |err| ~3e-5 on the
               maps) or 'fp32' (exact f32 products on the f32 matrix cores).
    batch_invariant: keep one accumulation order for every batch size (by default a lone frame's
               convolutions split their input channels over workgroups: ~2x lower latency, f32
               re-association ~1e-5 against the same frame in a batch).
    peak_branch: which of the reference's two compute_peaks_from_heatmaps branches ``__call__``
               follows: 'cpu' (default; pose_detector.py:82-110, scipy gaussian_filter + strict NMS,
               what a reference detector with device=-1 returns) or 'gpu' (pose_detector.py:111-132,
               the 17x17 unnormalised zero-padded Gaussian + >= NMS a reference detector built with
               device >= 0 runs).  ``detect_precise`` and ``compute_peaks_from_heatmaps`` take the
               CPU branch either way, as in the reference (NumPy heatmaps there).
    """

    def __init__(self, arch=None, weights_file=None, model=None, device=-1, precise=False, max_batch=1,
                 precision="bf16x3", batch_invariant=False, peak_branch="cpu"):
        self.arch = arch
        self.precise = precise
        if model is None and arch not in (None, "posenet"):
            raise ValueError("arch %r is not on this path (only 'posenet')" % (arch,))
        self.device = 0 if device is None or device < 0 else int(device)
        limits = _lib.OpLimits()
        limits.max_batch = int(max_batch)
        self._ctx = _lib.Context(self.device, _lib.params_from_dict(params), limits)
        self._ctx.set_precision(precision)
        if batch_invariant:  # one accumulation order for every batch size (op_set_batch_invariant)
            self._ctx.set_batch_invariant(True)
        if peak_branch != "cpu":  # the reference's GPU-branch peaks in __call__ (op_set_peak_mode)
            self._ctx.set_peak_mode(peak_branch, params["ksize"])
        if model is not None:
            w = model
        elif weights_file:
            print("Loading the model...")
            w = _weights.load_npz(weights_file)
        else:
            print("Loading the model...")
            w = _weights.random_weights(0)
        self._ctx.set_weights(w)

    # ---- helpers mirrored from the reference (host-side arithmetic only) ----
    def create_gaussian_kernel(self, sigma=1, ksize=5):
        """pose_detector.py:38-44 (the reference's GPU-branch kernel; kept for API parity)."""
        center = int(ksize / 2)
        d2 = (np.arange(ksize)[None, :] - center) ** 2 + (np.arange(ksize)[:, None] - center) ** 2
        return (np.exp(-0.5 * d2 / sigma ** 2) / (sigma ** 2 * 2 * np.pi)).astype("f")

    def pad_image(self, img, stride, pad_value):
        """pose_detector.py:46-55: pad bottom/right to a multiple of stride with pad_value (the
        reference's result is int64: uint8 zeros plus the pad tuple)."""
        h, w, _ = img.shape
        pad = [(stride - (h % stride)) % stride, (stride - (w % stride)) % stride]
        out = np.zeros((h + pad[0], w + pad[1], 3), "uint8") + np.asarray(pad_value)
        out[:h, :w, :] = img
        return out, pad

    def compute_optimal_size(self, orig_img, img_size, stride=8):
        """pose_detector.py:57-73: (w, h) with the short side = img_size, multiples of stride."""
        h, w = orig_img.shape[:2]
        aspect = h / w
        if h < w:
            sh, sw = img_size, int(np.round(img_size / aspect))
            sw += (stride - sw % stride) % stride
        else:
            sw, sh = img_size, int(np.round(img_size * aspect))
            sh += (stride - sh % stride) % stride
        return sw, sh

    def preprocess(self, img):
        """pose_detector.py:426-431 (x/255 - 0.5, HWC -> 1x3xHxW, BGR kept)."""
        x = img.astype("f")
        x /= 255
        x -= 0.5
        return x.transpose(2, 0, 1)[None]

    # ---- hot-path steps on the device ----
    def compute_peaks_from_heatmaps(self, heatmaps):
        """pose_detector.py:75-110 (CPU semantics): (19,H,W) -> all_peaks (N,5) or array([])."""
        peaks = self._ctx.compute_peaks(np.asarray(heatmaps, np.float32))
        return peaks if len(peaks) else np.array([])

    def compute_connections(self, pafs, all_peaks, img_len, params):
        """pose_detector.py:161-181 -> list of 19 (K,3) f64 arrays."""
        self._check_params(params)
        return self._ctx.compute_connections(np.asarray(pafs, np.float32), all_peaks, img_len)

    def grouping_key_points(self, all_connections, candidate_peaks, params):
        """pose_detector.py:183-250 -> (S,20) f64 subsets (raises IndexError like the reference)."""
        self._check_params(params)
        return self._ctx.grouping(all_connections, candidate_peaks)

    def subsets_to_pose_array(self, subsets, all_peaks):
        """pose_detector.py:252-265."""
        rows = []
        for subset in subsets:
            ids = subset[:len(JointType)].astype("i")
            pose = np.zeros((len(JointType), 3))
            have = ids >= 0
            pose[have, :2] = all_peaks[ids[have]][:, 1:3]
            pose[have, 2] = 2
            rows.append(pose)
        return np.array(rows)

    def _check_params(self, p):
        if p is not params:
            for k in ("n_integ_points", "n_integ_points_thresh", "inner_product_thresh", "limb_length_ratio",
                      "length_penalty_value", "n_subset_limbs_thresh", "subset_score_thresh"):
                if p.get(k) != params[k]:
                    raise ValueError("params[%r] differs from the context's; build a new PoseDetector" % k)

    def detect_precise(self, orig_img):
        """pose_detector.py:433-482: multi-scale inference (params['inference_scales'], cubic resizes),
        post-processed at the original resolution.  Like the reference it leaves the averaged maps in
        self.pafs (38, H, W) / self.heatmaps (19, H, W) and the peaks in self.all_peaks."""
        img = np.asarray(orig_img)
        if img.dtype != np.uint8 or img.ndim != 3 or img.shape[2] != 3:
            raise ValueError("expected an H x W x 3 uint8 BGR image")
        poses, scores, res, self.pafs, self.heatmaps = self._ctx.detect_precise(img, return_maps=True)
        self.all_peaks = self.compute_peaks_from_heatmaps(self.heatmaps)
        if res.n_peaks == 0:
            return np.empty((0, len(JointType), 3)), np.empty(0)
        if res.n_persons == 0:
            return np.array([]), np.empty(0)
        return poses, scores

    def __call__(self, orig_img):
        """pose_detector.py:484-517: BGR uint8 image -> (poses (P,18,3) f64, scores (P,) f64)."""
        if self.precise:
            return self.detect_precise(orig_img)
        img = np.asarray(orig_img)
        if img.dtype != np.uint8 or img.ndim != 3 or img.shape[2] != 3:
            raise ValueError("expected an H x W x 3 uint8 BGR image")
        poses, scores, res = self._ctx.detect(img)
        if res.n_peaks == 0:
            return np.empty((0, len(JointType), 3)), np.empty(0)
        if res.n_persons == 0:
            return np.array([]), np.empty(0)
        return poses, scores

    # ---- crops for the face / hand detectors (restating pose_detector.py:266-425; host-side, used
    # by demo.py).  The arithmetic follows the reference operation for operation (the crop SHA-256
    # fixtures in tests/golden/cpm/ pin it); the structure is this module's own. ----

    # unit-length divisors (pose_detector.py:278-290): nose-neck, shoulder-elbow(R), neck-waist(R),
    # left ear-shoulder, right ear-shoulder first; every limb's divisor as the fallback
    _UNIT_BASE = ([14, 3, 0, 13, 9], np.array([0.85, 2.2, 2.2, 0.85, 0.85]))
    _UNIT_ALL = np.array([2.2, 1.7, 1.7, 2.2, 1.7, 1.7, 0.6, 0.93, 0.65, 0.85, 0.6, 0.93, 0.65, 0.85, 1, 0.2,
                          0.2, 0.25, 0.25])

    def compute_limbs_length(self, joints):
        """pose_detector.py:266-276 -> (lengths (19,) f64, [[joint_a, joint_b] or None per limb]).
        Rows of a pose array are never None, so every limb gets a length (0 for absent joints at 0,0)."""
        limbs = [None if joints[a] is None or joints[b] is None else [joints[a], joints[b]]
                 for a, b in params["limbs_point"]]
        lengths = np.zeros(len(limbs))
        for i, limb in enumerate(limbs):
            if limb is not None:
                lengths[i] = np.linalg.norm(limb[1][:-1] - limb[0][:-1])
        return lengths, limbs

    def compute_unit_length(self, limbs_len):
        """pose_detector.py:278-290: mean of length / divisor over the base limbs that were found,
        else over every limb that was found."""
        def mean_scaled(lengths, divisors):
            found = lengths > 0
            return np.sum(lengths[found] / divisors[found]) / np.count_nonzero(found)
        idx, div = self._UNIT_BASE
        base = limbs_len[idx]
        return mean_scaled(base, div) if np.any(base > 0) else mean_scaled(limbs_len, self._UNIT_ALL)

    def get_unit_length(self, person_pose):
        """pose_detector.py:292-296."""
        return self.compute_unit_length(self.compute_limbs_length(person_pose)[0])

    def crop_around_keypoint(self, img, keypoint, crop_size):
        """pose_detector.py:298-307: square of half-size crop_size about keypoint."""
        x, y = keypoint
        bbox = tuple(int(v) for v in (x - crop_size, y - crop_size, x + crop_size, y + crop_size))
        return self.crop_image(img, bbox), bbox

    def crop_person(self, img, person_pose, unit_length):
        """pose_detector.py:309-352.  The reference uses ``sys.maxsize`` without importing sys, so
        every call raises NameError there; this mirror raises the same error."""
        raise NameError("name 'sys' is not defined")

    def crop_face(self, img, person_pose, unit_length):
        """pose_detector.py:354-369: (face_img, bbox) from 1.2 units above to 0.8 below the nose and
        one unit either side of it, or (None, None) without a nose."""
        nx, ny, nv = person_pose[JointType.Nose][:3]
        if not nv > 0:
            return None, None
        bbox = (int(nx - unit_length), int(ny - unit_length * 1.2), int(nx + unit_length), int(ny + unit_length * 0.8))
        return self.crop_image(img, bbox), bbox

    def crop_hands(self, img, person_pose, unit_length):
        """pose_detector.py:371-399: {'left'|'right': {'img', 'bbox'} or None}; the centre moves 0.3 of
        the elbow->hand vector past the hand.  Like the reference, that shift is written into
        person_pose itself (the centre is a view of the hand row)."""
        out = {}
        for side, hand, elbow in (("left", JointType.LeftHand, JointType.LeftElbow),
                                  ("right", JointType.RightHand, JointType.RightElbow)):
            out[side] = None
            if not person_pose[hand][2] > 0:
                continue
            centre = person_pose[hand][:-1]  # a view: the in-place shift below reaches person_pose
            if person_pose[elbow][2] > 0:
                centre += (0.3 * (person_pose[hand][:-1] - person_pose[elbow][:-1])).astype(centre.dtype)
            crop, bbox = self.crop_around_keypoint(img, centre, unit_length * 0.95)
            out[side] = {"img": crop, "bbox": bbox}
        return {"left": out["left"], "right": out["right"]}

    def crop_image(self, img, bbox):
        """pose_detector.py:401-425: the (left, top, right, bottom) box of img; the parts of the box
        outside the image are zeros."""
        left, top, right, bottom = bbox
        h, w, ch = img.shape
        out = np.zeros((bottom - top, right - left, ch), np.uint8)
        y0, y1 = max(0, top), min(h, bottom)
        x0, x1 = max(0, left), min(w, right)
        out[y0 - top:y1 - top, x0 - left:x1 - left] = img[y0:y1, x0:x1]
        return out
