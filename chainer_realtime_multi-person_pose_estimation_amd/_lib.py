"""ctypes binding of libopenpose_hip.so (C ABI: include/openpose_hip.h).

There is no CPU fallback: if the HIP library is missing or cannot load, every entry point
raises.  Status codes map to the exceptions the reference would raise (IndexError for the
grouping overflow at pose_detector.py:197) or to RuntimeError/ValueError.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# OP_LIB_VARIANT=<name> loads libopenpose_hip.<name>.so instead (kernel tuning experiments only)
LIB_PATH = os.path.join(_HERE, "libopenpose_hip%s.so" % (
    "." + os.environ["OP_LIB_VARIANT"] if os.environ.get("OP_LIB_VARIANT") else ""))

OP_OK, OP_ERR_INVALID, OP_ERR_HIP, OP_ERR_CAPACITY, OP_ERR_INDEX, OP_ERR_STATE, OP_ERR_TIMEOUT = range(7)
OP_COMM_ID_BYTES = 128
N_JOINTS, N_LIMBS, N_PAF, N_HEAT, N_LAYERS = 18, 19, 38, 19, 92

# Every symbol include/openpose_hip.h declares (checked by tests/test_abi.py).
EXPORTED = (
    "op_last_error", "op_build_info", "op_default_params", "op_default_limits", "op_layer_info", "op_create", "op_destroy",
    "op_set_weights", "op_detect", "op_preprocess", "op_forward", "op_forward_stages", "op_resize_images", "op_compute_peaks",
    "op_compute_connections", "op_grouping", "op_postprocess", "op_stage_frames", "op_stage_maps",
    "op_use_staged_maps", "op_run_staged", "op_run_staged_graph", "op_graph_info", "op_synchronize", "op_fetch_result",
    "op_last_timing", "op_forward_flops", "op_profile_enable", "op_profile_read", "op_profile_reset",
    "op_set_precision", "op_get_precision", "op_fetch_results", "op_fetch_maps", "op_upload_frames", "op_upload_wait", "op_conv_census", "op_host_alloc", "op_host_free",
    "op_pack_results", "op_comm_unique_id", "op_comm_create", "op_comm_destroy", "op_comm_gather_results",
    "op_comm_wait", "op_comm_overflow", "op_comm_overflow_result", "op_detect_precise", "op_resize_cubic",
    "op_set_conv_algo", "op_set_stage_layout", "op_set_batch_invariant", "op_set_peak_mode", "op_profile_classes", "op_run_staged_precise",
    "op_cpm_layer_count", "op_cpm_layer_info", "op_cpm_create", "op_cpm_destroy", "op_cpm_set_weights",
    "op_cpm_forward", "op_cpm_peaks", "op_cpm_detect", "op_cpm_detect_batch", "op_cpm_set_batch_invariant",
    "op_train_create", "op_train_destroy", "op_train_set_weights", "op_train_get_weights", "op_train_set_hyper",
    "op_train_enable_layer", "op_train_set_grad_scale", "op_train_step",
)
ARCH = {"facenet": 1, "handnet": 2}
MAX_SCALES = 8
PRECISION = {"fp32": 0, "bf16x3": 1}
PEAK_BRANCH = {"cpu": 0, "gpu": 1}  # OP_PEAKS_CPU_BRANCH / OP_PEAKS_GPU_BRANCH


class OpParams(ctypes.Structure):
    _fields_ = [
        ("inference_img_size", ctypes.c_int32), ("heatmap_size", ctypes.c_int32),
        ("gaussian_sigma", ctypes.c_double), ("n_integ_points", ctypes.c_int32),
        ("n_integ_points_thresh", ctypes.c_int32), ("heatmap_peak_thresh", ctypes.c_double),
        ("inner_product_thresh", ctypes.c_double), ("limb_length_ratio", ctypes.c_double),
        ("length_penalty_value", ctypes.c_double), ("n_subset_limbs_thresh", ctypes.c_int32),
        ("subset_score_thresh", ctypes.c_double), ("limbs_point", (ctypes.c_int32 * 2) * N_LIMBS),
        ("downscale", ctypes.c_int32), ("n_scales", ctypes.c_int32),
        ("inference_scales", ctypes.c_double * MAX_SCALES),
    ]


class OpLimits(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        "max_batch", "max_net_h", "max_net_w", "max_map_h", "max_map_w", "max_peaks_per_joint",
        "max_frame_h", "max_frame_w")]


class OpFrameResult(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        "status", "n_peaks", "n_persons", "map_w", "map_h", "net_w", "net_h")]


_lib = None


def lib():
    """Load the HIP library (fails loudly: there is no other implementation of this path)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError("libopenpose_hip.so is not built (%s); run __graft_entry__.build() or "
                           "make -C chainer_realtime_multi-person_pose_estimation_amd/csrc" % LIB_PATH)
    L = ctypes.CDLL(LIB_PATH)
    P, I32, I64, D = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_double
    sig = {
        "op_last_error": ([], ctypes.c_char_p),
        "op_build_info": ([ctypes.c_char_p, I32], ctypes.c_int),
        "op_default_params": ([P], ctypes.c_int),
        "op_default_limits": ([P], ctypes.c_int),
        "op_layer_info": ([ctypes.c_int, ctypes.POINTER(ctypes.c_char_p), P, P, P], ctypes.c_int),
        "op_create": ([P, P, ctypes.c_int, P], ctypes.c_int),
        "op_destroy": ([P], ctypes.c_int),
        "op_set_weights": ([P, P, P], ctypes.c_int),
        "op_detect": ([P, P, I32, I32, I64, P, P, I32, P], ctypes.c_int),
        "op_detect_precise": ([P, P, I32, I32, I64, P, P, I32, P, P, P], ctypes.c_int),
        "op_set_conv_algo": ([P, I32], ctypes.c_int),
        "op_set_stage_layout": ([P, I32], ctypes.c_int),
        "op_set_batch_invariant": ([P, I32], ctypes.c_int),
        "op_set_peak_mode": ([P, I32, I32], ctypes.c_int),
        "op_profile_classes": ([P, I32], ctypes.c_int),
        "op_resize_cubic": ([P, P, I32, I32, I32, I32, P, I32, I32], ctypes.c_int),
        "op_preprocess": ([P, P, I32, I32, I64, I32, I32, P], ctypes.c_int),
        "op_forward": ([P, P, I32, I32, I32, P, P], ctypes.c_int),
        "op_forward_stages": ([P, P, I32, I32, I32, P, P], ctypes.c_int),
        "op_resize_images": ([P, P, I32, I32, I32, I32, I32, P], ctypes.c_int),
        "op_compute_peaks": ([P, P, I32, I32, I32, P, I64, P], ctypes.c_int),
        "op_compute_connections": ([P, P, I32, I32, P, I64, D, P, I64, P], ctypes.c_int),
        "op_grouping": ([P, P, P, P, I64, P, I64, P], ctypes.c_int),
        "op_postprocess": ([P, P, P, I32, I32, I32, I32, P, P, I32, P], ctypes.c_int),
        "op_stage_frames": ([P, P, I32, I32, I32], ctypes.c_int),
        "op_stage_maps": ([P, P, I32, I32, I32], ctypes.c_int),
        "op_use_staged_maps": ([P, I32], ctypes.c_int),
        "op_run_staged": ([P], ctypes.c_int),
        "op_run_staged_graph": ([P], ctypes.c_int),
        "op_graph_info": ([P, P, P, P, P, P], ctypes.c_int),
        "op_run_staged_precise": ([P], ctypes.c_int),
        "op_synchronize": ([P], ctypes.c_int),
        "op_fetch_result": ([P, I32, P, P, I32, P], ctypes.c_int),
        "op_last_timing": ([P, P, P, P], ctypes.c_int),
        "op_forward_flops": ([I32, I32], D),
        "op_profile_enable": ([P, I32], ctypes.c_int),
        "op_profile_read": ([P, I32, P, P, P, P], ctypes.c_int),
        "op_profile_reset": ([P], ctypes.c_int),
        "op_set_precision": ([P, I32], ctypes.c_int),
        "op_get_precision": ([P, P], ctypes.c_int),
        "op_fetch_results": ([P, I32, I32, P, P, I32, P], ctypes.c_int),
        "op_cpm_layer_count": ([I32], ctypes.c_int),
        "op_cpm_layer_info": ([I32, I32, ctypes.POINTER(ctypes.c_char_p), P, P, P], ctypes.c_int),
        "op_cpm_create": ([I32, I32, P], ctypes.c_int),
        "op_cpm_destroy": ([P], ctypes.c_int),
        "op_cpm_set_weights": ([P, P, P], ctypes.c_int),
        "op_cpm_forward": ([P, P, I32, I32, I32, P], ctypes.c_int),
        "op_cpm_peaks": ([P, P, I32, I32, I32, ctypes.c_float, I32, P, P], ctypes.c_int),
        "op_cpm_detect": ([P, P, I32, I32, I64, ctypes.c_float, I32, P, P], ctypes.c_int),
        "op_cpm_detect_batch": ([P, I32, P, P, P, P, ctypes.c_float, P, P, P], ctypes.c_int),
        "op_pack_results": ([P, I32, I32, I32, ctypes.c_int64, I32, P], ctypes.c_int),
        "op_comm_unique_id": ([P], ctypes.c_int),
        "op_comm_create": ([P, I32, I32, P, ctypes.c_double, P], ctypes.c_int),
        "op_comm_destroy": ([P], ctypes.c_int),
        "op_comm_gather_results": ([P, P, I32, I32, I32, ctypes.c_int64, I32], ctypes.c_int),
        "op_comm_wait": ([P, ctypes.c_double, P, P, P], ctypes.c_int),
        "op_comm_overflow": ([P, P, P, P, I32, P], ctypes.c_int),
        "op_comm_overflow_result": ([P, P, I32, P, P, I32, P], ctypes.c_int),
        "op_upload_frames": ([P, P, I32, I32, I32], ctypes.c_int),
        "op_upload_wait": ([P], ctypes.c_int),
        "op_conv_census": ([P, I32, I32], ctypes.c_int),
        "op_host_alloc": ([ctypes.c_size_t, P], ctypes.c_int),
        "op_host_free": ([P], ctypes.c_int),
        "op_fetch_maps": ([P, I32, I32, P, P, P, P], ctypes.c_int),
        "op_cpm_set_batch_invariant": ([P, I32], ctypes.c_int),
        "op_train_create": ([I32, I32, I32, I32, P], ctypes.c_int),
        "op_train_destroy": ([P], ctypes.c_int),
        "op_train_set_weights": ([P, P, P], ctypes.c_int),
        "op_train_get_weights": ([P, P, P, P, P], ctypes.c_int),
        "op_train_set_hyper": ([P, D, D, D, D], ctypes.c_int),
        "op_train_enable_layer": ([P, I32, I32], ctypes.c_int),
        "op_train_set_grad_scale": ([P, I32, D], ctypes.c_int),
        "op_train_step": ([P, P, P, P, P, P], ctypes.c_int),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    return L


def build_info():
    """The provenance baked into the loaded library at build time: "sha256:<hex>;defs=<flags>" --
    the digest of its sources and the build flags beyond csrc/Makefile's own (empty for the
    product library)."""
    buf = ctypes.create_string_buffer(1024)
    check(lib().op_build_info(buf, len(buf)), "op_build_info")
    return buf.value.decode("ascii")


def build_digest():
    """The source-digest part of build_info() ("sha256:<hex>")."""
    return build_info().split(";", 1)[0]


def build_flags():
    """The build-flags part of build_info(): "" for the product library."""
    info = build_info()
    return info.split(";defs=", 1)[1] if ";defs=" in info else ""


def check_provenance():
    """Assert the loaded library is the product build of this tree: its source digest equals the
    checked-out sources' and it was built without extra flags.  Returns the digest, or None when
    the sources are absent (an install without csrc/: the digest cannot be verified, nor refuted)."""
    flags = build_flags()
    assert flags == "", "libopenpose_hip.so is an experiment build (flags %r): rebuild the product library" % flags
    tree = source_digest()
    if tree is None:
        return None
    built = build_digest()
    assert built == tree, "libopenpose_hip.so digest %s != sources %s: rebuild it" % (built, tree)
    return built


def source_digest(csrc=None):
    """The same digest recomputed from the checked-out sources (csrc/Makefile DIGEST_SRCS: sha256
    of the `sha256sum` listing of csrc/*.hip *.hpp *.cpp, csrc/Makefile and include/*.h, paths as
    written relative to csrc/, in sorted order); None when the sources are not present."""
    import glob
    import hashlib
    csrc = csrc or os.path.join(_HERE, "csrc")
    if not os.path.isfile(os.path.join(csrc, "Makefile")):
        return None
    names = ["Makefile"]
    for pat in ("*.hip", "*.hpp", "*.cpp"):
        names += [os.path.basename(p) for p in glob.glob(os.path.join(csrc, pat))]
    names += ["../../include/" + os.path.basename(p) for p in glob.glob(os.path.join(csrc, "..", "..", "include", "*.h"))]
    listing = ""
    for n in sorted(names, key=lambda v: v.encode()):
        with open(os.path.join(csrc, n), "rb") as f:
            listing += "%s  %s\n" % (hashlib.sha256(f.read()).hexdigest(), n)
    return "sha256:" + hashlib.sha256(listing.encode()).hexdigest()


def last_error():
    return (lib().op_last_error() or b"").decode("utf-8", "replace")


def check(rc, what=""):
    if rc == OP_OK:
        return
    msg = "%s: %s" % (what, last_error()) if what else last_error()
    if rc == OP_ERR_INDEX:
        raise IndexError("list assignment index out of range")
    if rc == OP_ERR_INVALID:
        raise ValueError(msg)
    if rc == OP_ERR_TIMEOUT:
        raise TimeoutError(msg)
    raise RuntimeError("%s (status %d)" % (msg, rc))


def ptr(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


def default_params():
    p = OpParams()
    check(lib().op_default_params(ctypes.byref(p)))
    return p


def params_from_dict(d):
    p = default_params()
    for k in ("inference_img_size", "heatmap_size", "n_integ_points", "n_integ_points_thresh",
              "n_subset_limbs_thresh", "downscale"):
        if k in d:
            setattr(p, k, int(d[k]))
    for k in ("gaussian_sigma", "heatmap_peak_thresh", "inner_product_thresh", "limb_length_ratio",
              "length_penalty_value", "subset_score_thresh"):
        if k in d:
            setattr(p, k, float(d[k]))
    if "inference_scales" in d:
        sc = list(d["inference_scales"])
        if not 1 <= len(sc) <= MAX_SCALES:
            raise ValueError("inference_scales: 1..%d entries" % MAX_SCALES)
        p.n_scales = len(sc)
        for i, v in enumerate(sc):
            p.inference_scales[i] = float(v)
    if "limbs_point" in d:
        for i, (a, b) in enumerate(d["limbs_point"]):
            p.limbs_point[i][0] = int(a)
            p.limbs_point[i][1] = int(b)
    return p


def layer_table():
    """[(name, ci, co, k)] in models/CocoPoseNet.py:26-129 order, from the library."""
    out = []
    name = ctypes.c_char_p()
    ci, co, k = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
    for i in range(N_LAYERS):
        check(lib().op_layer_info(i, ctypes.byref(name), ctypes.byref(ci), ctypes.byref(co), ctypes.byref(k)))
        out.append((name.value.decode(), ci.value, co.value, k.value))
    return out


CENSUS = {"7x7_splitk": 11, "7x7_other": 12, "3x3_w48": 13, "3x3_w32": 14, "3x3_pool": 15, "3x3_splitk": 16,
          "3x3_big": 17, "conv1_pair": 18, "3x3_r256": 19, "3x3_r128": 20, "3x3_r_pool": 21,
          "7x7_planar": 22, "7x7_frame_aligned": 23, "7x7_tight": 24,
          "cubic_fused": 25, "cubic_two_pass": 26,
          "cubic_rows": 28, "f32_lds": 29, "7x7_stag": 30, "7x7_plain_ring": 31,
          "7x7_q": 32, "7x7_circ": 33, "precise_side": 34, "7x7_q_iwg": 35, "7x7_lin": 36, "7x7_q_bpf": 37, "7x7_pers": 38}
CENSUS_SLOTS = 40


def conv_census(reset=False):
    """Process-wide launch counts of the bf16x3 conv kernels (op_conv_census): {"npx": {NPX: n}
    for the 7x7 raster kernel, plus the CENSUS slots by name}."""
    a = (ctypes.c_int32 * CENSUS_SLOTS)()
    check(lib().op_conv_census(a, CENSUS_SLOTS, 1 if reset else 0), "op_conv_census")
    out = {"npx": {i: a[i] for i in range(1, 11) if a[i]}}
    out.update({k: a[v] for k, v in CENSUS.items()})
    return out


def forward_flops(h, w):
    return float(lib().op_forward_flops(int(h), int(w)))


class Context(object):
    """Owns one op_ctx (one device, one stream, packed weights in HBM)."""

    def __init__(self, device=0, params=None, limits=None):
        L = lib()
        self._p = params if params is not None else default_params()
        self._l = limits if limits is not None else OpLimits()
        h = ctypes.c_void_p()
        check(L.op_create(ctypes.byref(self._p), ctypes.byref(self._l), int(device), ctypes.byref(h)), "op_create")
        self.h = h
        self.device = device

    def close(self):
        if getattr(self, "h", None) is not None and self.h.value:
            lib().op_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_precision(self, mode):
        """'bf16x3' (default: 3xBF16 split products, f32 accumulate) or 'fp32' (exact f32 MFMA)."""
        check(lib().op_set_precision(self.h, PRECISION[mode]), "op_set_precision")

    def get_precision(self):
        m = ctypes.c_int32()
        check(lib().op_get_precision(self.h, ctypes.byref(m)), "op_get_precision")
        return {v: k for k, v in PRECISION.items()}[m.value]

    def set_weights(self, weights):
        """weights: {layer name: (W (Co,Ci,k,k) f32, b (Co,) f32)}."""
        table = layer_table()
        keep = []
        Wp = (ctypes.c_void_p * N_LAYERS)()
        bp = (ctypes.c_void_p * N_LAYERS)()
        for i, (name, ci, co, k) in enumerate(table):
            if name not in weights:
                raise KeyError("missing weights for layer %s" % name)
            W, b = weights[name]
            W = np.ascontiguousarray(W, dtype=np.float32)
            b = np.ascontiguousarray(b, dtype=np.float32).reshape(-1)
            if W.shape != (co, ci, k, k) or b.shape != (co,):
                raise ValueError("layer %s: expected W%s b(%d,), got %s %s" % (name, (co, ci, k, k), co, W.shape, b.shape))
            keep += [W, b]
            Wp[i] = W.ctypes.data
            bp[i] = b.ctypes.data
        check(lib().op_set_weights(self.h, Wp, bp), "op_set_weights")

    # ---- results ----
    def _result_arrays(self, cap):
        return np.empty((cap, N_JOINTS, 3), np.float64), np.empty(cap, np.float64), OpFrameResult()

    def detect(self, img, cap=2048):
        img = np.ascontiguousarray(img, dtype=np.uint8)
        if img.ndim != 3 or img.shape[2] != 3:
            raise ValueError("expected an H x W x 3 uint8 BGR image")
        poses, scores, res = self._result_arrays(cap)
        rc = lib().op_detect(self.h, ptr(img), img.shape[0], img.shape[1], img.strides[0], ptr(poses), ptr(scores),
                             cap, ctypes.byref(res))
        if rc == OP_ERR_CAPACITY and res.n_persons > cap:  # more persons than rows: the frame stays staged
            return self.fetch_result(0, cap=res.n_persons)
        check(rc, "op_detect")
        return poses[:res.n_persons].copy(), scores[:res.n_persons].copy(), res

    def set_conv_algo(self, algo):
        """Kernel family of the bf16x3 convolutions (include/openpose_hip.h: op_set_conv_algo)."""
        check(lib().op_set_conv_algo(self.h, int(algo)), "op_set_conv_algo")

    def set_stage_layout(self, planar):
        """Chunk-planar (1, default) or [row][col][channels] (0) 7x7 stage tensors
        (include/openpose_hip.h: op_set_stage_layout); the maps are bit-identical either way."""
        check(lib().op_set_stage_layout(self.h, 1 if planar else 0), "op_set_stage_layout")

    def set_peak_mode(self, branch="cpu", ksize=None):
        """Peak semantics of the single-scale post-process (include/openpose_hip.h: op_set_peak_mode):
        'cpu' (default; pose_detector.py:82-110) or 'gpu', the reference's GPU branch
        (pose_detector.py:111-132: ksize x ksize unnormalised Gaussian with zero padding, >= NMS;
        ksize defaults to params['ksize'] = 17)."""
        if branch not in PEAK_BRANCH:
            raise ValueError("peak branch %r: 'cpu' or 'gpu'" % (branch,))
        k = int(ksize if ksize is not None else 17)
        check(lib().op_set_peak_mode(self.h, PEAK_BRANCH[branch], k), "op_set_peak_mode")

    def set_batch_invariant(self, enable=True):
        """One accumulation order for every batch size (include/openpose_hip.h: op_set_batch_invariant);
        off by default: lone frames split their 7x7 input channels over workgroups (~2x lower latency)."""
        check(lib().op_set_batch_invariant(self.h, int(bool(enable))), "op_set_batch_invariant")

    def detect_precise(self, img, cap=2048, return_maps=False):
        """detect_precise (pose_detector.py:433-482): (poses, scores, res[, pafs (38,h,w), heatmaps (19,h,w)])."""
        img = np.ascontiguousarray(img, dtype=np.uint8)
        if img.ndim != 3 or img.shape[2] != 3:
            raise ValueError("expected an H x W x 3 uint8 BGR image")
        h, w = img.shape[:2]
        poses, scores, res = self._result_arrays(cap)
        pafs = np.empty((N_PAF, h, w), np.float32) if return_maps else None
        heat = np.empty((N_HEAT, h, w), np.float32) if return_maps else None
        rc = lib().op_detect_precise(self.h, ptr(img), h, w, img.strides[0], ptr(poses), ptr(scores), cap,
                                     ctypes.byref(res), ptr(pafs) if return_maps else None,
                                     ptr(heat) if return_maps else None)
        if rc == OP_ERR_CAPACITY and res.n_persons > cap:  # more persons than rows: the frame stays staged
            out = self.fetch_result(0, cap=res.n_persons)
            return out + (pafs, heat) if return_maps else out
        try:
            check(rc, "op_detect_precise")
        except IndexError as e:  # the averaged maps are valid: keep them for inspection
            e.maps = (pafs, heat)
            raise
        out = (poses[:res.n_persons].copy(), scores[:res.n_persons].copy(), res)
        return out + (pafs, heat) if return_maps else out

    def resize_cubic(self, img, out_w, out_h):
        """cv2.resize(img, (out_w, out_h), interpolation=cv2.INTER_CUBIC) for uint8 / float32 H x W (x C)."""
        a = np.asarray(img)
        if a.dtype == np.uint8:
            dt = 0
        elif a.dtype == np.float32:
            dt = 1
        else:
            raise ValueError("uint8 or float32 image expected")
        a = np.ascontiguousarray(a)
        cn = 1 if a.ndim == 2 else a.shape[2]
        out = np.empty((out_h, out_w, cn), a.dtype)
        check(lib().op_resize_cubic(self.h, ptr(a), dt, a.shape[0], a.shape[1], cn, ptr(out), out_h, out_w),
              "op_resize_cubic")
        return out if a.ndim == 3 else out[:, :, 0]

    def preprocess(self, img, out_w, out_h):
        img = np.ascontiguousarray(img, dtype=np.uint8)
        x = np.empty((1, 3, out_h, out_w), np.float32)
        check(lib().op_preprocess(self.h, ptr(img), img.shape[0], img.shape[1], img.strides[0], out_w, out_h, ptr(x)),
              "op_preprocess")
        return x

    def forward(self, x):
        x = np.ascontiguousarray(x, dtype=np.float32)
        n, c, h, w = x.shape
        if c != 3:
            raise ValueError("expected (n, 3, h, w)")
        paf = np.empty((n, N_PAF, h // 8, w // 8), np.float32)
        heat = np.empty((n, N_HEAT, h // 8, w // 8), np.float32)
        check(lib().op_forward(self.h, ptr(x), n, h, w, ptr(paf), ptr(heat)), "op_forward")
        return paf, heat

    def forward_stages(self, x):
        """All six stages: pafs (6, n, 38, h/8, w/8), heatmaps (6, n, 19, h/8, w/8)."""
        x = np.ascontiguousarray(x, dtype=np.float32)
        n, c, h, w = x.shape
        if c != 3:
            raise ValueError("expected (n, 3, h, w)")
        paf = np.empty((6, n, N_PAF, h // 8, w // 8), np.float32)
        heat = np.empty((6, n, N_HEAT, h // 8, w // 8), np.float32)
        check(lib().op_forward_stages(self.h, ptr(x), n, h, w, ptr(paf), ptr(heat)), "op_forward_stages")
        return paf, heat

    def resize_images(self, x, oh, ow):
        x = np.ascontiguousarray(x, dtype=np.float32)
        c, h, w = x.shape
        y = np.empty((c, oh, ow), np.float32)
        check(lib().op_resize_images(self.h, ptr(x), c, h, w, oh, ow, ptr(y)), "op_resize_images")
        return y

    def compute_peaks(self, heatmaps):
        heatmaps = np.ascontiguousarray(heatmaps, dtype=np.float32)
        c, h, w = heatmaps.shape
        cap = max(1, N_JOINTS * 2048)
        while True:  # uncapped: on a too-small array the library reports the rows it needs
            out = np.empty((cap, 5), np.float64)
            n = ctypes.c_int64()
            rc = lib().op_compute_peaks(self.h, ptr(heatmaps), c, h, w, ptr(out), cap, ctypes.byref(n))
            if rc == OP_ERR_CAPACITY and n.value > cap:
                cap = n.value
                continue
            check(rc, "op_compute_peaks")
            return out[:n.value].copy()

    def compute_connections(self, pafs, peaks, img_len):
        pafs = np.ascontiguousarray(pafs, dtype=np.float32)
        peaks = np.ascontiguousarray(np.asarray(peaks, np.float64).reshape(-1, 5))
        _, h, w = pafs.shape
        cap = max(1, N_LIMBS * 2048)
        while True:
            conn = np.empty((cap, 3), np.float64)
            off = np.zeros(N_LIMBS + 1, np.int64)
            rc = lib().op_compute_connections(self.h, ptr(pafs), h, w, ptr(peaks), len(peaks), float(img_len),
                                              ptr(conn), cap, ptr(off))
            if rc == OP_ERR_CAPACITY and off[N_LIMBS] > cap:
                cap = int(off[N_LIMBS])
                continue
            check(rc, "op_compute_connections")
            return [conn[off[l]:off[l + 1]].copy() for l in range(N_LIMBS)]

    def grouping(self, connections, peaks):
        peaks = np.ascontiguousarray(np.asarray(peaks, np.float64).reshape(-1, 5))
        rows = [np.asarray(c, np.float64).reshape(-1, 3) for c in connections]
        conn = np.ascontiguousarray(np.concatenate(rows) if rows else np.zeros((0, 3)))
        off = np.zeros(N_LIMBS + 1, np.int64)
        off[1:] = np.cumsum([len(r) for r in rows])
        cap = 2048
        cptr = conn if len(conn) else np.zeros((1, 3))
        while True:
            subsets = np.empty((cap, 20), np.float64)
            n = ctypes.c_int64()
            rc = lib().op_grouping(self.h, ptr(cptr), ptr(off), ptr(peaks), len(peaks), ptr(subsets), cap,
                                   ctypes.byref(n))
            if rc == OP_ERR_CAPACITY and n.value > cap:
                cap = n.value
                continue
            check(rc, "op_grouping")
            return subsets[:n.value].copy()

    def postprocess(self, paf_low, heat_low, orig_h, orig_w, cap=2048):
        paf_low = np.ascontiguousarray(paf_low, dtype=np.float32)
        heat_low = np.ascontiguousarray(heat_low, dtype=np.float32)
        _, h, w = paf_low.shape
        while True:
            poses, scores, res = self._result_arrays(cap)
            rc = lib().op_postprocess(self.h, ptr(paf_low), ptr(heat_low), h, w, int(orig_h), int(orig_w),
                                      ptr(poses), ptr(scores), cap, ctypes.byref(res))
            if rc == OP_ERR_CAPACITY and res.n_persons > cap:
                cap = res.n_persons
                continue
            check(rc, "op_postprocess")
            return poses[:res.n_persons].copy(), scores[:res.n_persons].copy(), res

    # ---- staged batched path ----
    def stage_frames(self, frames):
        frames = np.ascontiguousarray(frames, dtype=np.uint8)
        n, h, w, c = frames.shape
        check(lib().op_stage_frames(self.h, ptr(frames), n, h, w), "op_stage_frames")

    def upload_frames(self, frames):
        """Asynchronous staging (op_upload_frames): the next run_staged* uses these frames; keep
        `frames` (ideally a PinnedFrames array) unchanged until the copy has completed
        (upload_wait(), synchronize(), or a later call that waited for the consuming run)."""
        if frames.dtype != np.uint8 or frames.ndim != 4 or frames.shape[3] != 3 or not frames.flags.c_contiguous:
            raise ValueError("expected contiguous (n, h, w, 3) uint8 frames")
        n, h, w, _ = frames.shape
        check(lib().op_upload_frames(self.h, ctypes.c_void_p(frames.ctypes.data), n, h, w), "op_upload_frames")

    def upload_wait(self):
        """Block until every upload_frames copy has finished reading its host buffer."""
        check(lib().op_upload_wait(self.h), "op_upload_wait")

    def stage_maps(self, maps):
        maps = np.ascontiguousarray(maps, dtype=np.float32)
        n, c, h, w = maps.shape
        if c != N_PAF + N_HEAT:
            raise ValueError("maps must be (n, 57, h, w): 38 PAF then 19 heatmap channels")
        check(lib().op_stage_maps(self.h, ptr(maps), n, h, w), "op_stage_maps")

    def use_staged_maps(self, enable):
        check(lib().op_use_staged_maps(self.h, 1 if enable else 0))

    def run_staged(self, graph=False):
        check((lib().op_run_staged_graph if graph else lib().op_run_staged)(self.h), "op_run_staged")

    def run_staged_precise(self):
        """detect_precise on every staged frame (batched per scale; op_run_staged_precise)."""
        check(lib().op_run_staged_precise(self.h), "op_run_staged_precise")

    def synchronize(self):
        check(lib().op_synchronize(self.h), "op_synchronize")

    def graph_info(self):
        """Node counts of the last captured step graph (op_graph_info)."""
        v = [ctypes.c_int32() for _ in range(5)]
        check(lib().op_graph_info(self.h, *[ctypes.byref(x) for x in v]), "op_graph_info")
        return dict(zip(("nodes", "kernels", "memsets", "memcpys", "host_nodes"), (x.value for x in v)))

    def fetch_result(self, frame, cap=2048):
        while True:
            poses, scores, res = self._result_arrays(cap)
            rc = lib().op_fetch_result(self.h, int(frame), ptr(poses), ptr(scores), cap, ctypes.byref(res))
            if rc == OP_ERR_CAPACITY and res.n_persons > cap:
                cap = res.n_persons
                continue
            check(rc, "op_fetch_result")
            return poses[:res.n_persons].copy(), scores[:res.n_persons].copy(), res

    def fetch_results(self, first, n, cap=64):
        """Results of staged frames [first, first+n) in three copies: [(poses, scores, res), ...]."""
        while True:
            poses = np.empty((n, cap, N_JOINTS, 3), np.float64)
            scores = np.empty((n, cap), np.float64)
            res = (OpFrameResult * n)()
            rc = lib().op_fetch_results(self.h, int(first), int(n), ptr(poses), ptr(scores), cap, res)
            most = max(r.n_persons for r in res)
            if rc == OP_ERR_CAPACITY and most > cap:
                cap = most
                continue
            check(rc, "op_fetch_results")
            break
        return [(poses[i, :res[i].n_persons].copy(), scores[i, :res[i].n_persons].copy(), res[i]) for i in range(n)]

    def fetch_maps(self, first=0, n=1):
        """Network maps of staged frames [first, first+n): (pafs (n,38,h,w), heatmaps (n,19,h,w)) --
        the last-stage maps of run_staged, or the averaged full-resolution maps of run_staged_precise."""
        mh, mw = ctypes.c_int32(), ctypes.c_int32()
        check(lib().op_fetch_maps(self.h, int(first), int(n), None, None, ctypes.byref(mh), ctypes.byref(mw)),
              "op_fetch_maps")
        pafs = np.empty((n, N_PAF, mh.value, mw.value), np.float32)
        heat = np.empty((n, N_HEAT, mh.value, mw.value), np.float32)
        check(lib().op_fetch_maps(self.h, int(first), int(n), ptr(pafs), ptr(heat), ctypes.byref(mh),
                                  ctypes.byref(mw)), "op_fetch_maps")
        return pafs, heat

    def last_timing(self):
        a, b, t = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        check(lib().op_last_timing(self.h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(t)), "op_last_timing")
        return a.value, b.value, t.value

    # ---- per-kernel-class event timing ----
    PROFILE_CLASSES = ("conv7x7", "conv3x3", "conv1x1", "postprocess", "input", "map_resize", "other")

    def profile(self, enable=True):
        check(lib().op_profile_enable(self.h, 1 if enable else 0), "op_profile_enable")

    def profile_classes(self, names):
        """Time only these classes (names from PROFILE_CLASSES) while profiling is enabled."""
        mask = 0
        for n in names:
            mask |= 1 << self.PROFILE_CLASSES.index(n)
        check(lib().op_profile_classes(self.h, mask), "op_profile_classes")

    def profile_reset(self):
        check(lib().op_profile_reset(self.h), "op_profile_reset")

    def profile_read(self):
        """{class: (ms, launches, algorithmic flops, algorithmic bytes)} since the last reset."""
        out = {}
        for i, name in enumerate(self.PROFILE_CLASSES):
            ms, n, fl, by = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double(), ctypes.c_double()
            check(lib().op_profile_read(self.h, i, ctypes.byref(ms), ctypes.byref(n), ctypes.byref(fl),
                                        ctypes.byref(by)), "op_profile_read")
            out[name] = (ms.value, n.value, fl.value, by.value)
        return out


def cpm_layer_table(arch):
    """[(name, ci, co, k)] of FaceNet / HandNet (models/FaceNet.py:11-76) from the library."""
    a = ARCH[arch]
    out = []
    name = ctypes.c_char_p()
    ci, co, k = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
    for i in range(lib().op_cpm_layer_count(a)):
        check(lib().op_cpm_layer_info(a, i, ctypes.byref(name), ctypes.byref(ci), ctypes.byref(co), ctypes.byref(k)))
        out.append((name.value.decode(), ci.value, co.value, k.value))
    return out


def _row_strided_u8(img):
    """A uint8 H x W x 3 view whose pixels are packed within each row (rows may be strided, e.g. a
    crop view into a larger image: the device upload packs them); anything else is copied."""
    a = np.asarray(img)
    if a.dtype != np.uint8 or a.ndim != 3 or a.strides[2] != 1 or a.strides[1] != 3 or a.strides[0] < a.shape[1] * 3:
        a = np.ascontiguousarray(a, np.uint8)
    return a


class PinnedFrames(object):
    """(n, h, w, 3) uint8 frames in page-locked host memory (op_host_alloc), the source of
    asynchronous uploads (Context.upload_frames)."""

    def __init__(self, n, h, w):
        nbytes = int(n) * int(h) * int(w) * 3
        p = ctypes.c_void_p()
        check(lib().op_host_alloc(nbytes, ctypes.byref(p)), "op_host_alloc")
        self._p = p
        buf = (ctypes.c_uint8 * nbytes).from_address(p.value)
        self.array = np.frombuffer(buf, np.uint8).reshape(int(n), int(h), int(w), 3)

    def close(self):
        if getattr(self, "_p", None) is not None and self._p.value:
            self.array = None
            lib().op_host_free(self._p)
            self._p = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class CpmContext(object):
    """Owns one op_cpm_ctx: a FaceNet or HandNet replica on one device (face/hand detectors)."""

    def __init__(self, arch, device=0):
        if arch not in ARCH:
            raise ValueError("arch must be one of %s" % sorted(ARCH))
        self.arch = arch
        self.table = cpm_layer_table(arch)
        self.n_maps = self.table[-1][2]
        h = ctypes.c_void_p()
        check(lib().op_cpm_create(ARCH[arch], int(device), ctypes.byref(h)), "op_cpm_create")
        self.h = h

    def set_batch_invariant(self, enable=True):
        """No split-K on small launches: a crop's keypoints and confidences do not depend on the
        other crops of its batch (include/openpose_hip.h: op_cpm_set_batch_invariant)."""
        check(lib().op_cpm_set_batch_invariant(self.h, int(bool(enable))), "op_cpm_set_batch_invariant")

    def close(self):
        if getattr(self, "h", None) is not None and self.h.value:
            lib().op_cpm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_weights(self, weights):
        """weights: {layer: (W (Co,Ci,k,k), b (Co,))} for every layer of the table."""
        Ws, bs = [], []
        for name, ci, co, k in self.table:
            W, b = weights[name]
            W = np.ascontiguousarray(W, np.float32)
            b = np.ascontiguousarray(b, np.float32)
            if W.shape != (co, ci, k, k) or b.shape != (co,):
                raise ValueError("%s: expected W %s b %s, got %s %s" % (name, (co, ci, k, k), (co,), W.shape, b.shape))
            Ws.append(W)
            bs.append(b)
        self._keep = (Ws, bs)
        Wp = (ctypes.c_void_p * len(Ws))(*[w.ctypes.data for w in Ws])
        bp = (ctypes.c_void_p * len(bs))(*[v.ctypes.data for v in bs])
        check(lib().op_cpm_set_weights(self.h, Wp, bp), "op_cpm_set_weights")

    def forward(self, x):
        x = np.ascontiguousarray(x, np.float32)
        n, _, h, w = x.shape
        out = np.empty((n, self.n_maps, h // 8, w // 8), np.float32)
        check(lib().op_cpm_forward(self.h, ptr(x), n, h, w, ptr(out)), "op_cpm_forward")
        return out

    @staticmethod
    def _keypoints(kp, found):
        return [[int(k[0]), int(k[1]), np.float32(k[2])] if f else None for k, f in zip(kp, found)]

    def peaks(self, heatmaps, thresh, flip=False):
        hm = np.ascontiguousarray(heatmaps, np.float32)
        c, h, w = hm.shape
        kp = np.zeros((max(c - 1, 0), 3), np.float64)
        found = np.zeros(max(c - 1, 0), np.int32)
        check(lib().op_cpm_peaks(self.h, ptr(hm), c, h, w, float(thresh), int(bool(flip)), ptr(kp), ptr(found)),
              "op_cpm_peaks")
        return self._keypoints(kp, found)

    def detect(self, bgr, thresh, flip_maps=False):
        img = _row_strided_u8(bgr)
        if img.ndim != 3 or img.shape[2] != 3:
            raise ValueError("expected an H x W x 3 uint8 BGR image")
        h, w = img.shape[:2]
        kp = np.zeros((self.n_maps - 1, 3), np.float64)
        found = np.zeros(self.n_maps - 1, np.int32)
        check(lib().op_cpm_detect(self.h, ctypes.c_void_p(img.ctypes.data), h, w, img.strides[0], float(thresh),
                                  int(bool(flip_maps)), ptr(kp),
                                  ptr(found)), "op_cpm_detect")
        return self._keypoints(kp, found)

    def detect_batch(self, crops, thresh, flip_maps=None):
        """``detect`` over a list of BGR crops (any sizes) in one batched forward; the keypoints of
        one ``detect`` call per crop (confidences up to f32 re-association)."""
        imgs = [_row_strided_u8(c) for c in crops]
        for img in imgs:
            if img.ndim != 3 or img.shape[2] != 3:
                raise ValueError("expected H x W x 3 uint8 BGR crops")
        n, np_ = len(imgs), self.n_maps - 1
        if n == 0:
            return []
        ptrs = (ctypes.c_void_p * n)(*[img.ctypes.data for img in imgs])
        hs = np.array([img.shape[0] for img in imgs], np.int32)
        ws = np.array([img.shape[1] for img in imgs], np.int32)
        rs = np.array([img.strides[0] for img in imgs], np.int64)
        fl = np.array([int(bool(f)) for f in (flip_maps or [False] * n)], np.int32)
        if len(fl) != n:
            raise ValueError("flip_maps needs one entry per crop")
        kp = np.zeros((n, np_, 3), np.float64)
        found = np.zeros((n, np_), np.int32)
        check(lib().op_cpm_detect_batch(self.h, n, ptrs, ptr(hs), ptr(ws), ptr(rs), float(thresh), ptr(fl), ptr(kp),
                                        ptr(found)), "op_cpm_detect_batch")
        return [self._keypoints(kp[i], found[i]) for i in range(n)]


class TrainContext(object):
    """Owns one op_train_ctx: CocoPoseNet master weights, Adam state and the activations of a batch
    of n frames of h x w on one device (train_coco_pose_estimation.py's Updater on the GPU)."""

    def __init__(self, n, h, w, device=0):
        self.n, self.h, self.w = int(n), int(h), int(w)
        self.table = layer_table()
        hdl = ctypes.c_void_p()
        check(lib().op_train_create(int(device), self.n, self.h, self.w, ctypes.byref(hdl)), "op_train_create")
        self.h_ = hdl

    def close(self):
        if getattr(self, "h_", None) is not None and self.h_.value:
            lib().op_train_destroy(self.h_)
            self.h_ = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_weights(self, weights):
        Ws, bs = [], []
        for name, ci, co, k in self.table:
            W, b = weights[name]
            W = np.ascontiguousarray(W, np.float32)
            b = np.ascontiguousarray(b, np.float32)
            if W.shape != (co, ci, k, k) or b.shape != (co,):
                raise ValueError("%s: expected W %s, got %s" % (name, (co, ci, k, k), W.shape))
            Ws.append(W)
            bs.append(b)
        Wp = (ctypes.c_void_p * len(Ws))(*[a.ctypes.data for a in Ws])
        bp = (ctypes.c_void_p * len(bs))(*[a.ctypes.data for a in bs])
        check(lib().op_train_set_weights(self.h_, Wp, bp), "op_train_set_weights")

    def get(self, grads=False):
        """{layer: (W, b)} of the current weights, or of the last step's (unscaled) gradients."""
        out = {name: (np.empty((co, ci, k, k), np.float32), np.empty(co, np.float32))
               for name, ci, co, k in self.table}
        Wp = (ctypes.c_void_p * len(self.table))(*[out[t[0]][0].ctypes.data for t in self.table])
        bp = (ctypes.c_void_p * len(self.table))(*[out[t[0]][1].ctypes.data for t in self.table])
        args = (None, None, Wp, bp) if grads else (Wp, bp, None, None)
        check(lib().op_train_get_weights(self.h_, *args), "op_train_get_weights")
        return out

    def set_hyper(self, alpha, beta1=0.9, beta2=0.999, eps=1e-8):
        check(lib().op_train_set_hyper(self.h_, float(alpha), float(beta1), float(beta2), float(eps)),
              "op_train_set_hyper")

    def enable(self, layer_index, on=True):
        check(lib().op_train_enable_layer(self.h_, int(layer_index), int(bool(on))), "op_train_enable_layer")

    def set_grad_scale(self, layer_index, scale):
        check(lib().op_train_set_grad_scale(self.h_, int(layer_index), float(scale)), "op_train_set_grad_scale")

    def step(self, x, pafs_t, heatmaps_t, ignore_mask):
        n, h8, w8 = self.n, self.h // 8, self.w // 8
        x = np.ascontiguousarray(x, np.float32)
        pt = np.ascontiguousarray(pafs_t, np.float32)
        ht = np.ascontiguousarray(heatmaps_t, np.float32)
        ig = np.ascontiguousarray(ignore_mask, np.uint8)
        if x.shape != (n, 3, self.h, self.w) or pt.shape != (n, 38, h8, w8) or ht.shape != (n, 19, h8, w8) \
                or ig.shape != (n, h8, w8):
            raise ValueError("train step: shapes (n,3,h,w) (n,38,h/8,w/8) (n,19,h/8,w/8) (n,h/8,w/8) expected")
        losses = np.zeros(12, np.float64)
        check(lib().op_train_step(self.h_, ptr(x), ptr(pt), ptr(ht), ptr(ig), ptr(losses)), "op_train_step")
        return losses
