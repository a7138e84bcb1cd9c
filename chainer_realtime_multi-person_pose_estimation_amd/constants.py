"""Hot-path constants.

``JointType`` restates the 18-joint enum of the reference (entity.py:9-46) and ``params`` holds the
inference entries of its params dict (entity.py:70-105) and the face / hand detector entries
(entity.py:126-150) under the same keys, so callers written against the reference
(``params['limbs_point']``, ``JointType.Neck`` ...) work unchanged.  Training entries are outside
this path and are not carried.
"""
from enum import IntEnum

from .nets import CocoPoseNet, FaceNet, HandNet

_JOINT_NAMES = ("Nose Neck RightShoulder RightElbow RightHand LeftShoulder LeftElbow LeftHand "
                "RightWaist RightKnee RightFoot LeftWaist LeftKnee LeftFoot RightEye LeftEye "
                "RightEar LeftEar").split()

JointType = IntEnum("JointType", [(n, i) for i, n in enumerate(_JOINT_NAMES)])

# limb l connects joint LIMBS[l][0] -> LIMBS[l][1] (PAF channels 2l, 2l+1); entity.py:85-105
_LIMB_PAIRS = ((1, 8), (8, 9), (9, 10), (1, 11), (11, 12), (12, 13), (1, 2), (2, 3), (3, 4), (2, 16),
               (1, 5), (5, 6), (6, 7), (5, 17), (1, 0), (0, 14), (0, 15), (14, 16), (15, 17))

params = dict(
    archs={"posenet": CocoPoseNet, "facenet": FaceNet, "handnet": HandNet},  # entity.py:50-54: classes
    insize=368,
    downscale=8,
    inference_img_size=368,
    inference_scales=[0.5, 1, 1.5, 2],
    heatmap_size=320,
    gaussian_sigma=2.5,
    ksize=17,
    n_integ_points=10,
    n_integ_points_thresh=8,
    heatmap_peak_thresh=0.05,
    inner_product_thresh=0.05,
    limb_length_ratio=1.0,
    length_penalty_value=1,
    n_subset_limbs_thresh=3,
    subset_score_thresh=0.2,
    limbs_point=[[JointType(a), JointType(b)] for a, b in _LIMB_PAIRS],
    # face params (entity.py:126-140)
    face_inference_img_size=368,
    face_heatmap_peak_thresh=0.1,
    face_crop_scale=1.5,
    face_line_indices=[[i, i + 1] for i in range(16)] + [[i, i + 1] for i in range(17, 21)]
    + [[i, i + 1] for i in range(22, 26)] + [[27, 28], [28, 29], [29, 30]] + [[i, i + 1] for i in range(31, 35)]
    + [[i, i + 1] for i in range(36, 41)] + [[41, 36]] + [[i, i + 1] for i in range(42, 47)] + [[47, 42]]
    + [[i, i + 1] for i in range(48, 59)] + [[59, 48]] + [[i, i + 1] for i in range(60, 67)] + [[67, 60]],
    # hand params (entity.py:142-150)
    hand_inference_img_size=368,
    hand_heatmap_peak_thresh=0.1,
    fingers_indices=[[[0, 1], [1, 2], [2, 3], [3, 4]], [[0, 5], [5, 6], [6, 7], [7, 8]],
                     [[0, 9], [9, 10], [10, 11], [11, 12]], [[0, 13], [13, 14], [14, 15], [15, 16]],
                     [[0, 17], [17, 18], [18, 19], [19, 20]]],
)

N_JOINTS = len(JointType)
N_LIMBS = len(_LIMB_PAIRS)
