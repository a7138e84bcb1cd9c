"""Hot-path constants.

``JointType`` restates the 18-joint enum of the reference (entity.py:9-46) and ``params`` holds the
inference entries of its params dict (entity.py:70-105) under the same keys, so callers written
against the reference (``params['limbs_point']``, ``JointType.Neck`` ...) work unchanged.
Training / face / hand entries are outside this path and are not carried.
"""
from enum import IntEnum

_JOINT_NAMES = ("Nose Neck RightShoulder RightElbow RightHand LeftShoulder LeftElbow LeftHand "
                "RightWaist RightKnee RightFoot LeftWaist LeftKnee LeftFoot RightEye LeftEye "
                "RightEar LeftEar").split()

JointType = IntEnum("JointType", [(n, i) for i, n in enumerate(_JOINT_NAMES)])

# limb l connects joint LIMBS[l][0] -> LIMBS[l][1] (PAF channels 2l, 2l+1); entity.py:85-105
_LIMB_PAIRS = ((1, 8), (8, 9), (9, 10), (1, 11), (11, 12), (12, 13), (1, 2), (2, 3), (3, 4), (2, 16),
               (1, 5), (5, 6), (6, 7), (5, 17), (1, 0), (0, 14), (0, 15), (14, 16), (15, 17))

params = dict(
    archs={"posenet": "CocoPoseNet"},
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
)

N_JOINTS = len(JointType)
N_LIMBS = len(_LIMB_PAIRS)
