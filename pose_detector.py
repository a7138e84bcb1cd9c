"""Drop-in shim: the reference's callers do ``from pose_detector import PoseDetector``
(pose_detector.py:15); this re-exports the MI355X implementation, including
``draw_person_pose`` and the reference's command line (``python pose_detector.py posenet W --img I``)."""
import importlib as _il

_pkg = _il.import_module("chainer_realtime_multi-person_pose_estimation_amd")
PoseDetector = _pkg.PoseDetector
params = _pkg.params
JointType = _pkg.JointType
draw_person_pose = _pkg.draw_person_pose

if __name__ == "__main__":
    import sys
    sys.exit(_il.import_module("chainer_realtime_multi-person_pose_estimation_amd.draw").main())
