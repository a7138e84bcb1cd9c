"""MI355X-native OpenPose inference path (drop-in for PoseDetector.__call__ of
nk35jk/Chainer_Realtime_Multi-Person_Pose_Estimation).  See DESIGN.md."""
from .constants import JointType, params  # noqa: F401
from .pose_detector import PoseDetector  # noqa: F401
from . import weights  # noqa: F401
from .draw import draw_person_pose  # noqa: F401
