"""Drop-in shim for ``from entity import params, JointType`` (entity.py:9-152 of the reference;
only the inference constants exist on this path)."""
import importlib as _il

_c = _il.import_module("chainer_realtime_multi-person_pose_estimation_amd.constants")
params = _c.params
JointType = _c.JointType
