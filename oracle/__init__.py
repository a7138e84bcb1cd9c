"""ORACLE — TEST INFRASTRUCTURE ONLY.

CPU restatement of the reference hot path (``PoseDetector.__call__``, pose_detector.py:484-517)
used as the *checker* for the MI355X path.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import it; the product package never does.

* ``oracle/postproc.c`` (+ ``postproc.py``): plain C restatement of pose_detector.py:75-265 and
  the Chainer/SciPy map ops.  Pinned: tests/golden/ holds outputs of the reference's own
  post-process code (run in the build container under import stubs) and the tests check this
  restatement reproduces them bit for bit.
* ``oracle/forward.py``: NumPy restatement of Chainer's CPU forward of models/CocoPoseNet.py.
  Chainer is absent: parity unpinned at that boundary, cross-checked against an independent
  float64 convolution.
* ``oracle/cvresize.py``: OpenCV INTER_LINEAR restatement.  OpenCV is absent: parity unpinned.
"""
from . import cvresize, forward, postproc  # noqa: F401
