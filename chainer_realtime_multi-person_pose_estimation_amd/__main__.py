"""python -m chainer_realtime_multi-person_pose_estimation_amd posenet WEIGHTS --img IMG [--precise]"""
import sys

from .draw import main

sys.exit(main())
