"""Layer tables of the three reference networks (host-side constants, no compute).

Each table is [(name, ci, co, k)] in the reference's declaration order:
  posenet  models/CocoPoseNet.py:26-129 (the HIP library's own table, op_layer_info, is the same;
           tests/test_convert.py checks it)
  facenet  models/FaceNet.py:11-76  (VGG-19 conv1-conv5 + conv5_3_CPM, stage 1 of two 1x1
           convs, stages 2-6 of 7x7 Mconv1-5 + 1x1 Mconv6-7 on concat(heat71, feature128) = 199)
  handnet  models/HandNet.py:11-76  (as FaceNet with 22 heatmaps: Mconv1 input 22 + 128 = 150)
and CONVERT_LAYERS[arch] is the reference converter's copy list (models/convert_model.py:8-248),
which for posenet omits conv5_5_CPM_L1 (that layer keeps its initial weights there).
"""


def _posenet():
    t = [("conv1_1", 3, 64, 3), ("conv1_2", 64, 64, 3), ("conv2_1", 64, 128, 3), ("conv2_2", 128, 128, 3),
         ("conv3_1", 128, 256, 3), ("conv3_2", 256, 256, 3), ("conv3_3", 256, 256, 3), ("conv3_4", 256, 256, 3),
         ("conv4_1", 256, 512, 3), ("conv4_2", 512, 512, 3), ("conv4_3_CPM", 512, 256, 3),
         ("conv4_4_CPM", 256, 128, 3)]
    for L, co in (("L1", 38), ("L2", 19)):
        t += [("conv5_1_CPM_" + L, 128, 128, 3), ("conv5_2_CPM_" + L, 128, 128, 3), ("conv5_3_CPM_" + L, 128, 128, 3),
              ("conv5_4_CPM_" + L, 128, 512, 1), ("conv5_5_CPM_" + L, 512, co, 1)]
    for st in range(2, 7):
        for L, co in (("L1", 38), ("L2", 19)):
            sfx = "_stage%d_%s" % (st, L)
            t += [("Mconv1" + sfx, 185, 128, 7)] + [("Mconv%d" % i + sfx, 128, 128, 7) for i in range(2, 6)]
            t += [("Mconv6" + sfx, 128, 128, 1), ("Mconv7" + sfx, 128, co, 1)]
    return t


def _cpm_single(n_maps):
    t = [("conv1_1", 3, 64, 3), ("conv1_2", 64, 64, 3), ("conv2_1", 64, 128, 3), ("conv2_2", 128, 128, 3),
         ("conv3_1", 128, 256, 3), ("conv3_2", 256, 256, 3), ("conv3_3", 256, 256, 3), ("conv3_4", 256, 256, 3),
         ("conv4_1", 256, 512, 3), ("conv4_2", 512, 512, 3), ("conv4_3", 512, 512, 3), ("conv4_4", 512, 512, 3),
         ("conv5_1", 512, 512, 3), ("conv5_2", 512, 512, 3), ("conv5_3_CPM", 512, 128, 3),
         ("conv6_1_CPM", 128, 512, 1), ("conv6_2_CPM", 512, n_maps, 1)]
    for st in range(2, 7):
        sfx = "_stage%d" % st
        t += [("Mconv1" + sfx, n_maps + 128, 128, 7)] + [("Mconv%d" % i + sfx, 128, 128, 7) for i in range(2, 6)]
        t += [("Mconv6" + sfx, 128, 128, 1), ("Mconv7" + sfx, 128, n_maps, 1)]
    return t


LAYERS = {"posenet": _posenet(), "facenet": _cpm_single(71), "handnet": _cpm_single(22)}

CONVERT_LAYERS = {
    "posenet": [n for n, _, _, _ in LAYERS["posenet"] if n != "conv5_5_CPM_L1"],
    "facenet": [n for n, _, _, _ in LAYERS["facenet"]],
    "handnet": [n for n, _, _, _ in LAYERS["handnet"]],
}


def layers(arch):
    if arch not in LAYERS:
        raise KeyError("unknown arch %r (expected one of %s)" % (arch, sorted(LAYERS)))
    return LAYERS[arch]


class _Net(dict):
    """A network's parameters as {layer: (W, b)}, built like the reference's Chainer models
    (models/CocoPoseNet.py:23-130, FaceNet.py / HandNet.py:10-76): every conv initialised with
    Chainer's defaults (LeCunNormal W, zero b; seeded here).  ``params['archs'][arch]()`` returns
    one, as pose_detector.py:23 expects; the detectors take it as ``model=`` and
    ``weights.load_npz(path, model)`` fills it in place like ``serializers.load_npz(path, model)``."""
    arch = None

    def __init__(self, seed=0):
        from .convert_model import initial_weights
        super().__init__(initial_weights(self.arch, seed))

    @property
    def layers(self):
        return layers(self.arch)


class CocoPoseNet(_Net):
    arch = "posenet"


class FaceNet(_Net):
    arch = "facenet"


class HandNet(_Net):
    arch = "handnet"
