"""Generate the FORWARD golden fixtures by running the REFERENCE's own network definitions.

Run in the build container only (it needs /root/reference, absent on the GPU box):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_forward.py

Chainer is not installed here, so the reference's ``models/CocoPoseNet.py``, ``models/FaceNet.py``
and ``models/HandNet.py`` are imported under op stubs and their UNMODIFIED ``__init__`` and
``__call__`` run:

* ``chainer.Chain.__init__(**links)`` registers each link as an attribute, in declaration order;
* ``L.Convolution2D(in_channels, out_channels, ksize, stride, pad)`` records its arguments (the
  layer table written to the fixture) and, when called, applies Chainer's CPU convolution as
  restated in ``oracle/forward.py`` (im2col + ``np.tensordot`` sgemm + bias, f32);
* ``F.relu`` / ``F.max_pooling_2d(ksize, stride)`` (pad 0, cover_all) / ``F.concat(axis=1)`` are
  the oracle's ops (Chainer CPU semantics).

So the wiring (layer order, which layers have a ReLU, where the pools sit, the concat order
``(paf, heat, feature)``, the six stage outputs) comes from the reference's own code; only the
per-op arithmetic is the restatement.  Weights come from
``chainer_realtime_multi-person_pose_estimation_amd.weights.random_weights(seed, arch=...)``
(NumPy PCG64 ``default_rng(seed)``: ``standard_normal(f32) * sqrt(g / (ci*k*k))`` per layer in
table order, g = 1 for the last conv of each stage, else 2, then ``uniform(-0.05, 0.05)`` biases);
the fixture stores a checksum of them so a changed generator is caught.  Inputs are
``default_rng(x_seed).uniform(-0.5, 0.5, shape)`` f32 (the range of ``x/255 - 0.5``), stored
for the small cases and regenerated from ``x_seed`` (checked against ``x_sum``) for the large ones.

Output: tests/golden/forward/<arch>_<n>x<h>x<w>.npz (data only, no code).
"""
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
OUT = os.path.join(HERE, "forward")
sys.path.insert(0, REPO)

from oracle import forward as OF  # noqa: E402

TRACE = []


class Convolution2D(object):
    """Recording stand-in for chainer.links.Convolution2D (Chainer 2+ keyword signature)."""

    def __init__(self, in_channels, out_channels, ksize=None, stride=1, pad=0, **kw):
        self.ci, self.co, self.k, self.stride, self.pad = in_channels, out_channels, ksize, stride, pad
        self.name = None
        self.W = self.b = None

    def __call__(self, x):
        assert self.stride == 1 and x.shape[1] == self.ci, (self.name, x.shape)
        y = OF.convolution_2d(x, self.W, self.b, self.pad)
        TRACE.append(("conv", self.name))
        return y


class Chain(object):
    def __init__(self, **links):
        self._links = []
        for name, link in links.items():  # kwargs keep declaration order (PEP 468)
            link.name = name
            setattr(self, name, link)
            self._links.append(name)


def relu(x):
    TRACE.append(("relu", ""))
    return OF.relu(x)


def max_pooling_2d(x, ksize, stride=None, pad=0, cover_all=True):
    assert pad == 0 and cover_all and ksize == 2 and (stride or ksize) == 2
    TRACE.append(("pool", ""))
    return OF.max_pooling_2d(x, ksize, stride or ksize)


def concat(xs, axis=1):
    TRACE.append(("concat", ",".join(str(v.shape[1]) for v in xs)))
    return np.concatenate(xs, axis=axis)


def install_stubs():
    for name in ["chainer", "chainer.functions", "chainer.links", "chainer.links.caffe"]:
        sys.modules[name] = types.ModuleType(name)
    ch = sys.modules["chainer"]
    ch.Chain = Chain
    ch.functions = F = sys.modules["chainer.functions"]
    ch.links = L = sys.modules["chainer.links"]
    L.caffe = sys.modules["chainer.links.caffe"]
    L.Convolution2D = Convolution2D
    F.relu, F.max_pooling_2d, F.concat = relu, max_pooling_2d, concat
    sys.path.insert(0, REF)


def weights_checksum(w, table):
    return np.array([float(np.float64(w[n][0]).sum()) + float(np.float64(w[n][1]).sum()) for n, _, _, _ in table])


def run(model, weights, x):
    for name in model._links:
        link = getattr(model, name)
        W, b = weights[name]
        assert W.shape == (link.co, link.ci, link.k, link.k), (name, W.shape)
        link.W, link.b = W, b
    del TRACE[:]
    return model(x)


def main():
    install_stubs()
    import importlib
    Wm = importlib.import_module("chainer_realtime_multi-person_pose_estimation_amd.weights")
    nets = importlib.import_module("chainer_realtime_multi-person_pose_estimation_amd.nets")
    from models.CocoPoseNet import CocoPoseNet
    from models.FaceNet import FaceNet
    from models.HandNet import HandNet
    os.makedirs(OUT, exist_ok=True)
    # (arch, class, weight seed, input seed, shape, keep every stage)
    cases = [
        ("posenet", CocoPoseNet, 0, 11, (1, 3, 64, 80), True),
        ("posenet", CocoPoseNet, 0, 12, (2, 3, 48, 48), True),
        ("posenet", CocoPoseNet, 0, 13, (1, 3, 184, 328), False),  # C4 scale 0.5 of 1280x720
        ("posenet", CocoPoseNet, 0, 14, (1, 3, 368, 368), False),  # the headline size
        ("facenet", FaceNet, 0, 21, (1, 3, 64, 64), True),
        ("facenet", FaceNet, 0, 22, (2, 3, 48, 40), True),
        ("handnet", HandNet, 0, 31, (1, 3, 64, 64), True),
        ("handnet", HandNet, 0, 32, (1, 3, 96, 128), True),
    ]
    wcache = {}
    for arch, cls, wseed, xseed, shape, every in cases:
        if (arch, wseed) not in wcache:
            wcache[arch, wseed] = Wm.random_weights(seed=wseed, arch=arch)
        weights = wcache[arch, wseed]
        model = cls()
        table = [(n, getattr(model, n).ci, getattr(model, n).co, getattr(model, n).k) for n in model._links]
        # the build's own layer tables must be the reference's declaration order and shapes
        assert table == [tuple(t) for t in nets.layers(arch)], arch
        pads = [getattr(model, n).pad for n in model._links]
        x = np.random.default_rng(xseed).uniform(-0.5, 0.5, shape).astype(np.float32)
        out = run(model, weights, x)
        rec = {"x_seed": xseed, "x_sum": np.float64(x).sum(), "weight_seed": wseed, "weights_checksum": weights_checksum(weights, table),
               "layer_names": np.array([t[0] for t in table]),
               "layer_shape": np.array([t[1:] + (p,) for t, p in zip(table, pads)], np.int32),  # ci, co, k, pad
               "trace_op": np.array([t[0] for t in TRACE]), "trace_arg": np.array([t[1] for t in TRACE])}
        if x.size <= 64 * 1024:
            rec["x"] = x  # larger inputs are regenerated from x_seed (checked against x_sum)
        if arch == "posenet":
            pafs, heats = out
            assert len(pafs) == len(heats) == 6
            stages = [(p, h) for p, h in zip(pafs, heats)]
            rec["paf"], rec["heat"] = pafs[-1], heats[-1]
            if every:
                rec["paf_stages"] = np.stack(pafs)
                rec["heat_stages"] = np.stack(heats)
            rec["stage_sums"] = np.array([[np.float64(p).sum(), np.float64(h).sum(), np.abs(np.float64(p)).sum(),
                                           np.abs(np.float64(h)).sum()] for p, h in stages])
        else:
            assert len(out) == 6
            rec["maps"] = out[-1]
            if every:
                rec["map_stages"] = np.stack(out)
            rec["stage_sums"] = np.array([[np.float64(m).sum(), np.abs(np.float64(m)).sum()] for m in out])
        name = "%s_%dx%dx%d" % (arch, shape[0], shape[2], shape[3])
        np.savez_compressed(os.path.join(OUT, name + ".npz"), **rec)
        print(name, "layers", len(table), "trace", len(TRACE), "max|out|",
              float(np.abs(rec["paf" if arch == "posenet" else "maps"]).max()))


if __name__ == "__main__":
    main()
