"""Network weights on the host: the Chainer npz format and a seeded random initialiser.

* ``load_npz`` reads what ``chainer.serializers.save_npz(model)`` writes for CocoPoseNet
  (pose_detector.py:26): keys ``<layer>/W`` (Co, Ci, k, k) f32 and ``<layer>/b`` (Co,), possibly
  under a prefix (e.g. ``predictor/``).  Only NumPy's non-pickle loader is used.
* ``random_weights`` builds random-init weights of the same architecture (He-normal, so the
  activations stay O(1) through the 92 layers) for benchmarking without trained weights.
* ``arch``: 'posenet' (CocoPoseNet, default), 'facenet' or 'handnet' (layer tables: nets.py).
"""
import numpy as np

from . import _lib
from . import nets


def layer_table(arch="posenet"):
    return _lib.layer_table() if arch == "posenet" else nets.layers(arch)


def load_npz(path, arch="posenet"):
    """-> {layer: (W, b)}.  ``load_npz(path, model)`` with a model from nets (``params['archs'][a]()``)
    fills that model in place and returns it, like ``serializers.load_npz(path, model)``."""
    model = None
    if isinstance(arch, nets._Net):
        model, arch = arch, arch.arch
    with np.load(path, allow_pickle=False) as z:
        keys = list(z.keys())
        out = {}
        for name, ci, co, k in layer_table(arch):
            wk = [key for key in keys if key == name + "/W" or key.endswith("/" + name + "/W")]
            bk = [key for key in keys if key == name + "/b" or key.endswith("/" + name + "/b")]
            if not wk or not bk:
                raise KeyError("%s: no weights for layer %s" % (path, name))
            W = np.asarray(z[wk[0]], np.float32)
            b = np.asarray(z[bk[0]], np.float32)
            out[name] = (W, b)
    if model is not None:
        model.update(out)
        return model
    return out


def random_weights(seed=0, bias_scale=0.05, arch="posenet"):
    rng = np.random.default_rng(seed)
    out = {}
    for name, ci, co, k in layer_table(arch):
        fan_in = ci * k * k
        last = name.startswith("conv5_5") or name.startswith("Mconv7") or name == "conv6_2_CPM"
        std = np.sqrt((1.0 if last else 2.0) / fan_in)
        W = (rng.standard_normal((co, ci, k, k), dtype=np.float32) * np.float32(std)).astype(np.float32)
        b = rng.uniform(-bias_scale, bias_scale, co).astype(np.float32)
        out[name] = (W, b)
    return out


def save_npz(path, weights):
    """Write weights in the Chainer npz key layout (``<layer>/W``, ``<layer>/b``)."""
    flat = {}
    for name, (W, b) in weights.items():
        flat[name + "/W"] = W
        flat[name + "/b"] = b
    np.savez(path, **flat)
