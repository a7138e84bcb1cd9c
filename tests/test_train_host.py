"""Training host side, CPU: preprocess (train_coco_pose_estimation.py:80-86), the
synthetic stand-in batches, and that the library exports the training ABI."""
import numpy as np

from conftest import pkg_module


def test_preprocess_matches_reference_formula():
    T = pkg_module("train")
    imgs = np.random.default_rng(0).integers(0, 256, (2, 16, 24, 3), dtype=np.uint8)
    x = imgs.astype("f")
    x /= 255
    x -= 0.5
    ref = x.transpose(0, 3, 1, 2)
    got = T.preprocess(imgs)
    assert got.dtype == np.float32 and got.shape == (2, 3, 16, 24) and np.array_equal(got, ref)


def test_synthetic_batch_shapes_and_ranges():
    T = pkg_module("train")
    imgs, paf, heat, ign = T.synthetic_batch(np.random.default_rng(1), 2, 64, 48)
    assert imgs.shape == (2, 64, 48, 3) and paf.shape == (2, 38, 8, 6) and heat.shape == (2, 19, 8, 6)
    assert ign.shape == (2, 8, 6) and ign.dtype == np.uint8
    assert heat.min() >= 0 and heat.max() <= 1 + 1e-6 and np.abs(paf).max() <= 1 + 1e-5
    assert np.allclose(heat[:, 18], 1 - heat[:, :18].max(axis=1))
    assert set(T.GRAD_SCALED) >= set(T.VGG_FROZEN) and len(T.GRAD_SCALED) == 12


def _schedule():
    import json
    import os
    with open(os.path.join(os.path.dirname(__file__), "golden", "train", "host_schedule.json")) as f:
        return json.load(f)


class FakeTrainContext(object):
    """Records what train.Updater asks of the device (no GPU): the layer table is the package's."""

    def __init__(self):
        self.table = pkg_module("weights").layer_table("posenet")
        self.enabled = {t[0]: True for t in self.table}
        self.scale = {t[0]: 1.0 for t in self.table}
        self.hyper = []
        self.events = []
        self.steps = 0

    def set_weights(self, w):
        pass

    def set_hyper(self, alpha, beta1=0.9, beta2=0.999, eps=1e-8):
        self.hyper.append((alpha, beta1, beta2, eps))

    def enable(self, i, on=True):
        self.enabled[self.table[i][0]] = bool(on)
        self.events.append((self.table[i][0], bool(on)))

    def set_grad_scale(self, i, s):
        self.scale[self.table[i][0]] = float(s)

    def step(self, x, pt, ht, ig):
        self.steps += 1
        return np.zeros(12)


def _fake_updater(resume=False):
    T = pkg_module("train")
    ctx = FakeTrainContext()
    up = T.Updater(1, 16, 16, model={}, ctx=ctx, resume=resume)
    return T, ctx, up


def test_updater_setup_equals_the_reference_main():
    """train_coco_pose_estimation.py's __main__ (:208-225) run under recording stubs
    (tests/golden/make_golden_train_host.py): Adam's hyperparameters, the GradientScaling hook's
    per-layer multiplier on all 92 layers (the reference's own __call__ applied to ones and random
    gradients), and the layers frozen at start."""
    g = _schedule()
    T, ctx, up = _fake_updater()
    assert [t[0] for t in ctx.table] == g["layer_order"]
    a = g["adam"]
    assert ctx.hyper[0] == (a["alpha"], a["beta1"], a["beta2"], a["eps"])
    assert (up.alpha, up.beta1, up.beta2, up.eps) == (a["alpha"], a["beta1"], a["beta2"], a["eps"])
    (hook,) = g["hooks"]
    assert [h.name for h in up.hooks] == [hook["name"]]
    assert list(up.hooks[0].layer_names) == hook["layer_names"] and up.hooks[0].scale == hook["scale"]
    assert ctx.scale == hook["multiplier_by_layer"]
    assert [n for n, on in ctx.events if not on] == g["frozen_at_start"]
    assert sorted(n for n, on in ctx.enabled.items() if not on) == sorted(g["frozen_at_start"])
    _, ctx2, _ = _fake_updater(resume=True)  # --resume: nothing frozen (:220)
    assert all(ctx2.enabled.values())


def test_updater_schedule_equals_the_reference_update_core():
    """The reference's own Updater.update_core (:90-126) driven at iterations around the schedule's
    edges: the layers it re-enables (all at 2000) and the optimizer alpha in force at each update."""
    g = _schedule()
    T, ctx, up = _fake_updater()
    batch = (np.zeros((1, 16, 16, 3), np.uint8), np.zeros((1, 38, 2, 2), np.float32),
             np.zeros((1, 19, 2, 2), np.float32), np.zeros((1, 2, 2), np.uint8))
    ctx.events.clear()
    alphas = []
    for it in g["iterations"]:
        up.iteration = it
        n0 = len(ctx.events)
        up.update(batch)
        alphas.append({"iteration": it, "alpha": ctx.hyper[-1][0]})
        for name, on in ctx.events[n0:]:
            assert on and {"layer": name, "iteration": it} in g["enable_events"], (it, name)
    assert alphas == g["updates"]
    assert [e[0] for e in ctx.events] == [e["layer"] for e in g["enable_events"]]
    assert all(ctx.enabled.values())
