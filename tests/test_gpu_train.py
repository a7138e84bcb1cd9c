"""Training iteration on the GPU against an independent float64 torch autograd
restatement of train_coco_pose_estimation.py:42-123 (CocoPoseNet.__call__ with every stage's maps,
compute_loss with the ignore mask, backward) and of Chainer's Adam + GradientScaling hook.  torch
is the checker here only (tests); the product path is op_train_step."""
import numpy as np
import pytest

from conftest import pkg_module

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def torch_step(W, x, pafs_t, heat_t, ignore):
    """(losses[12], grads {layer: (gW, gb)}) in float64."""
    tf = torch.nn.functional
    P = {k: (torch.tensor(w, dtype=torch.float64, requires_grad=True),
             torch.tensor(b, dtype=torch.float64, requires_grad=True)) for k, (w, b) in W.items()}

    def conv(name, h, act=True):
        w, b = P[name]
        y = tf.conv2d(h, w, b, padding=w.shape[2] // 2)
        return torch.relu(y) if act else y

    h = torch.tensor(x, dtype=torch.float64)
    for blk in (("conv1_1", "conv1_2"), ("conv2_1", "conv2_2"), ("conv3_1", "conv3_2", "conv3_3", "conv3_4")):
        for n in blk:
            h = conv(n, h)
        h = tf.max_pool2d(h, 2)
    for n in ("conv4_1", "conv4_2", "conv4_3_CPM", "conv4_4_CPM"):
        h = conv(n, h)
    feat = h
    outs = []
    h1, h2 = feat, feat
    for i in (1, 2, 3, 4):
        h1 = conv("conv5_%d_CPM_L1" % i, h1)
        h2 = conv("conv5_%d_CPM_L2" % i, h2)
    h1, h2 = conv("conv5_5_CPM_L1", h1, False), conv("conv5_5_CPM_L2", h2, False)
    outs.append((h1, h2))
    for s in range(2, 7):
        cat = torch.cat((h1, h2, feat), 1)
        t1, t2 = cat, cat
        for i in range(1, 7):
            t1 = conv("Mconv%d_stage%d_L1" % (i, s), t1)
            t2 = conv("Mconv%d_stage%d_L2" % (i, s), t2)
        h1, h2 = conv("Mconv7_stage%d_L1" % s, t1, False), conv("Mconv7_stage%d_L2" % s, t2, False)
        outs.append((h1, h2))
    pt = torch.tensor(pafs_t, dtype=torch.float64)
    ht = torch.tensor(heat_t, dtype=torch.float64)
    m = torch.tensor(ignore.astype(bool))[:, None]
    total = 0
    losses = []
    for py, hy in outs:  # compute_loss: masked targets take the prediction's value
        tp = torch.where(m.expand_as(py), py.detach(), pt)
        th = torch.where(m.expand_as(hy), hy.detach(), ht)
        lp, lh = ((py - tp) ** 2).mean(), ((hy - th) ** 2).mean()
        losses += [float(lp), float(lh)]
        total = total + lp + lh
    total.backward()
    return np.array(losses), {k: (w.grad.numpy(), b.grad.numpy()) for k, (w, b) in P.items()}


def _hook_multipliers():
    import json
    import os
    with open(os.path.join(os.path.dirname(__file__), "golden", "train", "host_schedule.json")) as f:
        return json.load(f)["hooks"][0]["multiplier_by_layer"]


def adam_ref(p, g, scale, t, alpha=1e-4, b1=0.9, b2=0.999, eps=1e-8):
    """Chainer AdamRule on fresh state after t identical-gradient steps is not what we test; one step."""
    g = (g * np.float32(scale)).astype(np.float32)
    m = (np.float32(1 - b1) * g).astype(np.float32)
    v = (np.float32(1 - b2) * g * g).astype(np.float32)
    lr = alpha * np.sqrt(1 - b2 ** t) / (1 - b1 ** t)
    return (p - np.float32(lr) * m / (np.sqrt(v) + np.float32(eps))).astype(np.float32)


def _data(n, h, w, seed):
    rng = np.random.default_rng(seed)
    x = rng.uniform(-0.5, 0.5, (n, 3, h, w)).astype(np.float32)
    pt = rng.uniform(-1, 1, (n, 38, h // 8, w // 8)).astype(np.float32)
    ht = rng.uniform(0, 1, (n, 19, h // 8, w // 8)).astype(np.float32)
    ig = (rng.random((n, h // 8, w // 8)) < 0.2).astype(np.uint8)
    return x, pt, ht, ig


@pytest.mark.parametrize("frozen", [False, True])
def test_train_step_vs_torch_float64(frozen):
    lib = pkg_module("_lib")
    W0 = pkg_module("weights").random_weights(seed=7)
    n, h, w = 2, 64, 48
    x, pt, ht, ig = _data(n, h, w, 3)
    ctx = lib.TrainContext(n, h, w, 0)
    try:
        ctx.set_weights(W0)
        ctx.set_hyper(1e-4)
        names = [t[0] for t in ctx.table]
        # the reference's GradientScaling hook, as its own __call__ applied it per layer
        # (tests/golden/train/host_schedule.json, make_golden_train_host.py)
        mult = _hook_multipliers()
        for nm, sc in mult.items():
            if sc != 1.0:
                ctx.set_grad_scale(names.index(nm), sc)
        vgg = pkg_module("train").VGG_FROZEN
        if frozen:
            for nm in vgg:
                ctx.enable(names.index(nm), False)
        losses = ctx.step(x, pt, ht, ig)
        grads = ctx.get(grads=True)
        W1 = ctx.get()
    finally:
        ctx.close()
    ref_losses, ref_grads = torch_step(W0, x, pt, ht, ig)
    np.testing.assert_allclose(losses, ref_losses, rtol=2e-5)
    worst = 0.0
    for nm in names:
        gW, gb = grads[nm]
        if frozen and nm in vgg:
            assert not gW.any() and not gb.any()
            assert np.array_equal(W1[nm][0], W0[nm][0]) and np.array_equal(W1[nm][1], W0[nm][1])
            continue
        rW, rb = ref_grads[nm]
        sW = max(np.abs(rW).max(), 1e-30)
        errW = np.abs(gW - rW).max() / sW
        errb = np.abs(gb - rb).max() / max(np.abs(rb).max(), 1e-30)
        worst = max(worst, errW, errb)
        assert errW <= 2e-3 and errb <= 2e-3, (nm, errW, errb)
        # the Adam step on the device's own gradients times the reference hook's multiplier
        sc = mult[nm]
        np.testing.assert_allclose(W1[nm][0], adam_ref(W0[nm][0], gW, sc, 1), rtol=0, atol=2e-7)
        np.testing.assert_allclose(W1[nm][1], adam_ref(W0[nm][1], gb, sc, 1), rtol=0, atol=2e-7)
    print("train step: max relative gradient error vs float64 = %.3g" % worst)


def test_updater_schedule_and_loss_decreases():
    T = pkg_module("train")
    up = T.Updater(2, 64, 64, model=pkg_module("weights").random_weights(seed=1))
    rng = np.random.default_rng(0)
    batch = T.synthetic_batch(rng, 2, 64, 64)
    first = up.update(batch)[0]
    for _ in range(5):
        last = up.update(batch)[0]
    assert up.iteration == 6 and last < first  # the same batch: Adam must make progress
    g = up.grads()
    assert not g["conv1_1"][0].any() and g["conv4_3_CPM"][0].any()  # VGG frozen until iteration 2000
    up.ctx.close()


@pytest.mark.parametrize("case", ["posenet_2x48x48", "posenet_1x64x80"])
def test_train_step_losses_vs_reference_compute_loss(case):
    """op_train_step's twelve per-stage losses against the REFERENCE's own compute_loss
    (train_coco_pose_estimation.py:41-73, tests/golden/train/, made by make_golden_train.py) on the
    reference network's own stage outputs for the same weights (seed 0) and input.  The device
    recomputes the forward itself (exact f32), so the losses agree to the forward's 1e-3-level map
    agreement, far tighter in relative terms: rtol 1e-4."""
    from test_train_golden import load_train_case
    from test_forward_golden import case_weights, load_case
    lib = pkg_module("_lib")
    g, _ = load_train_case(case)
    _, d = load_case(case)
    n, h, w = d["x"].shape[0], d["x"].shape[2], d["x"].shape[3]
    ctx = lib.TrainContext(n, h, w, 0)
    try:
        ctx.set_weights(case_weights("posenet", 0))
        losses = ctx.step(d["x"], g["pafs_t"], g["heatmaps_t"], g["ignore_mask"])
    finally:
        ctx.close()
    want = np.stack([g["paf_loss"], g["heat_loss"]], 1).reshape(-1)  # [paf, heat] per stage
    print(case, "max rel loss error vs reference compute_loss: %.3g" % float(np.max(np.abs(losses - want) / want)))
    np.testing.assert_allclose(losses, want, rtol=1e-4)
