"""The NumPy forward restatement (Chainer CPU semantics) against an independent float64 conv."""
import numpy as np
import torch

from oracle import forward as F


def _ref_conv64(x, W, b):
    y = torch.nn.functional.conv2d(torch.from_numpy(x.astype(np.float64)), torch.from_numpy(W.astype(np.float64)),
                                   torch.from_numpy(b.astype(np.float64)), padding=W.shape[2] // 2)
    return y.numpy()


def test_conv_restatement_matches_float64():
    rng = np.random.default_rng(0)
    for ci, co, k, h, w in [(3, 8, 3, 12, 10), (16, 32, 7, 9, 11), (24, 16, 1, 5, 7)]:
        x = rng.standard_normal((2, ci, h, w)).astype(np.float32)
        W = (rng.standard_normal((co, ci, k, k)) / np.sqrt(ci * k * k)).astype(np.float32)
        b = rng.standard_normal(co).astype(np.float32)
        y = F.convolution_2d(x, W, b, k // 2)
        assert y.dtype == np.float32 and y.shape == (2, co, h, w)
        np.testing.assert_allclose(y, _ref_conv64(x, W, b), rtol=1e-5, atol=1e-5)


def test_maxpool_cover_all():
    x = np.arange(2 * 3 * 6 * 4, dtype=np.float32).reshape(2, 3, 6, 4)
    y = F.max_pooling_2d(x)
    assert y.shape == (2, 3, 3, 2)
    np.testing.assert_array_equal(y, x.reshape(2, 3, 3, 2, 2, 2).max(axis=(3, 5)))
    z = F.max_pooling_2d(np.ones((1, 1, 5, 5), np.float32))  # odd size: cover_all adds a window
    assert z.shape == (1, 1, 3, 3)


def test_full_network_float64_crosscheck(rand_weights):
    """Whole CocoPoseNet at 32x40 against the same graph in float64 torch."""
    rng = np.random.default_rng(5)
    x = rng.uniform(-0.5, 0.5, (1, 3, 32, 40)).astype(np.float32)
    paf, heat = F.cocoposenet_forward(rand_weights, x)
    assert paf.shape == (1, 38, 4, 5) and heat.shape == (1, 19, 4, 5)

    def conv(name, h, act=True):
        W, b = rand_weights[name]
        y = _ref_conv64(h, W, b)
        return np.maximum(y, 0) if act else y

    def pool(h):
        t = torch.from_numpy(h)
        return torch.nn.functional.max_pool2d(t, 2, 2, ceil_mode=True).numpy()

    h = conv("conv1_2", conv("conv1_1", x))
    h = pool(h)
    h = pool(conv("conv2_2", conv("conv2_1", h)))
    for n in ("conv3_1", "conv3_2", "conv3_3", "conv3_4"):
        h = conv(n, h)
    h = pool(h)
    for n in ("conv4_1", "conv4_2", "conv4_3_CPM", "conv4_4_CPM"):
        h = conv(n, h)
    feat = h
    outs = []
    for br in ("L1", "L2"):
        t = feat
        for i in (1, 2, 3, 4):
            t = conv("conv5_%d_CPM_%s" % (i, br), t)
        outs.append(conv("conv5_5_CPM_%s" % br, t, act=False))
    for s in range(2, 7):
        cat = np.concatenate([outs[0], outs[1], feat], axis=1)
        new = []
        for br in ("L1", "L2"):
            t = cat
            for i in range(1, 7):
                t = conv("Mconv%d_stage%d_%s" % (i, s, br), t)
            new.append(conv("Mconv7_stage%d_%s" % (s, br), t, act=False))
        outs = new
    scale = max(1.0, float(np.abs(outs[0]).max()), float(np.abs(outs[1]).max()))
    np.testing.assert_allclose(paf, outs[0], atol=1e-4 * scale, rtol=0)
    np.testing.assert_allclose(heat, outs[1], atol=1e-4 * scale, rtol=0)
