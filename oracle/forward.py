"""ORACLE — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

NumPy restatement of the CocoPoseNet forward exactly as Chainer's CPU path runs it:
``Convolution2DFunction.forward_cpu`` = ``im2col_cpu`` + ``numpy.tensordot`` (sgemm) + bias,
``F.relu``, ``MaxPooling2D.forward_cpu`` (im2col with -inf padding, ``cover_all=True``),
``F.concat(axis=1)``.

Layer table and call order follow ``models/CocoPoseNet.py:23-130`` (links) and
``models/CocoPoseNet.py:132-262`` (``__call__``).  Chainer itself is not installed here, so this
restatement is the contract for the forward ("parity unpinned" at the Chainer boundary); it is
cross-checked against an independent float64 convolution in tests/test_oracle_forward.py.
"""
import numpy as np

# (name, Cin, Cout, ksize) in models/CocoPoseNet.py:26-129 order.
LAYERS = []


def _add(name, ci, co, k):
    LAYERS.append((name, ci, co, k))


for _n, _ci, _co in [("conv1_1", 3, 64), ("conv1_2", 64, 64), ("conv2_1", 64, 128),
                     ("conv2_2", 128, 128), ("conv3_1", 128, 256), ("conv3_2", 256, 256),
                     ("conv3_3", 256, 256), ("conv3_4", 256, 256), ("conv4_1", 256, 512),
                     ("conv4_2", 512, 512), ("conv4_3_CPM", 512, 256), ("conv4_4_CPM", 256, 128)]:
    _add(_n, _ci, _co, 3)
for _b, _out in (("L1", 38), ("L2", 19)):
    for _i in (1, 2, 3):
        _add("conv5_%d_CPM_%s" % (_i, _b), 128, 128, 3)
    _add("conv5_4_CPM_%s" % _b, 128, 512, 1)
    _add("conv5_5_CPM_%s" % _b, 512, _out, 1)
for _s in range(2, 7):
    for _b, _out in (("L1", 38), ("L2", 19)):
        _add("Mconv1_stage%d_%s" % (_s, _b), 185, 128, 7)
        for _i in (2, 3, 4, 5):
            _add("Mconv%d_stage%d_%s" % (_i, _s, _b), 128, 128, 7)
        _add("Mconv6_stage%d_%s" % (_s, _b), 128, 128, 1)
        _add("Mconv7_stage%d_%s" % (_s, _b), 128, _out, 1)

assert len(LAYERS) == 92


def get_conv_outsize(size, k, s, p, cover_all=False, d=1):
    """chainer.utils.conv.get_conv_outsize."""
    dk = k + (k - 1) * (d - 1)
    if cover_all:
        return (size + p * 2 - dk + s - 1) // s + 1
    return (size + p * 2 - dk) // s + 1


def im2col_cpu(img, kh, kw, sy, sx, ph, pw, pval=0, cover_all=False):
    """chainer.utils.conv.im2col_cpu (dilation 1)."""
    n, c, h, w = img.shape
    out_h = get_conv_outsize(h, kh, sy, ph, cover_all)
    out_w = get_conv_outsize(w, kw, sx, pw, cover_all)
    img = np.pad(img, ((0, 0), (0, 0), (ph, ph + sy - 1), (pw, pw + sx - 1)),
                 mode="constant", constant_values=(pval,))
    col = np.ndarray((n, c, kh, kw, out_h, out_w), dtype=img.dtype)
    for j in range(kh):
        j_lim = j + sy * out_h
        for i in range(kw):
            i_lim = i + sx * out_w
            col[:, :, j, i, :, :] = img[:, :, j:j_lim:sy, i:i_lim:sx]
    return col


def convolution_2d(x, W, b, pad):
    """Convolution2DFunction.forward_cpu: tensordot over (C, kh, kw), + b, NCHW out."""
    kh, kw = W.shape[2:]
    col = im2col_cpu(x, kh, kw, 1, 1, pad, pad)
    y = np.tensordot(col, W, ((1, 2, 3), (1, 2, 3))).astype(x.dtype, copy=False)
    if b is not None:
        y += b
    return np.ascontiguousarray(np.rollaxis(y, 3, 1))


def relu(x):
    return np.maximum(x, x.dtype.type(0))


def max_pooling_2d(x, k=2, s=2):
    """MaxPooling2D.forward_cpu with pad=0, cover_all=True (F.max_pooling_2d default)."""
    n, c, h, w = x.shape
    col = im2col_cpu(x, k, k, s, s, 0, 0, pval=-float("inf"), cover_all=True)
    return col.reshape(n, c, k * k, col.shape[4], col.shape[5]).max(axis=2)


def cocoposenet_forward(weights, x, all_stages=False):
    """models/CocoPoseNet.py:132-262.  weights: {name: (W (Co,Ci,k,k) f32, b (Co,) f32)}.

    Returns (pafs, heatmaps) of the last stage, or the full 6-stage lists if all_stages."""
    def conv(name, h, act=True):
        W, b = weights[name]
        y = convolution_2d(h, W, b, W.shape[2] // 2)
        return relu(y) if act else y

    h = conv("conv1_1", x)
    h = conv("conv1_2", h)
    h = max_pooling_2d(h)
    h = conv("conv2_1", h)
    h = conv("conv2_2", h)
    h = max_pooling_2d(h)
    for n in ("conv3_1", "conv3_2", "conv3_3", "conv3_4"):
        h = conv(n, h)
    h = max_pooling_2d(h)
    for n in ("conv4_1", "conv4_2", "conv4_3_CPM", "conv4_4_CPM"):
        h = conv(n, h)
    feature_map = h
    pafs, heatmaps = [], []
    h1 = feature_map
    for i in (1, 2, 3, 4):
        h1 = conv("conv5_%d_CPM_L1" % i, h1)
    h1 = conv("conv5_5_CPM_L1", h1, act=False)
    h2 = feature_map
    for i in (1, 2, 3, 4):
        h2 = conv("conv5_%d_CPM_L2" % i, h2)
    h2 = conv("conv5_5_CPM_L2", h2, act=False)
    pafs.append(h1)
    heatmaps.append(h2)
    for s in range(2, 7):
        h = np.concatenate((h1, h2, feature_map), axis=1)
        outs = []
        for br in ("L1", "L2"):
            t = h
            for i in range(1, 7):
                t = conv("Mconv%d_stage%d_%s" % (i, s, br), t)
            outs.append(conv("Mconv7_stage%d_%s" % (s, br), t, act=False))
        h1, h2 = outs
        pafs.append(h1)
        heatmaps.append(h2)
    if all_stages:
        return pafs, heatmaps
    return pafs[-1], heatmaps[-1]
