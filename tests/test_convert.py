"""Caffe -> npz converter (models/convert_model.py) on caffemodels written by an
independent protobuf encoder below, in each wire variant a caffemodel can use.  CPU only.

Parity unpinned: no caffemodel and no Caffe/Chainer exist here; the encoder follows the published
protobuf wire format and caffe.proto field numbers.
"""
import struct

import numpy as np
import pytest

from conftest import pkg_module

conv = pkg_module("convert_model")
nets = pkg_module("nets")
weights = pkg_module("weights")


def _vint(x):
    out = bytearray()
    while True:
        b = x & 0x7F
        x >>= 7
        if x:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(fn, wt):
    return _vint((fn << 3) | wt)


def _ld(fn, payload):
    return _key(fn, 2) + _vint(len(payload)) + payload


def _blob(arr, style):
    a = np.asarray(arr, np.float32)
    if style == "shape_packed":  # new-style: BlobShape dims packed, data packed
        dims = b"".join(_vint(d) for d in a.shape)
        return _ld(7, _ld(1, dims)) + _ld(5, a.astype("<f4").tobytes())
    if style == "shape_unpacked":  # dims as repeated varints, data as repeated fixed32
        dims = b"".join(_key(1, 0) + _vint(d) for d in a.shape)
        return _ld(7, dims) + b"".join(_key(5, 5) + struct.pack("<f", v) for v in a.ravel())
    if style == "legacy":  # num/channels/height/width, packed data
        shp = list(a.shape) + [1] * (4 - a.ndim) if a.ndim < 4 else list(a.shape)
        if a.ndim == 1:
            shp = [1, 1, 1, a.shape[0]]
        head = b"".join(_key(f, 0) + _vint(v) for f, v in zip((1, 2, 3, 4), shp))
        return head + _ld(5, a.astype("<f4").tobytes())
    if style == "double":
        dims = b"".join(_vint(d) for d in a.shape)
        return _ld(7, _ld(1, dims)) + _ld(8, a.astype("<f8").tobytes())
    raise ValueError(style)


def _layer(name, blobs, v1=False, style="shape_packed"):
    if v1:  # V1LayerParameter: name 4, type 5 (enum), blobs 6
        body = _ld(4, name.encode()) + _key(5, 0) + _vint(4)
        body += b"".join(_ld(6, _blob(b, style)) for b in blobs)
        return _ld(2, body)
    body = _ld(1, name.encode()) + _ld(2, b"Convolution") + _ld(3, b"bottom") + _ld(4, b"top")
    body += b"".join(_ld(7, _blob(b, style)) for b in blobs)
    return _ld(100, body)


def _model(arch, seed=1, style="shape_packed", v1=False, skip=(), bad=()):
    key = (arch, seed, style, v1, skip, bad)
    if key not in _CACHE:
        rng = np.random.default_rng(seed)
        ref = {}
        out = [_ld(1, b"net"), _ld(100, _ld(1, b"data") + _ld(2, b"Input"))]
        for name, ci, co, k in nets.layers(arch):
            W = rng.standard_normal((co, ci, k, k), dtype=np.float32)
            b = rng.standard_normal(co, dtype=np.float32)
            ref[name] = (W, b)
            if name in skip:
                continue
            Wf = W[:, :-1] if name in bad else W
            out.append(_layer(name, [Wf, b], v1=v1, style=style))
            out.append(_ld(100, _ld(1, (name + "_relu").encode()) + _ld(2, b"ReLU")))
        _CACHE.clear()  # one ~210 MB model at a time
        _CACHE[key] = (b"".join(out), ref)
    return _CACHE[key]


_CACHE = {}


def test_posenet_table_matches_library():
    assert nets.layers("posenet") == weights.layer_table()


def test_layer_tables():
    assert len(nets.layers("posenet")) == 92
    for arch, nm in (("facenet", 71), ("handnet", 22)):
        t = dict((n, (ci, co, k)) for n, ci, co, k in nets.layers(arch))
        assert len(t) == 17 + 5 * 7
        assert t["Mconv1_stage2"] == (nm + 128, 128, 7) and t["Mconv7_stage6"] == (128, nm, 1)
        assert t["conv6_2_CPM"] == (512, nm, 1)
    assert "conv5_5_CPM_L1" not in nets.CONVERT_LAYERS["posenet"]
    assert len(nets.CONVERT_LAYERS["posenet"]) == 91


@pytest.mark.parametrize("style,v1", [("shape_packed", False), ("legacy", True), ("double", False)])
def test_posenet_roundtrip(style, v1):
    buf, ref = _model("posenet", style=style, v1=v1)
    logs = []
    m = conv.convert("posenet", conv.read_caffemodel(buf), seed=3, log=logs.append)
    init = conv.initial_weights("posenet", seed=3)
    for name, (W, b) in ref.items():
        if name == "conv5_5_CPM_L1":  # the reference's copy list omits it: initial weights kept
            assert np.array_equal(m[name][0], init[name][0]) and not m[name][1].any()
        else:
            assert np.array_equal(m[name][0], W) and np.array_equal(m[name][1], b), name
    assert len(logs) == 91 and all(s.startswith("Succeed to copy layer ") for s in logs)


def test_unpacked_fixed32_blob():
    W = np.arange(2 * 3 * 3 * 3, dtype=np.float32).reshape(2, 3, 3, 3) / 7
    got = conv.parse_blob(_blob(W, "shape_unpacked"))
    assert got.shape == W.shape and np.array_equal(got, W)


def test_copy_all_and_seeded_initials():
    buf, ref = _model("posenet")
    m = conv.convert("posenet", buf, copy_all=True, log=lambda s: None)
    assert np.array_equal(m["conv5_5_CPM_L1"][0], ref["conv5_5_CPM_L1"][0])
    a = conv.initial_weights("posenet", seed=5)["conv1_1"][0]
    b = conv.initial_weights("posenet", seed=5)["conv1_1"][0]
    assert np.array_equal(a, b) and abs(a.std() - np.sqrt(1 / 27)) < 0.05


def test_shape_mismatch_is_not_copied_and_missing_layer_raises():
    buf, ref = _model("handnet", bad=("Mconv3_stage4",))
    logs = []
    m = conv.convert("handnet", buf, seed=0, log=logs.append)
    assert "Failed to copy layer Mconv3_stage4!" in logs
    assert np.array_equal(m["Mconv3_stage4"][0], conv.initial_weights("handnet", 0)["Mconv3_stage4"][0])
    assert np.array_equal(m["Mconv4_stage4"][0], ref["Mconv4_stage4"][0])
    buf2, _ = _model("facenet", skip=("conv4_4",))
    with pytest.raises(KeyError):
        conv.convert("facenet", buf2, log=lambda s: None)
    with pytest.raises(KeyError):
        nets.layers("bodynet")


def test_cli_writes_npz_loadable_by_pose_detector(tmp_path):
    buf, ref = _model("posenet", seed=7)
    src = tmp_path / "pose.caffemodel"
    src.write_bytes(buf)
    dst = tmp_path / "coco_posenet.npz"
    assert conv.main(["posenet", str(src), str(dst), "--copy-all"]) == 0
    w = weights.load_npz(str(dst))
    for name, (W, b) in ref.items():
        assert np.array_equal(w[name][0], W) and np.array_equal(w[name][1], b)
    with np.load(str(dst)) as z:
        assert sorted(z.keys()) == sorted(k for n in ref for k in (n + "/W", n + "/b"))


def test_copy_lists_match_reference_converter():
    """nets.CONVERT_LAYERS == models/convert_model.py:8-249's layer_names (extracted from the
    reference source with ast by tests/golden/make_golden_convert.py), order included."""
    import json
    import os
    d = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "convert_layer_names.json")))
    assert d["source"] == "models/convert_model.py:8-249"
    assert set(d["layer_names"]) == set(nets.CONVERT_LAYERS) == {"posenet", "facenet", "handnet"}
    for arch, names in d["layer_names"].items():
        assert list(nets.CONVERT_LAYERS[arch]) == names, arch


def test_params_archs_build_models(tmp_path):
    """entity.py:50-54 maps arch -> model class and pose_detector.py:23-26 does
    ``params['archs'][arch]()`` then ``serializers.load_npz(weights_file, model)``."""
    from conftest import pkg_module as pm
    params = pm("constants").params
    for arch, n in (("posenet", 92), ("facenet", 52), ("handnet", 52)):
        m = params["archs"][arch]()
        assert len(m) == n and m.arch == arch
        for name, ci, co, k in nets.layers(arch):
            W, b = m[name]
            assert W.shape == (co, ci, k, k) and W.dtype == np.float32 and not b.any()
    src = weights.random_weights(5)
    path = str(tmp_path / "w.npz")
    weights.save_npz(path, src)
    m = params["archs"]["posenet"]()
    assert weights.load_npz(path, m) is m
    assert all(np.array_equal(m[k][0], src[k][0]) and np.array_equal(m[k][1], src[k][1]) for k in src)
