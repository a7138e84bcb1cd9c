"""Caffe ``.caffemodel`` -> Chainer-layout npz (models/convert_model.py:1-282), SURVEY §8 f2.

    python -m chainer_realtime_multi-person_pose_estimation_amd.convert_model ARCH CAFFE_FILE CHAINER_FILE

The reference builds the Chainer model (random initial weights), loads the caffemodel with
``chainer.links.caffe.CaffeFunction`` and, for every name in its copy list, copies ``W``/``b``
when both shapes match ("Succeed to copy layer X") or leaves the layer alone ("Failed to copy
layer X!"), then ``serializers.save_npz`` writes ``<layer>/W`` (Co, Ci, kh, kw) f32 and
``<layer>/b`` (Co,) for every layer (models/convert_model.py:257-282).  Neither Caffe nor Chainer
is needed here: the caffemodel is a protobuf ``NetParameter`` read straight from its wire format
(field numbers of the published caffe.proto: NetParameter.layer = 100 / legacy layers = 2;
LayerParameter name = 1, blobs = 7; V1LayerParameter name = 4, blobs = 6; BlobProto num..width =
1-4, data = 5, shape = 7 {dim = 1}, double_data = 8).  A Convolution blob pair maps to W =
data.reshape(num, channels, height, width) (CaffeFunction._setup_convolution, group 1) and b.

Reproduced quirk: the posenet copy list omits ``conv5_5_CPM_L1`` (convert_model.py:24-33), so
that layer keeps the model's initial weights.  Chainer's default initialiser there is LeCunNormal
(N(0, 1/fan_in)) with zero bias from an unseeded RNG; this converter draws it from
``numpy.random.default_rng(seed)`` (``--seed``) so a conversion is reproducible, and
``--copy-all`` copies the layer instead (what the OpenPose weights intend).  Parity unpinned: no
caffemodel and no Caffe/Chainer exist in this environment; tests/test_convert.py round-trips
models written by an independent protobuf encoder in every wire variant.
"""
import argparse
import struct
import sys

import numpy as np

from . import nets


def _varint(buf, i):
    v = 0
    shift = 0
    while True:
        if i >= len(buf):
            raise ValueError("truncated varint")
        b = buf[i]
        i += 1
        v |= (b & 0x7F) << shift
        if not b & 0x80:
            return v, i
        shift += 7
        if shift > 70:
            raise ValueError("varint too long")


def fields(buf):
    """Yield (field_number, wire_type, value) of one protobuf message: value is an int (varint),
    bytes (length-delimited) or the raw 4/8 bytes (fixed32/fixed64)."""
    i, n = 0, len(buf)
    while i < n:
        key, i = _varint(buf, i)
        fn, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _varint(buf, i)
        elif wt == 1:
            v, i = buf[i:i + 8], i + 8
        elif wt == 2:
            ln, i = _varint(buf, i)
            v, i = buf[i:i + ln], i + ln
        elif wt == 5:
            v, i = buf[i:i + 4], i + 4
        else:
            raise ValueError("unsupported wire type %d (field %d)" % (wt, fn))
        if i > n:
            raise ValueError("truncated field %d" % fn)
        yield fn, wt, v


def _packed_varints(v):
    out, i = [], 0
    while i < len(v):
        x, i = _varint(v, i)
        out.append(x)
    return out


def parse_blob(buf):
    """BlobProto -> f32 ndarray shaped by shape.dim, else (num, channels, height, width)."""
    legacy = {}
    dims = []
    parts = []
    for fn, wt, v in fields(buf):
        if fn in (1, 2, 3, 4) and wt == 0:
            legacy[fn] = v
        elif fn == 5:  # data: packed floats (wt 2) or one fixed32 per element (wt 5)
            parts.append(np.frombuffer(v, "<f4") if wt == 2 else np.array(struct.unpack("<f", v), "<f4"))
        elif fn == 8:  # double_data
            parts.append((np.frombuffer(v, "<f8") if wt == 2 else np.array(struct.unpack("<d", v))).astype(np.float32))
        elif fn == 7 and wt == 2:  # BlobShape
            for sf, swt, sv in fields(v):
                if sf == 1:
                    dims += _packed_varints(sv) if swt == 2 else [sv]
    data = np.concatenate(parts).astype(np.float32) if parts else np.zeros(0, np.float32)
    if not dims and legacy:
        dims = [legacy.get(k, 1) for k in (1, 2, 3, 4)]
    if dims and int(np.prod(dims)) == data.size:
        return data.reshape(dims)
    return data


def read_caffemodel(path_or_bytes):
    """{layer name: [blob arrays]} for every layer that carries blobs, in file order."""
    buf = path_or_bytes if isinstance(path_or_bytes, (bytes, bytearray)) else open(path_or_bytes, "rb").read()
    out = {}
    for fn, wt, v in fields(bytes(buf)):
        if wt != 2 or fn not in (100, 2):
            continue
        name_f, blob_f = (1, 7) if fn == 100 else (4, 6)
        name, blobs = None, []
        for lf, lwt, lv in fields(v):
            if lf == name_f and lwt == 2:
                name = lv.decode("utf-8")
            elif lf == blob_f and lwt == 2:
                blobs.append(parse_blob(lv))
        if name is not None and blobs:
            out[name] = blobs
    return out


def _conv_params(blobs, co, ci, k):
    """(W, b) as CaffeFunction builds them, or None when the blobs cannot be this layer."""
    W = blobs[0]
    if W.ndim != 4:
        if W.size != co * ci * k * k:
            return None
        W = W.reshape(co, ci, k, k)
    b = blobs[1].reshape(-1) if len(blobs) > 1 else np.zeros(W.shape[0], np.float32)
    return np.ascontiguousarray(W, np.float32), np.ascontiguousarray(b, np.float32)


def initial_weights(arch, seed=0):
    """The model's initial parameters: LeCunNormal W (std sqrt(1/fan_in)), zero b (Chainer defaults)."""
    rng = np.random.default_rng(seed)
    out = {}
    for name, ci, co, k in nets.layers(arch):
        W = (rng.standard_normal((co, ci, k, k)) * np.sqrt(1.0 / (ci * k * k))).astype(np.float32)
        out[name] = (W, np.zeros(co, np.float32))
    return out


def convert(arch, caffe_model, seed=0, copy_all=False, log=print):
    """models/convert_model.py:257-282 without Chainer: returns {layer: (W, b)} for every layer."""
    model = initial_weights(arch, seed)
    caffe = caffe_model if isinstance(caffe_model, dict) else read_caffemodel(caffe_model)
    names = [n for n, _, _, _ in nets.layers(arch)] if copy_all else nets.CONVERT_LAYERS[arch]
    for name in names:
        if name not in caffe:
            raise KeyError("caffemodel has no layer %r" % name)
        Wm, bm = model[name]
        got = _conv_params(caffe[name], *Wm.shape[:2], Wm.shape[2])
        if got is not None and got[0].shape == Wm.shape and got[1].shape == bm.shape:
            model[name] = got
            log("Succeed to copy layer %s" % name)
        else:
            log("Failed to copy layer %s!" % name)
    return model


def save_npz(path, model):
    """Chainer save_npz key layout: <layer>/W, <layer>/b."""
    flat = {}
    for name, (W, b) in model.items():
        flat[name + "/W"] = W
        flat[name + "/b"] = b
    np.savez(path, **flat)


def main(argv=None):
    ap = argparse.ArgumentParser(description="Convert caffemodel into chainermodel")
    ap.add_argument("arch", help="model architecture: ['posenet', 'facenet', 'handnet']")
    ap.add_argument("caffe_file", help="caffe weights file path")
    ap.add_argument("chainer_file", help="file path to save chainer weights file")
    ap.add_argument("--seed", type=int, default=0, help="initial weights of layers left uncopied")
    ap.add_argument("--copy-all", action="store_true", help="also copy conv5_5_CPM_L1 (posenet)")
    args = ap.parse_args(argv)
    print("Loading %s..." % args.arch)
    nets.layers(args.arch)
    print("Loading caffemodel file...")
    caffe = read_caffemodel(args.caffe_file)
    model = convert(args.arch, caffe, seed=args.seed, copy_all=args.copy_all)
    print("Saving weights file into '%s'..." % args.chainer_file)
    save_npz(args.chainer_file, model)
    print("Done.")
    return 0


if __name__ == "__main__":
    sys.exit(main())
