# debugging aid: conv1_1 output (C11 buffer) of the VALU kernel vs a float64 reference conv
import ctypes, importlib, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
L = importlib.import_module("chainer_realtime_multi-person_pose_estimation_amd._lib")
W = importlib.import_module("chainer_realtime_multi-person_pose_estimation_amd.weights").random_weights(seed=0)
c = L.Context(0); c.set_weights(W)
h, w = 64, 80
x = np.random.default_rng(11).uniform(-0.5, 0.5, (1, 3, h, w)).astype(np.float32)
c.forward(x)
buf = np.empty(((h + 2) * (w + 2) * 64,), np.float32)
L.lib().op_debug_read_buffer.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int64]
L.check(L.lib().op_debug_read_buffer(c.h, 1, buf.ctypes.data, buf.nbytes))
raw = buf.view(np.uint16).reshape(h + 2, w + 2, 8, 2, 8)  # [y][x][group][hi/lo][8]
hi = (raw[:, :, :, 0, :].astype(np.uint32) << 16).view(np.float32)
lo = (raw[:, :, :, 1, :].astype(np.uint32) << 16).view(np.float32)
got = (hi.astype(np.float64) + lo).reshape(h + 2, w + 2, 64)[1:-1, 1:-1].transpose(2, 0, 1)
wt, b = W["conv1_1"]
xp = np.pad(x[0].astype(np.float64), ((0, 0), (1, 1), (1, 1)))
ref = np.zeros((64, h, w))
for ky in range(3):
    for kx in range(3):
        ref += np.einsum("oc,chw->ohw", wt[:, :, ky, kx].astype(np.float64), xp[:, ky:ky + h, kx:kx + w])
ref = np.maximum(ref + b[:, None, None], 0)
d = np.abs(got - ref)
print("max err", d.max(), "at", np.unravel_index(d.argmax(), d.shape), "frac bad", (d > 1e-3).mean())
print("halo sum", np.abs((hi.astype(np.float64) + lo)[0]).sum(), np.abs((hi.astype(np.float64) + lo)[:, 0]).sum())
x0 = np.empty(((h + 2) * (w + 2) * 16,), np.float32)
L.check(L.lib().op_debug_read_buffer(c.h, 0, x0.ctypes.data, x0.nbytes))
r0 = x0.view(np.uint16).reshape(h + 2, w + 2, 2, 2, 8)
xh = (r0[:, :, 0, 0, :].astype(np.uint32) << 16).view(np.float32)
xl = (r0[:, :, 0, 1, :].astype(np.uint32) << 16).view(np.float32)
xr = (xh.astype(np.float64) + xl)[1:-1, 1:-1, :3].transpose(2, 0, 1)
print("x0 recon err", np.abs(xr - x[0]).max())
# tile-mapping probe: which input offset best explains the GPU output?
for dy in (-1, 0, 1):
    for dx in (-1, 0, 1):
        sh = np.roll(np.roll(ref, dy, 1), dx, 2)
        print(dy, dx, np.abs(got - sh)[:, 2:-2, 2:-2].max())
def conv(wt4, bias):
    r = np.zeros((64, h, w))
    for ky in range(3):
        for kx in range(3):
            r += np.einsum("oc,chw->ohw", wt4[:, :, ky, kx].astype(np.float64), xp[:, ky:ky + h, kx:kx + w])
    return np.maximum(r + bias[:, None, None], 0)
hyp = {"transpose_k": conv(wt.transpose(0, 1, 3, 2), b), "ci_rev": conv(wt[:, ::-1], b), "nobias": conv(wt, 0 * b),
       "flip": conv(wt[:, :, ::-1, ::-1], b)}
for k, v in hyp.items():
    print(k, np.abs(got - v).max())
# raw layout reinterpretation used by the old packing ([tap][co][8] with ci) on w11 offsets
wf = wt.reshape(-1)
alt = np.zeros_like(wt)
for co in range(64):
    for ci in range(3):
        for t in range(9):
            idx = (t * 3 + ci) * 64 + co
            alt[co, ci, t // 3, t % 3] = wf[idx] if idx < wf.size else 0
print("w11 read as raw", np.abs(got - conv(alt, b)).max())
print("sample got", got[:3, 5, 5], "ref", ref[:3, 5, 5])
