"""Oracle of the multi-scale path (pose_detector.py:433-482): the cv2 INTER_CUBIC restatement
(oracle/cvcubic.c, OpenCV absent -> parity unpinned) cross-checked against an independent
bicubic (torch, A = -0.75, half-pixel centres, edge clamp, float64) and the size arithmetic."""
import numpy as np
import pytest

from oracle import precise as PR
from oracle import postproc as P


@pytest.mark.parametrize("h,w,oh,ow,cn", [(23, 41, 184, 328, 38), (46, 46, 368, 368, 19), (40, 30, 17, 13, 3),
                                          (6, 9, 48, 72, 19), (35, 61, 720, 1280, 2)])
def test_cubic_f32_matches_independent_bicubic(h, w, oh, ow, cn):
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(h * w)
    x = rng.standard_normal((h, w, cn)).astype(np.float32)
    got = PR.resize_cubic_f32(x, ow, oh)
    ref = torch.nn.functional.interpolate(torch.from_numpy(x.transpose(2, 0, 1)[None]).double(), size=(oh, ow),
                                          mode="bicubic", align_corners=False)[0].numpy().transpose(1, 2, 0)
    # the restated path rounds the source coordinate to f32 (OpenCV), torch keeps f64
    assert np.abs(got - ref).max() < 2e-4 * max(1.0, ow / w)


def test_cubic_u8_within_one_lsb_of_independent_bicubic():
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(1)
    x = rng.integers(0, 256, (50, 70, 3), dtype=np.uint8)
    got = PR.resize_cubic_u8(x, 91, 37).astype(np.int64)
    ref = torch.nn.functional.interpolate(torch.from_numpy(x.transpose(2, 0, 1)[None]).double(), size=(37, 91),
                                          mode="bicubic", align_corners=False)[0].numpy().transpose(1, 2, 0)
    assert np.abs(got - np.clip(np.rint(ref), 0, 255)).max() <= 1


def test_cubic_identity_and_constant():
    rng = np.random.default_rng(2)
    x = rng.standard_normal((13, 17, 5)).astype(np.float32)
    assert np.array_equal(PR.resize_cubic_f32(x, 17, 13), x)
    u = rng.integers(0, 256, (13, 17, 3), dtype=np.uint8)
    assert np.array_equal(PR.resize_cubic_u8(u, 17, 13), u)
    c = np.full((9, 11, 3), 77, np.uint8)
    assert np.all(PR.resize_cubic_u8(c, 40, 23) == 77)


def test_scale_sizes_720p():
    # padded inputs 328x184, 656x368, 984x552, 1312x736 for a 1280x720 frame
    got = PR.scale_sizes(720, 1280, P.PARAMS)
    assert [(pw, ph) for _, _, pw, ph in got] == [(328, 184), (656, 368), (984, 552), (1312, 736)]


def test_pad_image_matches_reference_semantics():
    img = np.arange(5 * 7 * 3, dtype=np.uint8).reshape(5, 7, 3)
    out, pad = PR.pad_image(img, 8, (104, 117, 123))
    assert pad == [3, 1] and out.shape == (8, 8, 3)  # (int64 like the reference: uint8 zeros + a tuple)
    assert np.array_equal(out[:5, :7], img) and np.all(out[5:, :, 0] == 104) and np.all(out[:, 7:, 2] == 123)


def test_precise_maps_small_runs(rand_weights_small):
    params = dict(P.PARAMS, inference_img_size=16)
    img = np.random.default_rng(3).integers(0, 256, (20, 28, 3), dtype=np.uint8)
    pafs, heat = PR.precise_maps(rand_weights_small, img, params)
    assert pafs.shape == (38, 20, 28) and heat.shape == (19, 20, 28)
    assert pafs.dtype == np.float32 and np.isfinite(pafs).all() and np.isfinite(heat).all()
