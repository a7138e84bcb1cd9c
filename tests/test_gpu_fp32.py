"""The exact-f32 precision's 3x3 / 7x7 convolutions on the LDS-halo kernel (round 5, VERDICT r04
item 6; csrc/conv_f32.hip conv_f32_lds).  It contracts the same operands in the same order as the
global-load kernel conv_mfma_f32 (conv.hip), so the network's maps must be BIT-IDENTICAL with
OP_F32_LDS=0 (which keeps every layer on conv_mfma_f32) -- across map widths that pick 16- or
32-column tiles, partial edge tiles, batches and both branches (groups = 2); and held to the CPU
oracle of the reference network (models/CocoPoseNet.py:132-262) at the north star's 1e-3 by
test_gpu_forward_golden.py's fp32 cases, which now run this kernel."""
import numpy as np
import pytest

from conftest import pkg_module
from oracle import forward as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def f32ctx(lib, rand_weights):
    c = lib.Context(0)
    c.set_weights(rand_weights)
    c.set_precision("fp32")
    yield c
    c.close()


@pytest.mark.parametrize("n,h,w", [(1, 64, 80), (2, 368, 368), (1, 368, 656), (3, 120, 200), (1, 56, 40)])
def test_lds_kernel_bit_identical_to_global_load_kernel(lib, f32ctx, monkeypatch, n, h, w):
    rng = np.random.default_rng(h * 1000 + w + n)
    x = rng.uniform(-0.5, 0.5, (n, 3, h, w)).astype(np.float32)
    out = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("OP_F32_LDS", mode)
        lib.conv_census(reset=True)
        out[mode] = f32ctx.forward(x)
        cen = lib.conv_census(reset=True)
        if mode == "1":
            assert cen["f32_lds"] > 0, cen  # every 3x3 / 7x7 layer (conv1_1 .. Mconv5)
        else:
            assert cen["f32_lds"] == 0, cen
    for a, b in zip(out["1"], out["0"]):
        assert a.shape == b.shape and np.array_equal(a, b), float(np.abs(a - b).max())


def test_lds_kernel_128_channel_waves_bit_identical(lib, f32ctx, monkeypatch):
    """OP_F32_CB=4 (A/B aid): 128 output channels per wave, the same per-output k order."""
    rng = np.random.default_rng(31)
    x = rng.uniform(-0.5, 0.5, (2, 3, 184, 200)).astype(np.float32)
    out = {}
    for cb in ("4", "2"):
        monkeypatch.setenv("OP_F32_CB", cb)
        out[cb] = f32ctx.forward(x)
    monkeypatch.delenv("OP_F32_CB")
    for a, b in zip(out["4"], out["2"]):
        assert np.array_equal(a, b), float(np.abs(a - b).max())


def test_lds_kernel_vs_oracle(f32ctx, rand_weights):
    rng = np.random.default_rng(7)
    x = rng.uniform(-0.5, 0.5, (1, 3, 96, 112)).astype(np.float32)
    paf, heat = f32ctx.forward(x)
    opaf, oheat = F.cocoposenet_forward(rand_weights, x)
    err = max(float(np.abs(paf - opaf).max()), float(np.abs(heat - oheat).max()))
    print("fp32 LDS kernel vs oracle: %.3g" % err)
    assert err <= 1e-4, err  # exact f32 products: ~1e-6 (summation order only)
