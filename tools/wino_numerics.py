"""Numerics study (CPU, NumPy): Winograd F(m x m, r x r) with the bf16x3 split (hi*hi + hi*lo +
lo*hi, f32 accumulate) against a float64 direct convolution, next to the direct bf16x3 error.

Decides whether a Winograd-domain conv kernel can hold the north star's 1e-3 map tolerance.
  python tools/wino_numerics.py [--ci 128] [--hw 46]
"""
import argparse

import numpy as np
import sympy


def wino_mats(pts, m, r):
    """A^T (m x n), G (n x r), B^T (n x n) for correlation y_k = sum_j d[k+j] g[j], k < m.
    Toom-Cook on points pts (n-1 finite) + infinity: s = V^-1 diag(Vr g) Vm h (convolution),
    transposed in h -> correlation."""
    n = m + r - 1
    assert len(pts) == n - 1

    def ev(k):
        rows = [[sympy.Rational(p) ** j for j in range(k)] for p in pts]
        rows.append([0] * (k - 1) + [1])
        return sympy.Matrix(rows)

    V, Vr, Vm = ev(n), ev(r), ev(m)
    BT = V.inv().T
    f = lambda M: np.array(M.tolist(), dtype=np.float64)
    return f(Vm.T), f(Vr), f(BT)


def bf16(x):
    x = np.ascontiguousarray(x, dtype=np.float32)
    u = x.view(np.uint32).astype(np.uint64)
    u = (u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000
    return u.astype(np.uint32).view(np.float32)


def split(x):
    x = x.astype(np.float32)
    hi = bf16(x)
    lo = bf16(x - hi)
    return hi, lo


def mm3(a, b, eq):
    """bf16x3 contraction with f32 accumulation (einsum in f32 as a stand-in for MFMA)."""
    ah, al = split(a)
    bh, bl = split(b)
    return (np.einsum(eq, ah, bh, dtype=np.float32) + np.einsum(eq, ah, bl, dtype=np.float32)
            + np.einsum(eq, al, bh, dtype=np.float32)).astype(np.float32)


def direct64(d, g):
    ci, H, W = d.shape
    co, _, r, _ = g.shape
    Ho, Wo = H - r + 1, W - r + 1
    y = np.zeros((co, Ho, Wo))
    for i in range(r):
        for j in range(r):
            y += np.einsum("oc,chw->ohw", g[:, :, i, j], d[:, i:i + Ho, j:j + Wo])
    return y


def direct3(d, g):
    ci, H, W = d.shape
    co, _, r, _ = g.shape
    Ho, Wo = H - r + 1, W - r + 1
    y = np.zeros((co, Ho, Wo), np.float32)
    for i in range(r):
        for j in range(r):
            y += mm3(g[:, :, i, j], d[:, i:i + Ho, j:j + Wo], "oc,chw->ohw")
    return y


def wino(d, g, m, pts, vdtype=np.float32):
    ci, H, W = d.shape
    co, _, r, _ = g.shape
    AT, G, BT = wino_mats(pts, m, r)
    n = m + r - 1
    Ho, Wo = H - r + 1, W - r + 1
    th, tw = Ho // m, Wo // m
    U = np.einsum("ai,ocij,bj->ocab", G, g.astype(np.float64), G).astype(np.float32)
    # input tiles (ci, th, tw, n, n)
    idx_h = (np.arange(th)[:, None] * m + np.arange(n)[None, :])
    idx_w = (np.arange(tw)[:, None] * m + np.arange(n)[None, :])
    tiles = d[:, idx_h[:, None, :, None], idx_w[None, :, None, :]].astype(vdtype)
    BTf = BT.astype(vdtype)
    V = np.einsum("ai,cxyij,bj->cxyab", BTf, tiles, BTf).astype(np.float32)
    M = mm3(U, V, "ocab,cxyab->oxyab")
    ATf = AT.astype(np.float32)
    Y = np.einsum("ia,oxyab,jb->oxyij", ATf, M, ATf).astype(np.float32)
    return Y.transpose(0, 1, 3, 2, 4).reshape(co, th * m, tw * m), np.abs(AT).max(), np.abs(BT).max()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ci", type=int, default=128)
    ap.add_argument("--co", type=int, default=32)
    ap.add_argument("--hw", type=int, default=24)
    args = ap.parse_args()
    rng = np.random.default_rng(0)
    cases = [
        (3, 2, [0, 1, -1]),
        (3, 4, [0, 1, -1, 2, -2]),
        (3, 4, [0, 1, -1, sympy.Rational(1, 2), -sympy.Rational(1, 2)]),
        (7, 2, [0, 1, -1, 2, -2, sympy.Rational(1, 2), -sympy.Rational(1, 2)]),
        (7, 3, [0, 1, -1, 2, -2, sympy.Rational(1, 2), -sympy.Rational(1, 2), 3]),
        (7, 4, [0, 1, -1, 2, -2, sympy.Rational(1, 2), -sympy.Rational(1, 2), 3, -3]),
    ]
    for r, m, pts in cases:
        hw = args.hw - args.hw % m
        d = np.maximum(rng.standard_normal((args.ci, hw + r - 1, hw + r - 1)), 0).astype(np.float32)
        g = (rng.standard_normal((args.co, args.ci, r, r)) * np.sqrt(2.0 / (args.ci * r * r))).astype(np.float32)
        ref = direct64(d.astype(np.float64), g.astype(np.float64))
        e_dir = np.abs(direct3(d, g) - ref).max()
        y, amax, bmax = wino(d, g, m, pts)
        e_w = np.abs(y - ref).max()
        print("F(%dx%d,%dx%d) pts=%s  |y|max %.3g  direct bf16x3 err %.2e  winograd err %.2e (x%.1f)  "
              "mult reduction %.2fx" % (m, m, r, r, [str(p) for p in pts], np.abs(ref).max(), e_dir, e_w,
                                          e_w / e_dir, (m * m * r * r) / (m + r - 1) ** 2))


if __name__ == "__main__":
    main()
