// Host-side weight packing and SciPy Gaussian taps shared by the CocoPoseNet runtime
// (runtime.hip) and the FaceNet / HandNet detectors (cpm.hip).
#pragma once
#include <stdint.h>
#include <string.h>

#include <cmath>
#include <vector>

namespace op {

inline uint16_t bf16_rne(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  if ((u & 0x7f800000u) == 0x7f800000u) return (uint16_t)(u >> 16);  // inf / nan: truncate
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

inline float bf16_f(uint16_t b) {
  const uint32_t u = (uint32_t)b << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

// Pack Chainer W (Co, Ci, k, k) into the split layout at output-channel offset co_off:
// element (c16, tap, co, h, part, j) = part 0: bf16(w), part 1: bf16(w - hi) for input channel
// 16*c16 + 8h + j, stored planar [c16][tap][plane = 2h + (0 hi | 1 lo)][cop][8].  cmap(p) gives the
// logical input channel of physical channel p (-1: zero padding).
template <class CMap>
void pack_split(std::vector<uint16_t>& dst, int cop, int cin16, int k, const float* W, int Co, int Ci, int co_off,
                CMap cmap) {
  const int taps = k * k;
  for (int co = 0; co < Co; ++co)
    for (int p = 0; p < cin16; ++p) {
      const int ci = cmap(p);
      if (ci < 0 || ci >= Ci) continue;
      const int c16 = p / 16, h = (p % 16) / 8, j = p % 8;
      for (int t = 0; t < taps; ++t) {
        const int ky = t / k, kx = t % k;
        const float v = W[(((size_t)co * Ci + ci) * k + ky) * k + kx];
        const uint16_t hb = bf16_rne(v);
        const uint16_t lb = bf16_rne(v - bf16_f(hb));
        const size_t tile = ((size_t)c16 * taps + t) * 4;
        dst[((tile + 2 * h) * cop + (co_off + co)) * 8 + j] = hb;
        dst[((tile + 2 * h + 1) * cop + (co_off + co)) * 8 + j] = lb;
      }
    }
}

// scipy.ndimage._gaussian_kernel1d(sigma, 0, int(4 * sigma + 0.5)): exp taps normalised by their
// NumPy pairwise sum; returns the radius.
inline int gaussian_taps(double sigma, std::vector<double>& w) {
  const int r = (int)(4.0 * sigma + 0.5);
  w.assign(2 * r + 1, 0.0);
  const double coef = -0.5 / (sigma * sigma);
  for (int i = 0; i <= 2 * r; ++i) w[i] = std::exp(coef * (double)((i - r) * (i - r)));
  const int n = 2 * r + 1;
  double s;
  if (n < 8) {
    s = 0;
    for (int i = 0; i < n; ++i) s += w[i];
  } else {
    double rr[8];
    for (int j = 0; j < 8; ++j) rr[j] = w[j];
    int i = 8;
    for (; i < n - (n % 8); i += 8)
      for (int j = 0; j < 8; ++j) rr[j] += w[i + j];
    s = ((rr[0] + rr[1]) + (rr[2] + rr[3])) + ((rr[4] + rr[5]) + (rr[6] + rr[7]));
    for (; i < n; ++i) s += w[i];
  }
  for (auto& v : w) v = v / s;
  return r;
}

// The GPU branch's kernel (pose_detector.py:38-44, built at :34 with params 'gaussian_sigma' /
// 'ksize'): K[dy][dx] = exp(-0.5 (dx^2 + dy^2) / sigma^2) / (2 pi sigma^2) over ksize x ksize, NOT
// normalised, is the outer product g g^T of g(d) = exp(-0.5 d^2 / sigma^2) / sqrt(2 pi sigma^2),
// d = -r .. r, r = ksize / 2: w = g (2r + 1 doubles), returns r.  The device filter runs the two
// 1-D passes (f64, f32 between them) instead of the reference's 2-D f32 convolution: the same
// products up to rounding (~1e-7 relative, tests/test_gpu_peak_mode.py).
inline int gpu_branch_taps(double sigma, int ksize, std::vector<double>& w) {
  const int r = ksize / 2;
  w.assign(2 * r + 1, 0.0);
  const double norm = std::sqrt(2.0 * 3.14159265358979323846 * sigma * sigma);
  for (int i = 0; i <= 2 * r; ++i) w[i] = std::exp(-0.5 * (double)((i - r) * (i - r)) / (sigma * sigma)) / norm;
  return r;
}

}  // namespace op
