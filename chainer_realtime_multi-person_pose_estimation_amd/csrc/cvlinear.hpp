// Device restatement of cv2.resize(INTER_LINEAR) on uint8 + the reference preprocess
// (pose_detector.py:493-494, 426-431); shared by the f32 and the split-bf16 input kernels.
#pragma once
#include "common.hpp"

namespace op {

// ---- cv2.resize(INTER_LINEAR, uint8) restatement + preprocess (pose_detector.py:493-494, 426-431) ----
// Same arithmetic as oracle/cvresize.py (OpenCV fixed point, 11-bit coefficients, SIMD-body
// vertical rounding); every double/float op is explicitly rounded, no contraction.
struct LinTap {
  int s0, s1;
  int c0, c1;
};

__device__ __forceinline__ LinTap cv_linear_tap(int d, int dsize, int ssize, bool clampx) {
  const double inv = __ddiv_rn((double)dsize, (double)ssize);
  const double scale = __ddiv_rn(1.0, inv);
  float f = __double2float_rn(__dsub_rn(__dmul_rn(__dadd_rn((double)d, 0.5), scale), 0.5));
  int sidx = (int)floorf(f);
  f = __fsub_rn(f, (float)sidx);
  if (clampx) {
    if (sidx < 0) {
      f = 0.0f;
      sidx = 0;
    }
    if (sidx >= ssize - 1) {
      f = 0.0f;
      sidx = ssize - 1;
    }
  }
  LinTap t;
  t.s0 = sidx;
  t.s1 = sidx + 1;
  t.c0 = __float2int_rn(__fmul_rn(__fsub_rn(1.0f, f), 2048.0f));
  t.c1 = __float2int_rn(__fmul_rn(f, 2048.0f));
  return t;
}

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// div: 255 (pose_detector.py:426-431) or 256 (face_detector.py:33, hand_detector.py:36)
__device__ __forceinline__ float cv_linear_px(const uint8_t* src, int64_t row_stride, int sh, int sw, const LinTap& tx,
                                              const LinTap& ty, int ch, float div = 255.0f) {
  const int x0 = tx.s0, x1 = tx.s1 < sw ? tx.s1 : sw - 1;
  const int r0 = clampi(ty.s0, 0, sh - 1), r1 = clampi(ty.s1, 0, sh - 1);
  const uint8_t* p0 = src + (int64_t)r0 * row_stride;
  const uint8_t* p1 = src + (int64_t)r1 * row_stride;
  const int h0 = (int)p0[x0 * 3 + ch] * tx.c0 + (int)p0[x1 * 3 + ch] * tx.c1;
  const int h1 = (int)p1[x0 * 3 + ch] * tx.c0 + (int)p1[x1 * 3 + ch] * tx.c1;
  int v = ((((h0 >> 4) * ty.c0) >> 16) + (((h1 >> 4) * ty.c1) >> 16) + 2) >> 2;
  v = clampi(v, 0, 255);
  return __fsub_rn(__fdiv_rn((float)v, div), 0.5f);
}


__device__ __forceinline__ float cv_linear_norm(const uint8_t* src, int64_t row_stride, int sh, int sw, int dx, int dy,
                                                int dw, int dh, int ch, float div = 255.0f) {
  const LinTap tx = cv_linear_tap(dx, dw, sw, true);
  const LinTap ty = cv_linear_tap(dy, dh, sh, false);
  return cv_linear_px(src, row_stride, sh, sw, tx, ty, ch, div);
}

}  // namespace op
