// Device restatement of cv2.resize(INTER_CUBIC) (pose_detector.py:443,461,463,465,467): the same
// arithmetic as oracle/cvcubic.c — source coordinate in double -> f32, interpolateCubic (A = -0.75)
// in f32, edge-clamped taps; uint8: 11-bit coefficients, int32 horizontal pass, vertical pass as
// OpenCV's SIMD body (first floor(W*cn/8)*8 elements of a row, f32 + round-half-even) or scalar
// tail ((sum + 2^21) >> 22); f32: left-to-right horizontal sum, vertical SIMD body (first
// floor(W*cn/4)*4 elements: S0*b0 + (S1*b1 + (S2*b2 + S3*b3))) or scalar tail (left to right).
// Every float op is an explicitly rounded intrinsic (no contraction).
#pragma once
#include "common.hpp"

namespace op {

struct CubicTap {
  int s;       // floor of the source coordinate; taps s-1 .. s+2 (edge-clamped)
  float c[4];  // interpolateCubic coefficients
};

// scale = 1 / (dsize / ssize) in double (OpenCV's inv_scale_x / scale_x); host launchers pass it
// precomputed (IEEE division on the host rounds the same), sparing two f64 divisions per thread
__host__ __device__ inline double cv_cubic_scale(int dsize, int ssize) { return 1.0 / ((double)dsize / (double)ssize); }

__device__ __forceinline__ CubicTap cv_cubic_tap_s(int d, double scale) {
  float f = __double2float_rn(__dsub_rn(__dmul_rn(__dadd_rn((double)d, 0.5), scale), 0.5));
  const int si = (int)floorf(f);
  f = __fsub_rn(f, (float)si);
  const float A = -0.75f;
  const float x1 = __fadd_rn(f, 1.0f);
  CubicTap t;
  t.s = si;
  // ((A*(x+1) - 5A)*(x+1) + 8A)*(x+1) - 4A
  t.c[0] = __fsub_rn(__fmul_rn(__fadd_rn(__fmul_rn(__fsub_rn(__fmul_rn(A, x1), -3.75f), x1), -6.0f), x1), -3.0f);
  // ((A+2)*x - (A+3))*x*x + 1
  t.c[1] = __fadd_rn(__fmul_rn(__fmul_rn(__fsub_rn(__fmul_rn(1.25f, f), 2.25f), f), f), 1.0f);
  const float y = __fsub_rn(1.0f, f);
  t.c[2] = __fadd_rn(__fmul_rn(__fmul_rn(__fsub_rn(__fmul_rn(1.25f, y), 2.25f), y), y), 1.0f);
  t.c[3] = __fsub_rn(__fsub_rn(__fsub_rn(1.0f, t.c[0]), t.c[1]), t.c[2]);
  return t;
}

__device__ __forceinline__ CubicTap cv_cubic_tap(int d, int dsize, int ssize) {
  const double inv = __ddiv_rn((double)dsize, (double)ssize);
  return cv_cubic_tap_s(d, __ddiv_rn(1.0, inv));
}

__device__ __forceinline__ int cv_cubic_fix(float c) {  // saturate_cast<short>(c * 2048)
  const float r = rintf(__fmul_rn(c, 2048.0f));
  return (int)(r < -32768.f ? -32768.f : (r > 32767.f ? 32767.f : r));
}

__device__ __forceinline__ int clampc(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// One uint8 output element (dx, dy, channel ch) of a cn-channel image; e = dx*cn + ch.
__device__ __forceinline__ int cv_cubic_u8(const uint8_t* src, int64_t sstride, int sh, int sw, int cn, int ch,
                                           const CubicTap& tx, const CubicTap& ty, int e, int simd_end) {
  int ia[4], ib[4], hs[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    ia[k] = cv_cubic_fix(tx.c[k]);
    ib[k] = cv_cubic_fix(ty.c[k]);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint8_t* row = src + (int64_t)clampc(ty.s - 1 + k, 0, sh - 1) * sstride;
    int v = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) v += (int)row[clampc(tx.s - 1 + j, 0, sw - 1) * cn + ch] * ia[j];
    hs[k] = v;
  }
  int r;
  if (e < simd_end) {
    const float sc = 1.0f / (2048.0f * 2048.0f);
    const float t3 = __fmul_rn((float)hs[3], __fmul_rn((float)ib[3], sc));
    const float t2 = __fadd_rn(__fmul_rn((float)hs[2], __fmul_rn((float)ib[2], sc)), t3);
    const float t1 = __fadd_rn(__fmul_rn((float)hs[1], __fmul_rn((float)ib[1], sc)), t2);
    const float t0 = __fadd_rn(__fmul_rn((float)hs[0], __fmul_rn((float)ib[0], sc)), t1);
    r = (int)rintf(t0);
  } else {
    const int v = hs[0] * ib[0] + hs[1] * ib[1] + hs[2] * ib[2] + hs[3] * ib[3];
    r = (v + (1 << 21)) >> 22;
  }
  return clampc(r, 0, 255);
}

// One f32 output element; src element (y, x, ch) at src[y*sstride + x*pstride + ch*cstride]
// (interleaved: cstride 1; planar: pstride 1, cstride = plane size).
__device__ __forceinline__ float cv_cubic_f32(const float* src, int64_t sstride, int pstride, int sh, int sw, int ch,
                                              const CubicTap& tx, const CubicTap& ty, int e, int simd_end,
                                              int64_t cstride = 1) {
  float hs[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float* row = src + (int64_t)clampc(ty.s - 1 + k, 0, sh - 1) * sstride + ch * cstride;
    float v = __fmul_rn(row[(int64_t)clampc(tx.s - 1, 0, sw - 1) * pstride], tx.c[0]);
    v = __fadd_rn(v, __fmul_rn(row[(int64_t)clampc(tx.s, 0, sw - 1) * pstride], tx.c[1]));
    v = __fadd_rn(v, __fmul_rn(row[(int64_t)clampc(tx.s + 1, 0, sw - 1) * pstride], tx.c[2]));
    v = __fadd_rn(v, __fmul_rn(row[(int64_t)clampc(tx.s + 2, 0, sw - 1) * pstride], tx.c[3]));
    hs[k] = v;
  }
  if (e < simd_end) {
    const float t3 = __fmul_rn(hs[3], ty.c[3]);
    const float t2 = __fadd_rn(__fmul_rn(hs[2], ty.c[2]), t3);
    const float t1 = __fadd_rn(__fmul_rn(hs[1], ty.c[1]), t2);
    return __fadd_rn(__fmul_rn(hs[0], ty.c[0]), t1);
  }
  return __fadd_rn(__fadd_rn(__fadd_rn(__fmul_rn(hs[0], ty.c[0]), __fmul_rn(hs[1], ty.c[1])), __fmul_rn(hs[2], ty.c[2])),
                   __fmul_rn(hs[3], ty.c[3]));
}

}  // namespace op
