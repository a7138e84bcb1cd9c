/* ORACLE — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).
 *
 * cv2.resize(..., interpolation=cv2.INTER_CUBIC) as used by PoseDetector.detect_precise
 * (pose_detector.py:443 on the uint8 frame, :461/:463 on the f32 PAF, :465/:467 on the f32 heat
 * maps).  OpenCV is not installed, so this restates its generic (non-IPP) resize path —
 * "parity unpinned":
 *   - source coordinate fx = (float)((dx + 0.5) * (1 / inv_scale) - 0.5), inv_scale = dw / sw
 *     (double); sx = floor(fx); fx -= sx;
 *   - interpolateCubic(fx) with A = -0.75 in f32; out-of-range taps clamp to the edge pixel;
 *   - uint8: coefficients saturate_cast<short>(c * 2048); horizontal pass in int32; vertical pass
 *     as VResizeCubicVec_32s8u computes it over the first floor(W*cn / 8) * 8 elements of a row
 *     (f32: S0*b0 + (S1*b1 + (S2*b2 + S3*b3)) with b = beta * 2^-22, round half-even, saturate)
 *     and the scalar VResizeCubic over the rest ((sum + 2^21) >> 22, saturate);
 *   - f32: horizontal ((S0*a0 + S1*a1) + S2*a2) + S3*a3; vertical VResizeCubicVec_32f over the
 *     first floor(W*cn / 4) * 4 elements (S0*b0 + (S1*b1 + (S2*b2 + S3*b3))) and the scalar
 *     ((S0*b0 + S1*b1) + S2*b2) + S3*b3 over the rest.
 * Every operation is rounded as written (compiled with -ffp-contract=off).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>

static void cubic_coeffs(float x, float c[4]) {
  const float A = -0.75f;
  c[0] = ((A * (x + 1) - 5 * A) * (x + 1) + 8 * A) * (x + 1) - 4 * A;
  c[1] = ((A + 2) * x - (A + 3)) * x * x + 1;
  c[2] = ((A + 2) * (1 - x) - (A + 3)) * (1 - x) * (1 - x) + 1;
  c[3] = 1.f - c[0] - c[1] - c[2];
}

static void cubic_tap(int d, int dsize, int ssize, int* s, float c[4]) {
  const double inv = (double)dsize / (double)ssize;
  const double scale = 1.0 / inv;
  float f = (float)((d + 0.5) * scale - 0.5);
  const int si = (int)floorf(f);
  f -= (float)si;
  *s = si;
  cubic_coeffs(f, c);
}

static int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

static short round_short(float v) {
  const float r = nearbyintf(v);
  return (short)(r < -32768.f ? -32768 : (r > 32767.f ? 32767 : r));
}

/* src: sh x sw x cn uint8 with row stride sstride bytes; dst: dh x dw x cn contiguous. */
void orc_resize_cubic_u8(const uint8_t* src, int sh, int sw, int cn, int64_t sstride, uint8_t* dst, int dh, int dw) {
  int* xs = (int*)malloc(sizeof(int) * dw);
  short* ia = (short*)malloc(sizeof(short) * 4 * dw);
  for (int dx = 0; dx < dw; ++dx) {
    float c[4];
    cubic_tap(dx, dw, sw, &xs[dx], c);
    for (int k = 0; k < 4; ++k) ia[4 * dx + k] = round_short(c[k] * 2048);
  }
  const int rowlen = dw * cn;
  const int simd_end = rowlen / 8 * 8;
  for (int dy = 0; dy < dh; ++dy) {
    int sy;
    float cy[4];
    short ib[4];
    cubic_tap(dy, dh, sh, &sy, cy);
    for (int k = 0; k < 4; ++k) ib[k] = round_short(cy[k] * 2048);
    const float scale = 1.f / (2048 * 2048);
    float bf[4];
    for (int k = 0; k < 4; ++k) bf[k] = ib[k] * scale;
    for (int dx = 0; dx < dw; ++dx)
      for (int ch = 0; ch < cn; ++ch) {
        int hs[4];
        for (int k = 0; k < 4; ++k) {
          const uint8_t* row = src + (int64_t)clampi(sy - 1 + k, 0, sh - 1) * sstride;
          int v = 0;
          for (int j = 0; j < 4; ++j) v += (int)row[clampi(xs[dx] - 1 + j, 0, sw - 1) * cn + ch] * ia[4 * dx + j];
          hs[k] = v;
        }
        const int e = dx * cn + ch;
        int r;
        if (e < simd_end) {
          const float t3 = (float)hs[3] * bf[3];
          const float t2 = (float)hs[2] * bf[2] + t3;
          const float t1 = (float)hs[1] * bf[1] + t2;
          const float t0 = (float)hs[0] * bf[0] + t1;
          r = (int)nearbyintf(t0);
        } else {
          const int v = hs[0] * ib[0] + hs[1] * ib[1] + hs[2] * ib[2] + hs[3] * ib[3];
          r = (v + (1 << 21)) >> 22;
        }
        dst[((int64_t)dy * dw + dx) * cn + ch] = (uint8_t)clampi(r, 0, 255);
      }
  }
  free(xs);
  free(ia);
}

/* src: sh x sw x cn f32 with row stride sstride elements; dst: dh x dw x cn contiguous. */
void orc_resize_cubic_f32(const float* src, int sh, int sw, int cn, int64_t sstride, float* dst, int dh, int dw) {
  int* xs = (int*)malloc(sizeof(int) * dw);
  float* al = (float*)malloc(sizeof(float) * 4 * dw);
  for (int dx = 0; dx < dw; ++dx) cubic_tap(dx, dw, sw, &xs[dx], al + 4 * dx);
  const int rowlen = dw * cn;
  const int simd_end = rowlen / 4 * 4;
  for (int dy = 0; dy < dh; ++dy) {
    int sy;
    float b[4];
    cubic_tap(dy, dh, sh, &sy, b);
    for (int dx = 0; dx < dw; ++dx)
      for (int ch = 0; ch < cn; ++ch) {
        float hs[4];
        for (int k = 0; k < 4; ++k) {
          const float* row = src + (int64_t)clampi(sy - 1 + k, 0, sh - 1) * sstride;
          const float* a = al + 4 * dx;
          float v = row[clampi(xs[dx] - 1, 0, sw - 1) * cn + ch] * a[0];
          v = v + row[clampi(xs[dx], 0, sw - 1) * cn + ch] * a[1];
          v = v + row[clampi(xs[dx] + 1, 0, sw - 1) * cn + ch] * a[2];
          v = v + row[clampi(xs[dx] + 2, 0, sw - 1) * cn + ch] * a[3];
          hs[k] = v;
        }
        const int e = dx * cn + ch;
        float r;
        if (e < simd_end) {
          const float t3 = hs[3] * b[3];
          const float t2 = hs[2] * b[2] + t3;
          const float t1 = hs[1] * b[1] + t2;
          r = hs[0] * b[0] + t1;
        } else {
          r = ((hs[0] * b[0] + hs[1] * b[1]) + hs[2] * b[2]) + hs[3] * b[3];
        }
        dst[((int64_t)dy * dw + dx) * cn + ch] = r;
      }
  }
  free(xs);
  free(al);
}
