// Kernels of the multi-scale path PoseDetector.detect_precise (pose_detector.py:433-482):
// cv2.resize(INTER_CUBIC) of the frame fused with pad_image + preprocess into the network input,
// and the cubic resizes of the last-stage maps (to the padded size, crop, to the original size)
// fused with the running sum over scales and the final division by the scale count.
#include "common.hpp"
#include "cvcubic.hpp"

namespace op {

__device__ __forceinline__ float norm_u8(int v) { return __fsub_rn(__fdiv_rn((float)v, 255.0f), 0.5f); }

// The cubic taps of output rows y0 .. y0 + TY - 1 (clamped to ylast), block-uniform: lane yy of the
// wave makes row yy's (one f64 tap computation per lane instead of TY per lane) and v_readlane
// moves them to scalar registers.  Lanes 0 .. TY-1 must be active (a lane that has returned holds
// no defined value for v_readlane).
template <int TY>
__device__ __forceinline__ void row_taps(int y0, int ylast, double scy, CubicTap (&ty)[TY]) {
  static_assert(TY <= 64, "one row per lane");
  const int lane = threadIdx.x & 63;
  const CubicTap t = cv_cubic_tap_s(min(y0 + min(lane, TY - 1), ylast), scy);
#pragma unroll
  for (int yy = 0; yy < TY; ++yy) {
    ty[yy].s = __builtin_amdgcn_readlane(t.s, yy);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      ty[yy].c[j] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, t.c[j]), yy));
  }
}

// Padded network input (h = ph, w = pw, 1-pixel zero halo): pixel (x, y) < (rw, rh) is the cubic
// resize of the frame, the rest the pad colour (104, 117, 123) (pose_detector.py:446, :46-55),
// normalised (x/255 - 0.5, :426-431).  SPLIT: 16 channels as bf16 hi/lo (split format), else
// 8 f32 channels.
// Frame blockIdx.y of the batch: bgr + y * src_fstride bytes -> out + y * dst_fbytes.
template <bool SPLIT>
__global__ __launch_bounds__(256) void preprocess_cubic(const uint8_t* __restrict__ bgr, int64_t row_stride, int sh,
                                                        int sw, int rh, int rw, int ph, int pw, char* __restrict__ out,
                                                        int64_t src_fstride, int64_t dst_fbytes) {
  const int wp = pw + 2, hp = ph + 2;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)hp * wp) return;
  bgr += blockIdx.y * src_fstride;
  out += blockIdx.y * dst_fbytes;
  const int px = (int)(i % wp), py = (int)(i / wp);
  float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const int dx = px - 1, dy = py - 1;
  if (dx >= 0 && dx < pw && dy >= 0 && dy < ph) {
    if (dx < rw && dy < rh) {
      const CubicTap tx = cv_cubic_tap(dx, rw, sw);
      const CubicTap ty = cv_cubic_tap(dy, rh, sh);
      const int simd_end = rw * 3 / 8 * 8;
      for (int ch = 0; ch < 3; ++ch)
        v[ch] = norm_u8(cv_cubic_u8(bgr, row_stride, sh, sw, 3, ch, tx, ty, dx * 3 + ch, simd_end));
    } else {
      v[0] = norm_u8(104);
      v[1] = norm_u8(117);
      v[2] = norm_u8(123);
    }
  }
  if constexpr (SPLIT) {
    unsigned short hs[8], ls[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const __bf16 h16 = (__bf16)v[k];
      const __bf16 l16 = (__bf16)(v[k] - (float)h16);
      hs[k] = __builtin_bit_cast(unsigned short, h16);
      ls[k] = __builtin_bit_cast(unsigned short, l16);
    }
    uint4* o = (uint4*)(out + i * 64);
    o[0] = *(const uint4*)hs;
    o[1] = *(const uint4*)ls;
    o[2] = make_uint4(0, 0, 0, 0);
    o[3] = make_uint4(0, 0, 0, 0);
  } else {
    floatx4* o = (floatx4*)(out + i * 32);
    o[0] = floatx4{v[0], v[1], v[2], v[3]};
    o[1] = floatx4{v[4], v[5], v[6], v[7]};
  }
}

int launch_preprocess_cubic(const uint8_t* bgr, int64_t row_stride, int32_t sh, int32_t sw, int32_t rh, int32_t rw,
                            int32_t ph, int32_t pw, bool split, float* out, int32_t n, int64_t src_fstride,
                            int64_t dst_ffloats, hipStream_t st) {
  const int64_t total = (int64_t)(ph + 2) * (pw + 2);
  const dim3 grid((unsigned)((total + 255) / 256), (unsigned)n);
  const int64_t dst_fbytes = dst_ffloats * (int64_t)sizeof(float);
  if (split)
    hipLaunchKernelGGL(preprocess_cubic<true>, grid, dim3(256), 0, st, bgr, row_stride, sh, sw, rh, rw, ph, pw,
                       (char*)out, src_fstride, dst_fbytes);
  else
    hipLaunchKernelGGL(preprocess_cubic<false>, grid, dim3(256), 0, st, bgr, row_stride, sh, sw, rh, rw, ph, pw,
                       (char*)out, src_fstride, dst_fbytes);
  OP_AFTER_LAUNCH("preprocess_cubic", st);
  OP_HIP_CHECK(hipGetLastError());
  return OP_OK;
}

// Generic cv2.resize(INTER_CUBIC) of a cn-channel f32 image (element (y, x, c) at
// src[y*sstride + x*pstride + c]) to dh x dw.
//   mode 0: dst NHWC (dh, dw, cn) contiguous;
//   mode 1/2/3: dst planar (cn, dh, dw): 1 store, 2 add to dst, 3 add then divide by `div`
//   (the running sum over scales of pose_detector.py:463/467 and its mean at :469-470).
__global__ __launch_bounds__(256) void resize_cubic_f32(const float* __restrict__ src, int64_t sstride, int pstride,
                                                        int sh, int sw, int cn, float* __restrict__ dst, int dh, int dw,
                                                        int mode, float div, double scx, double scy) {
  const int64_t total = (int64_t)cn * dh * dw;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  int x, y, c;
  if (mode == 0) {
    c = (int)(i % cn);
    x = (int)((i / cn) % dw);
    y = (int)(i / ((int64_t)cn * dw));
  } else {
    x = (int)(i % dw);
    y = (int)((i / dw) % dh);
    c = (int)(i / ((int64_t)dw * dh));
  }
  const CubicTap tx = cv_cubic_tap_s(x, scx);
  const CubicTap ty = cv_cubic_tap_s(y, scy);
  const float v = cv_cubic_f32(src, sstride, pstride, sh, sw, c, tx, ty, x * cn + c, dw * cn / 4 * 4);
  if (mode == 0) {
    dst[i] = v;
  } else if (mode == 1) {
    dst[i] = v;
  } else if (mode == 2) {
    dst[i] = __fadd_rn(dst[i], v);
  } else {
    dst[i] = __fdiv_rn(__fadd_rn(dst[i], v), div);
  }
}

int launch_resize_cubic_f32(const float* src, int64_t sstride, int32_t pstride, int32_t sh, int32_t sw, int32_t cn,
                            float* dst, int32_t dh, int32_t dw, int32_t mode, float div, hipStream_t st) {
  const int64_t total = (int64_t)cn * dh * dw;
  hipLaunchKernelGGL(resize_cubic_f32, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, src, sstride, pstride,
                     sh, sw, cn, dst, dh, dw, mode, div, cv_cubic_scale(dw, sw), cv_cubic_scale(dh, sh));
  OP_AFTER_LAUNCH("resize_cubic_f32", st);
  OP_HIP_CHECK(hipGetLastError());
  return OP_OK;
}

// Mode 1 for upsampling resizes, n frames per launch (round 3): a block is 256 output columns x
// kUpRows output rows of one (frame, channel).  Each thread makes the horizontal sums of the few
// source rows those output rows need -- once, instead of once per output row as resize_cubic_f32
// does -- keeps them in its own LDS column, then makes every output row's vertical sum from them.
// The f32 operations of each output element are resize_cubic_f32's (cv_cubic_f32), in its order.
// Round 4: kUpRows and the prefetch (every source row's four taps loaded before the first
// horizontal sum: one memory latency per block instead of one per source row) are build knobs.
#ifndef UP_ROWS
#define UP_ROWS 16
#endif
#ifndef UP_PREFETCH
#define UP_PREFETCH 1
#endif
constexpr int kUpRows = UP_ROWS, kUpSrc = 8;
__global__ __launch_bounds__(256) void resize_cubic_f32_up(const float* __restrict__ src, int64_t sstride, int pstride,
                                                           int64_t src_fstride, int sh, int sw, int cn,
                                                           float* __restrict__ dst, int64_t dst_fstride, int dh, int dw,
                                                           double scx, double scy) {
  __shared__ float hsum[kUpSrc][256];
  const int x = blockIdx.x * 256 + threadIdx.x;
  const int y0 = blockIdx.y * kUpRows;
  const int f = blockIdx.z / cn, c = blockIdx.z - (blockIdx.z / cn) * cn;
  // no barrier below: a thread reads only its own LDS column; whole waves past the right edge
  // leave (lanes 0 .. kUpRows-1 of a wave make its row taps)
  if (blockIdx.x * 256 + (threadIdx.x & ~63) >= dw) return;
  const bool live = x < dw;
  const int ylast = min(y0 + kUpRows - 1, dh - 1);
  // lane yy makes output row y0 + yy's taps (clamped to ylast); each row's are read out by
  // v_readlane where they are used (kUpRows rows of taps would not fit the scalar registers)
  const CubicTap tl = cv_cubic_tap_s(min(y0 + min((int)(threadIdx.x & 63), kUpRows - 1), ylast), scy);
  const int r0 = __builtin_amdgcn_readlane(tl.s, 0) - 1;
  const int nr = __builtin_amdgcn_readlane(tl.s, kUpRows - 1) + 2 - r0 + 1;  // <= kUpSrc (the launcher checks)
  const CubicTap tx = cv_cubic_tap_s(min(x, dw - 1), scx);
  int64_t col[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) col[j] = (int64_t)clampc(tx.s - 1 + j, 0, sw - 1) * pstride;
  const float* fs = src + (int64_t)f * src_fstride + c;
#if UP_PREFETCH
  float q[kUpSrc][4];
#pragma unroll
  for (int r = 0; r < kUpSrc; ++r) {
    if (r < nr) {
      const float* row = fs + (int64_t)clampc(r0 + r, 0, sh - 1) * sstride;
#pragma unroll
      for (int j = 0; j < 4; ++j) q[r][j] = row[col[j]];
    }
  }
#pragma unroll
  for (int r = 0; r < kUpSrc; ++r) {
    if (r < nr) {
      float h = __fmul_rn(q[r][0], tx.c[0]);
      h = __fadd_rn(h, __fmul_rn(q[r][1], tx.c[1]));
      h = __fadd_rn(h, __fmul_rn(q[r][2], tx.c[2]));
      h = __fadd_rn(h, __fmul_rn(q[r][3], tx.c[3]));
      hsum[r][threadIdx.x] = h;
    }
  }
#else
  for (int r = 0; r < nr; ++r) {
    const float* row = fs + (int64_t)clampc(r0 + r, 0, sh - 1) * sstride;
    float h = __fmul_rn(row[col[0]], tx.c[0]);
    h = __fadd_rn(h, __fmul_rn(row[col[1]], tx.c[1]));
    h = __fadd_rn(h, __fmul_rn(row[col[2]], tx.c[2]));
    h = __fadd_rn(h, __fmul_rn(row[col[3]], tx.c[3]));
    hsum[r][threadIdx.x] = h;
  }
#endif
  // dead lanes (x >= dw) stay to the end: lanes 0 .. kUpRows-1 hold the row taps read below
  const bool simd = x * cn + c < dw * cn / 4 * 4;
  float* o = dst + (int64_t)f * dst_fstride + ((int64_t)c * dh + y0) * dw + x;
#pragma unroll
  for (int yy = 0; yy < kUpRows; ++yy) {
    if (y0 + yy > ylast) continue;  // (not break: the loop stays unrolled, constant readlane lanes)
    CubicTap ty1;
    ty1.s = __builtin_amdgcn_readlane(tl.s, yy);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      ty1.c[j] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, tl.c[j]), yy));
    const int b = ty1.s - 1 - r0;
    const float h0 = hsum[b][threadIdx.x], h1 = hsum[b + 1][threadIdx.x];
    const float h2 = hsum[b + 2][threadIdx.x], h3 = hsum[b + 3][threadIdx.x];
    float v;
    if (simd) {
      const float t3 = __fmul_rn(h3, ty1.c[3]);
      const float t2 = __fadd_rn(__fmul_rn(h2, ty1.c[2]), t3);
      const float t1 = __fadd_rn(__fmul_rn(h1, ty1.c[1]), t2);
      v = __fadd_rn(__fmul_rn(h0, ty1.c[0]), t1);
    } else {
      v = __fadd_rn(__fadd_rn(__fadd_rn(__fmul_rn(h0, ty1.c[0]), __fmul_rn(h1, ty1.c[1])),
                              __fmul_rn(h2, ty1.c[2])),
                    __fmul_rn(h3, ty1.c[3]));
    }
    if (live) o[(int64_t)yy * dw] = v;
  }
}

int launch_resize_cubic_f32_frames(const float* src, int64_t sstride, int32_t pstride, int64_t src_fstride, int32_t sh,
                                   int32_t sw, int32_t cn, float* dst, int64_t dst_fstride, int32_t dh, int32_t dw,
                                   int32_t n, hipStream_t st) {
  const double scx = cv_cubic_scale(dw, sw), scy = cv_cubic_scale(dh, sh);
  // source rows one block of kUpRows output rows needs: at most ceil((kUpRows - 1) * scy) + 1 + 3
  const bool up = dh >= sh && dw >= sw && (int)((kUpRows - 1) * scy) + 5 <= kUpSrc;
  if (!up) {
    for (int f = 0; f < n; ++f) {
      const int rc = launch_resize_cubic_f32(src + (int64_t)f * src_fstride, sstride, pstride, sh, sw, cn,
                                             dst + (int64_t)f * dst_fstride, dh, dw, 1, 1.0f, st);
      if (rc) return rc;
    }
    return OP_OK;
  }
  hipLaunchKernelGGL(resize_cubic_f32_up, dim3((unsigned)((dw + 255) / 256), (unsigned)((dh + kUpRows - 1) / kUpRows),
                                               (unsigned)(cn * n)),
                     dim3(256), 0, st, src, sstride, pstride, src_fstride, sh, sw, cn, dst, dst_fstride, dh, dw, scx, scy);
  OP_AFTER_LAUNCH("resize_cubic_f32_up", st);
  OP_HIP_CHECK(hipGetLastError());
  return OP_OK;
}

// The same resize from a PLANAR source (element (y, x, c) at src[c*cstride + y*sstride + x]) into a
// planar destination (modes 1-3 as above); block = 256 consecutive x of one (row, channel), so the
// row's taps are block-uniform and the source rows are read coalesced.  Values identical to
// resize_cubic_f32 on the interleaved copy of the source (OpenCV's SIMD/tail split still follows
// the interleaved element index x*cn + c).
__global__ __launch_bounds__(256) void resize_cubic_f32_planar(const float* __restrict__ src, int64_t cstride,
                                                               int64_t sstride, int sh, int sw, int cn,
                                                               float* __restrict__ dst, int dh, int dw, int mode,
                                                               float div, double scx, double scy) {
  const int x = blockIdx.x * 256 + threadIdx.x;
  const int y = blockIdx.y, c = blockIdx.z;
  if (x >= dw) return;
  const CubicTap tx = cv_cubic_tap_s(x, scx);
  const CubicTap ty = cv_cubic_tap_s(y, scy);
  const float v = cv_cubic_f32(src, sstride, 1, sh, sw, c, tx, ty, x * cn + c, dw * cn / 4 * 4, cstride);
  const int64_t i = ((int64_t)c * dh + y) * dw + x;
  if (mode == 1) {
    dst[i] = v;
  } else if (mode == 2) {
    dst[i] = __fadd_rn(dst[i], v);
  } else {
    dst[i] = __fdiv_rn(__fadd_rn(dst[i], v), div);
  }
}

int launch_resize_cubic_f32_planar(const float* src, int64_t cstride, int64_t sstride, int32_t sh, int32_t sw,
                                   int32_t cn, float* dst, int32_t dh, int32_t dw, int32_t mode, float div,
                                   hipStream_t st) {
  if (mode < 1 || mode > 3) {
    set_error("resize_cubic_f32_planar: planar modes are 1..3");
    return OP_ERR_INVALID;
  }
  hipLaunchKernelGGL(resize_cubic_f32_planar, dim3((unsigned)((dw + 255) / 256), (unsigned)dh, (unsigned)cn),
                     dim3(256), 0, st, src, cstride, sstride, sh, sw, cn, dst, dh, dw, mode, div, cv_cubic_scale(dw, sw),
                     cv_cubic_scale(dh, sh));
  OP_AFTER_LAUNCH("resize_cubic_f32_planar", st);
  OP_HIP_CHECK(hipGetLastError());
  return OP_OK;
}

// All scales' second pass at once (pose_detector.py:461-470): for every output pixel and map
// channel, the cubic resize of each scale's cropped padded-size map, summed in scale order and
// divided by the scale count -- the same f32 operations, in the same order, as mode 1 / 2 / 3 of
// resize_cubic_f32_planar, without writing and re-reading the running sum once per scale.
// Channels 0..npaf-1 are the PAF map (its own cv2.resize call: SIMD/tail split over npaf
// interleaved channels), npaf.. the heatmap (nheat channels).
// Round 3: a block covers 256 outputs of one row for kMeanG consecutive channels; each thread makes
// a scale's taps once and applies them to its kMeanG channels (scales outer, channels inner, one
// running sum per channel, so every output's f32 operations and their order are unchanged): the
// per-(pixel, channel) f64 tap arithmetic and 64-bit tap addressing were most of the instructions.
constexpr int kMeanG = 8;
__global__ __launch_bounds__(256) void resize_cubic_f32_planar_mean(CubicMeanArgs a, float* __restrict__ dst, int dh,
                                                                    int dw, int npaf, int nheat) {
  const int x = blockIdx.x * 256 + threadIdx.x;
  const int y = blockIdx.y, c0 = blockIdx.z * kMeanG;
  if (x >= dw) return;
  const int nch = npaf + nheat;
  float sum[kMeanG];
  for (int k = 0; k < a.ns; ++k) {
    const CubicTap tx = cv_cubic_tap_s(x, a.scx[k]);
    const CubicTap ty = cv_cubic_tap_s(y, a.scy[k]);
    const int sh = a.sh[k], sw = a.sw[k];
    int64_t roff[4];
    int col[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      roff[r] = (int64_t)clampc(ty.s - 1 + r, 0, sh - 1) * a.sstride[k];
      col[r] = clampc(tx.s - 1 + r, 0, sw - 1);
    }
#pragma unroll
    for (int g = 0; g < kMeanG; ++g) {
      const int c = c0 + g;
      if (c >= nch) break;
      const bool paf = c < npaf;
      const int cn = paf ? npaf : nheat, ce = paf ? c : c - npaf;
      const float* p = a.src[k] + (int64_t)c * a.cstride[k];
      float hs[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {  // cv_cubic_f32 (pstride 1): left-to-right horizontal sums
        const float* row = p + roff[r];
        float h = __fmul_rn(row[col[0]], tx.c[0]);
        h = __fadd_rn(h, __fmul_rn(row[col[1]], tx.c[1]));
        h = __fadd_rn(h, __fmul_rn(row[col[2]], tx.c[2]));
        h = __fadd_rn(h, __fmul_rn(row[col[3]], tx.c[3]));
        hs[r] = h;
      }
      float v;
      if (x * cn + ce < dw * cn / 4 * 4) {  // its vertical orders (SIMD body / scalar tail)
        const float t3 = __fmul_rn(hs[3], ty.c[3]);
        const float t2 = __fadd_rn(__fmul_rn(hs[2], ty.c[2]), t3);
        const float t1 = __fadd_rn(__fmul_rn(hs[1], ty.c[1]), t2);
        v = __fadd_rn(__fmul_rn(hs[0], ty.c[0]), t1);
      } else {
        v = __fadd_rn(__fadd_rn(__fadd_rn(__fmul_rn(hs[0], ty.c[0]), __fmul_rn(hs[1], ty.c[1])), __fmul_rn(hs[2], ty.c[2])),
                      __fmul_rn(hs[3], ty.c[3]));
      }
      sum[g] = k == 0 ? v : __fadd_rn(sum[g], v);
    }
  }
  const int64_t plane = (int64_t)dh * dw;
  float* o = dst + (int64_t)y * dw + x;
#pragma unroll
  for (int g = 0; g < kMeanG; ++g)
    if (c0 + g < nch) o[(c0 + g) * plane] = __fdiv_rn(sum[g], (float)a.ns);
}

int launch_resize_cubic_f32_planar_mean(const CubicMeanArgs& a, float* dst, int32_t dh, int32_t dw, int32_t npaf,
                                        int32_t nheat, hipStream_t st) {
  if (a.ns < 1 || a.ns > OP_MAX_SCALES) {
    set_error("resize_cubic_f32_planar_mean: 1..OP_MAX_SCALES scales");
    return OP_ERR_INVALID;
  }
  hipLaunchKernelGGL(resize_cubic_f32_planar_mean, dim3((unsigned)((dw + 255) / 256), (unsigned)dh,
                                                        (unsigned)((npaf + nheat + kMeanG - 1) / kMeanG)),
                     dim3(256), 0, st, a, dst, dh, dw, npaf, nheat);
  OP_AFTER_LAUNCH("resize_cubic_f32_planar_mean", st);
  OP_HIP_CHECK(hipGetLastError());
  return OP_OK;
}

// The same second pass with a block of TY output rows x 256 columns x G channels, every frame in
// one launch (round 4): per scale a thread makes the horizontal sums of the source rows its block's
// output rows read ONCE, into its own LDS column (resize_cubic_f32_up's scheme, so no barrier), and
// every output row's vertical sum from them -- resize_cubic_f32_planar_mean makes four horizontal
// sums (16 gathers) per output row and scale.  The row taps are made once per scale, the column
// taps once per (scale, thread).  Each output's f32 operations and their order are unchanged:
// horizontal sums left to right, the SIMD-body / scalar-tail vertical orders, scales summed in
// order, one division by the scale count.  LDS: rcap rows x 256 floats (rcap >= the rows any
// block reads at any scale; the host checks).
#ifndef ROWS_UNROLL
#define ROWS_UNROLL 2
#endif
#ifndef ROWS_MINB
#define ROWS_MINB 1
#endif
template <int G, int TY>
__global__ __launch_bounds__(256, ROWS_MINB) void resize_cubic_f32_planar_mean_rows(CubicMeanArgs a, float* __restrict__ dst,
                                                                         int64_t dst_fstride, int dh, int dw, int npaf,
                                                                         int nheat, int ngroups, int rcap, int nbx,
                                                                         int nby, int nblocks) {
  extern __shared__ float hsl[];  // [rcap][256], each thread its own column
  // XCD-aware order: XCD k (= linear id mod 8) runs the k-th eighth of the (x, y, channel, frame)
  // blocks in order, so the blocks of neighbouring output rows -- which read the same source rows
  // -- share one L2 (round-robin placement put them on different XCDs: 1.76x the maps' bytes)
  const int per = (nblocks + 7) >> 3;
  const int lb = (blockIdx.x & 7) * per + (blockIdx.x >> 3);
  if (lb >= nblocks) return;
  const int bz = lb / (nbx * nby), rem = lb - bz * nbx * nby;
  const int by = rem / nbx, bx = rem - by * nbx;
  const int tid = threadIdx.x, x0 = bx * 256, x = x0 + tid;
  const int y0 = by * TY;
  const int f = bz / ngroups, c0 = (bz - f * ngroups) * G;
  if (x0 + (tid & ~63) >= dw) return;  // whole waves past the right edge only (lanes 0..TY-1 make row taps)
  const bool live = x < dw;
  const int nch = npaf + nheat;
  const int ylast = min(y0 + TY - 1, dh - 1);
  float sum[G][TY];
  for (int k = 0; k < a.ns; ++k) {
    const int sh = a.sh[k], sw = a.sw[k];
    CubicTap ty[TY];  // block-uniform: scalar registers
    row_taps<TY>(y0, ylast, a.scy[k], ty);
    const int r0 = ty[0].s - 1;                   // row y0's first tap
    const int nr = ty[TY - 1].s + 2 - r0 + 1;     // .. row ylast's last
    const bool fits = nr <= rcap;  // never false (host bound); else the outputs are NaN
    const CubicTap tx = cv_cubic_tap_s(min(x, dw - 1), a.scx[k]);
    int col[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) col[j] = clampc(tx.s - 1 + j, 0, sw - 1);
    const float* pf = a.src[k] + (int64_t)f * a.fstride[k];
#pragma unroll
    for (int g = 0; g < G; ++g) {  // unrolled: sum[g] stays in registers
      const int c = c0 + g;
      if (c >= nch) break;
      const bool paf = c < npaf;
      const int cn = paf ? npaf : nheat, ce = paf ? c : c - npaf;
      const float* p = pf + (int64_t)c * a.cstride[k];
#pragma unroll ROWS_UNROLL
      for (int r = 0; r < (fits ? nr : 0); ++r) {  // cv_cubic_f32 (pstride 1): left-to-right horizontal sums
        const float* row = p + clampc(r0 + r, 0, sh - 1) * (int)a.sstride[k];
        float h = __fmul_rn(row[col[0]], tx.c[0]);
        h = __fadd_rn(h, __fmul_rn(row[col[1]], tx.c[1]));
        h = __fadd_rn(h, __fmul_rn(row[col[2]], tx.c[2]));
        h = __fadd_rn(h, __fmul_rn(row[col[3]], tx.c[3]));
        hsl[r * 256 + tid] = h;
      }
      const bool simd = x * cn + ce < dw * cn / 4 * 4;
#pragma unroll
      for (int yy = 0; yy < TY; ++yy) {
        const int b = ty[yy].s - 1 - r0;
        const float h0 = hsl[b * 256 + tid], h1 = hsl[(b + 1) * 256 + tid];
        const float h2 = hsl[(b + 2) * 256 + tid], h3 = hsl[(b + 3) * 256 + tid];
        float v;
        if (!fits) {
          v = __builtin_nanf("");
        } else if (simd) {
          const float t3 = __fmul_rn(h3, ty[yy].c[3]);
          const float t2 = __fadd_rn(__fmul_rn(h2, ty[yy].c[2]), t3);
          const float t1 = __fadd_rn(__fmul_rn(h1, ty[yy].c[1]), t2);
          v = __fadd_rn(__fmul_rn(h0, ty[yy].c[0]), t1);
        } else {
          v = __fadd_rn(__fadd_rn(__fadd_rn(__fmul_rn(h0, ty[yy].c[0]), __fmul_rn(h1, ty[yy].c[1])),
                                  __fmul_rn(h2, ty[yy].c[2])),
                        __fmul_rn(h3, ty[yy].c[3]));
        }
        sum[g][yy] = k == 0 ? v : __fadd_rn(sum[g][yy], v);
      }
    }
  }
  if (!live) return;
  const int64_t plane = (int64_t)dh * dw;
#pragma unroll
  for (int g = 0; g < G; ++g) {
    if (c0 + g >= nch) break;
    float* o = dst + (int64_t)f * dst_fstride + (c0 + g) * plane + (int64_t)y0 * dw + x;
#pragma unroll
    for (int yy = 0; yy < TY; ++yy)
      if (y0 + yy < dh) o[(int64_t)yy * dw] = __fdiv_rn(sum[g][yy], (float)a.ns);
  }
}

#ifndef MEAN_ROWS_G
#define MEAN_ROWS_G 1
#endif
#ifndef MEAN_ROWS_TY
#define MEAN_ROWS_TY 12
#endif
// One launch of the row-block form with TY output rows per block; *taken false when a scale's
// rows exceed the 64-KiB LDS budget.
template <int TY>
static int mean_rows_ty(const CubicMeanArgs& a, float* dst, int64_t dst_fstride, int32_t n, int32_t dh, int32_t dw,
                        int32_t npaf, int32_t nheat, hipStream_t st, bool* taken) {
  constexpr int G = MEAN_ROWS_G;
  *taken = false;
  // rows TY consecutive outputs read: floor((TY - 1) * s) + 1 distinct tap origins + 3, + 1 for
  // the f32 rounding of the source coordinate, + 1 spare (as fused_lds)
  int rcap = 0;
  for (int k = 0; k < a.ns; ++k) rcap = std::max(rcap, (int)std::floor((TY - 1) * a.scy[k]) + 7);
  const size_t lds = (size_t)rcap * 256 * sizeof(float);
  if (lds > 64 * 1024) return OP_OK;
  static bool attr = false;
  if (!attr) {
    OP_HIP_CHECK(hipFuncSetAttribute((const void*)resize_cubic_f32_planar_mean_rows<G, TY>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024));
    attr = true;
  }
  const int ngroups = (npaf + nheat + G - 1) / G;
  const int nbx = (dw + 255) / 256, nby = (dh + TY - 1) / TY;
  const int64_t nb = (int64_t)nbx * nby * n * ngroups;
  if (nb > INT32_MAX - 8) {
    set_error("resize_cubic_f32_planar_mean_rows: grid too large");
    return OP_ERR_INVALID;
  }
  const unsigned grid = (unsigned)((nb + 7) / 8 * 8);
  hipLaunchKernelGGL((resize_cubic_f32_planar_mean_rows<G, TY>), dim3(grid), dim3(256), lds, st, a, dst, dst_fstride,
                     dh, dw, npaf, nheat, ngroups, rcap, nbx, nby, (int)nb);
  OP_AFTER_LAUNCH("resize_cubic_f32_planar_mean_rows", st);
  OP_HIP_CHECK(hipGetLastError());
  *taken = true;
  return OP_OK;
}

// MEAN_ROWS_TY (12) rows per block, or 8 where a scale's second resize shrinks its crop so much
// that 12 rows' source rows exceed the LDS budget (small frames: ~7.7x at 96x128); *taken false
// when neither fits (the caller runs the per-frame form).
int launch_resize_cubic_f32_planar_mean_rows(const CubicMeanArgs& a, float* dst, int64_t dst_fstride, int32_t n,
                                             int32_t dh, int32_t dw, int32_t npaf, int32_t nheat, hipStream_t st,
                                             bool* taken) {
  *taken = false;
  if (a.ns < 1 || a.ns > OP_MAX_SCALES) {
    set_error("resize_cubic_f32_planar_mean_rows: 1..OP_MAX_SCALES scales");
    return OP_ERR_INVALID;
  }
  const int rc = mean_rows_ty<MEAN_ROWS_TY>(a, dst, dst_fstride, n, dh, dw, npaf, nheat, st, taken);
  if (rc || *taken || MEAN_ROWS_TY == 8) return rc;
  return mean_rows_ty<8>(a, dst, dst_fstride, n, dh, dw, npaf, nheat, st, taken);
}

// The row-block second pass with each scale's source tile staged in LDS: the block's nr source
// rows x the ~256 * s + 4 source columns its outputs read are loaded once, coalesced (a row
// segment per pass of the block), and the four column taps of every horizontal sum come from LDS
// instead of four gathers from global memory per row.  One channel per block; the horizontal sums
// go to the thread's own LDS column as in _rows; the f32 operations and their order are unchanged.
// LDS: T [rcap][ccap] source tile + H [rcap][256] horizontal sums; rcap <= kTileRows, ccap <= 512.
constexpr int kTileRows = 16;
template <int TY>
__global__ __launch_bounds__(256) void resize_cubic_f32_planar_mean_tile(CubicMeanArgs a, float* __restrict__ dst,
                                                                         int64_t dst_fstride, int dh, int dw, int npaf,
                                                                         int nheat, int rcap, int ccap) {
  extern __shared__ float lds_t[];
  float* T = lds_t;                 // [rcap][ccap]
  float* H = lds_t + rcap * ccap;   // [rcap][256]
  const int nch = npaf + nheat;
  const int tid = threadIdx.x, x0 = blockIdx.x * 256, x = x0 + tid;
  const int y0 = blockIdx.y * TY;
  const int f = blockIdx.z / nch, c = blockIdx.z - f * nch;
  const bool live = x < dw;
  const int xc = min(x, dw - 1), xl = min(x0 + 255, dw - 1);
  const int ylast = min(y0 + TY - 1, dh - 1);
  const bool paf = c < npaf;
  const int cn = paf ? npaf : nheat, ce = paf ? c : c - npaf;
  const bool simd = xc * cn + ce < dw * cn / 4 * 4;
  float sum[TY];
  for (int k = 0; k < a.ns; ++k) {
    const int sh = a.sh[k], sw = a.sw[k];
    const int r0 = cv_cubic_tap_s(y0, a.scy[k]).s - 1;
    const int nr = cv_cubic_tap_s(ylast, a.scy[k]).s + 2 - r0 + 1;
    const int cx0 = clampc(cv_cubic_tap_s(x0, a.scx[k]).s - 1, 0, sw - 1);
    const int nc = clampc(cv_cubic_tap_s(xl, a.scx[k]).s + 2, 0, sw - 1) - cx0 + 1;
    const bool fits = nr <= rcap && nc <= ccap;  // never false (host bounds); else the outputs are NaN
    CubicTap ty[TY];  // block-uniform: scalar registers
    row_taps<TY>(y0, ylast, a.scy[k], ty);
    const CubicTap tx = cv_cubic_tap_s(xc, a.scx[k]);
    int col[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) col[j] = clampc(tx.s - 1 + j, 0, sw - 1) - cx0;
    const float* p = a.src[k] + (int64_t)f * a.fstride[k] + (int64_t)c * a.cstride[k] + cx0;
    if (k) __syncthreads();  // the previous scale's horizontal sums have read T
    if (fits) {  // every row's loads issued before the first LDS store (one memory latency per scale)
      float v0[kTileRows], v1[kTileRows];
      const bool c0ok = tid < nc, c1ok = tid + 256 < nc;
#pragma unroll
      for (int r = 0; r < kTileRows; ++r) {
        const float* row = p + clampc(r0 + min(r, nr - 1), 0, sh - 1) * (int)a.sstride[k];
        v0[r] = c0ok ? row[tid] : 0.f;
        v1[r] = c1ok ? row[tid + 256] : 0.f;
      }
#pragma unroll
      for (int r = 0; r < kTileRows; ++r) {
        if (r < nr) {
          if (c0ok) T[r * ccap + tid] = v0[r];
          if (c1ok) T[r * ccap + tid + 256] = v1[r];
        }
      }
    }
    __syncthreads();
    if (fits) {
#pragma unroll 2
      for (int r = 0; r < nr; ++r) {  // cv_cubic_f32 (pstride 1): left-to-right horizontal sums
        const float* row = T + r * ccap;
        float h = __fmul_rn(row[col[0]], tx.c[0]);
        h = __fadd_rn(h, __fmul_rn(row[col[1]], tx.c[1]));
        h = __fadd_rn(h, __fmul_rn(row[col[2]], tx.c[2]));
        h = __fadd_rn(h, __fmul_rn(row[col[3]], tx.c[3]));
        H[r * 256 + tid] = h;
      }
    }
#pragma unroll
    for (int yy = 0; yy < TY; ++yy) {
      const int b = ty[yy].s - 1 - r0;
      float v;
      if (!fits) {
        v = __builtin_nanf("");
      } else {
        const float h0 = H[b * 256 + tid], h1 = H[(b + 1) * 256 + tid];
        const float h2 = H[(b + 2) * 256 + tid], h3 = H[(b + 3) * 256 + tid];
        if (simd) {
          const float t3 = __fmul_rn(h3, ty[yy].c[3]);
          const float t2 = __fadd_rn(__fmul_rn(h2, ty[yy].c[2]), t3);
          const float t1 = __fadd_rn(__fmul_rn(h1, ty[yy].c[1]), t2);
          v = __fadd_rn(__fmul_rn(h0, ty[yy].c[0]), t1);
        } else {
          v = __fadd_rn(__fadd_rn(__fadd_rn(__fmul_rn(h0, ty[yy].c[0]), __fmul_rn(h1, ty[yy].c[1])),
                                  __fmul_rn(h2, ty[yy].c[2])),
                        __fmul_rn(h3, ty[yy].c[3]));
        }
      }
      sum[yy] = k == 0 ? v : __fadd_rn(sum[yy], v);
    }
  }
  if (live) {
    float* o = dst + (int64_t)f * dst_fstride + (int64_t)c * dh * dw + (int64_t)y0 * dw + x;
#pragma unroll
    for (int yy = 0; yy < TY; ++yy)
      if (y0 + yy < dh) o[(int64_t)yy * dw] = __fdiv_rn(sum[yy], (float)a.ns);
  }
}

int launch_resize_cubic_f32_planar_mean_tile(const CubicMeanArgs& a, float* dst, int64_t dst_fstride, int32_t n,
                                             int32_t dh, int32_t dw, int32_t npaf, int32_t nheat, hipStream_t st,
                                             bool* taken) {
  constexpr int TY = 8;
  *taken = false;
  if (a.ns < 1 || a.ns > OP_MAX_SCALES) {
    set_error("resize_cubic_f32_planar_mean_tile: 1..OP_MAX_SCALES scales");
    return OP_ERR_INVALID;
  }
  // extents as in _rows: T consecutive outputs read floor((T - 1) * s) + 5 source indices, + 1
  // for the f32 rounding of the coordinate, + 1 spare; columns padded to an odd count (banks)
  int rcap = 0, ccap = 0;
  for (int k = 0; k < a.ns; ++k) {
    rcap = std::max(rcap, (int)std::floor((TY - 1) * a.scy[k]) + 7);
    ccap = std::max(ccap, std::min((int)std::floor(255 * a.scx[k]) + 7, a.sw[k]));
  }
  ccap |= 1;
  const size_t lds = (size_t)rcap * (ccap + 256) * sizeof(float);
  if (lds > 64 * 1024 || rcap > kTileRows || ccap > 512) return OP_OK;  // caller runs another form
  static bool attr = false;
  if (!attr) {
    OP_HIP_CHECK(hipFuncSetAttribute((const void*)resize_cubic_f32_planar_mean_tile<TY>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024));
    attr = true;
  }
  hipLaunchKernelGGL((resize_cubic_f32_planar_mean_tile<TY>),
                     dim3((unsigned)((dw + 255) / 256), (unsigned)((dh + TY - 1) / TY), (unsigned)(n * (npaf + nheat))),
                     dim3(256), lds, st, a, dst, dst_fstride, dh, dw, npaf, nheat, rcap, ccap);
  OP_AFTER_LAUNCH("resize_cubic_f32_planar_mean_tile", st);
  OP_HIP_CHECK(hipGetLastError());
  *taken = true;
  return OP_OK;
}

// Last-stage maps -> planar [frame][dst_c0 + c][lh][lw] (the fused resize's input: each scale's maps
// copied out of its activation arena, ~6 MB per 1280x720 frame over the four scales).
__global__ __launch_bounds__(256) void maps_planar(const float* __restrict__ src, int64_t sstride, int pstride,
                                                   int64_t fstride, int lh, int lw, int cn, float* __restrict__ dst,
                                                   int dst_c0, int dst_nch, int n) {
  const int64_t plane = (int64_t)lh * lw;
  const int64_t total = (int64_t)n * cn * plane;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int64_t p = i % plane;
  const int c = (int)((i / plane) % cn);
  const int f = (int)(i / (plane * cn));
  const int y = (int)(p / lw), x = (int)(p - (int64_t)y * lw);
  dst[((int64_t)f * dst_nch + dst_c0 + c) * plane + p] = src[(int64_t)f * fstride + (int64_t)y * sstride +
                                                             (int64_t)x * pstride + c];
}

int launch_maps_planar(const float* src, int64_t sstride, int32_t pstride, int64_t fstride, int32_t lh, int32_t lw,
                       int32_t cn, float* dst, int32_t dst_c0, int32_t dst_nch, int32_t n, hipStream_t st) {
  const int64_t total = (int64_t)n * cn * lh * lw;
  hipLaunchKernelGGL(maps_planar, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, src, sstride, pstride,
                     fstride, lh, lw, cn, dst, dst_c0, dst_nch, n);
  OP_AFTER_LAUNCH("maps_planar", st);
  OP_HIP_CHECK(hipGetLastError());
  return OP_OK;
}

// Both map resizes of every scale (pose_detector.py:461-467) and the scale mean (:469-470) in one
// pass (round 4), without the padded-size maps in HBM.  cv2.resize(map, (pw, ph), CUBIC), the crop
// [:rh, :rw] and cv2.resize(crop, (w, h), CUBIC) of a channel are a chain of separable 4-tap
// filters; a block makes, for a TY x 256 tile of the output and one channel at a time, exactly the
// crop elements that tile's second resize reads, in LDS:
//   a. first resize, horizontal sums of the low-res rows those crop rows need   (H1)
//   b. first resize, vertical sums -> the crop elements                          (I)
//   c. second resize, horizontal sums over the crop rows, each thread its column (H2, own column)
//   d. second resize, vertical sums of the thread's column -> the output rows,
//      summed over the scales in scale order, divided by the scale count once.
// Every element's f32 operations and their order are those of resize_cubic_f32_up (the first
// resize, incl. its SIMD-body / scalar-tail orders over pw x cn) and resize_cubic_f32_planar_mean
// (the second resize and the mean), so the averaged maps are BIT-IDENTICAL to the two-pass path
// (tests/test_gpu_precise_full.py); HBM sees the low-res maps and the averaged output only: per
// 1280x720 frame ~1.04 GB of padded-size map writes and reads become 210 MB of output writes.
// kFusedTY = TY output rows per block: 16, or 8 where the scales' crops are large against the
// output (second-resize ratios over ~1.1) and 16 rows' extents would not fit the LDS budget.
// Loop order: scales outer, the block's kFusedG channels inner, the running sums of all of them
// in registers (sum[g][y]); per scale the taps are made once and the G channels' low-res patches
// are loaded into LDS in one round of global loads.
constexpr int kFusedTX = 256, kFusedG = 2;  // G unrolled: 8 made a ~117 KB kernel (I-cache bound, 12 ms)
template <int kFusedTY>
__global__ __launch_bounds__(256) void resize_cubic_fused_mean(CubicFusedArgs a, float* __restrict__ dst, int dh,
                                                               int dw, int npaf, int nheat) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int nch = npaf + nheat;
  const int ngroups = (nch + kFusedG - 1) / kFusedG;
  const int f = blockIdx.z / ngroups, c0 = (blockIdx.z - f * ngroups) * kFusedG;
  const int ng = min(kFusedG, nch - c0);
  const int x0 = blockIdx.x * kFusedTX, y0 = blockIdx.y * kFusedTY;
  const int tid = threadIdx.x, x = x0 + tid;
  const int xl = min(x0 + kFusedTX - 1, dw - 1), yl = min(y0 + kFusedTY - 1, dh - 1);
  const int rxc = a.rx_cap, ryc = a.ry_cap, lrc = a.lr_cap, pcc = a.pc_cap;
  CubicTap* t1x = (CubicTap*)lds;          // [rx_cap]   first resize, crop columns
  CubicTap* t1y = t1x + rxc;               // [ry_cap]   first resize, crop rows
  CubicTap* t2y = t1y + ryc;               // [TY]       second resize, output rows
  float* P = (float*)(t2y + kFusedTY);     // [G][lr_cap][pc_cap] low-res patches
  float* H1 = P + kFusedG * lrc * pcc;     // [lr_cap][rx_cap]
  float* I = H1 + lrc * rxc;               // [ry_cap][rx_cap]
  float* H2 = I + ryc * rxc;               // [ry_cap][TX]
  float sum[kFusedG][kFusedTY];
  for (int k = 0; k < a.ns; ++k) {
    const int lw = a.lw[k], lh = a.lh[k], rw = a.rw[k], rh = a.rh[k];
    // the crop columns / rows the tile reads, the low-res rows and columns those read (uniform)
    const int qx0 = clampc(cv_cubic_tap_s(x0, a.s2x[k]).s - 1, 0, rw - 1);
    const int NX = clampc(cv_cubic_tap_s(xl, a.s2x[k]).s + 2, 0, rw - 1) - qx0 + 1;
    const int qy0 = clampc(cv_cubic_tap_s(y0, a.s2y[k]).s - 1, 0, rh - 1);
    const int NY = clampc(cv_cubic_tap_s(yl, a.s2y[k]).s + 2, 0, rh - 1) - qy0 + 1;
    const int l0 = clampc(cv_cubic_tap_s(qy0, a.s1y[k]).s - 1, 0, lh - 1);
    const int NL = clampc(cv_cubic_tap_s(qy0 + NY - 1, a.s1y[k]).s + 2, 0, lh - 1) - l0 + 1;
    const int p0 = clampc(cv_cubic_tap_s(qx0, a.s1x[k]).s - 1, 0, lw - 1);
    const int NP = clampc(cv_cubic_tap_s(qx0 + NX - 1, a.s1x[k]).s + 2, 0, lw - 1) - p0 + 1;
    const bool fits = NX <= rxc && NY <= ryc && NL <= lrc && NP <= pcc;  // never false (host bounds)
    __syncthreads();  // the previous scale's last step c has read I; its taps are no longer read
    if (fits) {
      for (int i = tid; i < NX; i += 256) t1x[i] = cv_cubic_tap_s(qx0 + i, a.s1x[k]);
      for (int i = tid; i < NY; i += 256) t1y[i] = cv_cubic_tap_s(qy0 + i, a.s1y[k]);
      if (tid < kFusedTY) t2y[tid] = cv_cubic_tap_s(min(y0 + tid, dh - 1), a.s2y[k]);
      const float* src = a.low[k] + (int64_t)f * a.lframe[k] + (int64_t)c0 * lh * lw + (int64_t)l0 * lw + p0;
      for (int j = tid; j < ng * NL * pcc; j += 256) {
        const int row = j / pcc, col = j - row * pcc;  // row = g * NL + l
        const int g = row / NL, l = row - g * NL;
        if (col < NP) P[(g * lrc + l) * pcc + col] = src[((int64_t)g * lh + l) * lw + col];
      }
    }
    const CubicTap tx2 = cv_cubic_tap_s(min(x, dw - 1), a.s2x[k]);
    int col2[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) col2[j] = clampc(tx2.s - 1 + j, 0, rw - 1) - qx0;
    __syncthreads();
#pragma unroll
    for (int g = 0; g < kFusedG; ++g) {  // unrolled: sum[g] stays in registers
      if (g >= ng) break;
      const int c = c0 + g;
      const bool paf = c < npaf;
      const int cn = paf ? npaf : nheat, ce = paf ? c : c - npaf;
      if (fits) {
        // a. H1[l][i]: low-res row l0 + l, crop column qx0 + i (resize_cubic_f32_up's horizontal sum);
        //    work items of 4 rows x 1 column (16 independent LDS reads each)
        const float* pg = P + g * lrc * pcc;
        const int NLB = (NL + 3) >> 2;
        for (int j = tid; j < NX * NLB; j += 256) {
          const int lb = j / NX, i = j - lb * NX;
          const CubicTap t = t1x[i];
          int cc[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) cc[e] = clampc(t.s - 1 + e, 0, lw - 1) - p0;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int l = min(4 * lb + q, NL - 1);  // past the last row: recompute it (same value)
            const float* row = pg + l * pcc;
            float h = __fmul_rn(row[cc[0]], t.c[0]);
            h = __fadd_rn(h, __fmul_rn(row[cc[1]], t.c[1]));
            h = __fadd_rn(h, __fmul_rn(row[cc[2]], t.c[2]));
            h = __fadd_rn(h, __fmul_rn(row[cc[3]], t.c[3]));
            H1[l * rxc + i] = h;
          }
        }
        __syncthreads();
        // b. I[r][i]: the first resize's output at (qy0 + r, qx0 + i), its vertical order over pw x cn;
        //    work items of 4 rows x 1 column
        const int simd1 = a.pw[k] * cn / 4 * 4;
        const int NYB = (NY + 3) >> 2;
        for (int j = tid; j < NX * NYB; j += 256) {
          const int rb = j / NX, i = j - rb * NX;
          const bool simd = (qx0 + i) * cn + ce < simd1;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int r = min(4 * rb + q, NY - 1);
            const CubicTap t = t1y[r];
            const float h0 = H1[(clampc(t.s - 1, 0, lh - 1) - l0) * rxc + i];
            const float h1 = H1[(clampc(t.s, 0, lh - 1) - l0) * rxc + i];
            const float h2 = H1[(clampc(t.s + 1, 0, lh - 1) - l0) * rxc + i];
            const float h3 = H1[(clampc(t.s + 2, 0, lh - 1) - l0) * rxc + i];
            float v;
            if (simd) {
              const float t3 = __fmul_rn(h3, t.c[3]);
              const float t2 = __fadd_rn(__fmul_rn(h2, t.c[2]), t3);
              const float t1 = __fadd_rn(__fmul_rn(h1, t.c[1]), t2);
              v = __fadd_rn(__fmul_rn(h0, t.c[0]), t1);
            } else {
              v = __fadd_rn(__fadd_rn(__fadd_rn(__fmul_rn(h0, t.c[0]), __fmul_rn(h1, t.c[1])), __fmul_rn(h2, t.c[2])),
                            __fmul_rn(h3, t.c[3]));
            }
            I[r * rxc + i] = v;
          }
        }
        __syncthreads();
      }
      // c + d: this thread's output column (no barrier: H2's column is the thread's own)
      if (x < dw) {
        if (!fits) {
#pragma unroll
          for (int yy = 0; yy < kFusedTY; ++yy) sum[g][yy] = __builtin_nanf("");
          continue;
        }
#pragma unroll 4
        for (int r = 0; r < NY; ++r) {
          const float* row = I + r * rxc;
          float h = __fmul_rn(row[col2[0]], tx2.c[0]);
          h = __fadd_rn(h, __fmul_rn(row[col2[1]], tx2.c[1]));
          h = __fadd_rn(h, __fmul_rn(row[col2[2]], tx2.c[2]));
          h = __fadd_rn(h, __fmul_rn(row[col2[3]], tx2.c[3]));
          H2[r * kFusedTX + tid] = h;
        }
        const bool simd2 = x * cn + ce < dw * cn / 4 * 4;
#pragma unroll
        for (int yy = 0; yy < kFusedTY; ++yy) {
          const CubicTap ty = t2y[yy];
          int rr[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) rr[j] = clampc(ty.s - 1 + j, 0, rh - 1) - qy0;
          const float h0 = H2[rr[0] * kFusedTX + tid], h1 = H2[rr[1] * kFusedTX + tid];
          const float h2 = H2[rr[2] * kFusedTX + tid], h3 = H2[rr[3] * kFusedTX + tid];
          float v;
          if (simd2) {
            const float t3 = __fmul_rn(h3, ty.c[3]);
            const float t2 = __fadd_rn(__fmul_rn(h2, ty.c[2]), t3);
            const float t1 = __fadd_rn(__fmul_rn(h1, ty.c[1]), t2);
            v = __fadd_rn(__fmul_rn(h0, ty.c[0]), t1);
          } else {
            v = __fadd_rn(__fadd_rn(__fadd_rn(__fmul_rn(h0, ty.c[0]), __fmul_rn(h1, ty.c[1])), __fmul_rn(h2, ty.c[2])),
                          __fmul_rn(h3, ty.c[3]));
          }
          sum[g][yy] = k == 0 ? v : __fadd_rn(sum[g][yy], v);
        }
      }
    }
  }
  if (x < dw) {
    const int64_t plane = (int64_t)dh * dw;
#pragma unroll
    for (int g = 0; g < kFusedG; ++g) {
      if (g >= ng) break;
      float* o = dst + ((int64_t)f * nch + c0 + g) * plane + (int64_t)y0 * dw + x;
#pragma unroll
      for (int yy = 0; yy < kFusedTY; ++yy)
        if (y0 + yy < dh) o[(int64_t)yy * dw] = __fdiv_rn(sum[g][yy], (float)a.ns);
    }
  }
}

// LDS bytes of resize_cubic_fused_mean<TY> for these scales (and their extents into a), 0 when
// over its budget.  Extents: T consecutive outputs read source taps floor((x + 0.5) s - 0.5) - 1 ..
// + 2, at most floor((T - 1) s) + 1 + 4 distinct indices (+1 for the f32 rounding of the coordinate).
static size_t fused_lds(CubicFusedArgs& a, int ty) {
  int rx = 0, ry = 0, lr = 0, pc = 0;
  for (int k = 0; k < a.ns; ++k) {
    const int nx = std::min((int)std::floor((kFusedTX - 1) * a.s2x[k]) + 7, a.rw[k]);
    const int ny = std::min((int)std::floor((ty - 1) * a.s2y[k]) + 7, a.rh[k]);
    rx = std::max(rx, nx);
    ry = std::max(ry, ny);
    lr = std::max(lr, std::min((int)std::floor((ny - 1) * a.s1y[k]) + 7, a.lh[k]));
    pc = std::max(pc, std::min((int)std::floor((nx - 1) * a.s1x[k]) + 7, a.lw[k]));
  }
  a.rx_cap = rx;
  a.ry_cap = ry;
  a.lr_cap = lr;
  a.pc_cap = pc;
  const size_t lds = (size_t)(rx + ry + ty) * sizeof(CubicTap) +
                     4 * ((size_t)kFusedG * lr * pc + (size_t)lr * rx + (size_t)ry * rx + (size_t)ry * kFusedTX);
  return lds <= 96 * 1024 ? lds : 0;
}

size_t cubic_fused_lds(CubicFusedArgs& a) {
  const size_t l = fused_lds(a, 16);
  return l ? l : fused_lds(a, 8);
}

int launch_resize_cubic_fused_mean(CubicFusedArgs a, float* dst, int32_t n, int32_t dh, int32_t dw, int32_t npaf,
                                   int32_t nheat, hipStream_t st, bool* taken) {
  *taken = false;
  if (a.ns < 1 || a.ns > OP_MAX_SCALES) {
    set_error("resize_cubic_fused_mean: 1..OP_MAX_SCALES scales");
    return OP_ERR_INVALID;
  }
  int ty = 16;
  size_t lds = fused_lds(a, 16);
  if (!lds) {
    ty = 8;
    lds = fused_lds(a, 8);
  }
  if (!lds) return OP_OK;
  static bool attr = false;
  if (!attr) {
    OP_HIP_CHECK(hipFuncSetAttribute((const void*)resize_cubic_fused_mean<16>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024));
    OP_HIP_CHECK(hipFuncSetAttribute((const void*)resize_cubic_fused_mean<8>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024));
    attr = true;
  }
  const int ngroups = (npaf + nheat + kFusedG - 1) / kFusedG;
  const dim3 grid((unsigned)((dw + kFusedTX - 1) / kFusedTX), (unsigned)((dh + ty - 1) / ty), (unsigned)(n * ngroups));
  if (ty == 16)
    hipLaunchKernelGGL(resize_cubic_fused_mean<16>, grid, dim3(256), lds, st, a, dst, dh, dw, npaf, nheat);
  else
    hipLaunchKernelGGL(resize_cubic_fused_mean<8>, grid, dim3(256), lds, st, a, dst, dh, dw, npaf, nheat);
  OP_AFTER_LAUNCH("resize_cubic_fused_mean", st);
  OP_HIP_CHECK(hipGetLastError());
  *taken = true;
  return OP_OK;
}

// Generic cv2.resize(INTER_CUBIC) of a cn-channel uint8 image (row stride sstride bytes) to a
// contiguous dh x dw x cn image (the stage-level ABI op_resize_cubic).
__global__ __launch_bounds__(256) void resize_cubic_u8(const uint8_t* __restrict__ src, int64_t sstride, int sh, int sw,
                                                       int cn, uint8_t* __restrict__ dst, int dh, int dw) {
  const int64_t total = (int64_t)cn * dh * dw;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int c = (int)(i % cn);
  const int x = (int)((i / cn) % dw);
  const int y = (int)(i / ((int64_t)cn * dw));
  const CubicTap tx = cv_cubic_tap(x, dw, sw);
  const CubicTap ty = cv_cubic_tap(y, dh, sh);
  dst[i] = (uint8_t)cv_cubic_u8(src, sstride, sh, sw, cn, c, tx, ty, x * cn + c, dw * cn / 8 * 8);
}

int launch_resize_cubic_u8(const uint8_t* src, int64_t sstride, int32_t sh, int32_t sw, int32_t cn, uint8_t* dst,
                           int32_t dh, int32_t dw, hipStream_t st) {
  const int64_t total = (int64_t)cn * dh * dw;
  hipLaunchKernelGGL(resize_cubic_u8, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, src, sstride, sh, sw, cn,
                     dst, dh, dw);
  OP_AFTER_LAUNCH("resize_cubic_u8", st);
  OP_HIP_CHECK(hipGetLastError());
  return OP_OK;
}

}  // namespace op
