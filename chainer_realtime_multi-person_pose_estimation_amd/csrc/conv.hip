// CocoPoseNet forward kernels for gfx950 (models/CocoPoseNet.py:132-262).
//
// Direct convolution as an implicit GEMM on the f32-input matrix cores
// (v_mfma_f32_32x32x2_f32: exact f32 products, f32 accumulate — Chainer's fp32 semantics,
// no reduced-precision shortcut).  Activations live in HBM as NHWC with a zero halo of `pad`
// pixels, so every tap of a 3x3 / 7x7 window is a wave-uniform offset from a per-lane base
// pointer: no im2col buffer, no per-tap bounds checks.
//
// MFMA mapping (per wave): A = weights (32 output channels x 2 k), B = activations (2 k x 32 pixels).
// One 16-byte load per lane carries 4 consecutive input channels, feeding 4 MFMAs:
//   lanes 0-31 hold channels c..c+3 of pixel (lane), lanes 32-63 channels c+4..c+7 of the same pixel;
//   MFMA j contracts the k-pair {c+j, c+4+j}.  Weights are packed [c8][tap][co][8] so the A operand
//   has the identical k order and a wave's weight load is one contiguous 1 KiB line.
// A wave owns CB x PB blocks of 32 channels x 32 pixels; the 4 waves of a workgroup share the
// channel block (weights hit L1) and take consecutive pixel blocks.  Operand loads run two
// (tap, channel-chunk) iterations ahead of the MFMAs in two named register sets.
#include "common.hpp"
#include "cvlinear.hpp"

namespace op {

template <int KS, int CB, int PB>
__global__ __launch_bounds__(256) void conv_mfma_f32(ConvShape s, ConvGroup g0, ConvGroup g1) {
  const ConvGroup g = blockIdx.z == 0 ? g0 : g1;
  constexpr int KSQ = KS * KS;
  constexpr int R = KS / 2;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int co_base = blockIdx.y * (CB * 32);
  if (co_base >= g.cop) return;
  const int hw = s.h * s.w;
  const int total = s.n * hw;
  const int px_base = (blockIdx.x * 4 + wave) * (PB * 32);
  if (px_base >= total) return;
  const int l32 = lane & 31;
  const int hi = lane >> 5;
  const int wp_in = s.w + 2 * s.pin;
  const int hp_in = s.h + 2 * s.pin;

  const float* bptr[PB];
#pragma unroll
  for (int pb = 0; pb < PB; ++pb) {
    int p = px_base + pb * 32 + l32;
    if (p >= total) p = total - 1;
    const int n = p / hw;
    const int rem = p - n * hw;
    const int y = rem / s.w;
    const int x = rem - y * s.w;
    bptr[pb] = g.in + ((int64_t)(n * hp_in + y + s.pin - R) * wp_in + (x + s.pin - R)) * s.cs_in + 4 * hi;
  }
  const float* aptr = g.w + (int64_t)(co_base + l32) * 8 + 4 * hi;
  const int64_t wstep = (int64_t)g.cop * 8;
  const int n_it = s.c8 * KSQ;

  floatx16 acc[CB][PB];
#pragma unroll
  for (int cb = 0; cb < CB; ++cb)
#pragma unroll
    for (int pb = 0; pb < PB; ++pb)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[cb][pb][r] = 0.0f;

  auto load = [&](floatx4(&a)[CB], floatx4(&b)[PB], int it) {
    if (it >= n_it) it = n_it - 1;  // tail prefetch: reload a valid address, never consumed
    const int c = it / KSQ;
    const int t = it - c * KSQ;
    const int ky = t / KS;
    const int kx = t - ky * KS;
    const int64_t ioff = ((int64_t)ky * wp_in + kx) * s.cs_in + c * 8;
    const float* ap = aptr + (int64_t)it * wstep;
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) a[cb] = *(const floatx4*)(ap + cb * 256);
#pragma unroll
    for (int pb = 0; pb < PB; ++pb) b[pb] = *(const floatx4*)(bptr[pb] + ioff);
  };
  auto mma = [&](const floatx4(&a)[CB], const floatx4(&b)[PB]) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int cb = 0; cb < CB; ++cb)
#pragma unroll
        for (int pb = 0; pb < PB; ++pb)
          acc[cb][pb] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[cb][j], b[pb][j], acc[cb][pb], 0, 0, 0);
  };

  floatx4 a0[CB], b0[PB], a1[CB], b1[PB];
  load(a0, b0, 0);
  load(a1, b1, 1);
  int it = 0;
  for (; it + 2 <= n_it; it += 2) {
    mma(a0, b0);
    load(a0, b0, it + 2);
    mma(a1, b1);
    load(a1, b1, it + 3);
  }
  if (it < n_it) mma(a0, b0);

  // Epilogue: lane holds pixel (l32) and, per register group q, 4 consecutive output channels
  // 8q + 4hi .. +3 of each 32-channel block (C/D map: row = (r&3) + 8(r>>2) + 4(lane>>5)).
  const int wp_out = s.w + 2 * s.pout;
  const int hp_out = s.h + 2 * s.pout;
#pragma unroll
  for (int pb = 0; pb < PB; ++pb) {
    const int p = px_base + pb * 32 + l32;
    if (p >= total) continue;
    const int n = p / hw;
    const int rem = p - n * hw;
    const int y = rem / s.w;
    const int x = rem - y * s.w;
    float* optr = g.out + ((int64_t)(n * hp_out + y + s.pout) * wp_out + (x + s.pout)) * s.cs_out;
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int co = co_base + cb * 32 + 8 * q + 4 * hi;
        if (co >= g.cout_store) continue;
        const floatx4 bv = *(const floatx4*)(g.bias + co);
        floatx4 v;
        v[0] = acc[cb][pb][4 * q + 0] + bv[0];
        v[1] = acc[cb][pb][4 * q + 1] + bv[1];
        v[2] = acc[cb][pb][4 * q + 2] + bv[2];
        v[3] = acc[cb][pb][4 * q + 3] + bv[3];
        if (s.relu) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = v[e] > 0.0f ? v[e] : 0.0f;
        }
        *(floatx4*)(optr + co) = v;
      }
    }
  }
}

template <int KS, int CB, int PB>
static int launch_conv_t(const ConvShape& s, const ConvGroup* g, hipStream_t st) {
  const int64_t total = (int64_t)s.n * s.h * s.w;
  const int cop_max = s.groups > 1 ? (g[0].cop > g[1].cop ? g[0].cop : g[1].cop) : g[0].cop;
  dim3 grid((unsigned)((total + 4 * PB * 32 - 1) / (4 * PB * 32)), (unsigned)((cop_max + CB * 32 - 1) / (CB * 32)),
            (unsigned)s.groups);
  hipLaunchKernelGGL((conv_mfma_f32<KS, CB, PB>), grid, dim3(256), 0, st, s, g[0], s.groups > 1 ? g[1] : g[0]);
  OP_AFTER_LAUNCH("conv_mfma_f32<KS", st);
  OP_HIP_CHECK(hipGetLastError());
  return OP_OK;
}

int launch_conv(const ConvShape& s, const ConvGroup* g, hipStream_t st) {
  // Host-side shape checks: the kernel assumes these (no bounds checks inside).
  if (s.c8 <= 0 || (s.ks != 1 && s.ks != 3 && s.ks != 7) || s.pin < s.ks / 2 || s.cs_in % 4 || s.cs_out % 4) {
    set_error("launch_conv: unsupported shape");
    return OP_ERR_INVALID;
  }
  for (int i = 0; i < s.groups; ++i) {
    if (g[i].cop % 64 || g[i].cout_store % 4 || g[i].cout_store > g[i].cop) {
      set_error("launch_conv: channel padding");
      return OP_ERR_INVALID;
    }
  }
  int taken = 0;
  const int rc = launch_conv_f32_lds(s, g, st, &taken);  // 3x3 / 7x7: the LDS-halo form (conv_f32.hip)
  if (rc != OP_OK || taken) return rc;
  switch (s.ks) {
    case 1: return launch_conv_t<1, 2, 2>(s, g, st);
    case 3: return launch_conv_t<3, 2, 2>(s, g, st);
    default: return launch_conv_t<7, 2, 2>(s, g, st);
  }
}

// A branch's two closing 1x1 convs in one launch, exact f32 (conv5_4 + conv5_5, CocoPoseNet.py:
// 162-165; Mconv6 + Mconv7, :181-184 and the later stages): in -> a (bias, ReLU) -> b (bias) -> out,
// the intermediate kept in registers.  A wave owns 32 pixels; layer a runs in groups of 128 channels
// (4 blocks of 32, K = the input channels), and each group's ReLU'd accumulators feed layer b's
// K loop directly as B operands: the D layout of v_mfma_f32_32x32x2_f32 gives lane (pixel, hi)
// channels (r&3) + 8(r>>2) + 4hi of a block in register r, i.e. for chunk c8 = 4 block + (r>>2)
// and MFMA j = r&3 the k-pair {8c8 + j, 8c8 + 4 + j} that conv_mfma_f32 contracts with the same
// packed weights [c8][co][8].  Both layers therefore accumulate in conv_mfma_f32's order and the
// output is bit-identical to the two-launch path, without the intermediate's HBM round trip
// (stage 1: 512 channels per pixel).
template <int CB2>
__global__ __launch_bounds__(256) void conv_head_f32(HeadF32Shape s, HeadF32Group g0, HeadF32Group g1) {
  const HeadF32Group g = blockIdx.z == 0 ? g0 : g1;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int hw = s.h * s.w;
  const int total = s.n * hw;
  const int px_base = (blockIdx.x * 4 + wave) * 32;
  if (px_base >= total) return;
  const int l32 = lane & 31, hi = lane >> 5;
  const int wp_in = s.w + 2 * s.pin, hp_in = s.h + 2 * s.pin;
  const float* bptr;
  {
    int p = px_base + l32;
    if (p >= total) p = total - 1;
    const int n = p / hw, rem = p - n * hw;
    const int y = rem / s.w, x = rem - y * s.w;
    bptr = g.in + ((int64_t)(n * hp_in + y + s.pin) * wp_in + (x + s.pin)) * s.cs_in + 4 * hi;
  }
  const int64_t wstep1 = (int64_t)g.cop1 * 8, wstep2 = (int64_t)g.cop2 * 8;

  floatx16 accb[CB2];
#pragma unroll
  for (int cb = 0; cb < CB2; ++cb)
#pragma unroll
    for (int r = 0; r < 16; ++r) accb[cb][r] = 0.0f;

  for (int grp = 0; grp < s.co1 / 128; ++grp) {
    floatx16 acca[4];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
      for (int r = 0; r < 16; ++r) acca[cb][r] = 0.0f;
    const float* aptr = g.w1 + (int64_t)(grp * 128 + l32) * 8 + 4 * hi;
    auto load = [&](floatx4(&a)[4], floatx4& b, int c) {
      if (c >= s.c8) c = s.c8 - 1;  // tail prefetch: a valid address, never consumed
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) a[cb] = *(const floatx4*)(aptr + c * wstep1 + cb * 256);
      b = *(const floatx4*)(bptr + c * 8);
    };
    auto mma = [&](const floatx4(&a)[4], const floatx4& b) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) acca[cb] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[cb][j], b[j], acca[cb], 0, 0, 0);
    };
    floatx4 a0[4], a1[4], b0, b1;
    load(a0, b0, 0);
    load(a1, b1, 1);
    int c = 0;
    for (; c + 2 <= s.c8; c += 2) {
      mma(a0, b0);
      load(a0, b0, c + 2);
      mma(a1, b1);
      load(a1, b1, c + 3);
    }
    if (c < s.c8) mma(a0, b0);
    // layer a's bias + ReLU, in place
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const floatx4 bv = *(const floatx4*)(g.b1 + grp * 128 + cb * 32 + 8 * q + 4 * hi);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float v = acca[cb][4 * q + e] + bv[e];
          acca[cb][4 * q + e] = v > 0.0f ? v : 0.0f;
        }
      }
    // layer b over this group's 128 channels: chunk c8 = 16 grp + 4 cb + q
    const float* a2ptr = g.w2 + (int64_t)l32 * 8 + 4 * hi;
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int c8 = 16 * grp + 4 * cb + q;
        floatx4 a2[CB2];
#pragma unroll
        for (int cb2 = 0; cb2 < CB2; ++cb2) a2[cb2] = *(const floatx4*)(a2ptr + c8 * wstep2 + cb2 * 256);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int cb2 = 0; cb2 < CB2; ++cb2)
            accb[cb2] = __builtin_amdgcn_mfma_f32_32x32x2f32(a2[cb2][j], acca[cb][4 * q + j], accb[cb2], 0, 0, 0);
      }
  }

  // epilogue (conv_mfma_f32's): layer b's bias, no ReLU
  const int p = px_base + l32;
  if (p >= total) return;
  const int wp_out = s.w + 2 * s.pout, hp_out = s.h + 2 * s.pout;
  const int n = p / hw, rem = p - n * hw;
  const int y = rem / s.w, x = rem - y * s.w;
  float* optr = g.out + ((int64_t)(n * hp_out + y + s.pout) * wp_out + (x + s.pout)) * s.cs_out;
#pragma unroll
  for (int cb = 0; cb < CB2; ++cb)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int co = cb * 32 + 8 * q + 4 * hi;
      if (co >= g.cout_store) continue;
      const floatx4 bv = *(const floatx4*)(g.b2 + co);
      floatx4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = accb[cb][4 * q + e] + bv[e];
      *(floatx4*)(optr + co) = v;
    }
}

int launch_conv_head_f32(const HeadF32Shape& s, const HeadF32Group* g, hipStream_t st) {
  // the kernel's assumptions (no bounds checks inside)
  if (s.c8 <= 0 || s.co1 <= 0 || s.co1 % 128 || s.cs_in % 4 || s.cs_out % 4 || s.groups < 1 || s.groups > 2) {
    set_error("launch_conv_head_f32: unsupported shape");
    return OP_ERR_INVALID;
  }
  const int cop2 = g[0].cop2;
  for (int i = 0; i < s.groups; ++i) {
    if (g[i].cop1 < s.co1 || g[i].cop1 % 64 || g[i].cop2 != cop2 || (cop2 != 32 && cop2 != 64) ||
        g[i].cout_store % 4 || g[i].cout_store > cop2) {
      set_error("launch_conv_head_f32: channel padding");
      return OP_ERR_INVALID;
    }
  }
  const int64_t total = (int64_t)s.n * s.h * s.w;
  const dim3 grid((unsigned)((total + 127) / 128), 1, (unsigned)s.groups);
  const HeadF32Group& g1 = s.groups > 1 ? g[1] : g[0];
  if (cop2 == 64) hipLaunchKernelGGL((conv_head_f32<2>), grid, dim3(256), 0, st, s, g[0], g1);
  else hipLaunchKernelGGL((conv_head_f32<1>), grid, dim3(256), 0, st, s, g[0], g1);
  OP_AFTER_LAUNCH("conv_head_f32", st);
  OP_HIP_CHECK(hipGetLastError());
  return OP_OK;
}

// F.max_pooling_2d(h, ksize=2, stride=2) (CocoPoseNet.py:138,141,146); sizes are even here
// (multiples of 8, pose_detector.py:57-73), so cover_all adds no extra window.
__global__ __launch_bounds__(256) void maxpool2_nhwc(const float* __restrict__ in, int pin, float* __restrict__ out,
                                                     int pout, int n, int h, int w, int c4) {
  const int oh = h / 2, ow = w / 2;
  const int64_t total = (int64_t)n * oh * ow * c4;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int cc = (int)(i % c4);
  int64_t p = i / c4;
  const int ox = (int)(p % ow);
  p /= ow;
  const int oy = (int)(p % oh);
  const int nn = (int)(p / oh);
  const int wpi = w + 2 * pin, hpi = h + 2 * pin;
  const int C = c4 * 4;
  const float* b = in + ((int64_t)(nn * hpi + 2 * oy + pin) * wpi + (2 * ox + pin)) * C + cc * 4;
  floatx4 v0 = *(const floatx4*)b;
  floatx4 v1 = *(const floatx4*)(b + C);
  floatx4 v2 = *(const floatx4*)(b + (int64_t)wpi * C);
  floatx4 v3 = *(const floatx4*)(b + (int64_t)wpi * C + C);
  floatx4 r;
#pragma unroll
  for (int e = 0; e < 4; ++e) r[e] = fmaxf(fmaxf(v0[e], v1[e]), fmaxf(v2[e], v3[e]));
  const int wpo = ow + 2 * pout, hpo = oh + 2 * pout;
  *(floatx4*)(out + ((int64_t)(nn * hpo + oy + pout) * wpo + (ox + pout)) * C + cc * 4) = r;
}

int launch_maxpool2(const float* in, int32_t pin, float* out, int32_t pout, int32_t n, int32_t h, int32_t w,
                    int32_t c, hipStream_t st) {
  if ((h & 1) || (w & 1) || (c & 3)) {
    set_error("maxpool2: odd size");
    return OP_ERR_INVALID;
  }
  const int64_t total = (int64_t)n * (h / 2) * (w / 2) * (c / 4);
  hipLaunchKernelGGL(maxpool2_nhwc, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, in, pin, out, pout, n,
                     h, w, c / 4);
  OP_AFTER_LAUNCH("maxpool2_nhwc", st);
  OP_HIP_CHECK(hipGetLastError());
  return OP_OK;
}

// (n,3,h,w) f32 -> padded (n, h+2, w+2, 8) NHWC, zero halo and zero channels 3..7.
__global__ __launch_bounds__(256) void nchw_to_nhwc8(const float* __restrict__ x, float* __restrict__ out, int n, int h,
                                                     int w) {
  const int wp = w + 2, hp = h + 2;
  const int64_t total = (int64_t)n * hp * wp;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int px = (int)(i % wp);
  const int py = (int)((i / wp) % hp);
  const int nn = (int)(i / ((int64_t)wp * hp));
  floatx4 lo = {0.f, 0.f, 0.f, 0.f}, hi4 = {0.f, 0.f, 0.f, 0.f};
  const int y = py - 1, xx = px - 1;
  if (y >= 0 && y < h && xx >= 0 && xx < w) {
    const int64_t plane = (int64_t)h * w;
    const float* b = x + (int64_t)nn * 3 * plane + (int64_t)y * w + xx;
    lo[0] = b[0];
    lo[1] = b[plane];
    lo[2] = b[2 * plane];
  }
  *(floatx4*)(out + i * 8) = lo;
  *(floatx4*)(out + i * 8 + 4) = hi4;
}

int launch_nchw_to_nhwc8(const float* x, float* out, int32_t n, int32_t h, int32_t w, hipStream_t st) {
  const int64_t total = (int64_t)n * (h + 2) * (w + 2);
  hipLaunchKernelGGL(nchw_to_nhwc8, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, x, out, n, h, w);
  OP_AFTER_LAUNCH("nchw_to_nhwc8", st);
  OP_HIP_CHECK(hipGetLastError());
  return OP_OK;
}

// Stage-6 maps out of the stage-input buffer -> planar (n,38,h,w) and (n,19,h,w).
__global__ __launch_bounds__(256) void extract_maps(const float* __restrict__ cat, int n, int h, int w,
                                                    float* __restrict__ paf, float* __restrict__ heat) {
  const int64_t total = (int64_t)n * 57 * h * w;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int x = (int)(i % w);
  const int y = (int)((i / w) % h);
  const int c = (int)((i / ((int64_t)w * h)) % 57);
  const int nn = (int)(i / ((int64_t)w * h * 57));
  const int wp = w + 2 * kStagePad, hp = h + 2 * kStagePad;
  const float* px = cat + ((int64_t)(nn * hp + y + kStagePad) * wp + (x + kStagePad)) * kCatStride;
  if (c < 38)
    paf[(((int64_t)nn * 38 + c) * h + y) * w + x] = px[kCatPaf + c];
  else
    heat[(((int64_t)nn * 19 + (c - 38)) * h + y) * w + x] = px[kCatHeat + c - 38];
}

int launch_extract_maps(const float* cat, int32_t n, int32_t h, int32_t w, float* paf, float* heat, hipStream_t st) {
  const int64_t total = (int64_t)n * 57 * h * w;
  hipLaunchKernelGGL(extract_maps, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, cat, n, h, w, paf, heat);
  OP_AFTER_LAUNCH("extract_maps", st);
  OP_HIP_CHECK(hipGetLastError());
  return OP_OK;
}

// frames (n, sh, sw, 3) u8 -> padded (n, dh+2, dw+2, 8) NHWC f32 network input (zero halo).
__global__ __launch_bounds__(256) void preprocess_nhwc8(const uint8_t* __restrict__ frames, int64_t frame_bytes,
                                                        int64_t row_stride, int n, int sh, int sw, int dh, int dw,
                                                        float* __restrict__ out) {
  const int wp = dw + 2, hp = dh + 2;
  const int64_t total = (int64_t)n * hp * wp;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int px = (int)(i % wp);
  const int py = (int)((i / wp) % hp);
  const int nn = (int)(i / ((int64_t)wp * hp));
  floatx4 lo = {0.f, 0.f, 0.f, 0.f}, z = {0.f, 0.f, 0.f, 0.f};
  const int dy = py - 1, dx = px - 1;
  if (dy >= 0 && dy < dh && dx >= 0 && dx < dw) {
    const LinTap tx = cv_linear_tap(dx, dw, sw, true);
    const LinTap ty = cv_linear_tap(dy, dh, sh, false);
    const uint8_t* src = frames + (int64_t)nn * frame_bytes;
    lo[0] = cv_linear_px(src, row_stride, sh, sw, tx, ty, 0);
    lo[1] = cv_linear_px(src, row_stride, sh, sw, tx, ty, 1);
    lo[2] = cv_linear_px(src, row_stride, sh, sw, tx, ty, 2);
  }
  *(floatx4*)(out + i * 8) = lo;
  *(floatx4*)(out + i * 8 + 4) = z;
}

int launch_preprocess(const uint8_t* frames, int64_t frame_bytes, int64_t row_stride, int32_t n, int32_t sh,
                      int32_t sw, int32_t dh, int32_t dw, float* out, hipStream_t st) {
  const int64_t total = (int64_t)n * (dh + 2) * (dw + 2);
  hipLaunchKernelGGL(preprocess_nhwc8, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, frames, frame_bytes,
                     row_stride, n, sh, sw, dh, dw, out);
  OP_AFTER_LAUNCH("preprocess_nhwc8", st);
  OP_HIP_CHECK(hipGetLastError());
  return OP_OK;
}

// One frame -> planar (1, 3, dh, dw) (the reference's x_data, for the stage-level ABI).
__global__ __launch_bounds__(256) void preprocess_planar(const uint8_t* __restrict__ bgr, int64_t row_stride, int sh,
                                                         int sw, int dh, int dw, float* __restrict__ out) {
  const int64_t total = (int64_t)dh * dw;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int dx = (int)(i % dw), dy = (int)(i / dw);
  const LinTap tx = cv_linear_tap(dx, dw, sw, true);
  const LinTap ty = cv_linear_tap(dy, dh, sh, false);
  for (int c = 0; c < 3; ++c) out[c * total + i] = cv_linear_px(bgr, row_stride, sh, sw, tx, ty, c);
}

int launch_preprocess_planar(const uint8_t* bgr, int64_t row_stride, int32_t sh, int32_t sw, int32_t dh, int32_t dw,
                             float* out_nchw, hipStream_t st) {
  const int64_t total = (int64_t)dh * dw;
  hipLaunchKernelGGL(preprocess_planar, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, bgr, row_stride, sh,
                     sw, dh, dw, out_nchw);
  OP_AFTER_LAUNCH("preprocess_planar", st);
  OP_HIP_CHECK(hipGetLastError());
  return OP_OK;
}

}  // namespace op
