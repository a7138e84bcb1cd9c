// conv1_1 (CocoPoseNet.py:136: 3 -> 64 channels, 3x3, ReLU) on the split path as f32 FMAs
// (K = 27 is far too small for the matrix cores: 16-channel padding made the MFMA version do 5x
// the work at 27 TF/s).  FROM_FRAMES fuses the network-input kernel: each 16x16 output tile
// resamples its 18x18 input window straight from the uint8 frame (cv2 LINEAR + x/255 - 0.5,
// pose_detector.py:493-494, 426-431) into LDS, so the padded network input never touches HBM.
// Both variants see the same input values -- the split format's hi + lo of x -- so the staged
// path and op_forward produce identical conv1_1 outputs.
#include "common.hpp"
#include "cvlinear.hpp"

namespace op {

typedef unsigned short u16x4c __attribute__((ext_vector_type(4)));

// (Reading bf16 lanes as __builtin_bit_cast(__bf16, u16-vector element) was miscompiled for this
// kernel: channel 1 came back as channel 0.  The input is decoded from 32-bit words instead.)

__device__ __forceinline__ float split_recon(float v) {
  const __bf16 h = (__bf16)v;
  return (float)h + (float)(__bf16)(v - (float)h);
}

template <bool FROM_FRAMES>
__global__ __launch_bounds__(256) void conv11_split(const uint8_t* __restrict__ frames, int64_t frame_bytes,
                                                    int64_t row_stride, int sh, int sw, const char* __restrict__ x0,
                                                    int h, int w, const float* __restrict__ wt,
                                                    const float* __restrict__ bias, char* __restrict__ out) {
  __shared__ float tile[18][18][4];
  const int n = blockIdx.z;
  const int x0t = blockIdx.x * 16, y0t = blockIdx.y * 16;
  const int tid = threadIdx.x;

  for (int i = tid; i < 18 * 18; i += 256) {
    const int iy = i / 18, ix = i - (i / 18) * 18;
    const int gy = y0t - 1 + iy, gx = x0t - 1 + ix;
    float v[3] = {0.f, 0.f, 0.f};
    if (gy >= 0 && gy < h && gx >= 0 && gx < w) {
      if constexpr (FROM_FRAMES) {
        const uint8_t* src = frames + (int64_t)n * frame_bytes;
        const LinTap tx = cv_linear_tap(gx, w, sw, true);
        const LinTap ty = cv_linear_tap(gy, h, sh, false);
#pragma unroll
        for (int c = 0; c < 3; ++c) v[c] = split_recon(cv_linear_px(src, row_stride, sh, sw, tx, ty, c));
      } else {  // padded split16 input (h+2, w+2, 16): channels 0..7 hi at +0, lo at +16
        const char* p = x0 + (((int64_t)n * (h + 2) + gy + 1) * (w + 2) + gx + 1) * 64;
        const uint2 hv = *(const uint2*)p, lv = *(const uint2*)(p + 16);  // bf16 pairs (c0|c1<<16, c2|c3<<16)
        v[0] = __fadd_rn(__uint_as_float(hv.x << 16), __uint_as_float(lv.x << 16));
        v[1] = __fadd_rn(__uint_as_float(hv.x & 0xffff0000u), __uint_as_float(lv.x & 0xffff0000u));
        v[2] = __fadd_rn(__uint_as_float(hv.y << 16), __uint_as_float(lv.y << 16));
      }
    }
    tile[iy][ix][0] = v[0];
    tile[iy][ix][1] = v[1];
    tile[iy][ix][2] = v[2];
  }
  __syncthreads();
  const int tx = tid & 15, ty = tid >> 4;
  const int x = x0t + tx, y = y0t + ty;
  float acc[64];
#pragma unroll
  for (int co = 0; co < 64; ++co) acc[co] = 0.0f;
#pragma unroll
  for (int t = 0; t < 9; ++t) {
#pragma unroll
    for (int ci = 0; ci < 3; ++ci) {
      const float v = tile[ty + t / 3][tx + t % 3][ci];
#pragma unroll
      for (int co = 0; co < 64; ++co) acc[co] = __fmaf_rn(v, wt[(t * 3 + ci) * 64 + co], acc[co]);  // SGPR operand
    }
  }
  if (x >= w || y >= h) return;
  char* o = out + (((int64_t)n * (h + 2) + y + 1) * (w + 2) + x + 1) * 256;
#pragma unroll
  for (int gq = 0; gq < 8; ++gq) {
    u16x4c h0, h1, l0, l1;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float f = __fadd_rn(acc[gq * 8 + e], bias[gq * 8 + e]);
      f = f > 0.0f ? f : 0.0f;
      const __bf16 hh = (__bf16)f;
      const __bf16 ll = (__bf16)(f - (float)hh);
      if (e < 4) {
        h0[e] = __builtin_bit_cast(unsigned short, hh);
        l0[e] = __builtin_bit_cast(unsigned short, ll);
      } else {
        h1[e - 4] = __builtin_bit_cast(unsigned short, hh);
        l1[e - 4] = __builtin_bit_cast(unsigned short, ll);
      }
    }
    *(u16x4c*)(o + gq * 32) = h0;
    *(u16x4c*)(o + gq * 32 + 8) = h1;
    *(u16x4c*)(o + gq * 32 + 16) = l0;
    *(u16x4c*)(o + gq * 32 + 24) = l1;
  }
}

// frames != nullptr: fused from the uint8 frames (sh x sw, resized to h x w); else from the
// padded split16 input x0.  wt: conv1_1 as [tap][ci][co] f32; out: C11 (h+2, w+2, 64).
int launch_conv11_split(const uint8_t* frames, int64_t frame_bytes, int64_t row_stride, int32_t sh, int32_t sw,
                        const float* x0, int32_t n, int32_t h, int32_t w, const float* wt, const float* bias,
                        float* out, hipStream_t st) {
  const dim3 grid((unsigned)((w + 15) / 16), (unsigned)((h + 15) / 16), (unsigned)n);
  if (frames)
    hipLaunchKernelGGL(conv11_split<true>, grid, dim3(256), 0, st, frames, frame_bytes, row_stride, sh, sw, nullptr, h,
                       w, wt, bias, (char*)out);
  else
    hipLaunchKernelGGL(conv11_split<false>, grid, dim3(256), 0, st, nullptr, 0, 0, 0, 0, (const char*)x0, h, w, wt,
                       bias, (char*)out);
  OP_AFTER_LAUNCH("conv11_split", st);
  OP_HIP_CHECK(hipGetLastError());
  return OP_OK;
}

}  // namespace op
