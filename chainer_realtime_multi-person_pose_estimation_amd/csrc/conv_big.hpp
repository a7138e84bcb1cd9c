// Device helpers and tiling record shared by the halo-tiled conv kernels (conv_big.hip) and the
// 7x7 raster-tile kernel (conv_m16.hip, its own translation unit so it can take its own LLVM
// scheduler flags: Makefile FLAGS_conv_m16).
#pragma once
#include "common.hpp"

namespace op {

typedef __bf16 bf16x8g __attribute__((ext_vector_type(8)));
typedef unsigned short u16x4g __attribute__((ext_vector_type(4)));

#define LDS_PTR_G(p) ((__attribute__((address_space(3))) void*)(p))

struct BigTiling {
  int32_t tr, tc;            // tile rows x cols
  int32_t tiles_y, tiles_x;  // tiles per frame
  int32_t pitch;             // LDS halo row pitch in 16-B slots (halo_pitch)
  int32_t hrows;             // tr + ks - 1
  int32_t nh;                // 1-KiB halo pieces per plane
  int32_t units;             // weight sets = groups x channel tiles
  int32_t co_tiles;          // channel tiles per group
  int32_t per_unit;          // workgroups per weight set (= n * tiles_y * tiles_x)
  int32_t xpu;               // XCDs per weight set (8 / units), 0 = plain block order
  int32_t pair;              // > 1 (conv_m16r): channel tiles of one group sharing an XCD set, a
                             // pixel tile's tiles dispatched back to back (xpu = 8 * pair / units)
  int32_t hw, total;         // raster tiles: pixels per frame, pixels of the batch
  int32_t fa_tiles;          // > 0 (conv_m16): raster tiles aligned to frames, fa_tiles per frame
  int32_t per_xcd;           // > 0: pixel-major XCD order (conv_m16k): XCD x runs pixel tiles
                             // [x*per_xcd, (x+1)*per_xcd) for every weight set, sets adjacent
  int32_t ksplit;            // > 1 (conv_m16): input chunks split over blockIdx.y, f32 partials in ws
  float* ws;                 // ksplit partials [split][group][pixel][cop] (conv_m16_splitk_reduce)
  const void* zeros;         // conv_m16: >= 1 KiB of device zeros (the padding tap of an odd tap count)
  int32_t halo_trim;         // conv_m16 LIN: a tile within one frame loads only its own halo rows' pieces
  int32_t pers_blocks;       // conv_m16 PERS: the launch's tile count (the grid is one workgroup per CU)
};

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N <= 63, "vmcnt literal");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Epilogue of the 16x16x32 kernels: a lane holds 4 consecutive output channels c..c+3 of one pixel
// (D rows = channels, row kg = lane / 16), so rows kg and kg ^ 1 together hold one 8-channel group
// whose split record is [hi c..c+7 (16 B)][lo c..c+7 (16 B)].  own = this lane's {hi, hi, lo, lo}
// dwords; w = the same after v_permlane16_swap (odd rows of the hi operand <-> even rows of the lo
// operand): the even row then holds the group's 16 hi bytes and the odd row its 16 lo bytes, so one
// 16-B store per lane replaces two 8-B stores.  Every lane of the wave must execute this.
__device__ __forceinline__ void split_pair_swap(const floatx4& acc, const floatx4& bv, int relu, floatx4& v,
                                                uint32_t own[4], uint32_t w[4]) {
  unsigned short hb[4], lb[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float fv = acc[e] + bv[e];
    if (relu) fv = fv > 0.0f ? fv : 0.0f;
    v[e] = fv;
    const __bf16 h16 = (__bf16)fv;
    const __bf16 l16v = (__bf16)(fv - (float)h16);
    hb[e] = __builtin_bit_cast(unsigned short, h16);
    lb[e] = __builtin_bit_cast(unsigned short, l16v);
  }
  own[0] = hb[0] | ((uint32_t)hb[1] << 16);
  own[1] = hb[2] | ((uint32_t)hb[3] << 16);
  own[2] = lb[0] | ((uint32_t)lb[1] << 16);
  own[3] = lb[2] | ((uint32_t)lb[3] << 16);
  const auto r0 = __builtin_amdgcn_permlane16_swap(own[0], own[2], false, false);
  const auto r1 = __builtin_amdgcn_permlane16_swap(own[1], own[3], false, false);
  w[0] = r0[0];
  w[1] = r1[0];
  w[2] = r0[1];
  w[3] = r1[1];
}

// Store one lane's part of an 8-channel group (see split_pair_swap): one 16-B store when the whole
// group is stored, else (a group cut by cout_store) this lane's own two 8-B pieces.  pstride = bytes
// between the pixel's consecutive 16-B pieces: 16 in the [pixel][channels] layout, the plane size in
// the chunk-planar one (SplitConvShape::out_planar).
__device__ __forceinline__ void store_split_group(char* optr, int co, int kg, int cout_store, const uint32_t own[4],
                                                  const uint32_t w[4], int64_t pstride = 16) {
  char* gp = optr + (co >> 3) * 2 * pstride;
  if ((co | 7) < cout_store) {
    *(uint4*)(gp + (kg & 1) * pstride) = make_uint4(w[0], w[1], w[2], w[3]);
  } else {
    *(uint2*)(gp + (co & 7) * 2) = make_uint2(own[0], own[1]);
    *(uint2*)(gp + pstride + (co & 7) * 2) = make_uint2(own[2], own[3]);
  }
}

// One (pixel P of the batch, 4 channels co..co+3) of a split-K conv: the tl.ksplit f32 partials
// summed in split order onto the bias, the activation, and the split hi/lo (+ dense f32) store of
// the kernels' own epilogue; conv_m16_splitk_reduce runs it per thread (a launch boundary orders it
// after the conv).  Round 5: the round-4 experiment that finished split-K inside the conv kernel
// (last arriver at an agent-scope counter; measured slower, and its hand-off had no release /
// acquire pairing -- advisor r04) is removed.
// Round 4: every partial is loaded before the first add (a predicated, fully unrolled loop over at
// most kMaxSplitK splits), so a thread waits for memory once instead of once per split (the
// launch's 8 dependent load latencies were most of a one-frame reduce's 6.4 us); the adds keep
// the split order.
constexpr int kMaxSplitK = 16;
__device__ __forceinline__ void splitk_reduce_item(const SplitConvShape& s, const SplitConvGroup& g, int grp,
                                                   const BigTiling& tl, int wsc, int64_t P, int co) {
  floatx4 part[kMaxSplitK];
#pragma unroll
  for (int sp = 0; sp < kMaxSplitK; ++sp)
    if (sp < tl.ksplit)
      part[sp] = *(const floatx4*)(tl.ws + (((int64_t)sp * s.groups + grp) * tl.total + P) * wsc + co);
  floatx4 v = *(const floatx4*)(g.bias + co);
#pragma unroll
  for (int sp = 0; sp < kMaxSplitK; ++sp)
    if (sp < tl.ksplit) {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] += part[sp][e];
    }
  const int f = (int)(P / tl.hw), pp = (int)(P - (int64_t)f * tl.hw);
  const int y = pp / s.w, x = pp - y * s.w;
  const int wp_out = s.w + 2 * s.pout, hp_out = s.h + 2 * s.pout;
  const int64_t out_pc = split_piece_stride(s.out_planar, hp_out, wp_out);
  char* d = (char*)g.out + (int64_t)f * hp_out * wp_out * s.cs_out * 4 +
            ((int64_t)(y + s.pout) * wp_out + (x + s.pout)) * split_pixel_stride(s.out_planar, s.cs_out) +
            (co >> 3) * 2 * out_pc + (co & 7) * 2;
  u16x4g vh, vl;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    if (s.relu) v[e] = v[e] > 0.0f ? v[e] : 0.0f;
    const __bf16 h16 = (__bf16)v[e];
    const __bf16 l16v = (__bf16)(v[e] - (float)h16);
    vh[e] = __builtin_bit_cast(unsigned short, h16);
    vl[e] = __builtin_bit_cast(unsigned short, l16v);
  }
  *(u16x4g*)d = vh;
  *(u16x4g*)(d + out_pc) = vl;
  if (g.out32) *(floatx4*)(g.out32 + ((int64_t)(f * s.h + y) * s.w + x) * s.cs_out32 + g.out32_off + co) = v;
}

// conv_m16.hip: launch conv_m16_bf16x3<7, npx, deep> on a raster tiling made by conv_big.hip (picks
// the deep weight ring for small tiles; sets the kernels' LDS attribute on first use).
// conv_m16k_wide.hip: launch conv_m16k_bf16x3<false, 3, 6> (4 x 48 tiles; sets its LDS attribute).
int launch_m16k_wide(dim3 grid, int lds, hipStream_t st, const SplitConvShape& s, const SplitConvGroup& g0,
                     const SplitConvGroup& g1, const BigTiling& tl);

// conv_m16r.hip: the register-weight, double-buffered-halo 3x3 kernel (large launches); *taken = 0
// when the shape or launch size is outside it
int launch_conv_m16r(const SplitConvShape& s, const SplitConvGroup* g, bool pool, hipStream_t st, int* taken);

int launch_m16_7x7(int npx, hipStream_t st, const SplitConvShape& s, const SplitConvGroup& g0,
                   const SplitConvGroup& g1, const BigTiling& tl);
// conv_m16q.hip: the small-launch 7x7 kernel (tr x 16 tiles, split K over chunk pairs x nth tap
// ranges, f32 partials in tl.ws for conv_m16_splitk_reduce)
// conv_m16w.hip: the whole-depth register-weight 7x7 kernel (OP_M16W=1 A/B aid); *taken = 0 otherwise
int launch_conv_m16w(const SplitConvShape& s, const SplitConvGroup* g, int cop_max, hipStream_t st, int* taken);
int launch_m16q_7x7(int tr, int nth, int pf, hipStream_t st, const SplitConvShape& s, const SplitConvGroup& g0,
                    const SplitConvGroup& g1, const BigTiling& tl,
                    bool iwg, bool bpf);

}  // namespace op
