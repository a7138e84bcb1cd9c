// Fused 1x1 pair at the end of every branch (3xBF16 split, gfx950): conv5_4 + conv5_5
// (CocoPoseNet.py:157-158, 162-163: 128 -> 512 ReLU -> 38 | 19) and Mconv6 + Mconv7 of stages
// 2-6 (e.g. :174-175, 181-182: 128 -> 128 ReLU -> 38 | 19).
//
// The intermediate (512 or 128 channels per pixel) never reaches HBM: a workgroup owns 64
// consecutive pixels of the batch (raster order, crossing frame borders) of one branch.
//  * its input tile (64 px x Ci split channels) is copied once into LDS;
//  * for each 128-channel chunk of the intermediate, GEMM1 (v_mfma_f32_16x16x32_bf16, K = 32
//    input channels per step, products hi*hi + hi*lo + lo*hi) -> + bias, ReLU, hi/lo split ->
//    LDS, then GEMM2 accumulates that chunk's contribution to the <= 48 output channels in
//    registers;
//  * the epilogue adds the second bias and writes the split output (and the dense f32 copy of
//    the last stage's maps) straight into the stage-input (concat) buffer slices.
// Waves: 4; GEMM1: wave w = intermediate blocks 2w, 2w+1 (16 ch each) x 4 pixel blocks;
// GEMM2: wave w = pixel block w x all output blocks.  Weights come from L2 (the CU's tiles share
// them), issued a K step (GEMM2) or a chunk (GEMM1) ahead.  Mconv6+7 (one chunk): the intermediate
// overwrites the input tile, 33 KiB LDS, 4 workgroups per CU; conv5_4+5 (4 chunks): 67.5 KiB, 2.
#include "common.hpp"
#include "conv_big.hpp"

namespace op {

typedef __bf16 bf16x8h __attribute__((ext_vector_type(8)));
typedef unsigned short u16x4h __attribute__((ext_vector_type(4)));

constexpr int kHeadPx = 64;
// Round 4 experiment, OFF by default (-DHEAD_SWZ=1 builds it): LDS swizzle of the X / T rows.  A pixel row holds 16 groups of 8 channels (32 B: hi, lo);
// group cg of pixel px sits at slot cg ^ swz(px).  ds_read_b128 services a wave in 4 lane groups
// of 16 -- {0-3, 12-15, 20-27}, {4-11, 16-19, 28-31}, ... (MI355X_MICROARCH.md, LDS) -- which mix
// pixels 0-3 / 12-15 of one k group with pixels 4-11 of the next; at the 528-B pitch those
// collided 2-way in every lane group (SQ: 2.9-4.5 conflict cycles per LDS instruction).  Flipping
// the group bit 0 for pixels 4-11 of every 16 makes all four lane groups hit 64 distinct banks:
// conflict cycles per LDS instruction 4.48 -> 1.28 / 4.00 -> 2.29, yet the head launches ran
// slower, 2.42 vs 2.05 ms per 232-frame step in a 5-round A/B (profiles/r04/ab_r04s_*.log).
#ifndef HEAD_SWZ
#define HEAD_SWZ 0
#endif
__device__ __forceinline__ int head_swz(int px) { return HEAD_SWZ ? (((px & 15) + 4) >> 3) & 1 : 0; }

__device__ __forceinline__ floatx4 mfma3(const bf16x8h& ah, const bf16x8h& al, const bf16x8h& bh, const bf16x8h& bl,
                                        floatx4 acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, acc, 0, 0, 0);
  return acc;
}

// PXB (round 4, opt-in OP_HEAD_PX=128, measured slower): pixel blocks of 64 per workgroup.
// TPW (round 4, opt-in OP_HEAD_TPW, measured slower): 64-px tiles per workgroup, one after the other.  Mconv6 + Mconv7 (ONE) has a
// single 128-channel chunk, so a wave's GEMM1 weight fragments (64 KiB per workgroup, re-read from
// L2 by every workgroup: ~1 GB per 232-frame launch) are loaded once for TPW tiles.
// PL (round 6): channel-group-planar X / T tiles, [8-ch group][hi, lo][px][16 B].
// A ds_read_b128 lane group (above) then reads 16 consecutive pixels' 16-B pieces of planes that
// start a multiple of 256 B apart: 64 distinct banks, no swizzle; the T write pairs rows with
// v_permlane16_swap (split_pair_swap) into one 16-B store per lane, 8 consecutive pixels per
// ds_write_b128 cycle.  X's lo planes hold pixel px at slot px ^ 4 (a lane group's read stays a
// permutation of 16 slots), so the copy of a [pixel][channels] input can give 8 consecutive lanes
// the hi and lo pieces of 4 pixels (64-B runs of each pixel per 16 lanes) and still write 8 slots.
// (Round 6: 8 pixels x 16-B pieces per 16 lanes made conv5_4+5's copy 14 % slower.)
template <int NB2, bool ONE, int PXB = 1, int TPW = 1, int PL = 0>
#ifndef HEAD_TPW_OCC
#define HEAD_TPW_OCC 3  // workgroups per CU the TPW > 1 forms are built for (a1 stays live across tiles)
#endif
__global__ __launch_bounds__(256, ONE ? (TPW > 1 ? HEAD_TPW_OCC : 4 / PXB) : 2 / PXB) void conv_head_bf16x3(HeadShape s, HeadGroup g0,
                                                                                                  HeadGroup g1,
                                                                                  int32_t per_group) {
  constexpr int CI = 128;  // both pairs read 128 channels per branch
  constexpr int kPx = kHeadPx * PXB;
  static_assert(TPW == 1 || ONE, "several tiles per workgroup keep one chunk's weights");
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int grp = blockIdx.x >= (unsigned)per_group ? 1 : 0;
  const HeadGroup g = grp ? g1 : g0;
  const int wg = blockIdx.x - grp * per_group;
  const int hw = s.h * s.w;
  const int total = s.n * hw;
  constexpr int xpitch = CI * 4 + 16;  // +16 B: consecutive pixels start 4 banks apart
  constexpr int tpitch = 128 * 4 + 16;
  constexpr int plane = kPx * 16;  // PL: bytes of one (group, hi | lo) plane
  char* const X = lds;
  char* const T = ONE ? lds : lds + kPx * xpitch;  // ONE (co1 = 128): T overwrites X after GEMM1
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int l16 = lane & 15, kg = lane >> 4;
  const int wp_in = s.w + 2 * s.pin, hp_in = s.h + 2 * s.pin;

  const int64_t wpl1 = (int64_t)g.cop1 * 16;  // bytes per (c16, plane) of W1
  const int64_t wpl2 = (int64_t)g.cop2 * 16;
  const char* const w1 = (const char*)g.w1;
  const char* const w2 = (const char*)g.w2;
  const int kh = kg & 1;
  // A fragments of GEMM1 for one chunk: 4 K steps x 2 channel blocks x (hi, lo), issued ahead
  bf16x8h a1[4][2][2];
  auto load_a1 = [&](int chunk) {
    const int co_a = chunk + wave * 32 + l16;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int c16 = 2 * k + (kg >> 1);
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        const char* wa = w1 + (int64_t)(c16 * 4 + 2 * kh) * wpl1 + (int64_t)(co_a + 16 * cb) * 16;
        a1[k][cb][0] = *(const bf16x8h*)wa;
        a1[k][cb][1] = *(const bf16x8h*)(wa + wpl1);
      }
    }
  };
  load_a1(0);
  for (int tile = 0; tile < TPW; ++tile) {
  const int P0 = (wg * TPW + tile) * kPx;
  if (P0 >= total) break;  // block-uniform
  if (!ONE && tile > 0) load_a1(0);
  // ---- input tile -> LDS (16-B pieces; pixels past the batch repeat the last one) ----
  {
    // (chunk-planar input: consecutive threads take consecutive pixels of one plane, so a wave
    // reads 64 contiguous 16-B pieces; else one pixel's consecutive pieces)
    constexpr int pieces = CI / 4;
    const int64_t pcs = split_piece_stride(s.in_planar, hp_in, wp_in), pxs = split_pixel_stride(s.in_planar, s.cs_in);
    for (int i = threadIdx.x; i < kPx * pieces; i += 256) {
      int px, pc;
      if ((PL & 1) && !s.in_planar) {  // lanes (hi | lo piece, 4 pixels, 8 piece pairs): 64-B runs read
        const int lo = i & 63, hi = i >> 6;
        px = ((lo >> 1) & 3) + 4 * (hi % (kPx / 4));
        pc = (lo & 1) + 2 * (lo >> 3) + 16 * (hi / (kPx / 4));
      } else {
        px = s.in_planar ? i % kPx : i / pieces;
        pc = s.in_planar ? i / kPx : i - px * pieces;
      }
      const int P = min(P0 + px, total - 1);
      const int f = P / hw, pp = P - f * hw;
      const int y = pp / s.w, x = pp - y * s.w;
      const char* src = (const char*)g.in + (int64_t)f * hp_in * wp_in * s.cs_in * 4 +
                        ((int64_t)(y + s.pin) * wp_in + x + s.pin) * pxs + pc * pcs;
      if constexpr ((PL & 1) != 0)
        *(uint4*)(X + pc * plane + (px ^ (pc & 1) * 4) * 16) = *(const uint4*)src;
      else
        *(uint4*)(X + px * xpitch + (((pc >> 1) ^ head_swz(px)) * 32 + (pc & 1) * 16)) = *(const uint4*)src;
    }
  }
  __syncthreads();

  floatx4 acc2[PXB][NB2];
#pragma unroll
  for (int q = 0; q < PXB; ++q)
#pragma unroll
    for (int j = 0; j < NB2; ++j) acc2[q][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  for (int chunk = 0; chunk < (ONE ? 128 : s.co1); chunk += 128) {
    // ---- GEMM1: intermediate channels chunk + 32w .. +31 x kPx px ----
    floatx4 acc1[2][4 * PXB];
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int pb = 0; pb < 4 * PXB; ++pb) acc1[cb][pb] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
#pragma unroll
      for (int pb = 0; pb < 4 * PXB; ++pb) {
        const char* xb = (PL & 1) ? X + (4 * k + kg) * 2 * plane + (pb * 16 + l16) * 16
                            : X + (pb * 16 + l16) * xpitch + ((4 * k + kg) ^ head_swz(l16)) * 32;
        const bf16x8h bh = *(const bf16x8h*)xb;
        const bf16x8h bl = *(const bf16x8h*)((PL & 1) ? xb + plane + ((l16 ^ 4) - l16) * 16 : xb + 16);
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) acc1[cb][pb] = mfma3(a1[k][cb][0], a1[k][cb][1], bh, bl, acc1[cb][pb]);
      }
    }
    // GEMM2's A fragments of the first K step, in flight across the T write and barrier
    bf16x8h a2[NB2][2];
    auto load_a2 = [&](int k) {
      const int c16 = chunk / 16 + 2 * k + (kg >> 1);
#pragma unroll
      for (int j = 0; j < NB2; ++j) {
        const char* wa = w2 + (int64_t)(c16 * 4 + 2 * kh) * wpl2 + (int64_t)(j * 16 + l16) * 16;
        a2[j][0] = *(const bf16x8h*)wa;
        a2[j][1] = *(const bf16x8h*)(wa + wpl2);
      }
    };
    load_a2(0);
    if constexpr (ONE) __syncthreads();  // every wave is done with X before T overwrites it
    // ---- bias + ReLU + split -> T[px][chunk channel] ----
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      const int cl = wave * 32 + cb * 16 + 4 * kg;  // chunk-relative channel of e = 0
      const floatx4 bv = *(const floatx4*)(g.b1 + chunk + cl);
#pragma unroll
      for (int pb = 0; pb < 4 * PXB; ++pb) {
        if constexpr ((PL & 2) != 0) {
          floatx4 v;
          uint32_t own[4], w[4];
          split_pair_swap(acc1[cb][pb], bv, 1, v, own, w);
          *(uint4*)(T + ((cl >> 3) * 2 + (kg & 1)) * plane + (pb * 16 + l16) * 16) = make_uint4(w[0], w[1], w[2], w[3]);
          continue;
        }
        u16x4h vh, vl;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float v = acc1[cb][pb][e] + bv[e];
          v = v > 0.0f ? v : 0.0f;
          const __bf16 h16 = (__bf16)v;
          const __bf16 l16v = (__bf16)(v - (float)h16);
          vh[e] = __builtin_bit_cast(unsigned short, h16);
          vl[e] = __builtin_bit_cast(unsigned short, l16v);
        }
        char* d = T + (pb * 16 + l16) * tpitch + ((cl >> 3) ^ head_swz(l16)) * 32 + (cl & 7) * 2;
        *(u16x4h*)d = vh;
        *(u16x4h*)(d + 16) = vl;
      }
    }
    __syncthreads();
    // ---- GEMM2: pixel blocks wave, wave + 4 (PXB 2) x NB2 output blocks, K = this chunk ----
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      bf16x8h cur[NB2][2];
#pragma unroll
      for (int j = 0; j < NB2; ++j) {
        cur[j][0] = a2[j][0];
        cur[j][1] = a2[j][1];
      }
      if (k + 1 < 4) load_a2(k + 1);
#pragma unroll
      for (int q = 0; q < PXB; ++q) {
        const char* tb = (PL & 2) ? T + (4 * k + kg) * 2 * plane + ((wave + 4 * q) * 16 + l16) * 16
                            : T + ((wave + 4 * q) * 16 + l16) * tpitch + ((4 * k + kg) ^ head_swz(l16)) * 32;
        const bf16x8h bh = *(const bf16x8h*)tb;
        const bf16x8h bl = *(const bf16x8h*)(tb + ((PL & 2) ? plane : 16));
#pragma unroll
        for (int j = 0; j < NB2; ++j) acc2[q][j] = mfma3(cur[j][0], cur[j][1], bh, bl, acc2[q][j]);
      }
    }
    // next chunk's GEMM1 fragments: issued after GEMM2's (vmcnt retires in order)
    if (!ONE && chunk + 128 < s.co1) load_a1(chunk + 128);
    __syncthreads();  // T is rewritten by the next chunk
  }

  // ---- epilogue: + bias2 (no ReLU), split store into the concat slice (+ dense f32 copy) ----
#pragma unroll
  for (int q = 0; q < PXB; ++q) {
  const int P = P0 + (wave + 4 * q) * 16 + l16;
  if (P >= total) continue;
  const int f = P / hw, pp = P - f * hw;
  const int y = pp / s.w, x = pp - y * s.w;
  const int wp_out = s.w + 2 * s.pout, hp_out = s.h + 2 * s.pout;
  const int64_t opc = split_piece_stride(s.out_planar, hp_out, wp_out);
  char* const optr = (char*)g.out + (int64_t)f * hp_out * wp_out * s.cs_out * 4 +
                     ((int64_t)(y + s.pout) * wp_out + x + s.pout) * split_pixel_stride(s.out_planar, s.cs_out);
  float* const o32 = g.out32 ? g.out32 + (int64_t)P * s.cs_out32 + g.out32_off : nullptr;
#pragma unroll
  for (int j = 0; j < NB2; ++j) {
    const int co = j * 16 + 4 * kg;
    if (co >= g.cout_store) continue;
    const floatx4 bv = *(const floatx4*)(g.b2 + co);
    floatx4 v;
    u16x4h vh, vl;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float fv = acc2[q][j][e] + bv[e];
      v[e] = fv;
      const __bf16 h16 = (__bf16)fv;
      const __bf16 l16v = (__bf16)(fv - (float)h16);
      vh[e] = __builtin_bit_cast(unsigned short, h16);
      vl[e] = __builtin_bit_cast(unsigned short, l16v);
    }
    char* d = optr + (co >> 3) * 2 * opc + (co & 7) * 2;
    *(u16x4h*)d = vh;
    *(u16x4h*)(d + opc) = vl;
    if (o32) *(floatx4*)(o32 + co) = v;
  }
  }
  }
}

template <int NB2, bool ONE, int PXB, int PL>
static int launch_head_pl1(dim3 grid, int lds, hipStream_t st, const HeadShape& s, const HeadGroup& a,
                            const HeadGroup& b, int per) {
  static bool attr = false;
  if (!attr) {
    OP_HIP_CHECK(hipFuncSetAttribute((const void*)conv_head_bf16x3<NB2, ONE, PXB, 1, PL>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  hipLaunchKernelGGL((conv_head_bf16x3<NB2, ONE, PXB, 1, PL>), grid, dim3(256), lds, st, s, a, b, per);
  return OP_OK;
}

template <int NB2, bool ONE, int PXB>
static int launch_head_pl(int pl, dim3 grid, int lds, hipStream_t st, const HeadShape& s, const HeadGroup& a,
                           const HeadGroup& b, int per) {
  static_assert(PXB == 1, "planar tiles: 64-px workgroups");
  if (pl == 1) return launch_head_pl1<NB2, ONE, PXB, 1>(grid, lds, st, s, a, b, per);
  if (pl == 2) return launch_head_pl1<NB2, ONE, PXB, 2>(grid, lds, st, s, a, b, per);
  return launch_head_pl1<NB2, ONE, PXB, 3>(grid, lds, st, s, a, b, per);
}

template <int NB2, int PXB>
static int launch_head_px(const HeadShape& s, const HeadGroup* g, hipStream_t st) {
  constexpr int kPx = kHeadPx * PXB;
  const int total = s.n * s.h * s.w;
  const bool one = s.co1 == 128;
  // OP_HEAD_TPW=2 / 4: Mconv6 + Mconv7 with that many tiles per workgroup -- opt-in: 2.28 vs 2.14
  // ms per 232-frame step at TPW 4 (4-round A/B, profiles/r04/ab_r04t_head_tpw.log), so the heads
  // are not bound by re-reading their weights from L2 (2 workgroups per CU: 2.82)
  static const int tpw_env = getenv("OP_HEAD_TPW") ? atoi(getenv("OP_HEAD_TPW")) : 0;
  const int tiles = (total + kPx - 1) / kPx;
  int tpw = 1;
  if (one && PXB == 1 && (tpw_env == 2 || tpw_env == 4)) tpw = tpw_env;
  const int per = (tiles + tpw - 1) / tpw;
  // channel-group-planar LDS tiles (PL, round 6): bit 0 X, bit 1 T.  OP_HEAD_PLANAR (Mconv6+7) and
  // OP_HEAD_PLANAR1 (conv5_4+5) = 0..3, read per launch (the bit-identity test flips them in one
  // process).  Default 3 for both: LDS bank conflicts 4.00 / 4.48 -> 0.00 per LDS instruction.  At
  // equal time only with conv_head.o built under max-ilp (Makefile): under the default scheduler
  // conv5_4+5's four-chunk loop ran 10-12 % slower with ANY planar bit (the compiler reordered the
  // whole loop), profiles/r06/ab_r06j_head_planar.log.
  const char* pl_env = getenv(one ? "OP_HEAD_PLANAR" : "OP_HEAD_PLANAR1");
  const int pl = (PXB == 1 && tpw == 1) ? (pl_env ? (atoi(pl_env) & 3) : 3) : 0;
  const int lds = kPx * (128 * 4 + 16) * (one ? 1 : 2);
  static bool attr = false;
  if (!attr) {
    OP_HIP_CHECK(hipFuncSetAttribute((const void*)conv_head_bf16x3<NB2, false, PXB>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    OP_HIP_CHECK(hipFuncSetAttribute((const void*)conv_head_bf16x3<NB2, true, PXB>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    OP_HIP_CHECK(hipFuncSetAttribute((const void*)conv_head_bf16x3<NB2, true, PXB, 2>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    OP_HIP_CHECK(hipFuncSetAttribute((const void*)conv_head_bf16x3<NB2, true, PXB, 4>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  const dim3 grid((unsigned)(per * s.groups));
  int rc = OP_OK;
  if constexpr (PXB == 1) {
    if (pl && one) rc = launch_head_pl<NB2, true, PXB>(pl, grid, lds, st, s, g[0], s.groups > 1 ? g[1] : g[0], per);
    else if (pl) rc = launch_head_pl<NB2, false, PXB>(pl, grid, lds, st, s, g[0], s.groups > 1 ? g[1] : g[0], per);
  }
  if (rc) return rc;
  if (pl) {
  } else if (one && tpw == 4)
    hipLaunchKernelGGL((conv_head_bf16x3<NB2, true, PXB, 4>), dim3((unsigned)(per * s.groups)), dim3(256), lds, st, s,
                       g[0], s.groups > 1 ? g[1] : g[0], per);
  else if (one && tpw == 2)
    hipLaunchKernelGGL((conv_head_bf16x3<NB2, true, PXB, 2>), dim3((unsigned)(per * s.groups)), dim3(256), lds, st, s,
                       g[0], s.groups > 1 ? g[1] : g[0], per);
  else if (one)
    hipLaunchKernelGGL((conv_head_bf16x3<NB2, true, PXB>), dim3((unsigned)(per * s.groups)), dim3(256), lds, st, s,
                       g[0], s.groups > 1 ? g[1] : g[0], per);
  else
    hipLaunchKernelGGL((conv_head_bf16x3<NB2, false, PXB>), dim3((unsigned)(per * s.groups)), dim3(256), lds, st, s,
                       g[0], s.groups > 1 ? g[1] : g[0], per);
  OP_AFTER_LAUNCH("conv_head_bf16x3", st);
  OP_HIP_CHECK(hipGetLastError());
  return OP_OK;
}

// 64-px workgroups; OP_HEAD_PX=128 selects 128-px ones (half the weight fetches per pixel, but
// fewer waves per CU: 2.71 vs 2.04 ms per 232-frame step, profiles/r04/ab_r04p_head_px.log)
template <int NB2>
static int launch_head_t(const HeadShape& s, const HeadGroup* g, hipStream_t st) {
  static const bool big = getenv("OP_HEAD_PX") && atoi(getenv("OP_HEAD_PX")) == 128;
  return big ? launch_head_px<NB2, 2>(s, g, st) : launch_head_px<NB2, 1>(s, g, st);
}

// *taken = 0 when the shape is outside this kernel (the caller runs the two 1x1 convs).
int launch_conv_head(const HeadShape& s, const HeadGroup* g, hipStream_t st, int* taken) {
  *taken = 0;
  if (s.ci != 128 || s.co1 % 128 || s.cs_in % 8 || s.groups < 1 || s.groups > 2) return OP_OK;
  int store = 0;
  for (int i = 0; i < s.groups; ++i) {
    if (g[i].cop1 < s.co1 || g[i].cout_store % 4 || g[i].cout_store > 48 || g[i].cop2 < g[i].cout_store) return OP_OK;
    store = store > g[i].cout_store ? store : g[i].cout_store;
  }
  *taken = 1;
  if (store > 32) return launch_head_t<3>(s, g, st);
  if (store > 16) return launch_head_t<2>(s, g, st);
  return launch_head_t<1>(s, g, st);
}

}  // namespace op
