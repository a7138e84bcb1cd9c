// Exact-f32 3x3 / 7x7 convolutions with an LDS halo (round 5; the fp32 precision's default for
// those layers, models/CocoPoseNet.py:136-260 at Chainer's own fp32 arithmetic).
//
// Same MFMA mapping, weight layout and accumulation order as conv_mfma_f32 (conv.hip): per wave 2 x
// 2 blocks of 32 output channels x 32 pixels on v_mfma_f32_32x32x2_f32, the k loop over (input chunk
// of 8 channels, tap), each 16-B operand load feeding the 4 MFMAs of the k-pairs {c+j, c+4+j}, so
// every output is BIT-IDENTICAL to conv_mfma_f32's.  What changes is where the B operand comes
// from: conv_mfma_f32 reads each (pixel, 8-channel chunk) slice straight from global memory -- 32 B
// of a 128-B line per lane pair, re-fetched from L2 for each of the 49 taps (the per-CU L1 cannot
// hold 12 waves' rows), ~32 B per clock per CU at 0.71 of the f32 MFMA peak.  Here a workgroup
// stages the halo of its 256-pixel tile for one chunk in LDS once (2 planes: channels c..c+3 and
// c+4..c+7, 16 B per pixel), by LDS-DMA of whole rows, double-buffered: the next chunk's halo is
// issued when a chunk starts and waited for at its end (one barrier per chunk).  Weights stay
// register operands loaded two k steps ahead (the 4 waves of a workgroup read the same 1 KiB lines:
// L1 hits).
//
// Tile: 4 waves x 2 pixel blocks of 32; a block is TCW columns x 32 / TCW rows of one frame
// (TCW 16: 16 x 16 tiles for the 46 / 82-wide maps; 32: 32 x 8 tiles for wide maps).  LDS rows are
// padded to a multiple of 16 pixels, so a ds_read_b128's 16-lane groups (rows r, r + 1 of a
// 16-wide block) hit 64 distinct banks.
#include "common.hpp"

namespace op {

// LDS-DMA from inline asm (as conv_m16r.hip): invisible to the compiler's waitcnt pass, so the B
// reads of the current buffer do not wait for the next buffer's pieces.  Writes M0.
__device__ __forceinline__ void dma16_f32(const void* gsrc, uint32_t lds_byte) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(gsrc), "s"(lds_byte) : "memory");
}

// chunk boundary wait: every VMEM operation but the 2 * CB youngest (the weight loads of the two
// steps ahead, CB per step) has completed -- i.e. this wave's halo pieces, issued before them
template <int CB>
__device__ __forceinline__ void wait_vmcnt_f32() {
  static_assert(2 * CB <= 63, "vmcnt literal");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * CB) : "memory");
}

template <int KS, int TCW>
struct F32Tile {
  static constexpr int R = KS / 2;
  static constexpr int BR = 32 / TCW;          // rows per 32-pixel block
  static constexpr int TR = 4 * 2 * BR;         // tile rows: 4 waves x 2 blocks
  static constexpr int HR = TR + KS - 1;        // halo rows
  static constexpr int HC = TCW + KS - 1;       // halo columns
  static constexpr int HP = (HC + 15) / 16 * 16;  // LDS pitch (pixels)
  static constexpr int NP = (HR * HP + 63) / 64;  // 1-KiB pieces per plane
  static constexpr int PLANE = NP * 1024;
  static constexpr int BUF = 2 * PLANE;         // one chunk: channels c..c+3, c+4..c+7
  static constexpr int LDS = 2 * BUF;           // double-buffered
};

template <int KS, int TCW, int CB = 2>
__global__ __launch_bounds__(256, CB == 4 ? 2 : 1) void conv_f32_lds(ConvShape s, ConvGroup g0, ConvGroup g1, int tiles_x, int tiles_y) {
  using T = F32Tile<KS, TCW>;
  constexpr int KSQ = KS * KS;
  constexpr int R = T::R;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const ConvGroup g = blockIdx.z == 0 ? g0 : g1;
  const int co_base = blockIdx.y * (CB * 32);
  if (co_base >= g.cop) return;
  const int tpf = tiles_x * tiles_y;
  const int frame = blockIdx.x / tpf;
  const int tix = blockIdx.x - frame * tpf;
  const int ty = tix / tiles_x;
  const int y0 = ty * T::TR, x0 = (tix - ty * tiles_x) * TCW;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int l32 = lane & 31, hi = lane >> 5;
  const int wp_in = s.w + 2 * s.pin;
  const int hp_in = s.h + 2 * s.pin;
  const uint32_t lds0 = (uint32_t)(size_t)(__attribute__((address_space(3))) char*)lds;

  // halo pieces of chunk c into buffer b: piece j = plane j / NP, slots 64 (j % NP) .. + 63
  const float* const fin = g.in + (int64_t)frame * hp_in * wp_in * s.cs_in;
  auto issue_halo = [&](int c, int b) {
    for (int j = wave; j < 2 * T::NP; j += 4) {
      const int plane = j >= T::NP, i = j - plane * T::NP;
      const int slot = i * 64 + lane;
      const int hr = slot / T::HP, hc = slot - (slot / T::HP) * T::HP;
      const int yy = min(y0 - R + hr + s.pin, hp_in - 1), xx = min(x0 - R + hc + s.pin, wp_in - 1);
      dma16_f32(fin + ((int64_t)yy * wp_in + xx) * s.cs_in + c * 8 + plane * 4,
                lds0 + (uint32_t)(b * T::BUF + plane * T::PLANE + i * 1024));
    }
  };

  // this lane's pixel in pixel block pb of the wave: tile row / column
  int prow[2], pcol[2];
#pragma unroll
  for (int pb = 0; pb < 2; ++pb) {
    prow[pb] = (wave * 2 + pb) * T::BR + l32 / TCW;
    pcol[pb] = l32 % TCW;
  }
  // B operand byte offsets in a buffer (tap (0, 0)): plane hi, slot (row, col)
  const int boff0 = hi * T::PLANE + (prow[0] * T::HP + pcol[0]) * 16;
  const int boff1 = hi * T::PLANE + (prow[1] * T::HP + pcol[1]) * 16;

  const float* aptr = g.w + (int64_t)(co_base + l32) * 8 + 4 * hi;
  const int64_t wstep = (int64_t)g.cop * 8;
  const int n_it = s.c8 * KSQ;

  floatx16 acc[CB][2];
#pragma unroll
  for (int cb = 0; cb < CB; ++cb)
#pragma unroll
    for (int pb = 0; pb < 2; ++pb)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[cb][pb][r] = 0.0f;

  auto load_a = [&](floatx4(&a)[CB], int it) {
    if (it >= n_it) it = n_it - 1;  // tail prefetch: a valid address, never consumed
    const float* ap = aptr + (int64_t)it * wstep;
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) a[cb] = *(const floatx4*)(ap + cb * 256);
  };
  // the B operands of k step `it` (chunk c, tap t) from LDS
  auto read_b = [&](floatx4(&b)[2], int it) {
    const int c = it / KSQ, t = it - c * KSQ;
    const int ky = t / KS, kx = t - ky * KS;
    const char* bb = lds + (c & 1) * T::BUF + (ky * T::HP + kx) * 16;
    b[0] = *(const floatx4*)(bb + boff0);
    b[1] = *(const floatx4*)(bb + boff1);
  };
  // one k step: 16 MFMAs in conv_mfma_f32's order (round 5: reading the B operands one step ahead
  // measured slower, 431 -> 408 frames/s on the fp32 line: profiles/r05/ab_r05e_fp32_b_prefetch_not_kept.log)
  auto mma = [&](const floatx4(&a)[CB], const floatx4(&b)[2]) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int cb = 0; cb < CB; ++cb)
#pragma unroll
        for (int pb = 0; pb < 2; ++pb)
          acc[cb][pb] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[cb][j], b[pb][j], acc[cb][pb], 0, 0, 0);
  };

  // chunk boundary before step `it` (t == 0): chunk c's halo landed (every wave's pieces: the
  // weight loads of the two steps ahead are the only younger VMEM operations), the previous chunk's
  // buffer is free; then chunk c + 1's halo is issued into it
  auto boundary = [&](int it) {
    const int c = it / KSQ;
    if (it - c * KSQ != 0) return;
    wait_vmcnt_f32<CB>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (c + 1 < s.c8) issue_halo(c + 1, (c + 1) & 1);
  };

  issue_halo(0, 0);
  floatx4 a0[CB], a1[CB];
  load_a(a0, 0);
  load_a(a1, 1);
  int it = 0;
  auto step = [&](const floatx4(&a)[CB], int it) {
    floatx4 b[2];
    read_b(b, it);
    mma(a, b);
  };
  for (; it + 2 <= n_it; it += 2) {
    boundary(it);
    step(a0, it);
    load_a(a0, it + 2);
    boundary(it + 1);
    step(a1, it + 1);
    load_a(a1, it + 3);
  }
  if (it < n_it) {
    boundary(it);
    step(a0, it);
  }

  // epilogue (conv_mfma_f32's): lane holds pixel (prow, pcol) and, per register group q, output
  // channels 8q + 4hi .. +3 of each 32-channel block
  const int wp_out = s.w + 2 * s.pout;
  const int hp_out = s.h + 2 * s.pout;
#pragma unroll
  for (int pb = 0; pb < 2; ++pb) {
    const int y = y0 + prow[pb], x = x0 + pcol[pb];
    if (y >= s.h || x >= s.w) continue;
    float* optr = g.out + ((int64_t)(frame * hp_out + y + s.pout) * wp_out + (x + s.pout)) * s.cs_out;
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

template <int KS, int TCW, int CB>
static int launch_f32_lds_cb(const ConvShape& s, const ConvGroup* g, hipStream_t st) {
  using T = F32Tile<KS, TCW>;
  static bool attr = false;
  if (!attr) {
    OP_HIP_CHECK(hipFuncSetAttribute((const void*)conv_f32_lds<KS, TCW, CB>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     T::LDS));
    attr = true;
  }
  const int tiles_x = (s.w + TCW - 1) / TCW, tiles_y = (s.h + T::TR - 1) / T::TR;
  const int cop_max = s.groups > 1 ? std::max(g[0].cop, g[1].cop) : g[0].cop;
  const dim3 grid((unsigned)(s.n * tiles_x * tiles_y), (unsigned)((cop_max + CB * 32 - 1) / (CB * 32)), (unsigned)s.groups);
  hipLaunchKernelGGL((conv_f32_lds<KS, TCW, CB>), grid, dim3(256), T::LDS, st, s, g[0], s.groups > 1 ? g[1] : g[0],
                     tiles_x, tiles_y);
  OP_AFTER_LAUNCH("conv_f32_lds", st);
  OP_HIP_CHECK(hipGetLastError());
  return OP_OK;
}

template <int KS, int TCW>
static int launch_f32_lds_t(const ConvShape& s, const ConvGroup* g, hipStream_t st) {
  // OP_F32_CB=4: 128 output channels per wave (A/B aid, read per call; needs cop % 128 == 0)
  const char* e = getenv("OP_F32_CB");
  bool cb4 = e && atoi(e) == 4;
  for (int i = 0; i < s.groups; ++i) cb4 = cb4 && g[i].cop % 128 == 0;
  return cb4 ? launch_f32_lds_cb<KS, TCW, 4>(s, g, st) : launch_f32_lds_cb<KS, TCW, 2>(s, g, st);
}

// 3x3 / 7x7 on the LDS-halo kernel; *taken = 0 when the shape is outside it (conv_mfma_f32 runs).
// OP_F32_LDS=0 keeps every layer on conv_mfma_f32 (A/B and parity aid; read per call).
int launch_conv_f32_lds(const ConvShape& s, const ConvGroup* g, hipStream_t st, int* taken) {
  *taken = 0;
  const char* e = getenv("OP_F32_LDS");
  if ((e && atoi(e) == 0) || (s.ks != 3 && s.ks != 7) || s.pin < s.ks / 2 || s.cs_in % 4 || s.n < 1) return OP_OK;
  // tile width: 16 or 32 columns, whichever wastes fewer columns (ties: 32, fewer halo pixels)
  const double u16 = (double)s.w / (16.0 * ((s.w + 15) / 16)), u32 = (double)s.w / (32.0 * ((s.w + 31) / 32));
  const bool w32 = u32 >= u16 - 1e-9;
  const int64_t blocks = (int64_t)s.n * ((s.w + (w32 ? 31 : 15)) / (w32 ? 32 : 16)) * ((s.h + (w32 ? 7 : 15)) / (w32 ? 8 : 16));
  if (blocks >= (1ll << 31) - 1) return OP_OK;
  census_add(OP_CENSUS_F32_LDS);
  *taken = 1;
  if (s.ks == 3) return w32 ? launch_f32_lds_t<3, 32>(s, g, st) : launch_f32_lds_t<3, 16>(s, g, st);
  return w32 ? launch_f32_lds_t<7, 32>(s, g, st) : launch_f32_lds_t<7, 16>(s, g, st);
}

}  // namespace op
