// Tap-pair convolution on v_mfma_f32_16x16x32_bf16 (3xBF16 split, gfx950): the 7x7 stage convs.
//
// Why: in bare loops on random data the 16x16x32 bf16 MFMA sustains ~15 % more FLOP/s than the
// 32x32x16 form under the chip's power limit (measured here: 2.03 vs 1.76 PF with the conv's own
// accumulation pattern, tools/micro/mfma_peak.hip).  Its K = 32 is fed with TWO TAPS of one
// 16-channel chunk: lane group g = lane/16 holds k = 8g..8g+7, i.e. tap t + g/2, channel half
// g%2 -- so the activation halo and the weight ring keep the 16-channel layout of conv_big and the
// weights need no repacking (a pair's A operand is two consecutive ring slots).  A 7x7 chunk is
// 25 steps (the last pairs tap 48 with zero weights: 2 % waste).
//
// Workgroup = 8 waves, one per CU (1 WG/CU): 128 output channels x a TR x TC tile with TC a
// multiple of 16, so every 16-pixel block lies in one tile row and its LDS address is
// wave-uniform (scalar) -- a lane only adds its column.  Wave w: channel quarter w % 4 (32
// channels = 2 blocks of 16) x pixel group w / 4 (NPB blocks of 16 pixels): 2 x NPB accumulator
// tiles of 16x16 (4 registers each).  Halo, weight ring (6 slots, barrier per tap pair, 4 taps
// ahead) and XCD-aware block order as in conv_big.hip.
#include <cstdlib>
#include <vector>

#include "common.hpp"

namespace op {

typedef __bf16 bf16x8p __attribute__((ext_vector_type(8)));
typedef unsigned short u16x4p __attribute__((ext_vector_type(4)));

#define LDS_PTR_P(p) ((__attribute__((address_space(3))) void*)(p))

struct PairTiling {
  int32_t tr, tc;            // tile rows x cols (tc % 16 == 0, tr * tc == tile capacity)
  int32_t tiles_y, tiles_x;
  int32_t pitch;             // LDS halo row pitch (16-B slots) = tc + 16: bank-conflict-free wraps
  int32_t nh;                // 1-KiB halo pieces per plane
  int32_t units, co_tiles, per_unit, xpu;
};

template <int KS, int NPB>
__global__ __launch_bounds__(512, 1) void conv_pair_bf16x3(SplitConvShape s, SplitConvGroup g0, SplitConvGroup g1,
                                                           PairTiling tl) {
  constexpr int KSQ = KS * KS;
  constexpr int R = KS / 2;
  constexpr int PLANE_W = 128 * 16;  // one weight plane of the 128-channel tile
  constexpr int SLOT_W = 4 * PLANE_W;
  constexpr int RING = 6;
  extern __shared__ __attribute__((aligned(16))) char lds[];  // [W ring][halo: 4 planes]

  const int lin = blockIdx.x;
  int unit, widx;
  if (tl.xpu) {
    const int xcd = lin & 7, slot = lin >> 3;
    unit = xcd / tl.xpu;
    widx = slot * tl.xpu + (xcd - unit * tl.xpu);
  } else {
    unit = lin / tl.per_unit;
    widx = lin - unit * tl.per_unit;
  }
  if (unit >= tl.units || widx >= tl.per_unit) return;
  const int grp = unit / tl.co_tiles;
  const int co0 = (unit - grp * tl.co_tiles) * 128;
  const SplitConvGroup g = grp == 0 ? g0 : g1;
  if (co0 >= g.cop) return;
  const int tpf = tl.tiles_y * tl.tiles_x;
  const int frame = widx / tpf;
  const int tix = widx - frame * tpf;
  const int ty = tix / tl.tiles_x;
  const int y0 = ty * tl.tr, x0 = (tix - ty * tl.tiles_x) * tl.tc;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int cq = wave & 3;   // channel quarter: co0 + 32*cq .. +31
  const int pg = wave >> 2;  // pixel group: tile blocks pg*NPB .. +NPB-1
  const int l16 = lane & 15, lg = lane >> 4;
  const int tsel = lg >> 1, kh = lg & 1;  // this lane's tap (t + tsel) and channel half
  const int hplane = tl.nh * 1024;
  char* const halo = lds + RING * SLOT_W;
  const int wp_in = s.w + 2 * s.pin;
  const int hp_in = s.h + 2 * s.pin;
  const int64_t pix_bytes = (int64_t)s.cs_in * 4;
  const char* const fbase = (const char*)g.in + (int64_t)frame * hp_in * wp_in * pix_bytes;

  // weights: wave w copies plane w/2, channels 64*(w&1) .. +63 of the tap tile (one 1-KiB piece)
  const int64_t wplane = (int64_t)g.cop * 16;
  const int64_t wstep = 4 * wplane;
  const char* const wsrc = (const char*)g.w + (wave >> 1) * wplane + ((int64_t)co0 + 64 * (wave & 1) + lane) * 16;
  const int wdst = (wave >> 1) * PLANE_W + (wave & 1) * 1024;
  const int n_it = s.c16 * KSQ;
  auto stage_w = [&](int it) {
    char* dst = lds + (it % RING) * SLOT_W + wdst;
    if (it >= n_it) it = n_it - 1;
    __builtin_amdgcn_global_load_lds((const void*)(wsrc + (int64_t)it * wstep), LDS_PTR_P(dst), 16, 0, 0);
  };

  const int bpr = tl.tc >> 4;  // 16-pixel blocks per tile row
  const int rows_here = min(tl.tr, s.h - y0);

  floatx4 acc[2][NPB];
#pragma unroll
  for (int cb = 0; cb < 2; ++cb)
#pragma unroll
    for (int pb = 0; pb < NPB; ++pb) acc[cb][pb] = floatx4{0.f, 0.f, 0.f, 0.f};

  for (int i = 0; i < 4; ++i) stage_w(i);
  // this lane's A: plane (2*kh + part) of slot (t + tsel), channel co0 + 32*cq + 16*cb + l16
  const int a_lane = (2 * kh) * PLANE_W + (cq * 32 + l16) * 16;
  // this lane's B: plane (2*kh + part), slot (block row * pitch + block col + l16 + tap offset)
  char* const b_lane = halo + (2 * kh) * hplane + l16 * 16;
  int it = 0;
  for (int c = 0; c < s.c16; ++c) {
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    {
      const char* src0 = fbase + c * 64;
      for (int q = wave; q < 4 * tl.nh; q += 8) {
        const int plane = q / tl.nh, i = q - (q / tl.nh) * tl.nh;
        const int sl = i * 64 + lane;
        const int hr = sl / tl.pitch, hc = sl - (sl / tl.pitch) * tl.pitch;
        int yy = y0 - R + hr + s.pin, xx = x0 - R + hc + s.pin;
        yy = yy < hp_in - 1 ? yy : hp_in - 1;
        xx = xx < wp_in - 1 ? xx : wp_in - 1;
        __builtin_amdgcn_global_load_lds((const void*)(src0 + plane * 16 + ((int64_t)yy * wp_in + xx) * pix_bytes),
                                         LDS_PTR_P(halo + plane * hplane + i * 1024), 16, 0, 0);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#pragma unroll 1
    for (int t = 0; t < KSQ; t += 2) {
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");  // W(it), W(it+1) landed (see conv_big.hip)
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      stage_w(it + 4);
      stage_w(it + 5);
      const bool two = t + 1 < KSQ;
      const int tt = two ? t + tsel : t;  // a 1-tap tail: the upper lanes read tap t with zero weights
      const int toff = ((tt / KS) * tl.pitch + (tt - (tt / KS) * KS)) * 16;
      const char* wb = lds + ((it + tsel) % RING) * SLOT_W + a_lane;
      bf16x8p ah[2], al[2];
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        ah[cb] = *(const bf16x8p*)(wb + cb * 256);
        al[cb] = *(const bf16x8p*)(wb + PLANE_W + cb * 256);
      }
      if (!two && tsel) {
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          ah[cb] = bf16x8p{};
          al[cb] = bf16x8p{};
        }
      }
      const char* bl0 = b_lane + toff;
      auto boff = [&](int pb) -> int {  // wave-uniform LDS offset of block pb
        const int b = pg * NPB + pb;
        const int r = b / bpr;
        return (r * tl.pitch + ((b - r * bpr) << 4)) * 16;
      };
      bf16x8p bh[3], bl[3];
      bh[0] = *(const bf16x8p*)(bl0 + boff(0));
      bl[0] = *(const bf16x8p*)(bl0 + hplane + boff(0));
      bh[1] = *(const bf16x8p*)(bl0 + boff(1));
      bl[1] = *(const bf16x8p*)(bl0 + hplane + boff(1));
#pragma unroll
      for (int pb = 0; pb < NPB; ++pb) {
        if (pb + 2 < NPB) {
          bh[(pb + 2) % 3] = *(const bf16x8p*)(bl0 + boff(pb + 2));
          bl[(pb + 2) % 3] = *(const bf16x8p*)(bl0 + hplane + boff(pb + 2));
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          acc[cb][pb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[cb], bh[pb % 3], acc[cb][pb], 0, 0, 0);
          acc[cb][pb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[cb], bl[pb % 3], acc[cb][pb], 0, 0, 0);
          acc[cb][pb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[cb], bh[pb % 3], acc[cb][pb], 0, 0, 0);
        }
      }
      it += two ? 2 : 1;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // ---- epilogue: D(row = co, col = pixel): lane holds channels 4*lg .. +3 of pixel l16 ----
  const int wp_out = s.w + 2 * s.pout;
  const int hp_out = s.h + 2 * s.pout;
#pragma unroll
  for (int pb = 0; pb < NPB; ++pb) {
    const int b = pg * NPB + pb;
    const int r = b / bpr;
    const int x = x0 + ((b - r * bpr) << 4) + l16;
    if (r >= rows_here || x >= s.w) continue;
    const int y = y0 + r;
    char* optr = (char*)g.out + ((int64_t)(frame * hp_out + y + s.pout) * wp_out + (x + s.pout)) * (int64_t)s.cs_out * 4;
    float* o32 = g.out32 ? g.out32 + ((int64_t)(frame * s.h + y) * s.w + x) * s.cs_out32 + g.out32_off : nullptr;
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      const int co = co0 + cq * 32 + cb * 16 + 4 * lg;
      if (co >= g.cout_store) continue;
      const floatx4 bv = *(const floatx4*)(g.bias + co);
      floatx4 v;
      u16x4p vh, vl;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float f = acc[cb][pb][e] + bv[e];
        if (s.relu) f = f > 0.0f ? f : 0.0f;
        v[e] = f;
        const __bf16 h16 = (__bf16)f;
        const __bf16 l16b = (__bf16)(f - (float)h16);
        vh[e] = __builtin_bit_cast(unsigned short, h16);
        vl[e] = __builtin_bit_cast(unsigned short, l16b);
      }
      char* d = optr + (co >> 3) * 32 + (co & 7) * 2;
      *(u16x4p*)d = vh;
      *(u16x4p*)(d + 16) = vl;
      if (o32) *(floatx4*)(o32 + co) = v;
    }
  }
}

static int pair_halo_bytes(int tr, int tc, int ks) { return 4 * 1024 * (((tr + ks - 1) * (tc + 16) + 63) / 64); }

// Tile choice: tc a multiple of 16 dividing the tile capacity (cap = 2 * NPB * 16 pixels); among
// the tilings within 3 % of the best MFMA-lane utilisation, the least halo re-read.
static bool pair_tiling(int cap, int ks, int n, int h, int w, int groups, int cop_max, PairTiling& t) {
  const int budget = 160 * 1024 - 6 * 4 * 128 * 16;
  struct Cand {
    int tr, tc, tiles_y, tiles_x;
    double util, amp;
  };
  std::vector<Cand> cands;
  double best = 0.0;
  for (int tc = 16; tc <= cap; tc += 16) {
    if (cap % tc) continue;
    const int tr = cap / tc;
    if (pair_halo_bytes(tr, tc, ks) > budget) continue;
    if (tc >= w + 16) break;  // wider tiles only add masked columns
    const int tiles_x = (w + tc - 1) / tc, tiles_y = (h + tr - 1) / tr;
    const double util = (double)h * w / ((double)tiles_x * tiles_y * cap);
    const double amp = (double)(tr + ks - 1) * (tc + ks - 1) / ((double)tr * tc);
    cands.push_back({tr, tc, tiles_y, tiles_x, util, amp});
    best = util > best ? util : best;
  }
  if (best <= 0.0) return false;
  const Cand* pick = nullptr;
  for (const Cand& c : cands)
    if (c.util >= best - 0.03 && (!pick || c.amp < pick->amp - 1e-9)) pick = &c;
  t.tr = pick->tr;
  t.tc = pick->tc;
  t.tiles_y = pick->tiles_y;
  t.tiles_x = pick->tiles_x;
  t.pitch = t.tc + 16;
  t.nh = ((t.tr + ks - 1) * t.pitch + 63) / 64;
  t.co_tiles = (cop_max + 127) / 128;
  t.units = groups * t.co_tiles;
  t.per_unit = n * t.tiles_y * t.tiles_x;
  t.xpu = (t.units <= 8 && 8 % t.units == 0) ? 8 / t.units : 0;
  return true;
}

// 7x7 split-path convolution on 16x16x32 tap pairs; *taken = 0 when the shape is outside it.
int launch_conv_pair(const SplitConvShape& s, const SplitConvGroup* g, hipStream_t st, int* taken) {
  constexpr int NPB = 24;
  *taken = 0;
  if (s.ks != 7 || s.cs_in % 16 || s.pin < 3) return OP_OK;
  int cop_max = 0;
  for (int i = 0; i < s.groups; ++i) {
    if (g[i].cop % 128 || g[i].cin_off % 16) return OP_OK;
    cop_max = cop_max > g[i].cop ? cop_max : g[i].cop;
  }
  PairTiling tl;
  if (!pair_tiling(2 * NPB * 16, 7, s.n, s.h, s.w, s.groups, cop_max, tl)) return OP_OK;
  static bool attr = false;
  if (!attr) {
    OP_HIP_CHECK(hipFuncSetAttribute((const void*)conv_pair_bf16x3<7, NPB>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     160 * 1024));
    attr = true;
  }
  *taken = 1;
  const int lds = 6 * 4 * 128 * 16 + 4 * tl.nh * 1024;
  const unsigned blocks = tl.xpu ? 8u * (unsigned)((tl.per_unit + tl.xpu - 1) / tl.xpu)
                                 : (unsigned)(tl.units * tl.per_unit);
  hipLaunchKernelGGL((conv_pair_bf16x3<7, NPB>), dim3(blocks), dim3(512), lds, st, s, g[0], s.groups > 1 ? g[1] : g[0],
                     tl);
  OP_AFTER_LAUNCH("conv_pair_bf16x3", st);
  OP_HIP_CHECK(hipGetLastError());
  return OP_OK;
}

}  // namespace op
