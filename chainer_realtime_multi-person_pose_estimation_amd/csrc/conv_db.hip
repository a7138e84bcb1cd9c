// Double-buffered halo convolution on 8-channel chunks (3xBF16 split, gfx950): 3x3 and 7x7.
//
// conv_big.hip reloads its halo tile every 16 input channels with the whole CU waiting (measured:
// 19 % of the 3x3 time, 5 % of the 7x7).  Here a chunk is 8 channels, so two chunks' halos fit in
// the LDS one 16-channel halo took, and chunk q+1's halo is copied (global_load_lds) while chunk q
// computes.  The v_mfma_f32_32x32x16_bf16 K = 16 is fed with two consecutive (chunk, tap)
// ELEMENTS of the flat sequence e = chunk * KSQ + tap: lanes 0-31 hold element 2p, lanes 32-63
// element 2p+1 (possibly the next chunk's tap 0, read from the other halo buffer) -- no tap is
// wasted for odd KSQ except a single zero half at the very end.
//
// Workgroup = 8 waves, one per CU: CW output channels x a TR x TC tile.  Wave w: channel half
// w / PG (64 channels, 2 blocks of 32) x pixel group w % PG (NPB blocks of 32 pixels).  Weights
// per element: 2 planes (hi, lo) x CW channels x 16 B, an 8-slot LDS ring, one barrier per pair.
// In-order vmcnt accounting: pair p waits for the weight copy issued at pair p-2, i.e. all but
// the ops issued after it (the halo copies of pairs p-2 and p-1 and one weight copy); a chunk's
// halo is issued >= 3 pairs before its first use, so that wait also covers it.
#include <cstdlib>
#include <vector>

#include "common.hpp"

namespace op {

typedef __bf16 bf16x8d __attribute__((ext_vector_type(8)));
typedef unsigned short u16x4d __attribute__((ext_vector_type(4)));

#define LDS_PTR_D(p) ((__attribute__((address_space(3))) void*)(p))

struct DbTiling {
  int32_t tr, tc, tiles_y, tiles_x;
  int32_t pitch;  // LDS halo row pitch in 16-B slots (tc + 16 for ks > 1: conflict-free row wraps)
  int32_t nh;     // 1-KiB halo pieces per plane
  int32_t units, co_tiles, per_unit, xpu;
};


template <int KS, int NPB, int CW, bool POOL>
__global__ __launch_bounds__(512, 1) void conv_db_bf16x3(SplitConvShape s, SplitConvGroup g0, SplitConvGroup g1,
                                                         DbTiling tl) {
  constexpr int KSQ = KS * KS;
  constexpr int R = KS / 2;
  constexpr int CH = CW / 64;       // 64-channel halves
  constexpr int PG = 8 / CH;        // pixel groups
  constexpr int PLANE_W = CW * 16;  // one weight plane of one element
  constexpr int ESLOT = 2 * PLANE_W;
  constexpr int RING = 8;
  extern __shared__ __attribute__((aligned(16))) char lds[];  // [W ring][halo buffer 0][halo buffer 1]

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
  const int co0 = (unit - grp * tl.co_tiles) * CW;
  const SplitConvGroup g = grp == 0 ? g0 : g1;
  if (co0 >= g.cop) return;
  const int tpf = tl.tiles_y * tl.tiles_x;
  const int frame = widx / tpf;
  const int tix = widx - frame * tpf;
  const int ty = tix / tl.tiles_x;
  const int y0 = ty * tl.tr, x0 = (tix - ty * tl.tiles_x) * tl.tc;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ch = wave / PG, pg = wave % PG;
  const int l32 = lane & 31, hi = lane >> 5;
  const int hplane = tl.nh * 1024;
  char* const halo = lds + RING * ESLOT;
  const int wp_in = s.w + 2 * s.pin;
  const int hp_in = s.h + 2 * s.pin;
  const int64_t pix_bytes = (int64_t)s.cs_in * 4;
  const char* const fbase = (const char*)g.in + (int64_t)frame * hp_in * wp_in * pix_bytes;
  const int n_c8 = s.c16 * 2;
  const int E = n_c8 * KSQ;
  const int NP = (E + 1) >> 1;

  // weight piece of this wave: j = wave % (4*CH) -> element 2p + j/(2*CH), plane (j/CH)&1, half j%CH
  // (CH = 1: waves 4-7 repeat waves 0-3's copies so every wave issues one op per pair)
  const int64_t wplane = (int64_t)g.cop * 16;
  const int64_t wstep = 4 * wplane;
  const int wj = wave % (4 * CH);
  const int w_eo = wj / (2 * CH), w_plane = (wj / CH) & 1, w_half = wj % CH;
  const char* const wsrc = (const char*)g.w + w_plane * wplane + ((int64_t)co0 + 64 * w_half + lane) * 16;
  const int wdst = w_plane * PLANE_W + w_half * 1024;
  auto stage_w = [&](int p) {
    const int eu = 2 * p + w_eo;
    const int e = eu < E ? eu : E - 1;  // trailing copies: never read
    const int c8 = e / KSQ, t = e - (e / KSQ) * KSQ;
    const char* src = wsrc + ((int64_t)(c8 >> 1) * KSQ + t) * wstep + (c8 & 1) * 2 * wplane;
    __builtin_amdgcn_global_load_lds((const void*)src, LDS_PTR_D(lds + (eu % RING) * ESLOT + wdst), 16, 0, 0);
  };
  // halo of chunk q (8 channels = 32 B of each pixel: hi 16 B, lo 16 B) into buffer q & 1;
  // returns this wave's op count
  auto stage_halo = [&](int q) -> int {
    const char* src0 = fbase + q * 32;
    char* dst0 = halo + (q & 1) * 2 * hplane;
    int k = 0;
    for (int i = wave; i < 2 * tl.nh; i += 8, ++k) {
      const int plane = i >= tl.nh ? 1 : 0, idx = i - plane * tl.nh;
      const int sl = idx * 64 + lane;
      const int hr = sl / tl.pitch, hc = sl - (sl / tl.pitch) * tl.pitch;
      int yy = y0 - R + hr + s.pin, xx = x0 - R + hc + s.pin;
      yy = yy < hp_in - 1 ? yy : hp_in - 1;  // slots past the padded image only feed masked outputs
      xx = xx < wp_in - 1 ? xx : wp_in - 1;
      __builtin_amdgcn_global_load_lds((const void*)(src0 + plane * 16 + ((int64_t)yy * wp_in + xx) * pix_bytes),
                                       LDS_PTR_D(dst0 + plane * hplane + idx * 1024), 16, 0, 0);
    }
    return k;
  };

  const int rows_here = min(tl.tr, s.h - y0);
  const int cols_here = min(tl.tc, s.w - x0);
  int q0[NPB];
#pragma unroll
  for (int pb = 0; pb < NPB; ++pb) {
    const int p = (pg * NPB + pb) * 32 + l32;
    const int r = p / tl.tc, c = p - (p / tl.tc) * tl.tc;
    q0[pb] = (r < rows_here && c < cols_here) ? r * tl.pitch + c : 0;  // pad lanes: never stored
  }

  floatx16 acc[2][NPB];
#pragma unroll
  for (int cb = 0; cb < 2; ++cb)
#pragma unroll
    for (int pb = 0; pb < NPB; ++pb)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[cb][pb][e] = 0.0f;

  stage_w(0);
  stage_w(1);
  stage_halo(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  int k_p2 = 0, k_p1 = 0;  // halo ops this wave issued at pairs p-2, p-1
  int next_h = 1;
  const int wlane = (ch * 64 + l32) * 16;
#pragma unroll 1
  for (int p = 0; p < NP; ++p) {
    if (p >= 2) wait_vm_dyn(k_p2 + 1 + k_p1);  // the weight copy of pair p (issued at p-2) landed ...
    __builtin_amdgcn_s_barrier();              // ... for every wave; pair p-1's slots are free
    asm volatile("" ::: "memory");
    stage_w(p + 2);
    int k_now = 0;
    if (next_h < n_c8 && 2 * (p - 1) >= (next_h - 1) * KSQ) {  // chunk next_h-2 is done: its buffer is free
      k_now = stage_halo(next_h);
      ++next_h;
    }
    // this lane's element
    const int eu = 2 * p + hi;
    const bool live = eu < E;
    const int e = live ? eu : 2 * p;
    const int c8 = e / KSQ, t = e - (e / KSQ) * KSQ;
    const int toff = (t / KS) * tl.pitch + (t - (t / KS) * KS);
    const char* bp = halo + (c8 & 1) * 2 * hplane + toff * 16;
    const char* wb = lds + (eu % RING) * ESLOT + wlane;
    bf16x8d ah[2], al[2];
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      ah[cb] = live ? *(const bf16x8d*)(wb + cb * 512) : bf16x8d{};
      al[cb] = live ? *(const bf16x8d*)(wb + PLANE_W + cb * 512) : bf16x8d{};
    }
    bf16x8d bh[2], bl[2];
    bh[0] = *(const bf16x8d*)(bp + q0[0] * 16);
    bl[0] = *(const bf16x8d*)(bp + hplane + q0[0] * 16);
#pragma unroll
    for (int pb = 0; pb < NPB; ++pb) {
      const int cur = pb & 1;
      if (pb + 1 < NPB) {
        bh[cur ^ 1] = *(const bf16x8d*)(bp + q0[pb + 1] * 16);
        bl[cur ^ 1] = *(const bf16x8d*)(bp + hplane + q0[pb + 1] * 16);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        acc[cb][pb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[cb], bh[cur], acc[cb][pb], 0, 0, 0);
        acc[cb][pb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[cb], bl[cur], acc[cb][pb], 0, 0, 0);
        acc[cb][pb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[cb], bh[cur], acc[cb][pb], 0, 0, 0);
      }
    }
    k_p2 = k_p1;
    k_p1 = k_now;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain the trailing (never read) copies

  if constexpr (POOL) {
    // fused 2x2 max-pool (tiles are 32 wide: block pb is a tile row), as in conv_big.hip
    const int wp_out = s.w / 2 + 2 * s.pout;
    const int hp_out = s.h / 2 + 2 * s.pout;
#pragma unroll
    for (int pb = 0; pb < NPB; pb += 2) {
      const int r = pg * NPB + pb;
      const int x = x0 + l32;
      const bool store = r < rows_here && x < s.w && (l32 & 1) == 0;
      const int y = y0 + r;
      char* optr = (char*)g.out +
                   ((int64_t)(frame * hp_out + y / 2 + s.pout) * wp_out + (x / 2 + s.pout)) * (int64_t)s.cs_out * 4;
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int co = co0 + ch * 64 + cb * 32 + 8 * q + 4 * hi;
          const bool lv = co < g.cout_store;
          const floatx4 bv = lv ? *(const floatx4*)(g.bias + co) : floatx4{0.f, 0.f, 0.f, 0.f};
          u16x4d vh, vl;
#pragma unroll
          for (int e2 = 0; e2 < 4; ++e2) {
            float m = 0.0f;
#pragma unroll
            for (int k = 0; k < 2; ++k) {
              float f = acc[cb][pb + k][4 * q + e2] + bv[e2];
              if (s.relu) f = f > 0.0f ? f : 0.0f;
              const __bf16 h16 = (__bf16)f;
              const float rc = (float)h16 + (float)(__bf16)(f - (float)h16);
              m = k == 0 ? rc : fmaxf(m, rc);
            }
            m = fmaxf(m, __shfl_xor(m, 1));
            const __bf16 h16 = (__bf16)m;
            const __bf16 l16 = (__bf16)(m - (float)h16);
            vh[e2] = __builtin_bit_cast(unsigned short, h16);
            vl[e2] = __builtin_bit_cast(unsigned short, l16);
          }
          if (store && lv) {
            char* d = optr + (co >> 3) * 32 + (co & 7) * 2;
            *(u16x4d*)d = vh;
            *(u16x4d*)(d + 16) = vl;
          }
        }
    }
    return;
  }

  const int wp_out = s.w + 2 * s.pout;
  const int hp_out = s.h + 2 * s.pout;
#pragma unroll
  for (int pb = 0; pb < NPB; ++pb) {
    const int p = (pg * NPB + pb) * 32 + l32;
    const int r = p / tl.tc, cc = p - (p / tl.tc) * tl.tc;
    if (r >= rows_here || cc >= cols_here) continue;
    const int y = y0 + r, x = x0 + cc;
    char* optr = (char*)g.out + ((int64_t)(frame * hp_out + y + s.pout) * wp_out + (x + s.pout)) * (int64_t)s.cs_out * 4;
    float* o32 = g.out32 ? g.out32 + ((int64_t)(frame * s.h + y) * s.w + x) * s.cs_out32 + g.out32_off : nullptr;
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int co = co0 + ch * 64 + cb * 32 + 8 * q + 4 * hi;
        if (co >= g.cout_store) continue;
        const floatx4 bv = *(const floatx4*)(g.bias + co);
        floatx4 v;
        u16x4d vh, vl;
#pragma unroll
        for (int e2 = 0; e2 < 4; ++e2) {
          float f = acc[cb][pb][4 * q + e2] + bv[e2];
          if (s.relu) f = f > 0.0f ? f : 0.0f;
          v[e2] = f;
          const __bf16 h16 = (__bf16)f;
          const __bf16 l16 = (__bf16)(f - (float)h16);
          vh[e2] = __builtin_bit_cast(unsigned short, h16);
          vl[e2] = __builtin_bit_cast(unsigned short, l16);
        }
        char* d = optr + (co >> 3) * 32 + (co & 7) * 2;
        *(u16x4d*)d = vh;
        *(u16x4d*)(d + 16) = vl;
        if (o32) *(floatx4*)(o32 + co) = v;
      }
  }
}

// ---- host side ----
static int db_lds(int nh, int cw) { return 8 * 2 * cw * 16 + 4 * nh * 1024; }

static void db_finish(DbTiling& t, int ks, int cw, int n, int groups, int cop_max) {
  t.pitch = t.tc + (ks > 1 ? 16 * ((ks - 1 + 15) / 16) : 0);
  t.nh = ((t.tr + ks - 1) * t.pitch + 63) / 64;
  t.co_tiles = (cop_max + cw - 1) / cw;
  t.units = groups * t.co_tiles;
  t.per_unit = n * t.tiles_y * t.tiles_x;
  t.xpu = (t.units <= 8 && 8 % t.units == 0) ? 8 / t.units : 0;
}

// Tile choice as conv_big.hip: within 3 % of the best lane utilisation, the least halo re-read.
static bool db_tiling(int ks, int cap, int cw, int n, int h, int w, int groups, int cop_max, DbTiling& t) {
  struct Cand {
    int tr, tc, tiles_y, tiles_x;
    double util, amp;
  };
  std::vector<Cand> cands;
  double best = 0.0;
  for (int segs = 1; segs <= 32; ++segs) {
    const int tc = (w + segs - 1) / segs;
    if (tc > cap || tc < 1) continue;
    if (segs > 1 && (w + tc - 1) / tc != segs) continue;
    int tr = cap / tc;
    if (tr > h) tr = h;
    const int pitch = tc + (ks > 1 ? 16 : 0);
    while (tr >= 1 && db_lds(((tr + ks - 1) * pitch + 63) / 64, cw) > 160 * 1024) --tr;
    if (tr < 1) continue;
    const int tiles_y = (h + tr - 1) / tr;
    const int trb = (h + tiles_y - 1) / tiles_y;
    const double util = (double)h * w / ((double)tiles_y * segs * cap);
    const double amp = (double)(trb + ks - 1) * (tc + ks - 1) / ((double)trb * tc);
    cands.push_back({trb, tc, tiles_y, segs, util, amp});
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
  db_finish(t, ks, cw, n, groups, cop_max);
  return true;
}

template <int KS, int NPB, int CW, bool POOL>
static int launch_db_t(const SplitConvShape& s, const SplitConvGroup* g, const DbTiling& tl, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    OP_HIP_CHECK(hipFuncSetAttribute((const void*)conv_db_bf16x3<KS, NPB, CW, POOL>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  const unsigned blocks = tl.xpu ? 8u * (unsigned)((tl.per_unit + tl.xpu - 1) / tl.xpu)
                                 : (unsigned)(tl.units * tl.per_unit);
  hipLaunchKernelGGL((conv_db_bf16x3<KS, NPB, CW, POOL>), dim3(blocks), dim3(512), db_lds(tl.nh, CW), st, s, g[0],
                     s.groups > 1 ? g[1] : g[0], tl);
  OP_AFTER_LAUNCH("conv_db_bf16x3", st);
  OP_HIP_CHECK(hipGetLastError());
  return OP_OK;
}

// 3x3 / 7x7 split-path convolution with double-buffered 8-channel halos.  pool: fused 2x2
// max-pool (s.h x s.w is the conv size, the output buffer (s.h/2) x (s.w/2)).  *taken = 0 when
// the shape is outside this kernel.
int launch_conv_db(const SplitConvShape& s, const SplitConvGroup* g, hipStream_t st, bool pool, int* taken) {
  *taken = 0;
  if ((s.ks != 3 && s.ks != 7) || s.cs_in % 16 || s.pin < s.ks / 2) return OP_OK;
  int cop_max = 0;
  bool c128 = true;
  for (int i = 0; i < s.groups; ++i) {
    if (g[i].cop % 64 || g[i].cin_off % 16) return OP_OK;
    if (g[i].cop % 128) c128 = false;
    cop_max = cop_max > g[i].cop ? cop_max : g[i].cop;
  }
  DbTiling tl;
  if (pool) {
    if (s.ks != 3 || s.groups != 1 || (s.h & 1) || (s.w & 1) || !s.relu) return OP_OK;
    const int npb = c128 ? 4 : 2;  // even: window rows are blocks (pb, pb+1)
    const int cw = c128 ? 128 : 64;
    tl.tc = 32;
    tl.tr = (8 / (cw / 64)) * npb;
    tl.tiles_y = (s.h + tl.tr - 1) / tl.tr;
    tl.tiles_x = (s.w + 31) / 32;
    db_finish(tl, 3, cw, s.n, 1, cop_max);
    if (db_lds(tl.nh, cw) > 160 * 1024) return OP_OK;
    *taken = 1;
    if (c128) return launch_db_t<3, 4, 128, true>(s, g, tl, st);
    return launch_db_t<3, 2, 64, true>(s, g, tl, st);
  }
  if (!c128) {  // 64-channel layers: 8 pixel groups x 3 blocks
    if (!db_tiling(s.ks, 8 * 3 * 32, 64, s.n, s.h, s.w, s.groups, cop_max, tl)) return OP_OK;
    *taken = 1;
    if (s.ks == 3) return launch_db_t<3, 3, 64, false>(s, g, tl, st);
    return launch_db_t<7, 3, 64, false>(s, g, tl, st);
  }
  if (!db_tiling(s.ks, 4 * 6 * 32, 128, s.n, s.h, s.w, s.groups, cop_max, tl)) return OP_OK;
  *taken = 1;
  if (s.ks == 3) return launch_db_t<3, 6, 128, false>(s, g, tl, st);
  return launch_db_t<7, 6, 128, false>(s, g, tl, st);
}

}  // namespace op
