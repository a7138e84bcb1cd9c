// conv_m16r_bf16x3: 3x3 convs on v_mfma_f32_16x16x32_bf16 with register-resident weights and a
// double-buffered LDS halo (round 3; the default 3x3 kernel where the launch is large enough).
//
// Same arithmetic as conv_m16k_bf16x3 (conv_m16k.hpp): K = 32 of one MFMA is one tap over a PAIR of
// 16-channel input chunks (lane group g = lane / 16: chunk g / 2, channel half g % 2), three bf16
// products per f32-accurate MAC (hi*hi, hi*lo, lo*hi), accumulated per output in the order (chunk
// pair, tap, hi*hi, hi*lo, lo*hi) -- so every output is BIT-IDENTICAL to conv_m16k's.  What changes
// is where the operands come from:
//
// * A (weights): each wave owns 32 output channels and loads their fragments for a step straight
//   from global memory (L2) into VGPRs, two steps ahead -- no shared weight ring in LDS, so no
//   LDS-DMA staging of weights, no A reads from LDS and no workgroup barrier per tap (conv_m16k
//   pays all three every step: weight staging and the per-step barrier were ~8.5 % of its time in
//   round 2's traffic experiments).
// * B (pixels): every wave of the workgroup covers the SAME pixel tile (TR rows x 16*TCB columns),
//   read from an LDS halo of both chunks of the pair (8 planes of 16 B per pixel, tight pitch,
//   compile-time tap offsets: one ds_read_b128 with an immediate offset per fragment).  The halo is
//   double-buffered: the next chunk pair's halo is streamed in by LDS-DMA during taps 0..4 of the
//   current pair, so the once-per-pair reload (~10 % of conv_m16k's time) leaves the critical path;
//   one workgroup barrier per chunk pair swaps the buffers.
//
// NW waves x 32 channels = the workgroup's channel tile (NW = 8: 256 channels, one workgroup per
// CU; NW = 4: 128 channels, two per CU).  POOL: fused 2x2 max-pool epilogue (tile rows r, r + 1 =
// blocks pb, pb + TCB; columns = lanes l, l ^ 1).  Layer semantics: models/CocoPoseNet.py:136-163
// (conv + ReLU, the pools after conv1_2 / conv2_2 / conv3_4).
#include <type_traits>

#include "conv_big.hpp"

namespace op {

// LDS-DMA from inline asm: invisible to the compiler's waitcnt pass, so the B-fragment reads of the
// current buffer do not wait for the next buffer's pieces (with the builtin the pass cannot tell the
// two apart and would serialise them).  Writes M0; nothing else in this kernel uses M0.
__device__ __forceinline__ void dma16(const void* gsrc, uint32_t lds_byte) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(gsrc), "s"(lds_byte) : "memory");
}

template <int NW, int TCB, int TR, bool POOL, int CBW = 2>
__global__ __launch_bounds__(NW * 64, 2) void conv_m16r_bf16x3(SplitConvShape s, SplitConvGroup g0,
                                                                   SplitConvGroup g1, BigTiling tl) {
  // CBW = 16-channel blocks per wave: 2 (waves split the channels only and cover the whole pixel
  // tile) or 4 (NW = 4: two channel halves x two pixel halves -- every B fragment read from LDS
  // feeds twice the MFMAs, every weight fragment is loaded by two waves)
  static_assert(CBW == 2 || (CBW == 4 && NW == 4), "wave tiles: 32 channels, or 64 at NW 4");
  constexpr int PGN = CBW / 2;              // pixel groups
  constexpr int NCS = NW / PGN;             // channel slices
  constexpr int NPT = TR * TCB;             // 16-px blocks of the tile
  constexpr int NPX = NPT / PGN;            // 16-px blocks per wave
  constexpr int TC = 16 * TCB;
  constexpr int PITCH = TC + 2;
  constexpr int HROWS = TR + 2;
  constexpr int NH = (HROWS * PITCH + 63) / 64;  // 1-KiB pieces per halo plane
  constexpr int HPLANE = NH * 1024;
  constexpr int HBUF = 8 * HPLANE;               // 2 chunks x 4 planes (hi/lo x 2 channel halves)
  constexpr int PIECES = 8 * NH / NW;            // halo pieces per wave per chunk pair
  constexpr int HSTEPS = 5;                      // taps during which the next pair's halo is issued
  constexpr int PPS = (PIECES + HSTEPS - 1) / HSTEPS;
  constexpr int CW = NW * 32;
  static_assert((8 * NH) % NW == 0, "halo pieces split evenly over the waves");
  static_assert(NPT % PGN == 0 && (!POOL || (NPX % (2 * TCB)) == 0), "whole (pooled) row pairs per wave");
  static_assert(!POOL || (TR % 2 == 0), "pooled tiles hold whole row pairs");
  extern __shared__ __attribute__((aligned(16))) char lds[];  // [2][8 planes][NH KiB]

  const int lin = blockIdx.x;
  int unit, widx;
  if (tl.xpu) {
    // XCD set su runs weight sets su*P .. su*P+P-1; consecutive slots of one XCD are one pixel
    // tile's P channel tiles, so its input is read from HBM once per XCD set
    // (per_xcd > 0: XCD xo of the set runs the contiguous pixel tiles [xo * per_xcd, +per_xcd), so
    // vertically adjacent tiles run on one XCD at about the same time and share their halo rows
    // in its L2; else consecutive tiles go to consecutive XCDs of the set)
    const int xcd = lin & 7, slot = lin >> 3;
    const int P = tl.pair > 1 ? tl.pair : 1;
    const int su = xcd / tl.xpu, q = slot / P, xo = xcd - su * tl.xpu;
    unit = su * P + (slot - q * P);
    widx = tl.per_xcd > 0 ? xo * tl.per_xcd + q : q * tl.xpu + xo;
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
  const int y0 = ty * TR, x0 = (tix - ty * tl.tiles_x) * TC;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int cs = wave % NCS, pg = wave / NCS;  // channel slice, pixel group
  const int l16 = lane & 15, kg = lane >> 4;
  const int csel = kg >> 1, khalf = kg & 1;
  const int wp_in = s.w + 2 * s.pin;
  const int hp_in = s.h + 2 * s.pin;
  const int64_t pix_bytes = (int64_t)s.cs_in * 4;
  const char* const fbase = (const char*)g.in + (int64_t)frame * hp_in * wp_in * pix_bytes;
  const uint32_t lds0 = (uint32_t)(size_t)(__attribute__((address_space(3))) char*)lds;

  // ---- A: this wave's 16*CBW channels; weights [c16][tap][plane 2*khalf + hi/lo][cop][8 bf16] ----
  const int64_t wplane = (int64_t)g.cop * 16;
  const int cw0 = co0 + cs * 16 * CBW;
  const char* const wlane = (const char*)g.w + ((int64_t)csel * 9 * 4 + 2 * khalf) * wplane + (int64_t)(cw0 + l16) * 16;
  const int ncp = s.c16 / 2;
  const int n_it = ncp * 9;
  typedef bf16x8g AFrag[2 * CBW];  // [cb * 2 + hl]
  constexpr int NB = CBW == 2 ? 3 : 2;  // weight buffers: 2 or 1 steps ahead (64-channel waves: registers)
  AFrag abuf[NB];
  auto load_a = [&](int it, AFrag& a) {
    if (it >= n_it) it = n_it - 1;  // the last steps' prefetch re-reads the final step (unused)
    const int cp = it / 9, t = it - cp * 9;
    const char* p = wlane + (int64_t)((2 * cp * 9 + t) * 4) * wplane;
#pragma unroll
    for (int cb = 0; cb < CBW; ++cb) {
      a[2 * cb] = *(const bf16x8g*)(p + cb * 256);
      a[2 * cb + 1] = *(const bf16x8g*)(p + wplane + cb * 256);
    }
  };

  // ---- B: halo of one chunk pair; wave w DMAs pieces j = w, w + NW, ... (plane j / NH, piece j % NH) ----
  auto halo_piece = [&](int cp, int buf, int k) {  // k-th of this wave's PIECES pieces
    const int j = wave + k * NW;
    const int plane = j / NH, i = j - (j / NH) * NH;
    const int cj = plane >> 2, pl = plane & 3;
    const int slot = i * 64 + lane;
    const int hr = slot / PITCH, hc = slot - (slot / PITCH) * PITCH;
    const int yy = min(y0 - 1 + hr + s.pin, hp_in - 1), xx = min(x0 - 1 + hc + s.pin, wp_in - 1);
    const char* src = fbase + (int64_t)(yy * wp_in + xx) * pix_bytes + (2 * cp + cj) * 64 + pl * 16;
    dma16(src, lds0 + (uint32_t)(buf * HBUF + plane * HPLANE + i * 1024));
  };

  const int rows_here = min(TR, s.h - y0);
  const int cols_here = min(TC, s.w - x0);
  // this lane's halo byte offset within a buffer: plane of (chunk csel, half khalf, hi), pixel l16
  // of the wave's first block (pixel group pg: tile rows pg * NPX / TCB ..)
  const int bl0 = (csel * 4 + 2 * khalf) * HPLANE + (l16 + pg * (NPX / TCB) * PITCH) * 16;

  floatx4 acc[CBW][NPX];
#pragma unroll
  for (int cb = 0; cb < CBW; ++cb)
#pragma unroll
    for (int pb = 0; pb < NPX; ++pb) acc[cb][pb] = floatx4{0.f, 0.f, 0.f, 0.f};

  // prologue: chunk pair 0's halo into buffer 0, the first NB - 1 steps' weights
#pragma unroll
  for (int k = 0; k < PIECES; ++k) halo_piece(0, 0, k);
#pragma unroll
  for (int k = 0; k < NB - 1; ++k) load_a(k, abuf[k]);
  wait_vmcnt<0>();
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  // one chunk pair (9 taps); P = the pair's parity, so step it = 9 cp + t uses weight buffer
  // it % NB = (9 P + t) % NB at compile time (NB 3: t % 3; NB 2: the parity alternates per pair)
  auto chunk_pair = [&](int cp, auto parity) {
    constexpr int P = decltype(parity)::value;
    const int buf = cp & 1;
    const char* const hb = lds + buf * HBUF + bl0;
    const bool next = cp + 1 < ncp;
    // B fragments one 16-px block ahead, across tap boundaries (the first block of tap t + 1 is
    // read during the last block of tap t)
    // B fragments one block ahead (round 5: two blocks ahead, three register sets, measured neutral:
    // profiles/r05/ab_r05j_m16r_b_two_ahead_neutral.log)
    constexpr int NBB = 2;
    auto boff = [&](int idx) {  // byte offset of block idx's B fragment (compile-time after unrolling)
      const int t1 = idx / NPX, pb1 = idx % NPX;
      return (((t1 / 3) + pb1 / TCB) * PITCH + (t1 % 3) + (pb1 % TCB) * 16) * 16;
    };
    bf16x8g bh[NBB], bl[NBB];
#pragma unroll
    for (int k = 0; k < NBB - 1; ++k) {
      bh[k] = *(const bf16x8g*)(hb + boff(k));
      bl[k] = *(const bf16x8g*)(hb + boff(k) + HPLANE);
    }
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int it = cp * 9 + t;
      load_a(it + NB - 1, abuf[(9 * P + t + NB - 1) % NB]);  // NB - 1 steps ahead
      if (t < HSTEPS && next) {
#pragma unroll
        for (int k = t * PPS; k < (t + 1) * PPS && k < PIECES; ++k) halo_piece(cp + 1, buf ^ 1, k);
      }
      const AFrag& a = abuf[(9 * P + t) % NB];
#pragma unroll
      for (int pb = 0; pb < NPX; ++pb) {
        const int idx = t * NPX + pb, cur = idx % NBB;
        if (idx + NBB - 1 < 9 * NPX) {
          const int o1 = boff(idx + NBB - 1);
          bh[(idx + NBB - 1) % NBB] = *(const bf16x8g*)(hb + o1);
          bl[(idx + NBB - 1) % NBB] = *(const bf16x8g*)(hb + o1 + HPLANE);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int cb = 0; cb < CBW; ++cb) {
          acc[cb][pb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2 * cb], bh[cur], acc[cb][pb], 0, 0, 0);
          acc[cb][pb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2 * cb], bl[cur], acc[cb][pb], 0, 0, 0);
          acc[cb][pb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2 * cb + 1], bh[cur], acc[cb][pb], 0, 0, 0);
        }
      }
    }
    if (next) {
      // this wave's pieces of the next pair were issued by tap HSTEPS - 1; younger than them are
      // only the weight loads of taps HSTEPS..8 (2 CBW each, load_a): waiting down to that many
      // outstanding covers every piece and keeps those weight loads in flight across the barrier
      // (round 3 waited down to 8, which also drained half of them -- advisor finding;
      // M16R_WAIT8 builds that for the A/B)
#ifdef M16R_WAIT8
      constexpr int kYounger = 8;
#else
      constexpr int kYounger = (9 - HSTEPS) * 2 * CBW;
#endif
      static_assert(kYounger >= 0 && kYounger <= 63, "vmcnt literal");
      wait_vmcnt<kYounger>();
      __builtin_amdgcn_s_barrier();  // every wave's pieces landed; this pair's buffer is free
      asm volatile("" ::: "memory");
    }
  };
  if constexpr (NB == 3) {
    for (int cp = 0; cp < ncp; ++cp) chunk_pair(cp, std::integral_constant<int, 0>());
  } else {
    for (int cp = 0; cp < ncp; cp += 2) {
      chunk_pair(cp, std::integral_constant<int, 0>());
      if (cp + 1 < ncp) chunk_pair(cp + 1, std::integral_constant<int, 1>());
    }
  }
  wait_vmcnt<0>();

  if constexpr (POOL) {
    const int wp_out = s.w / 2 + 2 * s.pout;
    const int hp_out = s.h / 2 + 2 * s.pout;
#pragma unroll
    for (int pb = 0; pb < NPX; ++pb) {
      if ((pb / TCB) & 1) continue;  // odd tile rows are the pair partners
      const int r = pg * (NPX / TCB) + pb / TCB, c = (pb % TCB) * 16 + l16;
      const int y = y0 + r, x = x0 + c;
      const bool store = r < rows_here && c < cols_here && (l16 & 1) == 0;
      char* optr = (char*)g.out +
                   ((int64_t)(frame * hp_out + y / 2 + s.pout) * wp_out + (x / 2 + s.pout)) * (int64_t)s.cs_out * 4;
#pragma unroll
      for (int cb = 0; cb < CBW; ++cb) {
        const int co = cw0 + cb * 16 + 4 * kg;
        const bool live = co < g.cout_store;
        const floatx4 bv = live ? *(const floatx4*)(g.bias + co) : floatx4{0.f, 0.f, 0.f, 0.f};
        u16x4g vh, vl;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float m = 0.0f;
#pragma unroll
          for (int k = 0; k < 2; ++k) {
            float f = acc[cb][pb + k * TCB][e] + bv[e];
            if (s.relu) f = f > 0.0f ? f : 0.0f;
            const __bf16 h16 = (__bf16)f;
            const float rc = (float)h16 + (float)(__bf16)(f - (float)h16);
            m = k == 0 ? rc : fmaxf(m, rc);
          }
          m = fmaxf(m, __shfl_xor(m, 1));
          const __bf16 h16 = (__bf16)m;
          const __bf16 l16v = (__bf16)(m - (float)h16);
          vh[e] = __builtin_bit_cast(unsigned short, h16);
          vl[e] = __builtin_bit_cast(unsigned short, l16v);
        }
        if (store && live) {
          char* d = optr + (co >> 3) * 32 + (co & 7) * 2;
          *(u16x4g*)d = vh;
          *(u16x4g*)(d + 16) = vl;
        }
      }
    }
    return;
  }

  const int wp_out = s.w + 2 * s.pout;
  const int hp_out = s.h + 2 * s.pout;
#pragma unroll
  for (int pb = 0; pb < NPX; ++pb) {
    const int r = pg * (NPX / TCB) + pb / TCB, c = (pb % TCB) * 16 + l16;
    const bool live = r < rows_here && c < cols_here;
    const int y = y0 + r, x = x0 + c;
    char* optr = (char*)g.out + ((int64_t)(frame * hp_out + y + s.pout) * wp_out + (x + s.pout)) * (int64_t)s.cs_out * 4;
    float* o32 = g.out32 ? g.out32 + ((int64_t)(frame * s.h + y) * s.w + x) * s.cs_out32 + g.out32_off : nullptr;
#pragma unroll
    for (int cb = 0; cb < CBW; ++cb) {
      const int co = cw0 + cb * 16 + 4 * kg;
      floatx4 v;
      uint32_t own[4], w[4];
      split_pair_swap(acc[cb][pb], co < g.cop ? *(const floatx4*)(g.bias + co) : floatx4{0.f, 0.f, 0.f, 0.f}, s.relu, v,
                      own, w);
      if (!live || co >= g.cout_store) continue;
      store_split_group(optr, co, kg, g.cout_store, own, w);
      if (o32) *(floatx4*)(o32 + co) = v;
    }
  }
}

template <int NW, int TCB, int TR, bool POOL, int CBW>
static int launch_t(const SplitConvShape& s, const SplitConvGroup& g0, const SplitConvGroup& g1, const BigTiling& tl,
                    hipStream_t st) {
  constexpr int PITCH = 16 * TCB + 2;
  constexpr int NH = ((TR + 2) * PITCH + 63) / 64;
  constexpr int LDS = 2 * 8 * NH * 1024;
  static_assert(LDS <= 160 * 1024 / (8 / NW), "workgroups per CU x LDS fits 160 KiB");
  static bool attr = false;
  if (!attr) {
    OP_HIP_CHECK(hipFuncSetAttribute((const void*)conv_m16r_bf16x3<NW, TCB, TR, POOL, CBW>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, LDS));
    attr = true;
  }
  const unsigned blocks = tl.xpu ? 8u * (unsigned)((tl.per_unit + tl.xpu - 1) / tl.xpu * std::max(tl.pair, 1))
                                 : (unsigned)(tl.units * tl.per_unit);
  hipLaunchKernelGGL((conv_m16r_bf16x3<NW, TCB, TR, POOL, CBW>), dim3(blocks), dim3(NW * 64), LDS, st, s, g0, g1, tl);
  return OP_OK;
}

// Tiling + launch of conv_m16r_bf16x3 for a 3x3 split-format conv; *taken = 0 when the shape is
// outside it (the caller falls back to conv_m16k / conv_big).  mode: OP_M16R (0 off, 1 default:
// NW 4; 8: NW 8 where Co is a multiple of 256).
int launch_conv_m16r(const SplitConvShape& s, const SplitConvGroup* g, bool pool, hipStream_t st, int* taken) {
  *taken = 0;
  static const int mode = getenv("OP_M16R") ? atoi(getenv("OP_M16R")) : 1;
  if (!mode || s.ks != 3 || s.pin < 1 || s.cs_in % 16 || (s.c16 & 1) || s.halo_mode != 4 || !s.regw) return OP_OK;
  int cop_max = 0;
  for (int i = 0; i < s.groups; ++i) {
    if (g[i].cop % 128 || g[i].cin_off % 16) return OP_OK;
    cop_max = std::max(cop_max, g[i].cop);
  }
  if (pool && (s.groups != 1 || (s.h & 1) || (s.w & 1) || !s.relu)) return OP_OK;
  // NW = 4 (128 channels, two workgroups per CU with independent per-pair barriers) by default: in
  // an interleaved A/B it ran the 3x3 class 2 % faster than 256-channel workgroups on the
  // 256/512-channel layers (profiles/r03/ab_r03a_m16r_nw.log); OP_M16R=8 selects those
  const int nw = mode == 8 ? 8 : 4;
  if (nw == 8)
    for (int i = 0; i < s.groups; ++i)
      if (g[i].cop % 256) return OP_OK;
  // 4 x 48 tiles: 46- / 92- / 184-wide maps at 96 % column use
  constexpr int TCB = 3, TR = 4;
  BigTiling t{};
  t.tc = 16 * TCB;
  t.tr = TR;
  t.tiles_x = (s.w + t.tc - 1) / t.tc;
  t.tiles_y = (s.h + TR - 1) / TR;
  t.co_tiles = cop_max / (nw * 32);
  t.units = s.groups * t.co_tiles;
  t.per_unit = s.n * t.tiles_y * t.tiles_x;
  // channel tiles per XCD set: the most whose weights (split format, 4 B per weight) stay under
  // OP_M16R_PAIR_KB (0 = one tile per set, the input read from HBM once per tile).  5000 KB (pairs
  // for conv3_x / conv4_2 / conv4_3 / conv5_1, all four tiles of conv4_1): non-pooled reads 887 ->
  // 632 MiB FETCH_SIZE per launch, pooled 1752 -> 1446, the 3x3 class 21.73 -> 21.53 ms per 114
  // frames (profiles/r03/ab_r03d_*.log, fetch_r03d_*.txt); a 2600-KB cap pairs fewer layers and
  // measured no gain
  static const int pair_kb = getenv("OP_M16R_PAIR_KB") ? atoi(getenv("OP_M16R_PAIR_KB")) : 5000;
  const int64_t tile_wbytes = (int64_t)nw * 32 * s.c16 * 16 * 9 * 4;
  t.pair = 1;
  for (int p = t.co_tiles; p > 1; --p)
    if (t.co_tiles % p == 0 && p * tile_wbytes <= (int64_t)pair_kb * 1024 && (t.units / p) <= 8 &&
        8 % (t.units / p) == 0) {
      t.pair = p;
      break;
    }
  t.xpu = (t.units / t.pair <= 8 && 8 % (t.units / t.pair) == 0) ? 8 * t.pair / t.units : 0;
  if (!t.xpu) t.pair = 1;
  // contiguous pixel tiles per XCD (default; OP_M16R_XMAJ=0: consecutive tiles on consecutive XCDs):
  // 3x3 fabric reads 1325 -> 998 MB per non-pooled launch, 3035 -> 1980 pooled, the 3x3 class
  // 21.13 -> 20.94 ms per 114 frames (profiles/r03/ab_r03i_*.log, tcc_r03i_*.txt)
  static const int xmaj = getenv("OP_M16R_XMAJ") ? atoi(getenv("OP_M16R_XMAJ")) : 1;
  t.per_xcd = xmaj && t.xpu ? (t.per_unit + t.xpu - 1) / t.xpu : 0;
  // enough workgroups to fill the chip several times; small launches keep conv_m16k (split-K)
  const int64_t wgs = (int64_t)t.units * t.per_unit;
  if (wgs < (nw == 8 ? 2 * 256 : 4 * 256)) return OP_OK;
  *taken = 1;
  const SplitConvGroup& g1 = s.groups > 1 ? g[1] : g[0];
  census_add(pool ? OP_CENSUS_3X3_R_POOL : nw == 8 ? OP_CENSUS_3X3_R256 : OP_CENSUS_3X3_R128);
  // wave tile: 32 channels x the whole tile (CBW 2), or 64 channels x half the tile (CBW 4, NW 4)
  static const int cbw = getenv("OP_M16R_CBW") ? atoi(getenv("OP_M16R_CBW")) : 2;
  int rc;
  if (nw == 8)
    rc = pool ? launch_t<8, TCB, TR, true, 2>(s, g[0], g1, t, st) : launch_t<8, TCB, TR, false, 2>(s, g[0], g1, t, st);
  else if (cbw == 4)
    rc = pool ? launch_t<4, TCB, TR, true, 4>(s, g[0], g1, t, st) : launch_t<4, TCB, TR, false, 4>(s, g[0], g1, t, st);
  else
    rc = pool ? launch_t<4, TCB, TR, true, 2>(s, g[0], g1, t, st) : launch_t<4, TCB, TR, false, 2>(s, g[0], g1, t, st);
  if (rc != OP_OK) return rc;
  OP_AFTER_LAUNCH("conv_m16r_bf16x3", st);
  OP_HIP_CHECK(hipGetLastError());
  return OP_OK;
}

}  // namespace op
