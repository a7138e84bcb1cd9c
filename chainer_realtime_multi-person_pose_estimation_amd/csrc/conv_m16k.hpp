// conv_m16k_bf16x3: the default 3x3 kernel (definition shared by two translation units so each
// instantiation can take its own LLVM scheduler flags: conv_big.hip holds <false, 2, 8> and
// <true, 2, 8>, conv_m16k_wide.hip <false, 3, 6>).  Include after conv_big.hpp.
#pragma once
#include "conv_big.hpp"

namespace op {

// ---- 3x3 on v_mfma_f32_16x16x32_bf16 with K = 32 input channels (default 3x3 kernel) ----
// One step = one tap over a PAIR of 16-channel chunks: lane group g holds k = 8g..8g+7 = chunk
// g/2 of the pair, channel half g%2.  The halo holds both chunks (8 planes); the weight ring slot
// holds the tap's weights of both chunks.  Workgroup = 4 waves (2 channel halves x 2 pixel groups,
// two workgroups per CU at <= 80 KiB), tile = 8 rows x 32 columns; wave = 64 channels x 8 blocks
// of 16 px (block b = half a tile row).  POOL: fused 2x2 max-pool epilogue (rows = blocks b, b+2).
// TCB = 16-pixel blocks per tile row: 2 (8 x 32 tiles, NPX 8) or 3 (4 x 48 tiles, NPX 6: the 46- and
// 82-wide maps, where 32-column tiles leave 28 % / 15 % of the MFMA lanes on padding).
template <bool POOL, int TCB = 2, int NPX = 8>
__global__ __launch_bounds__(256, 2) void conv_m16k_bf16x3(SplitConvShape s, SplitConvGroup g0, SplitConvGroup g1,
                                                           BigTiling tl) {
  static_assert(!POOL || TCB == 2, "the pooled epilogue pairs blocks b, b + 2");
  static_assert((2 * NPX) % TCB == 0, "whole tile rows");
  constexpr int KS = 3, KSQ = 9, R = 1;
  constexpr int CW = 128, PG = 2;
  constexpr int PLANE_W = CW * 16;
  constexpr int CHUNK_W = 4 * PLANE_W;   // one chunk's (tap) weights
  constexpr int SLOT_W = 2 * CHUNK_W;    // a step: the chunk pair
  constexpr int RING = 2;
  extern __shared__ __attribute__((aligned(16))) char lds[];  // [W ring][halo: 2 chunks x 4 planes]

  const int lin = blockIdx.x;
  int unit, widx;
  if (tl.per_xcd) {  // the weight sets of one pixel tile run side by side on one XCD: its input
    const int xcd = lin & 7, slot = lin >> 3;  // tile is fetched from HBM once, then from L2
    const int wl = slot / tl.units;
    unit = slot - wl * tl.units;
    widx = wl < tl.per_xcd ? xcd * tl.per_xcd + wl : tl.per_unit;
  } else if (tl.xpu) {
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
  const int l16 = lane & 15, kg = lane >> 4;
  const int csel = kg >> 1, khalf = kg & 1;
  const int hplane = tl.nh * 1024;
  char* const halo = lds + RING * SLOT_W;
  const int wp_in = s.w + 2 * s.pin;
  const int hp_in = s.h + 2 * s.pin;
  const int64_t pix_bytes = (int64_t)s.cs_in * 4;
  const char* const fbase = (const char*)g.in + (int64_t)frame * hp_in * wp_in * pix_bytes;

  // weights: 16 1-KiB pieces per step; wave w copies j = 4w .. 4w+3: chunk j/8, plane (j/2)%4, half j%2
  const int64_t wplane = (int64_t)g.cop * 16;
  const int64_t wstep = 4 * wplane;  // one (chunk, tap)
  // split-K (tl.ksplit > 1): chunk pairs [cp0, cp1) of this workgroup (pooled launches too, round 4:
  // conv_m16_splitk_reduce_pool then sums, pools and stores)
  const int nsplit = tl.ksplit > 1 ? tl.ksplit : 1;
  const int split = nsplit > 1 ? (int)blockIdx.y : 0;
  const int cp0 = split * (s.c16 / 2 / nsplit), cp1 = cp0 + s.c16 / 2 / nsplit;
  const int n_it = cp1 * KSQ;
  auto stage_w = [&](int it) {
    char* dst = lds + (it % RING) * SLOT_W;
    if (it >= n_it) it = n_it - 1;
    const int cp = it / KSQ, t = it - (it / KSQ) * KSQ;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int j = wave * 4 + i;
      const int cj = j >> 3, pl = (j >> 1) & 3, hf = j & 1;
      const char* src = (const char*)g.w + ((int64_t)(2 * cp + cj) * KSQ + t) * wstep + pl * wplane +
                        ((int64_t)co0 + 64 * hf + lane) * 16;
      glds16((const void*)src, dst + cj * CHUNK_W + pl * PLANE_W + hf * 1024);
    }
  };

  const int rows_here = min(tl.tr, s.h - y0);
  const int cols_here = min(tl.tc, s.w - x0);
  uint32_t qp[NPX / 2];
#pragma unroll
  for (int pb = 0; pb < NPX; ++pb) {
    const int b = pg * NPX + pb;
    const int r = b / TCB, c = (b % TCB) * 16 + l16;
    const uint32_t q = (uint32_t)(r * tl.pitch + c);  // masked lanes read their own (unused) halo slot: no bank clash
    if (pb & 1) qp[pb >> 1] |= q << 16;
    else qp[pb >> 1] = q;
  }
  auto q0 = [&](int pb) -> int { return (int)((qp[pb >> 1] >> (16 * (pb & 1))) & 0xffffu); };

  floatx4 acc[4][NPX];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb)
#pragma unroll
    for (int pb = 0; pb < NPX; ++pb) acc[cb][pb] = floatx4{0.f, 0.f, 0.f, 0.f};

  stage_w(cp0 * KSQ);
  const char* const bplane = halo + (csel * 4 + 2 * khalf) * hplane;          // hi plane; lo at + hplane
  const int wlane = csel * CHUNK_W + (2 * khalf) * PLANE_W + (ch * 64 + l16) * 16;
  // halo reload: 8 planes x nh pieces over 4 waves; wave w: planes w and w + 4 (chunk 0 / 1)
  int it = cp0 * KSQ;
  for (int cp = cp0; cp < cp1; ++cp) {
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#pragma unroll
    for (int cj = 0; cj < 2; ++cj) {
      const char* src0 = fbase + (2 * cp + cj) * 64 + wave * 16;
      char* dst = halo + (cj * 4 + wave) * hplane;
      int hr = lane / tl.pitch, hc = lane - (lane / tl.pitch) * tl.pitch;
      for (int i = 0; i < tl.nh; ++i) {
        const int yy = min(y0 - R + hr + s.pin, hp_in - 1), xx = min(x0 - R + hc + s.pin, wp_in - 1);
        glds16((const void*)(src0 + (int64_t)(yy * wp_in + xx) * pix_bytes), dst);
        dst += 1024;
        hc += 64;
        while (hc >= tl.pitch) {
          hc -= tl.pitch;
          ++hr;
        }
      }
    }
    wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#pragma unroll 1
    for (int t = 0; t < KSQ; ++t, ++it) {
      if (t > 0) {
        wait_vmcnt<0>();  // W(it): the newest copy, issued one step back ...
        __builtin_amdgcn_s_barrier();  // ... landed for every wave; slot (it+1) % 2 is free
        asm volatile("" ::: "memory");
      }
      stage_w(it + 1);
      const char* wsl = lds + (it % RING) * SLOT_W + wlane;
      bf16x8g ah[4], al[4];
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        ah[cb] = *(const bf16x8g*)(wsl + cb * 256);
        al[cb] = *(const bf16x8g*)(wsl + PLANE_W + cb * 256);
      }
      const int toff = (t / KS) * tl.pitch + (t - (t / KS) * KS);
      bf16x8g bh[2], bl[2];
      bh[0] = *(const bf16x8g*)(bplane + (q0(0) + toff) * 16);
      bl[0] = *(const bf16x8g*)(bplane + hplane + (q0(0) + toff) * 16);
#pragma unroll
      for (int pb = 0; pb < NPX; ++pb) {
        const int cur = pb & 1;
        if (pb + 1 < NPX) {
          bh[cur ^ 1] = *(const bf16x8g*)(bplane + (q0(pb + 1) + toff) * 16);
          bl[cur ^ 1] = *(const bf16x8g*)(bplane + hplane + (q0(pb + 1) + toff) * 16);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) {
          acc[cb][pb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[cb], bh[cur], acc[cb][pb], 0, 0, 0);
          acc[cb][pb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[cb], bl[cur], acc[cb][pb], 0, 0, 0);
          acc[cb][pb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[cb], bh[cur], acc[cb][pb], 0, 0, 0);
        }
      }
    }
  }
  wait_vmcnt<0>();

  if (nsplit > 1) {  // raw partials in raster order (conv_m16_splitk_reduce finishes them)
    const int wsc = max(g0.cop, g1.cop);
    float* const wsg = tl.ws + ((int64_t)split * s.groups + grp) * (int64_t)tl.total * wsc;
#pragma unroll
    for (int pb = 0; pb < NPX; ++pb) {
      const int b = pg * NPX + pb;
      const int r = b / TCB, c = (b % TCB) * 16 + l16;
      if (r >= rows_here || c >= cols_here) continue;
      const int64_t P = ((int64_t)frame * s.h + y0 + r) * s.w + x0 + c;
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        const int co = co0 + ch * 64 + cb * 16 + 4 * kg;
        if (co < g.cop) *(floatx4*)(wsg + P * wsc + co) = acc[cb][pb];
      }
    }
    return;
  }
  if constexpr (POOL) {
    // rows (b, b+2) = tile rows (r, r+1); columns (l16, l16 ^ 1) = lanes (l, l ^ 1)
    const int wp_out = s.w / 2 + 2 * s.pout;
    const int hp_out = s.h / 2 + 2 * s.pout;
#pragma unroll
    for (int pb = 0; pb < NPX; ++pb) {
      if (pb & 2) continue;
      const int b = pg * NPX + pb;
      const int r = b >> 1, c = (b & 1) * 16 + l16;
      const int y = y0 + r, x = x0 + c;
      const bool store = r < rows_here && c < cols_here && (l16 & 1) == 0;
      char* optr = (char*)g.out +
                   ((int64_t)(frame * hp_out + y / 2 + s.pout) * wp_out + (x / 2 + s.pout)) * (int64_t)s.cs_out * 4;
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        const int co = co0 + ch * 64 + cb * 16 + 4 * kg;
        const bool live = co < g.cout_store;
        const floatx4 bv = live ? *(const floatx4*)(g.bias + co) : floatx4{0.f, 0.f, 0.f, 0.f};
        u16x4g vh, vl;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float m = 0.0f;
#pragma unroll
          for (int k = 0; k < 2; ++k) {
            float f = acc[cb][pb + 2 * k][e] + bv[e];
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
    const int b = pg * NPX + pb;
    const int r = b / TCB, c = (b % TCB) * 16 + l16;
    const bool live = r < rows_here && c < cols_here;
    const int y = y0 + r, x = x0 + c;
    char* optr = (char*)g.out + ((int64_t)(frame * hp_out + y + s.pout) * wp_out + (x + s.pout)) * (int64_t)s.cs_out * 4;
    float* o32 = g.out32 ? g.out32 + ((int64_t)(frame * s.h + y) * s.w + x) * s.cs_out32 + g.out32_off : nullptr;
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      const int co = co0 + ch * 64 + cb * 16 + 4 * kg;
      floatx4 v;
      uint32_t own[4], w[4];
      split_pair_swap(acc[cb][pb], co < g.cop ? *(const floatx4*)(g.bias + co) : floatx4{0.f, 0.f, 0.f, 0.f}, s.relu,
                      v, own, w);
      if (!live || co >= g.cout_store) continue;
      store_split_group(optr, co, kg, g.cout_store, own, w);
      if (o32) *(floatx4*)(o32 + co) = v;
    }
  }
}

}  // namespace op
