// Co-split halo convolution (3xBF16 split, gfx950) — the conv kernel of the split path.
//
// Workgroup = NWV waves; wave w owns output channels [co_base + 32w, +32) for ALL pixels of a
// rectangular tile of TR rows x TC columns of one frame (NPB blocks of 32 pixels, TR*TC <= NPB*32).
//  * Activations: for each 16-channel chunk the tile's input window plus its (KS-1)-pixel halo is
//    copied once into LDS as 4 planes (hi/lo x k-half) of 16 B per pixel, and every tap reads its
//    shifted window from there (reuse TR*TC*KS^2 / halo pixels: ~14x for 7x7, ~6x for 3x3).
//    B-operand reads are consecutive 16-B slots: bank-conflict-free.
//  * Weights: each wave streams ONLY its own 32-channel slice (2 KiB per (tap, chunk), packed in
//    4 planes) through a private 3-deep LDS ring with global_load_lds; nothing is shared, so the
//    main loop has no barrier -- each wave waits on its own counted vmcnt.  The only barriers are
//    the two around each chunk's halo reload.
//  * MFMA: v_mfma_f32_32x32x16_bf16, 3 products (hi*hi, hi*lo, lo*hi) per k-step into one f32
//    accumulator per 32-pixel block.
#include "common.hpp"

namespace op {

typedef __bf16 bf16x8h __attribute__((ext_vector_type(8)));
typedef unsigned short u16x4h __attribute__((ext_vector_type(4)));

#define LDS_PTR_H(p) ((__attribute__((address_space(3))) void*)(p))

template <int KS, int NPB, int NWV>
__global__ __launch_bounds__(NWV * 64, 2) void conv_halo_bf16x3(SplitConvShape s, SplitConvGroup g0, SplitConvGroup g1,
                                                                 HaloTiling tl) {
  constexpr int KSQ = KS * KS;
  constexpr int R = KS / 2;
  constexpr int W_SLOT = 2048;                 // one wave's weight tile per (tap, chunk)
  constexpr int W_RING = 3 * W_SLOT;           // per wave
  extern __shared__ __attribute__((aligned(16))) char lds[];  // [halo: 4 planes x hplane][W rings]

  const SplitConvGroup g = blockIdx.z == 0 ? g0 : g1;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int co_wave = blockIdx.y * (NWV * 32) + wave * 32;
  if (blockIdx.y * (NWV * 32) >= g.cop) return;  // whole workgroup
  const bool wave_active = co_wave < g.cop;      // uniform per wave; still joins the barriers
  const int tiles_per_frame = tl.tiles_y * tl.tiles_x;
  const int frame = blockIdx.x / tiles_per_frame;
  const int tix = blockIdx.x - frame * tiles_per_frame;
  const int ty = tix / tl.tiles_x, tx = tix - ty * tl.tiles_x;
  const int y0 = ty * tl.tr, x0 = tx * tl.tc;
  const int hcols = tl.tc + KS - 1;
  const int hrows = tl.tr + KS - 1;
  const int hpix = hrows * hcols;
  const int hplane = tl.nh * 1024;
  const int wp_in = s.w + 2 * s.pin;
  const int hp_in = s.h + 2 * s.pin;
  const int64_t pix_bytes = (int64_t)s.cs_in * 4;
  // halo pixel (hr, hc) <-> padded input (y0 + pin - R + hr, x0 + pin - R + hc) of this frame
  const char* hbase = (const char*)g.in + ((int64_t)(frame * hp_in + y0 + s.pin - R) * wp_in + (x0 + s.pin - R)) * pix_bytes;
  char* wring = lds + 4 * hplane + wave * W_RING;

  const int l32 = lane & 31, hi = lane >> 5;
  // weights: glds j covers planes 2j (lanes 0-31) and 2j+1 (lanes 32-63) of this wave's 32 channels
  const char* wsrc = (const char*)g.w + ((int64_t)hi * g.cop + (wave_active ? co_wave : 0) + l32) * 16;
  const int64_t wplane = (int64_t)g.cop * 16;
  const int64_t wstep = 4 * wplane;
  const int n_it = s.c16 * KSQ;

  // output pixels of this lane: tile-local p = pb*32 + l32 -> (r, c)
  int q0[NPB];
#pragma unroll
  for (int pb = 0; pb < NPB; ++pb) {
    const int p = pb * 32 + l32;
    int r = p / tl.tc, c = p - (p / tl.tc) * tl.tc;
    if (r >= tl.tr) {  // pad lanes of the last block: read a valid halo pixel, never stored
      r = 0;
      c = 0;
    }
    q0[pb] = r * hcols + c;
  }

  auto stage_w = [&](int it) {
    char* dst = wring + (it % 3) * W_SLOT;  // slot of the unclamped step (the clamped copy is never read)
    if (it >= n_it) it = n_it - 1;
    const char* src = wsrc + (int64_t)it * wstep;
    __builtin_amdgcn_global_load_lds((const void*)src, LDS_PTR_H(dst), 16, 0, 0);
    __builtin_amdgcn_global_load_lds((const void*)(src + 2 * wplane), LDS_PTR_H(dst + 1024), 16, 0, 0);
  };

  floatx16 acc[NPB];
#pragma unroll
  for (int pb = 0; pb < NPB; ++pb)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[pb][r] = 0.0f;

  stage_w(0);
  stage_w(1);
  int it = 0;
  for (int c = 0; c < s.c16; ++c) {
    // ---- halo reload: everyone is done with the previous chunk's halo ----
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    for (int pl = wave; pl < 4; pl += NWV) {
      char* dst = lds + pl * hplane;
      for (int i = 0; i < tl.nh; ++i) {
        int q = i * 64 + lane;
        if (q >= hpix) q = hpix - 1;
        int hr = q / hcols, hc = q - (q / hcols) * hcols;
        // rows / cols past this frame's padded image only feed masked (out-of-map) pixels: clamp
        // the source so a partial last tile never reads outside the frame (or the buffer)
        if (y0 + s.pin - R + hr > hp_in - 1) hr = hp_in - 1 - (y0 + s.pin - R);
        if (x0 + s.pin - R + hc > wp_in - 1) hc = wp_in - 1 - (x0 + s.pin - R);
        __builtin_amdgcn_global_load_lds((const void*)(hbase + ((int64_t)hr * wp_in + hc) * pix_bytes + c * 64 + pl * 16),
                                         LDS_PTR_H(dst + i * 1024), 16, 0, 0);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // own halo pieces (and in-flight weights) landed
    __builtin_amdgcn_s_barrier();                        // every wave's pieces landed
    asm volatile("" ::: "memory");
#pragma unroll 1
    for (int t = 0; t < KSQ; ++t, ++it) {
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");  // W(it) landed; W(it+1) may be in flight
      stage_w(it + 2);
      const char* wb = wring + (it % 3) * W_SLOT;
      const bf16x8h ah = *(const bf16x8h*)(wb + (2 * hi) * 512 + l32 * 16);
      const bf16x8h al = *(const bf16x8h*)(wb + (2 * hi + 1) * 512 + l32 * 16);
      const int ky = t / KS, kx = t - (t / KS) * KS;
      const int toff = ky * hcols + kx;
#pragma unroll
      for (int pb = 0; pb < NPB; ++pb) {
        const char* b = lds + (q0[pb] + toff) * 16;
        const bf16x8h bh = *(const bf16x8h*)(b + (2 * hi) * hplane);
        const bf16x8h bl = *(const bf16x8h*)(b + (2 * hi + 1) * hplane);
        acc[pb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc[pb], 0, 0, 0);
        acc[pb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc[pb], 0, 0, 0);
        acc[pb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc[pb], 0, 0, 0);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain the trailing (never read) weight copies
  if (!wave_active) return;

  // ---- epilogue: bias, ReLU, split store (+ dense f32 copy) ----
  const int wp_out = s.w + 2 * s.pout;
  const int hp_out = s.h + 2 * s.pout;
#pragma unroll
  for (int pb = 0; pb < NPB; ++pb) {
    const int p = pb * 32 + l32;
    const int r = p / tl.tc, cc = p - (p / tl.tc) * tl.tc;
    const int y = y0 + r, x = x0 + cc;
    if (r >= tl.tr || y >= s.h || x >= s.w) continue;
    char* optr = (char*)g.out + ((int64_t)(frame * hp_out + y + s.pout) * wp_out + (x + s.pout)) * (int64_t)s.cs_out * 4;
    float* o32 = g.out32 ? g.out32 + ((int64_t)(frame * s.h + y) * s.w + x) * s.cs_out32 : nullptr;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int co = co_wave + 8 * q + 4 * hi;
      if (co >= g.cout_store) continue;
      const floatx4 bv = *(const floatx4*)(g.bias + co);
      floatx4 v;
      u16x4h vh, vl;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float f = acc[pb][4 * q + e] + bv[e];
        if (s.relu) f = f > 0.0f ? f : 0.0f;
        v[e] = f;
        const __bf16 h16 = (__bf16)f;
        const __bf16 l16 = (__bf16)(f - (float)h16);
        vh[e] = __builtin_bit_cast(unsigned short, h16);
        vl[e] = __builtin_bit_cast(unsigned short, l16);
      }
      char* d = optr + (co >> 3) * 32 + (co & 7) * 2;
      *(u16x4h*)d = vh;
      *(u16x4h*)(d + 16) = vl;
      if (o32) *(floatx4*)(o32 + g.out32_off + co) = v;
    }
  }
}

// Choose the tile for an H x W map: TR full-width rows (TC = W) while W fits a tile, else one row
// split into equal segments; NPB = 32-pixel blocks per tile.
static HaloTiling make_tiling(int h, int w, int ks, int npb) {
  HaloTiling t;
  const int cap = npb * 32;
  if (w <= cap) {
    t.tc = w;
    t.tr = cap / w;
    if (t.tr > h) t.tr = h;
  } else {
    const int segs = (w + cap - 1) / cap;
    t.tc = (w + segs - 1) / segs;
    t.tr = 1;
  }
  t.tiles_y = (h + t.tr - 1) / t.tr;
  t.tiles_x = (w + t.tc - 1) / t.tc;
  const int hpix = (t.tr + ks - 1) * (t.tc + ks - 1);
  t.nh = (hpix + 63) / 64;
  return t;
}

static int lds_bytes(const HaloTiling& t, int nwv) { return 4 * t.nh * 1024 + nwv * 3 * 2048; }

template <int KS, int NPB, int NWV>
static int launch_halo_cs_t(const SplitConvShape& s, const SplitConvGroup* g, const HaloTiling& tl, hipStream_t st) {
  const int cop_max = s.groups > 1 ? (g[0].cop > g[1].cop ? g[0].cop : g[1].cop) : g[0].cop;
  const int lds = lds_bytes(tl, NWV);
  static int attr = 0;
  if (lds > attr) {
    OP_HIP_CHECK(hipFuncSetAttribute((const void*)conv_halo_bf16x3<KS, NPB, NWV>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = 160 * 1024;
  }
  dim3 grid((unsigned)(s.n * tl.tiles_y * tl.tiles_x), (unsigned)((cop_max + NWV * 32 - 1) / (NWV * 32)),
            (unsigned)s.groups);
  hipLaunchKernelGGL((conv_halo_bf16x3<KS, NPB, NWV>), grid, dim3(NWV * 64), lds, st, s, g[0],
                     s.groups > 1 ? g[1] : g[0], tl);
  OP_AFTER_LAUNCH("conv_halo_bf16x3", st);
  OP_HIP_CHECK(hipGetLastError());
  return OP_OK;
}

template <int KS, int NPB>
static int dispatch_nwv(const SplitConvShape& s, const SplitConvGroup* g, const HaloTiling& tl, hipStream_t st,
                        int nwv) {
  if (nwv == 2) return launch_halo_cs_t<KS, NPB, 2>(s, g, tl, st);
  return launch_halo_cs_t<KS, NPB, 4>(s, g, tl, st);
}

// The split-path convolution: picks the tile and instantiation.  *taken = 0 when the shape is
// outside this kernel (caller falls back to the gather kernel).
int launch_conv_halo(const SplitConvShape& s, const SplitConvGroup* g, hipStream_t st, int* taken) {
  *taken = 0;
  if (s.cs_in % 16 || s.pin < s.ks / 2) return OP_OK;
  int cop_max = 0;
  for (int i = 0; i < s.groups; ++i) {
    if (g[i].cop % 64 || g[i].cin_off % 16) return OP_OK;
    cop_max = cop_max > g[i].cop ? cop_max : g[i].cop;
  }
  const int nwv = cop_max >= 128 ? 4 : 2;
  // 6 or 8 pixel blocks per tile, whichever wastes fewer MFMA lanes on this map width
  const HaloTiling t6 = make_tiling(s.h, s.w, s.ks, 6), t8 = make_tiling(s.h, s.w, s.ks, 8);
  const double u6 = (double)s.h * s.w / ((double)t6.tiles_y * t6.tiles_x * 6 * 32);
  const double u8 = (double)s.h * s.w / ((double)t8.tiles_y * t8.tiles_x * 8 * 32);
  const bool use8 = u8 > u6 + 0.02;
  const HaloTiling tl = use8 ? t8 : t6;
  if (lds_bytes(tl, nwv) * 2 > 160 * 1024) return OP_OK;  // keep 2 workgroups per CU
  *taken = 1;
  if (use8) {
    switch (s.ks) {
      case 1: return dispatch_nwv<1, 8>(s, g, tl, st, nwv);
      case 3: return dispatch_nwv<3, 8>(s, g, tl, st, nwv);
      default: return dispatch_nwv<7, 8>(s, g, tl, st, nwv);
    }
  }
  switch (s.ks) {
    case 1: return dispatch_nwv<1, 6>(s, g, tl, st, nwv);
    case 3: return dispatch_nwv<3, 6>(s, g, tl, st, nwv);
    default: return dispatch_nwv<7, 6>(s, g, tl, st, nwv);
  }
}

}  // namespace op
