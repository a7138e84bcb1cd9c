// 3xBF16-split direct convolution for gfx950 (the fast path of models/CocoPoseNet.py:132-262).
//
// Every f32 value x is carried as the pair (hi, lo) = (bf16(x), bf16(x - hi)); a product is formed
// from the three significant partial products hi*hi + hi*lo + lo*hi on v_mfma_f32_32x32x16_bf16
// with f32 accumulation (~16 significant bits per product; the dropped lo*lo term is 2^-16
// relative).  Measured against float64 over the whole 92-layer network: 3e-5 max abs error on
// O(1) maps (the parity tests hold it to the north star's 1e-3).  Throughput: 3 bf16 MFMAs per
// k-step = 5.3x the f32-MFMA rate.
//
// Split activation format (same 4 B/element as f32, NHWC with a zero halo): per pixel, every
// group of 8 channels is 16 B of hi followed by 16 B of lo.  The producing conv's epilogue writes
// it directly.  Weights are pre-split on the host and packed in four planes per (c16, tap):
// [c16][tap][plane = 2*k-half + (hi|lo)][co][8 bf16], so a wave's A-operand reads (lanes = 32
// consecutive channels, 16 B apart) are LDS-bank-conflict-free.  The pixel operand rows are
// XOR-swizzled per 16-B part on the gather side (part ^ ((px >> 2) & 3)) for the same reason.
//
// Workgroup = 4 waves; wave w owns CB x PB blocks of 32 output channels x 32 pixels; the 4 waves
// share the channel tile.  Per (tap, 16-channel) step the workgroup stages the weight tile
// (CB*2 KiB) and each wave its own 32-pixel operand rows (PB*2 KiB) into LDS with
// global_load_lds (per-lane source addresses do the im2col gather; the LDS image is linear),
// through a 3-deep ring: stage it+2 is issued right after the barrier of step it, so the copies
// run two steps (2 x 24 MFMAs) ahead.  One raw s_barrier + counted vmcnt per step.
#include "common.hpp"
#include "cvlinear.hpp"

namespace op {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));

#define LDS_PTR(p) ((__attribute__((address_space(3))) void*)(p))

// Epilogue shared by the split kernels: bias, ReLU, split store (+ optional dense f32 copy).
// Lane holds pixel (lane & 31) of each 32-pixel block and, per register group q, output
// channels 8q + 4*(lane>>5) .. +3 of each 32-channel block (32x32 C/D map).
template <int CB, int PB>
__device__ __forceinline__ void store_tile(const SplitConvShape& s, const SplitConvGroup& g, floatx16 (&acc)[CB][PB],
                                           int co_base, int px_base, int total, int hw, int lane) {
  const int l32 = lane & 31, hi = lane >> 5;
  const int wp_out = s.w + 2 * s.pout;
  const int hp_out = s.h + 2 * s.pout;
#pragma unroll
  for (int pb = 0; pb < PB; ++pb) {
    const int p = px_base + pb * 32 + l32;
    if (p < 0 || p >= total) continue;
    const int n = p / hw;
    const int rem = p - n * hw;
    const int y = rem / s.w;
    const int x = rem - y * s.w;
    char* optr = (char*)g.out + ((int64_t)(n * hp_out + y + s.pout) * wp_out + (x + s.pout)) * (int64_t)s.cs_out * 4;
    float* o32 = g.out32 ? g.out32 + (int64_t)p * s.cs_out32 : nullptr;
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int co = co_base + cb * 32 + 8 * q + 4 * hi;
        if (co >= g.cout_store) continue;
        const floatx4 bv = *(const floatx4*)(g.bias + co);
        floatx4 v;
        u16x4 vh, vl;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float f = acc[cb][pb][4 * q + e] + bv[e];
          if (s.relu) f = f > 0.0f ? f : 0.0f;
          v[e] = f;
          const __bf16 h16 = (__bf16)f;
          const __bf16 l16 = (__bf16)(f - (float)h16);
          vh[e] = __builtin_bit_cast(unsigned short, h16);
          vl[e] = __builtin_bit_cast(unsigned short, l16);
        }
        char* d = optr + (co >> 3) * 32 + (co & 7) * 2;
        *(u16x4*)d = vh;
        *(u16x4*)(d + 16) = vl;
        if (o32) *(floatx4*)(o32 + g.out32_off + co) = v;
      }
    }
  }
}

template <int KS, int CB, int PB>
__global__ __launch_bounds__(256, 2) void conv_bf16x3(SplitConvShape s, SplitConvGroup g0, SplitConvGroup g1) {
  constexpr int KSQ = KS * KS;
  constexpr int R = KS / 2;
  constexpr int W_BYTES = CB * 32 * 64;      // weight tile per step
  constexpr int X_BYTES = PB * 32 * 64;      // one wave's pixel operand rows per step
  constexpr int STAGE = W_BYTES + 4 * X_BYTES;
  constexpr int NX = PB * 2;                 // glds per wave for X (16 pixels x 64 B each)
  constexpr int NW = W_BYTES / 4096;         // glds per wave for W (4 waves x 1 KiB each)
  static_assert(W_BYTES % 4096 == 0, "CB must be a multiple of 2");
  __shared__ __attribute__((aligned(16))) char lds[3 * STAGE];

  const SplitConvGroup g = blockIdx.z == 0 ? g0 : g1;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int co_base = blockIdx.y * (CB * 32);
  if (co_base >= g.cop) return;  // whole workgroup
  const int hw = s.h * s.w;
  const int total = s.n * hw;
  const int px_base = (blockIdx.x * 4 + wave) * (PB * 32);
  const int wp_in = s.w + 2 * s.pin;
  const int hp_in = s.h + 2 * s.pin;
  const int64_t in_pix_bytes = (int64_t)s.cs_in * 4;

  // per-lane gather sources: X glds i, lane L -> pixel px_base + i*16 + (L>>2), part (L&3)
  const char* xsrc[NX];
#pragma unroll
  for (int i = 0; i < NX; ++i) {
    int p = px_base + i * 16 + (lane >> 2);
    if (p >= total) p = total - 1;
    const int n = p / hw;
    const int rem = p - n * hw;
    const int y = rem / s.w;
    const int x = rem - y * s.w;
    // LDS slot (lane & 3) of pixel (i*16 + lane/4) holds global part (slot ^ ((px >> 2) & 3))
    const int pl = i * 16 + (lane >> 2);
    xsrc[i] = (const char*)g.in + ((int64_t)(n * hp_in + y + s.pin - R) * wp_in + (x + s.pin - R)) * in_pix_bytes +
              (((lane & 3) ^ ((pl >> 2) & 3)) * 16);
  }
  // weight pieces: piece k (= wave*NW + j) -> plane k / (CB/2), 64-channel half k % (CB/2)
  const char* wsrc[NW];
#pragma unroll
  for (int j = 0; j < NW; ++j) {
    const int k = wave * NW + j;
    wsrc[j] = (const char*)g.w + ((int64_t)(k / (CB / 2)) * g.cop + co_base + (k % (CB / 2)) * 64 + lane) * 16;
  }
  const int64_t wstep = (int64_t)g.cop * 64;
  const int n_it = s.c16 * KSQ;

  auto stage = [&](int it, int buf) {
    const int c = it / KSQ;
    const int t = it - c * KSQ;
    const int ky = t / KS;
    const int kx = t - ky * KS;
    const int64_t xoff = ((int64_t)ky * wp_in + kx) * in_pix_bytes + c * 64;
    char* base = lds + buf * STAGE;
#pragma unroll
    for (int j = 0; j < NW; ++j)
      __builtin_amdgcn_global_load_lds((const void*)(wsrc[j] + (int64_t)it * wstep),
                                       LDS_PTR(base + (wave * NW + j) * 1024), 16, 0, 0);
#pragma unroll
    for (int i = 0; i < NX; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(xsrc[i] + xoff), LDS_PTR(base + W_BYTES + wave * X_BYTES + i * 1024),
                                       16, 0, 0);
  };

  floatx16 acc[CB][PB];
#pragma unroll
  for (int cb = 0; cb < CB; ++cb)
#pragma unroll
    for (int pb = 0; pb < PB; ++pb)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[cb][pb][r] = 0.0f;

  const int l32 = lane & 31, hi = lane >> 5;
  stage(0, 0);
  if (n_it > 1) stage(1, 1);
  int buf = 0;
  for (int it = 0; it < n_it; ++it) {
    // this wave's copies for step `it` have landed once at most one younger stage is in flight
    if (it + 1 < n_it)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NW + NX) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's copies for `it` landed; everyone is done with it-1
    asm volatile("" ::: "memory");  // keep the next stage's LDS writes and this step's reads below the barrier
    if (it + 2 < n_it) stage(it + 2, buf == 0 ? 2 : buf - 1);
    const char* base = lds + buf * STAGE;
    bf16x8 ah[CB], al[CB], bh[PB], bl[PB];
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) {
      const char* a = base + (2 * hi) * (CB * 512) + (cb * 32 + l32) * 16;
      ah[cb] = *(const bf16x8*)a;
      al[cb] = *(const bf16x8*)(a + CB * 512);
    }
#pragma unroll
    for (int pb = 0; pb < PB; ++pb) {
      const int pl = pb * 32 + l32;
      const char* b = base + W_BYTES + wave * X_BYTES + pl * 64;
      const int sw = (pl >> 2) & 3;
      bh[pb] = *(const bf16x8*)(b + (((2 * hi) ^ sw) * 16));
      bl[pb] = *(const bf16x8*)(b + (((2 * hi + 1) ^ sw) * 16));
    }
#pragma unroll
    for (int cb = 0; cb < CB; ++cb)
#pragma unroll
      for (int pb = 0; pb < PB; ++pb) {
        acc[cb][pb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[cb], bh[pb], acc[cb][pb], 0, 0, 0);
        acc[cb][pb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[cb], bl[pb], acc[cb][pb], 0, 0, 0);
        acc[cb][pb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[cb], bh[pb], acc[cb][pb], 0, 0, 0);
      }
    buf = buf == 2 ? 0 : buf + 1;
  }

  store_tile<CB, PB>(s, g, acc, co_base, px_base, total, hw, lane);
}

template <int KS, int CB, int PB>
static int launch_bf16x3_t(const SplitConvShape& s, const SplitConvGroup* g, hipStream_t st) {
  const int64_t total = (int64_t)s.n * s.h * s.w;
  const int cop_max = s.groups > 1 ? (g[0].cop > g[1].cop ? g[0].cop : g[1].cop) : g[0].cop;
  dim3 grid((unsigned)((total + 4 * PB * 32 - 1) / (4 * PB * 32)), (unsigned)((cop_max + CB * 32 - 1) / (CB * 32)),
            (unsigned)s.groups);
  hipLaunchKernelGGL((conv_bf16x3<KS, CB, PB>), grid, dim3(256), 0, st, s, g[0], s.groups > 1 ? g[1] : g[0]);
  OP_AFTER_LAUNCH("conv_bf16x3<KS", st);
  OP_HIP_CHECK(hipGetLastError());
  return OP_OK;
}

int launch_conv_bf16x3(const SplitConvShape& s, const SplitConvGroup* g, hipStream_t st) {
  if (s.c16 <= 0 || (s.ks != 1 && s.ks != 3 && s.ks != 7) || s.pin < s.ks / 2 || s.cs_in % 16 || s.cs_out % 8) {
    set_error("launch_conv_bf16x3: unsupported shape");
    return OP_ERR_INVALID;
  }
  bool wide = true;
  for (int i = 0; i < s.groups; ++i) {
    if (g[i].cop % 64 || g[i].cout_store % 4 || g[i].cout_store > g[i].cop || g[i].cin_off % 16) {
      set_error("launch_conv_bf16x3: channel padding");
      return OP_ERR_INVALID;
    }
    if (g[i].cop % 128) wide = false;
  }
  // chunk-planar tensors (the stage buffers of stages 2-6): conv_m16_bf16x3 only
  if (s.in_planar || s.out_planar) {
    int taken = 0;
    const int rc = s.ks == 7 && s.halo_mode == 4 ? launch_conv_big(s, g, st, &taken) : OP_OK;
    if (rc || taken) return rc;
    set_error("launch_conv_bf16x3: chunk-planar tensors need the conv_m16 7x7 kernel");
    return OP_ERR_INVALID;
  }
  // conv algo 4 (default): the shared-weight halo kernels (conv_big.hip), then the co-split halo
  // kernel for the shapes they leave (the 1x1 convs, narrow maps); algo 3: the co-split halo
  // kernel first; algo 0 / anything neither takes: the per-tap gather kernel below
  if (s.halo_mode == 4) {
    int taken = 0;
    const int rc = launch_conv_big(s, g, st, &taken);
    if (rc || taken) return rc;
  }
  if (s.halo_mode == 3 || s.halo_mode == 4) {
    int taken = 0;
    const int rc = launch_conv_halo(s, g, st, &taken);
    if (rc || taken) return rc;
  }
  if (wide) {
    switch (s.ks) {
      case 1: return launch_bf16x3_t<1, 4, 2>(s, g, st);
      case 3: return launch_bf16x3_t<3, 4, 2>(s, g, st);
      default: return launch_bf16x3_t<7, 4, 2>(s, g, st);
    }
  }
  switch (s.ks) {
    case 1: return launch_bf16x3_t<1, 2, 2>(s, g, st);
    case 3: return launch_bf16x3_t<3, 2, 2>(s, g, st);
    default: return launch_bf16x3_t<7, 2, 2>(s, g, st);
  }
}

// ---- split-format helpers ----
__device__ __forceinline__ void split8(const float* v, u16x4& h0, u16x4& h1, u16x4& l0, u16x4& l1) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const __bf16 hh = (__bf16)v[e];
    const __bf16 ll = (__bf16)(v[e] - (float)hh);
    const unsigned short hb = __builtin_bit_cast(unsigned short, hh);
    const unsigned short lb = __builtin_bit_cast(unsigned short, ll);
    if (e < 4) {
      h0[e] = hb;
      l0[e] = lb;
    } else {
      h1[e - 4] = hb;
      l1[e - 4] = lb;
    }
  }
}

__device__ __forceinline__ float bf16_to_f(unsigned short b) { return __uint_as_float((unsigned)b << 16); }

// 8 channels (one 32-B group) of a split pixel -> f32 (hi + lo; exact in f32).
__device__ __forceinline__ void unsplit8(const char* p, float* v) {
  const u16x4 h0 = *(const u16x4*)p, h1 = *(const u16x4*)(p + 8);
  const u16x4 l0 = *(const u16x4*)(p + 16), l1 = *(const u16x4*)(p + 24);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    v[e] = bf16_to_f(h0[e]) + bf16_to_f(l0[e]);
    v[e + 4] = bf16_to_f(h1[e]) + bf16_to_f(l1[e]);
  }
}

__device__ __forceinline__ void store_split8(char* p, const float* v) {
  u16x4 h0, h1, l0, l1;
  split8(v, h0, h1, l0, l1);
  *(u16x4*)p = h0;
  *(u16x4*)(p + 8) = h1;
  *(u16x4*)(p + 16) = l0;
  *(u16x4*)(p + 24) = l1;
}

// 2x2 max-pool on split tensors (reconstructed values compared; the winner re-split is its own pair).
__global__ __launch_bounds__(256) void maxpool2_split(const char* __restrict__ in, int pin, char* __restrict__ out,
                                                      int pout, int n, int h, int w, int c8) {
  const int oh = h / 2, ow = w / 2;
  const int64_t total = (int64_t)n * oh * ow * c8;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int cc = (int)(i % c8);
  int64_t p = i / c8;
  const int ox = (int)(p % ow);
  p /= ow;
  const int oy = (int)(p % oh);
  const int nn = (int)(p / oh);
  const int wpi = w + 2 * pin, hpi = h + 2 * pin;
  const int64_t pix = (int64_t)c8 * 32;
  const char* b = in + ((int64_t)(nn * hpi + 2 * oy + pin) * wpi + (2 * ox + pin)) * pix + cc * 32;
  float v0[8], v1[8], v2[8], v3[8], r[8];
  unsplit8(b, v0);
  unsplit8(b + pix, v1);
  unsplit8(b + (int64_t)wpi * pix, v2);
  unsplit8(b + (int64_t)wpi * pix + pix, v3);
#pragma unroll
  for (int e = 0; e < 8; ++e) r[e] = fmaxf(fmaxf(v0[e], v1[e]), fmaxf(v2[e], v3[e]));
  const int wpo = ow + 2 * pout, hpo = oh + 2 * pout;
  store_split8(out + ((int64_t)(nn * hpo + oy + pout) * wpo + (ox + pout)) * pix + cc * 32, r);
}

int launch_maxpool2_split(const float* in, int32_t pin, float* out, int32_t pout, int32_t n, int32_t h, int32_t w,
                          int32_t c, hipStream_t st) {
  if ((h & 1) || (w & 1) || (c & 7)) {
    set_error("maxpool2_split: odd size");
    return OP_ERR_INVALID;
  }
  const int64_t total = (int64_t)n * (h / 2) * (w / 2) * (c / 8);
  hipLaunchKernelGGL(maxpool2_split, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, (const char*)in, pin,
                     (char*)out, pout, n, h, w, c / 8);
  OP_AFTER_LAUNCH("maxpool2_split", st);
  OP_HIP_CHECK(hipGetLastError());
  return OP_OK;
}

// (n,3,h,w) f32 -> padded (n, h+2, w+2, 16) split, zero halo and zero channels 3..15.
__global__ __launch_bounds__(256) void nchw_to_split16(const float* __restrict__ x, char* __restrict__ out, int n, int h,
                                                       int w) {
  const int wp = w + 2, hp = h + 2;
  const int64_t total = (int64_t)n * hp * wp;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int px = (int)(i % wp);
  const int py = (int)((i / wp) % hp);
  const int nn = (int)(i / ((int64_t)wp * hp));
  float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, z[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const int y = py - 1, xx = px - 1;
  if (y >= 0 && y < h && xx >= 0 && xx < w) {
    const int64_t plane = (int64_t)h * w;
    const float* b = x + (int64_t)nn * 3 * plane + (int64_t)y * w + xx;
    v[0] = b[0];
    v[1] = b[plane];
    v[2] = b[2 * plane];
  }
  store_split8(out + i * 64, v);
  store_split8(out + i * 64 + 32, z);
}

// 16-B piece i of pixel p (32 threads per pixel of a 128-channel slice: the reads are one
// contiguous run per pixel; the writes land in 4 * c16 planes, merged into lines in L2)
__global__ __launch_bounds__(256) void split_to_planar(const char* __restrict__ in, char* __restrict__ out, int32_t n,
                                                       int32_t h, int32_t w, int32_t pad, int32_t cs, int32_t c16) {
  const int pieces = 4 * c16;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)n * h * w * pieces) return;
  const int pc = (int)(i % pieces);
  const int64_t P = i / pieces;
  const int hw = h * w;
  const int f = (int)(P / hw), pp = (int)(P - (int64_t)f * hw);
  const int y = pp / w, x = pp - (pp / w) * w;
  const int hp = h + 2 * pad, wp = w + 2 * pad;
  const int64_t fb = (int64_t)f * hp * wp * cs * 4, pix = (int64_t)(y + pad) * wp + x + pad;
  const uint4 v = *(const uint4*)(in + fb + pix * cs * 4 + pc * 16);
  *(uint4*)(out + fb + (int64_t)pc * hp * wp * 16 + pix * 16) = v;
}

int launch_split_to_planar(const float* in, float* out, int32_t n, int32_t h, int32_t w, int32_t pad, int32_t cs,
                           int32_t c16, hipStream_t st) {
  if (cs % 16 || c16 * 16 > cs || n < 1) {
    set_error("split_to_planar: bad channel range");
    return OP_ERR_INVALID;
  }
  const int64_t items = (int64_t)n * h * w * 4 * c16;
  hipLaunchKernelGGL(split_to_planar, dim3((unsigned)((items + 255) / 256)), dim3(256), 0, st, (const char*)in,
                     (char*)out, n, h, w, pad, cs, c16);
  OP_AFTER_LAUNCH("split_to_planar", st);
  OP_HIP_CHECK(hipGetLastError());
  return OP_OK;
}

int launch_nchw_to_split16(const float* x, float* out, int32_t n, int32_t h, int32_t w, hipStream_t st) {
  const int64_t total = (int64_t)n * (h + 2) * (w + 2);
  hipLaunchKernelGGL(nchw_to_split16, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, x, (char*)out, n, h, w);
  OP_AFTER_LAUNCH("nchw_to_split16", st);
  OP_HIP_CHECK(hipGetLastError());
  return OP_OK;
}

// split (n, h+2, w+2, 16) network input written straight from the uint8 frames (preprocess fused).

__global__ __launch_bounds__(256) void preprocess_split16(const uint8_t* __restrict__ frames, int64_t frame_bytes,
                                                          int64_t row_stride, int n, int sh, int sw, int dh, int dw,
                                                          char* __restrict__ out, float div) {
  const int wp = dw + 2, hp = dh + 2;
  const int64_t total = (int64_t)n * hp * wp;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int px = (int)(i % wp);
  const int py = (int)((i / wp) % hp);
  const int nn = (int)(i / ((int64_t)wp * hp));
  float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, z[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const int dy = py - 1, dx = px - 1;
  if (dy >= 0 && dy < dh && dx >= 0 && dx < dw) {
    const uint8_t* src = frames + (int64_t)nn * frame_bytes;
    for (int c = 0; c < 3; ++c) v[c] = cv_linear_norm(src, row_stride, sh, sw, dx, dy, dw, dh, c, div);
  }
  store_split8(out + i * 64, v);
  store_split8(out + i * 64 + 32, z);
}

int launch_preprocess_split(const uint8_t* frames, int64_t frame_bytes, int64_t row_stride, int32_t n, int32_t sh,
                            int32_t sw, int32_t dh, int32_t dw, float* out, hipStream_t st, float div) {
  const int64_t total = (int64_t)n * (dh + 2) * (dw + 2);
  hipLaunchKernelGGL(preprocess_split16, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, frames, frame_bytes,
                     row_stride, n, sh, sw, dh, dw, (char*)out, div);
  OP_AFTER_LAUNCH("preprocess_split16", st);
  OP_HIP_CHECK(hipGetLastError());
  return OP_OK;
}

// f32 maps (n, lh, lw, cs) dense (paf at 0, heat at heat_off) -> planar (n,38,h,w), (n,19,h,w).
__global__ __launch_bounds__(256) void extract_maps32(const float* __restrict__ m, int cs, int heat_off, int n, int h,
                                                      int w, float* __restrict__ paf, float* __restrict__ heat) {
  const int64_t total = (int64_t)n * 57 * h * w;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int x = (int)(i % w);
  const int y = (int)((i / w) % h);
  const int c = (int)((i / ((int64_t)w * h)) % 57);
  const int nn = (int)(i / ((int64_t)w * h * 57));
  const float* px = m + (((int64_t)nn * h + y) * w + x) * cs;
  if (c < 38)
    paf[(((int64_t)nn * 38 + c) * h + y) * w + x] = px[c];
  else
    heat[(((int64_t)nn * 19 + (c - 38)) * h + y) * w + x] = px[heat_off + c - 38];
}

int launch_extract_maps32(const float* m, int32_t cs, int32_t heat_off, int32_t n, int32_t h, int32_t w, float* paf,
                          float* heat, hipStream_t st) {
  const int64_t total = (int64_t)n * 57 * h * w;
  hipLaunchKernelGGL(extract_maps32, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, m, cs, heat_off, n, h, w,
                     paf, heat);
  OP_AFTER_LAUNCH("extract_maps32", st);
  OP_HIP_CHECK(hipGetLastError());
  return OP_OK;
}

}  // namespace op
