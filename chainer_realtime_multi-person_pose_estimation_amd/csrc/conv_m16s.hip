// conv_m16s_bf16x3: the 7x7 stage convs (models/CocoPoseNet.py:167-260, Mconv1..Mconv5 of stages 2-6)
// with register-resident weights and a double-buffered raster halo (round 3; large launches).
//
// Same arithmetic and accumulation order as conv_m16_bf16x3 (conv_m16.hip): K = 32 of one
// v_mfma_f32_16x16x32_bf16 is a tap PAIR of one 16-channel chunk (lane group g: tap t + g/2, channel
// half g%2; the odd 49th tap pairs with zero weights), products hi*hi, hi*lo, lo*hi, summed per
// output over (chunk, tap pair) in order -- so every output is BIT-IDENTICAL to conv_m16's, and a
// frame's maps do not depend on which of the two kernels a launch picked.  What changes:
//
// * waves split the 128 output channels, not the pixels: wave w owns channels 32 (w % 4) .. + 31 of
//   pixel group w / 4 (two groups of NPXW 16-px blocks of the raster tile); its weight fragments
//   for a tap pair come straight from global memory (L2) into VGPRs, two pairs ahead -- no shared
//   weight ring in LDS, no LDS-DMA staging of weights and no workgroup barrier per tap pair;
// * the LDS holds two halo buffers: the next chunk's halo streams in by LDS-DMA during tap pairs
//   0..9 of the current chunk, so the once-per-chunk reload (about 5 % of conv_m16's time: its
//   waves all stall on it) leaves the critical path; one barrier per chunk swaps the buffers.
// Tiles are raster runs of CAP = 2 * NPXW * 16 pixels of the batch (may span two frames; each
// frame's rows carry their own 3-pixel border in the halo), at the tight pitch w + 6 so two halo
// buffers fit 160 KiB: 4 planes x 20 KiB each.
#include "conv_big.hpp"

#ifndef M16S_ABUF
#define M16S_ABUF 2  // weight fragment buffers per wave: 2 = one tap pair ahead, 3 = two
#endif

namespace op {

namespace {

// LDS-DMA from inline asm (invisible to the compiler's waitcnt pass, see conv_m16r.hip)
__device__ __forceinline__ void dma16s(const void* gsrc, uint32_t lds_byte) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(gsrc), "s"(lds_byte) : "memory");
}

constexpr int kSNh = 20;                 // 1-KiB pieces per halo plane (max)
constexpr int kSPlane = kSNh * 1024;
constexpr int kSBuf = 4 * kSPlane;      // one chunk: 4 planes (hi/lo x 2 channel halves)
constexpr int kSPieces = 4 * kSNh / 8;  // halo pieces per wave per chunk
constexpr int kSHalo = kSPieces;        // tap pairs during which the next chunk's halo is issued (1 each)

}  // namespace

template <int NPXW>
__global__ __launch_bounds__(512, 2) void conv_m16s_bf16x3(SplitConvShape s, SplitConvGroup g0, SplitConvGroup g1,
                                                           BigTiling tl) {
  constexpr int KS = 7, KSQ = 49, R = 3;
  constexpr int PAIRS = (KSQ + 1) / 2;  // 25 tap pairs per chunk (the last pairs tap 48 with zeros)
  constexpr int CAP = 2 * NPXW * 16;
  extern __shared__ __attribute__((aligned(16))) char lds[];  // [2 buffers][4 planes][kSPlane]

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
  const int P0 = widx * CAP;
  const int P1 = min(P0 + CAP, tl.total) - 1;
  const int frame = P0 / tl.hw;
  const int y0 = (P0 - frame * tl.hw) / s.w;
  const int fb = P1 / tl.hw;
  const int rowsA = fb != frame ? s.h - y0 + 2 * R : (1 << 30);

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int cs = wave & 3, pg = wave >> 2;  // channel slice, pixel group
  const int l16 = lane & 15, kg = lane >> 4;
  const int tsel = kg >> 1, khalf = kg & 1;
  const int wp_in = s.w + 2 * s.pin;
  const int hp_in = s.h + 2 * s.pin;
  const int64_t pix_bytes = (int64_t)s.cs_in * 4;
  const char* const fbase = (const char*)g.in + (int64_t)frame * hp_in * wp_in * pix_bytes;
  const char* const fbase_b = (const char*)g.in + (int64_t)fb * hp_in * wp_in * pix_bytes;
  const uint32_t lds0 = (uint32_t)(size_t)(__attribute__((address_space(3))) char*)lds;
  const int pitch = tl.pitch, nh = tl.nh;

  // ---- A: this wave's 32 channels; weights [c16][tap][plane 2*khalf + hi/lo][cop][8 bf16] ----
  const int64_t wplane = (int64_t)g.cop * 16;
  const int cw0 = co0 + cs * 32;
  const char* const wlane = (const char*)g.w + (int64_t)(2 * khalf) * wplane + (int64_t)(cw0 + l16) * 16;
  const int n_pairs = s.c16 * PAIRS;
  typedef bf16x8g AFrag[4];  // [cb * 2 + hl]
  auto load_a = [&](int p, AFrag& a) {
    if (p >= n_pairs) p = n_pairs - 1;  // the last pairs' prefetch re-reads the final pair (unused)
    const int c = p / PAIRS, j = p - (p / PAIRS) * PAIRS;
    // this lane group's tap; the padding tap (49) loads tap 48 and is zeroed before use (no lane
    // branch here: a masked load would make the compiler drain the prefetch queue)
    const int t = min(2 * j + tsel, KSQ - 1);
    const char* q = wlane + (int64_t)((c * KSQ + t) * 4) * wplane;
    a[0] = *(const bf16x8g*)q;
    a[1] = *(const bf16x8g*)(q + wplane);
    a[2] = *(const bf16x8g*)(q + 256);
    a[3] = *(const bf16x8g*)(q + wplane + 256);
  };

  // ---- halo of chunk c into buffer buf: wave w DMAs pieces j = w + 8k (plane j / nh, piece j % nh) ----
  auto halo_piece = [&](int c, int buf, int k) {
    const int j = wave + 8 * k;
    if (j >= 4 * nh) return;  // uniform per wave
    const int plane = j / nh, i = j - (j / nh) * nh;
    const int slot = i * 64 + lane;
    const int hr = slot / pitch, hc = slot - (slot / pitch) * pitch;
    const bool in_a = hr < rowsA;
    const int yy = min((in_a ? y0 - R + hr : hr - rowsA - R) + s.pin, hp_in - 1);
    const int xx = min(hc - R + s.pin, wp_in - 1);
    const char* src = (in_a ? fbase : fbase_b) + (int64_t)(yy * wp_in + xx) * pix_bytes + c * 64 + plane * 16;
    dma16s(src, lds0 + (uint32_t)(buf * kSBuf + plane * kSPlane + i * 1024));
  };

  // this lane's pixel of each block -> byte offset of its halo slot in its (2 khalf) hi plane,
  // two 16-bit offsets per register (< 64 KiB: 2 planes + 24 rows x 52 slots x 16 B)
  uint32_t qp[(NPXW + 1) / 2];
#pragma unroll
  for (int pb = 0; pb < NPXW; ++pb) {
    const int P = P0 + (pg * NPXW + pb) * 16 + l16;
    int q = 0;
    if (P <= P1) {
      const int f = P / tl.hw, pp = P - (P / tl.hw) * tl.hw;
      const int y = pp / s.w, x = pp - (pp / s.w) * s.w;
      q = (f == frame ? y - y0 : rowsA + y) * pitch + x;
    }
    const uint32_t o = (uint32_t)((2 * khalf) * kSPlane + q * 16);
    if (pb & 1) qp[pb >> 1] |= o << 16;
    else qp[pb >> 1] = o;
  }
  auto qb = [&](int pb) -> int { return (int)((qp[pb >> 1] >> (16 * (pb & 1))) & 0xffffu); };

  floatx4 acc[2][NPXW];
#pragma unroll
  for (int cb = 0; cb < 2; ++cb)
#pragma unroll
    for (int pb = 0; pb < NPXW; ++pb) acc[cb][pb] = floatx4{0.f, 0.f, 0.f, 0.f};

  // prologue: chunk 0's halo, the first two pairs' weights
#pragma unroll
  for (int k = 0; k < kSPieces; ++k) halo_piece(0, 0, k);
  AFrag abuf[M16S_ABUF];
#pragma unroll
  for (int k = 0; k < M16S_ABUF - 1; ++k) load_a(k, abuf[k]);
  wait_vmcnt<0>();
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  const int nchunks = s.c16;
  // one tap pair: prefetch the weights two pairs ahead, stream one halo piece of the next chunk
  // (pairs 0..9), the MFMAs; after the chunk's last pair, the buffer swap
  auto pair = [&](int p, AFrag& a, AFrag& a_ahead) {
    const int c = p / PAIRS, j = p - (p / PAIRS) * PAIRS;
    load_a(p + M16S_ABUF - 1, a_ahead);
    const bool next = c + 1 < nchunks;
    if (j < kSHalo && next) halo_piece(c + 1, (c + 1) & 1, j);
    const char* const hb = lds + (c & 1) * kSBuf;
    const int t0 = 2 * j, t1 = 2 * j + 1 < KSQ ? 2 * j + 1 : 2 * j;  // the padding tap reads tap 48's pixels
    const int toff0 = ((t0 / KS) * pitch + (t0 - (t0 / KS) * KS)) * 16;
    const int toff1 = ((t1 / KS) * pitch + (t1 - (t1 / KS) * KS)) * 16;
    const char* const hbt = hb + (tsel ? toff1 : toff0);
    if (j == PAIRS - 1 && tsel) {  // the padding tap: +0 weights (as conv_m16's zero-buffer tap)
      const bf16x8g z = {};
#pragma unroll
      for (int r = 0; r < 4; ++r) a[r] = z;
    }
    bf16x8g bh[2], bl[2];
    bh[0] = *(const bf16x8g*)(hbt + qb(0));
    bl[0] = *(const bf16x8g*)(hbt + qb(0) + kSPlane);
#pragma unroll
    for (int pb = 0; pb < NPXW; ++pb) {
      const int cur = pb & 1;
      if (pb + 1 < NPXW) {
        bh[cur ^ 1] = *(const bf16x8g*)(hbt + qb(pb + 1));
        bl[cur ^ 1] = *(const bf16x8g*)(hbt + qb(pb + 1) + kSPlane);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        acc[cb][pb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2 * cb], bh[cur], acc[cb][pb], 0, 0, 0);
        acc[cb][pb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2 * cb], bl[cur], acc[cb][pb], 0, 0, 0);
        acc[cb][pb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2 * cb + 1], bh[cur], acc[cb][pb], 0, 0, 0);
      }
    }
    if (j == PAIRS - 1 && next) {
      // this wave's pieces of the next chunk were issued by pair kSHalo - 1; younger than them are
      // only weight loads (4 per pair, 15 pairs): waiting down to 4 outstanding covers every piece
      wait_vmcnt<4>();
      __builtin_amdgcn_s_barrier();  // every wave's pieces landed; this chunk's buffer is free
      asm volatile("" ::: "memory");
    }
  };
#if M16S_ABUF == 3
  for (int p = 0; p < n_pairs; p += 3) {  // three weight buffers in rotation (two pairs ahead)
    pair(p, abuf[0], abuf[2]);
    if (p + 1 < n_pairs) pair(p + 1, abuf[1], abuf[0]);
    if (p + 2 < n_pairs) pair(p + 2, abuf[2], abuf[1]);
  }
#else
  for (int p = 0; p < n_pairs; p += 2) {  // two weight buffers (one pair ahead)
    pair(p, abuf[0], abuf[1]);
    if (p + 1 < n_pairs) pair(p + 1, abuf[1], abuf[0]);
  }
#endif
  wait_vmcnt<0>();

  const int wp_out = s.w + 2 * s.pout;
  const int hp_out = s.h + 2 * s.pout;
#pragma unroll
  for (int pb = 0; pb < NPXW; ++pb) {
    const int P = P0 + (pg * NPXW + pb) * 16 + l16;
    const int f = P / tl.hw, pp = P - f * tl.hw;
    const int y = pp / s.w, x = pp - y * s.w;
    char* optr = (char*)g.out + ((int64_t)(f * hp_out + y + s.pout) * wp_out + (x + s.pout)) * (int64_t)s.cs_out * 4;
    float* o32 = g.out32 ? g.out32 + ((int64_t)(f * s.h + y) * s.w + x) * s.cs_out32 + g.out32_off : nullptr;
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      const int co = cw0 + cb * 16 + 4 * kg;
      floatx4 v;
      uint32_t own[4], w[4];
      split_pair_swap(acc[cb][pb], co < g.cop ? *(const floatx4*)(g.bias + co) : floatx4{0.f, 0.f, 0.f, 0.f}, s.relu,
                      v, own, w);
      if (P > P1 || co >= g.cout_store) continue;
      store_split_group(optr, co, kg, g.cout_store, own, w);
      if (o32) *(floatx4*)(o32 + co) = v;
    }
  }
}

// Tiling + launch for a 7x7 split-format conv (Co multiple of 128, one or two groups); *taken = 0
// when the launch is small (conv_m16 picks its tile and split-K there) or a raster tile's halo does
// not fit kSNh pieces per plane at the tight pitch (maps much wider than 46).  zeros: >= 1 KiB of
// device zeros (the padding tap's weights).  OP_M16S=0 disables.
int launch_conv_m16s(const SplitConvShape& s, const SplitConvGroup* g, const void* zeros, hipStream_t st, int* taken) {
  *taken = 0;
  static const int mode = getenv("OP_M16S") ? atoi(getenv("OP_M16S")) : 1;
  constexpr int NPXW = 14, CAP = 2 * NPXW * 16, R = 3;
  if (!mode || !zeros || s.ks != 7 || s.cs_in % 16 || s.pin < R || s.halo_mode != 4 || !s.regw) return OP_OK;
  int cop_max = 0;
  for (int i = 0; i < s.groups; ++i) {
    if (g[i].cop % 128 || g[i].cin_off % 16) return OP_OK;
    cop_max = std::max(cop_max, g[i].cop);
  }
  const int hw = s.h * s.w;
  const int64_t total = (int64_t)s.n * hw;
  if (hw < CAP || total >= (1 << 30)) return OP_OK;
  const int tiles = (int)((total + CAP - 1) / CAP);
  BigTiling t{};
  t.co_tiles = cop_max / 128;
  t.units = s.groups * t.co_tiles;
  t.per_unit = tiles;
  if ((int64_t)t.units * t.per_unit < 2 * 256) return OP_OK;
  // worst halo of a raster tile: its rows of each frame it touches, each with a 2R border
  const int pitch = s.w + 2 * R;
  int rows_max = 0;
  for (int i = 0; i < tiles; ++i) {
    const int64_t a = (int64_t)i * CAP, b = std::min<int64_t>(a + CAP, total) - 1;
    const int f0 = (int)(a / hw), f1 = (int)(b / hw);
    const int ya = (int)((a - (int64_t)f0 * hw) / s.w), yb = (int)((b - (int64_t)f1 * hw) / s.w);
    const int rows = f0 == f1 ? yb - ya + 1 + 2 * R : (s.h - ya + 2 * R) + (yb + 1 + 2 * R);
    rows_max = std::max(rows_max, rows);
  }
  const int nh = (rows_max * pitch + 63) / 64;
  if (nh > kSNh) return OP_OK;
  t.tr = 0;
  t.tc = s.w;
  t.tiles_y = tiles;
  t.tiles_x = 1;
  t.pitch = pitch;
  t.hrows = rows_max;
  t.nh = nh;
  t.xpu = (t.units <= 8 && 8 % t.units == 0) ? 8 / t.units : 0;
  t.hw = hw;
  t.total = (int)total;
  t.ksplit = 1;
  t.zeros = zeros;
  static bool attr = false;
  if (!attr) {
    OP_HIP_CHECK(hipFuncSetAttribute((const void*)conv_m16s_bf16x3<NPXW>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     2 * kSBuf));
    attr = true;
  }
  *taken = 1;
  census_add(OP_CENSUS_7X7_S);
  const unsigned blocks = t.xpu ? 8u * (unsigned)((t.per_unit + t.xpu - 1) / t.xpu) : (unsigned)(t.units * t.per_unit);
  const SplitConvGroup& g1 = s.groups > 1 ? g[1] : g[0];
  hipLaunchKernelGGL((conv_m16s_bf16x3<NPXW>), dim3(blocks), dim3(512), 2 * kSBuf, st, s, g[0], g1, t);
  OP_AFTER_LAUNCH("conv_m16s_bf16x3", st);
  OP_HIP_CHECK(hipGetLastError());
  return OP_OK;
}

}  // namespace op
