// Halo-tiled convolution with weights shared across the workgroup (3xBF16 split, gfx950): the
// 7x7 stage convs (Mconv1..5 of stages 2-6, 68 % of the network's FLOPs) and the 3x3 convs.
//
// Workgroup = NWAVE waves; it owns CW output channels (128 or 64) x one TR x TC pixel tile of one
// frame.  Wave w holds 64 channels (channel half w / PG) for NPB 32-pixel blocks (pixel group
// w % PG): 2 x NPB accumulator tiles, so every B fragment read from LDS feeds 2 channel blocks and
// every A fragment NPB pixel blocks.
//  * Activations: per 16-channel chunk the tile's input rows plus halo are copied once into LDS
//    as 4 planes (hi/lo x k-half) of 16 B per pixel and all KSxKS taps read their shifted window
//    from there.  The LDS row pitch is TC + 16 slots when a 32-pixel block wraps a tile row (every
//    ds_read_b128 lane group stays on distinct banks), the tight TC + KS - 1 when TC % 32 == 0.
//  * Weights: (tap, chunk) tiles of CW channels x 4 planes stream through an LDS ring by
//    global_load_lds (each wave copies its pieces), one counted vmcnt + one s_barrier per tap
//    (PAIR = 0, 3-deep ring) or per pair of taps (PAIR = 1, 6-deep ring, 4 taps ahead; raster
//    tiles, whose two-frame halo needs the LDS, 4-deep ring, 2 taps ahead).
//  * The weight bytes fetched per MFMA-flop fall with the tile's pixel count: 7x7 uses one
//    8-wave workgroup per CU on 768-pixel raster tiles (consecutive pixels of the batch, crossing
//    frame borders, so no lane computes padding); 3x3 uses two 4-wave workgroups per CU on
//    384-pixel tiles so one workgroup's halo reload (every 9 taps) overlaps the other's MFMAs.
//  * Workgroup -> XCD: blocks are dealt to XCDs round-robin, so block b is remapped to make every
//    XCD work on ONE weight set (branch x channel tile), which its 4 MiB L2 then holds.
//  * MFMA: v_mfma_f32_32x32x16_bf16, products hi*hi + hi*lo + lo*hi into one f32 accumulator.
#include <atomic>
#include <array>
#include <map>
#include <mutex>
#include <tuple>
#include <cstdlib>
#include <vector>

#include "conv_big.hpp"
#include "conv_m16k.hpp"

namespace op {


// nt (1 or 2) consecutive taps t, t+1 of one chunk for one wave: 2 channel blocks x NPB pixel
// blocks.  The B fragments are software-pipelined one block ahead (also into the next tap), so
// each LDS read has a block's 6 MFMAs (~200 cycles) to land; A fragments are read per tap.
template <int NPB, int KS, int PLANE_W>
__device__ __forceinline__ void big_taps(int nt, floatx16 (&acc)[2][NPB], const char* bp0, int hplane,
                                         const uint32_t (&qp)[(NPB + 1) / 2], const char* wb0, const char* wb1,
                                         int t, int pitch, int hi) {
  bf16x8g bh[2], bl[2], ah[2], al[2];
  // halo slot of pixel block pb (two 16-bit slots per register)
  auto q0 = [&](int pb) -> int { return (int)((qp[pb >> 1] >> (16 * (pb & 1))) & 0xffffu); };
  int toff = (t / KS) * pitch + (t - (t / KS) * KS);
  bh[0] = *(const bf16x8g*)(bp0 + (q0(0) + toff) * 16);
  bl[0] = *(const bf16x8g*)(bp0 + hplane + (q0(0) + toff) * 16);
#pragma unroll 1
  for (int u = 0; u < nt; ++u) {
    const char* wb = u == 0 ? wb0 : wb1;
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      ah[cb] = *(const bf16x8g*)(wb + (2 * hi) * PLANE_W + cb * 512);
      al[cb] = *(const bf16x8g*)(wb + (2 * hi + 1) * PLANE_W + cb * 512);
    }
    const int tn = t + u + 1;
    const int toff_n = (tn / KS) * pitch + (tn - (tn / KS) * KS);
    const bool more = u + 1 < nt;
#pragma unroll
    for (int pb = 0; pb < NPB; ++pb) {
      // block pb's fragments sit in buffer (pb & 1) of this tap; an odd NPB flips the parity of
      // the next tap, so the prefetch into the next tap goes to buffer (NPB & 1)
      const int cur = pb & 1;
      if (pb + 1 < NPB) {
        bh[(pb + 1) & 1] = *(const bf16x8g*)(bp0 + (q0(pb + 1) + toff) * 16);
        bl[(pb + 1) & 1] = *(const bf16x8g*)(bp0 + hplane + (q0(pb + 1) + toff) * 16);
      } else if (more) {
        bh[NPB & 1] = *(const bf16x8g*)(bp0 + (q0(0) + toff_n) * 16);
        bl[NPB & 1] = *(const bf16x8g*)(bp0 + hplane + (q0(0) + toff_n) * 16);
      }
      __builtin_amdgcn_sched_barrier(0);  // keep the next block's reads ahead of this block's MFMAs
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        acc[cb][pb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[cb], bh[cur], acc[cb][pb], 0, 0, 0);
        acc[cb][pb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[cb], bl[cur], acc[cb][pb], 0, 0, 0);
        acc[cb][pb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[cb], bh[cur], acc[cb][pb], 0, 0, 0);
      }
    }
    toff = toff_n;
    if constexpr (NPB & 1) {  // the next tap starts on buffer 1: swap so block 0 reads buffer 0
      const bf16x8g th = bh[0], tl = bl[0];
      bh[0] = bh[1];
      bl[0] = bl[1];
      bh[1] = th;
      bl[1] = tl;
    }
  }
}

template <int KS, int NPB, int NWAVE, int CW, int PAIR, bool POOL, bool RASTER>
__global__ __launch_bounds__(NWAVE * 64, NWAVE == 8 ? 1 : 2) void conv_big_bf16x3(SplitConvShape s, SplitConvGroup g0,
                                                                                   SplitConvGroup g1, BigTiling tl) {
  constexpr int KSQ = KS * KS;
  constexpr int R = KS / 2;
  constexpr int CH = CW / 64;            // 64-channel halves per tile
  constexpr int PG = NWAVE / CH;         // pixel groups
  constexpr int PLANE_W = CW * 16;       // bytes of one weight plane of the tile
  constexpr int SLOT_W = 4 * PLANE_W;    // one (tap, chunk) weight tile
  constexpr int NWP = 4 * CH / NWAVE;    // 1-KiB weight pieces per wave per tap
  // tap pairs use a 4-slot ring (2 taps ahead) where LDS is tight: RASTER (tiles over the batch's
  // raster order, 2 halo regions) and 3x3 (2 workgroups per CU)
  constexpr bool RING4 = RASTER || KS == 3;
  constexpr int RING = PAIR ? (RING4 ? 4 : 6) : 3;
  constexpr int AHEAD = PAIR ? (RING4 ? 2 : 4) : 2;  // taps between a weight copy's issue and its use
  constexpr int CAP = PG * NPB * 32;     // output pixels per tile
  static_assert(NWP >= 1 && NWP <= 2 && PG >= 1, "wave / channel split");
  static_assert(!RASTER || !POOL, "raster tiles: plain epilogue");
  extern __shared__ __attribute__((aligned(16))) char lds[];  // [W ring][halo: 4 planes]

  // ---- which tile / weight set ----
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
  if (co0 >= g.cop) return;  // narrower second group
  // rect tiles: frame, rows y0.., cols x0..; raster tiles: batch raster pixels P0..P1, i.e. rows
  // y0.. of `frame` and, when the range runs into the next frame, rows 0.. of frame fb, whose halo
  // rows follow frame's (from halo row rowsA on)
  int frame, y0, x0 = 0, fb = 0, rowsA = 1 << 30, P0 = 0, P1 = 0;
  if constexpr (RASTER) {
    P0 = widx * CAP;
    P1 = min(P0 + CAP, tl.total) - 1;
    frame = P0 / tl.hw;
    y0 = (P0 - frame * tl.hw) / s.w;
    fb = P1 / tl.hw;
    if (fb != frame) rowsA = s.h - y0 + 2 * R;
  } else {
    const int tpf = tl.tiles_y * tl.tiles_x;
    frame = widx / tpf;
    const int tix = widx - frame * tpf;
    const int ty = tix / tl.tiles_x;
    y0 = ty * tl.tr;
    x0 = (tix - ty * tl.tiles_x) * tl.tc;
  }

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ch = wave / PG;  // channel half: channels co0 + 64*ch .. +63
  const int pg = wave % PG;  // pixel group: tile pixels pg*NPB*32 .. +NPB*32-1
  const int l32 = lane & 31, hi = lane >> 5;
  const int hplane = tl.nh * 1024;
  char* const halo = lds + RING * SLOT_W;
  const int wp_in = s.w + 2 * s.pin;
  const int hp_in = s.h + 2 * s.pin;
  const int64_t pix_bytes = (int64_t)s.cs_in * 4;
  const char* const fbase = (const char*)g.in + (int64_t)frame * hp_in * wp_in * pix_bytes;
  const char* const fbase_b = (const char*)g.in + (int64_t)fb * hp_in * wp_in * pix_bytes;

  // weights: wave w copies pieces j = w*NWP + i: plane j / CH, channels co0 + 64*(j % CH) + 0..63
  const int64_t wplane = (int64_t)g.cop * 16;
  const int64_t wstep = 4 * wplane;
  const char* wsrc[NWP];
  int wdst[NWP];
#pragma unroll
  for (int i = 0; i < NWP; ++i) {
    const int j = wave * NWP + i;
    wsrc[i] = (const char*)g.w + (j / CH) * wplane + ((int64_t)co0 + 64 * (j % CH) + lane) * 16;
    wdst[i] = (j / CH) * PLANE_W + (j % CH) * 1024;
  }
  // split-K (tl.ksplit > 1): this workgroup runs input chunks [cb0, cb1)
  const int nsplit = tl.ksplit > 1 ? tl.ksplit : 1;
  const int split = nsplit > 1 ? (int)blockIdx.y : 0;
  const int cb0 = split * (s.c16 / nsplit), cb1 = cb0 + s.c16 / nsplit;
  const int n_it = cb1 * KSQ;
  auto stage_w = [&](int it) {
    char* dst = lds + (it % RING) * SLOT_W;  // slot of the unclamped step
    if (it >= n_it) it = n_it - 1;           // trailing copies: never read
#pragma unroll
    for (int i = 0; i < NWP; ++i)
      glds16((const void*)(wsrc[i] + (int64_t)it * wstep), dst + wdst[i]);
  };

  // this lane's output pixels: tile-local p = (pg*NPB + pb)*32 + l32 -> (r, c) -> halo slot
  const int rows_here = min(tl.tr, s.h - y0);
  const int cols_here = min(tl.tc, s.w - x0);
  uint32_t qp[(NPB + 1) / 2];  // two 16-bit halo slots per register (hrows*pitch <= 4*nh*64 < 65536)
#pragma unroll
  for (int pb = 0; pb < NPB; ++pb) {
    const int p = (pg * NPB + pb) * 32 + l32;
    uint32_t q = 0u;  // pad lanes: never stored
    if constexpr (RASTER) {
      const int P = P0 + p;
      if (P <= P1) {
        const int f = P / tl.hw, pp = P - (P / tl.hw) * tl.hw;
        const int y = pp / s.w, x = pp - (pp / s.w) * s.w;
        q = (uint32_t)((f == frame ? y - y0 : rowsA + y) * tl.pitch + x);
      }
    } else {
      const int r = p / tl.tc, c = p - (p / tl.tc) * tl.tc;
      if (r < rows_here && c < cols_here) q = (uint32_t)(r * tl.pitch + c);
    }
    if (pb & 1) qp[pb >> 1] |= q << 16;
    else qp[pb >> 1] = q;
  }

  floatx16 acc[2][NPB];
#pragma unroll
  for (int cb = 0; cb < 2; ++cb)
#pragma unroll
    for (int pb = 0; pb < NPB; ++pb)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[cb][pb][e] = 0.0f;

#pragma unroll
  for (int i = 0; i < AHEAD; ++i) stage_w(i);
  const char* const bp0 = halo + (2 * hi) * hplane;  // this lane's k-half: hi plane, lo plane follows
  const int wlane = (ch * 64 + l32) * 16;
  constexpr int HSTEP = NWAVE / 4;
  const int h_plane = wave & 3, h_i0 = wave >> 2;
  const int h_sl0 = h_i0 * 64 + lane;
  const int h_r0 = h_sl0 / tl.pitch, h_c0 = h_sl0 - (h_sl0 / tl.pitch) * tl.pitch;
  int it = 0;
  for (int c = 0; c < s.c16; ++c) {
    // ---- halo reload; everyone is past the previous chunk's reads ----
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    {
      const char* src0 = fbase + c * 64 + h_plane * 16;
      const char* src0_b = fbase_b + c * 64 + h_plane * 16;
      // wave w copies plane w%4, pieces w/4, w/4 + NWAVE/4, ...: the halo slot advances by a
      // fixed stride, so (row, col) are stepped, not divided, per piece
      int hr = h_r0, hc = h_c0;
      char* dst = halo + h_plane * hplane + h_i0 * 1024;
      for (int i = h_i0; i < tl.nh; i += HSTEP) {
        // slots past the padded image (bottom / right of a partial tile, pitch gap) only feed
        // masked outputs or are never read: clamp the source inside this frame
        const bool in_a = hr < rowsA;  // raster tiles: halo rows past rowsA belong to frame fb
        const int yy = min((in_a ? y0 - R + hr : hr - rowsA - R) + s.pin, hp_in - 1);
        const int xx = min(x0 - R + hc + s.pin, wp_in - 1);
        glds16((const void*)((in_a ? src0 : src0_b) + (int64_t)(yy * wp_in + xx) * pix_bytes), dst);
        dst += HSTEP * 1024;
        hc += HSTEP * 64;
        while (hc >= tl.pitch) {
          hc -= tl.pitch;
          ++hr;
        }
      }
    }
    wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if constexpr (PAIR) {
#pragma unroll 1
      for (int t = 0; t < KSQ; t += 2) {
        // taps (t, t+1) share one barrier: W(it), W(it+1) landed for this wave (W(it+2), W(it+3)
        // may be in flight; after a 1-tap tail the count over-waits, which is safe) ...
        wait_vmcnt<AHEAD == 4 ? 2 * NWP : 0>();
        // ... and for every wave; every wave is also done with the slots of the previous pair
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        stage_w(it + AHEAD);
        stage_w(it + AHEAD + 1);
        const int nt = t + 1 < KSQ ? 2 : 1;
        big_taps<NPB, KS, PLANE_W>(nt, acc, bp0, hplane, qp, lds + (it % RING) * SLOT_W + wlane,
                                   lds + ((it + 1) % RING) * SLOT_W + wlane, t, tl.pitch, hi);
        it += nt;
      }
    } else {
#pragma unroll 1
      for (int t = 0; t < KSQ; ++t, ++it) {
        wait_vmcnt<NWP>();  // W(it) landed for this wave (W(it+1) may be in flight) ...
        __builtin_amdgcn_s_barrier();  // ... and for every wave; slot (it-1) % 3 is free
        asm volatile("" ::: "memory");
        stage_w(it + 2);
        const char* wb = lds + (it % RING) * SLOT_W + wlane;
        big_taps<NPB, KS, PLANE_W>(1, acc, bp0, hplane, qp, wb, wb, t, tl.pitch, hi);
      }
    }
  }
  wait_vmcnt<0>();  // drain the trailing (never read) weight copies

  if constexpr (POOL) {
    // ---- fused 2x2 max-pool epilogue (the following F.max_pooling_2d, CocoPoseNet.py:138/141/146)
    // Tiles are 32 wide, so block pb of a wave is one tile row: the window rows are blocks
    // (pb, pb+1) of this lane and the window columns lanes (l32, l32^1).  Exactly the unfused
    // path: ReLU(acc + b) split into hi/lo, the reconstructed hi+lo compared, the winner re-split.
    const int wp_out = s.w / 2 + 2 * s.pout;
    const int hp_out = s.h / 2 + 2 * s.pout;
#pragma unroll
    for (int pb = 0; pb < NPB; pb += 2) {
      const int r = pg * NPB + pb;  // even tile row
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
          const bool live = co < g.cout_store;
          const floatx4 bv = live ? *(const floatx4*)(g.bias + co) : floatx4{0.f, 0.f, 0.f, 0.f};
          u16x4g vh, vl;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float m = 0.0f;
#pragma unroll
            for (int k = 0; k < 2; ++k) {
              float f = acc[cb][pb + k][4 * q + e] + bv[e];
              if (s.relu) f = f > 0.0f ? f : 0.0f;
              const __bf16 h16 = (__bf16)f;
              const float rc = (float)h16 + (float)(__bf16)(f - (float)h16);
              m = k == 0 ? rc : fmaxf(m, rc);
            }
            m = fmaxf(m, __shfl_xor(m, 1));  // the window's other column (all lanes take part)
            const __bf16 h16 = (__bf16)m;
            const __bf16 l16 = (__bf16)(m - (float)h16);
            vh[e] = __builtin_bit_cast(unsigned short, h16);
            vl[e] = __builtin_bit_cast(unsigned short, l16);
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

  // ---- epilogue: bias, ReLU, split store (+ dense f32 copy) ----
  const int wp_out = s.w + 2 * s.pout;
  const int hp_out = s.h + 2 * s.pout;
#pragma unroll
  for (int pb = 0; pb < NPB; ++pb) {
    const int p = (pg * NPB + pb) * 32 + l32;
    int f = frame, y, x;
    if constexpr (RASTER) {
      const int P = P0 + p;
      if (P > P1) continue;
      f = P / tl.hw;
      const int pp = P - f * tl.hw;
      y = pp / s.w;
      x = pp - y * s.w;
    } else {
      const int r = p / tl.tc, cc = p - (p / tl.tc) * tl.tc;
      if (r >= rows_here || cc >= cols_here) continue;
      y = y0 + r;
      x = x0 + cc;
    }
    char* optr = (char*)g.out + ((int64_t)(f * hp_out + y + s.pout) * wp_out + (x + s.pout)) * (int64_t)s.cs_out * 4;
    float* o32 = g.out32 ? g.out32 + ((int64_t)(f * s.h + y) * s.w + x) * s.cs_out32 + g.out32_off : nullptr;
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int co = co0 + ch * 64 + cb * 32 + 8 * q + 4 * hi;
        if (co >= g.cout_store) continue;
        const floatx4 bv = *(const floatx4*)(g.bias + co);
        floatx4 v;
        u16x4g vh, vl;
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
        *(u16x4g*)d = vh;
        *(u16x4g*)(d + 16) = vl;
        if (o32) *(floatx4*)(o32 + co) = v;
      }
  }
}


// Device zeros per HIP device (the 7x7 padding tap's weights), allocated outside any stream capture
// by conv_big_device_init() when a context is created.
static std::mutex g_zeros_mu;
static std::map<int, void*> g_zeros;

int conv_big_device_init(int device) {
  std::lock_guard<std::mutex> lk(g_zeros_mu);
  if (g_zeros.count(device)) return OP_OK;
  void* z = nullptr;
  OP_HIP_CHECK(hipMalloc(&z, 4096));
  OP_HIP_CHECK(hipMemset(z, 0, 4096));
  OP_HIP_CHECK(hipDeviceSynchronize());
  g_zeros[device] = z;
  return OP_OK;
}

static std::atomic<int64_t> g_census[OP_CENSUS_SLOTS];
void census_add(int slot) {
  if (slot >= 0 && slot < OP_CENSUS_SLOTS) g_census[slot].fetch_add(1, std::memory_order_relaxed);
}

static const void* device_zeros() {
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lk(g_zeros_mu);
  auto it = g_zeros.find(d);
  return it == g_zeros.end() ? nullptr : it->second;
}

// Per-stream split-K workspace, owned by the context that owns the stream: grown on demand
// outside capture, released by splitk_ws_release() when the context destroys its stream.  While
// the stream is capturing a hipGraph and the buffer is too small the launch cannot allocate, so it
// records the size it needs and returns nullptr; the capturing caller checks
// splitk_ws_capture_short() after EndCapture, grows the buffer with splitk_ws_reserve() and
// captures again, so graph replays pick the same kernels (and sums) as eager runs.
struct SplitkWs {
  float* p = nullptr;
  size_t floats = 0;
  size_t short_by = 0;  // largest request refused during capture
  std::vector<float*> retired;  // outgrown buffers: a graph captured earlier may still read them
};
static std::mutex g_ws_mu;
static std::map<hipStream_t, SplitkWs> g_ws;

static float* splitk_ws(hipStream_t st, size_t floats) {
  std::lock_guard<std::mutex> lk(g_ws_mu);
  SplitkWs& e = g_ws[st];
  if (e.floats >= floats) return e.p;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) {
    e.short_by = std::max(e.short_by, floats);
    return nullptr;
  }
  float* p = nullptr;
  if (hipMalloc(&p, floats * sizeof(float)) != hipSuccess) return nullptr;
  if (e.p) e.retired.push_back(e.p);
  e.p = p;
  e.floats = floats;
  return p;
}

size_t splitk_ws_capture_short(hipStream_t st) {
  std::lock_guard<std::mutex> lk(g_ws_mu);
  auto it = g_ws.find(st);
  return it == g_ws.end() ? 0 : it->second.short_by;
}

int splitk_ws_reserve(hipStream_t st) {
  size_t need;
  {
    std::lock_guard<std::mutex> lk(g_ws_mu);
    SplitkWs& e = g_ws[st];
    need = e.short_by;
    e.short_by = 0;
    if (need <= e.floats) return 0;
  }
  return splitk_ws(st, need) ? 0 : -1;
}

void splitk_ws_release(hipStream_t st) {
  std::lock_guard<std::mutex> lk(g_ws_mu);
  auto it = g_ws.find(st);
  if (it == g_ws.end()) return;
  if (it->second.p) (void)hipFree(it->second.p);
  for (float* p : it->second.retired) (void)hipFree(p);
  g_ws.erase(it);
}

// Split-K epilogue of conv_m16_bf16x3: out = act(sum over splits (fixed order) + bias), stored
// like the kernel's own epilogue (split hi/lo planes + optional dense f32).  Thread = 4 channels.
__global__ __launch_bounds__(256) void conv_m16_splitk_reduce(SplitConvShape s, SplitConvGroup g0, SplitConvGroup g1,
                                                              BigTiling tl) {
  const int grp = blockIdx.y;
  const SplitConvGroup g = grp == 0 ? g0 : g1;
  const int q = g.cop / 4;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)tl.total * q) return;
  const int P = (int)(i / q), co = (int)(i - (int64_t)P * q) * 4;
  if (co >= g.cout_store) return;
  splitk_reduce_item(s, g, grp, tl, max(g0.cop, g1.cop), P, co);
}

// Split-K partials of a conv with the fused 2x2 max-pool (round 4: pooled 3x3 launches that fill
// few CUs, one frame's conv2_2 / conv3_4): one thread per (pooled pixel, 4 channels) sums the
// partials of its 4 conv pixels in split order onto the bias, then ReLU, the split round trip and
// the max as the pooled epilogue of conv_m16k_bf16x3<true>, and stores the pooled split value.
__global__ __launch_bounds__(256) void conv_m16_splitk_reduce_pool(SplitConvShape s, SplitConvGroup g,
                                                                   BigTiling tl) {
  const int q = g.cop / 4;
  const int ho = s.h / 2, wo = s.w / 2;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)s.n * ho * wo * q) return;
  const int64_t Po = i / q;
  const int co = (int)(i - Po * q) * 4;
  if (co >= g.cout_store) return;
  const int f = (int)(Po / ((int64_t)ho * wo)), pp = (int)(Po - (int64_t)f * ho * wo);
  const int yo = pp / wo, xo = pp - yo * wo;
  const floatx4 bv = *(const floatx4*)(g.bias + co);
  floatx4 m = {0.f, 0.f, 0.f, 0.f};
  // all 4 x ksplit partials loaded before the first add (splitk_reduce_item); split order kept
  constexpr int kMaxPoolSplit = 8;
  floatx4 part[4][kMaxPoolSplit];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t P = ((int64_t)f * s.h + 2 * yo + (k >> 1)) * s.w + 2 * xo + (k & 1);
#pragma unroll
    for (int sp = 0; sp < kMaxPoolSplit; ++sp)
      if (sp < tl.ksplit) part[k][sp] = *(const floatx4*)(tl.ws + ((int64_t)sp * tl.total + P) * g.cop + co);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    floatx4 v = bv;
#pragma unroll
    for (int sp = 0; sp < kMaxPoolSplit; ++sp)
      if (sp < tl.ksplit) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += part[k][sp][e];
      }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float fv = v[e];
      if (s.relu) fv = fv > 0.0f ? fv : 0.0f;
      const __bf16 h16 = (__bf16)fv;
      const float rc = (float)h16 + (float)(__bf16)(fv - (float)h16);
      m[e] = k == 0 ? rc : fmaxf(m[e], rc);
    }
  }
  const int wp_out = wo + 2 * s.pout, hp_out = ho + 2 * s.pout;
  char* d = (char*)g.out + (((int64_t)f * hp_out + yo + s.pout) * wp_out + (xo + s.pout)) * (int64_t)s.cs_out * 4 +
            (co >> 3) * 32 + (co & 7) * 2;
  u16x4g vh, vl;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const __bf16 h16 = (__bf16)m[e];
    const __bf16 l16v = (__bf16)(m[e] - (float)h16);
    vh[e] = __builtin_bit_cast(unsigned short, h16);
    vl[e] = __builtin_bit_cast(unsigned short, l16v);
  }
  *(u16x4g*)d = vh;
  *(u16x4g*)(d + 16) = vl;
}

// ---- 3x3: conv_m16k_bf16x3 (conv_m16k.hpp) ----

// ---- host side ----
struct BigConfig {
  int ks, npb, nwave, cw, pair, raster = 0;
  int cap_px = 0;  // pixels per tile when npb does not express it (conv_m16 with an odd block count)
  int cap() const { return cap_px ? cap_px : (nwave / (cw / 64)) * npb * 32; }  // pixels per tile
  int ring_bytes() const { return (pair ? ((raster || ks == 3) ? 4 : 6) : 3) * 4 * cw * 16; }
  int lds_budget() const { return (nwave == 8 ? 160 : 80) * 1024; }  // 1 or 2 workgroups per CU
  int halo_budget() const { return lds_budget() - ring_bytes(); }
};

// LDS halo row pitch (16-B slots): a 32-pixel block that wraps a tile row (tc % 32 != 0) needs
// (pitch - tc) % 16 == 0 to keep its ds_read_b128 lane groups on distinct banks; when tc % 32 == 0
// every block is one contiguous row segment and the tight tc + ks - 1 suffices.
static int halo_pitch(int tc, int ks) {
  if (ks == 1) return tc;
  return tc % 32 == 0 ? tc + ks - 1 : tc + 16 * ((ks - 1 + 15) / 16);
}

static int halo_bytes(int tr, int tc, int ks) {
  return 4 * 1024 * (((tr + ks - 1) * halo_pitch(tc, ks) + 63) / 64);
}

constexpr double BIG_UTIL_WIN = 0.03;

// Pick the tile (tr x tc) that fits LDS: among the tilings within 3 % of the best MFMA-lane
// utilisation, the one that loads the fewest halo slots per tile pixel (hrows x pitch / (tr tc)).
// Widths are the even splits of the image (ceil(w / segs)) and the multiples of 32 (tight pitch).
static bool big_tiling(const BigConfig& k, int n, int h, int w, int groups, int cop_max, BigTiling& t) {
  const int cap = k.cap();
  const int budget = k.halo_budget();
  struct Cand {
    int tr, tc, tiles_y, tiles_x;
    double util, amp;
  };
  std::vector<Cand> cands;
  double best = 0.0;
  std::vector<int> widths;
  for (int segs = 1; segs <= 32; ++segs) widths.push_back((w + segs - 1) / segs);
  for (int tc = 32; tc < w && tc <= cap; tc += 32) widths.push_back(tc);
  for (int tc : widths) {
    if (tc > cap || tc < 1) continue;
    const int segs = (w + tc - 1) / tc;
    int tr = cap / tc;
    if (tr > h) tr = h;
    while (tr >= 1 && halo_bytes(tr, tc, k.ks) > budget) --tr;
    if (tr < 1) continue;
    const int tiles_y = (h + tr - 1) / tr;
    const int trb = (h + tiles_y - 1) / tiles_y;  // even the rows out over the same tile count
    const double util = (double)h * w / ((double)tiles_y * segs * cap);
    const double amp = (double)(trb + k.ks - 1) * halo_pitch(tc, k.ks) / ((double)trb * tc);
    cands.push_back({trb, tc, tiles_y, segs, util, amp});
    best = util > best ? util : best;
  }
  if (best <= 0.0) return false;
  const Cand* pick = nullptr;
  for (const Cand& c : cands)
    if (c.util >= best - BIG_UTIL_WIN && (!pick || c.amp < pick->amp - 1e-9)) pick = &c;
  t.tr = pick->tr;
  t.tc = pick->tc;
  t.tiles_y = pick->tiles_y;
  t.tiles_x = pick->tiles_x;
  t.pitch = halo_pitch(t.tc, k.ks);
  t.hrows = t.tr + k.ks - 1;
  t.nh = (t.hrows * t.pitch + 63) / 64;
  t.co_tiles = (cop_max + k.cw - 1) / k.cw;
  t.units = groups * t.co_tiles;
  t.per_unit = n * t.tiles_y * t.tiles_x;
  t.xpu = (t.units <= 8 && 8 % t.units == 0) ? 8 / t.units : 0;
  return true;
}

template <int KS, int NPB, int NWAVE, int CW, int PAIR, bool POOL = false, bool RASTER = false>
static int launch_big_t(const SplitConvShape& s, const SplitConvGroup* g, const BigTiling& tl, hipStream_t st) {
  const BigConfig k{KS, NPB, NWAVE, CW, PAIR, RASTER};
  const int lds = k.ring_bytes() + 4 * tl.nh * 1024;
  static bool attr = false;
  if (!attr) {
    OP_HIP_CHECK(hipFuncSetAttribute((const void*)conv_big_bf16x3<KS, NPB, NWAVE, CW, PAIR, POOL, RASTER>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  const unsigned blocks = tl.xpu ? 8u * (unsigned)((tl.per_unit + tl.xpu - 1) / tl.xpu)
                                 : (unsigned)(tl.units * tl.per_unit);
  census_add(KS == 7 ? OP_CENSUS_7X7_OTHER : OP_CENSUS_3X3_BIG);
  hipLaunchKernelGGL((conv_big_bf16x3<KS, NPB, NWAVE, CW, PAIR, POOL, RASTER>), dim3(blocks), dim3(NWAVE * 64), lds, st, s, g[0],
                     s.groups > 1 ? g[1] : g[0], tl);
  OP_AFTER_LAUNCH("conv_big_bf16x3", st);
  OP_HIP_CHECK(hipGetLastError());
  return OP_OK;
}

// Raster tiles: tile i = pixels [i*cap, (i+1)*cap) of the batch in raster order, so a tile can run
// from the bottom rows of one frame into the top rows of the next and no MFMA lane computes padding
// (46 x 46 maps: 2116 px = 2.76 tiles of 768, where rectangular tiles pay 3).  The halo holds the
// tile's rows of each frame with their own KS-1 border rows; every frame is >= cap pixels, so a
// tile touches at most two.  false when the worst tile's halo does not fit LDS.
// wide: (conv_m16 only) when the batch-raster halo does not fit, also try the tight pitch (blocks
// that wrap a row then see a few 2-way bank conflicts) and then frame-aligned raster tiles (no
// tile crosses a frame: one border region instead of two; the last tile of a frame is partial),
// so the wide maps of the multi-scale path (82 .. 164 columns) stay on the raster kernel.
static bool raster_tiling(const BigConfig& k, int n, int h, int w, int groups, int cop_max, BigTiling& t,
                          bool wide = false) {
  const int cap = k.cap(), hw = h * w, R = k.ks / 2;
  const int64_t total = (int64_t)n * hw;
  if (hw < cap || total >= (1 << 30)) return false;
  const int budget = k.lds_budget() - k.ring_bytes();
  int tiles = 0, rows_max = 0, pitch = 0, nh = 0, fa = 0;
  bool ok = false;
  // conv_m16 (wide): the tight pitch w + ks - 1 first (round 6: the headline's 7x7 75.6 -> 75.2 ms per
  // step, profiles/r06/ab_r06a_tight_pitch_ring4.log -- the 16-B slots of a block that wraps a row
  // see a few 2-way bank conflicts, but 22 instead of 27 KiB halo planes load and fit a circular
  // second chunk, conv_m16.hip CIRC); OP_M16_TIGHT=0 (A/B aid) starts from w + 16
  static const bool tight_first = !(getenv("OP_M16_TIGHT") && atoi(getenv("OP_M16_TIGHT")) == 0);
  for (int variant = (wide && tight_first) ? 1 : 0; variant < (wide ? 4 : 1) && !ok; ++variant) {
    const bool aligned = variant >= 2;
    pitch = (variant & 1) ? w + k.ks - 1 : halo_pitch(w, k.ks);
    fa = aligned ? (hw + cap - 1) / cap : 0;
    tiles = aligned ? n * fa : (int)((total + cap - 1) / cap);
    rows_max = 0;
    const int nt = aligned ? fa : tiles;  // aligned: every frame has the same tiles
    for (int i = 0; i < nt; ++i) {
      const int P0 = i * cap;
      const int P1 = (int)std::min<int64_t>((int64_t)P0 + cap, aligned ? hw : total) - 1;
      const int f0 = P0 / hw, ya = (P0 - f0 * hw) / w, f1 = P1 / hw, yb = (P1 - f1 * hw) / w;
      const int rows = f0 == f1 ? yb - ya + 1 + 2 * R : (h - ya + 2 * R) + (yb + 1 + 2 * R);
      rows_max = std::max(rows_max, rows);
    }
    nh = (rows_max * pitch + 63) / 64;
    ok = 4 * nh * 1024 <= budget && nh * 64 < 65536;
  }
  if (!ok) return false;
  t.fa_tiles = fa;
  t.tr = 0;
  t.tc = w;
  t.tiles_y = tiles;
  t.tiles_x = 1;
  t.pitch = pitch;
  t.hrows = rows_max;
  t.nh = nh;
  t.co_tiles = (cop_max + k.cw - 1) / k.cw;
  t.units = groups * t.co_tiles;
  t.per_unit = tiles;
  t.xpu = (t.units <= 8 && 8 % t.units == 0) ? 8 / t.units : 0;
  t.hw = hw;
  t.total = (int)total;
  return true;
}

// Default 3x3 c128 layers with c16 even on
// conv_m16k_bf16x3 (8 x 32 tiles, 2 workgroups per CU: 32 KiB weight ring + 8-plane halo <= 48
// KiB; 2-19 % faster per layer than conv_big_bf16x3<3,..> in an interleaved A/B).  false when the
// shape does not fit (the 46-wide maps, conv1_2's 64 channels).
static bool m16k_tiling(const SplitConvShape& s, int groups, int cop_max, bool pool, BigTiling& t) {
  const int m = s.halo_mode;
  if (m != 4 || s.ks != 3 || cop_max % 128 || (s.c16 & 1) || s.pin < 1)
    return false;
  static const bool no48 = getenv("OP_M16K_NO48") && atoi(getenv("OP_M16K_NO48")) != 0;  // A/B aid
  // 8 x 32 tiles, or 4 x 48 where they waste fewer MFMA lanes (narrow maps; not with the pool)
  const double u32 = (double)s.w / (((s.w + 31) / 32) * 32) * s.h / (((s.h + 7) / 8) * 8);
  const double u48 = (double)s.w / (((s.w + 47) / 48) * 48) * s.h / (((s.h + 3) / 4) * 4);
  // round 4: on narrow maps where both tile shapes use the lanes equally (the 82 x 46 maps of
  // 1280x720 frames: 85 % either way), 4 x 48 tiles rather than falling back to conv_big below --
  // large launches then run conv_m16r (same arithmetic order as conv_m16k: a frame's bits do not
  // depend on the batch); OP_M16K_TIE48=0 restores the fallback (A/B aid)
  static const bool tie48 = !(getenv("OP_M16K_TIE48") && atoi(getenv("OP_M16K_TIE48")) == 0);
  const bool w48 = !pool && !no48 && (u48 > u32 + 0.02 || (tie48 && s.w < 128 && u48 >= u32 - 1e-9));
  t.tc = w48 ? 48 : 32;
  t.tr = w48 ? 4 : 8;
  t.tiles_x = (s.w + t.tc - 1) / t.tc;
  t.tiles_y = (s.h + t.tr - 1) / t.tr;
  if (!pool && !w48 && (double)s.w / (t.tiles_x * 32) < 0.9) return false;  // narrow maps: conv_big
  t.pitch = t.tc + 2;  // 16-px blocks never wrap a tile row: tight pitch
  t.hrows = t.tr + 2;
  t.nh = (t.hrows * t.pitch + 63) / 64;
  if (2 * 2 * 4 * 128 * 16 + 8 * t.nh * 1024 > 80 * 1024) return false;
  t.co_tiles = (cop_max + 127) / 128;
  t.units = groups * t.co_tiles;
  t.per_unit = s.n * t.tiles_y * t.tiles_x;
  t.xpu = (t.units <= 8 && 8 % t.units == 0) ? 8 / t.units : 0;
  // pixel-major XCD order when several weight sets share the input and all of them fit an XCD's
  // 4 MiB L2 beside the streamed halos (OP_M16K_PMAJ: 1 when they fit, 2 always; default off: no
  // gain in an interleaved A/B, the MALL already serves the second read)
  static const int pmaj = getenv("OP_M16K_PMAJ") ? atoi(getenv("OP_M16K_PMAJ")) : 0;
  const double wset = (double)s.c16 * 16 * 9 * 128 * 4;  // one weight set, split bf16 bytes
  t.per_xcd = 0;
  if (groups == 1 && t.co_tiles > 1 && (pmaj == 2 || (pmaj == 1 && t.units * wset <= 3.0 * 1024 * 1024)))
    t.per_xcd = (t.per_unit + 7) / 8;
  return true;
}

static int launch_m16k(const SplitConvShape& s, const SplitConvGroup* g, const BigTiling& tl, bool pool, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    OP_HIP_CHECK(hipFuncSetAttribute((const void*)conv_m16k_bf16x3<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     80 * 1024));
    OP_HIP_CHECK(hipFuncSetAttribute((const void*)conv_m16k_bf16x3<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     80 * 1024));
    attr = true;
  }
  const int lds = 2 * 2 * 4 * 128 * 16 + 8 * tl.nh * 1024;
  const unsigned blocks = tl.per_xcd ? 8u * (unsigned)(tl.per_xcd * tl.units)
                          : tl.xpu   ? 8u * (unsigned)((tl.per_unit + tl.xpu - 1) / tl.xpu)
                                     : (unsigned)(tl.units * tl.per_unit);
  const SplitConvGroup& g1 = s.groups > 1 ? g[1] : g[0];
  // split-K when the launch fills few of the 512 workgroup slots (two per CU): one frame's
  // 46-wide layers (12-48 workgroups); partials reduced by conv_m16_splitk_reduce
  BigTiling t = tl;
  t.ksplit = 1;
  t.ws = nullptr;
  static const int ks_force = getenv("OP_M16_KSPLIT") ? atoi(getenv("OP_M16_KSPLIT")) : 0;  // A/B aid: 1 = off
  // A/B aid: the split launch's workgroup cap (default 512 = two per CU)
  static const int split_wg = getenv("OP_M16K_SPLIT_WG") ? atoi(getenv("OP_M16K_SPLIT_WG")) : 512;
  if (s.splitk && (!pool || s.groups == 1)) {
    const int pairs = s.c16 / 2;
    int S = 1;
    if (ks_force > 0) S = pairs % ks_force == 0 ? ks_force : 1;
    else
      for (int cand : {8, 4, 2})
        if (pairs % cand == 0 && (int)blocks * cand <= split_wg) {
          S = cand;
          break;
        }
    if (S > (pool ? 8 : kMaxSplitK)) S = 1;  // the reduce kernels' unrolled partial loads
    if (S > 1) {
      int cop_max = g[0].cop;
      if (s.groups > 1) cop_max = std::max(cop_max, g[1].cop);
      t.hw = s.h * s.w;
      t.total = s.n * s.h * s.w;
      float* ws = splitk_ws(st, (size_t)S * s.groups * t.total * cop_max);
      if (ws) {
        t.ksplit = S;
        t.ws = ws;
      }
    }
  }
  const dim3 grid(blocks, (unsigned)t.ksplit);
  census_add(pool ? OP_CENSUS_3X3_POOL : tl.tc == 48 ? OP_CENSUS_3X3_W48 : OP_CENSUS_3X3_W32);
  if (t.ksplit > 1) census_add(OP_CENSUS_3X3_SPLITK);
  if (pool)
    hipLaunchKernelGGL(conv_m16k_bf16x3<true>, grid, dim3(256), lds, st, s, g[0], g1, t);
  else if (tl.tc == 48) {
    const int rc = launch_m16k_wide(grid, lds, st, s, g[0], g1, t);
    if (rc != OP_OK) return rc;
  } else
    hipLaunchKernelGGL(conv_m16k_bf16x3<false>, grid, dim3(256), lds, st, s, g[0], g1, t);
  OP_AFTER_LAUNCH("conv_m16k_bf16x3", st);
  if (t.ksplit > 1 && pool) {
    const int64_t items = (int64_t)s.n * (s.h / 2) * (s.w / 2) * (g[0].cop / 4);
    hipLaunchKernelGGL(conv_m16_splitk_reduce_pool, dim3((unsigned)((items + 255) / 256)), dim3(256), 0, st, s, g[0], t);
    OP_AFTER_LAUNCH("conv_m16_splitk_reduce_pool", st);
  } else if (t.ksplit > 1) {
    int cop_max = g[0].cop;
    if (s.groups > 1) cop_max = std::max(cop_max, g[1].cop);
    const int64_t items = (int64_t)t.total * (cop_max / 4);
    hipLaunchKernelGGL(conv_m16_splitk_reduce, dim3((unsigned)((items + 255) / 256), (unsigned)s.groups), dim3(256), 0,
                       st, s, g[0], g1, t);
    OP_AFTER_LAUNCH("conv_m16_splitk_reduce", st);
  }
  OP_HIP_CHECK(hipGetLastError());
  return OP_OK;
}

// 3x3 conv + ReLU + 2x2 max-pool in one launch: s.h x s.w is the conv size, the output buffer is
// (s.h/2) x (s.w/2) with halo s.pout.  Tiles are 32 columns x (pixel groups x NPB) rows.
// *taken = 0 when the shape is outside this kernel (the caller runs conv + pool).
int launch_conv_big_pool(const SplitConvShape& s, const SplitConvGroup* g, hipStream_t st, int* taken) {
  *taken = 0;
  if (s.ks != 3 || s.groups != 1 || s.cs_in % 16 || s.pin < 1 || (s.h & 1) || (s.w & 1) || g[0].cop % 64 ||
      g[0].cin_off % 16 || !s.relu)
    return OP_OK;
  const bool c128 = g[0].cop % 128 == 0;
  BigTiling t{};
  if (c128 && m16k_tiling(s, 1, g[0].cop, true, t)) {
    // large launches of the shapes conv_m16k takes run the register-weight kernel instead: the
    // same accumulation order, so a frame's result does not depend on which of the two ran
    const int rc = launch_conv_m16r(s, g, true, st, taken);
    if (rc != OP_OK || *taken) return rc;
    *taken = 1;
    return launch_m16k(s, g, t, true, st);
  }
  const BigConfig k = c128 ? BigConfig{3, 6, 4, 128, 0} : BigConfig{3, 4, 4, 64, 0};
  t.tc = 32;
  t.tr = k.cap() / 32;  // rows = pixel groups x NPB (even)
  if (halo_bytes(t.tr, t.tc, 3) > k.halo_budget()) return OP_OK;
  t.tiles_y = (s.h + t.tr - 1) / t.tr;
  t.tiles_x = (s.w + 31) / 32;
  t.pitch = halo_pitch(32, 3);
  t.hrows = t.tr + 2;
  t.nh = (t.hrows * t.pitch + 63) / 64;
  t.co_tiles = g[0].cop / k.cw;
  t.units = t.co_tiles;
  t.per_unit = s.n * t.tiles_y * t.tiles_x;
  t.xpu = (t.units <= 8 && 8 % t.units == 0) ? 8 / t.units : 0;
  *taken = 1;
  if (c128) return launch_big_t<3, 6, 4, 128, 0, true>(s, g, t, st);
  return launch_big_t<3, 4, 4, 64, 0, true>(s, g, t, st);
}

// The split-path convolution on shared-weight halo tiles (7x7 and 3x3).  *taken = 0 when the
// shape is outside these kernels (the caller falls back).
// whether launch_conv_big runs a 7x7 launch of this shape on conv_m16_bf16x3 (the only kernel
// that reads and writes chunk-planar tensors)
bool conv_m16_takes(int n, int h, int w, int groups, int cop_max) {
  BigTiling tl{};
  return cop_max % 128 == 0 && raster_tiling(BigConfig{7, 5, 8, 128, 1, 1}, n, h, w, groups, cop_max, tl, true);
}

// Small 7x7 launches (round 5): conv_m16q_bf16x3 (conv_m16q.hip) where split-K is allowed and the
// launch covers at most OP_M16Q_MAX_PX pixels (default 4800: one 368x368 frame's 46 x 46 maps, not
// C4's or C5's batches); OP_M16Q=0 (read per launch) keeps them on conv_m16.  Tiles of OP_M16Q_TR
// rows (2 / 4 / 8; default 4) x 16 columns, split K over the chunk pairs x OP_M16Q_NTH tap ranges
// (2..4, default 2, lowered until the splits fit kMaxSplitK), weights OP_M16Q_PF (2 / 4, default 2)
// taps ahead; the partials go through conv_m16_splitk_reduce like conv_m16's.  One frame's 7x7
// class 1.02 -> 0.95 ms (TR 2 / 8, NTH 3 / 4, PF 4 / 6 no better: profiles/r05/ab_r05s_*.log).
// *taken = 0 when the launch is outside it.
static int launch_conv_m16q(const SplitConvShape& s, const SplitConvGroup* g, int cop_max, hipStream_t st,
                            int* taken) {
  *taken = 0;
  const char* on = getenv("OP_M16Q");
  if ((on && atoi(on) == 0) || !s.splitk || s.ks != 7 || s.pin < 3 || (s.c16 & 1) || cop_max % 128) return OP_OK;
  static const int64_t max_px = getenv("OP_M16Q_MAX_PX") ? atoll(getenv("OP_M16Q_MAX_PX")) : 4800;
  if ((int64_t)s.n * s.h * s.w > max_px) return OP_OK;
  for (int i = 0; i < s.groups; ++i)
    if (g[i].cop % 128 || g[i].cin_off % 16) return OP_OK;
  const char* tr_env = getenv("OP_M16Q_TR");  // (read per launch: A/B and test aids)
  const char* nth_env = getenv("OP_M16Q_NTH");
  const char* pf_env = getenv("OP_M16Q_PF");
  const int tr = tr_env ? atoi(tr_env) : 4;
  const int nth0 = nth_env ? atoi(nth_env) : 2;
  const int pf = pf_env ? atoi(pf_env) : 2;
  if (tr != 2 && tr != 4 && tr != 8) return OP_OK;
  const int ncp = s.c16 / 2;
  // the instantiated kernels: TR 4 with 2..4 tap ranges and prefetch 2 / 4; TR 2 / 8 with 2 and 2
  int nth = tr == 4 ? std::max(2, std::min(nth0, 4)) : 2;
  const int pfk = tr == 4 && pf == 4 ? 4 : 2;
  while (nth > 2 && ncp * nth > kMaxSplitK) --nth;
  if (ncp * nth > kMaxSplitK) return OP_OK;
  // round 6, opt-in (OP_M16Q_IWG=1): the 2 tap ranges of a chunk pair in one 8-wave workgroup,
  // summed in LDS, so split K = the chunk pairs and the reduce reads half the partials -- measured
  // slower: one frame's 7x7 class 0.95 -> 0.99 ms (profiles/r06/ab_r06g_b1_m16q_iwg_not_kept.log),
  // the 8-wave workgroups' exchange and barrier cost more than the halved partial traffic saves
  const char* iwg_env = getenv("OP_M16Q_IWG");
  const bool iwg = tr == 4 && nth == 2 && pfk == 2 && iwg_env && atoi(iwg_env) == 1;
  BigTiling t{};
  t.tr = tr;
  t.tc = 16;
  t.tiles_x = (s.w + 15) / 16;
  t.tiles_y = (s.h + tr - 1) / tr;
  t.co_tiles = cop_max / 128;
  t.units = s.groups * t.co_tiles;
  t.per_unit = s.n * t.tiles_y * t.tiles_x;
  t.hw = s.h * s.w;
  t.total = s.n * t.hw;
  t.ksplit = iwg ? ncp : ncp * nth;
  float* ws = splitk_ws(st, (size_t)t.ksplit * s.groups * t.total * cop_max);
  if (!ws) return OP_OK;  // capturing with a short workspace: conv_m16 unsplit now, re-captured later
  t.ws = ws;
  *taken = 1;
  census_add(OP_CENSUS_7X7_Q);
  census_add(OP_CENSUS_7X7_SPLITK);
  if (s.in_planar) census_add(OP_CENSUS_7X7_PLANAR);
  const SplitConvGroup& g1 = s.groups > 1 ? g[1] : g[0];
  if (iwg) census_add(OP_CENSUS_7X7_Q_IWG);
  // round 6: B fragments one tap ahead, by default (OP_M16Q_BPF=0, read per launch, reads them at the
  // tap): one frame's 7x7 class 0.950-0.968 -> 0.943-0.959 ms in 5 interleaved rounds on two boxes
  // (profiles/r06/ab_r06r_b1_m16q_bpf_split_wg.log, ab_r06t_b1_m16q_bpf.log); bit-identical
  const char* bpf_env = getenv("OP_M16Q_BPF");
  const bool bpf = !iwg && tr == 4 && nth == 2 && pfk == 2 && !(bpf_env && atoi(bpf_env) == 0);
  if (bpf) census_add(OP_CENSUS_7X7_Q_BPF);
  const int rc = launch_m16q_7x7(tr, nth, pfk, st, s, g[0], g1, t, iwg, bpf);
  if (rc != OP_OK) return rc;
  OP_AFTER_LAUNCH("conv_m16q_bf16x3", st);
  const int64_t items = (int64_t)t.total * (cop_max / 4);
  hipLaunchKernelGGL(conv_m16_splitk_reduce, dim3((unsigned)((items + 255) / 256), (unsigned)s.groups), dim3(256), 0,
                     st, s, g[0], g1, t);
  OP_AFTER_LAUNCH("conv_m16_splitk_reduce", st);
  OP_HIP_CHECK(hipGetLastError());
  return OP_OK;
}

int launch_conv_big(const SplitConvShape& s, const SplitConvGroup* g, hipStream_t st, int* taken) {
  *taken = 0;
  if ((s.ks != 7 && s.ks != 3) || s.cs_in % 16 || s.pin < s.ks / 2) return OP_OK;
  int cop_max = 0;
  bool c128 = true;
  for (int i = 0; i < s.groups; ++i) {
    if (g[i].cop % 64 || g[i].cin_off % 16) return OP_OK;
    if (g[i].cop % 128) c128 = false;
    cop_max = cop_max > g[i].cop ? cop_max : g[i].cop;
  }
  static const bool plain_order = getenv("OP_BIG_PLAIN_ORDER") != nullptr;  // tuning aid: no XCD remap
  BigTiling tl{};
  if (s.ks == 7) {
    if (!c128) return OP_OK;
    {
      int rc = launch_conv_m16w(s, g, cop_max, st, taken);  // opt-in experiment (OP_M16W=1)
      if (rc != OP_OK || *taken) return rc;
      rc = launch_conv_m16q(s, g, cop_max, st, taken);
      if (rc != OP_OK || *taken) return rc;
    }
    if (raster_tiling(BigConfig{7, 5, 8, 128, 1, 1}, s.n, s.h, s.w, s.groups, cop_max, tl, true)) {
      // default: 16x16x32 tap pairs on raster tiles, 10 blocks of 16 px per wave = the 640-px tile of npb 5
      // Tile size per launch shape.  A workgroup's time grows as ~(2 + NPX) (fixed halo /
      // weight-ring / barrier work plus NPX 16-px blocks per wave; measured 0.17 / 0.25 / 0.50 ms
      // for NPX 2 / 4 / 10), one workgroup per CU, so a launch costs rounds x (2 + NPX) with
      // rounds = workgroups per XCD / 32 CUs, rounded up.  640-px tiles (NPX 10) stay unless a
      // smaller tile costs less (the 38-frame batch: 252 workgroups, one round, kept); the
      // candidates are NPX 8, 6, 5, 4, 3, 2 (one crop: 2; 16 frames: 5 -> 212
      // workgroups in one round instead of 106 at 2.4x the work each; 40-57 frames: 8, two
      // rounds of 512-px tiles instead of two of 640).
      static const int force = getenv("OP_M16_NPX") ? atoi(getenv("OP_M16_NPX")) : 0;  // A/B aid
      // channel tiles that share their input (one group, Mconv1's 256 channels): a pixel tile's
      // tiles back to back on one XCD -- OFF by default (OP_M16_PAIR=1 selects it): neutral in a
      // 3-run A/B on the headline (1869.3 vs 1868.0 frames/s, profiles/r04/ab_r04i_mconv1_pair.log),
      // so the round-3 mapping (one channel tile per XCD set) stays.  Applied to every candidate
      // tiling before it is costed (the grid grows to whole XCD rounds)
      static const bool m16_pair = getenv("OP_M16_PAIR") && atoi(getenv("OP_M16_PAIR")) == 1;
      auto pairmaj = [&](BigTiling& t) {
        t.pair = 1;
        if (m16_pair && !plain_order && t.xpu && s.groups == 1 && t.co_tiles > 1 && 8 % t.co_tiles == 0) {
          t.pair = t.co_tiles;
          t.xpu = 8;
        }
      };
      pairmaj(tl);
      auto rounds = [](const BigTiling& t) -> int {
        const int P = t.pair > 1 ? t.pair : 1;
        return t.xpu ? ((t.per_unit + t.xpu - 1) / t.xpu * P + 31) / 32 : (t.units * t.per_unit + 255) / 256;
      };
      // Split-K (launches that leave CUs idle: one frame, one crop; never in batch-invariant mode):
      // the input chunks are divided over blockIdx.y (f32 partials + conv_m16_splitk_reduce).  Round
      // 4: the tile size and the split S are chosen together -- a workgroup's time is ~ its chunks x
      // (2 + NPX), a launch's ~ rounds x that, plus ~0.2 of a unit per split for the partials and the
      // reduce launch (OP_M16_SPLIT_GAMMA) -- over S dividing the chunk count (2 .. 16, not just
      // 8 / 4 / 2): one 368x368 frame's Mconv2-5 take NPX 3 x S 8 (176 workgroups, one chunk each)
      // instead of NPX 2 x S 4 (136 workgroups, two chunks each), Mconv1 NPX 4 x S 12.
      static const int ks_force = getenv("OP_M16_KSPLIT") ? atoi(getenv("OP_M16_KSPLIT")) : 0;  // A/B aid: 1 = off
      static const bool joint = !(getenv("OP_M16_JOINT") && atoi(getenv("OP_M16_JOINT")) == 0);  // A/B aid
      static const double gamma = getenv("OP_M16_SPLIT_GAMMA") ? atof(getenv("OP_M16_SPLIT_GAMMA")) : 0.2;
      static const bool plain_small = !(getenv("OP_M16_PLAIN_SMALL") && atoi(getenv("OP_M16_PLAIN_SMALL")) == 0);
      auto wgs_of = [](const BigTiling& t) -> int {
        return t.xpu ? 8 * ((t.per_unit + t.xpu - 1) / t.xpu) * (t.pair > 1 ? t.pair : 1) : t.units * t.per_unit;
      };
      // every launch shape is evaluated once (the tilings loop over tiles) and cached
      static std::mutex sel_mu;
      static std::map<std::array<int, 7>, std::tuple<int, BigTiling, int>> sel_cache;
      const std::array<int, 7> key{s.n, s.h, s.w, s.groups, cop_max, s.c16, s.splitk};
      int npx = 10, S = 1;
      {
        std::lock_guard<std::mutex> lk(sel_mu);
        auto it = sel_cache.find(key);
        if (it != sel_cache.end()) {
          npx = std::get<0>(it->second);
          tl = std::get<1>(it->second);
          S = std::get<2>(it->second);
        } else {
          // round 4: NPX 9 and 7 as well (OP_M16_ODD=0: off), e.g. the C4 scale-1.5 launches: 472
          // workgroups of 576 px in 2 rounds instead of 448 of 640 px (1.75 rounds, cost 22 vs 24)
          static const bool odd = !(getenv("OP_M16_ODD") && atoi(getenv("OP_M16_ODD")) == 0);
          if (force != 10) {
            int best = rounds(tl) * (2 + 10);
            for (int cand : {9, 8, 7, 6, 5, 4, 3, 2}) {
              if (force && cand != force) continue;
              if (!odd && (cand == 9 || cand == 7)) continue;
              BigConfig k{7, 1, 8, 128, 1, 1};
              k.cap_px = 64 * cand;
              BigTiling tc{};
              if (!raster_tiling(k, s.n, s.h, s.w, s.groups, cop_max, tc, true)) continue;
              pairmaj(tc);
              const int cost = rounds(tc) * (2 + cand);
              if (force || cost < best) {
                best = cost;
                npx = cand;
                tl = tc;
              }
            }
          }
          if (s.splitk && ks_force > 0) {
            S = s.c16 % ks_force == 0 ? ks_force : 1;
          } else if (s.splitk && !joint) {  // round 3's rule: the no-split tile, the largest S of 8 / 4 / 2 that fits
            for (int cand : {8, 4, 2})
              if (s.c16 % cand == 0 && wgs_of(tl) * cand <= 256) {
                S = cand;
                break;
              }
          } else if (s.splitk && wgs_of(tl) < 256) {
            double best = (double)rounds(tl) * s.c16 * (2 + npx);
            static const bool odd_split = getenv("OP_M16_ODD_SPLIT") && atoi(getenv("OP_M16_ODD_SPLIT")) == 1;
            for (int cand : {10, 9, 8, 7, 6, 5, 4, 3, 2}) {
              if (force && cand != force) continue;
              if (!odd_split && (cand == 9 || cand == 7)) continue;
              BigConfig k{7, 1, 8, 128, 1, 1};
              k.cap_px = 64 * cand;
              BigTiling tc{};
              if (!raster_tiling(k, s.n, s.h, s.w, s.groups, cop_max, tc, true)) continue;
              pairmaj(tc);
              // round 4: also the plain block order -- the XCD-aware grid pads each XCD's share of
              // a weight set to whole slots, so a split launch of few tiles (one frame's Mconv1: 9
              // tiles x 2 sets x 12 splits = 216 workgroups) takes a second round it does not need
              // (288 grid slots); plain order keeps such a launch in one (OP_M16_PLAIN_SMALL=0: off)
              BigTiling tp = tc;
              tp.xpu = 0;
              tp.pair = 1;
              for (int ord = 0; ord < (plain_small ? 2 : 1); ++ord) {
                const BigTiling& tt = ord ? tp : tc;
                for (int sp : {2, 3, 4, 6, 8, 12, 16}) {
                  if (s.c16 % sp) continue;
                  const int r = (wgs_of(tt) * sp + 255) / 256;
                  const double cost = (double)r * (s.c16 / sp) * (2 + cand) + gamma * sp;
                  if (cost < best) {
                    best = cost;
                    npx = cand;
                    tl = tt;
                    S = sp;
                  }
                }
              }
            }
          }
          sel_cache[key] = std::make_tuple(npx, tl, S);
        }
      }
      if (plain_order) {
        tl.xpu = 0;
        tl.pair = 1;
      }
      tl.zeros = device_zeros();
      // round 6: LIN tiles within one frame load only their own halo rows (default; OP_M16_TRIM=0, read
      // per launch, loads the plane's nh pieces sized for the frame-crossing tiles)
      const char* trim_env = getenv("OP_M16_TRIM");
      tl.halo_trim = !(trim_env && atoi(trim_env) == 0);
      if (!tl.zeros) {
        set_error("conv_m16_bf16x3: conv_big_device_init was not called for this device");
        return OP_ERR_STATE;
      }
      *taken = 1;
      tl.ksplit = 1;
      tl.ws = nullptr;
      if (S > kMaxSplitK) S = 1;  // the reduce's unrolled partial loads
      if (s.splitk && S > 1) {
        float* ws = splitk_ws(st, (size_t)S * s.groups * tl.total * cop_max);
        if (ws) {
          tl.ksplit = S;
          tl.ws = ws;
        }
      }
      const SplitConvGroup& g1 = s.groups > 1 ? g[1] : g[0];
      census_add(npx);
      if (tl.ksplit > 1) census_add(OP_CENSUS_7X7_SPLITK);
      if (s.in_planar) census_add(OP_CENSUS_7X7_PLANAR);
      if (tl.fa_tiles) census_add(OP_CENSUS_7X7_FRAME_ALIGNED);
      if (tl.pitch == s.w + 6) census_add(OP_CENSUS_7X7_TIGHT);
      const int rc = launch_m16_7x7(npx, st, s, g[0], g1, tl);
      if (rc != OP_OK) return rc;
      if (tl.ksplit > 1) {
        OP_AFTER_LAUNCH("conv_m16_bf16x3", st);
        const int64_t items = (int64_t)tl.total * (cop_max / 4);
        hipLaunchKernelGGL(conv_m16_splitk_reduce, dim3((unsigned)((items + 255) / 256), (unsigned)s.groups), dim3(256),
                           0, st, s, g[0], g1, tl);
      }
      OP_AFTER_LAUNCH("conv_m16_bf16x3", st);
      OP_HIP_CHECK(hipGetLastError());
      return OP_OK;
    }
    if (s.in_planar || s.out_planar) return OP_OK;  // the caller reports it
    if (raster_tiling(BigConfig{7, 6, 8, 128, 1, 1}, s.n, s.h, s.w, s.groups, cop_max, tl)) {
      if (plain_order) tl.xpu = 0;
      *taken = 1;
      return launch_big_t<7, 6, 8, 128, 1, false, true>(s, g, tl, st);
    }
    if (!big_tiling(BigConfig{7, 6, 8, 128, 1}, s.n, s.h, s.w, s.groups, cop_max, tl)) return OP_OK;
    if (plain_order) tl.xpu = 0;
    *taken = 1;
    return launch_big_t<7, 6, 8, 128, 1>(s, g, tl, st);
  }
  if (c128) {
    if (m16k_tiling(s, s.groups, cop_max, false, tl)) {
      const int rc = launch_conv_m16r(s, g, false, st, taken);  // large launches (same order, above)
      if (rc != OP_OK || *taken) return rc;
      if (plain_order) tl.xpu = 0;
      *taken = 1;
      return launch_m16k(s, g, tl, false, st);
    }
    if (!big_tiling(BigConfig{3, 6, 4, 128, 0}, s.n, s.h, s.w, s.groups, cop_max, tl)) return OP_OK;
    if (plain_order) tl.xpu = 0;
    *taken = 1;
    return launch_big_t<3, 6, 4, 128, 0>(s, g, tl, st);
  }
  if (!big_tiling(BigConfig{3, 3, 4, 64, 0}, s.n, s.h, s.w, s.groups, cop_max, tl)) return OP_OK;
  if (plain_order) tl.xpu = 0;
  *taken = 1;
  return launch_big_t<3, 3, 4, 64, 0>(s, g, tl, st);
}

}  // namespace op

int op_conv_census(int32_t* counts, int32_t n, int32_t reset) {
  if (!counts || n < 1) return OP_ERR_INVALID;
  for (int i = 0; i < OP_CENSUS_SLOTS; ++i) {
    const int64_t v = reset ? op::g_census[i].exchange(0) : op::g_census[i].load();
    if (i < n) counts[i] = (int32_t)std::min<int64_t>(v, INT32_MAX);
  }
  for (int i = OP_CENSUS_SLOTS; i < n; ++i) counts[i] = 0;
  return OP_OK;
}
