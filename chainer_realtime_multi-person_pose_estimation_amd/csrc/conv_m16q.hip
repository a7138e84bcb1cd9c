// conv_m16q_bf16x3: the 7x7 stage convolutions of launches too small to fill the chip -- one
// 368x368 frame's Mconv1..5 (46 x 46 maps, CocoPoseNet.py:167-260) -- round 5.
//
// Same arithmetic as every bf16x3 kernel: v_mfma_f32_16x16x32_bf16, three bf16 products per
// f32-accurate MAC (hi*hi, hi*lo, lo*hi).  What differs from conv_m16_bf16x3 (the raster kernel
// that runs the batched launches) is the decomposition.  One frame's launch is 2 x 128 x 128 x 49
// MACs over 2116 pixels: conv_m16's 8-wave workgroups with a shared LDS weight ring take one CU
// each (176 of 256 at 192-px tiles x 8 chunk splits) and pay a ring barrier + weight LDS-DMA for
// every tap pair of only 3 pixel blocks per wave (29 us per launch, 0.23 of the 833 TF/s peak).
// Here:
//
// * a workgroup is 4 independent waves over one TR x 16 pixel tile of one frame, 32 output
//   channels each (128 per workgroup), and ONE input chunk pair (K = 32 of an MFMA = one tap of two
//   16-channel chunks, as in conv_m16r) over a RANGE of the 49 taps: the split-K index covers
//   (chunk pair, tap range), so one frame's Mconv2-5 run 36 tiles x 2 branches x 4 pairs x 2 tap
//   halves = 576 workgroups (2-3 per CU) instead of 176;
// * A (weights) stream from L2 into registers PF taps ahead, straight from the packed
//   [c16][tap][plane][cop][8] layout (no ring, no per-tap barrier); the workgroup's weight sets are
//   laid out so XCD x runs the sets = x mod 8, i.e. each XCD's L2 holds 1/8 of the launch's weights;
// * B (pixels) from an LDS halo of the chunk pair, staged once by LDS-DMA (one barrier per
//   workgroup);
// * f32 partials per split, summed in split order with the bias and ReLU by the existing
//   conv_m16_splitk_reduce (so the output layout, plain or chunk-planar, is the reduce's).
//
// Measured (profiles/r05/ab_r05s_*.log, m16q_stamps_r05s.txt): 27.2 us per Mconv2-5 launch vs 29.0
// on conv_m16, the one-frame 7x7 class 1.02 -> 0.95 ms.  The kernel is not MFMA-bound: with five
// of its six MFMAs per block removed it still took ~80 % of the time, and without the per-tap
// weight loads or with every tap reading tap 0's pixels ~97 %; its workgroups (2-3 per CU, all
// resident) spend 84 % in the tap loop at ~1800 cycles per tap per wave against 384 of MFMA issue.
// Prefetch 2 / 4 / 6 taps ahead, product-major MFMA order, a cap of 3 workgroups per CU and a
// rolled tap loop (a tenth of the code) measured within noise.
//
// Launch contract (launch_conv_m16q in conv_big.hip checks it): ks = 7, pin >= 3, c16 even, every
// group's cop a multiple of 128, tl.ksplit = (c16 / 2) * nth <= kMaxSplitK, tl.ws sized
// [ksplit][groups][total][max cop].
#include <type_traits>

#include "conv_big.hpp"

namespace op {

#ifndef M16Q_STAMPS
#define M16Q_STAMPS 0  // diagnostic build only: per-workgroup phase times (OP_M16Q_STAMPS=1 prints them)
#endif
#if M16Q_STAMPS
// [0] first start, [1] last end, [7] last start (s_memrealtime, 100 MHz); [2] workgroup cycles,
// [3] prologue, [4] tap loop, [5] epilogue (s_memtime sums); [6] workgroups
__device__ unsigned long long g_q_st[8];
#endif

// LDS-DMA of 16 B per lane (inline asm: the compiler's waitcnt pass does not track it, so the halo
// is waited for explicitly; nothing else in this kernel uses M0)
__device__ __forceinline__ void q_dma16(const void* gsrc, uint32_t lds_byte) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(gsrc), "s"(lds_byte) : "memory");
}

// IWG (round 6, opt-in OP_M16Q_IWG=1, measured slower at one frame): the NTH tap ranges of a chunk pair run in ONE workgroup of 4 x NTH waves (waves
// 4r .. 4r + 3: tap range r) over the shared halo, and the ranges' accumulators are summed in LDS
// (range 0 + range 1 + ..., exchanged through the halo's space) before the f32 partials are
// written: the split-K index is the chunk pair alone, so the partials and the reduce launch that
// reads them shrink NTH-fold (one frame's Mconv2-5: 8 -> 4 partials of 8.7 MB).
// BPF (round 6): the tap's B fragments (TR rows x hi / lo, 8 ds_read_b128 at TR 4) are read from LDS
// one tap ahead into PF + 1 register sets, so a tap's MFMAs start on fragments that landed a whole
// tap earlier; without it each tap waits for its own 8 LDS reads at its first MFMA and again for the
// last two in its middle (the compiled loop: s_waitcnt lgkmcnt(0) before the first MFMA of a tap).
template <int KS, int TR, int NTH, int PF, bool IWG = false, bool BPF = false>
__global__ __launch_bounds__(IWG ? 256 * NTH : 256, 3) void conv_m16q_bf16x3(SplitConvShape s, SplitConvGroup g0,
                                                                            SplitConvGroup g1, BigTiling tl) {
  constexpr int KSQ = KS * KS, R = KS / 2;
  constexpr int TC = 16;                 // tile columns (one 16-px block per tile row)
  constexpr int PITCH = TC + KS - 1;     // halo row pitch in 16-B slots
  constexpr int HROWS = TR + KS - 1;
  constexpr int NH = (HROWS * PITCH + 63) / 64;  // 1-KiB pieces per halo plane
  constexpr int HPLANE = NH * 1024;
  constexpr int NWV = IWG ? 4 * NTH : 4;  // waves per workgroup
  constexpr int PIECES = 8 * NH / NWV;   // 8 planes x NH pieces over the waves
  static_assert((8 * NH) % NWV == 0, "halo pieces split evenly over the waves");
  static_assert(!IWG || 4 * 64 * 2 * TR * 16 <= 8 * NH * 1024, "tap-range exchange fits the halo's LDS");
  extern __shared__ __attribute__((aligned(16))) char lds[];  // [8 planes][NH KiB]

  // block -> (pixel tile, weight set); weight set = (unit, split), split = (chunk pair, tap range)
  const int nws = tl.units * tl.ksplit;
  const int lin = blockIdx.x;
  const int tile = lin / nws, wsi = lin - (lin / nws) * nws;
  if (tile >= tl.per_unit) return;
  const int unit = wsi / tl.ksplit, sp = wsi - (wsi / tl.ksplit) * tl.ksplit;
  const int wave_ = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int cp = IWG ? sp : sp / NTH, th = IWG ? wave_ >> 2 : sp - (sp / NTH) * NTH;
  const int grp = unit / tl.co_tiles;
  const int co0 = (unit - grp * tl.co_tiles) * 128;
  const SplitConvGroup g = grp == 0 ? g0 : g1;
  if (co0 >= g.cop) return;
  const int t0 = th * KSQ / NTH, t1 = (th + 1) * KSQ / NTH;
  const int tpf = tl.tiles_y * tl.tiles_x;
  const int frame = tile / tpf;
  const int tix = tile - frame * tpf;
  const int ty = tix / tl.tiles_x;
  const int y0 = ty * TR, x0 = (tix - ty * tl.tiles_x) * TC;

#if M16Q_STAMPS
  const unsigned long long q_r0 = __builtin_amdgcn_s_memrealtime(), q_t0 = __builtin_amdgcn_s_memtime();
#endif
  const int lane = threadIdx.x & 63;
  const int wave = IWG ? (wave_ & 3) : wave_;  // this wave's 32-channel slice
  const int l16 = lane & 15, kg = lane >> 4;
  const int csel = kg >> 1, khalf = kg & 1;
  const int wp_in = s.w + 2 * s.pin;
  const int hp_in = s.h + 2 * s.pin;
  const int64_t pix_bytes = (int64_t)s.cs_in * 4;
  const int64_t in_pc = split_piece_stride(s.in_planar, hp_in, wp_in);
  const int64_t in_px = split_pixel_stride(s.in_planar, s.cs_in);
  const char* const fbase = (const char*)g.in + (int64_t)frame * hp_in * wp_in * pix_bytes;
  const uint32_t lds0 = (uint32_t)(size_t)(__attribute__((address_space(3))) char*)lds;

  // ---- A: this wave's 32 channels of chunk 2 cp + csel, k-half khalf, tap t ----
  const int64_t wplane = (int64_t)g.cop * 16;
  const int cw0 = co0 + wave * 32;
  const char* const wlane =
      (const char*)g.w + ((int64_t)((2 * cp + csel) * KSQ) * 4 + 2 * khalf) * wplane + (int64_t)(cw0 + l16) * 16;
  typedef bf16x8g AFrag[4];  // [cb * 2 + hl]
  auto load_a = [&](int t, AFrag& a) {
    if (t >= t1) t = t1 - 1;  // the last taps' prefetch re-reads the final tap (unused)
    const char* p = wlane + (int64_t)t * 4 * wplane;
    a[0] = *(const bf16x8g*)p;
    a[1] = *(const bf16x8g*)(p + wplane);
    a[2] = *(const bf16x8g*)(p + 256);
    a[3] = *(const bf16x8g*)(p + wplane + 256);
  };

  // ---- B: the chunk pair's halo, (TR + 6) x (16 + 6) slots per plane, 8 planes ----
#pragma unroll
  for (int k = 0; k < PIECES; ++k) {
    const int j = wave_ + NWV * k;
    const int plane = j / NH, i = j - (j / NH) * NH;
    const int cj = plane >> 2, pl = plane & 3;
    const int slot = i * 64 + lane;  // slots past the window read a clamped pixel, never used
    const int hr = slot / PITCH, hc = slot - (slot / PITCH) * PITCH;
    const int yy = min(y0 - R + hr + s.pin, hp_in - 1), xx = min(x0 - R + hc + s.pin, wp_in - 1);
    const char* src = fbase + (int64_t)((2 * cp + cj) * 4 + pl) * in_pc + (int64_t)(yy * wp_in + xx) * in_px;
    q_dma16(src, lds0 + (uint32_t)(plane * HPLANE + i * 1024));
  }
  // weights PF taps ahead (PF + 1 register sets; 2 by default, 4 instantiated for A/Bs)
  AFrag abuf[PF + 1];
#pragma unroll
  for (int k = 0; k < PF; ++k) load_a(t0 + k, abuf[k]);
  wait_vmcnt<0>();
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

#if M16Q_STAMPS
  const unsigned long long q_t1 = __builtin_amdgcn_s_memtime();
#endif
  floatx4 acc[2][TR];
#pragma unroll
  for (int cb = 0; cb < 2; ++cb)
#pragma unroll
    for (int pb = 0; pb < TR; ++pb) acc[cb][pb] = floatx4{0.f, 0.f, 0.f, 0.f};

  // this lane's slot in its (chunk csel, k-half khalf) hi plane; block pb = tile row pb
  const char* const hb = lds + (csel * 4 + 2 * khalf) * HPLANE + l16 * 16;
  typedef bf16x8g BFrag[TR][2];  // [pb][hi, lo]
  auto load_b = [&](int t, BFrag& b) {
    if (t >= t1) t = t1 - 1;  // the last tap's prefetch re-reads the final tap (unused)
    const int tr = t / KS, tc = t - (t / KS) * KS;
    const char* const tb = hb + (tr * PITCH + tc) * 16;
#pragma unroll
    for (int pb = 0; pb < TR; ++pb) {
      b[pb][0] = *(const bf16x8g*)(tb + pb * PITCH * 16);
      b[pb][1] = *(const bf16x8g*)(tb + pb * PITCH * 16 + HPLANE);
    }
  };
  BFrag bbuf[BPF ? 2 : 1];
  if constexpr (BPF) load_b(t0, bbuf[0]);
  // one tap: the weights of tap t + PF into buffer (B + PF) % (PF + 1), then tap t's MFMAs from
  // buffer B (K = the tap's index mod G, a compile-time constant; B = K mod PF + 1; BPF: the B
  // fragments of tap t + 1 into set (K + 1) mod 2, tap t's from set K mod 2)
  auto step = [&](int t, auto ksel) {
    constexpr int K = decltype(ksel)::value;
    constexpr int B = K % (PF + 1), BB = K % 2;
    load_a(t + PF, abuf[(B + PF) % (PF + 1)]);
    if constexpr (BPF) {
      // this tap's fragments (issued a tap ago) have landed before the next tap's are issued: at
      // most 8 LDS reads in flight (lgkmcnt is 4 bits); the builtin wait is visible to the
      // compiler's counter, so the MFMAs below need no further LDS wait
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0) (vmcnt 63, expcnt 7: no wait on those)
      load_b(t + 1, bbuf[BPF ? (BB + 1) % 2 : 0]);
    }
    __builtin_amdgcn_sched_barrier(0);  // keep the prefetch at the step's start
    const int tr = t / KS, tc = t - (t / KS) * KS;
    const char* const tb = hb + (tr * PITCH + tc) * 16;
    const AFrag& a = abuf[B];
#pragma unroll
    for (int pb = 0; pb < TR; ++pb) {
      const bf16x8g bh = BPF ? bbuf[BPF ? BB : 0][pb][0] : *(const bf16x8g*)(tb + pb * PITCH * 16);
      const bf16x8g bl = BPF ? bbuf[BPF ? BB : 0][pb][1] : *(const bf16x8g*)(tb + pb * PITCH * 16 + HPLANE);
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        acc[cb][pb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2 * cb], bh, acc[cb][pb], 0, 0, 0);
        acc[cb][pb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2 * cb], bl, acc[cb][pb], 0, 0, 0);
        acc[cb][pb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2 * cb + 1], bh, acc[cb][pb], 0, 0, 0);
      }
    }
    if constexpr (BPF) __builtin_amdgcn_sched_barrier(0);  // the next tap's loads stay behind these MFMAs
  };
  // A rolled loop of PF + 1 taps per iteration (each buffer index compile-time, so the back-edge
  // carries the buffers in place), then the 0..PF remaining taps: 989 instead of 2248 lines of
  // code with every tap unrolled, the same time (profiles/r05/ab_r05u_b1_m16q_rolled.log).
  // BPF: G = 2 (PF + 1) taps per iteration, so both the A and the B set indices are compile-time
  constexpr int G = BPF ? 2 * (PF + 1) : PF + 1;
  static_assert(G <= 6, "the unrolled iteration holds at most 6 taps");
  const int n = t1 - t0;
  const int ng = n / G;
  int t = t0;
#define M16Q_STEP(k) step(t + (k), std::integral_constant<int, ((k) < G ? (k) : 0)>())
#pragma unroll 1
  for (int i = 0; i < ng; ++i, t += G) {
    M16Q_STEP(0);
    M16Q_STEP(1);
    M16Q_STEP(2);
    if constexpr (G > 3) M16Q_STEP(3);
    if constexpr (G > 4) M16Q_STEP(4);
    if constexpr (G > 5) M16Q_STEP(5);
  }
  const int rem = n - ng * G;
  if (rem > 0) M16Q_STEP(0);
  if (rem > 1) M16Q_STEP(1);
  if constexpr (G > 3) {
    if (rem > 2) M16Q_STEP(2);
    if (rem > 3) M16Q_STEP(3);
  }
  if constexpr (G > 5) {
    if (rem > 4) M16Q_STEP(4);
  }
#undef M16Q_STEP

#if M16Q_STAMPS
  __builtin_amdgcn_sched_barrier(0);
  const unsigned long long q_t2 = __builtin_amdgcn_s_memtime();
  __builtin_amdgcn_sched_barrier(0);
#endif
  if constexpr (IWG) {
    // the tap ranges' sums: ranges 1 .. NTH-1 hand their accumulators to range 0 through LDS (the
    // halo's space, free once every wave is past its last tap), added in range order
    __syncthreads();
    float* const xch = (float*)lds;
    for (int r = 1; r < NTH; ++r) {
      if (th == r) {
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
#pragma unroll
          for (int pb = 0; pb < TR; ++pb) *(floatx4*)(xch + ((wave * 2 * TR + cb * TR + pb) * 64 + lane) * 4) = acc[cb][pb];
      }
      __syncthreads();
      if (th == 0) {
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
#pragma unroll
          for (int pb = 0; pb < TR; ++pb) {
            const floatx4 o = *(const floatx4*)(xch + ((wave * 2 * TR + cb * TR + pb) * 64 + lane) * 4);
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[cb][pb][e] += o[e];
          }
      }
      if (r + 1 < NTH) __syncthreads();
    }
    if (th != 0) return;
  }
  // ---- f32 partials of split sp: ws [split][group][pixel of the batch][wsc] ----
  const int wsc = max(g0.cop, g1.cop);
  float* const wsg = tl.ws + ((int64_t)sp * s.groups + grp) * (int64_t)tl.total * wsc;
  const int x = x0 + l16;
#pragma unroll
  for (int pb = 0; pb < TR; ++pb) {
    const int y = y0 + pb;
    if (y >= s.h || x >= s.w) continue;
    const int64_t P = (int64_t)frame * tl.hw + y * s.w + x;
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) *(floatx4*)(wsg + P * wsc + cw0 + cb * 16 + 4 * kg) = acc[cb][pb];
  }
#if M16Q_STAMPS
  wait_vmcnt<0>();
  __builtin_amdgcn_sched_barrier(0);
  const unsigned long long q_t3 = __builtin_amdgcn_s_memtime(), q_r3 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    atomicMin(&g_q_st[0], q_r0);
    atomicMax(&g_q_st[1], q_r3);
    atomicMax(&g_q_st[7], q_r0);
    atomicAdd(&g_q_st[2], q_t3 - q_t0);
    atomicAdd(&g_q_st[3], q_t1 - q_t0);
    atomicAdd(&g_q_st[4], q_t2 - q_t1);
    atomicAdd(&g_q_st[5], q_t3 - q_t2);
    atomicAdd(&g_q_st[6], 1ull);
  }
#endif
}

int launch_m16q_7x7(int tr, int nth, int pf, hipStream_t st, const SplitConvShape& s, const SplitConvGroup& g0,
                    const SplitConvGroup& g1, const BigTiling& tl, bool iwg, bool bpf) {
  // OP_M16Q_LDS_KB (A/B aid): allocate at least that much LDS per workgroup (caps workgroups per CU)
  static const int lds_min = getenv("OP_M16Q_LDS_KB") ? atoi(getenv("OP_M16Q_LDS_KB")) * 1024 : 0;
  auto lds_of = [](int r) { return std::max(lds_min, 8 * (((r + 6) * 22 + 63) / 64) * 1024); };
  const dim3 grid((unsigned)(tl.per_unit * tl.units * tl.ksplit));
#define M16Q_LAUNCH(R, T, P) \
  hipLaunchKernelGGL((conv_m16q_bf16x3<7, R, T, P>), grid, dim3(256), lds_of(R), st, s, g0, g1, tl)
  if (iwg) {  // one workgroup per chunk pair, its 2 tap ranges inside (tl.ksplit = chunk pairs)
    if (tr == 4 && nth == 2 && pf == 2) {
      hipLaunchKernelGGL((conv_m16q_bf16x3<7, 4, 2, 2, true>), grid, dim3(512), lds_of(4), st, s, g0, g1, tl);
    } else {
      set_error("conv_m16q_bf16x3 (tap ranges in one workgroup): tile rows 4, 2 tap ranges, prefetch 2 only");
      return OP_ERR_INVALID;
    }
  } else if (bpf) {  // B fragments one tap ahead (round 6): tile rows 4, prefetch 2, 2 tap ranges
    if (tr == 4 && nth == 2 && pf == 2) {
      hipLaunchKernelGGL((conv_m16q_bf16x3<7, 4, 2, 2, false, true>), grid, dim3(256), lds_of(4), st, s, g0, g1, tl);
    } else {
      set_error("conv_m16q_bf16x3 (B prefetch): tile rows 4, 2 tap ranges, prefetch 2 only");
      return OP_ERR_INVALID;
    }
  } else if (tr == 4 && (pf == 2 || pf == 4) && nth >= 2 && nth <= 4) {
#define M16Q_PF(P)                                  \
  if (pf == P) {                                    \
    if (nth == 2) M16Q_LAUNCH(4, 2, P);             \
    else if (nth == 3) M16Q_LAUNCH(4, 3, P);        \
    else M16Q_LAUNCH(4, 4, P);                      \
  }
    M16Q_PF(2)
    M16Q_PF(4)
#undef M16Q_PF
  } else if (tr == 2 && nth == 2 && pf == 2) {
    M16Q_LAUNCH(2, 2, 2);
  } else if (tr == 8 && nth == 2 && pf == 2) {
    M16Q_LAUNCH(8, 2, 2);
  } else {
    set_error("conv_m16q_bf16x3: tile rows " + std::to_string(tr) + ", tap ranges " + std::to_string(nth) +
              ", prefetch " + std::to_string(pf) + " not instantiated");
    return OP_ERR_INVALID;
  }
#undef M16Q_LAUNCH
#if M16Q_STAMPS
  static const bool dump = getenv("OP_M16Q_STAMPS") != nullptr;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (dump && hipStreamIsCapturing(st, &cs) == hipSuccess && cs == hipStreamCaptureStatusNone) {
    static double acc[8] = {};
    static int launches = 0;
    unsigned long long h[8];
    OP_HIP_CHECK(hipStreamSynchronize(st));
    OP_HIP_CHECK(hipMemcpyFromSymbol(h, HIP_SYMBOL(g_q_st), sizeof(h)));
    const unsigned long long z[8] = {~0ull, 0, 0, 0, 0, 0, 0, 0};
    OP_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_q_st), z, sizeof(z)));
    if (launches > 0 && h[6]) {  // (the first launch's minimum start is not initialised)
      acc[0] += (h[1] - h[0]) * 0.01;  // kernel span, us
      acc[1] += (h[7] - h[0]) * 0.01;  // start spread, us
      for (int i = 2; i < 6; ++i) acc[i] += (double)h[i] / h[6];
      acc[6] += 1;
    }
    if (++launches % 25 == 0 && acc[6] > 0) {
      const double n = acc[6];
      fprintf(stderr,
              "M16Q_STAMPS tr %d nth %d launches %.0f | span %.2f us, start spread %.2f us | per workgroup cycles %.0f: "
              "prologue %.0f, taps %.0f, epilogue %.0f\n",
              tr, nth, n, acc[0] / n, acc[1] / n, acc[2] / n, acc[3] / n, acc[4] / n, acc[5] / n);
    }
  }
#endif
  return OP_OK;
}

}  // namespace op
