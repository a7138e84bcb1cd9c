// conv1_1 + conv1_2 + 2x2 max-pool in one launch (CocoPoseNet.py:136-138), 3xBF16 split, gfx950.
//
// conv1_1 (3 -> 64, K = 27) is VALU work; conv1_2 (64 -> 64) is MFMA work.  Run separately, the
// 64-channel conv1_1 map (1.4 GB split at 38 frames of 368x368) is written once and read ~2x by
// conv1_2.  Here a workgroup owns an 8 x 32 tile of conv1_2 outputs (4 x 16 pooled) and:
//  * stages the 12 x 36 network-input window (cv2 LINEAR resize + x/255 - 0.5 from the uint8
//    frame, pose_detector.py:493-494, 426-431, or the padded split16 input) in LDS;
//  * per 32-channel half of conv1_1: computes conv1_1 + bias + ReLU on the 10 x 34 window conv1_2
//    reads (zero outside the image: conv1_2's own zero padding), in the same FMA order as
//    conv11_split, and writes it hi/lo split into 8 LDS planes (chunk x k-half x hi/lo);
//  * runs conv1_2's 9 taps of that half on v_mfma_f32_16x16x32_bf16 (K = 32 channels: lane group
//    g = chunk g/2, channel half g%2; products hi*hi + hi*lo + lo*hi), A fragments read from L2
//    one step ahead;
//  * pools 2x2 in the epilogue (rows = blocks b, b+2; columns = lanes l, l^1) into P1.
// Waves: 4, wave w = kP1CoW (32) channels x 16 / (4 / kP1Cg) (8) blocks of 16 px (tile rows
// 4 (w / 2) .. + 3): a wave's per-step A fragments (read from L2) feed 8 pixel blocks, where 64
// channels x 4 blocks read every A fragment in all four waves (conv1_pair -2.8 %; 16 x 16: +1.4 %).  LDS 48 KiB:
// three workgroups per CU, so one's conv1_1 (VALU) phase overlaps the others' MFMA phases.
#include "conv_big.hpp"  // split_pair_swap
#include "cvlinear.hpp"

namespace op {

typedef __bf16 bf16x8p __attribute__((ext_vector_type(8)));
typedef unsigned short u16x4p __attribute__((ext_vector_type(4)));
typedef unsigned short u16x8p __attribute__((ext_vector_type(8)));

constexpr int kP1R = 8, kP1C = 32;                 // conv1_2 tile
constexpr int kP1HR = kP1R + 2, kP1HC = kP1C + 2;  // conv1_1 window = conv1_2 halo (pitch kP1HC)
constexpr int kP1IR = kP1R + 4, kP1IC = kP1C + 4;  // network-input window
constexpr int kP1Slots = kP1HR * kP1HC;            // 340
// bytes per plane, a multiple of 256 so all 8 planes start on bank 0: a ds_read_b128 lane group
// spans two planes (k-halves), and with a 64-B plane offset their 16-B slots collided (2-way)
constexpr int kP1Plane = (kP1Slots * 16 + 255) / 256 * 256;  // (no measurable change in an A/B)
[[maybe_unused]] constexpr int kP1Items = 384;                      // conv1_1 work items per 16-channel group (6 waves)
#ifndef C1P_COW
#define C1P_COW 32
#endif
#ifndef C1P_SWAP
// 1: conv1_1's split stores as one ds_write_b128 per lane after a permlane16 row swap -- LDS
// conflicts 0.66 -> 0.28 per instruction, but neutral to slower (conv3x3 42.60 vs 42.56 ms per
// 232-frame step, 5-round A/B, profiles/r04/ab_r04s_*.log): off
#define C1P_SWAP 0
#endif
#ifndef C1P_MFMA11
#define C1P_MFMA11 1  // conv1_1 on MFMA (0: the f32 VALU form, in the CPU oracle's FMA order)
#endif
constexpr int kP1CoW = C1P_COW;             // conv1_2 output channels per wave (16, 32 or 64)
constexpr int kP1Ncb = kP1CoW / 16;         // 16-channel MFMA blocks per wave
constexpr int kP1Cg = 64 / kP1CoW;          // channel groups over the 4 waves
constexpr int kP1Npb = 16 / (4 / kP1Cg);    // 16-px blocks per wave (the tile has 16)

__device__ __forceinline__ float p1_recon(float v) {
  const __bf16 h = (__bf16)v;
  return (float)h + (float)(__bf16)(v - (float)h);
}

template <bool FROM_FRAMES>
__global__ __launch_bounds__(256, 2) void conv1_pair_bf16x3(const uint8_t* __restrict__ frames, int64_t frame_bytes,
                                                            int64_t row_stride, int sh, int sw,
                                                            const char* __restrict__ x0in, int h, int w,
                                                            const float* __restrict__ wt11,
                                                            const float* __restrict__ b11, const char* __restrict__ w12,
                                                            const float* __restrict__ b12, char* __restrict__ out,
                                                            int pout) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  char* const halo = lds;                           // 8 planes x 340 slots x 16 B
  float* const inw = (float*)(lds + 8 * kP1Plane);  // [3][12][36] f32, planar: lanes read consecutive words
  // cv2 LINEAR taps of the window's 36 columns and 12 rows, computed once per workgroup (f64 scale
  // arithmetic) instead of once per staged pixel
  LinTap* const taps = (LinTap*)(lds + 8 * kP1Plane + kP1IR * kP1IC * 12);  // [36 x][12 y]
  const int n = blockIdx.z;
  const int y0 = blockIdx.y * kP1R, x0 = blockIdx.x * kP1C;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int l16 = lane & 15, kg = lane >> 4;
  const int csel = kg >> 1, khalf = kg & 1;

  if constexpr (FROM_FRAMES) {
    if (tid < kP1IC) taps[tid] = cv_linear_tap(x0 - 2 + tid, w, sw, true);
    else if (tid < kP1IC + kP1IR) taps[tid] = cv_linear_tap(y0 - 2 + tid - kP1IC, h, sh, false);
    __syncthreads();
  }
  // ---- network-input window (zero outside the image: conv1_1's padding) ----
  for (int i = tid; i < kP1IR * kP1IC; i += 256) {
    const int iy = i / kP1IC, ix = i - (i / kP1IC) * kP1IC;
    const int gy = y0 - 2 + iy, gx = x0 - 2 + ix;
    float v[3] = {0.f, 0.f, 0.f};
    if (gy >= 0 && gy < h && gx >= 0 && gx < w) {
      if constexpr (FROM_FRAMES) {
        const uint8_t* src = frames + (int64_t)n * frame_bytes;
        const LinTap tx = taps[ix];
        const LinTap ty = taps[kP1IC + iy];
#pragma unroll
        for (int c = 0; c < 3; ++c) v[c] = p1_recon(cv_linear_px(src, row_stride, sh, sw, tx, ty, c));
      } else {  // padded split16 input (h+2, w+2, 16): channels 0..7 hi at +0, lo at +16
        const char* p = x0in + (((int64_t)n * (h + 2) + gy + 1) * (w + 2) + gx + 1) * 64;
        const uint2 hv = *(const uint2*)p, lv = *(const uint2*)(p + 16);
        v[0] = __fadd_rn(__uint_as_float(hv.x << 16), __uint_as_float(lv.x << 16));
        v[1] = __fadd_rn(__uint_as_float(hv.x & 0xffff0000u), __uint_as_float(lv.x & 0xffff0000u));
        v[2] = __fadd_rn(__uint_as_float(hv.y << 16), __uint_as_float(lv.y << 16));
      }
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) inw[c * kP1IR * kP1IC + i] = v[c];
  }

  const int cs = wave % kP1Cg, ph = wave / kP1Cg;  // channel group, pixel group of this wave
  // A fragments (conv1_2 weights, split layout [c16][tap][plane][64][8]) of step (half, tap)
  auto load_a = [&](int half, int t, bf16x8p(&ah)[kP1Ncb], bf16x8p(&al)[kP1Ncb]) {
    const int c16 = 2 * half + csel;
    const char* base = w12 + ((int64_t)((c16 * 9 + t) * 4 + 2 * khalf) * 64 + kP1CoW * cs + l16) * 16;
#pragma unroll
    for (int cb = 0; cb < kP1Ncb; ++cb) {
      ah[cb] = *(const bf16x8p*)(base + cb * 256);
      al[cb] = *(const bf16x8p*)(base + 64 * 16 + cb * 256);
    }
  };

  floatx4 acc[kP1Ncb][kP1Npb];
#pragma unroll
  for (int cb = 0; cb < kP1Ncb; ++cb)
#pragma unroll
    for (int pb = 0; pb < kP1Npb; ++pb) acc[cb][pb] = floatx4{0.f, 0.f, 0.f, 0.f};

  // this lane's halo slot for its pixel blocks (block b = kP1Npb ph + pb: row b/2, cols (b%2)*16 + l16)
  int q[kP1Npb];
#pragma unroll
  for (int pb = 0; pb < kP1Npb; ++pb) {
    const int b = kP1Npb * ph + pb;
    q[pb] = (b >> 1) * kP1HC + (b & 1) * 16 + l16;
  }
  const char* const bplane = halo + (csel * 4 + 2 * khalf) * kP1Plane;

  bf16x8p ah[kP1Ncb], al[kP1Ncb];
  load_a(0, 0, ah, al);
  for (int half = 0; half < 2; ++half) {
    __syncthreads();  // input window staged / the previous half's MFMAs are done with the halo
#if C1P_MFMA11
    // ---- conv1_1 for channels 32*half .. +31 on the 10 x 34 window -> split LDS planes, on MFMA:
    // K = the 27 (tap, input channel) products, then the bias (B = 1.0, A = b11: the bias rides in
    // the accumulation instead of a per-block load + add) and 4 zeros; im2col fragments built in
    // registers from the staged window with unconditional reads (a slot past the window reads its
    // last slot and is not stored); three bf16 products per MAC like every other layer (round 3:
    // the f32 VALU form below took ~75 % of the workgroup's MFMA time in issue slots) ----
    {
      bf16x8p a11h[2], a11l[2];
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        const int co = 32 * half + 16 * cb + l16;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int k = 8 * kg + j;
          const float v = k < 27 ? wt11[k * 64 + co] : (k == 27 ? b11[co] : 0.0f);
          const __bf16 h = (__bf16)v;
          a11h[cb][j] = h;
          a11l[cb][j] = (__bf16)(v - (float)h);
        }
      }
#ifdef C1P_PROBE_NO11  // timing probe only (wrong results): conv1_1 skipped, the planes keep stale data
      if (false)
#endif
      for (int blk = wave; blk < (kP1Slots + 15) / 16; blk += 4) {
        const int sl = blk * 16 + l16;  // window slot = halo slot (row-major, pitch kP1HC)
        const int slc = min(sl, kP1Slots - 1);
        const int ry = slc / kP1HC, rx = slc - (slc / kP1HC) * kP1HC;
        const float* const px = inw + ry * kP1IC + rx;
        bf16x8p bh, bl;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int k = 8 * kg + j;
          const int kk = k < 27 ? k : 0;
          const int t = kk / 3, ci = kk - (kk / 3) * 3;
          float v = px[ci * kP1IR * kP1IC + (t / 3) * kP1IC + t % 3];
          v = k < 27 ? v : (k == 27 ? 1.0f : 0.0f);
          const __bf16 h = (__bf16)v;
          bh[j] = h;
          bl[j] = (__bf16)(v - (float)h);
        }
        const int gy = y0 - 1 + ry, gx = x0 - 1 + rx;
        const bool inside = gy >= 0 && gy < h && gx >= 0 && gx < w;
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          floatx4 d = {0.f, 0.f, 0.f, 0.f};
          d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a11h[cb], bh, d, 0, 0, 0);
          d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a11h[cb], bl, d, 0, 0, 0);
          d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a11l[cb], bh, d, 0, 0, 0);
#if C1P_SWAP
          // round 4: rows kg, kg ^ 1 (channels 4 kg .. +3 and the other half of the same 8-channel
          // piece) swap halves with v_permlane16_swap (split_pair_swap: VALU, no LDS traffic), so
          // the even row stores the piece's 16 hi bytes and the odd row its 16 lo bytes, one
          // ds_write_b128 each: 8 lanes of a row = 128 contiguous bytes, conflict-free, where the
          // two 8-B stores per lane were 2-way conflicted (ds_write_b64 banks 16 lanes at once)
          // (conv1_2's zero padding outside the image)
          floatx4 dm, v;
#pragma unroll
          for (int e = 0; e < 4; ++e) dm[e] = inside ? d[e] : 0.0f;
          uint32_t own[4], wv[4];
          split_pair_swap(dm, floatx4{0.f, 0.f, 0.f, 0.f}, 1, v, own, wv);
          if (sl < kP1Slots)
            *(uint4*)(halo + (cb * 4 + 2 * (kg >> 1) + (kg & 1)) * kP1Plane + sl * 16) =
                make_uint4(wv[0], wv[1], wv[2], wv[3]);
#else
          // lane: channels 16 cb + 4 kg .. + 3 of slot sl -> 8 bytes of the (chunk cb, half kg / 2)
          // hi and lo planes (conv1_2's zero padding outside the image)
          u16x4p hv, lv;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float f = d[e] > 0.0f && inside ? d[e] : 0.0f;
            const __bf16 hh = (__bf16)f;
            hv[e] = __builtin_bit_cast(unsigned short, hh);
            lv[e] = __builtin_bit_cast(unsigned short, (__bf16)(f - (float)hh));
          }
          if (sl < kP1Slots) {
            char* dst = halo + (cb * 4 + 2 * (kg >> 1)) * kP1Plane + sl * 16 + (kg & 1) * 8;
            *(u16x4p*)dst = hv;
            *(u16x4p*)(dst + kP1Plane) = lv;
          }
#endif
        }
      }
    }
#else
    // ---- conv1_1 for channels 32*half .. +31 on the 10 x 34 window -> split LDS planes ----
    for (int it = tid; it < 2 * kP1Items; it += 256) {
      // 16-channel group within the half: wave-uniform (kP1Items is a multiple of 64), so the
      // weights are scalar operands as in conv11_split
      const int grp = __builtin_amdgcn_readfirstlane(it / kP1Items);
      const int s = it - grp * kP1Items;
      if (s >= kP1Slots) continue;
      // slot order: the 32 leading columns row by row (a 32-lane group reads one row of the input
      // window: consecutive words, no bank conflict), then the last 2 columns of every row (in
      // plain row-major order most groups straddle a row end, where the window pitch 36 skips 2
      // words: 2-way conflicts on every conv1_1 input read)
      constexpr int kLead = kP1HR * 32;  // 320 slots of the leading 32 columns
      const int ry = s < kLead ? s >> 5 : (s - kLead) >> 1;
      const int rx = s < kLead ? s & 31 : 32 + ((s - kLead) & 1);
      const int hs = ry * kP1HC + rx;  // halo slot
      const int gy = y0 - 1 + ry, gx = x0 - 1 + rx;
      const int cbase = 32 * half + 16 * grp;
      u16x8p hv[2], lv[2];
      if (gy >= 0 && gy < h && gx >= 0 && gx < w) {
        float a[16];
#pragma unroll
        for (int co = 0; co < 16; ++co) a[co] = 0.0f;
#pragma unroll
        for (int t = 0; t < 9; ++t) {
          const float* px = inw + (ry + t / 3) * kP1IC + rx + t % 3;
#pragma unroll
          for (int ci = 0; ci < 3; ++ci) {
            const float v = px[ci * kP1IR * kP1IC];
#pragma unroll
            for (int co = 0; co < 16; ++co) a[co] = __fmaf_rn(v, wt11[(t * 3 + ci) * 64 + cbase + co], a[co]);
          }
        }
#pragma unroll
        for (int co = 0; co < 16; ++co) {
          float f = __fadd_rn(a[co], b11[cbase + co]);
          f = f > 0.0f ? f : 0.0f;
          const __bf16 hh = (__bf16)f;
          const __bf16 ll = (__bf16)(f - (float)hh);
          hv[co >> 3][co & 7] = __builtin_bit_cast(unsigned short, hh);
          lv[co >> 3][co & 7] = __builtin_bit_cast(unsigned short, ll);
        }
      } else {
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          hv[k] = u16x8p{0, 0, 0, 0, 0, 0, 0, 0};
          lv[k] = u16x8p{0, 0, 0, 0, 0, 0, 0, 0};
        }
      }
      // planes: chunk grp, k-half k, hi / lo
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        *(u16x8p*)(halo + (grp * 4 + 2 * k) * kP1Plane + hs * 16) = hv[k];
        *(u16x8p*)(halo + (grp * 4 + 2 * k + 1) * kP1Plane + hs * 16) = lv[k];
      }
    }
#endif
    __syncthreads();
    // ---- conv1_2, the 9 taps of this half: K = 32 channels per step ----
#pragma unroll 1
    for (int t = 0; t < 9; ++t) {
      bf16x8p ch_[kP1Ncb], cl_[kP1Ncb];
#pragma unroll
      for (int cb = 0; cb < kP1Ncb; ++cb) {
        ch_[cb] = ah[cb];
        cl_[cb] = al[cb];
      }
      if (t + 1 < 9) load_a(half, t + 1, ah, al);
      else if (half == 0) load_a(1, 0, ah, al);
      const int toff = (t / 3) * kP1HC + t % 3;
#pragma unroll
      for (int pb = 0; pb < kP1Npb; ++pb) {
        const char* bp = bplane + (q[pb] + toff) * 16;
        const bf16x8p bh = *(const bf16x8p*)bp;
        const bf16x8p bl = *(const bf16x8p*)(bp + kP1Plane);
#pragma unroll
        for (int cb = 0; cb < kP1Ncb; ++cb) {
          acc[cb][pb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ch_[cb], bh, acc[cb][pb], 0, 0, 0);
          acc[cb][pb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ch_[cb], bl, acc[cb][pb], 0, 0, 0);
          acc[cb][pb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cl_[cb], bh, acc[cb][pb], 0, 0, 0);
        }
      }
    }
  }

  // ---- epilogue: + bias, ReLU, split round trip, 2x2 max-pool -> P1 (pad pout, 64 channels) ----
  const int wp_out = w / 2 + 2 * pout;
  const int hp_out = h / 2 + 2 * pout;
#pragma unroll
  for (int pb = 0; pb < kP1Npb; ++pb) {  // blocks pb (row 2i) and pb + 2 (row 2i + 1)
    if (pb & 2) continue;
    const int b = kP1Npb * ph + pb;
    const int r = b >> 1, c = (b & 1) * 16 + l16;
    const int y = y0 + r, x = x0 + c;
    const bool store = y < h && x < w && (l16 & 1) == 0;
    char* optr = out + ((int64_t)(n * hp_out + y / 2 + pout) * wp_out + (x / 2 + pout)) * 256;
#pragma unroll
    for (int cb = 0; cb < kP1Ncb; ++cb) {
      const int co = kP1CoW * cs + cb * 16 + 4 * kg;
      const floatx4 bv = *(const floatx4*)(b12 + co);
      u16x4p vh, vl;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float m = 0.0f;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          float f = acc[cb][pb + 2 * k][e] + bv[e];
          f = f > 0.0f ? f : 0.0f;
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
      if (store) {
        char* d = optr + (co >> 3) * 32 + (co & 7) * 2;
        *(u16x4p*)d = vh;
        *(u16x4p*)(d + 16) = vl;
      }
    }
  }
}

// conv1_1 + conv1_2 + pool: frames != nullptr reads the uint8 frames (sh x sw resized to h x w),
// else the padded split16 network input x0.  wt11: conv1_1 [tap][ci][co] f32; w12: conv1_2 split
// weights (cop 64); out: P1 (h/2 + 2 pout, w/2 + 2 pout, 64) split.
int launch_conv1_pair(const uint8_t* frames, int64_t frame_bytes, int64_t row_stride, int32_t sh, int32_t sw,
                      const float* x0, int32_t n, int32_t h, int32_t w, const float* wt11, const float* b11,
                      const void* w12, const float* b12, float* out, int32_t pout, hipStream_t st) {
  if (h % 2 || w % 2) {
    set_error("conv1_pair: odd map size");
    return OP_ERR_INVALID;
  }
  const int lds = 8 * kP1Plane + kP1IR * kP1IC * 12 + (kP1IC + kP1IR) * (int)sizeof(LinTap);
  static bool attr = false;
  if (!attr) {
    OP_HIP_CHECK(hipFuncSetAttribute((const void*)conv1_pair_bf16x3<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     160 * 1024));
    OP_HIP_CHECK(hipFuncSetAttribute((const void*)conv1_pair_bf16x3<false>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  const dim3 grid((unsigned)((w + kP1C - 1) / kP1C), (unsigned)((h + kP1R - 1) / kP1R), (unsigned)n);
  census_add(OP_CENSUS_CONV1_PAIR);
  if (frames)
    hipLaunchKernelGGL(conv1_pair_bf16x3<true>, grid, dim3(256), lds, st, frames, frame_bytes, row_stride, sh, sw,
                       nullptr, h, w, wt11, b11, (const char*)w12, b12, (char*)out, pout);
  else
    hipLaunchKernelGGL(conv1_pair_bf16x3<false>, grid, dim3(256), lds, st, nullptr, 0, 0, 0, 0, (const char*)x0, h, w,
                       wt11, b11, (const char*)w12, b12, (char*)out, pout);
  OP_AFTER_LAUNCH("conv1_pair_bf16x3", st);
  OP_HIP_CHECK(hipGetLastError());
  return OP_OK;
}

}  // namespace op
