// PAF post-process kernels for gfx950 (pose_detector.py:75-265, 501-517).
//
// Bit-exact restatement of the reference CPU path (the parity target):
//   heat_vpass      F.resize_images align-corners bilinear (f64 weights cast to f32) fused
//                   with scipy gaussian_filter's axis-0 pass: reflect, 21 taps, f64
//                   accumulate in NI_Correlate1D's symmetric order, f32 store           :501-502, :86
//   heat_hpass_nms  axis-1 pass + strict 4-neighbour NMS on an LDS tile                  :86-102
//   peak_sort       restores np.nonzero's row-major peak order per (frame, joint)        :104-108
//   limb_pairs      line integral over 10 linspace points, np.round half-to-even, PAF
//                   samples recomputed with the upsample formula (no full-res PAF write),
//                   fma(px,ux, py*uy) dot, NumPy pairwise sum                             :135-157
//   limb_greedy     greedy assignment in (score desc, enumeration asc) order = Python's
//                   stable sorted(reverse=True) then first-fit                            :158-177
//   grouping        person grouping, one wave per frame, subsets in LDS                   :183-265
// All f64/f32 arithmetic uses explicitly rounded intrinsics; the file is built with
// -ffp-contract=off so nothing is fused behind our back.
#include "common.hpp"

namespace op {

constexpr int kMaxSubsetsLds = 2048;
constexpr int kPeakScoreLds = 8192;  // grouping<false>: a frame's peak scores staged in LDS up to this count

__device__ __forceinline__ double linspace_at(double start, double stop, int num, int i) {
  if (num == 1) return start;
  if (i == num - 1) return stop;
  const double delta = __dsub_rn(stop, start);
  const double step = __ddiv_rn(delta, (double)(num - 1));
  double y;
  if (step == 0.0)
    y = __dmul_rn(__ddiv_rn((double)i, (double)(num - 1)), delta);
  else
    y = __dmul_rn((double)i, step);
  return __dadd_rn(y, start);
}

struct UpTap {
  int u0, v0;
  float w1, w2, w3, w4;
};
// One axis of the align-corners bilinear tap: source index i0 and the f64 distances to i0+1 / i0.
struct AxisTap {
  double d1, d0;
  int i0, pad_;
};
__device__ __forceinline__ AxisTap axis_tap(int o, int L, int oL) {
  const double u = linspace_at(0.0, (double)(L - 1), oL, o);
  int i0 = (int)floor(u);
  i0 = i0 > L - 2 ? L - 2 : i0;
  i0 = i0 < 0 ? 0 : i0;
  AxisTap t;
  t.i0 = i0;
  t.d1 = __dsub_rn((double)(i0 + 1), u);
  t.d0 = __dsub_rn(u, (double)i0);
  return t;
}
__device__ __forceinline__ UpTap up_tap2(const AxisTap& ty, const AxisTap& tx) {
  UpTap t;
  t.u0 = tx.i0;
  t.v0 = ty.i0;
  t.w1 = __double2float_rn(__dmul_rn(tx.d1, ty.d1));
  t.w2 = __double2float_rn(__dmul_rn(tx.d0, ty.d1));
  t.w3 = __double2float_rn(__dmul_rn(tx.d1, ty.d0));
  t.w4 = __double2float_rn(__dmul_rn(tx.d0, ty.d0));
  return t;
}
__device__ __forceinline__ UpTap up_tap(int oy, int ox, int H, int W, int oH, int oW) {
  return up_tap2(axis_tap(oy, H, oH), axis_tap(ox, W, oW));
}
__device__ __forceinline__ float up_combine(const UpTap& t, float x00, float x01, float x10, float x11) {
  float s = __fadd_rn(__fmul_rn(t.w1, x00), __fmul_rn(t.w2, x01));
  s = __fadd_rn(s, __fmul_rn(t.w3, x10));
  return __fadd_rn(s, __fmul_rn(t.w4, x11));
}

// Low-res NHWC (stage-input buffer) accessor for one frame.
struct LowMap {
  const float* f;  // frame base
  int wp, pad, cs;
  __device__ __forceinline__ float at(int c, int y, int x) const {
    return f[((int64_t)(y + pad) * wp + (x + pad)) * cs + c];
  }
};

__device__ __forceinline__ LowMap low_map(const MapSource& src, int lw, int frame) {
  LowMap m;
  m.f = src.base + (int64_t)frame * src.fstride;
  m.wp = lw + 2 * src.pad;
  m.pad = src.pad;
  m.cs = src.cs;
  return m;
}

__device__ __forceinline__ float up_sample(const LowMap& m, int c, const UpTap& t) {
  return up_combine(t, m.at(c, t.v0, t.u0), m.at(c, t.v0, t.u0 + 1), m.at(c, t.v0 + 1, t.u0),
                    m.at(c, t.v0 + 1, t.u0 + 1));
}

// Chainer resize for a planar (c,h,w) tensor (stage-level ABI).
__global__ __launch_bounds__(256) void resize_planar(const float* __restrict__ x, int c, int h, int w, int oh, int ow,
                                                     float* __restrict__ y) {
  const int64_t plane = (int64_t)oh * ow;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= plane * c) return;
  const int ox = (int)(i % ow);
  const int oy = (int)((i / ow) % oh);
  const int cc = (int)(i / plane);
  const UpTap t = up_tap(oy, ox, h, w, oh, ow);
  const float* p = x + (int64_t)cc * h * w;
  y[i] = up_combine(t, p[t.v0 * w + t.u0], p[t.v0 * w + t.u0 + 1], p[(t.v0 + 1) * w + t.u0],
                    p[(t.v0 + 1) * w + t.u0 + 1]);
}

// PAF sample at map pixel (y, x) of PAF channel c: recomputed from the low-res map with the
// upsample formula (identical f32 value to the full-res map the reference indexes), or read from a
// full-res planar map (stage-level ABI).
struct PafLow {
  LowMap m;
  int lh, lw, mh, mw, off;
  const AxisTap* ty = nullptr;  // per-block LDS tables of axis_tap over the map rows / columns
  const AxisTap* tx = nullptr;  // (round 3: the f64 linspace divisions once per block, not per sample)
  const float* p0 = nullptr;    // the limb's two low-res PAF planes staged in LDS ([lh][lw] each)
  const float* p1 = nullptr;
  __device__ __forceinline__ float at(int c, int y, int x) const {
    return up_sample(m, off + c, up_tap(y, x, lh, lw, mh, mw));
  }
  // both channels of limb l at one map pixel: one tap for the pair
  __device__ __forceinline__ void at2(int c, int y, int x, float& v0, float& v1) const {
    const UpTap t = ty ? up_tap2(ty[y], tx[x]) : up_tap(y, x, lh, lw, mh, mw);
    if (p0) {
      const int i = t.v0 * lw + t.u0;
      v0 = up_combine(t, p0[i], p0[i + 1], p0[i + lw], p0[i + lw + 1]);
      v1 = up_combine(t, p1[i], p1[i + 1], p1[i + lw], p1[i + lw + 1]);
    } else {
      v0 = up_sample(m, off + c, t);
      v1 = up_sample(m, off + c + 1, t);
    }
  }
};
struct PafFull {  // planar (38, mh, mw) of one frame (limb_pairs_full offsets p per frame)
  const float* p;
  int mh, mw;
  __device__ __forceinline__ float at(int c, int y, int x) const { return p[((int64_t)c * mh + y) * mw + x]; }
  __device__ __forceinline__ void at2(int c, int y, int x, float& v0, float& v1) const {
    v0 = at(c, y, x);
    v1 = at(c + 1, y, x);
  }
};

__device__ __forceinline__ int peak_count(const int32_t* cnt, int maxp) {
  const int c = *cnt;
  return c > maxp ? maxp : c;
}

// compute_candidate_connections for every limb of every frame; grid (frames, 19, G).
template <class Paf>
__device__ __forceinline__ void limb_pairs_body(const Paf& paf, const PostShape& s, const PostBuffers& b, int f, int l) {
  const int ja = s.limbs[l][0], jb = s.limbs[l][1];
  const int64_t fa = (int64_t)f * OP_N_JOINTS + ja, fb = (int64_t)f * OP_N_JOINTS + jb;
  const int na = peak_count(b.peak_cnt + fa, b.maxp), nb = peak_count(b.peak_cnt + fb, b.maxp);
  const int64_t npairs = (int64_t)na * nb;
  const int64_t fl = (int64_t)f * OP_N_LIMBS + l;
  const int np_ = s.n_integ;
  for (int64_t q = (int64_t)blockIdx.z * blockDim.x + threadIdx.x; q < npairs; q += (int64_t)gridDim.z * blockDim.x) {
    const int ia = (int)(q / nb), ib = (int)(q - (int64_t)ia * nb);
    const int32_t pa = b.peak_xy[fa * b.maxp + ia], pb = b.peak_xy[fb * b.maxp + ib];
    const double ax = (double)(pa & 0xffff), ay = (double)(pa >> 16);
    const double bx = (double)(pb & 0xffff), by = (double)(pb >> 16);
    const double vx = __dsub_rn(bx, ax), vy = __dsub_rn(by, ay);
    const double norm = __dsqrt_rn(__dadd_rn(__dmul_rn(vx, vx), __dmul_rn(vy, vy)));
    if (norm == 0.0) continue;
    const double ux = __ddiv_rn(vx, norm), uy = __ddiv_rn(vy, norm);
    double inner[16];
    int nvalid = 0;
    for (int i = 0; i < np_; ++i) {
      const int yi = (int)rint(linspace_at(ay, by, np_, i));
      const int xi = (int)rint(linspace_at(ax, bx, np_, i));
      float fx, fy;
      paf.at2(2 * l, yi, xi, fx, fy);
      const double px = (double)fx, py = (double)fy;
      const double ip = __fma_rn(px, ux, __dmul_rn(py, uy));
      inner[i] = ip;
      nvalid += ip > s.inner_thresh ? 1 : 0;
    }
    // NumPy pairwise sum (n < 8: sequential; 8 <= n <= 128: 8 partial accumulators)
    double sum;
    if (np_ < 8) {
      sum = 0.0;
      for (int i = 0; i < np_; ++i) sum = __dadd_rn(sum, inner[i]);
    } else {
      double r[8];
      for (int j = 0; j < 8; ++j) r[j] = inner[j];
      int i = 8;
      for (; i < np_ - (np_ % 8); i += 8)
        for (int j = 0; j < 8; ++j) r[j] = __dadd_rn(r[j], inner[i + j]);
      sum = __dadd_rn(__dadd_rn(__dadd_rn(r[0], r[1]), __dadd_rn(r[2], r[3])),
                      __dadd_rn(__dadd_rn(r[4], r[5]), __dadd_rn(r[6], r[7])));
      for (; i < np_; ++i) sum = __dadd_rn(sum, inner[i]);
    }
    const double integ = __ddiv_rn(sum, (double)np_);
    double pen = __dsub_rn(__ddiv_rn(__dmul_rn(s.len_ratio, s.img_len), norm), s.len_penalty);
    if (pen > 0.0) pen = 0.0;
    const double score = __dadd_rn(integ, pen);
    if (nvalid > s.n_integ_thresh && score > 0.0) {
      const int slot = atomicAdd(b.cand_cnt + fl, 1);
      if (slot < b.maxc) {
        b.cand_score[fl * b.maxc + slot] = score;
        b.cand_idx[fl * b.maxc + slot] = (int32_t)q;
      }
    }
  }
}

constexpr int64_t kPairsStage = 2048;  // candidate pairs of a (frame, limb) from which limb_pairs_low stages

__global__ __launch_bounds__(256) void limb_pairs_low(MapSource src, PostShape s, PostBuffers b, int tables) {
  const int f = blockIdx.x, l = blockIdx.y;
  extern __shared__ AxisTap tab[];  // tables: [mh] rows then [mw] columns; then (tables 2) the planes
  // this block's share of the limb's candidate pairs; the LDS tables / planes only where the pairs
  // repay their set-up (crowded frames), sparse frames sample the L2-resident map directly
  const int na = peak_count(b.peak_cnt + (int64_t)f * OP_N_JOINTS + s.limbs[l][0], b.maxp);
  const int nb = peak_count(b.peak_cnt + (int64_t)f * OP_N_JOINTS + s.limbs[l][1], b.maxp);
  const int64_t npairs = (int64_t)na * nb;
  if ((int64_t)blockIdx.z * blockDim.x >= npairs) return;
  if (npairs < kPairsStage) tables = 0;
  PafLow paf;
  if (tables) {
    for (int i = threadIdx.x; i < s.mh + s.mw; i += 256)
      tab[i] = i < s.mh ? axis_tap(i, s.lh, s.mh) : axis_tap(i - s.mh, s.lw, s.mw);
    paf.ty = tab;
    paf.tx = tab + s.mh;
  }
  paf.m = low_map(src, s.lw, f);
  if (tables == 2) {  // this limb's two PAF channels of the frame's low-res map -> LDS
    float* pl = (float*)(tab + s.mh + s.mw);
    const int area = s.lh * s.lw;
    for (int i = threadIdx.x; i < area; i += 256) {
      const int y = i / s.lw, x = i - (i / s.lw) * s.lw;
      pl[i] = paf.m.at(src.paf_off + 2 * l, y, x);
      pl[area + i] = paf.m.at(src.paf_off + 2 * l + 1, y, x);
    }
    paf.p0 = pl;
    paf.p1 = pl + area;
  }
  if (tables) __syncthreads();
  paf.lh = s.lh;
  paf.lw = s.lw;
  paf.mh = s.mh;
  paf.mw = s.mw;
  paf.off = src.paf_off;
  limb_pairs_body(paf, s, b, f, l);
}

__global__ __launch_bounds__(256) void limb_pairs_full(const float* __restrict__ paf_full, int64_t fstride, PostShape s,
                                                       PostBuffers b) {
  PafFull paf;
  paf.p = paf_full + blockIdx.x * fstride;
  paf.mh = s.mh;
  paf.mw = s.mw;
  limb_pairs_body(paf, s, b, blockIdx.x, blockIdx.y);
}

// Greedy assignment per (frame, limb): repeatedly accept the best remaining candidate whose two
// peaks are both unused, until min(|A|,|B|) connections (pose_detector.py:172-177).  Accepting
// the (score desc, index asc) maximum among still-valid candidates is exactly first-fit over
// the stably sorted list: every skipped candidate keeps a used endpoint forever.
// kBig: the used-peak bitsets live in HBM (b.used, [frame][limb][2][words]) for any peak count;
// otherwise in LDS (maxp <= 2048).
constexpr int kGreedySort = 4096;  // candidates per (frame, limb) sorted in LDS (48 KiB); more: argmax scans

template <bool kBig>
__global__ __launch_bounds__(256) void limb_greedy(PostShape s, PostBuffers b) {
  __shared__ unsigned used_lds[kBig ? 1 : 128];
  __shared__ double red_s[4];
  __shared__ int red_i[4];
  __shared__ unsigned long long skey[kGreedySort];  // sorted batches: score bits
  __shared__ int32_t sq[kGreedySort];               // and candidate (pair) indices
  __shared__ unsigned long long samp[256];          // sorted sample of the keys (K > kGreedySort)
  __shared__ int fill_n, got_s;
  const int f = blockIdx.x, l = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ja = s.limbs[l][0], jb = s.limbs[l][1];
  const int64_t fa = (int64_t)f * OP_N_JOINTS + ja, fb = (int64_t)f * OP_N_JOINTS + jb;
  const int na = peak_count(b.peak_cnt + fa, b.maxp), nb = peak_count(b.peak_cnt + fb, b.maxp);
  const int64_t fl = (int64_t)f * OP_N_LIMBS + l;
  int K = b.cand_cnt[fl];
  K = K > b.maxc ? (int)b.maxc : K;
  // global peak id bases (ids are consecutive over joints 0..17, pose_detector.py:106-108)
  int base_a = 0, base_b = 0;
  for (int j = 0; j < OP_N_JOINTS; ++j) {
    const int c = peak_count(b.peak_cnt + (int64_t)f * OP_N_JOINTS + j, b.maxp);
    if (j < ja) base_a += c;
    if (j < jb) base_b += c;
  }
  const int words = kBig ? (b.maxp + 31) / 32 : 64;
  unsigned* used_a = used_lds;
  if constexpr (kBig) used_a = b.used + fl * 2 * words;
  unsigned* used_b = used_a + (kBig ? words : 64);
  for (int i = tid; i < words; i += 256) {
    used_a[i] = 0;
    used_b[i] = 0;
  }
  __syncthreads();
  const int lim = na < nb ? na : nb;
  const double* cs = b.cand_score + fl * b.maxc;
  const int32_t* ci = b.cand_idx + fl * b.maxc;
  int got = 0;
  if (K > 0) {
    // round 3: first-fit over the candidates in (score desc, index asc) order (positive doubles
    // order like their bit patterns), taken in batches of keys [T, hi) that fit kGreedySort LDS
    // slots: a batch is collected by one scan, bitonic-sorted in LDS, and walked by one wave 64
    // candidates at a time -- each accepted candidate kills the later lanes that share one of its
    // peaks (a ballot per acceptance).  Thresholds T come from a sorted sample of 256 keys; a batch
    // that would still overflow (ties) hands the rest to the argmax scans below, which continue
    // correctly: every candidate of a finished batch is accepted or has a used endpoint.
    unsigned long long hi = ~0ull;  // exclusive upper key bound of the next batch
    int r = 0;                      // sample rank of the last threshold
    if (K > kGreedySort) {
      samp[tid] = (unsigned long long)__double_as_longlong(cs[(int)(((int64_t)tid * K) / 256)]);
      __syncthreads();
      for (int k = 2; k <= 256; k <<= 1)  // descending
        for (int j = k >> 1; j > 0; j >>= 1) {
          const int p = tid ^ j;
          const unsigned long long a = samp[tid], c = samp[p];
          __syncthreads();
          if (p > tid ? (((tid & k) == 0) ? a < c : a > c) : (((p & k) == 0) ? c < a : c > a)) samp[tid] = c;
          __syncthreads();
        }
    }
    bool done = false;
    while (!done) {
      // this batch's threshold: all the rest if it fits, else the sample rank whose count fits
      unsigned long long T = 0;
      int cnt = 0;
      if (K > kGreedySort) {
        int step = (int)((int64_t)kGreedySort * 256 * 3 / 4 / K);
        step = step < 1 ? 1 : step;
        for (;;) {
          int j = r + step;
          if (j >= 256) {
            T = 0;
          } else {
            while (j < 256 && samp[j] >= hi) ++j;  // ties with the previous threshold
            T = j < 256 ? samp[j] : 0ull;
          }
          // count and collect in one scan (a wave reserves its lanes' slots with one LDS atomic);
          // a batch past the cap is dropped and the step halves
          if (tid == 0) fill_n = 0;
          __syncthreads();
          for (int i0 = 0; i0 < K; i0 += 256) {
            const int i = i0 + tid;
            unsigned long long key = 0;
            bool in = false;
            if (i < K) {
              key = (unsigned long long)__double_as_longlong(cs[i]);
              in = key >= T && key < hi;
            }
            const unsigned long long m = __ballot(in);
            int base = 0;
            if (m) {
              if (lane == 0) base = atomicAdd(&fill_n, __popcll(m));
              base = __shfl(base, 0);
            }
            const int slot = base + __popcll(m & ((1ull << lane) - 1ull));
            if (in && slot < kGreedySort) {
              skey[slot] = key;
              sq[slot] = ci[i];
            }
          }
          __syncthreads();
          const int c = fill_n;
          __syncthreads();
          if (c <= kGreedySort) {
            cnt = c;
            r = j < 256 ? j : 256;
            break;
          }
          if (step == 1) {
            cnt = -1;  // a tie run longer than a batch: the argmax scans take over
            break;
          }
          step >>= 1;
        }
        if (cnt < 0) break;
      } else {
        cnt = K;
      }
      // the batch (any order; sorted next): collected by the counting scan, or all K at once
      if (K <= kGreedySort) {
        for (int i = tid; i < K; i += 256) {
          skey[i] = (unsigned long long)__double_as_longlong(cs[i]);
          sq[i] = ci[i];
        }
      }
      int n2 = 1;
      while (n2 < cnt) n2 <<= 1;
      for (int i = cnt + tid; i < n2; i += 256) {
        skey[i] = 0ull;  // padding sorts last
        sq[i] = 0x7fffffff;
      }
      __syncthreads();
      for (int k = 2; k <= n2; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
          for (int i = tid; i < n2; i += 256) {
            const int p = i ^ j;
            if (p > i) {
              const unsigned long long ki = skey[i], kp = skey[p];
              const int qi = sq[i], qp = sq[p];
              const bool i_first = ki > kp || (ki == kp && qi < qp);
              if (((i & k) == 0) != i_first) {
                skey[i] = kp;
                skey[p] = ki;
                sq[i] = qp;
                sq[p] = qi;
              }
            }
          }
          __syncthreads();
        }
      if (wave == 0) {
        for (int c0 = 0; c0 < cnt && got < lim; c0 += 64) {
          const int i = c0 + lane;
          int ia = -1, ib = -1;
          bool alive = false;
          if (i < cnt) {
            const int q = sq[i];
            ia = q / nb;
            ib = q - ia * nb;
            alive = !((used_a[ia >> 5] >> (ia & 31)) & 1u) && !((used_b[ib >> 5] >> (ib & 31)) & 1u);
          }
          unsigned long long m = __ballot(alive);
          while (m && got < lim) {
            const int jl = __ffsll((long long)m) - 1;
            const int ja_ = __shfl(ia, jl), jb_ = __shfl(ib, jl);
            if (lane == jl || ia == ja_ || ib == jb_) alive = false;
            if (lane == 0) {
              used_a[ja_ >> 5] |= 1u << (ja_ & 31);
              used_b[jb_ >> 5] |= 1u << (jb_ & 31);
              const int64_t o = fl * b.maxp + got;
              b.conn_ab[2 * o] = base_a + ja_;
              b.conn_ab[2 * o + 1] = base_b + jb_;
              b.conn_score[o] = __longlong_as_double((long long)skey[c0 + jl]);
            }
            if constexpr (kBig) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");  // HBM bitsets: the
            ++got;                                                                     // next chunk reads them
            m = __ballot(alive);
          }
        }
        if (lane == 0) got_s = got;
      }
      __syncthreads();
      got = got_s;
      done = T == 0 || got >= lim;
      hi = T;
      __syncthreads();  // skey / sq / fill_n are rewritten by the next batch
    }
    if (done) {
      if (tid == 0) b.conn_cnt[fl] = got;
      return;
    }
  }
  while (got < lim && K > 0) {
    double best = -1.0;  // every kept candidate has score > 0
    int bidx = 0x7fffffff;
    for (int i = tid; i < K; i += 256) {
      const int q = ci[i];
      const int ia = q / nb, ib = q - ia * nb;
      if ((used_a[ia >> 5] >> (ia & 31)) & 1u) continue;
      if ((used_b[ib >> 5] >> (ib & 31)) & 1u) continue;
      const double sc = cs[i];
      if (sc > best || (sc == best && q < bidx)) {
        best = sc;
        bidx = q;
      }
    }
    for (int off = 32; off > 0; off >>= 1) {
      const double os = __shfl_xor(best, off);
      const int oi = __shfl_xor(bidx, off);
      if (os > best || (os == best && oi < bidx)) {
        best = os;
        bidx = oi;
      }
    }
    if (lane == 0) {
      red_s[wave] = best;
      red_i[wave] = bidx;
    }
    __syncthreads();
    best = red_s[0];
    bidx = red_i[0];
    for (int w = 1; w < 4; ++w) {
      if (red_s[w] > best || (red_s[w] == best && red_i[w] < bidx)) {
        best = red_s[w];
        bidx = red_i[w];
      }
    }
    __syncthreads();
    if (bidx == 0x7fffffff) break;
    const int ia = bidx / nb, ib = bidx - ia * nb;
    if (tid == 0) {
      used_a[ia >> 5] |= 1u << (ia & 31);
      used_b[ib >> 5] |= 1u << (ib & 31);
      const int64_t o = fl * b.maxp + got;
      b.conn_ab[2 * o] = base_a + ia;
      b.conn_ab[2 * o + 1] = base_b + ib;
      b.conn_score[o] = best;
    }
    __syncthreads();
    ++got;
  }
  if (tid == 0) b.conn_cnt[fl] = got;
}

// wave-uniform-lane broadcasts (v_readlane_b32): lane must be the same for every lane of the wave
__device__ __forceinline__ int rl_i(int v, int lane) { return __builtin_amdgcn_readlane(v, lane); }
__device__ __forceinline__ double rl_d(double v, int lane) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), lane);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

#ifndef GROUP_REG
#define GROUP_REG 1
#endif
// grouping_key_points + subsets_to_pose_array, one wave per frame.
// kBig: the subsets live in HBM (b.sub_ids / b.sub_sc, b.maxs rows, int32 peak ids) for any
// peak and subset count; otherwise in LDS (<= kMaxSubsetsLds rows, int16 ids).
template <bool kBig>
__global__ __launch_bounds__(64) void grouping(PostShape s, PostBuffers b) {
  using IdT = typename std::conditional<kBig, int32_t, int16_t>::type;
  constexpr int kRows = kBig ? 1 : kMaxSubsetsLds;
  __shared__ int16_t ids_lds[kRows][OP_N_JOINTS];
  __shared__ double sc_lds[kRows][2];
  __shared__ int base[OP_N_JOINTS + 1];
  __shared__ int cnt[OP_N_JOINTS];
  __shared__ float pk_lds[kBig ? 1 : kPeakScoreLds];  // peak scores by global peak id
  const int f = blockIdx.x;
  IdT (*ids)[OP_N_JOINTS];
  double (*sc)[2];
  if constexpr (kBig) {
    ids = (IdT(*)[OP_N_JOINTS])(b.sub_ids + (int64_t)f * b.maxs * OP_N_JOINTS);
    sc = (double(*)[2])(b.sub_sc + (int64_t)f * b.maxs * 2);
  } else {
    ids = ids_lds;
    sc = sc_lds;
  }
  const int lane = threadIdx.x;
  if (lane < OP_N_JOINTS) cnt[lane] = b.peak_cnt[(int64_t)f * OP_N_JOINTS + lane];
  __syncthreads();
  int status = OP_OK;
  if (lane == 0) {
    int acc = 0;
    for (int j = 0; j < OP_N_JOINTS; ++j) {
      base[j] = acc;
      if (cnt[j] > b.maxp) status = OP_ERR_CAPACITY;
      acc += cnt[j] > b.maxp ? b.maxp : cnt[j];
    }
    base[OP_N_JOINTS] = acc;
  }
  status = __shfl(status, 0);
  __syncthreads();
  const int n_peaks = base[OP_N_JOINTS];
  int S = 0;
  // round 4: no chain of dependent global loads per limb.  The frame's peak scores go to LDS in one
  // pass (all loads in flight together), every limb's connection count is one lane's load, and a
  // limb's first 64 connections (ids, score; one per lane, broadcast from registers) are fetched
  // while the previous limb is processed.
  const bool pk_lds_ok = !kBig && n_peaks <= kPeakScoreLds;
  if (pk_lds_ok) {
    for (int i = lane; i < n_peaks; i += 64) {
      int j = 0;
      while (base[j + 1] <= i) ++j;
      pk_lds[i] = b.peak_score[((int64_t)f * OP_N_JOINTS + j) * b.maxp + (i - base[j])];
    }
  }
  const int kc = lane < OP_N_LIMBS ? b.conn_cnt[(int64_t)f * OP_N_LIMBS + lane] : 0;
  __syncthreads();
  auto pscore = [&](int joint, int id) -> double {
    if (pk_lds_ok) return (double)pk_lds[id];
    return (double)b.peak_score[((int64_t)f * OP_N_JOINTS + joint) * b.maxp + (id - base[joint])];
  };
  auto fetch = [&](int l, int cb, int& ia, int& ib, double& sc) {
    const int K = rl_i(kc, l);
    ia = 0;
    ib = 0;
    sc = 0.0;
    if (cb + lane < K) {
      const int64_t q = ((int64_t)f * OP_N_LIMBS + l) * b.maxp + cb + lane;
      ia = b.conn_ab[2 * q];
      ib = b.conn_ab[2 * q + 1];
      sc = b.conn_score[q];
    }
  };
  int nx_ia, nx_ib;
  double nx_sc;
  fetch(0, 0, nx_ia, nx_ib, nx_sc);
  // Round 5 (GROUP_REG, LDS subsets): lane r < 64 also holds subset row r's ids at the current
  // limb's two joints (cja, cjb) and its two scores (cs0, cs1) in registers, so the first 64 rows
  // are matched without LDS reads and a matched row is updated by its own lane from registers; the
  // LDS rows stay authoritative (every update writes through; merges and the final pass read them)
  constexpr bool kReg = !kBig && GROUP_REG;
  int cja = -1, cjb = -1;
  double cs0 = 0.0, cs1 = 0.0;
  for (int l = 0; l < OP_N_LIMBS && status == OP_OK; ++l) {
    const int ja = s.limbs[l][0], jb = s.limbs[l][1];
    if constexpr (kReg) {
      if (lane < S) {
        cja = ids[lane][ja];
        cjb = ids[lane][jb];
      }
    }
    const int K = rl_i(kc, l);
    int my_ia = nx_ia, my_ib = nx_ib;
    double my_sc = nx_sc;
    if (l + 1 < OP_N_LIMBS) fetch(l + 1, 0, nx_ia, nx_ib, nx_sc);
    for (int cb = 0; cb < K && status == OP_OK; cb += 64) {
    if (cb > 0) fetch(l, cb, my_ia, my_ib, my_sc);
    double my_pa = 0.0, my_pb = 0.0;
    if (cb + lane < K) {
      my_pa = pscore(ja, my_ia);
      my_pb = pscore(jb, my_ib);
    }
    const int ce = min(K - cb, 64);
    for (int c = 0; c < ce && status == OP_OK; ++c) {
      // lane c's values, read with v_readlane into scalar registers (c is wave-uniform): no LDS
      // round trip per broadcast, as __shfl's ds_bpermute would make (8 per connection)
      const int ia = rl_i(my_ia, c);
      const int ib = rl_i(my_ib, c);
      const double score = rl_d(my_sc, c);
      const double psa = rl_d(my_pa, c), psb = rl_d(my_pb, c);  // pscore(ja, ia), pscore(jb, ib)
      int found = 0, f0 = -1, f1 = -1;
      for (int s0 = 0; s0 < S; s0 += 64) {
        const int r = s0 + lane;
        const bool m = r < S && ((kReg && s0 == 0) ? (cja == ia || cjb == ib) : (ids[r][ja] == ia || ids[r][jb] == ib));
        unsigned long long bal = __ballot(m);
        while (bal) {
          const int k = __ffsll((long long)bal) - 1;
          bal &= bal - 1;
          if (found == 0) f0 = s0 + k;
          else if (found == 1) f1 = s0 + k;
          ++found;
        }
        if (found >= 3) break;
      }
      if (found >= 3) {
        status = OP_ERR_INDEX;
        break;
      }
      if (found == 1) {
        if (kReg && f0 < 64) {
          if (lane == f0 && cjb != ib) {
            ids[f0][jb] = (IdT)ib;
            cjb = ib;
            cs1 = __dadd_rn(cs1, 1.0);
            cs0 = __dadd_rn(cs0, __dadd_rn(psb, score));
            sc[f0][1] = cs1;
            sc[f0][0] = cs0;
          }
        } else if (lane == 0 && ids[f0][jb] != ib) {
          ids[f0][jb] = (IdT)ib;
          sc[f0][1] = __dadd_rn(sc[f0][1], 1.0);
          sc[f0][0] = __dadd_rn(sc[f0][0], __dadd_rn(psb, score));
        }
      } else if (found == 2) {
        const bool both = lane < OP_N_JOINTS && ids[f0][lane] >= 0 && ids[f1][lane] >= 0;
        if (__ballot(both) == 0ull) {
          if (lane < OP_N_JOINTS) ids[f0][lane] = (IdT)(ids[f0][lane] + ids[f1][lane] + 1);
          if (lane == 0) {
            sc[f0][0] = __dadd_rn(sc[f0][0], sc[f1][0]);
            sc[f0][1] = __dadd_rn(sc[f0][1], sc[f1][1]);
            sc[f0][0] = __dadd_rn(sc[f0][0], score);
            sc[f0][1] = __dadd_rn(sc[f0][1], score);
          }
          __syncthreads();
          // np.delete(subsets, f1): shift rows down, 64 rows per step (read all, then write)
          for (int r0 = f1; r0 < S - 1; r0 += 64) {
            const int r = r0 + lane;
            IdT row[OP_N_JOINTS];
            double s2[2];
            const bool act = r < S - 1;
            if (act) {
              for (int j = 0; j < OP_N_JOINTS; ++j) row[j] = ids[r + 1][j];
              s2[0] = sc[r + 1][0];
              s2[1] = sc[r + 1][1];
            }
            __syncthreads();
            if (act) {
              for (int j = 0; j < OP_N_JOINTS; ++j) ids[r][j] = row[j];
              sc[r][0] = s2[0];
              sc[r][1] = s2[1];
            }
            __syncthreads();
          }
          --S;
          if constexpr (kReg) {  // rows f0 and past f1 changed: reload every lane's row
            __syncthreads();
            if (lane < S) {
              cja = ids[lane][ja];
              cjb = ids[lane][jb];
              cs0 = sc[lane][0];
              cs1 = sc[lane][1];
            }
          }
        } else {
          const int fs[2] = {f0, f1};
          for (int q = 0; q < 2; ++q) {
            const int t = fs[q];
            if (kReg && t < 64) {
              if (lane == t) {
                if (cja == -1) {
                  ids[t][ja] = (IdT)ia;
                  cja = ia;
                  cs1 = __dadd_rn(cs1, 1.0);
                  cs0 = __dadd_rn(cs0, __dadd_rn(psa, score));
                  sc[t][1] = cs1;
                  sc[t][0] = cs0;
                } else if (cjb == -1) {
                  ids[t][jb] = (IdT)ib;
                  cjb = ib;
                  cs1 = __dadd_rn(cs1, 1.0);
                  cs0 = __dadd_rn(cs0, __dadd_rn(psb, score));
                  sc[t][1] = cs1;
                  sc[t][0] = cs0;
                }
              }
              continue;
            }
            if (lane != 0) continue;
            if (ids[t][ja] == -1) {
              ids[t][ja] = (IdT)ia;
              sc[t][1] = __dadd_rn(sc[t][1], 1.0);
              sc[t][0] = __dadd_rn(sc[t][0], __dadd_rn(psa, score));
            } else if (ids[t][jb] == -1) {
              ids[t][jb] = (IdT)ib;
              sc[t][1] = __dadd_rn(sc[t][1], 1.0);
              sc[t][0] = __dadd_rn(sc[t][0], __dadd_rn(psb, score));
            }
          }
        }
      } else if (l != 9 && l != 13) {
        if ((!kBig && S >= kMaxSubsetsLds) || S >= b.maxs) {
          status = OP_ERR_CAPACITY;
          break;
        }
        if (lane < OP_N_JOINTS) ids[S][lane] = (IdT)(lane == ja ? ia : (lane == jb ? ib : -1));
        if (lane == 0) {
          sc[S][1] = 2.0;
          sc[S][0] = __dadd_rn(__dadd_rn(psa, psb), score);
        }
        if (kReg && lane == S) {
          cja = ia;
          cjb = ib;
          cs1 = 2.0;
          cs0 = __dadd_rn(__dadd_rn(psa, psb), score);
        }
        ++S;
      }
      __syncthreads();
    }
    }
  }
  // keep filter (pose_detector.py:248) + subsets_to_pose_array + subsets dump, ordered compaction
  int kept = 0;
  if (status == OP_OK) {
    for (int r0 = 0; r0 < S; r0 += 64) {
      const int r = r0 + lane;
      bool keep = false;
      if (r < S) keep = sc[r][1] >= (double)s.subset_min && __ddiv_rn(sc[r][0], sc[r][1]) >= s.subset_score;
      const unsigned long long bal = __ballot(keep);
      const int pos = kept + __popcll(bal & ((1ull << lane) - 1ull));
      if (keep) {
        double* pose = b.res_poses + ((int64_t)f * b.maxs + pos) * OP_N_JOINTS * 3;
        double* sub = b.res_subsets + ((int64_t)f * b.maxs + pos) * 20;
        for (int j = 0; j < OP_N_JOINTS; ++j) {
          const int id = ids[r][j];
          sub[j] = (double)id;
          if (id >= 0) {
            const int32_t xy = b.peak_xy[((int64_t)f * OP_N_JOINTS + j) * b.maxp + (id - base[j])];
            pose[3 * j + 0] = __dmul_rn((double)(xy & 0xffff), s.sx);
            pose[3 * j + 1] = __dmul_rn((double)(xy >> 16), s.sy);
            pose[3 * j + 2] = 2.0;
          } else {
            pose[3 * j + 0] = 0.0;
            pose[3 * j + 1] = 0.0;
            pose[3 * j + 2] = 0.0;
          }
        }
        sub[18] = sc[r][0];
        sub[19] = sc[r][1];
        b.res_scores[(int64_t)f * b.maxs + pos] = sc[r][0];
      }
      kept += __popcll(bal);
    }
  }
  if (lane == 0) {
    b.res_hdr[4 * f + 0] = status;
    b.res_hdr[4 * f + 1] = n_peaks;
    b.res_hdr[4 * f + 2] = kept;
    b.res_hdr[4 * f + 3] = S;
  }
}

// ---- heat-map pipeline: fused (upsample + vertical + horizontal Gaussian + NMS) -> sort ----
// One block owns a kFT x kFT tile of one (frame, joint) plane.  The upsampled map is rebuilt in
// LDS over the tile plus the 1-pixel NMS border plus the Gaussian radius on each side, the two
// Gaussian passes run LDS to LDS in SciPy's order (f64 symmetric pairs, f32 between the passes),
// and nothing but the peak list touches HBM.  The reflect boundary is resolved once per LDS row /
// column: region row ly stands for image row reflect(y0 - 1 - r + ly), which is exactly the row the
// reference's correlate1d reads for the tap (pose_detector.py:84, scipy mode='reflect').
constexpr int kFT = 64;                    // output tile edge
constexpr int kMaxR = 16;                  // max Gaussian radius of the tiled kernel
static_assert(kMaxR == kMaxGaussR, "op_set_peak_mode checks ksize against kMaxGaussR");
constexpr int kFU = kFT + 2 + 2 * kMaxR;   // LDS region edge (upsampled map)
constexpr int kFW = 48;                    // low-res window edge staged in LDS
constexpr int kFN = 512;                   // threads per block (2 blocks / CU by LDS)

__device__ __forceinline__ int reflect_near(int i, int L) {
  if (i < 0) i = -i - 1;
  if (i >= L) i = 2 * L - 1 - i;
  return i < 0 ? 0 : (i >= L ? L - 1 : i);  // L > radius: one reflection suffices
}

// Smallest (hi = false) or largest (hi = true) of reflect_near(a, L) over a .. a + n - 1: the
// identity on 0 .. L-1, a decreasing piece below 0 (values 0 .. -a-1) and above L - 1 (2L-1-e .. L-1).
__device__ __forceinline__ int reflect_span(int a, int n, int L, bool hi) {
  const int e = a + n - 1;
  int lo = a < 0 ? 0 : a, up = e > L - 1 ? L - 1 : e;
  if (e > L - 1) lo = min(lo, 2 * L - 1 - e);
  if (a < 0) up = max(up, -a - 1);
  const int v = hi ? up : lo;
  return v < 0 ? 0 : (v > L - 1 ? L - 1 : v);
}

struct HeatLow {  // heat channels of the low-res stage output, upsampled on the fly
  static constexpr bool kLow = true;
  MapSource src;
  int lh, lw, mh, mw;
};
struct HeatFull {  // already-upsampled planes: frame f, joint j at p + f*fs + j*mh*mw
  static constexpr bool kLow = false;
  const float* p;
  int mh, mw;
  int64_t fs;
  __device__ __forceinline__ float at(int f, int j, int y, int x) const {
    return p[f * fs + ((int64_t)j * mh + y) * mw + x];
  }
};

// Early out of a tile: every value the NMS sees is a convex combination of the tile's source
// values (bilinear f32 weights >= 0 summing to 1 within 4 ulp, normalised non-negative Gaussian taps
// in f64, two f32 roundings), so it is <= M + |M| * 1e-6 for the source maximum M.  A tile whose
// sources all stay below thresh - |.| * 1e-4 cannot hold a value > thresh, hence no peak.
__device__ __forceinline__ bool may_reach(float v, float thresh) {
  return (double)v + fabs((double)v) * 1e-4 >= (double)thresh;
}

// R > 0: radius fixed at compile time (register-blocked passes, NV outputs per thread); R == 0: any
// radius <= kMaxR given at run time (one output per thread).
// Block order (round 4): a 1-D grid where XCD x (= linear block id mod 8) runs every tile of every
// joint of frames x, x + 8, ...: the 18 joints' blocks of a frame read the same low-res pixel
// records (38 + 19 of 64 interleaved channels per 256-B record), so those lines come from HBM
// once, into that XCD's L2, instead of once per XCD.  n_frames: frames of the launch; tx, ty:
// tiles per plane.  Only for launches of >= 8 frames (xcd_major): with fewer, every tile of a frame
// would run on one XCD (one frame: 32 of 256 CUs, 7/8 of the grid exiting at once), so small
// launches take the plain order, which spreads a frame's tiles over the whole chip (advisor r04).
// true when NO thread of the block has `live` (a barrier for every thread): a ballot per wave and one
// store per wave with a live lane -- __syncthreads_or had every lane OR into one LDS word, 64 lanes
// of an instruction on one bank (round 6).  *flag: zeroed before a barrier that precedes this call.
__device__ __forceinline__ bool block_none(bool live, int* flag) {
  if (__ballot(live) && (threadIdx.x & 63) == 0) *flag = 1;
  __syncthreads();
  return *flag == 0;
}

// G (round 6, op_set_peak_mode): the reference's GPU branch (pose_detector.py:111-132) -- the map
// zero-padded instead of reflected (F.convolution_2d pad = ksize / 2, :112-113), w = the 1-D factor
// of its unnormalised ksize x ksize kernel (host_pack.hpp gpu_branch_taps), and >= instead of > in
// the 4-neighbour test (:123-126); the threshold stays strict (:123).  Only HeatLow (the single-scale
// path): the reference's precise path and standalone calls hand it NumPy arrays (CPU branch).
template <class Src, int R, bool G = false>
__global__ __launch_bounds__(kFN) void heat_fused(Src src, int mh, int mw, const double* __restrict__ w, int rr,
                                                  float thresh, int cap, int32_t* __restrict__ stage_key,
                                                  float* __restrict__ stage_score, int32_t* __restrict__ peak_cnt,
                                                  int n_frames, int tx, int ty, int xcd_major) {
  // vertical-pass output pitch: 33 16-B slots (round 6; was kFU + 2 = 100 floats).  The horizontal
  // pass gives lane i the slot (i / 17) * pitch + i % 17 = i + 16 * (i / 17) (17 four-column groups
  // per row), so with a pitch of 1 (mod 16) slots every ds_read_b128 lane group reads 16 distinct
  // slots mod 16: conflict-free (at 25 slots the rows a group spans collided 2-way)
  constexpr int kTP = 4 * 33;
  static_assert(kTP >= kFU + 2 && (kTP / 4) % 16 == 1, "horizontal-pass pitch");
  constexpr int kHP = kFT + 4;  // filtered-map pitch
  constexpr int NB = 4;         // outputs per thread in the register-blocked passes
  __shared__ float up[(kFU + NB) * kFU];         // upsampled region; reused for the filtered map
  __shared__ float tmp[(kFT + 2 + 1) * kTP];     // vertical-pass output; low-res window before that
  // the region's row / column taps: weights (16 B, read by ds_read_b128) apart from the indices
  // (4 B) -- a 24-B AxisTap array put lanes 16 apart on one bank for the i0 reads (round 6)
  __shared__ double2 rtw[kFU], ctw[kFU];
  __shared__ int rti[kFU], cti[kFU];
  __shared__ int any_live;
  static_assert(!G || Src::kLow, "GPU-branch peaks: single-scale maps only");
  const int r = R > 0 ? R : rr;
  const int per_frame = tx * ty * OP_N_JOINTS;
  const int lin = blockIdx.x;
  int f, within;
  if (xcd_major) {
    const int xcd = lin & 7, slot = lin >> 3;
    f = (slot / per_frame) * 8 + xcd;
    within = slot - (slot / per_frame) * per_frame;
  } else {  // plain order: a frame's tiles spread over every XCD
    f = lin / per_frame;
    within = lin - f * per_frame;
  }
  if (f >= n_frames) return;
  const int j = within / (tx * ty), t = within - j * (tx * ty);
  const int fj = f * OP_N_JOINTS + j;
  const int x0 = (t % tx) * kFT, y0 = (t / tx) * kFT;
  const int hr = min(kFT + 2, mh + 1 - y0);  // filtered rows needed: image rows y0-1 .. <= mh-1
  const int hc = min(kFT + 2, mw + 1 - x0);
  const int ur = hr + 2 * r, uc = hc + 2 * r;
  const int uy0 = y0 - 1 - r, ux0 = x0 - 1 - r;
  if constexpr (Src::kLow) {
    for (int i = threadIdx.x; i < ur + uc; i += kFN) {
      const bool row = i < ur;
      const int k = row ? i : i - ur;
      const AxisTap t = row ? axis_tap(reflect_near(uy0 + k, mh), src.lh, mh)
                            : axis_tap(reflect_near(ux0 + k, mw), src.lw, mw);
      (row ? rtw : ctw)[k] = make_double2(t.d1, t.d0);
      (row ? rti : cti)[k] = t.i0;
    }
    if (threadIdx.x == 0) any_live = 0;  // ordered before the flag stores by the barrier below
    __syncthreads();
    // low-res window rows wy .. wy + nwy - 1 (columns likewise): the taps' i0 .. i0 + 1 over the
    // region.  i0 is non-decreasing in the image row, so its extremes come from the extreme rows
    // the reflected region reaches -- computed by every thread (round 6: the bounds were reduced
    // with LDS atomics by every tap, 64 lanes on one word, the bulk of this kernel's bank-conflict
    // cycles)
    const int wy = axis_tap(reflect_span(uy0, ur, mh, false), src.lh, mh).i0;
    const int wx = axis_tap(reflect_span(ux0, uc, mw, false), src.lw, mw).i0;
    const int nwy = axis_tap(reflect_span(uy0, ur, mh, true), src.lh, mh).i0 + 2 - wy;
    const int nwx = axis_tap(reflect_span(ux0, uc, mw, true), src.lw, mw).i0 + 2 - wx;

    const bool staged = nwy <= kFW && nwx <= kFW;  // block-uniform
    const LowMap m = low_map(src.src, src.lw, f);
    const int c = src.src.heat_off + j;
    float* win = tmp;
    bool live = !staged;
    if (staged)
      for (int i = threadIdx.x; i < nwy * nwx; i += kFN) {
        const int a = i / nwx;
        const float v = m.at(c, wy + a, wx + (i - a * nwx));
        win[i] = v;
        live |= may_reach(v, thresh);
      }
    // No low-res value of the window can lift the upsampled + smoothed tile above the peak
    // threshold: the tile has no peak, skip the passes (result identical, see may_reach).
    if (block_none(live, &any_live)) return;
    for (int i = threadIdx.x; i < ur * uc; i += kFN) {
      const int ly = i / uc, lx = i - ly * uc;
      AxisTap ty, tx;
      const double2 wy2 = rtw[ly], wx2 = ctw[lx];
      ty.d1 = wy2.x;
      ty.d0 = wy2.y;
      ty.i0 = rti[ly];
      tx.d1 = wx2.x;
      tx.d0 = wx2.y;
      tx.i0 = cti[lx];
      const UpTap t = up_tap2(ty, tx);
      float v;
      if (staged) {
        const float* q = win + (t.v0 - wy) * nwx + (t.u0 - wx);
        v = up_combine(t, q[0], q[1], q[nwx], q[nwx + 1]);
      } else {
        v = up_sample(m, c, t);
      }
      if constexpr (G) {  // zero padding: region rows / columns outside the map hold 0
        const int yy = uy0 + ly, xx = ux0 + lx;
        if (yy < 0 || yy >= mh || xx < 0 || xx >= mw) v = 0.0f;
      }
      up[ly * kFU + lx] = v;
    }
  } else {
    bool live = false;
    for (int i = threadIdx.x; i < ur * uc; i += kFN) {
      const int ly = i / uc, lx = i - ly * uc;
      const float v = src.at(f, j, reflect_near(uy0 + ly, mh), reflect_near(ux0 + lx, mw));
      up[ly * kFU + lx] = v;
      live |= may_reach(v, thresh);
    }
    if (!__syncthreads_or(live)) return;  // (HeatFull: the precise path's full-resolution planes)
  }
  __syncthreads();
  if constexpr (R > 0) {
    double wr[R + 1];
#pragma unroll
    for (int q = 0; q <= R; ++q) wr[q] = w[q];
    // vertical pass: NB consecutive rows of one column per thread, the 2R+NB inputs read once
    const int ngy = (hr + NB - 1) / NB;
    for (int i = threadIdx.x; i < ngy * uc; i += kFN) {
      const int g = i / uc, lx = i - g * uc;
      const int ly0 = g * NB;
      double v[2 * R + NB];
#pragma unroll
      for (int q = 0; q < 2 * R + NB; ++q) v[q] = (double)up[(ly0 + q) * kFU + lx];
#pragma unroll
      for (int q = 0; q < NB; ++q) {
        double o = __dmul_rn(v[q + R], wr[R]);
#pragma unroll
        for (int jj = -R; jj < 0; ++jj)
          o = __dadd_rn(o, __dmul_rn(__dadd_rn(v[q + R + jj], v[q + R - jj]), wr[R + jj]));
        if (ly0 + q < hr) tmp[(ly0 + q) * kTP + lx] = __double2float_rn(o);
      }
    }
    __syncthreads();
    // horizontal pass: NB consecutive columns of one row per thread (16-byte LDS reads)
    constexpr int ngx = (kFT + 2 + NB - 1) / NB;
    constexpr int NV4 = (2 * R + NB + 3) / 4;
    for (int i = threadIdx.x; i < (kFT + 2) * ngx; i += kFN) {
      const int ly = i / ngx, lx0 = (i - ly * ngx) * NB;
      floatx4 out = {0.0f, 0.0f, 0.0f, 0.0f};  // outside the image a neighbour counts as 0 (pose_detector.py:87-94)
      if (ly < hr && y0 - 1 + ly >= 0) {
        float fv[NV4 * 4];
        const floatx4* src4 = (const floatx4*)(tmp + ly * kTP + lx0);
#pragma unroll
        for (int q = 0; q < NV4; ++q) {
          const floatx4 t = src4[q];
          fv[4 * q + 0] = t[0];
          fv[4 * q + 1] = t[1];
          fv[4 * q + 2] = t[2];
          fv[4 * q + 3] = t[3];
        }
        double v[2 * R + NB];
#pragma unroll
        for (int q = 0; q < 2 * R + NB; ++q) v[q] = (double)fv[q];
#pragma unroll
        for (int q = 0; q < NB; ++q) {
          double o = __dmul_rn(v[q + R], wr[R]);
#pragma unroll
          for (int jj = -R; jj < 0; ++jj)
            o = __dadd_rn(o, __dmul_rn(__dadd_rn(v[q + R + jj], v[q + R - jj]), wr[R + jj]));
          const int lx = lx0 + q;
          if (lx < hc && x0 - 1 + lx >= 0) out[q] = __double2float_rn(o);
        }
      }
      *(floatx4*)(up + ly * kHP + lx0) = out;
    }
  } else {
    for (int i = threadIdx.x; i < hr * uc; i += kFN) {  // vertical pass
      const int ly = i / uc, lx = i - ly * uc;
      const float* col = up + (ly + r) * kFU + lx;
      double o = __dmul_rn((double)col[0], w[r]);
      for (int jj = -r; jj < 0; ++jj)
        o = __dadd_rn(o, __dmul_rn(__dadd_rn((double)col[jj * kFU], (double)col[-jj * kFU]), w[r + jj]));
      tmp[ly * kTP + lx] = __double2float_rn(o);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < (kFT + 2) * (kFT + 2); i += kFN) {  // horizontal pass
      const int ly = i / (kFT + 2), lx = i - ly * (kFT + 2);
      float v = 0.0f;  // outside the image a neighbour counts as 0 (pose_detector.py:87-94)
      if (ly < hr && lx < hc && y0 - 1 + ly >= 0 && x0 - 1 + lx >= 0) {
        const float* row = tmp + ly * kTP + lx + r;
        double o = __dmul_rn((double)row[0], w[r]);
        for (int jj = -r; jj < 0; ++jj)
          o = __dadd_rn(o, __dmul_rn(__dadd_rn((double)row[jj], (double)row[-jj]), w[r + jj]));
        v = __double2float_rn(o);
      }
      up[ly * kHP + lx] = v;
    }
  }
  __syncthreads();
  const float* hm = up;  // filtered map, (kFT + 2) rows of pitch kHP
  constexpr int P = kHP;
  for (int i = threadIdx.x; i < kFT * kFT; i += kFN) {  // strict 4-neighbour NMS (pose_detector.py:87-97)
    const int ly = i / kFT + 1, lx = i % kFT + 1;
    const int y = y0 + ly - 1, x = x0 + lx - 1;
    if (y >= mh || x >= mw) continue;
    const float v = hm[ly * P + lx];
    const bool peak = G ? (v > thresh && v >= hm[(ly - 1) * P + lx] && v >= hm[(ly + 1) * P + lx] &&
                           v >= hm[ly * P + lx - 1] && v >= hm[ly * P + lx + 1])
                        : (v > thresh && v > hm[(ly - 1) * P + lx] && v > hm[(ly + 1) * P + lx] &&
                           v > hm[ly * P + lx - 1] && v > hm[ly * P + lx + 1]);
    if (peak) {
      const int slot = atomicAdd(peak_cnt + fj, 1);
      if (slot < cap) {
        stage_key[(int64_t)fj * cap + slot] = y * mw + x;
        stage_score[(int64_t)fj * cap + slot] = v;
      }
    }
  }
}

// Per (frame, joint): bitonic sort of the staged peaks by y*mw + x (= np.nonzero row-major order).
__global__ __launch_bounds__(512) void peak_sort(const int32_t* __restrict__ stage_key,
                                                 const float* __restrict__ stage_score, int cap, int mw,
                                                 const int32_t* __restrict__ peak_cnt, int32_t* __restrict__ peak_xy,
                                                 float* __restrict__ peak_score) {
  __shared__ int32_t key[2048];
  __shared__ float val[2048];
  const int fj = blockIdx.x;
  int n = peak_cnt[fj];
  if (n > cap) n = cap;  // overflow is reported by the grouping kernel from peak_cnt
  int m = 1;
  while (m < n) m <<= 1;
  for (int i = threadIdx.x; i < m; i += 512) {
    key[i] = i < n ? stage_key[(int64_t)fj * cap + i] : 0x7fffffff;
    val[i] = i < n ? stage_score[(int64_t)fj * cap + i] : 0.0f;
  }
  __syncthreads();
  for (int k = 2; k <= m; k <<= 1)
    for (int jb = k >> 1; jb > 0; jb >>= 1) {
      for (int i = threadIdx.x; i < m; i += 512) {
        const int l = i ^ jb;
        if (l > i) {
          const bool up = (i & k) == 0;
          if ((key[i] > key[l]) == up) {
            const int32_t tk = key[i];
            key[i] = key[l];
            key[l] = tk;
            const float tv = val[i];
            val[i] = val[l];
            val[l] = tv;
          }
        }
      }
      __syncthreads();
    }
  for (int i = threadIdx.x; i < n; i += 512) {
    const int yx = key[i];
    const int y = yx / mw, x = yx - y * mw;
    peak_xy[(int64_t)fj * cap + i] = x | (y << 16);
    peak_score[(int64_t)fj * cap + i] = val[i];
  }
}

// Per (frame, joint), any peak count: each staged peak's rank in y*mw + x order (keys are distinct
// pixels) counted against every other key through LDS tiles; grid (planes, ceil(cap / 256)).
__global__ __launch_bounds__(256) void peak_sort_rank(const int32_t* __restrict__ stage_key,
                                                      const float* __restrict__ stage_score, int cap, int mw,
                                                      const int32_t* __restrict__ peak_cnt, int32_t* __restrict__ peak_xy,
                                                      float* __restrict__ peak_score) {
  __shared__ int32_t tile[2048];
  const int fj = blockIdx.x;
  int n = peak_cnt[fj];
  if (n > cap) n = cap;
  const int i = blockIdx.y * 256 + threadIdx.x;
  if ((int)blockIdx.y * 256 >= n) return;  // whole block idle (uniform)
  const int32_t* keys = stage_key + (int64_t)fj * cap;
  const int32_t ki = i < n ? keys[i] : 0x7fffffff;
  int rank = 0;
  for (int j0 = 0; j0 < n; j0 += 2048) {
    const int m = n - j0 < 2048 ? n - j0 : 2048;
    __syncthreads();
    for (int j = threadIdx.x; j < m; j += 256) tile[j] = keys[j0 + j];
    __syncthreads();
    for (int j = 0; j < m; ++j) rank += tile[j] < ki ? 1 : 0;
  }
  if (i < n) {
    const int y = ki / mw, x = ki - y * mw;
    peak_xy[(int64_t)fj * cap + rank] = x | (y << 16);
    peak_score[(int64_t)fj * cap + rank] = stage_score[(int64_t)fj * cap + i];
  }
}

// The step's counters zeroed by one launch (round 4): a hipMemsetAsync of a few dozen bytes runs as
// two fill kernels on this stack, four per frame for the peak and candidate counters
__global__ __launch_bounds__(256) void zero_counters(int32_t* __restrict__ a, int na, int32_t* __restrict__ b, int nb) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < na) a[i] = 0;
  else if (i - na < nb && b) b[i - na] = 0;
}

// also / also_n: a second counter array zeroed by the same launch (the candidate counts of the
// connection step that follows), or null
template <class Src>
static int run_heat_tiled(const Src& src, const PostShape& s, PostBuffers& b, hipStream_t st, int32_t* also = nullptr,
                          int also_n = 0) {
  const int planes = s.n * OP_N_JOINTS;
  hipLaunchKernelGGL(zero_counters, dim3((unsigned)((planes + also_n + 255) / 256)), dim3(256), 0, st, b.peak_cnt, planes,
                     also, also ? also_n : 0);
  OP_AFTER_LAUNCH("zero_counters", st);
  const int tx = (s.mw + kFT - 1) / kFT, ty = (s.mh + kFT - 1) / kFT;
  const int xm = s.n >= 8;
  const dim3 g((unsigned)((xm ? 8 * ((s.n + 7) / 8) : s.n) * tx * ty * OP_N_JOINTS));
  if (Src::kLow && s.peak_mode == OP_PEAKS_GPU_BRANCH) {  // op_set_peak_mode: the reference's GPU branch
    const double* wg = b.gauss_w + kGaussGpuOff;
    if (s.gpu_radius == 8)  // ksize 17, the reference's default
      hipLaunchKernelGGL((heat_fused<Src, 8, Src::kLow>), g, dim3(kFN), 0, st, src, s.mh, s.mw, wg, s.gpu_radius,
                         s.peak_thresh, b.maxp, b.stage_key, b.stage_score, b.peak_cnt, s.n, tx, ty, xm);
    else
      hipLaunchKernelGGL((heat_fused<Src, 0, Src::kLow>), g, dim3(kFN), 0, st, src, s.mh, s.mw, wg, s.gpu_radius,
                         s.peak_thresh, b.maxp, b.stage_key, b.stage_score, b.peak_cnt, s.n, tx, ty, xm);
  } else if (s.radius == 10)  // gaussian_sigma 2.5, the reference's default
    hipLaunchKernelGGL((heat_fused<Src, 10>), g, dim3(kFN), 0, st, src, s.mh, s.mw, b.gauss_w, s.radius,
                       s.peak_thresh, b.maxp, b.stage_key, b.stage_score, b.peak_cnt, s.n, tx, ty, xm);
  else
    hipLaunchKernelGGL((heat_fused<Src, 0>), g, dim3(kFN), 0, st, src, s.mh, s.mw, b.gauss_w, s.radius,
                       s.peak_thresh, b.maxp, b.stage_key, b.stage_score, b.peak_cnt, s.n, tx, ty, xm);
  OP_AFTER_LAUNCH("heat_fused<Src>", st);
  if (b.maxp <= 2048) {
    hipLaunchKernelGGL(peak_sort, dim3((unsigned)planes), dim3(512), 0, st, b.stage_key, b.stage_score, b.maxp, s.mw,
                       b.peak_cnt, b.peak_xy, b.peak_score);
    OP_AFTER_LAUNCH("peak_sort", st);
  } else {
    hipLaunchKernelGGL(peak_sort_rank, dim3((unsigned)planes, (unsigned)((b.maxp + 255) / 256)), dim3(256), 0, st,
                       b.stage_key, b.stage_score, b.maxp, s.mw, b.peak_cnt, b.peak_xy, b.peak_score);
    OP_AFTER_LAUNCH("peak_sort_rank", st);
  }
  OP_HIP_CHECK(hipGetLastError());
  return OP_OK;
}

// ---------------- launchers ----------------
static inline unsigned nblk(int64_t n) { return (unsigned)((n + 255) / 256); }

// Big mode (b.used != nullptr: the uncapped re-run of one frame, post_big.cpp-style buffers sized
// from the frame's own counts): HBM bitsets / subsets, rank sort, more candidate-pair blocks.
static inline bool big_mode(const PostBuffers& b) { return b.used != nullptr; }

static int launch_greedy(const PostShape& s, PostBuffers& b, hipStream_t st) {
  if (big_mode(b))
    hipLaunchKernelGGL(limb_greedy<true>, dim3(s.n, OP_N_LIMBS), dim3(256), 0, st, s, b);
  else
    hipLaunchKernelGGL(limb_greedy<false>, dim3(s.n, OP_N_LIMBS), dim3(256), 0, st, s, b);
  OP_AFTER_LAUNCH("limb_greedy", st);
  return OP_OK;
}

static int launch_group(const PostShape& s, PostBuffers& b, hipStream_t st) {
  if (big_mode(b))
    hipLaunchKernelGGL(grouping<true>, dim3(s.n), dim3(64), 0, st, s, b);
  else
    hipLaunchKernelGGL(grouping<false>, dim3(s.n), dim3(64), 0, st, s, b);
  OP_AFTER_LAUNCH("grouping", st);
  return OP_OK;
}

static inline unsigned pair_blocks(const PostBuffers& b) { return big_mode(b) ? 64u : 8u; }

static int check_shape(const PostShape& s, const PostBuffers& b) {
  if (s.mw > 0xffff || s.mh > 0x7fff || s.n_integ > 16 || s.n_integ < 2 || (b.maxp > 2048 && !big_mode(b)) ||
      s.radius > kMaxR || (s.peak_mode && (s.gpu_radius > kMaxR || s.mh <= s.gpu_radius || s.mw <= s.gpu_radius)) ||
      s.mh <= s.radius || s.mw <= s.radius || (int64_t)s.mh * s.mw >= 0x7fffffff) {
    set_error("post-process shape outside kernel limits");
    return OP_ERR_INVALID;
  }
  return OP_OK;
}

int launch_post_maps(const MapSource& src, const PostShape& s, PostBuffers& b, hipStream_t st) {
  int rc = check_shape(s, b);
  if (rc) return rc;
  HeatLow hs;
  hs.src = src;
  hs.lh = s.lh;
  hs.lw = s.lw;
  hs.mh = s.mh;
  hs.mw = s.mw;
  if ((rc = run_heat_tiled(hs, s, b, st, b.cand_cnt, s.n * OP_N_LIMBS))) return rc;  // zeroes cand_cnt too
  // axis-tap tables in LDS when they fit 48 KiB (368 x 368 maps: 17 KiB; 1280 x 720: 47 KiB), and
  // the limb's two low-res PAF planes next to them when both fit 64 KiB (46 x 46: +17 KiB): the
  // 80 map reads per candidate pair hit LDS instead of scattered L2 lines
  size_t tab = (size_t)(s.mh + s.mw) * sizeof(AxisTap);
  const size_t planes = (size_t)2 * s.lh * s.lw * sizeof(float);
  const int tables = tab + planes <= 64 * 1024 ? 2 : tab <= 48 * 1024 ? 1 : 0;
  if (tables == 2) tab += planes;
  static bool attr = false;
  if (!attr) {
    OP_HIP_CHECK(hipFuncSetAttribute((const void*)limb_pairs_low, hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024));
    attr = true;
  }
  hipLaunchKernelGGL(limb_pairs_low, dim3(s.n, OP_N_LIMBS, pair_blocks(b)), dim3(256), tables ? tab : 0, st, src, s, b,
                     tables);
  OP_AFTER_LAUNCH("limb_pairs_low", st);
  if ((rc = launch_greedy(s, b, st))) return rc;
  if ((rc = launch_group(s, b, st))) return rc;
  OP_HIP_CHECK(hipGetLastError());
  return OP_OK;
}

int launch_peaks_from_full(const float* heat_full, int32_t n_joint, int32_t mh, int32_t mw, const PostShape& s,
                           PostBuffers& b, hipStream_t st, int64_t fstride) {
  (void)n_joint;
  (void)mh;
  (void)mw;
  int rc = check_shape(s, b);
  if (rc) return rc;
  HeatFull hs;
  hs.p = heat_full;
  hs.mh = s.mh;
  hs.mw = s.mw;
  hs.fs = fstride ? fstride : (int64_t)OP_N_JOINTS * s.mh * s.mw;
  return run_heat_tiled(hs, s, b, st);
}

int launch_connections_full(const float* paf_full, int32_t mh, int32_t mw, const PostShape& s, PostBuffers& b,
                            hipStream_t st, int64_t fstride) {
  (void)mh;
  (void)mw;
  int rc = check_shape(s, b);
  if (rc) return rc;
  OP_HIP_CHECK(hipMemsetAsync(b.cand_cnt, 0, sizeof(int32_t) * s.n * OP_N_LIMBS, st));
  hipLaunchKernelGGL(limb_pairs_full, dim3(s.n, OP_N_LIMBS, pair_blocks(b)), dim3(256), 0, st, paf_full, fstride, s,
                     b);
  OP_AFTER_LAUNCH("limb_pairs_full", st);
  if ((rc = launch_greedy(s, b, st))) return rc;
  OP_HIP_CHECK(hipGetLastError());
  return OP_OK;
}

int launch_grouping(const PostShape& s, PostBuffers& b, hipStream_t st) {
  int rc = check_shape(s, b);
  if (rc) return rc;
  if ((rc = launch_group(s, b, st))) return rc;
  OP_HIP_CHECK(hipGetLastError());
  return OP_OK;
}

int launch_resize_images(const float* x, int32_t c, int32_t h, int32_t w, int32_t oh, int32_t ow, float* y,
                         hipStream_t st) {
  hipLaunchKernelGGL(resize_planar, dim3(nblk((int64_t)c * oh * ow)), dim3(256), 0, st, x, c, h, w, oh, ow, y);
  OP_AFTER_LAUNCH("resize_planar", st);
  OP_HIP_CHECK(hipGetLastError());
  return OP_OK;
}

}  // namespace op
