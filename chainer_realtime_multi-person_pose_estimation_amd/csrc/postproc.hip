// PAF post-process kernels for gfx950 (pose_detector.py:75-265, 501-517).
//
// Bit-exact restatement of the reference CPU path (the parity target):
//   upsample_heat   F.resize_images align-corners bilinear, f64 weights cast to f32      :501-502
//   gauss_v/gauss_h scipy gaussian_filter(sigma 2.5): reflect, 21 taps, f64 accumulate in
//                   NI_Correlate1D's symmetric order, f32 store between the two passes    :86
//   nms_compact     strict 4-neighbour NMS, peaks ordered (joint, y, x) by a block-wide
//                   ordered (ballot + prefix) compaction                                  :87-110
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

// Chainer <= 6 ResizeImages weights for output (oy, ox).
__device__ __forceinline__ UpTap up_tap(int oy, int ox, int H, int W, int oH, int oW) {
  const double v = linspace_at(0.0, (double)(H - 1), oH, oy);
  const double u = linspace_at(0.0, (double)(W - 1), oW, ox);
  int v0 = (int)floor(v);
  v0 = v0 > H - 2 ? H - 2 : v0;
  v0 = v0 < 0 ? 0 : v0;
  int u0 = (int)floor(u);
  u0 = u0 > W - 2 ? W - 2 : u0;
  u0 = u0 < 0 ? 0 : u0;
  const double du1 = __dsub_rn((double)(u0 + 1), u), du0 = __dsub_rn(u, (double)u0);
  const double dv1 = __dsub_rn((double)(v0 + 1), v), dv0 = __dsub_rn(v, (double)v0);
  UpTap t;
  t.u0 = u0;
  t.v0 = v0;
  t.w1 = __double2float_rn(__dmul_rn(du1, dv1));
  t.w2 = __double2float_rn(__dmul_rn(du0, dv1));
  t.w3 = __double2float_rn(__dmul_rn(du1, dv0));
  t.w4 = __double2float_rn(__dmul_rn(du0, dv0));
  return t;
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

// heat channels 0..17 (the background channel 18 is dropped, pose_detector.py:78) -> up[f][j][y][x]
__global__ __launch_bounds__(256) void upsample_heat(MapSource src, PostShape s, float* __restrict__ up) {
  const int64_t plane = (int64_t)s.mh * s.mw;
  const int64_t total = (int64_t)s.n * OP_N_JOINTS * plane;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int ox = (int)(i % s.mw);
  const int oy = (int)((i / s.mw) % s.mh);
  const int j = (int)((i / plane) % OP_N_JOINTS);
  const int f = (int)(i / (plane * OP_N_JOINTS));
  const UpTap t = up_tap(oy, ox, s.lh, s.lw, s.mh, s.mw);
  up[i] = up_sample(low_map(src, s.lw, f), src.heat_off + j, t);
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

__device__ __forceinline__ int reflect_index(int i, int L) {
  const int p = 2 * L;
  i %= p;
  if (i < 0) i += p;
  if (i >= L) i = p - 1 - i;
  return i;
}

// NI_Correlate1D symmetric branch along y (axis 0): o = x0*w0; o += (x[-k] + x[+k]) * w[-k] for k = r..1.
__global__ __launch_bounds__(256) void gauss_v(const float* __restrict__ in, float* __restrict__ out, int nplanes,
                                               int H, int W, const double* __restrict__ w, int r) {
  const int64_t plane = (int64_t)H * W;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= plane * nplanes) return;
  const int x = (int)(i % W);
  const int y = (int)((i / W) % H);
  const float* p = in + (i / plane) * plane;
  double o = __dmul_rn((double)p[(int64_t)y * W + x], w[r]);
  for (int jj = -r; jj < 0; ++jj) {
    const double a = (double)p[(int64_t)reflect_index(y + jj, H) * W + x];
    const double b = (double)p[(int64_t)reflect_index(y - jj, H) * W + x];
    o = __dadd_rn(o, __dmul_rn(__dadd_rn(a, b), w[r + jj]));
  }
  out[i] = __double2float_rn(o);
}

// Same along x (axis 1), one row per 256-thread block chunk.
__global__ __launch_bounds__(256) void gauss_h(const float* __restrict__ in, float* __restrict__ out, int nplanes, int H,
                                               int W, const double* __restrict__ w, int r) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)H * W * nplanes) return;
  const int x = (int)(i % W);
  const float* row = in + (i / W) * W;
  double o = __dmul_rn((double)row[x], w[r]);
  for (int jj = -r; jj < 0; ++jj) {
    const double a = (double)row[reflect_index(x + jj, W)];
    const double b = (double)row[reflect_index(x - jj, W)];
    o = __dadd_rn(o, __dmul_rn(__dadd_rn(a, b), w[r + jj]));
  }
  out[i] = __double2float_rn(o);
}

// Strict 4-neighbour NMS + ordered compaction, one 256-thread block per (frame, joint).
__global__ __launch_bounds__(256) void nms_compact(const float* __restrict__ hm, int H, int W, float thresh, int maxp,
                                                   int32_t* __restrict__ peak_xy, float* __restrict__ peak_score,
                                                   int32_t* __restrict__ peak_cnt) {
  __shared__ int wave_cnt[4];
  __shared__ int running;
  const int fj = blockIdx.x;  // frame * 18 + joint
  const float* m = hm + (int64_t)fj * H * W;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) running = 0;
  __syncthreads();
  const int64_t total = (int64_t)H * W;
  for (int64_t base = 0; base < total; base += 256) {
    const int64_t p = base + tid;
    bool pk = false;
    float v = 0.0f;
    int x = 0, y = 0;
    if (p < total) {
      y = (int)(p / W);
      x = (int)(p - (int64_t)y * W);
      v = m[p];
      const float up = y > 0 ? m[p - W] : 0.0f;
      const float dn = y < H - 1 ? m[p + W] : 0.0f;
      const float lf = x > 0 ? m[p - 1] : 0.0f;
      const float rt = x < W - 1 ? m[p + 1] : 0.0f;
      pk = v > thresh && v > up && v > dn && v > lf && v > rt;
    }
    const unsigned long long bal = __ballot(pk);
    if (lane == 0) wave_cnt[wave] = __popcll(bal);
    __syncthreads();
    int before = running;
    for (int q = 0; q < wave; ++q) before += wave_cnt[q];
    const int pos = before + __popcll(bal & ((1ull << lane) - 1ull));
    if (pk && pos < maxp) {
      peak_xy[(int64_t)fj * maxp + pos] = x | (y << 16);
      peak_score[(int64_t)fj * maxp + pos] = v;
    }
    __syncthreads();
    if (tid == 0) running += wave_cnt[0] + wave_cnt[1] + wave_cnt[2] + wave_cnt[3];
    __syncthreads();
  }
  if (tid == 0) peak_cnt[fj] = running;  // may exceed maxp: overflow is reported per frame
}

// PAF sample at map pixel (y, x) of PAF channel c: recomputed from the low-res map with the
// upsample formula (identical f32 value to the full-res map the reference indexes), or read from a
// full-res planar map (stage-level ABI).
struct PafLow {
  LowMap m;
  int lh, lw, mh, mw, off;
  __device__ __forceinline__ float at(int c, int y, int x) const {
    return up_sample(m, off + c, up_tap(y, x, lh, lw, mh, mw));
  }
};
struct PafFull {
  const float* p;
  int mh, mw;
  __device__ __forceinline__ float at(int c, int y, int x) const { return p[((int64_t)c * mh + y) * mw + x]; }
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
      const double px = (double)paf.at(2 * l, yi, xi);
      const double py = (double)paf.at(2 * l + 1, yi, xi);
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

__global__ __launch_bounds__(256) void limb_pairs_low(MapSource src, PostShape s, PostBuffers b) {
  const int f = blockIdx.x, l = blockIdx.y;
  PafLow paf;
  paf.m = low_map(src, s.lw, f);
  paf.lh = s.lh;
  paf.lw = s.lw;
  paf.mh = s.mh;
  paf.mw = s.mw;
  paf.off = src.paf_off;
  limb_pairs_body(paf, s, b, f, l);
}

__global__ __launch_bounds__(256) void limb_pairs_full(const float* __restrict__ paf_full, PostShape s, PostBuffers b) {
  PafFull paf;
  paf.p = paf_full;
  paf.mh = s.mh;
  paf.mw = s.mw;
  limb_pairs_body(paf, s, b, blockIdx.x, blockIdx.y);
}

// Greedy assignment per (frame, limb): repeatedly accept the best remaining candidate whose two
// peaks are both unused, until min(|A|,|B|) connections (pose_detector.py:172-177).  Accepting
// the (score desc, index asc) maximum among still-valid candidates is exactly first-fit over
// the stably sorted list: every skipped candidate keeps a used endpoint forever.
__global__ __launch_bounds__(256) void limb_greedy(PostShape s, PostBuffers b) {
  __shared__ unsigned used_a[64], used_b[64];  // maxp <= 2048
  __shared__ double red_s[4];
  __shared__ int red_i[4];
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
  for (int i = tid; i < 64; i += 256) {
    used_a[i] = 0;
    used_b[i] = 0;
  }
  __syncthreads();
  const int lim = na < nb ? na : nb;
  const double* cs = b.cand_score + fl * b.maxc;
  const int32_t* ci = b.cand_idx + fl * b.maxc;
  int got = 0;
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

// grouping_key_points + subsets_to_pose_array, one wave per frame.
__global__ __launch_bounds__(64) void grouping(PostShape s, PostBuffers b) {
  __shared__ int16_t ids[kMaxSubsetsLds][OP_N_JOINTS];
  __shared__ double sc[kMaxSubsetsLds][2];
  __shared__ int base[OP_N_JOINTS + 1];
  __shared__ int cnt[OP_N_JOINTS];
  const int f = blockIdx.x;
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
  auto pscore = [&](int joint, int id) -> double {
    return (double)b.peak_score[((int64_t)f * OP_N_JOINTS + joint) * b.maxp + (id - base[joint])];
  };
  for (int l = 0; l < OP_N_LIMBS && status == OP_OK; ++l) {
    const int ja = s.limbs[l][0], jb = s.limbs[l][1];
    const int64_t fl = (int64_t)f * OP_N_LIMBS + l;
    const int K = b.conn_cnt[fl];
    for (int c = 0; c < K && status == OP_OK; ++c) {
      const int ia = b.conn_ab[2 * (fl * b.maxp + c)];
      const int ib = b.conn_ab[2 * (fl * b.maxp + c) + 1];
      const double score = b.conn_score[fl * b.maxp + c];
      int found = 0, f0 = -1, f1 = -1;
      for (int s0 = 0; s0 < S; s0 += 64) {
        const int r = s0 + lane;
        const bool m = r < S && (ids[r][ja] == ia || ids[r][jb] == ib);
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
        if (lane == 0 && ids[f0][jb] != ib) {
          ids[f0][jb] = (int16_t)ib;
          sc[f0][1] = __dadd_rn(sc[f0][1], 1.0);
          sc[f0][0] = __dadd_rn(sc[f0][0], __dadd_rn(pscore(jb, ib), score));
        }
      } else if (found == 2) {
        const bool both = lane < OP_N_JOINTS && ids[f0][lane] >= 0 && ids[f1][lane] >= 0;
        if (__ballot(both) == 0ull) {
          if (lane < OP_N_JOINTS) ids[f0][lane] = (int16_t)(ids[f0][lane] + ids[f1][lane] + 1);
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
            int16_t row[OP_N_JOINTS];
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
        } else if (lane == 0) {
          const int fs[2] = {f0, f1};
          for (int q = 0; q < 2; ++q) {
            const int t = fs[q];
            if (ids[t][ja] == -1) {
              ids[t][ja] = (int16_t)ia;
              sc[t][1] = __dadd_rn(sc[t][1], 1.0);
              sc[t][0] = __dadd_rn(sc[t][0], __dadd_rn(pscore(ja, ia), score));
            } else if (ids[t][jb] == -1) {
              ids[t][jb] = (int16_t)ib;
              sc[t][1] = __dadd_rn(sc[t][1], 1.0);
              sc[t][0] = __dadd_rn(sc[t][0], __dadd_rn(pscore(jb, ib), score));
            }
          }
        }
      } else if (l != 9 && l != 13) {
        if (S >= kMaxSubsetsLds || S >= b.maxs) {
          status = OP_ERR_CAPACITY;
          break;
        }
        if (lane < OP_N_JOINTS) ids[S][lane] = (int16_t)(lane == ja ? ia : (lane == jb ? ib : -1));
        if (lane == 0) {
          sc[S][1] = 2.0;
          sc[S][0] = __dadd_rn(__dadd_rn(pscore(ja, ia), pscore(jb, ib)), score);
        }
        ++S;
      }
      __syncthreads();
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

// ---------------- launchers ----------------
static inline unsigned nblk(int64_t n) { return (unsigned)((n + 255) / 256); }

static int run_gauss_nms(const float* src_up, const PostShape& s, PostBuffers& b, hipStream_t st) {
  const int64_t planes = (int64_t)s.n * OP_N_JOINTS;
  const int64_t total = planes * s.mh * s.mw;
  hipLaunchKernelGGL(gauss_v, dim3(nblk(total)), dim3(256), 0, st, src_up, b.tmp, (int)planes, s.mh, s.mw, b.gauss_w,
                     s.radius);
  hipLaunchKernelGGL(gauss_h, dim3(nblk(total)), dim3(256), 0, st, b.tmp, b.hm, (int)planes, s.mh, s.mw, b.gauss_w,
                     s.radius);
  hipLaunchKernelGGL(nms_compact, dim3((unsigned)planes), dim3(256), 0, st, b.hm, s.mh, s.mw, s.peak_thresh, b.maxp,
                     b.peak_xy, b.peak_score, b.peak_cnt);
  OP_HIP_CHECK(hipGetLastError());
  return OP_OK;
}

static int check_shape(const PostShape& s, const PostBuffers& b) {
  if (s.mw > 0xffff || s.mh > 0x7fff || s.n_integ > 16 || s.n_integ < 2 || b.maxp > 2048 || s.radius > 32) {
    set_error("post-process shape outside kernel limits");
    return OP_ERR_INVALID;
  }
  return OP_OK;
}

int launch_post_maps(const MapSource& src, const PostShape& s, PostBuffers& b, hipStream_t st) {
  int rc = check_shape(s, b);
  if (rc) return rc;
  const int64_t total = (int64_t)s.n * OP_N_JOINTS * s.mh * s.mw;
  hipLaunchKernelGGL(upsample_heat, dim3(nblk(total)), dim3(256), 0, st, src, s, b.up);
  if ((rc = run_gauss_nms(b.up, s, b, st))) return rc;
  OP_HIP_CHECK(hipMemsetAsync(b.cand_cnt, 0, sizeof(int32_t) * s.n * OP_N_LIMBS, st));
  hipLaunchKernelGGL(limb_pairs_low, dim3(s.n, OP_N_LIMBS, 8), dim3(256), 0, st, src, s, b);
  hipLaunchKernelGGL(limb_greedy, dim3(s.n, OP_N_LIMBS), dim3(256), 0, st, s, b);
  hipLaunchKernelGGL(grouping, dim3(s.n), dim3(64), 0, st, s, b);
  OP_HIP_CHECK(hipGetLastError());
  return OP_OK;
}

int launch_peaks_from_full(const float* heat_full, int32_t n_joint, int32_t mh, int32_t mw, const PostShape& s,
                           PostBuffers& b, hipStream_t st) {
  (void)n_joint;
  (void)mh;
  (void)mw;
  int rc = check_shape(s, b);
  if (rc) return rc;
  return run_gauss_nms(heat_full, s, b, st);
}

int launch_connections_full(const float* paf_full, int32_t mh, int32_t mw, const PostShape& s, PostBuffers& b,
                            hipStream_t st) {
  (void)mh;
  (void)mw;
  int rc = check_shape(s, b);
  if (rc) return rc;
  OP_HIP_CHECK(hipMemsetAsync(b.cand_cnt, 0, sizeof(int32_t) * s.n * OP_N_LIMBS, st));
  hipLaunchKernelGGL(limb_pairs_full, dim3(s.n, OP_N_LIMBS, 8), dim3(256), 0, st, paf_full, s, b);
  hipLaunchKernelGGL(limb_greedy, dim3(s.n, OP_N_LIMBS), dim3(256), 0, st, s, b);
  OP_HIP_CHECK(hipGetLastError());
  return OP_OK;
}

int launch_grouping(const PostShape& s, PostBuffers& b, hipStream_t st) {
  int rc = check_shape(s, b);
  if (rc) return rc;
  hipLaunchKernelGGL(grouping, dim3(s.n), dim3(64), 0, st, s, b);
  OP_HIP_CHECK(hipGetLastError());
  return OP_OK;
}

int launch_resize_images(const float* x, int32_t c, int32_t h, int32_t w, int32_t oh, int32_t ow, float* y,
                         hipStream_t st) {
  hipLaunchKernelGGL(resize_planar, dim3(nblk((int64_t)c * oh * ow)), dim3(256), 0, st, x, c, h, w, oh, ow, y);
  OP_HIP_CHECK(hipGetLastError());
  return OP_OK;
}

}  // namespace op
