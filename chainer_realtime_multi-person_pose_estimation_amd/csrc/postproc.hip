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

// ---- heat-map pipeline: (upsample + vertical Gaussian) -> (horizontal Gaussian + NMS) -> sort ----
// Tiles are staged in LDS; the reflect boundary is resolved once per LDS row / column.
constexpr int kVT = 64;   // vertical-pass tile (rows x cols)
constexpr int kHTR = 16;  // horizontal-pass tile rows
constexpr int kHTC = 64;  // horizontal-pass tile cols
constexpr int kMaxR = 16; // max Gaussian radius of the tiled kernels

__device__ __forceinline__ int reflect_near(int i, int L) {
  if (i < 0) i = -i - 1;
  if (i >= L) i = 2 * L - 1 - i;
  return i < 0 ? 0 : (i >= L ? L - 1 : i);  // L > radius: one reflection suffices
}

struct HeatLow {
  MapSource src;
  int lh, lw, mh, mw;
  __device__ __forceinline__ float at(int f, int j, int y, int x) const {
    return up_sample(low_map(src, lw, f), src.heat_off + j, up_tap(y, x, lh, lw, mh, mw));
  }
};
struct HeatFull {  // already-upsampled planes [f*18 + j][mh][mw]
  const float* p;
  int mh, mw;
  __device__ __forceinline__ float at(int f, int j, int y, int x) const {
    return p[(((int64_t)f * OP_N_JOINTS + j) * mh + y) * mw + x];
  }
};

template <class Src>
__global__ __launch_bounds__(256) void heat_vpass(Src src, int mh, int mw, const double* __restrict__ w, int r,
                                                  float* __restrict__ tmp) {
  __shared__ float tile[kVT + 2 * kMaxR][kVT];
  const int fj = blockIdx.z;
  const int f = fj / OP_N_JOINTS, j = fj - f * OP_N_JOINTS;
  const int x0 = blockIdx.x * kVT, y0 = blockIdx.y * kVT;
  const int rows = kVT + 2 * r;
  for (int i = threadIdx.x; i < rows * kVT; i += 256) {
    const int ly = i / kVT, lx = i - ly * kVT;
    const int x = x0 + lx;
    float v = 0.0f;
    if (x < mw) v = src.at(f, j, reflect_near(y0 - r + ly, mh), x);
    tile[ly][lx] = v;
  }
  __syncthreads();
  const int lx = threadIdx.x & (kVT - 1);
  const int x = x0 + lx;
  if (x >= mw) return;
  for (int ly = threadIdx.x / kVT; ly < kVT; ly += 256 / kVT) {
    const int y = y0 + ly;
    if (y >= mh) break;
    double o = __dmul_rn((double)tile[ly + r][lx], w[r]);
    for (int jj = -r; jj < 0; ++jj)
      o = __dadd_rn(o, __dmul_rn(__dadd_rn((double)tile[ly + r + jj][lx], (double)tile[ly + r - jj][lx]), w[r + jj]));
    tmp[((int64_t)fj * mh + y) * mw + x] = __double2float_rn(o);
  }
}

// Horizontal pass + strict 4-neighbour NMS on a kHTR x kHTC tile; peaks are appended to the
// (frame, joint) staging list as (y*mw + x, score) -- order restored by peak_sort.
__global__ __launch_bounds__(256) void heat_hpass_nms(const float* __restrict__ tmp, int mh, int mw,
                                                      const double* __restrict__ w, int r, float thresh, int cap,
                                                      int32_t* __restrict__ stage_key, float* __restrict__ stage_score,
                                                      int32_t* __restrict__ peak_cnt) {
  __shared__ float src[kHTR + 2][kHTC + 2 + 2 * kMaxR];
  __shared__ float hm[kHTR + 2][kHTC + 2];
  const int fj = blockIdx.z;
  const int x0 = blockIdx.x * kHTC, y0 = blockIdx.y * kHTR;
  const int cols = kHTC + 2 + 2 * r;
  const float* plane = tmp + (int64_t)fj * mh * mw;
  for (int i = threadIdx.x; i < (kHTR + 2) * cols; i += 256) {
    const int ly = i / cols, lx = i - ly * cols;
    const int y = y0 - 1 + ly;
    float v = 0.0f;
    if (y >= 0 && y < mh) v = plane[(int64_t)y * mw + reflect_near(x0 - 1 - r + lx, mw)];
    src[ly][lx] = v;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < (kHTR + 2) * (kHTC + 2); i += 256) {
    const int ly = i / (kHTC + 2), lx = i - ly * (kHTC + 2);
    const int y = y0 - 1 + ly, x = x0 - 1 + lx;
    float v = 0.0f;  // outside the image a neighbour counts as 0 (pose_detector.py:87-94)
    if (y >= 0 && y < mh && x >= 0 && x < mw) {
      double o = __dmul_rn((double)src[ly][lx + r], w[r]);
      for (int jj = -r; jj < 0; ++jj)
        o = __dadd_rn(o, __dmul_rn(__dadd_rn((double)src[ly][lx + r + jj], (double)src[ly][lx + r - jj]), w[r + jj]));
      v = __double2float_rn(o);
    }
    hm[ly][lx] = v;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kHTR * kHTC; i += 256) {
    const int ly = i / kHTC + 1, lx = i % kHTC + 1;
    const int y = y0 + ly - 1, x = x0 + lx - 1;
    if (y >= mh || x >= mw) continue;
    const float v = hm[ly][lx];
    if (v > thresh && v > hm[ly - 1][lx] && v > hm[ly + 1][lx] && v > hm[ly][lx - 1] && v > hm[ly][lx + 1]) {
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

template <class Src>
static int run_heat_tiled(const Src& src, const PostShape& s, PostBuffers& b, hipStream_t st) {
  const int planes = s.n * OP_N_JOINTS;
  OP_HIP_CHECK(hipMemsetAsync(b.peak_cnt, 0, sizeof(int32_t) * planes, st));
  dim3 gv((unsigned)((s.mw + kVT - 1) / kVT), (unsigned)((s.mh + kVT - 1) / kVT), (unsigned)planes);
  hipLaunchKernelGGL((heat_vpass<Src>), gv, dim3(256), 0, st, src, s.mh, s.mw, b.gauss_w, s.radius, b.tmp);
  OP_AFTER_LAUNCH("heat_vpass<Src>", st);
  dim3 gh((unsigned)((s.mw + kHTC - 1) / kHTC), (unsigned)((s.mh + kHTR - 1) / kHTR), (unsigned)planes);
  hipLaunchKernelGGL(heat_hpass_nms, gh, dim3(256), 0, st, b.tmp, s.mh, s.mw, b.gauss_w, s.radius, s.peak_thresh,
                     b.maxp, b.stage_key, b.stage_score, b.peak_cnt);
  OP_AFTER_LAUNCH("heat_hpass_nms", st);
  hipLaunchKernelGGL(peak_sort, dim3((unsigned)planes), dim3(512), 0, st, b.stage_key, b.stage_score, b.maxp, s.mw,
                     b.peak_cnt, b.peak_xy, b.peak_score);
  OP_AFTER_LAUNCH("peak_sort", st);
  OP_HIP_CHECK(hipGetLastError());
  return OP_OK;
}

// ---------------- launchers ----------------
static inline unsigned nblk(int64_t n) { return (unsigned)((n + 255) / 256); }

static int check_shape(const PostShape& s, const PostBuffers& b) {
  if (s.mw > 0xffff || s.mh > 0x7fff || s.n_integ > 16 || s.n_integ < 2 || b.maxp > 2048 || s.radius > kMaxR ||
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
  if ((rc = run_heat_tiled(hs, s, b, st))) return rc;
  OP_HIP_CHECK(hipMemsetAsync(b.cand_cnt, 0, sizeof(int32_t) * s.n * OP_N_LIMBS, st));
  hipLaunchKernelGGL(limb_pairs_low, dim3(s.n, OP_N_LIMBS, 8), dim3(256), 0, st, src, s, b);
  OP_AFTER_LAUNCH("limb_pairs_low", st);
  hipLaunchKernelGGL(limb_greedy, dim3(s.n, OP_N_LIMBS), dim3(256), 0, st, s, b);
  OP_AFTER_LAUNCH("limb_greedy", st);
  hipLaunchKernelGGL(grouping, dim3(s.n), dim3(64), 0, st, s, b);
  OP_AFTER_LAUNCH("grouping", st);
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
  HeatFull hs;
  hs.p = heat_full;
  hs.mh = s.mh;
  hs.mw = s.mw;
  return run_heat_tiled(hs, s, b, st);
}

int launch_connections_full(const float* paf_full, int32_t mh, int32_t mw, const PostShape& s, PostBuffers& b,
                            hipStream_t st) {
  (void)mh;
  (void)mw;
  int rc = check_shape(s, b);
  if (rc) return rc;
  OP_HIP_CHECK(hipMemsetAsync(b.cand_cnt, 0, sizeof(int32_t) * s.n * OP_N_LIMBS, st));
  hipLaunchKernelGGL(limb_pairs_full, dim3(s.n, OP_N_LIMBS, 8), dim3(256), 0, st, paf_full, s, b);
  OP_AFTER_LAUNCH("limb_pairs_full", st);
  hipLaunchKernelGGL(limb_greedy, dim3(s.n, OP_N_LIMBS), dim3(256), 0, st, s, b);
  OP_AFTER_LAUNCH("limb_greedy", st);
  OP_HIP_CHECK(hipGetLastError());
  return OP_OK;
}

int launch_grouping(const PostShape& s, PostBuffers& b, hipStream_t st) {
  int rc = check_shape(s, b);
  if (rc) return rc;
  hipLaunchKernelGGL(grouping, dim3(s.n), dim3(64), 0, st, s, b);
  OP_AFTER_LAUNCH("grouping", st);
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
