/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into, loaded by, or called
 * from the product path (chainer_realtime_multi-person_pose_estimation_amd/).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it.
 *
 * Plain-C CPU restatement of the reference post-process, one function per
 * reference step.  Every arithmetic order below is the one NumPy / SciPy /
 * Chainer use in the reference (verified bit-for-bit against the reference's
 * own code run in the build container; fixtures in tests/golden/).
 * Build with -ffp-contract=off: every fused multiply-add here is explicit.
 *
 *   orc_resize_align_corners   Chainer<=6 F.resize_images      pose_detector.py:501-502
 *   orc_gaussian_weights       scipy _gaussian_kernel1d        pose_detector.py:86
 *   orc_gaussian_filter        scipy gaussian_filter (reflect) pose_detector.py:86
 *   orc_find_peaks             strict 4-neighbour NMS          pose_detector.py:75-110
 *   orc_candidate_connections  PAF line integral               pose_detector.py:135-159
 *   orc_connections            greedy per-limb assignment      pose_detector.py:161-181
 *   orc_grouping               person grouping                 pose_detector.py:183-250
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORC_OK 0
#define ORC_ERR_CAPACITY 3
#define ORC_ERR_INDEX 4 /* reference raises IndexError at pose_detector.py:197 */

/* Chainer <=6 ResizeImages.forward (align corners), recalled semantics:
 * u = linspace(0, W-1, oW) (f64), u0 = clip(floor(u), 0, W-2), u1 = u0+1,
 * weights formed in f64 then cast to f32, y = ((w1*x00 + w2*x01) + w3*x10) + w4*x11 in f32. */
static double linspace_at(double start, double stop, int num, int i) {
  if (num == 1) return start;
  if (i == num - 1) return stop;
  double step = (stop - start) / (double)(num - 1);
  double y;
  if (step == 0.0) {
    y = ((double)i / (double)(num - 1)) * (stop - start);
  } else {
    y = (double)i * step;
  }
  return y + start;
}

void orc_resize_align_corners(const float* x, int C, int H, int W, int oH, int oW, float* y) {
  for (int oy = 0; oy < oH; ++oy) {
    double v = linspace_at(0.0, (double)(H - 1), oH, oy);
    int v0 = (int)floor(v);
    if (v0 > H - 2) v0 = H - 2;
    if (v0 < 0) v0 = 0;
    int v1 = v0 + 1;
    for (int ox = 0; ox < oW; ++ox) {
      double u = linspace_at(0.0, (double)(W - 1), oW, ox);
      int u0 = (int)floor(u);
      if (u0 > W - 2) u0 = W - 2;
      if (u0 < 0) u0 = 0;
      int u1 = u0 + 1;
      float w1 = (float)(((double)u1 - u) * ((double)v1 - v));
      float w2 = (float)((u - (double)u0) * ((double)v1 - v));
      float w3 = (float)(((double)u1 - u) * (v - (double)v0));
      float w4 = (float)((u - (double)u0) * (v - (double)v0));
      for (int c = 0; c < C; ++c) {
        const float* p = x + (size_t)c * H * W;
        float a = w1 * p[v0 * W + u0];
        float b = w2 * p[v0 * W + u1];
        float s = a + b;
        s = s + w3 * p[v1 * W + u0];
        s = s + w4 * p[v1 * W + u1];
        y[((size_t)c * oH + oy) * oW + ox] = s;
      }
    }
  }
}

/* NumPy pairwise summation (numpy/_core/src/umath/loops_utils.h) for n <= 128. */
static double np_pairwise_sum(const double* a, int n) {
  if (n < 8) {
    double res = 0.0;
    for (int i = 0; i < n; ++i) res += a[i];
    return res;
  }
  double r[8];
  for (int j = 0; j < 8; ++j) r[j] = a[j];
  int i;
  for (i = 8; i < n - (n % 8); i += 8)
    for (int j = 0; j < 8; ++j) r[j] += a[i + j];
  double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; ++i) res += a[i];
  return res;
}

/* scipy.ndimage._filters._gaussian_kernel1d(sigma, 0, radius):
 * phi = exp(-0.5/sigma^2 * x^2); phi /= phi.sum().  Returns radius. */
int orc_gaussian_weights(double sigma, double truncate, double* w, int cap) {
  int radius = (int)(truncate * sigma + 0.5);
  int n = 2 * radius + 1;
  if (n > cap) return -1;
  double sigma2 = sigma * sigma;
  double coef = -0.5 / sigma2;
  for (int i = 0; i < n; ++i) {
    double xx = (double)((long)(i - radius) * (long)(i - radius));
    w[i] = exp(coef * xx);
  }
  double s = np_pairwise_sum(w, n);
  for (int i = 0; i < n; ++i) w[i] = w[i] / s;
  return radius;
}

/* scipy 'reflect' extension: (d c b a | a b c d | d c b a), period 2L. */
static int reflect_index(int i, int L) {
  int p = 2 * L;
  i %= p;
  if (i < 0) i += p;
  if (i >= L) i = p - 1 - i;
  return i;
}

/* NI_Correlate1D symmetric branch: o = x0*w0; for jj=-r..-1: o += (x[jj] + x[-jj]) * w[jj]  (all f64).
 * gaussian_filter runs axis 0 then axis 1, storing f32 between passes. w has 2r+1 entries. */
void orc_gaussian_filter(const float* in, float* out, float* tmp, int H, int W, const double* w, int r) {
  const double* fw = w + r;
  /* axis 0 (along y) */
  double* line = (double*)malloc(sizeof(double) * (size_t)(H > W ? H : W) + 16);
  for (int x = 0; x < W; ++x) {
    for (int y = 0; y < H; ++y) {
      double o = (double)in[(size_t)y * W + x] * fw[0];
      for (int jj = -r; jj < 0; ++jj) {
        double a = (double)in[(size_t)reflect_index(y + jj, H) * W + x];
        double b = (double)in[(size_t)reflect_index(y - jj, H) * W + x];
        o += (a + b) * fw[jj];
      }
      tmp[(size_t)y * W + x] = (float)o;
    }
  }
  /* axis 1 (along x) */
  for (int y = 0; y < H; ++y) {
    const float* row = tmp + (size_t)y * W;
    for (int x = 0; x < W; ++x) {
      double o = (double)row[x] * fw[0];
      for (int jj = -r; jj < 0; ++jj) {
        double a = (double)row[reflect_index(x + jj, W)];
        double b = (double)row[reflect_index(x - jj, W)];
        o += (a + b) * fw[jj];
      }
      out[(size_t)y * W + x] = (float)o;
    }
  }
  free(line);
}

/* pose_detector.py:82-110 (CPU branch).  hm: J filtered maps (J = 18).
 * Peak iff v > thresh (f32 compare, NumPy 2 weak-scalar rule) and strictly greater than
 * its 4 neighbours (out-of-image neighbours are 0).  Rows [joint, x, y, score, id], ordered by
 * joint, then y, then x (row-major nonzero).  Returns N, or -1 on capacity overflow. */
long orc_find_peaks(const float* hm, int J, int H, int W, float thresh, double* peaks, long cap) {
  long n = 0;
  for (int j = 0; j < J; ++j) {
    const float* m = hm + (size_t)j * H * W;
    for (int y = 0; y < H; ++y) {
      for (int x = 0; x < W; ++x) {
        float v = m[(size_t)y * W + x];
        float up = y > 0 ? m[(size_t)(y - 1) * W + x] : 0.0f;
        float dn = y < H - 1 ? m[(size_t)(y + 1) * W + x] : 0.0f;
        float lf = x > 0 ? m[(size_t)y * W + x - 1] : 0.0f;
        float rt = x < W - 1 ? m[(size_t)y * W + x + 1] : 0.0f;
        if (v > thresh && v > up && v > dn && v > lf && v > rt) {
          if (n >= cap) return -1;
          double* p = peaks + n * 5;
          p[0] = (double)j; p[1] = (double)x; p[2] = (double)y; p[3] = (double)v; p[4] = (double)n;
          ++n;
        }
      }
    }
  }
  return n;
}

typedef struct {
  int32_t n_integ_points;        /* 10   entity.py:77 */
  int32_t n_integ_points_thresh; /* 8    entity.py:78 */
  double inner_product_thresh;   /* 0.05 entity.py:80 */
  double limb_length_ratio;      /* 1.0  entity.py:81 */
  double length_penalty_value;   /* 1    entity.py:82 */
  int32_t n_subset_limbs_thresh; /* 3    entity.py:83 */
  double subset_score_thresh;    /* 0.2  entity.py:84 */
} orc_params;

typedef struct { double score; long idx; int32_t a, b; } orc_cand;

static int cand_cmp(const void* pa, const void* pb) {
  const orc_cand* a = (const orc_cand*)pa;
  const orc_cand* b = (const orc_cand*)pb;
  if (a->score > b->score) return -1;
  if (a->score < b->score) return 1;
  return (a->idx < b->idx) ? -1 : (a->idx > b->idx);
}

/* pose_detector.py:135-159.  paf_x/paf_y: one limb's 2 planes (H, W).  cand rows [x, y, score, id].
 * Output rows [id_a, id_b, score] sorted by score desc (Python's stable sorted(reverse=True)
 * == total order (score desc, enumeration index asc)).  Returns count or -1 on overflow. */
long orc_candidate_connections(const float* paf_x, const float* paf_y, int H, int W,
                               const double* cand_a, int na, const double* cand_b, int nb,
                               double img_len, const orc_params* prm, double* out, long cap) {
  int np_ = prm->n_integ_points;
  orc_cand* cs = (orc_cand*)malloc(sizeof(orc_cand) * ((size_t)na * nb + 1));
  double* inner = (double*)malloc(sizeof(double) * (size_t)(np_ + 1));
  long k = 0;
  for (int ia = 0; ia < na; ++ia) {
    const double* A = cand_a + (size_t)ia * 4;
    for (int ib = 0; ib < nb; ++ib) {
      const double* B = cand_b + (size_t)ib * 4;
      double vx = B[0] - A[0], vy = B[1] - A[1];
      double norm = sqrt(vx * vx + vy * vy); /* integer coordinates: exact */
      if (norm == 0.0) continue;
      double ux = vx / norm, uy = vy / norm;
      int nvalid = 0;
      for (int i = 0; i < np_; ++i) {
        double ys = linspace_at(A[1], B[1], np_, i);
        double xs = linspace_at(A[0], B[0], np_, i);
        int yi = (int)nearbyint(ys); /* np.round: half to even */
        int xi = (int)nearbyint(xs);
        double px = (double)paf_x[(size_t)yi * W + xi];
        double py = (double)paf_y[(size_t)yi * W + xi];
        double ip = fma(px, ux, py * uy); /* np.dot((10,2) f64, (2,)) via OpenBLAS dgemv_t */
        inner[i] = ip;
        if (ip > prm->inner_product_thresh) ++nvalid;
      }
      double integ = np_pairwise_sum(inner, np_) / (double)np_;
      double pen = prm->limb_length_ratio * img_len / norm - prm->length_penalty_value;
      if (pen > 0.0) pen = 0.0; /* min(pen, 0) */
      double score = integ + pen;
      if (nvalid > prm->n_integ_points_thresh && score > 0.0) {
        cs[k].score = score;
        cs[k].idx = (long)ia * nb + ib;
        cs[k].a = (int32_t)A[3];
        cs[k].b = (int32_t)B[3];
        ++k;
      }
    }
  }
  (void)H;
  qsort(cs, (size_t)k, sizeof(orc_cand), cand_cmp);
  if (k > cap) { free(cs); free(inner); return -1; }
  for (long i = 0; i < k; ++i) {
    out[i * 3 + 0] = (double)cs[i].a;
    out[i * 3 + 1] = (double)cs[i].b;
    out[i * 3 + 2] = cs[i].score;
  }
  free(cs);
  free(inner);
  return k;
}

/* pose_detector.py:161-181.  pafs: (2*L, H, W).  peaks: (N,5).  limbs: L pairs.
 * conn_out: rows [id_a, id_b, score], limb l's rows start at conn_off[l], conn_off[L] = total. */
int orc_connections(const float* pafs, int H, int W, const double* peaks, long N,
                    const int32_t* limbs, int L, double img_len, const orc_params* prm,
                    double* conn_out, long cap, long* conn_off) {
  long total = 0;
  for (int l = 0; l < L; ++l) {
    conn_off[l] = total;
    int ja = limbs[2 * l], jb = limbs[2 * l + 1];
    int na = 0, nb = 0;
    for (long i = 0; i < N; ++i) {
      if ((int)peaks[i * 5] == ja) ++na;
      if ((int)peaks[i * 5] == jb) ++nb;
    }
    if (na == 0 || nb == 0) continue;
    double* ca = (double*)malloc(sizeof(double) * 4 * (size_t)na);
    double* cb = (double*)malloc(sizeof(double) * 4 * (size_t)nb);
    int ka = 0, kb = 0;
    for (long i = 0; i < N; ++i) {
      if ((int)peaks[i * 5] == ja) { memcpy(ca + 4 * ka, peaks + i * 5 + 1, 4 * sizeof(double)); ++ka; }
      if ((int)peaks[i * 5] == jb) { memcpy(cb + 4 * kb, peaks + i * 5 + 1, 4 * sizeof(double)); ++kb; }
    }
    long kmax = (long)na * nb;
    double* cand = (double*)malloc(sizeof(double) * 3 * (size_t)(kmax + 1));
    long k = orc_candidate_connections(pafs + (size_t)(2 * l) * H * W, pafs + (size_t)(2 * l + 1) * H * W,
                                       H, W, ca, na, cb, nb, img_len, prm, cand, kmax);
    long lim = na < nb ? na : nb;
    long got = 0;
    for (long i = 0; i < k; ++i) {
      double ia = cand[i * 3], ib = cand[i * 3 + 1];
      int used = 0;
      for (long q = 0; q < got; ++q) {
        if (conn_out[(total + q) * 3] == ia || conn_out[(total + q) * 3 + 1] == ib) { used = 1; break; }
      }
      if (used) continue;
      if (total + got >= cap) { free(ca); free(cb); free(cand); return ORC_ERR_CAPACITY; }
      memcpy(conn_out + (total + got) * 3, cand + i * 3, 3 * sizeof(double));
      ++got;
      if (got >= lim) break;
    }
    total += got;
    free(ca); free(cb); free(cand);
  }
  conn_off[L] = total;
  return ORC_OK;
}

/* pose_detector.py:183-250.  Subset rows are 20 f64: 18 peak ids (-1 none), [18] score, [19] count.
 * Returns ORC_OK and *n_out kept rows in `subsets` (capacity cap rows, also used as workspace),
 * ORC_ERR_INDEX where the reference raises IndexError (a connection touching >= 3 subsets). */
int orc_grouping(const double* conn, const long* conn_off, const int32_t* limbs, int L,
                 const double* peaks, const orc_params* prm, double* subsets, long cap, long* n_out) {
  long S = 0;
  for (int l = 0; l < L; ++l) {
    int ja = limbs[2 * l], jb = limbs[2 * l + 1];
    for (long c = conn_off[l]; c < conn_off[l + 1]; ++c) {
      int ia = (int)conn[c * 3], ib = (int)conn[c * 3 + 1];
      double score = conn[c * 3 + 2];
      int found = 0;
      long fidx[2] = {-1, -1};
      for (long s = 0; s < S; ++s) {
        const double* row = subsets + s * 20;
        if (row[ja] == (double)ia || row[jb] == (double)ib) {
          if (found >= 2) return ORC_ERR_INDEX;
          fidx[found++] = s;
        }
      }
      if (found == 1) {
        double* f = subsets + fidx[0] * 20;
        if (f[jb] != (double)ib) {
          f[jb] = (double)ib;
          f[19] += 1.0;
          f[18] += peaks[(size_t)ib * 5 + 3] + score;
        }
      } else if (found == 2) {
        double* f1 = subsets + fidx[0] * 20;
        double* f2 = subsets + fidx[1] * 20;
        int overlap = 0;
        for (int j = 0; j < 18; ++j)
          if (f1[j] >= 0.0 && f2[j] >= 0.0) { overlap = 1; break; }
        if (!overlap) {
          for (int j = 0; j < 18; ++j) f1[j] += f2[j] + 1.0;
          f1[18] += f2[18];
          f1[19] += f2[19];
          f1[18] += score;
          f1[19] += score;
          memmove(subsets + fidx[1] * 20, subsets + (fidx[1] + 1) * 20, sizeof(double) * 20 * (size_t)(S - fidx[1] - 1));
          --S;
        } else {
          double* fs[2] = {f1, f2};
          for (int q = 0; q < 2; ++q) {
            double* f = fs[q];
            if (f[ja] == -1.0) {
              f[ja] = (double)ia;
              f[19] += 1.0;
              f[18] += peaks[(size_t)ia * 5 + 3] + score;
            } else if (f[jb] == -1.0) {
              f[jb] = (double)ib;
              f[19] += 1.0;
              f[18] += peaks[(size_t)ib * 5 + 3] + score;
            }
          }
        }
      } else if (found == 0 && l != 9 && l != 13) {
        if (S >= cap) return ORC_ERR_CAPACITY;
        double* row = subsets + S * 20;
        for (int j = 0; j < 20; ++j) row[j] = -1.0;
        row[ja] = (double)ia;
        row[jb] = (double)ib;
        row[19] = 2.0;
        row[18] = (peaks[(size_t)ia * 5 + 3] + peaks[(size_t)ib * 5 + 3]) + score;
        ++S;
      }
    }
  }
  long k = 0;
  for (long s = 0; s < S; ++s) {
    const double* row = subsets + s * 20;
    if (row[19] >= (double)prm->n_subset_limbs_thresh && row[18] / row[19] >= prm->subset_score_thresh) {
      if (k != s) memmove(subsets + k * 20, row, sizeof(double) * 20);
      ++k;
    }
  }
  *n_out = k;
  return ORC_OK;
}
