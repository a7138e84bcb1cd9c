// One CocoPoseNet training iteration on the device: Updater.update_core of
// train_coco_pose_estimation.py:93-123 — forward keeping every stage's maps, compute_loss
// (:42-77: per-stage masked MSE on PAFs and heat maps), backward, GradientScaling(1/4) on the VGG +
// CPM layers (:24-38, :218-222), frozen VGG layers (:225-230, enabled again by the caller), and
// Chainer's Adam (:214) — in exact f32 (the v_mfma_f32_32x32x2_f32 conv kernel of conv.hip for the
// forward and the input gradients; CDNA VALU f32 for the weight gradients).
//
// Layout: every tensor is NHWC f32 with a 3-pixel zero halo (so any conv reads any buffer), one
// buffer per layer output (the backward needs them all) and a same-shaped gradient buffer.  The
// stage inputs concat((paf, heat, feature)) (CocoPoseNet.py:168) are one 192-channel buffer per
// stage in the inference layout (feature 0..127, heat 128..146, paf 152..189): stage s-1's Mconv7
// writes its maps straight into stage s's buffer, conv4_4_CPM's feature is copied into stages 3-6.
//   input gradient  dX = conv(dY_pre, W') with W'[ci][co][K-1-ky][K-1-kx] (same padding);
//   weight gradient dW[co][ci][ky][kx] = sum_p dY_pre[p][co] * X[p + (ky-R, kx-R)][ci] (split over
//     pixel ranges, partials reduced in a fixed order: deterministic);
//   ReLU: dY_pre = dY * (Y > 0); max-pool: the gradient goes to the window's first maximum
//     (MaxPooling2D.backward: argmax over the window in (ky, kx) order).
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "common.hpp"

namespace op {
namespace {

constexpr int kPad = 3;
constexpr int kNL = 92;

struct TLayer {
  std::string name;
  int ci, co, k;
};

std::vector<TLayer> train_layers() {  // models/CocoPoseNet.py:26-129 order
  std::vector<TLayer> v = {{"conv1_1", 3, 64, 3},     {"conv1_2", 64, 64, 3},     {"conv2_1", 64, 128, 3},
                           {"conv2_2", 128, 128, 3},  {"conv3_1", 128, 256, 3},   {"conv3_2", 256, 256, 3},
                           {"conv3_3", 256, 256, 3},  {"conv3_4", 256, 256, 3},   {"conv4_1", 256, 512, 3},
                           {"conv4_2", 512, 512, 3},  {"conv4_3_CPM", 512, 256, 3}, {"conv4_4_CPM", 256, 128, 3}};
  const char* br[2] = {"L1", "L2"};
  const int out[2] = {38, 19};
  for (int b = 0; b < 2; ++b) {
    for (int i = 1; i <= 3; ++i) v.push_back({"conv5_" + std::to_string(i) + "_CPM_" + br[b], 128, 128, 3});
    v.push_back({std::string("conv5_4_CPM_") + br[b], 128, 512, 1});
    v.push_back({std::string("conv5_5_CPM_") + br[b], 512, out[b], 1});
  }
  for (int s = 2; s <= 6; ++s)
    for (int b = 0; b < 2; ++b) {
      const std::string sfx = "_stage" + std::to_string(s) + "_" + br[b];
      v.push_back({"Mconv1" + sfx, 185, 128, 7});
      for (int i = 2; i <= 5; ++i) v.push_back({"Mconv" + std::to_string(i) + sfx, 128, 128, 7});
      v.push_back({"Mconv6" + sfx, 128, 128, 1});
      v.push_back({"Mconv7" + sfx, 128, out[b], 1});
    }
  return v;
}

// buffers
enum {
  T_X0, T_C11, T_C12, T_P1, T_C21, T_C22, T_P2, T_C31, T_C32, T_C33, T_C34, T_P3, T_C41, T_C42, T_C43,
  T_CAT0,                 // 5 stage inputs: T_CAT0 + (s - 2), s = 2..6
  T_S1 = T_CAT0 + 5,      // stage 1: per branch conv5_1..conv5_4 outputs (4 each)
  T_M = T_S1 + 8,         // stages 2-6: per (stage, branch) Mconv1..Mconv6 outputs (6 each)
  T_OUT6 = T_M + 60,      // stage 6 maps: paf 0..37, heat 40..58
  T_NB
};

struct TBuf {
  int div, cs;
};

struct TConv {
  int layer;
  int in, cin_off, cin_phys;  // input buffer, first channel, physical channels read (c8 * 8)
  int out, cout_off, store;   // output buffer, first channel, channels written
  bool relu, cat;             // cat: the input is a stage buffer (physical channel map)
};

}  // namespace

// ---- kernels ----
struct TView {  // NHWC f32 view: element (f, y, x, c) at p + ((f*(h+2pad) + y+pad)*(w+2pad) + x+pad)*cs + c
  float* p;
  int h, w, pad, cs;
  __device__ __forceinline__ int64_t at(int f, int y, int x) const {
    return (((int64_t)f * (h + 2 * pad) + y + pad) * (w + 2 * pad) + x + pad) * cs;
  }
};

// network input (n, 3, h, w) f32 -> X (NHWC, 8 channels, channels 3..7 zero)
__global__ __launch_bounds__(256) void tr_input(const float* __restrict__ x, TView X, int n) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t hw = (int64_t)X.h * X.w;
  if (i >= (int64_t)n * 3 * hw) return;
  const int xx = (int)(i % X.w);
  const int y = (int)((i / X.w) % X.h);
  const int c = (int)((i / hw) % 3);
  const int f = (int)(i / (hw * 3));
  X.p[X.at(f, y, xx) + c] = x[i];
}

// g[.., 0:C] *= (y > 0)
__global__ __launch_bounds__(256) void tr_relu_bwd(TView g, TView y, int n, int C) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t total = (int64_t)n * g.h * g.w * C;
  if (i >= total) return;
  const int c = (int)(i % C);
  int64_t p = i / C;
  const int x = (int)(p % g.w);
  p /= g.w;
  const int yy = (int)(p % g.h);
  const int f = (int)(p / g.h);
  if (!(y.p[y.at(f, yy, x) + c] > 0.0f)) g.p[g.at(f, yy, x) + c] = 0.0f;
}

// dst[.., doff + c] += src[.., soff + c], c < C
__global__ __launch_bounds__(256) void tr_add(TView dst, int doff, TView src, int soff, int n, int C) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t total = (int64_t)n * dst.h * dst.w * C;
  if (i >= total) return;
  const int c = (int)(i % C);
  int64_t p = i / C;
  const int x = (int)(p % dst.w);
  p /= dst.w;
  const int yy = (int)(p % dst.h);
  const int f = (int)(p / dst.h);
  dst.p[dst.at(f, yy, x) + doff + c] += src.p[src.at(f, yy, x) + soff + c];
}

// dst[.., doff + c] = src[.., soff + c] (the feature copy into the later stage buffers)
__global__ __launch_bounds__(256) void tr_copy(TView dst, int doff, TView src, int soff, int n, int C) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t total = (int64_t)n * dst.h * dst.w * C;
  if (i >= total) return;
  const int c = (int)(i % C);
  int64_t p = i / C;
  const int x = (int)(p % dst.w);
  p /= dst.w;
  const int yy = (int)(p % dst.h);
  const int f = (int)(p / dst.h);
  dst.p[dst.at(f, yy, x) + doff + c] = src.p[src.at(f, yy, x) + soff + c];
}

// max-pool 2x2 backward: dX (zeroed) at the first maximum of each window of X gets dP
__global__ __launch_bounds__(256) void tr_pool_bwd(TView dP, TView X, TView dX, int n, int C) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t total = (int64_t)n * dP.h * dP.w * C;
  if (i >= total) return;
  const int c = (int)(i % C);
  int64_t p = i / C;
  const int ox = (int)(p % dP.w);
  p /= dP.w;
  const int oy = (int)(p % dP.h);
  const int f = (int)(p / dP.h);
  int best = 0;
  float bv = X.p[X.at(f, 2 * oy, 2 * ox) + c];
  for (int k = 1; k < 4; ++k) {
    const float v = X.p[X.at(f, 2 * oy + (k >> 1), 2 * ox + (k & 1)) + c];
    if (v > bv) {
      bv = v;
      best = k;
    }
  }
  dX.p[dX.at(f, 2 * oy + (best >> 1), 2 * ox + (best & 1)) + c] = dP.p[dP.at(f, oy, ox) + c];
}

// compute_loss for one map tensor: y = slice [yoff, yoff + C) of buffer Y, t (n, C, h, w) planar,
// ignore (n, h, w) u8.  t' = ignore ? y : t; partial sums of (y - t')^2 per block (f64) and
// dY[slice] += 2 (y - t') / numel.
__global__ __launch_bounds__(256) void tr_loss(TView Y, int yoff, TView dY, const float* __restrict__ t,
                                               const uint8_t* __restrict__ ign, int n, int C, float inv_numel2,
                                               double* __restrict__ part) {
  __shared__ double red[256];
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t hw = (int64_t)Y.h * Y.w;
  const int64_t total = (int64_t)n * C * hw;
  double sq = 0.0;
  if (i < total) {
    const int x = (int)(i % Y.w);
    const int yy = (int)((i / Y.w) % Y.h);
    const int c = (int)((i / hw) % C);
    const int f = (int)(i / (hw * C));
    const float yv = Y.p[Y.at(f, yy, x) + yoff + c];
    const float d = ign[(int64_t)f * hw + (int64_t)yy * Y.w + x] ? 0.0f : yv - t[i];
    sq = (double)d * (double)d;
    dY.p[dY.at(f, yy, x) + yoff + c] += d * inv_numel2;
  }
  red[threadIdx.x] = sq;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

// weight gradient partials: workgroup = 64 co x 64 ci of one tap over the pixel range of split z;
// thread = 4 co x 4 ci; 16-pixel steps staged in LDS.  part[z][tap][co][ci] (co, ci < cop, cip).
// The centre tap's first ci block also sums the staged G rows: bias partials bpart[z][co].
constexpr int kWgPx = 16;
__global__ __launch_bounds__(256) void tr_wgrad(TView G, int gch, TView X, int n, int cop, int cip, int ks,
                                                int px_per_split, float* __restrict__ part,
                                                float* __restrict__ bpart) {
  __shared__ float sg[kWgPx][64];
  __shared__ float sx[kWgPx][64];
  const int co0 = blockIdx.x * 64;
  const int taps = ks * ks;
  const int tap = blockIdx.y % taps, ci0 = (blockIdx.y / taps) * 64;
  const int z = blockIdx.z;
  const int R = ks / 2, dy = tap / ks - R, dx = tap % ks - R;
  const int hw = G.h * G.w, total = n * hw;
  const int p0 = z * px_per_split, p1 = min(p0 + px_per_split, total);
  const int tid = threadIdx.x;
  const int tco = (tid & 15) * 4, tci = (tid >> 4) * 4;
  const bool bwg = tap == taps / 2 && ci0 == 0;  // workgroup-uniform: this one also sums the bias
  float acc[4][4] = {};
  float bacc = 0.0f;  // bwg, threads 0..63: channel co0 + tid
  for (int pb = p0; pb < p1; pb += kWgPx) {
    // stage 16 px x 64 channels of G and of the shifted X (one float4 per thread each)
    {
      const int pp = tid >> 4, c4 = (tid & 15) * 4;
      const int p = pb + pp;
      floatx4 gv = {0.f, 0.f, 0.f, 0.f}, xv = {0.f, 0.f, 0.f, 0.f};
      if (p < p1) {
        const int f = p / hw, r = p - f * hw, y = r / G.w, x = r - y * G.w;
        if (co0 + c4 < gch) gv = *(const floatx4*)(G.p + G.at(f, y, x) + co0 + c4);  // stored channels only
        if (ci0 + c4 < cip) xv = *(const floatx4*)(X.p + X.at(f, y + dy, x + dx) + ci0 + c4);
      }
      *(floatx4*)&sg[pp][c4] = gv;
      *(floatx4*)&sx[pp][c4] = xv;
    }
    __syncthreads();
#pragma unroll 4
    for (int k = 0; k < kWgPx; ++k) {
      const floatx4 a = *(const floatx4*)&sg[k][tco];
      const floatx4 b = *(const floatx4*)&sx[k][tci];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __fmaf_rn(a[i], b[j], acc[i][j]);
    }
    if (bwg && tid < 64)
#pragma unroll
      for (int k = 0; k < kWgPx; ++k) bacc += sg[k][tid];
    __syncthreads();
  }
  if (bwg && tid < 64 && co0 + tid < cop) bpart[(int64_t)z * cop + co0 + tid] = bacc;
  float* o = part + ((int64_t)z * taps + tap) * (int64_t)cop * cip;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (co0 + tco + i < cop && ci0 + tci + j < cip) o[(int64_t)(co0 + tco + i) * cip + ci0 + tci + j] = acc[i][j];
}

// gW[co][ci_log][tap] = sum_z part[z][tap][co][ci_phys] (fixed order); cat: physical -> logical
__global__ __launch_bounds__(256) void tr_wreduce(const float* __restrict__ part, int splits, int taps, int cop, int cip,
                                                  int Co, int Ci, int cat, float* __restrict__ gW) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t total = (int64_t)taps * cop * cip;
  if (i >= total) return;
  const int pci = (int)(i % cip);
  const int co = (int)((i / cip) % cop);
  const int tap = (int)(i / ((int64_t)cip * cop));
  if (co >= Co) return;
  int ci = pci;
  if (cat) {
    if (pci >= kCatFeat && pci < kCatFeat + 128) ci = 57 + (pci - kCatFeat);
    else if (pci >= kCatHeat && pci < kCatHeat + 19) ci = 38 + (pci - kCatHeat);
    else if (pci >= kCatPaf && pci < kCatPaf + 38) ci = pci - kCatPaf;
    else return;
  }
  if (ci >= Ci) return;
  float s = 0.0f;
  for (int z = 0; z < splits; ++z) s += part[((int64_t)z * taps + tap) * (int64_t)cop * cip + (int64_t)co * cip + pci];
  gW[((int64_t)co * Ci + ci) * taps + tap] = s;
}

__global__ __launch_bounds__(256) void tr_breduce(const float* __restrict__ part, int splits, int cop, int Co,
                                                  float* __restrict__ gb) {
  const int co = blockIdx.x * 256 + threadIdx.x;
  if (co >= Co) return;
  float s = 0.0f;
  for (int z = 0; z < splits; ++z) s += part[(int64_t)z * cop + co];
  gb[co] = s;
}

// Chainer AdamRule.update_core (eta 1, no weight decay): grad *= scale (GradientScaling hook);
// m += (1 - b1)(g - m); v += (1 - b2)(g^2 - v); p -= lr * m / (sqrt(v) + eps)
__global__ __launch_bounds__(256) void tr_adam(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                                               float* __restrict__ v, int64_t n, float scale, float lr, float b1,
                                               float b2, float eps) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const float gr = g[i] * scale;
  const float mm = m[i] + (1.0f - b1) * (gr - m[i]);
  const float vv = v[i] + (1.0f - b2) * (gr * gr - v[i]);
  m[i] = mm;
  v[i] = vv;
  p[i] -= lr * mm / (sqrtf(vv) + eps);
}

// forward packing [c8][tap][cop][8] (input channel = physical p, cat map) and input-gradient packing
// (input channel = forward output co, output channel = forward physical input p, taps flipped)
__global__ __launch_bounds__(256) void tr_pack(const float* __restrict__ W, int Co, int Ci, int ks, int cin_phys, int cop,
                                               int cat, int dgrad, float* __restrict__ dst) {
  const int taps = ks * ks;
  const int in_ch = dgrad ? (Co + 7) / 8 * 8 : cin_phys;  // packed input channels
  const int64_t total = (int64_t)in_ch * taps * cop;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int j = (int)(i % 8);
  const int oc = (int)((i / 8) % cop);
  const int tap = (int)((i / (8 * (int64_t)cop)) % taps);
  const int c8 = (int)(i / (8 * (int64_t)cop * taps));
  const int ic = c8 * 8 + j;
  int co, p, t;
  if (dgrad) {
    co = ic;
    p = oc;
    t = taps - 1 - tap;
  } else {
    co = oc;
    p = ic;
    t = tap;
  }
  int ci = p;
  if (cat) {
    if (p >= kCatFeat && p < kCatFeat + 128) ci = 57 + (p - kCatFeat);
    else if (p >= kCatHeat && p < kCatHeat + 19) ci = 38 + (p - kCatHeat);
    else if (p >= kCatPaf && p < kCatPaf + 38) ci = p - kCatPaf;
    else ci = -1;
  }
  float v = 0.0f;
  if (co < Co && ci >= 0 && ci < Ci) v = W[((int64_t)co * Ci + ci) * taps + t];
  dst[i] = v;
}

}  // namespace op

using namespace op;

struct op_train_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  int n = 0, h = 0, w = 0;
  std::vector<TLayer> L;
  std::vector<TConv> convs;
  TBuf bdef[T_NB];
  TView act[T_NB], grad[T_NB];
  void* arena = nullptr;
  size_t arena_bytes = 0, grad_off = 0;
  // per layer: master W, b; grads; Adam state; packed forward / input-gradient weights
  float *W[kNL] = {}, *b[kNL] = {}, *gW[kNL] = {}, *gb[kNL] = {}, *mW[kNL] = {}, *vW[kNL] = {}, *mb[kNL] = {},
        *vb[kNL] = {}, *pf[kNL] = {}, *pd[kNL] = {}, *bpad[kNL] = {};
  int cop[kNL] = {}, cin_phys[kNL] = {}, dcop[kNL] = {};
  bool enabled[kNL] = {};
  int64_t t_step[kNL] = {};
  float scale[kNL] = {};
  float *zeros = nullptr, *tmp = nullptr, *part = nullptr;
  size_t tmp_floats = 0, part_floats = 0;
  double* lpart = nullptr;
  size_t lpart_n = 0;
  float *d_t = nullptr;
  uint8_t* d_ign = nullptr;
  float* d_x = nullptr;
  double alpha = 1e-4, beta1 = 0.9, beta2 = 0.999, eps = 1e-8;
  bool have_weights = false;
};

namespace op {
namespace {

int tr_check(op_train_ctx* c) {
  if (!c) {
    set_error("null op_train_ctx");
    return OP_ERR_INVALID;
  }
  OP_HIP_CHECK(hipSetDevice(c->device));
  return OP_OK;
}

#define TRC(x)           \
  do {                   \
    int _r = (x);        \
    if (_r) return _r;   \
  } while (0)

inline unsigned nb(int64_t n) { return (unsigned)((n + 255) / 256); }

void build_graph(op_train_ctx* c) {
  TBuf* B = c->bdef;
  auto setb = [&](int i, int div, int cs) { B[i] = TBuf{div, cs}; };
  setb(T_X0, 1, 8);
  setb(T_C11, 1, 64);
  setb(T_C12, 1, 64);
  setb(T_P1, 2, 64);
  setb(T_C21, 2, 128);
  setb(T_C22, 2, 128);
  setb(T_P2, 4, 128);
  for (int i = T_C31; i <= T_C34; ++i) setb(i, 4, 256);
  setb(T_P3, 8, 256);
  setb(T_C41, 8, 512);
  setb(T_C42, 8, 512);
  setb(T_C43, 8, 256);
  for (int s = 0; s < 5; ++s) setb(T_CAT0 + s, 8, kCatStride);
  for (int b = 0; b < 2; ++b)
    for (int i = 0; i < 4; ++i) setb(T_S1 + 4 * b + i, 8, i == 3 ? 512 : 128);
  for (int i = 0; i < 60; ++i) setb(T_M + i, 8, 128);
  setb(T_OUT6, 8, 64);
  auto conv = [&](int layer, int in, int cin_off, int out, int cout_off, int store, bool relu, bool cat = false) {
    const int ci = c->L[layer].ci;
    const int cin_phys = cat ? kCatStride : (ci + 7) / 8 * 8;
    c->convs.push_back(TConv{layer, in, cin_off, cin_phys, out, cout_off, store, relu, cat});
  };
  conv(0, T_X0, 0, T_C11, 0, 64, true);
  conv(1, T_C11, 0, T_C12, 0, 64, true);
  conv(2, T_P1, 0, T_C21, 0, 128, true);
  conv(3, T_C21, 0, T_C22, 0, 128, true);
  conv(4, T_P2, 0, T_C31, 0, 256, true);
  conv(5, T_C31, 0, T_C32, 0, 256, true);
  conv(6, T_C32, 0, T_C33, 0, 256, true);
  conv(7, T_C33, 0, T_C34, 0, 256, true);
  conv(8, T_P3, 0, T_C41, 0, 512, true);
  conv(9, T_C41, 0, T_C42, 0, 512, true);
  conv(10, T_C42, 0, T_C43, 0, 256, true);
  conv(11, T_C43, 0, T_CAT0, kCatFeat, 128, true);
  for (int b = 0; b < 2; ++b) {  // stage 1 (layers 12 + 5b ..)
    const int l0 = 12 + 5 * b, s1 = T_S1 + 4 * b;
    conv(l0, T_CAT0, kCatFeat, s1, 0, 128, true);
    conv(l0 + 1, s1, 0, s1 + 1, 0, 128, true);
    conv(l0 + 2, s1 + 1, 0, s1 + 2, 0, 128, true);
    conv(l0 + 3, s1 + 2, 0, s1 + 3, 0, 512, true);
    conv(l0 + 4, s1 + 3, 0, T_CAT0, b == 0 ? kCatPaf : kCatHeat, b == 0 ? 40 : 20, false);
  }
  for (int s = 0; s < 5; ++s)
    for (int b = 0; b < 2; ++b) {
      const int l0 = 22 + 14 * s + 7 * b, m = T_M + 12 * s + 6 * b;
      conv(l0, T_CAT0 + s, 0, m, 0, 128, true, true);
      for (int i = 1; i <= 4; ++i) conv(l0 + i, m + i - 1, 0, m + i, 0, 128, true);
      conv(l0 + 5, m + 4, 0, m + 5, 0, 128, true);
      const int dst = s == 4 ? T_OUT6 : T_CAT0 + s + 1;
      const int off = s == 4 ? (b == 0 ? 0 : 40) : (b == 0 ? kCatPaf : kCatHeat);
      conv(l0 + 6, m + 5, 0, dst, off, b == 0 ? 40 : 20, false);
    }
}

int tr_geometry(op_train_ctx* c) {
  size_t fl = 0;
  for (int i = 0; i < T_NB; ++i) {
    const int hh = c->h / c->bdef[i].div, ww = c->w / c->bdef[i].div;
    fl += ((size_t)c->n * (hh + 2 * kPad) * (ww + 2 * kPad) * c->bdef[i].cs + 63) / 64 * 64;
  }
  const size_t bytes = 2 * fl * sizeof(float);
  OP_HIP_CHECK(hipMalloc(&c->arena, bytes));
  c->arena_bytes = bytes;
  OP_HIP_CHECK(hipMemset(c->arena, 0, bytes));
  float* p = (float*)c->arena;
  for (int g = 0; g < 2; ++g)
    for (int i = 0; i < T_NB; ++i) {
      TView v;
      v.h = c->h / c->bdef[i].div;
      v.w = c->w / c->bdef[i].div;
      v.pad = kPad;
      v.cs = c->bdef[i].cs;
      v.p = p;
      p += ((size_t)c->n * (v.h + 2 * kPad) * (v.w + 2 * kPad) * v.cs + 63) / 64 * 64;
      (g == 0 ? c->act : c->grad)[i] = v;
    }
  c->grad_off = fl;
  // scratch: input-gradient temp (largest conv input) and weight-gradient partials
  size_t tmax = 0;
  for (const auto& cv : c->convs) {
    const TView& in = c->act[cv.in];
    tmax = std::max(tmax, (size_t)c->n * (in.h + 2 * kPad) * (in.w + 2 * kPad) * ((cv.cin_phys + 63) / 64 * 64));
  }
  c->tmp_floats = tmax;
  OP_HIP_CHECK(hipMalloc(&c->tmp, tmax * sizeof(float)));
  OP_HIP_CHECK(hipMemset(c->tmp, 0, tmax * sizeof(float)));
  return OP_OK;
}

ConvShape tshape(int n, const TView& in, const TView& out, int c8, int ks, bool relu) {
  ConvShape s;
  s.n = n;
  s.h = out.h;
  s.w = out.w;
  s.pin = in.pad;
  s.cs_in = in.cs;
  s.pout = out.pad;
  s.cs_out = out.cs;
  s.c8 = c8;
  s.ks = ks;
  s.relu = relu ? 1 : 0;
  s.groups = 1;
  return s;
}

int tr_pack_layer(op_train_ctx* c, int l, const TConv& cv) {
  const TLayer& d = c->L[l];
  const int taps = d.k * d.k;
  int64_t tot = (int64_t)cv.cin_phys * taps * c->cop[l];
  hipLaunchKernelGGL(tr_pack, dim3(nb(tot)), dim3(256), 0, c->stream, c->W[l], d.co, d.ci, d.k, cv.cin_phys, c->cop[l],
                     cv.cat ? 1 : 0, 0, c->pf[l]);
  if (c->pd[l]) {
    tot = (int64_t)((d.co + 7) / 8 * 8) * taps * c->dcop[l];
    hipLaunchKernelGGL(tr_pack, dim3(nb(tot)), dim3(256), 0, c->stream, c->W[l], d.co, d.ci, d.k, cv.cin_phys,
                       c->dcop[l], cv.cat ? 1 : 0, 1, c->pd[l]);
  }
  OP_HIP_CHECK(hipMemcpyAsync(c->bpad[l], c->b[l], d.co * sizeof(float), hipMemcpyDeviceToDevice, c->stream));
  OP_AFTER_LAUNCH("tr_pack", c->stream);
  OP_HIP_CHECK(hipGetLastError());
  return OP_OK;
}

int tr_forward(op_train_ctx* c) {
  for (size_t k = 0; k < c->convs.size(); ++k) {
    const TConv& cv = c->convs[k];
    const int l = cv.layer;
    const TView& in = c->act[cv.in];
    const TView& out = c->act[cv.out];
    ConvGroup g[2];
    g[0].in = in.p + cv.cin_off;
    g[0].out = out.p + cv.cout_off;
    g[0].w = c->pf[l];
    g[0].bias = c->bpad[l];
    g[0].cop = c->cop[l];
    g[0].cout_store = cv.store;
    g[1] = g[0];
    TRC(launch_conv(tshape(c->n, in, out, cv.cin_phys / 8, c->L[l].k, cv.relu), g, c->stream));
    // pools after conv1_2, conv2_2, conv3_4; the feature copy after conv4_4_CPM
    const int pool_in = l == 1 ? T_C12 : (l == 3 ? T_C22 : (l == 7 ? T_C34 : -1));
    if (pool_in >= 0) {
      const int pool_out = l == 1 ? T_P1 : (l == 3 ? T_P2 : T_P3);
      const TView& a = c->act[pool_in];
      const TView& o = c->act[pool_out];
      TRC(launch_maxpool2(a.p, a.pad, o.p, o.pad, c->n, a.h, a.w, a.cs, c->stream));
    }
    if (l == 11)
      for (int s = 1; s < 5; ++s) {
        const TView& d = c->act[T_CAT0 + s];
        hipLaunchKernelGGL(tr_copy, dim3(nb((int64_t)c->n * d.h * d.w * 128)), dim3(256), 0, c->stream, d, kCatFeat,
                           c->act[T_CAT0], kCatFeat, c->n, 128);
      }
  }
  OP_HIP_CHECK(hipGetLastError());
  return OP_OK;
}

// the 12 map tensors of compute_loss: (buffer, channel offset, C, paf?) per stage
struct MapT {
  int buf, off, C;
};
MapT stage_map(int s, int paf) {  // s = 1..6
  if (s == 6) return MapT{T_OUT6, paf ? 0 : 40, paf ? 38 : 19};
  return MapT{T_CAT0 + s - 1, paf ? kCatPaf : kCatHeat, paf ? 38 : 19};
}

int tr_backward(op_train_ctx* c, int lowest) {
  const int n = c->n;
  // layer -> conv index; the backward visits convs in reverse order
  for (int k = (int)c->convs.size() - 1; k >= 0; --k) {
    const TConv& cv = c->convs[k];
    const int l = cv.layer;
    if (l < lowest) break;
    const TLayer& d = c->L[l];
    TView gout = c->grad[cv.out];
    const TView& yout = c->act[cv.out];
    // the feature copy: stage 3-6 feature gradients flow into stage 2's buffer
    if (l == 11)
      for (int s = 1; s < 5; ++s) {
        const TView& g = c->grad[T_CAT0 + s];
        hipLaunchKernelGGL(tr_add, dim3(nb((int64_t)n * g.h * g.w * 128)), dim3(256), 0, c->stream, c->grad[T_CAT0],
                           kCatFeat, g, kCatFeat, n, 128);
      }
    // pools: the pooled gradient routes into the conv output gradient
    const int pool_in = l == 1 ? T_C12 : (l == 3 ? T_C22 : (l == 7 ? T_C34 : -1));
    if (pool_in >= 0) {
      const int pool_out = l == 1 ? T_P1 : (l == 3 ? T_P2 : T_P3);
      const TView& gp = c->grad[pool_out];
      hipLaunchKernelGGL(tr_pool_bwd, dim3(nb((int64_t)n * gp.h * gp.w * c->act[pool_in].cs)), dim3(256), 0,
                         c->stream, gp, c->act[pool_in], c->grad[pool_in], n, c->act[pool_in].cs);
    }
    // ReLU on this conv's output slice
    TView gs = gout, ys = yout;
    gs.p += cv.cout_off;
    ys.p += cv.cout_off;
    if (cv.relu)
      hipLaunchKernelGGL(tr_relu_bwd, dim3(nb((int64_t)n * gs.h * gs.w * cv.store)), dim3(256), 0, c->stream, gs, ys,
                         n, cv.store);
    const TView& xin = c->act[cv.in];
    const int taps = d.k * d.k;
    const int total = n * gs.h * gs.w;
    if (c->enabled[l]) {  // weight / bias gradients
      const int cop = c->cop[l], cip = cv.cin_phys;
      const int splits = std::max(1, std::min(64, total / 512));
      const int pps = ((total + splits - 1) / splits + kWgPx - 1) / kWgPx * kWgPx;
      const size_t need = (size_t)splits * taps * cop * cip + (size_t)splits * cop;  // + bias partials
      if (need > c->part_floats) {
        OP_HIP_CHECK(hipStreamSynchronize(c->stream));
        if (c->part) OP_HIP_CHECK(hipFree(c->part));
        OP_HIP_CHECK(hipMalloc(&c->part, need * sizeof(float)));
        c->part_floats = need;
      }
      TView xv = xin;
      xv.p += cv.cin_off;
      const dim3 grid((unsigned)((cop + 63) / 64), (unsigned)(taps * ((cip + 63) / 64)), (unsigned)splits);
      // (a v_mfma_f32_32x32x2_f32 version with operands straight from L2 measured slower: 154 vs
      // 144 ms per batch-10 iteration)
      float* bpart = c->part + (size_t)splits * taps * cop * cip;
      hipLaunchKernelGGL(tr_wgrad, grid, dim3(256), 0, c->stream, gs, cv.store, xv, n, cop, cip, d.k, pps, c->part,
                         bpart);
      hipLaunchKernelGGL(tr_wreduce, dim3(nb((int64_t)taps * cop * cip)), dim3(256), 0, c->stream, c->part, splits,
                         taps, cop, cip, d.co, d.ci, cv.cat ? 1 : 0, c->gW[l]);
      hipLaunchKernelGGL(tr_breduce, dim3(nb(d.co)), dim3(256), 0, c->stream, bpart, splits, cop, d.co, c->gb[l]);
    }
    if (l > lowest && l > 0) {  // input gradient: temp = conv(dY_pre, W'), then added to the input's gradient
      TView tv = xin;
      tv.cs = c->dcop[l];
      tv.p = c->tmp;
      ConvGroup g[2];
      g[0].in = gs.p;
      g[0].out = tv.p;
      g[0].w = c->pd[l];
      g[0].bias = c->zeros;
      g[0].cop = c->dcop[l];
      g[0].cout_store = cv.cin_phys;
      g[1] = g[0];
      TView gin = gs;
      gin.cs = gout.cs;
      TRC(launch_conv(tshape(n, gin, tv, (d.co + 7) / 8, d.k, false), g, c->stream));
      const TView& gx = c->grad[cv.in];
      hipLaunchKernelGGL(tr_add, dim3(nb((int64_t)n * gx.h * gx.w * cv.cin_phys)), dim3(256), 0, c->stream, gx,
                         cv.cin_off, tv, 0, n, cv.cin_phys);
    }
  }
  OP_AFTER_LAUNCH("tr_backward", c->stream);
  OP_HIP_CHECK(hipGetLastError());
  return OP_OK;
}

}  // namespace
}  // namespace op

extern "C" {

int op_train_create(int32_t device, int32_t n, int32_t h, int32_t w, op_train_ctx** out) {
  if (!out || n < 1 || h < 16 || w < 16 || h % 8 || w % 8) {
    set_error("op_train_create: bad arguments (n >= 1, h and w multiples of 8, >= 16)");
    return OP_ERR_INVALID;
  }
  *out = nullptr;
  int ndev = 0;
  OP_HIP_CHECK(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) {
    set_error("op_train_create: no HIP device " + std::to_string(device));
    return OP_ERR_INVALID;
  }
  OP_HIP_CHECK(hipSetDevice(device));
  op_train_ctx* c = new op_train_ctx();
  c->device = device;
  c->n = n;
  c->h = h;
  c->w = w;
  c->L = train_layers();
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    set_error("op_train_create: stream");
    return OP_ERR_HIP;
  }
  build_graph(c);
  int rc = tr_geometry(c);
  if (rc) {
    op_train_destroy(c);
    return rc;
  }
  for (const auto& cv : c->convs) {
    const int l = cv.layer;
    const TLayer& d = c->L[l];
    const size_t nw = (size_t)d.co * d.ci * d.k * d.k;
    c->cop[l] = (d.co + 63) / 64 * 64;
    c->cin_phys[l] = cv.cin_phys;
    c->dcop[l] = (cv.cin_phys + 63) / 64 * 64;
    c->scale[l] = 1.0f;  // no hook until op_train_set_grad_scale (the reference's GradientScaling)
    c->enabled[l] = true;
    float** arrs[] = {&c->W[l], &c->gW[l], &c->mW[l], &c->vW[l]};
    for (float** a : arrs) {
      if (hipMalloc(a, nw * sizeof(float)) != hipSuccess || hipMemset(*a, 0, nw * sizeof(float)) != hipSuccess) {
        op_train_destroy(c);
        set_error("op_train_create: out of device memory");
        return OP_ERR_HIP;
      }
    }
    float** barrs[] = {&c->b[l], &c->gb[l], &c->mb[l], &c->vb[l]};
    for (float** a : barrs) {
      if (hipMalloc(a, d.co * sizeof(float)) != hipSuccess || hipMemset(*a, 0, d.co * sizeof(float)) != hipSuccess) {
        op_train_destroy(c);
        set_error("op_train_create: out of device memory");
        return OP_ERR_HIP;
      }
    }
    const size_t pfn = (size_t)cv.cin_phys * d.k * d.k * c->cop[l];
    OP_HIP_CHECK(hipMalloc(&c->pf[l], pfn * sizeof(float)));
    if (l > 0) {
      const size_t pdn = (size_t)((d.co + 7) / 8 * 8) * d.k * d.k * c->dcop[l];
      OP_HIP_CHECK(hipMalloc(&c->pd[l], pdn * sizeof(float)));
    }
    OP_HIP_CHECK(hipMalloc(&c->bpad[l], c->cop[l] * sizeof(float)));
    OP_HIP_CHECK(hipMemset(c->bpad[l], 0, c->cop[l] * sizeof(float)));
  }
  OP_HIP_CHECK(hipMalloc(&c->zeros, 1024 * sizeof(float)));
  OP_HIP_CHECK(hipMemset(c->zeros, 0, 1024 * sizeof(float)));
  *out = c;
  return OP_OK;
}

int op_train_destroy(op_train_ctx* c) {
  if (!c) return OP_OK;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  for (int l = 0; l < kNL; ++l) {
    float* arrs[] = {c->W[l], c->b[l], c->gW[l], c->gb[l], c->mW[l], c->vW[l], c->mb[l], c->vb[l], c->pf[l], c->pd[l],
                     c->bpad[l]};
    for (float* a : arrs)
      if (a) (void)hipFree(a);
  }
  void* bufs[] = {c->arena, c->tmp, c->part, c->zeros, c->lpart, c->d_t, c->d_ign, c->d_x};
  for (void* a : bufs)
    if (a) (void)hipFree(a);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return OP_OK;
}

int op_train_set_weights(op_train_ctx* c, const float* const* W, const float* const* b) {
  TRC(tr_check(c));
  if (!W || !b) {
    set_error("null weights");
    return OP_ERR_INVALID;
  }
  for (int l = 0; l < kNL; ++l) {
    if (!W[l] || !b[l]) {
      set_error("missing weights for layer " + c->L[l].name);
      return OP_ERR_INVALID;
    }
    const TLayer& d = c->L[l];
    OP_HIP_CHECK(hipMemcpy(c->W[l], W[l], (size_t)d.co * d.ci * d.k * d.k * 4, hipMemcpyHostToDevice));
    OP_HIP_CHECK(hipMemcpy(c->b[l], b[l], (size_t)d.co * 4, hipMemcpyHostToDevice));
    OP_HIP_CHECK(hipMemset(c->mW[l], 0, (size_t)d.co * d.ci * d.k * d.k * 4));
    OP_HIP_CHECK(hipMemset(c->vW[l], 0, (size_t)d.co * d.ci * d.k * d.k * 4));
    OP_HIP_CHECK(hipMemset(c->mb[l], 0, (size_t)d.co * 4));
    OP_HIP_CHECK(hipMemset(c->vb[l], 0, (size_t)d.co * 4));
    c->t_step[l] = 0;
  }
  for (const auto& cv : c->convs) TRC(tr_pack_layer(c, cv.layer, cv));
  OP_HIP_CHECK(hipStreamSynchronize(c->stream));
  c->have_weights = true;
  return OP_OK;
}

int op_train_get_weights(op_train_ctx* c, float* const* W, float* const* b, float* const* gW, float* const* gb) {
  TRC(tr_check(c));
  OP_HIP_CHECK(hipStreamSynchronize(c->stream));
  for (int l = 0; l < kNL; ++l) {
    const TLayer& d = c->L[l];
    const size_t nw = (size_t)d.co * d.ci * d.k * d.k * 4;
    if (W && W[l]) OP_HIP_CHECK(hipMemcpy(W[l], c->W[l], nw, hipMemcpyDeviceToHost));
    if (b && b[l]) OP_HIP_CHECK(hipMemcpy(b[l], c->b[l], d.co * 4, hipMemcpyDeviceToHost));
    if (gW && gW[l]) OP_HIP_CHECK(hipMemcpy(gW[l], c->gW[l], nw, hipMemcpyDeviceToHost));
    if (gb && gb[l]) OP_HIP_CHECK(hipMemcpy(gb[l], c->gb[l], d.co * 4, hipMemcpyDeviceToHost));
  }
  return OP_OK;
}

int op_train_set_hyper(op_train_ctx* c, double alpha, double beta1, double beta2, double eps) {
  TRC(tr_check(c));
  c->alpha = alpha;
  c->beta1 = beta1;
  c->beta2 = beta2;
  c->eps = eps;
  return OP_OK;
}

int op_train_enable_layer(op_train_ctx* c, int32_t layer, int32_t enable) {
  TRC(tr_check(c));
  if (layer < 0 || layer >= kNL) {
    set_error("op_train_enable_layer: bad layer");
    return OP_ERR_INVALID;
  }
  if (!enable && c->enabled[layer]) {  // a disabled layer reports zero gradients (steps no longer write them)
    const TLayer& d = c->L[layer];
    OP_HIP_CHECK(hipMemsetAsync(c->gW[layer], 0, (size_t)d.co * d.ci * d.k * d.k * 4, c->stream));
    OP_HIP_CHECK(hipMemsetAsync(c->gb[layer], 0, (size_t)d.co * 4, c->stream));
  }
  c->enabled[layer] = enable != 0;
  return OP_OK;
}

int op_train_set_grad_scale(op_train_ctx* c, int32_t layer, double scale) {
  TRC(tr_check(c));
  if (layer < 0 || layer >= kNL || !(scale == scale)) {
    set_error("op_train_set_grad_scale: bad layer or scale");
    return OP_ERR_INVALID;
  }
  c->scale[layer] = (float)scale;  // grad *= scale in f32 (train_coco_pose_estimation.py:38)
  return OP_OK;
}

int op_train_step(op_train_ctx* c, const float* x, const float* pafs_t, const float* heat_t, const uint8_t* ignore,
                  double* losses) {
  TRC(tr_check(c));
  if (!c->have_weights) {
    set_error("op_train_step: weights not set");
    return OP_ERR_STATE;
  }
  if (!x || !pafs_t || !heat_t || !ignore) {
    set_error("op_train_step: null pointer");
    return OP_ERR_INVALID;
  }
  const int n = c->n, h8 = c->h / 8, w8 = c->w / 8;
  const size_t xin = (size_t)n * 3 * c->h * c->w, tp = (size_t)n * 38 * h8 * w8, th = (size_t)n * 19 * h8 * w8,
               ig = (size_t)n * h8 * w8;
  if (!c->d_x) {
    OP_HIP_CHECK(hipMalloc(&c->d_x, xin * 4));
    OP_HIP_CHECK(hipMalloc(&c->d_t, (tp + th) * 4));
    OP_HIP_CHECK(hipMalloc(&c->d_ign, ig));
  }
  OP_HIP_CHECK(hipMemcpyAsync(c->d_x, x, xin * 4, hipMemcpyHostToDevice, c->stream));
  OP_HIP_CHECK(hipMemcpyAsync(c->d_t, pafs_t, tp * 4, hipMemcpyHostToDevice, c->stream));
  OP_HIP_CHECK(hipMemcpyAsync(c->d_t + tp, heat_t, th * 4, hipMemcpyHostToDevice, c->stream));
  OP_HIP_CHECK(hipMemcpyAsync(c->d_ign, ignore, ig, hipMemcpyHostToDevice, c->stream));
  // preprocess happens on the host side of the reference (:80-86): x is the network input
  hipLaunchKernelGGL(tr_input, dim3(nb((int64_t)xin)), dim3(256), 0, c->stream, c->d_x, c->act[T_X0], n);
  TRC(tr_forward(c));
  // gradients start at zero (halos too: the input-gradient convs read them)
  OP_HIP_CHECK(hipMemsetAsync((float*)c->arena + c->grad_off, 0, c->grad_off * 4, c->stream));
  // (no per-step gradient clearing: every enabled layer's tr_wreduce / tr_breduce assigns its whole
  // gW / gb once per step; a disabled layer's gradients are zeroed when it is disabled)
  // compute_loss: 6 stages x (paf, heat), mean over n * C * h8 * w8 elements each
  const int64_t per = (int64_t)n * 38 * h8 * w8;
  const size_t nblocks = nb(per);
  if (c->lpart_n < 12 * nblocks) {
    if (c->lpart) OP_HIP_CHECK(hipFree(c->lpart));
    OP_HIP_CHECK(hipMalloc(&c->lpart, 12 * nblocks * sizeof(double)));
    c->lpart_n = 12 * nblocks;
  }
  OP_HIP_CHECK(hipMemsetAsync(c->lpart, 0, 12 * nblocks * sizeof(double), c->stream));
  for (int s = 1; s <= 6; ++s)
    for (int paf = 1; paf >= 0; --paf) {
      const MapT m = stage_map(s, paf);
      const int64_t numel = (int64_t)n * m.C * h8 * w8;
      const int slot = 2 * (s - 1) + (paf ? 0 : 1);
      hipLaunchKernelGGL(tr_loss, dim3(nb(numel)), dim3(256), 0, c->stream, c->act[m.buf], m.off, c->grad[m.buf],
                         paf ? c->d_t : c->d_t + tp, c->d_ign, n, m.C, (float)(2.0 / (double)numel),
                         c->lpart + slot * nblocks);
    }
  // backward down to the lowest enabled layer
  int lowest = kNL;
  for (int l = 0; l < kNL; ++l)
    if (c->enabled[l]) {
      lowest = l;
      break;
    }
  TRC(tr_backward(c, lowest));
  // Adam on the enabled layers (per-layer step counters, as Chainer's per-parameter rules)
  for (int l = 0; l < kNL; ++l) {
    if (!c->enabled[l]) continue;
    const TLayer& d = c->L[l];
    const int64_t t = ++c->t_step[l];
    const double fix1 = 1.0 - std::pow(c->beta1, (double)t), fix2 = 1.0 - std::pow(c->beta2, (double)t);
    const float lr = (float)(c->alpha * std::sqrt(fix2) / fix1);
    const int64_t nw = (int64_t)d.co * d.ci * d.k * d.k;
    hipLaunchKernelGGL(tr_adam, dim3(nb(nw)), dim3(256), 0, c->stream, c->W[l], c->gW[l], c->mW[l], c->vW[l], nw,
                       c->scale[l], lr, (float)c->beta1, (float)c->beta2, (float)c->eps);
    hipLaunchKernelGGL(tr_adam, dim3(nb(d.co)), dim3(256), 0, c->stream, c->b[l], c->gb[l], c->mb[l], c->vb[l],
                       (int64_t)d.co, c->scale[l], lr, (float)c->beta1, (float)c->beta2, (float)c->eps);
  }
  for (const auto& cv : c->convs)
    if (c->enabled[cv.layer]) TRC(tr_pack_layer(c, cv.layer, cv));
  std::vector<double> part(12 * nblocks);
  OP_HIP_CHECK(hipMemcpyAsync(part.data(), c->lpart, part.size() * 8, hipMemcpyDeviceToHost, c->stream));
  OP_HIP_CHECK(hipStreamSynchronize(c->stream));
  if (losses)
    for (int k = 0; k < 12; ++k) {
      const MapT m = stage_map(k / 2 + 1, k % 2 == 0);
      double s = 0.0;
      for (size_t i = 0; i < nblocks; ++i) s += part[k * nblocks + i];
      losses[k] = s / (double)((int64_t)n * m.C * h8 * w8);
    }
  return OP_OK;
}

}  // extern "C"
