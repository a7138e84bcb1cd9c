// Face / hand keypoint detectors on the CocoPoseNet conv kernels, gfx950.
//
// FaceNet / HandNet (models/FaceNet.py, models/HandNet.py) are single-branch CPM nets: VGG-19
// conv1_1 .. conv5_2 with three 2x2 pools (46x46 maps at 368x368), conv5_3_CPM -> the 128-channel
// feature map; stage 1 = conv6_1_CPM (1x1 128->512, ReLU) + conv6_2_CPM (1x1 512->C); stages 2-6 on
// concat((heatmaps C, feature 128)) = Mconv1-5 7x7 + Mconv6 1x1 (ReLU) + Mconv7 1x1 -> C maps
// (C = 71 face, 22 hand).  Plan on the device, every conv in the 3xBF16 split format:
//   preprocess_split16 (cv2 LINEAR + x/256 - 0.5, face_detector.py:32-33) -> conv1_pair (conv1_1 +
//   conv1_2 + pool) -> conv_m16k / conv_big 3x3 (pools fused into conv2_2, conv3_4) -> the stage
//   buffer CAT [feature 0..127 | heat 128..128+C-1 | zero pad to a 16-multiple] (concat free, Mconv1
//   weights permuted to it) -> conv_m16 7x7 raster tiles -> fused or plain 1x1 pairs writing their
//   heat slice of CAT; the last stage also writes a dense f32 copy.
// Detector post-process (face_detector.py:38-39, 58-72; hand_detector.py:41-49, 68-82):
//   F.resize_images to the crop size (resize_planar), SciPy gaussian_filter(sigma 2.5) as two f64
//   passes in SciPy's order with an f32 store between them (the pose path's arithmetic), then per
//   map one workgroup finds the max and the first two maxima in (optionally x-mirrored) row-major
//   order = np.where's order, from which the host forms [coords[1], coords[0], max].
#include <cstring>
#include <string>
#include <vector>

#include "common.hpp"
#include "host_pack.hpp"

namespace op {
namespace {

struct CpmLayer {
  std::string name;
  int ci, co, k;
};

// models/FaceNet.py:11-76 / models/HandNet.py:11-76 declaration order.
std::vector<CpmLayer> make_cpm_layers(int nm) {
  std::vector<CpmLayer> v = {{"conv1_1", 3, 64, 3},       {"conv1_2", 64, 64, 3},     {"conv2_1", 64, 128, 3},
                             {"conv2_2", 128, 128, 3},    {"conv3_1", 128, 256, 3},   {"conv3_2", 256, 256, 3},
                             {"conv3_3", 256, 256, 3},    {"conv3_4", 256, 256, 3},   {"conv4_1", 256, 512, 3},
                             {"conv4_2", 512, 512, 3},    {"conv4_3", 512, 512, 3},   {"conv4_4", 512, 512, 3},
                             {"conv5_1", 512, 512, 3},    {"conv5_2", 512, 512, 3},   {"conv5_3_CPM", 512, 128, 3},
                             {"conv6_1_CPM", 128, 512, 1}, {"conv6_2_CPM", 512, nm, 1}};
  for (int s = 2; s <= 6; ++s) {
    const std::string sfx = "_stage" + std::to_string(s);
    v.push_back({"Mconv1" + sfx, nm + 128, 128, 7});
    for (int i = 2; i <= 5; ++i) v.push_back({"Mconv" + std::to_string(i) + sfx, 128, 128, 7});
    v.push_back({"Mconv6" + sfx, 128, 128, 1});
    v.push_back({"Mconv7" + sfx, 128, nm, 1});
  }
  return v;
}

int n_maps_of(int arch) { return arch == OP_ARCH_FACENET ? 71 : (arch == OP_ARCH_HANDNET ? 22 : 0); }

const std::vector<CpmLayer>* cpm_table(int arch) {
  static const std::vector<CpmLayer> face = make_cpm_layers(71), hand = make_cpm_layers(22);
  return arch == OP_ARCH_FACENET ? &face : (arch == OP_ARCH_HANDNET ? &hand : nullptr);
}

constexpr int kNCpm = 17 + 5 * 7;
constexpr int kCpmFeat = 0, kCpmHeat = 128;

struct SConv {
  void* ws = nullptr;
  float* b = nullptr;
  int cop = 0, cin16 = 0, ks = 0;
};

struct CAct {
  float* p = nullptr;
  int pad = 0, cs = 0, h = 0, w = 0;
  size_t floats(int n) const { return (size_t)n * (h + 2 * pad) * (w + 2 * pad) * cs; }
};

enum CBuf { X0, P1, C21, C22, P2, C3A, C3B, C34, P3, C4A, C4B, CAT, BRA, BRB, S1, MAP32, NCBUF };

}  // namespace

// ---- kernels ----
// dense f32 maps (n*lh*lw, cs) -> planar (n, c, lh, lw)
__global__ __launch_bounds__(256) void cpm_planar(const float* __restrict__ m, int cs, int c, int n, int hw,
                                                  float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)n * c * hw) return;
  const int p = (int)(i % hw);
  const int ch = (int)((i / hw) % c);
  const int f = (int)(i / ((int64_t)hw * c));
  out[i] = m[((int64_t)f * hw + p) * cs + ch];
}

__device__ __forceinline__ int scipy_reflect(int i, int L) {  // mode='reflect' (d c b a | a b c d)
  if (L == 1) return 0;
  const int p = 2 * L;
  i %= p;
  if (i < 0) i += p;
  return i >= L ? p - 1 - i : i;
}

// one SciPy correlate1d pass (NI_Correlate1D symmetric: centre tap, then pairs outermost first,
// f64) along y (VERT) or x over the first `c` planes of (c, h, w); f32 result
template <bool VERT>
__global__ __launch_bounds__(256) void cpm_gauss(const float* __restrict__ in, int c, int h, int w,
                                                 const double* __restrict__ wt, int r, float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t plane = (int64_t)h * w;
  if (i >= plane * c) return;
  const int x = (int)(i % w);
  const int y = (int)((i / w) % h);
  const float* p = in + (i / plane) * plane;
  auto at = [&](int d) -> double {
    return VERT ? (double)p[(int64_t)scipy_reflect(y + d, h) * w + x] : (double)p[(int64_t)y * w + scipy_reflect(x + d, w)];
  };
  double o = __dmul_rn(at(0), wt[r]);
  for (int jj = -r; jj < 0; ++jj) o = __dadd_rn(o, __dmul_rn(__dadd_rn(at(jj), at(-jj)), wt[r + jj]));
  out[i] = __double2float_rn(o);
}

// per plane: max, number of maxima, first two maxima in row-major order of the (x-mirrored if
// flip) plane.  res[4 * plane] = {max bits, count, idx0, idx1}
constexpr int kArgT = 1024;
__global__ __launch_bounds__(kArgT) void cpm_argmax(const float* __restrict__ filt, int h, int w, int flip,
                                                    int32_t* __restrict__ res) {
  __shared__ float smax[kArgT / 64];
  __shared__ int scnt[kArgT / 64], s0[kArgT / 64], s1[kArgT / 64];
  const int64_t plane = (int64_t)h * w;
  const float* p = filt + blockIdx.x * plane;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float m = -INFINITY;
  for (int64_t i = threadIdx.x; i < plane; i += kArgT) m = fmaxf(m, p[i]);
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if (lane == 0) smax[wv] = m;
  __syncthreads();
  m = smax[0];
  for (int k = 1; k < kArgT / 64; ++k) m = fmaxf(m, smax[k]);
  // i = flattened index in the reference's (mirrored) order: (y, xr) with x = flip ? w-1-xr : xr
  int cnt = 0, i0 = 0x7fffffff, i1 = 0x7fffffff;
  for (int64_t i = threadIdx.x; i < plane; i += kArgT) {
    const int y = (int)(i / w), xr = (int)(i - (int64_t)y * w);
    const int x = flip ? w - 1 - xr : xr;
    if (p[(int64_t)y * w + x] == m) {
      ++cnt;
      if ((int)i < i0) {
        i1 = i0;
        i0 = (int)i;
      } else if ((int)i < i1) {
        i1 = (int)i;
      }
    }
  }
  for (int o = 32; o > 0; o >>= 1) {  // merge (count, two smallest)
    const int c2 = __shfl_xor(cnt, o), a2 = __shfl_xor(i0, o), b2 = __shfl_xor(i1, o);
    cnt += c2;
    const int lo = min(i0, a2), hi = max(i0, a2);
    i1 = min(hi, min(i1, b2));
    i0 = lo;
  }
  if (lane == 0) {
    scnt[wv] = cnt;
    s0[wv] = i0;
    s1[wv] = i1;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int c = 0, a = 0x7fffffff, b = 0x7fffffff;
    for (int k = 0; k < kArgT / 64; ++k) {
      c += scnt[k];
      const int lo = min(a, s0[k]), hi = max(a, s0[k]);
      b = min(hi, min(b, s1[k]));
      a = lo;
    }
    res[4 * blockIdx.x + 0] = __float_as_int(m);
    res[4 * blockIdx.x + 1] = c;
    res[4 * blockIdx.x + 2] = a;
    res[4 * blockIdx.x + 3] = b;
  }
}

}  // namespace op

using namespace op;

struct op_cpm_ctx {
  int device = 0, arch = 0, nm = 0;
  int cat_cs = 0;  // stage buffer channels: 128 + C rounded up to 16
  int st = 0;      // heat channels stored by the Mconv7 / conv6_2 epilogues (C rounded up to 8)
  hipStream_t stream = nullptr;
  bool have_weights = false;
  SConv L[kNCpm];
  float* w11 = nullptr;  // conv1_1 [tap][ci][co] f32 (conv1_pair)
  void* arena = nullptr;
  size_t arena_bytes = 0;
  int gn = 0, gh = 0, gw = 0;
  CAct buf[NCBUF];
  void* scratch = nullptr;
  size_t scratch_bytes = 0;
  double* d_gauss = nullptr;
  int gauss_r = 0;
  int splitk = 1;  // op_cpm_set_batch_invariant(0): small launches may split K (batch-dependent sums)
};

namespace op {
namespace {

int cpm_check(op_cpm_ctx* c, bool need_weights) {
  if (!c) {
    set_error("null op_cpm_ctx");
    return OP_ERR_INVALID;
  }
  OP_HIP_CHECK(hipSetDevice(c->device));
  if (need_weights && !c->have_weights) {
    set_error("op_cpm: weights not set");
    return OP_ERR_STATE;
  }
  return OP_OK;
}

int cpm_scratch(op_cpm_ctx* c, size_t bytes) {
  if (bytes <= c->scratch_bytes) return OP_OK;
  OP_HIP_CHECK(hipStreamSynchronize(c->stream));
  if (c->scratch) OP_HIP_CHECK(hipFree(c->scratch));
  c->scratch = nullptr;
  OP_HIP_CHECK(hipMalloc(&c->scratch, bytes));
  c->scratch_bytes = bytes;
  return OP_OK;
}

int cpm_geometry(op_cpm_ctx* c, int n, int h, int w) {
  if (h % 8 || w % 8 || h < 16 || w < 16 || n < 1) {
    set_error("network input must be >= 16 and a multiple of 8");
    return OP_ERR_INVALID;
  }
  if (c->gn == n && c->gh == h && c->gw == w) return OP_OK;
  struct D {
    int pad, cs, div;
  };
  const D d[NCBUF] = {{1, 16, 1},  {1, 64, 2},  {1, 128, 2}, {0, 128, 2}, {1, 128, 4},
                      {1, 256, 4}, {1, 256, 4}, {0, 256, 4}, {1, 256, 8}, {1, 512, 8}, {1, 512, 8},
                      {kStagePad, c->cat_cs, 8}, {kStagePad, 128, 8}, {kStagePad, 128, 8}, {0, 512, 8},
                      {0, c->st, 8}};
  CAct a[NCBUF];
  size_t total = 0;
  for (int i = 0; i < NCBUF; ++i) {
    a[i].pad = d[i].pad;
    a[i].cs = d[i].cs;
    a[i].h = h / d[i].div;
    a[i].w = w / d[i].div;
    total += (a[i].floats(n) + 63) / 64 * 64;
  }
  const size_t need = total * sizeof(float);
  if (need > c->arena_bytes) {
    OP_HIP_CHECK(hipStreamSynchronize(c->stream));
    if (c->arena) OP_HIP_CHECK(hipFree(c->arena));
    c->arena = nullptr;
    OP_HIP_CHECK(hipMalloc(&c->arena, need));
    c->arena_bytes = need;
  }
  OP_HIP_CHECK(hipMemsetAsync(c->arena, 0, need, c->stream));  // halos and channel padding stay 0
  float* p = (float*)c->arena;
  for (int i = 0; i < NCBUF; ++i) {
    a[i].p = p;
    p += (a[i].floats(n) + 63) / 64 * 64;
    c->buf[i] = a[i];
  }
  c->gn = n;
  c->gh = h;
  c->gw = w;
  return OP_OK;
}

SplitConvShape cshape(int n, const CAct& in, const CAct& out, int c16, int ks, bool relu, int splitk) {
  SplitConvShape s;
  s.n = n;
  s.h = out.h;
  s.w = out.w;
  s.pin = in.pad;
  s.cs_in = in.cs;
  s.pout = out.pad;
  s.cs_out = out.cs;
  s.c16 = c16;
  s.ks = ks;
  s.relu = relu ? 1 : 0;
  s.groups = 1;
  s.cs_out32 = 0;
  s.halo_mode = 4;
  s.splitk = splitk;
  s.regw = 1;
  return s;
}

int cconv(op_cpm_ctx* c, const CAct& in, int cin_off, const CAct& out, int cout_off, const SConv& pc, int store,
          bool relu, const CAct* out32 = nullptr) {
  SplitConvGroup g[2];
  g[0].in = in.p + cin_off;
  g[0].out = out.p + cout_off;
  g[0].w = pc.ws;
  g[0].bias = pc.b;
  g[0].cop = pc.cop;
  g[0].cout_store = store;
  g[0].cin_off = cin_off;
  g[0].out32 = out32 ? out32->p : nullptr;
  g[0].out32_off = 0;
  g[1] = g[0];
  SplitConvShape s = cshape(c->gn, in, out, pc.cin16 / 16, pc.ks, relu, c->splitk);
  if (out32) s.cs_out32 = out32->cs;
  return launch_conv_bf16x3(s, g, c->stream);
}

// 3x3 conv + ReLU + 2x2 pool: fused launch, else conv into `full` + pool kernel
int cconv_pool(op_cpm_ctx* c, const CAct& in, const CAct& full, const CAct& pooled, const SConv& pc, int ch) {
  SplitConvGroup g[2];
  g[0].in = in.p;
  g[0].out = pooled.p;
  g[0].w = pc.ws;
  g[0].bias = pc.b;
  g[0].cop = pc.cop;
  g[0].cout_store = ch;
  g[0].cin_off = 0;
  g[0].out32 = nullptr;
  g[0].out32_off = 0;
  g[1] = g[0];
  SplitConvShape s = cshape(c->gn, in, full, pc.cin16 / 16, pc.ks, true, c->splitk);
  s.pout = pooled.pad;
  s.cs_out = pooled.cs;
  int taken = 0;
  const int rc = launch_conv_big_pool(s, g, c->stream, &taken);
  if (rc || taken) return rc;
  const int r2 = cconv(c, in, 0, full, 0, pc, ch, true);
  return r2 ? r2 : launch_maxpool2_split(full.p, full.pad, pooled.p, pooled.pad, c->gn, full.h, full.w, ch, c->stream);
}

// 1x1 pair in -> a (ReLU) -> b -> out slice (+ dense f32 copy): fused head kernel when it fits
int cpair(op_cpm_ctx* c, const CAct& in, const CAct& mid, const CAct& out, int cout_off, const SConv& a, const SConv& b,
          const CAct* out32) {
  static const bool off = getenv("OP_HEAD_FUSED") && atoi(getenv("OP_HEAD_FUSED")) == 0;
  if (!off) {
    HeadShape s;
    s.n = c->gn;
    s.h = out.h;
    s.w = out.w;
    s.pin = in.pad;
    s.cs_in = in.cs;
    s.pout = out.pad;
    s.cs_out = out.cs;
    s.ci = a.cin16;
    s.co1 = a.cop;
    s.groups = 1;
    s.cs_out32 = out32 ? out32->cs : 0;
    HeadGroup g[2];
    g[0].in = in.p;
    g[0].w1 = a.ws;
    g[0].b1 = a.b;
    g[0].cop1 = a.cop;
    g[0].w2 = b.ws;
    g[0].b2 = b.b;
    g[0].cop2 = b.cop;
    g[0].out = out.p + cout_off;
    g[0].cout_store = c->st;
    g[0].out32 = out32 ? out32->p : nullptr;
    g[0].out32_off = 0;
    g[1] = g[0];
    int taken = 0;
    const int rc = launch_conv_head(s, g, c->stream, &taken);
    if (rc || taken) return rc;
  }
  CAct m = mid;
  m.cs = a.cop;
  const int r1 = cconv(c, in, 0, m, 0, a, a.cop, true);
  return r1 ? r1 : cconv(c, m, 0, out, cout_off, b, c->st, false, out32);
}

#define CRC(x)           \
  do {                   \
    int _r = (x);        \
    if (_r) return _r;   \
  } while (0)

int cpm_run(op_cpm_ctx* c) {
  CAct* B = c->buf;
  const SConv* L = c->L;
  CRC(launch_conv1_pair(nullptr, 0, 0, 0, 0, B[X0].p, c->gn, c->gh, c->gw, c->w11, L[0].b, L[1].ws, L[1].b, B[P1].p,
                        B[P1].pad, c->stream));
  CRC(cconv(c, B[P1], 0, B[C21], 0, L[2], 128, true));
  CRC(cconv_pool(c, B[C21], B[C22], B[P2], L[3], 128));
  CRC(cconv(c, B[P2], 0, B[C3A], 0, L[4], 256, true));
  CRC(cconv(c, B[C3A], 0, B[C3B], 0, L[5], 256, true));
  CRC(cconv(c, B[C3B], 0, B[C3A], 0, L[6], 256, true));
  CRC(cconv_pool(c, B[C3A], B[C34], B[P3], L[7], 256));
  CRC(cconv(c, B[P3], 0, B[C4A], 0, L[8], 512, true));
  CRC(cconv(c, B[C4A], 0, B[C4B], 0, L[9], 512, true));
  CRC(cconv(c, B[C4B], 0, B[C4A], 0, L[10], 512, true));
  CRC(cconv(c, B[C4A], 0, B[C4B], 0, L[11], 512, true));
  CRC(cconv(c, B[C4B], 0, B[C4A], 0, L[12], 512, true));
  CRC(cconv(c, B[C4A], 0, B[C4B], 0, L[13], 512, true));
  CRC(cconv(c, B[C4B], 0, B[CAT], kCpmFeat, L[14], 128, true));  // conv5_3_CPM: the feature map
  CRC(cpair(c, B[CAT], B[S1], B[CAT], kCpmHeat, L[15], L[16], nullptr));  // stage 1
  for (int s = 0; s < 5; ++s) {
    const SConv* M = L + 17 + 7 * s;
    CRC(cconv(c, B[CAT], 0, B[BRA], 0, M[0], 128, true));
    const CAct* src = &B[BRA];
    const CAct* dst = &B[BRB];
    for (int i = 1; i <= 4; ++i) {
      CRC(cconv(c, *src, 0, *dst, 0, M[i], 128, true));
      std::swap(src, dst);
    }
    CRC(cpair(c, *src, B[S1], B[CAT], kCpmHeat, M[5], M[6], s == 4 ? &B[MAP32] : nullptr));
  }
  return OP_OK;
}

}  // namespace
}  // namespace op

extern "C" {

int op_cpm_layer_count(int32_t arch) { return cpm_table(arch) ? kNCpm : 0; }

int op_cpm_layer_info(int32_t arch, int32_t index, const char** name, int32_t* ci, int32_t* co, int32_t* ksize) {
  const auto* t = cpm_table(arch);
  if (!t || index < 0 || index >= (int)t->size()) {
    set_error("op_cpm_layer_info: bad arch or index");
    return OP_ERR_INVALID;
  }
  const CpmLayer& d = (*t)[index];
  if (name) *name = d.name.c_str();
  if (ci) *ci = d.ci;
  if (co) *co = d.co;
  if (ksize) *ksize = d.k;
  return OP_OK;
}

int op_cpm_create(int32_t arch, int32_t device, op_cpm_ctx** out) {
  if (!out || !cpm_table(arch)) {
    set_error("op_cpm_create: bad arch or null out");
    return OP_ERR_INVALID;
  }
  *out = nullptr;
  int ndev = 0;
  OP_HIP_CHECK(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) {
    set_error("op_cpm_create: no HIP device " + std::to_string(device));
    return OP_ERR_INVALID;
  }
  OP_HIP_CHECK(hipSetDevice(device));
  op_cpm_ctx* c = new op_cpm_ctx();
  c->device = device;
  c->arch = arch;
  c->nm = n_maps_of(arch);
  c->cat_cs = (128 + c->nm + 15) / 16 * 16;
  c->st = (c->nm + 7) / 8 * 8;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    set_error("op_cpm_create: stream");
    return OP_ERR_HIP;
  }
  if (conv_big_device_init(device) != OP_OK) {
    hipStreamDestroy(c->stream);
    delete c;
    return OP_ERR_HIP;
  }
  std::vector<double> w;
  c->gauss_r = gaussian_taps(2.5, w);  // params['gaussian_sigma'] (entity.py:77)
  OP_HIP_CHECK(hipMalloc(&c->d_gauss, w.size() * sizeof(double)));
  OP_HIP_CHECK(hipMemcpy(c->d_gauss, w.data(), w.size() * sizeof(double), hipMemcpyHostToDevice));
  *out = c;
  return OP_OK;
}

static void cpm_free_weights(op_cpm_ctx* c) {
  for (auto& l : c->L) {
    if (l.ws) (void)hipFree(l.ws);
    if (l.b) (void)hipFree(l.b);
    l = SConv();
  }
  if (c->w11) (void)hipFree(c->w11);
  c->w11 = nullptr;
  c->have_weights = false;
}

int op_cpm_set_batch_invariant(op_cpm_ctx* c, int32_t enable) {
  CRC(cpm_check(c, false));
  c->splitk = enable ? 0 : 1;
  return OP_OK;
}

int op_cpm_destroy(op_cpm_ctx* c) {
  if (!c) return OP_OK;
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  cpm_free_weights(c);
  if (c->arena) (void)hipFree(c->arena);
  if (c->scratch) (void)hipFree(c->scratch);
  if (c->d_gauss) (void)hipFree(c->d_gauss);
  splitk_ws_release(c->stream);
  (void)hipStreamDestroy(c->stream);
  delete c;
  return OP_OK;
}

int op_cpm_set_weights(op_cpm_ctx* c, const float* const* W, const float* const* b) {
  CRC(cpm_check(c, false));
  if (!W || !b) {
    set_error("null weights");
    return OP_ERR_INVALID;
  }
  const auto& T = *cpm_table(c->arch);
  for (int i = 0; i < kNCpm; ++i)
    if (!W[i] || !b[i]) {
      set_error("missing weights for layer " + T[i].name);
      return OP_ERR_INVALID;
    }
  cpm_free_weights(c);
  const int nm = c->nm;
  for (int i = 0; i < kNCpm; ++i) {
    const CpmLayer& d = T[i];
    SConv& pc = c->L[i];
    const bool cat_in = d.name.rfind("Mconv1_", 0) == 0;
    pc.ks = d.k;
    pc.cop = (d.co + 63) / 64 * 64;
    pc.cin16 = cat_in ? c->cat_cs : (d.ci + 15) / 16 * 16;
    // stage input: physical [feature 0..127 | heat 128..128+C-1] <- logical concat((heat, feature))
    auto cmap = [&](int p) -> int {
      if (!cat_in) return p < d.ci ? p : -1;
      if (p < 128) return nm + p;
      return p < 128 + nm ? p - 128 : -1;
    };
    std::vector<uint16_t> ws((size_t)pc.cin16 * d.k * d.k * pc.cop * 2, 0);
    pack_split(ws, pc.cop, pc.cin16, d.k, W[i], d.co, d.ci, 0, cmap);
    std::vector<float> bias(pc.cop, 0.0f);
    memcpy(bias.data(), b[i], d.co * sizeof(float));
    OP_HIP_CHECK(hipMalloc(&pc.ws, ws.size() * sizeof(uint16_t)));
    OP_HIP_CHECK(hipMemcpy(pc.ws, ws.data(), ws.size() * sizeof(uint16_t), hipMemcpyHostToDevice));
    OP_HIP_CHECK(hipMalloc(&pc.b, bias.size() * sizeof(float)));
    OP_HIP_CHECK(hipMemcpy(pc.b, bias.data(), bias.size() * sizeof(float), hipMemcpyHostToDevice));
  }
  std::vector<float> w11(9 * 3 * 64);  // conv1_1 for conv1_pair: [tap][ci][co]
  for (int co = 0; co < 64; ++co)
    for (int ci = 0; ci < 3; ++ci)
      for (int t = 0; t < 9; ++t) w11[(t * 3 + ci) * 64 + co] = W[0][(co * 3 + ci) * 9 + t];
  OP_HIP_CHECK(hipMalloc(&c->w11, w11.size() * sizeof(float)));
  OP_HIP_CHECK(hipMemcpy(c->w11, w11.data(), w11.size() * sizeof(float), hipMemcpyHostToDevice));
  c->have_weights = true;
  return OP_OK;
}

int op_cpm_forward(op_cpm_ctx* c, const float* x, int32_t n, int32_t h, int32_t w, float* maps) {
  CRC(cpm_check(c, true));
  if (!x || !maps) {
    set_error("op_cpm_forward: null pointer");
    return OP_ERR_INVALID;
  }
  CRC(cpm_geometry(c, n, h, w));
  const size_t xin = (size_t)n * 3 * h * w * 4;
  const int lh = h / 8, lw = w / 8;
  const size_t outb = (size_t)n * c->nm * lh * lw * 4;
  CRC(cpm_scratch(c, xin + 256 + outb));
  float* dx = (float*)c->scratch;
  float* dmaps = (float*)((char*)c->scratch + (xin + 255) / 256 * 256);
  OP_HIP_CHECK(hipMemcpyAsync(dx, x, xin, hipMemcpyHostToDevice, c->stream));
  CRC(launch_nchw_to_split16(dx, c->buf[X0].p, n, h, w, c->stream));
  CRC(cpm_run(c));
  const int64_t tot = (int64_t)n * c->nm * lh * lw;
  hipLaunchKernelGGL(cpm_planar, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, c->stream, c->buf[MAP32].p,
                     c->buf[MAP32].cs, c->nm, n, lh * lw, dmaps);
  OP_AFTER_LAUNCH("cpm_planar", c->stream);
  OP_HIP_CHECK(hipMemcpyAsync(maps, dmaps, outb, hipMemcpyDeviceToHost, c->stream));
  OP_HIP_CHECK(hipStreamSynchronize(c->stream));
  return OP_OK;
}

// gaussian + argmax over the first c-1 planes of the device maps `heat` (c, h, w) -> dres
// (c-1 records of [max bits, count, first two row-major maxima], device)
static int cpm_peaks_launch(op_cpm_ctx* c, float* heat, float* tmp, float* filt, int32_t* dres, int ch, int h, int w,
                            int flip) {
  const int np = ch - 1;
  if (np < 1) return OP_OK;
  const int64_t tot = (int64_t)np * h * w;
  const unsigned nb = (unsigned)((tot + 255) / 256);
  hipLaunchKernelGGL(cpm_gauss<true>, dim3(nb), dim3(256), 0, c->stream, heat, np, h, w, c->d_gauss, c->gauss_r, tmp);
  OP_AFTER_LAUNCH("cpm_gauss_v", c->stream);
  hipLaunchKernelGGL(cpm_gauss<false>, dim3(nb), dim3(256), 0, c->stream, tmp, np, h, w, c->d_gauss, c->gauss_r, filt);
  OP_AFTER_LAUNCH("cpm_gauss_h", c->stream);
  hipLaunchKernelGGL(cpm_argmax, dim3((unsigned)np), dim3(kArgT), 0, c->stream, filt, h, w, flip, dres);
  OP_AFTER_LAUNCH("cpm_argmax", c->stream);
  OP_HIP_CHECK(hipGetLastError());
  return OP_OK;
}

static void cpm_peaks_decode(const int32_t* res, int ch, int w, float thresh, double* kp, int32_t* found);

static int cpm_peaks_dev(op_cpm_ctx* c, float* heat, float* tmp, float* filt, int32_t* dres, int ch, int h, int w,
                         float thresh, int flip, double* kp, int32_t* found) {
  const int np = ch - 1;
  if (np < 1) return OP_OK;
  CRC(cpm_peaks_launch(c, heat, tmp, filt, dres, ch, h, w, flip));
  std::vector<int32_t> res((size_t)np * 4);
  OP_HIP_CHECK(hipMemcpyAsync(res.data(), dres, res.size() * 4, hipMemcpyDeviceToHost, c->stream));
  OP_HIP_CHECK(hipStreamSynchronize(c->stream));
  cpm_peaks_decode(res.data(), ch, w, thresh, kp, found);
  return OP_OK;
}

static void cpm_peaks_decode(const int32_t* res, int ch, int w, float thresh, double* kp, int32_t* found) {
  const int np = ch - 1;
  for (int i = 0; i < np; ++i) {
    float m;
    memcpy(&m, &res[4 * i], 4);
    const int cnt = res[4 * i + 1], i0 = res[4 * i + 2], i1 = res[4 * i + 3];
    found[i] = m > thresh ? 1 : 0;
    double* k = kp + 3 * i;
    if (!found[i] || cnt < 1) {
      found[i] = 0;
      k[0] = k[1] = k[2] = 0.0;
      continue;
    }
    // coords = np.array(np.where(map == m)).flatten() = [y0, y1, ..., x0, x1, ...]
    const int y0 = i0 / w, x0 = i0 % w;
    k[0] = cnt == 1 ? (double)x0 : (double)(i1 / w);  // coords[1]
    k[1] = (double)y0;                                // coords[0]
    k[2] = (double)m;
  }
}

int op_cpm_peaks(op_cpm_ctx* c, const float* heatmaps, int32_t ch, int32_t h, int32_t w, float thresh, int32_t flip,
                 double* keypoints, int32_t* found) {
  CRC(cpm_check(c, false));
  if (!heatmaps || !keypoints || !found || ch < 2 || h < 1 || w < 1 || (int64_t)h * w >= (1ll << 31)) {
    set_error("op_cpm_peaks: bad arguments");
    return OP_ERR_INVALID;
  }
  const size_t pb = ((size_t)ch * h * w * 4 + 255) / 256 * 256;
  CRC(cpm_scratch(c, 3 * pb + (size_t)ch * 16));
  char* s = (char*)c->scratch;
  float* heat = (float*)s;
  OP_HIP_CHECK(hipMemcpyAsync(heat, heatmaps, (size_t)ch * h * w * 4, hipMemcpyHostToDevice, c->stream));
  return cpm_peaks_dev(c, heat, (float*)(s + pb), (float*)(s + 2 * pb), (int32_t*)(s + 3 * pb), ch, h, w, thresh,
                       flip, keypoints, found);
}

int op_cpm_detect(op_cpm_ctx* c, const uint8_t* bgr, int32_t h, int32_t w, int64_t row_stride, float thresh,
                  int32_t flip_maps, double* keypoints, int32_t* found) {
  CRC(cpm_check(c, true));
  if (!bgr || !keypoints || !found || h < 2 || w < 2 || row_stride < (int64_t)w * 3 ||
      (int64_t)h * w >= (1ll << 31)) {
    set_error("op_cpm_detect: bad arguments");
    return OP_ERR_INVALID;
  }
  const int S = 368;  // params['face_inference_img_size'] = params['hand_inference_img_size'] (entity.py:127, 143)
  CRC(cpm_geometry(c, 1, S, S));
  const int lh = S / 8, lw = S / 8, ch = c->nm;
  const int64_t packed = (int64_t)w * 3;  // rows are packed on upload (row_stride may span a wider image)
  const size_t ib = ((size_t)h * packed + 255) / 256 * 256;
  const size_t lb = ((size_t)ch * lh * lw * 4 + 255) / 256 * 256;
  const size_t pb = ((size_t)ch * h * w * 4 + 255) / 256 * 256;
  CRC(cpm_scratch(c, ib + lb + 3 * pb + (size_t)ch * 16));
  char* s = (char*)c->scratch;
  uint8_t* dimg = (uint8_t*)s;
  float* low = (float*)(s + ib);
  float* heat = (float*)(s + ib + lb);
  OP_HIP_CHECK(hipMemcpy2DAsync(dimg, packed, bgr, row_stride, packed, h, hipMemcpyHostToDevice, c->stream));
  CRC(launch_preprocess_split(dimg, 0, packed, 1, h, w, S, S, c->buf[X0].p, c->stream, 256.0f));
  CRC(cpm_run(c));
  const int64_t tot = (int64_t)ch * lh * lw;
  hipLaunchKernelGGL(cpm_planar, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, c->stream, c->buf[MAP32].p,
                     c->buf[MAP32].cs, ch, 1, lh * lw, low);
  OP_AFTER_LAUNCH("cpm_planar", c->stream);
  CRC(launch_resize_images(low, ch, lh, lw, h, w, heat, c->stream));
  return cpm_peaks_dev(c, heat, (float*)(s + ib + lb + pb), (float*)(s + ib + lb + 2 * pb),
                       (int32_t*)(s + ib + lb + 3 * pb), ch, h, w, thresh, flip_maps, keypoints, found);
}

int op_cpm_detect_batch(op_cpm_ctx* c, int32_t n, const uint8_t* const* bgr, const int32_t* h, const int32_t* w,
                        const int64_t* row_stride, float thresh, const int32_t* flip_maps, double* keypoints,
                        int32_t* found) {
  CRC(cpm_check(c, true));
  if (n < 0 || (n > 0 && (!bgr || !h || !w || !row_stride || !keypoints || !found))) {
    set_error("op_cpm_detect_batch: bad arguments");
    return OP_ERR_INVALID;
  }
  for (int i = 0; i < n; ++i)
    if (!bgr[i] || h[i] < 2 || w[i] < 2 || row_stride[i] < (int64_t)w[i] * 3 || (int64_t)h[i] * w[i] >= (1ll << 31)) {
      set_error("op_cpm_detect_batch: bad crop " + std::to_string(i));
      return OP_ERR_INVALID;
    }
  if (n == 0) return OP_OK;
  const int S = 368;  // as op_cpm_detect
  CRC(cpm_geometry(c, n, S, S));
  const int lh = S / 8, lw = S / 8, ch = c->nm, np = ch - 1;
  auto al = [](size_t b) { return (b + 255) / 256 * 256; };
  // scratch: every crop's bytes, the batch's low-resolution maps, one full-size heat / tmp / filt
  // set (the per-crop upsample + peak launches run in stream order), the argmax records
  std::vector<size_t> ioff(n);
  size_t off = 0, pb = 0;
  for (int i = 0; i < n; ++i) {
    ioff[i] = off;
    off += al((size_t)h[i] * w[i] * 3);
    pb = std::max(pb, al((size_t)ch * h[i] * w[i] * 4));
  }
  const size_t lb = al((size_t)n * ch * lh * lw * 4);
  const size_t low_off = off, heat_off = off + lb;
  const size_t res_off = heat_off + 3 * pb;
  CRC(cpm_scratch(c, res_off + (size_t)n * std::max(np, 1) * 16));
  char* s = (char*)c->scratch;
  const size_t fx = c->buf[X0].floats(1);
  for (int i = 0; i < n; ++i) {
    const int64_t packed = (int64_t)w[i] * 3;
    OP_HIP_CHECK(hipMemcpy2DAsync(s + ioff[i], packed, bgr[i], row_stride[i], packed, h[i], hipMemcpyHostToDevice,
                                  c->stream));
    CRC(launch_preprocess_split((const uint8_t*)(s + ioff[i]), 0, packed, 1, h[i], w[i], S, S,
                                c->buf[X0].p + (size_t)i * fx, c->stream, 256.0f));
  }
  CRC(cpm_run(c));
  float* low = (float*)(s + low_off);
  const int64_t tot = (int64_t)n * ch * lh * lw;
  hipLaunchKernelGGL(cpm_planar, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, c->stream, c->buf[MAP32].p,
                     c->buf[MAP32].cs, ch, n, lh * lw, low);
  OP_AFTER_LAUNCH("cpm_planar", c->stream);
  float* heat = (float*)(s + heat_off);
  int32_t* dres = (int32_t*)(s + res_off);
  for (int i = 0; i < n; ++i) {
    CRC(launch_resize_images(low + (size_t)i * ch * lh * lw, ch, lh, lw, h[i], w[i], heat, c->stream));
    CRC(cpm_peaks_launch(c, heat, (float*)(s + heat_off + pb), (float*)(s + heat_off + 2 * pb),
                         dres + (size_t)i * np * 4, ch, h[i], w[i], flip_maps ? flip_maps[i] : 0));
  }
  if (np < 1) return OP_OK;
  std::vector<int32_t> res((size_t)n * np * 4);
  OP_HIP_CHECK(hipMemcpyAsync(res.data(), dres, res.size() * 4, hipMemcpyDeviceToHost, c->stream));
  OP_HIP_CHECK(hipStreamSynchronize(c->stream));
  for (int i = 0; i < n; ++i)
    cpm_peaks_decode(res.data() + (size_t)i * np * 4, ch, w[i], thresh, keypoints + (size_t)i * np * 3,
                     found + (size_t)i * np);
  return OP_OK;
}

}  // extern "C"
