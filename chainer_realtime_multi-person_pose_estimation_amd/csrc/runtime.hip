// Runtime + C ABI of the MI355X OpenPose path (include/openpose_hip.h).
//
// One context = one device, one stream, weights packed once in HBM, an activation arena carved
// per (batch, net size) geometry, and the post-process buffers.  The forward plan is the layer
// sequence of models/CocoPoseNet.py:132-262 with the two refinement branches fused:
//   * Mconv1_stageN_L1/L2 and conv5_1_CPM_L1/L2 share their input -> one conv with Co = 256;
//   * the later branch layers run as one 2-group launch (grid.z = branch);
//   * F.concat((paf, heat, feature)) is a single 192-channel buffer whose slices the producing
//     convs write directly (no concat copy).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "common.hpp"
#include "host_pack.hpp"

namespace op {

static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }

// ---- debugging aid: guard bands (OP_GUARD=<bytes>) ----
// Every device buffer gets a band of 0xA5 bytes after it; guard_check() (after each debug-synced
// launch and at every synchronising entry point) reports the first band a kernel wrote into.
size_t g_guard = 0;
struct GuardBand {
  const char* name;
  const char* p;
};
static std::vector<GuardBand> g_bands;
static std::mutex g_band_mu;

static void guard_add(const char* name, void* p, hipStream_t st) {
  if (!g_guard) return;
  hipMemsetAsync(p, 0xA5, g_guard, st);
  std::lock_guard<std::mutex> lk(g_band_mu);
  g_bands.push_back({name, (const char*)p});
}

static void guard_forget(const void* base, size_t bytes) {
  if (!g_guard || !base) return;
  std::lock_guard<std::mutex> lk(g_band_mu);
  const char* b = (const char*)base;
  std::vector<GuardBand> keep;
  for (auto& g : g_bands)
    if (!(g.p >= b && g.p < b + bytes)) keep.push_back(g);
  g_bands.swap(keep);
}

static int guard_check(const char* where) {
  if (!g_guard) return OP_OK;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipDeviceSynchronize() != hipSuccess) return OP_OK;  // the caller reports the fault itself
  std::lock_guard<std::mutex> lk(g_band_mu);
  std::vector<unsigned char> h(g_guard);
  for (auto& g : g_bands) {
    if (hipMemcpy(h.data(), g.p, g_guard, hipMemcpyDeviceToHost) != hipSuccess) {
      (void)hipGetLastError();  // a band of a buffer freed without guard_forget: not a kernel fault,
      continue;                 // and the sticky error must not surface at the next launch check
    }
    for (size_t i = 0; i < g_guard; ++i)
      if (h[i] != 0xA5) {
        char msg[256];
        snprintf(msg, sizeof(msg), "guard band after buffer '%s' overwritten at +%zu (byte 0x%02x), seen after %s",
                 g.name, i, h[i], where);
        fprintf(stderr, "[openpose_hip] %s\n", msg);
        set_error(msg);
        (void)cs;
        return OP_ERR_STATE;
      }
  }
  return OP_OK;
}

bool g_debug_sync = false;
int debug_after_launch(const char* name, hipStream_t st) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone) return OP_OK;
  const hipError_t e1 = hipGetLastError();
  const hipError_t e2 = hipStreamSynchronize(st);
  if (e1 != hipSuccess || e2 != hipSuccess) {
    set_error(std::string("after kernel ") + name + ": " + hipGetErrorString(e1 != hipSuccess ? e1 : e2));
    fprintf(stderr, "[openpose_hip] fault after kernel %s: %s\n", name, hipGetErrorString(e1 != hipSuccess ? e1 : e2));
    return OP_ERR_HIP;
  }
  return guard_check(name);
}

struct LayerDef {
  const char* name;
  int ci, co, k;
};

// models/CocoPoseNet.py:26-129 declaration order.
static std::vector<LayerDef> make_layers() {
  std::vector<LayerDef> v;
  static const char* bb[] = {"conv1_1", "conv1_2", "conv2_1", "conv2_2", "conv3_1", "conv3_2",
                             "conv3_3", "conv3_4", "conv4_1", "conv4_2", "conv4_3_CPM", "conv4_4_CPM"};
  static const int bci[] = {3, 64, 64, 128, 128, 256, 256, 256, 256, 512, 512, 256};
  static const int bco[] = {64, 64, 128, 128, 256, 256, 256, 256, 512, 512, 256, 128};
  for (int i = 0; i < 12; ++i) v.push_back({bb[i], bci[i], bco[i], 3});
  static std::vector<std::string> names;  // storage for generated names
  names.reserve(200);
  auto add = [&](const std::string& n, int ci, int co, int k) {
    names.push_back(n);
    v.push_back({names.back().c_str(), ci, co, k});
  };
  const char* br[2] = {"L1", "L2"};
  const int out[2] = {38, 19};
  for (int b = 0; b < 2; ++b) {
    for (int i = 1; i <= 3; ++i) add("conv5_" + std::to_string(i) + "_CPM_" + br[b], 128, 128, 3);
    add(std::string("conv5_4_CPM_") + br[b], 128, 512, 1);
    add(std::string("conv5_5_CPM_") + br[b], 512, out[b], 1);
  }
  for (int s = 2; s <= 6; ++s)
    for (int b = 0; b < 2; ++b) {
      const std::string sfx = "_stage" + std::to_string(s) + "_" + br[b];
      add("Mconv1" + sfx, 185, 128, 7);
      for (int i = 2; i <= 5; ++i) add("Mconv" + std::to_string(i) + sfx, 128, 128, 7);
      add("Mconv6" + sfx, 128, 128, 1);
      add("Mconv7" + sfx, 128, out[b], 1);
    }
  return v;
}

static const std::vector<LayerDef>& layers() {
  static std::vector<LayerDef> L = make_layers();
  return L;
}

static int layer_index(const std::string& n) {
  const auto& L = layers();
  for (size_t i = 0; i < L.size(); ++i)
    if (n == L[i].name) return (int)i;
  return -1;
}

// ---- packed weights ----
struct PackedConv {
  float* w = nullptr;
  float* b = nullptr;
  int cop = 0, cin_phys = 0, ks = 0;
  int cin_log = 0, co_log = 0;  // logical (reference) channel counts, for algorithmic FLOPs
  void* ws = nullptr;           // 3xBF16 split weights [c16][tap][cop][k-half][hi8 lo8]
  int cin16 = 0;                // input channels padded to 16 (split path)
};

struct ProfPair {
  int cls;
  hipEvent_t a, b;
  double flops, bytes;
  int n;  // launches between a and b (a joined run of back-to-back launches of one class)
};

// Logical input channel of physical channel p in the stage-input buffer (-1 = zero pad).
// Logical order is F.concat((paf 38, heat 19, feature 128)) (CocoPoseNet.py:168).
static int cat_logical(int p) {
  if (p >= kCatFeat && p < kCatFeat + 128) return 57 + (p - kCatFeat);
  if (p >= kCatHeat && p < kCatHeat + 19) return 38 + (p - kCatHeat);
  if (p >= kCatPaf && p < kCatPaf + 38) return p - kCatPaf;
  return -1;
}

// Pack Chainer W (Co, Ci, k, k) into [c8][tap][cop][8] at output-channel offset co_off.
static void pack_into(std::vector<float>& dst, std::vector<float>& bias, int cop, int cin_phys, int k, const float* W,
                      const float* b, int Co, int Ci, int co_off, bool cat_input) {
  const int c8 = cin_phys / 8, taps = k * k;
  for (int co = 0; co < Co; ++co) {
    bias[co_off + co] = b[co];
    for (int p = 0; p < cin_phys; ++p) {
      const int ci = cat_input ? cat_logical(p) : (p < Ci ? p : -1);
      if (ci < 0) continue;
      for (int t = 0; t < taps; ++t) {
        const int ky = t / k, kx = t % k;
        const float v = W[(((size_t)co * Ci + ci) * k + ky) * k + kx];
        const size_t idx = ((((size_t)(p / 8) * taps + t) * cop) + (co_off + co)) * 8 + (p % 8);
        dst[idx] = v;
      }
    }
  }
  (void)c8;
}

// Pack Chainer W (Co, Ci, k, k) into the split layout at output-channel offset co_off (host_pack.hpp);
// cat_input: physical channels of the 192-channel stage input (cat_logical).
static void pack_split_into(std::vector<uint16_t>& dst, int cop, int cin16, int k, const float* W, int Co, int Ci,
                            int co_off, bool cat_input) {
  pack_split(dst, cop, cin16, k, W, Co, Ci, co_off, [&](int p) { return cat_input ? cat_logical(p) : (p < Ci ? p : -1); });
}

static int upload(PackedConv& pc, const std::vector<float>& w, const std::vector<float>& b) {
  OP_HIP_CHECK(hipMalloc(&pc.w, w.size() * sizeof(float)));
  OP_HIP_CHECK(hipMalloc(&pc.b, b.size() * sizeof(float)));
  OP_HIP_CHECK(hipMemcpy(pc.w, w.data(), w.size() * sizeof(float), hipMemcpyHostToDevice));
  OP_HIP_CHECK(hipMemcpy(pc.b, b.data(), b.size() * sizeof(float), hipMemcpyHostToDevice));
  return OP_OK;
}

static int upload_split(PackedConv& pc, const std::vector<uint16_t>& ws) {
  OP_HIP_CHECK(hipMalloc(&pc.ws, ws.size() * sizeof(uint16_t)));
  OP_HIP_CHECK(hipMemcpy(pc.ws, ws.data(), ws.size() * sizeof(uint16_t), hipMemcpyHostToDevice));
  return OP_OK;
}

static int round_up(int v, int m) { return (v + m - 1) / m * m; }

// ---- activation buffers ----
struct Act {
  float* p = nullptr;
  int pad = 0, cs = 0, h = 0, w = 0;
  int planar = 0;  // split layout: 0 [frame][hp][wp][cs], 1 chunk-planar (SplitConvShape::in_planar)
  size_t frame_floats() const { return (size_t)(h + 2 * pad) * (w + 2 * pad) * cs; }
};

// Input of the last batched post-process (0: none, 1: low-res maps through the fused upsample,
// 2: full-resolution planar maps of the precise path), kept so one frame can be re-run uncapped.
struct PostRecord {
  int kind = 0;
  MapSource low{};
  const float* full = nullptr;
  int64_t fstride = 0;
  PostShape s{};
};

// Per gather slot (gather.hip's two record slots): the post-process input of the frames whose
// record cannot carry the whole result (over the batched caps, or more persons than the record
// holds), copied aside on the device when the records are packed, so the owning rank can re-run
// them after the next step has overwritten the batched buffers (op_comm_overflow*).
struct KeepSlot {
  // kept frames are compacted into `slots` entries assigned by device counters.  Round 5 (advisor
  // r04): every frame of the pack gets a slot while their maps fit kKeepSlotBytes (the 368x368 maps
  // of 232 frames: 125 MB; 16 precise 1280x720 frames: 3.4 GB), at least 8 beyond that, and a
  // gather that had more overflow frames than slots grows the next packs' slots (`grow`);
  // OP_KEEP_FRAMES=<n> pins the count (test aid).  A frame left without a slot is reported as a
  // frame status through the overflow exchange (frames.py), never as an exception before it
  float* maps = nullptr;  // [slot][fstride] post-process input of frames over the batched caps
  size_t maps_cap = 0;  // bytes
  double* res = nullptr;  // [slot][maxs][54 + 1] rows of frames past max_persons not in h_rows
  size_t res_cap = 0;
  int slots = 0;
  int maxs = 0;
  int32_t* cnt = nullptr;
  size_t cnt_cap = 0;
  // n x kKeepHdr {status, n_peaks, n_persons, why: 0 whole record, 1 over the caps, 2 > max_persons,
  // where: why 1: its maps / cnt slot; why 2: >= 0 offset of its rows in h_rows (doubles), <= -2
  // res slot -2 - where; -1: not kept (more such frames than slots: OP_ERR_CAPACITY on collection)}
  int32_t* d_hdr = nullptr;
  int32_t* h_hdr = nullptr;  // pinned copy, complete when the slot's gather is
  size_t hdr_cap = 0;
  // rows of the frames past max_persons written by keep_overflow straight into page-locked host
  // memory (poses then scores per frame, packed by a device counter), so collecting them needs no
  // GPU copy: a copy on any stream would share a hardware queue with the next steps' compute
  // and wait for them (round 3: 65 ms per 114-frame step on the network-maps line)
  double* h_rows = nullptr;
  double* d_rows_view = nullptr;  // the device's address of h_rows (hipHostGetDevicePointer)
  int64_t h_rows_cap = 0;  // doubles
  int64_t rows_cap_now = 0;  // of them, usable by the current pack (OP_KEEP_ROWS_AVG)
  PostRecord rec{};
  int n = 0;
  int grow = 0;  // overflow frames of the largest gather seen that needed a slot
};
constexpr int kKeepHdr = 5;  // int32 per frame in KeepSlot::d_hdr / h_hdr
constexpr int64_t kKeepSlotBytes = 4ll << 30;  // keep-slot map bytes per gather slot (of 288 GB HBM)
constexpr int64_t kKeepGrowBytes = 16ll << 30;  // ceiling of the grown slots' map bytes per gather slot

enum BufId {
  B_X0, B_C11, B_C12, B_P1, B_C21, B_C22, B_P2, B_C3A, B_C3B, B_C34, B_P3, B_C41, B_C42, B_C43, B_CAT, B_BRA, B_BRB,
  B_S1, B_MAP32, B_PA, B_PB, B_CATP, B_COUNT
};

}  // namespace op

using namespace op;

struct op_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  op_params prm;
  op_limits lim;
  bool have_weights = false;
  // packed convolutions (see build_weights)
  PackedConv bb[12];           // backbone conv1_1 .. conv4_4_CPM
  PackedConv s1_first;         // conv5_1 L1|L2 fused (Co 256)
  PackedConv s1_g[2][3];       // [branch][conv5_2, conv5_3, conv5_4]
  PackedConv s1_last[2];       // conv5_5 L1 / L2
  PackedConv st_first[5];      // Mconv1 stage s, fused (Co 256, 192 phys in)
  PackedConv st_g[5][2][5];    // [stage][branch][Mconv2..Mconv6]
  PackedConv st_last[5][2];    // Mconv7
  float* w11 = nullptr;        // conv1_1 weights [tap][ci][co] f32 for the VALU kernel (conv11.hip)
  // activation arena of the current geometry, and every geometry's arena (multi-scale: one per
  // scale, kept so switching scales needs neither an allocation nor a re-zeroing memset)
  void* arena = nullptr;
  size_t arena_bytes = 0;
  struct GeomArena {
    int n, h, w;
    bool split;
    void* p;
    size_t bytes;
    uint64_t used;
  };
  std::vector<GeomArena> arenas;
  uint64_t arena_clock = 0;
  int gn = 0, gh = 0, gw = 0;  // current geometry (batch, net h, net w)
  bool split = true;           // 3xBF16 split convs (default) or exact f32 MFMA convs
  bool gsplit = true;          // format the arena is currently carved for
  int conv_algo = 4;           // split-path conv kernel family (op_set_conv_algo)
  int stage_planar = 1;        // chunk-planar 7x7 stage tensors where conv_m16 takes them (op_set_stage_layout)
  Act buf[B_COUNT];
  // post-process
  PostBuffers pb{};
  void* post_arena = nullptr;
  size_t post_bytes = 0;
  int pn = 0, pmh = 0, pmw = 0;  // post geometry
  std::vector<double> gauss_host;
  int gauss_r = 0;
  // op_set_peak_mode: 1 = the reference's GPU-branch peaks (ksize x ksize unnormalised Gaussian,
  // zero padding, >= NMS) in the single-scale post-process; gpu_taps = its 1-D factor (2 gpu_r + 1)
  int peak_mode = 0;
  int gpu_r = 0;
  std::vector<double> gpu_taps;
  // staging
  uint8_t* d_frames = nullptr;
  size_t frames_bytes = 0;
  // async frame uploads (op_upload_frames): a 2-slot device ring filled on copy_stream; the next
  // run waits for its slot's copy and moves it into d_frames on the compute stream
  hipStream_t copy_stream = nullptr;
  // detect_precise (round 6): the small scales' forwards run on side_stream, concurrent with the large
  // ones on the compute stream (fork / join events); while they are enqueued `stream` points at it
  hipStream_t side_stream = nullptr;
  hipStream_t main_stream = nullptr;  // the compute stream while `stream` is swapped to side_stream
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  uint8_t* d_ring[2] = {nullptr, nullptr};
  size_t ring_bytes[2] = {0, 0};
  hipEvent_t ev_up[2] = {nullptr, nullptr}, ev_free[2] = {nullptr, nullptr};
  int ring_next = 0, up_slot = -1, up_n = 0, up_h = 0, up_w = 0;
  int st_n = 0, st_h = 0, st_w = 0;
  bool st_precise = false;     // the staged results come from op_run_staged_precise
  int st_net_w = 0, st_net_h = 0;
  float* d_maps = nullptr;
  size_t maps_bytes = 0;
  int sm_n = 0, sm_h = 0, sm_w = 0;
  float* d_fmaps = nullptr;  // staged full-resolution maps for the precise post-process, planar (n, 57, h, w)
  size_t fmaps_bytes = 0;
  int fm_n = 0, fm_h = 0, fm_w = 0;
  bool use_maps = false;
  float* d_scratch = nullptr;
  size_t scratch_bytes = 0;
  // timing
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
  bool timed = false;
  // per-class launch profiling
  bool prof = false;
  int splitk = 1;  // op_set_batch_invariant(0): small 7x7 launches may split K
  int prof_mask = 0x7F;  // kernel classes timed while prof (op_profile_classes)
  // set by the forward around launches it issues back to back (the 7x7 Mconv1..Mconv5 of a stage):
  // a profiled launch then extends the previous pair of its class instead of adding an event pair
  // (an event record between two kernels costs ~10 us of stream idle time on this runtime)
  bool prof_join = false;
  std::vector<hipEvent_t> ev_pool;
  size_t ev_used = 0;
  std::vector<op::ProfPair> pending;
  double prof_ms[OP_PROFILE_CLASSES] = {}, prof_flops[OP_PROFILE_CLASSES] = {}, prof_bytes[OP_PROFILE_CLASSES] = {};
  int64_t prof_n[OP_PROFILE_CLASSES] = {};
  // graph
  hipGraphExec_t gexec = nullptr;
  hipGraph_t graph = nullptr;
  uintptr_t g_key[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  // multi-scale path: per-scale map intermediates and the running sums over scales
  float* d_pmid = nullptr;
  size_t pmid_bytes = 0;
  float* d_psum = nullptr;
  size_t psum_bytes = 0;
  // pinned host staging for batched result fetches
  char* host_stage = nullptr;
  size_t host_stage_bytes = 0;
  // pinned host staging for the one-frame uploads of op_detect / op_detect_precise: the caller's
  // (pageable, possibly row-strided) image is packed here by the host and copied with one plain
  // async copy on the compute stream -- no pageable or 2D copy path of the HIP runtime is involved
  uint8_t* up_pinned = nullptr;
  size_t up_pinned_bytes = 0;
  // uncapped post-process: the last batched post-process's input (to re-run one frame) and the
  // one-frame big-mode buffers sized from that frame's own counts
  op::PostRecord post_rec;
  op::KeepSlot keep[2];
  PostBuffers bigb{};
  void* bb_arena = nullptr;
  int big_frame = -1;  // frame of post_rec whose big-mode result sits in bb
};

namespace op {

static size_t geom_floats(op_ctx* c, int n, int h, int w, Act* out, bool split) {
  // (pad, channel stride, scale divisor) per buffer
  struct D {
    int pad, cs, div;
  };
  const D d[B_COUNT] = {{1, 8, 1},   {1, 64, 1},  {0, 64, 1},  {1, 64, 2},  {1, 128, 2}, {0, 128, 2},
                        {1, 128, 4}, {1, 256, 4}, {1, 256, 4}, {0, 256, 4}, {1, 256, 8}, {1, 512, 8},
                        {1, 512, 8}, {1, 256, 8}, {kStagePad, kCatStride, 8}, {kStagePad, 256, 8},
                        {kStagePad, 256, 8}, {0, 1024, 8}, {0, 64, 8}, {kStagePad, 256, 8}, {kStagePad, 256, 8},
                        {kStagePad, kCatStride, 8}};
  size_t total = 0;
  for (int i = 0; i < B_COUNT; ++i) {
    Act a;
    a.pad = d[i].pad;
    a.cs = (i == B_X0 && split) ? 16 : d[i].cs;
    a.h = h / d[i].div;
    a.w = w / d[i].div;
    a.planar = (i == B_PA || i == B_PB || i == B_CATP) ? 1 : 0;  // the 7x7 inputs of stages 2-6
    const size_t fl = a.frame_floats() * (size_t)n;
    if (out) {
      out[i] = a;
      out[i].p = nullptr;
    }
    total += (fl + 63) / 64 * 64 + g_guard / 4;  // 256-B alignment (+ debug guard band)
  }
  (void)c;
  return total;
}

static const char* const kBufName[B_COUNT] = {"X0",  "C11", "C12", "P1",  "C21", "C22", "P2",  "C3A", "C3B", "C34",
                                              "P3",  "C41", "C42", "C43", "CAT", "BRA", "BRB", "S1",  "MAP32",
                                              "PA",  "PB",  "CATP"};

static int ensure_geometry(op_ctx* c, int n, int h, int w) {
  if (h % 8 || w % 8 || h < 16 || w < 16 || n < 1) {
    set_error("network input must be >= 16 and a multiple of 8");
    return OP_ERR_INVALID;
  }
  if (c->gn == n && c->gh == h && c->gw == w && c->gsplit == c->split) return OP_OK;
  Act a[B_COUNT];
  const size_t need = geom_floats(c, n, h, w, a, c->split) * sizeof(float);
  op_ctx::GeomArena* ga = nullptr;
  for (auto& e : c->arenas)
    if (e.n == n && e.h == h && e.w == w && e.split == c->split) ga = &e;
  if (!ga) {
    // bounded cache: at most 6 geometries / 96 GiB of arenas, least recently used evicted first
    const size_t cap_bytes = (size_t)96 << 30;
    for (;;) {
      size_t tot = need;
      for (auto& e : c->arenas) tot += e.bytes;
      if (c->arenas.empty() || (c->arenas.size() < 6 && tot <= cap_bytes)) break;
      size_t lru = 0;
      for (size_t i = 1; i < c->arenas.size(); ++i)
        if (c->arenas[i].used < c->arenas[lru].used) lru = i;
      // every stream that may still read the arena: the compute stream and the upload ring's copy
      // stream (which touches only d_ring, but hipFree must not race any queued work)
      OP_HIP_CHECK(hipStreamSynchronize(c->stream));
      if (c->main_stream) OP_HIP_CHECK(hipStreamSynchronize(c->main_stream));
      if (c->side_stream) OP_HIP_CHECK(hipStreamSynchronize(c->side_stream));
      if (c->copy_stream) OP_HIP_CHECK(hipStreamSynchronize(c->copy_stream));
      guard_forget(c->arenas[lru].p, c->arenas[lru].bytes);
      OP_HIP_CHECK(hipFree(c->arenas[lru].p));
      c->arenas.erase(c->arenas.begin() + lru);
    }
    void* p = nullptr;
    OP_HIP_CHECK(hipMalloc(&p, need));
    // zero halos (and everything else) once per geometry; kernels only ever write interiors
    OP_HIP_CHECK(hipMemsetAsync(p, 0, need, c->stream));
    c->arenas.push_back(op_ctx::GeomArena{n, h, w, c->split, p, need, 0});
    ga = &c->arenas.back();
  }
  ga->used = ++c->arena_clock;
  if (c->arena) guard_forget(c->arena, c->arena_bytes);
  c->arena = ga->p;
  c->arena_bytes = ga->bytes;
  float* p = (float*)c->arena;
  for (int i = 0; i < B_COUNT; ++i) {
    a[i].p = p;
    const size_t fl = a[i].frame_floats() * (size_t)n;
    p += (fl + 63) / 64 * 64;
    guard_add(kBufName[i], p, c->stream);
    p += g_guard / 4;
    c->buf[i] = a[i];
  }
  c->gn = n;
  c->gh = h;
  c->gw = w;
  c->gsplit = c->split;
  return OP_OK;
}

// The device Gaussian table (PostBuffers::gauss_w): the CPU-branch taps (scipy's normalised 2r + 1)
// at 0, the GPU-branch 1-D factor (op_set_peak_mode) at kGaussGpuOff
static std::vector<double> gauss_table(const op_ctx* c) {
  // (a sigma whose radius passes kMaxR -- 2r + 1 > 33 taps -- is refused by check_shape before any
  // launch; its table is cut at the region's end rather than written past it)
  std::vector<double> t(op::kGaussTable, 0.0);
  const size_t nc = std::min<size_t>(c->gauss_host.size(), op::kGaussGpuOff);
  const size_t ng = std::min<size_t>(c->gpu_taps.size(), op::kGaussTable - op::kGaussGpuOff);
  std::copy(c->gauss_host.begin(), c->gauss_host.begin() + nc, t.begin());
  std::copy(c->gpu_taps.begin(), c->gpu_taps.begin() + ng, t.begin() + op::kGaussGpuOff);
  return t;
}

static int ensure_post(op_ctx* c, int n, int mh, int mw) {
  if (c->pn >= n && c->pmh * c->pmw >= mh * mw && c->pb.up) return OP_OK;
  const int nn = std::max(n, c->pn), area = std::max(mh * mw, c->pmh * c->pmw);
  PostBuffers b{};
  b.maxp = c->lim.max_peaks_per_joint;
  b.maxc = (int64_t)b.maxp * b.maxp;
  b.maxs = OP_N_LIMBS * b.maxp;
  if (b.maxs > 2048) b.maxs = 2048;
  struct Part {
    void** p;
    size_t bytes;
  };
  const size_t plane = (size_t)nn * OP_N_JOINTS * area * sizeof(float);
  std::vector<Part> parts = {
      {(void**)&b.up, plane},
      {(void**)&b.peak_xy, (size_t)nn * OP_N_JOINTS * b.maxp * 4},
      {(void**)&b.peak_score, (size_t)nn * OP_N_JOINTS * b.maxp * 4},
      {(void**)&b.peak_cnt, (size_t)nn * OP_N_JOINTS * 4},
      {(void**)&b.stage_key, (size_t)nn * OP_N_JOINTS * b.maxp * 4},
      {(void**)&b.stage_score, (size_t)nn * OP_N_JOINTS * b.maxp * 4},
      {(void**)&b.cand_score, (size_t)nn * OP_N_LIMBS * b.maxc * 8},
      {(void**)&b.cand_idx, (size_t)nn * OP_N_LIMBS * b.maxc * 4},
      {(void**)&b.cand_cnt, (size_t)nn * OP_N_LIMBS * 4},
      {(void**)&b.conn_ab, (size_t)nn * OP_N_LIMBS * b.maxp * 8},
      {(void**)&b.conn_score, (size_t)nn * OP_N_LIMBS * b.maxp * 8},
      {(void**)&b.conn_cnt, (size_t)nn * OP_N_LIMBS * 4},
      {(void**)&b.sub_ids, 16},
      {(void**)&b.sub_sc, 16},
      {(void**)&b.res_poses, (size_t)nn * b.maxs * OP_N_JOINTS * 3 * 8},
      {(void**)&b.res_scores, (size_t)nn * b.maxs * 8},
      {(void**)&b.res_subsets, (size_t)nn * b.maxs * 20 * 8},
      {(void**)&b.res_hdr, (size_t)nn * 4 * 4},
      {(void**)&b.gauss_w, op::kGaussTable * 8},
  };
  static const char* const part_name[] = {"up",       "peak_xy",    "peak_score",
                                          "peak_cnt", "stage_key", "stage_score", "cand_score", "cand_idx",
                                          "cand_cnt", "conn_ab",   "conn_score", "conn_cnt",   "sub_ids",
                                          "sub_sc",   "res_poses", "res_scores", "res_subsets", "res_hdr",
                                          "gauss_w"};
  size_t total = 0;
  for (auto& q : parts) total += (q.bytes + 255) / 256 * 256 + g_guard;
  OP_HIP_CHECK(hipStreamSynchronize(c->stream));
  if (c->post_arena) {
    guard_forget(c->post_arena, c->post_bytes);
    OP_HIP_CHECK(hipFree(c->post_arena));
  }
  c->post_arena = nullptr;
  OP_HIP_CHECK(hipMalloc(&c->post_arena, total));
  c->post_bytes = total;
  OP_HIP_CHECK(hipMemset(c->post_arena, 0, total));
  char* p = (char*)c->post_arena;
  for (size_t i = 0; i < parts.size(); ++i) {
    *parts[i].p = p;
    p += (parts[i].bytes + 255) / 256 * 256;
    guard_add(part_name[i], p, nullptr);
    p += g_guard;
  }
  OP_HIP_CHECK(hipDeviceSynchronize());
  const std::vector<double> gt = gauss_table(c);
  OP_HIP_CHECK(hipMemcpy(b.gauss_w, gt.data(), gt.size() * 8, hipMemcpyHostToDevice));
  c->pb = b;
  c->pn = nn;
  c->pmh = mh;
  c->pmw = area / mh;
  if (c->gexec) {
    hipGraphExecDestroy(c->gexec);
    c->gexec = nullptr;
  }
  return OP_OK;
}

// (Re)allocate a growable device buffer of `bytes` (+ debug guard band after it).
static int grow_buffer(op_ctx* c, void** p, size_t* cap, size_t bytes, const char* name) {
  if (bytes <= *cap) return OP_OK;
  OP_HIP_CHECK(hipStreamSynchronize(c->stream));
  if (c->main_stream) OP_HIP_CHECK(hipStreamSynchronize(c->main_stream));
  if (c->side_stream) OP_HIP_CHECK(hipStreamSynchronize(c->side_stream));
  if (*p) {
    guard_forget(*p, *cap + g_guard);
    OP_HIP_CHECK(hipFree(*p));
  }
  *p = nullptr;
  *cap = 0;  // a failed allocation below leaves no buffer, and says so
  OP_HIP_CHECK(hipMalloc(p, bytes + g_guard));
  *cap = bytes;
  guard_add(name, (char*)*p + bytes, nullptr);
  OP_HIP_CHECK(hipDeviceSynchronize());
  return OP_OK;
}

static int ensure_scratch(op_ctx* c, size_t bytes) {
  return grow_buffer(c, (void**)&c->d_scratch, &c->scratch_bytes, bytes, "scratch");
}

// ---- forward plan ----
static ConvGroup grp(const Act& in, int cin_off, const Act& out, int cout_off, const PackedConv& pc, int cout_store) {
  ConvGroup g;
  g.in = in.p + cin_off;
  g.out = out.p + cout_off;
  g.w = pc.w;
  g.bias = pc.b;
  g.cop = pc.cop;
  g.cout_store = cout_store;
  return g;
}

static ConvShape shp(int n, const Act& in, const Act& out, int c8, int ks, bool relu, int groups) {
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
  s.groups = groups;
  return s;
}

static hipEvent_t pool_event(op_ctx* c) {
  if (c->ev_used == c->ev_pool.size()) {
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    c->ev_pool.push_back(e);
  }
  return c->ev_pool[c->ev_used++];
}

// Record an event pair around `fn`'s launches when profiling is on.
template <class Fn>
static int profiled(op_ctx* c, int cls, double flops, double bytes, Fn fn) {
  if (!c->prof || !((c->prof_mask >> cls) & 1)) return fn();
  if (c->prof_join && !c->pending.empty() && c->pending.back().cls == cls) {
    ProfPair& p = c->pending.back();  // the previous launch of this run ended with p.b: move p.b past fn
    const int rc = fn();
    OP_HIP_CHECK(hipEventRecord(p.b, c->stream));
    p.flops += flops;
    p.bytes += bytes;
    p.n += 1;
    return rc;
  }
  hipEvent_t a = pool_event(c), b = pool_event(c);
  if (!a || !b) return fn();
  OP_HIP_CHECK(hipEventRecord(a, c->stream));
  const int rc = fn();
  OP_HIP_CHECK(hipEventRecord(b, c->stream));
  c->pending.push_back(ProfPair{cls, a, b, flops, bytes, 1});
  return rc;
}

static int conv_class(int ks) { return ks == 7 ? 0 : (ks == 3 ? 1 : 2); }
// the other op_profile_read classes (openpose_hip.h)
constexpr int kProfPost = 3, kProfInput = 4, kProfMapResize = 5, kProfOther = 6;

// algorithmic work of one conv group: 2*Ci*Co*k*k*N*H*W FLOPs; bytes = input + output + weights (fp32)
static void conv_work(const op_ctx* c, const Act& out, const PackedConv& pc, double* flops, double* bytes) {
  const double px = (double)c->gn * out.h * out.w;
  *flops += 2.0 * pc.cin_log * pc.co_log * pc.ks * pc.ks * px;
  *bytes += 4.0 * (px * pc.cin_log + px * pc.co_log + (double)pc.cin_log * pc.co_log * pc.ks * pc.ks + pc.co_log);
}

// first channel `off` (a multiple of 8) of a split tensor, in floats from its base, for its layout
static size_t chan_offset(const Act& a, int off) {
  return a.planar ? (size_t)off * (a.h + 2 * a.pad) * (a.w + 2 * a.pad) : (size_t)off;
}

static SplitConvGroup sgrp(const Act& in, int cin_off, const Act& out, int cout_off, const PackedConv& pc,
                          int cout_store) {
  SplitConvGroup g;
  g.in = in.p + chan_offset(in, cin_off);
  g.out = out.p + chan_offset(out, cout_off);
  g.w = pc.ws;
  g.bias = pc.b;
  g.cop = pc.cop;
  g.cout_store = cout_store;
  g.cin_off = cin_off;
  g.out32 = nullptr;
  g.out32_off = 0;
  return g;
}

// Default split-path conv kernel family of new contexts (op_set_conv_algo; OP_HALO_MODE env).
static int g_halo_mode = 4;

static SplitConvShape sshp(int n, const Act& in, const Act& out, int c16, int ks, bool relu, int groups, int algo,
                           int splitk) {
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
  s.groups = groups;
  s.cs_out32 = 0;
  s.halo_mode = algo == 5 ? 4 : algo;  // 5: the default family without the register-weight kernels
  s.regw = algo == 4 ? 1 : 0;
  s.splitk = splitk;
  s.in_planar = in.planar;
  s.out_planar = out.planar;
  return s;
}

static int conv1(op_ctx* c, const Act& in, int cin_off, const Act& out, int cout_off, const PackedConv& pc, int store,
                 bool relu) {
  if (c->split) {
    SplitConvGroup g[2];
    g[0] = sgrp(in, cin_off, out, cout_off, pc, store);
    g[1] = g[0];
    double fl = 0, by = 0;
    conv_work(c, out, pc, &fl, &by);
    return profiled(c, conv_class(pc.ks), fl, by, [&] {
      return launch_conv_bf16x3(sshp(c->gn, in, out, pc.cin16 / 16, pc.ks, relu, 1, c->conv_algo, c->splitk), g, c->stream);
    });
  }
  ConvGroup g[2];
  g[0] = grp(in, cin_off, out, cout_off, pc, store);
  g[1] = g[0];
  double fl = 0, by = 0;
  conv_work(c, out, pc, &fl, &by);
  return profiled(c, conv_class(pc.ks), fl, by,
                  [&] { return launch_conv(shp(c->gn, in, out, pc.cin_phys / 8, pc.ks, relu, 1), g, c->stream); });
}

static int pool(op_ctx* c, const Act& in, const Act& out, int ch);

// conv (3x3, ReLU) followed by F.max_pooling_2d(2) (CocoPoseNet.py:137-138, 140-141, 145-146):
// one fused launch on the split path with the conv_big families (the pooled tensor is the only
// output), else the conv into `full` and the pool kernel.
static int conv_pool(op_ctx* c, const Act& in, const Act& full, const Act& pooled, const PackedConv& pc, int ch) {
  if (c->split && (c->conv_algo == 4 || c->conv_algo == 5)) {
    SplitConvGroup g[2];
    g[0] = sgrp(in, 0, pooled, 0, pc, ch);
    g[1] = g[0];
    SplitConvShape sh = sshp(c->gn, in, full, pc.cin16 / 16, pc.ks, true, 1, c->conv_algo, c->splitk);
    sh.pout = pooled.pad;
    sh.cs_out = pooled.cs;
    double fl = 0, by = 0;
    conv_work(c, full, pc, &fl, &by);
    int taken = 0;
    const int rc = profiled(c, conv_class(pc.ks), fl, by, [&] {
      return launch_conv_big_pool(sh, g, c->stream, &taken);
    });
    if (rc || taken) return rc;
  }
  const int rc = conv1(c, in, 0, full, 0, pc, ch, true);
  return rc ? rc : pool(c, full, pooled, ch);
}

static int conv2(op_ctx* c, const Act& in, int ci0, int ci1, const Act& out, int co0, int co1, const PackedConv& p0,
                 const PackedConv& p1, int st0, int st1, bool relu, const Act* out32 = nullptr, int o32a = 0,
                 int o32b = 0) {
  if (c->split) {
    SplitConvGroup g[2];
    g[0] = sgrp(in, ci0, out, co0, p0, st0);
    g[1] = sgrp(in, ci1, out, co1, p1, st1);
    SplitConvShape sh = sshp(c->gn, in, out, p0.cin16 / 16, p0.ks, relu, 2, c->conv_algo, c->splitk);
    if (out32) {
      g[0].out32 = g[1].out32 = out32->p;
      g[0].out32_off = o32a;
      g[1].out32_off = o32b;
      sh.cs_out32 = out32->cs;
    }
    double fl = 0, by = 0;
    conv_work(c, out, p0, &fl, &by);
    conv_work(c, out, p1, &fl, &by);
    return profiled(c, conv_class(p0.ks), fl, by, [&] { return launch_conv_bf16x3(sh, g, c->stream); });
  }
  ConvGroup g[2];
  g[0] = grp(in, ci0, out, co0, p0, st0);
  g[1] = grp(in, ci1, out, co1, p1, st1);
  double fl = 0, by = 0;
  conv_work(c, out, p0, &fl, &by);
  conv_work(c, out, p1, &fl, &by);
  return profiled(c, conv_class(p0.ks), fl, by,
                  [&] { return launch_conv(shp(c->gn, in, out, p0.cin_phys / 8, p0.ks, relu, 2), g, c->stream); });
}

#define RC(x)            \
  do {                   \
    int _r = (x);        \
    if (_r) return _r;   \
  } while (0)

// Fused 1x1 pair per branch (conv5_4+conv5_5, Mconv6+Mconv7): in -> a (ReLU) -> b -> out, the
// intermediate kept on chip (conv_head.hip).  Returns -1 when not taken (the caller then runs the
// two convs through `mid`).  OP_HEAD_FUSED=0 disables it (A/B).
static bool head_fused_on() {  // read per forward (not cached): the parity tests A/B it in-process
  const char* e = getenv("OP_HEAD_FUSED");
  return !(e && atoi(e) == 0);
}

static int head2(op_ctx* c, const Act& in, int ci0, int ci1, const Act& out, int co0, int co1,
                 const PackedConv* a, const PackedConv* b, int st0, int st1, const Act* out32, int o32a, int o32b) {
  if (!head_fused_on()) return -1;
  if (!c->split) {  // exact f32: conv_head_f32 (bit-identical to the two conv2 launches)
    if (out32 || a[0].ks != 1 || b[0].ks != 1 || a[0].cop % 128 || a[0].cop != a[1].cop ||
        b[0].cin_phys != a[0].cop || b[1].cin_phys != a[1].cop || b[0].cop != b[1].cop)
      return -1;
    HeadF32Shape s;
    s.n = c->gn;
    s.h = out.h;
    s.w = out.w;
    s.pin = in.pad;
    s.cs_in = in.cs;
    s.pout = out.pad;
    s.cs_out = out.cs;
    s.c8 = a[0].cin_phys / 8;
    s.co1 = a[0].cop;
    s.groups = 2;
    HeadF32Group g[2];
    const int cis[2] = {ci0, ci1}, cos[2] = {co0, co1}, sts[2] = {st0, st1};
    for (int i = 0; i < 2; ++i) {
      g[i].in = in.p + cis[i];
      g[i].w1 = a[i].w;
      g[i].b1 = a[i].b;
      g[i].cop1 = a[i].cop;
      g[i].w2 = b[i].w;
      g[i].b2 = b[i].b;
      g[i].cop2 = b[i].cop;
      g[i].out = out.p + cos[i];
      g[i].cout_store = sts[i];
    }
    double fl = 0, by = 0;
    for (int i = 0; i < 2; ++i) {
      conv_work(c, out, a[i], &fl, &by);
      conv_work(c, out, b[i], &fl, &by);
    }
    const int rc = profiled(c, 2, fl, by, [&] { return launch_conv_head_f32(s, g, c->stream); });
    return rc ? rc : 0;
  }
  HeadShape s;
  s.n = c->gn;
  s.h = out.h;
  s.w = out.w;
  s.pin = in.pad;
  s.cs_in = in.cs;
  s.pout = out.pad;
  s.cs_out = out.cs;
  s.ci = a[0].cin16;
  s.co1 = a[0].cop;
  s.groups = 2;
  s.cs_out32 = out32 ? out32->cs : 0;
  s.in_planar = in.planar;
  s.out_planar = out.planar;
  HeadGroup g[2];
  const int cis[2] = {ci0, ci1}, cos[2] = {co0, co1}, sts[2] = {st0, st1}, o32[2] = {o32a, o32b};
  for (int i = 0; i < 2; ++i) {
    g[i].in = in.p + chan_offset(in, cis[i]);
    g[i].w1 = a[i].ws;
    g[i].b1 = a[i].b;
    g[i].cop1 = a[i].cop;
    g[i].w2 = b[i].ws;
    g[i].b2 = b[i].b;
    g[i].cop2 = b[i].cop;
    g[i].out = out.p + chan_offset(out, cos[i]);
    g[i].cout_store = sts[i];
    g[i].out32 = out32 ? out32->p : nullptr;
    g[i].out32_off = o32[i];
  }
  double fl = 0, by = 0;
  for (int i = 0; i < 2; ++i) {
    conv_work(c, out, a[i], &fl, &by);
    conv_work(c, out, b[i], &fl, &by);
  }
  int taken = 0;
  const int rc = profiled(c, 2, fl, by, [&] { return launch_conv_head(s, g, c->stream, &taken); });
  return rc ? rc : (taken ? 0 : -1);
}

static int pool(op_ctx* c, const Act& in, const Act& out, int ch) {
  return profiled(c, kProfOther, 0.0, 0.0, [&] {
    if (c->split) return launch_maxpool2_split(in.p, in.pad, out.p, out.pad, c->gn, in.h, in.w, ch, c->stream);
    return launch_maxpool2(in.p, in.pad, out.p, out.pad, c->gn, in.h, in.w, ch, c->stream);
  });
}

// frames != nullptr (split path): conv1_1 reads the uint8 frames directly (fused input kernel).
// stages != nullptr: every stage's (paf, heat) is also extracted to stages = paf [6][n][38][lh][lw]
// followed by heat [6][n][19][lh][lw] (op_forward_stages; the reference's pafs / heatmaps lists).
static int run_forward(op_ctx* c, const uint8_t* frames = nullptr, int64_t frame_bytes = 0, int64_t row_stride = 0,
                       int sh = 0, int sw = 0, float* stages = nullptr) {
  c->post_rec.kind = 0;  // the maps a recorded post-process read are overwritten from here on
  Act* B = c->buf;
  const size_t stage_px = (size_t)c->gn * (c->gh / 8) * (c->gw / 8);
  auto dump_stage = [&](int s) -> int {
    if (!stages) return OP_OK;
    float* paf = stages + (size_t)s * 38 * stage_px;
    float* heat = stages + (size_t)6 * 38 * stage_px + (size_t)s * 19 * stage_px;
    if (c->split) return launch_extract_maps32(B[B_MAP32].p, 64, 40, c->gn, c->gh / 8, c->gw / 8, paf, heat, c->stream);
    return launch_extract_maps(B[B_CAT].p, c->gn, c->gh / 8, c->gw / 8, paf, heat, c->stream);
  };
  static const bool c11_mfma = getenv("OP_CONV11_MFMA") != nullptr;  // debugging aid: the MFMA conv1_1
  // conv1_1 + conv1_2 + pool in one launch (conv1_pair.hip); OP_CONV1_FUSED=0: the two-kernel path
  static const bool c1_fused = !(getenv("OP_CONV1_FUSED") && atoi(getenv("OP_CONV1_FUSED")) == 0);
  bool conv1_done = false;
  if (c->split && c1_fused && !c11_mfma && (c->conv_algo == 4 || c->conv_algo == 5)) {
    const Act& o = B[B_C11];
    double fl = 0, by = 0;
    conv_work(c, o, c->bb[0], &fl, &by);
    conv_work(c, o, c->bb[1], &fl, &by);
    RC(profiled(c, conv_class(3), fl, by, [&] {
      return launch_conv1_pair(frames, frame_bytes, row_stride, sh, sw, B[B_X0].p, c->gn, o.h, o.w, c->w11,
                               c->bb[0].b, c->bb[1].ws, c->bb[1].b, B[B_P1].p, B[B_P1].pad, c->stream);
    }));
    conv1_done = true;
  } else if (c->split && !(c11_mfma && !frames)) {
    const Act& o = B[B_C11];
    double fl = 0, by = 0;
    conv_work(c, o, c->bb[0], &fl, &by);
    RC(profiled(c, conv_class(3), fl, by, [&] {
      return launch_conv11_split(frames, frame_bytes, row_stride, sh, sw, B[B_X0].p, c->gn, o.h, o.w, c->w11,
                                 c->bb[0].b, o.p, c->stream);
    }));
  } else {
    RC(conv1(c, B[B_X0], 0, B[B_C11], 0, c->bb[0], 64, true));
  }
  if (!conv1_done) RC(conv_pool(c, B[B_C11], B[B_C12], B[B_P1], c->bb[1], 64));
  RC(conv1(c, B[B_P1], 0, B[B_C21], 0, c->bb[2], 128, true));
  RC(conv_pool(c, B[B_C21], B[B_C22], B[B_P2], c->bb[3], 128));
  RC(conv1(c, B[B_P2], 0, B[B_C3A], 0, c->bb[4], 256, true));
  RC(conv1(c, B[B_C3A], 0, B[B_C3B], 0, c->bb[5], 256, true));
  RC(conv1(c, B[B_C3B], 0, B[B_C3A], 0, c->bb[6], 256, true));
  RC(conv_pool(c, B[B_C3A], B[B_C34], B[B_P3], c->bb[7], 256));
  RC(conv1(c, B[B_P3], 0, B[B_C41], 0, c->bb[8], 512, true));
  RC(conv1(c, B[B_C41], 0, B[B_C42], 0, c->bb[9], 512, true));
  RC(conv1(c, B[B_C42], 0, B[B_C43], 0, c->bb[10], 256, true));
  RC(conv1(c, B[B_C43], 0, B[B_CAT], kCatFeat, c->bb[11], 128, true));
  // Stages 2-6 run their 7x7 layers on chunk-planar tensors when conv_m16_bf16x3 takes every 7x7
  // launch of this geometry and the fused heads write the stage maps (op_set_stage_layout(ctx, 0)
  // or OP_STAGE_PLANAR=0: the [pixel][channels] buffers): Mconv1..Mconv5 outputs in PA / PB, and the Mconv1 input
  // (the 185-channel concat) in CATP -- the feature slice copied over from CAT once per forward
  // (stage 1's conv5_1 reads it from CAT), every stage's (paf, heat) written there by its head.
  const int sh8 = B[B_BRA].h, sw8 = B[B_BRA].w;
  const bool planar = c->split && (c->conv_algo == 4 || c->conv_algo == 5) && c->stage_planar && head_fused_on() &&
                      conv_m16_takes(c->gn, sh8, sw8, 1, 256) && conv_m16_takes(c->gn, sh8, sw8, 2, 128);
  if (planar)
    RC(profiled(c, kProfOther, 0.0, 0.0, [&] {
      return launch_split_to_planar(B[B_CAT].p, B[B_CATP].p, c->gn, sh8, sw8, B[B_CAT].pad, B[B_CAT].cs, 128 / 16,
                                    c->stream);
    }));
  const Act& catm = planar ? B[B_CATP] : B[B_CAT];  // stage maps + Mconv1 input
  // stage 1 (CocoPoseNet.py:153-165)
  const Act& cat = B[B_CAT];
  Act s1 = B[B_S1];
  RC(conv1(c, cat, kCatFeat, B[B_BRA], 0, c->s1_first, 256, true));
  RC(conv2(c, B[B_BRA], 0, 128, B[B_BRB], 0, 128, c->s1_g[0][0], c->s1_g[1][0], 128, 128, true));
  RC(conv2(c, B[B_BRB], 0, 128, B[B_BRA], 0, 128, c->s1_g[0][1], c->s1_g[1][1], 128, 128, true));
  {
    const Act* m32 = (c->split && stages) ? &B[B_MAP32] : nullptr;
    const PackedConv a[2] = {c->s1_g[0][2], c->s1_g[1][2]}, b[2] = {c->s1_last[0], c->s1_last[1]};
    const int h = head2(c, B[B_BRA], 0, 128, catm, kCatPaf, kCatHeat, a, b, 40, 20, m32, 0, 40);
    if (h > 0) return h;
    if (h < 0) {
      RC(conv2(c, B[B_BRA], 0, 128, s1, 0, 512, c->s1_g[0][2], c->s1_g[1][2], 512, 512, true));
      RC(conv2(c, s1, 0, 512, catm, kCatPaf, kCatHeat, c->s1_last[0], c->s1_last[1], 40, 20, false, m32, 0, 40));
    }
    RC(dump_stage(0));
  }
  // stages 2-6 (CocoPoseNet.py:167-260), on the chunk-planar buffers when `planar` (above)
  Act s6 = B[B_S1];
  s6.cs = 256;  // Mconv6 output reuses the stage-1 1x1 buffer (no halo) with a 256-channel stride
  const Act& SA = planar ? B[B_PA] : B[B_BRA];
  const Act& SB = planar ? B[B_PB] : B[B_BRB];
  for (int st = 0; st < 5; ++st) {
    RC(conv1(c, catm, 0, SA, 0, c->st_first[st], 256, true));
    const Act* src = &SA;
    const Act* dst = &SB;
    c->prof_join = true;  // Mconv2..Mconv5 follow Mconv1 back to back on the stream
    for (int i = 0; i < 4; ++i) {
      const int r = conv2(c, *src, 0, 128, *dst, 0, 128, c->st_g[st][0][i], c->st_g[st][1][i], 128, 128, true);
      if (r) {
        c->prof_join = false;
        return r;
      }
      std::swap(src, dst);
    }
    c->prof_join = false;
    // the last stage also leaves a dense f32 copy (paf at 0, heat at 40) for the post-process
    const Act* m32 = (c->split && (st == 4 || stages)) ? &B[B_MAP32] : nullptr;
    const PackedConv a[2] = {c->st_g[st][0][4], c->st_g[st][1][4]}, b[2] = {c->st_last[st][0], c->st_last[st][1]};
    const int h = head2(c, *src, 0, 128, catm, kCatPaf, kCatHeat, a, b, 40, 20, m32, 0, 40);
    if (h > 0) return h;
    if (h < 0) {
      RC(conv2(c, *src, 0, 128, s6, 0, 128, c->st_g[st][0][4], c->st_g[st][1][4], 128, 128, true));
      RC(conv2(c, s6, 0, 128, catm, kCatPaf, kCatHeat, c->st_last[st][0], c->st_last[st][1], 40, 20, false, m32, 0,
               40));
    }
    RC(dump_stage(st + 1));
  }
  return OP_OK;
}

static void post_shape(op_ctx* c, PostShape& s, int n, int lh, int lw, int mh, int mw, double img_len, double sx,
                       double sy) {
  s.n = n;
  s.lh = lh;
  s.lw = lw;
  s.mh = mh;
  s.mw = mw;
  s.radius = c->gauss_r;
  s.peak_mode = c->peak_mode;
  s.gpu_radius = c->gpu_r;
  s.img_len = img_len;
  s.sx = sx;
  s.sy = sy;
  s.peak_thresh = (float)c->prm.heatmap_peak_thresh;
  s.n_integ = c->prm.n_integ_points;
  s.n_integ_thresh = c->prm.n_integ_points_thresh;
  s.inner_thresh = c->prm.inner_product_thresh;
  s.len_ratio = c->prm.limb_length_ratio;
  s.len_penalty = c->prm.length_penalty_value;
  s.subset_min = c->prm.n_subset_limbs_thresh;
  s.subset_score = c->prm.subset_score_thresh;
  memcpy(s.limbs, c->prm.limbs_point, sizeof(s.limbs));
}

// compute_optimal_size (pose_detector.py:57-73); np.round is half-to-even (nearbyint).
static void optimal_size(int h, int w, int img_size, int stride, int* out_w, int* out_h) {
  const double aspect = (double)h / (double)w;
  int iw, ih;
  if (h < w) {
    ih = img_size;
    iw = (int)std::nearbyint((double)img_size / aspect);
    const int sur = iw % stride;
    if (sur) iw += stride - sur;
  } else {
    iw = img_size;
    ih = (int)std::nearbyint((double)img_size * aspect);
    const int sur = ih % stride;
    if (sur) ih += stride - sur;
  }
  *out_w = iw;
  *out_h = ih;
}

// ---- uncapped post-process (the reference has no caps, pose_detector.py:75-250) ----
// A frame whose peaks per joint exceed the batched buffers' cap, or whose subsets overflow the
// LDS grouping, is re-run alone in "big mode": one-frame buffers sized from its own counts (peaks
// per joint, candidates per limb, subsets <= connections + 1), greedy bitsets and subsets in HBM,
// a rank sort for the peak lists.  Only device memory bounds it (OP_ERR_CAPACITY if an allocation
// fails).
static int big_buffers(op_ctx* c, int maxp, int64_t maxc, PostBuffers** out) {
  maxp = std::max(maxp, 1);
  maxc = std::max<int64_t>(maxc, 1);
  if (c->bb_arena && c->bigb.maxp >= maxp && c->bigb.maxc >= maxc) {
    *out = &c->bigb;
    return OP_OK;
  }
  if (c->bb_arena) {
    maxp = std::max(maxp, c->bigb.maxp);
    maxc = std::max(maxc, c->bigb.maxc);
  }
  if ((int64_t)maxp * maxp >= ((int64_t)1 << 31)) {  // candidate pair indices are int32
    set_error("more than 46340 peaks for one joint");
    return OP_ERR_CAPACITY;
  }
  PostBuffers b{};
  b.maxp = maxp;
  b.maxc = maxc;
  b.maxs = OP_N_LIMBS * maxp + 1;  // every new subset consumes a connection (<= maxp per limb)
  const size_t words = ((size_t)maxp + 31) / 32, P = (size_t)maxp, S = (size_t)b.maxs, C = (size_t)maxc;
  struct Part {
    void** p;
    size_t bytes;
  };
  const Part parts[] = {
      {(void**)&b.peak_xy, OP_N_JOINTS * P * 4},   {(void**)&b.peak_score, OP_N_JOINTS * P * 4},
      {(void**)&b.peak_cnt, OP_N_JOINTS * 4},      {(void**)&b.stage_key, OP_N_JOINTS * P * 4},
      {(void**)&b.stage_score, OP_N_JOINTS * P * 4}, {(void**)&b.cand_score, OP_N_LIMBS * C * 8},
      {(void**)&b.cand_idx, OP_N_LIMBS * C * 4},   {(void**)&b.cand_cnt, OP_N_LIMBS * 4},
      {(void**)&b.conn_ab, OP_N_LIMBS * P * 8},    {(void**)&b.conn_score, OP_N_LIMBS * P * 8},
      {(void**)&b.conn_cnt, OP_N_LIMBS * 4},       {(void**)&b.sub_ids, S * OP_N_JOINTS * 4},
      {(void**)&b.sub_sc, S * 2 * 8},              {(void**)&b.res_poses, S * OP_N_JOINTS * 3 * 8},
      {(void**)&b.res_scores, S * 8},              {(void**)&b.res_subsets, S * 20 * 8},
      {(void**)&b.res_hdr, 4 * 4},                 {(void**)&b.gauss_w, op::kGaussTable * 8},
      {(void**)&b.used, OP_N_LIMBS * 2 * words * 4},
  };
  size_t total = 0;
  for (const Part& q : parts) total += (q.bytes + 255) / 256 * 256;
  OP_HIP_CHECK(hipStreamSynchronize(c->stream));
  if (c->bb_arena) OP_HIP_CHECK(hipFree(c->bb_arena));
  c->bb_arena = nullptr;
  c->bigb = PostBuffers{};
  c->big_frame = -1;
  if (hipMalloc(&c->bb_arena, total) != hipSuccess) {
    (void)hipGetLastError();
    c->bb_arena = nullptr;
    set_error("post-process of a frame needs more device memory than is free (" + std::to_string(total >> 20) +
              " MiB for " + std::to_string(maxp) + " peaks per joint)");
    return OP_ERR_CAPACITY;
  }
  char* p = (char*)c->bb_arena;
  for (const Part& q : parts) {
    *q.p = p;
    p += (q.bytes + 255) / 256 * 256;
  }
  const std::vector<double> gt = gauss_table(c);
  OP_HIP_CHECK(hipMemcpy(b.gauss_w, gt.data(), gt.size() * 8, hipMemcpyHostToDevice));
  c->bigb = b;
  *out = &c->bigb;
  return OP_OK;
}

// Run the post-process of `peaks` (frame 0 of B) from the recorded input of frame f.
static int post_one_frame(op_ctx* c, const PostRecord& r, int f, PostBuffers& B) {
  PostShape s1 = r.s;
  s1.n = 1;
  if (r.kind == 1) {
    MapSource src = r.low;
    src.base += (int64_t)f * src.fstride;
    return launch_post_maps(src, s1, B, c->stream);
  }
  const float* m = r.full + (int64_t)f * r.fstride;
  RC(launch_peaks_from_full(m + (size_t)OP_N_PAF * s1.mh * s1.mw, OP_N_JOINTS, s1.mh, s1.mw, s1, B, c->stream,
                            r.fstride));
  RC(launch_connections_full(m, s1.mh, s1.mw, s1, B, c->stream, r.fstride));
  return launch_grouping(s1, B, c->stream);
}

// Re-run frame f of the recorded post-process input r in big mode, sizing the buffers from the
// frame's batched peak counts at d_cnt (18 int32); *out = buffers holding its result.
static int rerun_big_rec(op_ctx* c, const PostRecord& r, int f, const int32_t* d_cnt, PostBuffers** out) {
  if (r.kind == 0 || f < 0 || f >= r.s.n) {
    set_error("post-process capacity exceeded and no recorded input to re-run the frame");
    return OP_ERR_CAPACITY;
  }
  OP_HIP_CHECK(hipStreamSynchronize(c->stream));
  int32_t cnt[OP_N_JOINTS];
  OP_HIP_CHECK(hipMemcpy(cnt, d_cnt, sizeof(cnt), hipMemcpyDeviceToHost));
  int maxp = 1;
  for (int j = 0; j < OP_N_JOINTS; ++j) maxp = std::max(maxp, cnt[j]);
  int64_t maxc = std::min<int64_t>((int64_t)maxp * maxp, (int64_t)1 << 20);
  PostBuffers* B = nullptr;
  c->big_frame = -1;
  for (;;) {
    RC(big_buffers(c, maxp, maxc, &B));
    RC(post_one_frame(c, r, f, *B));
    int32_t cc[OP_N_LIMBS];
    OP_HIP_CHECK(hipMemcpyAsync(cc, B->cand_cnt, sizeof(cc), hipMemcpyDeviceToHost, c->stream));
    OP_HIP_CHECK(hipStreamSynchronize(c->stream));
    int64_t need = 0;
    for (int l = 0; l < OP_N_LIMBS; ++l) need = std::max<int64_t>(need, cc[l]);
    if (need <= B->maxc) break;
    maxc = need;  // more candidates than the first guess: grow and run again
  }
  *out = B;
  return OP_OK;
}

// Re-run frame f of the last batched post-process in big mode (cached per frame).
static int rerun_big(op_ctx* c, int f, PostBuffers** out) {
  if (c->big_frame == f && c->bb_arena) {
    *out = &c->bigb;
    return OP_OK;
  }
  if (c->post_rec.kind == 0 || f < 0 || f >= c->post_rec.s.n) {
    set_error("post-process capacity exceeded and no recorded input to re-run the frame");
    return OP_ERR_CAPACITY;
  }
  RC(rerun_big_rec(c, c->post_rec, f, c->pb.peak_cnt + (size_t)f * OP_N_JOINTS, out));
  c->big_frame = f;
  return OP_OK;
}

// The result of a one-frame big-mode buffer set (frame 0 of B) into the caller's arrays.
static int read_big(PostBuffers* B, double* poses, double* scores, int cap, op_frame_result* res) {
  int32_t hdr[4];
  OP_HIP_CHECK(hipMemcpy(hdr, B->res_hdr, sizeof(hdr), hipMemcpyDeviceToHost));
  res->status = hdr[0];
  res->n_peaks = hdr[1];
  res->n_persons = hdr[0] == OP_OK ? hdr[2] : 0;
  if (hdr[0] != OP_OK) {
    set_error(hdr[0] == OP_ERR_INDEX ? "list assignment index out of range (grouping_key_points)"
                                     : "post-process capacity exceeded (peaks per joint / subsets)");
    return hdr[0];
  }
  if (hdr[2] > cap) {
    set_error("result capacity too small");
    return OP_ERR_CAPACITY;
  }
  if (hdr[2] > 0) {
    OP_HIP_CHECK(hipMemcpy(poses, B->res_poses, (size_t)hdr[2] * 54 * 8, hipMemcpyDeviceToHost));
    OP_HIP_CHECK(hipMemcpy(scores, B->res_scores, (size_t)hdr[2] * 8, hipMemcpyDeviceToHost));
  }
  return OP_OK;
}

static void post_record(op_ctx* c, int kind, const MapSource* low, const float* full, int64_t fstride,
                        const PostShape& s) {
  c->post_rec.kind = kind;
  if (low) c->post_rec.low = *low;
  c->post_rec.full = full;
  c->post_rec.fstride = fstride;
  c->post_rec.s = s;
  c->big_frame = -1;
}

static int read_result(op_ctx* c, int frame, double* poses, double* scores, int cap, op_frame_result* res) {
  int32_t hdr[4];
  OP_HIP_CHECK(hipMemcpy(hdr, c->pb.res_hdr + 4 * frame, sizeof(hdr), hipMemcpyDeviceToHost));
  const PostBuffers* B = &c->pb;
  int slot = frame;
  if (hdr[0] == OP_ERR_CAPACITY && c->post_rec.kind) {  // over the batched caps: re-run uncapped
    PostBuffers* big = nullptr;
    RC(rerun_big(c, frame, &big));
    OP_HIP_CHECK(hipMemcpy(hdr, big->res_hdr, sizeof(hdr), hipMemcpyDeviceToHost));
    B = big;
    slot = 0;
  }
  res->status = hdr[0];
  res->n_peaks = hdr[1];
  res->n_persons = hdr[2];
  if (hdr[0] != OP_OK) {
    set_error(hdr[0] == OP_ERR_INDEX ? "list assignment index out of range (grouping_key_points)"
                                     : "post-process capacity exceeded (peaks per joint / subsets)");
    return hdr[0];
  }
  if (hdr[2] > cap) {
    set_error("result capacity too small");
    return OP_ERR_CAPACITY;
  }
  if (hdr[2] > 0) {
    OP_HIP_CHECK(hipMemcpy(poses, B->res_poses + (size_t)slot * B->maxs * 54, (size_t)hdr[2] * 54 * 8,
                           hipMemcpyDeviceToHost));
    OP_HIP_CHECK(hipMemcpy(scores, B->res_scores + (size_t)slot * B->maxs, (size_t)hdr[2] * 8,
                           hipMemcpyDeviceToHost));
  }
  return OP_OK;
}

static int check_ctx(op_ctx* c, bool need_weights) {
  if (!c) {
    set_error("null context");
    return OP_ERR_INVALID;
  }
  if (need_weights && !c->have_weights) {
    set_error("weights not set (op_set_weights)");
    return OP_ERR_STATE;
  }
  OP_HIP_CHECK(hipSetDevice(c->device));
  return OP_OK;
}

}  // namespace op

// =============================== C ABI ===============================
extern "C" {

const char* op_last_error(void) { return op::g_err.c_str(); }

int op_default_params(op_params* p) {
  if (!p) return OP_ERR_INVALID;
  memset(p, 0, sizeof(*p));
  p->inference_img_size = 368;
  p->heatmap_size = 320;
  p->gaussian_sigma = 2.5;
  p->n_integ_points = 10;
  p->n_integ_points_thresh = 8;
  p->heatmap_peak_thresh = 0.05;
  p->inner_product_thresh = 0.05;
  p->limb_length_ratio = 1.0;
  p->length_penalty_value = 1.0;
  p->n_subset_limbs_thresh = 3;
  p->subset_score_thresh = 0.2;
  static const int32_t limbs[OP_N_LIMBS][2] = {{1, 8},  {8, 9},   {9, 10}, {1, 11},  {11, 12}, {12, 13}, {1, 2},
                                               {2, 3},  {3, 4},   {2, 16}, {1, 5},   {5, 6},   {6, 7},   {5, 17},
                                               {1, 0},  {0, 14},  {0, 15}, {14, 16}, {15, 17}};
  memcpy(p->limbs_point, limbs, sizeof(limbs));
  p->downscale = 8;
  p->n_scales = 4;
  p->inference_scales[0] = 0.5;
  p->inference_scales[1] = 1.0;
  p->inference_scales[2] = 1.5;
  p->inference_scales[3] = 2.0;
  return OP_OK;
}

int op_default_limits(op_limits* l) {
  if (!l) return OP_ERR_INVALID;
  l->max_batch = 1;
  l->max_net_h = 368;
  l->max_net_w = 656;
  l->max_map_h = 320;
  l->max_map_w = 576;
  l->max_peaks_per_joint = 512;
  l->max_frame_h = 720;
  l->max_frame_w = 1280;
  return OP_OK;
}

int op_layer_info(int index, const char** name, int32_t* ci, int32_t* co, int32_t* ksize) {
  const auto& L = op::layers();
  if (index < 0 || index >= (int)L.size()) return OP_ERR_INVALID;
  if (name) *name = L[index].name;
  if (ci) *ci = L[index].ci;
  if (co) *co = L[index].co;
  if (ksize) *ksize = L[index].k;
  return OP_OK;
}

double op_forward_flops(int32_t h, int32_t w) {
  double f = 0.0;
  const auto& L = op::layers();
  for (size_t i = 0; i < L.size(); ++i) {
    int div = 8;
    if (i < 2) div = 1;
    else if (i < 4) div = 2;
    else if (i < 8) div = 4;
    const double hw = (double)(h / div) * (double)(w / div);
    f += 2.0 * L[i].ci * L[i].co * L[i].k * L[i].k * hw;
  }
  return f;
}

int op_create(const op_params* params, const op_limits* limits, int device, op_ctx** out) {
  if (!out) return OP_ERR_INVALID;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
    op::set_error("no HIP device available (this path runs on MI355X only)");
    return OP_ERR_HIP;
  }
  if (device < 0 || device >= ndev) {
    op::set_error("device ordinal out of range");
    return OP_ERR_INVALID;
  }
  op_ctx* c = new op_ctx();
  c->device = device;
  if (params) c->prm = *params;
  else op_default_params(&c->prm);
  op_default_limits(&c->lim);
  if (limits) {
    if (limits->max_batch > 0) c->lim.max_batch = limits->max_batch;
    if (limits->max_net_h > 0) c->lim.max_net_h = limits->max_net_h;
    if (limits->max_net_w > 0) c->lim.max_net_w = limits->max_net_w;
    if (limits->max_map_h > 0) c->lim.max_map_h = limits->max_map_h;
    if (limits->max_map_w > 0) c->lim.max_map_w = limits->max_map_w;
    if (limits->max_peaks_per_joint > 0) c->lim.max_peaks_per_joint = limits->max_peaks_per_joint;
    if (limits->max_frame_h > 0) c->lim.max_frame_h = limits->max_frame_h;
    if (limits->max_frame_w > 0) c->lim.max_frame_w = limits->max_frame_w;
  }
  if (c->lim.max_peaks_per_joint > 2048 || c->prm.n_integ_points > 16 || c->prm.n_integ_points < 2 ||
      c->prm.n_scales < 0 || c->prm.n_scales > OP_MAX_SCALES || c->prm.downscale != 8) {
    op::set_error("parameters outside kernel support (max_peaks_per_joint <= 2048, 2 <= n_integ_points <= 16, "
                  "n_scales <= OP_MAX_SCALES, downscale == 8)");
    delete c;
    return OP_ERR_INVALID;
  }
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    op::set_error("hipStreamCreate failed");
    delete c;
    return OP_ERR_HIP;
  }
  if (op::conv_big_device_init(device) != OP_OK) {
    hipStreamDestroy(c->stream);
    delete c;
    return OP_ERR_HIP;
  }
  for (int i = 0; i < 4; ++i) hipEventCreate(&c->ev[i]);
  if (const char* e = getenv("OP_HALO_MODE")) {
    const int m = atoi(e);
    if (m == 0 || m == 3 || m == 4 || m == 5) op::g_halo_mode = m;
  }
  c->conv_algo = op::g_halo_mode;
  c->stage_planar = !(getenv("OP_STAGE_PLANAR") && atoi(getenv("OP_STAGE_PLANAR")) == 0);
  if (const char* e = getenv("OP_DEBUG_SYNC")) op::g_debug_sync = e[0] == '1';
  if (const char* e = getenv("OP_GUARD")) op::g_guard = ((size_t)atol(e) + 255) / 256 * 256;
  // scipy _gaussian_kernel1d(sigma, 0, int(4*sigma + 0.5)) taps (restated; pinned by the tests)
  c->gauss_r = op::gaussian_taps(c->prm.gaussian_sigma, c->gauss_host);
  *out = c;
  return OP_OK;
}

static void free_pc(op::PackedConv& p) {
  if (p.w) hipFree(p.w);
  if (p.b) hipFree(p.b);
  if (p.ws) hipFree(p.ws);
  p.w = p.b = nullptr;
  p.ws = nullptr;
}

static void free_weights(op_ctx* c) {
  if (c->w11) hipFree(c->w11);
  c->w11 = nullptr;
  for (auto& p : c->bb) free_pc(p);
  free_pc(c->s1_first);
  for (auto& a : c->s1_g)
    for (auto& p : a) free_pc(p);
  for (auto& p : c->s1_last) free_pc(p);
  for (auto& p : c->st_first) free_pc(p);
  for (auto& a : c->st_g)
    for (auto& b : a)
      for (auto& p : b) free_pc(p);
  for (auto& a : c->st_last)
    for (auto& p : a) free_pc(p);
  c->have_weights = false;
}

int op_destroy(op_ctx* c) {
  if (!c) return OP_OK;
  hipSetDevice(c->device);
  if (c->stream) hipStreamSynchronize(c->stream);
  if (c->side_stream) hipStreamSynchronize(c->side_stream);
  if (c->copy_stream) hipStreamSynchronize(c->copy_stream);
  if (c->gexec) hipGraphExecDestroy(c->gexec);
  if (c->graph) hipGraphDestroy(c->graph);
  free_weights(c);
  for (auto& e : c->arenas) {
    guard_forget(e.p, e.bytes);
    hipFree(e.p);
  }
  c->arenas.clear();
  c->arena = nullptr;
  guard_forget(c->post_arena, c->post_bytes);
  guard_forget(c->d_frames, c->frames_bytes + g_guard);
  guard_forget(c->d_maps, c->maps_bytes + g_guard);
  guard_forget(c->d_scratch, c->scratch_bytes + g_guard);
  guard_forget(c->d_fmaps, c->fmaps_bytes + g_guard);
  if (c->post_arena) hipFree(c->post_arena);
  if (c->d_frames) hipFree(c->d_frames);
  if (c->d_maps) hipFree(c->d_maps);
  if (c->d_fmaps) hipFree(c->d_fmaps);
  if (c->d_scratch) hipFree(c->d_scratch);
  guard_forget(c->d_pmid, c->pmid_bytes + g_guard);
  guard_forget(c->d_psum, c->psum_bytes + g_guard);
  if (c->d_pmid) hipFree(c->d_pmid);
  if (c->d_psum) hipFree(c->d_psum);
  if (c->host_stage) hipHostFree(c->host_stage);
  if (c->up_pinned) hipHostFree(c->up_pinned);
  for (auto& k : c->keep) {
    if (k.h_rows) hipHostFree(k.h_rows);
    if (k.maps) hipFree(k.maps);
    if (k.res) hipFree(k.res);
    if (k.cnt) hipFree(k.cnt);
    if (k.d_hdr) hipFree(k.d_hdr);
    if (k.h_hdr) hipHostFree(k.h_hdr);
  }
  if (c->bb_arena) hipFree(c->bb_arena);
  for (auto& e : c->ev)
    if (e) hipEventDestroy(e);
  for (auto& e : c->ev_pool) hipEventDestroy(e);
  if (c->copy_stream) {
    (void)hipStreamSynchronize(c->copy_stream);
    (void)hipStreamDestroy(c->copy_stream);
  }
  if (c->side_stream) {
    (void)hipStreamSynchronize(c->side_stream);
    splitk_ws_release(c->side_stream);
    (void)hipStreamDestroy(c->side_stream);
  }
  if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
  if (c->ev_join) (void)hipEventDestroy(c->ev_join);
  for (int i = 0; i < 2; ++i) {
    if (c->d_ring[i]) (void)hipFree(c->d_ring[i]);
    if (c->ev_up[i]) (void)hipEventDestroy(c->ev_up[i]);
    if (c->ev_free[i]) (void)hipEventDestroy(c->ev_free[i]);
  }
  if (c->stream) {
    (void)hipStreamSynchronize(c->stream);
    splitk_ws_release(c->stream);
    hipStreamDestroy(c->stream);
  }
  delete c;
  return OP_OK;
}

int op_set_weights(op_ctx* c, const float* const* W, const float* const* b) {
  using namespace op;
  int rc = check_ctx(c, false);
  if (rc) return rc;
  if (!W || !b) {
    set_error("null weights");
    return OP_ERR_INVALID;
  }
  for (int i = 0; i < OP_N_LAYERS; ++i)
    if (!W[i] || !b[i]) {
      set_error(std::string("missing weights for layer ") + layers()[i].name);
      return OP_ERR_INVALID;
    }
  free_weights(c);
  const auto& L = layers();
  auto single = [&](PackedConv& pc, int li, bool cat_in) -> int {
    const LayerDef& d = L[li];
    pc.ks = d.k;
    pc.cin_phys = cat_in ? kCatStride : round_up(d.ci, 8);
    pc.cop = round_up(d.co, 64);
    pc.cin_log = d.ci;
    pc.co_log = d.co;
    pc.cin16 = cat_in ? kCatStride : round_up(d.ci, 16);
    std::vector<float> w((size_t)pc.cin_phys * d.k * d.k * pc.cop, 0.0f), bias(pc.cop, 0.0f);
    pack_into(w, bias, pc.cop, pc.cin_phys, d.k, W[li], b[li], d.co, d.ci, 0, cat_in);
    std::vector<uint16_t> ws((size_t)pc.cin16 * d.k * d.k * pc.cop * 2, 0);
    pack_split_into(ws, pc.cop, pc.cin16, d.k, W[li], d.co, d.ci, 0, cat_in);
    RC(upload_split(pc, ws));
    return upload(pc, w, bias);
  };
  auto fused = [&](PackedConv& pc, int l1, int l2, bool cat_in) -> int {
    const LayerDef& d = L[l1];
    pc.ks = d.k;
    pc.cin_phys = cat_in ? kCatStride : round_up(d.ci, 8);
    pc.cop = 2 * d.co;
    pc.cin_log = d.ci;
    pc.co_log = 2 * d.co;
    pc.cin16 = cat_in ? kCatStride : round_up(d.ci, 16);
    std::vector<float> w((size_t)pc.cin_phys * d.k * d.k * pc.cop, 0.0f), bias(pc.cop, 0.0f);
    pack_into(w, bias, pc.cop, pc.cin_phys, d.k, W[l1], b[l1], d.co, d.ci, 0, cat_in);
    pack_into(w, bias, pc.cop, pc.cin_phys, d.k, W[l2], b[l2], d.co, d.ci, d.co, cat_in);
    std::vector<uint16_t> ws((size_t)pc.cin16 * d.k * d.k * pc.cop * 2, 0);
    pack_split_into(ws, pc.cop, pc.cin16, d.k, W[l1], d.co, d.ci, 0, cat_in);
    pack_split_into(ws, pc.cop, pc.cin16, d.k, W[l2], d.co, d.ci, d.co, cat_in);
    RC(upload_split(pc, ws));
    return upload(pc, w, bias);
  };
  for (int i = 0; i < 12; ++i) RC(single(c->bb[i], i, false));
  {  // conv1_1 for the VALU kernel: [tap][ci][co]
    std::vector<float> w11(9 * 3 * 64);
    for (int co = 0; co < 64; ++co)
      for (int ci = 0; ci < 3; ++ci)
        for (int t = 0; t < 9; ++t) w11[(t * 3 + ci) * 64 + co] = W[0][(co * 3 + ci) * 9 + t];
    OP_HIP_CHECK(hipMalloc(&c->w11, w11.size() * sizeof(float)));
    OP_HIP_CHECK(hipMemcpy(c->w11, w11.data(), w11.size() * sizeof(float), hipMemcpyHostToDevice));
  }
  const char* br[2] = {"L1", "L2"};
  RC(fused(c->s1_first, layer_index("conv5_1_CPM_L1"), layer_index("conv5_1_CPM_L2"), false));
  for (int bi = 0; bi < 2; ++bi) {
    for (int k = 0; k < 3; ++k)
      RC(single(c->s1_g[bi][k], layer_index("conv5_" + std::to_string(k + 2) + "_CPM_" + br[bi]), false));
    RC(single(c->s1_last[bi], layer_index(std::string("conv5_5_CPM_") + br[bi]), false));
  }
  for (int s = 0; s < 5; ++s) {
    const std::string st = "_stage" + std::to_string(s + 2) + "_";
    RC(fused(c->st_first[s], layer_index("Mconv1" + st + "L1"), layer_index("Mconv1" + st + "L2"), true));
    for (int bi = 0; bi < 2; ++bi) {
      for (int k = 0; k < 5; ++k) RC(single(c->st_g[s][bi][k], layer_index("Mconv" + std::to_string(k + 2) + st + br[bi]), false));
      RC(single(c->st_last[s][bi], layer_index("Mconv7" + st + br[bi]), false));
    }
  }
  c->have_weights = true;
  return OP_OK;
}

int op_preprocess(op_ctx* c, const uint8_t* bgr, int32_t h, int32_t w, int64_t row_stride, int32_t out_w,
                  int32_t out_h, float* x_out) {
  using namespace op;
  RC(check_ctx(c, false));
  if (!bgr || !x_out || h < 1 || w < 1 || out_w < 1 || out_h < 1 || row_stride < (int64_t)w * 3) {
    set_error("op_preprocess: bad arguments");
    return OP_ERR_INVALID;
  }
  const size_t in_bytes = (size_t)h * w * 3, out_bytes = (size_t)3 * out_h * out_w * 4;
  RC(ensure_scratch(c, in_bytes + 256 + out_bytes));
  uint8_t* din = (uint8_t*)c->d_scratch;
  float* dout = (float*)((char*)c->d_scratch + (in_bytes + 255) / 256 * 256);
  OP_HIP_CHECK(hipMemcpy2DAsync(din, (size_t)w * 3, bgr, (size_t)row_stride, (size_t)w * 3, h, hipMemcpyHostToDevice,
                                c->stream));
  RC(launch_preprocess_planar(din, (int64_t)w * 3, h, w, out_h, out_w, dout, c->stream));
  OP_HIP_CHECK(hipMemcpyAsync(x_out, dout, out_bytes, hipMemcpyDeviceToHost, c->stream));
  OP_HIP_CHECK(hipStreamSynchronize(c->stream));
  return OP_OK;
}

int op_forward_stages(op_ctx* c, const float* x, int32_t n, int32_t h, int32_t w, float* pafs, float* heatmaps) {
  using namespace op;
  RC(check_ctx(c, true));
  if (!x || !pafs || !heatmaps) {
    set_error("op_forward_stages: null pointer");
    return OP_ERR_INVALID;
  }
  RC(ensure_geometry(c, n, h, w));
  const size_t xin = (size_t)n * 3 * h * w * 4;
  const size_t px = (size_t)n * (h / 8) * (w / 8);
  const size_t outb = 6 * 57 * px * 4;
  RC(ensure_scratch(c, xin + 256 + outb));
  float* dx = c->d_scratch;
  float* dst = (float*)((char*)c->d_scratch + (xin + 255) / 256 * 256);
  OP_HIP_CHECK(hipMemcpyAsync(dx, x, xin, hipMemcpyHostToDevice, c->stream));
  if (c->split)
    RC(launch_nchw_to_split16(dx, c->buf[B_X0].p, n, h, w, c->stream));
  else
    RC(launch_nchw_to_nhwc8(dx, c->buf[B_X0].p, n, h, w, c->stream));
  RC(run_forward(c, nullptr, 0, 0, 0, 0, dst));
  OP_HIP_CHECK(hipMemcpyAsync(pafs, dst, 6 * 38 * px * 4, hipMemcpyDeviceToHost, c->stream));
  OP_HIP_CHECK(hipMemcpyAsync(heatmaps, dst + 6 * 38 * px, 6 * 19 * px * 4, hipMemcpyDeviceToHost, c->stream));
  OP_HIP_CHECK(hipStreamSynchronize(c->stream));
  return OP_OK;
}

int op_forward(op_ctx* c, const float* x, int32_t n, int32_t h, int32_t w, float* pafs, float* heatmaps) {
  using namespace op;
  RC(check_ctx(c, true));
  if (!x || !pafs || !heatmaps) {
    set_error("op_forward: null pointer");
    return OP_ERR_INVALID;
  }
  RC(ensure_geometry(c, n, h, w));
  const size_t xin = (size_t)n * 3 * h * w * 4;
  const int lh = h / 8, lw = w / 8;
  const size_t outb = (size_t)n * 57 * lh * lw * 4;
  RC(ensure_scratch(c, xin + 256 + outb));
  float* dx = c->d_scratch;
  float* dmaps = (float*)((char*)c->d_scratch + (xin + 255) / 256 * 256);
  OP_HIP_CHECK(hipMemcpyAsync(dx, x, xin, hipMemcpyHostToDevice, c->stream));
  if (c->split)
    RC(launch_nchw_to_split16(dx, c->buf[B_X0].p, n, h, w, c->stream));
  else
    RC(launch_nchw_to_nhwc8(dx, c->buf[B_X0].p, n, h, w, c->stream));
  RC(run_forward(c));
  float* dpaf = dmaps;
  float* dheat = dmaps + (size_t)n * 38 * lh * lw;
  if (c->split)
    RC(launch_extract_maps32(c->buf[B_MAP32].p, 64, 40, n, lh, lw, dpaf, dheat, c->stream));
  else
    RC(launch_extract_maps(c->buf[B_CAT].p, n, lh, lw, dpaf, dheat, c->stream));
  OP_HIP_CHECK(hipMemcpyAsync(pafs, dpaf, (size_t)n * 38 * lh * lw * 4, hipMemcpyDeviceToHost, c->stream));
  OP_HIP_CHECK(hipMemcpyAsync(heatmaps, dheat, (size_t)n * 19 * lh * lw * 4, hipMemcpyDeviceToHost, c->stream));
  OP_HIP_CHECK(hipStreamSynchronize(c->stream));
  return OP_OK;
}

int op_resize_images(op_ctx* c, const float* x, int32_t ch, int32_t h, int32_t w, int32_t oh, int32_t ow, float* y) {
  using namespace op;
  RC(check_ctx(c, false));
  if (!x || !y || ch < 1 || h < 2 || w < 2 || oh < 1 || ow < 1) {
    set_error("op_resize_images: bad arguments");
    return OP_ERR_INVALID;
  }
  const size_t inb = (size_t)ch * h * w * 4, outb = (size_t)ch * oh * ow * 4;
  RC(ensure_scratch(c, inb + 256 + outb));
  float* din = c->d_scratch;
  float* dout = (float*)((char*)c->d_scratch + (inb + 255) / 256 * 256);
  OP_HIP_CHECK(hipMemcpyAsync(din, x, inb, hipMemcpyHostToDevice, c->stream));
  RC(launch_resize_images(din, ch, h, w, oh, ow, dout, c->stream));
  OP_HIP_CHECK(hipMemcpyAsync(y, dout, outb, hipMemcpyDeviceToHost, c->stream));
  OP_HIP_CHECK(hipStreamSynchronize(c->stream));
  return OP_OK;
}

// Peaks per joint of (N,5) all_peaks rows (reference format: ordered by joint, ids = row index);
// OP_ERR_INVALID if the rows are not in that format.
static int peaks_per_joint(const double* peaks, int64_t n, int32_t* cnt) {
  for (int j = 0; j < OP_N_JOINTS; ++j) cnt[j] = 0;
  int prev = -1;
  for (int64_t i = 0; i < n; ++i) {
    const double* r = peaks + i * 5;
    const int j = (int)r[0];
    if (j < 0 || j >= OP_N_JOINTS || j < prev || (int64_t)r[4] != i || r[1] < 0 || r[2] < 0 || r[1] > 0xffff ||
        r[2] > 0x7fff) {
      set_error("peaks must be all_peaks rows [joint, x, y, score, id] ordered by joint with id = row");
      return OP_ERR_INVALID;
    }
    prev = j;
    cnt[j]++;
  }
  return OP_OK;
}

// The context's batched post buffers when maxp peaks per joint fit them (and !force_big), else the
// one-frame big-mode buffers sized for maxp / maxc (uncapped: only device memory bounds them).
static int pick_buffers(op_ctx* c, int maxp, int64_t maxc, bool force_big, PostBuffers** out) {
  if (!force_big && maxp <= c->pb.maxp && maxc <= c->pb.maxc) {
    *out = &c->pb;
    return OP_OK;
  }
  return big_buffers(c, std::max(maxp, c->pb.maxp), std::max<int64_t>(maxc, 1), out);
}

// Upload all_peaks rows into the per-joint peak arrays of frame 0 of B.
static int upload_peaks(op_ctx* c, PostBuffers& B, const double* peaks, int64_t n) {
  using namespace op;
  const int maxp = B.maxp;
  std::vector<int32_t> xy((size_t)OP_N_JOINTS * maxp, 0), cnt(OP_N_JOINTS, 0);
  std::vector<float> sc((size_t)OP_N_JOINTS * maxp, 0.0f);
  for (int64_t i = 0; i < n; ++i) {
    const double* r = peaks + i * 5;
    const int j = (int)r[0];
    if (cnt[j] >= maxp) {
      set_error("internal: peak buffers smaller than the peaks per joint");
      return OP_ERR_INVALID;
    }
    xy[(size_t)j * maxp + cnt[j]] = (int32_t)r[1] | ((int32_t)r[2] << 16);
    sc[(size_t)j * maxp + cnt[j]] = (float)r[3];
    cnt[j]++;
  }
  OP_HIP_CHECK(hipMemcpyAsync(B.peak_xy, xy.data(), xy.size() * 4, hipMemcpyHostToDevice, c->stream));
  OP_HIP_CHECK(hipMemcpyAsync(B.peak_score, sc.data(), sc.size() * 4, hipMemcpyHostToDevice, c->stream));
  OP_HIP_CHECK(hipMemcpyAsync(B.peak_cnt, cnt.data(), cnt.size() * 4, hipMemcpyHostToDevice, c->stream));
  OP_HIP_CHECK(hipStreamSynchronize(c->stream));
  return OP_OK;
}

int op_compute_peaks(op_ctx* c, const float* heatmaps, int32_t ch, int32_t h, int32_t w, double* peaks, int64_t cap,
                     int64_t* n_peaks) {
  using namespace op;
  RC(check_ctx(c, false));
  if (!heatmaps || !n_peaks || ch != OP_N_JOINTS + 1 || h < 2 || w < 2) {
    set_error("op_compute_peaks: heatmaps must be (19, h, w)");
    return OP_ERR_INVALID;
  }
  RC(ensure_post(c, 1, h, w));
  OP_HIP_CHECK(hipMemcpyAsync(c->pb.up, heatmaps, (size_t)OP_N_JOINTS * h * w * 4, hipMemcpyHostToDevice, c->stream));
  PostShape s;
  post_shape(c, s, 1, h, w, h, w, (double)w, 1.0, 1.0);
  PostBuffers* B = &c->pb;
  std::vector<int32_t> cnt(OP_N_JOINTS);
  for (;;) {
    RC(launch_peaks_from_full(c->pb.up, OP_N_JOINTS, h, w, s, *B, c->stream));
    OP_HIP_CHECK(hipMemcpyAsync(cnt.data(), B->peak_cnt, cnt.size() * 4, hipMemcpyDeviceToHost, c->stream));
    OP_HIP_CHECK(hipStreamSynchronize(c->stream));
    const int most = *std::max_element(cnt.begin(), cnt.end());
    if (most <= B->maxp) break;
    RC(pick_buffers(c, most, 1, true, &B));  // more peaks than the cap: again, uncapped
  }
  const int maxp = B->maxp;
  std::vector<int32_t> xy((size_t)OP_N_JOINTS * maxp);
  std::vector<float> sc((size_t)OP_N_JOINTS * maxp);
  OP_HIP_CHECK(hipMemcpyAsync(xy.data(), B->peak_xy, xy.size() * 4, hipMemcpyDeviceToHost, c->stream));
  OP_HIP_CHECK(hipMemcpyAsync(sc.data(), B->peak_score, sc.size() * 4, hipMemcpyDeviceToHost, c->stream));
  OP_HIP_CHECK(hipStreamSynchronize(c->stream));
  int64_t total = 0;
  for (int j = 0; j < OP_N_JOINTS; ++j) total += cnt[j];
  if (total > cap) {  // the caller's rows are too few: report how many are needed
    *n_peaks = total;
    set_error("peaks capacity too small");
    return OP_ERR_CAPACITY;
  }
  int64_t k = 0;
  for (int j = 0; j < OP_N_JOINTS; ++j) {
    for (int i = 0; i < cnt[j]; ++i) {
      const int32_t v = xy[(size_t)j * maxp + i];
      double* r = peaks + k * 5;
      r[0] = j;
      r[1] = v & 0xffff;
      r[2] = v >> 16;
      r[3] = (double)sc[(size_t)j * maxp + i];
      r[4] = (double)k;
      ++k;
    }
  }
  *n_peaks = k;
  return OP_OK;
}

int op_compute_connections(op_ctx* c, const float* pafs, int32_t h, int32_t w, const double* peaks, int64_t n_peaks,
                           double img_len, double* conn, int64_t cap, int64_t* conn_off) {
  using namespace op;
  RC(check_ctx(c, false));
  if (!pafs || !conn_off || (n_peaks > 0 && !peaks) || h < 1 || w < 1) {
    set_error("op_compute_connections: bad arguments");
    return OP_ERR_INVALID;
  }
  RC(ensure_post(c, 1, h, w));
  int32_t pj[OP_N_JOINTS];
  RC(peaks_per_joint(peaks, n_peaks, pj));
  const int most = *std::max_element(pj, pj + OP_N_JOINTS);
  const size_t pb = (size_t)OP_N_PAF * h * w * 4;
  RC(ensure_scratch(c, pb));
  OP_HIP_CHECK(hipMemcpyAsync(c->d_scratch, pafs, pb, hipMemcpyHostToDevice, c->stream));
  PostShape s;
  post_shape(c, s, 1, h, w, h, w, img_len, 1.0, 1.0);
  PostBuffers* B = nullptr;
  int64_t maxc = std::min<int64_t>((int64_t)most * most, (int64_t)1 << 20);
  RC(pick_buffers(c, most, most <= c->pb.maxp ? 1 : maxc, false, &B));
  std::vector<int32_t> ccnt(OP_N_LIMBS);
  for (;;) {
    RC(upload_peaks(c, *B, peaks, n_peaks));
    RC(launch_connections_full(c->d_scratch, h, w, s, *B, c->stream));
    OP_HIP_CHECK(hipMemcpyAsync(ccnt.data(), B->cand_cnt, ccnt.size() * 4, hipMemcpyDeviceToHost, c->stream));
    OP_HIP_CHECK(hipStreamSynchronize(c->stream));
    const int64_t need = *std::max_element(ccnt.begin(), ccnt.end());
    if (need <= B->maxc) break;
    RC(pick_buffers(c, most, need, true, &B));  // more candidates than the buffers hold: again
  }
  const int maxp = B->maxp;
  std::vector<int32_t> cnt(OP_N_LIMBS), ab((size_t)OP_N_LIMBS * maxp * 2);
  std::vector<double> sc((size_t)OP_N_LIMBS * maxp);
  OP_HIP_CHECK(hipMemcpyAsync(cnt.data(), B->conn_cnt, cnt.size() * 4, hipMemcpyDeviceToHost, c->stream));
  OP_HIP_CHECK(hipMemcpyAsync(ab.data(), B->conn_ab, ab.size() * 4, hipMemcpyDeviceToHost, c->stream));
  OP_HIP_CHECK(hipMemcpyAsync(sc.data(), B->conn_score, sc.size() * 8, hipMemcpyDeviceToHost, c->stream));
  OP_HIP_CHECK(hipStreamSynchronize(c->stream));
  int64_t total = 0;
  for (int l = 0; l < OP_N_LIMBS; ++l) total += cnt[l];
  if (total > cap) {  // the caller's rows are too few: report how many are needed
    conn_off[OP_N_LIMBS] = total;
    set_error("connection capacity too small");
    return OP_ERR_CAPACITY;
  }
  int64_t k = 0;
  for (int l = 0; l < OP_N_LIMBS; ++l) {
    conn_off[l] = k;
    for (int i = 0; i < cnt[l]; ++i) {
      conn[k * 3 + 0] = ab[((size_t)l * maxp + i) * 2];
      conn[k * 3 + 1] = ab[((size_t)l * maxp + i) * 2 + 1];
      conn[k * 3 + 2] = sc[(size_t)l * maxp + i];
      ++k;
    }
  }
  conn_off[OP_N_LIMBS] = k;
  return OP_OK;
}

int op_grouping(op_ctx* c, const double* conn, const int64_t* conn_off, const double* peaks, int64_t n_peaks,
                double* subsets, int64_t cap, int64_t* n_subsets) {
  using namespace op;
  RC(check_ctx(c, false));
  if (!conn_off || !n_subsets || (n_peaks > 0 && !peaks)) {
    set_error("op_grouping: bad arguments");
    return OP_ERR_INVALID;
  }
  // map size is irrelevant for grouping; keep whatever post buffers exist
  RC(ensure_post(c, 1, std::max(c->pmh, 8), std::max(c->pmw, 8)));
  int32_t pj[OP_N_JOINTS];
  RC(peaks_per_joint(peaks, n_peaks, pj));
  int most = *std::max_element(pj, pj + OP_N_JOINTS);
  // peak id ranges per joint (ids are row indices of all_peaks, grouped by joint)
  int64_t jlo[OP_N_JOINTS], jhi[OP_N_JOINTS];
  for (int j = 0; j < OP_N_JOINTS; ++j) {
    jlo[j] = 0;
    jhi[j] = -1;
  }
  for (int64_t i = n_peaks - 1; i >= 0; --i) jlo[(int)peaks[i * 5]] = i;
  for (int64_t i = 0; i < n_peaks; ++i) jhi[(int)peaks[i * 5]] = i;
  for (int l = 0; l < OP_N_LIMBS; ++l) {
    const int64_t k0 = conn_off[l], k1 = conn_off[l + 1];
    if (k1 < k0 || k1 - k0 > 0x7fffffff) {
      set_error("connection offsets must be non-decreasing");
      return OP_ERR_INVALID;
    }
    most = std::max<int64_t>(most, k1 - k0);
    const int ja = c->prm.limbs_point[l][0], jb = c->prm.limbs_point[l][1];
    for (int64_t i = k0; i < k1; ++i) {
      const int64_t ia = (int64_t)conn[i * 3], ib = (int64_t)conn[i * 3 + 1];
      if (ia < jlo[ja] || ia > jhi[ja] || ib < jlo[jb] || ib > jhi[jb]) {
        set_error("connection ids do not belong to the limb's joints");
        return OP_ERR_INVALID;
      }
    }
  }
  PostBuffers* B = nullptr;
  RC(pick_buffers(c, most, 1, false, &B));
  PostShape s;
  post_shape(c, s, 1, 64, 64, 64, 64, 64.0, 1.0, 1.0);  // map size is unused by grouping
  int32_t hdr[4];
  for (;;) {
    RC(upload_peaks(c, *B, peaks, n_peaks));
    const int maxp = B->maxp;
    std::vector<int32_t> cnt(OP_N_LIMBS, 0), ab((size_t)OP_N_LIMBS * maxp * 2, 0);
    std::vector<double> sc((size_t)OP_N_LIMBS * maxp, 0.0);
    for (int l = 0; l < OP_N_LIMBS; ++l) {
      const int64_t k0 = conn_off[l], k1 = conn_off[l + 1];
      cnt[l] = (int)(k1 - k0);
      for (int64_t i = k0; i < k1; ++i) {
        ab[((size_t)l * maxp + (i - k0)) * 2] = (int32_t)conn[i * 3];
        ab[((size_t)l * maxp + (i - k0)) * 2 + 1] = (int32_t)conn[i * 3 + 1];
        sc[(size_t)l * maxp + (i - k0)] = conn[i * 3 + 2];
      }
    }
    OP_HIP_CHECK(hipMemcpyAsync(B->conn_cnt, cnt.data(), cnt.size() * 4, hipMemcpyHostToDevice, c->stream));
    OP_HIP_CHECK(hipMemcpyAsync(B->conn_ab, ab.data(), ab.size() * 4, hipMemcpyHostToDevice, c->stream));
    OP_HIP_CHECK(hipMemcpyAsync(B->conn_score, sc.data(), sc.size() * 8, hipMemcpyHostToDevice, c->stream));
    RC(launch_grouping(s, *B, c->stream));
    OP_HIP_CHECK(hipMemcpyAsync(hdr, B->res_hdr, sizeof(hdr), hipMemcpyDeviceToHost, c->stream));
    OP_HIP_CHECK(hipStreamSynchronize(c->stream));
    if (hdr[0] != OP_ERR_CAPACITY || B != &c->pb) break;
    RC(pick_buffers(c, most, 1, true, &B));  // more subsets than the LDS grouping holds: again, in HBM
  }
  if (hdr[0] == OP_ERR_INDEX) {
    set_error("list assignment index out of range (grouping_key_points)");
    return OP_ERR_INDEX;
  }
  if (hdr[0] != OP_OK) {
    set_error("grouping capacity exceeded");
    return hdr[0];
  }
  if (hdr[2] > cap) {
    *n_subsets = hdr[2];
    set_error("subsets capacity too small");
    return OP_ERR_CAPACITY;
  }
  if (hdr[2] > 0)
    OP_HIP_CHECK(hipMemcpy(subsets, B->res_subsets, (size_t)hdr[2] * 20 * 8, hipMemcpyDeviceToHost));
  *n_subsets = hdr[2];
  return OP_OK;
}

// Pack planar (n, 57, lh, lw) maps [38 paf | 19 heat] into an NHWC (n, lh, lw, 57) device buffer.
static int stage_maps_dev(op_ctx* c, const float* maps, int n, int lh, int lw, float** out) {
  using namespace op;
  c->post_rec.kind = 0;  // staged maps are replaced
  const size_t fl = (size_t)n * 57 * lh * lw;
  std::vector<float> t(fl);
  for (int f = 0; f < n; ++f)
    for (int ch = 0; ch < 57; ++ch)
      for (int y = 0; y < lh; ++y)
        for (int x = 0; x < lw; ++x)
          t[(((size_t)f * lh + y) * lw + x) * 57 + ch] = maps[(((size_t)f * 57 + ch) * lh + y) * lw + x];
  RC(grow_buffer(c, (void**)&c->d_maps, &c->maps_bytes, fl * 4, "maps"));
  // the null-stream copy is not ordered against the (non-blocking) compute stream: a queued run may
  // still read the old maps
  OP_HIP_CHECK(hipStreamSynchronize(c->stream));
  OP_HIP_CHECK(hipMemcpy(c->d_maps, t.data(), fl * 4, hipMemcpyHostToDevice));
  *out = c->d_maps;
  return OP_OK;
}

int op_postprocess(op_ctx* c, const float* paf_low, const float* heat_low, int32_t h, int32_t w, int32_t orig_h,
                   int32_t orig_w, double* poses, double* scores, int32_t cap, op_frame_result* res) {
  using namespace op;
  RC(check_ctx(c, false));
  if (!paf_low || !heat_low || !res || h < 2 || w < 2 || orig_h < 1 || orig_w < 1) {
    set_error("op_postprocess: bad arguments");
    return OP_ERR_INVALID;
  }
  std::vector<float> maps((size_t)57 * h * w);
  memcpy(maps.data(), paf_low, (size_t)38 * h * w * 4);
  memcpy(maps.data() + (size_t)38 * h * w, heat_low, (size_t)19 * h * w * 4);
  float* dm = nullptr;
  RC(stage_maps_dev(c, maps.data(), 1, h, w, &dm));
  int map_w, map_h;
  optimal_size(orig_h, orig_w, c->prm.heatmap_size, 8, &map_w, &map_h);
  RC(ensure_post(c, 1, map_h, map_w));
  MapSource src{dm, (int64_t)57 * h * w, 0, 57, 0, 38};
  PostShape s;
  post_shape(c, s, 1, h, w, map_h, map_w, (double)map_w, (double)orig_w / map_w, (double)orig_h / map_h);
  post_record(c, 1, &src, nullptr, 0, s);
  RC(launch_post_maps(src, s, c->pb, c->stream));
  OP_HIP_CHECK(hipStreamSynchronize(c->stream));
  memset(res, 0, sizeof(*res));
  res->map_w = map_w;
  res->map_h = map_h;
  return read_result(c, 0, poses, scores, cap, res);
}

// Enqueue preprocess + forward + post-process for the staged batch on the context stream.
static int enqueue_staged(op_ctx* c, bool timing) {
  c->st_precise = false;
  using namespace op;
  int in_w, in_h, map_w, map_h;
  optimal_size(c->st_h, c->st_w, c->prm.inference_img_size, 8, &in_w, &in_h);
  optimal_size(c->st_h, c->st_w, c->prm.heatmap_size, 8, &map_w, &map_h);
  RC(ensure_geometry(c, c->st_n, in_h, in_w));
  RC(ensure_post(c, c->st_n, map_h, map_w));
  if (timing) OP_HIP_CHECK(hipEventRecord(c->ev[0], c->stream));
  if (c->split) {  // the network input is resampled inside the conv1_1 kernel
    RC(run_forward(c, c->d_frames, (int64_t)c->st_h * c->st_w * 3, (int64_t)c->st_w * 3, c->st_h, c->st_w));
  } else {
    RC(profiled(c, kProfInput, 0.0, 0.0, [&] {
      return launch_preprocess(c->d_frames, (int64_t)c->st_h * c->st_w * 3, (int64_t)c->st_w * 3, c->st_n, c->st_h,
                               c->st_w, in_h, in_w, c->buf[B_X0].p, c->stream);
    }));
    RC(run_forward(c));
  }
  if (timing) OP_HIP_CHECK(hipEventRecord(c->ev[1], c->stream));
  const int lh = in_h / 8, lw = in_w / 8;
  MapSource src;
  if (c->use_maps) {
    if (c->sm_n < c->st_n || c->sm_h != lh || c->sm_w != lw) {
      set_error("staged maps do not match the staged frames (n, h/8, w/8)");
      return OP_ERR_STATE;
    }
    src = MapSource{c->d_maps, (int64_t)57 * lh * lw, 0, 57, 0, 38};
  } else if (c->split) {
    const Act& m = c->buf[B_MAP32];
    src = MapSource{m.p, (int64_t)m.frame_floats(), 0, m.cs, 0, 40};
  } else {
    const Act& cat = c->buf[B_CAT];
    src = MapSource{cat.p, (int64_t)cat.frame_floats(), cat.pad, cat.cs, kCatPaf, kCatHeat};
  }
  PostShape s;
  post_shape(c, s, c->st_n, lh, lw, map_h, map_w, (double)map_w, (double)c->st_w / map_w, (double)c->st_h / map_h);
  // post-process algorithmic HBM bytes: 57-ch low-res read + 18-ch upsample write +
  // 2 x (read + write) Gaussian passes + NMS read, f32
  const double mp = (double)c->st_n * map_h * map_w;
  const double pbytes = 4.0 * ((double)c->st_n * 57 * lh * lw + 18 * mp + 2 * 2 * 18 * mp + 18 * mp);
  post_record(c, 1, &src, nullptr, 0, s);
  RC(profiled(c, kProfPost, 0.0, pbytes, [&] { return launch_post_maps(src, s, c->pb, c->stream); }));
  if (timing) OP_HIP_CHECK(hipEventRecord(c->ev[2], c->stream));
  c->timed = timing;
  return OP_OK;
}

int op_stage_frames(op_ctx* c, const uint8_t* frames, int32_t n, int32_t h, int32_t w) {
  using namespace op;
  RC(check_ctx(c, false));
  if (!frames || n < 1 || h < 8 || w < 8) {
    set_error("op_stage_frames: bad arguments");
    return OP_ERR_INVALID;
  }
  const size_t bytes = (size_t)n * h * w * 3;
  c->up_slot = -1;  // a pending op_upload_frames is replaced
  RC(grow_buffer(c, (void**)&c->d_frames, &c->frames_bytes, bytes, "frames"));
  OP_HIP_CHECK(hipMemcpyAsync(c->d_frames, frames, bytes, hipMemcpyHostToDevice, c->stream));
  OP_HIP_CHECK(hipStreamSynchronize(c->stream));
  if (c->st_n != n || c->st_h != h || c->st_w != w) {
    if (c->gexec) {
      hipGraphExecDestroy(c->gexec);
      c->gexec = nullptr;
    }
  }
  c->st_n = n;
  c->st_h = h;
  c->st_w = w;
  return OP_OK;
}

int op_stage_maps(op_ctx* c, const float* maps, int32_t n, int32_t mh, int32_t mw) {
  using namespace op;
  RC(check_ctx(c, false));
  if (!maps || n < 1 || mh < 2 || mw < 2) {
    set_error("op_stage_maps: bad arguments");
    return OP_ERR_INVALID;
  }
  if (c->st_n > 0 && mh == c->st_h && mw == c->st_w) {
    // full-resolution maps of the staged frames: the precise post-process input (kept planar)
    const size_t bytes = (size_t)n * 57 * mh * mw * 4;
    c->post_rec.kind = 0;  // staged maps are replaced
    RC(grow_buffer(c, (void**)&c->d_fmaps, &c->fmaps_bytes, bytes, "full_maps"));
    OP_HIP_CHECK(hipStreamSynchronize(c->stream));  // a queued precise run may still read the old maps
    OP_HIP_CHECK(hipMemcpy(c->d_fmaps, maps, bytes, hipMemcpyHostToDevice));
    c->fm_n = n;
    c->fm_h = mh;
    c->fm_w = mw;
  } else {
    float* dm;
    RC(stage_maps_dev(c, maps, n, mh, mw, &dm));
    c->sm_n = n;
    c->sm_h = mh;
    c->sm_w = mw;
  }
  if (c->gexec) {
    hipGraphExecDestroy(c->gexec);
    c->gexec = nullptr;
  }
  return OP_OK;
}

int op_use_staged_maps(op_ctx* c, int32_t enable) {
  if (!c) return OP_ERR_INVALID;
  c->use_maps = enable != 0;
  if (c->gexec) {
    hipGraphExecDestroy(c->gexec);
    c->gexec = nullptr;
  }
  return OP_OK;
}

// A pending op_upload_frames becomes the staged frame set: the compute stream waits for its copy
// and moves the ring slot into d_frames (the buffer kernels and captured graphs read).
static int take_upload(op_ctx* c) {
  if (c->up_slot < 0) return OP_OK;
  const int k = c->up_slot;
  c->up_slot = -1;
  const size_t bytes = (size_t)c->up_n * c->up_h * c->up_w * 3;
  RC(grow_buffer(c, (void**)&c->d_frames, &c->frames_bytes, bytes, "frames"));
  OP_HIP_CHECK(hipStreamWaitEvent(c->stream, c->ev_up[k], 0));
  OP_HIP_CHECK(hipMemcpyAsync(c->d_frames, c->d_ring[k], bytes, hipMemcpyDeviceToDevice, c->stream));
  OP_HIP_CHECK(hipEventRecord(c->ev_free[k], c->stream));
  if (c->st_n != c->up_n || c->st_h != c->up_h || c->st_w != c->up_w) {
    if (c->gexec) {
      OP_HIP_CHECK(hipStreamSynchronize(c->stream));
      hipGraphExecDestroy(c->gexec);
      c->gexec = nullptr;
    }
  }
  c->st_n = c->up_n;
  c->st_h = c->up_h;
  c->st_w = c->up_w;
  return OP_OK;
}

int op_upload_frames(op_ctx* c, const uint8_t* frames, int32_t n, int32_t h, int32_t w) {
  using namespace op;
  RC(check_ctx(c, false));
  if (!frames || n < 1 || h < 8 || w < 8) {
    set_error("op_upload_frames: bad arguments");
    return OP_ERR_INVALID;
  }
  if (!c->copy_stream) {
    OP_HIP_CHECK(hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking));
    for (int i = 0; i < 2; ++i) {
      OP_HIP_CHECK(hipEventCreateWithFlags(&c->ev_up[i], hipEventDisableTiming));
      OP_HIP_CHECK(hipEventCreateWithFlags(&c->ev_free[i], hipEventDisableTiming));
    }
  }
  RC(take_upload(c));  // an upload never run is still staged: this one replaces it afterwards
  const int k = c->ring_next;
  const size_t bytes = (size_t)n * h * w * 3;
  if (bytes > c->ring_bytes[k]) {
    OP_HIP_CHECK(hipStreamSynchronize(c->copy_stream));
    OP_HIP_CHECK(hipStreamSynchronize(c->stream));
    if (c->d_ring[k]) OP_HIP_CHECK(hipFree(c->d_ring[k]));
    c->d_ring[k] = nullptr;
    OP_HIP_CHECK(hipMalloc((void**)&c->d_ring[k], bytes));
    c->ring_bytes[k] = bytes;
  }
  // the slot's previous frames must have been moved out by the compute stream first
  OP_HIP_CHECK(hipStreamWaitEvent(c->copy_stream, c->ev_free[k], 0));
  OP_HIP_CHECK(hipMemcpyAsync(c->d_ring[k], frames, bytes, hipMemcpyHostToDevice, c->copy_stream));
  OP_HIP_CHECK(hipEventRecord(c->ev_up[k], c->copy_stream));
  c->up_slot = k;
  c->up_n = n;
  c->up_h = h;
  c->up_w = w;
  c->ring_next = k ^ 1;
  return OP_OK;
}

int op_upload_wait(op_ctx* c) {
  using namespace op;
  RC(check_ctx(c, false));
  for (int k = 0; k < 2; ++k)
    if (c->ev_up[k]) OP_HIP_CHECK(hipEventSynchronize(c->ev_up[k]));
  return OP_OK;
}

int op_host_alloc(size_t bytes, void** p) {
  if (!p || bytes == 0) return OP_ERR_INVALID;
  *p = nullptr;
  if (hipHostMalloc(p, bytes, hipHostMallocDefault) != hipSuccess) {
    (void)hipGetLastError();
    op::set_error("hipHostMalloc failed");
    return OP_ERR_HIP;
  }
  return OP_OK;
}

int op_host_free(void* p) {
  if (p && hipHostFree(p) != hipSuccess) return OP_ERR_HIP;
  return OP_OK;
}

int op_run_staged(op_ctx* c) {
  using namespace op;
  RC(check_ctx(c, true));
  RC(take_upload(c));
  if (c->st_n < 1) {
    set_error("no staged frames");
    return OP_ERR_STATE;
  }
  return enqueue_staged(c, true);
}

int op_run_staged_graph(op_ctx* c) {
  using namespace op;
  RC(check_ctx(c, true));
  RC(take_upload(c));
  if (c->st_n < 1) {
    set_error("no staged frames");
    return OP_ERR_STATE;
  }
  // geometry/buffers must exist before capture (allocation and memsets are not captured)
  int in_w, in_h, map_w, map_h;
  optimal_size(c->st_h, c->st_w, c->prm.inference_img_size, 8, &in_w, &in_h);
  optimal_size(c->st_h, c->st_w, c->prm.heatmap_size, 8, &map_w, &map_h);
  RC(ensure_geometry(c, c->st_n, in_h, in_w));
  RC(ensure_post(c, c->st_n, map_h, map_w));
  // the graph bakes in every pointer and size: replay only if none changed since capture
  const uintptr_t key[10] = {(uintptr_t)c->st_n, (uintptr_t)c->st_h, (uintptr_t)c->st_w, (uintptr_t)c->use_maps,
                             (uintptr_t)c->arena, (uintptr_t)c->post_arena, (uintptr_t)c->d_frames,
                             (uintptr_t)c->d_maps, (uintptr_t)c->gn, (uintptr_t)(c->gh * 65536 + c->gw) * 4 + (uintptr_t)c->split * 2 + (uintptr_t)c->splitk};
  if (c->gexec && memcmp(key, c->g_key, sizeof(key)) != 0) {
    hipGraphExecDestroy(c->gexec);
    c->gexec = nullptr;
  }
  if (!c->gexec) {
    OP_HIP_CHECK(hipStreamSynchronize(c->stream));
    memcpy(c->g_key, key, sizeof(key));
    const bool prof = c->prof;
    c->prof = false;  // no event records inside the capture
    if (c->graph) {
      hipGraphDestroy(c->graph);
      c->graph = nullptr;
    }
    hipGraph_t g = nullptr;
    for (int attempt = 0;; ++attempt) {
      OP_HIP_CHECK(hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
      int rc = enqueue_staged(c, false);
      hipError_t e = hipStreamEndCapture(c->stream, &g);
      if (rc || e != hipSuccess) {
        c->prof = prof;
        if (g) hipGraphDestroy(g);
        if (rc) return rc;
        OP_HIP_CHECK(e);
      }
      // a split-K launch that found its workspace too small during capture ran unsplit: grow the
      // workspace outside capture and capture again, so replays match eager runs
      if (splitk_ws_capture_short(c->stream) == 0) break;
      hipGraphDestroy(g);
      g = nullptr;
      if (attempt > 0 || splitk_ws_reserve(c->stream) != 0) {
        c->prof = prof;
        set_error("split-K workspace allocation failed");
        return OP_ERR_HIP;
      }
    }
    c->prof = prof;
    c->graph = g;
    OP_HIP_CHECK(hipGraphInstantiate(&c->gexec, g, nullptr, nullptr, 0));
    if (const char* d = getenv("OP_GRAPH_DUMP")) {  // debugging aid: DOT dump of every captured graph
      static int seq = 0;
      const std::string path = std::string(d) + "/graph_" + std::to_string(seq++) + ".dot";
      hipGraphDebugDotPrint(g, path.c_str(), hipGraphDebugDotFlagsVerbose);
    }
  }
  if (getenv("OP_GRAPH_DRYRUN")) return enqueue_staged(c, false);  // debugging aid: eager instead of replay
  OP_HIP_CHECK(hipGraphLaunch(c->gexec, c->stream));
  c->timed = false;
  return OP_OK;
}

static bool host_side(const void* p) {
  if (!p) return false;
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();  // unregistered (pageable) host memory
    return true;
  }
  return a.type != hipMemoryTypeDevice;
}

int op_graph_info(op_ctx* c, int32_t* nodes, int32_t* kernels, int32_t* memsets, int32_t* memcpys,
                  int32_t* host_nodes) {
  using namespace op;
  RC(check_ctx(c, false));
  if (!nodes || !kernels || !memsets || !memcpys || !host_nodes) {
    set_error("op_graph_info: null output");
    return OP_ERR_INVALID;
  }
  if (!c->graph) {
    set_error("op_graph_info: no captured graph");
    return OP_ERR_STATE;
  }
  size_t n = 0;
  OP_HIP_CHECK(hipGraphGetNodes(c->graph, nullptr, &n));
  std::vector<hipGraphNode_t> v(n);
  OP_HIP_CHECK(hipGraphGetNodes(c->graph, v.data(), &n));
  *nodes = (int32_t)n;
  *kernels = *memsets = *memcpys = *host_nodes = 0;
  for (hipGraphNode_t nd : v) {
    hipGraphNodeType t;
    OP_HIP_CHECK(hipGraphNodeGetType(nd, &t));
    if (t == hipGraphNodeTypeKernel) {
      ++*kernels;
    } else if (t == hipGraphNodeTypeMemset) {
      hipMemsetParams mp;
      OP_HIP_CHECK(hipGraphMemsetNodeGetParams(nd, &mp));
      ++*memsets;
      if (host_side(mp.dst)) ++*host_nodes;
    } else if (t == hipGraphNodeTypeMemcpy) {
      hipMemcpy3DParms mp;
      OP_HIP_CHECK(hipGraphMemcpyNodeGetParams(nd, &mp));
      ++*memcpys;
      const void* src = mp.srcArray ? nullptr : mp.srcPtr.ptr;
      const void* dst = mp.dstArray ? nullptr : mp.dstPtr.ptr;
      if (mp.kind == hipMemcpyHostToDevice || mp.kind == hipMemcpyDeviceToHost || mp.kind == hipMemcpyHostToHost ||
          host_side(src) || host_side(dst))
        ++*host_nodes;
    } else if (t != hipGraphNodeTypeEmpty) {
      ++*host_nodes;  // host callbacks, event records / waits, child graphs: not expected
    }
  }
  return OP_OK;
}

int op_synchronize(op_ctx* c) {
  using namespace op;
  RC(check_ctx(c, false));
  OP_HIP_CHECK(hipStreamSynchronize(c->stream));
  RC(guard_check("op_synchronize"));
  return OP_OK;
}

// network input / post-process map size of the staged results (single scale or precise)
static void staged_sizes(op_ctx* c, int* in_w, int* in_h, int* map_w, int* map_h) {
  if (c->st_precise) {
    *in_w = c->st_net_w;
    *in_h = c->st_net_h;
    *map_w = c->st_w;
    *map_h = c->st_h;
    return;
  }
  optimal_size(c->st_h, c->st_w, c->prm.inference_img_size, 8, in_w, in_h);
  optimal_size(c->st_h, c->st_w, c->prm.heatmap_size, 8, map_w, map_h);
}

int op_fetch_result(op_ctx* c, int32_t frame, double* poses, double* scores, int32_t cap, op_frame_result* res) {
  using namespace op;
  RC(check_ctx(c, false));
  if (!res || frame < 0 || frame >= c->st_n) {
    set_error("op_fetch_result: bad frame");
    return OP_ERR_INVALID;
  }
  memset(res, 0, sizeof(*res));
  int in_w, in_h, map_w, map_h;
  staged_sizes(c, &in_w, &in_h, &map_w, &map_h);
  res->map_w = map_w;
  res->map_h = map_h;
  res->net_w = in_w;
  res->net_h = in_h;
  return read_result(c, frame, poses, scores, cap, res);
}

int op_fetch_maps(op_ctx* c, int32_t first, int32_t n, float* pafs, float* heatmaps, int32_t* mh, int32_t* mw) {
  using namespace op;
  RC(check_ctx(c, false));
  if (first < 0 || n < 1 || first + n > c->st_n || !mh || !mw) {
    set_error("op_fetch_maps: bad range");
    return OP_ERR_INVALID;
  }
  int in_w, in_h, map_w, map_h;
  staged_sizes(c, &in_w, &in_h, &map_w, &map_h);
  const int h = c->st_precise ? c->st_h : in_h / 8, w = c->st_precise ? c->st_w : in_w / 8;
  *mh = h;
  *mw = w;
  if (!pafs && !heatmaps) return OP_OK;  // size query
  OP_HIP_CHECK(hipStreamSynchronize(c->stream));
  const size_t hw = (size_t)h * w;
  if (c->st_precise) {  // the averaged maps: planar (57, h, w) per frame
    const size_t fpl = (size_t)(OP_N_PAF + OP_N_HEAT) * hw;
    for (int i = 0; i < n; ++i) {
      const float* f = c->d_psum + (size_t)(first + i) * fpl;
      if (pafs) OP_HIP_CHECK(hipMemcpy(pafs + (size_t)i * OP_N_PAF * hw, f, OP_N_PAF * hw * 4, hipMemcpyDeviceToHost));
      if (heatmaps)
        OP_HIP_CHECK(hipMemcpy(heatmaps + (size_t)i * OP_N_HEAT * hw, f + OP_N_PAF * hw, OP_N_HEAT * hw * 4,
                               hipMemcpyDeviceToHost));
    }
    return OP_OK;
  }
  // single scale: the last-stage maps (NHWC) as the network wrote them
  const Act& m = c->split ? c->buf[B_MAP32] : c->buf[B_CAT];
  if (c->gn < first + n || m.h != h || m.w != w) {
    set_error("op_fetch_maps: no network maps of the staged frames (run op_run_staged first)");
    return OP_ERR_STATE;
  }
  const int paf_off = c->split ? 0 : kCatPaf, heat_off = c->split ? 40 : kCatHeat;
  std::vector<float> t(m.frame_floats());
  for (int i = 0; i < n; ++i) {
    OP_HIP_CHECK(hipMemcpy(t.data(), m.p + (size_t)(first + i) * m.frame_floats(), t.size() * 4, hipMemcpyDeviceToHost));
    const int pw = w + 2 * m.pad;
    for (int y = 0; y < h; ++y)
      for (int x = 0; x < w; ++x) {
        const float* px = t.data() + ((size_t)(y + m.pad) * pw + (x + m.pad)) * m.cs;
        if (pafs)
          for (int k = 0; k < OP_N_PAF; ++k) pafs[((size_t)i * OP_N_PAF + k) * hw + (size_t)y * w + x] = px[paf_off + k];
        if (heatmaps)
          for (int k = 0; k < OP_N_HEAT; ++k)
            heatmaps[((size_t)i * OP_N_HEAT + k) * hw + (size_t)y * w + x] = px[heat_off + k];
      }
  }
  return OP_OK;
}

// ---- fixed-size per-frame result records (the multi-GPU gather's payload, gather.hip) ----
// Record of frame i: int32 {status, n_peaks, n_persons, 0}, int64 global frame id, 8 pad bytes,
// then max_persons x 54 f64 poses and max_persons f64 scores (rows past n_persons zero).
__global__ __launch_bounds__(256) void pack_records(PostBuffers b, int first, int max_persons, int64_t frame_base,
                                                    int frame_stride, char* __restrict__ out, int64_t rec_bytes) {
  const int i = blockIdx.x;
  const int f = first + i;
  char* r = out + (int64_t)i * rec_bytes;
  const int status = b.res_hdr[4 * f];
  const int persons = status == OP_OK ? b.res_hdr[4 * f + 2] : 0;
  const int k = persons < max_persons ? persons : max_persons;
  if (threadIdx.x == 0) {
    int32_t* h = (int32_t*)r;
    h[0] = status;
    h[1] = b.res_hdr[4 * f + 1];
    h[2] = persons;
    h[3] = 0;
    *(int64_t*)(r + 16) = frame_base + (int64_t)i * frame_stride;
    *(int64_t*)(r + 24) = 0;
  }
  double* poses = (double*)(r + 32);
  double* scores = poses + (int64_t)max_persons * 54;
  const double* src = b.res_poses + (int64_t)f * b.maxs * 54;
  for (int e = threadIdx.x; e < max_persons * 54; e += 256) poses[e] = e < k * 54 ? src[e] : 0.0;
  for (int e = threadIdx.x; e < max_persons; e += 256) scores[e] = e < k ? b.res_scores[(int64_t)f * b.maxs + e] : 0.0;
}

int64_t record_bytes(int max_persons) { return 32 + (int64_t)max_persons * 55 * 8; }

// Keep slot plan (see KeepSlot; round 6): one block assigns every frame's keep
// entry in FRAME ORDER -- exclusive prefix counts over the frames before it -- so which frame goes
// without a slot when slots run short is always the same one (the last ones), whatever the block
// scheduling (the per-block atomic claims it replaces were first come, first served).  Per frame:
// why 2 (more persons than the record holds) takes page-locked rows while the rows of every earlier
// why-2 frame plus its own fit h_rows_cap, else a device res slot; why 1 (over the batched caps) a
// maps slot; a frame past `slots` such frames is not kept (where -1).
__global__ __launch_bounds__(1024) void keep_plan(PostBuffers b, int first, int n, int max_persons, int have_src,
                                                  int32_t* __restrict__ hdr, int64_t h_rows_cap, int slots) {
  __shared__ int64_t s_rows[1024];
  __shared__ int s_res[1024], s_map[1024];
  __shared__ int64_t c_rows;
  __shared__ int c_res, c_map;
  const int t = threadIdx.x;
  if (t == 0) {
    c_rows = 0;
    c_res = 0;
    c_map = 0;
  }
  for (int base = 0; base < n; base += 1024) {
    const int i = base + t;
    int status = 0, persons = 0, why = 0;
    if (i < n) {
      const int f = first + i;
      status = b.res_hdr[4 * f];
      persons = b.res_hdr[4 * f + 2];
      why = status == OP_ERR_CAPACITY ? 1 : (status == OP_OK && persons > max_persons) ? 2 : 0;
    }
    const int64_t rows = why == 2 ? (int64_t)persons * 55 : 0;
    __syncthreads();  // the carries of the previous chunk are visible, its scans are consumed
    const int64_t r0 = c_rows;
    s_rows[t] = rows;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {  // inclusive scan of the rows
      const int64_t v = t >= d ? s_rows[t - d] : 0;
      __syncthreads();
      s_rows[t] += v;
      __syncthreads();
    }
    const int64_t o = r0 + s_rows[t] - rows;  // doubles of h_rows before this frame's
    const bool in_rows = why == 2 && o + rows <= h_rows_cap;
    const int need_res = why == 2 && !in_rows, need_map = why == 1 && have_src;
    s_res[t] = need_res;
    s_map[t] = need_map;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {
      const int vr = t >= d ? s_res[t - d] : 0, vm = t >= d ? s_map[t - d] : 0;
      __syncthreads();
      s_res[t] += vr;
      s_map[t] += vm;
      __syncthreads();
    }
    if (i < n) {
      int off = -1;
      if (in_rows) off = (int)o;
      else if (need_res) {
        const int sl = c_res + s_res[t] - 1;
        if (sl < slots) off = -2 - sl;
      } else if (need_map) {
        const int sl = c_map + s_map[t] - 1;
        if (sl < slots) off = sl;
      }
      int32_t* h = hdr + kKeepHdr * i;
      h[0] = status;
      h[1] = b.res_hdr[4 * (first + i) + 1];
      h[2] = status == OP_OK ? persons : 0;
      h[3] = why;
      h[4] = off;
    }
    __syncthreads();
    if (t == 1023) {
      c_rows = r0 + s_rows[1023];
      c_res += s_res[1023];
      c_map += s_map[1023];
    }
  }
}

// The frame-order plan of frame i computed by its own block (keep_overflow with plan_self, packs
// of <= kKeepSelfPlan frames): the same prefix counts as keep_plan over frames 0 .. i-1 (each block
// reads the earlier frames' headers itself: O(n^2) reads, a few microseconds at the headline's
// 232 frames) -- one launch fewer per pack, which the one-frame latency path pays for in full.
constexpr int kKeepSelfPlan = 1024;
__device__ void keep_plan_self(const PostBuffers& b, int first, int i, int max_persons, int have_src,
                               int32_t* __restrict__ hdr, int64_t h_rows_cap, int slots) {
  __shared__ int64_t r_rows[4];
  __shared__ int r_res[4], r_map[4];
  const int t = threadIdx.x;
  auto why_of = [&](int j, int* persons) {
    const int f = first + j;
    const int status = b.res_hdr[4 * f];
    *persons = b.res_hdr[4 * f + 2];
    return status == OP_ERR_CAPACITY ? 1 : (status == OP_OK && *persons > max_persons) ? 2 : 0;
  };
  // rows of every earlier why-2 frame; the earlier frames needing a res / maps slot.  A why-2 frame
  // needs a res slot iff its rows did not fit: o_j + rows_j > cap, o_j the rows of those before it
  // (rows only grow, so once one misses, every later one misses: the count of misses is the count
  // of why-2 frames j < i whose inclusive row sum exceeds the cap)
  int64_t rows = 0;
  int nres = 0, nmap = 0;
  // pass 1: inclusive row sums need order -- each thread takes a contiguous run of earlier frames
  const int per = (i + 255) / 256, j0 = min(i, t * per), j1 = min(i, j0 + per);
  int64_t run = 0;
  for (int j = j0; j < j1; ++j) {
    int p;
    if (why_of(j, &p) == 2) run += (int64_t)p * 55;
  }
  // exclusive prefix of the runs over the threads (a block scan in LDS)
  __shared__ int64_t s_run[256];
  s_run[t] = run;
  __syncthreads();
  for (int d = 1; d < 256; d <<= 1) {
    const int64_t v = t >= d ? s_run[t - d] : 0;
    __syncthreads();
    s_run[t] += v;
    __syncthreads();
  }
  int64_t acc = s_run[t] - run;  // rows of the why-2 frames before this thread's run
  for (int j = j0; j < j1; ++j) {
    int p;
    const int w = why_of(j, &p);
    if (w == 2) {
      acc += (int64_t)p * 55;
      nres += acc > h_rows_cap;
    } else if (w == 1 && have_src) {
      ++nmap;
    }
  }
  rows = run;
  // block sums of the run rows (total before frame i), res and map counts
  for (int o = 32; o > 0; o >>= 1) {
    rows += __shfl_xor(rows, o);
    nres += __shfl_xor(nres, o);
    nmap += __shfl_xor(nmap, o);
  }
  if ((t & 63) == 0) {
    r_rows[t >> 6] = rows;
    r_res[t >> 6] = nres;
    r_map[t >> 6] = nmap;
  }
  __syncthreads();
  if (t == 0) {
    const int64_t o = r_rows[0] + r_rows[1] + r_rows[2] + r_rows[3];
    const int cres = r_res[0] + r_res[1] + r_res[2] + r_res[3], cmap = r_map[0] + r_map[1] + r_map[2] + r_map[3];
    int p;
    const int w = why_of(i, &p);
    const int f = first + i;
    const int status = b.res_hdr[4 * f];
    int off = -1;
    if (w == 2) {
      if (o + (int64_t)p * 55 <= h_rows_cap) off = (int)o;
      else if (cres < slots) off = -2 - cres;
    } else if (w == 1 && have_src) {
      if (cmap < slots) off = cmap;
    }
    int32_t* h = hdr + kKeepHdr * i;
    h[0] = status;
    h[1] = b.res_hdr[4 * f + 1];
    h[2] = status == OP_OK ? p : 0;
    h[3] = w;
    h[4] = off;
  }
  __syncthreads();
}

// Keep slot fill: per frame, as keep_plan (or the block itself, plan_self) assigned it.  A frame
// over the batched caps keeps its post-process input and batched peak counts (it is re-run alone in
// big mode); a frame with more persons than the record holds keeps its batched result rows (they
// are complete: copied out as they are).
__global__ __launch_bounds__(256) void keep_overflow(PostBuffers b, int first, const float* __restrict__ src,
                                                     int64_t fstride, float* __restrict__ dst, int32_t* __restrict__ cnt,
                                                     double* __restrict__ res, int32_t* __restrict__ hdr,
                                                     double* __restrict__ h_rows, int plan_self, int max_persons,
                                                     int64_t h_rows_cap, int slots) {
  const int i = blockIdx.x;
  const int f = first + i;
  if (plan_self) keep_plan_self(b, first, i, max_persons, src ? 1 : 0, hdr, h_rows_cap, slots);
  const int why = hdr[kKeepHdr * i + 3], off = hdr[kKeepHdr * i + 4];
  if (why == 2) {
    if (off == -1) return;
    const int persons = hdr[kKeepHdr * i + 2];
    const double* ps = b.res_poses + (int64_t)f * b.maxs * 54;
    const double* ss = b.res_scores + (int64_t)f * b.maxs;
    double* d = off >= 0 ? h_rows + off : res + (int64_t)(-2 - off) * b.maxs * 55;
    const int64_t sc = off >= 0 ? (int64_t)persons * 54 : (int64_t)b.maxs * 54;
    for (int e = threadIdx.x; e < persons * 54; e += 256) d[e] = ps[e];
    for (int e = threadIdx.x; e < persons; e += 256) d[sc + e] = ss[e];
    return;
  }
  if (why != 1 || !src || off < 0) return;
  if (threadIdx.x < OP_N_JOINTS) cnt[off * OP_N_JOINTS + threadIdx.x] = b.peak_cnt[f * OP_N_JOINTS + threadIdx.x];
  const float* s = src + (int64_t)f * fstride;
  float* d = dst + (int64_t)off * fstride;
  for (int64_t e = threadIdx.x; e < fstride; e += 256) d[e] = s[e];
}

// Enqueue the records of staged frames [first, first+n) into dst (device) on the context stream;
// keep_slot 0/1 also fills that keep slot (gather.hip passes its record slot) and copies its
// headers to pinned memory on the same stream.
int ctx_pack_records(op_ctx* c, int first, int n, int max_persons, int64_t frame_base, int frame_stride, void* dst,
                     hipStream_t* stream, int keep_slot) {
  if (first < 0 || n < 1 || first + n > c->st_n || first + n > c->pn || max_persons < 0 || keep_slot > 1) {
    set_error("pack records: bad frame range");
    return OP_ERR_INVALID;
  }
  if (keep_slot >= 0) {
    KeepSlot& k = c->keep[keep_slot];
    // page-locked rows for frames past max_persons: 256 persons per frame on average (the rest,
    // if ever, are read from the device copy in res; OP_KEEP_ROWS_AVG overrides the 256, 0 sends
    // every such frame through the device copy -- a test aid)
    const char* avg_env = getenv("OP_KEEP_ROWS_AVG");
    const int64_t avg = avg_env ? std::max(0, atoi(avg_env)) : 256;
    const int64_t want = (int64_t)n * avg * 55;
    k.rows_cap_now = std::min(want, k.h_rows_cap);
    if (want > k.h_rows_cap) {
      OP_HIP_CHECK(hipStreamSynchronize(c->stream));
      if (k.h_rows) OP_HIP_CHECK(hipHostFree(k.h_rows));
      k.h_rows = nullptr;
      k.h_rows_cap = 0;
      // coherent (fine-grained): the kernel's stores go straight to host memory
      OP_HIP_CHECK(hipHostMalloc((void**)&k.h_rows, (size_t)want * 8, hipHostMallocMapped | hipHostMallocCoherent));
      OP_HIP_CHECK(hipHostGetDevicePointer((void**)&k.d_rows_view, k.h_rows, 0));
      k.h_rows_cap = want;
      k.rows_cap_now = want;
    }
  }
  RC(profiled(c, kProfOther, 0.0, 0.0, [&] {
    hipLaunchKernelGGL(pack_records, dim3(n), dim3(256), 0, c->stream, c->pb, first, max_persons, frame_base,
                       frame_stride, (char*)dst, record_bytes(max_persons));
    OP_AFTER_LAUNCH("pack_records", c->stream);
    return OP_OK;
  }));
  if (keep_slot >= 0) {
    KeepSlot& k = c->keep[keep_slot];
    const PostRecord& r = c->post_rec;
    const float* src = r.kind == 1 ? r.low.base : r.kind == 2 ? r.full : nullptr;
    const int64_t fstride = r.kind == 1 ? r.low.fstride : r.fstride;
    const char* kf_env = getenv("OP_KEEP_FRAMES");
    const int64_t per = src ? std::max<int64_t>(1, fstride * 4) : 1;  // map bytes per kept frame
    int fit = n;  // the budget-sized count
    if (kf_env) {
      k.slots = std::min(n, std::max(1, atoi(kf_env)));
      fit = k.slots;
    } else {
      const char* kb_env = getenv("OP_KEEP_BYTES");  // test aid: the map-byte budget per gather slot
      const int64_t budget = kb_env ? std::max(0ll, atoll(kb_env)) : kKeepSlotBytes;
      fit = (int)std::min<int64_t>(n, std::max<int64_t>(8, budget / per));
      // a short gather grows the next packs' slots (`grow`), but never past kKeepGrowBytes of maps
      // (advisor r05: growth was unbounded; one gather with many over-cap frames sized every later
      // pack's slots for good, and a failed allocation then failed the pack instead of losing frames)
      const char* kg_env = getenv("OP_KEEP_GROW_BYTES");  // test aid: the growth ceiling
      const int64_t ceiling = kg_env ? std::max(0ll, atoll(kg_env)) : kKeepGrowBytes;
      const int64_t grown = std::min<int64_t>(std::max(c->keep[0].grow, c->keep[1].grow),
                                              std::max<int64_t>(8, ceiling / per));
      k.slots = (int)std::min<int64_t>(n, std::max<int64_t>(fit, grown));
    }
    // the slots' buffers; if the grown count cannot be allocated, fall back to the budget-sized one:
    // the frames beyond it travel as lost-frame statuses rather than failing the pack
    auto alloc = [&]() -> int {
      if (src) {
        RC(grow_buffer(c, (void**)&k.maps, &k.maps_cap, (size_t)k.slots * fstride * 4, "keep_maps"));
        RC(grow_buffer(c, (void**)&k.cnt, &k.cnt_cap, (size_t)k.slots * OP_N_JOINTS * 4, "keep_cnt"));
      }
      return grow_buffer(c, (void**)&k.res, &k.res_cap, (size_t)k.slots * c->pb.maxs * 55 * 8, "keep_res");
    };
    if (alloc() != OP_OK) {
      if (k.slots <= fit) return OP_ERR_HIP;
      (void)hipGetLastError();  // the failed hipMalloc's error: the smaller request below decides
      k.slots = fit;
      RC(alloc());
    }
    k.maxs = c->pb.maxs;
    const size_t hb = (size_t)n * kKeepHdr * 4;
    if (hb > k.hdr_cap) {
      OP_HIP_CHECK(hipStreamSynchronize(c->stream));
      if (k.d_hdr) OP_HIP_CHECK(hipFree(k.d_hdr));
      if (k.h_hdr) OP_HIP_CHECK(hipHostFree(k.h_hdr));
      k.d_hdr = nullptr;
      k.h_hdr = nullptr;
      k.hdr_cap = 0;
      OP_HIP_CHECK(hipMalloc((void**)&k.d_hdr, hb));
      OP_HIP_CHECK(hipHostMalloc((void**)&k.h_hdr, hb, hipHostMallocDefault));
      k.hdr_cap = hb;
    }
    RC(profiled(c, kProfOther, 0.0, 0.0, [&] {
      const char* kp_env = getenv("OP_KEEP_PLAN_KERNEL");  // test aid: 1 = the separate keep_plan launch
      const int self = n <= kKeepSelfPlan && !(kp_env && atoi(kp_env) == 1) ? 1 : 0;
      if (!self) {
        hipLaunchKernelGGL(keep_plan, dim3(1), dim3(1024), 0, c->stream, c->pb, first, n, max_persons, src ? 1 : 0,
                           k.d_hdr, k.rows_cap_now, k.slots);
        OP_AFTER_LAUNCH("keep_plan", c->stream);
      }
      hipLaunchKernelGGL(keep_overflow, dim3(n), dim3(256), 0, c->stream, c->pb, first, src, fstride, k.maps, k.cnt,
                         k.res, k.d_hdr, k.d_rows_view, self, max_persons, k.rows_cap_now, k.slots);
      OP_AFTER_LAUNCH("keep_overflow", c->stream);
      return OP_OK;
    }));
    OP_HIP_CHECK(hipMemcpyAsync(k.h_hdr, k.d_hdr, hb, hipMemcpyDeviceToHost, c->stream));
    k.rec = r;
    k.rec.s.n = n;
    if (r.kind == 1) k.rec.low.base = k.maps;
    else if (r.kind == 2) k.rec.full = k.maps;
    if (!src) k.rec.kind = 0;
    k.n = n;
  }
  OP_HIP_CHECK(hipGetLastError());
  *stream = c->stream;
  return OP_OK;
}

// This rank's frames (slot-relative) of keep slot `slot` whose record does not carry the whole
// result; valid once the slot's gather has completed (op_comm_wait).
int ctx_kept_overflow(op_ctx* c, int slot, int32_t* frames, int32_t* reasons, int32_t cap, int32_t* count) {
  if (slot < 0 || slot > 1 || !count || (cap > 0 && !frames)) {
    set_error("kept overflow: bad arguments");
    return OP_ERR_INVALID;
  }
  KeepSlot& k = c->keep[slot];
  int m = 0, need1 = 0, need2 = 0;
  for (int i = 0; i < k.n; ++i)
    if (k.h_hdr[kKeepHdr * i + 3]) {
      if (k.h_hdr[kKeepHdr * i + 3] == 1) ++need1;
      else if (k.h_hdr[kKeepHdr * i + 4] < 0) ++need2;  // rows past the page-locked buffer
      if (m < cap) {
        frames[m] = i;
        if (reasons) reasons[m] = k.h_hdr[kKeepHdr * i + 3];
      }
      ++m;
    }
  k.grow = std::max(k.grow, std::max(need1, need2));  // the next packs keep this many
  *count = m;
  return OP_OK;
}

// Full result of frame i of keep slot `slot` (re-run alone in big mode from the kept input).
int ctx_kept_result(op_ctx* c, int slot, int frame, double* poses, double* scores, int32_t cap, op_frame_result* res) {
  if (slot < 0 || slot > 1 || !res || !poses || !scores || frame < 0 || frame >= c->keep[slot].n) {
    set_error("kept result: bad arguments");
    return OP_ERR_INVALID;
  }
  KeepSlot& k = c->keep[slot];
  memset(res, 0, sizeof(*res));
  const int32_t* hd = k.h_hdr + kKeepHdr * frame;
  if (!hd[3]) {
    set_error("kept result: the frame's record carries its whole result");
    return OP_ERR_STATE;
  }
  if (hd[3] == 2) {  // complete batched rows, kept as they were
    const int p = hd[2];
    res->status = OP_OK;
    res->n_peaks = hd[1];
    res->n_persons = p;
    if (p > cap) {
      set_error("result capacity too small");
      return OP_ERR_CAPACITY;
    }
    if (hd[4] >= 0) {  // written to page-locked memory by keep_overflow (complete: the gather waited)
      const double* h = k.h_rows + hd[4];
      memcpy(poses, h, (size_t)p * 54 * 8);
      memcpy(scores, h + (size_t)p * 54, (size_t)p * 8);
      return OP_OK;
    }
    if (hd[4] == -1) {
      set_error("kept result: more frames past max_persons than keep slots (OP_KEEP_FRAMES) in this gather");
      return OP_ERR_CAPACITY;
    }
    const double* d = k.res + (size_t)(-2 - hd[4]) * k.maxs * 55;
    OP_HIP_CHECK(hipMemcpy(poses, d, (size_t)p * 54 * 8, hipMemcpyDeviceToHost));
    OP_HIP_CHECK(hipMemcpy(scores, d + (size_t)k.maxs * 54, (size_t)p * 8, hipMemcpyDeviceToHost));
    return OP_OK;
  }
  if (k.rec.kind == 0) {
    set_error("kept result: no recorded post-process input for this slot");
    return OP_ERR_STATE;
  }
  if (hd[4] < 0) {
    set_error("kept result: more frames over the post-process caps than keep slots (OP_KEEP_FRAMES) in this gather");
    return OP_ERR_CAPACITY;
  }
  PostBuffers* B = nullptr;
  RC(rerun_big_rec(c, k.rec, hd[4], k.cnt + (size_t)hd[4] * OP_N_JOINTS, &B));
  return read_big(B, poses, scores, cap, res);
}

int ctx_device(op_ctx* c) { return c->device; }

int op_pack_results(op_ctx* c, int32_t first, int32_t n, int32_t max_persons, int64_t frame_base, int32_t frame_stride,
                    void* host_records) {
  using namespace op;
  RC(check_ctx(c, false));
  if (!host_records) {
    set_error("op_pack_results: null output");
    return OP_ERR_INVALID;
  }
  const size_t bytes = (size_t)n * record_bytes(max_persons);
  RC(ensure_scratch(c, bytes));
  hipStream_t st;
  RC(ctx_pack_records(c, first, n, max_persons, frame_base, frame_stride, c->d_scratch, &st, -1));
  OP_HIP_CHECK(hipMemcpyAsync(host_records, c->d_scratch, bytes, hipMemcpyDeviceToHost, st));
  OP_HIP_CHECK(hipStreamSynchronize(st));
  return OP_OK;
}

int op_fetch_results(op_ctx* c, int32_t first, int32_t n, double* poses, double* scores, int32_t cap,
                     op_frame_result* res) {
  using namespace op;
  RC(check_ctx(c, false));
  if (!res || !poses || !scores || first < 0 || n < 1 || first + n > c->st_n || cap < 1) {
    set_error("op_fetch_results: bad range");
    return OP_ERR_INVALID;
  }
  std::vector<int32_t> hdr((size_t)n * 4);
  OP_HIP_CHECK(hipMemcpy(hdr.data(), c->pb.res_hdr + 4 * first, hdr.size() * 4, hipMemcpyDeviceToHost));
  int in_w, in_h, map_w, map_h;
  staged_sizes(c, &in_w, &in_h, &map_w, &map_h);
  int maxp = 0;
  std::vector<int> big;
  for (int i = 0; i < n; ++i) {
    op_frame_result& r = res[i];
    memset(&r, 0, sizeof(r));
    r.status = hdr[4 * i];
    r.n_peaks = hdr[4 * i + 1];
    r.n_persons = r.status == OP_OK ? hdr[4 * i + 2] : 0;
    if (r.status == OP_ERR_CAPACITY && c->post_rec.kind) {  // over the batched caps: uncapped re-run
      big.push_back(i);
      r.n_persons = 0;
      r.status = OP_OK;
    }
    r.map_w = map_w;
    r.map_h = map_h;
    r.net_w = in_w;
    r.net_h = in_h;
    maxp = std::max(maxp, r.n_persons);
  }
  if (maxp > cap) {
    set_error("result capacity too small");
    return OP_ERR_CAPACITY;
  }
  if (maxp > 0) {
    // strided device rows -> packed pinned staging (one async 2D copy each), then host rows
    const size_t prow = (size_t)maxp * 54 * 8, srow = (size_t)maxp * 8;
    const size_t need = (size_t)n * (prow + srow);
    if (need > c->host_stage_bytes) {
      if (c->host_stage) OP_HIP_CHECK(hipHostFree(c->host_stage));
      c->host_stage = nullptr;
      OP_HIP_CHECK(hipHostMalloc((void**)&c->host_stage, need, hipHostMallocDefault));
      c->host_stage_bytes = need;
    }
    char* hp = c->host_stage;
    char* hs = c->host_stage + (size_t)n * prow;
    OP_HIP_CHECK(hipMemcpy2DAsync(hp, prow, c->pb.res_poses + (size_t)first * c->pb.maxs * 54,
                                  (size_t)c->pb.maxs * 54 * 8, prow, n, hipMemcpyDeviceToHost, c->stream));
    OP_HIP_CHECK(hipMemcpy2DAsync(hs, srow, c->pb.res_scores + (size_t)first * c->pb.maxs, (size_t)c->pb.maxs * 8,
                                  srow, n, hipMemcpyDeviceToHost, c->stream));
    OP_HIP_CHECK(hipStreamSynchronize(c->stream));
    for (int i = 0; i < n; ++i) {
      const size_t k = (size_t)res[i].n_persons;
      memcpy((char*)poses + (size_t)i * cap * 54 * 8, hp + i * prow, k * 54 * 8);
      memcpy((char*)scores + (size_t)i * cap * 8, hs + i * srow, k * 8);
    }
  }
  for (int i : big) {  // frames over the batched caps, re-run one at a time in big mode
    op_frame_result& r = res[i];
    const int rc = read_result(c, first + i, poses + (size_t)i * cap * 54, scores + (size_t)i * cap, cap, &r);
    if (rc == OP_ERR_HIP || (rc == OP_ERR_CAPACITY && r.n_persons > cap)) return rc;
    if (rc) {
      r.status = rc;
      r.n_persons = 0;
    }
  }
  return OP_OK;
}

// One frame (h x w x 3 u8, row stride row_stride) from caller memory into d_frames on the compute
// stream, through the context's page-locked staging buffer (op_detect / op_detect_precise).
static int upload_one_frame(op_ctx* c, const uint8_t* bgr, int h, int w, int64_t row_stride) {
  const size_t row = (size_t)w * 3, bytes = row * h;
  RC(grow_buffer(c, (void**)&c->d_frames, &c->frames_bytes, bytes, "frames"));
  OP_HIP_CHECK(hipStreamSynchronize(c->stream));  // the staging buffer's previous copy has completed
  if (bytes > c->up_pinned_bytes) {
    if (c->up_pinned) OP_HIP_CHECK(hipHostFree(c->up_pinned));
    c->up_pinned = nullptr;
    c->up_pinned_bytes = 0;
    OP_HIP_CHECK(hipHostMalloc((void**)&c->up_pinned, bytes, hipHostMallocDefault));
    c->up_pinned_bytes = bytes;
  }
  for (int y = 0; y < h; ++y) memcpy(c->up_pinned + (size_t)y * row, bgr + (size_t)y * row_stride, row);
  OP_HIP_CHECK(hipMemcpyAsync(c->d_frames, c->up_pinned, bytes, hipMemcpyHostToDevice, c->stream));
  return OP_OK;
}

int op_detect(op_ctx* c, const uint8_t* bgr, int32_t h, int32_t w, int64_t row_stride, double* poses, double* scores,
              int32_t cap, op_frame_result* res) {
  using namespace op;
  RC(check_ctx(c, true));
  if (!bgr || !res || h < 8 || w < 8 || row_stride < (int64_t)w * 3) {
    set_error("op_detect: bad arguments");
    return OP_ERR_INVALID;
  }
  c->up_slot = -1;  // a pending op_upload_frames is replaced
  RC(upload_one_frame(c, bgr, h, w, row_stride));
  c->st_n = 1;
  c->st_h = h;
  c->st_w = w;
  const bool keep_maps = c->use_maps;
  c->use_maps = false;
  int rc = enqueue_staged(c, false);
  c->use_maps = keep_maps;
  if (rc) return rc;
  OP_HIP_CHECK(hipStreamSynchronize(c->stream));
  RC(guard_check("op_detect"));
  return op_fetch_result(c, 0, poses, scores, cap, res);
}

// detect_precise (pose_detector.py:433-482).  Sizes follow the reference's Python arithmetic:
// multiplier = scale * inference_img_size / min(h, w) and math.ceil(w * multiplier) in f64.
// detect_precise (pose_detector.py:433-482) for the n frames (h x w, contiguous) at c->d_frames:
// per scale one batched forward of the n frames (cubic resize + pad + normalise per frame), then
// per frame the cubic map resizes into its running mean (psum: [frame][38 paf | 19 heat][h][w]),
// then the full-resolution post-process of all n frames (results at frame index f).
static int precise_run(op_ctx* c, int n, int h, int w, int* net_w, int* net_h, bool staged) {
  const int ds = c->prm.downscale;
  const int ns = c->prm.n_scales;
  int rws[OP_MAX_SCALES], rhs[OP_MAX_SCALES], pws[OP_MAX_SCALES], phs[OP_MAX_SCALES];
  size_t mid_off[OP_MAX_SCALES + 1] = {0};  // floats: every scale's padded-size maps of every frame
  for (int k = 0; k < ns; ++k) {
    const double m = c->prm.inference_scales[k] * (double)c->prm.inference_img_size / (double)(h < w ? h : w);
    rws[k] = (int)std::ceil((double)w * m);
    rhs[k] = (int)std::ceil((double)h * m);
    pws[k] = rws[k] + (ds - rws[k] % ds) % ds;
    phs[k] = rhs[k] + (ds - rhs[k] % ds) % ds;
    if (rws[k] < 1 || rhs[k] < 1 || phs[k] < 16 || pws[k] < 16) {
      set_error("detect_precise: a scale gives a network input below 16 x 16");
      return OP_ERR_INVALID;
    }
    mid_off[k + 1] = mid_off[k] + (size_t)n * phs[k] * pws[k] * (OP_N_PAF + OP_N_HEAT);
  }
  const int64_t fplanes = (int64_t)(OP_N_PAF + OP_N_HEAT) * h * w;  // floats per frame of psum
  // round 4 experiment, OFF by default: both map resizes and the scale mean in one pass from each
  // scale's last-stage maps (copied planar into d_pmid at low_off[k]) -- bit-identical, but it
  // recomputes each tile's crop halo and makes ~4.5x the VALU instructions of the two-pass path,
  // which is VALU/issue-bound rather than HBM-bound: 12.5 vs 11.3 ms per 16 1280x720 frames
  // (SQ_INSTS_VALU, profiles/r04/c4_fused_cubic_not_kept.md).  OP_CUBIC_FUSED=1 selects it.
  CubicFusedArgs fa{};
  size_t low_off[OP_MAX_SCALES + 1] = {0};
  fa.ns = ns;
  for (int k = 0; k < ns; ++k) {
    fa.lh[k] = phs[k] / ds;
    fa.lw[k] = pws[k] / ds;
    fa.pw[k] = pws[k];
    fa.rh[k] = rhs[k];
    fa.rw[k] = rws[k];
    fa.s1x[k] = 1.0 / ((double)pws[k] / (double)fa.lw[k]);  // cv_cubic_scale (cvcubic.hpp)
    fa.s1y[k] = 1.0 / ((double)phs[k] / (double)fa.lh[k]);
    fa.s2x[k] = 1.0 / ((double)w / (double)rws[k]);
    fa.s2y[k] = 1.0 / ((double)h / (double)rhs[k]);
    fa.lframe[k] = (int64_t)(OP_N_PAF + OP_N_HEAT) * fa.lh[k] * fa.lw[k];
    low_off[k + 1] = low_off[k] + (size_t)n * fa.lframe[k];
  }
  const char* fenv = getenv("OP_CUBIC_FUSED");
  const bool fused = fenv && atoi(fenv) == 1 && cubic_fused_lds(fa) > 0;
  RC(grow_buffer(c, (void**)&c->d_pmid, &c->pmid_bytes, (fused ? low_off[ns] : mid_off[ns]) * 4, "precise_mid"));
  RC(grow_buffer(c, (void**)&c->d_psum, &c->psum_bytes, (size_t)n * fplanes * 4, "precise_sum"));
  const size_t fbytes = (size_t)h * w * 3;
  auto run_scale = [&](int k) -> int {
    const int rw = rws[k], rh = rhs[k], pw = pws[k], ph = phs[k];
    RC(ensure_geometry(c, n, ph, pw));
    const Act& x0 = c->buf[B_X0];
    RC(profiled(c, kProfInput, 0.0, 0.0, [&] {
      return launch_preprocess_cubic(c->d_frames, (int64_t)w * 3, h, w, rh, rw, ph, pw, c->split, x0.p, n,
                                     (int64_t)fbytes, (int64_t)x0.frame_floats(), c->stream);
    }));
    RC(run_forward(c));
    // last-stage maps (lh, lw, cs) with the PAF / heat channels at paf_off / heat_off
    const int lh = ph / 8, lw = pw / 8;
    const float* mbase;
    int64_t mrow, mframe;
    int mpx, paf_off, heat_off;
    if (c->split) {
      const Act& m = c->buf[B_MAP32];
      mbase = m.p;
      mrow = (int64_t)lw * m.cs;
      mframe = (int64_t)m.frame_floats();
      mpx = m.cs;
      paf_off = 0;
      heat_off = 40;
    } else {
      const Act& cat = c->buf[B_CAT];
      mrow = (int64_t)(lw + 2 * cat.pad) * cat.cs;
      mframe = (int64_t)cat.frame_floats();
      mbase = cat.p + cat.pad * mrow + (int64_t)cat.pad * cat.cs;
      mpx = cat.cs;
      paf_off = kCatPaf;
      heat_off = kCatHeat;
    }
    if (fused) {
      float* low = c->d_pmid + low_off[k];
      fa.low[k] = low;
      RC(profiled(c, kProfMapResize, 0.0, 0.0, [&] {
        RC(launch_maps_planar(mbase + paf_off, mrow, mpx, mframe, lh, lw, OP_N_PAF, low, 0, OP_N_PAF + OP_N_HEAT, n,
                              c->stream));
        return launch_maps_planar(mbase + heat_off, mrow, mpx, mframe, lh, lw, OP_N_HEAT, low, OP_N_PAF,
                                  OP_N_PAF + OP_N_HEAT, n, c->stream);
      }));
    } else {
      // :461 / :465 cubic to the padded size (the heat by fx = fy = downscale: the same mapping),
      // stored planar (cn, ph, pw) so the second resize reads coalesced rows; kept for every scale
      // and frame until the fused second pass below; every frame of the scale in one launch per map
      const int64_t pp = (int64_t)ph * pw;
      const int64_t mid_f = pp * (OP_N_PAF + OP_N_HEAT);
      float* mid_paf = c->d_pmid + mid_off[k];
      float* mid_heat = mid_paf + (size_t)pp * OP_N_PAF;
      RC(profiled(c, kProfMapResize, 0.0, 0.0, [&] {
        RC(launch_resize_cubic_f32_frames(mbase + paf_off, mrow, mpx, mframe, lh, lw, OP_N_PAF, mid_paf, mid_f, ph, pw,
                                          n, c->stream));
        return launch_resize_cubic_f32_frames(mbase + heat_off, mrow, mpx, mframe, lh, lw, OP_N_HEAT, mid_heat, mid_f, ph,
                                              pw, n, c->stream);
      }));
    }
    return OP_OK;
  };
  // Round 6: the scales whose padded input is at most a quarter of the
  // largest's (1280x720: scales 0.5 and 1.0) run on a second stream, enqueued first, so their
  // launches -- a fraction of a round of workgroups each -- fill the rounds the large scales'
  // launches leave partly idle.  Each scale has its own activation arena (ensure_geometry caches one
  // per geometry, up to 6), its own region of d_pmid and, per stream, its own split-K workspace;
  // the side stream starts after everything queued on the compute stream (the staged frames, the
  // previous step's reads of d_pmid) and the compute stream waits for it before the scale mean.
  // OP_PRECISE_STREAMS=1 (read per call) runs every scale on the compute stream; never under capture,
  // nor while per-class profiling is on (op_profile: event pairs on two streams would overlap, and
  // the per-class sums -- the 7x7 roofline's launch time -- would count the overlap twice).
  const char* ps_env = getenv("OP_PRECISE_STREAMS");
  hipStreamCaptureStatus cap_st = hipStreamCaptureStatusNone;
  OP_HIP_CHECK(hipStreamIsCapturing(c->stream, &cap_st));
  std::vector<int> side, mainv;
  int64_t big = 0;
  for (int k = 0; k < ns; ++k) big = std::max<int64_t>(big, (int64_t)phs[k] * pws[k]);
  for (int k = 0; k < ns; ++k) {
    const bool small = ns > 1 && 4 * (int64_t)phs[k] * pws[k] <= big;
    (small && !(ps_env && atoi(ps_env) == 1) && !c->prof && cap_st == hipStreamCaptureStatusNone ? side : mainv)
        .push_back(k);
  }
  if (!side.empty()) {
    if (!c->side_stream) {
      OP_HIP_CHECK(hipStreamCreateWithFlags(&c->side_stream, hipStreamNonBlocking));
      OP_HIP_CHECK(hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming));
      OP_HIP_CHECK(hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming));
    }
    OP_HIP_CHECK(hipEventRecord(c->ev_fork, c->stream));
    OP_HIP_CHECK(hipStreamWaitEvent(c->side_stream, c->ev_fork, 0));
    c->main_stream = c->stream;
    c->stream = c->side_stream;
    int rc = OP_OK;
    for (int k : side)
      if ((rc = run_scale(k)) != OP_OK) break;
    c->stream = c->main_stream;
    c->main_stream = nullptr;
    // the join is recorded and waited for even after a failure, so no later work on the compute
    // stream can overtake what the side stream still has queued
    OP_HIP_CHECK(hipEventRecord(c->ev_join, c->side_stream));
    if (rc != OP_OK) {
      OP_HIP_CHECK(hipStreamWaitEvent(c->stream, c->ev_join, 0));
      return rc;
    }
    census_add(OP_CENSUS_PRECISE_SIDE);
  }
  for (int k : mainv) {
    const int rc = run_scale(k);
    if (rc != OP_OK) {
      if (!side.empty()) OP_HIP_CHECK(hipStreamWaitEvent(c->stream, c->ev_join, 0));
      return rc;
    }
  }
  if (!side.empty()) OP_HIP_CHECK(hipStreamWaitEvent(c->stream, c->ev_join, 0));
  // :462-463 / :466-467 / :469-470 every scale's crop to rh x rw and cubic to h x w, summed in scale
  // order and divided by the scale count: one pass per frame over the PAF and heat planes
  census_add(fused ? OP_CENSUS_CUBIC_FUSED : OP_CENSUS_CUBIC_TWO_PASS);
  if (fused) {
    bool taken = false;
    RC(profiled(c, kProfMapResize, 0.0, 0.0, [&] {
      return launch_resize_cubic_fused_mean(fa, c->d_psum, n, h, w, OP_N_PAF, OP_N_HEAT, c->stream, &taken);
    }));
    if (!taken) {
      set_error("detect_precise: fused map resize refused a checked shape");
      return OP_ERR_STATE;
    }
  }
  // round 4: every frame in one launch, a block of 8 output rows making each source row's
  // horizontal sums once (resize_cubic_f32_planar_mean_rows); OP_CUBIC_ROWS=0 selects the per-frame
  // form (A/B aid, read per call)
  bool rows_done = false;
  const char* renv = getenv("OP_CUBIC_ROWS");
  if (!fused && !(renv && atoi(renv) == 0)) {
    CubicMeanArgs a{};
    a.ns = ns;
    for (int k = 0; k < ns; ++k) {
      const int64_t pp = (int64_t)phs[k] * pws[k];
      a.src[k] = c->d_pmid + mid_off[k];
      a.fstride[k] = pp * (OP_N_PAF + OP_N_HEAT);
      a.cstride[k] = pp;
      a.sstride[k] = pws[k];
      a.sh[k] = rhs[k];
      a.sw[k] = rws[k];
      a.scx[k] = 1.0 / ((double)w / (double)rws[k]);  // cv_cubic_scale (cvcubic.hpp)
      a.scy[k] = 1.0 / ((double)h / (double)rhs[k]);
    }
    const char* tenv = getenv("OP_CUBIC_TILE");
    const bool tile = tenv && atoi(tenv) == 1;
    RC(profiled(c, kProfMapResize, 0.0, 0.0, [&] {
      if (tile)
        RC(launch_resize_cubic_f32_planar_mean_tile(a, c->d_psum, fplanes, n, h, w, OP_N_PAF, OP_N_HEAT, c->stream,
                                                    &rows_done));
      if (rows_done) return OP_OK;
      return launch_resize_cubic_f32_planar_mean_rows(a, c->d_psum, fplanes, n, h, w, OP_N_PAF, OP_N_HEAT, c->stream,
                                                      &rows_done);
    }));
  }
  if (rows_done) census_add(OP_CENSUS_CUBIC_ROWS);
  for (int f = 0; f < n && !fused && !rows_done; ++f) {
    CubicMeanArgs a{};
    a.ns = ns;
    for (int k = 0; k < ns; ++k) {
      const int64_t pp = (int64_t)phs[k] * pws[k];
      a.src[k] = c->d_pmid + mid_off[k] + (size_t)f * pp * (OP_N_PAF + OP_N_HEAT);
      a.cstride[k] = pp;
      a.sstride[k] = pws[k];
      a.sh[k] = rhs[k];
      a.sw[k] = rws[k];
      a.scx[k] = 1.0 / ((double)w / (double)rws[k]);  // cv_cubic_scale (cvcubic.hpp): OpenCV's f64 inverse scale
      a.scy[k] = 1.0 / ((double)h / (double)rhs[k]);
    }
    RC(profiled(c, kProfMapResize, 0.0, 0.0, [&] {
      return launch_resize_cubic_f32_planar_mean(a, c->d_psum + f * fplanes, h, w, OP_N_PAF, OP_N_HEAT, c->stream);
    }));
  }
  // :474-482 post-process at the original resolution: img_len = orig_w, no rescale.  With staged
  // full-resolution maps (op_stage_maps at the frame size + op_use_staged_maps) the post-process
  // reads those instead of the averaged maps (which are still computed).
  const float* post_maps = c->d_psum;
  if (c->use_maps && staged) {
    if (c->fm_n < n || c->fm_h != h || c->fm_w != w) {
      set_error("staged full-resolution maps do not match the staged frames (n, h, w)");
      return OP_ERR_STATE;
    }
    post_maps = c->d_fmaps;
  }
  RC(ensure_post(c, n, h, w));
  PostShape s;
  post_shape(c, s, n, h, w, h, w, (double)w, 1.0, 1.0);
  post_record(c, 2, nullptr, post_maps, fplanes, s);
  const float* sum_heat0 = post_maps + (size_t)OP_N_PAF * h * w;
  RC(profiled(c, kProfPost, 0.0, 0.0, [&] {
    RC(launch_peaks_from_full(sum_heat0, OP_N_JOINTS, h, w, s, c->pb, c->stream, fplanes));
    RC(launch_connections_full(post_maps, h, w, s, c->pb, c->stream, fplanes));
    return launch_grouping(s, c->pb, c->stream);
  }));
  *net_w = pws[ns - 1];
  *net_h = phs[ns - 1];
  return OP_OK;
}

int op_detect_precise(op_ctx* c, const uint8_t* bgr, int32_t h, int32_t w, int64_t row_stride, double* poses,
                      double* scores, int32_t cap, op_frame_result* res, float* pafs_out, float* heat_out) {
  using namespace op;
  RC(check_ctx(c, true));
  if (!bgr || !res || h < 11 || w < 11 || row_stride < (int64_t)w * 3 || c->prm.n_scales < 1) {
    set_error("op_detect_precise: bad arguments (frame >= 11 x 11, at least one inference scale)");
    return OP_ERR_INVALID;
  }
  c->up_slot = -1;  // a pending op_upload_frames is replaced
  RC(upload_one_frame(c, bgr, h, w, row_stride));
  // the staged frame set is replaced by this frame (its result stays fetchable as frame 0)
  c->st_n = 0;
  int net_w = 0, net_h = 0;
  RC(precise_run(c, 1, h, w, &net_w, &net_h, false));
  c->st_n = 1;
  c->st_h = h;
  c->st_w = w;
  c->st_precise = true;
  c->st_net_w = net_w;
  c->st_net_h = net_h;
  const float* sum_paf = c->d_psum;
  const float* sum_heat = c->d_psum + (size_t)OP_N_PAF * h * w;
  if (pafs_out)
    OP_HIP_CHECK(hipMemcpyAsync(pafs_out, sum_paf, (size_t)OP_N_PAF * h * w * 4, hipMemcpyDeviceToHost, c->stream));
  if (heat_out)
    OP_HIP_CHECK(hipMemcpyAsync(heat_out, sum_heat, (size_t)OP_N_HEAT * h * w * 4, hipMemcpyDeviceToHost, c->stream));
  OP_HIP_CHECK(hipStreamSynchronize(c->stream));
  RC(guard_check("op_detect_precise"));
  memset(res, 0, sizeof(*res));
  res->map_w = w;
  res->map_h = h;
  res->net_w = net_w;
  res->net_h = net_h;
  return read_result(c, 0, poses, scores, cap, res);
}

int op_run_staged_precise(op_ctx* c) {
  using namespace op;
  RC(check_ctx(c, true));
  RC(take_upload(c));
  if (c->st_n < 1 || c->st_h < 11 || c->st_w < 11 || c->prm.n_scales < 1) {
    set_error("op_run_staged_precise: no staged frames (>= 11 x 11) or no inference scale");
    return OP_ERR_STATE;
  }
  int net_w = 0, net_h = 0;
  RC(precise_run(c, c->st_n, c->st_h, c->st_w, &net_w, &net_h, true));
  c->st_precise = true;
  c->st_net_w = net_w;
  c->st_net_h = net_h;
  return OP_OK;
}

int op_resize_cubic(op_ctx* c, const void* src, int32_t dtype, int32_t h, int32_t w, int32_t cn, void* dst,
                    int32_t out_h, int32_t out_w) {
  using namespace op;
  RC(check_ctx(c, false));
  if (!src || !dst || (dtype != 0 && dtype != 1) || h < 1 || w < 1 || cn < 1 || out_h < 1 || out_w < 1) {
    set_error("op_resize_cubic: bad arguments");
    return OP_ERR_INVALID;
  }
  const size_t es = dtype == 0 ? 1 : 4;
  const size_t inb = (size_t)h * w * cn * es, outb = (size_t)out_h * out_w * cn * es;
  RC(ensure_scratch(c, inb + 256 + outb));
  char* din = (char*)c->d_scratch;
  char* dout = din + (inb + 255) / 256 * 256;
  OP_HIP_CHECK(hipMemcpyAsync(din, src, inb, hipMemcpyHostToDevice, c->stream));
  if (dtype == 0)
    RC(launch_resize_cubic_u8((const uint8_t*)din, (int64_t)w * cn, h, w, cn, (uint8_t*)dout, out_h, out_w, c->stream));
  else
    RC(launch_resize_cubic_f32((const float*)din, (int64_t)w * cn, cn, h, w, cn, (float*)dout, out_h, out_w, 0, 1.0f,
                               c->stream));
  OP_HIP_CHECK(hipMemcpyAsync(dst, dout, outb, hipMemcpyDeviceToHost, c->stream));
  OP_HIP_CHECK(hipStreamSynchronize(c->stream));
  return OP_OK;
}

int op_set_precision(op_ctx* c, int32_t mode) {
  using namespace op;
  RC(check_ctx(c, false));
  if (mode != OP_PRECISION_FP32 && mode != OP_PRECISION_BF16X3) {
    set_error("precision must be OP_PRECISION_FP32 or OP_PRECISION_BF16X3");
    return OP_ERR_INVALID;
  }
  c->split = mode == OP_PRECISION_BF16X3;
  return OP_OK;
}

int op_set_batch_invariant(op_ctx* c, int32_t enable) {
  using namespace op;
  RC(check_ctx(c, false));
  const int sk = enable ? 0 : 1;
  if (sk != c->splitk && c->gexec) {  // captured launches bake in the split-K choice
    OP_HIP_CHECK(hipStreamSynchronize(c->stream));
    hipGraphExecDestroy(c->gexec);
    c->gexec = nullptr;
  }
  c->splitk = sk;
  return OP_OK;
}

int op_set_peak_mode(op_ctx* c, int32_t mode, int32_t ksize) {
  using namespace op;
  RC(check_ctx(c, false));
  if (mode != OP_PEAKS_CPU_BRANCH && mode != OP_PEAKS_GPU_BRANCH) {
    set_error("op_set_peak_mode: mode must be OP_PEAKS_CPU_BRANCH or OP_PEAKS_GPU_BRANCH");
    return OP_ERR_INVALID;
  }
  if (mode == OP_PEAKS_GPU_BRANCH && (ksize < 3 || ksize > 2 * kMaxGaussR + 1 || (ksize & 1) == 0)) {
    set_error("op_set_peak_mode: ksize must be odd, 3 .. " + std::to_string(2 * kMaxGaussR + 1));
    return OP_ERR_INVALID;
  }
  OP_HIP_CHECK(hipStreamSynchronize(c->stream));
  c->peak_mode = mode;
  if (mode == OP_PEAKS_GPU_BRANCH) {
    c->gpu_r = gpu_branch_taps(c->prm.gaussian_sigma, ksize, c->gpu_taps);
  } else {
    c->gpu_r = 0;
    c->gpu_taps.clear();
  }
  const std::vector<double> gt = gauss_table(c);
  for (PostBuffers* b : {&c->pb, &c->bigb})
    if (b->gauss_w) OP_HIP_CHECK(hipMemcpy(b->gauss_w, gt.data(), gt.size() * 8, hipMemcpyHostToDevice));
  if (c->gexec) {  // captured launches bake in the peak kernel
    hipGraphExecDestroy(c->gexec);
    c->gexec = nullptr;
  }
  return OP_OK;
}

int op_set_stage_layout(op_ctx* c, int32_t planar) {
  using namespace op;
  RC(check_ctx(c, false));
  c->stage_planar = planar ? 1 : 0;
  if (c->gexec) {  // captured launches bake in the buffers
    OP_HIP_CHECK(hipStreamSynchronize(c->stream));
    hipGraphExecDestroy(c->gexec);
    c->gexec = nullptr;
  }
  return OP_OK;
}

int op_set_conv_algo(op_ctx* c, int32_t algo) {
  using namespace op;
  RC(check_ctx(c, false));
  if (algo != 0 && algo != 3 && algo != 4 && algo != 5) {
    set_error("conv algo must be 0 (per-tap gather), 3 (co-split halo), 4 (default) or 5 (default without the "
              "register-weight kernels)");
    return OP_ERR_INVALID;
  }
  c->conv_algo = algo;
  if (c->gexec) {  // captured launches bake in the kernels
    OP_HIP_CHECK(hipStreamSynchronize(c->stream));
    hipGraphExecDestroy(c->gexec);
    c->gexec = nullptr;
  }
  return OP_OK;
}

int op_get_precision(op_ctx* c, int32_t* mode) {
  using namespace op;
  RC(check_ctx(c, false));
  if (mode) *mode = c->split ? OP_PRECISION_BF16X3 : OP_PRECISION_FP32;
  return OP_OK;
}

int op_profile_enable(op_ctx* c, int32_t enable) {
  using namespace op;
  RC(check_ctx(c, false));
  c->prof = enable != 0;
  return OP_OK;
}

int op_profile_classes(op_ctx* c, int32_t mask) {
  using namespace op;
  RC(check_ctx(c, false));
  c->prof_mask = mask & ((1 << OP_PROFILE_CLASSES) - 1);
  return OP_OK;
}

int op_profile_reset(op_ctx* c) {
  using namespace op;
  RC(check_ctx(c, false));
  OP_HIP_CHECK(hipStreamSynchronize(c->stream));
  c->pending.clear();
  c->ev_used = 0;
  for (int i = 0; i < OP_PROFILE_CLASSES; ++i) {
    c->prof_ms[i] = c->prof_flops[i] = c->prof_bytes[i] = 0.0;
    c->prof_n[i] = 0;
  }
  return OP_OK;
}

int op_profile_read(op_ctx* c, int32_t cls, double* ms, int64_t* launches, double* flops, double* bytes) {
  using namespace op;
  RC(check_ctx(c, false));
  if (cls < 0 || cls >= OP_PROFILE_CLASSES) {
    set_error("profile class out of range (OP_PROFILE_CLASSES)");
    return OP_ERR_INVALID;
  }
  OP_HIP_CHECK(hipStreamSynchronize(c->stream));
  for (const ProfPair& p : c->pending) {
    float t = 0.0f;
    OP_HIP_CHECK(hipEventElapsedTime(&t, p.a, p.b));
    c->prof_ms[p.cls] += t;
    c->prof_n[p.cls] += p.n;
    c->prof_flops[p.cls] += p.flops;
    c->prof_bytes[p.cls] += p.bytes;
  }
  c->pending.clear();
  c->ev_used = 0;
  if (ms) *ms = c->prof_ms[cls];
  if (launches) *launches = c->prof_n[cls];
  if (flops) *flops = c->prof_flops[cls];
  if (bytes) *bytes = c->prof_bytes[cls];
  return OP_OK;
}

int op_last_timing(op_ctx* c, double* conv_ms, double* post_ms, double* total_ms) {
  using namespace op;
  RC(check_ctx(c, false));
  if (!c->timed) {
    set_error("no timed run (use op_run_staged)");
    return OP_ERR_STATE;
  }
  OP_HIP_CHECK(hipEventSynchronize(c->ev[2]));
  float a = 0, b = 0;
  OP_HIP_CHECK(hipEventElapsedTime(&a, c->ev[0], c->ev[1]));
  OP_HIP_CHECK(hipEventElapsedTime(&b, c->ev[1], c->ev[2]));
  if (conv_ms) *conv_ms = a;
  if (post_ms) *post_ms = b;
  if (total_ms) *total_ms = (double)a + b;
  return OP_OK;
}

}  // extern "C"

// Debugging aid (not part of the public header): copy the first `bytes` of activation buffer `id`
// (BufId order) of the current geometry to the host.
extern "C" int op_debug_read_buffer(op_ctx* c, int32_t id, void* dst, int64_t bytes) {
  using namespace op;
  RC(check_ctx(c, false));
  if (id < 0 || id >= B_COUNT || !dst || bytes < 0) return OP_ERR_INVALID;
  OP_HIP_CHECK(hipStreamSynchronize(c->stream));
  OP_HIP_CHECK(hipMemcpy(dst, c->buf[id].p, (size_t)bytes, hipMemcpyDeviceToHost));
  return OP_OK;
}
