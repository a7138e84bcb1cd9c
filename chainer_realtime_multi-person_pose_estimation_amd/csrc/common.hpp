// Shared helpers for the gfx950 kernels and the runtime.  Compiled with -ffp-contract=off:
// every fused multiply-add in the numeric-parity kernels is written explicitly.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>
#include <type_traits>

#include "openpose_hip.h"

namespace op {

// Thread-local last error text for op_last_error().
void set_error(const std::string& msg);

// OP_DEBUG_SYNC=1: synchronise after every kernel launch (outside graph capture) and report the
// kernel a fault happened in.
extern bool g_debug_sync;
int debug_after_launch(const char* name, hipStream_t st);
#define OP_AFTER_LAUNCH(name, st)                         \
  do {                                                    \
    if (::op::g_debug_sync) {                             \
      int _r = ::op::debug_after_launch((name), (st));    \
      if (_r) return _r;                                  \
    }                                                     \
  } while (0)

#define OP_HIP_CHECK(expr)                                                                   \
  do {                                                                                       \
    hipError_t _e = (expr);                                                                  \
    if (_e != hipSuccess) {                                                                  \
      ::op::set_error(std::string(#expr) + ": " + hipGetErrorString(_e));                    \
      return OP_ERR_HIP;                                                                     \
    }                                                                                        \
  } while (0)

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

// Physical channel layout of the 185-channel stage input (F.concat((paf, heat, feature)),
// CocoPoseNet.py:168): feature first so every slice start is 16-B aligned for the stores.
constexpr int kCatStride = 192;
constexpr int kCatFeat = 0;    // 128 channels
constexpr int kCatHeat = 128;  // 19 channels (+1 zero pad)
constexpr int kCatPaf = 152;   // 38 channels (+2 zero pad); 8-channel aligned for the split format
constexpr int kStagePad = 3;   // halo of the 7x7 stage convs

// ---- LDS DMA: global_load_lds_dwordx4 (lane l's 16 B land at lds + 16 l; lds wave-uniform) ----
// OP_ASM_DMA=1 issues it from inline asm.  With the builtin anywhere in a kernel the compiler's
// waitcnt pass makes every later LDS read wait for lgkmcnt(0) (in the 7x7 loop: every second 16-px
// block waits for the B fragment issued just before); the asm form is invisible to that pass and
// the reads get exact lgkmcnt(N).  Measured (interleaved A/B, tools/ab_lib.py): no gain -- the
// second wave of the SIMD already covers those stalls -- so the builtin stays the default.  The
// asm form writes M0 without telling the compiler; no kernel here relies on M0 otherwise.
#ifndef OP_ASM_DMA
#define OP_ASM_DMA 0
#endif
__device__ __forceinline__ void glds16(const void* gsrc, void* lds_dst) {
#if OP_ASM_DMA
  const uint32_t a =
      __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(__attribute__((address_space(3))) char*)lds_dst);
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(gsrc), "s"(a) : "memory");
#else
  __builtin_amdgcn_global_load_lds(gsrc, (__attribute__((address_space(3))) void*)lds_dst, 16, 0, 0);
#endif
}

// global -> LDS copy with an explicit cache-policy operand (timing experiments: 2 = nt)
template <int AUX>
__device__ __forceinline__ void glds16a(const void* gsrc, void* lds_dst) {
  __builtin_amdgcn_global_load_lds(gsrc, (__attribute__((address_space(3))) void*)lds_dst, 16, 0, AUX);
}

// ---- launch helpers implemented in the .hip files ----
struct ConvGroup {
  const float* in;    // padded NHWC input, already offset by the group's first input channel
  float* out;         // padded NHWC output, already offset by the group's first output channel
  const float* w;     // packed weights [c8][tap][cop][8]
  const float* bias;  // [cop]
  int32_t cop;        // padded output channels (multiple of the co tile)
  int32_t cout_store; // channels actually written (multiple of 4)
};

struct ConvShape {
  int32_t n, h, w;       // batch and spatial size (stride 1, same padding)
  int32_t pin, cs_in;    // input buffer halo and channel stride
  int32_t pout, cs_out;  // output buffer halo and channel stride
  int32_t c8;            // input channels / 8
  int32_t ks;            // 1, 3, 7
  int32_t relu;
  int32_t groups;        // 1 or 2
};

int launch_conv(const ConvShape& s, const ConvGroup* g, hipStream_t st);
// conv_f32.hip: the 3x3 / 7x7 LDS-halo form of conv_mfma_f32 (bit-identical); *taken = 0 outside it
int launch_conv_f32_lds(const ConvShape& s, const ConvGroup* g, hipStream_t st, int* taken);

// a branch's two closing 1x1 convs fused, exact f32 (conv.hip conv_head_f32)
struct HeadF32Shape {
  int32_t n, h, w, pin, cs_in, pout, cs_out;
  int32_t c8;      // input channels / 8
  int32_t co1;     // layer a's channels (a multiple of 128)
  int32_t groups;  // 1 or 2 (the two branches)
};
struct HeadF32Group {
  const float* in;  // padded NHWC input, offset by the group's first input channel
  const float *w1, *b1, *w2, *b2;  // packed [c8][cop][8] weights and biases of layers a and b
  int32_t cop1, cop2;
  float* out;  // padded NHWC output, offset by the group's first output channel
  int32_t cout_store;
};
int launch_conv_head_f32(const HeadF32Shape& s, const HeadF32Group* g, hipStream_t st);

// ---- 3xBF16 split path (conv_bf16x3.hip) ----
struct SplitConvGroup {
  const float* in;      // split NHWC input, offset by the group's first input channel (multiple of 16)
  float* out;           // split NHWC output, offset by the group's first output channel (multiple of 8)
  const void* w;        // packed [c16][tap][cop][k-half][hi8 lo8] bf16
  const float* bias;    // [cop] f32
  int32_t cop, cout_store, cin_off;
  float* out32;         // optional dense f32 copy of the output (n*h*w, cs_out32), or null
  int32_t out32_off;
};
struct SplitConvShape {
  int32_t n, h, w, pin, cs_in, pout, cs_out, c16, ks, relu, groups, cs_out32;
  int32_t halo_mode;  // 0 gather kernel; 7x7 only: 1 shared-weight halo (x1 buffer), 2 (x2 buffers); 3 co-split halo (all)
  int32_t splitk;     // 1: the 7x7 raster kernel may split input chunks over workgroups (small launches)
  int32_t regw;       // 1: large launches may take the register-weight kernels (conv_m16r / conv_m16s)
  // 1: the input / output tensor is chunk-planar (only conv_m16_bf16x3 and its split-K reduce take
  // it): per frame [16-channel chunk][4 planes: hi 0-7, lo 0-7, hi 8-15, lo 8-15][hp][wp][16 B]
  // instead of [hp][wp][channels], same frame size, so a chunk's halo rows are contiguous runs
  int32_t in_planar = 0, out_planar = 0;
};
// Bytes between a split tensor's consecutive 16-B channel pieces / consecutive pixels of a row, for
// its layout (planar: [chunk][plane][hp][wp][16 B] per frame; else [hp][wp][cs])
__host__ __device__ __forceinline__ int64_t split_piece_stride(int planar, int hp, int wp) {
  return planar ? (int64_t)hp * wp * 16 : 16;
}
__host__ __device__ __forceinline__ int64_t split_pixel_stride(int planar, int cs) { return planar ? 16 : (int64_t)cs * 4; }
int launch_conv_bf16x3(const SplitConvShape& s, const SplitConvGroup* g, hipStream_t st);
// split-K workspace of a stream (conv_big.hip): floats a capture wanted but could not allocate,
// grow to that size (outside capture; 0 ok), free on stream destruction
size_t splitk_ws_capture_short(hipStream_t st);

int splitk_ws_reserve(hipStream_t st);
void splitk_ws_release(hipStream_t st);
// co-split halo kernel (conv_halo.hip): tile of tr rows x tc cols per workgroup, nh 1-KiB halo pieces per plane
struct HaloTiling {
  int32_t tr, tc, tiles_y, tiles_x, nh;
};
int launch_conv_halo(const SplitConvShape& s, const SplitConvGroup* g, hipStream_t st, int* taken);
// big-tile 7x7 kernel (conv_big.hip): one workgroup per CU, 128 channels x <= 768 pixels
int conv_big_device_init(int device);  // per-device constants; call once per context, outside capture
int launch_conv_big(const SplitConvShape& s, const SplitConvGroup* g, hipStream_t st, int* taken);
bool conv_m16_takes(int n, int h, int w, int groups, int cop_max);
// process-wide launch census of the bf16x3 conv kernels by instantiation (op_conv_census; slots in
// include/openpose_hip.h): incremented on the host at every launch (a graph replay adds nothing)
void census_add(int slot);
// 3x3 conv + ReLU + 2x2 max-pool fused (conv_big.hip)
int launch_conv_big_pool(const SplitConvShape& s, const SplitConvGroup* g, hipStream_t st, int* taken);
// fused 1x1 pair at the end of a branch (conv_head.hip): in -> W1 (ReLU) -> W2 (no ReLU) -> out
struct HeadGroup {
  const float* in;       // split NHWC input, offset by the group's first input channel
  const void* w1;        // split weights of the first 1x1 [c16][plane][cop1][8]
  const float* b1;
  int32_t cop1;
  const void* w2;        // split weights of the second 1x1 [c16][plane][cop2][8]
  const float* b2;
  int32_t cop2;
  float* out;            // split NHWC output, offset by the group's first output channel
  int32_t cout_store;    // channels written (multiple of 4, <= 48)
  float* out32;          // optional dense f32 copy (n*h*w, cs_out32), or null
  int32_t out32_off;
};
struct HeadShape {
  int32_t n, h, w, pin, cs_in, pout, cs_out, ci, co1, groups, cs_out32;
  int32_t in_planar = 0, out_planar = 0;  // 1: chunk-planar input / output (SplitConvShape::in_planar)
};
int launch_conv_head(const HeadShape& s, const HeadGroup* g, hipStream_t st, int* taken);
int launch_maxpool2_split(const float* in, int32_t pin, float* out, int32_t pout, int32_t n, int32_t h, int32_t w,
                          int32_t c, hipStream_t st);
int launch_nchw_to_split16(const float* x, float* out, int32_t n, int32_t h, int32_t w, hipStream_t st);
// the first c16 16-channel chunks of every interior pixel of a split [pixel][channels] tensor ->
// the same channels of a chunk-planar tensor of the same geometry (pad, channel stride cs)
int launch_split_to_planar(const float* in, float* out, int32_t n, int32_t h, int32_t w, int32_t pad, int32_t cs,
                           int32_t c16, hipStream_t st);
int launch_preprocess_split(const uint8_t* frames, int64_t frame_bytes, int64_t row_stride, int32_t n, int32_t sh,
                            int32_t sw, int32_t dh, int32_t dw, float* out, hipStream_t st, float div = 255.0f);
int launch_extract_maps32(const float* m, int32_t cs, int32_t heat_off, int32_t n, int32_t h, int32_t w, float* paf,
                          float* heat, hipStream_t st);
int launch_maxpool2(const float* in, int32_t pin, float* out, int32_t pout, int32_t n, int32_t h, int32_t w,
                    int32_t c, hipStream_t st);
int launch_nchw_to_nhwc8(const float* x, float* out, int32_t n, int32_t h, int32_t w, hipStream_t st);
int launch_extract_maps(const float* cat, int32_t n, int32_t h, int32_t w, float* paf, float* heat, hipStream_t st);
int launch_preprocess(const uint8_t* frames, int64_t frame_bytes, int64_t row_stride, int32_t n, int32_t sh,
                      int32_t sw, int32_t dh, int32_t dw, float* out, hipStream_t st);
int launch_preprocess_planar(const uint8_t* bgr, int64_t row_stride, int32_t sh, int32_t sw, int32_t dh,
                             int32_t dw, float* out_nchw, hipStream_t st);

// conv1_1 as f32 FMAs (conv11.hip); frames != nullptr fuses the cv2 LINEAR network-input resize
int launch_conv11_split(const uint8_t* frames, int64_t frame_bytes, int64_t row_stride, int32_t sh, int32_t sw,
                        const float* x0, int32_t n, int32_t h, int32_t w, const float* wt, const float* bias,
                        float* out, hipStream_t st);

// conv1_1 + conv1_2 + 2x2 max-pool fused (conv1_pair.hip); frames as for launch_conv11_split
int launch_conv1_pair(const uint8_t* frames, int64_t frame_bytes, int64_t row_stride, int32_t sh, int32_t sw,
                      const float* x0, int32_t n, int32_t h, int32_t w, const float* wt11, const float* b11,
                      const void* w12, const float* b12, float* out, int32_t pout, hipStream_t st);

// ---- multi-scale path (precise.hip) ----
// n frames: frame f at bgr + f * src_fstride bytes -> out + f * dst_ffloats floats (one launch)
int launch_preprocess_cubic(const uint8_t* bgr, int64_t row_stride, int32_t sh, int32_t sw, int32_t rh, int32_t rw,
                            int32_t ph, int32_t pw, bool split, float* out, int32_t n, int64_t src_fstride,
                            int64_t dst_ffloats, hipStream_t st);
int launch_resize_cubic_f32(const float* src, int64_t sstride, int32_t pstride, int32_t sh, int32_t sw, int32_t cn,
                            float* dst, int32_t dh, int32_t dw, int32_t mode, float div, hipStream_t st);
// mode 1 (planar destination) for n frames at once (source / destination frame strides in floats):
// upsampling resizes (dh >= sh, dw >= sw) share each source row's horizontal sums among the output
// rows of an 8-row block (round 3), the rest run resize_cubic_f32 per frame
int launch_resize_cubic_f32_frames(const float* src, int64_t sstride, int32_t pstride, int64_t src_fstride, int32_t sh,
                                   int32_t sw, int32_t cn, float* dst, int64_t dst_fstride, int32_t dh, int32_t dw,
                                   int32_t n, hipStream_t st);
// planar source (c*cstride + y*sstride + x) -> planar destination, modes 1-3 (precise.hip)
// Per scale k: the padded-size map of one frame (planar, cstride floats per channel, sstride per
// row), cropped to sh x sw, and the host-computed cubic scales to the output size.
struct CubicMeanArgs {
  const float* src[OP_MAX_SCALES];
  int64_t cstride[OP_MAX_SCALES], sstride[OP_MAX_SCALES];
  int64_t fstride[OP_MAX_SCALES];  // floats per frame (the _rows form: every frame in one launch)
  int sh[OP_MAX_SCALES], sw[OP_MAX_SCALES];
  double scx[OP_MAX_SCALES], scy[OP_MAX_SCALES];
  int ns;
};
int launch_resize_cubic_f32_planar_mean(const CubicMeanArgs& a, float* dst, int32_t dh, int32_t dw, int32_t npaf,
                                        int32_t nheat, hipStream_t st);
// n frames (src[k] = frame 0, fstride[k] apart; dst frames dst_fstride apart); *taken false when
// a scale's rows would exceed its LDS budget (then run the per-frame form)
int launch_resize_cubic_f32_planar_mean_rows(const CubicMeanArgs& a, float* dst, int64_t dst_fstride, int32_t n,
                                             int32_t dh, int32_t dw, int32_t npaf, int32_t nheat, hipStream_t st,
                                             bool* taken);
int launch_resize_cubic_f32_planar_mean_tile(const CubicMeanArgs& a, float* dst, int64_t dst_fstride, int32_t n,
                                             int32_t dh, int32_t dw, int32_t npaf, int32_t nheat, hipStream_t st,
                                             bool* taken);
// detect_precise's two map resizes per scale fused (round 4): the padded-size maps are never
// written; see precise.hip resize_cubic_fused_mean.  low[k]: scale k's last-stage maps, planar
// [frame][npaf + nheat][lh][lw] f32 (launch_maps_planar).
struct CubicFusedArgs {
  int ns;
  const float* low[OP_MAX_SCALES];
  int64_t lframe[OP_MAX_SCALES];                         // floats per frame of low[k]
  int lh[OP_MAX_SCALES], lw[OP_MAX_SCALES];              // last-stage map size
  int pw[OP_MAX_SCALES];                                 // first resize's width (padded input width)
  int rh[OP_MAX_SCALES], rw[OP_MAX_SCALES];              // crop = second resize's source size
  double s1x[OP_MAX_SCALES], s1y[OP_MAX_SCALES];         // first resize: cv_cubic_scale(pw, lw), (ph, lh)
  double s2x[OP_MAX_SCALES], s2y[OP_MAX_SCALES];         // second: cv_cubic_scale(w, rw), (h, rh)
  int rx_cap, ry_cap, lr_cap, pc_cap;                    // LDS extents (host bounds)
};
// false (and nothing launched) when a scale's tile extents exceed the kernel's LDS budget: the
// caller then runs the two-pass path
size_t cubic_fused_lds(CubicFusedArgs& a);  // sets a's extents; 0 = over the kernel's LDS budget
int launch_resize_cubic_fused_mean(CubicFusedArgs a, float* dst, int32_t n, int32_t dh, int32_t dw, int32_t npaf,
                                   int32_t nheat, hipStream_t st, bool* taken);
// (frames, lh, lw, cn) maps at src (row stride sstride, pixel stride pstride, frame stride fstride
// floats) -> planar dst [frame][dst_c0 + c][lh][lw] with dst_nch channels per frame
int launch_maps_planar(const float* src, int64_t sstride, int32_t pstride, int64_t fstride, int32_t lh, int32_t lw,
                       int32_t cn, float* dst, int32_t dst_c0, int32_t dst_nch, int32_t n, hipStream_t st);
int launch_resize_cubic_f32_planar(const float* src, int64_t cstride, int64_t sstride, int32_t sh, int32_t sw,
                                   int32_t cn, float* dst, int32_t dh, int32_t dw, int32_t mode, float div,
                                   hipStream_t st);
int launch_resize_cubic_u8(const uint8_t* src, int64_t sstride, int32_t sh, int32_t sw, int32_t cn, uint8_t* dst,
                           int32_t dh, int32_t dw, hipStream_t st);

// Post-process device state for a batch of frames.
struct PostBuffers {
  int32_t maxp;        // peaks per joint cap
  int64_t maxc;        // candidates per limb cap (= maxp*maxp)
  int32_t maxs;        // subsets per frame cap (= 19*maxp)
  float* up;           // [B][18][Hm][Wm] full-res heat planes handed in through op_compute_peaks
  int32_t* peak_xy;    // [B][18][maxp]  x | y << 16
  float* peak_score;   // [B][18][maxp]
  int32_t* peak_cnt;   // [B][18]
  int32_t* stage_key;  // [B][18][maxp] unordered peaks (y*mw + x) before peak_sort
  float* stage_score;  // [B][18][maxp]
  double* cand_score;  // [B][19][maxc]
  int32_t* cand_idx;   // [B][19][maxc]
  int32_t* cand_cnt;   // [B][19]
  int32_t* conn_ab;    // [B][19][maxp][2] global peak ids
  double* conn_score;  // [B][19][maxp]
  int32_t* conn_cnt;   // [B][19]
  int32_t* sub_ids;    // [B][maxs][18]
  double* sub_sc;      // [B][maxs][2]  score, count
  double* res_poses;   // [B][maxs][18][3]
  double* res_scores;  // [B][maxs]
  double* res_subsets; // [B][maxs][20] kept subset rows (grouping_key_points output)
  int32_t* res_hdr;    // [B][4]: status, n_peaks, n_persons, reserved
  double* gauss_w;     // [kGaussTable] device Gaussian taps: the CPU branch's 2r+1 at 0, the GPU branch's at kGaussGpuOff
  unsigned* used;      // big mode only (else null): [B][19][2][ceil(maxp/32)] greedy used-peak bitsets
};

constexpr int kGaussTable = 128;  // doubles in PostBuffers::gauss_w
constexpr int kGaussGpuOff = 64;  // the GPU-branch taps' offset in it
constexpr int kMaxGaussR = 16;    // largest radius of the tiled peak kernel (postproc.hip kMaxR)

struct PostShape {
  int32_t n;             // frames
  int32_t lh, lw;        // network map size (low res)
  int32_t mh, mw;        // post-process map size
  int32_t radius;        // Gaussian radius (10)
  int32_t peak_mode;     // op_set_peak_mode: 1 = GPU-branch peaks in the single-scale (HeatLow) path
  int32_t gpu_radius;    // its Gaussian radius (ksize / 2 = 8)
  double img_len;        // distance-prior length (map_w, pose_detector.py:511)
  double sx, sy;         // output rescale (orig_w / map_w, orig_h / map_h; 1 in precise mode)
  float peak_thresh;
  int32_t n_integ;       // 10
  int32_t n_integ_thresh;// 8
  double inner_thresh, len_ratio, len_penalty;
  int32_t subset_min;    // 3
  double subset_score;   // 0.2
  int32_t limbs[OP_N_LIMBS][2];
};

// Low-res network maps as the post-process reads them: the stage-input (concat) NHWC buffer layout,
// element (frame f, map channel c, y, x) at base + f*fstride + ((y+pad)*(lw+2*pad) + x+pad)*cs + c.
struct MapSource {
  const float* base;
  int64_t fstride;
  int32_t pad;
  int32_t cs;
  int32_t paf_off;   // channel of PAF 0
  int32_t heat_off;  // channel of heatmap 0
};

int launch_post_maps(const MapSource& src, const PostShape& s, PostBuffers& b, hipStream_t st);
// Sub-steps on already-upsampled inputs (stage-level ABI)
// full-resolution planar maps; fstride = floats between frames (0: 18 joint planes per frame)
int launch_peaks_from_full(const float* heat_full, int32_t n_joint, int32_t mh, int32_t mw, const PostShape& s,
                           PostBuffers& b, hipStream_t st, int64_t fstride = 0);
int launch_connections_full(const float* paf_full, int32_t mh, int32_t mw, const PostShape& s, PostBuffers& b,
                            hipStream_t st, int64_t fstride = 0);
int launch_grouping(const PostShape& s, PostBuffers& b, hipStream_t st);
int launch_resize_images(const float* x, int32_t c, int32_t h, int32_t w, int32_t oh, int32_t ow, float* y,
                         hipStream_t st);

// s_waitcnt vmcnt(n) for a wave-uniform run-time n (counted waits over interleaved load streams).
__device__ __forceinline__ void wait_vm_dyn(int n) {  // n is wave-uniform
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
    case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    case 11: asm volatile("s_waitcnt vmcnt(11)" ::: "memory"); break;
    case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    case 13: asm volatile("s_waitcnt vmcnt(13)" ::: "memory"); break;
    case 14: asm volatile("s_waitcnt vmcnt(14)" ::: "memory"); break;
    case 15: asm volatile("s_waitcnt vmcnt(15)" ::: "memory"); break;
    case 16: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
    case 17: asm volatile("s_waitcnt vmcnt(17)" ::: "memory"); break;
    case 18: asm volatile("s_waitcnt vmcnt(18)" ::: "memory"); break;
    case 19: asm volatile("s_waitcnt vmcnt(19)" ::: "memory"); break;
    case 20: asm volatile("s_waitcnt vmcnt(20)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

}  // namespace op
