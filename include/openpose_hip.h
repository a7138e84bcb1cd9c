/*
 * openpose_hip.h — C ABI of the MI355X (gfx950) OpenPose inference path.
 *
 * Drop-in replacement for the hot path of nk35jk/Chainer_Realtime_Multi-Person_Pose_Estimation:
 * PoseDetector.__call__ (pose_detector.py:484-517) = CocoPoseNet forward
 * (models/CocoPoseNet.py:132-262) + PAF post-process (pose_detector.py:75-265).
 * The reference has no FFI of its own (pure Python); every entry point below names the
 * reference function it replaces.  The Python host package
 * (chainer_realtime_multi-person_pose_estimation_amd/) binds these with ctypes.
 *
 * Conventions: plain pointers + sizes; all host pointers, row-major, C-contiguous.
 * Every function returns an int status (OP_OK = 0); op_last_error() describes the last failure
 * on the calling thread.  A context is single-threaded and owns one HIP stream on one device.
 */
#ifndef OPENPOSE_HIP_H
#define OPENPOSE_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OP_OK 0
#define OP_ERR_INVALID 1  /* bad argument / shape */
#define OP_ERR_HIP 2      /* HIP runtime failure */
#define OP_ERR_CAPACITY 3 /* a per-frame cap (peaks/persons) was exceeded */
#define OP_ERR_INDEX 4    /* reference raises IndexError (pose_detector.py:197): a connection hit >=3 subsets */
#define OP_ERR_STATE 5    /* weights not set / no staged frames */
#define OP_ERR_TIMEOUT 6  /* a multi-GPU gather did not complete in time (a rank stalled or died) */

#define OP_N_JOINTS 18 /* JointType, entity.py:9-46 */
#define OP_N_LIMBS 19  /* params['limbs_point'], entity.py:85-105 */
#define OP_N_PAF 38
#define OP_N_HEAT 19
#define OP_N_LAYERS 92 /* models/CocoPoseNet.py:26-129 */
#define OP_MAX_SCALES 8 /* inference_scales entries (entity.py:74) */

/* Inference parameters — entity.py:70-105 (same names and meaning). */
typedef struct op_params {
  int32_t inference_img_size;   /* 368 */
  int32_t heatmap_size;         /* 320 */
  double gaussian_sigma;        /* 2.5 (scipy gaussian_filter, truncate 4.0) */
  int32_t n_integ_points;       /* 10 */
  int32_t n_integ_points_thresh;/* 8 */
  double heatmap_peak_thresh;   /* 0.05 */
  double inner_product_thresh;  /* 0.05 */
  double limb_length_ratio;     /* 1.0 */
  double length_penalty_value;  /* 1 */
  int32_t n_subset_limbs_thresh;/* 3 */
  double subset_score_thresh;   /* 0.2 */
  int32_t limbs_point[OP_N_LIMBS][2];
  int32_t downscale;            /* 8 */
  int32_t n_scales;             /* len(inference_scales) = 4 (detect_precise) */
  double inference_scales[OP_MAX_SCALES]; /* [0.5, 1, 1.5, 2] */
} op_params;

/* Capacities of a context (device buffers are sized from these; 0 = default). */
typedef struct op_limits {
  int32_t max_batch;           /* frames per run (default 1) */
  int32_t max_net_h, max_net_w;/* largest network input, multiples of 8 (default 368 x 656) */
  int32_t max_map_h, max_map_w;/* largest post-process map (default 320 x 576) */
  int32_t max_peaks_per_joint; /* default 512 */
  int32_t max_frame_h, max_frame_w; /* largest raw BGR frame for the staged path (default 720 x 1280) */
} op_limits;

/* Per-frame result header.  status is the frame's OP_* code. */
typedef struct op_frame_result {
  int32_t status;
  int32_t n_peaks;   /* len(all_peaks) */
  int32_t n_persons; /* len(subsets) after the keep filter (pose_detector.py:248) */
  int32_t map_w, map_h;
  int32_t net_w, net_h;
} op_frame_result;

typedef struct op_ctx op_ctx;

const char* op_last_error(void);

/* Provenance of the loaded binary (no reference counterpart): writes "sha256:<64 hex>;defs=<flags>"
 * + NUL into out (OP_ERR_INVALID when cap is too small), the digest of the library's sources as
 * built -- sha256 of the `sha256sum` listing of csrc/ *.hip *.hpp *.cpp, csrc/Makefile and
 * include/ *.h (paths relative to csrc/, sorted), computed by the Makefile at build time;
 * _lib.source_digest() recomputes it from the tree -- and the build flags beyond the Makefile's own
 * (DEFS, FLAGS_* overrides; empty for the product library). */
int op_build_info(char* out, int32_t cap);
int op_default_params(op_params* p);
int op_default_limits(op_limits* l);

/* Layer table of models/CocoPoseNet.py:26-129 (name, Ci, Co, ksize) in declaration order. */
int op_layer_info(int index, const char** name, int32_t* ci, int32_t* co, int32_t* ksize);

/* PoseDetector.__init__ (pose_detector.py:16-35): context on HIP device `device`. */
int op_create(const op_params* params, const op_limits* limits, int device, op_ctx** out);
int op_destroy(op_ctx* ctx);

/* Arithmetic of the forward convolutions.  OP_PRECISION_BF16X3 (default): every f32 operand is
 * split into bf16 hi + lo and each product formed as hi*hi + hi*lo + lo*hi on the bf16 matrix
 * cores with f32 accumulation (~16-bit products, 5.3x the f32-MFMA rate; |err| ~3e-5 on the maps,
 * inside the 1e-3 parity tolerance).  OP_PRECISION_FP32: exact f32 products (v_mfma_f32_32x32x2_f32). */
#define OP_PRECISION_FP32 0
#define OP_PRECISION_BF16X3 1
int op_set_precision(op_ctx* ctx, int32_t mode);
int op_get_precision(op_ctx* ctx, int32_t* mode);

/* Kernel family of the bf16x3 convolutions (a tuning knob; every family computes the same
 * products, parity-tested): 4 (default): large 3x3 launches (>= 1024 workgroups) take the
 * register-weight kernel with a double-buffered halo, conv_m16r, which sums in exactly the order of
 * conv_m16k below, so results are bit-identical to 5; 5 = 4 without it: shared-weight halo tiles
 * (conv_big.hip): the 7x7 layers
 * on v_mfma_f32_16x16x32_bf16 tap pairs over raster tiles (640-pixel ranges of the batch that
 * span frame borders), the 3x3 layers on 16x16x32 with K = 32 input channels over 8 x 32 / 4 x 48
 * tiles (32x32x16 kernel for the 64-channel ones), the 1x1 layers on co-split halo tiles;
 * 3 co-split halo tiles for every layer (conv_halo.hip); 0 the per-tap gather kernel.  Shapes a
 * family does not take use the gather kernel.  (Round-1 experiment families -- double-buffered
 * halos, rectangular 7x7 tap pairs, register weights -- live in git history: tools/build_rev.sh
 * builds that revision as an A/B variant.) */
int op_set_conv_algo(op_ctx* ctx, int32_t algo);
/* Layout of the 7x7 stage tensors of stages 2-6 (default 1; env OP_STAGE_PLANAR=0 sets new
 * contexts to 0).  1: chunk-planar ([16-channel chunk][hi/lo plane][row][col] per frame) wherever
 * the 7x7 kernel conv_m16 takes every 7x7 launch of the geometry -- its halo loads are then
 * contiguous runs (about half the HBM reads); 0: [row][col][channels].  Same kernels, same
 * arithmetic and order: the maps are bit-identical either way.  No reference counterpart (the
 * reference's tensors live in Chainer/cuDNN). */
int op_set_stage_layout(op_ctx* ctx, int32_t planar);
/* Batch invariance (default off).  A launch that fills few CUs (one frame, one crop) splits the
 * 7x7 convolutions' input channels over several workgroups and sums their f32 partials, so a
 * frame's maps then differ from the same frame inside a larger batch by f32 re-association (~1e-5;
 * near-threshold peaks of noisy maps can flip).  enable != 0 keeps one accumulation order for
 * every batch size (single-frame latency ~2x). */
int op_set_batch_invariant(op_ctx* ctx, int32_t enable);
/* Peak semantics of the single-scale post-process (op_detect, op_postprocess, op_run_staged*).
 * The reference's compute_peaks_from_heatmaps has two branches and takes the one of the array it
 * is handed: the CPU branch (pose_detector.py:82-110: scipy gaussian_filter sigma 2.5, reflect
 * boundary, normalised 21 taps; strict > 4-neighbour NMS) for a CPU detector, the GPU branch
 * (:111-132: F.convolution_2d with the ksize x ksize kernel of create_gaussian_kernel :38-44 --
 * exp(-d^2 / 2 sigma^2) / (2 pi sigma^2), not normalised -- zero padding ksize/2; >= NMS) in
 * __call__ of a detector built with device >= 0 (:29-35, :496-508).  OP_PEAKS_CPU_BRANCH (0, the
 * default and the parity target of the golden fixtures) or OP_PEAKS_GPU_BRANCH (1; ksize odd,
 * 3 .. 33, entity.py's 'ksize' is 17).  op_detect_precise and op_compute_peaks keep the CPU branch in
 * either mode, as the reference does: their heatmaps are NumPy arrays there (:470-475). */
#define OP_PEAKS_CPU_BRANCH 0
#define OP_PEAKS_GPU_BRANCH 1
int op_set_peak_mode(op_ctx* ctx, int32_t mode, int32_t ksize);

/* serializers.load_npz(weights_file, model) (pose_detector.py:26): 92 layers in op_layer_info
 * order, W as Chainer (Co, Ci, k, k) f32 and b as (Co,) f32.  Packed into the kernel layout
 * and uploaded once. */
int op_set_weights(op_ctx* ctx, const float* const* W, const float* const* b);

/* PoseDetector.__call__ (pose_detector.py:484-517), single scale.  bgr: h x w x 3 uint8,
 * row_stride bytes per row.  poses: cap x 18 x 3 f64, scores: cap f64. */
int op_detect(op_ctx* ctx, const uint8_t* bgr, int32_t h, int32_t w, int64_t row_stride,
              double* poses, double* scores, int32_t cap, op_frame_result* res);

/* PoseDetector.detect_precise (pose_detector.py:433-482), the multi-scale mode (precise=True):
 * per scale of params.inference_scales a cv2.resize(INTER_CUBIC) of the frame to
 * ceil(w*m) x ceil(h*m), m = scale * inference_img_size / min(h, w), pad_image to a multiple of
 * `downscale` with BGR (104, 117, 123), the forward, cubic resizes of the last-stage maps to the
 * padded size, crop, cubic resize to h x w; the maps are averaged over the scales and
 * post-processed at the original resolution (img_len = w, no rescale).  pafs_out (38, h, w) and
 * heat_out (19, h, w) f32 receive the averaged maps (the reference's self.pafs / self.heatmaps)
 * when non-null. */
int op_detect_precise(op_ctx* ctx, const uint8_t* bgr, int32_t h, int32_t w, int64_t row_stride,
                      double* poses, double* scores, int32_t cap, op_frame_result* res,
                      float* pafs_out, float* heat_out);

/* ---- Stage entry points (same semantics as the named reference code; used by the parity tests) ---- */

/* cv2.resize(src, (out_w, out_h), interpolation=cv2.INTER_CUBIC) (pose_detector.py:443, 461-467):
 * src h x w x cn, dtype 0 = uint8, 1 = float32; dst out_h x out_w x cn of the same dtype. */
int op_resize_cubic(op_ctx* ctx, const void* src, int32_t dtype, int32_t h, int32_t w, int32_t cn, void* dst,
                    int32_t out_h, int32_t out_w);

/* cv2.resize(orig_img, (out_w, out_h)) + preprocess (pose_detector.py:493-494, 426-431):
 * x_out (1, 3, out_h, out_w) f32 = u8/255 - 0.5, BGR order kept. */
int op_preprocess(op_ctx* ctx, const uint8_t* bgr, int32_t h, int32_t w, int64_t row_stride,
                  int32_t out_w, int32_t out_h, float* x_out);

/* CocoPoseNet.__call__ (models/CocoPoseNet.py:132-262): x (n, 3, h, w) f32 -> last-stage
 * pafs (n, 38, h/8, w/8) and heatmaps (n, 19, h/8, w/8).  h, w multiples of 8. */
int op_forward(op_ctx* ctx, const float* x, int32_t n, int32_t h, int32_t w, float* pafs, float* heatmaps);

/* As op_forward, but every stage's outputs: the (pafs, heatmaps) lists CocoPoseNet.__call__ returns
 * (models/CocoPoseNet.py:164-165, 180-181, ..., 262).  pafs (6, n, 38, h/8, w/8), heatmaps
 * (6, n, 19, h/8, w/8); stage s at index s-1. */
int op_forward_stages(op_ctx* ctx, const float* x, int32_t n, int32_t h, int32_t w, float* pafs, float* heatmaps);

/* F.resize_images (pose_detector.py:501-502; Chainer <= 6 align-corners bilinear): (c,h,w) -> (c,oh,ow). */
int op_resize_images(op_ctx* ctx, const float* x, int32_t c, int32_t h, int32_t w, int32_t oh, int32_t ow, float* y);

/* Capacities.  Like the reference (pose_detector.py:75-250 has no caps) the post-process is
 * uncapped: a frame with more peaks per joint than op_limits.max_peaks_per_joint, or more subsets
 * than the batched grouping holds, is re-run alone with buffers sized from its own counts (only
 * device memory bounds it).  OP_ERR_CAPACITY then means either that device memory ran out, or
 * that the caller's output array is too small -- in which case the needed row count is written
 * to the count output (*n_peaks, conn_off[19], *n_subsets, res->n_persons) so the call can be
 * repeated with a larger array. */

/* compute_peaks_from_heatmaps (pose_detector.py:75-110, CPU semantics): heatmaps (c, h, w),
 * channel c-1 dropped.  peaks: rows [joint, x, y, score, id] f64. */
int op_compute_peaks(op_ctx* ctx, const float* heatmaps, int32_t c, int32_t h, int32_t w,
                     double* peaks, int64_t cap, int64_t* n_peaks);

/* compute_connections (pose_detector.py:161-181, with compute_candidate_connections :135-159):
 * pafs (38, h, w) at map resolution, peaks (n, 5).  conn rows [id_a, id_b, score]; limb l's rows
 * are conn[conn_off[l] .. conn_off[l+1]). */
int op_compute_connections(op_ctx* ctx, const float* pafs, int32_t h, int32_t w, const double* peaks,
                           int64_t n_peaks, double img_len, double* conn, int64_t cap, int64_t* conn_off);

/* grouping_key_points (pose_detector.py:183-250): subsets (S, 20) f64 after the keep filter. */
int op_grouping(op_ctx* ctx, const double* conn, const int64_t* conn_off, const double* peaks,
                int64_t n_peaks, double* subsets, int64_t cap, int64_t* n_subsets);

/* pose_detector.py:501-517 from the last-stage network maps (38,h,w) + (19,h,w) of one frame;
 * the image was orig_h x orig_w. */
int op_postprocess(op_ctx* ctx, const float* paf_low, const float* heat_low, int32_t h, int32_t w,
                   int32_t orig_h, int32_t orig_w, double* poses, double* scores, int32_t cap,
                   op_frame_result* res);

/* ---- Device-resident batched path (frame-parallel serving / bench) ---- */

/* Copy n BGR frames (n x h x w x 3 u8, contiguous) into the context's HBM staging area. */
int op_stage_frames(op_ctx* ctx, const uint8_t* frames, int32_t n, int32_t h, int32_t w);
/* Asynchronous staging for a frame stream: copy n BGR frames (n x h x w x 3 u8, contiguous;
 * page-locked memory from op_host_alloc makes the copy truly asynchronous) on the context's copy
 * stream into a 2-slot device ring and return.  The next op_run_staged* waits for that copy on the
 * compute stream and makes these frames the staged set, so the upload of step k+1 overlaps the
 * compute of step k (the reference uploads each frame inside __call__, pose_detector.py:496-497).
 * The copy may still be reading the host buffer after op_upload_frames and the consuming
 * op_run_staged* have returned: the buffer must stay unchanged until the copy has completed --
 * after op_upload_wait, op_synchronize, or any later call that waited for the consuming run. */
int op_upload_frames(op_ctx* ctx, const uint8_t* frames, int32_t n, int32_t h, int32_t w);
/* Block until every op_upload_frames copy issued so far has finished reading its host buffer (the
 * buffers may then be refilled).  No reference counterpart (the reference's uploads are
 * synchronous, pose_detector.py:496-497). */
int op_upload_wait(op_ctx* ctx);
/* Page-locked host memory for op_upload_frames sources. */
int op_host_alloc(size_t bytes, void** p);
int op_host_free(void* p);
/* Optional: post-process these maps (n x 57 x mh x mw: 38 PAF then 19 heat) instead of the network's
 * own (synthetic-map benchmarking; default off; op_use_staged_maps).  mh x mw = the network map size
 * (h/8 x w/8 of the network input) feeds op_run_staged; mh x mw = the staged frame size (stage the
 * frames first) feeds op_run_staged_precise's full-resolution post-process in place of the averaged
 * maps, which are still computed. */
int op_stage_maps(op_ctx* ctx, const float* maps, int32_t n, int32_t mh, int32_t mw);
int op_use_staged_maps(op_ctx* ctx, int32_t enable);
/* Enqueue the full path (resize+normalise, 92 convs, post-process) on the staged frames; async. */
int op_run_staged(op_ctx* ctx);
/* detect_precise (pose_detector.py:433-482) on every staged frame: per inference scale one batched
 * forward of all staged frames, per-frame cubic map resizes into the running mean, then the
 * full-resolution post-process; results via op_fetch_result(s) as for op_run_staged (map_w/h = the
 * frame size, net_w/h = the largest scale's network input).  Synchronous on the context stream. */
int op_run_staged_precise(op_ctx* ctx);
/* Capture op_run_staged as a hipGraph and replay it (same semantics, fewer launches). */
int op_run_staged_graph(op_ctx* ctx);
/* Contents of the step graph op_run_staged_graph captured last (debugging / regression aid; no
 * reference counterpart): node counts by kind.  host_nodes = memcpy nodes with a host-memory source
 * or destination, and host / event / other nodes -- none may exist: the step graph touches device
 * memory only (uploads and result fetches stay outside it, on their own streams / calls).
 * OP_ERR_STATE when no graph has been captured. */
int op_graph_info(op_ctx* ctx, int32_t* nodes, int32_t* kernels, int32_t* memsets, int32_t* memcpys,
                  int32_t* host_nodes);
int op_synchronize(op_ctx* ctx);
/* Results of staged frame i (after op_synchronize). */
int op_fetch_result(op_ctx* ctx, int32_t frame, double* poses, double* scores, int32_t cap, op_frame_result* res);

/* Results of staged frames [first, first+n) in three copies: poses (n x cap x 18 x 3 f64),
 * scores (n x cap f64), res (n headers).  A frame's status is in its header; the call itself
 * fails only on bad arguments / HIP errors or when a frame's person count exceeds cap. */
int op_fetch_results(op_ctx* ctx, int32_t first, int32_t n, double* poses, double* scores, int32_t cap,
                     op_frame_result* res);

/* Network maps of staged frames [first, first+n) after op_synchronize: the last-stage maps of
 * op_run_staged (pafs (n, 38, h/8, w/8), heatmaps (n, 19, h/8, w/8) of the network input h x w), or
 * after op_run_staged_precise the averaged full-resolution maps (n, 38|19, H, W) -- the
 * self.pafs / self.heatmaps detect_precise leaves (pose_detector.py:469-470).  *mh, *mw receive the
 * map size; pafs = heatmaps = NULL only queries it. */
int op_fetch_maps(op_ctx* ctx, int32_t first, int32_t n, float* pafs, float* heatmaps, int32_t* mh, int32_t* mw);
/* HIP-event timing of the last op_run_staged: ms spent in the conv kernels, the post-process kernels
 * and total, recorded on the context stream. */
int op_last_timing(op_ctx* ctx, double* conv_ms, double* post_ms, double* total_ms);
/* Per-kernel-class HIP-event timing of the launches enqueued by op_run_staged while enabled
 * (event pairs on the context stream around every launch of the class).  Classes:
 * 0 = 7x7 stage convs (the dominant kernel), 1 = 3x3 convs, 2 = 1x1 convs, 3 = post-process
 * (peaks, line integrals, greedy, grouping; single scale and detect_precise's full resolution),
 * 4 = frame input (resize + pad + normalise kernels not fused into a conv), 5 = map resizes
 * (detect_precise's cubic resizes of the last-stage maps and their scale mean), 6 = other (pools,
 * layout copies, result packing).  op_profile_read resolves pending pairs (after op_synchronize) and returns the totals since the
 * last reset: summed ms, launch count, algorithmic FLOPs and algorithmic HBM bytes. */
int op_profile_enable(op_ctx* ctx, int32_t enable);
int op_profile_read(op_ctx* ctx, int32_t cls, double* ms, int64_t* launches, double* flops, double* bytes);
int op_profile_reset(op_ctx* ctx);
/* Which classes op_profile_enable times (bit c = class c; default 0x7F = all). */
#define OP_PROFILE_CLASSES 7
int op_profile_classes(op_ctx* ctx, int32_t mask);

/* Launch census of the bf16x3 conv kernels (process-wide, all contexts; counted on the host when a
 * launch is enqueued, so a replayed hipGraph adds nothing): counts[i] for i < n, then the counts are
 * zeroed if reset.  Lets a test assert which kernel instantiation a configuration really ran (the
 * 7x7 tile size is picked per launch shape by a cost model).  No reference counterpart.
 * Slots: 1..10 = conv_m16_bf16x3<7, NPX> launches with NPX 16-px blocks per wave (640-px raster
 * tiles at 10), and: */
#define OP_CENSUS_7X7_SPLITK 11  /* 7x7 launches that split their input chunks (split-K) */
#define OP_CENSUS_7X7_OTHER 12   /* 7x7 on the conv_big fallback family */
#define OP_CENSUS_3X3_W48 13     /* conv_m16k_bf16x3<false> on 4 x 48 tiles */
#define OP_CENSUS_3X3_W32 14     /* conv_m16k_bf16x3<false> on 8 x 32 tiles */
#define OP_CENSUS_3X3_POOL 15    /* conv_m16k_bf16x3<true> (fused 2x2 max-pool) */
#define OP_CENSUS_3X3_SPLITK 16  /* conv_m16k launches with split-K */
#define OP_CENSUS_3X3_BIG 17     /* conv_big_bf16x3<3, ...> (shapes conv_m16k does not take) */
#define OP_CENSUS_CONV1_PAIR 18  /* conv1_pair_bf16x3 (fused conv1_1 + conv1_2 + pool) */
#define OP_CENSUS_3X3_R256 19    /* conv_m16r_bf16x3<8, ...> (register weights, 256 channels per workgroup) */
#define OP_CENSUS_3X3_R128 20    /* conv_m16r_bf16x3<4, ...> (128 channels per workgroup) */
#define OP_CENSUS_3X3_R_POOL 21  /* conv_m16r_bf16x3<., ., ., true> (fused 2x2 max-pool) */
#define OP_CENSUS_7X7_PLANAR 22  /* 7x7 launches on chunk-planar tensors (op_set_stage_layout) */
#define OP_CENSUS_7X7_FRAME_ALIGNED 23  /* conv_m16 7x7 launches on frame-aligned raster tiles (no tile
                                           crosses a frame; else batch rasters that do) */
#define OP_CENSUS_7X7_TIGHT 24   /* conv_m16 7x7 launches with the tight halo pitch w + 6 (wide maps) */
#define OP_CENSUS_CUBIC_FUSED 25 /* detect_precise map resizes as one fused pass (resize_cubic_fused_mean) */
#define OP_CENSUS_CUBIC_TWO_PASS 26 /* ... as the two-pass path (padded-size maps in HBM) */
/* slot 27: retired in round 5 (the in-kernel split-K experiment was removed) */
#define OP_CENSUS_CUBIC_ROWS 28  /* two-pass second resize as one row-block launch for the batch
                                    (resize_cubic_f32_planar_mean_rows), else one launch per frame */
#define OP_CENSUS_F32_LDS 29     /* exact-f32 3x3 / 7x7 launches on the LDS-halo kernel conv_f32_lds (round 5) */
#define OP_CENSUS_7X7_STAG 30       /* conv_m16 7x7 launches with the staggered halves (round 5) */
#define OP_CENSUS_7X7_PLAIN_RING 31 /* ... with one ring barrier per pair for all 8 waves */
#define OP_CENSUS_7X7_Q 32          /* 7x7 launches on the small-launch kernel conv_m16q_bf16x3 (round 5) */
#define OP_CENSUS_7X7_CIRC 33       /* staggered conv_m16 7x7 launches with circular halo planes (round 6) */
#define OP_CENSUS_PRECISE_SIDE 34   /* detect_precise runs whose small scales ran on the side stream (round 6) */
#define OP_CENSUS_7X7_Q_IWG 35      /* conv_m16q launches with both tap ranges in one 8-wave workgroup (round 6) */
#define OP_CENSUS_7X7_LIN 36        /* conv_m16 launches with linear halo sources (LIN, round 6) */
#define OP_CENSUS_7X7_Q_BPF 37      /* conv_m16q launches with B fragments one tap ahead (round 6) */
#define OP_CENSUS_7X7_PERS 38       /* conv_m16 launches as a persistent grid of one workgroup per CU (round 6) */
#define OP_CENSUS_SLOTS 40
int op_conv_census(int32_t* counts, int32_t n, int32_t reset);

/* Algorithmic FLOPs of the forward for one frame of net size h x w (2*Ci*Co*k*k*H*W summed). */
double op_forward_flops(int32_t h, int32_t w);

/* ---- Multi-GPU result gather: frames shard round-robin over one process per GPU; the
 * only exchange is the per-frame result records, gathered to rank 0 over RCCL from device memory ----
 *
 * Record of one frame (record_bytes = 32 + max_persons * 55 * 8): int32 {status, n_peaks,
 * n_persons, 0}, int64 global frame id (frame_base + i * frame_stride), 8 zero bytes, then
 * max_persons x 18 x 3 f64 poses and max_persons f64 scores (persons past max_persons are not
 * carried; n_persons still counts them; rows past n_persons are zero).  A frame over the batched
 * post-process caps carries status OP_ERR_CAPACITY (op_fetch_result re-runs it uncapped; in a
 * gather, op_comm_overflow_result). */
int op_pack_results(op_ctx* ctx, int32_t first, int32_t n, int32_t max_persons, int64_t frame_base,
                    int32_t frame_stride, void* host_records);
#define OP_COMM_ID_BYTES 128
typedef struct op_comm op_comm;
/* RCCL's unique id (ncclGetUniqueId), made by rank 0 and passed to every rank by the host. */
int op_comm_unique_id(uint8_t* id);
/* Communicator of `world` ranks on ctx's device (ncclCommInitRankConfig, non-blocking); gives up with
 * OP_ERR_TIMEOUT after timeout_s. */
int op_comm_create(op_ctx* ctx, int32_t world, int32_t rank, const uint8_t* id, double timeout_s, op_comm** out);
int op_comm_destroy(op_comm* comm);
/* Enqueue: pack the records of staged frames [first, first+n) after ctx's queued work, then
 * ncclGather them to rank 0 on the communicator's own stream (and copy them to pinned host memory
 * there).  Returns at once; at most two gathers outstanding (double-buffered: step k's gather
 * overlaps step k+1's compute).  Every rank passes the same n and max_persons. */
int op_comm_gather_results(op_comm* comm, op_ctx* ctx, int32_t first, int32_t n, int32_t max_persons,
                           int64_t frame_base, int32_t frame_stride);
/* Wait for the oldest outstanding gather, at most timeout_s (then the communicator is aborted and
 * OP_ERR_TIMEOUT returned).  Rank 0: *records = n_frames records of rec_bytes each in rank order
 * (valid until the gather two submits later); other ranks: *records = NULL, *n_frames = 0. */
int op_comm_wait(op_comm* comm, double timeout_s, const void** records, int32_t* n_frames, int64_t* rec_bytes);
/* Every frame reaches rank 0 whole (pose_detector.py:484-517 returns every frame's poses): after
 * op_comm_wait, each rank lists the frames of its own part of that gather whose record does not
 * carry the whole result -- status OP_ERR_CAPACITY (over the batched post-process caps) or more
 * persons than max_persons -- as indices i in [0, n) of its op_comm_gather_results call (global id
 * frame_base + i * frame_stride), with reasons[i] (may be NULL) = 1 over the caps, 2 past
 * max_persons.  When the records were packed, an over-cap frame's post-process input was copied
 * aside on the device (op_comm_overflow_result re-runs it alone, uncapped: the result
 * op_fetch_result would have given) and a frame past max_persons kept its complete result rows
 * (copied out as they are) -- so both are exact even after later steps have run; the host ships
 * them to rank 0 (frames.py: TCP).  Valid until the next op_comm_gather_results, which packs into
 * that gather's slot (after it, both calls return OP_ERR_STATE until the next op_comm_wait).
 * Device keep space per slot: OP_KEEP_FRAMES (env, default 8) frames of each kind, compacted (rows
 * past max_persons go to page-locked memory first, OP_KEEP_ROWS_AVG); a frame beyond that has no
 * copy and op_comm_overflow_result returns OP_ERR_CAPACITY for it. */
int op_comm_overflow(op_comm* comm, op_ctx* ctx, int32_t* frames, int32_t* reasons, int32_t cap, int32_t* count);
int op_comm_overflow_result(op_comm* comm, op_ctx* ctx, int32_t frame, double* poses, double* scores, int32_t cap,
                            op_frame_result* res);

/* ---- Face / hand keypoint detectors: FaceNet / HandNet single-branch CPM nets ----
 * face_detector.py:12-56 (FaceDetector), hand_detector.py:12-66 (HandDetector); the same conv kernels
 * as CocoPoseNet, bf16x3 arithmetic.  One context = one network on one device, one stream. */
#define OP_ARCH_FACENET 1 /* models/FaceNet.py: 71 heat maps (70 keypoints + background) */
#define OP_ARCH_HANDNET 2 /* models/HandNet.py: 22 heat maps (21 keypoints + background) */
typedef struct op_cpm_ctx op_cpm_ctx;
/* Number of conv layers of `arch` (52) and their table in models/FaceNet.py:11-76 order. */
int op_cpm_layer_count(int32_t arch);
int op_cpm_layer_info(int32_t arch, int32_t index, const char** name, int32_t* ci, int32_t* co, int32_t* ksize);
int op_cpm_create(int32_t arch, int32_t device, op_cpm_ctx** out);
int op_cpm_destroy(op_cpm_ctx* ctx);
/* serializers.load_npz(weights_file, self.model) (face_detector.py:16): layers in op_cpm_layer_info order. */
int op_cpm_set_weights(op_cpm_ctx* ctx, const float* const* W, const float* const* b);
/* FaceNet.__call__ / HandNet.__call__ (models/FaceNet.py:78-161): x (n, 3, h, w) f32 NCHW
 * (h, w multiples of 8) -> last-stage maps (n, C, h/8, w/8) f32. */
int op_cpm_forward(op_cpm_ctx* ctx, const float* x, int32_t n, int32_t h, int32_t w, float* maps);
/* compute_peaks_from_heatmaps, CPU branch (face_detector.py:58-84, hand_detector.py:68-94): for each
 * of the first c-1 maps of heatmaps (c, h, w): gaussian_filter(sigma 2.5), global max m; found[i] =
 * m > thresh (f32); keypoints[i] = [coords[1], coords[0], m] of np.where(map == m) flattened
 * ([x, y] for one maximum, [y1, y0] for several, as the reference).  flip != 0 reads the maps
 * mirrored in x (hand_detector.py:47-48: the left-hand maps are flipped before the peaks). */
int op_cpm_peaks(op_cpm_ctx* ctx, const float* heatmaps, int32_t c, int32_t h, int32_t w, float thresh,
                 int32_t flip, double* keypoints, int32_t* found);
/* FaceDetector.__call__ / HandDetector.__call__ on one BGR crop (h x w x 3 u8): cv2 LINEAR resize to
 * 368 x 368, x/256 - 0.5, forward, F.resize_images to (h, w), peaks as op_cpm_peaks (flip_maps: the
 * left-hand map flip; the left-hand input flip is the host copy the reference also makes).
 * keypoints (c-1, 3) f64, found (c-1,). */
int op_cpm_detect(op_cpm_ctx* ctx, const uint8_t* bgr, int32_t h, int32_t w, int64_t row_stride, float thresh,
                  int32_t flip_maps, double* keypoints, int32_t* found);
/* op_cpm_detect over n crops of any sizes in one batched forward (demo.py:38-56's per-person face /
 * hand calls, which the reference makes one at a time): crop i = bgr[i] (h[i] x w[i] x 3 u8, row
 * stride row_stride[i]), flip_maps[i] as above (may be NULL: none).  Results equal n op_cpm_detect
 * calls up to f32 re-association (a lone crop's 7x7 convs split their input chunks over workgroups):
 * keypoints (n, c-1, 3) f64, found (n, c-1). */
int op_cpm_detect_batch(op_cpm_ctx* ctx, int32_t n, const uint8_t* const* bgr, const int32_t* h, const int32_t* w,
                        const int64_t* row_stride, float thresh, const int32_t* flip_maps, double* keypoints,
                        int32_t* found);
/* enable != 0: no split-K on small launches, so a crop's result does not depend on how many crops
 * share its batch (op_cpm_detect_batch == op_cpm_detect bit for bit).  Like op_set_batch_invariant. */
int op_cpm_set_batch_invariant(op_cpm_ctx* ctx, int32_t enable);

/* ---- Training iteration: Updater.update_core of train_coco_pose_estimation.py:93-123 ----
 * One context = CocoPoseNet master weights (f32), Adam state and every activation of a batch of n
 * frames of h x w (multiples of 8) on one device.  Exact f32 (v_mfma_f32_32x32x2_f32 forward and
 * input-gradient convs).  Layers in op_layer_info order. */
typedef struct op_train_ctx op_train_ctx;
int op_train_create(int32_t device, int32_t n, int32_t h, int32_t w, op_train_ctx** out);
int op_train_destroy(op_train_ctx* ctx);
/* initmodel / copy_vgg_params (:183-189): weights + biases; resets the Adam state. */
int op_train_set_weights(op_train_ctx* ctx, const float* const* W, const float* const* b);
/* Current weights / biases and the last step's (unscaled) gradients; any array may be null. */
int op_train_get_weights(op_train_ctx* ctx, float* const* W, float* const* b, float* const* gW, float* const* gb);
/* optimizers.Adam(alpha, beta1, beta2, eps) (:214); the caller's alpha schedule (:104-107) sets alpha. */
int op_train_set_hyper(op_train_ctx* ctx, double alpha, double beta1, double beta2, double eps);
/* enable_update / disable_update of one layer (:225-230, :97-102). */
int op_train_enable_layer(op_train_ctx* ctx, int32_t layer, int32_t enable);
/* GradientScaling hook (train_coco_pose_estimation.py:25-38, registered at :213-217): the step
 * multiplies this layer's W and b gradients by `scale` (f32) before Adam.  Default 1 (no hook). */
int op_train_set_grad_scale(op_train_ctx* ctx, int32_t layer, double scale);
/* One iteration: x = preprocess(imgs) (n, 3, h, w) f32; pafs_t (n, 38, h/8, w/8), heat_t (n, 19, h/8,
 * w/8) f32; ignore (n, h/8, w/8) u8 (1 = ignored); losses[12] = per stage (paf, heat) MSE of
 * compute_loss (:42-77).  Forward, loss, backward, the per-layer gradient scales
 * (op_train_set_grad_scale), Adam on the enabled layers. */
int op_train_step(op_train_ctx* ctx, const float* x, const float* pafs_t, const float* heat_t, const uint8_t* ignore,
                  double* losses);

#ifdef __cplusplus
}
#endif
#endif /* OPENPOSE_HIP_H */
