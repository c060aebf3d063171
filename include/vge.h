/*
 * vge.h -- C ABI of libvge.so, the MI355X (gfx950) implementation of the Action-Consistency /
 * Temporal-Coherence scoring path of XThomasBU/video-gen-evals.
 *
 * The reference has no FFI layer: its boundary is the set of Python functions eval.py composes.
 * Each entry point below replaces one of them (reference file:line cited per function).
 *
 * Conventions
 *   - Plain pointers and sizes; no torch types.  Pointers marked "device" are HBM buffers owned by
 *     the caller (hipMalloc / torch), "host" pointers are ordinary host memory.
 *   - Every compute call is asynchronous on the hipStream_t passed in (nullptr = default stream)
 *     and never synchronises, allocates or frees inside (graph-capture safe), except the create /
 *     reserve / destroy calls.
 *   - Return value: 0 (VGE_OK) or a vge_status code; nothing throws across the ABI.
 *     vge_last_error() returns a static description of the most recent failure on this thread.
 *   - Feature-column order is the reference's feats layout (utils.py:496-514):
 *       raw  = vit[1024] | global_orient[9] | pose[207] | betas[10] | kp2d[120]      (1370)
 *       diff = vit[1024] | global_orient[3] | pose[69]  | betas[10] | kp2d[120]      (1226)
 *     or, when the reference runs without keypoints (keypoint_dir None: no kp2d columns, 4 modalities),
 *       raw  = vit[1024] | global_orient[9] | pose[207] | betas[10]                   (1250)
 *       diff = vit[1024] | global_orient[3] | pose[69]  | betas[10]                   (1106)
 */
#ifndef VGE_H
#define VGE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* vge_stream_t; /* == hipStream_t */

typedef enum {
  VGE_OK = 0,
  VGE_ERR_ARG = 1,            /* bad argument / unsupported shape */
  VGE_ERR_HIP = 2,            /* a HIP runtime call failed */
  VGE_ERR_MISSING_WEIGHT = 3, /* a required state_dict key is absent (the reference's
                                 load_state_dict(strict=False) would silently random-init it) */
  VGE_ERR_WEIGHT_SHAPE = 4,   /* a state_dict tensor has the wrong shape */
  VGE_ERR_NOMEM = 5,
  VGE_ERR_WORKSPACE = 6,      /* vge_encoder_reserve() was not called for this many windows */
  VGE_ERR_UNSUPPORTED = 7,    /* a model shape the kernels are not built for (vge_encoder_create): clip_len != 32,
                                 a modality set / input dims other than the reference's five or its keypoint-less
                                 four (clip / dino modalities, other vit or pose widths), or d_model / time_heads
                                 other than 256 / 8 outside the exact-f32 generic path (VGE_F32 only: d_model a
                                 multiple of 32 in [32, 256], head dim <= 64).  load_model (eval.py:136-165) reads
                                 these from the checkpoint; time_layers is free (any >= 1). */
  VGE_ERR_DEVICE = 8          /* a kernel detected a broken invariant and raised the encoder's status word (the
                                 staggered conv kernel's half-workgroup exchange wait ran out of its bound): the
                                 outputs of that launch are wrong.  Reported by vge_encoder_status, by
                                 vge_encoder_profile_read and by every later vge_encode until cleared. */
} vge_status;

/* Encoder compute modes.  VGE_F32: exact f32 MFMA (v_mfma_f32_16x16x4_f32, bitwise an fmaf chain).
 * VGE_F32X3: f32-class split precision -- every GEMM operand carried as fp16 hi + fp16 lo*2^11 and
 * each product formed as hi*hi + 2^-11 (hi*lo + lo*hi) on v_mfma_f32_32x32x16_f16 with f32
 * accumulation (relative error ~2^-21 per product; AC/TC within ~1e-7 of the f32 mode).  Its conv encoders
 * run staggered (vge_encoder_x3s.hip): each block's GroupNorm is folded into the next GEMM's weights and
 * epilogue, and GELU is a one-exp2 form within ~1 f32 ulp at |x| <= 6 (f32 rounding-level, as the reference's
 * own erf-based GELU); env VGE_X3S=0 keeps the unstaggered kernel and unfolded weights. */
typedef enum { VGE_F32 = 0, VGE_F32X3 = 1, VGE_F16 = 2 } vge_dtype;
/* VGE_F16: the throughput mode (BASELINE configs 2 / 5 "bf16" / "fp16 MFMA path"): the ten
 * MovementConvEncoders (85% of the FLOPs) take every GEMM operand as a single fp16 (the hi planes of the
 * VGE_F32X3 image, same power-of-two scaling), one v_mfma_f32_32x32x16_f16 per product, f32 accumulation
 * and f32 epilogues (GELU, GroupNorm); the transformer keeps the 3xfp16 split, because it carries most of
 * the fp16 error for ~10% of the FLOPs (env VGE_F16_MIX: bit 1 = transformer split [default 2], bit 0 =
 * stem split).  Measured AC/TC within 3e-5 of the reference on the golden set (tests/test_gpu_parity.py),
 * asserted at 1e-4 on the bench and config-5 workloads (tests/test_bench_parity.py); bench.py reports it. */

#define VGE_FEAT_DIM 2596
#define VGE_RAW_DIM 1370
#define VGE_FEAT_DIM_NOKP 2356 /* keypoint-less layout (keypoint_dir None) */
#define VGE_RAW_DIM_NOKP 1250

/* Feature layouts: which columns WindowDataset._try_one concatenates (utils.py:496-514).  The reference picks it by
 * whether keypoint_dir is set; infer_dims_from_stats (eval.py:104-133) then gives the model 5 or 4 modalities. */
typedef enum { VGE_LAYOUT_KP = 0, VGE_LAYOUT_NOKP = 1 } vge_layout;
int vge_layout_feat_dim(vge_layout layout); /* 2596 / 2356, 0 for an unknown layout */
#define VGE_CLIP_LEN 32
#define VGE_D_MODEL 256

/* Model shape (infer_dims_from_stats, eval.py:104-133; HumanActionScorer, model.py:102-148).
 * The kernels are built for the reference configuration: 5 modalities in the order
 * vit, global, pose, beta, kp2d with dims {1024,9,207,10,120} / {1024,3,69,10,120}, or the first 4 of them
 * (keypoint-less layout: 8 conv encoders, a 4-way fusion, feats rows of 2356), d_model 256, post-norm
 * layers, 8 heads, FFN 1024, clip_len 32.  Other checkpoint shapes (d_model 32..256 in steps of 32, any head count
 * with a head dim <= 64, FFN 4 d_model) run on the generic exact-f32 kernels (vge_encoder_gen.hip) when created
 * with VGE_F32; seq / frame embeddings are then d_model wide. */
typedef struct {
  int n_modalities;
  int dims_raw[8];
  int dims_diff[8];
  int d_model;
  int time_layers;
  int time_heads;
  int clip_len;
} vge_dims;

/* A named host tensor, named exactly as the reference state_dict key (model.py parameter names),
 * e.g. "state_enc.vit.blocks.0.conv1.weight" [256,256,5] or "temporal.layers.3.norm2.bias" [256]. */
typedef struct {
  const char* name;
  const float* data; /* host, contiguous float32 */
  int ndim;
  int64_t shape[4];
} vge_tensor_view;

typedef struct vge_encoder vge_encoder;

/* ---- frame store: the per-frame features of a set of videos, resident in HBM ----------------
 * Replaces the npz/keypoints.npy reads of WindowDataset._try_one (utils.py:383-425).
 * videos[v] = {frame_off, n_frames, kp_off, kp_frames} (int32, device); kp_frames = 0 means the
 * video has no keypoint file. */
typedef struct {
  const float* pose;   /* device [F,207] (23 rotmats) */
  const float* gori;   /* device [F,9]                */
  const float* betas;  /* device [F,10]               */
  const float* vit;    /* device [F,1024]             */
  const float* kp;     /* device [Fk,120]             */
  const int32_t* videos; /* device [V,4]              */
  int n_videos;
} vge_frame_store;

/* ---------------------------------------------------------------------------------------------
 * Featurisation.  Replaces WindowDataset._try_one (utils.py:383-516) incl. _slice_or_pad
 * (366-381), _vit_delta (142-147), _rotmat_delta/_log_so3 (130-140,165-174), _betas_delta
 * (161-163), _procrustes_kp_delta with LAPACK-convention 2x2 SVD (177-217) and the z-norm
 * (x-mean)/(std+1e-6) (472-494).
 *   windows : device int32 [n_windows,2] = {video index, start frame}
 *   mean,std: device float [2596] (ModalityStats in feats column order)
 *   feats   : device float [n_windows,32,2596]
 * vge_featurize_layout: the same for either layout; VGE_LAYOUT_NOKP (keypoint_dir None) reads no keypoints and
 *   takes mean/std [2356] and feats [n_windows,32,2356] in that layout's column order.
 */
int vge_featurize(const vge_frame_store* store, const int32_t* windows, int n_windows,
                  const float* mean, const float* std, float* feats, vge_stream_t stream);
int vge_featurize_layout(const vge_frame_store* store, const int32_t* windows, int n_windows, const float* mean,
                         const float* std, vge_layout layout, float* feats, vge_stream_t stream);

/* ---------------------------------------------------------------------------------------------
 * ModalityStats.  Replaces compute_stats_from_npz (utils.py:595-801) with _update_sum_sum2
 * (589-593): float64 per-column sum / sum of squares over all frames of the selected videos,
 * diffs on the full sequences; keypoint columns over keypoint frames only.
 *   host_videos    : host copy of store->videos [V,4] (tile planning happens on the host)
 *   host_video_sel : host int32 [n_sel] video indices into the store
 *   sums      : device double [2,2596] (sum, sum of squares) -- ACCUMULATED INTO (zero it first)
 *   counts    : host int64 [2] += {mesh frames, keypoint frames} of the selection
 *   workspace : device scratch of >= vge_stats_workspace_bytes(1) bytes; videos are processed in
 *               chunks of as many 32-frame tiles as fit (this call may synchronise the stream)
 * vge_stats_finalize turns (sums, counts) into float32 mean/std (std = sqrt(max(var,0)+1e-6),
 * utils.py:746-750).  Sums are the RCCL exchange payload when the real set is sharded.
 * vge_stats_finalize_layout writes mean/std in a layout's column order (VGE_LAYOUT_NOKP: [2356], the kp2d
 * columns dropped -- the reference's keypoint-less ModalityStats); the sums are always [2,2596].
 */
size_t vge_stats_workspace_bytes(int chunk_tiles);
int vge_stats_accumulate(const vge_frame_store* store, const int32_t* host_videos, const int32_t* host_video_sel,
                         int n_sel, double* sums, int64_t* counts, void* workspace, size_t workspace_bytes,
                         vge_stream_t stream);
int vge_stats_finalize(const double* sums, const int64_t* counts, float* mean, float* std, vge_stream_t stream);
int vge_stats_finalize_layout(const double* sums, const int64_t* counts, vge_layout layout, float* mean, float* std,
                              vge_stream_t stream);

/* ---------------------------------------------------------------------------------------------
 * Encoder.  Replaces load_model (eval.py:136-165) + HumanActionScorer.forward (model.py:162-193).
 * create: validates every required key (missing -> VGE_ERR_MISSING_WEIGHT) and repacks the
 * weights into the library's MFMA panel layout in HBM (the handle owns them).
 * reserve: allocates the activation workspace for up to max_windows windows (outside timed
 * regions; compute calls never allocate).
 * encode: feats device [B,T,D] -> seq_embed device [B,256] (L2-normalised CLS), D = vge_encoder_feat_dim
 *   (2596, or 2356 for a 4-modality keypoint-less model),
 *   frame_embed device [B,T+1,256] or NULL, tc_window device [B] (per-window temporal coherence,
 *   eval.py:216-224) or NULL.
 */
int vge_encoder_create(const vge_dims* dims, const vge_tensor_view* weights, int n_weights, vge_dtype compute,
                       vge_encoder** out);
int vge_encoder_reserve(vge_encoder* enc, int max_windows);
int vge_encoder_destroy(vge_encoder* enc);
int vge_encoder_feat_dim(const vge_encoder* enc); /* feats row width the encoder reads: 2596 or 2356 (0: null) */
int vge_encode(vge_encoder* enc, const float* feats, int B, int T, float* seq_embed, float* frame_embed,
               float* tc_window, vge_stream_t stream);
/* Pipelining hook (no reference counterpart; the reference featurises batch k+1 in DataLoader workers while batch k
 * is encoded, eval.py:410-418): make `stream` wait until the conv stage of the most recent vge_encode on this
 * encoder -- the last reader of its feats -- has finished, so the next batch's vge_featurize can overwrite feats on
 * `stream` while this batch's fusion / transformer still run. */
int vge_encoder_wait_conv(vge_encoder* enc, vge_stream_t stream);
/* Pipelining hook (no reference counterpart): subsequent vge_encode calls run the stages after the fusion (token
 * GEMM, transformer, output normalisation / TC) on `tail` instead of their own stream (NULL: back to it).  The encode
 * stream keeps the conv stage and the fusion, so the caller can featurise and encode the next batch there while this
 * batch's transformer runs; seq_embed / frame_embed / tc_window are complete in `tail`'s order (read them there).
 * The next vge_encode's fusion waits for the previous encode's tail stages, which read the buffer it overwrites. */
int vge_encoder_set_tail_stream(vge_encoder* enc, vge_stream_t tail);

/* Per-stage device time of vge_encode, measured with hipEvents recorded on the encode stream around
 * each stage (used by bench.py for the roofline line).  profile_begin pre-creates events for up to
 * max_calls subsequent vge_encode calls (no allocation inside encode); profile_read synchronises on
 * the recorded events and returns the summed milliseconds per stage and the number of calls seen.
 * Stages: 0 conv encoders (MovementConvEncoder x10), 1 fusion pool, 2 token GEMM (+CLS/PE),
 *         3 transformer layers, 4 output normalisation + per-window TC. */
#define VGE_N_STAGES 5
int vge_encoder_profile_begin(vge_encoder* enc, int max_calls);
int vge_encoder_profile_read(vge_encoder* enc, double* stage_ms, int* n_calls);

/* The encoder's device status word: VGE_OK, or VGE_ERR_DEVICE once a completed launch raised it (the word is
 * host-mapped: no synchronisation here -- synchronise the encode stream first to cover launches in flight).
 * vge_encoder_clear_status resets it (tests).  No reference counterpart: the reference's torch ops cannot fail this
 * way; this is the kernel-side guard that keeps a broken invariant from being a silent wrong score. */
int vge_encoder_status(const vge_encoder* enc);
int vge_encoder_clear_status(vge_encoder* enc);
/* Which of the VGE_N_STAGES + 1 stage-boundary events profiled vge_encode calls record (bit k = event before stage k;
 * default all): each event is a queue marker, so a timed loop that only needs the conv stage records 0x3 and
 * profile_read reports the stages both of whose events were recorded (the others as 0).  Mask 0: later calls are not
 * profiled and take no slot (a caller can sample every k-th call inside a timed loop). */
int vge_encoder_profile_mask(vge_encoder* enc, int event_mask);

/* ---------------------------------------------------------------------------------------------
 * Metrics.
 * vge_tc_windows: compute_temporal_coherence_scores' per-window term (eval.py:216-224):
 *   tc[w] = mean_t ||f[w,t+1]-f[w,t]||_2 over rows 1..T of frame_embed [B,T+1,d] (CLS dropped).
 * vge_score_videos: per-video AC (eval.py:229-257) and TC (np.mean over windows, eval.py:226):
 *   windows of video v are [video_first_win[v], video_first_win[v+1]) (device int32 [V+1]);
 *   video_class[v] = centroid row or -1 (class not in label_dict -> ac[v] = NaN, no "ac" key).
 *   ac: device float [V]; tc: device double [V].
 */
int vge_tc_windows(const float* frame_embed, int B, int T1, int d, float* tc, vge_stream_t stream);
int vge_score_videos(const float* seq_embed, const float* tc_window, const int32_t* video_first_win,
                     const int32_t* video_class, const float* centroids, int V, int d, float* ac, double* tc,
                     vge_stream_t stream);

/* ---------------------------------------------------------------------------------------------
 * Real-class centroids.  Replaces build_train_centroids_subset (utils.py:1018-1045):
 * sums.index_add_(0, y, z); counts.index_add_ -- a deterministic segmented reduction (segments of 512
 * windows, CENT_SEG in vge_score.hip, summed in window order, then the segment partials in segment order: the same bits for any
 * device or launch, within a few ulps of a sequential index_add_); d <= 256; class ids outside [0, C)
 * are ignored.  finalize = normalize(sums / counts.clamp_min(1)).
 * sums [C,d] / counts [C] (device float) are ACCUMULATED INTO and are the RCCL all-gather payload.
 */
int vge_centroid_accumulate(const float* seq_embed, const int32_t* class_id, int n_windows, int C, int d,
                            float* sums, float* counts, vge_stream_t stream);
int vge_centroid_finalize(const float* sums, const float* counts, int C, int d, float* centroids,
                          vge_stream_t stream);

const char* vge_last_error(void);
const char* vge_version(void);

#ifdef __cplusplus
}
#endif
#endif /* VGE_H */
