/*
 * vge_dwpose.h -- C ABI of the per-frame 2-D keypoint extractor in libvge.so: DWPose (RTMPose-l whole-body
 * pose model; YOLOX-L person boxes) on gfx950, writing the keypoints.npy rows the scoring path reads.
 *
 * Replaces (reference file:line):
 *   process_video.py:59-91          per-frame `pose(frame)` + flatten_first_person_no_padding (23-57) ->
 *                                   keypoints.npy [T', 120] float32
 *   dwpose_init.py:37-69            DWposeDetector.__call__: Wholebody() -> candidate / (W, H), subset < 0.3 ->
 *                                   -1, body = candidate[:, :18], hands = vstack(candidate[:, 92:113],
 *                                   candidate[:, 113:])  (the h[1] = person 1's LEFT hand quirk with >= 2 persons)
 * and the third-party pieces it calls (ControlNet annotator/dwpose, NOT in /root/reference, no pinned version,
 * models downloaded at run time): wholebody.py (neck insertion + mmpose -> OpenPose reorder), onnxpose.py
 * (bbox_xyxy2cs padding 1.25, aspect fix, affine warp 288x384, BGR mean / std, SimCC argmax decode),
 * dw-ll_ucoco_384.onnx = RTMPose-l (mmpose CSPNeXt-P5 + RTMCCHead).  Their structure is restated from the
 * published models; parity vs the upstream ONNX weights is UNPINNED.  Kernels are checked
 * against a torch-fp32 restatement (oracle/dwpose.py).
 *
 * Only persons 0 and 1 of a frame (detector order) can reach the 120-d row, so only they are posed.
 * Conventions as in vge.h: device pointers unless stated, asynchronous on the given stream, int status.
 * Arithmetic: bf16 operands, f32 accumulation, BatchNorm folded into the conv weights at load time.
 */
#ifndef VGE_DWPOSE_H
#define VGE_DWPOSE_H

#include "vge.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  int in_h, in_w;          /* model input 384 x 288 */
  int stem_ch;             /* CSPNeXt stem output channels (64) */
  int stage_ch[4];         /* 128, 256, 512, 1024 */
  int stage_blocks[4];     /* 3, 6, 6, 3 CSPNeXtBlocks */
  int keypoints;           /* 133 (COCO-WholeBody) */
  int gau_hidden, gau_s, gau_e;  /* 256, 128, 512 */
  int final_k;             /* 7 */
  int split;               /* SimCC split ratio 2 */
} vge_rtmpose_config;

typedef struct vge_dwpose vge_dwpose;

/* Weights: float32 host views with the mmpose RTMPose state_dict keys, e.g.
 *   backbone.stem.<0..2>.{conv.weight, bn.{weight,bias,running_mean,running_var}},
 *   backbone.stage<i>.0.* (3x3/s2 ConvModule), backbone.stage4.1.{conv1,conv2}.* (SPPBottleneck),
 *   backbone.stage<i>.<j>.{main_conv,short_conv,final_conv}.*, .blocks.<b>.{conv1, conv2.depthwise_conv,
 *   conv2.pointwise_conv}.*, .attention.fc.{weight,bias},
 *   head.final_layer.{weight,bias}, head.mlp.0.g, head.mlp.1.weight, head.gau.{uv.weight, gamma, beta,
 *   o.weight, ln.g, res_scale.scale}, head.cls_x.weight, head.cls_y.weight.
 * Missing key -> VGE_ERR_MISSING_WEIGHT, wrong shape -> VGE_ERR_WEIGHT_SHAPE. */
int vge_dwpose_create(const vge_rtmpose_config* cfg, const vge_tensor_view* weights, int n_weights, vge_dwpose** out);
/* workspace for up to max_instances pose instances per call (a frame is 1 or 2 instances) */
int vge_dwpose_reserve(vge_dwpose* m, int max_instances);
int vge_dwpose_destroy(vge_dwpose* m);

/* frames: device uint8 [F][H][W][3] RGB.  boxes: HOST float [F][max_persons][4] xyxy pixels in detector order
 * (may be NULL when every n_persons is 0); n_persons: HOST int [F] (0 -> the whole frame is the box, as
 * onnxpose.preprocess does).  keypoints: device float [F][120] = flatten_first_person_no_padding of every frame
 * (with a person box every frame yields a row, so T' = F).  simcc (optional, device f32 [n_inst][K][split *
 * (in_w + in_h)]) and lv (optional, device f32 [n_inst][K][3] = x, y in model-input pixels, score) expose the
 * head outputs for the parity tests; instances are numbered frame-major (person 0, then person 1). */
int vge_dwpose_keypoints(vge_dwpose* m, const uint8_t* frames, int n_frames, int H, int W, const float* boxes,
                         int max_persons, const int* n_persons, float* keypoints, float* simcc, float* lv,
                         vge_stream_t stream);

/* Device time of the dense convolutions (implicit GEMMs) and of everything else over the next max_calls
 * keypoint calls: stage_ms[0] = conv / Linear GEMMs, [1] = depthwise + pooling + attention + prep, [2] = GAU token
 * mixing + decode; gemm_flops_per_call = algorithmic GEMM FLOPs of the recorded calls / n_calls (the last call's
 * when none was recorded). */
int vge_dwpose_profile_begin(vge_dwpose* m, int max_calls);
int vge_dwpose_profile_read(vge_dwpose* m, double* stage_ms, int* n_calls, double* gemm_flops_per_call);

/* ---- YOLOX person detector (onnxdet.inference_detector: yolox_l.onnx, 640x640 letterbox) ---------------------
 * The published YOLOX-L (CSPDarknet + YOLOPAFPN + YOLOXHead, BaseConv = conv + BN(eps 1e-3) + SiLU) restated; only
 * class 0 (person) is computed, because multiclass_nms is class-aware and inference_detector keeps class 0 with
 * score > 0.3 only.  Output = what reaches DWPose: the first two persons of the greedy NMS in score order and
 * min(person count, 2) (0 -> the pose model falls back to the whole frame). */
typedef struct {
  int in_size;       /* 640 */
  int width;         /* base channels: 64 (YOLOX-L, wid_mul 1.0) */
  int depth;         /* base depth: 3 (dep_mul 1.0; CSP blocks 3, 9, 9, 3) */
  int head_ch;       /* 256 */
  int num_classes;   /* 80 (the cls_preds weight shape; only row 0 is used) */
} vge_yolox_config;

typedef struct vge_yolox vge_yolox;

/* Weights: float32 host views with the YOLOX state_dict keys: backbone.backbone.{stem.conv, dark2..dark5}.*,
 * backbone.{lateral_conv0, C3_p4, reduce_conv1, C3_p3, bu_conv2, C3_n3, bu_conv1, C3_n4}.*, head.{stems,
 * cls_convs, reg_convs}.<k>.*, head.{cls_preds, reg_preds, obj_preds}.<k>.{weight,bias}; BaseConv = .conv.weight
 * + .bn.{weight,bias,running_mean,running_var}. */
int vge_yolox_create(const vge_yolox_config* cfg, const vge_tensor_view* weights, int n_weights, vge_yolox** out);
/* frames processed per internal chunk (workspace ~90 MB per frame at 640) */
int vge_yolox_reserve(vge_yolox* m, int chunk_frames);
int vge_yolox_destroy(vge_yolox* m);
/* frames: device uint8 [F][H][W][3] RGB.  boxes: device float [F][2][4] xyxy frame pixels of persons 0 and 1
 * (zeros where absent); n_persons: device int [F] = min(count, 2).  cand (optional): device float [F][A][5] =
 * every anchor's decoded box and score (A = 3 * 16^2 * (in_size / 128)^2 ... = 8400 at 640), for tests. */
int vge_yolox_detect(vge_yolox* m, const uint8_t* frames, int n_frames, int H, int W, float* boxes, int* n_persons,
                     float* cand, vge_stream_t stream);
/* The same, plus scores: device float [F][2] = the scores of persons 0 and 1 (0 where absent).  The TokenHMR
 * front end's single-person gate (mesh_generator.py:103-111: exactly one person box with score > 0.5 after NMS)
 * reads them: since persons 0 / 1 are the first two boxes the greedy NMS keeps, "exactly one box > 0.5" is
 * scores[f][0] > 0.5 && scores[f][1] <= 0.5.  (The reference's detector there is detectron2's Faster R-CNN
 * X101-FPN, absent offline; this YOLOX-L is its stand-in: parity unpinned.) */
int vge_yolox_detect_scored(vge_yolox* m, const uint8_t* frames, int n_frames, int H, int W, float* boxes,
                            int* n_persons, float* scores, float* cand, vge_stream_t stream);
/* stage_ms[0] = convolutions (implicit GEMMs), [1] = letterbox / upsample / pooling / decode + NMS, summed over the
 * recorded calls; gemm_flops_per_call = their algorithmic GEMM FLOPs / n_calls (a pass's tail call is smaller). */
int vge_yolox_profile_begin(vge_yolox* m, int max_calls);
int vge_yolox_profile_read(vge_yolox* m, double* stage_ms, int* n_calls, double* gemm_flops_per_call);

/* Op-level entry point (parity tests; the kernel every dense layer uses): NHWC bf16 convolution as an implicit
 * GEMM.  x [n_img][H][W][ldx] bf16 (channels 0..Cin-1 used, Cin a power of two >= 8), w [Npad][Kp] bf16 packed
 * k = (kh * KW + kw) * Cin + ci (Kp = KH*KW*Cin rounded up to 32, Npad = Cout rounded up to 256, zero padded),
 * bias [Npad] f32, out [n_img][Ho][Wo][ldo].  act: 0 none, 1 SiLU, 2 sigmoid; out_f32: 0 bf16 (Cout % 8 == 0),
 * 1 f32; res_mode: 0 none, 1 bf16 residual [M][ldr] added after the activation, 2 f32 residual x rscale[col]. */
int vge_op_conv_bf16(const void* x, long ldx, const void* w, const float* bias, void* out, long ldo, const void* res,
                     long ldr, const float* rscale, int n_img, int H, int W, int Cin, int KH, int KW, int stride,
                     int pad, int Cout, int act, int out_f32, int res_mode, vge_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* VGE_DWPOSE_H */
