/*
 * vge_frcnn.h -- C ABI of TokenHMR's single-person gate detector in libvge.so: detectron2's COCO Faster R-CNN
 * X101-32x8d-FPN (ResNeXt-101 32x8d + FPN + RPN + ROIAlignV2 box head) on gfx950.
 *
 * Replaces (reference file:line):
 *   mesh_generator.py:69-73     get_cfg() + merge_from_file("COCO-Detection/faster_rcnn_X_101_32x8d_FPN_3x.yaml"),
 *                               ROI_HEADS.SCORE_THRESH_TEST = 0.25, DefaultPredictor(det2_cfg)
 *   mesh_generator.py:103-117   per frame: det2_predictor(f) -> instances; valid = (pred_classes == 0) & (scores >
 *                               0.5); a frame is used iff exactly one box is valid (its box is then the crop box);
 *                               a video with < 80 % such frames is rejected
 * and the third-party code it calls (detectron2, NOT in /root/reference, no pinned version, weights from the model
 * zoo at run time): DefaultPredictor (ResizeShortestEdge 800 / 1333 through PIL bilinear), GeneralizedRCNN
 * (pixel normalisation, size_divisibility 32), build_resnet_backbone (ResNeXt, FrozenBN, STRIDE_IN_1X1 False), FPN +
 * LastLevelMaxPool, StandardRPNHead + find_top_rpn_proposals, ROIPooler (ROIAlignV2), FastRCNNConvFCHead,
 * FastRCNNOutputLayers.inference, detector_postprocess.  Restated from the published code (oracle/frcnn.py lists every
 * convention); parity vs detectron2's trained weights is UNPINNED.
 *
 * Conventions as in vge.h: device pointers unless stated, asynchronous on the given stream, int status return.
 * Arithmetic: bf16 operands and activations, f32 accumulation / epilogues / box arithmetic, FrozenBN folded into the
 * conv weights at load.  Grouped 3x3 convolutions run as 64-channel block-diagonal slices of the implicit-GEMM conv.
 */
#ifndef VGE_FRCNN_H
#define VGE_FRCNN_H

#include "vge.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  int min_size, max_size;            /* INPUT.MIN_SIZE_TEST 800, MAX_SIZE_TEST 1333 */
  int depth;                         /* RESNETS.DEPTH 101 (blocks 3, 4, 23, 3); 50 and 152 accepted */
  int groups, width_per_group;       /* NUM_GROUPS 32, WIDTH_PER_GROUP 8 (bottleneck 256 .. 2048) */
  int stem_ch, res2_ch, fpn_ch;      /* 64, 256, 256 (fpn_ch must be 256) */
  int rpn_pre_topk, rpn_post_topk;   /* PRE_NMS_TOPK_TEST 1000, POST_NMS_TOPK_TEST 1000 (each <= 1024) */
  float rpn_nms;                     /* RPN.NMS_THRESH 0.7 */
  int fc_dim, num_classes;           /* ROI_BOX_HEAD.FC_DIM 1024, ROI_HEADS.NUM_CLASSES 80 */
  float score_thresh, nms_thresh;    /* 0.25 (mesh_generator.py:71), ROI_HEADS.NMS_THRESH_TEST 0.5 */
  int det_per_img;                   /* TEST.DETECTIONS_PER_IMAGE 100 */
  float gate_thresh;                 /* 0.5 (mesh_generator.py:106) */
} vge_frcnn_config;

typedef struct vge_frcnn vge_frcnn;

/* Weights: float32 host views with detectron2's state_dict keys:
 *   backbone.bottom_up.stem.conv1.{weight, norm.{weight,bias,running_mean,running_var}},
 *   backbone.bottom_up.res<2..5>.<b>.{conv1,conv2,conv3[,shortcut]}.{weight, norm.*} (conv2: [w, w / groups, 3, 3]),
 *   backbone.fpn_lateral<2..5>.{weight,bias}, backbone.fpn_output<2..5>.{weight,bias},
 *   proposal_generator.rpn_head.{conv, objectness_logits, anchor_deltas}.{weight,bias},
 *   roi_heads.box_head.{fc1,fc2}.{weight,bias}, roi_heads.box_predictor.{cls_score,bbox_pred}.{weight,bias}.
 * Missing key -> VGE_ERR_MISSING_WEIGHT, wrong shape -> VGE_ERR_WEIGHT_SHAPE. */
int vge_frcnn_create(const vge_frcnn_config* cfg, const vge_tensor_view* weights, int n_weights, vge_frcnn** out);
/* workspace for chunks of up to chunk_frames frames of H x W pixels (~250 MB per 800 x 800 frame) */
int vge_frcnn_reserve(vge_frcnn* m, int chunk_frames, int H, int W);
int vge_frcnn_destroy(vge_frcnn* m);

/* Geometry for frames of H x W: out[0..1] = resized (newh, neww), out[2..3] = padded (Hp, Wp), out[4 + 2 l],
 * out[5 + 2 l] = (h, w) of FPN level P(2 + l), l = 0..4; out[14] = row stride of the head tap (floats). */
int vge_frcnn_shapes(const vge_frcnn* m, int H, int W, int* out /* [15] */);

/* Optional intermediates for the parity tests (all device pointers, NULL = not wanted), frame-major: */
typedef struct {
  uint8_t* resized;       /* [F][newh][neww][3] RGB: the PIL bilinear resize of each frame */
  void* fpn[5];           /* bf16 [F][h_l][w_l][256]: P2..P6 */
  float* rpn[5];          /* f32 [F][h_l][w_l][16]: objectness logits (3) | anchor deltas (12) | unused */
  float* proposals;       /* f32 [F][rpn_post_topk][5]: x1 y1 x2 y2 (resized-image pixels), objectness logit */
  int32_t* n_proposals;   /* [F] */
  void* box_features;     /* bf16 [F][rpn_post_topk][49][256]: ROIAlign bins (ph, pw) x channels */
  float* head;            /* f32 [F][rpn_post_topk][shapes[14]]: cls logits (K + 1) | class box deltas (4 K) */
  float* pre_dets;        /* f32 [F][det_per_img][6]: fast_rcnn_inference output (resized-image pixels) */
  int32_t* n_pre_dets;    /* [F] */
} vge_frcnn_taps;

/* frames: device uint8 [F][H][W][3] RGB.  Outputs (device):
 *   dets      f32 [F][det_per_img][6] = x1 y1 x2 y2 (frame pixels), score, class -- the predictor's instances in
 *             score order (detector_postprocess applied); n_dets int32 [F]
 *   person    f32 [F][2][5] = box + score of the first two class-0 instances (zeros where absent)
 *   n_person  int32 [F] = number of class-0 instances with score > gate_thresh: the frame passes the gate of
 *             mesh_generator.py:106-108 iff it is 1 (the box is then person[f][0])
 * Any output may be NULL except n_person. */
int vge_frcnn_detect(vge_frcnn* m, const uint8_t* frames, int n_frames, int H, int W, float* dets, int32_t* n_dets,
                     float* person, int32_t* n_person, const vge_frcnn_taps* taps, vge_stream_t stream);

/* Device time over the next max_calls detect calls: stage_ms[0] = backbone + FPN + RPN convolutions (implicit
 * GEMMs), [1] = box head GEMMs (fc1 as a 7 x 7 valid conv, fc2, predictor), [2] = resize, pooling, proposal
 * selection / NMS, ROIAlign, box inference; flops_per_call[0] / [1] = the algorithmic GEMM FLOPs of stages 0 / 1
 * (grouped convolutions counted at their grouped size). */
int vge_frcnn_profile_begin(vge_frcnn* m, int max_calls);
int vge_frcnn_profile_read(vge_frcnn* m, double* stage_ms, int* n_calls, double* flops_per_call);

#ifdef __cplusplus
}
#endif
#endif /* VGE_FRCNN_H */
