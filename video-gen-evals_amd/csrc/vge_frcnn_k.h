// Launch interface of the gate detector's non-GEMM kernels (vge_frcnn_kernels.hip), used by vge_frcnn.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace vge {

constexpr int FR_MAXK = 1024;   // proposal slots per (frame, level) and per frame; detections per frame <= 1024
constexpr int FR_SEL = 8;       // floats per selected-proposal entry: x1 y1 x2 y2 logit valid . .
constexpr int FR_MAXCAND = 4096;  // box-head candidates per frame (<= 4 classes above 0.25 per proposal)

struct RpnLevel {       // one FPN level of the RPN head output: f32 [n][h][w][16] = logits (3) | deltas (12) | -
  const float* out;
  int h, w, stride, k;  // k = min(pre_nms_topk, h * w * 3); anchors of size 8 x stride, ratios (0.5, 1, 2)
};
struct RpnLevels {
  RpnLevel l[5];
};
struct RoiLevels {      // P2..P5 of a chunk: bf16 [n][h][w][256]
  const void* p[4];
  int h[4], w[4];
};
struct DetPostArgs {
  const float* head;    // f32 [n * P][ld]: logits (K + 1) | deltas (4 K)
  int ld, P, K, det_per_img;
  const float* props;   // f32 [n][P][5]
  const int* n_prop;    // [n]
  float img_h, img_w;   // resized image size (clip)
  float sx, sy;         // detector_postprocess scales (frame / resized), float32
  float out_h, out_w;   // frame size
  float score_thresh, nms_thresh, gate_thresh;
  float* scratch;       // [n][FR_MAXCAND][8] candidates + [n][FR_MAXK][16] u64 masks (det_post_scratch_bytes)
  float* pre_dets;      // optional f32 [n][det_per_img][6] (resized pixels); n_pre [n]
  int* n_pre;
  float* dets;          // optional f32 [n][det_per_img][6] (frame pixels); n_dets [n]
  int* n_dets;
  float* person;        // optional f32 [n][2][5]
  int* n_person;        // [n]
};

size_t det_post_scratch_bytes(int n_frames);

hipError_t launch_frcnn_resize_h(const uint8_t* src, int n, int H, int W, int nw, const int* xb, const int* kk, int ks,
                                 uint8_t* dst, hipStream_t s);
hipError_t launch_frcnn_resize_v_norm(const uint8_t* tmp, int n, int H, int nw, int nh, int hp, int wp, const int* yb,
                                      const int* kk, int ks, uint8_t* resized, void* out, hipStream_t s);
hipError_t launch_frcnn_pool_s2(const void* x, void* y, int n, int H, int W, int C, int K, hipStream_t s);
// the stem conv (7x7 / 2, 8-channel NHWC input, 64 outputs, weights [64][Kp] tap-major) + ReLU + max_pool2d(3, 2, 1)
hipError_t launch_frcnn_stem_pool(const void* in, const void* w, int Kp, const float* bias, void* out, int n, int hp,
                                  int wp, hipStream_t s);
hipError_t launch_rpn_select(const RpnLevels& lv, int n, float img_h, float img_w, float* sel, float* sel_max,
                             hipStream_t s);
hipError_t launch_rpn_nms(const RpnLevels& lv, const float* sel, const float* sel_max, int n, float thr, float* kept,
                          int* kcount, hipStream_t s);
hipError_t launch_rpn_merge(const float* kept, const int* kcount, int n, int post_k, float* props, int* n_prop,
                            hipStream_t s);
hipError_t launch_roi_align(const RoiLevels& lv, const float* props, const int* n_prop, int n, int P, void* out,
                            hipStream_t s);
hipError_t launch_det_post(const DetPostArgs& a, int n, hipStream_t s);
// vge_gconv.hip: the bottlenecks' grouped 3x3 conv (+ folded FrozenBN bias, ReLU), HBM-bound direct kernel
hipError_t launch_gconv3(const void* x, long ldx, const void* w, int Kp, const float* bias, void* out, long ldo,
                         int n_img, int H, int W, int C, int gw, int stride, hipStream_t s);

}  // namespace vge
