// Host-side launch interface of the CNN kernels (vge_cnn.hip, vge_pose_head.hip) shared by vge_dwpose.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace vge {

struct ConvLaunch {
  const void* x; long ldx;                  // NHWC bf16 input (channel offset folded into the pointer)
  const void* w; const float* bias;         // packed [Npad][Kp] bf16, bias [Npad]
  void* out; long ldo;                      // NHWC output
  const void* res; long ldr; const float* rscale;
  const void* zero;                         // >= 16 B of zeros in device memory
  int n_img, H, W, Cin, KH, KW, stride, pad, Kp, Cout, Npad;
  int act, out_f32, res_mode, tn;           // act 0 none / 1 SiLU / 2 sigmoid / 3 ReLU; res 0 / 1 bf16 (after
                                            // act) / 2 f32 scaled / 3 bf16 before act
  int gslice;                               // grouped conv slices (vge_cnn.hip ConvArgs::gslice): Cin == tn
  int variant;                              // 0 default; 1 128-row kernel (tn <= 128); 2 256 x 256 tiles, one per
                                            // workgroup; 3 256 x 256 tiles on the persistent grid (res_mode 0 only);
                                            // 5 256-row tiles with tn (64 / 128) columns; 6 512 x 128 tiles on
                                            // the persistent grid
};

struct WarpInst {  // warp_prep_kernel: source frame and affine map of one pose instance
  int frame;
  float cx, cy, k;
};
struct PoseInst {  // kp120_kernel: box center and aspect-fixed scale
  float cx, cy, sw, sh;
};

hipError_t launch_conv_bf16(const ConvLaunch& c, hipStream_t s);
// the GEMM epilogue (vge_gemm.h) that runs c as variant 9 (a 1x1 stride-1 conv on gemm_bf16_kernel), -1 = none
int conv_gemm_epi(const ConvLaunch& c);
int conv_lib_epi(const ConvLaunch& c);
bool conv_gemm_persist_ok(const ConvLaunch& c);  // variant 10 applies (the persistent GEMM, vge_vit.hip gemmp)
hipError_t launch_dwconv(const void* x, long ldx, const float* w, const float* b, void* y, long ldy, int n_img, int H,
                         int W, int C, int K, hipStream_t s);
hipError_t launch_spp_pool(void* buf, long ld, int n_img, int H, int W, int C, int k0, int k1, int k2, hipStream_t s);
hipError_t launch_chan_attn(void* x, long ld, int n_img, int HW, int C, const float* Wt, const float* b, float* mean,
                            float* att, hipStream_t s);
hipError_t launch_warp_prep(const uint8_t* frames, int H, int W, const void* inst, int n_inst, int oh, int ow, void* out,
                            hipStream_t s);
hipError_t launch_letterbox_focus(const uint8_t* frames, int n, int H, int W, int S, int rh, int rw, float inv_rx,
                                  float inv_ry, void* out, hipStream_t s);
hipError_t launch_upsample2x(const void* x, long ldx, void* y, long ldy, int n_img, int H, int W, int C, hipStream_t s);
struct DetLevel {      // one YOLOX head level: f32 [n][g*g][8] = reg xywh, obj logit, cls-0 logit
  const float* out;
  int grid, stride;
};
hipError_t launch_yolox_decode_nms(DetLevel l0, DetLevel l1, DetLevel l2, int F, float ratio, float* boxes, int* n_out,
                                   float* scores, float* cand, hipStream_t s);
hipError_t launch_head_sn_t(const float* y, long ldy, int hw, int K, int Kp, float g, long n_rows, void* out,
                            hipStream_t s);
hipError_t launch_scalenorm_rows(const float* x, int D, float g, long rows, void* y, hipStream_t s);
size_t gau_lds_bytes(int S);
hipError_t launch_gau_attn(const float* uv, int n_inst, int K, int E, int S, const float* gamma, const float* beta,
                           void* out, hipStream_t s);
hipError_t launch_simcc_decode(const float* logits, long ld, int WX, int WY, float split, long rows, float* lv,
                               hipStream_t s);
hipError_t launch_kp120(const float* lv, const void* inst, const int* inst_of_frame, int F, int K, int in_w, int in_h,
                        int H, int W, float* out, hipStream_t s);

}  // namespace vge
