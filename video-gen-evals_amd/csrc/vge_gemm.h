// The bf16 GEMM of vge_vit.hip (gemm_bf16_kernel): C = A W^T + epilogue on v_mfma_f32_32x32x16_bf16, 256 x 256 tiles.
// Shared by the ViT-H extractor (vge_hmr.cpp) and, as a tuner candidate for 1x1 stride-1 convolutions, by the conv
// launcher (vge_cnn.hip).  A rows: any M (the last row tile's loads clamp to row M - 1, its stores stop at M);
// N % 256 == 0, K % 64 == 0, 16-B aligned rows.
#pragma once
#include <hip/hip_runtime.h>

namespace vge {

enum GemmEpiPublic {
  GEMM_BF16 = 0,           // + bias -> bf16
  GEMM_GELU_BF16 = 1,      // GELU(+ bias) -> bf16
  GEMM_RES_F32 = 2,        // + bias + res (f32) -> f32
  GEMM_PE_F32 = 3,         // + bias + position embedding -> f32
  GEMM_F32 = 4,            // + bias -> f32
  GEMM_RELU_BF16 = 5,      // ReLU(+ bias) -> bf16
  GEMM_RESB_BF16 = 6,      // + bias + resb (bf16) -> bf16
  GEMM_RESB_RELU_BF16 = 7, // ReLU(+ bias + resb) -> bf16
  GEMM_SILU_BF16 = 8       // SiLU(+ bias) -> bf16 (library path only: the YOLOX / RTMPose 1x1 convs)
};

struct GemmBf16 {
  const void* A; long lda;
  const void* W; long ldw;
  void* out; long ldo;
  const float* bias;
  const float* res; long ldr;   // f32 residual (GEMM_RES_F32) or, with resb, the bf16 residual's row stride
  const float* pos; int tokens;
  int M, N, K;
  const void* resb;             // bf16 residual [M][ldr] (GEMM_RESB_*)
};

hipError_t launch_gemm_bf16(int epi, const GemmBf16& a, hipStream_t s);
// the persistent form (gemmp_bf16_kernel: one workgroup per CU, one continuous LDS ring across tiles, the epilogue
// from registers under the next tile's first loads) for the residual-free bf16 epilogues; hipErrorInvalidValue where
// it does not apply (gemm_persist_ok)
hipError_t launch_gemm_bf16_persistent(int epi, const GemmBf16& a, hipStream_t s);
bool gemm_persist_ok(int epi, const GemmBf16& a);
// the same product through hipBLASLt (vge_blaslt.cpp) for the epilogues a library epilogue expresses (bias, ReLU, a
// bf16 residual before the ReLU, the f32 residual stream, f32 out); hipErrorNotSupported where it does not apply or
// VGE_GEMM_LIB=0 (callers then run launch_gemm_bf16)
hipError_t launch_gemm_lib(int epi, const GemmBf16& a, hipStream_t s);
bool gemm_lib_ok(int epi);
void gemm_lib_set(int on);

}  // namespace vge
