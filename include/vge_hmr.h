/*
 * vge_hmr.h -- C ABI of the per-frame mesh extractor in libvge.so: TokenHMR (HMR2 ViT-H/16 backbone +
 * SMPL token-decoder head) on gfx950, writing the frame-store arrays the scoring path reads.
 *
 * Replaces (reference file:line):
 *   MeshGenerator.process_video       modifications/mesh_generator.py:119-171 (batched model(batch) over
 *                                     the single-person frames, bs 8, keeps body_pose / betas /
 *                                     global_orient / token_out)
 *   SMPLTokenDecoderHead.forward      modifications/token_head.py:180-246 (zero token -> 6-layer cross-
 *                                     attention decoder -> readouts -> rot6d_to_rotmat)
 *   extract_mesh.py:35-43             the npz arrays pose[T,23,3,3] / global_orient[T,1,3,3] / betas[T,10] /
 *                                     vit[T,1024] (here: rows of the HBM frame store, no npz round trip)
 * The person crop (ViTDetDataset) is vge_hmr_crop below; the person detector of mesh_generator.py:103-117
 * (detectron2 Faster R-CNN) is stood in for by the YOLOX-L of vge_dwpose.h (vge_yolox_detect_scored).  The ViT backbone, pose_transformer and the
 * TokenHMR tokenizer are third-party code absent from /root/reference (TokenHMR / 4D-Humans at HEAD, no
 * pinned version, no weights offline): their structure is restated from the published models, the
 * token classifier's codebook decoder is a documented stand-in, and parity vs the upstream weights is
 * UNPINNED.  Kernels are checked against a torch-fp32 restatement (oracle/hmr.py).
 *
 * Conventions as in vge.h: device pointers, asynchronous on the given stream, int status return.
 * Arithmetic: bf16 operands, f32 accumulation, f32 residual streams and LayerNorm statistics.
 */
#ifndef VGE_HMR_H
#define VGE_HMR_H

#include "vge.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  int in_h, in_w;           /* input crop: 256 x 256 (ViTDetDataset output size) */
  int img_h, img_w;         /* backbone input: all rows, columns (in_w - img_w)/2 .. : 256 x 192 */
  int patch, pad;           /* patch-embed Conv2d kernel = stride 16, padding 2 -> 16 x 12 tokens */
  int embed_dim, depth, heads, mlp_dim;                       /* ViT-H: 1280, 32, 16, 5120 */
  int dec_dim, dec_depth, dec_heads, dec_dim_head, dec_mlp;   /* decoder: 1024, 6, 8, 64, 1024 */
  int tok_num, tok_classes, tok_code_dim;                     /* token classifier: 160, 2048, 256 */
} vge_hmr_config;

typedef struct vge_hmr vge_hmr;

/* Weights are named views (float32 host) with the upstream state_dict keys, e.g.
 *   backbone.patch_embed.proj.weight [E,3,16,16], backbone.pos_embed [1,T+1,E],
 *   backbone.blocks.<i>.{norm1,attn.qkv,attn.proj,norm2,mlp.fc1,mlp.fc2}.{weight,bias}, backbone.last_norm.*,
 *   smpl_head.transformer.{to_token_embedding.*,pos_embedding},
 *   smpl_head.transformer.transformer.layers.<l>.{0.norm,0.fn.to_qkv,0.fn.to_out.0,1.norm,1.fn.to_q,1.fn.to_kv,
 *       1.fn.to_out.0,2.norm,2.fn.net.0,2.fn.net.3}.*,
 *   smpl_head.{decpose_grot,decpose_hands,decshape,deccam}.*, smpl_head.init_{body_pose,betas,cam},
 *   smpl_head.decpose.{cls.weight,cls.bias,codebook,dec.weight,dec.bias} (stand-in naming).
 * Missing key -> VGE_ERR_MISSING_WEIGHT, wrong shape -> VGE_ERR_WEIGHT_SHAPE. */
int vge_hmr_create(const vge_hmr_config* cfg, const vge_tensor_view* weights, int n_weights, vge_hmr** out);
int vge_hmr_reserve(vge_hmr* m, int max_frames);
int vge_hmr_destroy(vge_hmr* m);

/* The TokenHMR front end's crop (ViTDetDataset.__getitem__ in 4D-Humans, driven by mesh_generator.py:119-145):
 * crop i is the 256 x 256 RGB patch of frame frame_of[i] (frame_of NULL: frame i) around boxes[i] (HOST float
 * [n_crops][4] xyxy frame pixels -- the single-person box of the frame, after the gate of mesh_generator.py:103-117):
 * center, 2.5x box scale expanded to the 192:256 aspect, the anti-alias Gaussian when the patch is downsampled by
 * more than 2.2x, cv2.warpAffine INTER_LINEAR with border 0, rounded to uint8.  frames: device uint8 [n_frames][H][W]
 * [3] RGB; crops: device uint8 [n_crops][256][256][3], the input of vge_hmr_extract.  Synchronises `stream`
 * before returning (the host instance table is released).  Parity unpinned (third-party geometry, restated). */
int vge_hmr_crop(const uint8_t* frames, int n_frames, int H, int W, const float* boxes, const int32_t* frame_of,
                 int n_crops, uint8_t* crops, vge_stream_t stream);

/* frames: device uint8 [F, in_h, in_w, 3] RGB.  Outputs (device float32, row strides as in the frame store):
 * pose [F,207] (23 rotation matrices, row-major), gori [F,9], betas [F,10], vit [F,dec_dim] (token_out). */
int vge_hmr_extract(vge_hmr* m, const uint8_t* frames, int n_frames, float* pose, float* gori, float* betas,
                    float* vit, vge_stream_t stream);

/* Device time of the backbone GEMMs / attention / rest over the next max_calls extract calls (hipEvents on
 * the extract stream).  stage_ms[0] = patch-embed + transformer-block GEMMs, [1] = attention, [2] = LayerNorms,
 * [3] = decoder head + readouts; flops[0] = algorithmic GEMM FLOPs per call of the backbone. */
int vge_hmr_profile_begin(vge_hmr* m, int max_calls);
int vge_hmr_profile_read(vge_hmr* m, double* stage_ms, int* n_calls, double* gemm_flops_per_call);

/* Op-level entry points (used by the parity tests; same kernels as vge_hmr_extract).
 * epi: 0 bf16 out (+bias), 1 bf16 GELU(x+bias), 2 f32 out = x + bias + res, 3 f32 out = x + bias +
 * pos[1 + row % tokens] + pos[0], 4 f32 out = x + bias.  Requires M % 256 == N % 256 == K % 64 == 0 and
 * lda / ldw % 8 == 0.  A [M][lda] bf16, W [N][ldw] bf16 (nn.Linear layout). */
int vge_op_gemm_bf16(int epi, const void* A, long lda, const void* W, long ldw, void* out, long ldo, const float* bias,
                     const float* res, long ldr, const float* pos, int tokens, int M, int N, int K,
                     vge_stream_t stream);
/* The same product through hipBLASLt (the extractor's library path for the bias, f32-residual and f32-out
 * epilogues 0, 2, 4; any M, N, K): VGE_ERR_UNSUPPORTED for the epilogues it does not take (GELU, PE) or with the
 * library path off (VGE_GEMM_LIB=0). */
int vge_op_gemm_lib(int epi, const void* A, long lda, const void* W, long ldw, void* out, long ldo, const float* bias,
                    const float* res, long ldr, int M, int N, int K, vge_stream_t stream);
/* qkv bf16 [F*192][3D] -> out bf16 [F*192][D]; head dim D / heads in {64, 80} */
int vge_op_vit_attention(const void* qkv, void* out, int F, int D, int heads, vge_stream_t stream);
/* LayerNorm f32 [rows][D] -> bf16, D in {256, 512, 768, 1024, 1280} */
int vge_op_layernorm_bf16(const float* x, void* y, const float* w, const float* b, int rows, int D, float eps,
                          vge_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* VGE_HMR_H */
