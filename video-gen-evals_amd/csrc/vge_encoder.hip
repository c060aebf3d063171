// HumanActionScorer forward (model.py:102-193) on gfx950, f32 in / f32 accumulate MFMA.
//
// Kernels (one launch each, in order):
//   conv_encoder_kernel   MovementConvEncoder x10 (model.py:21-58): stem (k=1) -> 4 x TemporalConvBlock
//                         (dilated k=5 conv, GELU, conv, +res, GELU, GroupNorm(1)) -> proj.  One workgroup =
//                         one encoder x 2 windows (64 rows); the whole chain runs out of LDS, weights stream
//                         through a 2-deep LDS ring by global_load_lds.  This is ~85% of the FLOPs.
//   fuse_kernel           per-modality sum + LN (model.py:169-178) and MinimalPerFrameFusion's softmax pool
//                         (model.py:79-98) with the constant query folded: logit_m = (Wk^T q).kv_m, and
//                         Wo(Wv(sum_m A_m kv_m)) computed as one GEMM with Wov = Wo Wv.
//   gemm_kernel<EPI>      [M,K] x [K,N] panel GEMM with fused epilogues: +PE/CLS token assembly,
//                         +bias, +bias+ReLU, +bias+residual+LayerNorm (post-norm transformer, model.py:145).
//   attn_kernel           33x33 softmax attention per (window, head).
//   embed_tc_kernel       L2-normalise tokens (model.py:190-193) and the per-window TC term (eval.py:223-224).
//
// MFMA: v_mfma_f32_16x16x4_f32 (exact f32 fmaf chain).  Fragment maps: lane l holds A[i=l&15][k=l>>4],
// B[k=l>>4][j=l&15]; C col = l&15, row = (l>>4)*4 + r.  K is processed in 256-wide "panels"; a panel is
// 64 MFMA K-steps of 4, K-step s of a panel uses k = s + 64*(l>>4), so one ds_read_b128 gives a lane the A
// values of 4 consecutive K-steps.  Weights are packed on the host into 16 KB "chunks" (4 K-steps x 256
// output columns) in the exact LDS image [g][n][q] = W[n][64g + 4c + q] that the B reads use.
#include "vge_common.h"
#include <cstring>

namespace {

constexpr int CHUNK_F = 4096;          // floats per weight chunk (16 KB)
constexpr int CHUNKS_PER_PANEL = 16;   // 64 K-steps / 4

// ------------------------------------------------------------------ weight-chunk ring (2 x 16 KB in LDS)
__device__ __forceinline__ void stage_chunk(const float* __restrict__ chunk, float* bst, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int piece = wave * 4 + i;  // 1 KB pieces, wave-uniform LDS base
    glds16(chunk + piece * 256 + lane * 4, bst + piece * 256);
  }
}

template <int NT>
__device__ __forceinline__ void mma_chunk(floatx4 (&acc)[NT], const floatx4 a, const float* bst, int nt0, int lane) {
  const int j = lane & 15, g = lane >> 4;
  floatx4 b[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) b[nt] = *reinterpret_cast<const floatx4*>(bst + ((g * 256 + (nt0 + nt) * 16 + j) << 2));
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[nt] = mfma16x16x4(a[q], b[nt][q], acc[nt]);
}

// Stream `nchunks` weight chunks through a 3-slot LDS ring; afn(c) returns this lane's A fragment for
// chunk c.  Chunk c+2 is DMA'd while chunk c is multiplied; the end-of-chunk wait is a counted vmcnt(4)
// that retires chunk c+1 (issued a whole chunk earlier) and leaves c+2 in flight across the barrier.
// Callers must have no other vector-memory ops outstanding except LDS-DMA they want retired with chunk 0.
template <int NT, class AFn>
__device__ __forceinline__ void run_stream(floatx4 (&acc)[NT], const float* __restrict__ chunks, int nchunks, float* bst,
                                           AFn afn, int nt0, int wave, int lane) {
  stage_chunk(chunks, bst, wave, lane);
  if (nchunks > 1) {
    stage_chunk(chunks + CHUNK_F, bst + CHUNK_F, wave, lane);
    vmcnt<4>();
  } else {
    vmcnt<0>();
  }
  lds_barrier();
  int slot = 0;
  for (int c = 0; c < nchunks; ++c) {
    const float* cur = bst + slot * CHUNK_F;
    const int slot2 = (slot >= 1) ? slot - 1 : 2;  // (slot + 2) % 3
    if (c + 2 < nchunks) stage_chunk(chunks + (size_t)(c + 2) * CHUNK_F, bst + slot2 * CHUNK_F, wave, lane);
    const floatx4 a = afn(c);
    mma_chunk<NT>(acc, a, cur, nt0, lane);
    if (c + 2 < nchunks) vmcnt<4>(); else vmcnt<0>();
    lds_barrier();
    slot = (slot == 2) ? 0 : slot + 1;
  }
}

template <int NT>
__device__ __forceinline__ void zero_acc(floatx4 (&acc)[NT]) {
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) acc[nt] = floatx4{0.f, 0.f, 0.f, 0.f};
}

// ------------------------------------------------------------------ encoder descriptors
struct EncDesc {
  const float* stem;   // n_stem_panels * 16 chunks
  const float* conv;   // 4 blocks x 2 convs x 5 taps x 16 chunks
  const float* proj;   // 16 chunks
  const float* gn_w;   // [4][256]
  const float* gn_b;   // [4][256]
  int in_col;          // column offset of this encoder's input in feats
  int d_in;
  int n_stem_panels;
  int ld;              // feats row width (2596, or 2356 keypoint-less)
};

// ------------------------------------------------------------------ conv encoder chain
// grid: n_enc * n_pairs blocks (XCD-aware order: concurrent blocks on one XCD share an encoder);
// block: 256 threads = 4 waves, wave w owns rows 16w..16w+15 = window (w>>1), frames (w&1)*16 + 0..15.
constexpr int CONV_LDS_BYTES = (64 * VGE_LDX + 3 * CHUNK_F + 64) * 4;

__global__ void __launch_bounds__(256, 1) conv_encoder_kernel(const float* __restrict__ feats, int n_windows,
                                                               const EncDesc* __restrict__ encs, int n_enc,
                                                               float* __restrict__ enc_out) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* X = lds;                          // [64][260] activations of the 2 windows
  float* bst = lds + 64 * VGE_LDX;         // 3 x 4096 weight ring
  float* red = bst + 3 * CHUNK_F;          // [16] reduction scratch

  const int n_pairs = (n_windows + 1) >> 1;
  const int nblk = n_enc * n_pairs;
  // bijective XCD remap: blocks b, b+8, ... share an XCD; give each XCD a contiguous run of work ids
  const int b = blockIdx.x;
  const int q8 = nblk >> 3, r8 = nblk & 7, x8 = b & 7;
  const int work = (x8 < r8 ? x8 * (q8 + 1) : r8 * (q8 + 1) + (x8 - r8) * q8) + (b >> 3);
  const int e = work / n_pairs, pair = work % n_pairs;
  const EncDesc ed = encs[e];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wl = wave >> 1, t0 = (wave & 1) * 16;
  const int i = lane & 15, g = lane >> 4;
  const int win = pair * 2 + wl;
  const bool win_valid = win < n_windows;
  const int rowq = (lane >> 4) * 4;  // C-layout row offset of this lane inside the wave's 16 rows

  floatx4 acc[16], res[16];

  // ---------------- stem: Conv1d(d_in -> 256, k=1, no bias)
  zero_acc(acc);
  for (int p = 0; p < ed.n_stem_panels; ++p) {
    __syncthreads();
    // stage this panel of the input (64 rows x 256 cols, zero-padded past d_in / past the last window)
    const int c = tid;  // column within the panel
    const int kcol = p * 256 + c;
    for (int r = 0; r < 64; ++r) {
      const int w = pair * 2 + (r >> 5);
      float v = 0.f;
      if (kcol < ed.d_in && w < n_windows) v = feats[((size_t)w * VGE_T + (r & 31)) * ed.ld + ed.in_col + kcol];
      X[r * VGE_LDX + c] = v;
    }
    __syncthreads();
    auto afn = [&](int cc) -> floatx4 {
      return *reinterpret_cast<const floatx4*>(X + (wl * 32 + t0 + i) * VGE_LDX + 64 * g + 4 * cc);
    };
    run_stream<16>(acc, ed.stem + (size_t)p * CHUNKS_PER_PANEL * CHUNK_F, CHUNKS_PER_PANEL, bst, afn, 0, wave, lane);
  }
#pragma unroll
  for (int nt = 0; nt < 16; ++nt) res[nt] = acc[nt];
  __syncthreads();
#pragma unroll
  for (int nt = 0; nt < 16; ++nt)
#pragma unroll
    for (int r = 0; r < 4; ++r) X[(wl * 32 + t0 + rowq + r) * VGE_LDX + nt * 16 + i] = acc[nt][r];
  __syncthreads();

  // ---------------- 4 TemporalConvBlocks
  for (int blk = 0; blk < 4; ++blk) {
    const int dil = 1 << blk;
    for (int cv = 0; cv < 2; ++cv) {
      zero_acc(acc);
      auto afn = [&](int c) -> floatx4 {
        const int tap = c >> 4, cc = c & 15;
        const int tt = t0 + i + (tap - 2) * dil;
        const bool ok = (unsigned)tt < 32u;
        const floatx4 v = *reinterpret_cast<const floatx4*>(X + (wl * 32 + (ok ? tt : 0)) * VGE_LDX + 64 * g + 4 * cc);
        return ok ? v : floatx4{0.f, 0.f, 0.f, 0.f};
      };
      run_stream<16>(acc, ed.conv + (size_t)(blk * 2 + cv) * 5 * CHUNKS_PER_PANEL * CHUNK_F, 5 * CHUNKS_PER_PANEL, bst,
                     afn, 0, wave, lane);
      if (cv == 0) {
        // y = GELU(conv1(x)); dropout is identity in eval
#pragma unroll
        for (int nt = 0; nt < 16; ++nt)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[nt][r] = gelu_erf(acc[nt][r]);
      } else {
        // z = GELU(conv2(y) + x); GroupNorm(1, 256) over the window's 256 x 32 values
        float s = 0.f;
#pragma unroll
        for (int nt = 0; nt < 16; ++nt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            acc[nt][r] = gelu_erf(acc[nt][r] + res[nt][r]);
            s += acc[nt][r];
          }
        s = wave_sum(s);
        if (lane == 0) red[wave] = s;
        __syncthreads();
        const float mean = (red[wl * 2] + red[wl * 2 + 1]) / 8192.0f;
        float v = 0.f;
#pragma unroll
        for (int nt = 0; nt < 16; ++nt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float d = acc[nt][r] - mean;
            v += d * d;
          }
        v = wave_sum(v);
        if (lane == 0) red[4 + wave] = v;
        __syncthreads();
        const float var = (red[4 + wl * 2] + red[4 + wl * 2 + 1]) / 8192.0f;
        const float rstd = 1.0f / sqrtf(var + 1e-5f);
        const float* gw = ed.gn_w + blk * 256;
        const float* gb = ed.gn_b + blk * 256;
#pragma unroll
        for (int nt = 0; nt < 16; ++nt) {
          const float w_ = gw[nt * 16 + i], b_ = gb[nt * 16 + i];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            acc[nt][r] = (acc[nt][r] - mean) * rstd * w_ + b_;
            res[nt][r] = acc[nt][r];
          }
        }
      }
      // all waves are past the barrier that ended the stream: X (input of this conv) is dead
#pragma unroll
      for (int nt = 0; nt < 16; ++nt)
#pragma unroll
        for (int r = 0; r < 4; ++r) X[(wl * 32 + t0 + rowq + r) * VGE_LDX + nt * 16 + i] = acc[nt][r];
      __syncthreads();
    }
  }

  // ---------------- proj: Linear(256 -> 256, no bias)
  zero_acc(acc);
  {
    auto afn = [&](int cc) -> floatx4 {
      return *reinterpret_cast<const floatx4*>(X + (wl * 32 + t0 + i) * VGE_LDX + 64 * g + 4 * cc);
    };
    run_stream<16>(acc, ed.proj, CHUNKS_PER_PANEL, bst, afn, 0, wave, lane);
  }
  if (win_valid) {
    float* o = enc_out + ((size_t)e * n_windows * VGE_T + (size_t)win * VGE_T + t0 + rowq) * VGE_D;
#pragma unroll
    for (int nt = 0; nt < 16; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r * VGE_D + nt * 16 + i] = acc[nt][r];
  }
}

// ------------------------------------------------------------------ modality fusion (one wave per frame row)
struct FuseParams {
  const float* kv_w;     // [256]
  const float* kv_b;     // [256]
  const float* u;        // [256] = Wk^T (Wq LN(latent))   (folded constant query)
  float inv_tau[8];      // 1 / (softplus(logit_temp) + 1e-3)
  float bias[8];         // logit_bias
  int n_mod;
  int has_motion[8];
};

// NMOD modalities in infer_dims_from_stats order: vit, global, pose, beta[, kp2d] (5, or 4 keypoint-less); enc_out
// planes 0..NMOD-1 are the state encoders, NMOD..2 NMOD-1 the motion encoders
// wave sum broadcast to every lane by DPP row reductions + one readlane (VALU latency): the shuffle butterfly's
// six LDS-latency steps per sum made a row's 25 dependent sums the fusion's long pole
__device__ __forceinline__ float wave_sum_bc(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, wave_sum_last(x)), 63));
}

template <int NMOD>
__global__ void __launch_bounds__(256) fuse_kernel(const float* __restrict__ enc_out, int n_rows, FuseParams fp,
                                                   float* __restrict__ pooled) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= n_rows) return;
  const size_t plane = (size_t)n_rows * VGE_D;
  const floatx4 kw = reinterpret_cast<const floatx4*>(fp.kv_w)[lane];
  const floatx4 kb = reinterpret_cast<const floatx4*>(fp.kv_b)[lane];
  const floatx4 u = reinterpret_cast<const floatx4*>(fp.u)[lane];
  floatx4 kv[NMOD];
  float logit[NMOD];
#pragma unroll
  for (int m = 0; m < NMOD; ++m) {
    floatx4 s = reinterpret_cast<const floatx4*>(enc_out + (size_t)m * plane + (size_t)row * VGE_D)[lane];
    if (fp.has_motion[m]) {
      const floatx4 mo = reinterpret_cast<const floatx4*>(enc_out + (size_t)(NMOD + m) * plane + (size_t)row * VGE_D)[lane];
      s = s + mo;
    }
    // F.layer_norm(s, (256,)) -- no affine
    float mu = wave_sum_bc(s[0] + s[1] + s[2] + s[3]) / 256.0f;
    floatx4 d = s - mu;
    float var = wave_sum_bc(d[0] * d[0] + d[1] * d[1] + d[2] * d[2] + d[3] * d[3]) / 256.0f;
    float rstd = 1.0f / sqrtf(var + 1e-5f);
    s = d * rstd;
    // kv_ln (affine)
    mu = wave_sum_bc(s[0] + s[1] + s[2] + s[3]) / 256.0f;
    d = s - mu;
    var = wave_sum_bc(d[0] * d[0] + d[1] * d[1] + d[2] * d[2] + d[3] * d[3]) / 256.0f;
    rstd = 1.0f / sqrtf(var + 1e-5f);
    kv[m] = d * rstd * kw + kb;
    const float qk = wave_sum_bc(u[0] * kv[m][0] + u[1] * kv[m][1] + u[2] * kv[m][2] + u[3] * kv[m][3]);
    logit[m] = (qk / 16.0f) * fp.inv_tau[m] + fp.bias[m];
  }
  float mx = logit[0];
#pragma unroll
  for (int m = 1; m < NMOD; ++m) mx = fmaxf(mx, logit[m]);
  float den = 0.f;
#pragma unroll
  for (int m = 0; m < NMOD; ++m) {
    logit[m] = expf(logit[m] - mx);
    den += logit[m];
  }
  floatx4 o = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int m = 0; m < NMOD; ++m) o += (logit[m] / den) * kv[m];
  reinterpret_cast<floatx4*>(pooled + (size_t)row * VGE_D)[lane] = o;
}

// ------------------------------------------------------------------ panel GEMM with fused epilogues
// out[M, N] = A[M, K] * W[N, K]^T.  Block = 4 waves = 2 row strips (16 rows) x 2 column halves (128 cols):
// BM = 32 rows, BN = 256 cols; grid = (ceil(M/32), N/256).  A panels (32 x 256) staged by global_load_lds.
enum Epi { EPI_TOKENS = 0, EPI_BIAS = 1, EPI_BIAS_RELU = 2, EPI_BIAS_RES_LN = 3 };

struct GemmArgs {
  const float* A;  int lda;     // rows padded to a multiple of 32 (pad rows are finite)
  const float* W;               // packed chunks [N/256][K/256][16][4096]
  float* out;      int ldo;
  int M, K, N;
  const float* bias;            // [N]
  const float* res;  int ldr;   // residual (EPI_BIAS_RES_LN)
  const float* ln_w; const float* ln_b;
  const float* pe;              // EPI_TOKENS: pos_enc.pe [5000,256]
  const float* cls;             // EPI_TOKENS: cls [256]
};

constexpr int GEMM_LDS_BYTES = (32 * VGE_LDX + 3 * CHUNK_F + 64) * 4;

template <int EPI>
__global__ void __launch_bounds__(256) gemm_kernel(GemmArgs ga) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* As = lds;                   // [32][260]
  float* bst = lds + 32 * VGE_LDX;   // weight ring (3 slots)
  float* red = bst + 3 * CHUNK_F;    // [32][2]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ws = wave >> 1, wn = wave & 1;  // row strip, column half
  const int i = lane & 15, g = lane >> 4, rowq = (lane >> 4) * 4;
  const int row0 = blockIdx.x * 32, nb = blockIdx.y;
  const int n_panels = ga.K / 256;

  floatx4 acc[8];
  zero_acc(acc);
  for (int p = 0; p < n_panels; ++p) {
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int r = wave * 8 + k;
      glds16(ga.A + (size_t)(row0 + r) * ga.lda + p * 256 + lane * 4, As + r * VGE_LDX);
    }
    auto afn = [&](int cc) -> floatx4 {
      return *reinterpret_cast<const floatx4*>(As + (ws * 16 + i) * VGE_LDX + 64 * g + 4 * cc);
    };
    run_stream<8>(acc, ga.W + ((size_t)nb * n_panels + p) * CHUNKS_PER_PANEL * CHUNK_F, CHUNKS_PER_PANEL, bst, afn,
                  wn * 8, wave, lane);
  }

  const int colb = nb * 256 + wn * 128;
  if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_RELU) {
#pragma unroll
    for (int nt = 0; nt < 8; ++nt) {
      const int col = colb + nt * 16 + i;
      const float bb = ga.bias[col];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = row0 + ws * 16 + rowq + r;
        float v = acc[nt][r] + bb;
        if (EPI == EPI_BIAS_RELU) v = fmaxf(v, 0.f);
        if (row < ga.M) ga.out[(size_t)row * ga.ldo + col] = v;
      }
    }
  } else if constexpr (EPI == EPI_TOKENS) {
    // rows are frames (w*32 + t) -> token row w*33 + 1 + t; + pos_enc.pe[1 + t]; CLS row = cls + pe[0]
#pragma unroll
    for (int nt = 0; nt < 8; ++nt) {
      const int col = colb + nt * 16 + i;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = row0 + ws * 16 + rowq + r;
        if (row < ga.M) {
          const int w = row >> 5, t = row & 31;
          ga.out[((size_t)w * VGE_TOK + 1 + t) * ga.ldo + col] = acc[nt][r] + ga.pe[(1 + t) * VGE_D + col];
          if (t == 0) ga.out[(size_t)w * VGE_TOK * ga.ldo + col] = ga.cls[col] + ga.pe[col];
        }
      }
    }
  } else {  // EPI_BIAS_RES_LN: LayerNorm(res + acc + bias) over the 256 columns (N == 256)
    float s[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int nt = 0; nt < 8; ++nt) {
      const int col = colb + nt * 16 + i;
      const float bb = ga.bias[col];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = row0 + ws * 16 + rowq + r;
        acc[nt][r] = acc[nt][r] + bb + ga.res[(size_t)row * ga.ldr + col];
        s[r] += acc[nt][r];
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      s[r] = group16_sum(s[r]);
      if (i == 0) red[(ws * 16 + rowq + r) * 2 + wn] = s[r];
    }
    __syncthreads();
    float mean[4], v[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int lr = ws * 16 + rowq + r;
      mean[r] = (red[lr * 2] + red[lr * 2 + 1]) / 256.0f;
    }
#pragma unroll
    for (int nt = 0; nt < 8; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float d = acc[nt][r] - mean[r];
        v[r] += d * d;
      }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      v[r] = group16_sum(v[r]);
      if (i == 0) red[(ws * 16 + rowq + r) * 2 + wn] = v[r];
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int lr = ws * 16 + rowq + r;
      const float var = (red[lr * 2] + red[lr * 2 + 1]) / 256.0f;
      v[r] = 1.0f / sqrtf(var + 1e-5f);
    }
#pragma unroll
    for (int nt = 0; nt < 8; ++nt) {
      const int col = colb + nt * 16 + i;
      const float lw = ga.ln_w[col], lb = ga.ln_b[col];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = row0 + ws * 16 + rowq + r;
        if (row < ga.M) ga.out[(size_t)row * ga.ldo + col] = (acc[nt][r] - mean[r]) * v[r] * lw + lb;
      }
    }
  }
}

// ------------------------------------------------------------------ self-attention, 33 tokens, head dim 32
// grid (n_windows, heads/4), block 256 = 4 waves, one head per wave; lane t < 33 owns query row t.
__global__ void __launch_bounds__(256) attn_kernel(const float* __restrict__ qkv, float* __restrict__ out) {
  __shared__ float Ks[4][VGE_TOK][33];
  __shared__ float Vs[4][VGE_TOK][32];
  const int w = blockIdx.x, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int h = blockIdx.y * 4 + wave;
  const float* base = qkv + (size_t)w * VGE_TOK * 768;
  for (int idx = lane; idx < VGE_TOK * 32; idx += 64) {
    const int t = idx >> 5, d = idx & 31;
    Ks[wave][t][d] = base[(size_t)t * 768 + 256 + h * 32 + d];
    Vs[wave][t][d] = base[(size_t)t * 768 + 512 + h * 32 + d];
  }
  __syncthreads();
  if (lane >= VGE_TOK) return;
  const float scale = 0.17677669529663687f;  // 1/sqrt(32)
  float q[32];
#pragma unroll
  for (int d = 0; d < 32; ++d) q[d] = base[(size_t)lane * 768 + h * 32 + d] * scale;
  float sc[VGE_TOK];
  float mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < VGE_TOK; ++j) {
    float a = 0.f;
#pragma unroll
    for (int d = 0; d < 32; ++d) a += q[d] * Ks[wave][j][d];
    sc[j] = a;
    mx = fmaxf(mx, a);
  }
  float den = 0.f;
#pragma unroll
  for (int j = 0; j < VGE_TOK; ++j) {
    sc[j] = expf(sc[j] - mx);
    den += sc[j];
  }
  const float inv = 1.0f / den;
  float o[32];
#pragma unroll
  for (int d = 0; d < 32; ++d) o[d] = 0.f;
#pragma unroll
  for (int j = 0; j < VGE_TOK; ++j) {
    const float pj = sc[j] * inv;
#pragma unroll
    for (int d = 0; d < 32; ++d) o[d] += pj * Vs[wave][j][d];
  }
  float* orow = out + ((size_t)w * VGE_TOK + lane) * VGE_D + h * 32;
#pragma unroll
  for (int d = 0; d < 32; d += 4) *reinterpret_cast<floatx4*>(orow + d) = floatx4{o[d], o[d + 1], o[d + 2], o[d + 3]};
}

// ------------------------------------------------------------------ outputs + per-window TC (one wave per window)
__global__ void __launch_bounds__(256) embed_tc_kernel(const float* __restrict__ x, int n_windows,
                                                       float* __restrict__ seq_embed, float* __restrict__ frame_embed,
                                                       float* __restrict__ tc) {
  const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (w >= n_windows) return;
  floatx4 prev = {0.f, 0.f, 0.f, 0.f};
  float tcsum = 0.f;
  for (int r = 0; r < VGE_TOK; ++r) {
    const floatx4 v = reinterpret_cast<const floatx4*>(x + ((size_t)w * VGE_TOK + r) * VGE_D)[lane];
    const float n = fmaxf(sqrtf(wave_sum(v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3])), 1e-12f);
    const floatx4 f = v / n;
    if (frame_embed) reinterpret_cast<floatx4*>(frame_embed + ((size_t)w * VGE_TOK + r) * VGE_D)[lane] = f;
    if (r == 0) reinterpret_cast<floatx4*>(seq_embed + (size_t)w * VGE_D)[lane] = f;
    if (r >= 2) {
      const floatx4 d = f - prev;
      tcsum += sqrtf(wave_sum(d[0] * d[0] + d[1] * d[1] + d[2] * d[2] + d[3] * d[3]));
    }
    prev = f;
  }
  if (tc && lane == 0) tc[w] = tcsum / (float)(VGE_TOK - 2);
}

}  // namespace

// ================================================================== host launchers
namespace vge {

struct EncDescHost {
  const float* stem; const float* conv; const float* proj; const float* gn_w; const float* gn_b;
  int in_col, d_in, n_stem_panels, ld;
};
static_assert(sizeof(EncDescHost) == sizeof(EncDesc), "EncDesc layout");

struct FuseParamsHost {
  const float* kv_w; const float* kv_b; const float* u;
  float inv_tau[8]; float bias[8]; int n_mod; int has_motion[8];
};
static_assert(sizeof(FuseParamsHost) == sizeof(FuseParams), "FuseParams layout");

struct GemmArgsHost {
  const float* A; int lda; const float* W; float* out; int ldo; int M, K, N;
  const float* bias; const float* res; int ldr; const float* ln_w; const float* ln_b; const float* pe; const float* cls;
};
static_assert(sizeof(GemmArgsHost) == sizeof(GemmArgs), "GemmArgs layout");

hipError_t encoder_kernel_setup() {
  hipError_t e = hipFuncSetAttribute((const void*)conv_encoder_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     CONV_LDS_BYTES);
  if (e != hipSuccess) return e;
  const void* gk[4] = {(const void*)gemm_kernel<EPI_TOKENS>, (const void*)gemm_kernel<EPI_BIAS>,
                       (const void*)gemm_kernel<EPI_BIAS_RELU>, (const void*)gemm_kernel<EPI_BIAS_RES_LN>};
  for (auto k : gk) {
    e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, GEMM_LDS_BYTES);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t launch_conv_encoders(const float* feats, int n_windows, const void* encs, int n_enc, float* enc_out,
                                hipStream_t s) {
  const int n_pairs = (n_windows + 1) / 2;
  hipLaunchKernelGGL(conv_encoder_kernel, dim3(n_enc * n_pairs), dim3(256), CONV_LDS_BYTES, s, feats, n_windows,
                     reinterpret_cast<const EncDesc*>(encs), n_enc, enc_out);
  return hipGetLastError();
}

hipError_t launch_fuse(const float* enc_out, int n_rows, const FuseParamsHost& fp, float* pooled, hipStream_t s) {
  FuseParams p;
  memcpy(&p, &fp, sizeof(p));
  if (fp.n_mod == 4)
    hipLaunchKernelGGL(fuse_kernel<4>, dim3((n_rows + 3) / 4), dim3(256), 0, s, enc_out, n_rows, p, pooled);
  else if (fp.n_mod == 5)
    hipLaunchKernelGGL(fuse_kernel<5>, dim3((n_rows + 3) / 4), dim3(256), 0, s, enc_out, n_rows, p, pooled);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_gemm(int epi, const GemmArgsHost& a, hipStream_t s) {
  GemmArgs g;
  memcpy(&g, &a, sizeof(g));
  dim3 grid((a.M + 31) / 32, a.N / 256);
  switch (epi) {
    case EPI_TOKENS: hipLaunchKernelGGL(gemm_kernel<EPI_TOKENS>, grid, dim3(256), GEMM_LDS_BYTES, s, g); break;
    case EPI_BIAS: hipLaunchKernelGGL(gemm_kernel<EPI_BIAS>, grid, dim3(256), GEMM_LDS_BYTES, s, g); break;
    case EPI_BIAS_RELU: hipLaunchKernelGGL(gemm_kernel<EPI_BIAS_RELU>, grid, dim3(256), GEMM_LDS_BYTES, s, g); break;
    default: hipLaunchKernelGGL(gemm_kernel<EPI_BIAS_RES_LN>, grid, dim3(256), GEMM_LDS_BYTES, s, g); break;
  }
  return hipGetLastError();
}

hipError_t launch_attn(const float* qkv, int n_windows, float* out, hipStream_t s) {
  hipLaunchKernelGGL(attn_kernel, dim3(n_windows, 2), dim3(256), 0, s, qkv, out);
  return hipGetLastError();
}

hipError_t launch_embed_tc(const float* x, int n_windows, float* seq, float* frame, float* tc, hipStream_t s) {
  hipLaunchKernelGGL(embed_tc_kernel, dim3((n_windows + 3) / 4), dim3(256), 0, s, x, n_windows, seq, frame, tc);
  return hipGetLastError();
}

}  // namespace vge
