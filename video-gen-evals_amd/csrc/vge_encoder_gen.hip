// HumanActionScorer forward (model.py:102-193) for checkpoints of any shape load_model accepts (eval.py:136-158 reads
// d_model, time_layers and time_heads from the checkpoint): exact f32 on the VALU, one kernel per stage.  The tiled
// MFMA kernels (vge_encoder.hip, vge_encoder_x3*.hip, vge_transformer_x3.hip) are built around d_model 256 and 8 heads
// of 32; this path serves every other d_model (32 .. 256, a multiple of 32) and head count (head dim <= 64).
//
//   gen_conv_kernel      Conv1d (stem k = 1, dilated k = 5 convs with "same" padding inside the 32-frame window) and
//                        Linear (proj): one workgroup per (window, 64 output channels), input rows + halo and the
//                        weight tile staged in LDS per 64 input channels; epilogue GELU / GELU(x + res)
//   gen_groupnorm_kernel GroupNorm(1, d) per window over its 32 x d values (biased variance, eps 1e-5, affine)
//   gen_fuse_kernel      per-modality sum + LayerNorm, kv_ln, the folded query's logits, softmax over modalities,
//                        sum of a_m kv_m (the Wo Wv product follows as one GEMM)
//   gen_gemm_kernel      out = A W^T + bias (+ ReLU / + residual / token assembly with the positional encoding)
//   gen_attn_kernel      33 x 33 softmax attention per (window, head)
//   gen_add_ln_kernel    LayerNorm(a + b) per token row (post-norm encoder layer)
//   gen_embed_tc_kernel  normalize (model.py:190-193) + the per-window TC term (eval.py:209-226)
#include "vge_common.h"

namespace {

constexpr int GT = 32;   // frames per window
constexpr int GTOK = 33; // CLS + frames

__device__ __forceinline__ float gelu_exact(float x) { return x * 0.5f * (1.0f + erff(x * 0.70710678118654752440f)); }

__device__ __forceinline__ float block_sum256(float v, float* red) {  // 256 threads
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) red[wave] = v;
  __syncthreads();
  const float s = red[0] + red[1] + red[2] + red[3];
  __syncthreads();
  return s;
}

// out[w*32 + t][co] (ld cout) = sum_{tap, ci} W[co][ci][tap] x[w*32 + t + (tap - taps/2) dil][xcol + ci]
// (rows outside the window read 0); epi 0: plain, 1: GELU, 2: GELU(v + res[row][co])
__global__ void __launch_bounds__(256) gen_conv_kernel(const float* __restrict__ x, int ldx, int xcol, int cin,
                                                       const float* __restrict__ Wt, int cout, int taps, int dil,
                                                       int epi, const float* __restrict__ res,
                                                       float* __restrict__ out) {
  __shared__ float xs[GT + 32][65];  // rows -pad .. 32 + pad (pad <= 16), 64 input channels
  __shared__ float ws[64][65];       // one tap's [ci][co] tile
  const int w = blockIdx.x, co0 = blockIdx.y * 64;
  const int tid = threadIdx.x, t = tid >> 3, cg = tid & 7;
  const int pad = (taps / 2) * dil;
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  for (int ci0 = 0; ci0 < cin; ci0 += 64) {
    const int nci = min(64, cin - ci0);
    for (int q = tid; q < (GT + 2 * pad) * 64; q += 256) {
      const int r = q >> 6, c = q & 63, tt = r - pad;
      xs[r][c] = (c < nci && tt >= 0 && tt < GT) ? x[((size_t)w * GT + tt) * ldx + xcol + ci0 + c] : 0.f;
    }
    for (int tap = 0; tap < taps; ++tap) {
      for (int q = tid; q < 64 * 64; q += 256) {
        const int co = q >> 6, c = q & 63;
        ws[c][co] = (co0 + co < cout && c < nci) ? Wt[((size_t)(co0 + co) * cin + ci0 + c) * taps + tap] : 0.f;
      }
      __syncthreads();
      const int r = t + pad + (tap - taps / 2) * dil;
      for (int c = 0; c < nci; ++c) {
        const float xv = xs[r][c];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = fmaf(xv, ws[c][cg + 8 * j], acc[j]);
      }
      __syncthreads();
    }
  }
  const size_t row = (size_t)w * GT + t;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int co = co0 + cg + 8 * j;
    if (co >= cout) continue;
    float v = acc[j];
    if (epi == 1) v = gelu_exact(v);
    if (epi == 2) v = gelu_exact(v + res[row * cout + co]);
    out[row * cout + co] = v;
  }
}

// GroupNorm(1, d) in place on window w's rows [32][d]
__global__ void __launch_bounds__(256) gen_groupnorm_kernel(float* __restrict__ x, int d, const float* __restrict__ g,
                                                            const float* __restrict__ b) {
  __shared__ float red[4];
  float* p = x + (size_t)blockIdx.x * GT * d;
  const int n = GT * d;
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) s += p[i];
  const float mean = block_sum256(s, red) / (float)n;
  float v = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) {
    const float q = p[i] - mean;
    v += q * q;
  }
  const float var = block_sum256(v, red) / (float)n;
  const float rstd = 1.0f / sqrtf(var + 1e-5f);
  for (int i = threadIdx.x; i < n; i += 256) {
    const int c = i % d;
    p[i] = (p[i] - mean) * rstd * g[c] + b[c];
  }
}

struct GenFuse {
  const float* kv_w; const float* kv_b; const float* u;  // [d] each (u = Wk^T Wq q_ln(latent))
  float inv_tau[8], bias[8];
  int n_mod, d;
  int has_motion[8];
};

// one wave per frame row; lane holds columns lane + 64 j (j < 4)
__global__ void __launch_bounds__(256) gen_fuse_kernel(const float* __restrict__ enc_out, int n_rows, GenFuse f,
                                                       float* __restrict__ pooled_pre) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= n_rows) return;
  const int d = f.d, M = f.n_mod;
  const size_t plane = (size_t)n_rows * d;
  float kv[8][4], logit[8];
  const float invd = 1.0f / (float)d, isq = 1.0f / sqrtf((float)d);
  for (int m = 0; m < M; ++m) {
    float s[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = lane + 64 * j;
      s[j] = 0.f;
      if (c < d) {
        s[j] = enc_out[(size_t)m * plane + (size_t)row * d + c];
        if (f.has_motion[m]) s[j] += enc_out[(size_t)(M + m) * plane + (size_t)row * d + c];
      }
    }
    for (int pass = 0; pass < 2; ++pass) {  // F.layer_norm (no affine), then kv_ln (affine)
      const float mu = wave_sum(s[0] + s[1] + s[2] + s[3]) * invd;
      float q = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (lane + 64 * j < d) q += (s[j] - mu) * (s[j] - mu);
      const float rstd = 1.0f / sqrtf(wave_sum(q) * invd + 1e-5f);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = lane + 64 * j;
        s[j] = c < d ? (pass ? (s[j] - mu) * rstd * f.kv_w[c] + f.kv_b[c] : (s[j] - mu) * rstd) : 0.f;
      }
    }
    float qk = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      kv[m][j] = s[j];
      if (lane + 64 * j < d) qk += f.u[lane + 64 * j] * s[j];
    }
    logit[m] = (wave_sum(qk) * isq) * f.inv_tau[m] + f.bias[m];
  }
  float mx = logit[0];
  for (int m = 1; m < M; ++m) mx = fmaxf(mx, logit[m]);
  float den = 0.f;
  for (int m = 0; m < M; ++m) {
    logit[m] = expf(logit[m] - mx);
    den += logit[m];
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = lane + 64 * j;
    if (c >= d) continue;
    float o = 0.f;
    for (int m = 0; m < M; ++m) o += (logit[m] / den) * kv[m][j];
    pooled_pre[(size_t)row * d + c] = o;
  }
}

// out[r][n] = sum_k A[r][k] W[n][k] (+ bias); 64 x 64 tiles, 256 threads x 4 x 4 outputs
// epi 0: + bias; 1: relu(+ bias); 2: + bias + res[r][n]; 3: tokens (rows = frames w*32 + t -> token row w*33 + 1 + t,
// + pe[1 + t]; the CLS row w*33 = cls + pe[0] written by the t == 0 rows)
__global__ void __launch_bounds__(256) gen_gemm_kernel(const float* __restrict__ A, int lda, const float* __restrict__ Wt,
                                                       int M, int N, int K, const float* __restrict__ bias, int epi,
                                                       const float* __restrict__ res, const float* __restrict__ pe,
                                                       const float* __restrict__ cls, float* __restrict__ out, int ldo) {
  __shared__ float As[16][65], Bs[16][65];
  const int m0 = blockIdx.x * 64, n0 = blockIdx.y * 64;
  const int tid = threadIdx.x, tr = tid >> 4, tc = tid & 15;
  float acc[4][4] = {};
  for (int k0 = 0; k0 < K; k0 += 16) {
    for (int q = tid; q < 16 * 64; q += 256) {
      const int r = q >> 4, k = q & 15;
      As[k][r] = (m0 + r < M && k0 + k < K) ? A[(size_t)(m0 + r) * lda + k0 + k] : 0.f;
      Bs[k][r] = (n0 + r < N && k0 + k < K) ? Wt[(size_t)(n0 + r) * K + k0 + k] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      float a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        a[i] = As[k][tr * 4 + i];
        b[i] = Bs[k][tc * 4 + i];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(a[i], b[j], acc[i][j]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = m0 + tr * 4 + i;
    if (r >= M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + tc * 4 + j;
      if (n >= N) continue;
      float v = acc[i][j] + (bias ? bias[n] : 0.f);
      if (epi == 1) v = fmaxf(v, 0.f);
      if (epi == 2) v += res[(size_t)r * N + n];
      if (epi == 3) {
        const int w = r / GT, t = r - w * GT;
        out[((size_t)w * GTOK + 1 + t) * ldo + n] = v + pe[(size_t)(1 + t) * N + n];
        if (t == 0) out[(size_t)w * GTOK * ldo + n] = cls[n] + pe[n];
      } else {
        out[(size_t)r * ldo + n] = v;
      }
    }
  }
}

// softmax attention of one (window, head): qkv [B*33][3d] (q | k | v, heads of hd contiguous inside each)
__global__ void __launch_bounds__(64) gen_attn_kernel(const float* __restrict__ qkv, int d, int heads,
                                                      float* __restrict__ out) {
  const int w = blockIdx.x, h = blockIdx.y, hd = d / heads, lane = threadIdx.x;
  __shared__ float Qs[GTOK][65], Ks[GTOK][65], Vs[GTOK][65], Ss[GTOK][GTOK + 1];
  const float* base = qkv + (size_t)w * GTOK * 3 * d;
  const float scale = 1.0f / sqrtf((float)hd);
  for (int q = lane; q < GTOK * hd; q += 64) {
    const int t = q / hd, c = q - t * hd;
    Qs[t][c] = base[(size_t)t * 3 * d + h * hd + c] * scale;
    Ks[t][c] = base[(size_t)t * 3 * d + d + h * hd + c];
    Vs[t][c] = base[(size_t)t * 3 * d + 2 * d + h * hd + c];
  }
  __syncthreads();
  if (lane >= GTOK) return;
  float mx = -INFINITY;
  for (int j = 0; j < GTOK; ++j) {
    float a = 0.f;
    for (int c = 0; c < hd; ++c) a = fmaf(Qs[lane][c], Ks[j][c], a);
    Ss[lane][j] = a;
    mx = fmaxf(mx, a);
  }
  float den = 0.f;
  for (int j = 0; j < GTOK; ++j) {
    const float e = expf(Ss[lane][j] - mx);
    Ss[lane][j] = e;
    den += e;
  }
  const float inv = 1.0f / den;
  float* o = out + ((size_t)w * GTOK + lane) * d + h * hd;
  for (int c = 0; c < hd; ++c) {
    float a = 0.f;
    for (int j = 0; j < GTOK; ++j) a = fmaf(Ss[lane][j] * inv, Vs[j][c], a);
    o[c] = a;
  }
}

// out[r] = LayerNorm(a[r] + b[r]) (eps 1e-5, affine), one wave per row, d <= 256
__global__ void __launch_bounds__(256) gen_add_ln_kernel(const float* __restrict__ a, const float* __restrict__ b, int rows,
                                                         int d, const float* __restrict__ g, const float* __restrict__ be,
                                                         float* __restrict__ out) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= rows) return;
  float s[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = lane + 64 * j;
    s[j] = c < d ? a[(size_t)row * d + c] + b[(size_t)row * d + c] : 0.f;
  }
  const float invd = 1.0f / (float)d;
  const float mu = wave_sum(s[0] + s[1] + s[2] + s[3]) * invd;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (lane + 64 * j < d) q += (s[j] - mu) * (s[j] - mu);
  const float rstd = 1.0f / sqrtf(wave_sum(q) * invd + 1e-5f);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = lane + 64 * j;
    if (c < d) out[(size_t)row * d + c] = (s[j] - mu) * rstd * g[c] + be[c];
  }
}

// one wave per window: F.normalize of every token row (eps 1e-12), seq = row 0, TC = mean over t of
// |f_{t+1} - f_t| of the 32 frame rows (rows 1..32)
__global__ void __launch_bounds__(256) gen_embed_tc_kernel(const float* __restrict__ x, int n_windows, int d,
                                                           float* __restrict__ seq, float* __restrict__ frame,
                                                           float* __restrict__ tc) {
  const int w = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (w >= n_windows) return;
  float prev[4] = {0.f, 0.f, 0.f, 0.f}, tcs = 0.f;
  for (int r = 0; r < GTOK; ++r) {
    float v[4], ss = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = lane + 64 * j;
      v[j] = c < d ? x[((size_t)w * GTOK + r) * d + c] : 0.f;
      ss += v[j] * v[j];
    }
    const float nrm = fmaxf(sqrtf(wave_sum(ss)), 1e-12f);
    float dd = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = lane + 64 * j;
      v[j] = v[j] / nrm;
      if (c < d) {
        if (frame) frame[((size_t)w * GTOK + r) * d + c] = v[j];
        if (r == 0) seq[(size_t)w * d + c] = v[j];
      }
      dd += (v[j] - prev[j]) * (v[j] - prev[j]);
      prev[j] = v[j];
    }
    dd = wave_sum(dd);
    if (r >= 2) tcs += sqrtf(dd);
  }
  if (tc && lane == 0) tc[w] = tcs / (float)(GTOK - 2);
}

}  // namespace

namespace vge {

struct GenFuseHost {
  const float* kv_w; const float* kv_b; const float* u;
  float inv_tau[8], bias[8];
  int n_mod, d;
  int has_motion[8];
};

hipError_t launch_gen_conv(const float* x, int ldx, int xcol, int cin, const float* W, int cout, int taps, int dil, int epi,
                           const float* res, float* out, int n_windows, hipStream_t s) {
  if (taps > 5 || (taps / 2) * dil > 16) return hipErrorInvalidValue;
  hipLaunchKernelGGL(gen_conv_kernel, dim3(n_windows, (cout + 63) / 64), dim3(256), 0, s, x, ldx, xcol, cin, W, cout, taps,
                     dil, epi, res, out);
  return hipGetLastError();
}
hipError_t launch_gen_groupnorm(float* x, int n_windows, int d, const float* g, const float* b, hipStream_t s) {
  hipLaunchKernelGGL(gen_groupnorm_kernel, dim3(n_windows), dim3(256), 0, s, x, d, g, b);
  return hipGetLastError();
}
hipError_t launch_gen_fuse(const float* enc_out, int n_rows, const GenFuseHost& f, float* pooled_pre, hipStream_t s) {
  GenFuse g;
  g.kv_w = f.kv_w;
  g.kv_b = f.kv_b;
  g.u = f.u;
  g.n_mod = f.n_mod;
  g.d = f.d;
  for (int m = 0; m < 8; ++m) {
    g.inv_tau[m] = f.inv_tau[m];
    g.bias[m] = f.bias[m];
    g.has_motion[m] = f.has_motion[m];
  }
  hipLaunchKernelGGL(gen_fuse_kernel, dim3((n_rows + 3) / 4), dim3(256), 0, s, enc_out, n_rows, g, pooled_pre);
  return hipGetLastError();
}
hipError_t launch_gen_gemm(const float* A, int lda, const float* W, int M, int N, int K, const float* bias, int epi,
                           const float* res, const float* pe, const float* cls, float* out, int ldo, hipStream_t s) {
  hipLaunchKernelGGL(gen_gemm_kernel, dim3((M + 63) / 64, (N + 63) / 64), dim3(256), 0, s, A, lda, W, M, N, K, bias, epi,
                     res, pe, cls, out, ldo);
  return hipGetLastError();
}
hipError_t launch_gen_attn(const float* qkv, int n_windows, int d, int heads, float* out, hipStream_t s) {
  if (d % heads || d / heads > 64) return hipErrorInvalidValue;
  hipLaunchKernelGGL(gen_attn_kernel, dim3(n_windows, heads), dim3(64), 0, s, qkv, d, heads, out);
  return hipGetLastError();
}
hipError_t launch_gen_add_ln(const float* a, const float* b, int rows, int d, const float* g, const float* be, float* out,
                             hipStream_t s) {
  hipLaunchKernelGGL(gen_add_ln_kernel, dim3((rows + 3) / 4), dim3(256), 0, s, a, b, rows, d, g, be, out);
  return hipGetLastError();
}
hipError_t launch_gen_embed_tc(const float* x, int n_windows, int d, float* seq, float* frame, float* tc, hipStream_t s) {
  hipLaunchKernelGGL(gen_embed_tc_kernel, dim3((n_windows + 3) / 4), dim3(256), 0, s, x, n_windows, d, seq, frame, tc);
  return hipGetLastError();
}

}  // namespace vge
