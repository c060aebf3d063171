// RTMPose whole-body head + DWPose output composition on gfx950 (the dense layers run on conv_bf16_kernel,
// vge_cnn.hip).
//
//   head_sn_t_kernel     RTMCCHead: flatten(final_layer(x), 2) -> ScaleNorm over the h*w positions of each
//                        keypoint channel -> bf16 rows [inst * K + k][hw (zero padded)]
//   scalenorm_rows_kernel RTMCCBlock.ln: ScaleNorm over the hidden dim -> bf16
//   gau_attn_kernel      RTMCCBlock token mixing of one instance: q / k = base * gamma + beta, kernel =
//                        relu(q k^T / sqrt(s))^2, out = u * (kernel @ v) (f32 on the VALU, K x K kernel in LDS)
//   simcc_decode_kernel  get_simcc_maximum: first-index argmax over the x / y bins, vals = min of the maxima,
//                        locs = -1 where vals <= 0, / split ratio
//   kp120_kernel         onnxpose.postprocess (float64) + wholebody neck / OpenPose reorder + dwpose_init's
//                        normalisation (/ W, / H; hand points with score < 0.3 -> -1, body points unmasked) +
//                        flatten_first_person_no_padding
#include "vge_common.h"
#include "vge_lds_attr.h"
#include "vge_cnn.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>

namespace {

typedef __bf16 bf16;
typedef float floatx16 __attribute__((ext_vector_type(16)));

__global__ void __launch_bounds__(256) head_sn_t_kernel(const float* __restrict__ y, long ldy, int hw, int K, int Kp,
                                                        float g, float inv_sqrt_hw, long n_rows, bf16* __restrict__ out) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);  // row = inst * K + k
  const int lane = threadIdx.x & 63;
  if (row >= n_rows) return;
  const long inst = row / K;
  const int k = (int)(row - inst * K);
  float v[4];
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int p = lane + 64 * j;
    v[j] = p < hw ? y[(inst * hw + p) * ldy + k] : 0.f;
    ss = fmaf(v[j], v[j], ss);
  }
  ss = wave_sum(ss);
  const float norm = fmaxf(sqrtf(ss) * inv_sqrt_hw, 1e-5f);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int p = lane + 64 * j;
    if (p < Kp) out[row * Kp + p] = (bf16)(p < hw ? v[j] / norm * g : 0.f);
  }
}

// D = 256 per row (RTMPose hidden dims), one wave per row, 4 values per lane
__global__ void __launch_bounds__(256) scalenorm_rows_kernel(const float* __restrict__ x, int D, float g,
                                                             float inv_sqrt_d, long rows, bf16* __restrict__ y) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  float v[8];
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = lane + 64 * j;
    v[j] = c < D ? x[row * D + c] : 0.f;
    ss = fmaf(v[j], v[j], ss);
  }
  ss = wave_sum(ss);
  const float norm = fmaxf(sqrtf(ss) * inv_sqrt_d, 1e-5f);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = lane + 64 * j;
    if (c < D) y[row * D + c] = (bf16)(v[j] / norm * g);
  }
}

// One workgroup (4 waves) per instance.  uv [inst * K + t][2E + S] f32 (SiLU already applied): u = cols
// [0, E), v = [E, 2E), base = [2E, 2E + S).  LDS: k-matrix [K][S + 1], kernel [K][KP], one q row per wave.
template <int KMAX>
__global__ void __launch_bounds__(256) gau_attn_kernel(const float* __restrict__ uv, int K, int E, int S,
                                                       const float* __restrict__ gamma, const float* __restrict__ beta,
                                                       float sqrt_s, bf16* __restrict__ out) {
  extern __shared__ float sm[];
  constexpr int KP = KMAX + 1;
  const int SP = S + 1;
  float* kk = sm;                       // [K][SP]
  float* A = kk + KMAX * SP;            // [K][KP]
  float* qrow = A + KMAX * KP;          // [4][S]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const long base_row = (long)blockIdx.x * K;
  const int ld = 2 * E + S;
  for (int idx = tid; idx < K * S; idx += 256) {
    const int j = idx / S, s = idx - j * S;
    kk[j * SP + s] = uv[(base_row + j) * ld + 2 * E + s] * gamma[S + s] + beta[S + s];
  }
  __syncthreads();
  for (int i = wave; i < K; i += 4) {
    for (int s = lane; s < S; s += 64) qrow[wave * S + s] = uv[(base_row + i) * ld + 2 * E + s] * gamma[s] + beta[s];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    for (int j = lane; j < K; j += 64) {
      float d = 0.f;
      for (int s = 0; s < S; ++s) d = fmaf(qrow[wave * S + s], kk[j * SP + s], d);
      const float r = fmaxf(d / sqrt_s, 0.f);
      A[i * KP + j] = r * r;
    }
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();
  // out[i][e] = u[i][e] * sum_j A[i][j] v[j][e]: 128-column chunks of v staged in LDS over the (dead) k-matrix;
  // thread = one column e (coalesced v / u / out) x 4-row groups, the two thread halves take alternate groups
  float* vs = kk;  // [K][128]
  const int el = tid & 127, half = tid >> 7;
  for (int e0 = 0; e0 < E; e0 += 128) {
    __syncthreads();
    for (int j = half; j < K; j += 2) vs[j * 128 + el] = uv[(base_row + j) * ld + E + e0 + el];
    __syncthreads();
    for (int i0 = 4 * half; i0 < K; i0 += 8) {
      float acc[4] = {0.f, 0.f, 0.f, 0.f};
      for (int j = 0; j < K; ++j) {
        const float v = vs[j * 128 + el];
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[r] = fmaf(A[(i0 + r) * KP + j], v, acc[r]);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (i0 + r < K)
          out[(base_row + i0 + r) * E + e0 + el] = (bf16)(uv[(base_row + i0 + r) * ld + e0 + el] * acc[r]);
    }
  }
}

// The same token mixing on exact-f32 MFMAs (v_mfma_f32_32x32x2_f32): lane l supplies A[m = l % 32][k = l / 32] and
// B[k = l / 32][n = l % 32], register r of D is row (r & 3) + 8 (r >> 2) + 4 (l / 32), column l % 32.  One
// workgroup (4 waves) per instance; tokens padded to 160 rows (5 tiles), pad rows / keys read as 0.
//   phase 1  base = uv[:, 2E : 2E + S] -> LDS [K][S + 1] (conflict-free column reads)
//   phase 2  kernel tile (ti, tj) = sum_k q[m][k] k[n][k], q = base * gamma0 + beta0, k = base * gamma1 + beta1
//            formed per element as torch does (a product, then a sum), relu(x / sqrt(s))^2 -> LDS [K][K | 1]
//   phase 3  u * (kernel @ v): v staged 128 columns at a time in LDS over the dead base rows (row stride 160:
//            the two k rows of a step land in opposite bank halves), 5 x 4 tiles per round
constexpr int GAU_M_TILES = 5;  // 160 padded tokens
__device__ __forceinline__ floatx16 mfma_f32x2(float a, float b, floatx16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
__global__ void __launch_bounds__(256) gau_mfma_kernel(const float* __restrict__ uv, int K, int E, int S,
                                                       const float* __restrict__ gamma, const float* __restrict__ beta,
                                                       float sqrt_s, bf16* __restrict__ out) {
#pragma clang fp contract(off)
  extern __shared__ float sm[];
  const int SP = S + 1, AP = K | 1, VS = 160;
  const int KP2 = (K + 1) & ~1;
  float* base = sm;                                            // [K][SP], later V [KP2][VS]
  float* A = sm + max(K * SP, KP2 * VS);                       // [K][AP]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 31, lh = lane >> 5;
  const long row0 = (long)blockIdx.x * K;
  const int ld = 2 * E + S;
  for (int idx = tid; idx < K * S; idx += 256) {
    const int j = idx / S, c = idx - j * S;
    base[j * SP + c] = uv[(row0 + j) * ld + 2 * E + c];
  }
  __syncthreads();
  // phase 2: 25 tiles over the 4 waves
  for (int tile = wave; tile < GAU_M_TILES * GAU_M_TILES; tile += 4) {
    const int ti = tile / GAU_M_TILES, tj = tile - ti * GAU_M_TILES;
    const int m = ti * 32 + li, n = tj * 32 + li;
    floatx16 acc = {};
    for (int ks = 0; ks < S; ks += 2) {
      const int kk = ks + lh;
      const float qa = m < K ? __fadd_rn(__fmul_rn(base[m * SP + kk], gamma[kk]), beta[kk]) : 0.f;
      const float kb = n < K ? __fadd_rn(__fmul_rn(base[n * SP + kk], gamma[S + kk]), beta[S + kk]) : 0.f;
      acc = mfma_f32x2(qa, kb, acc);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int mm = ti * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
      if (mm < K && n < K) {
        const float x = fmaxf(acc[r] / sqrt_s, 0.f);
        A[mm * AP + n] = x * x;
      }
    }
  }
  __syncthreads();
  // phase 3: rounds of 128 v columns
  float* V = base;
  for (int e0 = 0; e0 < E; e0 += 128) {
    for (int idx = tid; idx < KP2 * 128; idx += 256) {
      const int j = idx >> 7, c = idx & 127;
      V[j * VS + c] = j < K ? uv[(row0 + j) * ld + E + e0 + c] : 0.f;
    }
    __syncthreads();
    for (int tile = wave; tile < GAU_M_TILES * 4; tile += 4) {
      const int ti = tile >> 2, tn = tile & 3;
      const int m = ti * 32 + li;
      floatx16 acc = {};
      for (int ks = 0; ks < KP2; ks += 2) {
        const int kk = ks + lh;
        const float a = (m < K && kk < K) ? A[m * AP + kk] : 0.f;
        acc = mfma_f32x2(a, V[kk * VS + tn * 32 + li], acc);
      }
      const int col = e0 + tn * 32 + li;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int mm = ti * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (mm < K) out[(row0 + mm) * E + col] = (bf16)(uv[(row0 + mm) * ld + col] * acc[r]);
      }
    }
    __syncthreads();
  }
}

// one wave per (inst, k): logits row [x bins | y bins] (f32, row stride ld)
__global__ void __launch_bounds__(256) simcc_decode_kernel(const float* __restrict__ logits, long ld, int WX, int WY,
                                                           float split, long rows, float* __restrict__ lv) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float* p = logits + row * ld;
  float mx[2];
  int ix[2];
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    const int n = a ? WY : WX, off = a ? WX : 0;
    float best = -INFINITY;
    int bi = 0x7fffffff;
    for (int c = lane; c < n; c += 64) {
      const float v = p[off + c];
      if (v > best) { best = v; bi = c; }  // strictly greater: the first index per lane
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      const float ob = __shfl_xor(best, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
    }
    mx[a] = best;
    ix[a] = bi;
  }
  if (lane == 0) {
    const float val = fminf(mx[0], mx[1]);  // max_val_x[mask] = max_val_y[mask] where x > y
    float lx = (float)ix[0], ly = (float)ix[1];
    if (val <= 0.f) { lx = -1.f; ly = -1.f; }
    lv[row * 3 + 0] = lx / split;
    lv[row * 3 + 1] = ly / split;
    lv[row * 3 + 2] = val;
  }
}

using vge::PoseInst;

__constant__ int c_body18[18] = {0, 17, 6, 8, 10, 5, 7, 9, 12, 14, 16, 11, 13, 15, 2, 1, 4, 3};

// inst_of_frame [F][2]: pose instance of person 0 and of person 1 (-1 when the frame has < 2 persons)
__global__ void __launch_bounds__(128) kp120_kernel(const float* __restrict__ lv, const PoseInst* __restrict__ inst,
                                                    const int* __restrict__ inst_of_frame, int F, int K, int in_w,
                                                    int in_h, int H, int W, float* __restrict__ out) {
  const int f = blockIdx.x, e = threadIdx.x;
  if (f >= F || e >= 120) return;
  const int j = e >> 1, xy = e & 1;
  int person = 0, wb;
  if (j < 18) {
    wb = c_body18[j];
  } else if (j < 39) {
    wb = 91 + (j - 18);
  } else if (inst_of_frame[2 * f + 1] >= 0) {
    person = 1;
    wb = 91 + (j - 39);
  } else {
    wb = 112 + (j - 39);
  }
  const int ii = inst_of_frame[2 * f + person];
  const PoseInst P = inst[ii];
  const double in = xy ? (double)in_h : (double)in_w, sc = xy ? (double)P.sh : (double)P.sw;
  const double ce = xy ? (double)P.cy : (double)P.cx;
  auto coord = [&](int k) -> double { return (double)lv[((long)ii * K + k) * 3 + xy] / in * sc + ce - sc / 2.0; };
  double c, s;
  if (wb == 17) {  // neck: mean of the shoulders; score 1 if both > 0.3 else 0
    c = (coord(5) + coord(6)) / 2.0;
    const double s5 = lv[((long)ii * K + 5) * 3 + 2], s6 = lv[((long)ii * K + 6) * 3 + 2];
    s = (s5 > 0.3 && s6 > 0.3) ? 1.0 : 0.0;
  } else {
    c = coord(wb);
    s = lv[((long)ii * K + wb) * 3 + 2];
  }
  c /= xy ? (double)H : (double)W;
  // dwpose_init.py:45-59: the body rows are copied before `candidate[subset < 0.3] = -1`, so only hand points
  // are masked
  out[(long)f * 120 + e] = (j >= 18 && s < 0.3) ? -1.0f : (float)c;
}

// ------------------------------------------------------------------------------------ YOLOX decode + NMS
// onnxdet.demo_postprocess + xyxy / ratio + score = sigmoid(obj) * sigmoid(cls0), then the part of the class-aware
// greedy NMS (+1-pixel IoU, keep if ovr <= 0.45) and the score > 0.3 person filter that can reach DWPose: person 0
// = the best-scoring anchor above 0.3, person 1 = the best one above 0.3 that person 0 does not suppress.  Ties ->
// lowest anchor index.  One workgroup per frame.
struct DetBox {
  float x0, y0, x1, y1, score;
};

__device__ __forceinline__ DetBox det_anchor(const vge::DetLevel& L0, const vge::DetLevel& L1, const vge::DetLevel& L2,
                                             int f, int a, float ratio) {
#pragma clang fp contract(off)
  const vge::DetLevel* L = &L0;
  int i = a;
  const int a0 = L0.grid * L0.grid, a1 = L1.grid * L1.grid;
  if (i >= a0) {
    i -= a0;
    L = &L1;
    if (i >= a1) {
      i -= a1;
      L = &L2;
    }
  }
  const int g = L->grid;
  const float* o = L->out + ((long)f * g * g + i) * 8;
  const int gy = i / g, gx = i - gy * g;
  const double st = (double)L->stride;
  const float cx = (float)(((double)o[0] + gx) * st), cy = (float)(((double)o[1] + gy) * st);
  const float w = (float)((double)expf(o[2]) * st), h = (float)((double)expf(o[3]) * st);
  DetBox b;
  b.x0 = (cx - w / 2.0f) / ratio;
  b.y0 = (cy - h / 2.0f) / ratio;
  b.x1 = (cx + w / 2.0f) / ratio;
  b.y1 = (cy + h / 2.0f) / ratio;
  const float so = 1.0f / (1.0f + expf(-o[4])), sc = 1.0f / (1.0f + expf(-o[5]));
  b.score = so * sc;
  return b;
}

__device__ __forceinline__ float iou_plus1(const DetBox& a, const DetBox& b) {
#pragma clang fp contract(off)
  const float area_a = (a.x1 - a.x0 + 1.0f) * (a.y1 - a.y0 + 1.0f);
  const float area_b = (b.x1 - b.x0 + 1.0f) * (b.y1 - b.y0 + 1.0f);
  const float w = fmaxf(0.0f, fminf(a.x1, b.x1) - fmaxf(a.x0, b.x0) + 1.0f);
  const float h = fmaxf(0.0f, fminf(a.y1, b.y1) - fmaxf(a.y0, b.y0) + 1.0f);
  const float inter = w * h;
  return inter / (area_a + area_b - inter);
}

// block argmax of (score, -index) over anchors passing `ok`; 256 threads
template <class OK>
__device__ int block_argmax(const vge::DetLevel& L0, const vge::DetLevel& L1, const vge::DetLevel& L2, int f, int A,
                            float ratio, OK ok, float* s_best, int* s_idx) {
  float best = -INFINITY;
  int bi = 0x7fffffff;
  for (int a = threadIdx.x; a < A; a += blockDim.x) {
    const DetBox b = det_anchor(L0, L1, L2, f, a, ratio);
    if (b.score > 0.3f && ok(b, a) && (b.score > best)) {
      best = b.score;
      bi = a;
    }
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const float ob = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
  }
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    s_best[wave] = best;
    s_idx[wave] = bi;
  }
  __syncthreads();
  float b = s_best[0];
  int idx = s_idx[0];
  for (int w = 1; w < (int)(blockDim.x >> 6); ++w)
    if (s_best[w] > b || (s_best[w] == b && s_idx[w] < idx)) { b = s_best[w]; idx = s_idx[w]; }
  __syncthreads();
  return b > 0.3f ? idx : -1;
}

__global__ void __launch_bounds__(256) yolox_decode_nms_kernel(vge::DetLevel L0, vge::DetLevel L1, vge::DetLevel L2,
                                                               float ratio, float* __restrict__ boxes,
                                                               int* __restrict__ n_out, float* __restrict__ scores,
                                                               float* __restrict__ cand) {
  __shared__ float s_best[4];
  __shared__ int s_idx[4];
  const int f = blockIdx.x;
  const int A = L0.grid * L0.grid + L1.grid * L1.grid + L2.grid * L2.grid;
  if (cand)
    for (int a = threadIdx.x; a < A; a += blockDim.x) {
      const DetBox b = det_anchor(L0, L1, L2, f, a, ratio);
      float* c = cand + ((long)f * A + a) * 5;
      c[0] = b.x0; c[1] = b.y0; c[2] = b.x1; c[3] = b.y1; c[4] = b.score;
    }
  const int i0 = block_argmax(L0, L1, L2, f, A, ratio, [](const DetBox&, int) { return true; }, s_best, s_idx);
  int i1 = -1;
  if (i0 >= 0) {
    const DetBox k0 = det_anchor(L0, L1, L2, f, i0, ratio);
    i1 = block_argmax(L0, L1, L2, f, A, ratio,
                      [&](const DetBox& b, int a) { return a != i0 && iou_plus1(k0, b) <= 0.45f; }, s_best, s_idx);
  }
  if (threadIdx.x < 8) {
    const int p = threadIdx.x >> 2, c = threadIdx.x & 3;
    const int ii = p ? i1 : i0;
    float v = 0.f;
    if (ii >= 0) {
      const DetBox b = det_anchor(L0, L1, L2, f, ii, ratio);
      v = c == 0 ? b.x0 : c == 1 ? b.y0 : c == 2 ? b.x1 : b.y1;
    }
    boxes[(long)f * 8 + threadIdx.x] = v;
    if (scores && c == 0) scores[(long)f * 2 + p] = ii >= 0 ? det_anchor(L0, L1, L2, f, ii, ratio).score : 0.f;
  }
  if (threadIdx.x == 0) n_out[f] = i0 < 0 ? 0 : (i1 < 0 ? 1 : 2);
}

}  // namespace

namespace vge {

hipError_t launch_head_sn_t(const float* y, long ldy, int hw, int K, int Kp, float g, long n_rows, void* out,
                            hipStream_t s) {
  if (n_rows == 0) return hipSuccess;
  hipLaunchKernelGGL(head_sn_t_kernel, dim3((unsigned)((n_rows + 3) / 4)), dim3(256), 0, s, y, ldy, hw, K, Kp, g,
                     (float)(1.0 / std::sqrt((double)hw)), n_rows, static_cast<bf16*>(out));
  return hipGetLastError();
}

hipError_t launch_scalenorm_rows(const float* x, int D, float g, long rows, void* y, hipStream_t s) {
  if (rows == 0) return hipSuccess;
  hipLaunchKernelGGL(scalenorm_rows_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s, x, D, g,
                     (float)(1.0 / std::sqrt((double)D)), rows, static_cast<bf16*>(y));
  return hipGetLastError();
}

constexpr int GAU_KMAX = 136;

size_t gau_lds_bytes(int S) { return sizeof(float) * ((size_t)GAU_KMAX * (S + 1) + GAU_KMAX * (GAU_KMAX + 1) + 4 * S); }

size_t gau_mfma_lds_bytes(int K, int S) {
  const int KP2 = (K + 1) & ~1;
  return sizeof(float) * ((size_t)std::max(K * (S + 1), KP2 * 160) + (size_t)K * (K | 1));
}

hipError_t launch_gau_attn(const float* uv, int n_inst, int K, int E, int S, const float* gamma, const float* beta,
                           void* out, hipStream_t s) {
  if (n_inst == 0) return hipSuccess;
  static int use_valu = -1;  // VGE_GAU_VALU=1: the VALU kernel (A/B timing)
  if (use_valu < 0) {
    const char* e = getenv("VGE_GAU_VALU");
    use_valu = (e && atoi(e) == 1) ? 1 : 0;
  }
  const size_t mb = gau_mfma_lds_bytes(K, S);
  if (!use_valu && K <= GAU_M_TILES * 32 && S % 2 == 0 && E % 128 == 0 && mb <= 160 * 1024) {
    static LdsAttrOnce mattr;
    if (const hipError_t e = mattr(reinterpret_cast<const void*>(&gau_mfma_kernel), 160 * 1024); e != hipSuccess) return e;
    hipLaunchKernelGGL(gau_mfma_kernel, dim3(n_inst), dim3(256), mb, s, uv, K, E, S, gamma, beta,
                       (float)std::sqrt((double)S), static_cast<bf16*>(out));
    return hipGetLastError();
  }
  const size_t bytes = gau_lds_bytes(S);
  static LdsAttrOnce attr;
  if (const hipError_t e = attr(reinterpret_cast<const void*>(&gau_attn_kernel<GAU_KMAX>), 160 * 1024); e != hipSuccess) return e;
  hipLaunchKernelGGL(gau_attn_kernel<GAU_KMAX>, dim3(n_inst), dim3(256), bytes, s, uv, K, E, S, gamma, beta,
                     (float)std::sqrt((double)S), static_cast<bf16*>(out));
  return hipGetLastError();
}

hipError_t launch_simcc_decode(const float* logits, long ld, int WX, int WY, float split, long rows, float* lv,
                               hipStream_t s) {
  if (rows == 0) return hipSuccess;
  hipLaunchKernelGGL(simcc_decode_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s, logits, ld, WX, WY, split,
                     rows, lv);
  return hipGetLastError();
}

hipError_t launch_yolox_decode_nms(DetLevel l0, DetLevel l1, DetLevel l2, int F, float ratio, float* boxes, int* n_out,
                                   float* scores, float* cand, hipStream_t s) {
  if (F == 0) return hipSuccess;
  hipLaunchKernelGGL(yolox_decode_nms_kernel, dim3(F), dim3(256), 0, s, l0, l1, l2, ratio, boxes, n_out, scores, cand);
  return hipGetLastError();
}

hipError_t launch_kp120(const float* lv, const void* inst, const int* inst_of_frame, int F, int K, int in_w, int in_h,
                        int H, int W, float* out, hipStream_t s) {
  if (F == 0) return hipSuccess;
  hipLaunchKernelGGL(kp120_kernel, dim3(F), dim3(128), 0, s, lv, static_cast<const PoseInst*>(inst), inst_of_frame, F,
                     K, in_w, in_h, H, W, out);
  return hipGetLastError();
}

}  // namespace vge
