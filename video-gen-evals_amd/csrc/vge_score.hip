// AC / TC reductions and real-class centroid accumulation (gfx950).
//
//   centroid_partial_kernel + centroid_combine_kernel
//                          build_train_centroids_subset (utils.py:1018-1043): sums.index_add_(0, y, z),
//                          counts.index_add_, as a deterministic segmented reduction: the windows are cut into
//                          segments of CENT_SEG (a function of n only); one workgroup per (segment, 64 columns,
//                          block of 64 classes) walks its windows in order, lane j owning column j of every
//                          class row in LDS (runs of one class summed in a register first; no atomics, no
//                          races), then the segment partials are added in a fixed order.  Same result for any grid / device; the order
//                          of the f32 additions differs from a sequential index_add_ only by the segment
//                          split (a few ulps of the sums, far inside the 2e-5 centroid tolerance).
//                          HBM-bound: reads n x d x 4 B + 4n B once.
//   centroid_final_kernel  normalize(sums / counts.clamp_min(1)), eps 1e-12.
//   tc_windows_kernel      eval.py:216-224 per-window term (mean consecutive L2 over frames 1..T).
//   score_videos_kernel    eval.py:226 (np.mean over a video's windows, float64) and eval.py:238-255
//                          (AC = || normalize(mean_w seq_embed) - centroid[label] ||_2, float32).
// Roofline: HBM-bound; per window the metrics read 33 x 256 x 4 + 1,024 B (0 B when fused into the
// encoder's embed_tc_kernel, which is the default path) and write 8 B.
#include "vge_common.h"

namespace {

constexpr int CENT_SEG = 512;     // windows per segment (a function of nothing but n: the result is launch-independent)
constexpr int CENT_CB = 64;       // classes per workgroup

// grid (n_seg, ceil(d / 64), ceil(C / 64)), 4 waves; lane = column (64 per workgroup).  Wave q walks windows
// [q SEG/4, (q+1) SEG/4) of the segment in order: consecutive windows of one class (real-set windows come grouped by
// video and class) are summed in a register and flushed to the wave's own LDS row when the class changes; rows are
// loaded 32 ahead (one memory round trip per 32 windows).  Then the 4 wave partials are added in wave order.
// part [n_seg][C][d], pcnt [n_seg][C].
constexpr int CENT_QW = CENT_SEG / 4, CENT_B = 32;
__global__ void __launch_bounds__(256) centroid_partial_kernel(const float* __restrict__ seq,
                                                               const int* __restrict__ cls, int n, int C, int d,
                                                               float* __restrict__ part, float* __restrict__ pcnt) {
  __shared__ float acc[4][CENT_CB][64];
  __shared__ float cnt[4][CENT_CB];
  const int lane = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int seg = blockIdx.x, j = blockIdx.y * 64 + lane, c0 = blockIdx.z * CENT_CB;
  const int nc = min(CENT_CB, C - c0);
  for (int c = 0; c < nc; ++c) acc[q][c][lane] = 0.f;
  if (lane < nc) cnt[q][lane] = 0.f;
  const int w0 = seg * CENT_SEG + q * CENT_QW, w1 = min(n, w0 + CENT_QW);
  // the wave's 128 class ids, two per lane; read back as scalars with v_readlane (no LDS round trip per window)
  int yv[CENT_QW / 64];
#pragma unroll
  for (int h = 0; h < CENT_QW / 64; ++h) {
    const int k = h * 64 + lane;
    const int y = (w0 + k < w1) ? cls[w0 + k] - c0 : -1;
    yv[h] = (unsigned)y < (unsigned)nc ? y : -1;
  }
  __syncthreads();  // the zeroed LDS rows
  float run = 0.f, rcnt = 0.f;
  int cur = -1;
  auto load = [&](int b, float (&x)[CENT_B]) {
#pragma unroll
    for (int k = 0; k < CENT_B; ++k)
      x[k] = (w0 + b + k < w1 && j < d) ? seq[(size_t)(w0 + b + k) * d + j] : 0.f;
  };
  float xa[CENT_B], xb[CENT_B];
  load(0, xa);
#pragma unroll
  for (int b = 0; b < CENT_QW; b += 2 * CENT_B) {
    load(b + CENT_B, xb);  // rows past the segment read as 0 and carry class -1
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      float (&x)[CENT_B] = h ? xb : xa;
      const int bb = b + h * CENT_B;
      if (h == 1 && bb + CENT_B < CENT_QW) load(bb + CENT_B, xa);
#pragma unroll
      for (int k = 0; k < CENT_B; ++k) {
        const int y = __builtin_amdgcn_readlane(yv[(bb + k) >> 6], (bb + k) & 63);
        if (y != cur) {  // uniform: flush the finished run of class `cur`
          if (cur >= 0) {
            acc[q][cur][lane] += run;
            if (lane == 0) cnt[q][cur] += rcnt;
          }
          run = 0.f;
          rcnt = 0.f;
          cur = y;
        }
        run += x[k];
        rcnt += 1.0f;
      }
    }
  }
  if (cur >= 0) {
    acc[q][cur][lane] += run;
    if (lane == 0) cnt[q][cur] += rcnt;
  }
  __syncthreads();
  for (int c = q; c < nc; c += 4)
    if (j < d) part[((size_t)seg * C + c0 + c) * d + j] = ((acc[0][c][lane] + acc[1][c][lane]) + acc[2][c][lane]) +
                                                          acc[3][c][lane];
  if (blockIdx.y == 0 && q == 0 && lane < nc)
    pcnt[(size_t)seg * C + c0 + lane] = ((cnt[0][lane] + cnt[1][lane]) + cnt[2][lane]) + cnt[3][lane];
}

// sums[e] += sum over segments of part[g][e] (e over C d sums then C counts): 64 elements per workgroup, wave q
// adds segments q, q + 4, ... (8 loads in flight), then the 4 wave partials in wave order.
__global__ void __launch_bounds__(256) centroid_combine_kernel(const float* __restrict__ part,
                                                               const float* __restrict__ pcnt, int n_seg, int C,
                                                               int d, float* __restrict__ sums,
                                                               float* __restrict__ counts) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int e = blockIdx.x * 64 + lane, n_sum = C * d;
  const bool is_cnt = e >= n_sum;
  const float* src = is_cnt ? pcnt + (e - n_sum) : part + e;
  const size_t stride = is_cnt ? (size_t)C : (size_t)n_sum;
  float s = 0.f;
  if (e < n_sum + C) {
    for (int g = q; g < n_seg; g += 32) {
      float x[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) x[k] = (g + 4 * k < n_seg) ? src[(size_t)(g + 4 * k) * stride] : 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) s += x[k];
    }
  }
  red[q][lane] = s;
  __syncthreads();
  if (q == 0 && e < n_sum + C) {
    const float t = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
    if (is_cnt) counts[e - n_sum] += t;
    else sums[e] += t;
  }
}

__global__ void centroid_final_kernel(const float* __restrict__ sums, const float* __restrict__ counts, int C, int d,
                                      float* __restrict__ cent) {
  // one wave per class; d <= 256 (4 values per lane)
  const int c = blockIdx.x;
  const int lane = threadIdx.x;
  const float cnt = fmaxf(counts[c], 1.0f);
  float v[4];
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int j = lane + 64 * k;
    v[k] = (j < d) ? sums[(size_t)c * d + j] / cnt : 0.f;
    ss += v[k] * v[k];
  }
  const float n = fmaxf(sqrtf(wave_sum(ss)), 1e-12f);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int j = lane + 64 * k;
    if (j < d) cent[(size_t)c * d + j] = v[k] / n;
  }
}

__global__ void tc_windows_kernel(const float* __restrict__ fe, int B, int T1, int d, float* __restrict__ tc) {
  const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (w >= B) return;
  float sum = 0.f;
  for (int t = 2; t < T1; ++t) {
    float ss = 0.f;
    for (int j = lane; j < d; j += 64) {
      const float x = fe[((size_t)w * T1 + t) * d + j] - fe[((size_t)w * T1 + t - 1) * d + j];
      ss += x * x;
    }
    sum += sqrtf(wave_sum(ss));
  }
  if (lane == 0) tc[w] = (T1 >= 3) ? sum / (float)(T1 - 2) : nanf("");
}

__global__ void score_videos_kernel(const float* __restrict__ seq, const float* __restrict__ tcw,
                                    const int* __restrict__ first, const int* __restrict__ vcls,
                                    const float* __restrict__ cent, int V, int d, float* __restrict__ ac,
                                    double* __restrict__ tc) {
  const int v = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (v >= V) return;
  const int w0 = first[v], w1 = first[v + 1];
  const int n = w1 - w0;
  // TC: float64 mean of the per-window floats (np.mean of python floats)
  double ts = 0.0;
  for (int w = w0 + lane; w < w1; w += 64) ts += (double)tcw[w];
  ts = wave_sum_d(ts);
  if (lane == 0) tc[v] = (n > 0) ? ts / (double)n : nan("");
  // AC: torch.stack(embeds).mean(0) in float32, F.normalize, ||z - c||_2
  const int c = vcls[v];
  if (c < 0 || n <= 0) {
    if (lane == 0) ac[v] = nanf("");
    return;
  }
  float z[4];
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int j = lane + 64 * k;
    float s = 0.f;
    if (j < d)
      for (int w = w0; w < w1; ++w) s += seq[(size_t)w * d + j];
    z[k] = s / (float)n;
    ss += z[k] * z[k];
  }
  const float nz = fmaxf(sqrtf(wave_sum(ss)), 1e-12f);
  float dd = 0.f;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int j = lane + 64 * k;
    if (j < d) {
      const float x = z[k] / nz - cent[(size_t)c * d + j];
      dd += x * x;
    }
  }
  dd = wave_sum(dd);
  if (lane == 0) ac[v] = sqrtf(dd);
}

}  // namespace

namespace vge {

// d <= 256.  The segment partials live in a stream-ordered scratch allocation (n_seg x (C d + C) floats).
hipError_t launch_centroid_accum(const float* seq, const int* cls, int n, int C, int d, float* sums, float* counts,
                                 hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const int n_seg = (n + CENT_SEG - 1) / CENT_SEG;
  float* part = nullptr;
  const size_t nf = (size_t)n_seg * ((size_t)C * d + C);
  hipError_t e = hipMallocAsync(reinterpret_cast<void**>(&part), nf * sizeof(float), s);
  if (e != hipSuccess) return e;
  float* pcnt = part + (size_t)n_seg * C * d;
  hipLaunchKernelGGL(centroid_partial_kernel, dim3(n_seg, (d + 63) / 64, (C + CENT_CB - 1) / CENT_CB), dim3(256), 0,
                     s, seq, cls, n, C, d, part, pcnt);
  const int total = C * d + C;
  hipLaunchKernelGGL(centroid_combine_kernel, dim3((total + 63) / 64), dim3(256), 0, s, part, pcnt, n_seg, C, d, sums,
                     counts);
  e = hipGetLastError();
  const hipError_t f = hipFreeAsync(part, s);
  return e != hipSuccess ? e : f;
}

hipError_t launch_centroid_final(const float* sums, const float* counts, int C, int d, float* cent, hipStream_t s) {
  hipLaunchKernelGGL(centroid_final_kernel, dim3(C), dim3(64), 0, s, sums, counts, C, d, cent);
  return hipGetLastError();
}

hipError_t launch_tc_windows(const float* fe, int B, int T1, int d, float* tc, hipStream_t s) {
  hipLaunchKernelGGL(tc_windows_kernel, dim3((B + 3) / 4), dim3(256), 0, s, fe, B, T1, d, tc);
  return hipGetLastError();
}

hipError_t launch_score_videos(const float* seq, const float* tcw, const int* first, const int* vcls, const float* cent,
                               int V, int d, float* ac, double* tc, hipStream_t s) {
  hipLaunchKernelGGL(score_videos_kernel, dim3((V + 3) / 4), dim3(256), 0, s, seq, tcw, first, vcls, cent, V, d, ac, tc);
  return hipGetLastError();
}

}  // namespace vge
