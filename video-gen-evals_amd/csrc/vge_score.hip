// AC / TC reductions and real-class centroid accumulation (gfx950).
//
//   centroid_accum_kernel  build_train_centroids_subset (utils.py:1018-1043): sums.index_add_(0, y, z),
//                          counts.index_add_ -- one thread per (class, dim) walks the windows in order, so the
//                          f32 sums are bit-identical to index_add_'s sequential accumulation.
//   centroid_final_kernel  normalize(sums / counts.clamp_min(1)), eps 1e-12.
//   tc_windows_kernel      eval.py:216-224 per-window term (mean consecutive L2 over frames 1..T).
//   score_videos_kernel    eval.py:226 (np.mean over a video's windows, float64) and eval.py:238-255
//                          (AC = || normalize(mean_w seq_embed) - centroid[label] ||_2, float32).
// Roofline: HBM-bound; per window the metrics read 33 x 256 x 4 + 1,024 B (0 B when fused into the
// encoder's embed_tc_kernel, which is the default path) and write 8 B.
#include "vge_common.h"

namespace {

__global__ void centroid_accum_kernel(const float* __restrict__ seq, const int* __restrict__ cls, int n, int C, int d,
                                      float* __restrict__ sums, float* __restrict__ counts) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= C * d) return;
  const int c = idx / d, j = idx % d;
  float s = sums[idx];
  float cnt = (j == 0) ? counts[c] : 0.f;
  for (int w = 0; w < n; ++w) {
    if (cls[w] == c) {
      s += seq[(size_t)w * d + j];
      if (j == 0) cnt += 1.0f;
    }
  }
  sums[idx] = s;
  if (j == 0) counts[c] = cnt;
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

hipError_t launch_centroid_accum(const float* seq, const int* cls, int n, int C, int d, float* sums, float* counts,
                                 hipStream_t s) {
  const int total = C * d;
  hipLaunchKernelGGL(centroid_accum_kernel, dim3((total + 255) / 256), dim3(256), 0, s, seq, cls, n, C, d, sums, counts);
  return hipGetLastError();
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
