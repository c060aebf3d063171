// MFMA shape probe (gfx950): the split stream's inner loop -- A fragments (hi, lo) re-read from LDS every step, B
// fragments in registers, the three split products into one accumulator tile per 32 output columns -- on
// v_mfma_f32_32x32x16_f16 (SHAPE 0) vs v_mfma_f32_16x16x32_f16 (SHAPE 1, same rows x columns x k per step),
// 512 threads (2 waves per SIMD) per CU, random fp16 data.  Prints TFLOP/s and the in-kernel clock
// (s_memtime / s_memrealtime at 100 MHz).  Build: hipcc --offload-arch=gfx950 -O3 -o probe mfma_shape_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int ROWS = 128, XSB = 528;  // 4 row tiles of 32, LDS rows as in the conv kernel (256 + 8 pad fp16)

template <int SHAPE>
__global__ void __launch_bounds__(512, 1) probe(const half8* __restrict__ src, float* __restrict__ out, int iters,
                                                long long* __restrict__ clk) {
  __shared__ __attribute__((aligned(16))) char lds[2 * ROWS * XSB];
  const int tid = threadIdx.x, lane = tid & 63;
  for (int k = tid; k < 2 * ROWS * XSB / 16; k += 512)
    reinterpret_cast<half8*>(lds)[k] = src[(blockIdx.x * 977 + k) % 65536];
  __syncthreads();
  half8 bh[2], bl[2];
  for (int j = 0; j < 2; ++j) {
    bh[j] = src[(blockIdx.x * 131 + tid * 2 + j) % 65536];
    bl[j] = src[(blockIdx.x * 171 + tid * 2 + j + 7) % 65536] * (_Float16)0.0005f;
  }
  long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  float res = 0.f;
  if constexpr (SHAPE == 0) {
    floatx16 acc[4] = {};
    const int i = lane & 31, h = lane >> 5;
    for (int it = 0; it < iters; it += 2) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {  // (static B register index)
        const int c = (it + s) & 15;  // 16 k-chunks of 16 per 256-wide row
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const char* p = lds + (t * 32 + i) * XSB + c * 32 + h * 16;
          const half8 ah = *reinterpret_cast<const half8*>(p);
          const half8 al = *reinterpret_cast<const half8*>(p + ROWS * XSB);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh[s], acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl[s], acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh[s], acc[t], 0, 0, 0);
        }
      }
    }
    for (int t = 0; t < 4; ++t)
      for (int r = 0; r < 16; ++r) res += acc[t][r];
  } else {
    // the same 128 rows x 32 columns x 32 k per two steps: 8 row tiles x 2 column tiles of 16 x 16, k 32 per MFMA
    floatx4 acc[8][2] = {};
    const int i = lane & 15, q = lane >> 4;
    for (int it = 0; it < iters; it += 2) {
      const int c = (it >> 1) & 7;  // 8 k-chunks of 32
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const char* p = lds + (t * 16 + i) * XSB + c * 64 + q * 16;
        const half8 ah = *reinterpret_cast<const half8*>(p);
        const half8 al = *reinterpret_cast<const half8*>(p + ROWS * XSB);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          acc[t][u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh[u], acc[t][u], 0, 0, 0);
          acc[t][u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl[u], acc[t][u], 0, 0, 0);
          acc[t][u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh[u], acc[t][u], 0, 0, 0);
        }
      }
    }
    for (int t = 0; t < 8; ++t)
      for (int u = 0; u < 2; ++u)
        for (int r = 0; r < 4; ++r) res += acc[t][u][r];
  }
  long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * 512 + tid] = res;  // keeps the work live
  if (tid == 0) {
    clk[blockIdx.x * 2] = t1 - t0;
    clk[blockIdx.x * 2 + 1] = r1 - r0;
  }
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 200000, reps = argc > 2 ? atoi(argv[2]) : 5;
  hipDeviceProp_t pr;
  if (hipGetDeviceProperties(&pr, 0) != hipSuccess) return 1;
  const int G = pr.multiProcessorCount;
  std::vector<_Float16> h(65536 * 8);
  srand(1);
  for (auto& x : h) x = (_Float16)((rand() / (float)RAND_MAX) * 2.f - 1.f);
  half8* d_src; float* d_out; long long* d_clk;
  if (hipMalloc(&d_src, h.size() * 2) || hipMalloc(&d_out, (size_t)G * 512 * 4) || hipMalloc(&d_clk, (size_t)G * 16))
    return 1;
  if (hipMemcpy(d_src, h.data(), h.size() * 2, hipMemcpyHostToDevice)) return 1;
  std::vector<long long> clk(G * 2);
  for (int rep = 0; rep < reps; ++rep)
    for (int shape = 0; shape < 2; ++shape) {
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      hipEventRecord(e0);
      if (shape == 0) hipLaunchKernelGGL(probe<0>, dim3(G), dim3(512), 0, 0, d_src, d_out, iters, d_clk);
      else hipLaunchKernelGGL(probe<1>, dim3(G), dim3(512), 0, 0, d_src, d_out, iters, d_clk);
      hipEventRecord(e1);
      if (hipEventSynchronize(e1) != hipSuccess) return 2;
      float ms = 0.f;
      hipEventElapsedTime(&ms, e0, e1);
      hipMemcpy(clk.data(), d_clk, G * 16, hipMemcpyDeviceToHost);
      double ghz = 0;
      for (int b = 0; b < G; ++b) ghz += (double)clk[2 * b] / (clk[2 * b + 1] * 10.0);  // memrealtime = 100 MHz
      ghz /= G;
      // per step and wave: 4 row tiles x 32 x 32 x 16 x 2 flop x 3 products; 8 waves per CU
      const double flop = (double)G * 8 * iters * 4.0 * 32 * 32 * 16 * 2 * 3;
      printf("{\"shape\": \"%s\", \"rep\": %d, \"ms\": %.3f, \"tflops\": %.1f, \"ghz\": %.3f}\n",
             shape ? "16x16x32" : "32x32x16", rep, ms, flop / ms / 1e9, ghz);
      hipEventDestroy(e0);
      hipEventDestroy(e1);
    }
  return 0;
}
