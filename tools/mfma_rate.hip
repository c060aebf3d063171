// Calibration micro-benchmark (not product code): cycles per v_mfma_f32_32x32x16_f16 on one SIMD at 1 and 2
// waves per SIMD, operands in registers, the same 4-accumulator / 6-MFMA-per-step pattern the 3xfp16 encoder
// uses (acc.x chains two MFMAs per step).
//   hipcc -O3 --offload-arch=gfx950 tools/mfma_rate.hip -o /tmp/mfma_rate && /tmp/mfma_rate
#include <hip/hip_runtime.h>
#include <cstdio>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

__global__ void mfma_loop(float* out, long long* cyc, int iters) {
  half8 a0, a1, b0, b1, b2, b3;
  for (int j = 0; j < 8; ++j) {
    a0[j] = (_Float16)(threadIdx.x * 0.001f + j);
    a1[j] = (_Float16)(j * 0.5f);
    b0[j] = (_Float16)(j * 0.25f);
    b1[j] = (_Float16)(j * 0.125f);
    b2[j] = (_Float16)(j * 0.3f);
    b3[j] = (_Float16)(j * 0.7f);
  }
  floatx16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b0, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b1, c1, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, b0, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b2, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b3, c3, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, b2, c3, 0, 0, 0);
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  for (int r = 0; r < 16; ++r) s += c0[r] + c1[r] + c2[r] + c3[r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  const int iters = 20000, blocks = 256;
  float* out;
  long long* cyc;
  hipMalloc(&out, sizeof(float) * blocks * 512);
  hipMalloc(&cyc, sizeof(long long) * blocks);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int threads : {256, 512}) {
    hipLaunchKernelGGL(mfma_loop, dim3(blocks), dim3(threads), 0, 0, out, cyc, iters);
    hipEventRecord(e0);
    hipLaunchKernelGGL(mfma_loop, dim3(blocks), dim3(threads), 0, 0, out, cyc, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    long long c[blocks];
    hipMemcpy(c, cyc, sizeof(c), hipMemcpyDeviceToHost);
    double avg = 0;
    for (int b = 0; b < blocks; ++b) avg += c[b];
    avg /= blocks;
    const double mfma_per_simd = 6.0 * iters * (threads / 64) / 4.0;
    const double flops = 6.0 * iters * 32768.0 * (threads / 64) * blocks;
    printf("waves/SIMD %d: %.3f ms, %.1f TFLOP/s f16, s_memtime cycles/MFMA/SIMD %.2f, wall ns/MFMA/SIMD %.2f\n",
           threads / 256, ms, flops / (ms * 1e-3) / 1e12, avg / mfma_per_simd, ms * 1e6 / mfma_per_simd);
  }
  return 0;
}
