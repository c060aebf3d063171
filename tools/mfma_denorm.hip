// Calibration check (not product code): does v_mfma_f32_32x32x16_f16 keep fp16 subnormal inputs?
//   hipcc -O3 --offload-arch=gfx950 tools/mfma_denorm.hip -o tools/mfma_denorm.bin && ./tools/mfma_denorm.bin
#include <hip/hip_runtime.h>
#include <cstdio>
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
__global__ void k(float* out, float aval, float bval) {
  half8 a, b;
  for (int j = 0; j < 8; ++j) { a[j] = (_Float16)aval; b[j] = (_Float16)bval; }
  floatx16 c = {};
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  if (threadIdx.x == 0) out[0] = c[0];
}
int main() {
  float* d; hipMalloc(&d, 4);
  const float as[] = {1.0f, 0x1p-14f, 0x1p-20f, 0x1p-24f, 3.0f * 0x1p-24f};
  for (float a : as) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, a, 1.0f);
    float h; hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
    printf("a=%a (fp16 %s) b=1: sum over k=16 -> %a, expected %a\n", a, a < 0x1p-14f ? "subnormal" : "normal", h, 16 * a);
  }
  return 0;
}
