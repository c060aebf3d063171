// Shared device helpers for the gfx950 kernels of libvge (CDNA4: wave64, f32-input MFMA).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx2 __attribute__((ext_vector_type(2)));

#define VGE_WAVE 64
#define VGE_D 256            // d_model
#define VGE_T 32             // clip_len
#define VGE_TOK 33           // clip_len + CLS
#define VGE_FD 2596          // feats row width
#define VGE_LDX 260          // LDS row stride (floats) of a 256-wide activation panel: 16-B shift per
                             // row keeps ds_read_b128 fragment reads conflict-free (see vge_encoder.hip)

// ---- wave64 reductions (all lanes receive the result) ---------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
// sum over the 16 lanes that share (lane >> 4): xor offsets 1..8 stay inside a 16-lane group
__device__ __forceinline__ float group16_sum(float v) {
#pragma unroll
  for (int o = 8; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// exact-erf GELU (nn.GELU() default; ATen: x * 0.5 * (1 + erf(x * M_SQRT1_2)))
#if defined(VGE_ABL) && (VGE_ABL & 16)
__device__ __forceinline__ float gelu_erf(float x) { return x; }
#else
__device__ __forceinline__ float gelu_erf(float x) { return x * 0.5f * (1.0f + erff(x * 0.70710678118654752440f)); }
#endif

// v_mfma_f32_16x16x4_f32: exact f32 (bitwise an fmaf chain over k).  Lane l supplies
// A[i = l&15][k = l>>4] and B[k = l>>4][j = l&15]; C/D: col = l&15, row = (l>>4)*4 + r.
__device__ __forceinline__ floatx4 mfma16x16x4(float a, float b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// 16-B global -> LDS DMA (global_load_lds_dwordx4).  The LDS destination of a wave-instruction is
// the wave-uniform `lds_wave_base` + lane*16; the global source is per lane.
__device__ __forceinline__ void glds16(const void* gsrc, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)gsrc,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

__device__ __forceinline__ void vmcnt0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
template <int N>
__device__ __forceinline__ void vmcnt() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
// workgroup barrier that does NOT drain vector-memory (LDS-DMA in flight survives it): own LDS reads
// retired first (WAR safety for the ring slot being refilled), then s_barrier.  The "memory" clobber
// keeps the compiler from moving loads/stores across it.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
