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

// exact-erf GELU (nn.GELU() default; ATen: x * 0.5 * (1 + erf(x * M_SQRT1_2))), branch free.
// erf(a), a = |z|: a + a q(a^2) for a < 1, 1 - exp(-p(a)) for a >= 1, with the minimax coefficients of the
// ROCm device library's erff (ocml) but both pieces evaluated and selected (no divergent branches), and
// exp via v_exp_f32.  Max |error| vs erf in double 7.4e-8 over [-8, 8] (tools: host check in
// tests/test_lib_abi.py::test_erf_branch_free_accuracy); the packed form runs two values per v_pk_fma_f32.
__device__ __forceinline__ floatx2 erf2(floatx2 z) {
  const floatx2 a = __builtin_elementwise_abs(z);
  const floatx2 s = a * a;
  floatx2 q = __builtin_elementwise_fma(s, (floatx2)(-0x1.268bc20000000p-11f), (floatx2)(0x1.4208280000000p-8f));
  q = __builtin_elementwise_fma(s, q, (floatx2)(-0x1.b593700000000p-6f));
  q = __builtin_elementwise_fma(s, q, (floatx2)(0x1.ce077c0000000p-4f));
  q = __builtin_elementwise_fma(s, q, (floatx2)(-0x1.8126600000000p-2f));
  q = __builtin_elementwise_fma(s, q, (floatx2)(0x1.06eba00000000p-3f));
  const floatx2 rs = __builtin_elementwise_fma(a, q, a);
  floatx2 p = __builtin_elementwise_fma(a, (floatx2)(0x1.1d31560000000p-16f), (floatx2)(-0x1.8d12900000000p-12f));
  p = __builtin_elementwise_fma(a, p, (floatx2)(0x1.f9a6d20000000p-9f));
  p = __builtin_elementwise_fma(a, p, (floatx2)(-0x1.8c31640000000p-6f));
  p = __builtin_elementwise_fma(a, p, (floatx2)(0x1.b4e9c80000000p-4f));
  p = __builtin_elementwise_fma(a, p, (floatx2)(0x1.4515fa0000000p-1f));
  p = __builtin_elementwise_fma(a, p, (floatx2)(0x1.078e500000000p-3f));
  p = __builtin_elementwise_fma(a, p, a);
  const floatx2 l = p * (floatx2)(-1.44269504f);
  floatx2 t;
  t.x = __builtin_amdgcn_exp2f(l.x);
  t.y = __builtin_amdgcn_exp2f(l.y);
  const floatx2 rb = 1.0f - t;
  floatx2 r;
  r.x = a.x < 1.0f ? rs.x : rb.x;
  r.y = a.y < 1.0f ? rs.y : rb.y;
  return __builtin_elementwise_copysign(r, z);
}
#if defined(VGE_ABL) && (VGE_ABL & 16)
__device__ __forceinline__ floatx2 gelu2(floatx2 x) { return x; }
__device__ __forceinline__ float gelu_erf(float x) { return x; }
#else
__device__ __forceinline__ floatx2 gelu2(floatx2 x) {
  const floatx2 hx = x * 0.5f;
  return __builtin_elementwise_fma(hx, erf2(x * 0.70710678118654752440f), hx);
}
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
