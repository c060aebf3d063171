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
#define VGE_FD_NOKP 2356     // feats row width of the keypoint-less layout (keypoint_dir None)
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
// ---- DPP reductions (no LDS round trips): the result is valid in the LAST lane of the group only ------
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ float dpp_f(float old, float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, old), __builtin_bit_cast(int, x),
                                                               CTRL, ROW_MASK, 0xf, false));
}
#define VGE_DPP_QP_XOR1 0xB1        // quad_perm [1,0,3,2]
#define VGE_DPP_QP_XOR2 0x4E        // quad_perm [2,3,0,1]
#define VGE_DPP_ROW_HALF_MIRROR 0x141
#define VGE_DPP_ROW_MIRROR 0x140
#define VGE_DPP_ROW_BCAST15 0x142
#define VGE_DPP_ROW_BCAST31 0x143
// sum over each 16-lane row, in every lane of the row
__device__ __forceinline__ float row16_sum(float x) {
  x += dpp_f<VGE_DPP_QP_XOR1, 0xf>(0.f, x);
  x += dpp_f<VGE_DPP_QP_XOR2, 0xf>(0.f, x);
  x += dpp_f<VGE_DPP_ROW_HALF_MIRROR, 0xf>(0.f, x);
  x += dpp_f<VGE_DPP_ROW_MIRROR, 0xf>(0.f, x);
  return x;
}
__device__ __forceinline__ float row16_max(float x) {
  x = fmaxf(x, dpp_f<VGE_DPP_QP_XOR1, 0xf>(x, x));
  x = fmaxf(x, dpp_f<VGE_DPP_QP_XOR2, 0xf>(x, x));
  x = fmaxf(x, dpp_f<VGE_DPP_ROW_HALF_MIRROR, 0xf>(x, x));
  x = fmaxf(x, dpp_f<VGE_DPP_ROW_MIRROR, 0xf>(x, x));
  return x;
}
// sum over each 32-lane half: valid in lanes 31 and 63
__device__ __forceinline__ float half_sum_last(float x) {
  x = row16_sum(x);
  return x + dpp_f<VGE_DPP_ROW_BCAST15, 0xa>(0.f, x);
}
// sum / max over the wave: valid in lane 63
__device__ __forceinline__ float wave_sum_last(float x) {
  x = half_sum_last(x);
  return x + dpp_f<VGE_DPP_ROW_BCAST31, 0xc>(0.f, x);
}
__device__ __forceinline__ float wave_max_last(float x) {
  x = row16_max(x);
  x = fmaxf(x, dpp_f<VGE_DPP_ROW_BCAST15, 0xa>(x, x));
  return fmaxf(x, dpp_f<VGE_DPP_ROW_BCAST31, 0xc>(x, x));
}
// wave max broadcast to every lane (lane 63's value via readlane)
__device__ __forceinline__ float wave_max_all(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, wave_max_last(x)), 63));
}

// sum over the 16 lanes that share (lane >> 4): xor offsets 1..8 stay inside a 16-lane group
__device__ __forceinline__ float group16_sum(float v) {
#pragma unroll
  for (int o = 8; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// exact-erf GELU (nn.GELU() default; ATen: x * 0.5 * (1 + erf(x * M_SQRT1_2))).  gelu_erf: scalar, ocml
// erff (f32 path).  gelu2_many: branch free and packed (two values per v_pk_fma_f32): erf(a), a = |z|, is
// a + a q(a^2) for a < 1 and 1 - exp(-p(a)) for a >= 1 with the minimax coefficients of ocml's erff, both
// pieces evaluated and selected, exp via v_exp_f32.  Max |error| vs erf in double 7.4e-8 over [-8, 8]
// (host restatement checked in tests/test_lib_abi.py::test_erf_branch_free_accuracy).
#if defined(VGE_ABL) && (VGE_ABL & 16)
__device__ __forceinline__ float gelu_erf(float x) { return x; }
#else
__device__ __forceinline__ float gelu_erf(float x) { return x * 0.5f * (1.0f + erff(x * 0.70710678118654752440f)); }
#endif
// K pairs at once, written stage by stage so K independent dependency chains interleave (one pair's
// chain alone is ~20 dependent packed ops with hazard nops between them)
template <int K>
__device__ __forceinline__ void gelu2_many(floatx2 (&y)[K]) {
#if !(defined(VGE_ABL) && (VGE_ABL & 16))
  floatx2 z[K], a[K], s[K], q[K], p[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    z[k] = y[k] * 0.70710678118654752440f;
    a[k] = __builtin_elementwise_abs(z[k]);
    s[k] = a[k] * a[k];
  }
#define VGE_STAGE(dst, x, c1, c0)                                                                  \
  _Pragma("unroll") for (int k = 0; k < K; ++k) dst[k] = __builtin_elementwise_fma(x[k], c1, c0);
  VGE_STAGE(q, s, (floatx2)(-0x1.268bc2p-11f), (floatx2)(0x1.420828p-8f))
  VGE_STAGE(p, a, (floatx2)(0x1.1d3156p-16f), (floatx2)(-0x1.8d129p-12f))
#undef VGE_STAGE
#pragma unroll
  for (int k = 0; k < K; ++k) {
    q[k] = __builtin_elementwise_fma(s[k], q[k], (floatx2)(-0x1.b5937p-6f));
    p[k] = __builtin_elementwise_fma(a[k], p[k], (floatx2)(0x1.f9a6d2p-9f));
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    q[k] = __builtin_elementwise_fma(s[k], q[k], (floatx2)(0x1.ce077cp-4f));
    p[k] = __builtin_elementwise_fma(a[k], p[k], (floatx2)(-0x1.8c3164p-6f));
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    q[k] = __builtin_elementwise_fma(s[k], q[k], (floatx2)(-0x1.81266p-2f));
    p[k] = __builtin_elementwise_fma(a[k], p[k], (floatx2)(0x1.b4e9c8p-4f));
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    q[k] = __builtin_elementwise_fma(s[k], q[k], (floatx2)(0x1.06eba0p-3f));
    p[k] = __builtin_elementwise_fma(a[k], p[k], (floatx2)(0x1.4515fap-1f));
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    q[k] = __builtin_elementwise_fma(a[k], q[k], a[k]);  // erf(a), a < 1
    p[k] = __builtin_elementwise_fma(a[k], p[k], (floatx2)(0x1.078e5p-3f));
  }
#pragma unroll
  for (int k = 0; k < K; ++k) p[k] = __builtin_elementwise_fma(a[k], p[k], a[k]) * (floatx2)(-1.44269504f);
#pragma unroll
  for (int k = 0; k < K; ++k) {
    p[k].x = __builtin_amdgcn_exp2f(p[k].x);
    p[k].y = __builtin_amdgcn_exp2f(p[k].y);
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    floatx2 r;
    r.x = a[k].x < 1.0f ? q[k].x : 1.0f - p[k].x;
    r.y = a[k].y < 1.0f ? q[k].y : 1.0f - p[k].y;
    const floatx2 hx = y[k] * 0.5f;
    y[k] = __builtin_elementwise_fma(hx, __builtin_elementwise_copysign(r, z[k]), hx);
  }
#endif
}

// GELU for the single-fp16 conv path (VGE_F16), whose operands are rounded to fp16 (2^-11) anyway: one exp2 and no
// branch pieces.  erf(|x| / sqrt 2) = 1 - 2^(-a P(a)), a = min(|x|, 4 sqrt 2), P of degree 5 (weighted least-squares
// fit of -log2(erfc(a / sqrt 2)) / a), and GELU(x) = 0.5 x + |x| (0.5 - 0.5 * 2^(-a P(a))), which is
// 0.5 x (1 + erf(x / sqrt 2)) for either sign.  Max |error| vs the exact GELU 4.8e-7 over [-10, 10] in f32
// (host restatement: tests/test_lib_abi.py::test_gelu_fast_accuracy); ~2/3 of gelu2_many's VALU slots.
template <int K>
__device__ __forceinline__ void gelu2_fast(floatx2 (&y)[K]) {
#if !(defined(VGE_ABL) && (VGE_ABL & 16))
  floatx2 a[K], p[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    a[k].x = fminf(fabsf(y[k].x), 0x1.6a09e6p+2f);
    a[k].y = fminf(fabsf(y[k].y), 0x1.6a09e6p+2f);
    p[k] = __builtin_elementwise_fma(a[k], (floatx2)(-0x1.f5fbdcp-16f), (floatx2)(0x1.83e48ap-11f));
  }
#pragma unroll
  for (int k = 0; k < K; ++k) p[k] = __builtin_elementwise_fma(a[k], p[k], (floatx2)(-0x1.05672ep-7f));
#pragma unroll
  for (int k = 0; k < K; ++k) p[k] = __builtin_elementwise_fma(a[k], p[k], (floatx2)(0x1.b42062p-5f));
#pragma unroll
  for (int k = 0; k < K; ++k) p[k] = __builtin_elementwise_fma(a[k], p[k], (floatx2)(0x1.d5ee02p-2f));
#pragma unroll
  for (int k = 0; k < K; ++k) p[k] = __builtin_elementwise_fma(a[k], p[k], (floatx2)(0x1.26b194p+0f)) * a[k];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    p[k].x = __builtin_amdgcn_exp2f(-p[k].x);
    p[k].y = __builtin_amdgcn_exp2f(-p[k].y);
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const floatx2 eh = __builtin_elementwise_fma(p[k], (floatx2)(-0.5f), (floatx2)(0.5f));
    const floatx2 hx = y[k] * 0.5f;
    y[k].x = fmaf(fabsf(y[k].x), eh.x, hx.x);
    y[k].y = fmaf(fabsf(y[k].y), eh.y, hx.y);
  }
#endif
}

// Scalar forms of gelu2_many / gelu2_fast (same operations, so the same results), for code that runs beside MFMA
// streams: packed f32 VALU (v_pk_fma_f32 ...) issued next to a busy matrix pipe costs ~22 cycles more than two scalar
// ops (MI355X_MICROARCH.md, filler price row); build such files with -fno-slp-vectorize so they stay scalar.
template <int K>
__device__ __forceinline__ void gelu_many_s(float (&y)[K]) {
#if !(defined(VGE_ABL) && (VGE_ABL & 16))
  float z[K], a[K], s[K], q[K], p[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    z[k] = y[k] * 0.70710678118654752440f;
    a[k] = fabsf(z[k]);
    s[k] = a[k] * a[k];
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    q[k] = fmaf(s[k], -0x1.268bc2p-11f, 0x1.420828p-8f);
    p[k] = fmaf(a[k], 0x1.1d3156p-16f, -0x1.8d129p-12f);
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    q[k] = fmaf(s[k], q[k], -0x1.b5937p-6f);
    p[k] = fmaf(a[k], p[k], 0x1.f9a6d2p-9f);
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    q[k] = fmaf(s[k], q[k], 0x1.ce077cp-4f);
    p[k] = fmaf(a[k], p[k], -0x1.8c3164p-6f);
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    q[k] = fmaf(s[k], q[k], -0x1.81266p-2f);
    p[k] = fmaf(a[k], p[k], 0x1.b4e9c8p-4f);
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    q[k] = fmaf(s[k], q[k], 0x1.06eba0p-3f);
    p[k] = fmaf(a[k], p[k], 0x1.4515fap-1f);
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    q[k] = fmaf(a[k], q[k], a[k]);  // erf(a), a < 1
    p[k] = fmaf(a[k], p[k], 0x1.078e5p-3f);
  }
#pragma unroll
  for (int k = 0; k < K; ++k) p[k] = __builtin_amdgcn_exp2f(fmaf(a[k], p[k], a[k]) * -1.44269504f);
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const float r = a[k] < 1.0f ? q[k] : 1.0f - p[k];
    const float hx = y[k] * 0.5f;
    y[k] = fmaf(hx, copysignf(r, z[k]), hx);
  }
#endif
}
template <int K>
__device__ __forceinline__ void gelu_fast_s(float (&y)[K]) {
#if !(defined(VGE_ABL) && (VGE_ABL & 16))
  float a[K], p[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    a[k] = fminf(fabsf(y[k]), 0x1.6a09e6p+2f);
    p[k] = fmaf(a[k], -0x1.f5fbdcp-16f, 0x1.83e48ap-11f);
  }
#pragma unroll
  for (int k = 0; k < K; ++k) p[k] = fmaf(a[k], p[k], -0x1.05672ep-7f);
#pragma unroll
  for (int k = 0; k < K; ++k) p[k] = fmaf(a[k], p[k], 0x1.b42062p-5f);
#pragma unroll
  for (int k = 0; k < K; ++k) p[k] = fmaf(a[k], p[k], 0x1.d5ee02p-2f);
#pragma unroll
  for (int k = 0; k < K; ++k) p[k] = fmaf(a[k], p[k], 0x1.26b194p+0f) * a[k];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const float eh = fmaf(__builtin_amdgcn_exp2f(-p[k]), -0.5f, 0.5f);
    y[k] = fmaf(fabsf(y[k]), eh, y[k] * 0.5f);
  }
#endif
}

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

// The same waits as builtins (gfx9 s_waitcnt simm16: vmcnt[3:0] | expcnt[6:4] | lgkmcnt[11:8] | vmcnt_hi[15:14]):
// unlike an asm statement, hipcc's waitcnt insertion sees them and knows what they retired, so it does not add a
// conservative lgkmcnt(0) before later uses of registers loaded earlier.
template <int N>
__device__ __forceinline__ void vmcnt_b() {
  __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | 0x70 | 0xF00);
}
__device__ __forceinline__ void lds_barrier_b() {
  asm volatile("" ::: "memory");  // the builtins are IntrNoMem: keep LDS / global_load_lds ops on their side
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
