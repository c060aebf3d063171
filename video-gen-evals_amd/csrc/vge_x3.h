// Shared device pieces of the split-precision ("3xfp16") MFMA kernels (vge_encoder_x3.hip,
// vge_transformer_x3.hip): operand planes, fragments, and the direct-to-register weight stream.
// See vge_encoder_x3.hip for the arithmetic and layout description.
#pragma once
#include "vge_common.h"

namespace vge {
// Persistent schedule of the quad / pair conv kernels.  Work units: Q quads (4 windows) then the pairs (2 windows)
// covering the rest of each encoder's windows; encoder e takes q_e quads (windows [0, 4 q_e)) and the pairs after
// them.  Grid = G blocks (one per CU); unit u runs on block u % G in round u / G, so with Q a multiple of G every CU
// does the same number of quads and at most one pair.  Within a round the block index is remapped so the 8 XCDs
// (blocks dealt round robin) take contiguous runs of G / 8 units, i.e. the same encoders' weights in their L2.
// q_e: whole XCD runs where that tiles Q (conv_quad_sched: then every XCD streams ONE encoder per round, and the
// encoders with multi-panel stems -- `heavy`, a bit mask -- take the pairs), else nearly equal.  qpre / ppre: prefix
// sums of the quads / pairs per encoder.
constexpr int CONV_MAX_ENC = 16;
struct ConvSched {
  int n_windows, n_enc, G, Q, n_units;
  int qpre[CONV_MAX_ENC + 1], ppre[CONV_MAX_ENC + 1];
};
ConvSched conv_quad_sched(int n_windows, int n_enc, unsigned heavy = 0);  // vge_encoder_x3.hip (host)
}  // namespace vge

#ifndef VGE_ABL
#define VGE_ABL 0  // timing-only ablation builds (tools/ablate.sh), a bit mask: 1 no MFMA, 2 no B loads after the
                   // prologue, 4 no A reads, 16 identity GELU; 0 = the product
#endif

namespace {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef _Float16 half2v __attribute__((ext_vector_type(2)));

constexpr int XS = 264;              // fp16 per LDS activation row (256 + 8 pad: conflict-free b128 reads)
constexpr int XSB = XS * 2;          // bytes per activation row
constexpr int CHUNK_B = 16384;       // bytes per weight chunk
constexpr int PLANE_B = 8192;        // bytes between the hi and lo planes of a chunk
constexpr int STREAM_GROUP = 8;      // weight streams are packed as multiples of 8 chunks
constexpr int CONV_PF = 4;           // weight chunks in flight per wave: conv (a quad wave holds 128 x 64 outputs)
#ifndef VGE_CONV_PF16
#define VGE_CONV_PF16 8
#endif
constexpr int CONV_PF16 = VGE_CONV_PF16;  // ... in the single-fp16 mode (half the bytes per chunk)
#ifndef VGE_CONV_PF16W
#define VGE_CONV_PF16W 4
#endif
constexpr int CONV_PF16W = VGE_CONV_PF16W;  // ... 4-wave fp16 blocks (a wave's chunk = 2 column tiles)
constexpr int GEMM_PF = 4;           // ... and GEMM waves (32 x 32 outputs, 4 waves per SIMD)

__device__ __forceinline__ floatx16 mfma32(half8 a, half8 b, floatx16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

// x of lane l combined with x of lane l ^ 32 (v_permlane32_swap: no LDS round trip)
__device__ __forceinline__ float halves_sum(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float halves_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

__device__ __forceinline__ void split_store(_Float16* hi, _Float16* lo, float v) {
  const _Float16 h = (_Float16)v;
  *hi = h;
  *lo = (_Float16)(v - (float)h);
}

__device__ __forceinline__ int fp16_range_exp(float m) {  // 2^-e brings m into [2^8, 2^9); 2^+-e stays normal
  return (m > 0.f && m <= 3.0e38f) ? max(ilogbf(m) - 8, -100) : 0;
}

// A wave's output tile: R row tiles x N column tiles of 32 x 32, one f32 accumulator each
template <int R, int N>
struct Acc {
  floatx16 c[R][N];
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int t = 0; t < R; ++t)
#pragma unroll
      for (int n = 0; n < N; ++n)
#pragma unroll
        for (int r = 0; r < 16; ++r) c[t][n][r] = 0.f;
  }
};

template <int R>
struct AFrag {  // A fragments (hi, lo) of one 16-K chunk for R row tiles
  half8 h[R], l[R];
};

template <int N>
struct BFrag {  // B fragments (hi, lo) of one 16-K chunk for N column tiles
  half8 h[N], l[N];
};

// SP (split): true = the 3xfp16 product (hi*hi + hi*lo + lo*hi); false = the single-fp16 throughput mode
// (VGE_F16: hi planes only, one MFMA per product; the lo fragments are never loaded)
template <bool SP = true, int R, int N>
__device__ __forceinline__ void mma_chunk(Acc<R, N>& acc, const AFrag<R>& a, const BFrag<N>& b) {
#if !(VGE_ABL & 1)
#pragma unroll
  for (int n = 0; n < N; ++n)
#pragma unroll
    for (int t = 0; t < R; ++t) {
      acc.c[t][n] = mfma32(a.h[t], b.h[n], acc.c[t][n]);
      if constexpr (SP) {
        acc.c[t][n] = mfma32(a.h[t], b.l[n], acc.c[t][n]);
        acc.c[t][n] = mfma32(a.l[t], b.h[n], acc.c[t][n]);
      }
    }
#else
  asm volatile("" ::"v"(a.h[0]), "v"(a.l[R - 1]), "v"(b.h[0]), "v"(b.l[N - 1]));
#endif
}

typedef const __attribute__((address_space(1))) char* gchar;  // global (not flat) loads: counted by vmcnt only
typedef const __attribute__((address_space(1))) half8* ghalf8;

// column tile n of this lane sits 32 columns (512 B) after tile n - 1
template <int N, bool SP = true>
__device__ __forceinline__ void load_b(gchar g, int c, unsigned loff, BFrag<N>& b) {
  gchar p = g + (size_t)c * CHUNK_B + loff;
#pragma unroll
  for (int n = 0; n < N; ++n) {
    b.h[n] = *reinterpret_cast<ghalf8>(p + n * 512);
    if constexpr (SP) b.l[n] = *reinterpret_cast<ghalf8>(p + n * 512 + PLANE_B);
  }
}

// Multiply a wave's output tile by a stream of n weight chunks (n a multiple of PF, >= PF, PF | 8).  afn(c, AFrag&)
// reads the A fragments of chunk c from LDS (one chunk ahead).  B fragments are loaded PF - 1 chunks ahead
// into a register ring; the loop is unrolled by PF so every ring index is static and the compiler's counted
// vmcnt waits retire exactly the chunk being consumed.
template <int PF, bool SP = true, int R, int N, class AFn>
__device__ __forceinline__ void run_stream(Acc<R, N>& acc, const void* gw, int n, unsigned loff, AFn afn) {
  const gchar g = (gchar)gw;
  BFrag<N> b[PF];
#pragma unroll
  for (int j = 0; j < PF - 1; ++j) load_b<N, SP>(g, j, loff, b[j]);
  AFrag<R> a[2];
  afn(0, a[0]);
  for (int c0 = 0; c0 < n; c0 += PF) {
#pragma unroll
    for (int j = 0; j < PF; ++j) {
      const int c = c0 + j;
#if !(VGE_ABL & 2)
      load_b<N, SP>(g, min(c + PF - 1, n - 1), loff, b[(j + PF - 1) % PF]);
#endif
#if !(VGE_ABL & 4)
      afn(min(c + 1, n - 1), a[(j + 1) & 1]);
#endif
      mma_chunk<SP>(acc, a[j & 1], b[j]);
      // pin this step's loads in place: without it the compiler hoists every A read of the unrolled group
      // and sinks the B loads next to their use, which collapses the prefetch to vmcnt(0) waits
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    }
#if !(VGE_ABL & 8)
    // keep the two waves of each SIMD abreast (a raw s_barrier: LDS reads retired, loads stay in flight);
    // a wave left alone at the end of a stream has too few loads in flight to keep the MFMA pipe busy
    lds_barrier();
#endif
  }
}

// One MovementConvEncoder's weights (model.py:21-58) as the x3 conv kernels read them.
struct EncDescX3 {
  const _Float16* stem;  // stem chunks; panel p (256 K) starts at chunk 16p, padded to STREAM_GROUP chunks
  const _Float16* conv;  // 8 convs x 5 taps x 16 chunks
  const _Float16* proj;  // 16 chunks
  const float* gn_w;     // [4][256]
  const float* gn_b;     // [4][256]
  const float* cs;       // [10][256] weight column scales: stem, conv 0..7, proj
  // staggered split kernel only (vge_encoder_x3s.hip), else null: the GroupNorm-folded corrections of blocks 1..3's
  // conv1, [3 blocks][256 cols][16] = per-tap sums over input channels of W1 gamma (taps 0..4), then of W1 beta (at 8..12),
  // then the proj's [256][2] (sums of P gamma, P beta)
  const float* fold;
  int in_col, d_in, n_stem_panels, ld;  // ld: feats row width (2596, or 2356 keypoint-less)
  float gn_gmax[4], gn_bmax[4];  // max |gamma|, max |beta| of each GroupNorm (split-exponent bounds)
};

__host__ __device__ __forceinline__ int xcd_remap(int b, int nblk) {
  const int q8 = nblk >> 3, r8 = nblk & 7, x8 = b & 7;
  return (x8 < r8 ? x8 * (q8 + 1) : r8 * (q8 + 1) + (x8 - r8) * q8) + (b >> 3);
}

// Unit u of a ConvSched: encoder e, first window w0, quad (true) or pair.  Uniform over the block (scalar loop over
// the <= 16 prefix sums in kernel-argument memory).
__host__ __device__ __forceinline__ bool conv_unit(const vge::ConvSched& cs, int u, int& e, int& w0) {
  const bool quad = u < cs.Q;
  const int v = quad ? u : u - cs.Q;
  const int* pre = quad ? cs.qpre : cs.ppre;
  int ee = 0, lo = 0, qa = 0, qb = cs.qpre[1];
  for (int k = 1; k < cs.n_enc; ++k)  // fixed trip count, no dynamic index into the argument block
    if (v >= pre[k]) {
      ee = k;
      lo = pre[k];
      qa = cs.qpre[k];
      qb = cs.qpre[k + 1];
    }
  w0 = quad ? 4 * (v - lo) : 4 * (qb - qa) + 2 * (v - lo);
  e = ee;
#ifdef __HIP_DEVICE_COMPILE__
  e = __builtin_amdgcn_readfirstlane(e);
  w0 = __builtin_amdgcn_readfirstlane(w0);
#endif
  return quad;
}

}  // namespace
