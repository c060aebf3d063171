// Split-precision ("3xfp16") MFMA path of the fusion encoder (gfx950).
//
// Every GEMM operand x is carried as two fp16 planes, hi = f16(x) and lo = f16(x - hi), and each product
// is formed as hi_a*hi_b + hi_a*lo_b + lo_a*hi_b by three v_mfma_f32_32x32x16_f16 into one f32
// accumulator.  The dropped lo*lo term and the fp16 rounding of lo leave a relative error of ~2^-21 per
// product, i.e. f32-class results (AC/TC within ~1e-7 of the exact f32 path, tests/test_gpu_parity.py),
// at 3 f16 MFMAs per K=16 step instead of 4 f32 MFMAs per K=4 step: 5.3x the f32 MFMA rate.  Both
// operands are scaled by powers of two (exact) so that a block's largest |value| sits in [2^8, 2^9): the
// planes never overflow and the residual lo keeps ~11 significant bits (fp16 subnormals are kept by the
// MFMA).  Activations: per row of a stem panel, per window inside the conv chain, per 64-row tile and
// panel in the GEMMs; weights: per output column at pack time (vge_api.cpp pack_linear_x3, factor `cs`).
//
//   conv_encoder_x3_kernel   MovementConvEncoder x10 (model.py:21-58): one workgroup = 1 encoder x 2 windows
//                            (64 rows), 8 waves, wave w owns output columns 32w..32w+31 of all 64 rows.
//                            Activations stay in LDS as hi/lo planes for the whole chain (the A operand);
//                            each wave streams its own 32 weight columns (the B operand) straight from
//                            L2 into registers, PF chunks deep, so the K loop has no barrier and no LDS
//                            traffic besides the A fragment reads.
//   gemm_x3_kernel<EPI>      transformer / token GEMMs, same tiling (BM = 64, BN = 256), with the fused
//                            epilogues of the f32 path.
//
// MFMA maps (v_mfma_f32_32x32x16_f16): lane l (i = l&31, h = l>>5) supplies A[row i][k = 8h + j] and
// B[k = 8h + j][col i], j = 0..7; C/D: col = l&31, row = (r&3) + 8(r>>2) + 4(l>>5), r = 0..15.
// A weight chunk = 16 K x 256 columns: [plane][h][n][8] fp16 = 16 KB, so a lane's B fragment of a chunk
// is one 16-B load per plane and a wave's 32 columns are two contiguous 512-B runs per plane.
#include "vge_x3.h"
#include <algorithm>
#include <vector>
#include <cstdlib>
#include <cstring>


#ifndef VGE_TRACE_ROUND
#define VGE_TRACE_ROUND 0  // VGE_TRACE builds stamp the units of this round of the persistent schedule
#endif
#ifdef VGE_TRACE  // timing-only builds (tools/trace_encoder.py): s_memtime stamps of every wave of blocks 0..63
__device__ long long g_vge_trace[64 * 8 * 32];
#define STAMP(k)                                                                                        \
  do {                                                                                                  \
    if (tr_on && blockIdx.x < 64 && (threadIdx.x & 63) == 0)                                            \
      g_vge_trace[(blockIdx.x * 8 + (threadIdx.x >> 6)) * 32 + (k)] = __builtin_amdgcn_s_memtime();     \
  } while (0)
#else
#define STAMP(k) \
  do {           \
  } while (0)
#endif

namespace {

// ------------------------------------------------------------------ conv encoder chain (EncDescX3: vge_x3.h)
// One workgroup = one encoder x W windows (32 W rows) on CW waves; wave w owns output columns
// 32 N w .. 32 N w + 32 N - 1 (N = 8 / CW column tiles) of all rows, so every weight byte streamed into the
// workgroup feeds 32 W rows.  Used as W = 4 / 2 with CW = 8 (one workgroup per CU, two waves per SIMD).
// (Measured alternative, not kept: pairs on 4 waves with two unsynchronised workgroups per CU -- equal
// steady-state rate, twice the L2->CU weight traffic, worse tail at 256 windows.)
// Row tiles whose residual lives in LDS (f32, lane-private) instead of registers in conv_f16w_body: from 4 windows
// on, the last one or two tiles' residuals go to LDS (what the 160 KB leave beside the single activation plane), so
// a hex unit's accumulators (96) + residuals (80) + fragments fit a wave's 256 VGPRs.
template <int W>
constexpr int res_lds_tiles() {
  return W == 6 ? 1 : (W >= 4 ? 2 : 0);
}
// NPL activation planes: 2 (hi, lo) when the convs or the stem are split, 1 in the pure fp16 mode
template <int W, int CW, int NPL = 2>
constexpr int conv_lds_bytes() {
  return NPL * (32 * W + 1) * XSB + (6 * W * CW + 2 * 32 * W) * 4 + (NPL == 1 ? res_lds_tiles<W>() : 0) * 32 * 256 * 4;
}
template <int CW, int NPL>
constexpr int conv_lds_bytes_max() {  // over W = 1..6
  return std::max({conv_lds_bytes<1, CW, NPL>(), conv_lds_bytes<2, CW, NPL>(), conv_lds_bytes<3, CW, NPL>(),
                   conv_lds_bytes<4, CW, NPL>(), conv_lds_bytes<5, CW, NPL>(), conv_lds_bytes<6, CW, NPL>()});
}

// blocks [0, n_quad) take 4 windows, the rest 2: quads stream each weight byte for twice the rows, pairs
// fill the last round (see launch_conv_encoders_x3)
// SP: the 3xfp16 split for the conv blocks and proj; SPS: for the stem (its z-scored inputs carry the widest
// dynamic range; the f16 mode may keep the stem split)
template <int W, int CW, bool SP, bool SPS = SP>
__device__ __forceinline__ void conv_encoder_body(const float* __restrict__ feats, int n_windows, int win0,
                                                  const EncDescX3& ed, int e, float* __restrict__ enc_out,
                                                  char* lds_raw, [[maybe_unused]] bool tr_on) {
  constexpr int R = W, N = 8 / CW, ROWS = 32 * W, XROWS = ROWS + 1;
  constexpr int CONV_WAVES = CW;
  static_assert(CW * N == 8, "8 column tiles of 32 per workgroup");
  _Float16* Xh = reinterpret_cast<_Float16*>(lds_raw);                   // [XROWS][XS]
  _Float16* Xl = Xh + XROWS * XS;                                        // [XROWS][XS]
  float* red = reinterpret_cast<float*>(lds_raw + 2 * XROWS * XSB);      // [6 slots][W][waves] partials
  int* rexp = reinterpret_cast<int*>(red + 6 * W * CONV_WAVES);          // [2][ROWS] stem row exponents

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int i = lane & 31, h = lane >> 5;
  const int col0 = wave * 32 * N + i;                           // this lane's columns: col0 + 32 n
  const unsigned loff = (unsigned)((h * 256 + col0) * 16);      // its B fragment (column tile 0) in a chunk
  const char* xa = reinterpret_cast<const char*>(Xh) + h * 16;  // its 8 k-values of a 16-K chunk column
  auto crow = [&](int t, int r) { return t * 32 + (r & 3) + 8 * (r >> 2) + 4 * h; };  // C-layout row

  Acc<R, N> acc;
  floatx16 res[R][N];
  for (int c = tid; c < XS; c += 64 * CW) {  // the zero row
    Xh[ROWS * XS + c] = (_Float16)0.0f;
    if constexpr (SP) Xl[ROWS * XS + c] = (_Float16)0.0f;
  }

  // Combine one value per window over the 8 waves.  `slot` picks one of 4 partial buffers so back-to-back
  // reductions need only the one barrier inside.
  auto block_reduce = [&](const float (&v)[R], int slot, bool is_max, float (&out)[R]) {
#pragma unroll
    for (int t = 0; t < R; ++t) {
      const float w = is_max ? wave_max_last(v[t]) : wave_sum_last(v[t]);
      if (lane == 63) red[(slot * R + t) * CONV_WAVES + wave] = w;
    }
    __syncthreads();
#pragma unroll
    for (int t = 0; t < R; ++t) {
      const float* p = red + (slot * R + t) * CONV_WAVES;
      float a = p[0];
#pragma unroll
      for (int w = 1; w < CONV_WAVES; ++w) a = is_max ? fmaxf(a, p[w]) : a + p[w];
      out[t] = a;
    }
  };

  // Store the next conv's input as window * 2^-ex[t] (exact), the window's largest |value| in [2^8, 2^9)
  // -- from a block-wide max, or, when `bound` is given, from that per-window upper bound (a few times the
  // max at most: the split stays exact to 2^-22 relative) -- the consumer multiplies its accumulators
  // back by 2^ex[t].  The block-wide max's barrier orders the writes after every wave's reads of X; with
  // a bound the caller has passed such a barrier since the last stream.
  auto store_x = [&](const floatx16 (&v)[R][N], int (&ex)[R], const float* bound) {
    float mm[R];
    if (bound) {
#pragma unroll
      for (int t = 0; t < R; ++t) mm[t] = bound[t];
    } else {
      float m[R];
#pragma unroll
      for (int t = 0; t < R; ++t) {
        m[t] = 0.f;
#pragma unroll
        for (int n = 0; n < N; ++n)
#pragma unroll
          for (int r = 0; r < 16; ++r) m[t] = fmaxf(m[t], fabsf(v[t][n][r]));
      }
#if !(VGE_ABL & 512)
      block_reduce(m, 3, true, mm);
#else
#pragma unroll
      for (int t = 0; t < R; ++t) mm[t] = m[t];  // timing ablation: no block-wide max (wrong results)
#endif
    }
#pragma unroll
    for (int t = 0; t < R; ++t) {
      ex[t] = fp16_range_exp(mm[t]);
      const float sc = ldexpf(1.0f, -ex[t]);
#pragma unroll
      for (int n = 0; n < N; ++n) {
        // byte bases of this lane's column in row tile t (plane hi, lo); row r of the tile sits at a constant
        // offset (an immediate of ds_write_b16), so no per-store address register stays live
        char* bh = reinterpret_cast<char*>(Xh) + ((t * 32 + 4 * h) * XS + col0 + 32 * n) * 2;
        char* bl = bh + XROWS * XSB;
#pragma unroll
        for (int r = 0; r < 16; r += 2) {  // two rows per packed conversion (v_cvt_pk_f16_f32)
          const floatx2 y = (floatx2){v[t][n][r], v[t][n][r + 1]} * sc;
          const half2v hi = __builtin_convertvector(y, half2v);
          const half2v lo = __builtin_convertvector(y - __builtin_convertvector(hi, floatx2), half2v);
          const int off = ((r & 3) + 8 * (r >> 2)) * XSB;  // rows r and r + 1 of the tile are adjacent
          *reinterpret_cast<_Float16*>(bh + off) = hi[0];
          *reinterpret_cast<_Float16*>(bh + off + XSB) = hi[1];
#if !(VGE_ABL & 256)  // timing ablation: hi plane only (wrong results)
          if constexpr (SP) {
            *reinterpret_cast<_Float16*>(bl + off) = lo[0];
            *reinterpret_cast<_Float16*>(bl + off + XSB) = lo[1];
          }
#endif
        }
      }
    }
  };

  auto afn_rows = [&](int c, AFrag<R>& f) {  // A fragments of the block's own rows
#pragma unroll
    for (int t = 0; t < R; ++t) {
      const char* q = xa + (t * 32 + i) * XSB + c * 32;
      f.h[t] = *reinterpret_cast<const half8*>(q);
      if constexpr (SP) f.l[t] = *reinterpret_cast<const half8*>(q + XROWS * XSB);
    }
  };
  auto afn_stem = [&](int c, AFrag<R>& f) {
#pragma unroll
    for (int t = 0; t < R; ++t) {
      const char* q = xa + (t * 32 + i) * XSB + c * 32;
      f.h[t] = *reinterpret_cast<const half8*>(q);
      if constexpr (SPS) f.l[t] = *reinterpret_cast<const half8*>(q + XROWS * XSB);
    }
  };

  STAMP(0);
  // ---------------- stem: Conv1d(d_in -> 256, k=1, no bias), K streamed in 256-wide panels.
  // Per-row power-of-two scale: z-scored features leave the fp16 range when a column's train-set std is ~0
  // ((x - mean) / (std + 1e-6)), so row m of panel p is split as A[m,:] * 2^-e (exact) with the panel row's
  // largest |value| in [2^8, 2^9); the accumulators (held as C * 2^-e per row) are rescaled when e changes
  // between panels and multiplied back by 2^e at the end (all exact).  rexp[parity][row] holds e.
  acc.zero();
  for (int p = 0; p < ed.n_stem_panels; ++p) {
    const int kw = min(256, ed.d_in - p * 256);
    int* ecur = rexp + (p & 1) * ROWS;
    // wave w stages rows w*RPW .. w*RPW + RPW - 1 (RPW = 32 W / CW) in groups of 4; lane l columns l,
    // l+64, l+128, l+192
    constexpr int RPW = 32 * W / CW;
#pragma unroll
    for (int g8 = 0; g8 < RPW / 4; ++g8) {
      float a[4][4];
#pragma unroll
      for (int jr = 0; jr < 4; ++jr) {
        const int r = wave * RPW + g8 * 4 + jr;
        const int w = win0 + (r >> 5);
        const float* src = feats + ((size_t)w * VGE_T + (r & 31)) * ed.ld + ed.in_col + p * 256;
#pragma unroll
        for (int jc = 0; jc < 4; ++jc) {
          const int c = lane + 64 * jc;
          a[jr][jc] = (c < kw && w < n_windows) ? src[c] : 0.f;
        }
      }
#pragma unroll
      for (int jr = 0; jr < 4; ++jr) {
        float m = fmaxf(fmaxf(fabsf(a[jr][0]), fabsf(a[jr][1])), fmaxf(fabsf(a[jr][2]), fabsf(a[jr][3])));
        m = wave_max_all(m);
        const int ex = fp16_range_exp(m);
        const int r = wave * RPW + g8 * 4 + jr;
        if (lane == 0) ecur[r] = ex;
#pragma unroll
        for (int jc = 0; jc < 4; ++jc) {
          const int c = lane + 64 * jc;
          if constexpr (SPS) split_store(Xh + r * XS + c, Xl + r * XS + c, ldexpf(a[jr][jc], -ex));
          else Xh[r * XS + c] = (_Float16)ldexpf(a[jr][jc], -ex);
        }
      }
    }
    __syncthreads();  // X and ecur complete
    if (p == 0) STAMP(1);
    if (p > 0) {
      const int* eprev = rexp + ((p - 1) & 1) * ROWS;
#pragma unroll
      for (int t = 0; t < R; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float f = ldexpf(1.0f, eprev[crow(t, r)] - ecur[crow(t, r)]);
#pragma unroll
          for (int n = 0; n < N; ++n) acc.c[t][n][r] *= f;
        }
    }
    run_stream<SPS ? CONV_PF : CONV_PF16, SPS>(acc, reinterpret_cast<const char*>(ed.stem) + (size_t)p * 16 * CHUNK_B,
                             ((kw + 127) >> 7) * STREAM_GROUP, loff, afn_stem);
    __syncthreads();  // every wave is done reading X
  }
  {
    const int* efin = rexp + ((ed.n_stem_panels - 1) & 1) * ROWS;
#pragma unroll
    for (int n = 0; n < N; ++n) {
      const float wcs = ed.cs[col0 + 32 * n];
#pragma unroll
      for (int t = 0; t < R; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) res[t][n][r] = ldexpf(acc.c[t][n][r] * wcs, efin[crow(t, r)]);
    }
  }
  STAMP(2);
  int xexp[R];
  store_x(res, xexp, nullptr);
  __syncthreads();
  STAMP(3);

  // ---------------- 4 TemporalConvBlocks
  for (int blk = 0; blk < 4; ++blk) {
    const int dil = 1 << blk;
    for (int cv = 0; cv < 2; ++cv) {
      acc.zero();
      auto afn = [&](int c, AFrag<R>& f) {
        const int tap = c >> 4, cc = c & 15;
        const int tt = i + (tap - 2) * dil;
        const bool in = (unsigned)tt < 32u;
#pragma unroll
        for (int t = 0; t < R; ++t) {
          const int row = in ? t * 32 + tt : ROWS;  // out of the window -> zero row
          const char* q = xa + row * XSB + cc * 32;
          f.h[t] = *reinterpret_cast<const half8*>(q);
          if constexpr (SP) f.l[t] = *reinterpret_cast<const half8*>(q + XROWS * XSB);
        }
      };
      run_stream<SP ? CONV_PF : CONV_PF16, SP>(acc, reinterpret_cast<const char*>(ed.conv) + (size_t)(blk * 2 + cv) * 5 * 16 * CHUNK_B,
                          5 * 16, loff, afn);
      STAMP(4 + (blk * 2 + cv) * 2);
      // epilogue in packed f32 (v_pk_fma_f32: two rows per instruction), in place:
      // acc * 2^xexp * column scale -> [+ residual] -> GELU [-> GroupNorm]
      floatx16 (&v)[R][N] = acc.c;
      floatx2 s2[R];
#pragma unroll
      for (int t = 0; t < R; ++t) s2[t] = 0.f;
#pragma unroll
      for (int n = 0; n < N; ++n) {
        const float wcs = ed.cs[(1 + blk * 2 + cv) * 256 + col0 + 32 * n];
#pragma unroll
        for (int t = 0; t < R; ++t) {
          const float xs = ldexpf(1.0f, xexp[t]) * wcs;
          floatx2 y[8];
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            y[k] = (floatx2){v[t][n][2 * k], v[t][n][2 * k + 1]} * xs;
            if (cv == 1) y[k] += (floatx2){res[t][n][2 * k], res[t][n][2 * k + 1]};
          }
          gelu2_many(y);  // 8 independent chains interleaved
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            s2[t] += y[k];
            v[t][n][2 * k] = y[k].x;
            v[t][n][2 * k + 1] = y[k].y;
          }
          __builtin_amdgcn_sched_barrier(0);  // one tile's temporaries at a time
        }
      }
      STAMP(22 + blk * 2 + cv);
      float gbound[R];  // cv == 1: a bound on each window's |GroupNorm output| for the split exponent
      if (cv == 1) {
        // GroupNorm(1, 256) per window over its 32 x 256 values, spread over the waves
        float s[R], mean[R], q[R], var[R];
#pragma unroll
        for (int t = 0; t < R; ++t) s[t] = s2[t].x + s2[t].y;
        block_reduce(s, 0, false, mean);
#pragma unroll
        for (int t = 0; t < R; ++t) {
          mean[t] *= 1.0f / 8192.0f;
          floatx2 q2 = 0.f;
#pragma unroll
          for (int n = 0; n < N; ++n)
#pragma unroll
            for (int r = 0; r < 16; r += 2) {
              const floatx2 d = (floatx2){v[t][n][r], v[t][n][r + 1]} - mean[t];
              q2 = __builtin_elementwise_fma(d, d, q2);
            }
          q[t] = q2.x + q2.y;
        }
        block_reduce(q, 1, false, var);
        // |normalised| <= sqrt(8191) (the 8192 squares sum to at most 8192), so |out| <= 90.51 max|gamma| +
        // max|beta| -- a static bound, typically ~20x the max: the split keeps 2^-22 relative precision
#pragma unroll
        for (int t = 0; t < R; ++t) gbound[t] = 90.51f * ed.gn_gmax[blk] + ed.gn_bmax[blk];
#pragma unroll
        for (int n = 0; n < N; ++n) {
          const float gw = ed.gn_w[blk * 256 + col0 + 32 * n], gb = ed.gn_b[blk * 256 + col0 + 32 * n];
#pragma unroll
          for (int t = 0; t < R; ++t) {
            const float rstd = 1.0f / sqrtf(var[t] * (1.0f / 8192.0f) + 1e-5f);
            const float sc = rstd * gw, sh = gb - mean[t] * sc;  // (v - mean) * rstd * w + b
#pragma unroll
            for (int r = 0; r < 16; r += 2) {
              const floatx2 y =
                  __builtin_elementwise_fma((floatx2){v[t][n][r], v[t][n][r + 1]}, (floatx2)sc, (floatx2)sh);
              v[t][n][r] = res[t][n][r] = y.x;
              v[t][n][r + 1] = res[t][n][r + 1] = y.y;
            }
          }
        }
      }
      // cv == 0: store_x's block-wide max is the barrier after every wave's reads of X (this conv's A
      // operand); cv == 1: the GroupNorm reductions are
      store_x(v, xexp, cv == 1 ? gbound : nullptr);
      __syncthreads();
      STAMP(5 + (blk * 2 + cv) * 2);
    }
  }

  // ---------------- proj: Linear(256 -> 256, no bias)
  acc.zero();
  run_stream<SP ? CONV_PF : CONV_PF16, SP>(acc, reinterpret_cast<const char*>(ed.proj), 16, loff, afn_rows);
  STAMP(20);
#pragma unroll
  for (int t = 0; t < R; ++t) {
    const int win = win0 + t;
    if (win < n_windows) {
      float* o = enc_out + ((size_t)e * n_windows * VGE_T + (size_t)win * VGE_T) * VGE_D;
#pragma unroll
      for (int n = 0; n < N; ++n) {
        const float xs = ldexpf(1.0f, xexp[t]) * ed.cs[9 * 256 + col0 + 32 * n];
#pragma unroll
        for (int r = 0; r < 16; ++r) o[crow(0, r) * VGE_D + col0 + 32 * n] = acc.c[t][n][r] * xs;
      }
    }
  }
  STAMP(21);
#ifdef VGE_TRACE
  if (tr_on && blockIdx.x < 64 && threadIdx.x == 0) g_vge_trace[blockIdx.x * 8 * 32 + 31] = e;
#endif
}

// Persistent schedule.  Work units: Q quads (4 windows) then the pairs (2 windows) covering the rest of each
// encoder's windows; encoder e takes q_e = qa + (e < qr) quads (windows [0, 4 q_e)) and the pairs after them.
// Grid = G blocks (one per CU); unit u runs on block u % G in round u / G, so with Q a multiple of G every
// CU does the same number of quads and at most one pair.  Within a round the block index is remapped so the
// 8 XCDs (blocks dealt round robin) take contiguous units, i.e. the same encoders' weights in their L2.
// (ConvSched, xcd_remap: vge_x3.h)

template <bool SP, bool SPS>
__global__ void __launch_bounds__(512, 1) conv_encoder_x3_kernel(const float* __restrict__ feats,
                                                                  const EncDescX3* __restrict__ encs, vge::ConvSched cs,
                                                                  float* __restrict__ enc_out) {
  extern __shared__ __attribute__((aligned(16))) char lds_raw[];
  const int n = cs.n_windows;
  for (int round = 0; round * cs.G < cs.n_units; ++round) {
    const int u = round * cs.G + xcd_remap(blockIdx.x, cs.G);
    if (u >= cs.n_units) break;  // uniform over the block
    if (round > 0) __syncthreads();  // the previous unit's LDS is free
    int e, w0;
    if (conv_unit(cs, u, e, w0))
      conv_encoder_body<4, 8, SP, SPS>(feats, n, w0, encs[e], e, enc_out, lds_raw, round == VGE_TRACE_ROUND);
    else
      conv_encoder_body<2, 8, SP, SPS>(feats, n, w0, encs[e], e, enc_out, lds_raw, round == VGE_TRACE_ROUND);
  }
}

// Multiply a wave's output tile by a stream of n weight chunks (the single-fp16 form of run_stream) with ONE A
// fragment per row tile: tile t's fragment of chunk c + 1 is read from LDS right after the N MFMAs of chunk c that
// use it, so its latency hides behind the other tiles' MFMAs and no second A buffer is live (a hex unit needs
// those registers).  afn1(c, t) returns tile t's fragment of chunk c.
template <int PF, int R, int N, class AFn1>
__device__ __forceinline__ void run_stream1(Acc<R, N>& acc, const void* gw, int n, unsigned loff, AFn1 afn1) {
  const gchar g = (gchar)gw;
  BFrag<N> b[PF];
#pragma unroll
  for (int j = 0; j < PF - 1; ++j) load_b<N, false>(g, j, loff, b[j]);
  half8 a[R];
#pragma unroll
  for (int t = 0; t < R; ++t) a[t] = afn1(0, t);
  for (int c0 = 0; c0 < n; c0 += PF) {
#pragma unroll
    for (int j = 0; j < PF; ++j) {
      const int c = c0 + j;
#if !(VGE_ABL & 2)
      load_b<N, false>(g, min(c + PF - 1, n - 1), loff, b[(j + PF - 1) % PF]);
#endif
      const int cn = min(c + 1, n - 1);
#pragma unroll
      for (int t = 0; t < R; ++t) {
#if !(VGE_ABL & 1)
#pragma unroll
        for (int q = 0; q < N; ++q) acc.c[t][q] = mfma32(a[t], b[j].h[q], acc.c[t][q]);
#endif
#if !(VGE_ABL & 4)
        a[t] = afn1(cn, t);
#endif
      }
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    }
    // no per-group barrier (unlike run_stream): measured without it the waves drift within a conv and meet at the
    // epilogue's first block reduction -- 443 k -> 419 k cycles per 5-window unit; every LDS write that could race a
    // slower wave's A reads comes after that reduction's barrier
  }
}

// The MovementConvEncoder chain of one unit = one encoder x W windows on CW waves (wave w: columns 32Nw..32Nw+32N-1
// of all 32 W rows, N = 8 / CW), single fp16 operands (VGE_F16, nothing split).  Same arithmetic as conv_encoder_body<W, CW,
// false> -- same chunk order and MFMA per output, same epilogue operations -- with epilogues that stream tile by
// tile instead of holding the unit's activations in registers: each exponent comes from a max pass over the
// accumulators (stem output; |pre-GELU value| for the first conv of a block, an upper bound of |GELU|) or from the
// GroupNorm bound, so every tile is computed, stored and dropped in one pass.  Only the second conv of a block holds
// its GELU outputs for the GroupNorm statistics, while the residuals it consumes die.
template <int W, int CW>
__device__ __forceinline__ void conv_f16w_body(const float* __restrict__ feats, int n_windows, int win0,
                                               const EncDescX3& ed, int e, float* __restrict__ enc_out,
                                               char* lds_raw, [[maybe_unused]] bool tr_on) {
  constexpr int R = W, N = 8 / CW, NWV = CW, ROWS = 32 * W, XROWS = ROWS + 1;
  constexpr int RL = res_lds_tiles<W>(), RREG = R - RL;
#ifndef VGE_HEX_PF
#define VGE_HEX_PF CONV_PF16W
#endif
  constexpr int PFW = W >= 6 ? VGE_HEX_PF : 2 * CONV_PF16W;  // weight chunks in flight (registers allowing)
  _Float16* X = reinterpret_cast<_Float16*>(lds_raw);                 // [XROWS][XS]
  float* red = reinterpret_cast<float*>(lds_raw + XROWS * XSB);       // [6 slots][W][waves]
  int* rexp = reinterpret_cast<int*>(red + 6 * W * NWV);              // [2][ROWS] stem row exponents
  // residual tiles in LDS: [RL][waves][N][4][64 lanes] floatx4 (tile stride = 32 rows x 256 columns)
  floatx4* resl = reinterpret_cast<floatx4*>(rexp + 2 * ROWS) + (threadIdx.x >> 6) * (N * 4 * 64) + (threadIdx.x & 63);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int i = lane & 31, h = lane >> 5;
  const int col0 = wave * 32 * N + i;                          // this lane's columns: col0 + 32 n
  const unsigned loff = (unsigned)((h * 256 + col0) * 16);     // its B fragment (column tile 0) in a chunk
  const char* xa = reinterpret_cast<const char*>(X) + h * 16;  // its 8 k-values of a 16-K chunk column
  auto crow = [&](int t, int r) { return t * 32 + (r & 3) + 8 * (r >> 2) + 4 * h; };  // C-layout row
  char* xb = reinterpret_cast<char*>(X) + (4 * h * XS + col0) * 2;  // this lane's column, row 4h of tile 0

  Acc<R, N> acc;
  floatx16 res[RREG > 0 ? RREG : 1][N];
  auto res_set = [&](int t, int n, const floatx16& x) {
    if (t < RREG) {
      res[t][n] = x;
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        resl[(t - RREG) * (NWV * N * 4 * 64) + (n * 4 + q) * 64] = (floatx4){x[4 * q], x[4 * q + 1], x[4 * q + 2], x[4 * q + 3]};
    }
  };
  auto res_get = [&](int t, int n) -> floatx16 {
    if (t < RREG) return res[t][n];
    floatx16 x;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const floatx4 y = resl[(t - RREG) * (NWV * N * 4 * 64) + (n * 4 + q) * 64];
      x[4 * q] = y.x; x[4 * q + 1] = y.y; x[4 * q + 2] = y.z; x[4 * q + 3] = y.w;
    }
    return x;
  };
  for (int c = tid; c < XS; c += 64 * NWV) X[ROWS * XS + c] = (_Float16)0.0f;  // the zero row

  auto block_reduce = [&](const float (&v)[R], int slot, bool is_max, float (&out)[R]) {
#pragma unroll
    for (int t = 0; t < R; ++t) {
      const float w = is_max ? wave_max_last(v[t]) : wave_sum_last(v[t]);
      if (lane == 63) red[(slot * R + t) * NWV + wave] = w;
    }
    __syncthreads();
#pragma unroll
    for (int t = 0; t < R; ++t) {
      const float* p = red + (slot * R + t) * NWV;
      float a = p[0];
#pragma unroll
      for (int w = 1; w < NWV; ++w) a = is_max ? fmaxf(a, p[w]) : a + p[w];
      out[t] = a;
    }
  };
  // fp16 store of a lane's 16 values of column tile n of row tile t, scaled by 2^-ex (immediate-offset ds_write_b16)
  auto store_tile = [&](const floatx16& v, int t, int n, int ex) {
    const float sc = ldexpf(1.0f, -ex);
    char* bh = xb + (t * 32 * XS + 32 * n) * 2;
#pragma unroll
    for (int r = 0; r < 16; r += 2) {
      const floatx2 y = (floatx2){v[r], v[r + 1]} * sc;
      const half2v hv = __builtin_convertvector(y, half2v);
      const int off = ((r & 3) + 8 * (r >> 2)) * XSB;
      *reinterpret_cast<_Float16*>(bh + off) = hv[0];
      *reinterpret_cast<_Float16*>(bh + off + XSB) = hv[1];
    }
  };
  auto afn_rows = [&](int c, int t) { return *reinterpret_cast<const half8*>(xa + (t * 32 + i) * XSB + c * 32); };

  // ---------------- stem: Conv1d(d_in -> 256, k=1, no bias), K in 256-wide panels, per-row exponents (see
  // conv_encoder_body)
  STAMP(0);
  acc.zero();
  for (int p = 0; p < ed.n_stem_panels; ++p) {
    const int kw = min(256, ed.d_in - p * 256);
    int* ecur = rexp + (p & 1) * ROWS;
    constexpr int RPW = 32 * W / NWV;
    // every row load of the panel in flight at once (the staging is HBM-latency bound: ~20 k cycles per unit with
    // 16 loads in flight per wave); the acc registers are zero and no residual is live yet
    float a[RPW][4];
#pragma unroll
    for (int jr = 0; jr < RPW; ++jr) {
      const int r = wave * RPW + jr;
      const int w = win0 + (r >> 5);
      const float* src = feats + ((size_t)w * VGE_T + (r & 31)) * ed.ld + ed.in_col + p * 256;
#pragma unroll
      for (int jc = 0; jc < 4; ++jc) {
        const int c = lane + 64 * jc;
        a[jr][jc] = (c < kw && w < n_windows) ? src[c] : 0.f;
      }
    }
#pragma unroll
    for (int jr = 0; jr < RPW; ++jr) {
      float m = fmaxf(fmaxf(fabsf(a[jr][0]), fabsf(a[jr][1])), fmaxf(fabsf(a[jr][2]), fabsf(a[jr][3])));
      m = wave_max_all(m);
      const int ex = fp16_range_exp(m);
      const int r = wave * RPW + jr;
      if (lane == 0) ecur[r] = ex;
#pragma unroll
      for (int jc = 0; jc < 4; ++jc) X[r * XS + lane + 64 * jc] = (_Float16)ldexpf(a[jr][jc], -ex);
    }
    __syncthreads();  // X and ecur complete
    if (p == 0) STAMP(1);
    if (p > 0) {
      const int* eprev = rexp + ((p - 1) & 1) * ROWS;
#pragma unroll
      for (int t = 0; t < R; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float f = ldexpf(1.0f, eprev[crow(t, r)] - ecur[crow(t, r)]);
#pragma unroll
          for (int n = 0; n < N; ++n) acc.c[t][n][r] *= f;
        }
    }
    run_stream1<PFW>(acc, reinterpret_cast<const char*>(ed.stem) + (size_t)p * 16 * CHUNK_B,
                            ((kw + 127) >> 7) * STREAM_GROUP, loff, afn_rows);
    __syncthreads();  // every wave is done reading X
  }
  STAMP(2);
  int xexp[R];
  {
    const int* efin = rexp + ((ed.n_stem_panels - 1) & 1) * ROWS;
    float wcs[N];
#pragma unroll
    for (int n = 0; n < N; ++n) wcs[n] = ed.cs[col0 + 32 * n];
    auto stem_out = [&](int t, int n, int r) { return ldexpf(acc.c[t][n][r] * wcs[n], efin[crow(t, r)]); };
    float m[R], mm[R];
#pragma unroll
    for (int t = 0; t < R; ++t) {
      m[t] = 0.f;
#pragma unroll
      for (int n = 0; n < N; ++n)
#pragma unroll
        for (int r = 0; r < 16; ++r) m[t] = fmaxf(m[t], fabsf(stem_out(t, n, r)));
    }
    block_reduce(m, 3, true, mm);
#pragma unroll
    for (int t = 0; t < R; ++t) {
      xexp[t] = fp16_range_exp(mm[t]);
#pragma unroll
      for (int n = 0; n < N; ++n) {
        floatx16 v;
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = stem_out(t, n, r);
        res_set(t, n, v);
        store_tile(v, t, n, xexp[t]);
      }
    }
  }
  __syncthreads();
  STAMP(3);

  // ---------------- 4 TemporalConvBlocks (the two convs of a block written out: each epilogue is its own code)
#pragma unroll 1
  for (int blk = 0; blk < 4; ++blk) {
    const int dil = 1 << blk;
#pragma unroll
    for (int cv = 0; cv < 2; ++cv) {
      acc.zero();
      auto afn = [&](int c, int t) {
        const int tap = c >> 4, cc = c & 15;
        const int tt = i + (tap - 2) * dil;
        const int row = (unsigned)tt < 32u ? t * 32 + tt : ROWS;  // out of the window -> zero row
        return *reinterpret_cast<const half8*>(xa + row * XSB + cc * 32);
      };
      run_stream1<PFW>(acc, reinterpret_cast<const char*>(ed.conv) + (size_t)(blk * 2 + cv) * 5 * 16 * CHUNK_B,
                              5 * 16, loff, afn);
      STAMP(4 + (blk * 2 + cv) * 2);
      float wcs[N];
#pragma unroll
      for (int n = 0; n < N; ++n) wcs[n] = ed.cs[(1 + blk * 2 + cv) * 256 + col0 + 32 * n];
      if (cv == 0) {
        // GELU(y) with y = acc * 2^xexp * column scale; |GELU(y)| <= max(|y|, 0.17), so the pre-GELU block max
        // gives the next operand's exponent without holding the GELU outputs
        float m[R], mm[R];
#pragma unroll
        for (int t = 0; t < R; ++t) {
          m[t] = 0.17f;
#pragma unroll
          for (int n = 0; n < N; ++n) {
            float a0 = 0.f;
#pragma unroll
            for (int r = 0; r < 16; ++r) a0 = fmaxf(a0, fabsf(acc.c[t][n][r]));
            m[t] = fmaxf(m[t], a0 * fabsf(ldexpf(1.0f, xexp[t]) * wcs[n]));
          }
        }
        STAMP(22 + blk * 2 + cv);
        block_reduce(m, 3, true, mm);  // its barrier also orders the stores after every wave's reads of X
#pragma unroll
        for (int t = 0; t < R; ++t) {
          const int ex = fp16_range_exp(mm[t]);
#pragma unroll
          for (int n = 0; n < N; ++n) {
            const float xs = ldexpf(1.0f, xexp[t]) * wcs[n];
            floatx16 v;
#pragma unroll
            for (int k0 = 0; k0 < 8; k0 += 4) {
              floatx2 y[4];
#pragma unroll
              for (int k = 0; k < 4; ++k) y[k] = (floatx2){acc.c[t][n][2 * (k0 + k)], acc.c[t][n][2 * (k0 + k) + 1]} * xs;
              gelu2_fast(y);
#pragma unroll
              for (int k = 0; k < 4; ++k) {
                v[2 * (k0 + k)] = y[k].x;
                v[2 * (k0 + k) + 1] = y[k].y;
              }
            }
            store_tile(v, t, n, ex);
            __builtin_amdgcn_sched_barrier(0);  // one tile's temporaries at a time
          }
          xexp[t] = ex;
        }
      } else {
        // GELU(acc * scale + residual) -> GroupNorm(1, 256) per window -> the next block's input and residual
        floatx2 s2[R];
#pragma unroll
        for (int t = 0; t < R; ++t) {
          s2[t] = 0.f;
#pragma unroll
          for (int n = 0; n < N; ++n) {
            const float xs = ldexpf(1.0f, xexp[t]) * wcs[n];
            const floatx16 rt = res_get(t, n);
#pragma unroll
            for (int k0 = 0; k0 < 8; k0 += 4) {
              floatx2 y[4];
#pragma unroll
              for (int k = 0; k < 4; ++k)
                y[k] = (floatx2){acc.c[t][n][2 * (k0 + k)], acc.c[t][n][2 * (k0 + k) + 1]} * xs +
                       (floatx2){rt[2 * (k0 + k)], rt[2 * (k0 + k) + 1]};
              gelu2_fast(y);
#pragma unroll
              for (int k = 0; k < 4; ++k) {
                s2[t] += y[k];
                acc.c[t][n][2 * (k0 + k)] = y[k].x;
                acc.c[t][n][2 * (k0 + k) + 1] = y[k].y;
              }
            }
            __builtin_amdgcn_sched_barrier(0);
          }
        }
        float sm[R], mean[R], q[R], var[R];
#pragma unroll
        for (int t = 0; t < R; ++t) sm[t] = s2[t].x + s2[t].y;
        STAMP(22 + blk * 2 + cv);
        block_reduce(sm, 0, false, mean);
#pragma unroll
        for (int t = 0; t < R; ++t) {
          mean[t] *= 1.0f / 8192.0f;
          floatx2 q2 = 0.f;
#pragma unroll
          for (int n = 0; n < N; ++n)
#pragma unroll
            for (int r = 0; r < 16; r += 2) {
              const floatx2 d = (floatx2){acc.c[t][n][r], acc.c[t][n][r + 1]} - mean[t];
              q2 = __builtin_elementwise_fma(d, d, q2);
            }
          q[t] = q2.x + q2.y;
        }
        block_reduce(q, 1, false, var);
        const int ex = fp16_range_exp(90.51f * ed.gn_gmax[blk] + ed.gn_bmax[blk]);  // as conv_encoder_body
#pragma unroll
        for (int t = 0; t < R; ++t) {
          const float rstd = 1.0f / sqrtf(var[t] * (1.0f / 8192.0f) + 1e-5f);
#pragma unroll
          for (int n = 0; n < N; ++n) {
            const float gw = ed.gn_w[blk * 256 + col0 + 32 * n], gb = ed.gn_b[blk * 256 + col0 + 32 * n];
            const float sc = rstd * gw, sh = gb - mean[t] * sc;
            floatx16 v;
#pragma unroll
            for (int r = 0; r < 16; r += 2) {
              const floatx2 y =
                  __builtin_elementwise_fma((floatx2){acc.c[t][n][r], acc.c[t][n][r + 1]}, (floatx2)sc, (floatx2)sh);
              v[r] = y.x;
              v[r + 1] = y.y;
            }
            res_set(t, n, v);
            store_tile(v, t, n, ex);
          }
          xexp[t] = ex;
        }
      }
      __syncthreads();
      STAMP(5 + (blk * 2 + cv) * 2);
    }
  }

  // ---------------- proj: Linear(256 -> 256, no bias)
  acc.zero();
  run_stream1<PFW>(acc, reinterpret_cast<const char*>(ed.proj), 16, loff, afn_rows);
  STAMP(20);
#pragma unroll
  for (int t = 0; t < R; ++t) {
    const int win = win0 + t;
    if (win < n_windows) {
      float* o = enc_out + ((size_t)e * n_windows * VGE_T + (size_t)win * VGE_T) * VGE_D;
#pragma unroll
      for (int n = 0; n < N; ++n) {
        const float xs = ldexpf(1.0f, xexp[t]) * ed.cs[9 * 256 + col0 + 32 * n];
#pragma unroll
        for (int r = 0; r < 16; ++r) o[crow(0, r) * VGE_D + col0 + 32 * n] = acc.c[t][n][r] * xs;
      }
    }
  }
  STAMP(21);
#ifdef VGE_TRACE
  if (tr_on && blockIdx.x < 64 && threadIdx.x == 0) {
    g_vge_trace[blockIdx.x * 8 * 32 + 31] = e;
    g_vge_trace[blockIdx.x * 8 * 32 + 30] = W;
  }
#endif
}

// Pure fp16 mode (VGE_F16 with nothing split): one 512-thread workgroup per CU (8 waves, wave w = columns 32w..32w+31
// of all rows), units of 1..6 windows of one encoder from a table (conv_f16w_schedule; built on the device by
// conv_f16w_table_kernel), run by
// conv_f16w_body.  The weight stream is paid per unit (~28.5 k cycles per conv whatever the unit's rows), so the
// number of units per CU is what sets the time: at 256 windows every CU runs two units (quint + quint, or hex +
// quad; 10 windows) instead of the quad kernel's three (quad + quad + pair).  Measured (256 / 4,096 windows):
// 0.61 / 8.07 ms against 0.745 / 10.55 ms for conv_encoder_x3_kernel<false, false>.  Measured and dropped: the same
// body on 4 waves (one per SIMD, accumulators in AGPRs, at most 5 windows: the hex spills) -- 0.65-0.67 / 9.5 ms.
// Table entry: encoder | W << 4 | first window << 8, -1 = idle; [round][position], position = xcd_remap(block).
constexpr int F16W_MAX = 6;  // windows per unit

constexpr int F16W_WAVES = 8;

__global__ void __launch_bounds__(512, 1) conv_encoder_f16w_kernel(const float* __restrict__ feats,
                                                                    const EncDescX3* __restrict__ encs, int n_windows,
                                                                    int G, int n_rounds, const int* __restrict__ units,
                                                                    float* __restrict__ enc_out) {
  extern __shared__ __attribute__((aligned(16))) char lds_raw[];
  const int pos = xcd_remap(blockIdx.x, G);
  for (int round = 0; round < n_rounds; ++round) {
    const int u = __builtin_amdgcn_readfirstlane(units[round * G + pos]);
    if (u < 0) continue;  // uniform over the block
    if (round > 0) __syncthreads();  // the previous unit's LDS is free
    const int e = u & 15, w = (u >> 4) & 7, w0 = u >> 8;
#ifdef VGE_F16W_ONLY  // register-pressure probes: one instantiation only
    conv_f16w_body<VGE_F16W_ONLY, F16W_WAVES>(feats, n_windows, w0, encs[e], e, enc_out, lds_raw, round == VGE_TRACE_ROUND);
    (void)w;
#else
    switch (w) {
      case 6: conv_f16w_body<6, F16W_WAVES>(feats, n_windows, w0, encs[e], e, enc_out, lds_raw, round == VGE_TRACE_ROUND); break;
      case 5: conv_f16w_body<5, F16W_WAVES>(feats, n_windows, w0, encs[e], e, enc_out, lds_raw, round == VGE_TRACE_ROUND); break;
      case 4: conv_f16w_body<4, F16W_WAVES>(feats, n_windows, w0, encs[e], e, enc_out, lds_raw, round == VGE_TRACE_ROUND); break;
      case 3: conv_f16w_body<3, F16W_WAVES>(feats, n_windows, w0, encs[e], e, enc_out, lds_raw, round == VGE_TRACE_ROUND); break;
      case 2: conv_f16w_body<2, F16W_WAVES>(feats, n_windows, w0, encs[e], e, enc_out, lds_raw, round == VGE_TRACE_ROUND); break;
      default: conv_f16w_body<1, F16W_WAVES>(feats, n_windows, w0, encs[e], e, enc_out, lds_raw, round == VGE_TRACE_ROUND); break;
    }
#endif
  }
}

// ------------------------------------------------------------------ panel GEMM (3xfp16) with fused epilogues
enum Epi { EPI_TOKENS = 0, EPI_BIAS = 1, EPI_BIAS_RELU = 2, EPI_BIAS_RES_LN = 3 };

struct GemmArgsX3 {
  const float* A;  int lda;
  const _Float16* W;            // chunks [N/256][K/16][16 KB]
  float* out;      int ldo;
  int M, K, N;
  const float* bias;
  const float* res;  int ldr;
  const float* ln_w; const float* ln_b;
  const float* pe;
  const float* cls;
  const float* cs;              // [N] weight column scales
};

// block = 8 waves, BM = 32 RT rows x BN = 256 columns, wave w owns columns 32w..32w+31 of all BM rows.
// RT = 1: 32-row blocks, small enough (LDS 34 KB, <= 128 VGPRs) for several workgroups per CU, so one
// workgroup's staging / epilogue latency hides behind another's MFMAs on these short (K <= 1024) GEMMs.
constexpr int NWAVE = 8, GEMM_RT = 1;
template <int RT>
constexpr int gemm_lds_bytes() {
  return 2 * 32 * RT * XSB + (32 * RT * NWAVE + NWAVE) * 4;
}

template <int EPI, int RT>
__global__ void __launch_bounds__(512, 4) gemm_x3_kernel(GemmArgsX3 ga) {  // 4 waves per SIMD
  constexpr int BM = 32 * RT;
  extern __shared__ __attribute__((aligned(16))) char lds_raw[];
  _Float16* Xh = reinterpret_cast<_Float16*>(lds_raw);
  _Float16* Xl = Xh + BM * XS;
  float* red = reinterpret_cast<float*>(lds_raw + 2 * BM * XSB);  // [BM rows][8 waves] + [8] maxima
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int i = lane & 31, h = lane >> 5;
  const int row0 = blockIdx.x * BM, nb = blockIdx.y;
  const int n_panels = ga.K / 256;
  const unsigned loff = (unsigned)((h * 256 + wave * 32 + i) * 16);
  const char* xa = reinterpret_cast<const char*>(Xh) + i * XSB + h * 16;
  auto lrow = [&](int t, int r) { return t * 32 + (r & 3) + 8 * (r >> 2) + 4 * h; };

  Acc<RT, 1> acc;
  acc.zero();
  int aexp = 0;  // the accumulators hold C * 2^-aexp
  for (int p = 0; p < n_panels; ++p) {
    // the BM x 256 A panel (rows >= M read as 0) as hi/lo planes of panel * 2^-e, its largest |value| in
    // [2^8, 2^9): exact power-of-two scaling that keeps fp16 in range; the accumulators are rescaled to match
    const int c = tid & 255;
    float a[BM / 2];
    float m = 0.f;
#pragma unroll
    for (int j = 0; j < BM / 2; ++j) {
      const int row = row0 + (tid >> 8) + 2 * j;
      a[j] = (row < ga.M) ? ga.A[(size_t)row * ga.lda + p * 256 + c] : 0.f;
      m = fmaxf(m, fabsf(a[j]));
    }
    m = wave_max_last(m);
    if (lane == 63) red[BM * NWAVE + wave] = m;
    __syncthreads();  // also: every wave is past the previous panel's stream
    float mm = red[BM * NWAVE];
#pragma unroll
    for (int w = 1; w < NWAVE; ++w) mm = fmaxf(mm, red[BM * NWAVE + w]);
    const int e = fp16_range_exp(mm);
    if (p > 0 && e != aexp) {
      const float f = ldexpf(1.0f, aexp - e);
#pragma unroll
      for (int t = 0; t < RT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc.c[t][0][r] *= f;
    }
    aexp = e;
#pragma unroll
    for (int j = 0; j < BM / 2; ++j) {
      const int r = (tid >> 8) + 2 * j;
      split_store(Xh + r * XS + c, Xl + r * XS + c, ldexpf(a[j], -e));
    }
    __syncthreads();
    auto afn = [&](int cc, AFrag<RT>& f) {
#pragma unroll
      for (int t = 0; t < RT; ++t) {
        const char* q = xa + t * 32 * XSB + cc * 32;
        f.h[t] = *reinterpret_cast<const half8*>(q);
        f.l[t] = *reinterpret_cast<const half8*>(q + BM * XSB);
      }
    };
    run_stream<GEMM_PF>(acc, reinterpret_cast<const char*>(ga.W) + ((size_t)nb * (ga.K / 16) + p * 16) * CHUNK_B, 16,
                        loff, afn);
    __syncthreads();  // every wave is done reading the panel
  }

  const int col = nb * 256 + wave * 32 + i;
  float v[RT][16];
  const float as = ldexpf(1.0f, aexp) * ga.cs[col];
#pragma unroll
  for (int t = 0; t < RT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) v[t][r] = acc.c[t][0][r] * as;

  if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_RELU) {
    const float bb = ga.bias[col];
#pragma unroll
    for (int t = 0; t < RT; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = row0 + lrow(t, r);
        float x = v[t][r] + bb;
        if (EPI == EPI_BIAS_RELU) x = fmaxf(x, 0.f);
        if (row < ga.M) ga.out[(size_t)row * ga.ldo + col] = x;
      }
  } else if constexpr (EPI == EPI_TOKENS) {
#pragma unroll
    for (int t = 0; t < RT; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = row0 + lrow(t, r);
        if (row < ga.M) {
          const int w = row >> 5, tt = row & 31;
          ga.out[((size_t)w * VGE_TOK + 1 + tt) * ga.ldo + col] = v[t][r] + ga.pe[(1 + tt) * VGE_D + col];
          if (tt == 0) ga.out[(size_t)w * VGE_TOK * ga.ldo + col] = ga.cls[col] + ga.pe[col];
        }
      }
  } else {  // EPI_BIAS_RES_LN over the 256 columns (N == 256, one column block), one 32-row tile at a time
    // the token buffers are padded to whole 64-row tiles (vge_encoder_reserve): rows past M read and write
    // that padding (never consumed; A staging zeroes them), so the epilogue needs no row guards
    const float bb = ga.bias[col], lw = ga.ln_w[col], lb = ga.ln_b[col];
    // row sums (in place): over the 32 lanes that share h (xor 1..16 stays inside a 32-lane half), then over
    // the 8 waves' column slices through LDS
    auto row_reduce = [&](float (&q)[16], int t) {
#pragma unroll
      for (int r = 0; r < 16; ++r) q[r] = half_sum_last(q[r]);  // valid in lanes 31 and 63
      if (i == 31) {
#pragma unroll
        for (int r = 0; r < 16; ++r) red[lrow(t, r) * NWAVE + wave] = q[r];
      }
      __syncthreads();
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float* rr = red + lrow(t, r) * NWAVE;
        float a = rr[0];
#pragma unroll
        for (int w = 1; w < NWAVE; ++w) a += rr[w];
        q[r] = a;
      }
      __syncthreads();  // every wave has read the partials before they are reused
    };
    auto tile = [&](float (&vt)[16], int t) {
      const float* rbase = ga.res + (size_t)(row0 + t * 32) * ga.ldr + col;
      float s[16], q[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        vt[r] += bb + rbase[lrow(0, r) * ga.ldr];
        s[r] = vt[r];
      }
      row_reduce(s, t);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        s[r] *= 1.0f / 256.0f;  // row means
        const float d = vt[r] - s[r];
        q[r] = d * d;
      }
      row_reduce(q, t);
      float* obase = ga.out + (size_t)(row0 + t * 32) * ga.ldo + col;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float rstd = 1.0f / sqrtf(q[r] * (1.0f / 256.0f) + 1e-5f);
        obase[lrow(0, r) * ga.ldo] = (vt[r] - s[r]) * rstd * lw + lb;
      }
    };
#pragma unroll
    for (int t = 0; t < RT; ++t) tile(v[t], t);
  }
}

// ------------------------------------------------------------------ fused FFN block (3xfp16)
// out = LN2(X1 + relu(X1 W1^T + b1) W2^T + b2)  (TransformerEncoderLayer post-norm FFN, model.py:145-146)
// for a 32-row block, with the 1024-wide hidden activation never leaving the CU: the hidden dimension is
// processed in 4 chunks of 256; each chunk's relu(X1 W1_chunk^T + b1) is split into LDS hi/lo planes and
// immediately multiplied into the running FFN2 accumulator (K panel = that chunk).
struct FfnArgsX3 {
  const float* X1;  // [M (padded to 64)][256] input, also the residual
  float* out;       // [M][256]
  int M;
  const _Float16* W1; const float* cs1; const float* b1;  // linear1 [1024][256]: 4 column blocks x 16 chunks
  const _Float16* W2; const float* cs2; const float* b2;  // linear2 [256][1024]: 64 chunks (4 K panels)
  const float* ln_w; const float* ln_b;
};

constexpr int FFN_LDS_BYTES = 4 * 32 * XSB + (32 * NWAVE + 2 * NWAVE) * 4;

__global__ void __launch_bounds__(512, 4) ffn_x3_kernel(FfnArgsX3 fa) {
  extern __shared__ __attribute__((aligned(16))) char lds_raw[];
  _Float16* Xh = reinterpret_cast<_Float16*>(lds_raw);
  _Float16* Xl = Xh + 32 * XS;
  _Float16* Hh = Xl + 32 * XS;  // Hl = Hh + 32 * XS
  float* red = reinterpret_cast<float*>(lds_raw + 4 * 32 * XSB);  // [32 rows][8 waves] + 2 x [8] maxima
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int i = lane & 31, h = lane >> 5;
  const int row0 = blockIdx.x * 32;
  const int col = wave * 32 + i;  // this lane's column of every 256-wide block
  const unsigned loff = (unsigned)((h * 256 + col) * 16);
  auto lrow = [&](int r) { return (r & 3) + 8 * (r >> 2) + 4 * h; };
  auto block_max = [&](float m, int slot) {  // over the 512 threads, every thread gets it
    m = wave_max_last(m);
    if (lane == 63) red[32 * NWAVE + slot * NWAVE + wave] = m;
    __syncthreads();
    float mm = red[32 * NWAVE + slot * NWAVE];
#pragma unroll
    for (int w = 1; w < NWAVE; ++w) mm = fmaxf(mm, red[32 * NWAVE + slot * NWAVE + w]);
    return mm;
  };

  // ---- X1 panel (32 x 256) as hi/lo planes of X1 * 2^-ex (exact)
  int ex;
  {
    const int c = tid & 255;
    float a[16];
    float m = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int row = row0 + (tid >> 8) + 2 * j;
      a[j] = (row < fa.M) ? fa.X1[(size_t)row * 256 + c] : 0.f;
      m = fmaxf(m, fabsf(a[j]));
    }
    ex = fp16_range_exp(block_max(m, 0));
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int r = (tid >> 8) + 2 * j;
      split_store(Xh + r * XS + c, Xl + r * XS + c, ldexpf(a[j], -ex));
    }
  }
  __syncthreads();
  const char* xa = reinterpret_cast<const char*>(Xh) + i * XSB + h * 16;
  const char* ha = reinterpret_cast<const char*>(Hh) + i * XSB + h * 16;
  auto afn_x = [&](int cc, AFrag<1>& f) {
    f.h[0] = *reinterpret_cast<const half8*>(xa + cc * 32);
    f.l[0] = *reinterpret_cast<const half8*>(xa + cc * 32 + 32 * XSB);
  };
  auto afn_h = [&](int cc, AFrag<1>& f) {
    f.h[0] = *reinterpret_cast<const half8*>(ha + cc * 32);
    f.l[0] = *reinterpret_cast<const half8*>(ha + cc * 32 + 32 * XSB);
  };
  char* hb = reinterpret_cast<char*>(Hh) + (4 * h * XS + col) * 2;  // this lane's H column, C-layout rows

  Acc<1, 1> acc2;
  acc2.zero();
  int hexp = 0;  // acc2 holds (H W2^T) * 2^-hexp
  for (int hc = 0; hc < 4; ++hc) {
    Acc<1, 1> acc1;
    acc1.zero();
    run_stream<GEMM_PF, 1>(acc1, reinterpret_cast<const char*>(fa.W1) + (size_t)hc * 16 * CHUNK_B, 16, loff, afn_x);
    // hidden chunk: relu(acc1 * 2^ex * cs1 + b1)
    const float s1 = ldexpf(1.0f, ex) * fa.cs1[hc * 256 + col], bb = fa.b1[hc * 256 + col];
    float v[16];
    float m = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      v[r] = fmaxf(acc1.c[0][0][r] * s1 + bb, 0.f);
      m = fmaxf(m, v[r]);
    }
    const int e = fp16_range_exp(block_max(m, 1));  // its barrier also retires the previous chunk's H reads
    if (hc > 0 && e != hexp) {
      const float f = ldexpf(1.0f, hexp - e);
#pragma unroll
      for (int r = 0; r < 16; ++r) acc2.c[0][0][r] *= f;
    }
    hexp = e;
    const float sc = ldexpf(1.0f, -e);
#pragma unroll
    for (int r = 0; r < 16; r += 2) {
      const floatx2 y = (floatx2){v[r], v[r + 1]} * sc;
      const _Float16 h0 = (_Float16)y.x, h1 = (_Float16)y.y;
      const floatx2 lo = y - (floatx2){(float)h0, (float)h1};
      const int off = ((r & 3) + 8 * (r >> 2)) * XSB;
      *reinterpret_cast<_Float16*>(hb + off) = h0;
      *reinterpret_cast<_Float16*>(hb + off + XSB) = h1;
      *reinterpret_cast<_Float16*>(hb + off + 32 * XSB) = (_Float16)lo.x;  // the Hl plane: 32 rows on
      *reinterpret_cast<_Float16*>(hb + off + XSB + 32 * XSB) = (_Float16)lo.y;
    }
    __syncthreads();
    run_stream<GEMM_PF, 1>(acc2, reinterpret_cast<const char*>(fa.W2) + (size_t)hc * 16 * CHUNK_B, 16, loff, afn_h);
  }

  // ---- epilogue: LN2(X1 + acc2 * 2^hexp * cs2 + b2), one row tile, no row guards (padded token buffers)
  const float s2 = ldexpf(1.0f, hexp) * fa.cs2[col], bb2 = fa.b2[col], lw = fa.ln_w[col], lb = fa.ln_b[col];
  const float* rbase = fa.X1 + (size_t)row0 * 256 + col;
  float vt[16], s[16], q[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    vt[r] = acc2.c[0][0][r] * s2 + bb2 + rbase[lrow(r) * 256];
    s[r] = vt[r];
  }
  auto row_reduce = [&](float (&x)[16]) {
#pragma unroll
    for (int r = 0; r < 16; ++r) x[r] = half_sum_last(x[r]);  // valid in lanes 31 and 63
    if (i == 31) {
#pragma unroll
      for (int r = 0; r < 16; ++r) red[lrow(r) * NWAVE + wave] = x[r];
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float* rr = red + lrow(r) * NWAVE;
      float a = rr[0];
#pragma unroll
      for (int w = 1; w < NWAVE; ++w) a += rr[w];
      x[r] = a;
    }
    __syncthreads();
  };
  row_reduce(s);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    s[r] *= 1.0f / 256.0f;
    const float d = vt[r] - s[r];
    q[r] = d * d;
  }
  row_reduce(q);
  float* obase = fa.out + (size_t)row0 * 256 + col;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const float rstd = 1.0f / sqrtf(q[r] * (1.0f / 256.0f) + 1e-5f);
    obase[lrow(r) * 256] = (vt[r] - s[r]) * rstd * lw + lb;
  }
}

// ------------------------------------------------------------------ weight packing (load time)
// Device twin of vge_api.cpp pack_linear_x3 (the host packer, kept as VGE_HOST_PACK=1): W[N][K] (or the conv
// weight [256][256][5] read as K = tap * 256 + ci) -> chunks [N/256][nch][plane 2][h 2][n 256][8] fp16 of
// w * 2^s_n, hi = f16(w'), lo = f16(w' - hi), with the column exponent s_n = min(8 - ilogb(max_k |w|), 100).
// Same operations in the same order as the host code (RNE conversions, exact ldexp), so the images are
// bit-identical (tests/test_gpu_parity.py compares them byte for byte).
__device__ __forceinline__ float pack_w(const float* __restrict__ W, int conv, int ldk, int n, int k) {
  return conv ? W[((size_t)n * 256 + (k & 255)) * 5 + (k >> 8)] : W[(size_t)n * ldk + k];
}

// one block per column: s_n and the column scale 2^-s_n; any non-finite weight raises *bad
__global__ void __launch_bounds__(256) pack_x3_colexp_kernel(const float* __restrict__ W, int K_real, int ldk, int conv,
                                                             int* __restrict__ sh, float* __restrict__ cs,
                                                             int* __restrict__ bad) {
  __shared__ float red[4];
  const int n = blockIdx.x, tid = threadIdx.x;
  float m = 0.f;
  bool nf = false;
  for (int k = tid; k < K_real; k += 256) {
    const float v = pack_w(W, conv, ldk, n, k);
    nf |= !isfinite(v);
    m = fmaxf(m, fabsf(v));  // NaN-ignoring like the host's std::max(m, |v|)
  }
  if (nf) *bad = 1;
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if ((tid & 63) == 0) red[tid >> 6] = m;
  __syncthreads();
  if (tid == 0) {
    m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    const int s = m > 0.f ? min(8 - ilogbf(m), 100) : 0;
    sh[n] = s;
    cs[n] = ldexpf(1.0f, -s);
  }
}

// one thread per (column block, chunk, h, column): 8 k-values -> one 16-B store per plane
__global__ void __launch_bounds__(256) pack_x3_kernel(const float* __restrict__ W, int N, int K_real, int ldk, int conv,
                                                      int nch, const int* __restrict__ sh, _Float16* __restrict__ out) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= (N / 256) * nch * 512) return;
  const int n = t & 255, h = (t >> 8) & 1, c = (t >> 9) % nch, nb = (t >> 9) / nch;
  const int col = nb * 256 + n, s = sh[col];
  half8 hi, lo;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = 16 * c + 8 * h + j;
    const float w = k < K_real ? ldexpf(pack_w(W, conv, ldk, col, k), s) : 0.0f;
    const _Float16 x = (_Float16)w;
    hi[j] = x;
    lo[j] = (_Float16)(w - (float)x);
  }
  _Float16* ch = out + ((size_t)nb * nch + c) * 8192;
  *reinterpret_cast<half8*>(ch + ((0 * 2 + h) * 256 + n) * 8) = hi;
  *reinterpret_cast<half8*>(ch + ((1 * 2 + h) * 256 + n) * 8) = lo;
}

}  // namespace

// ================================================================== host launchers
namespace vge {

static int conv_cu_count();

hipError_t launch_pack_x3(const float* W, int N, int K_real, int ldk, int conv, int nch, int* sh, float* cs, int* bad,
                          _Float16* out, hipStream_t s) {
  if (N % 256 || K_real < 1 || nch * 16 < K_real) return hipErrorInvalidValue;
  hipLaunchKernelGGL(pack_x3_colexp_kernel, dim3(N), dim3(256), 0, s, W, K_real, ldk, conv, sh, cs, bad);
  const int nt = (N / 256) * nch * 512;
  hipLaunchKernelGGL(pack_x3_kernel, dim3((nt + 255) / 256), dim3(256), 0, s, W, N, K_real, ldk, conv, nch, sh, out);
  return hipGetLastError();
}

struct EncDescX3Host {
  const _Float16* stem; const _Float16* conv; const _Float16* proj; const float* gn_w; const float* gn_b;
  const float* cs; const float* fold;
  int in_col, d_in, n_stem_panels, ld;
  float gn_gmax[4], gn_bmax[4];
};
static_assert(sizeof(EncDescX3Host) == sizeof(EncDescX3), "EncDescX3 layout");

struct GemmArgsX3Host {
  const float* A; int lda; const _Float16* W; float* out; int ldo; int M, K, N;
  const float* bias; const float* res; int ldr; const float* ln_w; const float* ln_b; const float* pe; const float* cls;
  const float* cs;
};
static_assert(sizeof(GemmArgsX3Host) == sizeof(GemmArgsX3), "GemmArgsX3 layout");

hipError_t encoder_x3_kernel_setup() {
  const void* ck[3] = {(const void*)conv_encoder_x3_kernel<true, true>, (const void*)conv_encoder_x3_kernel<false, true>,
                       (const void*)conv_encoder_x3_kernel<false, false>};
  hipError_t e = hipSuccess;
  for (auto k : ck) {
    e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, conv_lds_bytes<4, 8>());
    if (e != hipSuccess) return e;
  }
  e = hipFuncSetAttribute((const void*)conv_encoder_f16w_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                          conv_lds_bytes_max<F16W_WAVES, 1>());
  if (e != hipSuccess) return e;
  const void* gk[4] = {(const void*)gemm_x3_kernel<EPI_TOKENS, GEMM_RT>, (const void*)gemm_x3_kernel<EPI_BIAS, GEMM_RT>,
                       (const void*)gemm_x3_kernel<EPI_BIAS_RELU, GEMM_RT>,
                       (const void*)gemm_x3_kernel<EPI_BIAS_RES_LN, GEMM_RT>};
  for (auto k : gk) {
    e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, gemm_lds_bytes<GEMM_RT>());
    if (e != hipSuccess) return e;
  }
  return hipFuncSetAttribute((const void*)ffn_x3_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, FFN_LDS_BYTES);
}

// Quads (4 windows per block) halve the weight bytes per row; pairs fill the remainder.  With G = min(CUs,
// units) persistent blocks and m = ceil(pair units / G) per block, Q = G * floor(m / 2) quads (as many as
// fit) make every block run floor(m / 2) quads and at most one pair.
// split: 3xfp16 (VGE_F32X3); otherwise single fp16 with the stem split (stem_split) or not
// Quads per encoder: any split of Q with q_e <= n / 4 gives the same pair count (sum of ceil((n - 4 q_e) / 2)), so
// the split is chosen for the L2s and the balance.  When Q is a whole number K of XCD runs (G / 8 units; xcd_remap),
// the K runs go to the encoders whose stem is one K panel first, as many as each takes (n / 4 quads), then to the
// `heavy` ones (vit: a 4-panel stem), so every run of an XCD in a round is one encoder's and the heavy encoders'
// windows end up in the pairs, spread over all CUs instead of as a longer quad on some.  256 windows x 10 encoders on
// 256 CUs: the 8 light encoders take 64 quads each (two rounds), the two vit encoders 128 pairs each (the third
// round); every CU runs two quads and one vit pair; 24 encoder weight streams per launch against ~41 with nearly equal
// q_e.  Otherwise nearly equal q_e.
ConvSched conv_quad_sched(int n_windows, int n_enc, unsigned heavy) {
  const int n_cu = conv_cu_count();
  const int pair_units = n_enc * ((n_windows + 1) / 2);
  const int G0 = std::min(n_cu, pair_units);
  const int m = (pair_units + G0 - 1) / G0;
  const int Q = std::min(G0 * (m / 2), n_enc * (n_windows / 4));
  ConvSched cs;
  memset(&cs, 0, sizeof(cs));
  cs.n_windows = n_windows;
  cs.n_enc = std::min(n_enc, CONV_MAX_ENC);
  cs.Q = Q;
  int q[CONV_MAX_ENC];
  const int X = G0 % 8 == 0 ? G0 / 8 : 0, qmax = n_windows / 4;
  static const int align = [] {  // VGE_QUAD_ALIGN=0: nearly equal q_e always; 1: whole runs, heavy stems not
    const char* v = getenv("VGE_QUAD_ALIGN");  // preferred in the pairs (A/B of the L2 alignment and the stem split)
    return v ? atoi(v) : 2;
  }();
  if (align < 2) heavy = 0;
  bool whole = align && X > 0 && Q % X == 0;
  if (whole) {
    int K = Q / X;
    const int kmax = qmax / X;
    for (int pass = 0; pass < 2; ++pass) {  // light encoders, then heavy: nearly equal runs within each class
      int cls = 0;
      for (int e = 0; e < cs.n_enc; ++e) cls += ((heavy >> e) & 1) == (unsigned)pass;
      if (pass == 0) {
        for (int e = 0; e < cs.n_enc; ++e) q[e] = 0;
      }
      if (cls == 0) continue;
      const int take = std::min(K, cls * kmax);
      int j = 0;
      for (int e = 0; e < cs.n_enc; ++e)
        if (((heavy >> e) & 1) == (unsigned)pass) q[e] = X * (take / cls + (j++ < take % cls));
      K -= take;
    }
    whole = K == 0;
  }
  if (!whole)
    for (int e = 0; e < cs.n_enc; ++e) q[e] = Q / cs.n_enc + (e < Q % cs.n_enc);
  for (int e = 0; e < cs.n_enc; ++e) {
    cs.qpre[e + 1] = cs.qpre[e] + q[e];
    cs.ppre[e + 1] = cs.ppre[e] + (n_windows - 4 * q[e] + 1) / 2;
  }
  cs.n_units = Q + cs.ppre[cs.n_enc];
  cs.G = std::min(n_cu, cs.n_units);
  return cs;
}

hipError_t launch_conv_encoders_x3(const float* feats, int n_windows, const void* encs, int n_enc, unsigned heavy,
                                   float* enc_out, bool split, bool stem_split, hipStream_t s) {
  if (n_windows < 1 || n_enc < 1) return hipSuccess;
  const ConvSched cs = conv_quad_sched(n_windows, n_enc, heavy);
  auto k = split ? conv_encoder_x3_kernel<true, true>
                 : (stem_split ? conv_encoder_x3_kernel<false, true> : conv_encoder_x3_kernel<false, false>);
  hipLaunchKernelGGL(k, dim3(cs.G), dim3(512), (conv_lds_bytes<4, 8>()), s, feats,
                     reinterpret_cast<const EncDescX3*>(encs), cs, enc_out);
  return hipGetLastError();
}

static int conv_cu_count() {
  static int n_cu = 0;
  if (n_cu == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n_cu < 1)
      n_cu = 256;
  }
  return n_cu;
}

// Unit table of conv_encoder_f16w_kernel for n_windows x n_enc (window, encoder) pairs on G = min(CUs, units)
// persistent blocks and R rounds: the fewest rounds whose units fit wmax (<= F16W_MAX) windows; encoder e is cut into u_e
// nearly equal units of consecutive windows (u_e = U / n_enc, +1 for the first U % n_enc encoders).  The units,
// encoder-major, are sorted by size (largest first, stable: the same encoder's units stay together) and dealt in
// snake order over the positions (round 0 left to right, round 1 right to left, ...), so a position holding a
// large unit in one round holds a small one in the next and consecutive positions -- one XCD's CUs, xcd_remap -- run the same encoder's units together.
// Returns false if n_enc > 16 or n_windows > 2^23 (the entry's bit fields).
bool conv_f16w_schedule(int n_windows, int n_enc, int wmax, std::vector<int>& table, int& G, int& R) {
  if (n_windows < 1 || n_enc < 1 || n_enc > 16 || n_windows > (1 << 23)) return false;
  wmax = std::max(1, std::min(wmax, F16W_MAX));
  const long long P = (long long)n_windows * n_enc;
  const int n_cu = conv_cu_count();
  struct U { int e, w0, w; };
  std::vector<U> units;
  for (R = 1;; ++R) {
    const long long Ul = std::min<long long>((long long)n_cu * R, P);
    const int Ut = (int)Ul;
    units.clear();
    bool ok = true;
    for (int e = 0; e < n_enc && ok; ++e) {
      const int ue = std::min(n_windows, Ut / n_enc + (e < Ut % n_enc));
      if (ue < 1 || (n_windows + ue - 1) / ue > wmax) { ok = false; break; }
      for (int k = 0; k < ue; ++k) {
        const int a = (int)((long long)k * n_windows / ue), b = (int)((long long)(k + 1) * n_windows / ue);
        units.push_back({e, a, b - a});
      }
    }
    if (ok) break;
  }
  const int Ut = (int)units.size();
  G = std::min(n_cu, Ut);
  R = (Ut + G - 1) / G;
  std::stable_sort(units.begin(), units.end(), [](const U& x, const U& y) { return x.w > y.w; });
  table.assign((size_t)R * G, -1);
  for (int k = 0; k < Ut; ++k) {
    const int r = k / G, j = k % G, p = (r & 1) ? G - 1 - j : j;
    table[(size_t)r * G + p] = units[k].e | (units[k].w << 4) | (units[k].w0 << 8);
  }
  return true;
}

// The plan of conv_f16w_schedule without the table: grid G, rounds R and unit count U (upper bound of the table:
// R * G <= 10 * n_windows + CUs).
bool conv_f16w_plan(int n_windows, int n_enc, int wmax, int& G, int& R, int& U) {
  if (n_windows < 1 || n_enc < 1 || n_enc > 16 || n_windows > (1 << 23)) return false;
  wmax = std::max(1, std::min(wmax, F16W_MAX));
  const long long P = (long long)n_windows * n_enc;
  const int n_cu = conv_cu_count();
  for (R = 1;; ++R) {
    const int Ut = (int)std::min<long long>((long long)n_cu * R, P);
    bool ok = true;
    U = 0;
    for (int e = 0; e < n_enc && ok; ++e) {
      const int ue = std::min(n_windows, Ut / n_enc + (e < Ut % n_enc));
      ok = ue >= 1 && (n_windows + ue - 1) / ue <= wmax;
      U += ue;
    }
    if (ok) break;
  }
  G = std::min(n_cu, U);
  R = (U + G - 1) / G;
  return true;
}

}  // namespace vge
namespace {
// Device twin of conv_f16w_schedule's table (so vge_encode builds it without host round trips: capture-safe): the
// same units (encoder e cut into u_e nearly equal runs of q_e = n / u_e or q_e + 1 windows), the same stable order
// (size descending, then encoder-major, then run index), the same snake dealing.  One thread per unit computes its
// rank in closed form: of the first j runs of encoder e, floor(j n / u_e) - j q_e have q_e + 1 windows.
__global__ void __launch_bounds__(1024) conv_f16w_table_kernel(int n_windows, int n_enc, int G, int R, int U,
                                                               int* __restrict__ table) {
  for (int i = threadIdx.x; i < G * R; i += blockDim.x) table[i] = -1;
  __syncthreads();
  auto ue_of = [&](int e) { return min(n_windows, U / n_enc + (e < U % n_enc)); };
  auto count = [&](int e, int sz) {  // runs of encoder e with sz windows
    const int ue = ue_of(e), q = n_windows / ue, big = n_windows - q * ue;
    return sz == q + 1 ? big : (sz == q ? ue - big : 0);
  };
  for (int e = 0; e < n_enc; ++e) {
    const int ue = ue_of(e), q = n_windows / ue;
    for (int j = threadIdx.x; j < ue; j += blockDim.x) {
      const int a = (int)((long long)j * n_windows / ue), b = (int)((long long)(j + 1) * n_windows / ue);
      const int sz = b - a;
      int k = 0;
      for (int s2 = F16W_MAX; s2 > sz; --s2)
        for (int e2 = 0; e2 < n_enc; ++e2) k += count(e2, s2);
      for (int e2 = 0; e2 < e; ++e2) k += count(e2, sz);
      const int bigs = a - j * q;  // runs of q + 1 windows before run j
      k += sz == q + 1 ? bigs : j - bigs;
      const int r = k / G, p = k % G, pos = (r & 1) ? G - 1 - p : p;
      table[r * G + pos] = e | (sz << 4) | (a << 8);
    }
  }
}
}  // namespace
namespace vge {

hipError_t launch_conv_f16w_table(int n_windows, int n_enc, int G, int R, int U, int* d_table, hipStream_t s) {
  hipLaunchKernelGGL(conv_f16w_table_kernel, dim3(1), dim3(1024), 0, s, n_windows, n_enc, G, R, U, d_table);
  return hipGetLastError();
}

hipError_t launch_conv_encoders_f16w(const float* feats, int n_windows, const void* encs, float* enc_out,
                                     const int* d_units, int G, int R, hipStream_t s) {
  if (n_windows < 1) return hipSuccess;
  hipLaunchKernelGGL(conv_encoder_f16w_kernel, dim3(G), dim3(512), (conv_lds_bytes_max<F16W_WAVES, 1>()), s, feats,
                     reinterpret_cast<const EncDescX3*>(encs), n_windows, G, R, d_units, enc_out);
  return hipGetLastError();
}

hipError_t launch_gemm_x3(int epi, const GemmArgsX3Host& a, hipStream_t s) {
  GemmArgsX3 g;
  memcpy(&g, &a, sizeof(g));
  constexpr int BM = 32 * GEMM_RT, L = gemm_lds_bytes<GEMM_RT>();
  dim3 grid((a.M + BM - 1) / BM, a.N / 256);
  switch (epi) {
    case EPI_TOKENS: hipLaunchKernelGGL((gemm_x3_kernel<EPI_TOKENS, GEMM_RT>), grid, dim3(512), L, s, g); break;
    case EPI_BIAS: hipLaunchKernelGGL((gemm_x3_kernel<EPI_BIAS, GEMM_RT>), grid, dim3(512), L, s, g); break;
    case EPI_BIAS_RELU: hipLaunchKernelGGL((gemm_x3_kernel<EPI_BIAS_RELU, GEMM_RT>), grid, dim3(512), L, s, g); break;
    default: hipLaunchKernelGGL((gemm_x3_kernel<EPI_BIAS_RES_LN, GEMM_RT>), grid, dim3(512), L, s, g); break;
  }
  return hipGetLastError();
}

struct FfnArgsX3Host {
  const float* X1; float* out; int M;
  const _Float16* W1; const float* cs1; const float* b1;
  const _Float16* W2; const float* cs2; const float* b2;
  const float* ln_w; const float* ln_b;
};
static_assert(sizeof(FfnArgsX3Host) == sizeof(FfnArgsX3), "FfnArgsX3 layout");

hipError_t launch_ffn_x3(const FfnArgsX3Host& a, hipStream_t s) {
  FfnArgsX3 f;
  memcpy(&f, &a, sizeof(f));
  hipLaunchKernelGGL(ffn_x3_kernel, dim3((a.M + 31) / 32), dim3(512), FFN_LDS_BYTES, s, f);
  return hipGetLastError();
}

}  // namespace vge

// Test hook (host only, tests/test_lib_abi.py): the f16w unit table for n_windows x 10 encoders, n_cu CUs.
extern "C" int vge_debug_conv_schedule(int n_windows, int wmax, int* table, int cap, int* G, int* R) {
  std::vector<int> t;
  if (!vge::conv_f16w_schedule(n_windows, 10, wmax, t, *G, *R) || (int)t.size() > cap) return -1;
  std::copy(t.begin(), t.end(), table);
  return (int)t.size();
}

// Test hook (host only, tests/test_lib_abi.py): the quad / pair schedule of n_windows x n_enc, as the kernels read it
// (conv_unit on xcd_remap'd positions): units[3 (round * G + block) + {0, 1, 2}] = encoder, first window, windows
// (-1 for an idle slot); heavy: the multi-panel-stem encoder mask.  Returns the entry count (rounds x G) and G.
extern "C" int vge_debug_quad_schedule(int n_windows, int n_enc, unsigned heavy, int* units, int cap, int* G) {
  if (n_windows < 1 || n_enc < 1 || n_enc > vge::CONV_MAX_ENC) return -1;
  const vge::ConvSched cs = vge::conv_quad_sched(n_windows, n_enc, heavy);
  const int R = (cs.n_units + cs.G - 1) / cs.G;
  if (R * cs.G > cap) return -1;
  for (int r = 0; r < R; ++r)
    for (int b = 0; b < cs.G; ++b) {
      int* o = units + 3 * (r * cs.G + b);
      const int u = r * cs.G + xcd_remap(b, cs.G);
      int e = -1, w0 = -1;
      o[2] = u < cs.n_units ? (conv_unit(cs, u, e, w0) ? 4 : 2) : -1;
      o[0] = e;
      o[1] = w0;
    }
  *G = cs.G;
  return R * cs.G;
}

#ifdef VGE_TRACE
extern "C" int vge_debug_x3_trace(long long* host, int n) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_vge_trace), sizeof(long long) * (size_t)n);
}
#endif
