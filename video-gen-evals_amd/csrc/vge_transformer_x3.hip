// Fused split-precision transformer (gfx950): for ONE window per workgroup, on chip end to end,
//   tokens      X = [cls + pe_0 ; pooled Wov^T + pe_1..32]                   (model.py:79-98 fold, 187-188)
//   4 x layer   X = LN2(X1 + W2 relu(W1 X1 + b1) + b2),  X1 = LN1(X + Wo MHA(X) + bo)   (model.py:145-146,
//               nn.TransformerEncoderLayer post-norm, 8 heads of 32, FFN 1024, ReLU, LN eps 1e-5)
//   outputs     seq = normalize(X_0), frame = normalize(X_t), tc = mean_t |f_{t+1} - f_t|  (model.py:190-193,
//               eval.py:209-226)
// Rows: the 32 frame tokens are one 32-row MFMA tile; the CLS token (row 0) is computed beside it on the
// VALU (v_dot2_f32_f16 over the same B fragments, same hi/lo split), so no MFMA work is spent on padding.
// 4 waves (one per SIMD, 512 registers each: nothing spills), wave w owns output columns 64w..64w+63 of
// every 256-wide block (two 32-column MFMA tiles) and attention heads 2w, 2w+1.  All weights of the
// whole transformer are ONE continuous stream of 16 KB chunks (token 16, per layer QKV 48 + out 16 +
// FFN 128) in "segments" of 16 chunks: each wave keeps its B fragments PF chunks ahead in registers across
// segment boundaries, so the loads of the next weights are in flight during a segment's epilogue (bias,
// attention, LayerNorm, ReLU, the next A operand's split store).  Same 3xfp16 arithmetic as
// vge_encoder_x3.hip; weight chunks as packed by pack_linear_x3 (vge_api.cpp).
#include "vge_x3.h"
#include <cstdlib>
#include <cstring>

#ifdef VGE_TRACE  // timing-only builds (tools/trace_transformer.py): s_memtime stamps, every wave of blocks 0..63
__device__ long long g_vge_tx_trace[64 * 4 * 128];
#define TSTAMP(k)                                                                                       \
  do {                                                                                                  \
    if (blockIdx.x < 64 && (threadIdx.x & 63) == 0)                                                     \
      g_vge_tx_trace[(blockIdx.x * 4 + (threadIdx.x >> 6)) * 128 + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define TSTAMP(k) \
  do {            \
  } while (0)
#endif

namespace {

constexpr int TX_MAX_LAYERS = 8;

struct TxLayerX3 {
  const _Float16* in_w;  const float* in_cs; const float* in_b;     // in_proj [768][256]: 3 col blocks x 16
  const _Float16* out_w; const float* out_cs; const float* out_b;   // out_proj [256][256]: 16 chunks
  const float* n1_w; const float* n1_b;
  const _Float16* l1_w; const float* l1_cs; const float* l1_b;      // linear1 [1024][256]: 4 col blocks x 16
  const _Float16* l2_w; const float* l2_cs; const float* l2_b;      // linear2 [256][1024]: 4 K panels x 16
  const float* n2_w; const float* n2_b;
  int e_x1, e_x2, e_h, pad;  // static split exponents: LN1 / LN2 outputs, FFN hidden (host: range bounds)
};

struct TxArgsX3 {  // by value: the layer table is kernel-argument memory (scalar loads, no vmcnt waits)
  const float* pooled;  // [B*32][256] fused per-frame vectors (fuse_kernel)
  int n_windows, n_layers;
  const _Float16* ov_w; const float* ov_cs;  // Wov = Wo Wv of the fusion (16 chunks)
  const float* cls; const float* pe;         // [256], [33][256]
  float* seq; float* frame; float* tc;       // [B][256], [B][33][256] | null, [B] | null
  TxLayerX3 layers[TX_MAX_LAYERS];
};

constexpr int TOK = 33;          // CLS + 32 frames
constexpr int AROWS = TOK;       // rows of an A operand plane
constexpr int QS = 260;          // f32 row stride of the final-embedding staging (bank shift)
constexpr int QH = 36;           // f32 row stride of a wave's one-head Q / K / V staging (conflict-free b128 rows)
#ifndef VGE_TX_PF
#define VGE_TX_PF 4
#endif
constexpr int TX_PF = VGE_TX_PF;  // weight chunks in flight per wave (ring depth)
static_assert(16 % TX_PF == 0, "ring slots restart per 16-chunk segment: the depth must divide 16");
constexpr int TX_NW = 4;         // waves
template <bool SPA>
constexpr int ap_bytes() { return (SPA ? 2 : 1) * AROWS * XSB; }  // hi (/ lo) planes of one window's A operand
constexpr int HEAD_BYTES = 3 * TOK * QH * 4;         // one wave's Q, K, V of one head (f32)
constexpr int F_BYTES = TOK * QS * 4;                // one window's final embeddings (f32)
// U (the union): the 4 waves' head staging | W windows' FFN hidden planes | W windows' final embeddings
template <int W, bool SPA>
constexpr int tx_u_bytes() {
  constexpr int a = TX_NW * HEAD_BYTES, b = W * ap_bytes<SPA>(), c = W * F_BYTES;
  return a > b ? (a > c ? a : c) : (b > c ? b : c);
}
template <int W>
constexpr int tx_red_floats() {  // row partials x2, block maxima x2, tc
  return 2 * W * TOK * TX_NW + 2 * W * TX_NW + W * TX_NW;
}
template <int W, bool SPA>
constexpr int tx_lds_bytes() {
  return W * ap_bytes<SPA>() + tx_u_bytes<W, SPA>() + tx_red_floats<W>() * 4;
}
static_assert(tx_lds_bytes<2, true>() <= 160 * 1024, "LDS");
// single fp16 (no lo planes), one window: two workgroups fit a CU's LDS, so one's epilogues can run beside the
// other's weight stream (OCC = 2: 256 registers per wave)
static_assert(2 * tx_lds_bytes<1, false>() <= 160 * 1024, "LDS, two single-fp16 workgroups per CU");

// CLS rows: W = 1 on the VALU (v_dot2_f32_f16 over the same B fragments, same split products), so no MFMA work is
// spent on a mostly empty tile; W = 2 as one extra MFMA tile holding both windows' CLS rows (rows 0, 1): two windows'
// dot products would cost the VALU ~2x the MFMA time of the tile (8-cycle v_dot2, measured: 700 k vs 400 k stream
// cycles per window pair)
#ifndef VGE_TX_CLSM1
#define VGE_TX_CLSM1 0  // 1: the CLS row on an MFMA tile at W = 1 too (measured: 0.303 -> 0.325 ms at 256 windows)
#endif
template <int W>
constexpr bool tx_cls_mfma() { return W >= 2 || VGE_TX_CLSM1; }
template <int W>
struct AFragT {  // one chunk's A operands of W windows: the 32 frame rows and the CLS row(s)
  static constexpr int NC = tx_cls_mfma<W>() ? 1 : W;
  half8 h[W], l[W], h0[NC], l0[NC];
};

// CLS row on the VALU: c += x . w over this lane's 8 k of the chunk, the same 3 products as the MFMAs, in TX_CLS_NC
// independent partial sums (k pairs p -> sum p % NC): dependent v_dot2 chains of 12 / NC instead of 12, so the dots
// of a chunk finish while its MFMAs run
#ifndef VGE_TX_CLS_NC
#define VGE_TX_CLS_NC 1
#endif
constexpr int TX_CLS_NC = VGE_TX_CLS_NC;
template <bool SPA, bool SPW>
__device__ __forceinline__ void cls_dot(float (&c)[TX_CLS_NC], half8 xh, half8 xl, half8 wh, half8 wl) {
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    float& cp = c[p % TX_CLS_NC];
    const half2v a = {xh[2 * p], xh[2 * p + 1]};
    const half2v b = {wh[2 * p], wh[2 * p + 1]};
    if constexpr (SPA) {
      const half2v al = {xl[2 * p], xl[2 * p + 1]};
      cp = __builtin_amdgcn_fdot2(al, b, cp, false);
    }
    if constexpr (SPW) {
      const half2v bl = {wl[2 * p], wl[2 * p + 1]};
      cp = __builtin_amdgcn_fdot2(a, bl, cp, false);
    }
    cp = __builtin_amdgcn_fdot2(a, b, cp, false);
  }
}
__device__ __forceinline__ float cls_total(const float (&c)[TX_CLS_NC]) {
  float t = c[0];
#pragma unroll
  for (int k = 1; k < TX_CLS_NC; ++k) t += c[k];
  return t;
}

// SPA / SPW: activations / weights carried as hi + lo fp16 planes.  Both: 3xfp16 (VGE_F32X3, hi*hi + hi*lo +
// lo*hi); neither: single fp16, one MFMA per product; SPA only: (hi_a + lo_a) * hi_w, two MFMAs on the fp16 weight
// stream (half the bytes of the split).
// W windows per workgroup share every weight chunk a wave loads (W x 2 MFMA tiles per chunk): W = 2 when there are
// more windows than CUs.  A wave's Q / K / V columns are exactly its own two heads (2 wave + {0, 1}), so Q and K
// wait in registers for V and each head's attention stages only its own Q / K / V (14 KB per wave) in LDS: the
// windows' A planes and hidden planes (70 KB each at W = 2) then fit beside it.
template <bool SPA, bool SPW, int W, int OCC = 1>
__global__ void __launch_bounds__(256, OCC) transformer_x3_kernel(TxArgsX3 ta) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  constexpr int AP_BYTES = ap_bytes<SPA>();
  char* Ap = lds;                                   // [W] A planes: hi rows [0, AROWS), lo at + AROWS * XSB
  char* U = lds + W * AP_BYTES;                     // head staging | [W] hidden planes | [W] embeddings
  float* red = reinterpret_cast<float*>(U + tx_u_bytes<W, SPA>());  // [2][W][TOK][4] rows, [2][W][4] maxima, [W][4] tc
  // consecutive reductions alternate between two buffers, so none needs a trailing barrier: the writes of
  // reduction k + 2 come after reduction k + 1's barrier, which every read of reduction k precedes
  int rs_buf = 0, bm_buf = 0;
  [[maybe_unused]] int tr_s = -1;  // VGE_TRACE: the current segment, for the fine stamps of layer 0's epilogues
#ifdef VGE_TRACE
#define TSTAMP_FINE(k) do { if (tr_s == 4) TSTAMP(100 + (k)); else if (tr_s == 12) TSTAMP(110 + (k)); } while (0)
#else
#define TSTAMP_FINE(k) do { } while (0)
#endif
  const int wb0 = blockIdx.x * W;                   // first window of the block
  const int nv = min(W, ta.n_windows - wb0);        // its windows (the last block may hold fewer)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  int i = lane & 31, h = lane >> 5;
  int col0 = wave * 64 + i;                         // this lane's columns: col0 + 32 n, n = 0, 1
  const unsigned loff = (unsigned)((h * 256 + col0) * 16);
  // token row held in C-layout register r (the MFMA tile covers tokens 1..32; token 0 = CLS is `x0`)
  auto trow = [&](int r) { return 1 + (r & 3) + 8 * (r >> 2) + 4 * h; };
  const unsigned aoff = (unsigned)((1 + i) * XSB + h * 16), aoff0 = (unsigned)(h * 16);

  // ---- helpers (all W windows at once: one barrier per reduction) ------------------------------------------
  auto block_max = [&](float (&m)[W]) {  // in place: the workgroup max of each window's m
    float* rb = red + 2 * W * TOK * TX_NW + bm_buf * W * TX_NW;
    bm_buf ^= 1;
#pragma unroll
    for (int v = 0; v < W; ++v) {
      const float mv = wave_max_last(m[v]);
      if (lane == 63) rb[v * TX_NW + wave] = mv;
    }
    __syncthreads();
#pragma unroll
    for (int v = 0; v < W; ++v) {
      const floatx4 p = *reinterpret_cast<const floatx4*>(rb + v * TX_NW);
      m[v] = fmaxf(fmaxf(p[0], p[1]), fmaxf(p[2], p[3]));
    }
  };
  // row sums over the 256 columns, in place: x (token rows trow(r), both column tiles get the row sum),
  // x0 (CLS; the same value in both lane halves)
  auto row_sums = [&](float (&x)[W][2][16], float (&x0)[W][2]) {
    float* rb = red + rs_buf * W * TOK * TX_NW;
    rs_buf ^= 1;
#pragma unroll
    for (int v = 0; v < W; ++v) {
      float y[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) y[r] = half_sum_last(x[v][0][r] + x[v][1][r]);  // valid in lanes 31 and 63
      const float y0 = half_sum_last(x0[v][0] + x0[v][1]);
      if (i == 31) {
#pragma unroll
        for (int r = 0; r < 16; ++r) rb[(v * TOK + trow(r)) * TX_NW + wave] = y[r];
        if (h == 0) rb[v * TOK * TX_NW + wave] = y0;
      }
    }
    __syncthreads();
    auto sum4 = [&](int v, int row) {
      const floatx4 a = *reinterpret_cast<const floatx4*>(rb + (v * TOK + row) * TX_NW);
      return (a[0] + a[1]) + (a[2] + a[3]);
    };
#pragma unroll
    for (int v = 0; v < W; ++v) {
#pragma unroll
      for (int r = 0; r < 16; ++r) x[v][0][r] = x[v][1][r] = sum4(v, trow(r));
      x0[v][0] = x0[v][1] = sum4(v, 0);
    }
  };
  // LayerNorm over 256 columns (in place), affine w, b [256], eps 1e-5
  auto layer_norm = [&](float (&vv)[W][2][16], float (&v0)[W][2], const float (&lw)[2], const float (&lb)[2]) {
    float s[W][2][16], s0[W][2];
#pragma unroll
    for (int v = 0; v < W; ++v)
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        s0[v][n] = v0[v][n];
#pragma unroll
        for (int r = 0; r < 16; ++r) s[v][n][r] = vv[v][n][r];
      }
    TSTAMP_FINE(1);
    row_sums(s, s0);
    TSTAMP_FINE(2);
    float q[W][2][16], q0[W][2];
#pragma unroll
    for (int v = 0; v < W; ++v)
#pragma unroll
      for (int n = 0; n < 2; ++n) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          s[v][n][r] *= 1.0f / 256.0f;
          const float d = vv[v][n][r] - s[v][n][r];
          q[v][n][r] = d * d;
        }
        s0[v][n] *= 1.0f / 256.0f;
        q0[v][n] = (v0[v][n] - s0[v][n]) * (v0[v][n] - s0[v][n]);
      }
    row_sums(q, q0);
    TSTAMP_FINE(3);
    // 1 / sqrt(var + eps) once per row (v_rsq_f32, ~1 ulp; the IEEE sqrt + divide sequences cost ~50
    // instructions per value)
#pragma unroll
    for (int v = 0; v < W; ++v) {
      float rstd[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) rstd[r] = __builtin_amdgcn_rsqf(q[v][0][r] * (1.0f / 256.0f) + 1e-5f);
      const float rstd0 = __builtin_amdgcn_rsqf(q0[v][0] * (1.0f / 256.0f) + 1e-5f);
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const float gw = lw[n], gb = lb[n];
#pragma unroll
        for (int r = 0; r < 16; ++r) vv[v][n][r] = (vv[v][n][r] - s[v][n][r]) * rstd[r] * gw + gb;
        v0[v][n] = (v0[v][n] - s0[v][n]) * rstd0 * gw + gb;
      }
    }
  };
  // split one window's rows into hi/lo planes at `plane` as v * 2^-e (no barrier: the caller orders the writes
  // after every read of the planes' previous content and barriers before they are read)
  auto split_rows_e = [&](char* plane, const float (&v)[2][16], const float (&v0)[2], int e) {
    const float sc = ldexpf(1.0f, -e);
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      char* bh = plane + ((1 + 4 * h) * XS + col0 + 32 * n) * 2;
#pragma unroll
      for (int r = 0; r < 16; r += 2) {  // two rows per packed conversion (v_cvt_pk_f16_f32)
        const floatx2 y = floatx2{v[n][r], v[n][r + 1]} * sc;
        const half2v hi = __builtin_convertvector(y, half2v);
        const half2v lo = __builtin_convertvector(y - __builtin_convertvector(hi, floatx2), half2v);
        const int off = ((r & 3) + 8 * (r >> 2)) * XSB;
        *reinterpret_cast<_Float16*>(bh + off) = hi[0];
        *reinterpret_cast<_Float16*>(bh + off + XSB) = hi[1];
        if constexpr (SPA) {
          *reinterpret_cast<_Float16*>(bh + off + AROWS * XSB) = lo[0];
          *reinterpret_cast<_Float16*>(bh + off + XSB + AROWS * XSB) = lo[1];
        }
      }
      if (h == 0) {
        const float y = v0[n] * sc;
        const _Float16 hi = (_Float16)y;
        reinterpret_cast<_Float16*>(plane)[col0 + 32 * n] = hi;
        if constexpr (SPA) reinterpret_cast<_Float16*>(plane + AROWS * XSB)[col0 + 32 * n] = (_Float16)(y - (float)hi);
      }
    }
  };
  // every window's rows with its own exponent from the workgroup-wide max |v| (the barrier inside also retires
  // every read of the planes' previous content issued before it)
  auto split_rows = [&](char* plane, const float (&v)[W][2][16], const float (&v0)[W][2], int (&ex)[W]) {
    float m[W];
#pragma unroll
    for (int w = 0; w < W; ++w) {
      m[w] = fmaxf(fabsf(v0[w][0]), fabsf(v0[w][1]));
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int r = 0; r < 16; ++r) m[w] = fmaxf(m[w], fabsf(v[w][n][r]));
    }
    block_max(m);
#pragma unroll
    for (int w = 0; w < W; ++w) {
      ex[w] = fp16_range_exp(m[w]);
      split_rows_e(plane + w * AP_BYTES, v[w], v0[w], ex[w]);
    }
  };

  TSTAMP(124);
  // ---- token A operands: row 0 zero (the CLS token is not a product), rows 1..32 the window's pooled frames
#pragma unroll
  for (int v = 0; v < W; ++v) {
    reinterpret_cast<_Float16*>(Ap + v * AP_BYTES)[tid] = (_Float16)0.0f;
    if constexpr (SPA) reinterpret_cast<_Float16*>(Ap + v * AP_BYTES + AROWS * XSB)[tid] = (_Float16)0.0f;
  }
  int ax[W];  // the accumulators of the current segment hold (A_v * 2^-ax[v]) W
  {
    float a[W][32];
    float m[W];
#pragma unroll
    for (int v = 0; v < W; ++v) {
      m[v] = 0.f;
      const float* src = ta.pooled + (size_t)(wb0 + v) * 32 * 256 + tid;
#pragma unroll
      for (int j = 0; j < 32; ++j) {
        a[v][j] = v < nv ? src[j * 256] : 0.f;
        m[v] = fmaxf(m[v], fabsf(a[v][j]));
      }
    }
    block_max(m);
#pragma unroll
    for (int v = 0; v < W; ++v) {
      ax[v] = fp16_range_exp(m[v]);
      char* P = Ap + v * AP_BYTES;
#pragma unroll
      for (int j = 0; j < 32; ++j) {
        if constexpr (SPA)
          split_store(reinterpret_cast<_Float16*>(P + (1 + j) * XSB) + tid,
                      reinterpret_cast<_Float16*>(P + (AROWS + 1 + j) * XSB) + tid, ldexpf(a[v][j], -ax[v]));
        else
          reinterpret_cast<_Float16*>(P + (1 + j) * XSB)[tid] = (_Float16)ldexpf(a[v][j], -ax[v]);
      }
    }
  }
  __syncthreads();

  // ---- the segment stream -----------------------------------------------------------------------------
  // Segments (16 chunks each): tokens; per layer in_proj 0..2, out_proj, then linear1 / linear2 panel pairs.
  // in_proj's 768 outputs are packed in the order (vge_encoder_create) that makes wave w's two 32-column tiles
  //   in_proj 0: q, k of head 2w;   in_proj 1: v of head 2w, q of head 2w + 1;   in_proj 2: k, v of head 2w + 1
  // so head 2w's attention runs after in_proj 1 and only one head's q waits in registers.  The segments are
  // straight-line code per layer (not one loop over a segment index): what waits in registers between two
  // segments is then live only there.
  const int nseg = 1 + 12 * ta.n_layers;
  auto seg_base = [&](int s) -> gchar {
#if VGE_ABL & 32
    return (gchar)ta.ov_w;  // timing ablation: every segment re-reads the 256 KB token matrix (L2 resident)
#endif
    if (s >= nseg) s = nseg - 1;  // (the last segment's ring refill re-reads its own chunks)
    if (s == 0) return (gchar)ta.ov_w;
    const TxLayerX3& L = ta.layers[(s - 1) / 12];
    const int p = (s - 1) % 12;
    if (p < 3) return (gchar)L.in_w + (size_t)p * 16 * CHUNK_B;
    if (p == 3) return (gchar)L.out_w;
    const int hc = (p - 4) >> 1;
    return ((p - 4) & 1) ? (gchar)L.l2_w + (size_t)hc * 16 * CHUNK_B : (gchar)L.l1_w + (size_t)hc * 16 * CHUNK_B;
  };

  Acc<1, 2> acc[W], acc2[W];  // acc: the segment's accumulators; acc2: the FFN2 sum across its K panels
  constexpr bool CLSM = tx_cls_mfma<W>();
  float c0[W][2][TX_CLS_NC], c02[W][2];  // the CLS row's partial sums (this lane's half of the k) | the linear2 sum
  Acc<1, 2> accc;             // CLSM: the CLS tile (row v = window v's CLS row)
  accc.zero();
  float X[W][2][16], x0[W][2];  // the layer input / residual: token rows trow(r), CLS
#pragma unroll
  for (int v = 0; v < W; ++v) {
    acc[v].zero();
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int k = 0; k < TX_CLS_NC; ++k) c0[v][n][k] = 0.f;
  }

  // the token epilogue's constants, loaded before the first weight loads (see the epilogue parameters below)
#pragma unroll
  for (int n = 0; n < 2; ++n) {
    float pe[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) pe[r] = ta.pe[trow(r) * 256 + col0 + 32 * n];
    const float c = ta.cls[col0 + 32 * n] + ta.pe[col0 + 32 * n];
#pragma unroll
    for (int v = 0; v < W; ++v) {
#pragma unroll
      for (int r = 0; r < 16; ++r) X[v][n][r] = pe[r];
      x0[v][n] = c;
    }
  }

  // chunk order inside a segment rotated per workgroup (VGE_TX_ROT: the CUs of an XCD, which share its L2, then read
  // different chunks of the same segment at a time instead of all hitting one chunk's lines together)
#ifndef VGE_TX_ROT
#define VGE_TX_ROT 1
#endif
  const int rot = VGE_TX_ROT ? __builtin_amdgcn_readfirstlane(((blockIdx.x >> 3) * VGE_TX_ROT) & 15) : 0;
  BFrag<2> b[TX_PF];
#pragma unroll
  for (int j = 0; j < TX_PF - 1; ++j) load_b<2, SPW>(seg_base(0), (j + rot) & 15, loff, b[j]);

  int s = 0;  // the current segment
  // lane-derived values re-derived per segment: stops the compiler from hoisting the ~100 (64-bit, loop-invariant)
  // epilogue addresses out of the loops, where they would hold registers throughout
  auto rederive = [&]() __attribute__((always_inline)) {
    int lo = lane;
    asm volatile("" : "+v"(lo));
    i = lo & 31;
    h = lo >> 5;
    col0 = wave * 64 + i;
  };
  // a segment's epilogue parameters (column scales, bias, LayerNorm affine), loaded before its weight stream:
  // vmcnt retires in order, so a load issued in the epilogue would wait for the prefetched chunks
  float ecs[2], eb[2], eg[2], ebt[2];
  auto consts = [&](const float* pcs, const float* pb, const float* pg, const float* pbt) __attribute__((always_inline)) {
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      ecs[n] = pcs[col0 + 32 * n];
      eb[n] = pb ? pb[col0 + 32 * n] : 0.f;
      eg[n] = pg ? pg[col0 + 32 * n] : 0.f;
      ebt[n] = pg ? pbt[col0 + 32 * n] : 0.f;
    }
  };
  // segment s's 16 chunks into acc (A operands: window v's planes at abase + v * AP_BYTES), B fragments TX_PF - 1
  // chunks ahead across the boundary into segment s + 1; then cl = the CLS row (both k halves) and xs = the
  // accumulator scales
  float xs[W], cl[W][2];
  auto stream = [&](const char* abase) __attribute__((always_inline)) {
    auto afn = [&](int c, AFragT<W>& f) __attribute__((always_inline)) {
      if (VGE_TX_ROT) c = (c + rot) & 15;
#pragma unroll
      for (int v = 0; v < W; ++v) {
        const char* ab = abase + v * AP_BYTES;
        f.h[v] = *reinterpret_cast<const half8*>(ab + aoff + c * 32);
        if constexpr (SPA) f.l[v] = *reinterpret_cast<const half8*>(ab + aoff + c * 32 + AROWS * XSB);
        if constexpr (!CLSM) {
          f.h0[v] = *reinterpret_cast<const half8*>(ab + aoff0 + c * 32);
          if constexpr (SPA) f.l0[v] = *reinterpret_cast<const half8*>(ab + aoff0 + c * 32 + AROWS * XSB);
        }
      }
      if constexpr (CLSM) {  // CLS tile row i = window i's row 0 (lanes i < W), zero rows below
        const char* ab = abase + (i < W ? i : 0) * AP_BYTES + aoff0 + c * 32;
        const half8 z = {};
        const half8 x = *reinterpret_cast<const half8*>(ab);
        f.h0[0] = i < W ? x : z;
        if constexpr (SPA) {
          const half8 y = *reinterpret_cast<const half8*>(ab + AROWS * XSB);
          f.l0[0] = i < W ? y : z;
        }
      }
    };
    TSTAMP(2 * s);
    AFragT<W> a[2];
    afn(0, a[0]);
    const gchar seg_cur = seg_base(s), seg_nxt = seg_base(s + 1);
#pragma unroll
    for (int c = 0; c < 16; ++c) {
#if !(VGE_ABL & 2)
      if (c + TX_PF - 1 < 16) load_b<2, SPW>(seg_cur, (c + TX_PF - 1 + rot) & 15, loff, b[(c + TX_PF - 1) % TX_PF]);
      else load_b<2, SPW>(seg_nxt, (c + TX_PF - 1 - 16 + rot) & 15, loff, b[(c + TX_PF - 1) % TX_PF]);
#endif
      if (c + 1 < 16 && (!(VGE_ABL & 4) || c == 0)) afn(c + 1, a[(c + 1) & 1]);
      const AFragT<W>& f = a[c & 1];
      const BFrag<2>& bb = b[c % TX_PF];
#pragma unroll
      for (int v = 0; v < W; ++v)
#pragma unroll
        for (int n = 0; n < 2; ++n) {
#if !(VGE_ABL & 1)
          acc[v].c[0][n] = mfma32(f.h[v], bb.h[n], acc[v].c[0][n]);
          if constexpr (SPW) acc[v].c[0][n] = mfma32(f.h[v], bb.l[n], acc[v].c[0][n]);
          if constexpr (SPA) acc[v].c[0][n] = mfma32(f.l[v], bb.h[n], acc[v].c[0][n]);
#else
          asm volatile("" ::"v"(f.h[v]), "v"(f.l[v]), "v"(bb.h[n]), "v"(bb.l[n]));
#endif
#if !(VGE_ABL & 64)
          if constexpr (!CLSM) cls_dot<SPA, SPW>(c0[v][n], f.h0[v], f.l0[v], bb.h[n], bb.l[n]);
#endif
        }
      if constexpr (CLSM) {
#pragma unroll
        for (int n = 0; n < 2; ++n) {
#if !(VGE_ABL & 64)
          accc.c[0][n] = mfma32(f.h0[0], bb.h[n], accc.c[0][n]);
          if constexpr (SPW) accc.c[0][n] = mfma32(f.h0[0], bb.l[n], accc.c[0][n]);
          if constexpr (SPA) accc.c[0][n] = mfma32(f.l0[0], bb.h[n], accc.c[0][n]);
#endif
        }
      } else {
        // the CLS dot products stay in their step (else they are sunk past the loop and the ring stays live)
#pragma unroll
        for (int v = 0; v < W; ++v)
#pragma unroll
          for (int k = 0; k < TX_CLS_NC; ++k) asm volatile("" : "+v"(c0[v][0][k]), "+v"(c0[v][1][k]));
      }
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      // keep the waves abreast (see run_stream); the barrier after the last chunk also orders every
      // epilogue's LDS writes after all waves' reads of the segment's A planes
      if (c % TX_PF == TX_PF - 1 && (!(VGE_ABL & 128) || c == 15)) lds_barrier();
    }
    TSTAMP(2 * s + 1);
    tr_s = s;
    ++s;
#pragma unroll
    for (int v = 0; v < W; ++v) {
      xs[v] = ldexpf(1.0f, ax[v]);
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        if constexpr (CLSM) {
          cl[v][n] = halves_sum(accc.c[0][n][v]);  // row v: register v of the h = 0 lanes (h = 1 holds row 4 + v = 0)
        } else {
          cl[v][n] = halves_sum(cls_total(c0[v][n]));
#pragma unroll
          for (int k = 0; k < TX_CLS_NC; ++k) c0[v][n][k] = 0.f;
        }
      }
    }
    if constexpr (CLSM) accc.zero();
  };
  // the finished values of tile n (bias added) -> y, CLS -> y0
  auto tile_out = [&](int v, int n, floatx16& y, float& y0) __attribute__((always_inline)) {
    const float cs = ecs[n] * xs[v], bb = eb[n];
#pragma unroll
    for (int r = 0; r < 16; ++r) y[r] = acc[v].c[0][n][r] * cs + bb;
    y0 = cl[v][n] * cs + bb;
  };

  // attention, head 2 wave + e of window v (scale 1/sqrt(32)), exact f32 MFMAs (v_mfma_f32_32x32x2_f32) for the
  // 32 x 32 frame block, the CLS query / CLS key on the VALU; the head's Q, K, V staged in this wave's own LDS
  // rows (no other wave reads them: no barrier):
  //   S^T[k][q] = K_k . Q_q (frame keys k, frame queries q, C layout: lane = query, registers = keys)
  //   softmax over the keys of a query = over a lane's 16 registers, its partner half and the CLS key
  //   O^T[d][q] = sum_k V^T[d][k] P^T[k][q] (B operand = P^T straight from the C registers)
  floatx16 ot[W][2];  // O[1 + i][d], d = (r & 3) + 8 (r >> 2) + 4 h
  float oc[W][2];     // O[0][d = i] (CLS query), lanes with h == 0
  float am[W];        // max |O| of each window (the att planes' exponent)
  auto attend = [&](int v, int e, const floatx16& qt, float q0v, const floatx16& kt, float k0v, const floatx16& vt,
                    float v0v) __attribute__((always_inline)) {
    float* const Qh = reinterpret_cast<float*>(U) + wave * (3 * TOK * QH);
    float* const Kh = Qh + TOK * QH;
    float* const Vh = Qh + 2 * TOK * QH;
    constexpr float kScale = 0.17677669529663687f;
    // stage (the previous head's reads of these rows were issued first: LDS is in order per wave)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      Qh[trow(r) * QH + i] = qt[r];
      Kh[trow(r) * QH + i] = kt[r];
      Vh[trow(r) * QH + i] = vt[r];
    }
    if (h == 0) {
      Qh[i] = q0v;
      Kh[i] = k0v;
      Vh[i] = v0v;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // frame block scores; d ordered so lane half h reads d = 16 h .. 16 h + 15 contiguously
    floatx4 ka[4], qb[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      ka[j] = *reinterpret_cast<const floatx4*>(Kh + (1 + i) * QH + 16 * h + 4 * j);
      qb[j] = *reinterpret_cast<const floatx4*>(Qh + (1 + i) * QH + 16 * h + 4 * j);
    }
    floatx16 st = {};
#pragma unroll
    for (int t = 0; t < 16; ++t)
      st = __builtin_amdgcn_mfma_f32_32x32x2f32(ka[t >> 2][t & 3], qb[t >> 2][t & 3], st, 0, 0, 0);
    // CLS key score of query 1 + i (halves split d, then combine)
    float sc = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const floatx4 k0 = *reinterpret_cast<const floatx4*>(Kh + 16 * h + 4 * j);
      sc += qb[j][0] * k0[0] + qb[j][1] * k0[1] + qb[j][2] * k0[2] + qb[j][3] * k0[3];
    }
    sc = halves_sum(sc) * kScale;
    float mx = sc;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      st[r] *= kScale;
      mx = fmaxf(mx, st[r]);
    }
    mx = halves_max(mx);
    float den = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      st[r] = expf(st[r] - mx);
      den += st[r];
    }
    const float pc = expf(sc - mx);
    den = halves_sum(den) + pc;
    // P V over the frame keys: A = V^T[d = i][key of register t of half h], B = P^T (register t)
    floatx16 o = {};
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const float va = Vh[(1 + (t & 3) + 8 * (t >> 2) + 4 * h) * QH + i];
      o = __builtin_amdgcn_mfma_f32_32x32x2f32(va, st[t], o, 0, 0, 0);
    }
    // + the CLS key's value row, then normalise
    const float inv = 1.0f / den;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const floatx4 v0 = *reinterpret_cast<const floatx4*>(Vh + 8 * g + 4 * h);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        o[4 * g + k] = (o[4 * g + k] + pc * v0[k]) * inv;
        am[v] = fmaxf(am[v], fabsf(o[4 * g + k]));
      }
    }
    ot[v][e] = o;
    // CLS query: lane l <= 32 scores key l, the wave reduces; lane d < 32 then sums P V over the keys
    float s0 = -INFINITY;
    if (lane < TOK) {
      float a = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const floatx4 q0 = *reinterpret_cast<const floatx4*>(Qh + 4 * j);
        const floatx4 kl = *reinterpret_cast<const floatx4*>(Kh + lane * QH + 4 * j);
        a += q0[0] * kl[0] + q0[1] * kl[1] + q0[2] * kl[2] + q0[3] * kl[3];
      }
      s0 = a * kScale;
    }
    const float m0 = wave_max_all(s0);
    const float p0 = (lane < TOK) ? expf(s0 - m0) : 0.f;
    const float d0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(wave_sum_last(p0)), 63));
    float acc0[3] = {0.f, 0.f, 0.f};  // three chains (33 keys)
#pragma unroll
    for (int k = 0; k < TOK; ++k)
      acc0[k % 3] += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(p0), k)) * Vh[k * QH + i];
    oc[v][e] = ((acc0[0] + acc0[1]) + acc0[2]) / d0;
    if (h == 0) am[v] = fmaxf(am[v], fabsf(oc[v][e]));
  };

  // ---- tokens: CLS = cls + pe_0, frames = pooled Wov^T + pe_t
  consts(ta.ov_cs, nullptr, nullptr, nullptr);
  stream(Ap);
#pragma unroll
  for (int v = 0; v < W; ++v) {
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      const float cs = ecs[n] * xs[v];
#pragma unroll
      for (int r = 0; r < 16; ++r) X[v][n][r] += acc[v].c[0][n][r] * cs;  // X holds pe, x0 cls + pe_0
    }
    acc[v].zero();
  }
  split_rows(Ap, X, x0, ax);
  __syncthreads();

#pragma unroll 1
  for (int l = 0; l < ta.n_layers; ++l) {
    const TxLayerX3& L = ta.layers[l];
    // ---- in_proj 0: q, k of head 2 wave
    rederive();
    consts(L.in_cs, L.in_b, nullptr, nullptr);
    stream(Ap);
    floatx16 qa[W], ka[W];
    float qa0[W], ka0[W];
#pragma unroll
    for (int v = 0; v < W; ++v) {
      tile_out(v, 0, qa[v], qa0[v]);
      tile_out(v, 1, ka[v], ka0[v]);
      acc[v].zero();
    }
    // ---- in_proj 1: v of head 2 wave (-> its attention), q of head 2 wave + 1
    consts(L.in_cs + 256, L.in_b + 256, nullptr, nullptr);
    stream(Ap);
    floatx16 qb[W];
    float qb0[W];
#pragma unroll
    for (int v = 0; v < W; ++v) {
      floatx16 va;
      float va0;
      tile_out(v, 0, va, va0);
      tile_out(v, 1, qb[v], qb0[v]);
      acc[v].zero();
      am[v] = 0.f;
      attend(v, 0, qa[v], qa0[v], ka[v], ka0[v], va, va0);
    }
    // ---- in_proj 2: k, v of head 2 wave + 1 (-> its attention)
    consts(L.in_cs + 512, L.in_b + 512, nullptr, nullptr);
    stream(Ap);
#pragma unroll
    for (int v = 0; v < W; ++v) {
      floatx16 kb, vb;
      float kb0, vb0;
      tile_out(v, 0, kb, kb0);
      tile_out(v, 1, vb, vb0);
      acc[v].zero();
      attend(v, 1, qb[v], qb0[v], kb, kb0, vb, vb0);
    }
    block_max(am);
#pragma unroll
    for (int v = 0; v < W; ++v) {  // att -> the A planes of out_proj: frame rows 1 + i, CLS row 0 (every wave's
      ax[v] = fp16_range_exp(am[v]);  // reads of the X planes ended with in_proj 2's stream)
      const float scl = ldexpf(1.0f, -ax[v]);
      char* const P = Ap + v * AP_BYTES;
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        char* rh = P + (1 + i) * XSB + (2 * wave + e) * 64;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          typedef _Float16 half4v __attribute__((ext_vector_type(4)));
          half4v hv, lv;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const float y = ot[v][e][4 * g + k] * scl;
            hv[k] = (_Float16)y;
            lv[k] = (_Float16)(y - (float)hv[k]);
          }
          *reinterpret_cast<half4v*>(rh + (8 * g + 4 * h) * 2) = hv;
          if constexpr (SPA) *reinterpret_cast<half4v*>(rh + (8 * g + 4 * h) * 2 + AROWS * XSB) = lv;
        }
        if (h == 0) {
          const float y = oc[v][e] * scl;
          const _Float16 hi = (_Float16)y;
          reinterpret_cast<_Float16*>(P)[(2 * wave + e) * 32 + i] = hi;
          if constexpr (SPA)
            reinterpret_cast<_Float16*>(P + AROWS * XSB)[(2 * wave + e) * 32 + i] = (_Float16)(y - (float)hi);
        }
      }
    }
    __syncthreads();

    // ---- out_proj + bias + residual -> LN1 -> X1 (kept in X) and the A planes of linear1
    rederive();
    consts(L.out_cs, L.out_b, L.n1_w, L.n1_b);
    stream(Ap);
#pragma unroll
    for (int v = 0; v < W; ++v) {
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const float cs = ecs[n] * xs[v], bb = eb[n];
#pragma unroll
        for (int r = 0; r < 16; ++r) X[v][n][r] += acc[v].c[0][n][r] * cs + bb;
        x0[v][n] += cl[v][n] * cs + bb;
      }
      acc[v].zero();
    }
    layer_norm(X, x0, eg, ebt);
    // a LayerNorm output's range is known statically; the barrier orders the writes after every wave's reads of
    // the att planes (the out_proj stream) -- those all precede the LayerNorm's reductions
    TSTAMP_FINE(4);
#pragma unroll
    for (int v = 0; v < W; ++v) {
      split_rows_e(Ap + v * AP_BYTES, X[v], x0[v], L.e_x1);
      ax[v] = L.e_x1;
    }
    TSTAMP_FINE(5);
    __syncthreads();
    TSTAMP_FINE(6);

    // ---- FFN: linear1 chunk hc -> ReLU -> hidden planes (one static exponent for all four: the running
    // linear2 sum needs no rescale), linear2 K panel hc accumulated in acc2
#pragma unroll 1
    for (int hc = 0; hc < 4; ++hc) {
      rederive();
      consts(L.l1_cs + hc * 256, L.l1_b + hc * 256, nullptr, nullptr);
      stream(Ap);
#pragma unroll
      for (int v = 0; v < W; ++v) {
        float hv[2][16], h0[2];
#pragma unroll
        for (int n = 0; n < 2; ++n) {
          const float cs = ecs[n] * xs[v], bb = eb[n];
#pragma unroll
          for (int r = 0; r < 16; ++r) hv[n][r] = fmaxf(acc[v].c[0][n][r] * cs + bb, 0.f);
          h0[n] = fmaxf(cl[v][n] * cs + bb, 0.f);
        }
        split_rows_e(U + v * AP_BYTES, hv, h0, L.e_h);
        if (hc == 0) {
          acc[v].zero();
        } else {
          acc[v] = acc2[v];
          if constexpr (!CLSM) {
#pragma unroll
            for (int n = 0; n < 2; ++n) c0[v][n][0] = (h == 0) ? c02[v][n] : 0.f;  // c02: both k halves, one carries it
          }
        }
      }
      __syncthreads();
      if (hc == 3) {
        consts(L.l2_cs, L.l2_b, L.n2_w, L.n2_b);
      } else {
        consts(L.l2_cs, L.l2_b, nullptr, nullptr);  // (unused until the last panel)
      }
      stream(U);
      if (hc < 3) {
#pragma unroll
        for (int v = 0; v < W; ++v) {
          acc2[v] = acc[v];
#pragma unroll
          for (int n = 0; n < 2; ++n) c02[v][n] = (CLSM && hc > 0) ? c02[v][n] + cl[v][n] : cl[v][n];
          acc[v].zero();
        }
      }
    }
#pragma unroll
    for (int v = 0; v < W; ++v) {  // (the linear2 sum holds (H W2^T) 2^-e_h; ax stays the X1 planes' exponent)
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        if constexpr (CLSM) cl[v][n] += c02[v][n];  // the CLS tile restarts per K panel: its panel sums
        const float cs = ecs[n] * ldexpf(1.0f, L.e_h), bb = eb[n];
#pragma unroll
        for (int r = 0; r < 16; ++r) X[v][n][r] += acc[v].c[0][n][r] * cs + bb;
        x0[v][n] += cl[v][n] * cs + bb;
      }
      acc[v].zero();
    }
    layer_norm(X, x0, eg, ebt);
    if (l + 1 < ta.n_layers) {  // (every wave's reads of the X1 planes precede the LayerNorm's barriers)
      TSTAMP_FINE(4);
#pragma unroll
      for (int v = 0; v < W; ++v) {
        split_rows_e(Ap + v * AP_BYTES, X[v], x0[v], L.e_x2);
        ax[v] = L.e_x2;
      }
      TSTAMP_FINE(5);
      __syncthreads();
      TSTAMP_FINE(6);
    }
  }

  TSTAMP(125);
  // ---- outputs: L2-normalised tokens, the CLS row as seq_embed, the window's temporal-coherence term
  float ss[W][2][16], ss0[W][2];
#pragma unroll
  for (int v = 0; v < W; ++v)
#pragma unroll
    for (int n = 0; n < 2; ++n) {
#pragma unroll
      for (int r = 0; r < 16; ++r) ss[v][n][r] = X[v][n][r] * X[v][n][r];
      ss0[v][n] = x0[v][n] * x0[v][n];
    }
  row_sums(ss, ss0);
#pragma unroll
  for (int v = 0; v < W; ++v) {
    // F.normalize: x / max(||x||, 1e-12), as x * (1 / max(...)) once per row
    float inv_norm[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) inv_norm[r] = 1.0f / fmaxf(sqrtf(ss[v][0][r]), 1e-12f);
    const float inv_norm0 = 1.0f / fmaxf(sqrtf(ss0[v][0]), 1e-12f);
    float* F = reinterpret_cast<float*>(U + v * F_BYTES);  // [TOK][QS] normalised tokens
    const bool out = v < nv;
    const size_t w = (size_t)(wb0 + v);
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      const int col = col0 + 32 * n;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float f = X[v][n][r] * inv_norm[r];
        F[trow(r) * QS + col] = f;
        if (ta.frame && out) ta.frame[(w * TOK + trow(r)) * 256 + col] = f;
      }
      if (h == 0) {
        const float f0 = x0[v][n] * inv_norm0;
        F[col] = f0;
        if (out) {
          if (ta.frame) ta.frame[w * TOK * 256 + col] = f0;
          ta.seq[w * 256 + col] = f0;
        }
      }
    }
  }
  __syncthreads();
  if (ta.tc) {
    // |f_r - f_{r-1}| for r = 2..32 (frame_embeds[1:], eval.py:221-224): wave k takes rows 2+k, 6+k, ...
    float* rt = red + 2 * W * TOK * TX_NW + 2 * W * TX_NW;
#pragma unroll
    for (int v = 0; v < W; ++v) {
      const float* F = reinterpret_cast<const float*>(U + v * F_BYTES);
      float tsum = 0.f;
      for (int r = 2 + wave; r < TOK; r += TX_NW) {
        float d2 = 0.f;
#pragma unroll
        for (int c = lane; c < 256; c += 64) {
          const float d = F[r * QS + c] - F[(r - 1) * QS + c];
          d2 += d * d;
        }
        tsum += sqrtf(wave_sum(d2));
      }
      if (lane == 0) rt[v * TX_NW + wave] = tsum;
    }
    __syncthreads();
    if (tid < nv) {
      const float* q = rt + tid * TX_NW;
      ta.tc[wb0 + tid] = ((q[0] + q[1]) + (q[2] + q[3])) / (float)(TOK - 2);
    }
  }
  TSTAMP(126);
}

}  // namespace

namespace vge {

struct TxLayerX3Host {
  const _Float16* in_w;  const float* in_cs; const float* in_b;
  const _Float16* out_w; const float* out_cs; const float* out_b;
  const float* n1_w; const float* n1_b;
  const _Float16* l1_w; const float* l1_cs; const float* l1_b;
  const _Float16* l2_w; const float* l2_cs; const float* l2_b;
  const float* n2_w; const float* n2_b;
  int e_x1, e_x2, e_h, pad;
};
static_assert(sizeof(TxLayerX3Host) == sizeof(TxLayerX3), "TxLayerX3 layout");

struct TxArgsX3Host {
  const float* pooled; int n_windows, n_layers;
  const _Float16* ov_w; const float* ov_cs;
  const float* cls; const float* pe;
  const TxLayerX3Host* layers;  // host array [n_layers], n_layers <= 8
  float* seq; float* frame; float* tc;
};

hipError_t transformer_x3_kernel_setup() {
  const struct {
    const void* k;
    int lds;
  } ks[7] = {{(const void*)transformer_x3_kernel<true, true, 1>, tx_lds_bytes<1, true>()},
             {(const void*)transformer_x3_kernel<true, false, 1>, tx_lds_bytes<1, true>()},
             {(const void*)transformer_x3_kernel<false, false, 1>, tx_lds_bytes<1, false>()},
             {(const void*)transformer_x3_kernel<false, false, 1, 2>, tx_lds_bytes<1, false>()},
             {(const void*)transformer_x3_kernel<true, true, 2>, tx_lds_bytes<2, true>()},
             {(const void*)transformer_x3_kernel<true, false, 2>, tx_lds_bytes<2, true>()},
             {(const void*)transformer_x3_kernel<false, false, 2>, tx_lds_bytes<2, false>()}};
  for (const auto& k : ks) {
    const hipError_t e = hipFuncSetAttribute(k.k, hipFuncAttributeMaxDynamicSharedMemorySize, k.lds);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// Windows per workgroup (each weight chunk a wave streams then feeds two windows' rows at W = 2).  A W = 2 workgroup
// takes 1.7x (single fp16) / 1.9x (3xfp16 split) the time of a W = 1 one (its epilogues are per window, and the
// split's stream turns MFMA-bound), so W = 2 pays once every CU holds several windows: measured (stage times,
// tools/gpu_tx_modes.sh) split 2.35 -> 2.29 ms at 2,048 but 0.89 -> 1.10 ms at 600 (round tails).  Single fp16 keeps
// one window per workgroup and runs two workgroups per CU once there are more windows than CUs (76 KB of LDS each,
// so one's epilogues run beside the other's weight stream; tools/gpu_tx_occ.sh): 0.686 -> 0.50 ms at 1,024 windows
// and 2.67 -> 1.94 ms at 4,096 (W = 2: 0.61 / 2.39); at 256 windows the dispatcher would pair workgroups on some CUs
// and leave others idle (0.175 -> 0.18-0.19 ms).  VGE_TX_W=1|2 and VGE_TX_OCC=1|2 force either.
static int g_tx_w_forced = -1;  // -1: not read yet, 0: automatic, 1 | 2 (VGE_TX_W, vge_debug_set_tx_windows)
static int g_tx_occ = -1;       // single fp16, one window per workgroup: -1 not read yet, 0 automatic, 1 | 2 forced
static int tx_n_cu() {
  static int n_cu = 0;
  if (n_cu == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n_cu < 1)
      n_cu = 256;
  }
  return n_cu;
}
static int tx_windows_per_block(int n_windows, int mode) {
  if (g_tx_w_forced < 0) {
    const char* v = getenv("VGE_TX_W");
    g_tx_w_forced = (v && (v[0] == '1' || v[0] == '2')) ? v[0] - '0' : 0;
  }
  if (g_tx_w_forced) return g_tx_w_forced;
  if (mode == 0) return 1;
  return n_windows >= (mode == 2 ? 8 : 4) * tx_n_cu() ? 2 : 1;
}
static int tx_blocks_per_cu(int n_windows) {  // single fp16, W = 1
  if (g_tx_occ < 0) {
    const char* v = getenv("VGE_TX_OCC");
    g_tx_occ = (v && (v[0] == '1' || v[0] == '2')) ? v[0] - '0' : 0;
  }
  if (g_tx_occ) return g_tx_occ;
  return n_windows > tx_n_cu() ? 2 : 1;
}

// mode: 0 single fp16, 1 activations split (fp16 weights), 2 3xfp16
hipError_t launch_transformer_x3(const TxArgsX3Host& a, int mode, hipStream_t s) {
  if (a.n_windows < 1) return hipSuccess;
  if (a.n_layers < 0 || a.n_layers > TX_MAX_LAYERS) return hipErrorInvalidValue;
  TxArgsX3 t;
  memset(&t, 0, sizeof(t));
  t.pooled = a.pooled;
  t.n_windows = a.n_windows;
  t.n_layers = a.n_layers;
  t.ov_w = a.ov_w;
  t.ov_cs = a.ov_cs;
  t.cls = a.cls;
  t.pe = a.pe;
  t.seq = a.seq;
  t.frame = a.frame;
  t.tc = a.tc;
  memcpy(t.layers, a.layers, sizeof(TxLayerX3) * a.n_layers);
  if (tx_windows_per_block(a.n_windows, mode) == 2) {
    if (mode == 2)
      hipLaunchKernelGGL((transformer_x3_kernel<true, true, 2>), dim3((a.n_windows + 1) / 2), dim3(256),
                         (tx_lds_bytes<2, true>()), s, t);
    else if (mode == 1)
      hipLaunchKernelGGL((transformer_x3_kernel<true, false, 2>), dim3((a.n_windows + 1) / 2), dim3(256),
                         (tx_lds_bytes<2, true>()), s, t);
    else
      hipLaunchKernelGGL((transformer_x3_kernel<false, false, 2>), dim3((a.n_windows + 1) / 2), dim3(256),
                         (tx_lds_bytes<2, false>()), s, t);
  } else {
    if (mode == 2)
      hipLaunchKernelGGL((transformer_x3_kernel<true, true, 1>), dim3(a.n_windows), dim3(256), (tx_lds_bytes<1, true>()), s, t);
    else if (mode == 1)
      hipLaunchKernelGGL((transformer_x3_kernel<true, false, 1>), dim3(a.n_windows), dim3(256), (tx_lds_bytes<1, true>()), s,
                         t);
    else if (tx_blocks_per_cu(a.n_windows) == 2)
      hipLaunchKernelGGL((transformer_x3_kernel<false, false, 1, 2>), dim3(a.n_windows), dim3(256),
                         (tx_lds_bytes<1, false>()), s, t);
    else
      hipLaunchKernelGGL((transformer_x3_kernel<false, false, 1>), dim3(a.n_windows), dim3(256),
                         (tx_lds_bytes<1, false>()), s, t);
  }
  return hipGetLastError();
}

}  // namespace vge

// Test hook: force the fused transformer's windows per workgroup (1 or 2; 0 = automatic).  Returns the previous
// setting.
extern "C" int vge_debug_set_tx_windows(int w) {
  const int prev = vge::g_tx_w_forced < 0 ? 0 : vge::g_tx_w_forced;
  vge::g_tx_w_forced = (w == 1 || w == 2) ? w : 0;
  return prev;
}

#ifdef VGE_TRACE
extern "C" int vge_debug_tx_trace(long long* host, int n) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_vge_tx_trace), sizeof(long long) * (size_t)n);
}
#endif
