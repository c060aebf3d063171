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
constexpr int QS = 260;          // f32 row stride of the Q / K / V / final-embedding staging (bank shift)
#ifndef VGE_TX_PF
#define VGE_TX_PF 4
#endif
constexpr int TX_PF = VGE_TX_PF;  // weight chunks in flight per wave (ring depth)
constexpr int TX_NW = 4;         // waves
constexpr int AP_BYTES = 2 * AROWS * XSB;            // hi / lo planes of the current A operand
constexpr int U_BYTES = 3 * TOK * QS * 4;             // Q, K, V (f32) | FFN hidden planes | final embeddings
constexpr int RED_FLOATS = 2 * TOK * TX_NW + 2 * TX_NW + TX_NW;  // row partials x2, maxima x2, tc
constexpr int TX_LDS_BYTES = AP_BYTES + U_BYTES + RED_FLOATS * 4;
static_assert(2 * AROWS * XSB <= U_BYTES, "hidden planes fit the union");
static_assert(TX_LDS_BYTES <= 160 * 1024, "LDS");

struct AFragT {  // one chunk's A operand: the 32 frame rows (MFMA) and the CLS row (VALU dot products)
  half8 h, l, h0, l0;
};

// CLS row on the VALU: c += x . w over this lane's 8 k of the chunk, the same 3 products as the MFMAs
template <bool SPA, bool SPW>
__device__ __forceinline__ float cls_dot(float c, half8 xh, half8 xl, half8 wh, half8 wl) {
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const half2v a = {xh[2 * p], xh[2 * p + 1]};
    const half2v b = {wh[2 * p], wh[2 * p + 1]};
    if constexpr (SPA) {
      const half2v al = {xl[2 * p], xl[2 * p + 1]};
      c = __builtin_amdgcn_fdot2(al, b, c, false);
    }
    if constexpr (SPW) {
      const half2v bl = {wl[2 * p], wl[2 * p + 1]};
      c = __builtin_amdgcn_fdot2(a, bl, c, false);
    }
    c = __builtin_amdgcn_fdot2(a, b, c, false);
  }
  return c;
}

// SPA / SPW: activations / weights carried as hi + lo fp16 planes.  Both: 3xfp16 (VGE_F32X3, hi*hi + hi*lo +
// lo*hi); neither: single fp16, one MFMA per product; SPA only: (hi_a + lo_a) * hi_w, two MFMAs on the fp16 weight
// stream (half the bytes of the split).
template <bool SPA, bool SPW = SPA>
__global__ void __launch_bounds__(256, 1) transformer_x3_kernel(TxArgsX3 ta) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  char* Ap = lds;                                   // A planes: hi rows [0, AROWS), lo at + AROWS * XSB
  char* U = lds + AP_BYTES;                         // Q/K/V f32 [3][TOK][QS] | hidden planes | embeddings
  float* red = reinterpret_cast<float*>(U + U_BYTES);  // [2][TOK][4] row partials, [2][4] maxima, [4] tc
  // consecutive reductions alternate between two buffers, so none needs a trailing barrier: the writes of
  // reduction k + 2 come after reduction k + 1's barrier, which every read of reduction k precedes
  int rs_buf = 0, bm_buf = 0;
  [[maybe_unused]] int tr_s = -1;  // VGE_TRACE: the current segment, for the fine stamps of layer 0's epilogues
#ifdef VGE_TRACE
#define TSTAMP_FINE(k) do { if (tr_s == 4) TSTAMP(100 + (k)); else if (tr_s == 12) TSTAMP(110 + (k)); } while (0)
#else
#define TSTAMP_FINE(k) do { } while (0)
#endif
  const int w = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  int i = lane & 31, h = lane >> 5;
  int col0 = wave * 64 + i;                         // this lane's columns: col0 + 32 n, n = 0, 1
  const unsigned loff = (unsigned)((h * 256 + col0) * 16);
  // token row held in C-layout register r (the MFMA tile covers tokens 1..32; token 0 = CLS is `x0`)
  auto trow = [&](int r) { return 1 + (r & 3) + 8 * (r >> 2) + 4 * h; };
  const unsigned aoff = (unsigned)((1 + i) * XSB + h * 16), aoff0 = (unsigned)(h * 16);

  // ---- helpers -----------------------------------------------------------------------------------------
  auto block_max = [&](float m) {  // over the workgroup, every thread gets it
    float* rb = red + 2 * TOK * TX_NW + bm_buf * TX_NW;
    bm_buf ^= 1;
    m = wave_max_last(m);
    if (lane == 63) rb[wave] = m;
    __syncthreads();
    const floatx4 p = *reinterpret_cast<const floatx4*>(rb);
    return fmaxf(fmaxf(p[0], p[1]), fmaxf(p[2], p[3]));
  };
  // row sums over the 256 columns, in place: x (token rows trow(r), both column tiles get the row sum),
  // x0 (CLS; the same value in both lane halves)
  auto row_sums = [&](float (&x)[2][16], float (&x0)[2]) {
    float* rb = red + rs_buf * TOK * TX_NW;
    rs_buf ^= 1;
    auto sum4 = [&](int row) {
      const floatx4 a = *reinterpret_cast<const floatx4*>(rb + row * TX_NW);
      return (a[0] + a[1]) + (a[2] + a[3]);
    };
    float y[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) y[r] = half_sum_last(x[0][r] + x[1][r]);  // valid in lanes 31 and 63
    const float y0 = half_sum_last(x0[0] + x0[1]);
    if (i == 31) {
#pragma unroll
      for (int r = 0; r < 16; ++r) rb[trow(r) * TX_NW + wave] = y[r];
      if (h == 0) rb[wave] = y0;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; ++r) x[0][r] = x[1][r] = sum4(trow(r));
    x0[0] = x0[1] = sum4(0);
  };
  // LayerNorm over 256 columns (in place), affine w, b [256], eps 1e-5
  auto layer_norm = [&](float (&v)[2][16], float (&v0)[2], const float (&lw)[2], const float (&lb)[2]) {
    float s[2][16], s0[2] = {v0[0], v0[1]};
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int r = 0; r < 16; ++r) s[n][r] = v[n][r];
    TSTAMP_FINE(1);
    row_sums(s, s0);
    TSTAMP_FINE(2);
    float q[2][16], q0[2];
#pragma unroll
    for (int n = 0; n < 2; ++n) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        s[n][r] *= 1.0f / 256.0f;
        const float d = v[n][r] - s[n][r];
        q[n][r] = d * d;
      }
      s0[n] *= 1.0f / 256.0f;
      q0[n] = (v0[n] - s0[n]) * (v0[n] - s0[n]);
    }
    row_sums(q, q0);
    TSTAMP_FINE(3);
    // 1 / sqrt(var + eps) once per row (v_rsq_f32, ~1 ulp; the IEEE sqrt + divide sequences cost ~50
    // instructions per value)
    float rstd[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) rstd[r] = __builtin_amdgcn_rsqf(q[0][r] * (1.0f / 256.0f) + 1e-5f);
    const float rstd0 = __builtin_amdgcn_rsqf(q0[0] * (1.0f / 256.0f) + 1e-5f);
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      const float gw = lw[n], gb = lb[n];
#pragma unroll
      for (int r = 0; r < 16; ++r) v[n][r] = (v[n][r] - s[n][r]) * rstd[r] * gw + gb;
      v0[n] = (v0[n] - s0[n]) * rstd0 * gw + gb;
    }
  };
  // split rows into hi/lo planes at `plane` as v * 2^-e, e from the workgroup-wide max |v| (the barrier
  // inside also retires every read of the planes' previous content issued before it); returns e.  The
  // caller barriers before the planes are read.
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
    return e;
  };
  auto split_rows = [&](char* plane, const float (&v)[2][16], const float (&v0)[2]) {
    float m = fmaxf(fabsf(v0[0]), fabsf(v0[1]));
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int r = 0; r < 16; ++r) m = fmaxf(m, fabsf(v[n][r]));
    return split_rows_e(plane, v, v0, fp16_range_exp(block_max(m)));
  };
  auto both_halves = [&](float c) { return halves_sum(c); };

  TSTAMP(124);
  // ---- token A operand: row 0 zero (the CLS token is not a product), rows 1..32 the window's pooled frames
  reinterpret_cast<_Float16*>(Ap)[tid] = (_Float16)0.0f;
  reinterpret_cast<_Float16*>(Ap + AROWS * XSB)[tid] = (_Float16)0.0f;
  int ax;  // the accumulators of the current segment hold (A * 2^-ax) W
  {
    float a[32];
    float m = 0.f;
    const float* src = ta.pooled + (size_t)w * 32 * 256 + tid;
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      a[j] = src[j * 256];
      m = fmaxf(m, fabsf(a[j]));
    }
    ax = fp16_range_exp(block_max(m));
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      if constexpr (SPA)
        split_store(reinterpret_cast<_Float16*>(Ap + (1 + j) * XSB) + tid,
                    reinterpret_cast<_Float16*>(Ap + (AROWS + 1 + j) * XSB) + tid, ldexpf(a[j], -ax));
      else
        reinterpret_cast<_Float16*>(Ap + (1 + j) * XSB)[tid] = (_Float16)ldexpf(a[j], -ax);
    }
  }
  __syncthreads();

  // ---- the segment stream -----------------------------------------------------------------------------
  const int nseg = 1 + 12 * ta.n_layers;
  auto seg_base = [&](int s) -> gchar {
#if VGE_ABL & 32
    return (gchar)ta.ov_w;  // timing ablation: every segment re-reads the 256 KB token matrix (L2 resident)
#endif
    if (s == 0) return (gchar)ta.ov_w;
    const TxLayerX3& L = ta.layers[(s - 1) / 12];
    const int p = (s - 1) % 12;
    if (p < 3) return (gchar)L.in_w + (size_t)p * 16 * CHUNK_B;
    if (p == 3) return (gchar)L.out_w;
    const int hc = (p - 4) >> 1;
    return ((p - 4) & 1) ? (gchar)L.l2_w + (size_t)hc * 16 * CHUNK_B : (gchar)L.l1_w + (size_t)hc * 16 * CHUNK_B;
  };

  Acc<1, 2> acc, acc2;  // acc: the segment's accumulators; acc2: the FFN2 sum across its K panels
  acc.zero();
  acc2.zero();
  float c0[2] = {0.f, 0.f}, c02[2] = {0.f, 0.f};  // the CLS row's partial sums (this lane's half of the k)
  float X[2][16], x0[2] = {0.f, 0.f};             // the layer input / residual: token rows trow(r), CLS
  int hexp = 0;                                    // acc2 / c02 hold (H W2^T) * 2^-hexp

  // the token epilogue's constants, loaded before the first weight loads (see the epilogue parameters below)
#pragma unroll
  for (int n = 0; n < 2; ++n) {
#pragma unroll
    for (int r = 0; r < 16; ++r) X[n][r] = ta.pe[trow(r) * 256 + col0 + 32 * n];
    x0[n] = ta.cls[col0 + 32 * n] + ta.pe[col0 + 32 * n];
  }

  BFrag<2> b[TX_PF];
  gchar seg_next = seg_base(0);
#pragma unroll
  for (int j = 0; j < TX_PF - 1; ++j) load_b<2, SPW>(seg_next, j, loff, b[j]);

  for (int s = 0; s < nseg; ++s) {
    {  // lane-derived values re-derived per segment: stops the compiler from hoisting the ~100 (64-bit,
       // loop-invariant) epilogue addresses out of the loop, where they would hold registers throughout
      int lo = lane;
      asm volatile("" : "+v"(lo));
      i = lo & 31;
      h = lo >> 5;
      col0 = wave * 64 + i;
    }
    const int p = (s == 0) ? -1 : (s - 1) % 12;
    const int l = (s == 0) ? 0 : (s - 1) / 12;
    const bool use_h = (p >= 5) && (((p - 4) & 1) == 1);
    const char* abase = use_h ? U : Ap;
    auto afn = [&](int c, AFragT& f) {
      f.h = *reinterpret_cast<const half8*>(abase + aoff + c * 32);
      f.h0 = *reinterpret_cast<const half8*>(abase + aoff0 + c * 32);
      if constexpr (SPA) {
        f.l = *reinterpret_cast<const half8*>(abase + aoff + c * 32 + AROWS * XSB);
        f.l0 = *reinterpret_cast<const half8*>(abase + aoff0 + c * 32 + AROWS * XSB);
      }
    };
    TSTAMP(2 * s);
    // this segment's epilogue parameters (column scales, bias, LayerNorm affine), loaded before its weight
    // stream: vmcnt retires in order, so a load issued in the epilogue would wait for the prefetched chunks
    float ecs[2] = {0.f, 0.f}, eb[2] = {0.f, 0.f}, eg[2] = {0.f, 0.f}, ebt[2] = {0.f, 0.f};
    {
      const float *pcs = nullptr, *pb = nullptr, *pg = nullptr, *pbt = nullptr;
      if (s == 0) {
        pcs = ta.ov_cs;
      } else {
        const TxLayerX3& L = ta.layers[l];
        const int hc = (p - 4) >> 1;
        if (p < 3) {
          pcs = L.in_cs + p * 256;
          pb = L.in_b + p * 256;
        } else if (p == 3) {
          pcs = L.out_cs; pb = L.out_b; pg = L.n1_w; pbt = L.n1_b;
        } else if (((p - 4) & 1) == 0) {
          pcs = L.l1_cs + hc * 256;
          pb = L.l1_b + hc * 256;
        } else if (hc == 3) {
          pcs = L.l2_cs; pb = L.l2_b; pg = L.n2_w; pbt = L.n2_b;
        }
      }
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        if (pcs) ecs[n] = pcs[col0 + 32 * n];
        if (pb) eb[n] = pb[col0 + 32 * n];
        if (pg) {
          eg[n] = pg[col0 + 32 * n];
          ebt[n] = pbt[col0 + 32 * n];
        }
      }
    }
    AFragT a[2];
    afn(0, a[0]);
    // chunk c + PF - 1 of this segment, or chunk c + PF - 17 of the next (the last segment re-reads its own)
    const gchar seg_cur = seg_next;
    seg_next = seg_base(s + 1 < nseg ? s + 1 : s);
#pragma unroll
    for (int c = 0; c < 16; ++c) {
#if !(VGE_ABL & 2)
      if (c + TX_PF - 1 < 16) load_b<2, SPW>(seg_cur, c + TX_PF - 1, loff, b[(c + TX_PF - 1) % TX_PF]);
      else load_b<2, SPW>(seg_next, c + TX_PF - 1 - 16, loff, b[(c + TX_PF - 1) % TX_PF]);
#endif
      if (c + 1 < 16) afn(c + 1, a[(c + 1) & 1]);
      const AFragT& f = a[c & 1];
      const BFrag<2>& bb = b[c % TX_PF];
#pragma unroll
      for (int n = 0; n < 2; ++n) {
#if !(VGE_ABL & 1)
        acc.c[0][n] = mfma32(f.h, bb.h[n], acc.c[0][n]);
        if constexpr (SPW) acc.c[0][n] = mfma32(f.h, bb.l[n], acc.c[0][n]);
        if constexpr (SPA) acc.c[0][n] = mfma32(f.l, bb.h[n], acc.c[0][n]);
#else
        asm volatile("" ::"v"(f.h), "v"(f.l), "v"(bb.h[n]), "v"(bb.l[n]));
#endif
#if !(VGE_ABL & 64)
        c0[n] = cls_dot<SPA, SPW>(c0[n], f.h0, f.l0, bb.h[n], bb.l[n]);
#endif
      }
      // the CLS dot products stay in their step (else they are sunk past the loop and the ring stays live)
      asm volatile("" : "+v"(c0[0]), "+v"(c0[1])::"memory");
      __builtin_amdgcn_sched_barrier(0);
      // keep the waves abreast (see run_stream); the barrier after the last chunk also orders every
      // epilogue's LDS writes after all waves' reads of the segment's A planes
      if (c % TX_PF == TX_PF - 1 && (!(VGE_ABL & 128) || c == 15)) lds_barrier();
    }

    TSTAMP(2 * s + 1);
    tr_s = s;
    // ---- segment epilogues ------------------------------------------------------------------------------
    const float xs = ldexpf(1.0f, ax);
    float cl[2];  // the CLS row of this segment's product (both k halves)
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      cl[n] = both_halves(c0[n]);
      c0[n] = 0.f;
    }
    if (s == 0) {
      // tokens: CLS = cls + pe_0, frames = pooled Wov^T + pe_t
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const float cs = ecs[n] * xs;
#pragma unroll
        for (int r = 0; r < 16; ++r) X[n][r] += acc.c[0][n][r] * cs;  // X holds pe, x0 cls + pe_0
      }
      acc.zero();
      ax = split_rows(Ap, X, x0);
      __syncthreads();
      continue;
    }
    const TxLayerX3& L = ta.layers[l];
    if (p < 3) {
      // q / k / v block p -> f32 staging U[p][row][col]
      float* dst = reinterpret_cast<float*>(U) + p * TOK * QS;
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const int col = col0 + 32 * n;
        const float cs = ecs[n] * xs, bb = eb[n];
#pragma unroll
        for (int r = 0; r < 16; ++r) dst[trow(r) * QS + col] = acc.c[0][n][r] * cs + bb;
        if (h == 0) dst[col] = cl[n] * cs + bb;
      }
      acc.zero();
      if (p == 2) {
        __syncthreads();  // q, k, v complete; every wave is done reading the X planes
        // attention, heads 2 wave + e (scale 1/sqrt(32)), exact f32 MFMAs (v_mfma_f32_32x32x2_f32) for the
        // 32 x 32 frame block, the CLS query / CLS key on the VALU:
        //   S^T[k][q] = K_k . Q_q (frame keys k, frame queries q, C layout: lane = query, registers = keys)
        //   softmax over the keys of a query = over a lane's 16 registers, its partner half and the CLS key
        //   O^T[d][q] = sum_k V^T[d][k] P^T[k][q] (B operand = P^T straight from the C registers)
        const float* Uf = reinterpret_cast<const float*>(U);
        constexpr float kScale = 0.17677669529663687f;
        floatx16 ot[2];   // O[1 + i][d], d = (r & 3) + 8 (r >> 2) + 4 h
        float oc[2];      // O[0][d = i] (CLS query), lanes with h == 0
        float m = 0.f;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const float* Qh = Uf + (2 * wave + e) * 32;
          const float* Kh = Qh + TOK * QS;
          const float* Vh = Qh + 2 * TOK * QS;
          // frame block scores; d ordered so lane half h reads d = 16 h .. 16 h + 15 contiguously
          floatx4 ka[4], qb[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            ka[j] = *reinterpret_cast<const floatx4*>(Kh + (1 + i) * QS + 16 * h + 4 * j);
            qb[j] = *reinterpret_cast<const floatx4*>(Qh + (1 + i) * QS + 16 * h + 4 * j);
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
            const float va = Vh[(1 + (t & 3) + 8 * (t >> 2) + 4 * h) * QS + i];
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
              m = fmaxf(m, fabsf(o[4 * g + k]));
            }
          }
          ot[e] = o;
          // CLS query: lane l <= 32 scores key l, the wave reduces; lane d < 32 then sums P V over the keys
          float s0 = -INFINITY;
          if (lane < TOK) {
            float a = 0.f;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const floatx4 q0 = *reinterpret_cast<const floatx4*>(Qh + 4 * j);
              const floatx4 kl = *reinterpret_cast<const floatx4*>(Kh + lane * QS + 4 * j);
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
            acc0[k % 3] += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(p0), k)) * Vh[k * QS + i];
          oc[e] = ((acc0[0] + acc0[1]) + acc0[2]) / d0;
          if (h == 0) m = fmaxf(m, fabsf(oc[e]));
        }
        ax = fp16_range_exp(block_max(m));
        {  // att -> the A planes of out_proj: frame rows 1 + i, CLS row 0
          const float scl = ldexpf(1.0f, -ax);
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            char* rh = Ap + (1 + i) * XSB + (2 * wave + e) * 64;
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              typedef _Float16 half4v __attribute__((ext_vector_type(4)));
              half4v hv, lv;
#pragma unroll
              for (int k = 0; k < 4; ++k) {
                const float y = ot[e][4 * g + k] * scl;
                hv[k] = (_Float16)y;
                lv[k] = (_Float16)(y - (float)hv[k]);
              }
              *reinterpret_cast<half4v*>(rh + (8 * g + 4 * h) * 2) = hv;
              if constexpr (SPA) *reinterpret_cast<half4v*>(rh + (8 * g + 4 * h) * 2 + AROWS * XSB) = lv;
            }
            if (h == 0) {
              const float y = oc[e] * scl;
              const _Float16 hi = (_Float16)y;
              reinterpret_cast<_Float16*>(Ap)[(2 * wave + e) * 32 + i] = hi;
              if constexpr (SPA)
                reinterpret_cast<_Float16*>(Ap + AROWS * XSB)[(2 * wave + e) * 32 + i] = (_Float16)(y - (float)hi);
            }
          }
        }
        __syncthreads();
      }
      continue;
    }
    if (p == 3) {
      // out_proj + bias + residual -> LN1 -> X1 (kept in X) and the A planes of linear1
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const float cs = ecs[n] * xs, bb = eb[n];
#pragma unroll
        for (int r = 0; r < 16; ++r) X[n][r] += acc.c[0][n][r] * cs + bb;
        x0[n] += cl[n] * cs + bb;
      }
      acc.zero();
      layer_norm(X, x0, eg, ebt);
      // a LayerNorm output's range is known statically; the barrier orders the writes after every wave's
      // reads of the att planes (the out_proj stream) -- those all precede the LayerNorm's reductions
      TSTAMP_FINE(4);
      ax = split_rows_e(Ap, X, x0, L.e_x1);
      TSTAMP_FINE(5);
      __syncthreads();
      TSTAMP_FINE(6);
      continue;
    }
    const int hc = (p - 4) >> 1;
    if (((p - 4) & 1) == 0) {
      // linear1 chunk hc: H = relu(X1 W1_hc^T + b1) -> hidden planes; acc <- the FFN2 running sum
      float hv[2][16], h0[2];
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const float cs = ecs[n] * xs, bb = eb[n];
#pragma unroll
        for (int r = 0; r < 16; ++r) hv[n][r] = fmaxf(acc.c[0][n][r] * cs + bb, 0.f);
        h0[n] = fmaxf(cl[n] * cs + bb, 0.f);
      }
      // one static exponent for all four hidden chunks: the running FFN2 sum needs no rescale
      hexp = split_rows_e(U, hv, h0, L.e_h);
      if (hc == 0) {
        acc.zero();
      } else {
        acc = acc2;
#pragma unroll
        for (int n = 0; n < 2; ++n) c0[n] = (h == 0) ? c02[n] : 0.f;  // c02 holds both k halves: one half carries it
      }
      __syncthreads();
      continue;
    }
    // linear2 K panel hc done
    if (hc < 3) {
      acc2 = acc;
#pragma unroll
      for (int n = 0; n < 2; ++n) c02[n] = cl[n];
      acc.zero();
      continue;
    }
    {
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const float cs = ecs[n] * ldexpf(1.0f, hexp), bb = eb[n];
#pragma unroll
        for (int r = 0; r < 16; ++r) X[n][r] += acc.c[0][n][r] * cs + bb;
        x0[n] += cl[n] * cs + bb;
      }
      acc.zero();
      layer_norm(X, x0, eg, ebt);
      if (l + 1 < ta.n_layers) {  // (every wave's reads of the X1 planes precede the LayerNorm's barriers)
        TSTAMP_FINE(4);
        ax = split_rows_e(Ap, X, x0, L.e_x2);
        TSTAMP_FINE(5);
        __syncthreads();
        TSTAMP_FINE(6);
      }
    }
  }

  TSTAMP(125);
  // ---- outputs: L2-normalised tokens, the CLS row as seq_embed, the window's temporal-coherence term
  float ss[2][16], ss0[2];
#pragma unroll
  for (int n = 0; n < 2; ++n) {
#pragma unroll
    for (int r = 0; r < 16; ++r) ss[n][r] = X[n][r] * X[n][r];
    ss0[n] = x0[n] * x0[n];
  }
  row_sums(ss, ss0);
  // F.normalize: x / max(||x||, 1e-12), as x * (1 / max(...)) once per row
  float inv_norm[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) inv_norm[r] = 1.0f / fmaxf(sqrtf(ss[0][r]), 1e-12f);
  const float inv_norm0 = 1.0f / fmaxf(sqrtf(ss0[0]), 1e-12f);
  float* F = reinterpret_cast<float*>(U);  // [TOK][QS] normalised tokens
#pragma unroll
  for (int n = 0; n < 2; ++n) {
    const int col = col0 + 32 * n;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float f = X[n][r] * inv_norm[r];
      F[trow(r) * QS + col] = f;
      if (ta.frame) ta.frame[((size_t)w * TOK + trow(r)) * 256 + col] = f;
    }
    if (h == 0) {
      const float f0 = x0[n] * inv_norm0;
      F[col] = f0;
      if (ta.frame) ta.frame[(size_t)w * TOK * 256 + col] = f0;
      ta.seq[(size_t)w * 256 + col] = f0;
    }
  }
  __syncthreads();
  if (ta.tc) {
    // |f_r - f_{r-1}| for r = 2..32 (frame_embeds[1:], eval.py:221-224): wave k takes rows 2+k, 6+k, ...
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
    float* rt = red + 2 * TOK * TX_NW + 2 * TX_NW;
    if (lane == 0) rt[wave] = tsum;
    __syncthreads();
    if (tid == 0) ta.tc[w] = ((rt[0] + rt[1]) + (rt[2] + rt[3])) / (float)(TOK - 2);
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
  const void* k[3] = {(const void*)transformer_x3_kernel<true, true>, (const void*)transformer_x3_kernel<true, false>,
                      (const void*)transformer_x3_kernel<false, false>};
  for (auto f : k) {
    const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, TX_LDS_BYTES);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
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
  auto k = mode == 2 ? transformer_x3_kernel<true, true>
                     : (mode == 1 ? transformer_x3_kernel<true, false> : transformer_x3_kernel<false, false>);
  hipLaunchKernelGGL(k, dim3(a.n_windows), dim3(256), TX_LDS_BYTES, s, t);
  return hipGetLastError();
}

}  // namespace vge

#ifdef VGE_TRACE
extern "C" int vge_debug_tx_trace(long long* host, int n) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_vge_tx_trace), sizeof(long long) * (size_t)n);
}
#endif
