// Split-precision ("3xfp16") MFMA path of the fusion encoder (gfx950).
//
// Every GEMM operand x is carried as two fp16 planes, hi = f16(x) and lo = f16((x - hi) * 2^11), and
// each product is formed as hi_a*hi_b + 2^-11 (hi_a*lo_b + lo_a*hi_b) with v_mfma_f32_32x32x16_f16
// (f32 accumulate; two accumulators, combined in the epilogue).  The dropped lo*lo term and the fp16
// rounding of lo leave a relative error of ~2^-21 per product, i.e. f32-class results (measured AC/TC
// deviation from the exact f32 path ~1e-7, see tests/test_gpu_parity.py), at 3 f16 MFMAs per K=16
// step instead of 4 f32 MFMAs per K=4 step: 5.3x the f32 MFMA rate.
//
//   conv_encoder_x3_kernel   MovementConvEncoder x10 (model.py:21-58), one workgroup = 1 encoder x 2 windows,
//                            activations in LDS as hi/lo planes for the whole chain, weights streamed through
//                            a 5-slot LDS ring of 16 KB chunks by global_load_lds (chunk c+4 in flight while
//                            chunk c is multiplied; counted vmcnt + raw s_barrier).
//   gemm_x3_kernel<EPI>      transformer / token GEMMs with the same fused epilogues as the f32 path.
//
// MFMA maps (v_mfma_f32_32x32x16_f16): lane l (i = l&31, h = l>>5) supplies A[row i][k = 8h + j] and
// B[k = 8h + j][col i], j = 0..7; C/D: col = l&31, row = (r&3) + 8(r>>2) + 4(l>>5), r = 0..15.
// A chunk = 16 K x 256 columns: [plane][h][n][8] fp16 = 16 KB, the exact LDS image the B reads use.
#include "vge_common.h"
#include <cstring>

namespace {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

#ifndef VGE_ABL
#define VGE_ABL 0  // kernel ablation builds (tools/time_encoder.py); 0 = the product
#endif
constexpr int XS = 264;              // fp16 per LDS activation row (256 + 8 pad: conflict-free b128 reads)
constexpr int CHUNK_H = 8192;        // fp16 per weight chunk (16 KB)
constexpr int NSLOT = 5;             // LDS ring depth
constexpr float LO_SCALE = 2048.0f;  // 2^11
constexpr float LO_INV = 1.0f / 2048.0f;

__device__ __forceinline__ floatx16 mfma32(half8 a, half8 b, floatx16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void split_store(_Float16* hi, _Float16* lo, float v) {
  const _Float16 h = (_Float16)v;
  *hi = h;
  *lo = (_Float16)((v - (float)h) * LO_SCALE);
}

__device__ __forceinline__ void stage_chunk16(const _Float16* __restrict__ chunk, _Float16* slot, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int piece = wave * 4 + i;  // 1 KB = 512 fp16 per wave-instruction
    glds16(chunk + piece * 512 + lane * 8, slot + piece * 512);
  }
}

template <int NT>
struct Acc {
  floatx16 hh[NT];
  floatx16 x[NT];
};

template <int NT>
__device__ __forceinline__ void acc_zero(Acc<NT>& a) {
#pragma unroll
  for (int n = 0; n < NT; ++n) {
#pragma unroll
    for (int r = 0; r < 16; ++r) { a.hh[n][r] = 0.f; a.x[n][r] = 0.f; }
  }
}

// A and B fragments of one 16-K chunk for NT n-tiles
template <int NT>
struct Frag {
  half8 ah, al;
  half8 bh[NT], bl[NT];
};

template <int NT>
__device__ __forceinline__ void load_b(Frag<NT>& f, const _Float16* slot, int nb0, int lane) {
  const int i = lane & 31, h = lane >> 5;
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    const int col = nb0 + n * 32 + i;
    f.bh[n] = *reinterpret_cast<const half8*>(slot + ((0 * 2 + h) * 256 + col) * 8);
    f.bl[n] = *reinterpret_cast<const half8*>(slot + ((1 * 2 + h) * 256 + col) * 8);
  }
}

template <int NT>
__device__ __forceinline__ void mma_frag(Acc<NT>& acc, const Frag<NT>& f) {
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    acc.hh[n] = mfma32(f.ah, f.bh[n], acc.hh[n]);
    acc.x[n] = mfma32(f.ah, f.bl[n], acc.x[n]);
    acc.x[n] = mfma32(f.al, f.bh[n], acc.x[n]);
  }
}

// vmcnt(4 * k) for a runtime k in [0, 3]
__device__ __forceinline__ void vmcnt_chunks(int k) {
  if (k >= 3) vmcnt<12>();
  else if (k == 2) vmcnt<8>();
  else if (k == 1) vmcnt<4>();
  else vmcnt<0>();
}

// Stream nchunks 16 KB weight chunks through the NSLOT-deep LDS ring.  afn(c, ah, al) loads this lane's
// A fragments of chunk c.  Fragments are double-buffered in registers: iteration c multiplies chunk c
// from registers while the ds_reads of chunk c+1 and the DMA of chunk c+NSLOT are in flight.  One
// counted vmcnt (retire chunk c+1, leave the newer DMA in flight) + raw s_barrier per chunk.
template <int NT, class AFn>
__device__ __forceinline__ void stream_step(Acc<NT>& acc, Frag<NT>& use, Frag<NT>& nxt, const _Float16* __restrict__ chunks,
                                            int nchunks, _Float16* ring, AFn& afn, int nb0, int wave, int lane, int c) {
  // retire chunk c+1 (issued chunks newer than it: c+2 .. min(c+NSLOT-1, n-1))
  vmcnt_chunks(min(c + NSLOT - 1, nchunks - 1) - (c + 1));
  lds_barrier();  // every wave's reads of chunk c's slot are done; chunk c+1 visible
#if VGE_ABL != 2
  if (c + NSLOT < nchunks) stage_chunk16(chunks + (size_t)(c + NSLOT) * CHUNK_H, ring + (c % NSLOT) * CHUNK_H, wave, lane);
#endif
  if (c + 1 < nchunks) {
    afn(c + 1, nxt.ah, nxt.al);
#if VGE_ABL != 3
    load_b(nxt, ring + ((c + 1) % NSLOT) * CHUNK_H, nb0, lane);
#endif
  }
#if VGE_ABL != 1
  mma_frag(acc, use);
#else
  asm volatile("" ::"v"(use.ah), "v"(use.bh[0]), "v"(use.bl[NT - 1]));
#endif
}

template <int NT, class AFn>
__device__ __forceinline__ void run_stream_x3(Acc<NT>& acc, const _Float16* __restrict__ chunks, int nchunks, _Float16* ring,
                                              AFn afn, int nb0, int wave, int lane) {
  const int pre = min(nchunks, NSLOT);
  for (int c = 0; c < pre; ++c) stage_chunk16(chunks + (size_t)c * CHUNK_H, ring + c * CHUNK_H, wave, lane);
  vmcnt_chunks(pre - 1);  // chunk 0 landed
  lds_barrier();
  Frag<NT> f0, f1;
  afn(0, f0.ah, f0.al);
  load_b(f0, ring, nb0, lane);
  for (int c = 0; c < nchunks; c += 2) {
    stream_step(acc, f0, f1, chunks, nchunks, ring, afn, nb0, wave, lane, c);
    if (c + 1 < nchunks) stream_step(acc, f1, f0, chunks, nchunks, ring, afn, nb0, wave, lane, c + 1);
  }
  vmcnt<0>();
  lds_barrier();  // ring and X free for the caller
}

// ------------------------------------------------------------------ conv encoder chain
struct EncDescX3 {
  const _Float16* stem;  // stem chunks, panel-major: panel p has stem_chunks_p chunks
  const _Float16* conv;  // 8 convs x 5 taps x 16 chunks
  const _Float16* proj;  // 16 chunks
  const float* gn_w;     // [4][256]
  const float* gn_b;     // [4][256]
  int in_col, d_in, n_stem_panels, pad;
};

constexpr int XROWS = 65;  // 64 activation rows + one all-zero row that masked (out-of-window) taps read
constexpr int CONVX3_LDS_BYTES = 2 * XROWS * XS * 2 + NSLOT * CHUNK_H * 2 + 64 * 4;

__global__ void __launch_bounds__(256, 1) conv_encoder_x3_kernel(const float* __restrict__ feats, int n_windows,
                                                                  const EncDescX3* __restrict__ encs, int n_enc,
                                                                  float* __restrict__ enc_out) {
  extern __shared__ __attribute__((aligned(16))) _Float16 ldsh[];
  _Float16* Xh = ldsh;                       // [65][XS]
  _Float16* Xl = ldsh + XROWS * XS;          // [65][XS]
  _Float16* ring = ldsh + 2 * XROWS * XS;    // NSLOT x CHUNK_H
  float* red = reinterpret_cast<float*>(ring + NSLOT * CHUNK_H);  // [16]

  const int n_pairs = (n_windows + 1) >> 1;
  const int nblk = n_enc * n_pairs;
  const int b = blockIdx.x;
  const int q8 = nblk >> 3, r8 = nblk & 7, x8 = b & 7;
  const int work = (x8 < r8 ? x8 * (q8 + 1) : r8 * (q8 + 1) + (x8 - r8) * q8) + (b >> 3);
  const int e = work / n_pairs, pair = work % n_pairs;
  const EncDescX3 ed = encs[e];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int rt = wave >> 1;          // row tile = window within the pair
  const int nb0 = (wave & 1) * 128;  // this wave's 128 output columns
  const int i = lane & 31, h = lane >> 5;
  const int win = pair * 2 + rt;
  const bool win_valid = win < n_windows;

  Acc<4> acc;
  floatx16 res[4];
  for (int c = threadIdx.x; c < XS; c += 256) {  // the zero row
    Xh[64 * XS + c] = (_Float16)0.0f;
    Xl[64 * XS + c] = (_Float16)0.0f;
  }

  auto store_x = [&](const floatx16 (&v)[4]) {
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = rt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int col = nb0 + n * 32 + i;
        split_store(Xh + row * XS + col, Xl + row * XS + col, v[n][r]);
      }
  };

  // ---------------- stem: Conv1d(d_in -> 256, k=1, no bias), K streamed in 256-wide panels
  acc_zero(acc);
  const _Float16* stem_chunks = ed.stem;
  for (int p = 0; p < ed.n_stem_panels; ++p) {
    const int kw = min(256, ed.d_in - p * 256);
    const int nch = (kw + 15) >> 4;
    __syncthreads();
    for (int r = 0; r < 64; ++r) {
      const int w = pair * 2 + (r >> 5);
      float v = 0.f;
      if (tid < kw && w < n_windows) v = feats[((size_t)w * VGE_T + (r & 31)) * VGE_FD + ed.in_col + p * 256 + tid];
      split_store(Xh + r * XS + tid, Xl + r * XS + tid, v);
    }
    __syncthreads();
    auto afn = [&](int c, half8& ah, half8& al) {
      const int off = (rt * 32 + i) * XS + 16 * c + 8 * h;
      ah = *reinterpret_cast<const half8*>(Xh + off);
      al = *reinterpret_cast<const half8*>(Xl + off);
    };
    run_stream_x3<4>(acc, stem_chunks, nch, ring, afn, nb0, wave, lane);
    stem_chunks += (size_t)nch * CHUNK_H;
  }
#pragma unroll
  for (int n = 0; n < 4; ++n)
#pragma unroll
    for (int r = 0; r < 16; ++r) res[n][r] = acc.hh[n][r] + acc.x[n][r] * LO_INV;
  store_x(res);
  __syncthreads();

  // ---------------- 4 TemporalConvBlocks
  for (int blk = 0; blk < 4; ++blk) {
    const int dil = 1 << blk;
    for (int cv = 0; cv < 2; ++cv) {
      acc_zero(acc);
      auto afn = [&](int c, half8& ah, half8& al) {
        const int tap = c >> 4, cc = c & 15;
        const int tt = i + (tap - 2) * dil;
        const int row = ((unsigned)tt < 32u) ? rt * 32 + tt : 64;  // out of the window -> zero row
        const int off = row * XS + 16 * cc + 8 * h;
        ah = *reinterpret_cast<const half8*>(Xh + off);
        al = *reinterpret_cast<const half8*>(Xl + off);
      };
      run_stream_x3<4>(acc, ed.conv + (size_t)(blk * 2 + cv) * 5 * 16 * CHUNK_H, 5 * 16, ring, afn, nb0, wave, lane);
      floatx16 (&v)[4] = acc.hh;  // combine in place: hh + 2^-11 x
      if (cv == 0) {
#pragma unroll
        for (int n = 0; n < 4; ++n)
#pragma unroll
          for (int r = 0; r < 16; ++r) v[n][r] = gelu_erf(acc.hh[n][r] + acc.x[n][r] * LO_INV);
      } else {
        float s = 0.f;
#pragma unroll
        for (int n = 0; n < 4; ++n)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            v[n][r] = gelu_erf(acc.hh[n][r] + acc.x[n][r] * LO_INV + res[n][r]);
            s += v[n][r];
          }
        s = wave_sum(s);
        if (lane == 0) red[wave] = s;
        __syncthreads();
        const float mean = (red[rt * 2] + red[rt * 2 + 1]) / 8192.0f;
        float q = 0.f;
#pragma unroll
        for (int n = 0; n < 4; ++n)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float d = v[n][r] - mean;
            q += d * d;
          }
        q = wave_sum(q);
        if (lane == 0) red[4 + wave] = q;
        __syncthreads();
        const float var = (red[4 + rt * 2] + red[4 + rt * 2 + 1]) / 8192.0f;
        const float rstd = 1.0f / sqrtf(var + 1e-5f);
#pragma unroll
        for (int n = 0; n < 4; ++n) {
          const int col = nb0 + n * 32 + i;
          const float w_ = ed.gn_w[blk * 256 + col], b_ = ed.gn_b[blk * 256 + col];
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            v[n][r] = (v[n][r] - mean) * rstd * w_ + b_;
            res[n][r] = v[n][r];
          }
        }
      }
      store_x(v);  // the stream's final barrier retired every read of X
      __syncthreads();
    }
  }

  // ---------------- proj: Linear(256 -> 256, no bias)
  acc_zero(acc);
  {
    auto afn = [&](int c, half8& ah, half8& al) {
      const int off = (rt * 32 + i) * XS + 16 * c + 8 * h;
      ah = *reinterpret_cast<const half8*>(Xh + off);
      al = *reinterpret_cast<const half8*>(Xl + off);
    };
    run_stream_x3<4>(acc, ed.proj, 16, ring, afn, nb0, wave, lane);
  }
  if (win_valid) {
    float* o = enc_out + ((size_t)e * n_windows * VGE_T + (size_t)win * VGE_T) * VGE_D;
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
        o[row * VGE_D + nb0 + n * 32 + i] = acc.hh[n][r] + acc.x[n][r] * LO_INV;
      }
  }
}

// ------------------------------------------------------------------ panel GEMM (3xfp16) with fused epilogues
enum Epi { EPI_TOKENS = 0, EPI_BIAS = 1, EPI_BIAS_RELU = 2, EPI_BIAS_RES_LN = 3 };

struct GemmArgsX3 {
  const float* A;  int lda;
  const _Float16* W;            // chunks [N/256][K/16][CHUNK_H]
  float* out;      int ldo;
  int M, K, N;
  const float* bias;
  const float* res;  int ldr;
  const float* ln_w; const float* ln_b;
  const float* pe;
  const float* cls;
};

// block = 4 waves = 2 row tiles (32 rows) x 2 column halves (128 cols): BM = 64, BN = 256
constexpr int GEMMX3_LDS_BYTES = 2 * 64 * XS * 2 + NSLOT * CHUNK_H * 2 + 128 * 4;

template <int EPI>
__global__ void __launch_bounds__(256, 1) gemm_x3_kernel(GemmArgsX3 ga) {
  extern __shared__ __attribute__((aligned(16))) _Float16 ldsh[];
  _Float16* Xh = ldsh;
  _Float16* Xl = ldsh + 64 * XS;
  _Float16* ring = ldsh + 2 * 64 * XS;
  float* red = reinterpret_cast<float*>(ring + NSLOT * CHUNK_H);  // [64 rows][2]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int rt = wave >> 1, nb0 = (wave & 1) * 128;
  const int i = lane & 31, h = lane >> 5;
  const int row0 = blockIdx.x * 64, nb = blockIdx.y;
  const int n_panels = ga.K / 256;

  Acc<4> acc;
  acc_zero(acc);
  for (int p = 0; p < n_panels; ++p) {
    __syncthreads();
    // stage the 64 x 256 A panel as hi/lo planes (rows >= M read as 0)
    for (int r = 0; r < 64; ++r) {
      const int row = row0 + r;
      const float v = (row < ga.M) ? ga.A[(size_t)row * ga.lda + p * 256 + tid] : 0.f;
      split_store(Xh + r * XS + tid, Xl + r * XS + tid, v);
    }
    __syncthreads();
    auto afn = [&](int c, half8& ah, half8& al) {
      const int off = (rt * 32 + i) * XS + 16 * c + 8 * h;
      ah = *reinterpret_cast<const half8*>(Xh + off);
      al = *reinterpret_cast<const half8*>(Xl + off);
    };
    run_stream_x3<4>(acc, ga.W + ((size_t)nb * (ga.K / 16) + p * 16) * CHUNK_H, 16, ring, afn, nb0, wave, lane);
  }

  float v[4][16];
#pragma unroll
  for (int n = 0; n < 4; ++n)
#pragma unroll
    for (int r = 0; r < 16; ++r) v[n][r] = acc.hh[n][r] + acc.x[n][r] * LO_INV;
  const int colb = nb * 256 + nb0;
  auto rowof = [&](int r) { return row0 + rt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h; };

  if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_RELU) {
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int col = colb + n * 32 + i;
      const float bb = ga.bias[col];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = rowof(r);
        float x = v[n][r] + bb;
        if (EPI == EPI_BIAS_RELU) x = fmaxf(x, 0.f);
        if (row < ga.M) ga.out[(size_t)row * ga.ldo + col] = x;
      }
    }
  } else if constexpr (EPI == EPI_TOKENS) {
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int col = colb + n * 32 + i;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = rowof(r);
        if (row < ga.M) {
          const int w = row >> 5, t = row & 31;
          ga.out[((size_t)w * VGE_TOK + 1 + t) * ga.ldo + col] = v[n][r] + ga.pe[(1 + t) * VGE_D + col];
          if (t == 0) ga.out[(size_t)w * VGE_TOK * ga.ldo + col] = ga.cls[col] + ga.pe[col];
        }
      }
    }
  } else {  // EPI_BIAS_RES_LN over the 256 columns (N == 256, one column block)
    float s[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) s[r] = 0.f;
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int col = colb + n * 32 + i;
      const float bb = ga.bias[col];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = rowof(r);
        v[n][r] += bb + ((row < ga.M) ? ga.res[(size_t)row * ga.ldr + col] : 0.f);
        s[r] += v[n][r];
      }
    }
    // row sums: reduce over the 32 lanes that share h (xor 1..16 stays inside a 32-lane half)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
#pragma unroll
      for (int o = 16; o >= 1; o >>= 1) s[r] += __shfl_xor(s[r], o, 64);
    }
    __syncthreads();
    if (i == 0) {
#pragma unroll
      for (int r = 0; r < 16; ++r) red[(rt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h) * 2 + (wave & 1)] = s[r];
    }
    __syncthreads();
    float mean[16], q[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int lr = rt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
      mean[r] = (red[lr * 2] + red[lr * 2 + 1]) / 256.0f;
      q[r] = 0.f;
    }
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float d = v[n][r] - mean[r];
        q[r] += d * d;
      }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
#pragma unroll
      for (int o = 16; o >= 1; o >>= 1) q[r] += __shfl_xor(q[r], o, 64);
    }
    __syncthreads();
    if (i == 0) {
#pragma unroll
      for (int r = 0; r < 16; ++r) red[(rt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h) * 2 + (wave & 1)] = q[r];
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int lr = rt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
      q[r] = 1.0f / sqrtf((red[lr * 2] + red[lr * 2 + 1]) / 256.0f + 1e-5f);
    }
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int col = colb + n * 32 + i;
      const float lw = ga.ln_w[col], lb = ga.ln_b[col];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = rowof(r);
        if (row < ga.M) ga.out[(size_t)row * ga.ldo + col] = (v[n][r] - mean[r]) * q[r] * lw + lb;
      }
    }
  }
}

}  // namespace

// ================================================================== host launchers
namespace vge {

struct EncDescX3Host {
  const _Float16* stem; const _Float16* conv; const _Float16* proj; const float* gn_w; const float* gn_b;
  int in_col, d_in, n_stem_panels, pad;
};
static_assert(sizeof(EncDescX3Host) == sizeof(EncDescX3), "EncDescX3 layout");

struct GemmArgsX3Host {
  const float* A; int lda; const _Float16* W; float* out; int ldo; int M, K, N;
  const float* bias; const float* res; int ldr; const float* ln_w; const float* ln_b; const float* pe; const float* cls;
};
static_assert(sizeof(GemmArgsX3Host) == sizeof(GemmArgsX3), "GemmArgsX3 layout");

hipError_t encoder_x3_kernel_setup() {
  hipError_t e = hipFuncSetAttribute((const void*)conv_encoder_x3_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     CONVX3_LDS_BYTES);
  if (e != hipSuccess) return e;
  const void* gk[4] = {(const void*)gemm_x3_kernel<EPI_TOKENS>, (const void*)gemm_x3_kernel<EPI_BIAS>,
                       (const void*)gemm_x3_kernel<EPI_BIAS_RELU>, (const void*)gemm_x3_kernel<EPI_BIAS_RES_LN>};
  for (auto k : gk) {
    e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, GEMMX3_LDS_BYTES);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t launch_conv_encoders_x3(const float* feats, int n_windows, const void* encs, int n_enc, float* enc_out,
                                   hipStream_t s) {
  const int n_pairs = (n_windows + 1) / 2;
  hipLaunchKernelGGL(conv_encoder_x3_kernel, dim3(n_enc * n_pairs), dim3(256), CONVX3_LDS_BYTES, s, feats, n_windows,
                     reinterpret_cast<const EncDescX3*>(encs), n_enc, enc_out);
  return hipGetLastError();
}

hipError_t launch_gemm_x3(int epi, const GemmArgsX3Host& a, hipStream_t s) {
  GemmArgsX3 g;
  memcpy(&g, &a, sizeof(g));
  dim3 grid((a.M + 63) / 64, a.N / 256);
  switch (epi) {
    case EPI_TOKENS: hipLaunchKernelGGL(gemm_x3_kernel<EPI_TOKENS>, grid, dim3(256), GEMMX3_LDS_BYTES, s, g); break;
    case EPI_BIAS: hipLaunchKernelGGL(gemm_x3_kernel<EPI_BIAS>, grid, dim3(256), GEMMX3_LDS_BYTES, s, g); break;
    case EPI_BIAS_RELU: hipLaunchKernelGGL(gemm_x3_kernel<EPI_BIAS_RELU>, grid, dim3(256), GEMMX3_LDS_BYTES, s, g); break;
    default: hipLaunchKernelGGL(gemm_x3_kernel<EPI_BIAS_RES_LN>, grid, dim3(256), GEMMX3_LDS_BYTES, s, g); break;
  }
  return hipGetLastError();
}

}  // namespace vge
