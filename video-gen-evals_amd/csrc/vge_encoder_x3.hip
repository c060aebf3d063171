// Split-precision ("3xfp16") MFMA path of the fusion encoder (gfx950).
//
// Every GEMM operand x is carried as two fp16 planes, hi = f16(x) and lo = f16((x - hi) * 2^11), and
// each product is formed as hi_a*hi_b + 2^-11 (hi_a*lo_b + lo_a*hi_b) with v_mfma_f32_32x32x16_f16
// (f32 accumulate; two accumulators, combined in the epilogue).  The dropped lo*lo term and the fp16
// rounding of lo leave a relative error of ~2^-21 per product, i.e. f32-class results (measured AC/TC
// deviation from the exact f32 path ~1e-7, see tests/test_gpu_parity.py), at 3 f16 MFMAs per K=16
// step instead of 4 f32 MFMAs per K=4 step: 5.3x the f32 MFMA rate.
//
//   conv_encoder_x3_kernel   MovementConvEncoder x10 (model.py:21-58): one workgroup = 1 encoder x 2 windows
//                            (64 rows), 8 waves = 2 row tiles x 4 column quarters.  Activations stay in LDS
//                            as hi/lo planes for the whole chain; weights stream through a 5-slot LDS ring of
//                            16 KB chunks by global_load_lds (chunk c+5 issued while chunk c is multiplied;
//                            counted vmcnt + raw s_barrier; fragments double-buffered in registers).
//   gemm_x3_kernel<EPI>      transformer / token GEMMs, same tiling, with the fused epilogues of the f32 path.
//
// MFMA maps (v_mfma_f32_32x32x16_f16): lane l (i = l&31, h = l>>5) supplies A[row i][k = 8h + j] and
// B[k = 8h + j][col i], j = 0..7; C/D: col = l&31, row = (r&3) + 8(r>>2) + 4(l>>5), r = 0..15.
// A chunk = 16 K x 256 columns: [plane][h][n][8] fp16 = 16 KB, the exact LDS image the B reads use.
#include "vge_common.h"
#include <cstring>

#ifndef VGE_ABL
#define VGE_ABL 0  // timing-only ablation builds (tools/ablate.sh), a bit mask: 1 no MFMA, 2 no DMA after the
                   // prologue, 4 no B reads, 8 no stream barriers, 16 identity GELU; 0 = the product
#endif

namespace {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int XS = 264;              // fp16 per LDS activation row (256 + 8 pad: conflict-free b128 reads)
constexpr int XSB = XS * 2;          // bytes per activation row
constexpr int XROWS = 65;            // 64 activation rows + one all-zero row that masked conv taps read
constexpr int CHUNK_B = 16384;       // bytes per weight chunk
constexpr int PLANE_B = 8192;        // bytes between the hi and lo planes of a chunk
constexpr int NSLOT = 5;             // LDS ring depth (chunks)
constexpr int NWAVE = 8;             // waves per workgroup
constexpr int NT = 2;                // 32-column n-tiles per wave
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

struct Acc {
  floatx16 hh[NT];
  floatx16 x[NT];
};

__device__ __forceinline__ void acc_zero(Acc& a) {
#pragma unroll
  for (int n = 0; n < NT; ++n) {
#pragma unroll
    for (int r = 0; r < 16; ++r) { a.hh[n][r] = 0.f; a.x[n][r] = 0.f; }
  }
}

// A and B fragments of one 16-K chunk
struct Frag {
  half8 ah, al;
  half8 bh[NT], bl[NT];
};

__device__ __forceinline__ void mma_frag(Acc& acc, const Frag& f) {
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    acc.hh[n] = mfma32(f.ah, f.bh[n], acc.hh[n]);
    acc.x[n] = mfma32(f.ah, f.bl[n], acc.x[n]);
    acc.x[n] = mfma32(f.al, f.bh[n], acc.x[n]);
  }
}

// One workgroup's weight stream: n 16 KB chunks in HBM, a 5-slot ring in LDS.
struct Ring {
  const char* g;   // chunk 0 of the stream
  char* lds;       // ring base
  int n;           // chunks in the stream
  int wave;        // wave id (scalar)
  int lane;
  unsigned boff;   // this lane's B-fragment byte offset inside a chunk (n-tile 0, hi plane)

  // a chunk is 16 x 1 KB wave-pieces, 2 per wave (the LDS destination of a piece is wave-uniform)
  __device__ __forceinline__ void stage(int c, int slot) const {
#if !(VGE_ABL & 2)
    const char* src = g + (size_t)c * CHUNK_B + wave * 1024 + lane * 16;
    char* dst = lds + slot * CHUNK_B + wave * 1024;
    glds16(src, dst);
    glds16(src + NWAVE * 1024, dst + NWAVE * 1024);
#endif
  }
  __device__ __forceinline__ void load_b(Frag& f, int slot) const {
#if !(VGE_ABL & 4)
    const char* p = lds + slot * CHUNK_B + boff;
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      f.bh[n] = *reinterpret_cast<const half8*>(p + n * 512);
      f.bl[n] = *reinterpret_cast<const half8*>(p + n * 512 + PLANE_B);
    }
#endif
  }
};

// leave k newer chunks (2 DMA instructions each) in flight, k in [0, 3]
__device__ __forceinline__ void vm_wait_chunks(int k) {
  if (k >= 3) vmcnt<6>();
  else if (k == 2) vmcnt<4>();
  else if (k == 1) vmcnt<2>();
  else vmcnt<0>();
}

__device__ __forceinline__ int next_slot(int s) { return s == NSLOT - 1 ? 0 : s + 1; }

// One chunk step: retire chunk c+1, barrier, issue chunk c+NSLOT into chunk c's slot, read chunk c+1's
// fragments, multiply chunk c from registers.  STEADY: chunks c+2..c+4 are in flight (constant vmcnt).
template <bool STEADY, class AFn>
__device__ __forceinline__ void stream_step(Acc& acc, const Frag& use, Frag& nxt, const Ring& R, AFn& afn, int c,
                                            int slot) {
  if (STEADY) vmcnt<6>();
  else vm_wait_chunks(min(c + NSLOT - 1, R.n - 1) - (c + 1));
#if !(VGE_ABL & 8)
  lds_barrier();  // every wave's reads of chunk c's slot are done; chunk c+1 has landed for all waves
#endif
  if (c + NSLOT < R.n) R.stage(c + NSLOT, slot);
  if (STEADY || c + 1 < R.n) {
    afn(c + 1, nxt);
    R.load_b(nxt, next_slot(slot));
  }
#if !(VGE_ABL & 1)
  mma_frag(acc, use);
#else
  asm volatile("" ::"v"(use.ah), "v"(use.bh[0]), "v"(use.bl[NT - 1]));
#endif
}

// afn(c, frag) loads this lane's A fragments of chunk c
template <class AFn>
__device__ __forceinline__ void run_stream(Acc& acc, const Ring& R, AFn afn) {
  const int n = R.n;
  const int pre = min(n, NSLOT);
  for (int c = 0; c < pre; ++c) R.stage(c, c);
  vm_wait_chunks(pre - 1);  // chunk 0 landed
  lds_barrier();
  Frag f0, f1;
  afn(0, f0);
  R.load_b(f0, 0);
  int c = 0, slot = 0;
  for (; c + 1 <= n - NSLOT; c += 2) {
    stream_step<true>(acc, f0, f1, R, afn, c, slot);
    slot = next_slot(slot);
    stream_step<true>(acc, f1, f0, R, afn, c + 1, slot);
    slot = next_slot(slot);
  }
  for (; c < n; c += 2) {
    stream_step<false>(acc, f0, f1, R, afn, c, slot);
    slot = next_slot(slot);
    if (c + 1 < n) {
      stream_step<false>(acc, f1, f0, R, afn, c + 1, slot);
      slot = next_slot(slot);
    }
  }
  vmcnt<0>();
  lds_barrier();  // ring and activations free for the caller
}

// ------------------------------------------------------------------ conv encoder chain
struct EncDescX3 {
  const _Float16* stem;  // stem chunks; panel p (256 K) starts at chunk 16p, the last panel may be short
  const _Float16* conv;  // 8 convs x 5 taps x 16 chunks
  const _Float16* proj;  // 16 chunks
  const float* gn_w;     // [4][256]
  const float* gn_b;     // [4][256]
  int in_col, d_in, n_stem_panels, pad;
};

constexpr int CONVX3_LDS_BYTES = 2 * XROWS * XSB + NSLOT * CHUNK_B + (24 + 128) * 4;

__global__ void __launch_bounds__(512, 1) conv_encoder_x3_kernel(const float* __restrict__ feats, int n_windows,
                                                                  const EncDescX3* __restrict__ encs, int n_enc,
                                                                  float* __restrict__ enc_out) {
  extern __shared__ __attribute__((aligned(16))) char lds_raw[];
  _Float16* Xh = reinterpret_cast<_Float16*>(lds_raw);            // [65][XS]
  _Float16* Xl = Xh + XROWS * XS;                                 // [65][XS]
  char* ring = lds_raw + 2 * XROWS * XSB;                         // NSLOT x 16 KB
  float* red = reinterpret_cast<float*>(ring + NSLOT * CHUNK_B);  // [24]: GN sums, GN squares, |x| maxima
  int* rexp = reinterpret_cast<int*>(red + 24);                   // [2][64] stem row scale exponents

  // XCD-aware remap: the 8 XCDs take contiguous work ranges, so co-resident blocks of an XCD share an encoder
  const int n_pairs = (n_windows + 1) >> 1;
  const int nblk = n_enc * n_pairs;
  const int b = blockIdx.x;
  const int q8 = nblk >> 3, r8 = nblk & 7, x8 = b & 7;
  const int work = (x8 < r8 ? x8 * (q8 + 1) : r8 * (q8 + 1) + (x8 - r8) * q8) + (b >> 3);
  const int e = work / n_pairs, pair = work % n_pairs;
  const EncDescX3 ed = encs[e];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int rt = wave >> 2;         // row tile = window within the pair
  const int nb0 = (wave & 3) * 64;  // this wave's 64 output columns
  const int i = lane & 31, h = lane >> 5;
  const int win = pair * 2 + rt;
  const unsigned boff = (unsigned)((h * 256 + nb0 + i) * 16);
  const char* xa = reinterpret_cast<const char*>(Xh) + h * 16;  // this lane's 8 k-values of a 16-K chunk column

  Acc acc;
  floatx16 res[NT];
  if (tid < XS) {  // the zero row
    Xh[64 * XS + tid] = (_Float16)0.0f;
    Xl[64 * XS + tid] = (_Float16)0.0f;
  }

  // Store the next conv's input as window * 2^-e (exact) with the window's largest |value| in [2^8, 2^9), so
  // the fp16 planes neither overflow nor lose small values; returns e (the same for the row tile's 4 waves)
  // for the consumer to multiply its accumulators back by.  Caller guarantees X is no longer being read.
  auto store_x = [&](const floatx16 (&v)[NT]) -> int {
    float m = 0.f;
#pragma unroll
    for (int n = 0; n < NT; ++n)
#pragma unroll
      for (int r = 0; r < 16; ++r) m = fmaxf(m, fabsf(v[n][r]));
    m = wave_max(m);
    if (lane == 0) red[16 + wave] = m;
    __syncthreads();
    const float* rm = red + 16 + rt * 4;
    const float mm = fmaxf(fmaxf(rm[0], rm[1]), fmaxf(rm[2], rm[3]));
    const int e = (mm > 0.f && mm <= 3.0e38f) ? ilogbf(mm) - 8 : 0;
#pragma unroll
    for (int n = 0; n < NT; ++n)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = rt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int col = nb0 + n * 32 + i;
        split_store(Xh + row * XS + col, Xl + row * XS + col, ldexpf(v[n][r], -e));
      }
    return e;
  };
  auto a_at = [&](int row_byte, int cc, Frag& f) {
    const char* p = xa + row_byte + cc * 32;
    f.ah = *reinterpret_cast<const half8*>(p);
    f.al = *reinterpret_cast<const half8*>(p + XROWS * XSB);
  };
  const int own_row_b = (rt * 32 + i) * XSB;

  // ---------------- stem: Conv1d(d_in -> 256, k=1, no bias), K streamed in 256-wide panels
  // Per-row power-of-two scale: z-scored features leave the fp16 range when a column's train-set std is ~0
  // ((x - mean) / (std + 1e-6)), so row m of panel p is split as A[m,:] * 2^-e (exact) with the panel row's
  // largest |value| in [2^8, 2^9); the accumulators (held as C * 2^-e per row) are rescaled when e changes
  // between panels and multiplied back by 2^e at the end (all exact).  rexp[parity][row] holds e.
  acc_zero(acc);
  for (int p = 0; p < ed.n_stem_panels; ++p) {
    const int kw = min(256, ed.d_in - p * 256);
    int* ecur = rexp + (p & 1) * 64;
    // wave w stages rows 8w..8w+7, lane l columns l, l+64, l+128, l+192: 32 independent coalesced loads
    float a[8][4];
#pragma unroll
    for (int jr = 0; jr < 8; ++jr) {
      const int r = wave * 8 + jr;
      const int w = pair * 2 + (r >> 5);
      const float* src = feats + ((size_t)w * VGE_T + (r & 31)) * VGE_FD + ed.in_col + p * 256;
#pragma unroll
      for (int jc = 0; jc < 4; ++jc) {
        const int c = lane + 64 * jc;
        a[jr][jc] = (c < kw && w < n_windows) ? src[c] : 0.f;
      }
    }
#pragma unroll
    for (int jr = 0; jr < 8; ++jr) {
      float m = fmaxf(fmaxf(fabsf(a[jr][0]), fabsf(a[jr][1])), fmaxf(fabsf(a[jr][2]), fabsf(a[jr][3])));
      m = wave_max(m);
      const int e = (m > 0.f && m <= 3.0e38f) ? ilogbf(m) - 8 : 0;
      const int r = wave * 8 + jr;
      if (lane == 0) ecur[r] = e;
#pragma unroll
      for (int jc = 0; jc < 4; ++jc) {
        const int c = lane + 64 * jc;
        split_store(Xh + r * XS + c, Xl + r * XS + c, ldexpf(a[jr][jc], -e));
      }
    }
    __syncthreads();  // X and ecur complete (the previous stream's final barrier retired every read of X)
    if (p > 0) {
      const int* eprev = rexp + ((p - 1) & 1) * 64;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = rt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const float f = ldexpf(1.0f, eprev[row] - ecur[row]);
#pragma unroll
        for (int n = 0; n < NT; ++n) { acc.hh[n][r] *= f; acc.x[n][r] *= f; }
      }
    }
    auto afn = [&](int c, Frag& f) { a_at(own_row_b, c, f); };
    const Ring R{reinterpret_cast<const char*>(ed.stem) + (size_t)p * 16 * CHUNK_B, ring, (kw + 15) >> 4, wave, lane,
                 boff};
    run_stream(acc, R, afn);
  }
  {
    const int* efin = rexp + ((ed.n_stem_panels - 1) & 1) * 64;
#pragma unroll
    for (int n = 0; n < NT; ++n)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        res[n][r] = ldexpf(acc.hh[n][r] + acc.x[n][r] * LO_INV, efin[rt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h]);
  }
  int xexp = store_x(res);
  __syncthreads();

  // ---------------- 4 TemporalConvBlocks
  for (int blk = 0; blk < 4; ++blk) {
    const int dil = 1 << blk;
    for (int cv = 0; cv < 2; ++cv) {
      acc_zero(acc);
      auto afn = [&](int c, Frag& f) {
        const int tap = c >> 4, cc = c & 15;
        const int tt = i + (tap - 2) * dil;
        const int row = ((unsigned)tt < 32u) ? rt * 32 + tt : 64;  // out of the window -> zero row
        a_at(row * XSB, cc, f);
      };
      const Ring R{reinterpret_cast<const char*>(ed.conv) + (size_t)(blk * 2 + cv) * 5 * 16 * CHUNK_B, ring, 5 * 16,
                   wave, lane, boff};
      run_stream(acc, R, afn);
      floatx16 (&v)[NT] = acc.hh;  // combine in place: (hh + 2^-11 x) * 2^xexp
      const float xs = ldexpf(1.0f, xexp);
      if (cv == 0) {
#pragma unroll
        for (int n = 0; n < NT; ++n)
#pragma unroll
          for (int r = 0; r < 16; ++r) v[n][r] = gelu_erf((acc.hh[n][r] + acc.x[n][r] * LO_INV) * xs);
      } else {
        // GroupNorm(1, 256) over the window: 32 x 256 values held by the row tile's 4 waves
        float s = 0.f;
#pragma unroll
        for (int n = 0; n < NT; ++n)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            v[n][r] = gelu_erf((acc.hh[n][r] + acc.x[n][r] * LO_INV) * xs + res[n][r]);
            s += v[n][r];
          }
        s = wave_sum(s);
        if (lane == 0) red[wave] = s;
        __syncthreads();
        const float mean = (red[rt * 4] + red[rt * 4 + 1] + red[rt * 4 + 2] + red[rt * 4 + 3]) / 8192.0f;
        float q = 0.f;
#pragma unroll
        for (int n = 0; n < NT; ++n)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float d = v[n][r] - mean;
            q += d * d;
          }
        q = wave_sum(q);
        if (lane == 0) red[8 + wave] = q;
        __syncthreads();
        const float var =
            (red[8 + rt * 4] + red[8 + rt * 4 + 1] + red[8 + rt * 4 + 2] + red[8 + rt * 4 + 3]) / 8192.0f;
        const float rstd = 1.0f / sqrtf(var + 1e-5f);
#pragma unroll
        for (int n = 0; n < NT; ++n) {
          const int col = nb0 + n * 32 + i;
          const float w_ = ed.gn_w[blk * 256 + col], b_ = ed.gn_b[blk * 256 + col];
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            v[n][r] = (v[n][r] - mean) * rstd * w_ + b_;
            res[n][r] = v[n][r];
          }
        }
      }
      xexp = store_x(v);  // the stream's final barrier retired every read of X
      __syncthreads();
    }
  }

  // ---------------- proj: Linear(256 -> 256, no bias)
  acc_zero(acc);
  {
    auto afn = [&](int c, Frag& f) { a_at(own_row_b, c, f); };
    const Ring R{reinterpret_cast<const char*>(ed.proj), ring, 16, wave, lane, boff};
    run_stream(acc, R, afn);
  }
  if (win < n_windows) {
    const float xs = ldexpf(1.0f, xexp);
    float* o = enc_out + ((size_t)e * n_windows * VGE_T + (size_t)win * VGE_T) * VGE_D;
#pragma unroll
    for (int n = 0; n < NT; ++n)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
        o[row * VGE_D + nb0 + n * 32 + i] = (acc.hh[n][r] + acc.x[n][r] * LO_INV) * xs;
      }
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
};

// block = 8 waves = 2 row tiles (32 rows) x 4 column quarters (64 cols): BM = 64, BN = 256
constexpr int GEMMX3_LDS_BYTES = 2 * 64 * XSB + NSLOT * CHUNK_B + (64 * 4 + 8) * 4;

template <int EPI>
__global__ void __launch_bounds__(512, 1) gemm_x3_kernel(GemmArgsX3 ga) {
  extern __shared__ __attribute__((aligned(16))) char lds_raw[];
  _Float16* Xh = reinterpret_cast<_Float16*>(lds_raw);
  _Float16* Xl = Xh + 64 * XS;
  char* ring = lds_raw + 2 * 64 * XSB;
  float* red = reinterpret_cast<float*>(ring + NSLOT * CHUNK_B);  // [64 rows][4 column quarters] + [8] maxima
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int rt = wave >> 2, cq = wave & 3, nb0 = cq * 64;
  const int i = lane & 31, h = lane >> 5;
  const int row0 = blockIdx.x * 64, nb = blockIdx.y;
  const int n_panels = ga.K / 256;
  const unsigned boff = (unsigned)((h * 256 + nb0 + i) * 16);
  const char* xa = reinterpret_cast<const char*>(Xh) + (rt * 32 + i) * XSB + h * 16;

  Acc acc;
  acc_zero(acc);
  int aexp = 0;  // the accumulators hold C * 2^-aexp
  for (int p = 0; p < n_panels; ++p) {
    // the 64 x 256 A panel (rows >= M read as 0) as hi/lo planes of panel * 2^-e, its largest |value| in
    // [2^8, 2^9): exact power-of-two scaling that keeps fp16 in range; the accumulators are rescaled to match
    const int c = tid & 255;
    float a[32];
    float m = 0.f;
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      const int row = row0 + (tid >> 8) + 2 * j;
      a[j] = (row < ga.M) ? ga.A[(size_t)row * ga.lda + p * 256 + c] : 0.f;
      m = fmaxf(m, fabsf(a[j]));
    }
    m = wave_max(m);
    if (lane == 0) red[256 + wave] = m;
    __syncthreads();  // also: every wave is past the previous panel's stream
    float mm = red[256];
#pragma unroll
    for (int w = 1; w < NWAVE; ++w) mm = fmaxf(mm, red[256 + w]);
    const int e = (mm > 0.f && mm <= 3.0e38f) ? ilogbf(mm) - 8 : 0;
    if (p > 0 && e != aexp) {
      const float f = ldexpf(1.0f, aexp - e);
#pragma unroll
      for (int n = 0; n < NT; ++n)
#pragma unroll
        for (int r = 0; r < 16; ++r) { acc.hh[n][r] *= f; acc.x[n][r] *= f; }
    }
    aexp = e;
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      const int r = (tid >> 8) + 2 * j;
      split_store(Xh + r * XS + c, Xl + r * XS + c, ldexpf(a[j], -e));
    }
    __syncthreads();
    auto afn = [&](int cc, Frag& f) {
      f.ah = *reinterpret_cast<const half8*>(xa + cc * 32);
      f.al = *reinterpret_cast<const half8*>(xa + cc * 32 + 64 * XSB);
    };
    const Ring R{reinterpret_cast<const char*>(ga.W) + ((size_t)nb * (ga.K / 16) + p * 16) * CHUNK_B, ring, 16, wave,
                 lane, boff};
    run_stream(acc, R, afn);
  }

  float v[NT][16];
  const float as = ldexpf(1.0f, aexp);
#pragma unroll
  for (int n = 0; n < NT; ++n)
#pragma unroll
    for (int r = 0; r < 16; ++r) v[n][r] = (acc.hh[n][r] + acc.x[n][r] * LO_INV) * as;
  const int colb = nb * 256 + nb0;
  auto lrow = [&](int r) { return rt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h; };

  if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_RELU) {
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      const int col = colb + n * 32 + i;
      const float bb = ga.bias[col];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = row0 + lrow(r);
        float x = v[n][r] + bb;
        if (EPI == EPI_BIAS_RELU) x = fmaxf(x, 0.f);
        if (row < ga.M) ga.out[(size_t)row * ga.ldo + col] = x;
      }
    }
  } else if constexpr (EPI == EPI_TOKENS) {
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      const int col = colb + n * 32 + i;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = row0 + lrow(r);
        if (row < ga.M) {
          const int w = row >> 5, t = row & 31;
          ga.out[((size_t)w * VGE_TOK + 1 + t) * ga.ldo + col] = v[n][r] + ga.pe[(1 + t) * VGE_D + col];
          if (t == 0) ga.out[(size_t)w * VGE_TOK * ga.ldo + col] = ga.cls[col] + ga.pe[col];
        }
      }
    }
  } else {  // EPI_BIAS_RES_LN over the 256 columns (N == 256, one column block)
    float s[16], q[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) s[r] = 0.f;
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      const int col = colb + n * 32 + i;
      const float bb = ga.bias[col];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = row0 + lrow(r);
        v[n][r] += bb + ((row < ga.M) ? ga.res[(size_t)row * ga.ldr + col] : 0.f);
        s[r] += v[n][r];
      }
    }
    // row sums: reduce over the 32 lanes that share h (xor 1..16 stays inside a 32-lane half), then over
    // the 4 column-quarter waves through LDS
#pragma unroll
    for (int r = 0; r < 16; ++r) {
#pragma unroll
      for (int o = 16; o >= 1; o >>= 1) s[r] += __shfl_xor(s[r], o, 64);
    }
    if (i == 0) {
#pragma unroll
      for (int r = 0; r < 16; ++r) red[lrow(r) * 4 + cq] = s[r];
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float* rr = red + lrow(r) * 4;
      s[r] = (rr[0] + rr[1] + rr[2] + rr[3]) / 256.0f;  // mean
      q[r] = 0.f;
    }
#pragma unroll
    for (int n = 0; n < NT; ++n)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float d = v[n][r] - s[r];
        q[r] += d * d;
      }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
#pragma unroll
      for (int o = 16; o >= 1; o >>= 1) q[r] += __shfl_xor(q[r], o, 64);
    }
    __syncthreads();  // every wave has read the sums
    if (i == 0) {
#pragma unroll
      for (int r = 0; r < 16; ++r) red[lrow(r) * 4 + cq] = q[r];
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float* rr = red + lrow(r) * 4;
      q[r] = 1.0f / sqrtf((rr[0] + rr[1] + rr[2] + rr[3]) / 256.0f + 1e-5f);
    }
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      const int col = colb + n * 32 + i;
      const float lw = ga.ln_w[col], lb = ga.ln_b[col];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = row0 + lrow(r);
        if (row < ga.M) ga.out[(size_t)row * ga.ldo + col] = (v[n][r] - s[r]) * q[r] * lw + lb;
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
  hipLaunchKernelGGL(conv_encoder_x3_kernel, dim3(n_enc * n_pairs), dim3(512), CONVX3_LDS_BYTES, s, feats, n_windows,
                     reinterpret_cast<const EncDescX3*>(encs), n_enc, enc_out);
  return hipGetLastError();
}

hipError_t launch_gemm_x3(int epi, const GemmArgsX3Host& a, hipStream_t s) {
  GemmArgsX3 g;
  memcpy(&g, &a, sizeof(g));
  dim3 grid((a.M + 63) / 64, a.N / 256);
  switch (epi) {
    case EPI_TOKENS: hipLaunchKernelGGL(gemm_x3_kernel<EPI_TOKENS>, grid, dim3(512), GEMMX3_LDS_BYTES, s, g); break;
    case EPI_BIAS: hipLaunchKernelGGL(gemm_x3_kernel<EPI_BIAS>, grid, dim3(512), GEMMX3_LDS_BYTES, s, g); break;
    case EPI_BIAS_RELU: hipLaunchKernelGGL(gemm_x3_kernel<EPI_BIAS_RELU>, grid, dim3(512), GEMMX3_LDS_BYTES, s, g); break;
    default: hipLaunchKernelGGL(gemm_x3_kernel<EPI_BIAS_RES_LN>, grid, dim3(512), GEMMX3_LDS_BYTES, s, g); break;
  }
  return hipGetLastError();
}

}  // namespace vge
