// Staggered split-precision ("3xfp16") MovementConvEncoder chain (model.py:21-58, x10) on the 16x16x32 MFMA shape,
// gfx950.
//
// The schedule, arithmetic and exchanges are those of conv_encoder_x3s_kernel (vge_encoder_x3s.hip; read its header
// first): units of one encoder x 4 (quad) or 2 (pair) windows per 512-thread workgroup, group A = waves 0-3 (output
// columns 0..127) one phase ahead of group B = waves 4-7 (128..255), a GEMM's K streamed in two parts (P1 = the
// channels A produced, P2 = B's) so every epilogue of one half runs beside the other half's MFMA stream; GroupNorm
// folded into the next GEMM; per-half split exponents exchanged through LDS with an arrival counter.
//
// What changes is the matrix instruction: v_mfma_f32_16x16x32_f16 instead of v_mfma_f32_32x32x16_f16.  Same cycles
// per FLOP, but the chip holds a higher clock under it at this power-bound load (the stagger
// probe measured 8.5-10 % less wall time for this structure).  The shape reorganises every register mapping:
//
// * Row tiles are 16 rows: a quad has 8 (tile t = frames 4t..4t+3 of all four windows, MFMA row i = window i / 4,
//   frame 4t + i % 4), a pair 4 (frames 8t..8t+7 of both windows).  A tap that puts all of a tile's frames outside
//   the window is skipped by that tile (dilations 4 and 8; the finer tiles skip a little more than 32-row ones).
// * C layout: lane l holds columns (l & 15) and 16 + (l & 15) of its wave's 32, rows 4 (l >> 4) .. + 3 of each tile,
//   so a lane's values all belong to ONE window (quad: window l >> 4, frames 4t + r; pair: window l >> 5, frames
//   8t + 4 ((l >> 4) & 1) + r).  Per-window quantities (exponents, GroupNorm statistics) are one register per lane,
//   and their wave reductions are 16-lane DPP row reductions.
// * A fragments are read from LDS one row tile at a time through a small rolling window (X3T_AD tiles in flight),
//   not held for every tile: with 8 row tiles the per-tile buffering of the 32x32 kernel would take 64 registers.
// * Weights keep their packing (16 KB chunks of 16 K x 256 columns x {hi, lo}, [plane][h][n][8]): a 32-K step is two
//   chunks, and lane l's B fragment (column n, k = 8 (l >> 4) ..) is one 16-B load from chunk (l >> 5), half
//   (l >> 4) & 1 -- a per-lane constant offset of the buffer load.
// * Activation rows are 1,056 B ([hi 256 + 8 | lo 256 + 8] fp16) and quads' window blocks 128 B apart, which keeps
//   this shape's ds_read_b128 lane groups conflict-free (bank model over every tile, quads and pairs).
// * The GroupNorm fold corrections (the per-tap sums of W gamma / W beta over the taps inside the window) take five
//   values per column and dilation; which one a frame takes is decided at compile time (the epilogue of a block's
//   first conv is instantiated per block).
#include "vge_x3.h"
#include <type_traits>

namespace {

#ifndef X3T_GELU
#define X3T_GELU 1  // 1: gelu_fast_s (one exp2), 0: gelu_many_s (exact-erf pieces)
#endif
#ifndef X3T_PRIO
#define X3T_PRIO 1  // s_setprio 1 for the streaming half
#endif
#ifndef X3T_SKIP
#define X3T_SKIP 1  // 1: a row tile skips the taps that put all its frames outside the window (dilated convs)
#endif
#ifndef X3T_AD
#define X3T_AD 2  // row tiles whose A fragments are in flight ahead of the MFMAs
#endif
#ifndef X3T_PF_QUAD
#define X3T_PF_QUAD 2  // 32-K weight steps in flight per wave in a quad's streams (4 chunks, as the 32x32 kernel)
#endif
#ifndef X3T_PF_PAIR
#define X3T_PF_PAIR 4  // ... in a pair's
#endif
constexpr int T_WMAX = 4;
constexpr int TXR = 528;    // fp16 per row
constexpr int TXRB = 1056;  // bytes per row
constexpr int TXLO = 528;   // byte offset of the lo plane in a row
template <int W>
constexpr int t_gf() { return 16 / W; }  // frames of each window in one 16-row tile
template <int W>
constexpr int t_nt() { return 2 * W; }   // row tiles of a unit
template <int W>
constexpr int t_wsb() { return 32 * TXRB + (W >= 4 ? 128 : 0); }  // bytes per window block
template <int W>
constexpr int t_zr() { return W * t_wsb<W>(); }  // byte offset of the all-zero row
template <int W, bool SKIP>
__device__ __forceinline__ bool t_tap_ok(int t, int o) {
  constexpr int G = t_gf<W>();
  return !(X3T_SKIP && SKIP) || (G * t + G - 1 + o >= 0 && G * t + o <= 31);
}
constexpr int T_AUX_OFF = (t_zr<T_WMAX>() + TXRB + 15) / 16 * 16;

struct X3tAux {
  int rexp[2][32 * T_WMAX];       // stem row exponents, by panel parity
  float stats[2][T_WMAX][8][2];   // [block parity][window][wave] (mean, M2) of x = GELU(conv2 + res)
  float mx[2][2][T_WMAX][4];      // [exchange parity][group][window][wave in group] maxima
  int ex[2][2][T_WMAX];           // [GEMM-input parity][group][window] exponents of the stored activations
  int cnt[2];                     // exchange arrivals per group (monotonic over the launch)
};
constexpr int T_LDS_BYTES = T_AUX_OFF + (int)sizeof(X3tAux);
static_assert(T_AUX_OFF % 16 == 0, "aux alignment");
static_assert(T_LDS_BYTES <= 160 * 1024, "LDS");

template <int W>
struct Acc16 {
  floatx4 c[2 * W][2];
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int t = 0; t < 2 * W; ++t)
#pragma unroll
      for (int j = 0; j < 2; ++j) c[t][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  }
};
struct BFrag16 {  // one 32-K step of the wave's two 16-column tiles, hi and lo planes
  half8 h[2], l[2];
};

__device__ __forceinline__ floatx4 mfma16(half8 a, half8 b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// a global-address-space load (a generic pointer would become a flat load, which also counts on lgkmcnt)
__device__ __forceinline__ float tgload(const float* p) {
  return *(const __attribute__((address_space(1))) float*)p;
}

// One part of a GEMM without barriers: ntap taps x NS 32-K steps.  wb: the part's first chunk; tap k's step s reads
// chunks k * 16 + 2 s, + 1.  B fragments PF steps deep in a register ring whose slots restart at every tap; A
// fragments X3T_AD row tiles ahead.  xa: this lane's A base (the activation planes + its 16-B k block + the part's
// channel offset).  Row tile t of tap k reads, for MFMA row i, frame G t + i % G + (k - ctr) dil of window i / G, or
// the all-zero row outside the window.
template <int W, bool SKIP, int NS>
__device__ __forceinline__ void stream16(Acc16<W>& acc, const char* wb, int ntap, unsigned lb, const char* xa, int i,
                                         int dil, int ctr) {
  constexpr int NT = t_nt<W>(), G = t_gf<W>(), AD = X3T_AD;
  constexpr int PF = W >= 4 ? X3T_PF_QUAD : X3T_PF_PAIR;
  static_assert(NS % PF == 0, "ring slots restart at every tap: step s of a tap sits in slot s % PF");
  static_assert(NT % AD == 0 && AD <= NT, "A slots");
  const char* xw = xa + (i / G) * t_wsb<W>();
  const int fi = i % G;
  const char* xz = xa + t_zr<W>();
  auto rowp = [&](int k, int t) -> const char* {
    const int tt = G * t + fi + (k - ctr) * dil;
    return (unsigned)tt < 32u ? xw + tt * TXRB : xz;
  };
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(wb), (short)0, 0x7FFFFFF0, 0x00020000);
  auto ldb = [&](int k, int s, BFrag16& b) {
    const int so = (k * 16 + 2 * s) * CHUNK_B;
    b.h[0] = __builtin_bit_cast(half8, __builtin_amdgcn_raw_buffer_load_b128(rs, lb, so, 0));
    b.h[1] = __builtin_bit_cast(half8, __builtin_amdgcn_raw_buffer_load_b128(rs, lb + 256, so, 0));
    b.l[0] = __builtin_bit_cast(half8, __builtin_amdgcn_raw_buffer_load_b128(rs, lb + PLANE_B, so, 0));
    b.l[1] = __builtin_bit_cast(half8, __builtin_amdgcn_raw_buffer_load_b128(rs, lb + PLANE_B + 256, so, 0));
  };
  BFrag16 b[PF];
#pragma unroll
  for (int j = 0; j < PF - 1; ++j) ldb(0, j, b[j]);
  half8 ah[AD], al[AD];
  const char* pt[NT];
  bool okc[NT];  // tile t takes part in the current tap (uniform)
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    pt[t] = rowp(0, t);
    okc[t] = t_tap_ok<W, SKIP>(t, -ctr * dil);
  }
#pragma unroll
  for (int t = 0; t < AD; ++t)
    if (okc[t]) {
      ah[t] = *reinterpret_cast<const half8*>(pt[t]);
      al[t] = *reinterpret_cast<const half8*>(pt[t] + TXLO);
    }
#pragma unroll 1
  for (int k = 0; k < ntap; ++k) {
    const bool more = k + 1 < ntap;
    const int kn = more ? k + 1 : k;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
#if !(VGE_ABL & 2)
      {
        const int sn = s + PF - 1;
        if (sn < NS) ldb(k, sn, b[sn % PF]);
        else ldb(kn, more ? sn - NS : NS - 1, b[sn % PF]);  // (past the end: reload the last step)
      }
#endif
      const BFrag16& bb = b[s % PF];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int sl = t % AD;
#if !(VGE_ABL & 1)
        if (okc[t]) {
          acc.c[t][0] = mfma16(ah[sl], bb.h[0], acc.c[t][0]);
          acc.c[t][1] = mfma16(ah[sl], bb.h[1], acc.c[t][1]);
          acc.c[t][0] = mfma16(ah[sl], bb.l[0], acc.c[t][0]);
          acc.c[t][1] = mfma16(ah[sl], bb.l[1], acc.c[t][1]);
          acc.c[t][0] = mfma16(al[sl], bb.h[0], acc.c[t][0]);
          acc.c[t][1] = mfma16(al[sl], bb.h[1], acc.c[t][1]);
        }
#endif
#if !(VGE_ABL & 4)
        // the fragments of the tile AD ahead (this step, the next step, or the next tap's first step)
        const int tn = t + AD;
        const char* q = nullptr;
        bool okq;
        if (tn < NT) {
          okq = okc[tn];
          q = pt[tn] + s * 64;
        } else if (s + 1 < NS) {
          okq = okc[tn - NT];
          q = pt[tn - NT] + (s + 1) * 64;
        } else {
          okq = more && t_tap_ok<W, SKIP>(tn - NT, (kn - ctr) * dil);
          q = rowp(kn, tn - NT);
        }
        if (okq) {
          ah[sl] = *reinterpret_cast<const half8*>(q);
          al[sl] = *reinterpret_cast<const half8*>(q + TXLO);
        }
#endif
        __builtin_amdgcn_sched_barrier(0);  // tile by tile: the next fragments reuse this tile's slot
      }
      asm volatile("" ::: "memory");
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      pt[t] = rowp(kn, t);
      okc[t] = t_tap_ok<W, SKIP>(t, (kn - ctr) * dil);
    }
  }
}

template <int W>
__device__ __forceinline__ void conv_x3t_body(const float* __restrict__ feats, int n_windows, int win0,
                                              const EncDescX3& ed, int e, float* __restrict__ enc_out, char* lds_raw,
                                              int& n_ex, int* __restrict__ status, int spin_limit) {
  constexpr int NT = t_nt<W>(), G = t_gf<W>(), WSB = t_wsb<W>();
  char* Xb = lds_raw;  // W blocks of 32 rows of TXR fp16 (hi at +0, lo at +TXLO bytes), then the zero row
  X3tAux& ax = *reinterpret_cast<X3tAux*>(lds_raw + T_AUX_OFF);

  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave >> 2, wg = wave & 3;
  // Lane-derived values are recomputed from an opaque copy of the thread index at the top of every phase: hoisted
  // out of the phase loop they would stay live across all of it and spill.
  int lane, i, kb, lw, fb;
  unsigned lb;      // this lane's B fragment offset in a chunk pair
  const char* xa;   // this lane's A base (its 16-B k block)
  auto lane_setup = [&]() {
    int t = tid;
    asm volatile("" : "+v"(t));
    lane = t & 63;
    i = lane & 15;
    kb = lane >> 4;
    lw = kb * W / 4;               // the window of every C value of this lane
    fb = (4 * kb) % G;             // frame of C register r of tile t: G t + fb + r
    lb = (unsigned)((kb >> 1) * CHUNK_B + ((kb & 1) * 256 + wave * 32 + i) * 16);
    xa = Xb + kb * 16;
  };
  lane_setup();
  // logical row (window * 32 + frame) of C register r of tile t; LDS byte offset of that row without the lane's part
  auto crow = [&](int t, int r) { return lw * 32 + G * t + fb + r; };

  Acc16<W> acc;
  floatx4 res[NT][2];
  for (int c = tid; c < TXR; c += 512)  // the zero row (out-of-window taps)
    *reinterpret_cast<_Float16*>(Xb + t_zr<W>() + 2 * c) = (_Float16)0.0f;

  // ---------------- stem: Conv1d(d_in -> 256, k=1, no bias), both halves together: per-row power-of-two exponents,
  // K in 256-wide panels (the rows of PG panels loaded before any is used: one HBM round trip per PG panels)
  acc.zero();
  constexpr int RPW = 32 * W / 8;  // rows per wave
  constexpr int PG = W <= 2 ? 2 : 1;
  for (int p0 = 0; p0 < ed.n_stem_panels; p0 += PG) {
    float a[PG][RPW][4];
#pragma unroll
    for (int q = 0; q < PG; ++q) {
      const int p = p0 + q;
      const int kw = p < ed.n_stem_panels ? min(256, ed.d_in - p * 256) : 0;
#pragma unroll
      for (int jr = 0; jr < RPW; ++jr) {
        const int r = wave * RPW + jr;
        const int w = win0 + (r >> 5);
        const float* src = feats + ((size_t)w * VGE_T + (r & 31)) * ed.ld + ed.in_col + p * 256;
#pragma unroll
        for (int jc = 0; jc < 4; ++jc) {
          const int c = lane + 64 * jc;
          a[q][jr][jc] = (c < kw && w < n_windows) ? tgload(src + c) : 0.f;
        }
      }
    }
#pragma unroll
    for (int q = 0; q < PG; ++q) {
      const int p = p0 + q;
      if (p >= ed.n_stem_panels) break;
      const int kw = min(256, ed.d_in - p * 256);
      int* ecur = ax.rexp[p & 1];
#pragma unroll
      for (int jr = 0; jr < RPW; ++jr) {
        float m = fmaxf(fmaxf(fabsf(a[q][jr][0]), fabsf(a[q][jr][1])), fmaxf(fabsf(a[q][jr][2]), fabsf(a[q][jr][3])));
        m = wave_max_all(m);
        const int ex = fp16_range_exp(m);
        const int r = wave * RPW + jr;  // logical row: window r / 32, frame r % 32
        if (lane == 0) ecur[r] = ex;
        _Float16* xr = reinterpret_cast<_Float16*>(Xb + (r >> 5) * WSB + (r & 31) * TXRB);
#pragma unroll
        for (int jc = 0; jc < 4; ++jc) {
          const int c = lane + 64 * jc;
          split_store(xr + c, xr + TXLO / 2 + c, ldexpf(a[q][jr][jc], -ex));
        }
      }
      __syncthreads();  // X and ecur complete
      if (p > 0) {
        const int* eprev = ax.rexp[(p - 1) & 1];
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float f = ldexpf(1.0f, eprev[crow(t, r)] - ecur[crow(t, r)]);
            acc.c[t][0][r] *= f;
            acc.c[t][1][r] *= f;
          }
      }
      const char* wst = reinterpret_cast<const char*>(ed.stem) + (size_t)p * 16 * CHUNK_B;
      if (kw > 128) stream16<W, false, 8>(acc, wst, 1, lb, xa, i, 0, 0);
      else stream16<W, false, 4>(acc, wst, 1, lb, xa, i, 0, 0);
      __syncthreads();  // every wave is done reading X
    }
  }

  // ---------------- the staggered chain
  // max over the group's 4 waves of this lane's window (every lane gets its own window's result)
  auto group_max = [&](float m) -> float {
    const int par = n_ex & 1;
    m = row16_max(m);
    if constexpr (W == 2) m = fmaxf(m, __shfl_xor(m, 16, 64));  // a pair's window spans two 16-lane rows
    if (i == 0 && (W == 4 || (kb & 1) == 0)) ax.mx[par][grp][lw][wg] = m;
    ++n_ex;
    __builtin_amdgcn_s_waitcnt(0xC07F);  // this wave's maxima are in LDS before its arrival is counted
    if (lane == 0) __hip_atomic_fetch_add(&ax.cnt[grp], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    // Bounded: a wave that never arrives would be a bug.  A wave that gives up raises the status word (host-mapped;
    // vge_encode / vge_encoder_profile_read / vge_encoder_status return VGE_ERR_DEVICE), so its wrong results are
    // never silent.
    int spin = 0;
    for (; spin < spin_limit && __builtin_amdgcn_readfirstlane(__hip_atomic_load(
                                    &ax.cnt[grp], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) < 4 * n_ex;
         ++spin)
      __builtin_amdgcn_s_sleep(1);
    if (spin >= spin_limit &&
        __builtin_amdgcn_readfirstlane(__hip_atomic_load(&ax.cnt[grp], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) <
            4 * n_ex &&
        lane == 0)
      __hip_atomic_store(status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const floatx4 v = *reinterpret_cast<const floatx4*>(&ax.mx[par][grp][lw][0]);
    return fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3]));
  };
  // Store this wave's columns of the next GEMM's input (get(t, j) = the values), its window scaled by 2^-ex with the
  // group's largest |value| in [2^8, 2^9) (exact), and publish the exponent for parity `par`.
  auto store_act = [&](auto get, int par) {
    float m = 0.f;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const floatx4& x = get(t, j);
        m = fmaxf(m, fmaxf(fmaxf(fabsf(x[0]), fabsf(x[1])), fmaxf(fabsf(x[2]), fabsf(x[3]))));
      }
    m = group_max(m);
    const int ex = fp16_range_exp(m);
    if (wg == 0 && i == 0 && (W == 4 || (kb & 1) == 0)) ax.ex[par][grp][lw] = ex;
    const float sc = ldexpf(1.0f, -ex);
    char* bh = Xb + lw * WSB + fb * TXRB + (wave * 32 + i) * 2;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const floatx4& x = get(t, j);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float y = x[r] * sc;
          const _Float16 hi = (_Float16)y;
          const int off = (G * t + r) * TXRB + j * 32;
          *reinterpret_cast<_Float16*>(bh + off) = hi;
          *reinterpret_cast<_Float16*>(bh + TXLO + off) = (_Float16)(y - (float)hi);
        }
      }
  };
  // GroupNorm statistics of block b's x over both halves, this lane's window: mean and 1 / sqrt(var + eps)
  auto gn_stats = [&](int b, float& mu, float& rstd) {
    const float(*s)[2] = ax.stats[b & 1][lw];
    const float m = (((s[0][0] + s[1][0]) + (s[2][0] + s[3][0])) + ((s[4][0] + s[5][0]) + (s[6][0] + s[7][0]))) * 0.125f;
    float q = 0.f, d = 0.f;
#pragma unroll
    for (int w = 0; w < 8; ++w) {
      q += s[w][1];
      const float dm = s[w][0] - m;
      d = fmaf(dm, dm, d);
    }
    mu = m;
    rstd = 1.0f / sqrtf(fmaf(d, 1024.0f, q) * (1.0f / 8192.0f) + 1e-5f);
  };
  auto gelu4 = [&](floatx4& v) {
    float y[4] = {v[0], v[1], v[2], v[3]};
#if X3T_GELU
    gelu_fast_s(y);
#else
    gelu_many_s(y);
#endif
    v = floatx4{y[0], y[1], y[2], y[3]};
  };

  // this half's stem epilogue: the stem output is block 0's residual and conv 0's input
  auto stem_epilogue = [&]() {
    const int* efin = ax.rexp[(ed.n_stem_panels - 1) & 1];
    float wcs[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) wcs[j] = tgload(ed.cs + wave * 32 + j * 16 + i);
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ex = efin[crow(t, r)];
#pragma unroll
        for (int j = 0; j < 2; ++j) res[t][j][r] = ldexpf(acc.c[t][j][r] * wcs[j], ex);
      }
    store_act([&](int t, int j) -> const floatx4& { return res[t][j]; }, 0);
  };

  // The epilogue's global operands (column scales; GroupNorm affine and folded corrections; the proj's corrections)
  // are loaded at the start of the phase before it (P2 of the same GEMM), so their latency hides behind that stream.
  float pre_wcs[2], pre_gw[2], pre_gb[2], pre_sx[2], pre_sy[2];
  floatx4 pre_g[2], pre_b[2];  // per-tap sums of W1 gamma / W1 beta, taps 0..3
  float pre_g4[2], pre_b4[2];  // ... tap 4
  auto prefetch = [&](auto kind_tag, int gi) {
    constexpr int KIND = decltype(kind_tag)::value;
    const int blk = gi >> 1;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = wave * 32 + j * 16 + i;
      pre_wcs[j] = tgload(ed.cs + (1 + gi) * 256 + col);
      if constexpr (KIND == 2) {
        pre_sx[j] = tgload(ed.fold + 3 * 256 * 16 + col * 2);
        pre_sy[j] = tgload(ed.fold + 3 * 256 * 16 + col * 2 + 1);
      } else if constexpr (KIND == 0) {
        if (blk > 0) {
          pre_gw[j] = tgload(ed.gn_w + (blk - 1) * 256 + col);
          pre_gb[j] = tgload(ed.gn_b + (blk - 1) * 256 + col);
          typedef const __attribute__((address_space(1))) floatx4* gf4;
          const float* fbp = ed.fold + ((size_t)(blk - 1) * 256 + col) * 16;
          pre_g[j] = *(gf4)fbp;
          pre_g4[j] = tgload(fbp + 4);
          pre_b[j] = *(gf4)(fbp + 8);
          pre_b4[j] = tgload(fbp + 12);
        }
      }
    }
  };

  // epilogue of a block's first conv, block BLK (compile time: the fold classes of every frame are static)
  auto epilogue_k0 = [&](auto blk_tag) {
    constexpr int BLK = decltype(blk_tag)::value;
    constexpr int gi = 2 * BLK, par = gi & 1;
    float scv;  // this lane's window: the accumulators' exponent x ...
    {
      scv = ldexpf(1.0f, ax.ex[par][1][lw]);
    }
    if constexpr (BLK == 0) {
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          floatx4& x = acc.c[t][j];
          const float s = scv * pre_wcs[j];
#pragma unroll
          for (int r = 0; r < 4; ++r) x[r] *= s;
          gelu4(x);
        }
    } else {
      // conv1(GN(x)) = rstd (conv_{W gamma}(x) - mu C_gamma(f)) + C_beta(f); C(f) = the sums over the taps of frame
      // f that fall inside the window: five classes per column (f < d | < 2d | interior | >= 32 - 2d | >= 32 - d)
      constexpr int D = 1 << BLK;
      float mu, rstd;
      gn_stats(BLK - 1, mu, rstd);
      float cg[2][5], cb[2][5], gs[2], gsh[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const float g2 = pre_g[j][2], g234 = (g2 + pre_g[j][3]) + pre_g4[j];
        cg[j][0] = g234;                                       // f < d:            taps 2, 3, 4
        cg[j][1] = pre_g[j][1] + g234;                         // d <= f < 2d:      taps 1..4
        cg[j][2] = (((pre_g[j][0] + pre_g[j][1]) + g2) + pre_g[j][3]) + pre_g4[j];  // interior: all five
        cg[j][3] = ((pre_g[j][0] + pre_g[j][1]) + g2) + pre_g[j][3];                // 32 - 2d <= f < 32 - d
        cg[j][4] = (pre_g[j][0] + pre_g[j][1]) + g2;                                // f >= 32 - d
        const float b2 = pre_b[j][2], b234 = (b2 + pre_b[j][3]) + pre_b4[j];
        cb[j][0] = b234;
        cb[j][1] = pre_b[j][1] + b234;
        cb[j][2] = (((pre_b[j][0] + pre_b[j][1]) + b2) + pre_b[j][3]) + pre_b4[j];
        cb[j][3] = ((pre_b[j][0] + pre_b[j][1]) + b2) + pre_b[j][3];
        cb[j][4] = (pre_b[j][0] + pre_b[j][1]) + b2;
        gs[j] = rstd * pre_gw[j];
        gsh[j] = fmaf(-mu, gs[j], pre_gb[j]);
      }
      auto cls = [](int f) { return f < D ? 0 : f < 2 * D ? 1 : f < 32 - 2 * D ? 2 : f < 32 - D ? 3 : 4; };
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          floatx4& x = acc.c[t][j];
          const float s = scv * pre_wcs[j];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            // frame G t + fb + r: fb is 0 for quads; a pair's lanes take fb = 0 or 4 (the two candidates are static)
            int c;
            if constexpr (W == 4) {
              c = cls(G * t + r);
            } else {
              const int c0 = cls(G * t + r), c1 = cls(G * t + 4 + r);
              c = (c0 == c1) ? c0 : (fb ? c1 : c0);
            }
            float g = cg[j][0], bb = cb[j][0];
#pragma unroll
            for (int q = 1; q < 5; ++q)
              if (c == q) {
                g = cg[j][q];
                bb = cb[j][q];
              }
            res[t][j][r] = fmaf(res[t][j][r], gs[j], gsh[j]);  // (x - mu) rstd gamma + beta
            x[r] = fmaf(rstd, fmaf(-mu, g, x[r] * s), bb);
          }
          gelu4(x);
        }
    }
    store_act([&](int t, int j) -> const floatx4& { return acc.c[t][j]; }, (gi + 1) & 1);
  };

  // epilogue of a block's second conv: x = GELU(conv2(h) + residual), stored pre-GroupNorm, kept as the residual,
  // per-wave partial statistics published
  auto epilogue_k1 = [&](int gi) {
    const int par = gi & 1, blk = gi >> 1;
    const float scv = ldexpf(1.0f, ax.ex[par][1][lw]);
    float sum = 0.f;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        floatx4& x = acc.c[t][j];
        const float s = scv * pre_wcs[j];
#pragma unroll
        for (int r = 0; r < 4; ++r) x[r] = fmaf(x[r], s, res[t][j][r]);
        gelu4(x);
        res[t][j] = x;
        sum += (x[0] + x[1]) + (x[2] + x[3]);
      }
    // per-wave GroupNorm partials of this lane's window: mean, then M2 about it (two-pass, in registers)
    sum = row16_sum(sum);
    if constexpr (W == 2) sum += __shfl_xor(sum, 16, 64);
    const float mw = sum * (1.0f / 1024.0f);
    float q = 0.f;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float d = res[t][j][r] - mw;
          q = fmaf(d, d, q);
        }
    q = row16_sum(q);
    if constexpr (W == 2) q += __shfl_xor(q, 16, 64);
    if (i == 0 && (W == 4 || (kb & 1) == 0)) {
      ax.stats[blk & 1][lw][wave][0] = mw;
      ax.stats[blk & 1][lw][wave][1] = q;
    }
    store_act([&](int t, int j) -> const floatx4& { return acc.c[t][j]; }, (gi + 1) & 1);
  };

  // the proj's epilogue: proj(GN_3(x)) = rstd (P gamma x - mu S_gamma) + S_beta; rows past n_windows are not written
  auto epilogue_proj = [&]() {
    const float scv = ldexpf(1.0f, ax.ex[0][1][lw]);
    float mu, rstd;
    gn_stats(3, mu, rstd);
    const int win = win0 + lw;
    if (win < n_windows) {
      float* ob = enc_out + ((size_t)e * n_windows + win) * VGE_T * VGE_D + wave * 32 + i;
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const float s = scv * pre_wcs[j];
#pragma unroll
          for (int r = 0; r < 4; ++r)
            ob[(G * t + fb + r) * VGE_D + j * 16] = fmaf(rstd, fmaf(acc.c[t][j][r], s, -mu * pre_sx[j]), pre_sy[j]);
        }
    }
  };

  // SKIP (compile time): the tap-skipping stream code only where taps can be skipped (blocks 2, 3: dilation 4, 8)
  auto stream = [&](auto skip_tag, int gi, int part) {
    constexpr bool SKIP = decltype(skip_tag)::value;
    if (part == 0) {
      acc.zero();
    } else {  // channels of B: the accumulators move from A's exponent to B's (exact)
      const float f = ldexpf(1.0f, ax.ex[gi & 1][0][lw] - ax.ex[gi & 1][1][lw]);
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc.c[t][j] *= f;
    }
    const bool proj = gi == 8;
    const char* wb = reinterpret_cast<const char*>(proj ? ed.proj : ed.conv + (size_t)gi * 80 * (CHUNK_B / 2)) +
                     (size_t)part * 8 * CHUNK_B;
    if (X3T_PRIO) __builtin_amdgcn_s_setprio(1);
    stream16<W, SKIP, 4>(acc, wb, proj ? 1 : 5, lb, xa + part * 256, i, proj ? 0 : 1 << (gi >> 1), proj ? 0 : 2);
    __builtin_amdgcn_s_setprio(0);
  };

  using K0 = std::integral_constant<int, 0>;
  using K1 = std::integral_constant<int, 1>;
  using K2 = std::integral_constant<int, 2>;
  auto phase_end = [&]() {
    lds_barrier();
    lane_setup();
  };
  if (grp == 1) phase_end();
  else lane_setup();
  stem_epilogue();
  phase_end();
  using NoSkip = std::integral_constant<bool, false>;
  using Skip = std::integral_constant<bool, true>;
  // blocks are compile-time (each block's straight-line code is its own: a runtime block loop keeps more values live
  // across its back edge and spilled 96-226 scratch instructions against 7 this way)
  auto block = [&](auto skip_tag, auto blk_tag) {
    constexpr int blk = decltype(blk_tag)::value;
    stream(skip_tag, 2 * blk, 0);
    phase_end();
    prefetch(K0{}, 2 * blk);
    stream(skip_tag, 2 * blk, 1);
    phase_end();
    epilogue_k0(blk_tag);
    phase_end();
    stream(skip_tag, 2 * blk + 1, 0);
    phase_end();
    prefetch(K1{}, 2 * blk + 1);
    stream(skip_tag, 2 * blk + 1, 1);
    phase_end();
    epilogue_k1(2 * blk + 1);
    phase_end();
  };
  block(NoSkip{}, std::integral_constant<int, 0>{});
  block(NoSkip{}, std::integral_constant<int, 1>{});
  block(Skip{}, std::integral_constant<int, 2>{});
  block(Skip{}, std::integral_constant<int, 3>{});
  stream(NoSkip{}, 8, 0);
  phase_end();
  prefetch(K2{}, 8);
  stream(NoSkip{}, 8, 1);
  phase_end();
  epilogue_proj();
  phase_end();
  if (grp == 0) phase_end();
}

__global__ void __launch_bounds__(512, 1) conv_encoder_x3t_kernel(const float* __restrict__ feats,
                                                                   const EncDescX3* __restrict__ encs, vge::ConvSched cs,
                                                                   float* __restrict__ enc_out, int* __restrict__ status,
                                                                   int spin_limit) {
  extern __shared__ __attribute__((aligned(16))) char lds_raw[];
  X3tAux& ax = *reinterpret_cast<X3tAux*>(lds_raw + T_AUX_OFF);
  if (threadIdx.x < 2) ax.cnt[threadIdx.x] = 0;  // ordered before any exchange by the stem staging's barriers
  int n_ex = 0;
  const int n = cs.n_windows;
  for (int round = 0; round * cs.G < cs.n_units; ++round) {
    const int u = round * cs.G + xcd_remap(blockIdx.x, cs.G);
    if (u >= cs.n_units) break;  // uniform over the block
    int e, w0;
    if (conv_unit(cs, u, e, w0)) conv_x3t_body<4>(feats, n, w0, encs[e], e, enc_out, lds_raw, n_ex, status, spin_limit);
    else conv_x3t_body<2>(feats, n, w0, encs[e], e, enc_out, lds_raw, n_ex, status, spin_limit);
  }
}

}  // namespace

namespace vge {

hipError_t encoder_x3t_kernel_setup() {
  return hipFuncSetAttribute((const void*)conv_encoder_x3t_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                             T_LDS_BYTES);
}

extern int g_x3s_spin_limit_value();

hipError_t launch_conv_encoders_x3t(const float* feats, int n_windows, const void* encs, int n_enc, unsigned heavy,
                                    float* enc_out, int* status, hipStream_t s) {
  if (n_windows < 1 || n_enc < 1) return hipSuccess;
  if (!status) return hipErrorInvalidValue;
  const ConvSched cs = conv_quad_sched(n_windows, n_enc, heavy);
  hipLaunchKernelGGL(conv_encoder_x3t_kernel, dim3(cs.G), dim3(512), T_LDS_BYTES, s, feats,
                     reinterpret_cast<const EncDescX3*>(encs), cs, enc_out, status, g_x3s_spin_limit_value());
  return hipGetLastError();
}

}  // namespace vge
