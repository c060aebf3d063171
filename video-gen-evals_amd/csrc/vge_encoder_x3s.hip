// Staggered split-precision ("3xfp16") MovementConvEncoder chain (model.py:21-58, x10), gfx950.
//
// Same arithmetic as conv_encoder_x3_kernel (vge_encoder_x3.hip: hi/lo fp16 planes, three v_mfma_f32_32x32x16_f16
// per product, power-of-two scaled operands, f32 accumulation and epilogues), same units (an encoder x 4 or 2
// windows per 512-thread workgroup, wave w = output columns 32w..32w+31 of all rows), but the two halves of the
// workgroup run half a conv apart so that every epilogue of one half runs beside the other half's MFMA stream.
// In the unstaggered kernel all 8 waves reach each epilogue together and the matrix pipes idle through it (~20 %
// of a quad's cycles: tools/trace_encoder.py).
//
// Group A = waves 0-3 (output columns 0..127), group B = waves 4-7 (128..255); SIMD s holds waves s and s + 4, one
// of each group.  A GEMM's K (tap x 256 input channels) is streamed in two parts: P1 = the channels group A
// produced (0..127; 5 taps x 8 chunks for a conv), P2 = group B's.  Each half runs the task sequence
// stem-epilogue, then P1(g), P2(g), E(g) for g = conv 0..7, proj; B runs one phase behind A and every phase ends
// with a workgroup barrier:
//
//   phase 3g+1: A P1(g) | B E(g-1)      phase 3g+2: A P2(g) | B P1(g)      phase 3g+3: A E(g) | B P2(g)
//
// One buffer of activations satisfies every dependency: A's P2(g) reads what B's E(g-1) wrote a phase earlier; A's
// E(g) overwrites channels 0..127 after B's P1(g) read them (previous phase); B's E(g) overwrites 128..255 after
// A's P2(g) and B's own P2(g).  In phases 3g+1 and 3g+3 one wave per SIMD streams -- one accumulation chain of
// this MFMA keeps a SIMD's matrix pipe busy on its own (MI355X_MICROARCH.md, cycle constants) -- while its partner
// runs the epilogue's VALU work.
//
// Two reductions of the unstaggered kernel span the whole 256-column row, which one half cannot finish alone:
// * GroupNorm(1, 256) (per window over its 32 x 256 values).  A's epilogue of a block's second conv runs while B
//   is still streaming that conv, so the normalisation is folded into the next GEMM: the epilogue stores
//   x = GELU(conv2 + res) itself, keeps it as the residual and writes per-wave partial statistics; the next GEMM's
//   weights were packed as W diag(gamma) (vge_encoder_create) and its epilogue, which runs after both halves' E,
//   corrects per window: conv(GN(x)) = rstd (conv_{W gamma}(x) - mu C_gamma(r)) + C_beta(r), with C(r) the sums of
//   W gamma / W beta over the taps of row r that fall inside the window (EncDescX3::fold, host-computed in double);
//   the residual becomes (x - mu) rstd gamma + beta in registers.  Statistics: each wave's mean and M2 (two-pass in
//   registers) combined in a fixed order (Chan et al.), identical in every wave.
// * the split exponent of stored activations.  Each half stores its channels with its own per-window exponent (the
//   max over its 4 waves, exchanged through LDS with an arrival counter -- no barrier, the other half is
//   streaming), and a consumer rescales its accumulators between P1 and P2 (exact powers of two).
#include "vge_x3.h"
#include <type_traits>

#ifdef VGE_TRACE  // timing-only builds (tools/trace_x3s.py): s_memtime stamps of every wave of blocks 0..63, first unit
__device__ long long g_x3s_trace[64 * 8 * 128];
#define XTS(k)                                                                                                       \
  do {                                                                                                              \
    if (tr_on && blockIdx.x < 64 && (threadIdx.x & 63) == 0)                                                        \
      g_x3s_trace[(blockIdx.x * 8 + (threadIdx.x >> 6)) * 128 + (k)] = __builtin_amdgcn_s_memtime();                 \
  } while (0)
#else
#define XTS(k) \
  do {         \
  } while (0)
#endif

namespace {

#ifndef X3S_TRACE_ROUND
#define X3S_TRACE_ROUND 0  // VGE_TRACE builds stamp the units of this round of the persistent schedule
#endif
#ifndef X3S_GELU
#define X3S_GELU 1  // 1: gelu_fast_s (one exp2; f32 rounding-level error, see DESIGN), 0: gelu_many_s (exact-erf pieces)
#endif
#ifndef X3S_PRIO
#define X3S_PRIO 1  // s_setprio 1 for the streaming half
#endif
constexpr int X3S_WMAX = 4;     // windows per unit (quads; pairs fill the remainder)
#ifndef X3S_PF_QUAD
#define X3S_PF_QUAD 4  // weight chunks in flight per wave in a quad's conv streams
#endif
#ifndef X3S_PF_PAIR
#define X3S_PF_PAIR 8  // ... in a pair's
#endif
#ifndef X3S_PF16_QUAD
#define X3S_PF16_QUAD 8  // ... single-fp16 mode (VGE_F16): half the bytes per chunk, a third of the MFMAs
#endif
#ifndef X3S_PF16_PAIR
#define X3S_PF16_PAIR 8
#endif
#ifndef X3S_ROT
#define X3S_ROT 0  // 1: chunk order inside a tap rotated per workgroup (see stream_part; measured 1-2 % slower)
#endif
#ifndef X3S_SKIP
#define X3S_SKIP 1  // 1: a row tile skips the taps that put all its frames outside the window (dilated convs)
#endif
// Activation rows in LDS interleave the planes: [hi 256 + 8 pad | lo 256 + 8 pad | 8 pad] fp16 = 1,072 B, so one row
// base addresses both planes with immediate offsets (lo at +528 B).  A unit's windows are 32-row blocks WSB bytes
// apart, and an MFMA row tile is a row GROUP across the windows: tile t of a quad = frames 8t..8t+7 of all four
// windows (MFMA row i = window i / 8, frame 8t + i % 8), of a pair = frames 16t..16t+15 of both.  A dilated tap that
// puts all of a tile's frames outside the window then contributes exact zeros to the whole tile, and the tile skips
// it: of a block's 5 taps x 4 tiles, dilation 8 keeps 14, dilation 4 keeps 18 (quads; pairs: 8 of 10 at dilation 8).
// The quads' 128-B block padding keeps the ds_read_b128 lane groups, which mix rows of all four windows, on distinct
// banks (pairs: none needed).
constexpr int XR = 536;                         // fp16 per row
constexpr int XRB = 2 * XR;                     // bytes per row
constexpr int XLO = 528;                        // byte offset of the lo plane in a row
template <int W>
constexpr int x3s_g() { return 32 / W; }        // frames of each window in one row tile
template <int W>
constexpr int x3s_wsb() { return 32 * XRB + (W >= 4 ? 128 : 0); }  // bytes per window block
template <int W>
constexpr int x3s_zr() { return W * x3s_wsb<W>(); }  // byte offset of the all-zero row (out-of-window taps)
// C-layout register r of a lane (h = lane / 32) holds row rho = (r & 3) + 8 (r >> 2) + 4 h of its tile: window
// rho / G, frame G t + rho % G; the h part (4 h) never crosses a window, so a register's window is r's alone
template <int W>
__host__ __device__ constexpr int x3s_rwin(int r) { return ((r & 3) + 8 * (r >> 2)) / x3s_g<W>(); }
template <int W>
__host__ __device__ constexpr int x3s_rfr0(int t, int r) {  // frame without the lane's 4 h
  return x3s_g<W>() * t + ((r & 3) + 8 * (r >> 2)) % x3s_g<W>();
}
// does row tile t (frames G t .. G t + G - 1) see any in-window frame through tap offset o
template <int W, bool SKIP>
__device__ __forceinline__ bool x3s_tap_ok(int t, int o) {
  constexpr int G = x3s_g<W>();
  return !(X3S_SKIP && SKIP) || (G * t + G - 1 + o >= 0 && G * t + o <= 31);
}
constexpr int X3S_AUX_OFF = (x3s_zr<X3S_WMAX>() + XRB + 15) / 16 * 16;  // fixed LDS offset of the auxiliary area

struct X3sAux {
  int rexp[2][32 * X3S_WMAX];       // stem row exponents, by panel parity
  float stats[2][X3S_WMAX][8][2];   // [block parity][window][wave] (mean, M2) of x = GELU(conv2 + res)
  float mx[2][2][X3S_WMAX][4];      // [exchange parity][group][window][wave in group] maxima
  int ex[2][2][X3S_WMAX];           // [GEMM-input parity][group][window] exponents of the stored activations
  int cnt[2];                       // exchange arrivals per group (monotonic over the launch)
};
// Per wave: the next block-conv1 epilogue's fold operands of its 32 columns, landed by LDS-DMA during the stream
// before it (registers held across that stream spilled): [32 columns][16 floats] of EncDescX3::fold, then
// GroupNorm gamma [32] | beta [32]
constexpr int X3S_PRE_WAVE = 32 * 64 + 256;
constexpr int X3S_PRE_OFF = (X3S_AUX_OFF + (int)sizeof(X3sAux) + 15) / 16 * 16;
constexpr int X3S_LDS_BYTES = X3S_PRE_OFF + 8 * X3S_PRE_WAVE;
static_assert(X3S_AUX_OFF % 16 == 0, "aux alignment");
static_assert(X3S_LDS_BYTES <= 160 * 1024, "LDS");

// One part of a conv / proj GEMM without barriers: ntap taps x 8 chunks (input-channel blocks cb0..cb0+7 of each
// tap).  B fragments 3 chunks ahead in a register ring; A fragments single-buffered per row tile (tile t's fragments
// of the next chunk are read right after the three MFMAs of this chunk that use them: their latency hides behind the
// other tiles' MFMAs).  Addresses are formed once per tap -- LDS row bases (the zero row for taps outside the window)
// plus immediate chunk offsets, uniform weight pointers plus the lane's offset -- so the stream issues almost no VALU
// work besides its MFMAs (its partner wave's epilogue shares the SIMD's issue slots).
template <int W, bool SKIP, bool SP>
__device__ __forceinline__ void stream_part(Acc<W, 1>& acc, const char* wb, int ntap, unsigned loff, const char* xa,
                                            int i, int dil, int ctr, int rot) {
  constexpr int R = W, G = x3s_g<W>();
  // chunks in flight: a pair's chunk is only 6 MFMAs (192 cycles) -- 3 chunks ahead would not cover the weight
  // stream's L2 latency while one wave per SIMD streams -- and it has the registers for 7
  constexpr int PF = SP ? (R >= 4 ? X3S_PF_QUAD : X3S_PF_PAIR) : (R >= 4 ? X3S_PF16_QUAD : X3S_PF16_PAIR);
  // the ring's slots restart at every tap (chunk j of a tap sits in slot j % PF, and the last steps of a tap load the
  // next tap's first chunks into the slots they will be read from): a depth that does not divide a tap's 8 chunks
  // reads the wrong chunk (measured: depths 3 / 6 / 12 gave wrong scores)
  static_assert(8 % PF == 0, "ring depth must divide a tap's 8 chunks");
  const char* xw = xa + (i / G) * x3s_wsb<W>();  // this lane's MFMA row: its window's block ...
  const int fi = i % G;                          // ... and its frame within the tile's group
  const char* xz = xa + x3s_zr<W>();
  auto rowp = [&](int k, int t) -> const char* {
    const int tt = G * t + fi + (k - ctr) * dil;
    return (unsigned)tt < 32u ? xw + tt * XRB : xz;
  };
  // weights through a buffer resource: the chunk offset in an SGPR, the lane's offset (+ the lo plane) in VGPRs
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(wb), (short)0, 0x7FFFFFF0, 0x00020000);
  const unsigned loff_l = loff + PLANE_B;
  // rot: this workgroup's chunk order inside a tap (logical chunk j is input-channel block (j + rot) & 7): the CUs of
  // an XCD stream the same encoder's weights together, and rotated they do not all read one chunk's lines at once
  auto ldb = [&](int k, int j, BFrag<1>& b) {  // chunk j (0..7) of tap k
    const int so = (k * 16 + ((j + rot) & 7)) * CHUNK_B;
    b.h[0] = __builtin_bit_cast(half8, __builtin_amdgcn_raw_buffer_load_b128(rs, loff, so, 0));
    if constexpr (SP) b.l[0] = __builtin_bit_cast(half8, __builtin_amdgcn_raw_buffer_load_b128(rs, loff_l, so, 0));
  };
  BFrag<1> b[PF];
#pragma unroll
  for (int j = 0; j < PF - 1; ++j) ldb(0, j, b[j]);
  half8 ah[R], al[R];
  const char* pt[R];
  bool okc[R];  // tile t takes part in the current tap (uniform)
#pragma unroll
  for (int t = 0; t < R; ++t) {
    pt[t] = rowp(0, t);
    okc[t] = x3s_tap_ok<W, SKIP>(t, -ctr * dil);
    if (okc[t]) {
      ah[t] = *reinterpret_cast<const half8*>(pt[t] + rot * 32);
      if constexpr (SP) al[t] = *reinterpret_cast<const half8*>(pt[t] + rot * 32 + XLO);
    }
  }
  for (int k = 0; k < ntap; ++k) {
    const bool more = k + 1 < ntap;
    const int kn = more ? k + 1 : k;
    const char* pn[R];
    bool okn[R];
#pragma unroll
    for (int t = 0; t < R; ++t) {
      pn[t] = rowp(kn, t);
      okn[t] = x3s_tap_ok<W, SKIP>(t, (kn - ctr) * dil);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
#if !(VGE_ABL & 2)
      if (j + PF - 1 < 8) ldb(k, j + PF - 1, b[(j + PF - 1) % PF]);
      else ldb(kn, more ? j + PF - 1 - 8 : 7, b[(j + PF - 1) % PF]);  // (past the end: reload the last chunk)
#endif
#pragma unroll
      for (int t = 0; t < R; ++t) {
#if !(VGE_ABL & 1)
        if (okc[t]) {
          acc.c[t][0] = mfma32(ah[t], b[j % PF].h[0], acc.c[t][0]);
          if constexpr (SP) {
            acc.c[t][0] = mfma32(ah[t], b[j % PF].l[0], acc.c[t][0]);
            acc.c[t][0] = mfma32(al[t], b[j % PF].h[0], acc.c[t][0]);
          }
        }
#endif
#if !(VGE_ABL & 4)
        if (j < 7 ? okc[t] : okn[t]) {
          const char* q = j < 7 ? pt[t] + ((j + 1 + rot) & 7) * 32 : pn[t] + rot * 32;
          ah[t] = *reinterpret_cast<const half8*>(q);
          if constexpr (SP) al[t] = *reinterpret_cast<const half8*>(q + XLO);
        }
#endif
        __builtin_amdgcn_sched_barrier(0);  // tile by tile: the next fragments reuse this tile's registers
      }
      asm volatile("" ::: "memory");
    }
#pragma unroll
    for (int t = 0; t < R; ++t) {
      pt[t] = pn[t];
      okc[t] = okn[t];
    }
  }
}

// a global-address-space load (a generic pointer would become a flat load, which also counts on lgkmcnt)
__device__ __forceinline__ float gload(const float* p) {
  return *(const __attribute__((address_space(1))) float*)p;
}

template <int W, bool SP>
__device__ __forceinline__ void conv_x3s_body(const float* __restrict__ feats, int n_windows, int win0,
                                              const EncDescX3& ed, int e, float* __restrict__ enc_out, char* lds_raw,
                                              int& n_ex, int* __restrict__ status, int spin_limit,
                                              [[maybe_unused]] bool tr_on) {
  constexpr int R = W, G = x3s_g<W>(), WSB = x3s_wsb<W>();
  _Float16* X = reinterpret_cast<_Float16*>(lds_raw);  // W blocks of 32 rows of XR (hi at +0, lo at +XLO bytes), zero row
  char* Xb = lds_raw;
  X3sAux& ax = *reinterpret_cast<X3sAux*>(lds_raw + X3S_AUX_OFF);

  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave >> 2, wg = wave & 3;
  // Lane-derived values are recomputed from an opaque copy of the thread index at the top of every phase: hoisted
  // out of the phase loop (per-row addresses of every task kind) they would stay live across all of it and spill.
  int lane, i, h, col;
  unsigned loff;
  const char* xa;
  auto lane_setup = [&]() {
    int t = tid;
    asm volatile("" : "+v"(t));
    lane = t & 63;
    i = lane & 31;
    h = lane >> 5;
    col = wave * 32 + i;                                   // this lane's output column
    loff = (unsigned)((h * 256 + col) * 16);               // its B fragment in a chunk
    xa = reinterpret_cast<const char*>(X) + h * 16;        // its 8 k-values of a 16-K chunk column
  };
  lane_setup();
  // logical row (window * 32 + frame) of C-layout register r of tile t (the rexp index)
  auto crow = [&](int t, int r) { return x3s_rwin<W>(r) * 32 + x3s_rfr0<W>(t, r) + 4 * h; };
  // LDS byte offset of that row, without the lane's 4 h rows (compile-time for static t, r)
  auto cofs = [&](int t, int r) { return x3s_rwin<W>(r) * WSB + x3s_rfr0<W>(t, r) * XRB; };

  Acc<R, 1> acc;
  floatx16 res[R];
  for (int c = tid; c < XR; c += 512)  // the zero row (out-of-window taps)
    *reinterpret_cast<_Float16*>(Xb + x3s_zr<W>() + 2 * c) = (_Float16)0.0f;

  // ---------------- stem: Conv1d(d_in -> 256, k=1, no bias), both halves together (conv_encoder_body's staging:
  // per-row power-of-two exponents, K in 256-wide panels)
  auto afn_stem = [&](int c, AFrag<R>& f) {
#pragma unroll
    for (int t = 0; t < R; ++t) {  // MFMA row i of tile t: window i / G, frame G t + i % G
      const char* q = xa + (i / G) * WSB + (G * t + i % G) * XRB + c * 32;
      f.h[t] = *reinterpret_cast<const half8*>(q);
      if constexpr (SP) f.l[t] = *reinterpret_cast<const half8*>(q + XLO);
    }
  };
  XTS(0);
  acc.zero();
  // Every row of PG panels is loaded before any is used (one HBM round trip per PG panels: a pair's 4-panel vit stem
  // loads two panels at a time; the loads of a panel group are all issued before its first weight stream, so no
  // stream's counted vmcnt wait can stall on them), then each panel is split into LDS and streamed in turn.
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
          a[q][jr][jc] = (c < kw && w < n_windows) ? gload(src + c) : 0.f;
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
        _Float16* xr = reinterpret_cast<_Float16*>(Xb + (r >> 5) * WSB + (r & 31) * XRB);
#pragma unroll
        for (int jc = 0; jc < 4; ++jc) {
          const int c = lane + 64 * jc;
          if constexpr (SP) split_store(xr + c, xr + XLO / 2 + c, ldexpf(a[q][jr][jc], -ex));
          else xr[c] = (_Float16)ldexpf(a[q][jr][jc], -ex);
        }
      }
      __syncthreads();  // X and ecur complete
      if (p == 0) XTS(122);
      if (p > 0) {
        const int* eprev = ax.rexp[(p - 1) & 1];
#pragma unroll
        for (int t = 0; t < R; ++t)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc.c[t][0][r] *= ldexpf(1.0f, eprev[crow(t, r)] - ecur[crow(t, r)]);
      }
      run_stream<SP ? CONV_PF : CONV_PF16, SP>(acc, reinterpret_cast<const char*>(ed.stem) + (size_t)p * 16 * CHUNK_B,
                                ((kw + 127) >> 7) * STREAM_GROUP, loff, afn_stem);
      if (p == 0) XTS(123);
      __syncthreads();  // every wave is done reading X
    }
  }

  // ---------------- the staggered chain
  // An epilogue computes every tile in place in the accumulators, then exchanges the windows' maxima with the other
  // 3 waves of its half once, then stores.
  // max over the group's 4 waves of one value per window (every wave of the group gets the same results)
  auto group_max = [&](float (&m)[R]) {
    const int par = n_ex & 1;
#pragma unroll
    for (int t = 0; t < R; ++t) {
      const float w = wave_max_last(m[t]);
      if (lane == 63) ax.mx[par][grp][t][wg] = w;
    }
    ++n_ex;
    if (lane == 63) __hip_atomic_fetch_add(&ax.cnt[grp], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    // Bounded: a wave that never arrives would be a bug.  The bound ends the wait instead of hanging the device, and a
    // wave that gives up raises the encoder's status word (host-mapped; vge_encode / vge_encoder_profile_read /
    // vge_encoder_status return VGE_ERR_DEVICE once it is set), so the wrong results it leaves are never silent.
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
#pragma unroll
    for (int t = 0; t < R; ++t)
      m[t] = fmaxf(fmaxf(ax.mx[par][grp][t][0], ax.mx[par][grp][t][1]),
                   fmaxf(ax.mx[par][grp][t][2], ax.mx[par][grp][t][3]));
  };
  // Store this wave's columns of the next GEMM's input (v = the accumulators or the residuals), window v scaled by
  // 2^-ex[v] with the group's largest |value| in [2^8, 2^9) (exact), and publish the exponents for parity `par`.  Row
  // of register r of tile t at an immediate offset of ds_write_b16.
  [[maybe_unused]] int tslot = 64;  // trace: epilogue stamp base (64 + 4 * epilogue index)
  auto store_act = [&](auto get, int par) {
    XTS(tslot + 1);
    float m[R];
#pragma unroll
    for (int v = 0; v < R; ++v) m[v] = 0.f;
#pragma unroll
    for (int t = 0; t < R; ++t) {
      const floatx16& x = get(t);
#pragma unroll
      for (int r = 0; r < 16; ++r) m[x3s_rwin<W>(r)] = fmaxf(m[x3s_rwin<W>(r)], fabsf(x[r]));
    }
    group_max(m);
    XTS(tslot + 2);
    float scv[R];
#pragma unroll
    for (int v = 0; v < R; ++v) {
      const int ex = fp16_range_exp(m[v]);
      if (wg == 0 && lane == 0) ax.ex[par][grp][v] = ex;
      scv[v] = ldexpf(1.0f, -ex);
    }
    char* bh = Xb + (4 * h * XR + col) * 2;
#pragma unroll
    for (int t = 0; t < R; ++t) {
      const floatx16& x = get(t);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float y = x[r] * scv[x3s_rwin<W>(r)];
        const _Float16 hi = (_Float16)y;
        const int off = cofs(t, r);
        *reinterpret_cast<_Float16*>(bh + off) = hi;
        if constexpr (SP) *reinterpret_cast<_Float16*>(bh + XLO + off) = (_Float16)(y - (float)hi);
      }
    }
    XTS(tslot + 3);
    tslot += 4;
  };
  // GroupNorm statistics of block b's x over both halves, window t: mean and 1 / sqrt(var + eps)
  auto gn_stats = [&](int b, int t, float& mu, float& rstd) {
    const float(*s)[2] = ax.stats[b & 1][t];
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
  // GELU of a tile's 16 values in place (8 independent packed chains)
  auto gelu_tile = [&](floatx16& v) {
    float y[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) y[k] = v[k];
#if X3S_GELU
    gelu_fast_s(y);
#else
    gelu_many_s(y);
#endif
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = y[k];
  };

  // this half's stem epilogue: the stem output is block 0's residual and conv 0's input
  auto stem_epilogue = [&]() {
    XTS(tslot);
    const int* efin = ax.rexp[(ed.n_stem_panels - 1) & 1];
    const float wcs = gload(ed.cs + col);
#pragma unroll
    for (int t = 0; t < R; ++t) {
#pragma unroll
      for (int r = 0; r < 16; ++r) res[t][r] = ldexpf(acc.c[t][0][r] * wcs, efin[crow(t, r)]);
    }
    store_act([&](int t) -> const floatx16& { return res[t]; }, 0);
  };

  // epilogue of GEMM gi; KIND (compile time) = 0: a block's conv1, 1: its conv2, 2: the proj
  // The epilogue's global operands (column scale; GroupNorm affine and folded corrections; the proj's corrections)
  // are loaded at the start of the phase before it (P2 of the same GEMM), so their latency -- long while the other
  // half streams weights -- hides behind that stream.
  float pre_wcs = 0.f, pre_sx = 0.f, pre_sy = 0.f;
  char* pre_lds = lds_raw + X3S_PRE_OFF + wave * X3S_PRE_WAVE;  // this wave's fold operands (X3S_PRE_WAVE)
  auto prefetch = [&](auto kind_tag, int gi) {
    constexpr int KIND = decltype(kind_tag)::value;
    const int blk = gi >> 1;
    pre_wcs = gload(ed.cs + (1 + gi) * 256 + col);
    if constexpr (KIND == 2) {
      pre_sx = gload(ed.fold + 3 * 256 * 16 + col * 2);
      pre_sy = gload(ed.fold + 3 * 256 * 16 + col * 2 + 1);
    } else if constexpr (KIND == 0) {
      if (blk > 0) {  // LDS-DMA: the wave's 32 columns x 16 floats (2 KB, contiguous), then gamma | beta
        const float* fb = ed.fold + ((size_t)(blk - 1) * 256 + wave * 32) * 16;
        glds16(fb + lane * 4, pre_lds);
        glds16(fb + 256 + lane * 4, pre_lds + 1024);
        const float* gsrc = (h ? ed.gn_b : ed.gn_w) + (blk - 1) * 256 + col;
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)gsrc,
                                         (__attribute__((address_space(3))) void*)(pre_lds + 2048), 4, 0, 0);
        asm volatile("" ::: "memory");
      }
    }
  };

  auto epilogue = [&](auto kind_tag, int gi) {
    constexpr int KIND = decltype(kind_tag)::value;
    XTS(tslot);
    const int par = gi & 1, blk = gi >> 1;
    const float wcs = pre_wcs;
    float scv[R];  // per window: the accumulators' exponent x the column scale
#pragma unroll
    for (int v = 0; v < R; ++v) scv[v] = ldexpf(1.0f, ax.ex[par][1][v]) * wcs;
    if constexpr (KIND == 2) {
      // proj(GN_3(x)) = rstd (P gamma x - mu S_gamma) + S_beta; rows past n_windows are not written
      const float2 sp = {pre_sx, pre_sy};
      float* ob = enc_out + (size_t)e * n_windows * VGE_T * VGE_D + col;
#pragma unroll
      for (int v = 0; v < R; ++v) {  // window by window: its statistics live only while its rows are written
        float mu, rstd;
        gn_stats(3, v, mu, rstd);
        const int win = win0 + v;
        if (win < n_windows) {
#pragma unroll
          for (int t = 0; t < R; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r)
              if (x3s_rwin<W>(r) == v)
                ob[((size_t)win * VGE_T + x3s_rfr0<W>(t, r) + 4 * h) * VGE_D] =
                    fmaf(rstd, fmaf(acc.c[t][0][r], scv[v], -mu * sp.x), sp.y);
        }
      }
    } else {
      // K0, blocks 1..3: the corrections of this lane's frames (the taps of the frame inside the window); a lane's
      // frame depends on (t, r % (G / 2)) only: 16 values, as when a tile was one window
      constexpr int GH = G / 2;
      float cg[16], cb[16], gsv[R], gshv[R], muv[R], rstdv[R];
      if constexpr (KIND == 0) {
        if (blk > 0) {
          const int dil = 1 << blk;
          vmcnt0();  // this wave's LDS-DMA of the fold operands (issued before the stream) has landed
          const char* pl = pre_lds + i * 64;
          const floatx4 pre_g = *reinterpret_cast<const floatx4*>(pl);
          const float pre_g4 = *reinterpret_cast<const float*>(pl + 16);
          const floatx4 pre_b = *reinterpret_cast<const floatx4*>(pl + 32);
          const float pre_b4 = *reinterpret_cast<const float*>(pl + 48);
          const float pre_gw = *reinterpret_cast<const float*>(pre_lds + 2048 + i * 4);
          const float pre_gb = *reinterpret_cast<const float*>(pre_lds + 2048 + 128 + i * 4);
#pragma unroll
          for (int f = 0; f < 16; ++f) {
            const int row = x3s_rfr0<W>(f / GH, f % GH) + 4 * h;  // row + (tap - 2) dil in [0, 32)
            const bool k0 = row >= 2 * dil, k1 = row >= dil, k3 = row < 32 - dil, k4 = row < 32 - 2 * dil;
            cg[f] = (((k0 ? pre_g.x : 0.f) + (k1 ? pre_g.y : 0.f)) + pre_g.z) + (k3 ? pre_g.w : 0.f) + (k4 ? pre_g4 : 0.f);
            cb[f] = (((k0 ? pre_b.x : 0.f) + (k1 ? pre_b.y : 0.f)) + pre_b.z) + (k3 ? pre_b.w : 0.f) + (k4 ? pre_b4 : 0.f);
          }
#pragma unroll
          for (int v = 0; v < R; ++v) {
            gn_stats(blk - 1, v, muv[v], rstdv[v]);
            gsv[v] = rstdv[v] * pre_gw;
            gshv[v] = fmaf(-muv[v], gsv[v], pre_gb);
          }
        }
      }
#pragma unroll
      for (int t = 0; t < R; ++t) {
        floatx16& x = acc.c[t][0];
        if constexpr (KIND == 0) {
          // GELU(conv1(block input)); for blocks 1..3 the input is GN_{blk-1}(x), folded (file comment), and the
          // residual becomes GN_{blk-1}(x) here
          if (blk > 0) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int v = x3s_rwin<W>(r), f = t * GH + r % GH;
              res[t][r] = fmaf(res[t][r], gsv[v], gshv[v]);  // (x - mu) rstd gamma + beta, as conv_encoder_body
              x[r] = fmaf(rstdv[v], fmaf(-muv[v], cg[f], x[r] * scv[v]), cb[f]);
            }
          } else {
#pragma unroll
            for (int r = 0; r < 16; ++r) x[r] *= scv[x3s_rwin<W>(r)];  // (the stem output needs no correction)
          }
          gelu_tile(x);
        } else {
          // x = GELU(conv2(h) + residual): stored pre-GroupNorm, kept as the residual, partial statistics published
#pragma unroll
          for (int r = 0; r < 16; ++r) x[r] = fmaf(x[r], scv[x3s_rwin<W>(r)], res[t][r]);
          gelu_tile(x);
          res[t] = x;
        }
        __builtin_amdgcn_sched_barrier(0);  // one tile's temporaries at a time
      }
      if constexpr (KIND == 1) {
        // per-wave GroupNorm partials of every window: mean, then M2 about it (two-pass, in registers)
        float mw[R], q[R];
#pragma unroll
        for (int v = 0; v < R; ++v) mw[v] = q[v] = 0.f;
#pragma unroll
        for (int t = 0; t < R; ++t)
#pragma unroll
          for (int r = 0; r < 16; ++r) mw[x3s_rwin<W>(r)] += res[t][r];
#pragma unroll
        for (int v = 0; v < R; ++v) {
          mw[v] = wave_sum_last(mw[v]);
          mw[v] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, mw[v]), 63)) *
                  (1.0f / 1024.0f);
        }
#pragma unroll
        for (int t = 0; t < R; ++t)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float d = res[t][r] - mw[x3s_rwin<W>(r)];
            q[x3s_rwin<W>(r)] = fmaf(d, d, q[x3s_rwin<W>(r)]);
          }
#pragma unroll
        for (int v = 0; v < R; ++v) q[v] = wave_sum_last(q[v]);
        if (lane == 63) {
#pragma unroll
          for (int v = 0; v < R; ++v) {
            ax.stats[blk & 1][v][wave][0] = mw[v];
            ax.stats[blk & 1][v][wave][1] = q[v];
          }
        }
      }
      store_act([&](int t) -> const floatx16& { return acc.c[t][0]; }, (gi + 1) & 1);
    }
  };

  // SKIP (compile time): the tap-skipping stream code only where taps can be skipped (blocks 2, 3: dilation 4, 8);
  // the branch-free form for the others (same-box A/B: 1.099-1.108 ms with the skipping code everywhere, 1.084-1.090
  // this way)
  auto stream = [&](auto skip_tag, int gi, int part) {
    constexpr bool SKIP = decltype(skip_tag)::value;
    if (part == 0) {
      acc.zero();
    } else {  // channels of B: the accumulators move from A's exponent to B's (exact), window by window
      float f[R];
#pragma unroll
      for (int v = 0; v < R; ++v) f[v] = ldexpf(1.0f, ax.ex[gi & 1][0][v] - ax.ex[gi & 1][1][v]);
#pragma unroll
      for (int t = 0; t < R; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc.c[t][0][r] *= f[x3s_rwin<W>(r)];
    }
    const bool proj = gi == 8;
    const char* wb = reinterpret_cast<const char*>(proj ? ed.proj : ed.conv + (size_t)gi * 80 * (CHUNK_B / 2)) +
                     (size_t)part * 8 * CHUNK_B;
    if (X3S_PRIO) __builtin_amdgcn_s_setprio(1);
    stream_part<W, SKIP, SP>(acc, wb, proj ? 1 : 5, loff, xa + part * 8 * 32, i, proj ? 0 : 1 << (gi >> 1),
                             proj ? 0 : 2, X3S_ROT ? __builtin_amdgcn_readfirstlane((int)(blockIdx.x >> 3) & 7) : 0);
    __builtin_amdgcn_s_setprio(0);
  };

  // The task sequence of a half (file comment) is the same code for both: B starts it one barrier later and A ends
  // with one more, so B runs one phase behind.
  using K0 = std::integral_constant<int, 0>;
  using K1 = std::integral_constant<int, 1>;
  using K2 = std::integral_constant<int, 2>;
  [[maybe_unused]] int ph = 0;  // trace: this wave's phase index
  auto phase_end = [&]() {
    XTS(2 + 2 * ph);
    lds_barrier();
    XTS(3 + 2 * ph);
    ++ph;
    lane_setup();
  };
  XTS(1);
  if (grp == 1) phase_end();
  else lane_setup();
  stem_epilogue();
  phase_end();
  using NoSkip = std::integral_constant<bool, false>;
  using Skip = std::integral_constant<bool, true>;
  auto block = [&](auto skip_tag, int blk) {
    stream(skip_tag, 2 * blk, 0);
    phase_end();
    prefetch(K0{}, 2 * blk);
    stream(skip_tag, 2 * blk, 1);
    phase_end();
    epilogue(K0{}, 2 * blk);
    phase_end();
    stream(skip_tag, 2 * blk + 1, 0);
    phase_end();
    prefetch(K1{}, 2 * blk + 1);
    stream(skip_tag, 2 * blk + 1, 1);
    phase_end();
    epilogue(K1{}, 2 * blk + 1);
    phase_end();
  };
#pragma unroll 1
  for (int blk = 0; blk < 2; ++blk) block(NoSkip{}, blk);
#pragma unroll 1
  for (int blk = 2; blk < 4; ++blk) block(Skip{}, blk);
  stream(NoSkip{}, 8, 0);
  phase_end();
  prefetch(K2{}, 8);
  stream(NoSkip{}, 8, 1);
  phase_end();
  epilogue(K2{}, 8);
  phase_end();
  if (grp == 0) phase_end();
}

template <bool SP>
__global__ void __launch_bounds__(512, 1) conv_encoder_x3s_kernel(const float* __restrict__ feats,
                                                                   const EncDescX3* __restrict__ encs, vge::ConvSched cs,
                                                                   float* __restrict__ enc_out, int* __restrict__ status,
                                                                   int spin_limit) {
  extern __shared__ __attribute__((aligned(16))) char lds_raw[];
  X3sAux& ax = *reinterpret_cast<X3sAux*>(lds_raw + X3S_AUX_OFF);
  if (threadIdx.x < 2) ax.cnt[threadIdx.x] = 0;  // ordered before any exchange by the stem staging's barriers
#ifdef VGE_TRACE
  if (blockIdx.x < 64 && (threadIdx.x & 63) == 0)
    g_x3s_trace[(blockIdx.x * 8 + (threadIdx.x >> 6)) * 128 + 120] = __builtin_amdgcn_s_memtime();
#endif
  int n_ex = 0;
  const int n = cs.n_windows;
  const int bp = xcd_remap(blockIdx.x, cs.G);
  // Round order per XCD.  The blocks of XCD x start at round x % R (R rounds; at 256 windows two quad rounds, then
  // the vit pairs), so at any time about a third of the XCDs run the L2-bound vit pairs and their HBM stem loads
  // while the rest run MFMA-bound quads, instead of every CU hitting the same kind of round at once; inside an XCD
  // all CUs still stream one encoder in lockstep (its L2 shared).  A partial last round becomes a skipped slot in a
  // rotated block's order.  600 windows: 2.433-2.442 -> 2.422-2.423 ms; 4,096: unchanged.  Same box, interleaved
  // (profiles/ab_r04j_conv_round_order*.log): plain order 1.019-1.023 ms and 374 MB of fabric fetches (FETCH_SIZE x 2)
  // per launch, per XCD (this) 1.006-1.009 ms and 373 MB, per block (bp % 3: pairs beside quads inside every XCD)
  // 1.000-1.002 ms but 914 MB (the XCD's CUs then stream different encoders and the L2 sharing is lost).  Each unit's
  // results are unchanged.  VGE_X3S_ROT: 0 plain order, 3 per block (three full rounds), 4 per XCD; 1 / 2: blocks with bit
  // VGE_X3S_ROT_BIT of bp set start at that round.
#ifndef VGE_X3S_ROT
#define VGE_X3S_ROT 4
#endif
#ifndef VGE_X3S_ROT_BIT
#define VGE_X3S_ROT_BIT 0
#endif
#if VGE_X3S_ROT == 3
  const int rot = cs.n_units == 3 * cs.G ? bp % 3 : 0;  // (three full rounds only)
#elif VGE_X3S_ROT == 4
  const int rot = cs.G % 8 == 0 ? (bp / (cs.G / 8)) % ((cs.n_units + cs.G - 1) / cs.G) : 0;
#else
  const int rot = (VGE_X3S_ROT && cs.n_units == 3 * cs.G && ((bp >> VGE_X3S_ROT_BIT) & 1)) ? VGE_X3S_ROT : 0;
#endif
  const int n_rounds = (cs.n_units + cs.G - 1) / cs.G;
  for (int k = 0; k < n_rounds; ++k) {
    const int round = rot ? (k + rot) % n_rounds : k;
    const int u = round * cs.G + bp;
    if (u >= cs.n_units) continue;  // uniform over the block (only the last round is partial)
    if (u < cs.Q) {
      int e, w0;
      conv_unit(cs, u, e, w0);
      conv_x3s_body<4, SP>(feats, n, w0, encs[e], e, enc_out, lds_raw, n_ex, status, spin_limit,
                       round == X3S_TRACE_ROUND);
    } else {
      int e, w0;
      conv_unit(cs, u, e, w0);
      conv_x3s_body<2, SP>(feats, n, w0, encs[e], e, enc_out, lds_raw, n_ex, status, spin_limit,
                       round == X3S_TRACE_ROUND);
    }
  }
#ifdef VGE_TRACE
  if (blockIdx.x < 64 && (threadIdx.x & 63) == 0)
    g_x3s_trace[(blockIdx.x * 8 + (threadIdx.x >> 6)) * 128 + 121] = __builtin_amdgcn_s_memtime();
#endif
}

}  // namespace

namespace vge {

hipError_t encoder_x3s_kernel_setup() {
  hipError_t e = hipFuncSetAttribute((const void*)conv_encoder_x3s_kernel<true>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, X3S_LDS_BYTES);
  if (e == hipSuccess)
    e = hipFuncSetAttribute((const void*)conv_encoder_x3s_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            X3S_LDS_BYTES);
  return e;
}

// spin bound of the half-workgroup exchange (test hook vge_debug_set_x3s_spin_limit: 0 makes every wave that arrives
// before its group's last one give up, which must surface as VGE_ERR_DEVICE)
static int g_x3s_spin_limit = 1 << 22;

hipError_t launch_conv_encoders_x3s(const float* feats, int n_windows, const void* encs, int n_enc, unsigned heavy,
                                    float* enc_out, int* status, bool split, hipStream_t s) {
  if (n_windows < 1 || n_enc < 1) return hipSuccess;
  if (!status) return hipErrorInvalidValue;
  const ConvSched cs = conv_quad_sched(n_windows, n_enc, heavy);
  if (split)
    hipLaunchKernelGGL(conv_encoder_x3s_kernel<true>, dim3(cs.G), dim3(512), X3S_LDS_BYTES, s, feats,
                       reinterpret_cast<const EncDescX3*>(encs), cs, enc_out, status, g_x3s_spin_limit);
  else  // VGE_F16 (staggered single-fp16: hi planes only, one MFMA per product)
    hipLaunchKernelGGL(conv_encoder_x3s_kernel<false>, dim3(cs.G), dim3(512), X3S_LDS_BYTES, s, feats,
                       reinterpret_cast<const EncDescX3*>(encs), cs, enc_out, status, g_x3s_spin_limit);
  return hipGetLastError();
}

}  // namespace vge

// Test hook: the conv kernel's exchange spin bound (default 2^22 sleeps; < 0 restores it).  Returns the previous one.
extern "C" int vge_debug_set_x3s_spin_limit(int n) {
  const int prev = vge::g_x3s_spin_limit;
  vge::g_x3s_spin_limit = n < 0 ? (1 << 22) : n;
  return prev;
}

#ifdef VGE_TRACE
extern "C" int vge_debug_x3s_trace(long long* host, int n) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_x3s_trace), sizeof(long long) * (size_t)n);
}
#endif
