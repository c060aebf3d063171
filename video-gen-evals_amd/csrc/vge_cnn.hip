// Convolutional-network kernels of the per-frame keypoint extractor (DWPose: RTMPose-l whole-body and the
// YOLOX-L person detector) on gfx950.  Activations are NHWC bf16 with an explicit pixel stride, so a
// torch.cat along channels is just an output written at a channel offset of a wider buffer.
//
//   conv_bf16_kernel<TN,ACT,OUT,RES>  implicit-GEMM convolution on v_mfma_f32_32x32x16_bf16: C[pixel][cout] =
//       sum_k A[pixel][k] W[cout][k], k = tap * Cin + ci (tap-major, Cin a power of two >= 8).  A rows are
//       gathered straight from the NHWC input by global_load_lds (16 B = 8 channels per lane); taps that fall
//       in the zero padding (and K / M padding) read a zero page instead of being masked, so the LDS ring is
//       filled exactly like a dense GEMM's.  128 x TN output tile per 256-thread workgroup, 32-deep K stages in
//       a 3-slot ring, LDS image XOR-swizzled on the source address (conflict-free ds_read_b128 fragments),
//       XCD-contiguous tile ranges.  Epilogue through LDS, row-major: + bias (folded BatchNorm), SiLU /
//       sigmoid, + residual (bf16 identity of CSPNeXtBlock, or f32 x per-column scale for RTMCCBlock's
//       res_scale), bf16 or f32 store.  Every nn.Linear of the head runs here too (1x1 "image").
//   dwconv_kernel        depthwise KxK conv + folded BN + SiLU (one thread = 8 channels of one pixel).
//   spp_pool_kernel      SPPBottleneck's stride-1 max pools (5, 9, 13) written beside their input.
//   chan_mean_kernel / chan_attn_fc_kernel / chan_scale_kernel   ChannelAttention: avgpool -> 1x1 conv ->
//                        hardsigmoid -> x * a.
//   warp_prep_kernel     onnxpose.preprocess: per-instance affine crop (bilinear, border 0, uint8 round) of the
//                        RGB frame, BGR mean/std normalisation -> NHWC bf16 with 8 channels (3 used).
//   letterbox_focus_kernel  onnxdet.preprocess (resize by r, pad 114) + YOLOX Focus space-to-depth -> 16 ch.
#include "vge_common.h"
#include "vge_lds_attr.h"
#include "vge_cnn.h"
#include "vge_gemm.h"

#include <cstdlib>
#include <algorithm>
#include <type_traits>

namespace {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef unsigned uintx2_t __attribute__((ext_vector_type(2)));
typedef unsigned uintx4_t __attribute__((ext_vector_type(4)));

constexpr int CV_M = 128, CV_K = 32, CV_ST = 3;

enum { ACT_NONE = 0, ACT_SILU = 1, ACT_SIGMOID = 2, ACT_RELU = 3 };
enum { OUT_BF16 = 0, OUT_F32 = 1 };
enum { RES_NONE = 0, RES_BF16 = 1, RES_F32S = 2, RES_BF16_PRE = 3 };  // _PRE: added before the activation

struct ConvArgs {
  const bf16* x;       // NHWC input, pixel stride ldx elements (channel offset folded into the pointer)
  const bf16* w;       // [Npad][Kp] bf16, k = tap * Cin + ci, zero padded
  const float* bias;   // [Npad]
  void* out;           // NHWC output, pixel stride ldo
  const void* res;     // residual [M][ldr] (bf16 or f32)
  const float* rscale; // RES_F32S: per-column scale [Npad]
  const bf16* zero;    // >= 16 B of zeros (the source of padding taps)
  long ldx, ldo, ldr;
  int H, W, cin_log2, Ho, Wo, KW, kw_magic, stride, pad, taps, Kp, Cout, M;
  int gslice;          // grouped conv as block-diagonal slices: the tile of output columns n0.. reads input channels
                       // n0 .. n0 + Cin - 1 (Cin = the tile width; weights [Cout][taps * Cin], zero off the groups)
};

__device__ __forceinline__ int xcd_remap(int b, int nblk) {  // bijective: each XCD takes a contiguous range
  const int q8 = nblk >> 3, r8 = nblk & 7, x8 = b & 7;
  return (x8 < r8 ? x8 * (q8 + 1) : r8 * (q8 + 1) + (x8 - r8) * q8) + (b >> 3);
}

// Implicit-GEMM gather state of one A row (the tile rows a lane fetches): the address of the row's (kh, kw) = (0, 0)
// tap plus this lane's 16-B chunk (lc8 = 8 lc channels), and (ih0 << 16) | (iw0 & 0xFFFF) (a row past M gets ih0 =
// -16384, which fails every tap's bounds check).
struct RowState {
  const bf16* p;
  int hw0;
};
__device__ __forceinline__ RowState row_state(const ConvArgs& a, int m, int lc8) {
  const int hw = a.Ho * a.Wo;
  const int img = m / hw, rem = m - img * hw;
  const int oh = rem / a.Wo, ow = rem - oh * a.Wo;
  const int ih0 = m < a.M ? oh * a.stride - a.pad : -16384, iw0 = ow * a.stride - a.pad;
  // 64-bit row offset (n_img * H * W may pass 2^31 elements); a row past M keeps the base pointer (its taps all fail
  // the bounds check and read the zero page, so no out-of-range address is ever formed for it)
  const long off = m < a.M ? ((long)img * a.H + ih0) * a.W + iw0 : 0;
  return {a.x + off * a.ldx + lc8, (ih0 << 16) | (iw0 & 0xFFFF)};
}
// The 32-k stage starting at k0 of NR rows into LDS (row j's 1 KB wave-instruction at dst(j)).  Cin >= 32: the stage
// lies inside one tap, so the tap, its (kh, kw) and the channel base are uniform (scalar) and a row's source is its
// base + one scalar offset; Cin 8 / 16: a lane's chunk may fall in the next tap (per-lane tap).  Taps outside the
// image, past the kernel's taps, and rows past M read the zero page.
// The sources of the 32-k stage starting at k0 for NR rows: src[j] = row j's source or the zero page (taps outside
// the image, past the kernel's taps, rows past M).  Cin >= 32: the stage lies inside one tap, so the tap, its (kh, kw)
// and the channel base are uniform (scalar) and a row's source is its base + one scalar offset; Cin 8 / 16: a lane's
// chunk may fall in the next tap (per-lane tap).  Kept in registers: callers compute them while their MFMAs run and
// issue the loads at the top of the next step.
template <int NR>
__device__ __forceinline__ void gather_srcs(const ConvArgs& a, const RowState (&rs)[NR], int k0, int lc8,
                                            const bf16* (&src)[NR]) {
  int kh, kw, tap;
  long off;
  if (a.cin_log2 >= 5) {
    tap = k0 >> a.cin_log2;
    kh = (tap * a.kw_magic) >> 16;
    kw = tap - kh * a.KW;
    off = (long)(kh * a.W + kw) * a.ldx + (k0 & ((1 << a.cin_log2) - 1));
  } else {
    const int k = k0 + lc8;
    tap = k >> a.cin_log2;
    kh = (tap * a.kw_magic) >> 16;
    kw = tap - kh * a.KW;
    off = (long)(kh * a.W + kw) * a.ldx + (k & ((1 << a.cin_log2) - 1)) - lc8;
  }
#pragma unroll
  for (int j = 0; j < NR; ++j) {
    const int ih = (rs[j].hw0 >> 16) + kh, iw = (int)(short)rs[j].hw0 + kw;
    const bool ok = tap < a.taps && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
    const unsigned long v = ok ? reinterpret_cast<unsigned long>(rs[j].p + off) : reinterpret_cast<unsigned long>(a.zero);
    src[j] = reinterpret_cast<const bf16*>(v);
  }
}

__device__ __forceinline__ float silu(float v) { return v / (1.0f + __expf(-v)); }
__device__ __forceinline__ float sigm(float v) { return 1.0f / (1.0f + __expf(-v)); }

// 256 threads = 4 waves on 32x32x16 MFMAs.  BM = 128: 2 along M x 2 along N, wave tile 64 x TN/2; BM = 256 ("tall",
// for small Cout): 4 along M, wave tile 64 x TN, so each A byte in LDS feeds twice the MFMAs of the 128-row form.
template <int TN, int ACT, int OUT, int RES, int BM = CV_M>
__global__ void __launch_bounds__(256) conv_bf16_kernel(ConvArgs a) {
  constexpr int MW = BM / 64, NWV = 4 / MW;   // waves along M / N
  constexpr int AJ = BM / 64;                 // A wave-instructions (16 rows each) per wave per stage
  constexpr int TA = BM * CV_K * 2;           // A stage
  constexpr int TB = TN * CV_K * 2;           // B stage
  constexpr int SLOT = TA + TB;
  constexpr int NB = TN / (32 * NWV);         // 32-col MFMA tiles per wave
  constexpr int BQ = TN / 16 / 4;             // B wave-instructions per wave per stage
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / NWV, wn = wave % NWV;
  const int ntn = (a.Cout + TN - 1) / TN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = bid / ntn, nt = bid - mt * ntn;
  const int m0 = mt * BM, n0 = nt * TN;
  const int nk = a.Kp / CV_K;

  // per-lane gather state of this lane's AJ A rows (row = 16 q + lane / 4, q = AJ wave + j)
  const int lc = (lane & 3) ^ ((lane >> 4) & 3);  // logical 16-B chunk this lane fetches (pre-swizzled)
  const int lc8 = lc * 8;
  RowState rws[AJ];
#pragma unroll
  for (int j = 0; j < AJ; ++j) {
    rws[j] = row_state(a, m0 + 16 * (AJ * wave + j) + (lane >> 2), lc8);
    if (a.gslice) rws[j].p += n0;  // grouped: this column tile's input channel slice
  }
  const bf16* wrow[BQ];
#pragma unroll
  for (int j = 0; j < BQ; ++j) wrow[j] = a.w + (size_t)(n0 + 16 * (BQ * wave + j) + (lane >> 2)) * a.Kp + lc8;

  // software-pipelined ring: prep(st) computes stage st's A sources (after a step's MFMAs are issued, so the VALU work
  // runs beside them), fire(st) issues its loads at the top of the next step
  const bf16* nsrc[AJ];
  auto prep = [&](int st) { gather_srcs<AJ>(a, rws, st * CV_K, lc8, nsrc); };
  auto fire = [&](int st) {
    char* slot = lds + (st % CV_ST) * SLOT;
#pragma unroll
    for (int j = 0; j < AJ; ++j) glds16(nsrc[j], slot + (AJ * wave + j) * 1024);
#pragma unroll
    for (int j = 0; j < BQ; ++j) glds16(wrow[j] + st * CV_K, slot + TA + (BQ * wave + j) * 1024);
  };

  floatx16 acc[2][NB];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int u = 0; u < NB; ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[t][u][r] = 0.f;

  const int h = lane >> 5;
  const int swz = (lane >> 2) & 3;
  const int rowoff = (lane & 31) * 64;
  constexpr int LPS = AJ + BQ;  // global_load_lds per thread per stage
  for (int st = 0; st < CV_ST - 1; ++st) {
    prep(min(st, nk - 1));
    fire(min(st, nk - 1));
  }
  prep(min(CV_ST - 1, nk - 1));
  for (int kt = 0; kt < nk; ++kt) {
    vmcnt_b<LPS>();     // stage kt landed (stage kt + 1 may still be in flight)
    lds_barrier_b();    // ... for every wave; every wave is done reading stage kt - 1's slot
    fire(min(kt + CV_ST - 1, nk - 1));  // past the end: re-fetch the last stage into its own slot (same bytes)
    const char* cur = lds + (kt % CV_ST) * SLOT;
    const char* As = cur + wm * 64 * 64 + rowoff;
    const char* Bs = cur + TA + wn * (TN / NWV) * 64 + rowoff;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int co = ((2 * s + h) ^ swz) * 16;
      bf16x8 fa[2], fb[NB];
#pragma unroll
      for (int t = 0; t < 2; ++t) fa[t] = *reinterpret_cast<const bf16x8*>(As + t * 32 * 64 + co);
#pragma unroll
      for (int u = 0; u < NB; ++u) fb[u] = *reinterpret_cast<const bf16x8*>(Bs + u * 32 * 64 + co);
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int u = 0; u < NB; ++u)
          acc[t][u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[t], fb[u], acc[t][u], 0, 0, 0);
    }
    prep(min(kt + CV_ST, nk - 1));
  }

  // epilogue through LDS in BM / 64 row quarters / halves (64 rows of f32 each), row-major re-read: 8 columns per
  // thread
  vmcnt_b<0>();
  lds_barrier_b();
  constexpr int LDC = TN + 4;
  float* cs = reinterpret_cast<float*>(lds);
  constexpr int TPR = TN / 8;       // threads per row
  constexpr int RPP = 256 / TPR;    // rows per pass
#pragma unroll
  for (int half = 0; half < MW; ++half) {
    if (wm == half) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int u = 0; u < NB; ++u)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            cs[(t * 32 + (r & 3) + 8 * (r >> 2) + 4 * h) * LDC + wn * (TN / NWV) + u * 32 + (lane & 31)] = acc[t][u][r];
    }
    __syncthreads();
    const int c8 = (tid % TPR) * 8;
    const int col = n0 + c8;
    floatx4 b0 = *reinterpret_cast<const floatx4*>(a.bias + col);
    floatx4 b1 = *reinterpret_cast<const floatx4*>(a.bias + col + 4);
#pragma unroll
    for (int p = 0; p < 64 / RPP; ++p) {
      const int rl = p * RPP + tid / TPR;
      const int m = m0 + half * 64 + rl;
      if (m >= a.M || col >= a.Cout) continue;
      float v[8];
      const floatx4 x0 = *reinterpret_cast<const floatx4*>(cs + rl * LDC + c8) + b0;
      const floatx4 x1 = *reinterpret_cast<const floatx4*>(cs + rl * LDC + c8 + 4) + b1;
      v[0] = x0.x; v[1] = x0.y; v[2] = x0.z; v[3] = x0.w; v[4] = x1.x; v[5] = x1.y; v[6] = x1.z; v[7] = x1.w;
      if constexpr (RES == RES_BF16_PRE) {
        const bf16x8 r8 = *reinterpret_cast<const bf16x8*>(reinterpret_cast<const bf16*>(a.res) + (size_t)m * a.ldr + col);
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] += (float)r8[i];
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if constexpr (ACT == ACT_SILU) v[i] = silu(v[i]);
        if constexpr (ACT == ACT_SIGMOID) v[i] = sigm(v[i]);
        if constexpr (ACT == ACT_RELU) v[i] = fmaxf(v[i], 0.f);
      }
      if constexpr (RES == RES_BF16) {
        const bf16x8 r8 = *reinterpret_cast<const bf16x8*>(reinterpret_cast<const bf16*>(a.res) + (size_t)m * a.ldr + col);
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] += (float)r8[i];
      }
      if constexpr (RES == RES_F32S) {
        const float* rr = reinterpret_cast<const float*>(a.res) + (size_t)m * a.ldr + col;
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = fmaf(a.rscale[col + i], rr[i], v[i]);
      }
      if constexpr (OUT == OUT_BF16) {  // Cout % 8 == 0 (host-checked)
        bf16x8 o;
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = (bf16)v[i];
        *reinterpret_cast<bf16x8*>(reinterpret_cast<bf16*>(a.out) + (size_t)m * a.ldo + col) = o;
      } else {
        float* o = reinterpret_cast<float*>(a.out) + (size_t)m * a.ldo + col;
        if (col + 8 <= a.Cout && (a.ldo & 3) == 0) {
          *reinterpret_cast<floatx4*>(o) = floatx4{v[0], v[1], v[2], v[3]};
          *reinterpret_cast<floatx4*>(o + 4) = floatx4{v[4], v[5], v[6], v[7]};
        } else {
#pragma unroll
          for (int i = 0; i < 8; ++i)
            if (col + i < a.Cout) o[i] = v[i];
        }
      }
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------ conv v2 (wide tiles)
// The same implicit GEMM on 256 x BN tiles with 8 waves and gemm_bf16_kernel's schedule (vge_vit.hip): 32-deep
// stages in a 5-slot ring with three stages in flight (counted vmcnt, one barrier per stage), the next stage's
// fragments read into a second register set while the current one's MFMAs run, loads and LDS reads interleaved
// between the MFMAs (sched_group_barrier).  BN 256: waves 2 (M) x 4 (N) of 128 x 64; BN 128: 4 x 2 of 64 x 64.
// Epilogue through LDS (wave-private 64-row chunks re-read row-major, 4 columns per lane).
constexpr int C2_M = 256, C2_ST = 5;

// BM = 512 ("wide-M", BN 128 only): 8 waves of 128 x 64 as in the 256 x 256 tile, for layers with 128 output
// channels; 40 KB stages, so the ring has 4 slots (all 160 KB of LDS) and two stages in flight instead of three
template <int BN, int BM = C2_M>
struct C2Cfg {
  static_assert(BM == C2_M || (BM == 512 && BN == 128), "tile shapes");
  static constexpr int WM = BN == 256 ? 2 : 4, WN = 8 / WM;
  static constexpr int WR = BM / WM, WC = BN / WN;            // wave tile
  static constexpr int TM = WR / 32, TN = WC / 32;            // 32x32 MFMA tiles per wave
  static constexpr int TA = BM * CV_K * 2, TB = BN * CV_K * 2, SLOT = TA + TB;
  static constexpr int AJ = BM / 128;                         // A wave-instructions (16 rows each) per wave per stage
  static constexpr int BQ = BN / 128;                         // B wave-instructions per wave per stage
  static constexpr int LPS = AJ + BQ;                         // global_load_lds per thread per stage
  static constexpr int ST = BM == C2_M ? C2_ST : 4;           // ring slots
  static constexpr int RING = ST * SLOT, EPI = 8 * 64 * WC * 4;
  static constexpr int LDS = RING > EPI ? RING : EPI;
};

// SH = 1: the same wave tile on v_mfma_f32_16x16x32_bf16 (2 TM x 2 TN tiles of 16 x 16, one MFMA per 32-k stage and
// tile; gemm_bf16_kernel's SH form): the same LDS fragment bytes, MFMA cycles and K order, bit-identical outputs, and
// the chip holds a higher clock on this shape (MI355X_MICROARCH.md, DVFS give-back item 7)
template <int BN, int ACT, int OUT, int RES, int SH = 0>
__global__ void __launch_bounds__(512, 1) conv2_bf16_kernel(ConvArgs a) {
  using Cf = C2Cfg<BN>;
  constexpr int TM = Cf::TM, TN = Cf::TN, LPS = Cf::LPS, BQ = Cf::BQ;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / Cf::WN, wn = wave % Cf::WN;
  const int ntn = (a.Cout + BN - 1) / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = bid / ntn, nt = bid - mt * ntn;
  const int m0 = mt * C2_M, n0 = nt * BN;
  const int nk = a.Kp / CV_K;
  const int lc = (lane & 3) ^ ((lane >> 4) & 3);
  const int lc8 = lc * 8;
  RowState rws[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) rws[j] = row_state(a, m0 + 16 * (2 * wave + j) + (lane >> 2), lc8);
  const bf16* wrow[BQ];
#pragma unroll
  for (int j = 0; j < BQ; ++j) wrow[j] = a.w + (size_t)(n0 + 16 * (BQ * wave + j) + (lane >> 2)) * a.Kp + lc8;

  // software-pipelined ring (as conv2p_bf16_kernel): prep after a step's MFMAs, fire at the top of the next step
  const bf16* nsrc[2];
  auto prep = [&](int st) { gather_srcs<2>(a, rws, st * CV_K, lc8, nsrc); };
  auto fire = [&](int st) {
    char* slot = lds + (st % C2_ST) * Cf::SLOT;
#pragma unroll
    for (int j = 0; j < 2; ++j) glds16(nsrc[j], slot + (2 * wave + j) * 1024);
#pragma unroll
    for (int j = 0; j < BQ; ++j) glds16(wrow[j] + st * CV_K, slot + Cf::TA + (BQ * wave + j) * 1024);
  };
  const int h = lane >> 5, swz = (lane >> 2) & 3, rowoff = (lane & 31) * 64;
  struct Frag {
    bf16x8 a[2][TM], b[2][TN];
  };
  auto read = [&](int st, Frag& f) {
    const char* cur = lds + (st % C2_ST) * Cf::SLOT;
    if constexpr (SH == 0) {
      const char* As = cur + wm * Cf::WR * 64 + rowoff;
      const char* Bs = cur + Cf::TA + wn * Cf::WC * 64 + rowoff;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int co = ((2 * s + h) ^ swz) * 16;
#pragma unroll
        for (int t = 0; t < TM; ++t) f.a[s][t] = *reinterpret_cast<const bf16x8*>(As + t * 32 * 64 + co);
#pragma unroll
        for (int u = 0; u < TN; ++u) f.b[s][u] = *reinterpret_cast<const bf16x8*>(Bs + u * 32 * 64 + co);
      }
    } else {
      // 16x16x32 fragments: lane -> row (lane & 15) of a 16-row tile, k chunk lane >> 4 of the stage's 32;
      // a[t / TM][t % TM] = 16-row tile t, b[u / TN][u % TN] = 16-column tile u
      const int co = ((lane >> 4) ^ ((lane >> 2) & 3)) * 16, ro = (lane & 15) * 64;
      const char* As = cur + wm * Cf::WR * 64 + ro + co;
      const char* Bs = cur + Cf::TA + wn * Cf::WC * 64 + ro + co;
#pragma unroll
      for (int t = 0; t < 2 * TM; ++t) f.a[t / TM][t % TM] = *reinterpret_cast<const bf16x8*>(As + t * 16 * 64);
#pragma unroll
      for (int u = 0; u < 2 * TN; ++u) f.b[u / TN][u % TN] = *reinterpret_cast<const bf16x8*>(Bs + u * 16 * 64);
    }
  };
  floatx16 acc[SH ? 1 : TM][SH ? 1 : TN];
  floatx4 acq[SH ? 2 * TM : 1][SH ? 2 * TN : 1];  // SH = 1: [16-row tile][16-column tile]
#pragma unroll
  for (int t = 0; t < (SH ? 1 : TM); ++t)
#pragma unroll
    for (int u = 0; u < (SH ? 1 : TN); ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[t][u][r] = 0.f;
#pragma unroll
  for (int t = 0; t < (SH ? 2 * TM : 1); ++t)
#pragma unroll
    for (int u = 0; u < (SH ? 2 * TN : 1); ++u) acq[t][u] = floatx4{0.f, 0.f, 0.f, 0.f};
  auto mma = [&](const Frag& f, int s) {  // SH = 1: s = 16-row tiles TM s .. TM s + TM - 1
    if constexpr (SH == 0) {
#pragma unroll
      for (int t = 0; t < TM; ++t)
#pragma unroll
        for (int u = 0; u < TN; ++u)
          acc[t][u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.a[s][t], f.b[s][u], acc[t][u], 0, 0, 0);
    } else {
#pragma unroll
      for (int t = 0; t < TM; ++t)
#pragma unroll
        for (int u = 0; u < 2 * TN; ++u)
          acq[TM * s + t][u] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.a[s][t], f.b[u / TN][u % TN], acq[TM * s + t][u], 0, 0, 0);
    }
  };
  constexpr int NM = TM * TN * (SH ? 2 : 1);  // MFMAs per half-stage call of mma
  auto step = [&](int kt, Frag& cur, Frag& nxt) {
    vmcnt_b<2 * LPS>();  // stage kt + 1 landed (kt + 2, kt + 3 in flight)
    lds_barrier_b();
    fire(min(kt + 4, nk - 1));  // past the end: the last stage again, into its own slot (same bytes)
    read(min(kt + 1, nk - 1), nxt);
    mma(cur, 0);
    mma(cur, 1);
    prep(min(kt + 5, nk - 1));
#pragma unroll
    for (int j = 0; j < LPS; ++j) {
      __builtin_amdgcn_sched_group_barrier(0x008, NM / LPS > 0 ? NM / LPS : 1, 0);  // MFMA
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);                            // VMEM (global_load_lds)
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      __builtin_amdgcn_sched_group_barrier(0x008, NM / 4 > 0 ? NM / 4 : 1, 0);      // MFMA
      __builtin_amdgcn_sched_group_barrier(0x100, (2 * (TM + TN) + 3) / 4, 0);     // DS read
      __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);                            // VALU (the next stage's sources)
    }
  };
  for (int st = 0; st < C2_ST - 1; ++st) {
    prep(min(st, nk - 1));
    fire(min(st, nk - 1));
  }
  prep(min(C2_ST - 1, nk - 1));
  vmcnt_b<3 * LPS>();  // stage 0 landed
  lds_barrier_b();
  Frag f0, f1;
  read(0, f0);
  int kt = 0;
  for (; kt + 1 < nk; kt += 2) {
    step(kt, f0, f1);
    step(kt + 1, f1, f0);
  }
  if (kt < nk) step(kt, f0, f1);

  // epilogue: each wave stages 64-row chunks of its tile (C layout) in its private LDS region and re-reads them
  // row-major, 4 columns per lane (in-order LDS: no barrier between a wave's own stores and loads)
  vmcnt_b<0>();
  lds_barrier_b();
  constexpr int WC = Cf::WC, RPI = 256 / WC;  // rows per read instruction
  float* my = reinterpret_cast<float*>(lds) + wave * (64 * WC);
  const int lr = lane / (WC / 4), c4 = (lane % (WC / 4)) * 4;
  const int gcol = n0 + wn * WC + c4;
  const floatx4 bb = *reinterpret_cast<const floatx4*>(a.bias + gcol);
  floatx4 rsc = {0.f, 0.f, 0.f, 0.f};
  if constexpr (RES == RES_F32S) rsc = *reinterpret_cast<const floatx4*>(a.rscale + gcol);
#pragma unroll
  for (int half = 0; half < TM / 2; ++half) {
    if constexpr (SH == 0) {
#pragma unroll
      for (int tt = 0; tt < 2; ++tt)
#pragma unroll
        for (int u = 0; u < TN; ++u)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            my[(tt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h) * WC + u * 32 + (lane & 31)] = acc[2 * half + tt][u][r];
    } else {
#pragma unroll
      for (int tt = 0; tt < 4; ++tt)
#pragma unroll
        for (int u = 0; u < 2 * TN; ++u)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            my[(tt * 16 + 4 * (lane >> 4) + r) * WC + u * 16 + (lane & 15)] = acq[4 * half + tt][u][r];
    }
#pragma unroll 4
    for (int it = 0; it < 64 / RPI; ++it) {
      const int rl = it * RPI + lr;
      const int m = m0 + wm * Cf::WR + half * 64 + rl;
      floatx4 v = *reinterpret_cast<const floatx4*>(my + rl * WC + c4) + bb;
      if (m >= a.M || gcol >= a.Cout) continue;
      float e[4] = {v.x, v.y, v.z, v.w};
      if constexpr (RES == RES_BF16_PRE) {
        typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
        const bf16x4_t r4 = *reinterpret_cast<const bf16x4_t*>(reinterpret_cast<const bf16*>(a.res) + (size_t)m * a.ldr + gcol);
#pragma unroll
        for (int i = 0; i < 4; ++i) e[i] += (float)r4[i];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if constexpr (ACT == ACT_SILU) e[i] = silu(e[i]);
        if constexpr (ACT == ACT_SIGMOID) e[i] = sigm(e[i]);
        if constexpr (ACT == ACT_RELU) e[i] = fmaxf(e[i], 0.f);
      }
      if constexpr (RES == RES_BF16) {
        typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
        const bf16x4_t r4 = *reinterpret_cast<const bf16x4_t*>(reinterpret_cast<const bf16*>(a.res) + (size_t)m * a.ldr + gcol);
#pragma unroll
        for (int i = 0; i < 4; ++i) e[i] += (float)r4[i];
      }
      if constexpr (RES == RES_F32S) {
        const floatx4 r4 = *reinterpret_cast<const floatx4*>(reinterpret_cast<const float*>(a.res) + (size_t)m * a.ldr + gcol);
        e[0] = fmaf(rsc.x, r4.x, e[0]);
        e[1] = fmaf(rsc.y, r4.y, e[1]);
        e[2] = fmaf(rsc.z, r4.z, e[2]);
        e[3] = fmaf(rsc.w, r4.w, e[3]);
      }
      if constexpr (OUT == OUT_BF16) {
        typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
        bf16x4_t o;
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = (bf16)e[i];
        *reinterpret_cast<bf16x4_t*>(reinterpret_cast<bf16*>(a.out) + (size_t)m * a.ldo + gcol) = o;
      } else {
        float* o = reinterpret_cast<float*>(a.out) + (size_t)m * a.ldo + gcol;
        if (gcol + 4 <= a.Cout && (a.ldo & 3) == 0) {
          *reinterpret_cast<floatx4*>(o) = floatx4{e[0], e[1], e[2], e[3]};
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (gcol + i < a.Cout) o[i] = e[i];
        }
      }
    }
  }
}

// ------------------------------------------------------------------------- conv v2, persistent (default)
// conv2_bf16_kernel's tiles and schedule on a persistent grid (one workgroup per CU, tiles b, b + G, b + 2G, ...
// with G a multiple of 8, so a workgroup stays on its XCD's contiguous tile range) with ONE stage stream across
// its tiles: the ring issues stage g + 4 of the global sequence (tile g / nk, k-stage g % nk), so the next tile's
// first four stages are in flight while this tile's epilogue runs, and the next tile's first fragments are read
// during this tile's last MFMAs.  The epilogue leaves the LDS (ring) alone: the C-layout accumulators are turned
// row-major inside each 4-lane quad (two DPP quad_perm exchange rounds: lane i of a quad then holds row i, four
// consecutive columns) and stored straight to global memory, 8 B (bf16) / 16 B (f32) per lane.  vmcnt counts the
// epilogue's stores in issue order between the ring stages, so the three steps after an epilogue allow NST more
// outstanding operations.
// Tile id -> (row panel, column panel): groups of C2_GM row panels walk the column panels with the row panel fastest,
// so the ~32 consecutive ids an XCD runs at once cover ~8 row panels x ~4 column panels (A and W panels re-read from
// the XCD's L2 instead of the fabric when Cout spans many column panels; the same order as gemm_bf16_kernel's)
constexpr int C2_GM = 8;
__device__ __forceinline__ void c2_tile(int bid, int ntn, int mtn, int& mt, int& nt) {
  const int grp = bid / (C2_GM * ntn), rem = bid - grp * (C2_GM * ntn);
  const int gm = min(C2_GM, mtn - grp * C2_GM);
  mt = grp * C2_GM + rem % gm;
  nt = rem / gm;
}

template <int CTRL>
__device__ __forceinline__ float dppq(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}
// 4x4 transpose inside each quad: on entry lane i holds column i of rows 0..3 (v0..v3), on exit row i, columns 0..3
__device__ __forceinline__ void quad_t4(float& v0, float& v1, float& v2, float& v3, bool o1, bool o2) {
  float x = o1 ? v0 : v1, y = dppq<0xB1>(x);  // quad_perm [1,0,3,2]
  v0 = o1 ? y : v0;
  v1 = o1 ? v1 : y;
  x = o1 ? v2 : v3;
  y = dppq<0xB1>(x);
  v2 = o1 ? y : v2;
  v3 = o1 ? v3 : y;
  x = o2 ? v0 : v2;
  y = dppq<0x4E>(x);  // quad_perm [2,3,0,1]
  v0 = o2 ? y : v0;
  v2 = o2 ? v2 : y;
  x = o2 ? v1 : v3;
  y = dppq<0x4E>(x);
  v1 = o2 ? y : v1;
  v3 = o2 ? v3 : y;
}

template <int BN, int ACT, int OUT, int RES, int BM>
__global__ void __launch_bounds__(512, 1) conv2p_bf16_kernel(ConvArgs a) {
  using Cf = C2Cfg<BN, BM>;
  constexpr int TM = Cf::TM, TN = Cf::TN, LPS = Cf::LPS, BQ = Cf::BQ, AJ = Cf::AJ, ST = Cf::ST;
  constexpr int NST = TM * TN * 4;  // epilogue stores per thread
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / Cf::WN, wn = wave % Cf::WN;
  const int ntn = (a.Cout + BN - 1) / BN, ntiles = ((a.M + BM - 1) / BM) * ntn;
  const int G = gridDim.x, b = blockIdx.x;
  const int T = (ntiles - b + G - 1) / G;  // host: G <= ntiles, G % 8 == 0 unless G == ntiles
  const int nk = (a.Kp / CV_K + 1) & ~1, total = T * nk;  // even: an odd K gets one all-zero stage (zero page)
  const int lc = (lane & 3) ^ ((lane >> 4) & 3);

  // ---- issue side: gather state of the tile whose stages are being issued
  const int lc8 = lc * 8;
  RowState rws[AJ];
  const bf16* wrow[BQ];
  auto setup = [&](int i) {
    int mt, nt;
    c2_tile(xcd_remap(b + i * G, ntiles), ntn, ntiles / ntn, mt, nt);
    const int m0 = mt * BM, n0 = nt * BN;
#pragma unroll
    for (int j = 0; j < AJ; ++j) rws[j] = row_state(a, m0 + 16 * (AJ * wave + j) + (lane >> 2), lc8);
#pragma unroll
    for (int j = 0; j < BQ; ++j) wrow[j] = a.w + (size_t)(n0 + 16 * (BQ * wave + j) + (lane >> 2)) * a.Kp + lc * 8;
  };
  int is_t = 0, is_k = -1, is_g = -1;  // last prepared stage (tile, k-stage, global index)
  setup(0);
  // The ring is software-pipelined: prep(g) moves the issue state to stage g and computes its A sources (VALU work,
  // done right after a step's MFMAs are issued, so it runs beside them); fire() issues the prepared stage's loads at
  // the top of the next step.  Past the end, prep keeps the last stage: it is re-fetched into its own slot (same
  // bytes).
  const bf16* nsrc[AJ];
  auto prep = [&](int g) {  // g == is_g + 1, or past the end
    if (g < total) {
      is_g = g;
      if (++is_k == nk) {
        is_k = 0;
        setup(++is_t);
      }
    }
    gather_srcs<AJ>(a, rws, is_k * CV_K, lc8, nsrc);
  };
  auto fire = [&]() {
    char* slot = lds + (is_g % ST) * Cf::SLOT;
#pragma unroll
    for (int j = 0; j < AJ; ++j) glds16(nsrc[j], slot + (AJ * wave + j) * 1024);
    const bool kin = is_k * CV_K < a.Kp;
#pragma unroll
    for (int j = 0; j < BQ; ++j) glds16(kin ? wrow[j] + is_k * CV_K : a.zero, slot + Cf::TA + (BQ * wave + j) * 1024);
  };

  // ---- compute side
  const int h = lane >> 5, swz = (lane >> 2) & 3, rowoff = (lane & 31) * 64;
  struct Frag {
    bf16x8 a[2][TM], b[2][TN];
  };
  auto read = [&](int g, Frag& f) {
    const char* cur = lds + (g % ST) * Cf::SLOT;
    const char* As = cur + wm * Cf::WR * 64 + rowoff;
    const char* Bs = cur + Cf::TA + wn * Cf::WC * 64 + rowoff;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int co = ((2 * s + h) ^ swz) * 16;
#pragma unroll
      for (int t = 0; t < TM; ++t) f.a[s][t] = *reinterpret_cast<const bf16x8*>(As + t * 32 * 64 + co);
#pragma unroll
      for (int u = 0; u < TN; ++u) f.b[s][u] = *reinterpret_cast<const bf16x8*>(Bs + u * 32 * 64 + co);
    }
  };
  floatx16 acc[TM][TN];
  auto zero = [&]() {
#pragma unroll
    for (int t = 0; t < TM; ++t)
#pragma unroll
      for (int u = 0; u < TN; ++u)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[t][u][r] = 0.f;
  };
  zero();
  auto mma = [&](const Frag& f, int s) {
#pragma unroll
    for (int t = 0; t < TM; ++t)
#pragma unroll
      for (int u = 0; u < TN; ++u)
        acc[t][u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.a[s][t], f.b[s][u], acc[t][u], 0, 0, 0);
  };

  // epilogue: quad i of lanes holds (after quad_t4) row 8 q + 4 h + i of each 32-row block, columns 4 (lane % 32 / 4)
  // .. + 3.  Residual loads and output stores are raw buffer accesses on per-tile descriptors (rows past M and columns
  // past Cout get an out-of-range offset: loads return 0, stores are dropped), so the epilogue is one branch-free block
  // and the compiler's in-order vmcnt accounting stays exact.  The tile's bias / rscale are loaded at the top of its
  // last step (before that step's ring loads); residual rows are loaded one 32-row block ahead of their use.
  const bool o1 = lane & 1, o2 = lane & 2;
  const int qrow = 4 * h + (lane & 3), qcol = 4 * ((lane & 31) >> 2);
  constexpr int OE = OUT == OUT_BF16 ? 2 : 4;  // output element bytes
  constexpr int RE = RES == RES_F32S ? 4 : 2;  // residual element bytes
  typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
  typedef typename std::conditional<RES == RES_F32S, uintx4_t, uintx2_t>::type RV;
  floatx4 bb[TN], rs[TN];
  auto tile_mn = [&](int i, int& m0, int& n0) {
    int mt, nt;
    c2_tile(xcd_remap(b + i * G, ntiles), ntn, ntiles / ntn, mt, nt);
    m0 = mt * BM;
    n0 = nt * BN;
  };
  // bias / rscale: asm loads, invisible to hipcc's waitcnt pass (which answers any load issued among LDS-DMA ring
  // loads and stores with vmcnt(0)); consts_wait retires them by count, naming the registers so nothing reads them
  // earlier (cdna_hip_programming.md 5.7 item 1 form ii)
  constexpr int NCL = RES == RES_F32S ? 2 * TN : TN;  // asm loads per load_consts
  auto load_consts = [&](int i) {
    int m0, n0;
    tile_mn(i, m0, n0);
    const int cw = n0 + wn * Cf::WC + qcol;
#pragma unroll
    for (int u = 0; u < TN; ++u) {
      asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(bb[u]) : "v"(a.bias + cw + 32 * u) : "memory");
      if constexpr (RES == RES_F32S)
        asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(rs[u]) : "v"(a.rscale + cw + 32 * u) : "memory");
    }
  };
  auto consts_wait = [&]() {  // issued after them: two steps' ring loads (the last step's vmcnt(LPS) retired them)
    static_assert(TN == 2, "consts_wait names two registers");
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (RES == RES_F32S)
      asm volatile("s_waitcnt vmcnt(%4)" : "+v"(bb[0]), "+v"(bb[1]), "+v"(rs[0]), "+v"(rs[1]) : "i"(2 * LPS) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(%2)" : "+v"(bb[0]), "+v"(bb[1]) : "i"(2 * LPS) : "memory");
    (void)NCL;
  };
  auto epilogue = [&](int i) {
    consts_wait();
    int m0, n0;
    tile_mn(i, m0, n0);
    const int rows = min(BM, a.M - m0);
    const __amdgpu_buffer_rsrc_t ob = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<char*>(a.out) + (size_t)m0 * a.ldo * OE, (short)0, (int)((size_t)rows * a.ldo * OE), 0x00020000);
    __amdgpu_buffer_rsrc_t rb = ob;
    if constexpr (RES != RES_NONE)
      rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(reinterpret_cast<const char*>(a.res)) + (size_t)m0 * a.ldr * RE,
                                             (short)0, (int)((size_t)rows * a.ldr * RE), 0x00020000);
    const int rw = wm * Cf::WR + qrow, cw = n0 + wn * Cf::WC + qcol;
    auto offs = [&](int t, int u, int q, long ld, int eb) {
      const int r = rw + 32 * t + 8 * q, col = cw + 32 * u;
      return (r < rows && col + 4 <= a.Cout) ? (r * (int)ld + col) * eb : 0x7FFFFFF0;  // host: Cout % 4 == 0
    };
    RV rv[2][4];  // residual of one 32 x 32 block, loaded one block ahead
    auto rload = [&](int blk, RV (&d)[4]) {
      const int t = blk / TN, u = blk % TN;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if constexpr (RES == RES_BF16 || RES == RES_BF16_PRE)
          d[q] = __builtin_amdgcn_raw_buffer_load_b64(rb, offs(t, u, q, a.ldr, RE), 0, 0);
        if constexpr (RES == RES_F32S) d[q] = __builtin_amdgcn_raw_buffer_load_b128(rb, offs(t, u, q, a.ldr, RE), 0, 0);
      }
    };
    if constexpr (RES != RES_NONE) rload(0, rv[0]);
#pragma unroll
    for (int t = 0; t < TM; ++t)
#pragma unroll
      for (int u = 0; u < TN; ++u) {
        const int blk = t * TN + u;
        if constexpr (RES != RES_NONE)
          if (blk + 1 < TM * TN) rload(blk + 1, rv[(blk + 1) & 1]);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float e[4] = {acc[t][u][4 * q], acc[t][u][4 * q + 1], acc[t][u][4 * q + 2], acc[t][u][4 * q + 3]};
          quad_t4(e[0], e[1], e[2], e[3], o1, o2);
          e[0] += bb[u].x;
          e[1] += bb[u].y;
          e[2] += bb[u].z;
          e[3] += bb[u].w;
          if constexpr (RES == RES_BF16_PRE) {
            const bf16x4_t r4 = __builtin_bit_cast(bf16x4_t, rv[blk & 1][q]);
#pragma unroll
            for (int c = 0; c < 4; ++c) e[c] += (float)r4[c];
          }
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            if constexpr (ACT == ACT_SILU) e[c] = silu(e[c]);
            if constexpr (ACT == ACT_SIGMOID) e[c] = sigm(e[c]);
            if constexpr (ACT == ACT_RELU) e[c] = fmaxf(e[c], 0.f);
          }
          if constexpr (RES == RES_BF16) {
            const bf16x4_t r4 = __builtin_bit_cast(bf16x4_t, rv[blk & 1][q]);
#pragma unroll
            for (int c = 0; c < 4; ++c) e[c] += (float)r4[c];
          }
          if constexpr (RES == RES_F32S) {
            const floatx4 r4 = __builtin_bit_cast(floatx4, rv[blk & 1][q]);
            e[0] = fmaf(rs[u].x, r4.x, e[0]);
            e[1] = fmaf(rs[u].y, r4.y, e[1]);
            e[2] = fmaf(rs[u].z, r4.z, e[2]);
            e[3] = fmaf(rs[u].w, r4.w, e[3]);
          }
          const int oo = offs(t, u, q, a.ldo, OE);
          if constexpr (OUT == OUT_BF16) {
            bf16x4_t o;
#pragma unroll
            for (int c = 0; c < 4; ++c) o[c] = (bf16)e[c];
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(uintx2_t, o), ob, oo, 0, 0);
          } else {
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(uintx4_t, floatx4{e[0], e[1], e[2], e[3]}), ob, oo, 0, 0);
          }
        }
    }
  };

  constexpr int NM = TM * TN;
  // one 32-deep stage; kk = its index in the tile; after an epilogue (tile i > 0) its NST stores sit between the
  // ring stages for three steps
  // mode 0: plain step; 1: the tile's second-to-last step, which loads its bias / rscale ahead of its ring loads;
  // 2: the last step, whose wait also retires them (and every store of the previous epilogue)
  // ST slots: a step waits for stage g + 1 with ST - 3 later stages in flight and issues stage g + ST - 1; an
  // epilogue's stores stay between the ring stages for ST - 2 steps
  auto body = [&](int g, int kk, int i, Frag& cur, Frag& nxt, int mode) {
    if (mode == 2)
      vmcnt_b<LPS>();
    else if (i > 0 && kk < ST - 2)
      vmcnt_b<(ST - 3) * LPS + NST>();
    else
      vmcnt_b<(ST - 3) * LPS>();
    lds_barrier_b();
    if (mode == 1) load_consts(i);
    fire();  // stage g + ST - 1
    read(min(g + 1, total - 1), nxt);
    mma(cur, 0);
    mma(cur, 1);
    prep(g + ST);
#pragma unroll
    for (int j = 0; j < LPS; ++j) {
      __builtin_amdgcn_sched_group_barrier(0x008, NM / LPS > 0 ? NM / LPS : 1, 0);  // MFMA
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);                            // VMEM (global_load_lds)
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      __builtin_amdgcn_sched_group_barrier(0x008, NM / 4 > 0 ? NM / 4 : 1, 0);      // MFMA
      __builtin_amdgcn_sched_group_barrier(0x100, (2 * (TM + TN) + 3) / 4, 0);     // DS read
      __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);                            // VALU (the next stage's sources)
    }
  };
  auto last = [&](int g, int kk, int i, Frag& cur, Frag& nxt) {  // the tile's last stage + its epilogue
    body(g, kk, i, cur, nxt, 2);
    epilogue(i);
    zero();
  };
  for (int st = 0; st < ST - 1; ++st) {
    prep(st);
    fire();
  }
  prep(ST - 1);
  vmcnt_b<(ST - 2) * LPS>();  // stage 0 landed
  lds_barrier_b();
  Frag f0, f1;
  read(0, f0);
  int g = 0;
  for (int i = 0; i < T; ++i) {  // every tile starts with its first fragments in f0
    for (int kk = 0; kk < nk - 2; kk += 2, g += 2) {
      body(g, kk, i, f0, f1, 0);
      body(g + 1, kk + 1, i, f1, f0, 0);
    }
    body(g, nk - 2, i, f0, f1, 1);
    last(g + 1, nk - 1, i, f1, f0);
    g += 2;
  }
  vmcnt_b<0>();
}

// ------------------------------------------------------------------------------------ depthwise
// y[p][c] = SiLU(b[c] + sum_{kh,kw} w[kh*K+kw][c] x[p + (kh - pad, kw - pad)][c]), stride 1, f32 weights.
template <int K>
__global__ void __launch_bounds__(256) dwconv_kernel(const bf16* __restrict__ x, long ldx, const float* __restrict__ w,
                                                     const float* __restrict__ b, bf16* __restrict__ y, long ldy,
                                                     int n_img, int H, int W, int C) {
  const int cg = C >> 3;
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (long)n_img * H * W * cg) return;
  const int c8 = (int)(gid % cg) * 8;
  const long pix = gid / cg;
  const int ow = (int)(pix % W), oh = (int)((pix / W) % H);
  const long img = pix / ((long)W * H);
  float acc[8];
  {
    const floatx4 b0 = *reinterpret_cast<const floatx4*>(b + c8), b1 = *reinterpret_cast<const floatx4*>(b + c8 + 4);
    acc[0] = b0.x; acc[1] = b0.y; acc[2] = b0.z; acc[3] = b0.w; acc[4] = b1.x; acc[5] = b1.y; acc[6] = b1.z; acc[7] = b1.w;
  }
  constexpr int P = K / 2;
#pragma unroll
  for (int kh = 0; kh < K; ++kh) {
    const int ih = oh + kh - P;
    if ((unsigned)ih >= (unsigned)H) continue;
#pragma unroll
    for (int kw = 0; kw < K; ++kw) {
      const int iw = ow + kw - P;
      if ((unsigned)iw >= (unsigned)W) continue;
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(x + ((img * H + ih) * W + iw) * ldx + c8);
      const float* wt = w + (kh * K + kw) * C + c8;
      const floatx4 w0 = *reinterpret_cast<const floatx4*>(wt), w1 = *reinterpret_cast<const floatx4*>(wt + 4);
      acc[0] = fmaf(w0.x, (float)v[0], acc[0]);
      acc[1] = fmaf(w0.y, (float)v[1], acc[1]);
      acc[2] = fmaf(w0.z, (float)v[2], acc[2]);
      acc[3] = fmaf(w0.w, (float)v[3], acc[3]);
      acc[4] = fmaf(w1.x, (float)v[4], acc[4]);
      acc[5] = fmaf(w1.y, (float)v[5], acc[5]);
      acc[6] = fmaf(w1.z, (float)v[6], acc[6]);
      acc[7] = fmaf(w1.w, (float)v[7], acc[7]);
    }
  }
  bf16x8 o;
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = (bf16)silu(acc[i]);
  *reinterpret_cast<bf16x8*>(y + pix * ldy + c8) = o;
}

// Sliding-window form: one thread = 4 channels of RB (32) consecutive output rows of one column.  A 5 x 5 window of raw
// bf16x4 pixels slides down the column in registers, so each output row loads one new input row (5 pixels, 8 B
// each): 1/5 of the loads of the form above, weights for the 4 channels held in registers.  Per output the taps
// are summed in (kh, kw) order with out-of-range taps adding 0 -- the same sums as dwconv_kernel.
typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
template <int RB>
__global__ void __launch_bounds__(256) dwconv5_rb_kernel(const bf16* __restrict__ x, long ldx, const float* __restrict__ w,
                                                         const float* __restrict__ b, bf16* __restrict__ y, long ldy,
                                                         int n_img, int H, int W, int C) {
  const int cg = C >> 2, nstrip = (H + RB - 1) / RB;
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (long)n_img * nstrip * W * cg) return;
  const int c4 = (int)(gid % cg) * 4;
  long t = gid / cg;
  const int ow = (int)(t % W);
  t /= W;
  const int oh0 = (int)(t % nstrip) * RB;
  const long img = t / nstrip;
  float wr[25][4];
#pragma unroll
  for (int k = 0; k < 25; ++k) {
    const floatx4 v = *reinterpret_cast<const floatx4*>(w + k * C + c4);
    wr[k][0] = v.x; wr[k][1] = v.y; wr[k][2] = v.z; wr[k][3] = v.w;
  }
  const floatx4 bb = *reinterpret_cast<const floatx4*>(b + c4);
  const bf16* colp = x + img * H * W * ldx + c4;
  auto load_row = [&](int ih, bf16x4_t (&raw)[5]) {
#pragma unroll
    for (int kw = 0; kw < 5; ++kw) {
      const int iw = ow - 2 + kw;
      raw[kw] = bf16x4_t{(bf16)0.f, (bf16)0.f, (bf16)0.f, (bf16)0.f};
      if ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W)
        raw[kw] = *reinterpret_cast<const bf16x4_t*>(colp + ((long)ih * W + iw) * ldx);
    }
  };
  // the window lives in f32, input row ih in slot (ih - oh0 + 2) % 5; the output loop is unrolled by 5 so every
  // slot index is static (no register moves); the next input row is loaded one output ahead
  float wf[5][5][4];
  bf16x4_t nxt[5];
  auto to_slot = [&](const bf16x4_t (&raw)[5], float (&slot)[5][4]) {
#pragma unroll
    for (int kw = 0; kw < 5; ++kw)
#pragma unroll
      for (int c = 0; c < 4; ++c) slot[kw][c] = (float)raw[kw][c];
  };
#pragma unroll
  for (int kh = 0; kh < 4; ++kh) {
    load_row(oh0 - 2 + kh, nxt);
    to_slot(nxt, wf[kh]);
  }
  load_row(oh0 + 2, nxt);
  const int rows = min(RB, H - oh0);
#pragma unroll 1
  for (int r = 0; r < rows; r += 5) {
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      if (r + j >= rows) break;
      to_slot(nxt, wf[(j + 4) % 5]);
      load_row(oh0 + r + j + 3, nxt);  // in flight while this output's 100 FMAs run
      float acc[4] = {bb.x, bb.y, bb.z, bb.w};
#pragma unroll
      for (int kh = 0; kh < 5; ++kh)
#pragma unroll
        for (int kw = 0; kw < 5; ++kw)
#pragma unroll
          for (int c = 0; c < 4; ++c) acc[c] = fmaf(wr[kh * 5 + kw][c], wf[(j + kh) % 5][kw][c], acc[c]);
      bf16x4_t o;
#pragma unroll
      for (int c = 0; c < 4; ++c) o[c] = (bf16)silu(acc[c]);
      *reinterpret_cast<bf16x4_t*>(y + ((img * H + oh0 + r + j) * W + ow) * ldy + c4) = o;
    }
  }
}

// ------------------------------------------------------------------------------------ SPP max pools
// buf[p][0:C] is the input; writes max_pool(k)(input) for k = k0, k1, k2 at channel offsets C, 2C, 3C.
__global__ void __launch_bounds__(256) spp_pool_kernel(bf16* __restrict__ buf, long ld, int n_img, int H, int W, int C,
                                                       int k0, int k1, int k2) {
  const int cg = C >> 3;
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (long)n_img * H * W * cg) return;
  const int c8 = (int)(gid % cg) * 8;
  const long pix = gid / cg;
  const int ow = (int)(pix % W), oh = (int)((pix / W) % H);
  const long img = pix / ((long)W * H);
  const int r2 = k2 / 2, r1 = k1 / 2, r0 = k0 / 2;
  float m0[8], m1[8], m2[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) m0[i] = m1[i] = m2[i] = -INFINITY;
  for (int dy = -r2; dy <= r2; ++dy) {
    const int ih = oh + dy;
    if ((unsigned)ih >= (unsigned)H) continue;
    for (int dx = -r2; dx <= r2; ++dx) {
      const int iw = ow + dx;
      if ((unsigned)iw >= (unsigned)W) continue;
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(buf + ((img * H + ih) * W + iw) * ld + c8);
      const bool in1 = dy >= -r1 && dy <= r1 && dx >= -r1 && dx <= r1;
      const bool in0 = dy >= -r0 && dy <= r0 && dx >= -r0 && dx <= r0;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float f = (float)v[i];
        m2[i] = fmaxf(m2[i], f);
        if (in1) m1[i] = fmaxf(m1[i], f);
        if (in0) m0[i] = fmaxf(m0[i], f);
      }
    }
  }
  bf16x8 o0, o1, o2;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    o0[i] = (bf16)m0[i];
    o1[i] = (bf16)m1[i];
    o2[i] = (bf16)m2[i];
  }
  bf16* d = buf + pix * ld + c8;
  *reinterpret_cast<bf16x8*>(d + C) = o0;
  *reinterpret_cast<bf16x8*>(d + 2 * C) = o1;
  *reinterpret_cast<bf16x8*>(d + 3 * C) = o2;
}

// The same three pools from LDS: one workgroup per (image, 64-channel slab) holds the whole map, and
// max_pool(9) = max_pool(5) o max_pool(5), max_pool(13) = max_pool(5)^3 (stride 1, -inf padding: SPPF's identity),
// each pool5 done as a row pass and a column pass.  Maps of up to 400 positions (3 x 50 KB of LDS).
constexpr int SPP_LDS_MAX_HW = 400;
__device__ __forceinline__ bf16x8 max8(bf16x8 a, bf16x8 b) {
  bf16x8 r;
#pragma unroll
  for (int i = 0; i < 8; ++i) r[i] = (bf16)fmaxf((float)a[i], (float)b[i]);
  return r;
}
__global__ void __launch_bounds__(256) spp_lds_kernel(bf16* __restrict__ buf, long ld, int H, int W, int C) {
  extern __shared__ __attribute__((aligned(16))) char sm[];
  const int HW = H * W;
  bf16x8* P = reinterpret_cast<bf16x8*>(sm);          // [HW][8 groups]
  bf16x8* T = P + SPP_LDS_MAX_HW * 8;
  bf16x8* Q = T + SPP_LDS_MAX_HW * 8;
  const long img = blockIdx.x;
  const int c0 = blockIdx.y * 64;
  const int groups = min(8, (C - c0) / 8);
  const int items = HW * 8;
  bf16* base = buf + img * HW * ld + c0;
  for (int it = threadIdx.x; it < items; it += 256) {
    const int px = it >> 3, g = it & 7;
    if (g < groups) P[it] = *reinterpret_cast<const bf16x8*>(base + px * ld + g * 8);
  }
  __syncthreads();
  bf16x8* src = P;
  bf16x8* dst = Q;
  for (int k = 1; k <= 3; ++k) {
    for (int it = threadIdx.x; it < items; it += 256) {  // row pass src -> T
      const int px = it >> 3, g = it & 7, y = px / W, x = px - y * W;
      bf16x8 m = src[it];
#pragma unroll
      for (int d = -2; d <= 2; ++d)
        if (d && (unsigned)(x + d) < (unsigned)W) m = max8(m, src[((y * W) + x + d) * 8 + g]);
      T[it] = m;
    }
    __syncthreads();
    for (int it = threadIdx.x; it < items; it += 256) {  // column pass T -> dst, and out to channel slice k
      const int px = it >> 3, g = it & 7, y = px / W, x = px - y * W;
      bf16x8 m = T[it];
#pragma unroll
      for (int d = -2; d <= 2; ++d)
        if (d && (unsigned)(y + d) < (unsigned)H) m = max8(m, T[(((y + d) * W) + x) * 8 + g]);
      dst[it] = m;
      if (g < groups) *reinterpret_cast<bf16x8*>(base + px * ld + k * C + g * 8) = m;
    }
    __syncthreads();
    bf16x8* t = src;  // the next pool reads this pool's output; the old input buffer is free
    src = dst;
    dst = t;
  }
}

// ------------------------------------------------------------------------------------ ChannelAttention
// per-(image, channel) sums over the H*W pixels, split over `chunks` pixel ranges so a whole map is read by many
// workgroups: grid (image, 256-channel slab, chunk) -> part[image][chunk][C] (summed in a fixed order by the fc
// kernel: deterministic)
__global__ void __launch_bounds__(256) chan_mean_kernel(const bf16* __restrict__ x, long ld, int HW, int C, int chunks,
                                                        float* __restrict__ part) {
  __shared__ float red[256][9];
  const int img = blockIdx.x, slab = blockIdx.y * 256, chunk = blockIdx.z;
  const int per = (HW + chunks - 1) / chunks, p0 = chunk * per, p1 = min(HW, p0 + per);
  const int cw = min(256, C - slab);         // channels in this slab (multiple of 8)
  const int lanes_per_pix = cw / 8, g = threadIdx.x % lanes_per_pix;
  const int pr = threadIdx.x / lanes_per_pix, npr = 256 / lanes_per_pix;  // pixel rows in flight
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (pr < npr)
    for (int p = p0 + pr; p < p1; p += npr) {
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(x + ((long)img * HW + p) * ld + slab + g * 8);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] += (float)v[i];
    }
#pragma unroll
  for (int i = 0; i < 8; ++i) red[threadIdx.x][i] = acc[i];
  __syncthreads();
  if (threadIdx.x < cw) {
    const int c = threadIdx.x, gg = c / 8, ii = c % 8;
    float s = 0.f;
    for (int r = 0; r < npr; ++r) s += red[r * lanes_per_pix + gg][ii];
    part[((long)img * chunks + chunk) * C + slab + c] = s;
  }
}

// a[img][c] = hardsigmoid(b[c] + sum_k Wt[k][c] mean[img][k])  (Wt = fc.weight transposed, f32); mean from the
// chunk partial sums
__global__ void __launch_bounds__(256) chan_attn_fc_kernel(const float* __restrict__ part, int chunks, int HW,
                                                           const float* __restrict__ Wt, const float* __restrict__ b,
                                                           float* __restrict__ att, int C) {
  extern __shared__ float mrow[];
  const int img = blockIdx.y;
  for (int k = threadIdx.x; k < C; k += blockDim.x) {
    float s = 0.f;
    for (int q = 0; q < chunks; ++q) s += part[((long)img * chunks + q) * C + k];
    mrow[k] = s / (float)HW;
  }
  __syncthreads();
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float s = b[c];
  for (int k = 0; k < C; ++k) s = fmaf(Wt[(long)k * C + c], mrow[k], s);
  att[(long)img * C + c] = fminf(fmaxf(s + 3.0f, 0.0f), 6.0f) / 6.0f;  // nn.Hardsigmoid: relu6(x + 3) / 6
}

__global__ void __launch_bounds__(256) chan_scale_kernel(bf16* __restrict__ x, long ld, int HW, int C,
                                                         const float* __restrict__ att, long n_pix) {
  const int cg = C >> 3;
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= n_pix * cg) return;
  const int c8 = (int)(gid % cg) * 8;
  const long pix = gid / cg;
  const long img = pix / HW;
  bf16x8* p = reinterpret_cast<bf16x8*>(x + pix * ld + c8);
  bf16x8 v = *p;
  const float* a = att + img * C + c8;
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = (bf16)((float)v[i] * a[i]);
  *p = v;
}

// ------------------------------------------------------------------------------------ input preparation
using vge::WarpInst;

// onnxpose.preprocess restated in float (no contraction, so the host oracle reproduces every uint8)
__global__ void __launch_bounds__(256) warp_prep_kernel(const uint8_t* __restrict__ frames, int H, int W,
                                                        const WarpInst* __restrict__ inst, int n_inst, int oh, int ow,
                                                        bf16* __restrict__ out) {
#pragma clang fp contract(off)
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (long)n_inst * oh * ow) return;
  const int u = (int)(gid % ow), v = (int)((gid / ow) % oh);
  const int i = (int)(gid / ((long)ow * oh));
  const WarpInst in = inst[i];
  const float sx = in.cx + ((float)u - 0.5f * (float)ow) * in.k;
  const float sy = in.cy + ((float)v - 0.5f * (float)oh) * in.k;
  const float x0f = floorf(sx), y0f = floorf(sy);
  const float fx = sx - x0f, fy = sy - y0f;
  const int x0 = (int)x0f, y0 = (int)y0f;
  const uint8_t* fr = frames + (long)in.frame * H * W * 3;
  const float mean[3] = {123.675f, 116.28f, 103.53f}, stdv[3] = {58.395f, 57.12f, 57.375f};
  bf16x8 o;
#pragma unroll
  for (int c = 0; c < 3; ++c) {  // model channel c = BGR[c] = RGB[2 - c]
    auto px = [&](int yy, int xx) -> float {
      return ((unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W) ? (float)fr[((long)yy * W + xx) * 3 + 2 - c] : 0.f;
    };
    const float top = (1.0f - fx) * px(y0, x0) + fx * px(y0, x0 + 1);
    const float bot = (1.0f - fx) * px(y0 + 1, x0) + fx * px(y0 + 1, x0 + 1);
    const float val = (1.0f - fy) * top + fy * bot;
    const float q = rintf(fminf(fmaxf(val, 0.f), 255.f));
    o[c] = (bf16)((q - mean[c]) / stdv[c]);
  }
#pragma unroll
  for (int c = 3; c < 8; ++c) o[c] = (bf16)0.f;
  *reinterpret_cast<bf16x8*>(out + gid * 8) = o;
}

// onnxdet.preprocess (cv2.resize INTER_LINEAR by r into the top-left of a 114-filled S x S canvas, BGR,
// uint8 values) + YOLOX Focus (channels: [::2, ::2], [1::2, ::2], [::2, 1::2], [1::2, 1::2], 3 each) ->
// NHWC bf16 [F][S/2][S/2][16] (12 used).  cv2.resize maps dst x to src (x + 0.5) / r - 0.5, clamped.
__global__ void __launch_bounds__(256) letterbox_focus_kernel(const uint8_t* __restrict__ frames, int n, int H, int W,
                                                              int S, int rh, int rw, float inv_rx, float inv_ry,
                                                              bf16* __restrict__ out) {
#pragma clang fp contract(off)
  const int S2 = S / 2;
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (long)n * S2 * S2) return;
  const int u = (int)(gid % S2), v = (int)((gid / S2) % S2);
  const int f = (int)(gid / ((long)S2 * S2));
  const uint8_t* fr = frames + (long)f * H * W * 3;
  bf16 o[16];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int dy = q & 1, dx = q >> 1;  // Focus order: (0,0), (1,0), (0,1), (1,1) as (row, col) parity
    const int yy = 2 * v + dy, xx = 2 * u + dx;
    float val[3] = {114.f, 114.f, 114.f};
    if (yy < rh && xx < rw) {
      float sx = ((float)xx + 0.5f) * inv_rx - 0.5f, sy = ((float)yy + 0.5f) * inv_ry - 0.5f;
      sx = fmaxf(sx, 0.f);
      sy = fmaxf(sy, 0.f);
      int x0 = (int)floorf(sx), y0 = (int)floorf(sy);
      float fx = sx - (float)x0, fy = sy - (float)y0;
      if (x0 >= W - 1) { x0 = W - 1; fx = 0.f; }
      if (y0 >= H - 1) { y0 = H - 1; fy = 0.f; }
      const int x1 = min(x0 + 1, W - 1), y1 = min(y0 + 1, H - 1);
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float p00 = fr[((long)y0 * W + x0) * 3 + 2 - c], p01 = fr[((long)y0 * W + x1) * 3 + 2 - c];
        const float p10 = fr[((long)y1 * W + x0) * 3 + 2 - c], p11 = fr[((long)y1 * W + x1) * 3 + 2 - c];
        const float top = (1.0f - fx) * p00 + fx * p01, bot = (1.0f - fx) * p10 + fx * p11;
        val[c] = rintf(fminf(fmaxf((1.0f - fy) * top + fy * bot, 0.f), 255.f));
      }
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) o[q * 3 + c] = (bf16)val[c];
  }
#pragma unroll
  for (int c = 12; c < 16; ++c) o[c] = (bf16)0.f;
  bf16x8* d = reinterpret_cast<bf16x8*>(out + gid * 16);
  bf16x8 lo, hi;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    lo[i] = o[i];
    hi[i] = o[8 + i];
  }
  d[0] = lo;
  d[1] = hi;
}

// nearest 2x upsample (F.interpolate(scale_factor=2, mode="nearest")) of an NHWC slice into a wider buffer
__global__ void __launch_bounds__(256) upsample2x_kernel(const bf16* __restrict__ x, long ldx, bf16* __restrict__ y,
                                                         long ldy, int n_img, int H, int W, int C) {
  const int cg = C >> 3;
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (long)n_img * 4 * H * W * cg) return;
  const int c8 = (int)(gid % cg) * 8;
  const long pix = gid / cg;  // output pixel
  const int ow = (int)(pix % (2 * W)), oh = (int)((pix / (2 * W)) % (2 * H));
  const long img = pix / (4L * W * H);
  *reinterpret_cast<bf16x8*>(y + pix * ldy + c8) =
      *reinterpret_cast<const bf16x8*>(x + ((img * H + (oh >> 1)) * W + (ow >> 1)) * ldx + c8);
}

}  // namespace

// ------------------------------------------------------------------------------------ launchers
namespace vge {

static int ilog2(int v) {
  int l = 0;
  while ((1 << l) < v) ++l;
  return l;
}

static int g_conv_persist = -1;  // VGE_CONV_PERSIST=0: one tile per workgroup (conv2_bf16_kernel, A/B timing)

static int persistent_grid(int ntiles) {  // one workgroup per CU, a multiple of 8 (whole XCDs)
  static int cus = 0;
  if (cus == 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      n = 256;
    cus = std::max(8, n / 8 * 8);
  }
  return ntiles <= cus ? ntiles : cus;
}

template <int BN, int ACT, int OUT, int RES, int BM = C2_M>
static hipError_t conv2p_go(const ConvArgs& a, hipStream_t s) {
  constexpr int BYTES = C2Cfg<BN, BM>::RING;
  static LdsAttrOnce attr;
  if (const hipError_t e = attr(reinterpret_cast<const void*>(&conv2p_bf16_kernel<BN, ACT, OUT, RES, BM>), BYTES); e != hipSuccess) return e;
  const int ntiles = ((a.M + BM - 1) / BM) * ((a.Cout + BN - 1) / BN);
  const int grid = g_conv_persist == 2 ? ntiles : persistent_grid(ntiles);  // 2: A/B of the schedule alone
  hipLaunchKernelGGL((conv2p_bf16_kernel<BN, ACT, OUT, RES, BM>), dim3(grid), dim3(512), BYTES, s, a);
  return hipGetLastError();
}

// pmode: -1 = VGE_CONV_PERSIST (default on), 0 = one tile per workgroup, 1 = persistent
template <int BN, int ACT, int OUT, int RES>
static hipError_t conv2_go(const ConvArgs& a, hipStream_t s, int pmode) {
  if (g_conv_persist < 0) {
    const char* e = getenv("VGE_CONV_PERSIST");
    g_conv_persist = (e && atoi(e) == 0) ? 0 : 1;
  }
  if (pmode == 7) {  // the 16x16x32 form (variant 12)
    if constexpr (C2Cfg<BN>::TM % 2 == 0) {
      constexpr int BYTES = C2Cfg<BN>::LDS;
      static LdsAttrOnce attr;
      if (const hipError_t e = attr(reinterpret_cast<const void*>(&conv2_bf16_kernel<BN, ACT, OUT, RES, 1>), BYTES);
          e != hipSuccess)
        return e;
      const int grid = ((a.M + C2_M - 1) / C2_M) * ((a.Cout + BN - 1) / BN);
      hipLaunchKernelGGL((conv2_bf16_kernel<BN, ACT, OUT, RES, 1>), dim3(grid), dim3(512), BYTES, s, a);
      return hipGetLastError();
    }
    return hipErrorInvalidValue;
  }
  if constexpr (RES == RES_NONE)  // residual epilogues stay on conv2_bf16_kernel (their loads need vmcnt drains)
    if (pmode < 0 ? g_conv_persist : pmode) return conv2p_go<BN, ACT, OUT, RES>(a, s);
  constexpr int BYTES = C2Cfg<BN>::LDS;
  static LdsAttrOnce attr;
  if (const hipError_t e = attr(reinterpret_cast<const void*>(&conv2_bf16_kernel<BN, ACT, OUT, RES>), BYTES); e != hipSuccess) return e;
  const int grid = ((a.M + C2_M - 1) / C2_M) * ((a.Cout + BN - 1) / BN);
  hipLaunchKernelGGL((conv2_bf16_kernel<BN, ACT, OUT, RES>), dim3(grid), dim3(512), BYTES, s, a);
  return hipGetLastError();
}

static int g_conv_v1 = -1;  // VGE_CONV_V1=1: every layer on the 128-row kernel (A/B timing)
static int g_conv_force = 0;  // vge_debug_set_conv_variant(v): untuned launches (variant 0) take variant v (tests, A/B)
static int g_conv_tall = 0;  // vge_debug_set_conv_tall(1): 256-row tiles for the 64 / 128-column layers (A/B timing)

template <int TN, int ACT, int OUT, int RES, int BM>
static hipError_t conv1_go(const ConvArgs& a, int grid, hipStream_t s) {
  constexpr int LDS = CV_ST * (BM * CV_K * 2 + TN * CV_K * 2);
  constexpr int EPI = 64 * (TN + 4) * 4;
  constexpr int BYTES = LDS > EPI ? LDS : EPI;
  static LdsAttrOnce attr;
  if (const hipError_t e = attr(reinterpret_cast<const void*>(&conv_bf16_kernel<TN, ACT, OUT, RES, BM>), BYTES); e != hipSuccess) return e;
  hipLaunchKernelGGL((conv_bf16_kernel<TN, ACT, OUT, RES, BM>), dim3(grid), dim3(256), BYTES, s, a);
  return hipGetLastError();
}

template <int TN, int ACT, int OUT, int RES>
static hipError_t conv_go(const ConvArgs& a, int grid, hipStream_t s, int pmode) {
  if (g_conv_v1 < 0) {
    const char* e = getenv("VGE_CONV_V1");
    g_conv_v1 = (e && atoi(e) == 1) ? 1 : 0;
  }
  if constexpr (TN == 256) {
    return g_conv_v1 && pmode < 0 ? conv_go<128, ACT, OUT, RES>(a, grid, s, pmode) : conv2_go<256, ACT, OUT, RES>(a, s, pmode);
  } else if (pmode == 5) {  // 256-row ("tall") tiles
    return conv1_go<TN, ACT, OUT, RES, 256>(a, ((a.M + 255) / 256) * ((a.Cout + TN - 1) / TN), s);
  } else if (pmode == 6) {  // 512 x 128 tiles on the persistent grid
    if constexpr (TN == 128) return conv2p_go<128, ACT, OUT, RES, 512>(a, s);
    return hipErrorInvalidValue;
  } else {
    return conv1_go<TN, ACT, OUT, RES, CV_M>(a, grid, s);
  }
}

// variant 9: a 1x1 stride-1 conv as the bf16 GEMM of vge_vit.hip (out = act(x W^T + b (+ bf16 residual before the
// activation))), for the shapes that kernel takes; -1 = not applicable
int conv_gemm_epi(const ConvLaunch& c) {
  if (c.KH != 1 || c.KW != 1 || c.stride != 1 || c.pad != 0 || c.gslice || c.out_f32 || c.Cout % 256 ||
      c.Cin % 64 || c.Kp != c.Cin || c.ldx % 8 || c.ldo % 4)
    return -1;
  if (c.res_mode == RES_NONE) return c.act == ACT_NONE ? GEMM_BF16 : c.act == ACT_RELU ? GEMM_RELU_BF16 : -1;
  if (c.ldr % 4) return -1;
  // (residual after a ReLU is not the same as before it; with no activation both orders agree)
  if (c.res_mode == RES_BF16_PRE) return c.act == ACT_NONE ? GEMM_RESB_BF16 : c.act == ACT_RELU ? GEMM_RESB_RELU_BF16 : -1;
  if (c.res_mode == RES_BF16 && c.act == ACT_NONE) return GEMM_RESB_BF16;
  return -1;
}

// the library GEMM path (variant 11, vge_blaslt.cpp) for a 1x1 stride-1 conv: any Cin / Cout (16-B rows), the epilogues
// a library epilogue expresses (bias; + ReLU or SiLU; a bf16 residual before the ReLU or with no activation); -1 = no
int conv_lib_epi(const ConvLaunch& c) {
  if (c.KH != 1 || c.KW != 1 || c.stride != 1 || c.pad != 0 || c.gslice || c.out_f32 || c.Cout % 8 || c.Cin % 8 ||
      c.Kp < c.Cin || c.Kp % 8 || c.ldx % 8 || c.ldo % 8)
    return -1;
  if (c.res_mode == RES_NONE)
    return c.act == ACT_NONE ? GEMM_BF16 : c.act == ACT_RELU ? GEMM_RELU_BF16 : c.act == ACT_SILU ? GEMM_SILU_BF16 : -1;
  if (c.ldr % 8) return -1;
  if (c.res_mode == RES_BF16_PRE) return c.act == ACT_NONE ? GEMM_RESB_BF16 : c.act == ACT_RELU ? GEMM_RESB_RELU_BF16 : -1;
  if (c.res_mode == RES_BF16 && c.act == ACT_NONE) return GEMM_RESB_BF16;
  return -1;
}

bool conv_gemm_persist_ok(const ConvLaunch& c) {
  const int epi = conv_gemm_epi(c);
  if (epi < 0) return false;
  GemmBf16 g{};
  g.lda = c.ldx;
  g.ldw = c.Kp;
  g.ldo = c.ldo;
  g.bias = c.bias;
  g.M = c.n_img * ((c.H + 2 * c.pad - c.KH) / c.stride + 1) * ((c.W + 2 * c.pad - c.KW) / c.stride + 1);
  g.N = c.Cout;
  g.K = c.Cin;
  return gemm_persist_ok(epi, g);
}

hipError_t launch_conv_bf16(const ConvLaunch& c, hipStream_t s) {
  ConvArgs a;
  a.x = static_cast<const bf16*>(c.x);
  a.w = static_cast<const bf16*>(c.w);
  a.bias = c.bias;
  a.out = c.out;
  a.res = c.res;
  a.rscale = c.rscale;
  a.zero = static_cast<const bf16*>(c.zero);
  a.ldx = c.ldx;
  a.ldo = c.ldo;
  a.ldr = c.ldr;
  a.H = c.H;
  a.W = c.W;
  a.cin_log2 = ilog2(c.Cin);
  a.Ho = (c.H + 2 * c.pad - c.KH) / c.stride + 1;
  a.Wo = (c.W + 2 * c.pad - c.KW) / c.stride + 1;
  a.KW = c.KW;
  a.kw_magic = (65536 + c.KW - 1) / c.KW;
  a.stride = c.stride;
  a.pad = c.pad;
  a.taps = c.KH * c.KW;
  a.Kp = c.Kp;
  a.Cout = c.Cout;
  a.M = c.n_img * a.Ho * a.Wo;
  a.gslice = c.gslice;
  int tn = c.tn, pmode = -1;
  int variant = c.variant == 0 && g_conv_force > 0 && !c.gslice ? g_conv_force : c.variant;
  if (variant == 11) {  // the library GEMM (vge_blaslt.cpp; conv_tuned_launch's choice for the shapes it takes)
    const int epi = conv_lib_epi(c);
    if (epi >= 0) {
      GemmBf16 g{};
      g.A = c.x;
      g.lda = c.ldx;
      g.W = c.w;
      g.ldw = c.Kp;
      g.out = c.out;
      g.ldo = c.ldo;
      g.bias = c.bias;
      g.ldr = c.ldr;
      g.resb = c.res;
      g.M = a.M;
      g.N = c.Cout;
      g.K = c.Cin;
      const hipError_t e = launch_gemm_lib(epi, g, s);
      if (e != hipErrorNotSupported) return e;
    }
    variant = 9;  // not on the library path: the GEMM kernel where it applies, else the default below
  }
  if (variant == 9 || variant == 10) {  // the GEMM kernel (tuner candidates, or forced by vge_debug_set_conv_variant)
    const int epi = conv_gemm_epi(c);
    if (epi >= 0) {
      GemmBf16 g{};
      g.A = c.x;
      g.lda = c.ldx;
      g.W = c.w;
      g.ldw = c.Kp;
      g.out = c.out;
      g.ldo = c.ldo;
      g.bias = c.bias;
      g.ldr = c.ldr;
      g.resb = c.res;
      g.M = a.M;
      g.N = c.Cout;
      g.K = c.Cin;
      if (variant == 10) {  // its persistent form (one workgroup per CU, the epilogue under the next tile's loads)
        if (gemm_persist_ok(epi, g)) return launch_gemm_bf16_persistent(epi, g, s);
        if (c.variant == 10) return hipErrorInvalidValue;
      }
      return launch_gemm_bf16(epi, g, s);
    }
    if (c.variant == 9 || c.variant == 10) return hipErrorInvalidValue;
    variant = 0;  // forced globally (or the library's fallback): layers the GEMM cannot take keep the default kernel
  }
  // grouped slices run on the 128- / 256-row kernel only, with the slice width as the column tile
  if (c.gslice && (variant == 2 || variant == 3 || variant == 6 || variant == 12 || (c.tn != 64 && c.tn != 128) || c.Cin != c.tn ||
                   c.Cout % c.tn))
    return hipErrorInvalidValue;
  if (variant == 6) {  // 512 x 128 persistent tiles
    tn = 128;
    pmode = 6;
  }
  if (variant == 1 || variant == 5) tn = tn > 128 ? 128 : tn;
  if (variant == 5 || (variant == 0 && g_conv_tall && tn < 256)) pmode = 5;  // 256-row tiles, 64 / 128 columns
  if (variant == 2 || variant == 3 || variant == 12) {
    if (c.Npad % 256) return hipErrorInvalidValue;
    tn = 256;
    pmode = variant == 3 ? 1 : variant == 12 ? 7 : 0;
  }
  const int tn1 = tn > 128 ? 128 : tn;  // v1 grid (the tn 256 case runs conv2 with its own grid)
  const int grid = ((a.M + CV_M - 1) / CV_M) * ((c.Cout + tn1 - 1) / tn1);
  if (a.M <= 0) return hipSuccess;
#define VGE_CONV_CASE(ACT, OUT, RES)                                                              \
  if (c.act == ACT && c.out_f32 == OUT && c.res_mode == RES)                                      \
    return tn == 64 ? conv_go<64, ACT, OUT, RES>(a, grid, s, pmode)                               \
                    : tn == 128 ? conv_go<128, ACT, OUT, RES>(a, grid, s, pmode)                  \
                                : conv_go<256, ACT, OUT, RES>(a, grid, s, pmode);
  if (tn != 64 && tn != 128 && tn != 256) return hipErrorInvalidValue;
  VGE_CONV_CASE(ACT_SILU, OUT_BF16, RES_NONE)
  VGE_CONV_CASE(ACT_SILU, OUT_BF16, RES_BF16)
  VGE_CONV_CASE(ACT_NONE, OUT_BF16, RES_NONE)
  VGE_CONV_CASE(ACT_NONE, OUT_BF16, RES_F32S)
  VGE_CONV_CASE(ACT_NONE, OUT_F32, RES_NONE)
  VGE_CONV_CASE(ACT_SILU, OUT_F32, RES_NONE)
  VGE_CONV_CASE(ACT_SIGMOID, OUT_F32, RES_NONE)
  VGE_CONV_CASE(ACT_RELU, OUT_BF16, RES_NONE)       // Faster R-CNN: conv + FrozenBN + ReLU, RPN conv, box head fc
  VGE_CONV_CASE(ACT_RELU, OUT_BF16, RES_BF16_PRE)   // bottleneck conv3: relu(conv + shortcut)
  VGE_CONV_CASE(ACT_NONE, OUT_BF16, RES_BF16)       // FPN lateral + top-down sum
#undef VGE_CONV_CASE
  return hipErrorInvalidValue;
}

hipError_t launch_dwconv(const void* x, long ldx, const float* w, const float* b, void* y, long ldy, int n_img, int H,
                         int W, int C, int K, hipStream_t s) {
  const long n = (long)n_img * H * W * (C / 8);
  if (n == 0) return hipSuccess;
  const int grid = (int)((n + 255) / 256);
  if (K == 5) {
    constexpr int RB = 32;  // output rows per thread: the 25 weight vectors a thread loads serve 32 outputs
    const long nt = (long)n_img * ((H + RB - 1) / RB) * W * (C / 4);
    hipLaunchKernelGGL(dwconv5_rb_kernel<RB>, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, s,
                       static_cast<const bf16*>(x), ldx, w, b, static_cast<bf16*>(y), ldy, n_img, H, W, C);
  } else if (K == 55)  // the one-thread-per-output form (kept for A/B timing)
    hipLaunchKernelGGL(dwconv_kernel<5>, dim3(grid), dim3(256), 0, s, static_cast<const bf16*>(x), ldx, w, b,
                       static_cast<bf16*>(y), ldy, n_img, H, W, C);
  else if (K == 3)
    hipLaunchKernelGGL(dwconv_kernel<3>, dim3(grid), dim3(256), 0, s, static_cast<const bf16*>(x), ldx, w, b,
                       static_cast<bf16*>(y), ldy, n_img, H, W, C);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_spp_pool(void* buf, long ld, int n_img, int H, int W, int C, int k0, int k1, int k2, hipStream_t s) {
  const long n = (long)n_img * H * W * (C / 8);
  if (n == 0) return hipSuccess;
  if (k0 == 5 && k1 == 9 && k2 == 13 && H * W <= SPP_LDS_MAX_HW) {
    static LdsAttrOnce attr;
    const int bytes = 3 * SPP_LDS_MAX_HW * 8 * 16;
    if (const hipError_t e = attr(reinterpret_cast<const void*>(&spp_lds_kernel), bytes); e != hipSuccess) return e;
    hipLaunchKernelGGL(spp_lds_kernel, dim3(n_img, (C + 63) / 64), dim3(256), bytes, s, static_cast<bf16*>(buf), ld, H,
                       W, C);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(spp_pool_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, static_cast<bf16*>(buf), ld,
                     n_img, H, W, C, k0, k1, k2);
  return hipGetLastError();
}

hipError_t launch_chan_attn(void* x, long ld, int n_img, int HW, int C, const float* Wt, const float* b, float* mean,
                            float* att, hipStream_t s) {
  if (n_img == 0) return hipSuccess;
  // `mean` holds n_img x 2048 floats (vge_dwpose_reserve): pixel chunks of >= 512 within that budget
  const int chunks = std::max(1, std::min((HW + 511) / 512, 2048 / C));
  hipLaunchKernelGGL(chan_mean_kernel, dim3(n_img, (C + 255) / 256, chunks), dim3(256), 0, s,
                     static_cast<const bf16*>(x), ld, HW, C, chunks, mean);
  hipLaunchKernelGGL(chan_attn_fc_kernel, dim3((C + 255) / 256, n_img), dim3(256), C * sizeof(float), s, mean, chunks,
                     HW, Wt, b, att, C);
  const long n = (long)n_img * HW * (C / 8);
  hipLaunchKernelGGL(chan_scale_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, static_cast<bf16*>(x), ld,
                     HW, C, att, (long)n_img * HW);
  return hipGetLastError();
}

hipError_t launch_warp_prep(const uint8_t* frames, int H, int W, const void* inst, int n_inst, int oh, int ow, void* out,
                            hipStream_t s) {
  const long n = (long)n_inst * oh * ow;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(warp_prep_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, frames, H, W,
                     static_cast<const WarpInst*>(inst), n_inst, oh, ow, static_cast<bf16*>(out));
  return hipGetLastError();
}

hipError_t launch_letterbox_focus(const uint8_t* frames, int n, int H, int W, int S, int rh, int rw, float inv_rx,
                                  float inv_ry, void* out, hipStream_t s) {
  const long tot = (long)n * (S / 2) * (S / 2);
  if (tot == 0) return hipSuccess;
  hipLaunchKernelGGL(letterbox_focus_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, frames, n, H, W, S,
                     rh, rw, inv_rx, inv_ry, static_cast<bf16*>(out));
  return hipGetLastError();
}

hipError_t launch_upsample2x(const void* x, long ldx, void* y, long ldy, int n_img, int H, int W, int C, hipStream_t s) {
  const long tot = (long)n_img * 4 * H * W * (C / 8);
  if (tot == 0) return hipSuccess;
  hipLaunchKernelGGL(upsample2x_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, static_cast<const bf16*>(x),
                     ldx, static_cast<bf16*>(y), ldy, n_img, H, W, C);
  return hipGetLastError();
}

}  // namespace vge

extern "C" int vge_debug_set_conv_v1(int on) {  // A/B timing (tools/conv_bench.py)
  vge::g_conv_v1 = on ? 1 : 0;
  return 0;
}

extern "C" int vge_debug_set_conv_tall(int on) {  // A/B timing (tools/conv_bench.py)
  vge::g_conv_tall = on ? 1 : 0;
  return 0;
}

extern "C" int vge_debug_set_conv_variant(int v) {  // tests / A/B: untuned launches take variant v (0 = default)
  const int prev = vge::g_conv_force;
  vge::g_conv_force = v;
  return prev;
}

extern "C" int vge_debug_set_conv_persist(int mode) {  // A/B timing (tools/conv_bench.py): 0 off, 1 on, 2 one tile each
  vge::g_conv_persist = mode;
  return 0;
}
