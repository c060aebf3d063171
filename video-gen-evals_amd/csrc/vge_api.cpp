// C ABI of libvge.so (include/vge.h): argument checking, weight repacking into the MFMA panel layout,
// workspace management and the launch sequences.  No exception crosses the ABI.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <string>
#include <unordered_map>
#include <vector>
#include <memory>
#include <thread>
#include <atomic>

#include "../../include/vge.h"

namespace vge {
// launchers (vge_featurize.hip / vge_encoder.hip / vge_score.hip)
hipError_t launch_featurize_tiles(const float*, const float*, const float*, const float*, const float*, const int*,
                                  const void*, const int*, int, const float*, const float*, float*, int, hipStream_t);
hipError_t launch_stats_colsum(const float*, const void*, int, int, int, double*, double*, hipStream_t);
hipError_t launch_stats_finalize(const double*, long long, long long, float*, float*, int, hipStream_t);
struct EncDescHost {
  const float* stem; const float* conv; const float* proj; const float* gn_w; const float* gn_b;
  int in_col, d_in, n_stem_panels, ld;
};
struct FuseParamsHost {
  const float* kv_w; const float* kv_b; const float* u;
  float inv_tau[8]; float bias[8]; int n_mod; int has_motion[8];
};
struct GemmArgsHost {
  const float* A; int lda; const float* W; float* out; int ldo; int M, K, N;
  const float* bias; const float* res; int ldr; const float* ln_w; const float* ln_b; const float* pe; const float* cls;
};
hipError_t encoder_kernel_setup();
hipError_t encoder_x3_kernel_setup();
hipError_t launch_pack_x3(const float* W, int N, int K_real, int ldk, int conv, int nch, int* sh, float* cs, int* bad,
                          _Float16* out, hipStream_t s);
struct EncDescX3Host {
  const _Float16* stem; const _Float16* conv; const _Float16* proj; const float* gn_w; const float* gn_b;
  const float* cs; const float* fold;
  int in_col, d_in, n_stem_panels, ld;
  float gn_gmax[4], gn_bmax[4];  // max |gamma|, max |beta| per GroupNorm
};
struct GemmArgsX3Host {
  const float* A; int lda; const _Float16* W; float* out; int ldo; int M, K, N;
  const float* bias; const float* res; int ldr; const float* ln_w; const float* ln_b; const float* pe; const float* cls;
  const float* cs;
};
hipError_t launch_conv_encoders_x3(const float*, int, const void*, int, unsigned, float*, bool, bool, hipStream_t);
hipError_t encoder_x3s_kernel_setup();
hipError_t launch_conv_encoders_x3s(const float*, int, const void*, int, unsigned, float*, int*, bool, hipStream_t);

bool conv_f16w_plan(int n_windows, int n_enc, int wmax, int& G, int& R, int& U);
hipError_t launch_conv_f16w_table(int n_windows, int n_enc, int G, int R, int U, int* d_table, hipStream_t s);
hipError_t launch_conv_encoders_f16w(const float*, int, const void*, float*, const int*, int, int, hipStream_t);
hipError_t launch_gemm_x3(int, const GemmArgsX3Host&, hipStream_t);
struct FfnArgsX3Host {
  const float* X1; float* out; int M;
  const _Float16* W1; const float* cs1; const float* b1;
  const _Float16* W2; const float* cs2; const float* b2;
  const float* ln_w; const float* ln_b;
};
hipError_t launch_ffn_x3(const FfnArgsX3Host&, hipStream_t);
struct TxLayerX3Host {  // vge_transformer_x3.hip
  const _Float16* in_w;  const float* in_cs; const float* in_b;
  const _Float16* out_w; const float* out_cs; const float* out_b;
  const float* n1_w; const float* n1_b;
  const _Float16* l1_w; const float* l1_cs; const float* l1_b;
  const _Float16* l2_w; const float* l2_cs; const float* l2_b;
  const float* n2_w; const float* n2_b;
  int e_x1, e_x2, e_h, pad;  // static split exponents of LN1 / LN2 outputs and of the FFN hidden
};
struct TxArgsX3Host {
  const float* pooled; int n_windows, n_layers;
  const _Float16* ov_w; const float* ov_cs;
  const float* cls; const float* pe;
  const TxLayerX3Host* layers;  // host array [n_layers], n_layers <= 8 (passed as kernel arguments)
  float* seq; float* frame; float* tc;
};
hipError_t transformer_x3_kernel_setup();
hipError_t launch_transformer_x3(const TxArgsX3Host&, int, hipStream_t);
hipError_t launch_conv_encoders(const float*, int, const void*, int, float*, hipStream_t);
hipError_t launch_fuse(const float*, int, const FuseParamsHost&, float*, hipStream_t);
hipError_t launch_gemm(int, const GemmArgsHost&, hipStream_t);
hipError_t launch_attn(const float*, int, float*, hipStream_t);
hipError_t launch_embed_tc(const float*, int, float*, float*, float*, hipStream_t);
// the generic-shape exact-f32 path (vge_encoder_gen.hip)
struct GenFuseHost {
  const float* kv_w; const float* kv_b; const float* u;
  float inv_tau[8], bias[8];
  int n_mod, d;
  int has_motion[8];
};
hipError_t launch_gen_conv(const float* x, int ldx, int xcol, int cin, const float* W, int cout, int taps, int dil, int epi,
                           const float* res, float* out, int n_windows, hipStream_t s);
hipError_t launch_gen_groupnorm(float* x, int n_windows, int d, const float* g, const float* b, hipStream_t s);
hipError_t launch_gen_fuse(const float* enc_out, int n_rows, const GenFuseHost& f, float* pooled_pre, hipStream_t s);
hipError_t launch_gen_gemm(const float* A, int lda, const float* W, int M, int N, int K, const float* bias, int epi,
                           const float* res, const float* pe, const float* cls, float* out, int ldo, hipStream_t s);
hipError_t launch_gen_attn(const float* qkv, int n_windows, int d, int heads, float* out, hipStream_t s);
hipError_t launch_gen_add_ln(const float* a, const float* b, int rows, int d, const float* g, const float* be, float* out,
                             hipStream_t s);
hipError_t launch_gen_embed_tc(const float* x, int n_windows, int d, float* seq, float* frame, float* tc, hipStream_t s);
hipError_t launch_centroid_accum(const float*, const int*, int, int, int, float*, float*, hipStream_t);
hipError_t launch_centroid_final(const float*, const float*, int, int, float*, hipStream_t);
hipError_t launch_tc_windows(const float*, int, int, int, float*, hipStream_t);
hipError_t launch_score_videos(const float*, const float*, const int*, const int*, const float*, int, int, float*,
                               double*, hipStream_t);
enum { EPI_TOKENS = 0, EPI_BIAS = 1, EPI_BIAS_RELU = 2, EPI_BIAS_RES_LN = 3 };
}  // namespace vge

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIPCHK(expr)                                                                         \
  do {                                                                                       \
    hipError_t _e = (expr);                                                                  \
    if (_e != hipSuccess) return fail(VGE_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

hipStream_t S(vge_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

const char* kMods[5] = {"vit", "global", "pose", "beta", "kp2d"};
const int kDimsRaw[5] = {1024, 9, 207, 10, 120};
const int kDimsDiff[5] = {1024, 3, 69, 10, 120};
constexpr int CHUNK_F = 4096;

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Pack W[N][K] (row-major, K_real valid columns, row stride ldk) into [N/256][P][16][4096] chunks:
// chunk(nb, p, c)[(g*256 + n)*4 + q] = W[nb*256 + n][p*256 + 64g + 4c + q]
void pack_linear(const float* W, int N, int K_real, int ldk, int P, std::vector<float>& out) {
  const size_t base = out.size();
  out.resize(base + (size_t)(N / 256) * P * 16 * CHUNK_F, 0.f);
  float* o = out.data() + base;
  for (int nb = 0; nb < N / 256; ++nb)
    for (int p = 0; p < P; ++p)
      for (int c = 0; c < 16; ++c) {
        float* ch = o + (((size_t)nb * P + p) * 16 + c) * CHUNK_F;
        for (int g = 0; g < 4; ++g)
          for (int n = 0; n < 256; ++n)
            for (int q = 0; q < 4; ++q) {
              const int k = p * 256 + 64 * g + 4 * c + q;
              ch[(g * 256 + n) * 4 + q] = (k < K_real) ? W[(size_t)(nb * 256 + n) * ldk + k] : 0.f;
            }
      }
}

// Conv1d weight [256][256][5] -> 5 taps x 16 chunks: chunk(tap, c)[(g*256+n)*4+q] = W[n][64g+4c+q][tap]
void pack_conv(const float* W, std::vector<float>& out) {
  const size_t base = out.size();
  out.resize(base + (size_t)5 * 16 * CHUNK_F, 0.f);
  float* o = out.data() + base;
  for (int tap = 0; tap < 5; ++tap)
    for (int c = 0; c < 16; ++c) {
      float* ch = o + ((size_t)tap * 16 + c) * CHUNK_F;
      for (int g = 0; g < 4; ++g)
        for (int n = 0; n < 256; ++n)
          for (int q = 0; q < 4; ++q) {
            const int ci = 64 * g + 4 * c + q;
            ch[(g * 256 + n) * 4 + q] = W[((size_t)n * 256 + ci) * 5 + tap];
          }
    }
}

// 3xfp16 image: W[N][K] -> chunks [N/256][ceil(K/16)][plane 2][h 2][n 256][8] fp16 of w' = w * 2^s_n, the
// power-of-two column scale s_n bringing column n's largest |w| into [2^8, 2^9); plane 0 = hi = f16(w'),
// plane 1 = lo = f16(w' - hi) (an fp16 residual, subnormals kept by the MFMA); chunk c covers
// k = 16c + 8h + j (zero past K_real).  cs receives 2^-s_n per column (the kernels' epilogue factor).
// host twin of fp16_range_exp (vge_x3.h): 2^-e brings m into [2^8, 2^9)
int range_exp(double m) {
  if (!(m > 0.0) || !(m <= 3.0e38)) return 0;
  return std::max(std::ilogb(m) - 8, -100);
}

// run f(i) for i in [0, n) on up to hardware_concurrency host threads (weight packing at load time)
template <class F>
void parallel_for(int n, F f) {
  const int nt = std::max(1, std::min<int>(n, (int)std::thread::hardware_concurrency()));
  if (nt <= 1 || n < 4) {
    for (int i = 0; i < n; ++i) f(i);
    return;
  }
  std::vector<std::thread> th;
  std::atomic<int> next{0};
  for (int t = 0; t < std::min(nt, 32); ++t)
    th.emplace_back([&] {
      for (int i = next++; i < n; i = next++) f(i);
    });
  for (auto& x : th) x.join();
}

template <class Get>
void pack_linear_x3(Get W, int N, int K_real, std::vector<_Float16>& out, std::vector<float>& cs, int chunk_mult = 1) {
  const int nch = ((K_real + 15) / 16 + chunk_mult - 1) / chunk_mult * chunk_mult;  // streams run in groups of chunk_mult
  std::vector<int> sh(N);
  parallel_for(N, [&](int n) {
    float m = 0.f;
    for (int k = 0; k < K_real; ++k) m = std::max(m, std::fabs(W(n, k)));
    sh[n] = (m > 0.f) ? std::min(8 - std::ilogb(m), 100) : 0;
  });
  for (int n = 0; n < N; ++n) cs.push_back(std::ldexp(1.0f, -sh[n]));
  const size_t base = out.size();
  out.resize(base + (size_t)(N / 256) * nch * 8192, (_Float16)0.0f);
  _Float16* o = out.data() + base;
  parallel_for((N / 256) * nch, [&](int idx) {
    const int nb = idx / nch, c = idx % nch;
    {
      _Float16* ch = o + ((size_t)nb * nch + c) * 8192;
      for (int h = 0; h < 2; ++h)
        for (int n = 0; n < 256; ++n)
          for (int j = 0; j < 8; ++j) {
            const int k = 16 * c + 8 * h + j;
            const float w = (k < K_real) ? std::ldexp(W(nb * 256 + n, k), sh[nb * 256 + n]) : 0.0f;
            const _Float16 hi = (_Float16)w;
            const _Float16 lo = (_Float16)(w - (float)hi);
            ch[((0 * 2 + h) * 256 + n) * 8 + j] = hi;
            ch[((1 * 2 + h) * 256 + n) * 8 + j] = lo;
          }
    }
  });
}

}  // namespace

// A checkpoint whose d_model / time_heads differ from the tiled kernels' 256 / 8 (load_model reads both from the
// checkpoint, eval.py:139-158): the exact-f32 VALU kernels of vge_encoder_gen.hip, reference weights as they are.
struct GenModel {
  int d = 0, heads = 0, layers = 0, ffn = 0, M = 0;
  float* wbuf = nullptr;
  struct Enc {
    const float *stem, *conv[8], *proj, *gw[4], *gb[4];
    int in_col, d_in;
  };
  std::vector<Enc> encs;
  vge::GenFuseHost fuse{};
  const float *Wov = nullptr, *cls = nullptr, *pe = nullptr;
  struct Lyr {
    const float *in_w, *in_b, *out_w, *out_b, *n1w, *n1b, *l1w, *l1b, *l2w, *l2b, *n2w, *n2b;
  };
  std::vector<Lyr> L;
  int cap = 0;
  float* ws = nullptr;
  float *enc_out = nullptr, *a = nullptr, *b = nullptr, *c = nullptr, *pp = nullptr, *x = nullptr, *qkv = nullptr,
        *att = nullptr, *x1 = nullptr, *h = nullptr, *tmp = nullptr;
  ~GenModel() {
    if (wbuf) (void)hipFree(wbuf);
    if (ws) (void)hipFree(ws);
  }
};

struct vge_encoder {
  GenModel* gen = nullptr;  // set: every stage on the generic-shape exact-f32 kernels
  int mode = VGE_F32;
  int n_layers = 4;
  int n_mod = 5, n_enc = 10;     // modalities (5, or 4 keypoint-less) and conv encoders (state + motion)
  int feat_dim = VGE_FEAT_DIM;   // feats row width of this model's layout (2596 / 2356)
  // weights: f32 image (all modes: norms, biases, constants; f32-mode matrices) + fp16 hi/lo chunks (x3 mode)
  float* wbuf = nullptr;
  _Float16* hbuf = nullptr;
  size_t n_half = 0, n_f32 = 0;   // element counts of hbuf / wbuf (vge_debug_encoder_images)
  void* d_encs = nullptr;         // EncDescHost[10] or EncDescX3Host[10]
  std::vector<vge::TxLayerX3Host> tx_layers;  // x3: the fused transformer kernel's layer table
  bool tx_fused = true;           // x3: one fused transformer launch (VGE_X3_UNFUSED=1: per-layer kernels)
  unsigned stem_heavy = 0;        // bit e: encoder e's stem spans more than one 256-wide K panel (vit)
  bool x3s = false;               // VGE_F32X3: the staggered conv kernel on GroupNorm-folded weights (VGE_X3S=0: off)
  int f16_mix = 0;                // VGE_F16: stages kept in 3xfp16 (bit 0 stem, bit 1 transformer; VGE_F16_MIX)
  // VGE_F16 with the stem unsplit: the unit-table conv kernel with units of up to `f16w` windows (VGE_F16W; 0 = the
  // quad / pair kernel); its table for batch units_B lives in d_units (sized by vge_encoder_reserve, built on the
  // device by vge_encode when the batch size changes)
  int f16w = 6;
  // Up to kUnitTables tables are kept (one slot of units_cap entries each, least recently used replaced): config 5
  // alternates a full chunk and its tail, and each table is built once.
  static constexpr int kUnitTables = 4;
  int* d_units = nullptr;
  size_t units_cap = 0;  // entries per slot (>= R * G for any batch <= cap; checked per build)
  struct UnitTable { int B = 0, G = 0, R = 0; unsigned long long used = 0; };
  UnitTable tables[kUnitTables];
  unsigned long long units_clock = 0;
  int units_last = -1;  // slot of the last vge_encode (test hook vge_debug_encoder_units)
  hipEvent_t conv_done = nullptr;  // recorded after the conv stage of every vge_encode (vge_encoder_wait_conv)
  // device status word (host-mapped, coherent): a kernel that detects a broken invariant (the staggered conv kernel's
  // exchange wait running out) stores 1; vge_encode / vge_encoder_profile_read / vge_encoder_status report it
  int* status_h = nullptr;
  int* status_d = nullptr;
  // vge_encoder_set_tail_stream: the stages after the fusion run on `tail`; fuse_done hands the fusion output over,
  // tail_done (after the last tail stage) makes the next fusion wait before it overwrites `pooled`
  hipStream_t tail = nullptr;
  bool tail_set = false, tail_pending = false;
  hipEvent_t fuse_done = nullptr, tail_done = nullptr;
  vge::FuseParamsHost fuse{};
  const void* Wov = nullptr;      // packed (f32 chunks or fp16 chunks)
  const float* Wov_cs = nullptr;  // x3: its column scales
  struct Layer {
    const void *in_w, *out_w, *l1_w, *l2_w;  // packed matrices
    const float *in_b, *out_b, *l1_b, *l2_b, *n1_w, *n1_b, *n2_w, *n2_b;
    const float *in_cs, *out_cs, *l1_cs, *l2_cs;  // x3: per-column weight scales
    int e_x1, e_x2, e_h;                          // x3: static split exponents (see LOff)
  };
  std::vector<Layer> layers;
  const float* cls = nullptr;
  const float* pe = nullptr;
  // profiling (hipEvents recorded around the stages of vge_encode)
  std::vector<hipEvent_t> prof_ev;   // (VGE_N_STAGES + 1) per call
  int prof_max = 0, prof_calls = 0;
  int prof_mask = (1 << (VGE_N_STAGES + 1)) - 1;  // which stage-boundary events vge_encode records (profile_mask)
  hipEvent_t last_conv = nullptr;                 // the event vge_encoder_wait_conv waits on
  // workspace
  int cap = 0;
  float* ws = nullptr;
  float *enc_out = nullptr, *pooled = nullptr, *x = nullptr, *qkv = nullptr, *att = nullptr, *x1 = nullptr,
        *h = nullptr;
};

namespace vge {
void set_last_error(const std::string& msg) { g_err = msg; }  // vge_hmr.cpp
}  // namespace vge

extern "C" {

const char* vge_last_error(void) { return g_err.c_str(); }
const char* vge_version(void) { return "vge 0.2 (gfx950: f32 MFMA + 3xfp16 split MFMA)"; }

// ------------------------------------------------------------------ featurise
int vge_featurize_layout(const vge_frame_store* st, const int32_t* windows, int n_windows, const float* mean,
                         const float* std_, vge_layout layout, float* feats, vge_stream_t stream) {
  if (!st || !windows || !feats || n_windows < 0 || !mean || !std_) return fail(VGE_ERR_ARG, "vge_featurize: null argument");
  if (layout != VGE_LAYOUT_KP && layout != VGE_LAYOUT_NOKP) return fail(VGE_ERR_ARG, "vge_featurize: unknown layout");
  HIPCHK(vge::launch_featurize_tiles(st->pose, st->gori, st->betas, st->vit, st->kp, st->videos, nullptr, windows,
                                     n_windows, mean, std_, feats, layout == VGE_LAYOUT_KP, S(stream)));
  return VGE_OK;
}

int vge_featurize(const vge_frame_store* st, const int32_t* windows, int n_windows, const float* mean, const float* std_,
                  float* feats, vge_stream_t stream) {
  return vge_featurize_layout(st, windows, n_windows, mean, std_, VGE_LAYOUT_KP, feats, stream);
}

int vge_layout_feat_dim(vge_layout layout) {
  return layout == VGE_LAYOUT_KP ? VGE_FEAT_DIM : layout == VGE_LAYOUT_NOKP ? VGE_FEAT_DIM_NOKP : 0;
}

// ------------------------------------------------------------------ stats
static const int kColChunk = 4;   // tiles per column-sum partial (128 rows: enough chunks to fill the chip)

size_t vge_stats_workspace_bytes(int ct) {
  if (ct < 1) ct = 1;
  const size_t nch = (ct + kColChunk - 1) / kColChunk;
  return align_up((size_t)ct * 32, 256) + align_up((size_t)ct * 32 * VGE_FEAT_DIM * 4, 256) +
         align_up(nch * 2 * VGE_FEAT_DIM * 8, 256);
}

int vge_stats_accumulate(const vge_frame_store* st, const int32_t* host_videos, const int32_t* sel, int n_sel,
                         double* sums, int64_t* counts, void* workspace, size_t wsb, vge_stream_t stream) {
  if (!st || !host_videos || (!sel && n_sel) || !sums || !counts || !workspace) return fail(VGE_ERR_ARG, "vge_stats_accumulate: null argument");
  // largest chunk of tiles that fits the workspace
  int ct = 1;
  while (vge_stats_workspace_bytes(ct * 2) <= wsb && ct < (1 << 20)) ct *= 2;
  while (vge_stats_workspace_bytes(ct + 1) <= wsb && ct < (1 << 20)) ++ct;
  if (vge_stats_workspace_bytes(ct) > wsb) return fail(VGE_ERR_WORKSPACE, "vge_stats_accumulate: workspace too small");
  char* w = static_cast<char*>(workspace);
  int32_t* d_tiles = reinterpret_cast<int32_t*>(w);
  float* d_feats = reinterpret_cast<float*>(w + align_up((size_t)ct * 32, 256));
  double* d_part = reinterpret_cast<double*>(w + align_up((size_t)ct * 32, 256) + align_up((size_t)ct * 32 * VGE_FEAT_DIM * 4, 256));
  std::vector<int32_t> tiles;
  tiles.reserve((size_t)ct * 8);
  auto flush = [&]() -> int {
    const int n = (int)(tiles.size() / 8);
    if (n == 0) return VGE_OK;
    HIPCHK(hipMemcpyAsync(d_tiles, tiles.data(), tiles.size() * 4, hipMemcpyHostToDevice, S(stream)));
    HIPCHK(vge::launch_featurize_tiles(st->pose, st->gori, st->betas, st->vit, st->kp, st->videos, d_tiles, nullptr, n,
                                       nullptr, nullptr, d_feats, 1, S(stream)));
    const int nch = (n + kColChunk - 1) / kColChunk;
    HIPCHK(vge::launch_stats_colsum(d_feats, d_tiles, n, kColChunk, nch, d_part, sums, S(stream)));
    HIPCHK(hipStreamSynchronize(S(stream)));  // host tile buffer is reused
    tiles.clear();
    return VGE_OK;
  };
  for (int s = 0; s < n_sel; ++s) {
    const int v = sel[s];
    if (v < 0 || v >= st->n_videos) return fail(VGE_ERR_ARG, "vge_stats_accumulate: video index out of range");
    const int T = host_videos[4 * v + 1], Tk = host_videos[4 * v + 3];
    counts[0] += T;
    counts[1] += Tk;
    const int nt = (std::max(T, Tk) + 31) / 32;
    for (int i = 0; i < nt; ++i) {
      if ((int)(tiles.size() / 8) == ct) {
        int r = flush();
        if (r) return r;
      }
      const int out_row = (int)(tiles.size() / 8) * 32;
      const int mc = std::min(32, std::max(0, T - 32 * i)), kc = std::min(32, std::max(0, Tk - 32 * i));
      const int32_t td[8] = {v, 1, 32 * i, mc, 32 * i, kc, out_row, 0};
      tiles.insert(tiles.end(), td, td + 8);
    }
  }
  return flush();
}

int vge_stats_finalize_layout(const double* sums, const int64_t* counts, vge_layout layout, float* mean, float* std_,
                              vge_stream_t stream) {
  if (!sums || !counts || !mean || !std_) return fail(VGE_ERR_ARG, "vge_stats_finalize: null argument");
  if (layout != VGE_LAYOUT_KP && layout != VGE_LAYOUT_NOKP) return fail(VGE_ERR_ARG, "vge_stats_finalize: unknown layout");
  HIPCHK(vge::launch_stats_finalize(sums, counts[0], counts[1], mean, std_, layout == VGE_LAYOUT_KP, S(stream)));
  return VGE_OK;
}

int vge_stats_finalize(const double* sums, const int64_t* counts, float* mean, float* std_, vge_stream_t stream) {
  return vge_stats_finalize_layout(sums, counts, VGE_LAYOUT_KP, mean, std_, stream);
}

// ------------------------------------------------------------------ encoder
int vge_encoder_create(const vge_dims* dims, const vge_tensor_view* weights, int n_weights, vge_dtype compute,
                       vge_encoder** out) {
  if (!dims || !weights || !out) return fail(VGE_ERR_ARG, "vge_encoder_create: null argument");
  *out = nullptr;
  if (compute != VGE_F32 && compute != VGE_F32X3 && compute != VGE_F16)
    return fail(VGE_ERR_ARG, "vge_encoder_create: unsupported compute dtype");
  // VGE_F16 shares the 3xfp16 weight image (its kernels read the hi planes only)
  const bool x3 = compute == VGE_F32X3 || compute == VGE_F16;
  if (dims->time_layers < 1) return fail(VGE_ERR_ARG, "vge_encoder_create: time_layers must be >= 1");
  // 5 modalities (keypoint_dir given) or the keypoint-less 4 (utils.py:496-514; infer_dims_from_stats, eval.py:104-133)
  const int M = dims->n_modalities;
  // d_model / heads other than 256 / 8: the generic exact-f32 kernels (d_model a multiple of 32 up to 256, head dim
  // <= 64), requested as VGE_F32; the tiled 3xfp16 / fp16 kernels are built around 256 columns x 8 heads of 32
  const int Dm = dims->d_model, Hn = dims->time_heads;
  const bool generic = Dm != 256 || Hn != 8;
  const bool gen_ok = compute == VGE_F32 && Dm >= 32 && Dm <= 256 && Dm % 32 == 0 && Hn >= 1 && Dm % Hn == 0 &&
                      Dm / Hn <= 64;
  if ((M != 5 && M != 4) || dims->clip_len != 32 || (generic && !gen_ok))
    return fail(VGE_ERR_UNSUPPORTED,
                "vge_encoder_create: kernels are built for 5 (or 4, keypoint-less) modalities, clip 32, d_model 256 with "
                "8 heads (any compute) or, on the exact-f32 path (VGE_F32), d_model a multiple of 32 up to 256 with a "
                "head dim <= 64 (got " +
                    std::to_string(dims->n_modalities) + " modalities, d_model " + std::to_string(Dm) + ", " +
                    std::to_string(Hn) + " heads, clip " + std::to_string(dims->clip_len) + ")");
  for (int m = 0; m < M; ++m)
    if (dims->dims_raw[m] != kDimsRaw[m] || dims->dims_diff[m] != kDimsDiff[m])
      return fail(VGE_ERR_UNSUPPORTED, std::string("vge_encoder_create: unsupported dims for modality ") + kMods[m]);

  std::unordered_map<std::string, const vge_tensor_view*> wm;
  for (int i = 0; i < n_weights; ++i)
    if (weights[i].name) wm[weights[i].name] = &weights[i];
  std::string err;
  auto get = [&](const std::string& k, std::initializer_list<int64_t> shape) -> const float* {
    auto it = wm.find(k);
    if (it == wm.end()) {
      if (err.empty()) err = "missing weight: " + k;
      return nullptr;
    }
    const vge_tensor_view* t = it->second;
    int i = 0;
    bool ok = t->ndim == (int)shape.size() && t->data != nullptr;
    for (int64_t sh : shape) ok = ok && i < t->ndim && t->shape[i++] == sh;
    if (!ok && err.empty()) err = "bad shape for weight: " + k;
    return ok ? t->data : nullptr;
  };
  auto bail = [&]() { return fail(err.rfind("missing", 0) == 0 ? VGE_ERR_MISSING_WEIGHT : VGE_ERR_WEIGHT_SHAPE, err); };

  if (generic) {  // ---- the generic-shape exact-f32 model: reference weights uploaded as they are (+ the fusion fold)
    const int d = Dm, L = dims->time_layers, ffn = 4 * d;   // model.py:145: dim_feedforward = 4 * d_model
    std::vector<float> hw;
    std::vector<std::pair<const float**, size_t>> fix;      // device pointers resolved after the upload
    auto put = [&](const float* src, size_t n, const float** dst) {
      fix.push_back({dst, hw.size()});
      hw.insert(hw.end(), src, src + n);
      hw.resize((hw.size() + 63) / 64 * 64, 0.f);
    };
    auto* gm = new GenModel();
    std::unique_ptr<GenModel> guard(gm);
    gm->d = d; gm->heads = Hn; gm->layers = L; gm->ffn = ffn; gm->M = M;
    gm->encs.resize(2 * M);
    int col_raw = 0, col_diff = M == 5 ? VGE_RAW_DIM : VGE_RAW_DIM_NOKP;
    for (int kind = 0; kind < 2; ++kind)
      for (int m = 0; m < M; ++m) {
        GenModel::Enc& E = gm->encs[kind * M + m];
        const std::string pre = std::string(kind == 0 ? "state_enc." : "motion_enc.") + kMods[m];
        const int d_in = kind == 0 ? kDimsRaw[m] : kDimsDiff[m];
        E.d_in = d_in;
        E.in_col = kind == 0 ? col_raw : col_diff;
        if (kind == 0) col_raw += d_in; else col_diff += d_in;
        const float* st = get(pre + ".stem.weight", {d, d_in, 1});
        if (st) put(st, (size_t)d * d_in, &E.stem);
        for (int b = 0; b < 4; ++b) {
          for (int cv = 0; cv < 2; ++cv) {
            const float* w = get(pre + ".blocks." + std::to_string(b) + ".conv" + std::to_string(cv + 1) + ".weight",
                                 {d, d, 5});
            if (w) put(w, (size_t)d * d * 5, &E.conv[b * 2 + cv]);
          }
          const float* g = get(pre + ".blocks." + std::to_string(b) + ".norm.weight", {d});
          const float* be = get(pre + ".blocks." + std::to_string(b) + ".norm.bias", {d});
          if (g && be) {
            put(g, d, &E.gw[b]);
            put(be, d, &E.gb[b]);
          }
        }
        const float* pj = get(pre + ".proj.weight", {d, d});
        if (pj) put(pj, (size_t)d * d, &E.proj);
      }
    const float* latent = get("fusion.latent", {1, 1, d});
    const float* qw = get("fusion.q_ln.weight", {d});
    const float* qb = get("fusion.q_ln.bias", {d});
    const float* kvw = get("fusion.kv_ln.weight", {d});
    const float* kvb = get("fusion.kv_ln.bias", {d});
    const float* Wq = get("fusion.Wq.weight", {d, d});
    const float* Wk = get("fusion.Wk.weight", {d, d});
    const float* Wv = get("fusion.Wv.weight", {d, d});
    const float* Wo = get("fusion.Wo.weight", {d, d});
    const float* ltemp = get("fusion.logit_temp", {M});
    const float* lbias = get("fusion.logit_bias", {M});
    const float* clsw = get("cls", {1, 1, d});
    const float* pe = nullptr;
    {
      auto it = wm.find("pos_enc.pe");
      if (it == wm.end()) {
        if (err.empty()) err = "missing weight: pos_enc.pe";
      } else if (it->second->ndim == 3 && it->second->shape[0] == 1 && it->second->shape[1] >= 33 &&
                 it->second->shape[2] == d && it->second->data) {
        pe = it->second->data;
      } else if (err.empty()) {
        err = "bad shape for weight: pos_enc.pe";
      }
    }
    std::vector<const float*> lw;
    for (int l = 0; l < L; ++l) {
      const std::string p = "temporal.layers." + std::to_string(l);
      lw.push_back(get(p + ".self_attn.in_proj_weight", {3 * d, d}));
      lw.push_back(get(p + ".self_attn.in_proj_bias", {3 * d}));
      lw.push_back(get(p + ".self_attn.out_proj.weight", {d, d}));
      lw.push_back(get(p + ".self_attn.out_proj.bias", {d}));
      lw.push_back(get(p + ".norm1.weight", {d}));
      lw.push_back(get(p + ".norm1.bias", {d}));
      lw.push_back(get(p + ".linear1.weight", {ffn, d}));
      lw.push_back(get(p + ".linear1.bias", {ffn}));
      lw.push_back(get(p + ".linear2.weight", {d, ffn}));
      lw.push_back(get(p + ".linear2.bias", {d}));
      lw.push_back(get(p + ".norm2.weight", {d}));
      lw.push_back(get(p + ".norm2.bias", {d}));
    }
    if (!err.empty()) return bail();
    // fusion fold (double): q = q_ln(latent), u = Wk^T Wq q; Wov = Wo Wv (model.py:79-98)
    std::vector<double> q(d), Q(d);
    {
      double mu = 0, var = 0;
      for (int i = 0; i < d; ++i) mu += latent[i];
      mu /= d;
      for (int i = 0; i < d; ++i) var += (latent[i] - mu) * (latent[i] - mu);
      var /= d;
      const double rstd = 1.0 / std::sqrt(var + 1e-5);
      for (int i = 0; i < d; ++i) q[i] = (latent[i] - mu) * rstd * qw[i] + qb[i];
      for (int j = 0; j < d; ++j) {
        double a = 0;
        for (int i = 0; i < d; ++i) a += q[i] * Wq[(size_t)j * d + i];
        Q[j] = a;
      }
    }
    std::vector<float> u(d), wov((size_t)d * d);
    for (int i = 0; i < d; ++i) {
      double a = 0;
      for (int j = 0; j < d; ++j) a += Q[j] * Wk[(size_t)j * d + i];
      u[i] = (float)a;
    }
    for (int i = 0; i < d; ++i)
      for (int j = 0; j < d; ++j) {
        double a = 0;
        for (int k = 0; k < d; ++k) a += (double)Wo[(size_t)i * d + k] * Wv[(size_t)k * d + j];
        wov[(size_t)i * d + j] = (float)a;
      }
    put(u.data(), d, &gm->fuse.u);
    put(kvw, d, &gm->fuse.kv_w);
    put(kvb, d, &gm->fuse.kv_b);
    put(wov.data(), (size_t)d * d, &gm->Wov);
    put(clsw, d, &gm->cls);
    put(pe, (size_t)33 * d, &gm->pe);
    gm->fuse.n_mod = M;
    gm->fuse.d = d;
    for (int m = 0; m < M; ++m) {
      const float x = ltemp[m];
      const float sp = x > 20.0f ? x : log1pf(expf(x));  // F.softplus (beta 1, threshold 20)
      gm->fuse.inv_tau[m] = 1.0f / (sp + 1e-3f);
      gm->fuse.bias[m] = lbias[m];
      gm->fuse.has_motion[m] = 1;
    }
    gm->L.resize(L);
    for (int l = 0; l < L; ++l) {
      GenModel::Lyr& Y = gm->L[l];
      const float* const* w = lw.data() + 12 * l;
      put(w[0], (size_t)3 * d * d, &Y.in_w);
      put(w[1], (size_t)3 * d, &Y.in_b);
      put(w[2], (size_t)d * d, &Y.out_w);
      put(w[3], d, &Y.out_b);
      put(w[4], d, &Y.n1w);
      put(w[5], d, &Y.n1b);
      put(w[6], (size_t)ffn * d, &Y.l1w);
      put(w[7], ffn, &Y.l1b);
      put(w[8], (size_t)d * ffn, &Y.l2w);
      put(w[9], d, &Y.l2b);
      put(w[10], d, &Y.n2w);
      put(w[11], d, &Y.n2b);
    }
    hipError_t he = hipMalloc(&gm->wbuf, hw.size() * sizeof(float));
    if (he == hipSuccess) he = hipMemcpy(gm->wbuf, hw.data(), hw.size() * sizeof(float), hipMemcpyHostToDevice);
    if (he != hipSuccess) return fail(VGE_ERR_HIP, std::string("vge_encoder_create: ") + hipGetErrorString(he));
    for (auto& f : fix) *f.first = gm->wbuf + f.second;
    vge_encoder* enc = new vge_encoder();
    enc->gen = guard.release();
    enc->mode = VGE_F32;
    enc->n_mod = M;
    enc->n_enc = 2 * M;
    enc->feat_dim = M == 5 ? VGE_FEAT_DIM : VGE_FEAT_DIM_NOKP;
    enc->n_layers = L;
    he = hipEventCreateWithFlags(&enc->conv_done, hipEventDisableTiming);
    if (he == hipSuccess) he = hipEventCreateWithFlags(&enc->fuse_done, hipEventDisableTiming);
    if (he == hipSuccess) he = hipEventCreateWithFlags(&enc->tail_done, hipEventDisableTiming);
    if (he != hipSuccess) {
      vge_encoder_destroy(enc);
      return fail(VGE_ERR_HIP, std::string("vge_encoder_create: ") + hipGetErrorString(he));
    }
    *out = enc;
    return VGE_OK;
  }

  if (compute == VGE_F16 && dims->time_layers > 8)
    return fail(VGE_ERR_UNSUPPORTED, "vge_encoder_create: VGE_F16 runs the fused transformer, at most 8 layers");
  const int L = dims->time_layers;
  std::vector<float> pk;      // f32 device image
  // x3: the fp16 hi/lo image is packed on the device after the upload (launch_pack_x3, one job per matrix; the
  // column scales land in pk's placeholders); VGE_HOST_PACK=1 packs it on host threads instead (A/B check)
  struct PackJob { const float* W; int N, K_real, ldk, conv, nch; size_t off, cs; };
  std::vector<PackJob> jobs;
  size_t ph_n = 0;
  // a packed matrix lives in pk (f32 mode) or the fp16 image (x3 mode)
  struct Mat { size_t off, cs; };  // packed matrix (pk or fp16 image offset); x3: column scales at pk[cs]
  auto add_job = [&](const float* W, int N, int K_real, int ldk, int conv, int chunk_mult) -> Mat {
    const int nch = ((K_real + 15) / 16 + chunk_mult - 1) / chunk_mult * chunk_mult;
    const Mat m{ph_n, pk.size()};
    jobs.push_back(PackJob{W, N, K_real, ldk, conv, nch, ph_n, pk.size()});
    pk.resize(pk.size() + N, 0.f);
    ph_n += (size_t)(N / 256) * nch * 8192;
    return m;
  };
  auto pack_lin = [&](const float* W, int N, int K_real, int ldk, int P) -> Mat {
    // the x3 kernels stream weights in groups of 8 chunks (zero chunks pad a short last panel)
    if (x3) return add_job(W, N, K_real, ldk, 0, 8);
    const size_t o = pk.size();
    pack_linear(W, N, K_real, ldk, P, pk);
    return {o, 0};
  };
  auto pack_cv = [&](const float* W) -> Mat {
    if (x3) return add_job(W, 256, 5 * 256, 0, 1, 1);  // K index = tap * 256 + ci (tap-major panels)
    const size_t o = pk.size();
    pack_conv(W, pk);
    return {o, 0};
  };

  // VGE_F32X3 runs the staggered conv kernel (vge_encoder_x3s.hip) unless VGE_X3S=0: each block's GroupNorm is folded
  // into the next GEMM -- conv1 of blocks 1..3 and proj packed as W diag(gamma) -- plus the per-row corrections
  // (sums of W gamma and W beta over the taps that fall inside the window; double, then f32)
  // VGE_F16 (with the stem unsplit): the same staggered kernel in single fp16 (hi planes only) unless VGE_F16_X3S=0
  // selects conv_encoder_f16w_kernel (1..6-window units): conv 0.512 -> 0.489 ms at 256 windows, 6.95-6.99 -> 6.58-6.65
  // ms per 4,096-window chunk (profiles/ab_r05x_f16_conv.json, ab_r05w_cfg5.json)
  const char* x3s_env = getenv("VGE_X3S");
  const char* f16s_env = getenv("VGE_F16_X3S");
  const char* mix_env = getenv("VGE_F16_MIX");
  const bool f16_x3s = compute == VGE_F16 && !(f16s_env && f16s_env[0] == '0') && !((mix_env ? atoi(mix_env) : 2) & 1);
  const bool x3s = (compute == VGE_F32X3 && !(x3s_env && x3s_env[0] == '0')) || f16_x3s;
  std::vector<std::vector<float>> folded;  // folded weight copies, alive until packed
  struct Off { Mat stem, conv, proj; size_t gnw, gnb, fold; int in_col, d_in, P; };
  const int n_enc = 2 * M;
  const int feat_dim = M == 5 ? VGE_FEAT_DIM : VGE_FEAT_DIM_NOKP;
  std::vector<Off> eoff(n_enc);
  int col_raw = 0, col_diff = M == 5 ? VGE_RAW_DIM : VGE_RAW_DIM_NOKP;
  for (int kind = 0; kind < 2; ++kind) {
    for (int m = 0; m < M; ++m) {
      const int e = kind * M + m;
      const std::string pre = std::string(kind == 0 ? "state_enc." : "motion_enc.") + kMods[m];
      const int d_in = kind == 0 ? kDimsRaw[m] : kDimsDiff[m];
      Off& o = eoff[e];
      o.d_in = d_in;
      o.P = (d_in + 255) / 256;
      o.in_col = kind == 0 ? col_raw : col_diff;
      if (kind == 0) col_raw += d_in; else col_diff += d_in;
      const float* stem = get(pre + ".stem.weight", {256, d_in, 1});
      const float* cw[8];
      for (int b = 0; b < 4; ++b)
        for (int cv = 0; cv < 2; ++cv)
          cw[b * 2 + cv] = get(pre + ".blocks." + std::to_string(b) + ".conv" + std::to_string(cv + 1) + ".weight", {256, 256, 5});
      const float* proj = get(pre + ".proj.weight", {256, 256});
      const float *gw[4], *gb[4];
      for (int b = 0; b < 4; ++b) {
        gw[b] = get(pre + ".blocks." + std::to_string(b) + ".norm.weight", {256});
        gb[b] = get(pre + ".blocks." + std::to_string(b) + ".norm.bias", {256});
      }
      if (!err.empty()) return bail();
      const float* projw = proj;
      o.fold = 0;
      if (x3s) {
        pk.resize((pk.size() + 63) / 64 * 64, 0.f);  // 256-B aligned: the kernel reads 16-B vectors
        o.fold = pk.size();
        pk.resize(pk.size() + 3 * 256 * 16 + 512, 0.f);
        for (int b = 1; b <= 4; ++b) {  // GroupNorm b-1 folded into block b's conv1 (b < 4) or the proj (b == 4)
          const float* g = gw[b - 1];
          const float* be = gb[b - 1];
          const float* src = b < 4 ? cw[2 * b] : proj;
          const int ntap = b < 4 ? 5 : 1;
          folded.emplace_back((size_t)256 * 256 * ntap);
          float* f = folded.back().data();
          for (size_t q = 0; q < folded.back().size(); ++q) f[q] = src[q] * g[(q / ntap) & 255];
          parallel_for(256, [&](int n) {
            double sg[5] = {0, 0, 0, 0, 0}, sb[5] = {0, 0, 0, 0, 0};
            for (int ci = 0; ci < 256; ++ci)
              for (int tap = 0; tap < ntap; ++tap) {
                const size_t q = ((size_t)n * 256 + ci) * ntap + tap;
                sg[tap] += f[q];
                sb[tap] += (double)src[q] * be[ci];
              }
            if (b == 4) {
              pk[o.fold + 3 * 256 * 16 + n * 2] = (float)sg[0];
              pk[o.fold + 3 * 256 * 16 + n * 2 + 1] = (float)sb[0];
              return;
            }
            // per-tap sums: the kernel adds the taps that fall inside the window for each of its rows
            for (int tap = 0; tap < 5; ++tap) {
              pk[o.fold + ((size_t)(b - 1) * 256 + n) * 16 + tap] = (float)sg[tap];
              pk[o.fold + ((size_t)(b - 1) * 256 + n) * 16 + 8 + tap] = (float)sb[tap];
            }
          });
          if (b < 4) cw[2 * b] = f;
          else projw = f;
        }
      }
      o.stem = pack_lin(stem, 256, d_in, d_in, o.P);
      o.conv = pack_cv(cw[0]);
      for (int c = 1; c < 8; ++c) pack_cv(cw[c]);
      o.proj = pack_lin(projw, 256, 256, 256, 1);
      o.gnw = pk.size();
      for (int b = 0; b < 4; ++b) pk.insert(pk.end(), gw[b], gw[b] + 256);
      o.gnb = pk.size();
      for (int b = 0; b < 4; ++b) pk.insert(pk.end(), gb[b], gb[b] + 256);
    }
  }
  // fusion: fold the constant query  u = Wk^T (Wq q_ln(latent)),  Wov = Wo Wv
  const float* latent = get("fusion.latent", {1, 1, 256});
  const float* qw = get("fusion.q_ln.weight", {256});
  const float* qb = get("fusion.q_ln.bias", {256});
  const float* kvw = get("fusion.kv_ln.weight", {256});
  const float* kvb = get("fusion.kv_ln.bias", {256});
  const float* Wq = get("fusion.Wq.weight", {256, 256});
  const float* Wk = get("fusion.Wk.weight", {256, 256});
  const float* Wv = get("fusion.Wv.weight", {256, 256});
  const float* Wo = get("fusion.Wo.weight", {256, 256});
  const float* ltemp = get("fusion.logit_temp", {M});
  const float* lbias = get("fusion.logit_bias", {M});
  const float* cls = get("cls", {1, 1, 256});
  auto pe_it = wm.find("pos_enc.pe");
  if (pe_it == wm.end() && err.empty()) err = "missing weight: pos_enc.pe";
  const float* pe = nullptr;
  if (pe_it != wm.end()) {
    const vge_tensor_view* t = pe_it->second;
    if (t->ndim == 3 && t->shape[0] == 1 && t->shape[1] >= 33 && t->shape[2] == 256 && t->data) pe = t->data;
    else if (err.empty()) err = "bad shape for weight: pos_enc.pe";
  }
  if (!err.empty()) return bail();

  std::vector<double> q(256), Q(256);
  {
    double mu = 0, var = 0;
    for (int i = 0; i < 256; ++i) mu += latent[i];
    mu /= 256;
    for (int i = 0; i < 256; ++i) var += (latent[i] - mu) * (latent[i] - mu);
    var /= 256;
    const double rstd = 1.0 / std::sqrt(var + 1e-5);
    for (int i = 0; i < 256; ++i) q[i] = (latent[i] - mu) * rstd * qw[i] + qb[i];
    for (int j = 0; j < 256; ++j) {
      double a = 0;
      for (int i = 0; i < 256; ++i) a += q[i] * Wq[(size_t)j * 256 + i];
      Q[j] = a;
    }
  }
  const size_t off_u = pk.size();
  for (int i = 0; i < 256; ++i) {
    double a = 0;
    for (int j = 0; j < 256; ++j) a += Q[j] * Wk[(size_t)j * 256 + i];
    pk.push_back((float)a);
  }
  const size_t off_kvw = pk.size();
  pk.insert(pk.end(), kvw, kvw + 256);
  const size_t off_kvb = pk.size();
  pk.insert(pk.end(), kvb, kvb + 256);
  std::vector<float> wov(256 * 256);
  parallel_for(256, [&](int i) {
    for (int j = 0; j < 256; ++j) {
      double a = 0;
      for (int k = 0; k < 256; ++k) a += (double)Wo[(size_t)i * 256 + k] * Wv[(size_t)k * 256 + j];
      wov[(size_t)i * 256 + j] = (float)a;
    }
  });
  const Mat m_wov = pack_lin(wov.data(), 256, 256, 256, 1);
  const size_t off_cls = pk.size();
  pk.insert(pk.end(), cls, cls + 256);
  const size_t off_pe = pk.size();
  pk.insert(pk.end(), pe, pe + 33 * 256);

  struct LOff { Mat in_w, out_w, l1_w, l2_w; size_t in_b, out_b, l1_b, l2_b, n1_w, n1_b, n2_w, n2_b; int e_x1, e_x2, e_h; };
  std::vector<LOff> loff(L);
  // the fused transformer (x3 modes, <= 8 layers, unless VGE_X3_UNFUSED=1) reads in_proj's outputs in head order
  // (vge_transformer_x3.hip): output block j, wave w, tile t <- the original block (q | k | v) and head half of
  // kInPerm[j][t], rows 64 w + 32 half .. + 31; the per-layer kernels of the unfused path keep q | k | v
  const char* uf_env = getenv("VGE_X3_UNFUSED");
  const bool tx_fused = x3 && (!(uf_env && uf_env[0] == '1') || compute == VGE_F16) && L <= 8;
  static const int kInPerm[3][2][2] = {{{0, 0}, {1, 0}}, {{2, 0}, {0, 1}}, {{1, 1}, {2, 1}}};  // {block, half}
  auto in_perm_row = [](int nr) {
    const int j = nr >> 8, c = nr & 255, w = c >> 6, t = (c >> 5) & 1, i = c & 31;
    return kInPerm[j][t][0] * 256 + 64 * w + 32 * kInPerm[j][t][1] + i;
  };
  std::vector<std::vector<float>> in_perm;  // permuted in_proj copies, alive until packed
  for (int l = 0; l < L; ++l) {
    const std::string p = "temporal.layers." + std::to_string(l);
    const float* inw = get(p + ".self_attn.in_proj_weight", {768, 256});
    const float* inb = get(p + ".self_attn.in_proj_bias", {768});
    const float* ow = get(p + ".self_attn.out_proj.weight", {256, 256});
    const float* ob = get(p + ".self_attn.out_proj.bias", {256});
    const float* l1w = get(p + ".linear1.weight", {1024, 256});
    const float* l1b = get(p + ".linear1.bias", {1024});
    const float* l2w = get(p + ".linear2.weight", {256, 1024});
    const float* l2b = get(p + ".linear2.bias", {256});
    const float* n1w = get(p + ".norm1.weight", {256});
    const float* n1b = get(p + ".norm1.bias", {256});
    const float* n2w = get(p + ".norm2.weight", {256});
    const float* n2b = get(p + ".norm2.bias", {256});
    if (!err.empty()) return bail();
    LOff& o = loff[l];
    if (tx_fused) {
      in_perm.emplace_back((size_t)768 * 257);
      float* pw = in_perm.back().data();
      for (int nr = 0; nr < 768; ++nr) {
        std::copy(inw + (size_t)in_perm_row(nr) * 256, inw + (size_t)in_perm_row(nr) * 256 + 256, pw + (size_t)nr * 256);
        pw[768 * 256 + nr] = inb[in_perm_row(nr)];
      }
      inw = pw;
      inb = pw + 768 * 256;
    }
    o.in_w = pack_lin(inw, 768, 256, 256, 1);
    o.out_w = pack_lin(ow, 256, 256, 256, 1);
    o.l1_w = pack_lin(l1w, 1024, 256, 256, 1);
    o.l2_w = pack_lin(l2w, 256, 1024, 1024, 4);
    o.in_b = pk.size(); pk.insert(pk.end(), inb, inb + 768);
    o.out_b = pk.size(); pk.insert(pk.end(), ob, ob + 256);
    o.l1_b = pk.size(); pk.insert(pk.end(), l1b, l1b + 1024);
    o.l2_b = pk.size(); pk.insert(pk.end(), l2b, l2b + 256);
    o.n1_w = pk.size(); pk.insert(pk.end(), n1w, n1w + 256);
    o.n1_b = pk.size(); pk.insert(pk.end(), n1b, n1b + 256);
    o.n2_w = pk.size(); pk.insert(pk.end(), n2w, n2w + 256);
    o.n2_b = pk.size(); pk.insert(pk.end(), n2b, n2b + 256);
    // static operand scales of the fused x3 transformer (vge_transformer_x3.hip): a LayerNorm output is
    // bounded by 16 max|gamma| + max|beta| (sum_j z_j^2 <= 256), ReLU(X1 W1^T + b1) by
    // max_n sum_k |W1[n][k]| * that + |b1[n]|
    auto ln_bound = [](const float* g, const float* b) {
      double mg = 0.0, mb = 0.0;
      for (int j = 0; j < 256; ++j) {
        mg = std::max(mg, (double)std::fabs(g[j]));
        mb = std::max(mb, (double)std::fabs(b[j]));
      }
      return 16.0 * mg + mb;
    };
    const double b1 = ln_bound(n1w, n1b), b2 = ln_bound(n2w, n2b);
    double bh = 0.0;
    for (int n = 0; n < 1024; ++n) {
      double a = 0.0;
      for (int k = 0; k < 256; ++k) a += std::fabs((double)l1w[(size_t)n * 256 + k]);
      bh = std::max(bh, a * b1 + std::fabs((double)l1b[n]));
    }
    o.e_x1 = range_exp(b1);
    o.e_x2 = range_exp(b2);
    o.e_h = range_exp(bh);
  }

  vge_encoder* enc = new vge_encoder();
  enc->mode = compute;
  enc->n_mod = M;
  enc->n_enc = n_enc;
  enc->feat_dim = feat_dim;
  if (compute == VGE_F16) {  // default: the transformer keeps the split (most of the f16 error, ~10% of the FLOPs)
    const char* mx = getenv("VGE_F16_MIX");
    enc->f16_mix = mx ? atoi(mx) : 2;
    const char* fw = getenv("VGE_F16W");
    enc->f16w = fw ? atoi(fw) : 6;
  }
  enc->n_layers = L;
  auto hipfail = [&](hipError_t he) {
    vge_encoder_destroy(enc);
    return fail(VGE_ERR_HIP, std::string("vge_encoder_create: ") + hipGetErrorString(he));
  };
  // column scaling keeps every finite weight in the fp16 planes' range; a non-finite one cannot be split
  const char* hp_env = getenv("VGE_HOST_PACK");
  const bool host_pack = x3 && hp_env && hp_env[0] == '1';
  std::vector<_Float16> ph;
  if (host_pack) {
    for (const PackJob& j : jobs) {
      std::vector<float> cs;
      const float* W = j.W;
      const int ldk = j.ldk;
      if (j.conv)
        pack_linear_x3([&](int n, int k) { return W[((size_t)n * 256 + (k & 255)) * 5 + (k >> 8)]; }, j.N, j.K_real,
                       ph, cs, 1);
      else
        pack_linear_x3([&](int n, int k) { return W[(size_t)n * ldk + k]; }, j.N, j.K_real, ph, cs, 8);
      std::copy(cs.begin(), cs.end(), pk.begin() + j.cs);
    }
    for (const _Float16 v : ph)
      if (!std::isfinite((float)v)) {
        vge_encoder_destroy(enc);
        return fail(VGE_ERR_ARG, "vge_encoder_create: non-finite weight, not representable by the 3xfp16 split; use VGE_F32");
      }
  }
  enc->x3s = x3s;
  hipError_t he = x3 ? vge::encoder_x3_kernel_setup() : vge::encoder_kernel_setup();
  if (he == hipSuccess && x3s) he = vge::encoder_x3s_kernel_setup();

  if (he == hipSuccess) he = hipMalloc(&enc->wbuf, pk.size() * sizeof(float));
  if (he == hipSuccess) he = hipMemcpy(enc->wbuf, pk.data(), pk.size() * sizeof(float), hipMemcpyHostToDevice);
  if (he == hipSuccess && x3) he = hipMalloc(&enc->hbuf, ph_n * sizeof(_Float16));
  if (he == hipSuccess && host_pack) he = hipMemcpy(enc->hbuf, ph.data(), ph_n * sizeof(_Float16), hipMemcpyHostToDevice);
  if (he != hipSuccess) return hipfail(he);
  enc->n_half = x3 ? ph_n : 0;
  enc->n_f32 = pk.size();
  if (x3 && !host_pack) {
    // raw f32 weights staged in HBM (one buffer), then packed by launch_pack_x3 straight into hbuf / wbuf
    size_t raw = 0, ncol = 0;
    std::vector<size_t> roff(jobs.size());
    for (size_t i = 0; i < jobs.size(); ++i) {
      roff[i] = raw;
      raw += (size_t)jobs[i].N * (jobs[i].conv ? 1280 : jobs[i].ldk);
      ncol = std::max(ncol, (size_t)jobs[i].N);
    }
    float* d_raw = nullptr;
    int* d_sh = nullptr;  // [jobs][ncol] column exponents, then the non-finite flag
    he = hipMalloc(&d_raw, raw * sizeof(float));
    if (he == hipSuccess) he = hipMalloc(&d_sh, (jobs.size() * ncol + 1) * sizeof(int));
    if (he == hipSuccess) he = hipMemset(d_sh + jobs.size() * ncol, 0, sizeof(int));
    for (size_t i = 0; i < jobs.size() && he == hipSuccess; ++i) {
      const PackJob& j = jobs[i];
      he = hipMemcpyAsync(d_raw + roff[i], j.W, (size_t)j.N * (j.conv ? 1280 : j.ldk) * sizeof(float),
                          hipMemcpyHostToDevice, nullptr);
      if (he == hipSuccess)
        he = vge::launch_pack_x3(d_raw + roff[i], j.N, j.K_real, j.ldk, j.conv, j.nch, d_sh + i * ncol,
                                 enc->wbuf + j.cs, d_sh + jobs.size() * ncol, enc->hbuf + j.off, nullptr);
    }
    int bad = 0;
    if (he == hipSuccess) he = hipMemcpy(&bad, d_sh + jobs.size() * ncol, sizeof(int), hipMemcpyDeviceToHost);
    if (d_raw) (void)hipFree(d_raw);
    if (d_sh) (void)hipFree(d_sh);
    if (he != hipSuccess) return hipfail(he);
    if (bad) {
      vge_encoder_destroy(enc);
      return fail(VGE_ERR_ARG, "vge_encoder_create: non-finite weight, not representable by the 3xfp16 split; use VGE_F32");
    }
  }
  float* wb = enc->wbuf;
  _Float16* hb = enc->hbuf;
  auto mat = [&](const Mat& m) -> const void* { return x3 ? (const void*)(hb + m.off) : (const void*)(wb + m.off); };
  if (x3) {
    std::vector<vge::EncDescX3Host> descs(n_enc);
    for (int e = 0; e < n_enc; ++e)
    {
      descs[e] = vge::EncDescX3Host{hb + eoff[e].stem.off, hb + eoff[e].conv.off, hb + eoff[e].proj.off,
                                    wb + eoff[e].gnw, wb + eoff[e].gnb, wb + eoff[e].stem.cs,  // [10][256] scales
                                    x3s ? wb + eoff[e].fold : nullptr, eoff[e].in_col, eoff[e].d_in, eoff[e].P,
                                    feat_dim, {}, {}};
      for (int b = 0; b < 4; ++b) {
        float gm = 0.f, bm = 0.f;
        for (int c = 0; c < 256; ++c) {
          gm = std::max(gm, std::fabs(pk[eoff[e].gnw + b * 256 + c]));
          bm = std::max(bm, std::fabs(pk[eoff[e].gnb + b * 256 + c]));
        }
        descs[e].gn_gmax[b] = gm;
        descs[e].gn_bmax[b] = bm;
      }
    }
    for (int e = 0; e < n_enc; ++e)
      if (eoff[e].P > 1) enc->stem_heavy |= 1u << e;
    he = hipMalloc(&enc->d_encs, sizeof(vge::EncDescX3Host) * n_enc);
    if (he == hipSuccess)
      he = hipMemcpy(enc->d_encs, descs.data(), sizeof(vge::EncDescX3Host) * n_enc, hipMemcpyHostToDevice);
  } else {
    std::vector<vge::EncDescHost> descs(n_enc);
    for (int e = 0; e < n_enc; ++e)
      descs[e] = vge::EncDescHost{wb + eoff[e].stem.off, wb + eoff[e].conv.off, wb + eoff[e].proj.off, wb + eoff[e].gnw,
                                  wb + eoff[e].gnb, eoff[e].in_col, eoff[e].d_in, eoff[e].P, feat_dim};
    he = hipMalloc(&enc->d_encs, sizeof(vge::EncDescHost) * n_enc);
    if (he == hipSuccess) he = hipMemcpy(enc->d_encs, descs.data(), sizeof(vge::EncDescHost) * n_enc, hipMemcpyHostToDevice);
  }
  if (he != hipSuccess) return hipfail(he);
  enc->fuse.kv_w = wb + off_kvw;
  enc->fuse.kv_b = wb + off_kvb;
  enc->fuse.u = wb + off_u;
  enc->fuse.n_mod = M;
  for (int m = 0; m < M; ++m) {
    const float x = ltemp[m];
    const float sp = x > 20.0f ? x : log1pf(expf(x));  // F.softplus (beta 1, threshold 20)
    enc->fuse.inv_tau[m] = 1.0f / (sp + 1e-3f);
    enc->fuse.bias[m] = lbias[m];
    enc->fuse.has_motion[m] = 1;
  }
  enc->Wov = mat(m_wov);
  enc->Wov_cs = x3 ? wb + m_wov.cs : nullptr;
  enc->cls = wb + off_cls;
  enc->pe = wb + off_pe;
  enc->layers.resize(L);
  for (int l = 0; l < L; ++l) {
    const LOff& o = loff[l];
    auto csp = [&](const Mat& m) -> const float* { return x3 ? wb + m.cs : nullptr; };
    enc->layers[l] = vge_encoder::Layer{mat(o.in_w), mat(o.out_w), mat(o.l1_w), mat(o.l2_w), wb + o.in_b, wb + o.out_b,
                                        wb + o.l1_b, wb + o.l2_b, wb + o.n1_w, wb + o.n1_b, wb + o.n2_w, wb + o.n2_b,
                                        csp(o.in_w), csp(o.out_w), csp(o.l1_w), csp(o.l2_w), o.e_x1, o.e_x2, o.e_h};
  }
  if (x3) {
    enc->tx_fused = tx_fused;  // the f16 mode has the fused kernel only; it takes up to 8 layers
    std::vector<vge::TxLayerX3Host>& tl = enc->tx_layers;
    tl.resize(L);
    for (int l = 0; l < L; ++l) {
      const vge_encoder::Layer& y = enc->layers[l];
      tl[l] = vge::TxLayerX3Host{(const _Float16*)y.in_w, y.in_cs, y.in_b, (const _Float16*)y.out_w, y.out_cs, y.out_b,
                                 y.n1_w, y.n1_b, (const _Float16*)y.l1_w, y.l1_cs, y.l1_b, (const _Float16*)y.l2_w,
                                 y.l2_cs, y.l2_b, y.n2_w, y.n2_b, y.e_x1, y.e_x2, y.e_h, 0};
    }
    he = vge::transformer_x3_kernel_setup();
    if (he != hipSuccess) return hipfail(he);
  }
  he = hipEventCreateWithFlags(&enc->conv_done, hipEventDisableTiming);
  if (he != hipSuccess) return hipfail(he);
  he = hipHostMalloc(reinterpret_cast<void**>(&enc->status_h), sizeof(int), hipHostMallocMapped | hipHostMallocCoherent);
  if (he == hipSuccess) {
    *enc->status_h = 0;
    he = hipHostGetDevicePointer(reinterpret_cast<void**>(&enc->status_d), enc->status_h, 0);
  }
  if (he != hipSuccess) return hipfail(he);
  *out = enc;
  return VGE_OK;
}

int vge_encoder_reserve(vge_encoder* enc, int B) {
  if (!enc || B < 1) return fail(VGE_ERR_ARG, "vge_encoder_reserve: bad argument");
  if (B <= enc->cap) return VGE_OK;
  if (enc->gen) {  // the generic-shape model's planes, [rows][d_model] each
    GenModel& g = *enc->gen;
    if (g.ws) (void)hipFree(g.ws);
    g.ws = nullptr;
    enc->cap = 0;
    const size_t d = g.d, frames = (size_t)B * 32, tok = (size_t)B * 33;
    const size_t n_enc = 2 * (size_t)g.M * frames * d, n_f = frames * d, n_t = tok * d;
    const size_t total = n_enc + 4 * n_f + 4 * n_t + tok * 3 * d + tok * g.ffn;
    hipError_t he = hipMalloc(&g.ws, total * sizeof(float));
    if (he == hipSuccess) he = hipMemset(g.ws, 0, total * sizeof(float));
    if (he != hipSuccess) return fail(VGE_ERR_NOMEM, std::string("vge_encoder_reserve: ") + hipGetErrorString(he));
    float* p = g.ws;
    g.enc_out = p; p += n_enc;
    g.a = p; p += n_f;
    g.b = p; p += n_f;
    g.c = p; p += n_f;
    g.pp = p; p += n_f;
    g.x = p; p += n_t;
    g.att = p; p += n_t;
    g.x1 = p; p += n_t;
    g.tmp = p; p += n_t;
    g.qkv = p; p += tok * 3 * d;
    g.h = p;
    enc->cap = g.cap = B;
    return VGE_OK;
  }
  if (enc->ws) {
    (void)hipFree(enc->ws);
    enc->ws = nullptr;
    enc->cap = 0;
  }
  const size_t frames = (size_t)B * 32, tok = align_up((size_t)B * 33, 64);
  const size_t n_enc_out = 10 * frames * 256, n_pooled = frames * 256, n_x = tok * 256, n_qkv = tok * 768,
               n_att = tok * 256, n_x1 = tok * 256, n_h = tok * 1024;
  const size_t total = n_enc_out + n_pooled + n_x + n_qkv + n_att + n_x1 + n_h;
  hipError_t he = hipMalloc(&enc->ws, total * sizeof(float));
  if (he == hipSuccess) he = hipMemset(enc->ws, 0, total * sizeof(float));
  if (he != hipSuccess) return fail(VGE_ERR_NOMEM, std::string("vge_encoder_reserve: ") + hipGetErrorString(he));
  float* p = enc->ws;
  enc->enc_out = p; p += n_enc_out;
  enc->pooled = p; p += n_pooled;
  enc->x = p; p += n_x;
  enc->qkv = p; p += n_qkv;
  enc->att = p; p += n_att;
  enc->x1 = p; p += n_x1;
  enc->h = p;
  if (enc->d_units) (void)hipFree(enc->d_units);
  enc->d_units = nullptr;
  for (auto& t : enc->tables) t = vge_encoder::UnitTable{};
  enc->units_last = -1;
  {  // the largest R * G over batches <= B (R * G <= n_enc B + CUs - 1, conv_f16w_plan)
    int G = 0, R = 0, U = 0;
    enc->units_cap = (size_t)enc->n_enc * B + 1024;
    if (vge::conv_f16w_plan(B, enc->n_enc, enc->f16w > 0 ? enc->f16w : 6, G, R, U))
      enc->units_cap = std::max(enc->units_cap, (size_t)G * R);
  }
  he = hipMalloc(&enc->d_units, enc->units_cap * vge_encoder::kUnitTables * sizeof(int));
  if (he != hipSuccess) return fail(VGE_ERR_NOMEM, std::string("vge_encoder_reserve: ") + hipGetErrorString(he));
  enc->cap = B;
  return VGE_OK;
}

int vge_encoder_profile_mask(vge_encoder* enc, int event_mask) {
  if (!enc || event_mask < 0 || event_mask >= (1 << (VGE_N_STAGES + 1)))
    return fail(VGE_ERR_ARG, "vge_encoder_profile_mask: bad argument");
  enc->prof_mask = event_mask;
  return VGE_OK;
}

int vge_encoder_set_tail_stream(vge_encoder* enc, vge_stream_t tail) {
  if (!enc) return fail(VGE_ERR_ARG, "vge_encoder_set_tail_stream: null encoder");
  if (!enc->fuse_done) {
    HIPCHK(hipEventCreateWithFlags(&enc->fuse_done, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&enc->tail_done, hipEventDisableTiming));
  }
  enc->tail = S(tail);
  enc->tail_set = tail != nullptr;
  return VGE_OK;
}

int vge_encoder_wait_conv(vge_encoder* enc, vge_stream_t stream) {
  if (!enc) return fail(VGE_ERR_ARG, "vge_encoder_wait_conv: null encoder");
  if (enc->last_conv) HIPCHK(hipStreamWaitEvent(S(stream), enc->last_conv, 0));
  return VGE_OK;
}

int vge_encoder_profile_begin(vge_encoder* enc, int max_calls) {
  if (!enc || max_calls < 0) return fail(VGE_ERR_ARG, "vge_encoder_profile_begin: bad argument");
  const size_t need = (size_t)max_calls * (VGE_N_STAGES + 1);
  while (enc->prof_ev.size() < need) {
    hipEvent_t e;
    HIPCHK(hipEventCreate(&e));
    enc->prof_ev.push_back(e);
  }
  enc->prof_max = max_calls;
  enc->prof_calls = 0;
  return VGE_OK;
}

int vge_encoder_profile_read(vge_encoder* enc, double* stage_ms, int* n_calls) {
  if (!enc || !stage_ms || !n_calls) return fail(VGE_ERR_ARG, "vge_encoder_profile_read: bad argument");
  for (int k = 0; k < VGE_N_STAGES; ++k) stage_ms[k] = 0.0;
  const int n = std::min(enc->prof_calls, enc->prof_max);
  int last = VGE_N_STAGES;
  while (last > 0 && !((enc->prof_mask >> last) & 1)) --last;
  for (int c = 0; c < n; ++c) {
    hipEvent_t* ev = enc->prof_ev.data() + (size_t)c * (VGE_N_STAGES + 1);
    HIPCHK(hipEventSynchronize(ev[last]));
    for (int k = 0; k < VGE_N_STAGES; ++k) {
      if (!((enc->prof_mask >> k) & 1) || !((enc->prof_mask >> (k + 1)) & 1)) continue;  // stage not bracketed
      float ms = 0.f;
      HIPCHK(hipEventElapsedTime(&ms, ev[k], ev[k + 1]));
      stage_ms[k] += ms;
    }
  }
  *n_calls = n;
  enc->prof_max = 0;
  return vge_encoder_status(enc);  // the profiled launches are complete: any invariant they broke is visible now
}

static int device_fault(const vge_encoder* enc) {
  return fail(VGE_ERR_DEVICE, "a conv encoder launch gave up waiting in its half-workgroup exchange (status word "
                              "set): its outputs are wrong; the encoder stays in this state (vge_encoder_clear_status)");
}

int vge_encoder_status(const vge_encoder* enc) {
  if (!enc) return fail(VGE_ERR_ARG, "vge_encoder_status: null encoder");
  if (enc->status_h && __atomic_load_n(enc->status_h, __ATOMIC_ACQUIRE) != 0) return device_fault(enc);
  return VGE_OK;
}

int vge_encoder_clear_status(vge_encoder* enc) {
  if (!enc) return fail(VGE_ERR_ARG, "vge_encoder_clear_status: null encoder");
  if (enc->status_h) __atomic_store_n(enc->status_h, 0, __ATOMIC_RELEASE);
  return VGE_OK;
}

// Device images of a created encoder (test hook: tests/test_gpu_parity.py compares the device-packed fp16 image
// with VGE_HOST_PACK=1's byte for byte).
extern "C" int vge_debug_encoder_images(const vge_encoder* enc, const void** hbuf, size_t* n_half, const void** wbuf,
                                        size_t* n_f32) {
  if (!enc || !hbuf || !n_half || !wbuf || !n_f32) return fail(VGE_ERR_ARG, "vge_debug_encoder_images: null argument");
  *hbuf = enc->hbuf;
  *n_half = enc->n_half;
  *wbuf = enc->wbuf;
  *n_f32 = enc->n_f32;
  return VGE_OK;
}

// Test hook: the device-built unit table of the last vge_encode's batch (tests compare it with the host spec,
// vge_debug_conv_schedule).
extern "C" int vge_debug_encoder_units(const vge_encoder* enc, const void** table, int* G, int* R) {
  if (!enc || !table || !G || !R) return fail(VGE_ERR_ARG, "vge_debug_encoder_units: null argument");
  const int k = enc->units_last;
  *table = k >= 0 ? enc->d_units + (size_t)k * enc->units_cap : nullptr;
  *G = k >= 0 ? enc->tables[k].G : 0;
  *R = k >= 0 ? enc->tables[k].R : 0;
  return VGE_OK;
}

int vge_encoder_feat_dim(const vge_encoder* enc) { return enc ? enc->feat_dim : 0; }

int vge_encoder_destroy(vge_encoder* enc) {
  if (!enc) return VGE_OK;
  for (hipEvent_t e : enc->prof_ev) (void)hipEventDestroy(e);
  if (enc->ws) (void)hipFree(enc->ws);
  if (enc->d_encs) (void)hipFree(enc->d_encs);
  if (enc->wbuf) (void)hipFree(enc->wbuf);
  if (enc->d_units) (void)hipFree(enc->d_units);
  if (enc->conv_done) (void)hipEventDestroy(enc->conv_done);
  if (enc->fuse_done) (void)hipEventDestroy(enc->fuse_done);
  if (enc->tail_done) (void)hipEventDestroy(enc->tail_done);
  if (enc->hbuf) (void)hipFree(enc->hbuf);
  if (enc->status_h) (void)hipHostFree(enc->status_h);
  delete enc->gen;
  delete enc;
  return VGE_OK;
}

int vge_encode(vge_encoder* enc, const float* feats, int B, int T, float* seq_embed, float* frame_embed, float* tc_window,
               vge_stream_t stream) {
  if (!enc || !feats || !seq_embed) return fail(VGE_ERR_ARG, "vge_encode: null argument");
  if (T != 32) return fail(VGE_ERR_ARG, "vge_encode: clip_len must be 32");
  if (B <= 0) return VGE_OK;
  if (B > enc->cap) return fail(VGE_ERR_WORKSPACE, "vge_encode: call vge_encoder_reserve(B) first");
  // an earlier launch that completed with its status word raised (no synchronisation: a host read of the word)
  if (enc->status_h && __atomic_load_n(enc->status_h, __ATOMIC_ACQUIRE) != 0) return device_fault(enc);
  hipStream_t s = S(stream);
  const int frames = B * 32, M = B * 33;
  hipEvent_t* ev = nullptr;
  // (mask 0: this call is not profiled and takes no slot -- callers sample every k-th call)
  if (enc->prof_mask != 0 && enc->prof_calls < enc->prof_max)
    ev = enc->prof_ev.data() + (size_t)(enc->prof_calls++) * (VGE_N_STAGES + 1);
  auto mark = [&](int k) -> hipError_t {
    return (ev && ((enc->prof_mask >> k) & 1)) ? hipEventRecord(ev[k], s) : hipSuccess;
  };
  auto tail_end = [&]() -> hipError_t {
    if (!enc->tail_set) return hipSuccess;
    enc->tail_pending = true;
    return hipEventRecord(enc->tail_done, s);
  };
  if (enc->gen) {  // ---- generic-shape exact-f32 path (vge_encoder_gen.hip): one launch per stage
    const GenModel& g = *enc->gen;
    const int d = g.d;
    HIPCHK(mark(0));
    for (int e = 0; e < 2 * g.M; ++e) {  // MovementConvEncoder (model.py:43-58): stem, 4 dilated blocks, proj
      const GenModel::Enc& E = g.encs[e];
      float *cur = g.a, *tmp = g.b, *nxt = g.c;
      HIPCHK(vge::launch_gen_conv(feats, enc->feat_dim, E.in_col, E.d_in, E.stem, d, 1, 1, 0, nullptr, cur, B, s));
      for (int b = 0; b < 4; ++b) {  // TemporalConvBlock (model.py:21-40), dilation 1, 2, 4, 8
        HIPCHK(vge::launch_gen_conv(cur, d, 0, d, E.conv[2 * b], d, 5, 1 << b, 1, nullptr, tmp, B, s));
        HIPCHK(vge::launch_gen_conv(tmp, d, 0, d, E.conv[2 * b + 1], d, 5, 1 << b, 2, cur, nxt, B, s));
        HIPCHK(vge::launch_gen_groupnorm(nxt, B, d, E.gw[b], E.gb[b], s));
        std::swap(cur, nxt);
      }
      HIPCHK(vge::launch_gen_gemm(cur, d, E.proj, frames, d, d, nullptr, 0, nullptr, nullptr, nullptr,
                                  g.enc_out + (size_t)e * frames * d, d, s));
    }
    HIPCHK(hipEventRecord(enc->conv_done, s));
    enc->last_conv = enc->conv_done;
    HIPCHK(mark(1));
    if (enc->tail_pending) HIPCHK(hipStreamWaitEvent(s, enc->tail_done, 0));
    HIPCHK(vge::launch_gen_fuse(g.enc_out, frames, g.fuse, g.pp, s));
    HIPCHK(mark(2));
    if (enc->tail_set) {
      HIPCHK(hipEventRecord(enc->fuse_done, s));
      HIPCHK(hipStreamWaitEvent(enc->tail, enc->fuse_done, 0));
      s = enc->tail;
    }
    // frame tokens = pooled (Wo Wv)^T, CLS + sinusoidal positions (model.py:184-188)
    HIPCHK(vge::launch_gen_gemm(g.pp, d, g.Wov, frames, d, d, nullptr, 3, nullptr, g.pe, g.cls, g.x, d, s));
    HIPCHK(mark(3));
    for (int l = 0; l < g.layers; ++l) {  // nn.TransformerEncoderLayer, post-norm, ReLU FFN of 4 d_model
      const GenModel::Lyr& Y = g.L[l];
      HIPCHK(vge::launch_gen_gemm(g.x, d, Y.in_w, M, 3 * d, d, Y.in_b, 0, nullptr, nullptr, nullptr, g.qkv, 3 * d, s));
      HIPCHK(vge::launch_gen_attn(g.qkv, B, d, g.heads, g.att, s));
      HIPCHK(vge::launch_gen_gemm(g.att, d, Y.out_w, M, d, d, Y.out_b, 0, nullptr, nullptr, nullptr, g.tmp, d, s));
      HIPCHK(vge::launch_gen_add_ln(g.x, g.tmp, M, d, Y.n1w, Y.n1b, g.x1, s));
      HIPCHK(vge::launch_gen_gemm(g.x1, d, Y.l1w, M, g.ffn, d, Y.l1b, 1, nullptr, nullptr, nullptr, g.h, g.ffn, s));
      HIPCHK(vge::launch_gen_gemm(g.h, g.ffn, Y.l2w, M, d, g.ffn, Y.l2b, 0, nullptr, nullptr, nullptr, g.tmp, d, s));
      HIPCHK(vge::launch_gen_add_ln(g.x1, g.tmp, M, d, Y.n2w, Y.n2b, g.x, s));
    }
    HIPCHK(mark(4));
    HIPCHK(vge::launch_gen_embed_tc(g.x, B, d, seq_embed, frame_embed, tc_window, s));
    HIPCHK(mark(5));
    HIPCHK(tail_end());
    return VGE_OK;
  }
  const bool x3 = enc->mode == VGE_F32X3 || enc->mode == VGE_F16, split = enc->mode != VGE_F16;
  // one GEMM launcher for both modes (same epilogues; x3 = 3xfp16 split MFMA, f32 = exact f32 MFMA)
  auto gemm = [&](int epi, const float* A, int lda, const void* W, const float* cs, float* o, int ldo, int Mr, int K,
                  int N, const float* bias, const float* res, const float* lw, const float* lb) -> hipError_t {
    if (x3) {
      vge::GemmArgsX3Host g{A, lda, (const _Float16*)W, o, ldo, Mr, K, N, bias, res, 256, lw, lb, enc->pe, enc->cls, cs};
      return vge::launch_gemm_x3(epi, g, s);
    }
    vge::GemmArgsHost g{A, lda, (const float*)W, o, ldo, Mr, K, N, bias, res, 256, lw, lb, enc->pe, enc->cls};
    return vge::launch_gemm(epi, g, s);
  };
  HIPCHK(mark(0));
  if (x3 && !split && !(enc->f16_mix & 1) && enc->f16w > 0 && !enc->x3s) {
    // the unit table of this batch size: cached, else built on the device (stream-ordered, no host copy) into the
    // least recently used slot
    int k = -1;
    for (int j = 0; j < vge_encoder::kUnitTables; ++j)
      if (enc->tables[j].B == B) k = j;
    if (k < 0) {
      int G = 0, R = 0, U = 0;
      if (!vge::conv_f16w_plan(B, enc->n_enc, enc->f16w, G, R, U)) return fail(VGE_ERR_ARG, "vge_encode: batch too large");
      if ((size_t)G * R > enc->units_cap) return fail(VGE_ERR_WORKSPACE, "vge_encode: unit table exceeds its slot");
      k = 0;
      for (int j = 1; j < vge_encoder::kUnitTables; ++j)
        if (enc->tables[j].used < enc->tables[k].used) k = j;
      HIPCHK(vge::launch_conv_f16w_table(B, enc->n_enc, G, R, U, enc->d_units + (size_t)k * enc->units_cap, s));
      enc->tables[k] = vge_encoder::UnitTable{B, G, R, 0};
    }
    enc->tables[k].used = ++enc->units_clock;
    enc->units_last = k;
    HIPCHK(vge::launch_conv_encoders_f16w(feats, B, enc->d_encs, enc->enc_out, enc->d_units + (size_t)k * enc->units_cap,
                                          enc->tables[k].G, enc->tables[k].R, s));
  } else if (x3 && enc->x3s) {
    HIPCHK(vge::launch_conv_encoders_x3s(feats, B, enc->d_encs, enc->n_enc, enc->stem_heavy, enc->enc_out,
                                         enc->status_d, split, s));
  } else if (x3) {
    HIPCHK(vge::launch_conv_encoders_x3(feats, B, enc->d_encs, enc->n_enc, enc->stem_heavy, enc->enc_out, split, enc->f16_mix & 1, s));
  } else {
    HIPCHK(vge::launch_conv_encoders(feats, B, enc->d_encs, enc->n_enc, enc->enc_out, s));
  }
  if (ev && (enc->prof_mask & 2)) {  // the conv-end profiling event doubles as the conv-done event (one marker)
    HIPCHK(mark(1));
    enc->last_conv = ev[1];
  } else {
    HIPCHK(hipEventRecord(enc->conv_done, s));
    enc->last_conv = enc->conv_done;
    HIPCHK(mark(1));
  }
  // the fusion overwrites `pooled`, which the previous encode's token stage reads (on the tail stream, if one was set)
  if (enc->tail_pending) HIPCHK(hipStreamWaitEvent(s, enc->tail_done, 0));
  HIPCHK(vge::launch_fuse(enc->enc_out, frames, enc->fuse, enc->pooled, s));
  HIPCHK(mark(2));
  if (enc->tail_set) {  // the rest of this encode on the tail stream (mark / gemm follow `s`)
    HIPCHK(hipEventRecord(enc->fuse_done, s));
    HIPCHK(hipStreamWaitEvent(enc->tail, enc->fuse_done, 0));
    s = enc->tail;
  }
  if (x3 && enc->tx_fused) {  // tokens + all layers + outputs in one launch, one window per workgroup
    HIPCHK(mark(3));
    const vge::TxArgsX3Host ta{enc->pooled, B, enc->n_layers, (const _Float16*)enc->Wov, enc->Wov_cs, enc->cls, enc->pe,
                               enc->tx_layers.data(), seq_embed, frame_embed, tc_window};
    HIPCHK(vge::launch_transformer_x3(ta, (split || (enc->f16_mix & 2)) ? 2 : ((enc->f16_mix & 4) ? 1 : 0), s));
    HIPCHK(mark(4));
    HIPCHK(mark(5));
    HIPCHK(tail_end());
    return VGE_OK;
  }
  HIPCHK(gemm(vge::EPI_TOKENS, enc->pooled, 256, enc->Wov, enc->Wov_cs, enc->x, 256, frames, 256, 256, nullptr, nullptr,
              nullptr, nullptr));
  HIPCHK(mark(3));
  for (int l = 0; l < enc->n_layers; ++l) {
    const vge_encoder::Layer& Ly = enc->layers[l];
    HIPCHK(gemm(vge::EPI_BIAS, enc->x, 256, Ly.in_w, Ly.in_cs, enc->qkv, 768, M, 256, 768, Ly.in_b, nullptr, nullptr,
                nullptr));
    HIPCHK(vge::launch_attn(enc->qkv, B, enc->att, s));
    HIPCHK(gemm(vge::EPI_BIAS_RES_LN, enc->att, 256, Ly.out_w, Ly.out_cs, enc->x1, 256, M, 256, 256, Ly.out_b, enc->x,
                Ly.n1_w, Ly.n1_b));
    if (x3) {  // fused FFN block: the 1024-wide hidden stays on chip
      const vge::FfnArgsX3Host fa{enc->x1, enc->x, M, (const _Float16*)Ly.l1_w, Ly.l1_cs, Ly.l1_b,
                                  (const _Float16*)Ly.l2_w, Ly.l2_cs, Ly.l2_b, Ly.n2_w, Ly.n2_b};
      HIPCHK(vge::launch_ffn_x3(fa, s));
    } else {
      HIPCHK(gemm(vge::EPI_BIAS_RELU, enc->x1, 256, Ly.l1_w, Ly.l1_cs, enc->h, 1024, M, 256, 1024, Ly.l1_b, nullptr,
                  nullptr, nullptr));
      HIPCHK(gemm(vge::EPI_BIAS_RES_LN, enc->h, 1024, Ly.l2_w, Ly.l2_cs, enc->x, 256, M, 1024, 256, Ly.l2_b, enc->x1,
                  Ly.n2_w, Ly.n2_b));
    }
  }
  HIPCHK(mark(4));
  HIPCHK(vge::launch_embed_tc(enc->x, B, seq_embed, frame_embed, tc_window, s));
  HIPCHK(mark(5));
  HIPCHK(tail_end());
  return VGE_OK;
}

// ------------------------------------------------------------------ metrics / centroids
int vge_tc_windows(const float* fe, int B, int T1, int d, float* tc, vge_stream_t stream) {
  if (!fe || !tc || B < 0 || T1 < 1 || d < 1) return fail(VGE_ERR_ARG, "vge_tc_windows: bad argument");
  if (B == 0) return VGE_OK;
  HIPCHK(vge::launch_tc_windows(fe, B, T1, d, tc, S(stream)));
  return VGE_OK;
}

int vge_score_videos(const float* seq, const float* tcw, const int32_t* first, const int32_t* vcls, const float* cent, int V,
                     int d, float* ac, double* tc, vge_stream_t stream) {
  if (!seq || !tcw || !first || !vcls || !ac || !tc || V < 0 || d < 1 || d > 256)
    return fail(VGE_ERR_ARG, "vge_score_videos: bad argument");
  if (V == 0) return VGE_OK;
  HIPCHK(vge::launch_score_videos(seq, tcw, first, vcls, cent, V, d, ac, tc, S(stream)));
  return VGE_OK;
}

int vge_centroid_accumulate(const float* seq, const int32_t* cls, int n, int C, int d, float* sums, float* counts,
                            vge_stream_t stream) {
  if (!seq || !cls || !sums || !counts || n < 0 || C < 1 || d < 1 || d > 256)
    return fail(VGE_ERR_ARG, "vge_centroid_accumulate: bad argument");
  if (n == 0) return VGE_OK;
  HIPCHK(vge::launch_centroid_accum(seq, cls, n, C, d, sums, counts, S(stream)));
  return VGE_OK;
}

int vge_centroid_finalize(const float* sums, const float* counts, int C, int d, float* cent, vge_stream_t stream) {
  if (!sums || !counts || !cent || C < 1 || d < 1 || d > 256) return fail(VGE_ERR_ARG, "vge_centroid_finalize: bad argument");
  HIPCHK(vge::launch_centroid_final(sums, counts, C, d, cent, S(stream)));
  return VGE_OK;
}

}  // extern "C"
