// Host-side helpers shared by the CNN model loaders (vge_dwpose.cpp: RTMPose, vge_yolox.cpp: YOLOX): device
// allocations owned by a model, state_dict lookups with shape checks, BatchNorm folding, NHWC bf16 weight
// packing for conv_bf16_kernel, and the conv launch wrapper.
#pragma once
#include <hip/hip_runtime.h>
#include "vge_gemm.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>
#include <map>
#include <array>
#include <cstdlib>

#ifndef VGE_LIB_MIN_K_DEFAULT
#define VGE_LIB_MIN_K_DEFAULT 128  // Cin 64 layers: the tuner's kernels, YOLOX -0.8 % (profiles/ab_r06ai_lib_min_k.json)
#endif
#include <cstdlib>

#include "../../include/vge.h"
#include "vge_cnn.h"

namespace vge {
void set_last_error(const std::string& msg);  // vge_api.cpp (vge_last_error)

namespace cnnh {

inline int fail(int code, const std::string& msg) {
  set_last_error(msg);
  return code;
}

#define VGE_HIPCHK(expr)                                                                                             \
  do {                                                                                                               \
    hipError_t _e = (expr);                                                                                          \
    if (_e != hipSuccess) return ::vge::cnnh::fail(VGE_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

inline hipStream_t S(vge_stream_t s) { return reinterpret_cast<hipStream_t>(s); }
inline int rup(int x, int a) { return (x + a - 1) / a * a; }
inline bool pow2(int v) { return v > 0 && (v & (v - 1)) == 0; }
inline int pow2_at_least(int v, int lo) {
  int p = lo;
  while (p < v) p <<= 1;
  return p;
}
inline uint16_t to_bf16(float f) {  // round to nearest even (torch .to(bfloat16))
  uint32_t u;
  memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return 0x7fc0;
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

struct DevAllocs {
  std::vector<void*> allocs;
  DevAllocs() = default;
  DevAllocs(const DevAllocs&) = delete;
  DevAllocs& operator=(const DevAllocs&) = delete;
  ~DevAllocs() {
    for (void* p : allocs) (void)hipFree(p);
  }
  void* dmalloc(size_t bytes) {
    void* p = nullptr;
    if (hipMalloc(&p, std::max<size_t>(bytes, 256)) != hipSuccess) return nullptr;
    allocs.push_back(p);
    return p;
  }
};

template <class T>
bool upload(DevAllocs& d, const std::vector<T>& h, T** out) {
  *out = static_cast<T*>(d.dmalloc(h.size() * sizeof(T)));
  return *out && hipMemcpy(*out, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice) == hipSuccess;
}

struct WeightMap {
  std::unordered_map<std::string, const vge_tensor_view*> m;
  std::string missing, badshape;
  WeightMap(const vge_tensor_view* w, int n) {
    for (int i = 0; i < n; ++i)
      if (w[i].name) m[w[i].name] = &w[i];
  }
  const vge_tensor_view* get(const std::string& k, std::initializer_list<int64_t> shape) {
    auto it = m.find(k);
    if (it == m.end()) {
      if (missing.empty()) missing = k;
      return nullptr;
    }
    const vge_tensor_view* v = it->second;
    bool ok = v->ndim == (int)shape.size() && v->data;
    int i = 0;
    for (int64_t s : shape) ok = ok && v->shape[i++] == s;
    if (!ok && badshape.empty()) badshape = k;
    return ok ? v : nullptr;
  }
  int status(const std::string& who) const {
    if (!missing.empty()) return fail(VGE_ERR_MISSING_WEIGHT, who + ": missing weight " + missing);
    if (!badshape.empty()) return fail(VGE_ERR_WEIGHT_SHAPE, who + ": wrong shape for " + badshape);
    return fail(VGE_ERR_HIP, who + ": device allocation / upload failed");
  }
};

struct ConvW {  // packed dense conv / Linear: bf16 [Npad][Kp], k = tap * Cinp + ci; bias f32 [Npad]
  void* w = nullptr;
  float* b = nullptr;
  int Cin = 0, Cinp = 0, Cout = 0, KH = 1, KW = 1, Kp = 0, Npad = 0;
};

// W [Cout][Cin][KH][KW] (f32, already folded) -> bf16 [Npad][Kp] tap-major with Cin padded to Cinp
inline bool pack_conv(DevAllocs& d, const float* W, const float* bias, int Cout, int Cin, int Cinp, int KH, int KW,
                      ConvW& L) {
  L.Cin = Cin;
  L.Cinp = Cinp;
  L.Cout = Cout;
  L.KH = KH;
  L.KW = KW;
  L.Kp = rup(KH * KW * Cinp, 32);
  L.Npad = rup(Cout, 256);  // conv2_bf16_kernel reads 256-row weight tiles
  std::vector<uint16_t> h((size_t)L.Npad * L.Kp, 0);
  for (int n = 0; n < Cout; ++n)
    for (int ci = 0; ci < Cin; ++ci)
      for (int t = 0; t < KH * KW; ++t)
        h[(size_t)n * L.Kp + (size_t)t * Cinp + ci] = to_bf16(W[((size_t)n * Cin + ci) * KH * KW + t]);
  std::vector<float> b(L.Npad, 0.f);
  if (bias) memcpy(b.data(), bias, Cout * 4);
  uint16_t* dw = nullptr;
  if (!upload(d, h, &dw)) return false;
  L.w = dw;
  return upload(d, b, &L.b);
}

// ConvModule / BaseConv: conv.weight + bn.{weight,bias,running_mean,running_var} -> (w * s, beta - mean * s),
// s = gamma / sqrt(var + eps), in f32 with the operation order of torch (no contraction)
#pragma clang fp contract(off)
inline bool fold(WeightMap& wm, const std::string& p, int Cout, int Cin_g, int K, float eps, std::vector<float>& W,
                 std::vector<float>& b) {
  const vge_tensor_view* w = wm.get(p + ".conv.weight", {Cout, Cin_g, K, K});
  const vge_tensor_view* g = wm.get(p + ".bn.weight", {Cout});
  const vge_tensor_view* be = wm.get(p + ".bn.bias", {Cout});
  const vge_tensor_view* mu = wm.get(p + ".bn.running_mean", {Cout});
  const vge_tensor_view* var = wm.get(p + ".bn.running_var", {Cout});
  if (!w || !g || !be || !mu || !var) return false;
  const size_t per = (size_t)Cin_g * K * K;
  W.resize((size_t)Cout * per);
  b.resize(Cout);
  for (int n = 0; n < Cout; ++n) {
    const float s = g->data[n] / std::sqrt(var->data[n] + eps);
    for (size_t i = 0; i < per; ++i) W[n * per + i] = w->data[n * per + i] * s;
    b[n] = be->data[n] - mu->data[n] * s;
  }
  return true;
}
#pragma clang fp contract(on)

// two ConvModules / BaseConvs over the same input (CSP main + short 1x1s) as ONE conv with both weight sets along
// Cout: output channels [first | second] = the CSP concat order, written straight into the concat buffer
inline bool fold_pair(WeightMap& wm, const std::string& p0, const std::string& p1, int Cout, int Cin, int K, float eps,
                      std::vector<float>& W, std::vector<float>& b) {
  std::vector<float> W1, b1;
  if (!fold(wm, p0, Cout, Cin, K, eps, W, b) || !fold(wm, p1, Cout, Cin, K, eps, W1, b1)) return false;
  W.insert(W.end(), W1.begin(), W1.end());
  b.insert(b.end(), b1.begin(), b1.end());
  return true;
}

// Per-layer kernel choice, measured on first use: the implicit-GEMM conv has bit-identical variants (128- or 256-row
// tiles with 64 or 128 columns, 256 x 256 tiles one per workgroup, 256 x 256 or 512 x 128 tiles on the persistent grid) whose
// ranking depends on K, Cout and the tile count (tools/conv_bench.py).  The first launch of each layer shape times
// every applicable variant on the layer's own operands (one warm launch + 3 timed, hipEvents on its stream) and keeps
// the fastest; layers whose output is also an input (in-place residual) are not re-run and take the default.
// VGE_CONV_TUNE=0 turns it off.
struct ConvTuner {
  std::map<std::array<long, 10>, int> best;  // (H, W, Cin, Cout, KH, stride, act, out_f32, res, ldo) -> variant / tn
  hipEvent_t e0 = nullptr, e1 = nullptr;
  int on = -1;
  bool lib = true;  // the library path (variant 11) for the layers it takes; the pose extractors' tuners turn it off
  ~ConvTuner() {
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
  }
  bool enabled() {
    if (on < 0) {
      const char* e = getenv("VGE_CONV_TUNE");
      on = (e && atoi(e) == 0) ? 0 : 1;
    }
    return on == 1;
  }
};

struct ConvCtx {
  const void* zero;      // >= 16 B of device zeros (padding taps)
  double* flops;         // accumulates algorithmic 2 x MACs of every launch
  ConvTuner* tune = nullptr;
};

// encoded choice: variant * 1000 + tn
// hipBLASLt's stream-K GEMMs rely on their workgroups being resident together; two of them on two streams at once
// (the e2e bench runs the gate detector + TokenHMR beside YOLOX + DWPose) were seen to hang, so only one extractor
// side uses the library: the pose extractors' 1x1 convs stay on the tuner's kernels unless VGE_POSE_GEMM_LIB=1
inline bool pose_gemm_lib() {
  static const bool on = getenv("VGE_POSE_GEMM_LIB") && getenv("VGE_POSE_GEMM_LIB")[0] == '1';
  return on;
}

inline hipError_t conv_tuned_launch(ConvTuner& t, ConvLaunch& c, const std::array<long, 10>& key, hipStream_t s) {
  auto it = t.best.find(key);
  // 1x1 stride-1 convs with the epilogues the library expresses (bias, ReLU / SiLU, a bf16 residual before the ReLU)
  // go to hipBLASLt without a timing contest
  // (vge_blaslt.cpp: 1,165 vs 934-943 TFLOP/s on the detector's res4 shapes, profiles/lib_gemm_probe_r06t.json): a
  // choice that never depends on timing noise, so a layer's outputs do not change from run to run
  static const int lib_min_k = [] {  // VGE_LIB_MIN_K: layers with fewer input channels stay on the tuner's kernels
    const char* e = getenv("VGE_LIB_MIN_K");
    return e ? atoi(e) : VGE_LIB_MIN_K_DEFAULT;
  }();
  if (it == t.best.end() && t.lib && c.Cin >= lib_min_k && conv_lib_epi(c) >= 0 && gemm_lib_ok(conv_lib_epi(c)))
    it = t.best.emplace(key, 11000 + 256).first;
  if (it == t.best.end()) {
    if (!t.e0 && (hipEventCreate(&t.e0) != hipSuccess || hipEventCreate(&t.e1) != hipSuccess)) return hipErrorUnknown;
    // (12: variant 2 on the 16x16x32 MFMA form, bit-identical; VGE_CONV_SH=0 keeps it out)
    static const bool sh_ok = !(getenv("VGE_CONV_SH") && getenv("VGE_CONV_SH")[0] == '0');
    std::vector<int> cand = {1000 + 128, 5000 + 128, 2000 + 256};
    if (sh_ok) cand.push_back(12000 + 256);
    if (c.Cout <= 192) {
      cand.push_back(1000 + 64);
      cand.push_back(5000 + 64);
    }
    if (c.res_mode == 0 && c.Cout % 4 == 0) cand.push_back(3000 + 256);
    // 512 x 128 persistent tile: residual-free layers only, like variant 3 (conv2_go keeps residual epilogues off the
    // persistent kernels: its hand-counted vmcnt budget is reasoned for RES_NONE)
    if (c.res_mode == 0 && c.Cout > 64 && c.Cout <= 128 && c.Cout % 4 == 0) cand.push_back(6000 + 128);
    // 1x1 stride-1 convs with a ReLU / no activation: the bf16 GEMM kernel of the ViT (vge_vit.hip), whose 256 x 256
    // tiles and LDS-staged epilogue run these shapes ~20 % faster than the implicit GEMM (tools/gemm_vs_conv.py);
    // VGE_CONV_GEMM=0 keeps it out
    static const bool gemm_ok = !(getenv("VGE_CONV_GEMM") && getenv("VGE_CONV_GEMM")[0] == '0');
    if (gemm_ok && conv_gemm_epi(c) >= 0) cand.push_back(9000 + 256);
    // ... and its persistent form where it applies (residual-free bf16 epilogues, more 256 x 256 tiles than CUs) with
    // VGE_CONV_GEMMP=1: measured no faster on the detector (236.2 vs 236.6 ms per 256 frames, the tuner keeps the
    // one-tile kernel) and 7-20 % slower on the ViT-H shapes (profiles/ab_r06b_gemmp.json), so off by default
    static const bool gemmp_ok = getenv("VGE_CONV_GEMMP") && getenv("VGE_CONV_GEMMP")[0] == '1';
    if (gemm_ok && gemmp_ok && conv_gemm_persist_ok(c)) cand.push_back(10000 + 256);
    int pick = -1;
    float best_ms = 0.f;
    for (int v : cand) {
      c.variant = v / 1000;
      c.tn = v % 1000;
      hipError_t e = launch_conv_bf16(c, s);
      if (e != hipSuccess) return e;
      if ((e = hipEventRecord(t.e0, s)) != hipSuccess) return e;
      for (int r = 0; r < 3; ++r)
        if ((e = launch_conv_bf16(c, s)) != hipSuccess) return e;
      if ((e = hipEventRecord(t.e1, s)) != hipSuccess || (e = hipEventSynchronize(t.e1)) != hipSuccess) return e;
      float ms = 0.f;
      if ((e = hipEventElapsedTime(&ms, t.e0, t.e1)) != hipSuccess) return e;
      if (pick < 0 || ms < best_ms) {
        pick = v;
        best_ms = ms;
      }
    }
    it = t.best.emplace(key, pick).first;
  }
  c.variant = it->second / 1000;
  c.tn = it->second % 1000;
  return launch_conv_bf16(c, s);
}

// output-channel tile: 256-wide tiles (conv2_bf16_kernel, 8 waves) when Cout fills them, else the 128-row kernel
// with whichever of 64 / 128 pads Cout least (tools/conv_bench.py: conv2 wins at Cout 256 / 512, loses at 128)
inline int conv_tile_n(int Cout) {
  if (Cout % 256 == 0) return 256;
  return rup(Cout, 64) < rup(Cout, 128) ? 64 : 128;
}

// act 0 none / 1 SiLU / 2 sigmoid; res_mode 0 / 1 bf16 (after act) / 2 f32 x rscale
inline int conv(const ConvCtx& cx, const ConvW& L, const void* x, long ldx, int n, int H, int W, int stride, void* out,
                long ldo, hipStream_t s, int act = 1, int out_f32 = 0, int res_mode = 0, const void* res = nullptr,
                long ldr = 0, const float* rscale = nullptr) {
  ConvLaunch c{};
  c.x = x;
  c.ldx = ldx;
  c.w = L.w;
  c.bias = L.b;
  c.out = out;
  c.ldo = ldo;
  c.res = res;
  c.ldr = ldr;
  c.rscale = rscale;
  c.zero = cx.zero;
  c.n_img = n;
  c.H = H;
  c.W = W;
  c.Cin = L.Cinp;
  c.KH = L.KH;
  c.KW = L.KW;
  c.stride = stride;
  c.pad = L.KH / 2;
  c.Kp = L.Kp;
  c.Cout = L.Cout;
  c.Npad = L.Npad;
  c.act = act;
  c.out_f32 = out_f32;
  c.res_mode = res_mode;
  c.tn = conv_tile_n(L.Cout);
  if (cx.tune && cx.tune->enabled() && out != x && (res == nullptr || res != out)) {
    const std::array<long, 10> key = {H, W, L.Cinp, L.Cout, L.KH, stride, act, out_f32, res_mode, ldo};
    VGE_HIPCHK(conv_tuned_launch(*cx.tune, c, key, s));
  } else {
    VGE_HIPCHK(launch_conv_bf16(c, s));
  }
  const int Ho = (H + 2 * c.pad - L.KH) / stride + 1, Wo = (W + 2 * c.pad - L.KW) / stride + 1;
  if (cx.flops) *cx.flops += 2.0 * n * Ho * Wo * (double)L.Cout * L.KH * L.KW * L.Cin;
  return VGE_OK;
}

// event pairs around launches, by kind (per-call profiling of a model's forward)
struct Profiler {
  std::vector<hipEvent_t> ev;
  std::vector<int> kind;
  int max_calls = 0, calls = 0, per_call = 0;
  size_t pair = 0;
  bool on = false;
  double flops = 0;  // algorithmic GEMM FLOPs of the recorded calls (calls differ in size: a pass's tail)
  ~Profiler() {
    for (auto e : ev) (void)hipEventDestroy(e);
  }
  int begin(int n_calls, int pairs_per_call) {
    for (auto e : ev) (void)hipEventDestroy(e);
    per_call = pairs_per_call;
    ev.assign((size_t)n_calls * per_call * 2, nullptr);
    kind.assign((size_t)n_calls * per_call, -1);
    for (auto& e : ev) VGE_HIPCHK(hipEventCreate(&e));
    max_calls = n_calls;
    calls = 0;
    flops = 0;
    return VGE_OK;
  }
  void start_call() {
    on = calls < max_calls;
    pair = on ? (size_t)calls * per_call : 0;
  }
  void end_call(double call_flops) {
    if (on) ++calls, flops += call_flops;
    on = false;
  }
  double flops_per_call(double fallback) const { return calls ? flops / calls : fallback; }
  int beg(int k, hipStream_t s) {
    if (on && pair < (size_t)(calls + 1) * per_call) {
      kind[pair] = k;
      VGE_HIPCHK(hipEventRecord(ev[2 * pair], s));
    }
    return VGE_OK;
  }
  int end(hipStream_t s) {
    if (on && pair < (size_t)(calls + 1) * per_call) VGE_HIPCHK(hipEventRecord(ev[2 * pair++ + 1], s));
    return VGE_OK;
  }
  int read(double* ms, int n_kinds, int* n_calls) {
    for (int i = 0; i < n_kinds; ++i) ms[i] = 0;
    for (size_t p = 0; p < (size_t)calls * per_call; ++p) {
      if (kind[p] < 0) continue;
      float t;
      VGE_HIPCHK(hipEventSynchronize(ev[2 * p + 1]));
      VGE_HIPCHK(hipEventElapsedTime(&t, ev[2 * p], ev[2 * p + 1]));
      ms[kind[p]] += t;
    }
    *n_calls = calls;
    return VGE_OK;
  }
};

}  // namespace cnnh
}  // namespace vge
