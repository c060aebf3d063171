// C ABI of the DWPose keypoint extractor (include/vge_dwpose.h): BatchNorm folding and NHWC weight packing at
// load time, workspace, per-frame instance table (persons 0 and 1), and the launch sequence of one batched
// RTMPose-l whole-body forward.  Kernels: vge_cnn.hip (convolutions, prep), vge_pose_head.hip (head, decode).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/vge_dwpose.h"
#include "vge_cnn.h"
#include "vge_cnn_host.h"

using namespace vge::cnnh;
#define HIPCHK VGE_HIPCHK

namespace {

constexpr float BN_EPS = 1e-5f;  // mmpose RTMPose configs: SyncBN, default eps

struct DwW {  // depthwise: f32 [K*K][C] + bias
  float* w = nullptr;
  float* b = nullptr;
  int C = 0, K = 0;
};
struct AttW {  // ChannelAttention fc: f32 W^T [C][C] + bias
  float* Wt = nullptr;
  float* b = nullptr;
  int C = 0;
};
struct CspW {
  ConvW ms, fin;  // ms = main_conv | short_conv fused along Cout (cat order)
  std::vector<ConvW> c1, pw;
  std::vector<DwW> dw;
  AttW att;
  bool add = true;
};
struct StageW {
  ConvW down, spp1, spp2;
  bool spp = false;
  CspW csp;
};

}  // namespace

struct vge_dwpose {
  vge_rtmpose_config c{};
  DevAllocs dev;
  ConvW stem[3];
  StageW st[4];
  ConvW fin, mlp, uv, o, cls;
  float *gamma = nullptr, *beta = nullptr, *rscale = nullptr;
  float mlp_g = 1.f, ln_g = 1.f;
  void* zero = nullptr;
  int hw = 0, hwp = 0;  // head feature map positions (in_h/32 * in_w/32) and their padded row width
  // workspace
  int max_inst = 0;
  size_t act_elems = 0;  // per buffer (bf16 elements)
  void *in = nullptr, *X = nullptr, *D = nullptr, *SPP = nullptr, *CAT = nullptr, *Ma = nullptr, *Mb = nullptr,
       *T1 = nullptr, *T2 = nullptr;
  float *mean = nullptr, *att = nullptr;
  float *hf = nullptr, *hx = nullptr, *uvb = nullptr, *logits = nullptr, *lv = nullptr;
  void *ha = nullptr, *hxn = nullptr, *go = nullptr, *hy = nullptr;
  void *winst = nullptr, *pinst = nullptr;
  int* iof = nullptr;
  std::vector<vge::WarpInst> h_w;
  std::vector<vge::PoseInst> h_p;
  std::vector<int> h_iof;
  void *pin_w = nullptr, *pin_p = nullptr, *pin_iof = nullptr;  // pinned staging of the instance tables
  hipEvent_t staged = nullptr;                                   // their last copies to the device
  // profiling
  std::vector<hipEvent_t> ev;
  std::vector<int> ev_kind;
  int prof_max = 0, prof_calls = 0, ev_per_call = 0;
  double gemm_flops = 0, prof_flops = 0;  // prof_flops: summed over the recorded calls (instance counts differ)
  ~vge_dwpose() {
    for (auto e : ev) (void)hipEventDestroy(e);
    if (staged) (void)hipEventSynchronize(staged), (void)hipEventDestroy(staged);
    for (void* p : {pin_w, pin_p, pin_iof})
      if (p) (void)hipHostFree(p);
  }
  void* dmalloc(size_t bytes) { return dev.dmalloc(bytes); }
  ConvTuner tuner;  // per-layer conv variant, measured on first use
  ConvCtx cx() { return ConvCtx{zero, &gemm_flops, &tuner}; }
};

namespace {

// Two passes over the same load sequence: dry (key / shape checks only, no device work) then real (upload).
struct Loader {
  vge_dwpose* m;
  WeightMap& wm;
  bool dry = false;
  bool ok = true;
  void convmod(const std::string& p, int Cin, int Cout, int K, ConvW& L, int Cinp = 0) {
    std::vector<float> W, b;
    if (!ok || !fold(wm, p, Cout, Cin, K, BN_EPS, W, b)) return (void)(ok = false);
    if (dry) return;
    ok = pack_conv(m->dev, W.data(), b.data(), Cout, Cin, Cinp ? Cinp : Cin, K, K, L);
  }
  void convpair(const std::string& p0, const std::string& p1, int Cin, int Cout, ConvW& L) {  // 1x1 pair
    std::vector<float> W, b;
    if (!ok || !fold_pair(wm, p0, p1, Cout, Cin, 1, BN_EPS, W, b)) return (void)(ok = false);
    if (dry) return;
    ok = pack_conv(m->dev, W.data(), b.data(), 2 * Cout, Cin, Cin, 1, 1, L);
  }
  void dwmod(const std::string& p, int C, int K, DwW& L) {
    std::vector<float> W, b;
    if (!ok || !fold(wm, p, C, 1, K, BN_EPS, W, b)) return (void)(ok = false);
    if (dry) return;
    std::vector<float> t((size_t)K * K * C);
    for (int c = 0; c < C; ++c)
      for (int i = 0; i < K * K; ++i) t[(size_t)i * C + c] = W[(size_t)c * K * K + i];
    L.C = C;
    L.K = K;
    ok = upload(m->dev, t, &L.w) && upload(m->dev, b, &L.b);
  }
  void attn(const std::string& p, int C, AttW& L) {
    const vge_tensor_view* w = wm.get(p + ".fc.weight", {C, C, 1, 1});
    const vge_tensor_view* b = wm.get(p + ".fc.bias", {C});
    if (!ok || !w || !b) return (void)(ok = false);
    if (dry) return;
    std::vector<float> t((size_t)C * C), bb(b->data, b->data + C);
    for (int c = 0; c < C; ++c)
      for (int k = 0; k < C; ++k) t[(size_t)k * C + c] = w->data[(size_t)c * C + k];
    L.C = C;
    ok = upload(m->dev, t, &L.Wt) && upload(m->dev, bb, &L.b);
  }
  void linear(const std::string& k, int N, int K, int Kpow2, ConvW& L) {  // no bias, as a 1x1 conv
    const vge_tensor_view* w = wm.get(k, {N, K});
    if (!ok || !w) return (void)(ok = false);
    if (dry) return;
    ok = pack_conv(m->dev, w->data, nullptr, N, K, Kpow2, 1, 1, L);
  }
  void vec(const std::string& k, std::initializer_list<int64_t> shape, size_t npad, float** out) {
    const vge_tensor_view* t = wm.get(k, shape);
    if (!ok || !t) return (void)(ok = false);
    if (dry) return;
    size_t n = 1;
    for (int64_t s : shape) n *= (size_t)s;
    std::vector<float> h(std::max(n, npad), 0.f);
    memcpy(h.data(), t->data, n * 4);
    ok = upload(m->dev, h, out);
  }
  float scalar(const std::string& k) {
    const vge_tensor_view* t = wm.get(k, {1});
    if (!ok || !t) return (ok = false), 0.f;
    return t->data[0];
  }
};

bool cfg_ok(const vge_rtmpose_config& c, std::string& why) {
  if (c.in_h <= 0 || c.in_w <= 0 || c.in_h % 32 || c.in_w % 32) return why = "in_h / in_w must be multiples of 32", false;
  if (!pow2(c.stem_ch) || c.stem_ch < 16) return why = "stem_ch must be a power of two >= 16", false;
  for (int i = 0; i < 4; ++i) {
    if (!pow2(c.stage_ch[i]) || c.stage_ch[i] < 16 || c.stage_ch[i] > 2048)
      return why = "stage_ch must be powers of two in [16, 2048]", false;
    if (c.stage_blocks[i] < 0) return why = "stage_blocks must be >= 0", false;
  }
  if (c.keypoints < 133 || c.keypoints > 136)
    return why = "keypoints must be 133..136 (COCO-WholeBody indices feed the 120-d row)", false;
  if (!pow2(c.gau_hidden) || c.gau_hidden > 512 || !pow2(c.gau_e) || c.gau_e < 128 || c.gau_s <= 0 ||
      c.gau_s > 256 || c.gau_s % 8)
    return why = "gau_hidden / gau_e powers of two (hidden <= 512, e >= 128), gau_s % 8 == 0 and <= 256", false;
  if (c.final_k <= 0 || c.final_k % 2 == 0 || c.final_k > 9) return why = "final_k must be odd and <= 9", false;
  if (c.split <= 0) return why = "split must be positive", false;
  const int hw = (c.in_h / 32) * (c.in_w / 32);
  if (hw > 256) return why = "head feature map must have <= 256 positions", false;
  return true;
}

}  // namespace

namespace {
std::string I(int i) { return std::to_string(i); }
}  // namespace

namespace {
void load_all(Loader& ld, const vge_rtmpose_config& c) {
  vge_dwpose* m = ld.m;
  WeightMap& wm = ld.wm;
  const int s0 = c.stem_ch;
  ld.convmod("backbone.stem.0", 3, s0 / 2, 3, m->stem[0], 8);  // the prepared input carries 8 channels (3 used)
  ld.convmod("backbone.stem.1", s0 / 2, s0 / 2, 3, m->stem[1]);
  ld.convmod("backbone.stem.2", s0 / 2, s0, 3, m->stem[2]);
  int cin = s0;
  for (int i = 0; i < 4 && ld.ok; ++i) {
    const int C = c.stage_ch[i], mid = C / 2;
    const std::string p = "backbone.stage" + I(i + 1);
    StageW& S = m->st[i];
    ld.convmod(p + ".0", cin, C, 3, S.down);
    int j = 1;
    if (i == 3) {
      S.spp = true;
      ld.convmod(p + ".1.conv1", C, C / 2, 1, S.spp1);
      ld.convmod(p + ".1.conv2", (C / 2) * 4, C, 1, S.spp2);
      j = 2;
    }
    const std::string q = p + "." + I(j);
    CspW& L = S.csp;
    L.add = i < 3;
    ld.convpair(q + ".main_conv", q + ".short_conv", C, mid, L.ms);
    ld.convmod(q + ".final_conv", 2 * mid, C, 1, L.fin);
    L.c1.resize(c.stage_blocks[i]);
    L.pw.resize(c.stage_blocks[i]);
    L.dw.resize(c.stage_blocks[i]);
    for (int b = 0; b < c.stage_blocks[i]; ++b) {
      const std::string bp = q + ".blocks." + I(b);
      ld.convmod(bp + ".conv1", mid, mid, 3, L.c1[b]);
      ld.dwmod(bp + ".conv2.depthwise_conv", mid, 5, L.dw[b]);
      ld.convmod(bp + ".conv2.pointwise_conv", mid, mid, 1, L.pw[b]);
    }
    ld.attn(q + ".attention", 2 * mid, L.att);
    cin = C;
  }
  // head
  const int K = c.keypoints, H = c.gau_hidden, E = c.gau_e, Sg = c.gau_s, fk = c.final_k;
  m->hw = (c.in_h / 32) * (c.in_w / 32);
  m->hwp = pow2_at_least(m->hw, 8);
  if (ld.ok) {
    const vge_tensor_view* w = wm.get("head.final_layer.weight", {K, cin, fk, fk});
    const vge_tensor_view* b = wm.get("head.final_layer.bias", {K});
    ld.ok = w && b && (ld.dry || pack_conv(m->dev, w->data, b->data, K, cin, cin, fk, fk, m->fin));
  }
  m->mlp_g = ld.scalar("head.mlp.0.g");
  ld.linear("head.mlp.1.weight", H, m->hw, m->hwp, m->mlp);
  m->ln_g = ld.scalar("head.gau.ln.g");
  ld.linear("head.gau.uv.weight", 2 * E + Sg, H, H, m->uv);
  ld.linear("head.gau.o.weight", H, E, E, m->o);
  ld.vec("head.gau.gamma", {2, Sg}, 0, &m->gamma);
  ld.vec("head.gau.beta", {2, Sg}, 0, &m->beta);
  ld.vec("head.gau.res_scale.scale", {H}, (size_t)rup(H, 128), &m->rscale);
  {
    const int WX = c.split * c.in_w, WY = c.split * c.in_h;
    const vge_tensor_view* wx = wm.get("head.cls_x.weight", {WX, H});
    const vge_tensor_view* wy = wm.get("head.cls_y.weight", {WY, H});
    if (ld.ok && wx && wy && !ld.dry) {
      std::vector<float> Wc((size_t)(WX + WY) * H);
      memcpy(Wc.data(), wx->data, (size_t)WX * H * 4);
      memcpy(Wc.data() + (size_t)WX * H, wy->data, (size_t)WY * H * 4);
      ld.ok = pack_conv(m->dev, Wc.data(), nullptr, WX + WY, H, H, 1, 1, m->cls);
    } else if (!wx || !wy) {
      ld.ok = false;
    }
  }
  if (ld.ok && !ld.dry) {
    std::vector<uint16_t> z(128, 0);
    uint16_t* zp = nullptr;
    ld.ok = upload(m->dev, z, &zp);
    m->zero = zp;
  }
}

}  // namespace

extern "C" {

int vge_dwpose_create(const vge_rtmpose_config* cfg, const vge_tensor_view* weights, int n_weights, vge_dwpose** out) {
  if (!cfg || !out || (n_weights > 0 && !weights)) return fail(VGE_ERR_ARG, "vge_dwpose_create: null argument");
  *out = nullptr;
  std::string why;
  if (!cfg_ok(*cfg, why)) return fail(VGE_ERR_ARG, "vge_dwpose_create: unsupported config: " + why);
  const vge_rtmpose_config c = *cfg;
  WeightMap wm(weights, n_weights);
  auto* m = new vge_dwpose();
  m->tuner.lib = pose_gemm_lib();
  m->c = c;
  bool ok_all = true;
  for (int pass = 0; pass < 2 && ok_all; ++pass) {
    Loader ld{m, wm, pass == 0};
    load_all(ld, c);
    ok_all = ld.ok;
  }
  if (!ok_all) {
    delete m;
    return wm.status("vge_dwpose_create");
  }
  *out = m;
  return VGE_OK;
}

int vge_dwpose_reserve(vge_dwpose* m, int max_inst) {
  if (!m || max_inst <= 0) return fail(VGE_ERR_ARG, "vge_dwpose_reserve: bad argument");
  if (max_inst <= m->max_inst) return VGE_OK;
  const vge_rtmpose_config& c = m->c;
  // largest activation per instance: every tensor of the backbone is at most this many bf16 elements
  size_t per = (size_t)(c.in_h / 2) * (c.in_w / 2) * c.stem_ch;
  int h = c.in_h / 2, w = c.in_w / 2;
  for (int i = 0; i < 4; ++i) {
    h = (h + 1) / 2;
    w = (w + 1) / 2;
    per = std::max(per, (size_t)h * w * c.stage_ch[i] * (i == 3 ? 2 : 1));  // SPP concat = 2 C
  }
  const size_t N = (size_t)max_inst, K = c.keypoints, rows = N * K;
  const int WXY = c.split * (c.in_w + c.in_h);
  struct B { void** p; size_t bytes; };
  const B bufs[] = {
      {&m->in, N * c.in_h * c.in_w * 8 * 2},
      {&m->X, N * per * 2}, {&m->D, N * per * 2}, {&m->SPP, N * per * 2}, {&m->CAT, N * per * 2},
      {&m->Ma, N * per * 2}, {&m->Mb, N * per * 2}, {&m->T1, N * per * 2}, {&m->T2, N * per * 2},
      {(void**)&m->mean, N * 2048 * 4}, {(void**)&m->att, N * 2048 * 4},
      {(void**)&m->hf, N * m->hw * rup(c.keypoints, 8) * 4},
      {&m->ha, rows * m->hwp * 2},
      {(void**)&m->hx, rows * c.gau_hidden * 4},
      {&m->hxn, rows * c.gau_hidden * 2},
      {(void**)&m->uvb, rows * (2 * c.gau_e + c.gau_s) * 4},
      {&m->go, rows * c.gau_e * 2},
      {&m->hy, rows * c.gau_hidden * 2},
      {(void**)&m->logits, rows * WXY * 4},
      {(void**)&m->lv, rows * 3 * 4},
      {&m->winst, N * sizeof(vge::WarpInst)},
      {&m->pinst, N * sizeof(vge::PoseInst)},
      {(void**)&m->iof, N * 2 * sizeof(int)},
  };
  if (!m->staged) HIPCHK(hipEventCreateWithFlags(&m->staged, hipEventDisableTiming));
  HIPCHK(hipEventSynchronize(m->staged));
  for (void* p : {m->pin_w, m->pin_p, m->pin_iof})
    if (p) HIPCHK(hipHostFree(p));
  HIPCHK(hipHostMalloc(&m->pin_w, N * sizeof(vge::WarpInst)));
  HIPCHK(hipHostMalloc(&m->pin_p, N * sizeof(vge::PoseInst)));
  HIPCHK(hipHostMalloc(&m->pin_iof, N * 2 * sizeof(int)));
  for (const B& b : bufs) {
    void* p = m->dmalloc(b.bytes);
    if (!p) return fail(VGE_ERR_NOMEM, "vge_dwpose_reserve: hipMalloc failed");
    HIPCHK(hipMemset(p, 0, b.bytes));
    *b.p = p;
  }
  m->act_elems = N * per;
  m->max_inst = max_inst;
  return VGE_OK;
}

int vge_dwpose_destroy(vge_dwpose* m) {
  delete m;
  return VGE_OK;
}

int vge_dwpose_profile_begin(vge_dwpose* m, int max_calls) {
  if (!m || max_calls < 0) return fail(VGE_ERR_ARG, "vge_dwpose_profile_begin: bad argument");
  for (auto e : m->ev) (void)hipEventDestroy(e);
  m->ev_per_call = 2 * 512;
  m->ev.assign((size_t)max_calls * m->ev_per_call, nullptr);
  m->ev_kind.assign((size_t)max_calls * m->ev_per_call / 2, -1);
  for (auto& e : m->ev) HIPCHK(hipEventCreate(&e));
  m->prof_max = max_calls;
  m->prof_calls = 0;
  m->prof_flops = 0;
  return VGE_OK;
}

int vge_dwpose_profile_read(vge_dwpose* m, double* stage_ms, int* n_calls, double* gemm_flops_per_call) {
  if (!m || !stage_ms || !n_calls) return fail(VGE_ERR_ARG, "vge_dwpose_profile_read: bad argument");
  for (int i = 0; i < 3; ++i) stage_ms[i] = 0;
  for (size_t p = 0; p < (size_t)m->prof_calls * m->ev_per_call / 2; ++p) {
    if (m->ev_kind[p] < 0) continue;
    float t;
    HIPCHK(hipEventSynchronize(m->ev[2 * p + 1]));
    HIPCHK(hipEventElapsedTime(&t, m->ev[2 * p], m->ev[2 * p + 1]));
    stage_ms[m->ev_kind[p]] += t;
  }
  *n_calls = m->prof_calls;
  if (gemm_flops_per_call) *gemm_flops_per_call = m->prof_calls ? m->prof_flops / m->prof_calls : m->gemm_flops;
  return VGE_OK;
}

int vge_dwpose_keypoints(vge_dwpose* m, const uint8_t* frames, int F, int H, int W, const float* boxes,
                         int max_persons, const int* n_persons, float* keypoints, float* simcc, float* lv_out,
                         vge_stream_t stream) {
  if (!m || F < 0 || (F > 0 && (!frames || !n_persons || !keypoints || H <= 0 || W <= 0)) || max_persons < 0)
    return fail(VGE_ERR_ARG, "vge_dwpose_keypoints: bad argument");
  if (F == 0) return VGE_OK;
  const vge_rtmpose_config& c = m->c;
  // ---- instance table: persons 0 and 1 of every frame (no person -> the whole frame, onnxpose.preprocess)
  m->h_w.clear();
  m->h_p.clear();
  m->h_iof.assign((size_t)2 * F, -1);
  auto add = [&](int f, float x0, float y0, float x1, float y1) {
#pragma clang fp contract(off)
    const float cx = (x0 + x1) * 0.5f, cy = (y0 + y1) * 0.5f;
    const float w = (x1 - x0) * 1.25f, h = (y1 - y0) * 1.25f;
    const float ar = (float)c.in_w / (float)c.in_h;
    float sw, sh;
    if (w > h * ar) {
      sw = w;
      sh = w / ar;
    } else {
      sw = h * ar;
      sh = h;
    }
    m->h_w.push_back({f, cx, cy, sw / (float)c.in_w});
    m->h_p.push_back({cx, cy, sw, sh});
  };
  for (int f = 0; f < F; ++f) {
    const int n = n_persons[f];
    if (n < 0 || (n > 0 && (!boxes || n > max_persons))) return fail(VGE_ERR_ARG, "vge_dwpose_keypoints: bad n_persons");
    if (n == 0) {
      m->h_iof[2 * f] = (int)m->h_w.size();
      add(f, 0.f, 0.f, (float)W, (float)H);
      continue;
    }
    for (int p = 0; p < std::min(n, 2); ++p) {
      const float* b = boxes + ((size_t)f * max_persons + p) * 4;
      m->h_iof[2 * f + p] = (int)m->h_w.size();
      add(f, b[0], b[1], b[2], b[3]);
    }
  }
  const int N = (int)m->h_w.size();
  if (N > m->max_inst) return fail(VGE_ERR_WORKSPACE, "vge_dwpose_keypoints: call vge_dwpose_reserve(>= instances)");
  hipStream_t s = S(stream);
  // instance tables -> pinned staging (the previous call's copies must have read it) -> device.  F <= N because
  // every frame has at least one instance, so the frame map fits the max_inst-sized buffers.
  HIPCHK(hipEventSynchronize(m->staged));
  memcpy(m->pin_w, m->h_w.data(), N * sizeof(vge::WarpInst));
  memcpy(m->pin_p, m->h_p.data(), N * sizeof(vge::PoseInst));
  memcpy(m->pin_iof, m->h_iof.data(), (size_t)2 * F * sizeof(int));
  HIPCHK(hipMemcpyAsync(m->winst, m->pin_w, N * sizeof(vge::WarpInst), hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(m->pinst, m->pin_p, N * sizeof(vge::PoseInst), hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(m->iof, m->pin_iof, (size_t)2 * F * sizeof(int), hipMemcpyHostToDevice, s));
  HIPCHK(hipEventRecord(m->staged, s));
  const bool prof = m->prof_calls < m->prof_max;
  size_t pair = prof ? (size_t)m->prof_calls * m->ev_per_call / 2 : 0;
  auto beg = [&](int kind) -> int {
    if (prof) {
      m->ev_kind[pair] = kind;
      HIPCHK(hipEventRecord(m->ev[2 * pair], s));
    }
    return VGE_OK;
  };
  auto end = [&]() -> int {
    if (prof) HIPCHK(hipEventRecord(m->ev[2 * pair++ + 1], s));
    return VGE_OK;
  };
  m->gemm_flops = 0;
  int rc;
#define RC(x)                            \
  do {                                   \
    if ((rc = (x)) != VGE_OK) return rc; \
  } while (0)
#define CONV(...)            \
  do {                       \
    RC(beg(0));              \
    RC(conv(m->cx(), __VA_ARGS__)); \
    RC(end());               \
  } while (0)
#define OTHER(kind, expr) \
  do {                    \
    RC(beg(kind));        \
    HIPCHK(expr);         \
    RC(end());            \
  } while (0)
  OTHER(1, vge::launch_warp_prep(frames, H, W, m->winst, N, c.in_h, c.in_w, m->in, s));
  int h = c.in_h / 2, w = c.in_w / 2;
  const int s0 = c.stem_ch;
  CONV(m->stem[0], m->in, 8, N, c.in_h, c.in_w, 2, m->T1, s0 / 2, s);
  CONV(m->stem[1], m->T1, s0 / 2, N, h, w, 1, m->T2, s0 / 2, s);
  CONV(m->stem[2], m->T2, s0 / 2, N, h, w, 1, m->X, s0, s);
  int cin = s0;
  for (int i = 0; i < 4; ++i) {
    const StageW& St = m->st[i];
    const int C = c.stage_ch[i], mid = C / 2;
    CONV(St.down, m->X, cin, N, h, w, 2, m->D, C, s);
    h = (h + 1) / 2;
    w = (w + 1) / 2;
    const void* src = m->D;
    if (St.spp) {
      CONV(St.spp1, m->D, C, N, h, w, 1, m->SPP, 2 * C, s);
      OTHER(1, vge::launch_spp_pool(m->SPP, 2 * C, N, h, w, C / 2, 5, 9, 13, s));
      CONV(St.spp2, m->SPP, 2 * C, N, h, w, 1, m->X, C, s);
      src = m->X;
    }
    const CspW& L = St.csp;
    uint16_t* cat = static_cast<uint16_t*>(m->CAT);  // bf16 NHWC, (main | short) channel halves
    CONV(L.ms, src, C, N, h, w, 1, cat, C, s);  // [main | short] straight into the concat buffer
    const int nb = (int)L.c1.size();
    const void* Ma = cat;  // current main branch and its pixel stride
    long lda = C;
    void* scratch[2] = {m->Ma, m->Mb};
    for (int b = 0; b < nb; ++b) {
      CONV(L.c1[b], Ma, lda, N, h, w, 1, m->T1, mid, s);
      OTHER(1, vge::launch_dwconv(m->T1, mid, L.dw[b].w, L.dw[b].b, m->T2, mid, N, h, w, mid, 5, s));
      const bool last = b == nb - 1;
      void* out = last ? (void*)cat : scratch[b & 1];
      const long ldo = last ? C : mid;
      CONV(L.pw[b], m->T2, mid, N, h, w, 1, out, ldo, s, 1, 0, L.add ? 1 : 0, L.add ? Ma : nullptr, lda);
      Ma = out;
      lda = ldo;
    }
    OTHER(1, vge::launch_chan_attn(cat, C, N, h * w, C, L.att.Wt, L.att.b, m->mean, m->att, s));
    CONV(L.fin, cat, C, N, h, w, 1, m->X, C, s);
    cin = C;
  }
  // ---- RTMCCHead
  const int K = c.keypoints, Hd = c.gau_hidden, E = c.gau_e, Sg = c.gau_s;
  const int WX = c.split * c.in_w, WY = c.split * c.in_h;
  const long rows = (long)N * K;
  const int ldf = rup(K, 8);
  CONV(m->fin, m->X, cin, N, h, w, 1, m->hf, ldf, s, 0, 1);
  OTHER(2, vge::launch_head_sn_t(m->hf, ldf, m->hw, K, m->hwp, m->mlp_g, rows, m->ha, s));
  CONV(m->mlp, m->ha, m->hwp, (int)rows, 1, 1, 1, m->hx, Hd, s, 0, 1);
  OTHER(2, vge::launch_scalenorm_rows(m->hx, Hd, m->ln_g, rows, m->hxn, s));
  CONV(m->uv, m->hxn, Hd, (int)rows, 1, 1, 1, m->uvb, 2 * E + Sg, s, 1, 1);
  OTHER(2, vge::launch_gau_attn(m->uvb, N, K, E, Sg, m->gamma, m->beta, m->go, s));
  CONV(m->o, m->go, E, (int)rows, 1, 1, 1, m->hy, Hd, s, 0, 0, 2, m->hx, Hd, m->rscale);
  float* logits = simcc ? simcc : m->logits;
  CONV(m->cls, m->hy, Hd, (int)rows, 1, 1, 1, logits, WX + WY, s, 0, 1);
  float* lv = lv_out ? lv_out : m->lv;
  OTHER(2, vge::launch_simcc_decode(logits, WX + WY, WX, WY, (float)c.split, rows, lv, s));
  OTHER(2, vge::launch_kp120(lv, m->pinst, m->iof, F, K, c.in_w, c.in_h, H, W, keypoints, s));
#undef OTHER
#undef CONV
#undef RC
  if (prof) ++m->prof_calls, m->prof_flops += m->gemm_flops;
  return VGE_OK;
}

// ------------------------------------------------------------------ op-level entry point (tests)
int vge_op_conv_bf16(const void* x, long ldx, const void* w, const float* bias, void* out, long ldo, const void* res,
                     long ldr, const float* rscale, int n_img, int H, int W, int Cin, int KH, int KW, int stride,
                     int pad, int Cout, int act, int out_f32, int res_mode, vge_stream_t stream) {
  static void* zero = nullptr;
  if (!x || !w || !bias || !out || n_img <= 0 || H <= 0 || W <= 0 || !pow2(Cin) || Cin < 8 || KH <= 0 || KW <= 0 ||
      KW > 16 || stride <= 0 || pad < 0 || Cout <= 0 || act < 0 || act > 3 || out_f32 < 0 || out_f32 > 1 ||
      res_mode < 0 || res_mode > 3 || (res_mode == 1 && ((act != 1 && act != 0) || out_f32)) || (res_mode == 2 && (act || out_f32)) ||
      (res_mode == 3 && ((act != 0 && act != 3) || out_f32)) || (act == 3 && out_f32) ||
      (act == 2 && !out_f32) || ldx < Cin || ldx % 8 || ldo < Cout || (!out_f32 && (Cout % 8 || ldo % 8)) ||
      (res_mode && (!res || ldr < Cout)) || (res_mode == 2 && !rscale))
    return fail(VGE_ERR_ARG, "vge_op_conv_bf16: unsupported shape / arguments");
  if (!zero) {
    HIPCHK(hipMalloc(&zero, 256));
    HIPCHK(hipMemset(zero, 0, 256));
  }
  vge::ConvLaunch c{};
  c.x = x; c.ldx = ldx; c.w = w; c.bias = bias; c.out = out; c.ldo = ldo; c.res = res; c.ldr = ldr; c.rscale = rscale;
  c.zero = zero; c.n_img = n_img; c.H = H; c.W = W; c.Cin = Cin; c.KH = KH; c.KW = KW; c.stride = stride; c.pad = pad;
  c.Kp = rup(KH * KW * Cin, 32); c.Cout = Cout; c.Npad = rup(Cout, 256); c.act = act; c.out_f32 = out_f32;
  c.res_mode = res_mode; c.tn = conv_tile_n(Cout);
  HIPCHK(vge::launch_conv_bf16(c, S(stream)));
  return VGE_OK;
}

}  // extern "C"
