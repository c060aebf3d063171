// C ABI of DWPose's YOLOX person detector (include/vge_dwpose.h, vge_yolox_*): BatchNorm folding / NHWC weight
// packing, workspace, and the launch sequence of one chunk: letterbox + Focus -> CSPDarknet -> YOLOPAFPN ->
// decoupled head (person class only) -> decode + two-person NMS.  Concats are free: every producer writes its
// channel slice of the concatenated buffer (pixel stride = the concat width).
#include <hip/hip_runtime.h>

#include "../../include/vge_dwpose.h"
#include "vge_cnn.h"
#include "vge_cnn_host.h"

using namespace vge::cnnh;
#define HIPCHK VGE_HIPCHK

namespace {

constexpr float BN_EPS = 1e-3f;  // YOLOX init_yolo: BatchNorm eps 1e-3

struct YCsp {  // YOLOX CSPLayer: conv1 | conv2 (one fused 1x1 -> [x_1 | x_2]), n Bottlenecks (1x1, 3x3 [+x]), conv3
  ConvW c12, c3;
  std::vector<ConvW> m1, m2;
  bool shortcut = false;
  int hid = 0;
};
struct YHead {
  ConvW stem, first, cls1, reg1, regobj, cls0;  // first = cls_convs.0 | reg_convs.0 fused along Cout
};

std::string I(int i) { return std::to_string(i); }

}  // namespace

struct vge_yolox {
  vge_yolox_config c{};
  DevAllocs dev;
  ConvW stem, d2, d3, d4, d5, spp1, spp2, lat0, red1, bu2, bu1;
  YCsp c2, c3, c4, c5, p4, p3, n3, n4;
  YHead head[3];
  void* zero = nullptr;
  int chunk = 0;
  void *in = nullptr, *A = nullptr, *B = nullptr, *X2b = nullptr, *CAT = nullptr, *Ma = nullptr, *Mb = nullptr,
       *T = nullptr, *Cat8 = nullptr, *Cat16 = nullptr, *Pcat16 = nullptr, *Pcat32 = nullptr, *SPP = nullptr,
       *B2 = nullptr, *X0 = nullptr, *F0 = nullptr, *PAN[3] = {nullptr, nullptr, nullptr}, *HS = nullptr,
       *HB = nullptr, *CF = nullptr, *RF = nullptr;
  float* OUT[3] = {nullptr, nullptr, nullptr};
  Profiler prof;
  double gemm_flops = 0;
  ConvTuner tuner;  // per-layer conv variant, measured on first use
  ConvCtx cx() { return ConvCtx{zero, &gemm_flops, &tuner}; }
};

namespace {

struct YLoader {
  vge_yolox* m;
  WeightMap& wm;
  bool dry;
  bool ok = true;
  void base(const std::string& p, int Cin, int Cout, int K, ConvW& L, int Cinp = 0) {
    std::vector<float> W, b;
    if (!ok || !fold(wm, p, Cout, Cin, K, BN_EPS, W, b)) return (void)(ok = false);
    if (!dry) ok = pack_conv(m->dev, W.data(), b.data(), Cout, Cin, Cinp ? Cinp : Cin, K, K, L);
  }
  void csp(const std::string& p, int Cin, int Cout, int n, bool shortcut, YCsp& L) {
    const int hid = Cout / 2;
    L.hid = hid;
    L.shortcut = shortcut;
    {
      std::vector<float> W, b;
      if (!ok || !fold_pair(wm, p + ".conv1", p + ".conv2", hid, Cin, 1, BN_EPS, W, b)) return (void)(ok = false);
      if (!dry) ok = pack_conv(m->dev, W.data(), b.data(), 2 * hid, Cin, Cin, 1, 1, L.c12);
    }
    base(p + ".conv3", 2 * hid, Cout, 1, L.c3);
    L.m1.resize(n);
    L.m2.resize(n);
    for (int i = 0; i < n; ++i) {
      base(p + ".m." + I(i) + ".conv1", hid, hid, 1, L.m1[i]);
      base(p + ".m." + I(i) + ".conv2", hid, hid, 3, L.m2[i]);
    }
  }
  // cls_convs.k.0 and reg_convs.k.0 read the same stem output: one conv with both weight sets along Cout
  void fused_first(const std::string& k, int hc, ConvW& L) {
    std::vector<float> W0, b0, W1, b1;
    if (!ok || !fold(wm, "head.cls_convs." + k + ".0", hc, hc, 3, BN_EPS, W0, b0) ||
        !fold(wm, "head.reg_convs." + k + ".0", hc, hc, 3, BN_EPS, W1, b1))
      return (void)(ok = false);
    if (dry) return;
    W0.insert(W0.end(), W1.begin(), W1.end());
    b0.insert(b0.end(), b1.begin(), b1.end());
    ok = pack_conv(m->dev, W0.data(), b0.data(), 2 * hc, hc, hc, 3, 3, L);
  }
  // reg_preds (4) + obj_preds (1) as one 1x1 conv with bias; cls_preds row 0 as another
  void preds(const std::string& k, int hc, int nc, ConvW& regobj, ConvW& cls0) {
    const vge_tensor_view* rw = wm.get("head.reg_preds." + k + ".weight", {4, hc, 1, 1});
    const vge_tensor_view* rb = wm.get("head.reg_preds." + k + ".bias", {4});
    const vge_tensor_view* ow = wm.get("head.obj_preds." + k + ".weight", {1, hc, 1, 1});
    const vge_tensor_view* ob = wm.get("head.obj_preds." + k + ".bias", {1});
    const vge_tensor_view* cw = wm.get("head.cls_preds." + k + ".weight", {nc, hc, 1, 1});
    const vge_tensor_view* cb = wm.get("head.cls_preds." + k + ".bias", {nc});
    if (!ok || !rw || !rb || !ow || !ob || !cw || !cb) return (void)(ok = false);
    if (dry) return;
    std::vector<float> W((size_t)5 * hc), b(5);
    memcpy(W.data(), rw->data, (size_t)4 * hc * 4);
    memcpy(W.data() + (size_t)4 * hc, ow->data, (size_t)hc * 4);
    memcpy(b.data(), rb->data, 16);
    b[4] = ob->data[0];
    ok = pack_conv(m->dev, W.data(), b.data(), 5, hc, hc, 1, 1, regobj) &&
         pack_conv(m->dev, cw->data, cb->data, 1, hc, hc, 1, 1, cls0);
  }
};

void load_all(YLoader& ld, const vge_yolox_config& c) {
  vge_yolox* m = ld.m;
  const int w0 = c.width, d = c.depth, hc = c.head_ch;
  const std::string bb = "backbone.backbone.";
  ld.base(bb + "stem.conv", 12, w0, 3, m->stem, 16);  // Focus input: 12 channels carried as 16
  ld.base(bb + "dark2.0", w0, 2 * w0, 3, m->d2);
  ld.csp(bb + "dark2.1", 2 * w0, 2 * w0, d, true, m->c2);
  ld.base(bb + "dark3.0", 2 * w0, 4 * w0, 3, m->d3);
  ld.csp(bb + "dark3.1", 4 * w0, 4 * w0, 3 * d, true, m->c3);
  ld.base(bb + "dark4.0", 4 * w0, 8 * w0, 3, m->d4);
  ld.csp(bb + "dark4.1", 8 * w0, 8 * w0, 3 * d, true, m->c4);
  ld.base(bb + "dark5.0", 8 * w0, 16 * w0, 3, m->d5);
  ld.base(bb + "dark5.1.conv1", 16 * w0, 8 * w0, 1, m->spp1);
  ld.base(bb + "dark5.1.conv2", 32 * w0, 16 * w0, 1, m->spp2);
  ld.csp(bb + "dark5.2", 16 * w0, 16 * w0, d, false, m->c5);
  const int c3 = 4 * w0, c4 = 8 * w0, c5 = 16 * w0;
  ld.base("backbone.lateral_conv0", c5, c4, 1, m->lat0);
  ld.csp("backbone.C3_p4", 2 * c4, c4, d, false, m->p4);
  ld.base("backbone.reduce_conv1", c4, c3, 1, m->red1);
  ld.csp("backbone.C3_p3", 2 * c3, c3, d, false, m->p3);
  ld.base("backbone.bu_conv2", c3, c3, 3, m->bu2);
  ld.csp("backbone.C3_n3", 2 * c3, c4, d, false, m->n3);
  ld.base("backbone.bu_conv1", c4, c4, 3, m->bu1);
  ld.csp("backbone.C3_n4", 2 * c4, c5, d, false, m->n4);
  const int cin[3] = {c3, c4, c5};
  for (int k = 0; k < 3; ++k) {
    YHead& H = m->head[k];
    ld.base("head.stems." + I(k), cin[k], hc, 1, H.stem);
    ld.fused_first(I(k), hc, H.first);
    ld.base("head.cls_convs." + I(k) + ".1", hc, hc, 3, H.cls1);
    ld.base("head.reg_convs." + I(k) + ".1", hc, hc, 3, H.reg1);
    ld.preds(I(k), hc, c.num_classes, H.regobj, H.cls0);
  }
  if (ld.ok && !ld.dry) {
    std::vector<uint16_t> z(128, 0);
    uint16_t* zp = nullptr;
    ld.ok = upload(m->dev, z, &zp);
    m->zero = zp;
  }
}

bool cfg_ok(const vge_yolox_config& c, std::string& why) {
  if (c.in_size <= 0 || c.in_size % 32) return why = "in_size must be a multiple of 32", false;
  if (!pow2(c.width) || c.width < 8 || c.width > 128) return why = "width must be a power of two in [8, 128]", false;
  if (c.depth < 0) return why = "depth must be >= 0", false;
  if (!pow2(c.head_ch) || c.head_ch < 16 || c.head_ch > 512) return why = "head_ch must be a power of two <= 512", false;
  if (c.num_classes < 1) return why = "num_classes must be >= 1", false;
  return true;
}

// CSPLayer: out = conv3(cat(m(conv1(x)), conv2(x))); conv1 | conv2 write [x_1 | x_2] into the concat buffer and the
// last Bottleneck overwrites x_1 in place (its identity read and its store touch the same element)
int ycsp(vge_yolox* m, const YCsp& L, const void* x, long ldx, int n, int h, int w, void* out, long ldo, hipStream_t s,
         int& rc_kind) {
  (void)rc_kind;
  const int hid = L.hid, nb = (int)L.m1.size();
  uint16_t* cat = static_cast<uint16_t*>(m->CAT);
  int rc;
  if ((rc = conv(m->cx(), L.c12, x, ldx, n, h, w, 1, cat, 2 * hid, s)) != VGE_OK) return rc;
  const void* Ma = cat;
  long lda = 2 * hid;
  void* scratch[2] = {m->Ma, m->Mb};
  for (int b = 0; b < nb; ++b) {
    const bool last = b == nb - 1;
    void* o = last ? (void*)cat : scratch[b & 1];
    const long ldb = last ? 2 * hid : hid;
    if ((rc = conv(m->cx(), L.m1[b], Ma, lda, n, h, w, 1, m->T, hid, s)) != VGE_OK) return rc;
    if ((rc = conv(m->cx(), L.m2[b], m->T, hid, n, h, w, 1, o, ldb, s, 1, 0, L.shortcut ? 1 : 0,
                   L.shortcut ? Ma : nullptr, lda)) != VGE_OK)
      return rc;
    Ma = o;
    lda = ldb;
  }
  return conv(m->cx(), L.c3, cat, 2 * hid, n, h, w, 1, out, ldo, s);
}

}  // namespace

extern "C" {

int vge_yolox_create(const vge_yolox_config* cfg, const vge_tensor_view* weights, int n_weights, vge_yolox** out) {
  if (!cfg || !out || (n_weights > 0 && !weights)) return fail(VGE_ERR_ARG, "vge_yolox_create: null argument");
  *out = nullptr;
  std::string why;
  if (!cfg_ok(*cfg, why)) return fail(VGE_ERR_ARG, "vge_yolox_create: unsupported config: " + why);
  WeightMap wm(weights, n_weights);
  auto* m = new vge_yolox();
  m->tuner.lib = pose_gemm_lib();
  m->c = *cfg;
  bool ok = true;
  for (int pass = 0; pass < 2 && ok; ++pass) {
    YLoader ld{m, wm, pass == 0};
    load_all(ld, *cfg);
    ok = ld.ok;
  }
  if (!ok) {
    delete m;
    return wm.status("vge_yolox_create");
  }
  *out = m;
  return VGE_OK;
}

int vge_yolox_reserve(vge_yolox* m, int chunk) {
  if (!m || chunk <= 0) return fail(VGE_ERR_ARG, "vge_yolox_reserve: bad argument");
  if (chunk <= m->chunk) return VGE_OK;
  const vge_yolox_config& c = m->c;
  const size_t S = c.in_size, w0 = c.width, hc = c.head_ch, N = chunk;
  const size_t s2 = (S / 2) * (S / 2), s4 = (S / 4) * (S / 4), s8 = (S / 8) * (S / 8), s16 = (S / 16) * (S / 16),
               s32 = (S / 32) * (S / 32);
  struct B { void** p; size_t bytes; };
  const B bufs[] = {
      {&m->in, N * s2 * 16 * 2},       {&m->A, N * s2 * w0 * 2},         {&m->B, N * s4 * 2 * w0 * 2},
      {&m->X2b, N * s4 * 2 * w0 * 2},  {&m->CAT, N * s4 * 2 * w0 * 2},   {&m->Ma, N * s4 * w0 * 2},
      {&m->Mb, N * s4 * w0 * 2},       {&m->T, N * s4 * w0 * 2},         {&m->Cat8, N * s8 * 8 * w0 * 2},
      {&m->Cat16, N * s16 * 16 * w0 * 2}, {&m->Pcat16, N * s16 * 8 * w0 * 2}, {&m->Pcat32, N * s32 * 16 * w0 * 2},
      {&m->SPP, N * s32 * 32 * w0 * 2}, {&m->B2, N * s32 * 16 * w0 * 2},  {&m->X0, N * s32 * 16 * w0 * 2},
      {&m->F0, N * s16 * 8 * w0 * 2},  {&m->PAN[0], N * s8 * 4 * w0 * 2}, {&m->PAN[1], N * s16 * 8 * w0 * 2},
      {&m->PAN[2], N * s32 * 16 * w0 * 2}, {&m->HS, N * s8 * hc * 2},     {&m->HB, N * s8 * 2 * hc * 2},
      {&m->CF, N * s8 * hc * 2},       {&m->RF, N * s8 * hc * 2},
      {(void**)&m->OUT[0], N * s8 * 8 * 4}, {(void**)&m->OUT[1], N * s16 * 8 * 4}, {(void**)&m->OUT[2], N * s32 * 8 * 4},
  };
  for (const B& b : bufs) {
    void* p = m->dev.dmalloc(b.bytes);
    if (!p) return fail(VGE_ERR_NOMEM, "vge_yolox_reserve: hipMalloc failed");
    HIPCHK(hipMemset(p, 0, b.bytes));
    *b.p = p;
  }
  m->chunk = chunk;
  return VGE_OK;
}

int vge_yolox_destroy(vge_yolox* m) {
  delete m;
  return VGE_OK;
}

int vge_yolox_profile_begin(vge_yolox* m, int max_calls) {
  if (!m || max_calls < 0) return fail(VGE_ERR_ARG, "vge_yolox_profile_begin: bad argument");
  return m->prof.begin(max_calls, 1024);
}

int vge_yolox_profile_read(vge_yolox* m, double* stage_ms, int* n_calls, double* gemm_flops_per_call) {
  if (!m || !stage_ms || !n_calls) return fail(VGE_ERR_ARG, "vge_yolox_profile_read: bad argument");
  int rc = m->prof.read(stage_ms, 2, n_calls);
  if (gemm_flops_per_call) *gemm_flops_per_call = m->prof.flops_per_call(m->gemm_flops);
  return rc;
}

int vge_yolox_detect(vge_yolox* m, const uint8_t* frames, int F, int H, int W, float* boxes, int* n_persons,
                     float* cand, vge_stream_t stream) {
  return vge_yolox_detect_scored(m, frames, F, H, W, boxes, n_persons, nullptr, cand, stream);
}

int vge_yolox_detect_scored(vge_yolox* m, const uint8_t* frames, int F, int H, int W, float* boxes, int* n_persons,
                            float* scores, float* cand, vge_stream_t stream) {
  if (!m || F < 0 || (F > 0 && (!frames || !boxes || !n_persons || H <= 0 || W <= 0)))
    return fail(VGE_ERR_ARG, "vge_yolox_detect: bad argument");
  if (F == 0) return VGE_OK;
  if (m->chunk <= 0) return fail(VGE_ERR_WORKSPACE, "vge_yolox_detect: call vge_yolox_reserve first");
  const vge_yolox_config& c = m->c;
  const int Sz = c.in_size, w0 = c.width, hc = c.head_ch;
  const double r = std::min((double)Sz / H, (double)Sz / W);
  const int rh = (int)(H * r), rw = (int)(W * r);
  if (rh <= 0 || rw <= 0) return fail(VGE_ERR_ARG, "vge_yolox_detect: frame too small for the letterbox");
  const float inv_rx = (float)((double)W / rw), inv_ry = (float)((double)H / rh);
  const int A = (Sz / 8) * (Sz / 8) + (Sz / 16) * (Sz / 16) + (Sz / 32) * (Sz / 32);
  hipStream_t s = S(stream);
  (void)A;
  m->gemm_flops = 0;
  m->prof.start_call();
  int rc;
#define RC(x)                            \
  do {                                   \
    if ((rc = (x)) != VGE_OK) return rc; \
  } while (0)
#define CONV(...)                   \
  do {                              \
    RC(m->prof.beg(0, s));          \
    RC(conv(m->cx(), __VA_ARGS__)); \
    RC(m->prof.end(s));             \
  } while (0)
#define CSP(...)                    \
  do {                              \
    int k_ = 0;                     \
    RC(m->prof.beg(0, s));          \
    RC(ycsp(m, __VA_ARGS__, s, k_)); \
    RC(m->prof.end(s));             \
  } while (0)
#define OTHER(expr)        \
  do {                     \
    RC(m->prof.beg(1, s)); \
    HIPCHK(expr);          \
    RC(m->prof.end(s));    \
  } while (0)
  const int c3 = 4 * w0, c4 = 8 * w0, c5 = 16 * w0;
  for (int f0 = 0; f0 < F; f0 += m->chunk) {
    const int n = std::min(m->chunk, F - f0);
    OTHER(vge::launch_letterbox_focus(frames + (size_t)f0 * H * W * 3, n, H, W, Sz, rh, rw, inv_rx, inv_ry, m->in, s));
    const int h2 = Sz / 2, h4 = Sz / 4, h8 = Sz / 8, h16 = Sz / 16, h32 = Sz / 32;
    uint16_t* cat8 = static_cast<uint16_t*>(m->Cat8);
    uint16_t* cat16 = static_cast<uint16_t*>(m->Cat16);
    uint16_t* pcat16 = static_cast<uint16_t*>(m->Pcat16);
    uint16_t* pcat32 = static_cast<uint16_t*>(m->Pcat32);
    CONV(m->stem, m->in, 16, n, h2, h2, 1, m->A, w0, s);
    CONV(m->d2, m->A, w0, n, h2, h2, 2, m->B, 2 * w0, s);
    CSP(m->c2, m->B, 2 * w0, n, h4, h4, m->X2b, 2 * w0);
    CONV(m->d3, m->X2b, 2 * w0, n, h4, h4, 2, m->B, c3, s);
    CSP(m->c3, m->B, c3, n, h8, h8, cat8 + c3, 2 * c3);                 // x2 -> second half of Cat8
    CONV(m->d4, cat8 + c3, 2 * c3, n, h8, h8, 2, m->B, c4, s);
    CSP(m->c4, m->B, c4, n, h16, h16, cat16 + c4, 2 * c4);              // x1 -> second half of Cat16
    CONV(m->d5, cat16 + c4, 2 * c4, n, h16, h16, 2, m->B, c5, s);
    CONV(m->spp1, m->B, c5, n, h32, h32, 1, m->SPP, 2 * c5, s);
    OTHER(vge::launch_spp_pool(m->SPP, 2 * c5, n, h32, h32, c5 / 2, 5, 9, 13, s));
    CONV(m->spp2, m->SPP, 2 * c5, n, h32, h32, 1, m->B2, c5, s);
    CSP(m->c5, m->B2, c5, n, h32, h32, m->X0, c5);
    CONV(m->lat0, m->X0, c5, n, h32, h32, 1, pcat32 + c4, 2 * c4, s);   // fpn_out0 -> second half of Pcat32
    OTHER(vge::launch_upsample2x(pcat32 + c4, 2 * c4, cat16, 2 * c4, n, h32, h32, c4, s));
    CSP(m->p4, cat16, 2 * c4, n, h16, h16, m->F0, c4);
    CONV(m->red1, m->F0, c4, n, h16, h16, 1, pcat16 + c3, 2 * c3, s);   // fpn_out1 -> second half of Pcat16
    OTHER(vge::launch_upsample2x(pcat16 + c3, 2 * c3, cat8, 2 * c3, n, h16, h16, c3, s));
    CSP(m->p3, cat8, 2 * c3, n, h8, h8, m->PAN[0], c3);
    CONV(m->bu2, m->PAN[0], c3, n, h8, h8, 2, pcat16, 2 * c3, s);
    CSP(m->n3, pcat16, 2 * c3, n, h16, h16, m->PAN[1], c4);
    CONV(m->bu1, m->PAN[1], c4, n, h16, h16, 2, pcat32, 2 * c4, s);
    CSP(m->n4, pcat32, 2 * c4, n, h32, h32, m->PAN[2], c5);
    const int cin[3] = {c3, c4, c5}, hk[3] = {h8, h16, h32};
    for (int k = 0; k < 3; ++k) {
      const YHead& Hd = m->head[k];
      const int g = hk[k];
      uint16_t* hb = static_cast<uint16_t*>(m->HB);
      CONV(Hd.stem, m->PAN[k], cin[k], n, g, g, 1, m->HS, hc, s);
      CONV(Hd.first, m->HS, hc, n, g, g, 1, m->HB, 2 * hc, s);
      CONV(Hd.cls1, hb, 2 * hc, n, g, g, 1, m->CF, hc, s);
      CONV(Hd.reg1, hb + hc, 2 * hc, n, g, g, 1, m->RF, hc, s);
      CONV(Hd.regobj, m->RF, hc, n, g, g, 1, m->OUT[k], 8, s, 0, 1);
      CONV(Hd.cls0, m->CF, hc, n, g, g, 1, m->OUT[k] + 5, 8, s, 0, 1);
    }
    const vge::DetLevel L0{m->OUT[0], h8, 8}, L1{m->OUT[1], h16, 16}, L2{m->OUT[2], h32, 32};
    OTHER(vge::launch_yolox_decode_nms(L0, L1, L2, n, (float)r, boxes + (size_t)f0 * 8, n_persons + f0,
                                       scores ? scores + (size_t)f0 * 2 : nullptr,
                                       cand ? cand + (size_t)f0 * A * 5 : nullptr, s));
  }
#undef OTHER
#undef CSP
#undef CONV
#undef RC
  m->prof.end_call(m->gemm_flops);
  return VGE_OK;
}

}  // extern "C"
