// C ABI of TokenHMR's gate detector (include/vge_frcnn.h, vge_frcnn_*): detectron2's Faster R-CNN X101-32x8d-FPN.
// FrozenBN folding and NHWC bf16 weight packing (grouped 3x3 convs as 64-channel block-diagonal slices, fc1 as a 7 x 7
// valid conv over the ROI bins), the chunk workspace, and the launch sequence of one chunk of frames:
//   PIL resize + normalise -> stem + max pool -> res2..res5 bottlenecks -> FPN (P2..P6) -> RPN head per level ->
//   proposal selection / NMS / merge -> ROIAlignV2 -> fc1, fc2, predictor -> box inference + postprocess + gate count.
#include <hip/hip_runtime.h>

#include <memory>

#include "../../include/vge_frcnn.h"
#include "vge_cnn.h"
#include "vge_cnn_host.h"
#include "vge_frcnn_k.h"

using namespace vge::cnnh;
#define HIPCHK VGE_HIPCHK

#pragma clang fp contract(off)  // the FrozenBN fold in float32 as the oracle evaluates it

namespace {

constexpr float BN_EPS = 1e-5f;  // FrozenBatchNorm2d
constexpr int GSLICE = 64;       // grouped-conv slice width (output = input channels of one column tile)

struct Block {
  ConvW c1, c2, c3, sc;
  bool has_sc = false;
  int stride = 1, in_ch = 0, width = 0, out_ch = 0, cg = 0;
};

bool stage_blocks(int depth, int (&nb)[4]) {
  const int t[3][5] = {{50, 3, 4, 6, 3}, {101, 3, 4, 23, 3}, {152, 3, 8, 36, 3}};
  for (const auto& r : t)
    if (r[0] == depth) {
      for (int i = 0; i < 4; ++i) nb[i] = r[i + 1];
      return true;
    }
  return false;
}

// detectron2 ResizeShortestEdge.get_output_shape
void output_shape(int h, int w, int short_edge, int max_size, int& nh, int& nw) {
  const double size = short_edge * 1.0;
  double scale = size / std::min(h, w), newh, neww;
  if (h < w) {
    newh = size;
    neww = scale * w;
  } else {
    newh = scale * h;
    neww = size;
  }
  if (std::max(newh, neww) > max_size) {
    scale = max_size * 1.0 / std::max(newh, neww);
    newh = newh * scale;
    neww = neww * scale;
  }
  nw = (int)(neww + 0.5);
  nh = (int)(newh + 0.5);
}

// Pillow Resample.c precompute_coeffs (bilinear filter, the whole axis as the box) + normalize_coeffs_8bpc
void pil_coeffs(int in, int out, std::vector<int>& bounds, std::vector<int>& kk, int& ks) {
  const double scale = (double)in / out;
  const double filterscale = scale < 1.0 ? 1.0 : scale;
  const double support = 1.0 * filterscale;
  ks = (int)std::ceil(support) * 2 + 1;
  kk.assign((size_t)out * ks, 0);
  bounds.assign((size_t)2 * out, 0);
  std::vector<double> w(ks);
  for (int xx = 0; xx < out; ++xx) {
    const double center = (xx + 0.5) * scale;
    const double ss = 1.0 / filterscale;
    int xmin = (int)(center - support + 0.5);
    if (xmin < 0) xmin = 0;
    int xmax = (int)(center + support + 0.5);
    if (xmax > in) xmax = in;
    xmax -= xmin;
    double ww = 0.0;
    for (int x = 0; x < xmax; ++x) {
      double t = (x + xmin - center + 0.5) * ss;
      if (t < 0.0) t = -t;
      w[x] = t < 1.0 ? 1.0 - t : 0.0;
      ww += w[x];
    }
    for (int x = 0; x < xmax; ++x) {
      const double k = ww != 0.0 ? w[x] / ww : w[x];
      kk[(size_t)xx * ks + x] = k < 0 ? (int)(-0.5 + k * (1 << 22)) : (int)(0.5 + k * (1 << 22));
    }
    bounds[2 * xx] = xmin;
    bounds[2 * xx + 1] = xmax;
  }
}

std::string I(int i) { return std::to_string(i); }

}  // namespace

struct vge_frcnn {
  vge_frcnn_config c{};
  DevAllocs dev;
  ConvW stem, lat[4], outc[4], rpn_conv, rpn_head, fc1, fc2, pred;
  std::vector<Block> blocks[4];
  int nb[4] = {0, 0, 0, 0};
  int ld_head = 0;
  void* zero = nullptr;
  // workspace for chunks of `chunk` frames of rH x rW
  std::unique_ptr<DevAllocs> ws;
  int chunk = 0, rH = 0, rW = 0;
  int nh = 0, nw = 0, hp = 0, wp = 0, lh[5] = {0}, lw[5] = {0};
  int *xb = nullptr, *xk = nullptr, *yb = nullptr, *yk = nullptr, ksx = 0, ksy = 0;
  uint8_t* tmp = nullptr;
  void *in = nullptr, *stemo = nullptr, *pool = nullptr, *R[4] = {nullptr, nullptr, nullptr, nullptr}, *Y = nullptr,
       *T1 = nullptr, *T2 = nullptr, *SC = nullptr, *P[5] = {nullptr, nullptr, nullptr, nullptr, nullptr},
       *PV[2] = {nullptr, nullptr}, *UP = nullptr, *RT = nullptr, *BOXF = nullptr, *FC1 = nullptr, *FC2 = nullptr;
  float *RO[5] = {nullptr, nullptr, nullptr, nullptr, nullptr}, *SEL = nullptr, *SELMAX = nullptr, *KEPT = nullptr,
        *PROPS = nullptr, *HEAD = nullptr, *SCR = nullptr;
  int *KCNT = nullptr, *NPROP = nullptr;
  Profiler prof;
  double flops[2] = {0, 0};
  ConvTuner tuner;
  ConvCtx cx(int k) { return ConvCtx{zero, &flops[k], &tuner}; }
};

namespace {

// grouped 3x3 weight [width][cg][3][3] (BN folded) -> 64-channel slices [Npad][9 * 64]: k = tap * 64 + (input channel -
// slice base), zero outside the output channel's group; bias [Npad]
void pack_gconv(const float* W, const float* b, int width, int cg, std::vector<uint16_t>& h, std::vector<float>& bb) {
  const int Npad = rup(width, 256), Kp = 9 * GSLICE;
  h.assign((size_t)Npad * Kp, 0);
  for (int n = 0; n < width; ++n) {
    const int g = n / cg, base = (n / GSLICE) * GSLICE;
    for (int ci = 0; ci < cg; ++ci)
      for (int t = 0; t < 9; ++t)
        h[(size_t)n * Kp + (size_t)t * GSLICE + (g * cg + ci - base)] = to_bf16(W[((size_t)n * cg + ci) * 9 + t]);
  }
  bb.assign(Npad, 0.f);
  memcpy(bb.data(), b, width * 4);
}

struct FLoader {
  vge_frcnn* m;
  WeightMap& wm;
  bool dry;
  bool ok = true;
  // Conv2d(bias=False, norm=FrozenBatchNorm2d): name.weight + name.norm.{weight,bias,running_mean,running_var}
  bool fold_bn(const std::string& p, int Cout, int Cin_g, int K, std::vector<float>& W, std::vector<float>& b) {
    const vge_tensor_view* w = wm.get(p + ".weight", {Cout, Cin_g, K, K});
    const vge_tensor_view* g = wm.get(p + ".norm.weight", {Cout});
    const vge_tensor_view* be = wm.get(p + ".norm.bias", {Cout});
    const vge_tensor_view* mu = wm.get(p + ".norm.running_mean", {Cout});
    const vge_tensor_view* var = wm.get(p + ".norm.running_var", {Cout});
    if (!w || !g || !be || !mu || !var) return false;
    if (dry) return true;
    const size_t per = (size_t)Cin_g * K * K;
    W.resize((size_t)Cout * per);
    b.resize(Cout);
    for (int n = 0; n < Cout; ++n) {
      const float s = g->data[n] / std::sqrt(var->data[n] + BN_EPS);
      for (size_t i = 0; i < per; ++i) W[n * per + i] = w->data[n * per + i] * s;
      b[n] = be->data[n] - mu->data[n] * s;
    }
    return true;
  }
  void conv_bn(const std::string& p, int Cin, int Cout, int K, ConvW& L, int Cinp = 0) {
    std::vector<float> W, b;
    if (!ok || !fold_bn(p, Cout, Cin, K, W, b)) return (void)(ok = false);
    if (!dry) ok = pack_conv(m->dev, W.data(), b.data(), Cout, Cin, Cinp ? Cinp : Cin, K, K, L);
  }
  // grouped 3x3: weight [width][cg][3][3] -> 64-channel slices, k = tap * 64 + (input channel - slice base), zero
  // outside the output channel's group
  void gconv_bn(const std::string& p, int width, int cg, ConvW& L) {
    std::vector<float> W, b;
    if (!ok || !fold_bn(p, width, cg, 3, W, b)) return (void)(ok = false);
    if (dry) return;
    L.Cin = L.Cinp = GSLICE;
    L.Cout = width;
    L.KH = L.KW = 3;
    L.Kp = 9 * GSLICE;
    L.Npad = rup(width, 256);
    std::vector<uint16_t> h;
    std::vector<float> bb;
    pack_gconv(W.data(), b.data(), width, cg, h, bb);
    uint16_t* dw = nullptr;
    ok = upload(m->dev, h, &dw) && upload(m->dev, bb, &L.b);
    L.w = dw;
  }
  // Conv2d / Linear with bias (no norm); several state_dict tensors stacked along Cout
  void plain(const std::vector<std::pair<std::string, int>>& parts, int Cin, int K, ConvW& L, bool linear = false) {
    std::vector<float> W, b;
    int Cout = 0;
    for (const auto& pt : parts) {
      const vge_tensor_view* w = linear ? wm.get(pt.first + ".weight", {pt.second, (int64_t)Cin * K * K})
                                        : wm.get(pt.first + ".weight", {pt.second, Cin, K, K});
      const vge_tensor_view* bv = wm.get(pt.first + ".bias", {pt.second});
      if (!w || !bv) return (void)(ok = false);
      if (!dry) {
        W.insert(W.end(), w->data, w->data + (size_t)pt.second * Cin * K * K);
        b.insert(b.end(), bv->data, bv->data + pt.second);
      }
      Cout += pt.second;
    }
    if (!dry && ok) ok = pack_conv(m->dev, W.data(), b.data(), Cout, Cin, Cin, K, K, L);
  }
};

void load_all(FLoader& ld, const vge_frcnn_config& c) {
  vge_frcnn* m = ld.m;
  const std::string bb = "backbone.bottom_up.";
  ld.conv_bn(bb + "stem.conv1", 3, c.stem_ch, 7, m->stem, 8);
  int in_ch = c.stem_ch, width = c.groups * c.width_per_group, out_ch = c.res2_ch;
  for (int s = 0; s < 4; ++s) {
    m->blocks[s].assign(m->nb[s], Block{});
    for (int b = 0; b < m->nb[s]; ++b) {
      Block& B = m->blocks[s][b];
      const std::string p = bb + "res" + I(s + 2) + "." + I(b);
      B.in_ch = b == 0 ? in_ch : out_ch;
      B.width = width;
      B.out_ch = out_ch;
      B.cg = width / c.groups;
      B.stride = (b == 0 && s > 0) ? 2 : 1;
      B.has_sc = b == 0;
      if (B.has_sc) ld.conv_bn(p + ".shortcut", B.in_ch, out_ch, 1, B.sc);
      ld.conv_bn(p + ".conv1", B.in_ch, width, 1, B.c1);
      ld.gconv_bn(p + ".conv2", width, B.cg, B.c2);
      ld.conv_bn(p + ".conv3", width, out_ch, 1, B.c3);
    }
    in_ch = out_ch;
    width *= 2;
    out_ch *= 2;
  }
  const int F = c.fpn_ch;
  for (int l = 0; l < 4; ++l) {
    ld.plain({{"backbone.fpn_lateral" + I(l + 2), F}}, c.res2_ch << l, 1, m->lat[l]);
    ld.plain({{"backbone.fpn_output" + I(l + 2), F}}, F, 3, m->outc[l]);
  }
  ld.plain({{"proposal_generator.rpn_head.conv", F}}, F, 3, m->rpn_conv);
  ld.plain({{"proposal_generator.rpn_head.objectness_logits", 3}, {"proposal_generator.rpn_head.anchor_deltas", 12}}, F,
           1, m->rpn_head);
  ld.plain({{"roi_heads.box_head.fc1", c.fc_dim}}, F, 7, m->fc1, true);  // [fc][256 * 49] = [fc][256][7][7]
  ld.plain({{"roi_heads.box_head.fc2", c.fc_dim}}, c.fc_dim, 1, m->fc2, true);
  ld.plain({{"roi_heads.box_predictor.cls_score", c.num_classes + 1},
            {"roi_heads.box_predictor.bbox_pred", 4 * c.num_classes}},
           c.fc_dim, 1, m->pred, true);
  if (ld.ok && !ld.dry) {
    std::vector<uint16_t> z(128, 0);
    uint16_t* zp = nullptr;
    ld.ok = upload(m->dev, z, &zp);
    m->zero = zp;
  }
}

bool cfg_ok(const vge_frcnn_config& c, std::string& why) {
  int nb[4];
  if (c.min_size <= 0 || c.max_size < c.min_size) return why = "min_size / max_size", false;
  if (!stage_blocks(c.depth, nb)) return why = "depth must be 50, 101 or 152", false;
  const int w0 = c.groups * c.width_per_group;
  if (c.groups <= 0 || c.width_per_group <= 0 || w0 % GSLICE || GSLICE % c.width_per_group)
    return why = "bottleneck width must be a multiple of 64 and the group width divide 64", false;
  if (c.stem_ch != 64 || !pow2(c.res2_ch) || c.res2_ch < 64) return why = "stem_ch 64, res2_ch a power of two", false;
  if (c.fpn_ch != 256) return why = "fpn_ch must be 256", false;
  if (c.rpn_pre_topk < 1 || c.rpn_pre_topk > vge::FR_MAXK || c.rpn_post_topk < 1 || c.rpn_post_topk > vge::FR_MAXK)
    return why = "rpn top-k must be in [1, 1024]", false;
  if (c.num_classes < 1 || c.num_classes + 1 > 128) return why = "num_classes must be in [1, 127]", false;
  if (c.det_per_img < 1 || c.det_per_img > vge::FR_MAXK) return why = "det_per_img must be in [1, 1024]", false;
  if (!pow2(c.fc_dim) || c.fc_dim < 64) return why = "fc_dim must be a power of two >= 64", false;
  // det_post_kernel keeps at most 4 candidate classes per proposal (vge_frcnn_kernels.hip, FR_MAXCAND = 4,096 slots):
  // exact when no proposal can have 5 classes above the threshold, i.e. 5 x score_thresh >= 1 (softmax sums to 1);
  // the reference's gate runs at 0.25 (mesh_generator.py:71)
  if (!(c.score_thresh >= 0.2f && c.score_thresh < 1.f))
    return why = "score_thresh must be in [0.2, 1): at most 4 classes per proposal pass it (det_post_kernel)", false;
  if (!(c.nms_thresh > 0.f && c.nms_thresh <= 1.f) || !(c.rpn_nms > 0.f && c.rpn_nms <= 1.f))
    return why = "NMS thresholds must be in (0, 1]", false;
  return true;
}

int g_stem_split = -1;  // vge_debug_set_stem_split(1) / VGE_STEM_FUSED=0: the stem conv and the max pool as two kernels

bool stem_fused(const ConvW& L) {
  if (g_stem_split < 0) {
    const char* e = getenv("VGE_STEM_FUSED");
    g_stem_split = (e && e[0] == '0') ? 1 : 0;
  }
  return !g_stem_split && L.Cinp == 8 && L.Cout == 64 && L.KH == 7 && L.KW == 7 && L.Kp >= 400;
}

int gconv(vge_frcnn* m, const ConvW& L, int cg, const void* x, int n, int H, int W, int stride, void* out,
          hipStream_t s) {
  const int Ho = (H + 2 - 3) / stride + 1, Wo = (W + 2 - 3) / stride + 1;
  static const bool direct = !(getenv("VGE_FRCNN_GCONV") && getenv("VGE_FRCNN_GCONV")[0] == '0');
  // the direct grouped kernel (vge_gconv.hip) for group widths below 64 channels; at 64 (res5) a 64-channel slice
  // is one whole group, the implicit GEMM wastes nothing and is faster (92 vs 157 us per 32 frames, r05h trace);
  // VGE_FRCNN_GCONV=0: the implicit GEMM everywhere
  if (direct && cg < GSLICE) {
    HIPCHK(vge::launch_gconv3(x, L.Cout, L.w, L.Kp, L.b, out, L.Cout, n, H, W, L.Cout, cg, stride, s));
    m->flops[0] += 2.0 * n * Ho * Wo * (double)L.Cout * 9 * cg;
    return VGE_OK;
  }
  vge::ConvLaunch c{};
  c.x = x;
  c.ldx = L.Cout;
  c.w = L.w;
  c.bias = L.b;
  c.out = out;
  c.ldo = L.Cout;
  c.zero = m->zero;
  c.n_img = n;
  c.H = H;
  c.W = W;
  c.Cin = GSLICE;
  c.KH = c.KW = 3;
  c.stride = stride;
  c.pad = 1;
  c.Kp = L.Kp;
  c.Cout = L.Cout;
  c.Npad = L.Npad;
  c.act = 3;
  c.tn = GSLICE;
  c.gslice = 1;
  c.variant = 1;
  HIPCHK(vge::launch_conv_bf16(c, s));
  m->flops[0] += 2.0 * n * Ho * Wo * (double)L.Cout * 9 * cg;  // the grouped conv's own FLOPs
  return VGE_OK;
}

}  // namespace

extern "C" {

int vge_frcnn_create(const vge_frcnn_config* cfg, const vge_tensor_view* weights, int n_weights, vge_frcnn** out) {
  if (!cfg || !out || (n_weights > 0 && !weights)) return fail(VGE_ERR_ARG, "vge_frcnn_create: null argument");
  *out = nullptr;
  std::string why;
  if (!cfg_ok(*cfg, why)) return fail(VGE_ERR_ARG, "vge_frcnn_create: unsupported config: " + why);
  WeightMap wm(weights, n_weights);
  auto* m = new vge_frcnn();
  m->c = *cfg;
  stage_blocks(cfg->depth, m->nb);
  m->ld_head = rup(5 * cfg->num_classes + 1, 8);
  bool ok = true;
  for (int pass = 0; pass < 2 && ok; ++pass) {
    FLoader ld{m, wm, pass == 0};
    load_all(ld, *cfg);
    ok = ld.ok;
  }
  if (!ok) {
    delete m;
    return wm.status("vge_frcnn_create");
  }
  *out = m;
  return VGE_OK;
}

int vge_frcnn_shapes(const vge_frcnn* m, int H, int W, int* out) {
  if (!m || !out || H <= 0 || W <= 0) return fail(VGE_ERR_ARG, "vge_frcnn_shapes: bad argument");
  int nh, nw;
  output_shape(H, W, m->c.min_size, m->c.max_size, nh, nw);
  const int hp = rup(nh, 32), wp = rup(nw, 32);
  out[0] = nh;
  out[1] = nw;
  out[2] = hp;
  out[3] = wp;
  for (int l = 0; l < 4; ++l) {
    out[4 + 2 * l] = hp >> (l + 2);
    out[5 + 2 * l] = wp >> (l + 2);
  }
  out[12] = ((hp >> 5) - 1) / 2 + 1;  // P6 = max_pool2d(P5, 1, 2)
  out[13] = ((wp >> 5) - 1) / 2 + 1;
  out[14] = m->ld_head;
  return VGE_OK;
}

int vge_frcnn_reserve(vge_frcnn* m, int chunk, int H, int W) {
  if (!m || chunk <= 0 || H <= 0 || W <= 0) return fail(VGE_ERR_ARG, "vge_frcnn_reserve: bad argument");
  if (chunk <= m->chunk && H == m->rH && W == m->rW) return VGE_OK;
  int sh[15];
  vge_frcnn_shapes(m, H, W, sh);
  {  // index widths: every kernel addresses activations through 64-bit offsets; what stays 32-bit is a layer's row
     // count (n x h x w, the GEMM M) and the thread count of the elementwise kernels (resize: one per padded pixel,
     // pool / upsample: one per 8 channels of a pixel) -- both must stay under 2^31 for the chunk
    const size_t s2 = (size_t)(sh[2] / 2) * (sh[3] / 2), s4 = (size_t)sh[4] * sh[5];
    const size_t w0 = (size_t)m->c.groups * m->c.width_per_group;
    const size_t per = std::max({(size_t)sh[2] * sh[3], s2 * m->c.stem_ch / 8,
                                 s4 * std::max({(size_t)m->c.res2_ch, 2 * w0, (size_t)m->c.fpn_ch}) / 8});
    if ((size_t)chunk * per >= (1ull << 31))
      return fail(VGE_ERR_ARG, "vge_frcnn_reserve: chunk too large for " + std::to_string(H) + " x " + std::to_string(W) +
                                   " frames (at most " + std::to_string(((1ull << 31) - 1) / per) + ")");
  }
  (void)hipDeviceSynchronize();  // the previous workspace (if any) is released only after its kernels completed
  m->ws.reset();
  m->ws = std::make_unique<DevAllocs>();
  DevAllocs& d = *m->ws;
  m->chunk = 0;
  m->nh = sh[0];
  m->nw = sh[1];
  m->hp = sh[2];
  m->wp = sh[3];
  for (int l = 0; l < 5; ++l) {
    m->lh[l] = sh[4 + 2 * l];
    m->lw[l] = sh[5 + 2 * l];
  }
  std::vector<int> b, k;
  if (pil_coeffs(W, m->nw, b, k, m->ksx), !upload(d, b, &m->xb) || !upload(d, k, &m->xk))
    return fail(VGE_ERR_NOMEM, "vge_frcnn_reserve: upload failed");
  if (pil_coeffs(H, m->nh, b, k, m->ksy), !upload(d, b, &m->yb) || !upload(d, k, &m->yk))
    return fail(VGE_ERR_NOMEM, "vge_frcnn_reserve: upload failed");
  const size_t N = chunk, s2 = (size_t)(m->hp / 2) * (m->wp / 2), s4 = (size_t)m->lh[0] * m->lw[0];
  const int w0 = m->c.groups * m->c.width_per_group, r2 = m->c.res2_ch, F = m->c.fpn_ch, P = m->c.rpn_post_topk;
  struct Buf {
    void** p;
    size_t bytes;
  };
  std::vector<Buf> bufs = {
      {(void**)&m->tmp, N * H * m->nw * 3},
      {&m->in, N * m->hp * m->wp * 8 * 2},
      {&m->pool, N * s4 * m->c.stem_ch * 2},
      {&m->Y, N * s4 * std::max(r2, w0) * 2},
      {&m->T1, N * s4 * 2 * w0 * 2},
      {&m->T2, N * s4 * w0 * 2},
      {&m->SC, N * s4 * r2 * 2},
      {&m->PV[0], N * s4 * F * 2},
      {&m->PV[1], N * s4 * F * 2},
      {&m->FC1, N * P * m->c.fc_dim * 2},
      {&m->FC2, N * P * m->c.fc_dim * 2},
      {(void**)&m->HEAD, N * P * m->ld_head * 4},
      {(void**)&m->SEL, N * 5 * vge::FR_MAXK * vge::FR_SEL * 4},
      {(void**)&m->SELMAX, N * 5 * 4},
      {(void**)&m->KEPT, N * 5 * vge::FR_MAXK * vge::FR_SEL * 4},
      {(void**)&m->KCNT, N * 5 * 4},
      {(void**)&m->PROPS, N * P * 5 * 4},
      {(void**)&m->NPROP, N * 4},
      {(void**)&m->SCR, vge::det_post_scratch_bytes(chunk)},
  };
  for (int s = 0; s < 4; ++s) bufs.push_back({&m->R[s], N * (s4 >> (2 * s)) * (size_t)(r2 << s) * 2});
  for (int l = 0; l < 5; ++l) {
    const size_t px = (size_t)m->lh[l] * m->lw[l];
    bufs.push_back({&m->P[l], N * px * F * 2});
    bufs.push_back({(void**)&m->RO[l], N * px * 16 * 4});
  }
  for (const Buf& bf : bufs) {
    void* p = d.dmalloc(bf.bytes);
    if (!p) return fail(VGE_ERR_NOMEM, "vge_frcnn_reserve: hipMalloc failed");
    HIPCHK(hipMemset(p, 0, bf.bytes));
    *bf.p = p;
  }
  // buffers whose lifetimes do not overlap share memory (-86 MB per 800-px frame, a quarter of the workspace): the
  // stem output (split-stem path only) lives before res2.0's conv1 writes T1; the FPN's upsampled top-down sum and
  // the RPN conv's output after the backbone, in the shortcut / grouped-conv buffers; the ROI features after the RPN,
  // in T1.  An alias too small for another frame size gets its own allocation.
  struct Alias {
    void** p;
    size_t bytes;
    void* over;
    size_t over_bytes;
  };
  const Alias al[] = {{&m->stemo, N * s2 * m->c.stem_ch * 2, m->T1, N * s4 * 2 * w0 * 2},
                      {&m->UP, N * s4 * F * 2, m->SC, N * s4 * r2 * 2},
                      {&m->RT, N * s4 * F * 2, m->T2, N * s4 * w0 * 2},
                      {&m->BOXF, N * P * 49 * F * 2, m->T1, N * s4 * 2 * w0 * 2}};
  for (const Alias& a : al) {
    if (a.bytes <= a.over_bytes) {
      *a.p = a.over;
      continue;
    }
    void* p = d.dmalloc(a.bytes);
    if (!p) return fail(VGE_ERR_NOMEM, "vge_frcnn_reserve: hipMalloc failed");
    HIPCHK(hipMemset(p, 0, a.bytes));
    *a.p = p;
  }
  m->chunk = chunk;
  m->rH = H;
  m->rW = W;
  return VGE_OK;
}

int vge_frcnn_destroy(vge_frcnn* m) {
  if (m) (void)hipDeviceSynchronize();
  delete m;
  return VGE_OK;
}

int vge_frcnn_profile_begin(vge_frcnn* m, int max_calls) {
  if (!m || max_calls < 0) return fail(VGE_ERR_ARG, "vge_frcnn_profile_begin: bad argument");
  // event pairs per call: ~190 launches per chunk of frames, and a call may span several chunks
  return m->prof.begin(max_calls, 8192);
}

int vge_frcnn_profile_read(vge_frcnn* m, double* stage_ms, int* n_calls, double* flops_per_call) {
  if (!m || !stage_ms || !n_calls) return fail(VGE_ERR_ARG, "vge_frcnn_profile_read: bad argument");
  int rc = m->prof.read(stage_ms, 3, n_calls);
  if (flops_per_call) {
    // Profiler keeps one FLOP total per call; the split between the two GEMM stages is that of the last call
    const double tot = m->flops[0] + m->flops[1];
    const double per = m->prof.flops_per_call(tot);
    flops_per_call[0] = tot > 0 ? per * m->flops[0] / tot : 0.0;
    flops_per_call[1] = tot > 0 ? per * m->flops[1] / tot : 0.0;
  }
  return rc;
}

int vge_frcnn_detect(vge_frcnn* m, const uint8_t* frames, int F, int H, int W, float* dets, int32_t* n_dets,
                     float* person, int32_t* n_person, const vge_frcnn_taps* taps, vge_stream_t stream) {
  if (!m || F < 0 || (F > 0 && (!frames || !n_person || H <= 0 || W <= 0)))
    return fail(VGE_ERR_ARG, "vge_frcnn_detect: bad argument");
  if (F == 0) return VGE_OK;
  if (m->chunk <= 0) return fail(VGE_ERR_WORKSPACE, "vge_frcnn_detect: call vge_frcnn_reserve first");
  if (H != m->rH || W != m->rW) {
    const int rc = vge_frcnn_reserve(m, m->chunk, H, W);
    if (rc != VGE_OK) return rc;
  }
  const vge_frcnn_config& c = m->c;
  hipStream_t s = S(stream);
  const int Fc = c.fpn_ch, P = c.rpn_post_topk;
  const int h4 = m->lh[0], w4 = m->lw[0];
  m->flops[0] = m->flops[1] = 0;
  m->prof.start_call();
  int rc;
#define RC(x)                            \
  do {                                   \
    if ((rc = (x)) != VGE_OK) return rc; \
  } while (0)
#define STAGE(k, expr)     \
  do {                     \
    RC(m->prof.beg(k, s)); \
    RC(expr);              \
    RC(m->prof.end(s));    \
  } while (0)
#define OTHER(expr)        \
  do {                     \
    RC(m->prof.beg(2, s)); \
    HIPCHK(expr);          \
    RC(m->prof.end(s));    \
  } while (0)
  vge::RpnLevels rl{};
  vge::RoiLevels ro{};
  for (int l = 0; l < 5; ++l) {
    vge::RpnLevel& L = rl.l[l];
    L.h = m->lh[l];
    L.w = m->lw[l];
    L.stride = 4 << l;
    L.k = std::min(c.rpn_pre_topk, L.h * L.w * 3);
  }
  const float sx = (float)((double)W / m->nw), sy = (float)((double)H / m->nh);
  for (int f0 = 0; f0 < F; f0 += m->chunk) {
    const int n = std::min(m->chunk, F - f0);
    // ---- DefaultPredictor preprocessing
    OTHER(vge::launch_frcnn_resize_h(frames + (size_t)f0 * H * W * 3, n, H, W, m->nw, m->xb, m->xk, m->ksx, m->tmp, s));
    OTHER(vge::launch_frcnn_resize_v_norm(m->tmp, n, H, m->nw, m->nh, m->hp, m->wp, m->yb, m->yk, m->ksy,
                                          taps && taps->resized ? taps->resized + (size_t)f0 * m->nh * m->nw * 3 : nullptr,
                                          m->in, s));
    // ---- ResNeXt: stem, max pool, bottlenecks
    if (stem_fused(m->stem)) {  // the stem conv + ReLU + max pool in one kernel (no stem output in HBM)
      RC(m->prof.beg(0, s));
      HIPCHK(vge::launch_frcnn_stem_pool(m->in, m->stem.w, m->stem.Kp, m->stem.b, m->pool, n, m->hp, m->wp, s));
      RC(m->prof.end(s));
      m->flops[0] += 2.0 * n * (m->hp / 2) * (m->wp / 2) * (double)m->stem.Cout * 49 * m->stem.Cinp;
    } else {
      STAGE(0, conv(m->cx(0), m->stem, m->in, 8, n, m->hp, m->wp, 2, m->stemo, c.stem_ch, s, 3));
      OTHER(vge::launch_frcnn_pool_s2(m->stemo, m->pool, n, m->hp / 2, m->wp / 2, c.stem_ch, 3, s));
    }
    const void* x = m->pool;
    int h = h4, w = w4;
    for (int st = 0; st < 4; ++st) {
      const int nbk = m->nb[st];
      for (int b = 0; b < nbk; ++b) {
        const Block& B = m->blocks[st][b];
        const int ho = (h - 1) / B.stride + 1, wo = (w - 1) / B.stride + 1;
        void* o = ((nbk - 1 - b) % 2 == 0) ? m->R[st] : m->Y;
        const void* res = x;
        if (B.has_sc) {
          STAGE(0, conv(m->cx(0), B.sc, x, B.in_ch, n, h, w, B.stride, m->SC, B.out_ch, s, 0));
          res = m->SC;
        }
        STAGE(0, conv(m->cx(0), B.c1, x, B.in_ch, n, h, w, 1, m->T1, B.width, s, 3));
        STAGE(0, gconv(m, B.c2, B.cg, m->T1, n, h, w, B.stride, m->T2, s));
        STAGE(0, conv(m->cx(0), B.c3, m->T2, B.width, n, ho, wo, 1, o, B.out_ch, s, 3, 0, 3, res, B.out_ch));
        x = o;
        h = ho;
        w = wo;
      }
    }
    // ---- FPN (top-down from res5), P6
    STAGE(0, conv(m->cx(0), m->lat[3], m->R[3], c.res2_ch << 3, n, m->lh[3], m->lw[3], 1, m->PV[1], Fc, s, 0));
    STAGE(0, conv(m->cx(0), m->outc[3], m->PV[1], Fc, n, m->lh[3], m->lw[3], 1, m->P[3], Fc, s, 0));
    for (int l = 2, pv = 1; l >= 0; --l, pv ^= 1) {
      OTHER(vge::launch_upsample2x(m->PV[pv], Fc, m->UP, Fc, n, m->lh[l + 1], m->lw[l + 1], Fc, s));
      STAGE(0, conv(m->cx(0), m->lat[l], m->R[l], c.res2_ch << l, n, m->lh[l], m->lw[l], 1, m->PV[pv ^ 1], Fc, s, 0, 0, 1,
                    m->UP, Fc));
      STAGE(0, conv(m->cx(0), m->outc[l], m->PV[pv ^ 1], Fc, n, m->lh[l], m->lw[l], 1, m->P[l], Fc, s, 0));
    }
    OTHER(vge::launch_frcnn_pool_s2(m->P[3], m->P[4], n, m->lh[3], m->lw[3], Fc, 1, s));
    // ---- RPN head per level, proposals
    for (int l = 0; l < 5; ++l) {
      STAGE(0, conv(m->cx(0), m->rpn_conv, m->P[l], Fc, n, m->lh[l], m->lw[l], 1, m->RT, Fc, s, 3));
      STAGE(0, conv(m->cx(0), m->rpn_head, m->RT, Fc, n, m->lh[l], m->lw[l], 1, m->RO[l], 16, s, 0, 1));
      rl.l[l].out = m->RO[l];
    }
    OTHER(vge::launch_rpn_select(rl, n, (float)m->nh, (float)m->nw, m->SEL, m->SELMAX, s));
    OTHER(vge::launch_rpn_nms(rl, m->SEL, m->SELMAX, n, c.rpn_nms, m->KEPT, m->KCNT, s));
    OTHER(vge::launch_rpn_merge(m->KEPT, m->KCNT, n, P, m->PROPS, m->NPROP, s));
    // ---- box head: ROIAlignV2 7x7 over P2..P5, fc1 (a 7 x 7 valid conv over the bins), fc2, predictor
    for (int l = 0; l < 4; ++l) {
      ro.p[l] = m->P[l];
      ro.h[l] = m->lh[l];
      ro.w[l] = m->lw[l];
    }
    OTHER(vge::launch_roi_align(ro, m->PROPS, m->NPROP, n, P, m->BOXF, s));
    {
      vge::ConvLaunch fc{};
      fc.x = m->BOXF;
      fc.ldx = Fc;
      fc.w = m->fc1.w;
      fc.bias = m->fc1.b;
      fc.out = m->FC1;
      fc.ldo = c.fc_dim;
      fc.zero = m->zero;
      fc.n_img = n * P;
      fc.H = fc.W = 7;
      fc.Cin = Fc;
      fc.KH = fc.KW = 7;
      fc.stride = 1;
      fc.pad = 0;
      fc.Kp = m->fc1.Kp;
      fc.Cout = c.fc_dim;
      fc.Npad = m->fc1.Npad;
      fc.act = 3;
      fc.tn = conv_tile_n(c.fc_dim);
      RC(m->prof.beg(1, s));
      if (m->tuner.enabled()) {
        const std::array<long, 10> key = {7, 7, Fc, c.fc_dim, 7, -1, 3, 0, 0, c.fc_dim};  // (stride -1: pad 0)
        HIPCHK(conv_tuned_launch(m->tuner, fc, key, s));
      } else {
        HIPCHK(vge::launch_conv_bf16(fc, s));
      }
      RC(m->prof.end(s));
      m->flops[1] += 2.0 * n * P * (double)c.fc_dim * 49 * Fc;
    }
    STAGE(1, conv(m->cx(1), m->fc2, m->FC1, c.fc_dim, n * P, 1, 1, 1, m->FC2, c.fc_dim, s, 3));
    STAGE(1, conv(m->cx(1), m->pred, m->FC2, c.fc_dim, n * P, 1, 1, 1, m->HEAD, m->ld_head, s, 0, 1));
    // ---- FastRCNNOutputLayers.inference + detector_postprocess + the gate's person count
    vge::DetPostArgs da{};
    da.head = m->HEAD;
    da.ld = m->ld_head;
    da.P = P;
    da.K = c.num_classes;
    da.det_per_img = c.det_per_img;
    da.props = m->PROPS;
    da.n_prop = m->NPROP;
    da.img_h = (float)m->nh;
    da.img_w = (float)m->nw;
    da.sx = sx;
    da.sy = sy;
    da.out_h = (float)H;
    da.out_w = (float)W;
    da.score_thresh = c.score_thresh;
    da.nms_thresh = c.nms_thresh;
    da.gate_thresh = c.gate_thresh;
    da.scratch = m->SCR;
    da.pre_dets = taps && taps->pre_dets ? taps->pre_dets + (size_t)f0 * c.det_per_img * 6 : nullptr;
    da.n_pre = taps && taps->n_pre_dets ? taps->n_pre_dets + f0 : nullptr;
    da.dets = dets ? dets + (size_t)f0 * c.det_per_img * 6 : nullptr;
    da.n_dets = n_dets ? n_dets + f0 : nullptr;
    da.person = person ? person + (size_t)f0 * 10 : nullptr;
    da.n_person = n_person + f0;
    OTHER(vge::launch_det_post(da, n, s));
    // ---- parity taps
    if (taps) {
      for (int l = 0; l < 5; ++l) {
        const size_t px = (size_t)m->lh[l] * m->lw[l];
        if (taps->fpn[l])
          HIPCHK(hipMemcpyAsync(static_cast<char*>(taps->fpn[l]) + (size_t)f0 * px * Fc * 2, m->P[l], n * px * Fc * 2,
                                hipMemcpyDeviceToDevice, s));
        if (taps->rpn[l])
          HIPCHK(hipMemcpyAsync(taps->rpn[l] + (size_t)f0 * px * 16, m->RO[l], n * px * 16 * 4, hipMemcpyDeviceToDevice, s));
      }
      if (taps->proposals)
        HIPCHK(hipMemcpyAsync(taps->proposals + (size_t)f0 * P * 5, m->PROPS, (size_t)n * P * 5 * 4,
                              hipMemcpyDeviceToDevice, s));
      if (taps->n_proposals)
        HIPCHK(hipMemcpyAsync(taps->n_proposals + f0, m->NPROP, (size_t)n * 4, hipMemcpyDeviceToDevice, s));
      if (taps->box_features)
        HIPCHK(hipMemcpyAsync(static_cast<char*>(taps->box_features) + (size_t)f0 * P * 49 * Fc * 2, m->BOXF,
                              (size_t)n * P * 49 * Fc * 2, hipMemcpyDeviceToDevice, s));
      if (taps->head)
        HIPCHK(hipMemcpyAsync(taps->head + (size_t)f0 * P * m->ld_head, m->HEAD, (size_t)n * P * m->ld_head * 4,
                              hipMemcpyDeviceToDevice, s));
    }
  }
#undef OTHER
#undef STAGE
#undef RC
  m->prof.end_call(m->flops[0] + m->flops[1]);
  return VGE_OK;
}

// Test hook: the grouped 3x3 conv alone (tests/test_frcnn.py vs torch conv2d(groups)); x / out device NHWC bf16,
// w [C][gw][3][3] and b [C] host f32 (packed as the detector packs them); the block-diagonal implicit GEMM with
// VGE_FRCNN_GCONV=0
int vge_debug_gconv3(const void* x, int n, int H, int W, int C, int gw, int stride, const float* w, const float* b,
                     void* out, vge_stream_t stream) {
  if (!x || !w || !b || !out || n < 1 || C % GSLICE || gw < 1 || GSLICE % gw)
    return fail(VGE_ERR_ARG, "vge_debug_gconv3: bad argument");
  std::vector<uint16_t> h;
  std::vector<float> bb;
  pack_gconv(w, b, C, gw, h, bb);
  vge_frcnn tmp;
  ConvW L;
  L.Cin = L.Cinp = GSLICE;
  L.Cout = C;
  L.KH = L.KW = 3;
  L.Kp = 9 * GSLICE;
  L.Npad = rup(C, 256);
  uint16_t* dw = nullptr;
  std::vector<uint16_t> z(128, 0);
  uint16_t* zp = nullptr;
  if (!upload(tmp.dev, h, &dw) || !upload(tmp.dev, bb, &L.b) || !upload(tmp.dev, z, &zp))
    return fail(VGE_ERR_NOMEM, "vge_debug_gconv3: upload");
  L.w = dw;
  tmp.zero = zp;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int r = gconv(&tmp, L, gw, x, n, H, W, stride, out, s);
  if (r != VGE_OK) return r;
  HIPCHK(hipStreamSynchronize(s));
  return VGE_OK;
}

}  // extern "C"

extern "C" int vge_debug_set_stem_split(int on) {  // tests / A/B: 1 = the stem conv and the max pool as two kernels
  g_stem_split = on ? 1 : 0;
  return 0;
}
