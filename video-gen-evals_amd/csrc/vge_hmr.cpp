// C ABI of the TokenHMR extractor (include/vge_hmr.h): weight upload (f32 state_dict views -> bf16 panels in
// HBM), workspace, and the launch sequence of one batched forward.  Kernels: vge_vit.hip.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/vge_hmr.h"
#include "vge_gemm.h"

namespace vge {
void set_last_error(const std::string& msg);  // vge_api.cpp (vge_last_error)
hipError_t vit_kernels_setup();
hipError_t launch_hmr_crop(const uint8_t*, int, int, const float*, const int*, int, uint8_t*, hipStream_t);
hipError_t launch_ln_bf16(const float*, long, void*, long, const float*, const float*, int, int, float, hipStream_t);
hipError_t launch_cast_bf16(const float*, long, void*, long, int, int, hipStream_t);
hipError_t launch_bcast_rows(const float*, float*, int, int, hipStream_t);
hipError_t launch_patchify(const uint8_t*, int, int, int, int, int, int, int, int, int, int, const float*, const float*,
                           void*, hipStream_t);
hipError_t launch_vit_attn(const void*, long, void*, long, int, int, int, int, hipStream_t);
hipError_t launch_xattn1(const void*, long, const void*, long, void*, long, int, int, int, int, hipStream_t);
hipError_t launch_softmax_rows(const float*, void*, int, int, hipStream_t);
hipError_t launch_readout(const float*, int, const float*, int, const float*, const float*, float*, float*, float*, int,
                          hipStream_t);
hipError_t launch_copy_rows(const float*, long, float*, long, int, int, hipStream_t);
}  // namespace vge

namespace {

enum { GE_BF16 = 0, GE_GELU_BF16 = 1, GE_RES_F32 = 2, GE_PE_F32 = 3, GE_F32 = 4 };
constexpr int NTOK = 192;  // 16 x 12 patches of the 256 x 192 backbone input (the attention kernel's tile)

int fail(int code, const std::string& msg) {
  vge::set_last_error(msg);
  return code;
}

#define HIPCHK(expr)                                                                                    \
  do {                                                                                                  \
    hipError_t _e = (expr);                                                                             \
    if (_e != hipSuccess) return fail(VGE_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

hipStream_t S(vge_stream_t s) { return reinterpret_cast<hipStream_t>(s); }
int rup(int x, int a) { return (x + a - 1) / a * a; }

uint16_t to_bf16(float f) {  // round to nearest even (torch .to(bfloat16))
  uint32_t u;
  memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return 0x7fc0;
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

struct Lin {
  void* W = nullptr;     // bf16 [Npad][K]
  float* b = nullptr;    // f32 [Npad] (zeros when the Linear has no bias)
  int N = 0, K = 0, Npad = 0;
};

struct Vec {
  float* p = nullptr;
  int n = 0;
};

struct VitBlock {
  Vec n1w, n1b, n2w, n2b;
  Lin qkv, proj, fc1, fc2;
};

struct DecLayer {
  Vec sa_nw, sa_nb, ca_nw, ca_nb, ff_nw, ff_nb;
  Lin sa_v, sa_o, ca_q, ca_kv, ca_o, ff1, ff2;
};

}  // namespace

struct vge_hmr {
  vge_hmr_config c{};
  std::vector<void*> allocs;
  Lin pe;
  Vec pos, lnw, lnb, tok0, init_pose, init_betas;
  std::vector<VitBlock> blocks;
  std::vector<DecLayer> dec;
  Lin readout, cls, codebook, decoder;
  // workspace
  int max_frames = 0;
  void *ape = nullptr, *h = nullptr, *qkv = nullptr, *ao = nullptr, *hid = nullptr;
  float* x = nullptr;
  float *xd = nullptr, *rd = nullptr, *logits = nullptr, *bp = nullptr;
  void *hd = nullptr, *qb = nullptr, *cab = nullptr, *hm = nullptr, *xdb = nullptr, *probs = nullptr, *qz = nullptr;
  // profiling: event pairs around every launch of the backbone, by kind (0 GEMM, 1 attention, 2 LayerNorm /
  // patchify), and one pair around the head (kind 3)
  std::vector<hipEvent_t> ev;
  std::vector<int> ev_kind;
  int prof_max = 0, prof_calls = 0, ev_per_call = 0;
  double gemm_flops = 0;
  ~vge_hmr() {
    for (auto e : ev) (void)hipEventDestroy(e);
    for (void* p : allocs) (void)hipFree(p);
  }
  void* dmalloc(size_t bytes) {
    void* p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
    allocs.push_back(p);
    return p;
  }
};

namespace {

struct WeightMap {
  std::unordered_map<std::string, const vge_tensor_view*> m;
  std::string missing, badshape;
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
};

bool upload_f32(vge_hmr* m, const float* src, size_t n, size_t npad, Vec& out) {
  std::vector<float> h(npad, 0.f);
  if (src) memcpy(h.data(), src, n * 4);
  out.p = static_cast<float*>(m->dmalloc(npad * 4));
  out.n = (int)n;
  return out.p && hipMemcpy(out.p, h.data(), npad * 4, hipMemcpyHostToDevice) == hipSuccess;
}

// W [N][K] f32 (row stride ldk, column offset k0) -> bf16 [Npad][K]; rows >= N zero
bool upload_lin(vge_hmr* m, const float* W, int N, int K, long ldk, const float* bias, Lin& L) {
  L.N = N;
  L.K = K;
  L.Npad = rup(N, 256);
  std::vector<uint16_t> h((size_t)L.Npad * K, 0);
  for (int n = 0; n < N; ++n)
    for (int k = 0; k < K; ++k) h[(size_t)n * K + k] = to_bf16(W[(size_t)n * ldk + k]);
  L.W = m->dmalloc(h.size() * 2);
  if (!L.W || hipMemcpy(L.W, h.data(), h.size() * 2, hipMemcpyHostToDevice) != hipSuccess) return false;
  Vec b;
  if (!upload_f32(m, bias, bias ? N : 0, L.Npad, b)) return false;
  L.b = b.p;
  return true;
}

int gemm(int epi, const void* A, long lda, const Lin& L, void* out, long ldo, int M, hipStream_t s,
         const float* res = nullptr, long ldr = 0, const float* pos = nullptr, int tokens = 1) {
  vge::GemmBf16 g{A, lda, L.W, (long)L.K, out, ldo, L.b, res, ldr, pos, tokens, M, L.Npad, L.K};
  if (vge::gemm_lib_ok(epi)) {  // bias / f32-residual epilogues: hipBLASLt (vge_blaslt.cpp); GELU, PE: the kernel
    const hipError_t e = vge::launch_gemm_lib(epi, g, s);
    if (e == hipSuccess) return VGE_OK;
    if (e != hipErrorNotSupported) HIPCHK(e);
  }
  HIPCHK(vge::launch_gemm_bf16(epi, g, s));
  return VGE_OK;
}

bool cfg_ok(const vge_hmr_config& c, std::string& why) {
  if (c.in_h <= 0 || c.in_w <= 0 || c.img_h != c.in_h || c.img_w <= 0 || c.img_w > c.in_w || (c.in_w - c.img_w) % 2)
    return why = "crop geometry (img_h must equal in_h, img_w <= in_w, even margin)", false;
  if (c.patch != 16 || (c.img_h + 2 * c.pad - c.patch) / c.patch + 1 != 16 ||
      (c.img_w + 2 * c.pad - c.patch) / c.patch + 1 != 12)
    return why = "patch grid must be 16 x 12 (192 tokens) with a 16-pixel patch", false;
  if (c.embed_dim % 256 || c.embed_dim > 1280 || c.heads <= 0 || c.embed_dim % c.heads ||
      (c.embed_dim / c.heads != 64 && c.embed_dim / c.heads != 80))
    return why = "embed_dim must be a multiple of 256 (<= 1280) with head dim 64 or 80", false;
  if (c.mlp_dim % 256 || c.depth < 0) return why = "mlp_dim must be a multiple of 256", false;
  if (c.dec_dim % 256 || c.dec_dim > 1280 || c.dec_dim_head != 64 || c.dec_heads <= 0 ||
      (c.dec_heads * 64) % 256 || c.dec_mlp % 256 || c.dec_depth < 0)
    return why = "decoder: dim % 256, dim_head 64, heads * 64 % 256, mlp % 256", false;
  if (c.tok_num <= 0 || c.tok_classes % 256 || c.tok_code_dim % 256 || (c.tok_num * c.tok_code_dim) % 64)
    return why = "token classifier: classes and code dim multiples of 256", false;
  return true;
}

}  // namespace

namespace {
std::string I(int i) { return std::to_string(i); }
}  // namespace

extern "C" {

int vge_hmr_create(const vge_hmr_config* cfg, const vge_tensor_view* weights, int n_weights, vge_hmr** out) {
  if (!cfg || !out || (n_weights > 0 && !weights)) return fail(VGE_ERR_ARG, "vge_hmr_create: null argument");
  *out = nullptr;
  std::string why;
  if (!cfg_ok(*cfg, why)) return fail(VGE_ERR_ARG, "vge_hmr_create: unsupported config: " + why);
  HIPCHK(vge::vit_kernels_setup());
  const vge_hmr_config c = *cfg;
  WeightMap wm;
  for (int i = 0; i < n_weights; ++i)
    if (weights[i].name) wm.m[weights[i].name] = &weights[i];
  const int E = c.embed_dim, P = c.patch, T = NTOK, Dd = c.dec_dim, inner = c.dec_heads * 64;
  auto* m = new vge_hmr();
  m->c = c;
  bool ok = true;
  auto lin = [&](const std::string& k, int N, int K, bool bias, Lin& L, std::initializer_list<int64_t> wshape = {}) {
    const vge_tensor_view* w = wshape.size() ? wm.get(k + ".weight", wshape) : wm.get(k + ".weight", {N, K});
    const vge_tensor_view* b = bias ? wm.get(k + ".bias", {N}) : nullptr;
    if (!w || (bias && !b)) return (void)(ok = false);
    ok = ok && upload_lin(m, w->data, N, K, K, b ? b->data : nullptr, L);
  };
  auto vec = [&](const std::string& k, int n, Vec& v) {
    const vge_tensor_view* t = wm.get(k, {n});
    if (!t) return (void)(ok = false);
    ok = ok && upload_f32(m, t->data, n, n, v);
  };
  lin("backbone.patch_embed.proj", E, 3 * P * P, true, m->pe, {E, 3, P, P});
  if (const vge_tensor_view* t = wm.get("backbone.pos_embed", {1, T + 1, E}))
    ok = ok && upload_f32(m, t->data, (size_t)(T + 1) * E, (size_t)(T + 1) * E, m->pos);
  else
    ok = false;
  m->blocks.resize(c.depth);
  for (int i = 0; i < c.depth && ok; ++i) {
    const std::string p = "backbone.blocks." + I(i) + ".";
    VitBlock& B = m->blocks[i];
    vec(p + "norm1.weight", E, B.n1w);
    vec(p + "norm1.bias", E, B.n1b);
    vec(p + "norm2.weight", E, B.n2w);
    vec(p + "norm2.bias", E, B.n2b);
    lin(p + "attn.qkv", 3 * E, E, true, B.qkv);
    lin(p + "attn.proj", E, E, true, B.proj);
    lin(p + "mlp.fc1", c.mlp_dim, E, true, B.fc1);
    lin(p + "mlp.fc2", E, c.mlp_dim, true, B.fc2);
  }
  vec("backbone.last_norm.weight", E, m->lnw);
  vec("backbone.last_norm.bias", E, m->lnb);
  // decoder input token: to_token_embedding(zeros[.., 1]) + pos_embedding = bias + pos_embedding
  {
    const vge_tensor_view* tw = wm.get("smpl_head.transformer.to_token_embedding.weight", {Dd, 1});
    const vge_tensor_view* tb = wm.get("smpl_head.transformer.to_token_embedding.bias", {Dd});
    const vge_tensor_view* tp = wm.get("smpl_head.transformer.pos_embedding", {1, 1, Dd});
    if (tw && tb && tp) {
      std::vector<float> t0(Dd);
      for (int i = 0; i < Dd; ++i) t0[i] = tb->data[i] + tp->data[i];
      ok = ok && upload_f32(m, t0.data(), Dd, Dd, m->tok0);
    } else {
      ok = false;
    }
  }
  m->dec.resize(c.dec_depth);
  for (int l = 0; l < c.dec_depth && ok; ++l) {
    const std::string p = "smpl_head.transformer.transformer.layers." + I(l) + ".";
    DecLayer& L = m->dec[l];
    vec(p + "0.norm.weight", Dd, L.sa_nw);
    vec(p + "0.norm.bias", Dd, L.sa_nb);
    if (const vge_tensor_view* w = wm.get(p + "0.fn.to_qkv.weight", {3 * inner, Dd}))  // v = rows [2 inner, 3 inner)
      ok = ok && upload_lin(m, w->data + (size_t)2 * inner * Dd, inner, Dd, Dd, nullptr, L.sa_v);
    else
      ok = false;
    lin(p + "0.fn.to_out.0", Dd, inner, true, L.sa_o);
    vec(p + "1.norm.weight", Dd, L.ca_nw);
    vec(p + "1.norm.bias", Dd, L.ca_nb);
    lin(p + "1.fn.to_q", inner, Dd, false, L.ca_q);
    lin(p + "1.fn.to_kv", 2 * inner, E, false, L.ca_kv);
    lin(p + "1.fn.to_out.0", Dd, inner, true, L.ca_o);
    vec(p + "2.norm.weight", Dd, L.ff_nw);
    vec(p + "2.norm.bias", Dd, L.ff_nb);
    lin(p + "2.fn.net.0", c.dec_mlp, Dd, true, L.ff1);
    lin(p + "2.fn.net.3", Dd, c.dec_mlp, true, L.ff2);
  }
  // readouts as one GEMM: grot 0..5 | hands 6..17 | shape 18..27 | cam 28..30
  {
    const char* names[4] = {"smpl_head.decpose_grot", "smpl_head.decpose_hands", "smpl_head.decshape",
                            "smpl_head.deccam"};
    const int rows[4] = {6, 12, 10, 3};
    std::vector<float> W((size_t)31 * Dd), b(31);
    int r0 = 0;
    for (int i = 0; i < 4 && ok; ++i) {
      const vge_tensor_view* w = wm.get(std::string(names[i]) + ".weight", {rows[i], Dd});
      const vge_tensor_view* bb = wm.get(std::string(names[i]) + ".bias", {rows[i]});
      if (!w || !bb) {
        ok = false;
        break;
      }
      memcpy(W.data() + (size_t)r0 * Dd, w->data, (size_t)rows[i] * Dd * 4);
      memcpy(b.data() + r0, bb->data, rows[i] * 4);
      r0 += rows[i];
    }
    ok = ok && upload_lin(m, W.data(), 31, Dd, Dd, b.data(), m->readout);
  }
  lin("smpl_head.decpose.cls", c.tok_num * c.tok_classes, Dd, true, m->cls);
  if (const vge_tensor_view* cb = wm.get("smpl_head.decpose.codebook", {c.tok_classes, c.tok_code_dim})) {
    std::vector<float> t((size_t)c.tok_code_dim * c.tok_classes);  // codebook^T: [code][classes]
    for (int k = 0; k < c.tok_classes; ++k)
      for (int d = 0; d < c.tok_code_dim; ++d) t[(size_t)d * c.tok_classes + k] = cb->data[(size_t)k * c.tok_code_dim + d];
    ok = ok && upload_lin(m, t.data(), c.tok_code_dim, c.tok_classes, c.tok_classes, nullptr, m->codebook);
  } else {
    ok = false;
  }
  lin("smpl_head.decpose.dec", 21 * 6, c.tok_num * c.tok_code_dim, true, m->decoder);
  if (const vge_tensor_view* t = wm.get("smpl_head.init_body_pose", {1, 144}))
    ok = ok && upload_f32(m, t->data, 144, 144, m->init_pose);
  else
    ok = false;
  if (const vge_tensor_view* t = wm.get("smpl_head.init_betas", {1, 10}))
    ok = ok && upload_f32(m, t->data, 10, 10, m->init_betas);
  else
    ok = false;
  if (!ok) {
    const std::string miss = wm.missing, bad = wm.badshape;
    delete m;
    if (!miss.empty()) return fail(VGE_ERR_MISSING_WEIGHT, "vge_hmr_create: missing weight " + miss);
    if (!bad.empty()) return fail(VGE_ERR_WEIGHT_SHAPE, "vge_hmr_create: wrong shape for " + bad);
    return fail(VGE_ERR_HIP, "vge_hmr_create: device allocation / upload failed");
  }
  // algorithmic GEMM FLOPs of the backbone per frame (patch embed + per block qkv, proj, fc1, fc2)
  m->gemm_flops = 2.0 * T * ((double)E * 3 * P * P + c.depth * ((double)E * 3 * E + (double)E * E + 2.0 * E * c.mlp_dim));
  *out = m;
  return VGE_OK;
}

int vge_hmr_reserve(vge_hmr* m, int max_frames) {
  if (!m || max_frames <= 0) return fail(VGE_ERR_ARG, "vge_hmr_reserve: bad argument");
  if (max_frames <= m->max_frames) return VGE_OK;
  const vge_hmr_config& c = m->c;
  const size_t Mv = rup(max_frames * NTOK, 256), Fp = rup(max_frames, 256);
  const size_t E = c.embed_dim, Dd = c.dec_dim, inner = c.dec_heads * 64;
  const size_t K0 = 3 * c.patch * c.patch;
  struct B { void** p; size_t bytes; };
  const B bufs[] = {
      {&m->ape, Mv * K0 * 2},
      {(void**)&m->x, Mv * E * 4},
      {&m->h, Mv * E * 2},
      {&m->qkv, Mv * std::max(3 * E, 2 * inner) * 2},
      {&m->ao, Mv * E * 2},
      {&m->hid, Mv * c.mlp_dim * 2},
      {(void**)&m->xd, Fp * Dd * 4},
      {&m->hd, Fp * Dd * 2},
      {&m->qb, Fp * inner * 2},
      {&m->cab, Fp * inner * 2},
      {&m->hm, Fp * c.dec_mlp * 2},
      {&m->xdb, Fp * Dd * 2},
      {(void**)&m->rd, Fp * 256 * 4},
      {(void**)&m->logits, Fp * c.tok_num * c.tok_classes * 4},
      {&m->probs, Fp * c.tok_num * c.tok_classes * 2},
      {&m->qz, Fp * c.tok_num * c.tok_code_dim * 2},
      {(void**)&m->bp, Fp * 256 * 4},
  };
  for (const B& b : bufs) {
    void* p = m->dmalloc(b.bytes);
    if (!p) return fail(VGE_ERR_NOMEM, "vge_hmr_reserve: hipMalloc failed");
    HIPCHK(hipMemset(p, 0, b.bytes));  // pad rows stay finite
    *b.p = p;
  }
  m->max_frames = max_frames;
  return VGE_OK;
}

int vge_hmr_destroy(vge_hmr* m) {
  delete m;
  return VGE_OK;
}

int vge_hmr_profile_begin(vge_hmr* m, int max_calls) {
  if (!m || max_calls < 0) return fail(VGE_ERR_ARG, "vge_hmr_profile_begin: bad argument");
  for (auto e : m->ev) (void)hipEventDestroy(e);
  m->ev_per_call = 2 * (2 + 7 * m->c.depth + 2);
  m->ev.assign((size_t)max_calls * m->ev_per_call, nullptr);
  m->ev_kind.assign((size_t)max_calls * m->ev_per_call / 2, -1);
  for (auto& e : m->ev) HIPCHK(hipEventCreate(&e));
  m->prof_max = max_calls;
  m->prof_calls = 0;
  return VGE_OK;
}

int vge_hmr_profile_read(vge_hmr* m, double* stage_ms, int* n_calls, double* gemm_flops_per_call) {
  if (!m || !stage_ms || !n_calls) return fail(VGE_ERR_ARG, "vge_hmr_profile_read: bad argument");
  for (int i = 0; i < 4; ++i) stage_ms[i] = 0;
  for (size_t p = 0; p < (size_t)m->prof_calls * m->ev_per_call / 2; ++p) {
    if (m->ev_kind[p] < 0) continue;
    float t;
    HIPCHK(hipEventSynchronize(m->ev[2 * p + 1]));
    HIPCHK(hipEventElapsedTime(&t, m->ev[2 * p], m->ev[2 * p + 1]));
    stage_ms[m->ev_kind[p]] += t;
  }
  *n_calls = m->prof_calls;
  if (gemm_flops_per_call) *gemm_flops_per_call = m->gemm_flops;
  return VGE_OK;
}

int vge_hmr_crop(const uint8_t* frames, int n_frames, int H, int W, const float* boxes, const int32_t* frame_of,
                 int n_crops, uint8_t* crops, vge_stream_t stream) {
  if (n_crops < 0 || n_frames < 0 || (n_crops > 0 && (!frames || !boxes || !crops || H <= 0 || W <= 0)))
    return fail(VGE_ERR_ARG, "vge_hmr_crop: bad argument");
  for (int i = 0; i < n_crops; ++i) {
    const int f = frame_of ? frame_of[i] : i;
    const float* b = boxes + 4 * (size_t)i;
    if (f < 0 || f >= n_frames) return fail(VGE_ERR_ARG, "vge_hmr_crop: frame index out of range");
    if (!(b[2] > b[0]) || !(b[3] > b[1]) || !std::isfinite(b[0] + b[1] + b[2] + b[3]))
      return fail(VGE_ERR_ARG, "vge_hmr_crop: empty or non-finite box");
  }
  const hipError_t e = vge::launch_hmr_crop(frames, H, W, boxes, frame_of, n_crops, crops, S(stream));
  if (e == hipErrorInvalidValue)  // the only argument check inside: the anti-alias radius
    return fail(VGE_ERR_ARG, "vge_hmr_crop: box too large (anti-alias Gaussian radius > 32)");
  HIPCHK(e);
  return VGE_OK;
}

int vge_hmr_extract(vge_hmr* m, const uint8_t* frames, int F, float* pose, float* gori, float* betas, float* vit,
                    vge_stream_t stream) {
  if (!m || F < 0 || (F > 0 && (!frames || !pose || !gori || !betas || !vit)))
    return fail(VGE_ERR_ARG, "vge_hmr_extract: bad argument");
  if (F == 0) return VGE_OK;
  if (F > m->max_frames) return fail(VGE_ERR_WORKSPACE, "vge_hmr_extract: call vge_hmr_reserve(>= n_frames) first");
  const vge_hmr_config& c = m->c;
  hipStream_t s = S(stream);
  const int Mv = rup(F * NTOK, 256), Fp = rup(F, 256);
  const int E = c.embed_dim, Dd = c.dec_dim, inner = c.dec_heads * 64, K0 = 3 * c.patch * c.patch;
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
  int rc;
#define RC(x)                       \
  do {                              \
    if ((rc = (x)) != VGE_OK) return rc; \
  } while (0)
  static const float mean[3] = {123.675f, 116.28f, 103.53f}, stdv[3] = {58.395f, 57.12f, 57.375f};
  RC(beg(2));
  HIPCHK(vge::launch_patchify(frames, F, c.in_h, c.in_w, (c.in_w - c.img_w) / 2, c.img_h, c.img_w, c.patch, c.pad, 16,
                              12, mean, stdv, m->ape, s));
  RC(end());
  RC(beg(0));
  RC(gemm(GE_PE_F32, m->ape, K0, m->pe, m->x, E, Mv, s, nullptr, 0, m->pos.p, NTOK));
  RC(end());
  for (int i = 0; i < c.depth; ++i) {
    const VitBlock& B = m->blocks[i];
    RC(beg(2));
    HIPCHK(vge::launch_ln_bf16(m->x, E, m->h, E, B.n1w.p, B.n1b.p, Mv, E, 1e-6f, s));
    RC(end());
    RC(beg(0));
    RC(gemm(GE_BF16, m->h, E, B.qkv, m->qkv, 3 * E, Mv, s));
    RC(end());
    RC(beg(1));
    HIPCHK(vge::launch_vit_attn(m->qkv, 3 * E, m->ao, E, F, E, c.heads, E / c.heads, s));
    RC(end());
    RC(beg(0));
    RC(gemm(GE_RES_F32, m->ao, E, B.proj, m->x, E, Mv, s, m->x, E));
    RC(end());
    RC(beg(2));
    HIPCHK(vge::launch_ln_bf16(m->x, E, m->h, E, B.n2w.p, B.n2b.p, Mv, E, 1e-6f, s));
    RC(end());
    RC(beg(0));
    RC(gemm(GE_GELU_BF16, m->h, E, B.fc1, m->hid, c.mlp_dim, Mv, s));
    RC(end());
    RC(beg(0));
    RC(gemm(GE_RES_F32, m->hid, c.mlp_dim, B.fc2, m->x, E, Mv, s, m->x, E));
    RC(end());
  }
  RC(beg(2));
  HIPCHK(vge::launch_ln_bf16(m->x, E, m->h, E, m->lnw.p, m->lnb.p, Mv, E, 1e-6f, s));  // context tokens
  RC(end());
  RC(beg(3));
  // ---- SMPL token-decoder head (rows = frames, padded to Fp)
  HIPCHK(vge::launch_bcast_rows(m->tok0.p, m->xd, Fp, Dd, s));
  for (int l = 0; l < c.dec_depth; ++l) {
    const DecLayer& L = m->dec[l];
    // self-attention over the single token: softmax over one key is 1, so it is to_out(v(LN(x)))
    HIPCHK(vge::launch_ln_bf16(m->xd, Dd, m->hd, Dd, L.sa_nw.p, L.sa_nb.p, Fp, Dd, 1e-5f, s));
    RC(gemm(GE_BF16, m->hd, Dd, L.sa_v, m->qb, inner, Fp, s));
    RC(gemm(GE_RES_F32, m->qb, inner, L.sa_o, m->xd, Dd, Fp, s, m->xd, Dd));
    // cross-attention to the 192 context tokens of the frame
    HIPCHK(vge::launch_ln_bf16(m->xd, Dd, m->hd, Dd, L.ca_nw.p, L.ca_nb.p, Fp, Dd, 1e-5f, s));
    RC(gemm(GE_BF16, m->hd, Dd, L.ca_q, m->qb, inner, Fp, s));
    RC(gemm(GE_BF16, m->h, E, L.ca_kv, m->qkv, 2 * inner, Mv, s));
    HIPCHK(vge::launch_xattn1(m->qb, inner, m->qkv, 2 * inner, m->cab, inner, F, inner, c.dec_heads, NTOK, s));
    RC(gemm(GE_RES_F32, m->cab, inner, L.ca_o, m->xd, Dd, Fp, s, m->xd, Dd));
    // feed-forward
    HIPCHK(vge::launch_ln_bf16(m->xd, Dd, m->hd, Dd, L.ff_nw.p, L.ff_nb.p, Fp, Dd, 1e-5f, s));
    RC(gemm(GE_GELU_BF16, m->hd, Dd, L.ff1, m->hm, c.dec_mlp, Fp, s));
    RC(gemm(GE_RES_F32, m->hm, c.dec_mlp, L.ff2, m->xd, Dd, Fp, s, m->xd, Dd));
  }
  HIPCHK(vge::launch_cast_bf16(m->xd, Dd, m->xdb, Dd, Fp, Dd, s));
  RC(gemm(GE_F32, m->xdb, Dd, m->readout, m->rd, 256, Fp, s));
  const int NC = c.tok_num * c.tok_classes;
  RC(gemm(GE_F32, m->xdb, Dd, m->cls, m->logits, NC, Fp, s));
  HIPCHK(vge::launch_softmax_rows(m->logits, m->probs, Fp * c.tok_num, c.tok_classes, s));
  RC(gemm(GE_BF16, m->probs, c.tok_classes, m->codebook, m->qz, c.tok_code_dim, Fp * c.tok_num, s));
  RC(gemm(GE_F32, m->qz, (long)c.tok_num * c.tok_code_dim, m->decoder, m->bp, 256, Fp, s));
  HIPCHK(vge::launch_readout(m->rd, 256, m->bp, 256, m->init_pose.p, m->init_betas.p, pose, gori, betas, F, s));
  HIPCHK(vge::launch_copy_rows(m->xd, Dd, vit, Dd, F, Dd, s));
  RC(end());
#undef RC
  if (prof) ++m->prof_calls;
  return VGE_OK;
}

// ------------------------------------------------------------------ op-level entry points (tests)
int vge_op_gemm_bf16(int epi, const void* A, long lda, const void* W, long ldw, void* out, long ldo, const float* bias,
                     const float* res, long ldr, const float* pos, int tokens, int M, int N, int K,
                     vge_stream_t stream) {
  if (epi < 0 || epi > 4 || !A || !W || !out || M <= 0 || N <= 0 || K <= 0 || M % 256 || N % 256 || K % 64 ||
      lda % 8 || ldw % 8 || lda < K || ldw < K || ldo < N || (epi == GE_RES_F32 && (!res || ldr < N)) ||
      (epi == GE_PE_F32 && (!pos || tokens <= 0)))
    return fail(VGE_ERR_ARG, "vge_op_gemm_bf16: unsupported shape / arguments");
  HIPCHK(vge::vit_kernels_setup());
  vge::GemmBf16 g{A, lda, W, ldw, out, ldo, bias, res, ldr, pos, tokens, M, N, K};
  HIPCHK(vge::launch_gemm_bf16(epi, g, S(stream)));
  return VGE_OK;
}

int vge_op_gemm_lib(int epi, const void* A, long lda, const void* W, long ldw, void* out, long ldo, const float* bias,
                    const float* res, long ldr, int M, int N, int K, vge_stream_t stream) {
  if (epi < 0 || epi > 4 || !A || !W || !out || M <= 0 || N <= 0 || K <= 0 || lda < K || ldw < K || ldo < N ||
      (epi == GE_RES_F32 && (!res || ldr < N)))
    return fail(VGE_ERR_ARG, "vge_op_gemm_lib: unsupported shape / arguments");
  if (!vge::gemm_lib_ok(epi)) return fail(VGE_ERR_UNSUPPORTED, "vge_op_gemm_lib: epilogue not on the library path");
  vge::GemmBf16 g{A, lda, W, ldw, out, ldo, bias, res, ldr, nullptr, 1, M, N, K};
  const hipError_t e = vge::launch_gemm_lib(epi, g, S(stream));
  if (e == hipErrorNotSupported) return fail(VGE_ERR_UNSUPPORTED, "vge_op_gemm_lib: no library algorithm");
  HIPCHK(e);
  return VGE_OK;
}

void vge_debug_set_gemm_lib(int on) { vge::gemm_lib_set(on); }

int vge_op_vit_attention(const void* qkv, void* out, int F, int D, int heads, vge_stream_t stream) {
  if (!qkv || !out || F <= 0 || heads <= 0 || D % heads || (D / heads != 64 && D / heads != 80) || D % 8)
    return fail(VGE_ERR_ARG, "vge_op_vit_attention: head dim must be 64 or 80");
  HIPCHK(vge::vit_kernels_setup());
  HIPCHK(vge::launch_vit_attn(qkv, 3L * D, out, D, F, D, heads, D / heads, S(stream)));
  return VGE_OK;
}

int vge_op_layernorm_bf16(const float* x, void* y, const float* w, const float* b, int rows, int D, float eps,
                          vge_stream_t stream) {
  if (!x || !y || !w || !b || rows <= 0 || (D != 256 && D != 512 && D != 768 && D != 1024 && D != 1280))
    return fail(VGE_ERR_ARG, "vge_op_layernorm_bf16: unsupported width");
  HIPCHK(vge::launch_ln_bf16(x, D, y, D, w, b, rows, D, eps, S(stream)));
  return VGE_OK;
}

}  // extern "C"
