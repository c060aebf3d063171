// Library GEMMs (hipBLASLt) for the extractors' plain linear layers: out = act(A W^T + bias (+ C)) with A [M][K] and
// W [N][K] bf16 row-major, the epilogues of vge_gemm.h that a library epilogue expresses exactly in kind -- bias, bias
// + ReLU, bias + SiLU (Swish), a bf16 residual added before the ReLU, the ViT's f32 residual stream -- and f32
// accumulation throughout.
// The hand-written gemm_bf16_kernel (vge_vit.hip) stays for GELU (the library's is the tanh form, the reference's
// nn.GELU is erf), the position-embedding epilogue, and every shape or epilogue below; it is also what the tuner's
// bit-identity tests pin.  Measured on the MI355X (tools/lib_gemm_probe.py, profiles/lib_gemm_probe_r06t.json):
// hipBLASLt 1,120-1,340 TFLOP/s on the ViT-H and the detector's res4 / box-head shapes where gemm_bf16_kernel runs
// 930-1,150.
//
// Row-major to the library's column-major: out^T [N][M] = W [N][K] x A^T, i.e. the library's A operand is W (K x N,
// ld = ldw, transposed), its B is A (K x M, ld = lda), C / D are N x M with ld = ldr / ldo, and the bias vector (length
// N = the library's rows of D) broadcasts along its columns: out[m][n] += bias[n].
//
// One algorithm per (device, epilogue, N, K, strides, C use): the library heuristic's first choice for the first M seen,
// reused for every later M, so that a layer's per-element arithmetic does not change with the chunk size.
#include "vge_gemm.h"

#include <hipblaslt/hipblaslt.h>

#include <cstdlib>
#include <map>
#include <mutex>
#include <tuple>

namespace vge {
namespace {

constexpr size_t LT_WS_BYTES = 64ull << 20;  // per-device workspace (split-K algorithms)

struct LtDev {
  hipblasLtHandle_t h = nullptr;
  void* ws = nullptr;
};
struct LtAlgo {
  hipblasLtMatmulAlgo_t algo;
  size_t ws;
};
using LtKey = std::tuple<int, int, int, int, long, long, long, long, int>;  // dev, epi, N, K, lda, ldw, ldo, ldr, C

std::mutex g_lt_mu;
std::map<int, LtDev> g_lt_dev;
std::map<LtKey, LtAlgo> g_lt_algo;
int g_lt_on = -1;  // VGE_GEMM_LIB=0: the library path off (hand-written kernel everywhere)

struct LtDescs {  // RAII of one call's descriptors
  hipblasLtMatmulDesc_t op = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr, ld = nullptr;
  hipblasLtMatmulPreference_t pref = nullptr;
  ~LtDescs() {
    if (pref) (void)hipblasLtMatmulPreferenceDestroy(pref);
    if (ld) (void)hipblasLtMatrixLayoutDestroy(ld);
    if (lc) (void)hipblasLtMatrixLayoutDestroy(lc);
    if (lb) (void)hipblasLtMatrixLayoutDestroy(lb);
    if (la) (void)hipblasLtMatrixLayoutDestroy(la);
    if (op) (void)hipblasLtMatmulDescDestroy(op);
  }
};

#define LT_OK(x)                                           \
  do {                                                     \
    if ((x) != HIPBLAS_STATUS_SUCCESS) return hipErrorUnknown; \
  } while (0)

}  // namespace

bool gemm_lib_enabled() {
  if (g_lt_on < 0) {
    const char* e = getenv("VGE_GEMM_LIB");
    g_lt_on = (e && e[0] == '0') ? 0 : 1;
  }
  return g_lt_on == 1;
}

void gemm_lib_set(int on) { g_lt_on = on ? 1 : 0; }

bool gemm_lib_ok(int epi) {
  return gemm_lib_enabled() && (epi == GEMM_BF16 || epi == GEMM_RELU_BF16 || epi == GEMM_RESB_BF16 ||
                                epi == GEMM_RESB_RELU_BF16 || epi == GEMM_RES_F32 || epi == GEMM_F32 ||
                                epi == GEMM_SILU_BF16);
}

hipError_t launch_gemm_lib(int epi, const GemmBf16& a, hipStream_t s) {
  if (!gemm_lib_ok(epi) || a.M <= 0 || a.N <= 0 || a.K <= 0) return hipErrorNotSupported;
  const bool out_f32 = epi == GEMM_RES_F32 || epi == GEMM_F32;
  const bool relu = epi == GEMM_RELU_BF16 || epi == GEMM_RESB_RELU_BF16;
  const void* C = epi == GEMM_RES_F32 ? static_cast<const void*>(a.res)
                  : (epi == GEMM_RESB_BF16 || epi == GEMM_RESB_RELU_BF16) ? a.resb : nullptr;
  if ((epi == GEMM_RES_F32 || epi == GEMM_RESB_BF16 || epi == GEMM_RESB_RELU_BF16) && (!C || a.ldr < a.N))
    return hipErrorInvalidValue;
  const long ldc = C ? a.ldr : a.ldo;
  const hipDataType tout = out_f32 ? HIP_R_32F : HIP_R_16BF;

  int dev = 0;
  hipError_t he = hipGetDevice(&dev);
  if (he != hipSuccess) return he;
  std::lock_guard<std::mutex> lk(g_lt_mu);
  LtDev& D = g_lt_dev[dev];
  if (!D.h) {
    LT_OK(hipblasLtCreate(&D.h));
    if ((he = hipMalloc(&D.ws, LT_WS_BYTES)) != hipSuccess) return he;
  }
  LtDescs d;
  LT_OK(hipblasLtMatmulDescCreate(&d.op, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  const hipblasOperation_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
  LT_OK(hipblasLtMatmulDescSetAttribute(d.op, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)));
  LT_OK(hipblasLtMatmulDescSetAttribute(d.op, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)));
  const bool silu = epi == GEMM_SILU_BF16;  // Swish(x, 1) = x sigmoid(x) = SiLU
  const hipblasLtEpilogue_t ep =
      a.bias ? (relu ? HIPBLASLT_EPILOGUE_RELU_BIAS : silu ? HIPBLASLT_EPILOGUE_SWISH_BIAS_EXT : HIPBLASLT_EPILOGUE_BIAS)
             : (relu ? HIPBLASLT_EPILOGUE_RELU : silu ? HIPBLASLT_EPILOGUE_SWISH_EXT : HIPBLASLT_EPILOGUE_DEFAULT);
  LT_OK(hipblasLtMatmulDescSetAttribute(d.op, HIPBLASLT_MATMUL_DESC_EPILOGUE, &ep, sizeof(ep)));
  if (a.bias) {
    const void* bp = a.bias;
    const hipDataType bt = HIP_R_32F;
    LT_OK(hipblasLtMatmulDescSetAttribute(d.op, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bp, sizeof(bp)));
    LT_OK(hipblasLtMatmulDescSetAttribute(d.op, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)));
  }
  LT_OK(hipblasLtMatrixLayoutCreate(&d.la, HIP_R_16BF, a.K, a.N, a.ldw));
  LT_OK(hipblasLtMatrixLayoutCreate(&d.lb, HIP_R_16BF, a.K, a.M, a.lda));
  LT_OK(hipblasLtMatrixLayoutCreate(&d.lc, tout, a.N, a.M, ldc));
  LT_OK(hipblasLtMatrixLayoutCreate(&d.ld, tout, a.N, a.M, a.ldo));

  const LtKey key{dev, epi, a.N, a.K, a.lda, a.ldw, a.ldo, ldc, (C ? 1 : 0) + (a.bias ? 2 : 0)};
  auto it = g_lt_algo.find(key);
  if (it == g_lt_algo.end()) {
    LT_OK(hipblasLtMatmulPreferenceCreate(&d.pref));
    const uint64_t wsb = LT_WS_BYTES;
    LT_OK(hipblasLtMatmulPreferenceSetAttribute(d.pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb, sizeof(wsb)));
    hipblasLtMatmulHeuristicResult_t r[1];
    int n = 0;
    LT_OK(hipblasLtMatmulAlgoGetHeuristic(D.h, d.op, d.la, d.lb, d.lc, d.ld, d.pref, 1, r, &n));
    if (n < 1 || r[0].state != HIPBLAS_STATUS_SUCCESS || r[0].workspaceSize > LT_WS_BYTES) return hipErrorNotSupported;
    it = g_lt_algo.emplace(key, LtAlgo{r[0].algo, r[0].workspaceSize}).first;
  }
  const float alpha = 1.f, beta = C ? 1.f : 0.f;
  if (hipblasLtMatmul(D.h, d.op, &alpha, a.W, d.la, a.A, d.lb, &beta, C ? C : a.out, d.lc, a.out, d.ld,
                      &it->second.algo, D.ws, it->second.ws, s) == HIPBLAS_STATUS_SUCCESS)
    return hipSuccess;
  // the cached algorithm does not take this M: this call's own heuristic choice (not cached)
  if (!d.pref) {
    LT_OK(hipblasLtMatmulPreferenceCreate(&d.pref));
    const uint64_t wsb = LT_WS_BYTES;
    LT_OK(hipblasLtMatmulPreferenceSetAttribute(d.pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb, sizeof(wsb)));
  }
  hipblasLtMatmulHeuristicResult_t r[1];
  int n = 0;
  LT_OK(hipblasLtMatmulAlgoGetHeuristic(D.h, d.op, d.la, d.lb, d.lc, d.ld, d.pref, 1, r, &n));
  if (n < 1 || r[0].state != HIPBLAS_STATUS_SUCCESS || r[0].workspaceSize > LT_WS_BYTES) return hipErrorNotSupported;
  LT_OK(hipblasLtMatmul(D.h, d.op, &alpha, a.W, d.la, a.A, d.lb, &beta, C ? C : a.out, d.lc, a.out, d.ld, &r[0].algo,
                        D.ws, r[0].workspaceSize, s));
  return hipSuccess;
}

}  // namespace vge
