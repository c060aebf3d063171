// The gate detector's non-GEMM kernels (include/vge_frcnn.h; the convolutions and Linears run on the implicit-GEMM
// kernels of vge_cnn.hip): detectron2's Faster R-CNN inference path around the network, restated for gfx950.
//
//   frcnn_resize_h_kernel / frcnn_resize_v_norm_kernel   ResizeShortestEdge through PIL's bilinear Image.resize on
//       uint8 (Resample.c: 22-bit fixed-point coefficients from the host, horizontal pass then vertical pass, each
//       rounded to uint8) + (x - PIXEL_MEAN) / PIXEL_STD in BGR order -> NHWC bf16 with 8 channels, zero padding to a
//       multiple of 32 (ImageList size_divisibility)
//   frcnn_pool_s2_kernel<K>   max_pool2d(3, 2, 1) after the stem, max_pool2d(1, 2, 0) for P6 (LastLevelMaxPool)
//   rpn_select_kernel         find_top_rpn_proposals, one workgroup per (frame, level): the top-k objectness logits by
//       an 8-bit radix select on order-preserving keys (ties: lower anchor index), a bitonic sort of the k winners,
//       anchor + Box2BoxTransform decode, clip, nonempty, and the level's largest kept coordinate
//   rpn_nms_kernel            batched_nms(0.7) per (frame, level): torchvision's coordinate trick (boxes + level x
//       (max + 1)), the IoU > thr upper triangle as 64-bit ballot words in LDS, the greedy scan by one wave (bit scan
//       to the next live box), the kept boxes copied out after it
//   rpn_merge_kernel          the levels' kept boxes in (score desc, level, rank) order = one stable sort of the
//       concatenation, first post_nms_topk (rank by binary search in the other levels' sorted lists)
//   roi_align_sep_kernel      ROIPooler: level = floor(4 + log2(sqrt(area) / 224 + 1e-8)) in [2, 5], ROIAlignV2
//       (aligned, adaptive sampling grid) as separable per-bin cell weights, 8 channels per lane (default);
//       roi_align_kernel the same in torchvision's sample / weight / sum order
//   det_post_kernel           FastRCNNOutputLayers.inference + detector_postprocess per frame: softmax, per-class
//       decode (10, 10, 5, 5) + clip, candidates with score > thresh in (proposal, class) order, per-class NMS
//       (coordinate trick, bitmask + greedy scan), top det_per_img by (score desc, candidate order), scaling to the
//       frame, clip, nonempty, and the gate's person count
// Every float expression keeps its operations separately rounded (no contraction), as the oracle (oracle/frcnn.py)
// evaluates them.
#include "vge_common.h"
#include "vge_lds_attr.h"
#include "vge_frcnn_k.h"

#include <algorithm>

#pragma clang fp contract(off)

namespace {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned long long u64;
typedef unsigned uintx4_t __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr float SCALE_CLAMP = 4.135166556742356f;  // log(1000 / 16), Box2BoxTransform

__device__ __forceinline__ unsigned okey(float f) {  // order-preserving unsigned key of a float
  const unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ int clip8(int v) {
  v >>= 22;  // PRECISION_BITS
  return v < 0 ? 0 : (v > 255 ? 255 : v);
}
__device__ __forceinline__ u64 readlane64(u64 v, int l) {
  const unsigned lo = __builtin_amdgcn_readlane((int)(unsigned)v, l);
  const unsigned hi = __builtin_amdgcn_readlane((int)(unsigned)(v >> 32), l);
  return ((u64)hi << 32) | lo;
}

// Box2BoxTransform.apply_deltas for one box
__device__ __forceinline__ void apply_delta(float ax1, float ay1, float ax2, float ay2, float d0, float d1, float d2,
                                            float d3, float wx, float wy, float ww, float wh, float& x1, float& y1,
                                            float& x2, float& y2) {
  const float w = ax2 - ax1, h = ay2 - ay1;
  const float cx = ax1 + 0.5f * w, cy = ay1 + 0.5f * h;
  const float dx = d0 / wx, dy = d1 / wy;
  const float dw = fminf(d2 / ww, SCALE_CLAMP), dh = fminf(d3 / wh, SCALE_CLAMP);
  const float pcx = dx * w + cx, pcy = dy * h + cy;
  const float pw = expf(dw) * w, ph = expf(dh) * h;
  x1 = pcx - 0.5f * pw;
  y1 = pcy - 0.5f * ph;
  x2 = pcx + 0.5f * pw;
  y2 = pcy + 0.5f * ph;
}
__device__ __forceinline__ float clampf(float v, float hi) { return fminf(fmaxf(v, 0.f), hi); }

// torchvision devIoU > threshold (areas of the same, possibly offset, boxes)
__device__ __forceinline__ bool iou_gt(float4 a, float sa, float4 b, float sb, float thr) {
  const float left = fmaxf(a.x, b.x), right = fminf(a.z, b.z);
  const float top = fmaxf(a.y, b.y), bottom = fminf(a.w, b.w);
  const float width = fmaxf(right - left, 0.f), height = fmaxf(bottom - top, 0.f);
  const float inter = width * height;
  return inter / ((sa + sb) - inter) > thr;
}

// bitonic sort of N keys in LDS by T threads (ascending, or descending)
template <int N, int T, bool DESC>
__device__ void bitonic(u64* k) {
  for (int size = 2; size <= N; size <<= 1)
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      __syncthreads();
      for (int t = threadIdx.x; t < N / 2; t += T) {
        const int i = 2 * t - (t & (stride - 1)), j = i + stride;
        const bool up = (i & size) == 0;
        const u64 a = k[i], b = k[j];
        if (DESC ? ((a < b) == up) : ((a > b) == up)) {
          k[i] = b;
          k[j] = a;
        }
      }
    }
  __syncthreads();
}

// exclusive prefix sum over a 1024-thread block (wsum: 16 ints of LDS); *total = the block's sum
__device__ int block_excl_scan(int v, int* wsum, int* total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) wsum[wave] = x;
  __syncthreads();
  int off = 0, tot = 0;
  for (int w = 0; w < 16; ++w) {
    off += w < wave ? wsum[w] : 0;
    tot += wsum[w];
  }
  __syncthreads();
  *total = tot;
  return off + x - v;
}

__device__ __forceinline__ float block_max(float v, float* red) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_max(v);
  if (lane == 0) red[wave] = v;
  __syncthreads();
  float m = -INFINITY;
  for (int w = 0; w < nw; ++w) m = fmaxf(m, red[w]);
  __syncthreads();
  return m;
}

// ------------------------------------------------------------------------------------------------ resize
__global__ void __launch_bounds__(256) frcnn_resize_h_kernel(const uint8_t* __restrict__ src, int n, int H, int W,
                                                             int nw, const int* __restrict__ xb,
                                                             const int* __restrict__ kk, int ks,
                                                             uint8_t* __restrict__ dst) {
  const long gid = (long)blockIdx.x * 256 + threadIdx.x;
  if (gid >= (long)n * H * nw) return;
  const int xx = (int)(gid % nw);
  const uint8_t* s = src + (gid / nw) * W * 3;
  const int xmin = xb[2 * xx], xmax = xb[2 * xx + 1];
  const int* k = kk + (long)xx * ks;
  int a0 = 1 << 21, a1 = 1 << 21, a2 = 1 << 21;
  for (int x = 0; x < xmax; ++x) {
    const int w = k[x];
    const uint8_t* p = s + (xmin + x) * 3;
    a0 += (int)p[0] * w;
    a1 += (int)p[1] * w;
    a2 += (int)p[2] * w;
  }
  uint8_t* d = dst + gid * 3;
  d[0] = (uint8_t)clip8(a0);
  d[1] = (uint8_t)clip8(a1);
  d[2] = (uint8_t)clip8(a2);
}

// vertical pass + normalisation: tmp uint8 [n][H][nw][3] RGB -> out bf16 [n][hp][wp][8] (B, G, R, 0 ...)
__global__ void __launch_bounds__(256) frcnn_resize_v_norm_kernel(const uint8_t* __restrict__ tmp, int n, int H,
                                                                  int nw, int nh, int hp, int wp,
                                                                  const int* __restrict__ yb,
                                                                  const int* __restrict__ kk, int ks,
                                                                  uint8_t* __restrict__ resized, bf16* __restrict__ out) {
  const long gid = (long)blockIdx.x * 256 + threadIdx.x;
  if (gid >= (long)n * hp * wp) return;
  const int x = (int)(gid % wp), y = (int)((gid / wp) % hp);
  const long img = gid / ((long)wp * hp);
  bf16x8 o;
#pragma unroll
  for (int c = 0; c < 8; ++c) o[c] = (bf16)0.f;
  if (y < nh && x < nw) {
    const int ymin = yb[2 * y], ymax = yb[2 * y + 1];
    const int* k = kk + (long)y * ks;
    int a0 = 1 << 21, a1 = 1 << 21, a2 = 1 << 21;
    for (int j = 0; j < ymax; ++j) {
      const int w = k[j];
      const uint8_t* p = tmp + ((img * H + ymin + j) * nw + x) * 3;
      a0 += (int)p[0] * w;
      a1 += (int)p[1] * w;
      a2 += (int)p[2] * w;
    }
    const int r = clip8(a0), g = clip8(a1), b = clip8(a2);
    if (resized) {
      uint8_t* q = resized + ((img * nh + y) * nw + x) * 3;
      q[0] = (uint8_t)r;
      q[1] = (uint8_t)g;
      q[2] = (uint8_t)b;
    }
    o[0] = (bf16)(((float)b - 103.530f) / 57.375f);
    o[1] = (bf16)(((float)g - 116.280f) / 57.120f);
    o[2] = (bf16)(((float)r - 123.675f) / 58.395f);
  }
  *reinterpret_cast<bf16x8*>(out + gid * 8) = o;
}

// ------------------------------------------------------------------------------------------------ pooling
template <int K>
__global__ void __launch_bounds__(256) frcnn_pool_s2_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, int n,
                                                            int H, int W, int C, int Ho, int Wo) {
  const int cg = C >> 3;
  const long gid = (long)blockIdx.x * 256 + threadIdx.x;
  if (gid >= (long)n * Ho * Wo * cg) return;
  const int c8 = (int)(gid % cg) * 8;
  const long pix = gid / cg;
  const int ow = (int)(pix % Wo), oh = (int)((pix / Wo) % Ho);
  const long img = pix / ((long)Wo * Ho);
  float m[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) m[i] = -INFINITY;
#pragma unroll
  for (int dy = 0; dy < K; ++dy) {
    const int ih = 2 * oh - K / 2 + dy;
    if ((unsigned)ih >= (unsigned)H) continue;
#pragma unroll
    for (int dx = 0; dx < K; ++dx) {
      const int iw = 2 * ow - K / 2 + dx;
      if ((unsigned)iw >= (unsigned)W) continue;
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(x + ((img * H + ih) * W + iw) * C + c8);
#pragma unroll
      for (int i = 0; i < 8; ++i) m[i] = fmaxf(m[i], (float)v[i]);
    }
  }
  bf16x8 o;
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = (bf16)m[i];
  *reinterpret_cast<bf16x8*>(y + pix * C + c8) = o;
}

// ------------------------------------------------------------------------------------------------ RPN
// field-wise uniform selects (a dynamically indexed by-value kernel argument would be copied to scratch)
__device__ __forceinline__ vge::RpnLevel pick_level(const vge::RpnLevels& L, int l) {
  vge::RpnLevel r;
#define VGE_PICK(fld) r.fld = l == 0 ? L.l[0].fld : l == 1 ? L.l[1].fld : l == 2 ? L.l[2].fld : l == 3 ? L.l[3].fld : L.l[4].fld
  VGE_PICK(out);
  VGE_PICK(h);
  VGE_PICK(w);
  VGE_PICK(stride);
  VGE_PICK(k);
#undef VGE_PICK
  return r;
}
// DefaultAnchorGenerator._generate_cell_anchors in double (python floats), then float32: size 8 x stride, ratio
// (0.5, 1, 2)[a]; c = x1, y1, x2, y2
__device__ __forceinline__ float cell(const vge::RpnLevel& lv, int a, int c) {
  const double size = 8.0 * lv.stride, area = size * size, ratio = a == 0 ? 0.5 : (a == 1 ? 1.0 : 2.0);
  const double w = sqrt(area / ratio), h = ratio * w;
  const double v = c == 0 ? -w / 2.0 : c == 1 ? -h / 2.0 : c == 2 ? w / 2.0 : h / 2.0;
  return (float)v;
}

__global__ void __launch_bounds__(1024) rpn_select_kernel(vge::RpnLevels L, float img_h, float img_w,
                                                          float* __restrict__ sel, float* __restrict__ sel_max) {
  const int f = blockIdx.x, l = blockIdx.y;
  const vge::RpnLevel lv = pick_level(L, l);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float* out = lv.out + (size_t)f * lv.h * lv.w * 16;
  const int N = lv.h * lv.w * 3, k = lv.k;
  auto keyof = [&](int i) -> unsigned {
    const int loc = i / 3;
    return okey(out[(size_t)loc * 16 + (i - 3 * loc)]);
  };
  __shared__ unsigned hist[16][256];
  __shared__ u64 keys[vge::FR_MAXK];
  __shared__ unsigned s_prefix, s_krem, s_cnt, s_eqbase;
  __shared__ unsigned wcnt[16];
  __shared__ float red[16];

  // ---- the k-th largest key: 4 rounds of 8-bit digits, most significant first
  unsigned prefix = 0, pmask = 0, krem = (unsigned)k;
  for (int shift = 24; shift >= 0; shift -= 8) {
    for (int i = tid; i < 16 * 256; i += 1024) (&hist[0][0])[i] = 0u;
    __syncthreads();
    for (int i = tid; i < N; i += 1024) {
      const unsigned kk = keyof(i);
      if ((kk & pmask) == prefix) atomicAdd(&hist[wave][(kk >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (tid < 256) {
      unsigned t = 0;
      for (int w = 0; w < 16; ++w) t += hist[w][tid];
      hist[0][tid] = t;
    }
    __syncthreads();
    if (tid == 0) {
      unsigned cum = 0;
      int d = 255;
      for (; d > 0; --d) {
        if (cum + hist[0][d] >= krem) break;
        cum += hist[0][d];
      }
      s_krem = krem - cum;
      s_prefix = prefix | ((unsigned)d << shift);
    }
    __syncthreads();
    krem = s_krem;
    prefix = s_prefix;
    pmask |= 255u << shift;
    __syncthreads();
  }
  // ---- the winners: every key above the threshold key, and the `need` lowest-index keys equal to it
  const unsigned T = prefix, need = krem, ngt = (unsigned)k - need;
  if (tid == 0) {
    s_cnt = 0;
    s_eqbase = 0;
  }
  keys[tid] = 0ull;
  __syncthreads();
  for (int base = 0; base < N; base += 1024) {
    const int i = base + tid;
    const unsigned kk = i < N ? keyof(i) : 0u;
    const bool gt = i < N && kk > T, eq = i < N && kk == T;
    const u64 pk = ((u64)kk << 32) | (0xFFFFFFFFu - (unsigned)i);
    if (gt) keys[atomicAdd(&s_cnt, 1u)] = pk;
    const u64 bal = __ballot(eq);
    const unsigned pre = (unsigned)__popcll(bal & ((1ull << lane) - 1ull));
    if (lane == 0) wcnt[wave] = (unsigned)__popcll(bal);
    __syncthreads();
    unsigned woff = 0, tot = 0;
    for (int w = 0; w < 16; ++w) {
      woff += w < wave ? wcnt[w] : 0u;
      tot += wcnt[w];
    }
    const unsigned eqb = s_eqbase;
    if (eq && eqb + woff + pre < need) keys[ngt + eqb + woff + pre] = pk;
    __syncthreads();
    if (tid == 0) s_eqbase = eqb + tot;
    __syncthreads();
  }
  bitonic<vge::FR_MAXK, 1024, true>(keys);  // (key desc, anchor index asc)

  // ---- decode, clip, nonempty
  float* so = sel + ((size_t)(f * 5 + l) * vge::FR_MAXK + tid) * vge::FR_SEL;
  float e[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float mx = -INFINITY;
  if (tid < k) {
    const u64 v = keys[tid];
    const int i = (int)(0xFFFFFFFFu - (unsigned)(v & 0xFFFFFFFFull));
    const int loc = i / 3, a = i - 3 * loc;
    const float* row = out + (size_t)loc * 16;
    const float lg = row[a];
    const int y = loc / lv.w, x = loc - y * lv.w;
    const float sx = (float)(x * lv.stride), sy = (float)(y * lv.stride);
    float x1, y1, x2, y2;
    apply_delta(sx + cell(lv, a, 0), sy + cell(lv, a, 1), sx + cell(lv, a, 2), sy + cell(lv, a, 3), row[3 + 4 * a],
                row[4 + 4 * a], row[5 + 4 * a], row[6 + 4 * a], 1.f, 1.f, 1.f, 1.f, x1, y1, x2, y2);
    const bool fin = isfinite(x1) && isfinite(y1) && isfinite(x2) && isfinite(y2) && isfinite(lg);
    x1 = clampf(x1, img_w);
    y1 = clampf(y1, img_h);
    x2 = clampf(x2, img_w);
    y2 = clampf(y2, img_h);
    const bool ok = fin && (x2 - x1) > 0.f && (y2 - y1) > 0.f;
    e[0] = x1;
    e[1] = y1;
    e[2] = x2;
    e[3] = y2;
    e[4] = lg;
    e[5] = ok ? 1.f : 0.f;
    if (ok) mx = fmaxf(fmaxf(x1, y1), fmaxf(x2, y2));
  }
  *reinterpret_cast<floatx4*>(so) = floatx4{e[0], e[1], e[2], e[3]};
  *reinterpret_cast<floatx4*>(so + 4) = floatx4{e[4], e[5], e[6], e[7]};
  mx = block_max(mx, red);
  if (tid == 0) sel_max[f * 5 + l] = mx;
}

constexpr int NMS_LDS = vge::FR_MAXK * 16 + vge::FR_MAXK * 4 + vge::FR_MAXK * 4 + vge::FR_MAXK * 16 * 8;

__global__ void __launch_bounds__(1024) rpn_nms_kernel(vge::RpnLevels L, const float* __restrict__ sel,
                                                       const float* __restrict__ sel_max, float thr,
                                                       float* __restrict__ kept, int* __restrict__ kcount) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  float4* bx = reinterpret_cast<float4*>(lds);
  float* area = reinterpret_cast<float*>(lds + vge::FR_MAXK * 16);
  int* vld = reinterpret_cast<int*>(lds + vge::FR_MAXK * 20);
  u64* mask = reinterpret_cast<u64*>(lds + vge::FR_MAXK * 24);
  const int f = blockIdx.x, l = blockIdx.y;
  const int k = pick_level(L, l).k;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float maxc = -INFINITY;
#pragma unroll
  for (int j = 0; j < 5; ++j) maxc = fmaxf(maxc, sel_max[f * 5 + j]);
  const float off = (float)l * (maxc + 1.0f);
  const float* sl = sel + (size_t)(f * 5 + l) * vge::FR_MAXK * vge::FR_SEL;
  {
    const floatx4 b = *reinterpret_cast<const floatx4*>(sl + tid * vge::FR_SEL);
    const float v = sl[tid * vge::FR_SEL + 5];
    const float4 o = make_float4(b.x + off, b.y + off, b.z + off, b.w + off);
    bx[tid] = o;
    area[tid] = (o.z - o.x) * (o.w - o.y);
    vld[tid] = tid < k && v != 0.f;
  }
  __syncthreads();
  const int nw = (k + 63) >> 6;
  // the upper triangle only: row i's words from i's own (the scan never reads a word below it: those boxes are
  // decided); a pair without intersection is not > thr (thr >= 0) and skips the division
  for (int i = wave; i < k; i += 16) {
    if (!vld[i]) {
      for (int w = i >> 6; w < nw; ++w)
        if (lane == 0) mask[i * 16 + w] = 0ull;
      continue;
    }
    const float4 bi = bx[i];
    const float ai = area[i];
    for (int w = i >> 6; w < nw; ++w) {
      const int j = 64 * w + lane;
      bool sup = false;
      if (j > i && j < k && vld[j]) {
        const float4 bj = bx[j];
        const float left = fmaxf(bi.x, bj.x), right = fminf(bi.z, bj.z);
        const float top = fmaxf(bi.y, bj.y), bottom = fminf(bi.w, bj.w);
        const float inter = fmaxf(right - left, 0.f) * fmaxf(bottom - top, 0.f);
        if (inter > 0.f || thr < 0.f) sup = inter / ((ai + area[j]) - inter) > thr;  // iou_gt
      }
      const u64 bits = __ballot(sup);
      if (lane == 0) mask[i * 16 + w] = bits;
    }
  }
  __syncthreads();
  // the greedy scan by one wave: lane w holds the removed-bits word of boxes 64w .. 64w + 63 (invalid boxes start
  // removed), the next live box is the lowest clear bit (a box only suppresses later ones, so this is torchvision's
  // order), and only the kept boxes' indices are recorded (in LDS, over the areas); the copy-out runs after the scan
  __shared__ int s_nk;
  int* keep = reinterpret_cast<int*>(area);
  if (wave == 0) {
    u64 remv = 0;
    for (int w = 0; w < nw; ++w) {
      const int j = 64 * w + lane;
      const u64 v = __ballot(j < k && vld[j]);
      if (lane == w) remv = ~v;
    }
    int nk = 0;
    for (int w = 0; w < nw; ++w) {
      for (;;) {
        const u64 live = ~readlane64(remv, w);
        if (live == 0ull) break;
        const int b = __builtin_ctzll(live), i = 64 * w + b;
        if (lane < nw) remv |= mask[i * 16 + lane];
        if (lane == w) remv |= 1ull << b;
        if (lane == 0) keep[nk] = i;
        ++nk;
      }
    }
    if (lane == 0) {
      s_nk = nk;
      kcount[f * 5 + l] = nk;
    }
  }
  __syncthreads();
  float* ko = kept + (size_t)(f * 5 + l) * vge::FR_MAXK * vge::FR_SEL;
  for (int t = tid; t < s_nk * 5; t += 1024) {
    const int r = t / 5, q = t - 5 * r;
    ko[r * vge::FR_SEL + q] = sl[keep[r] * vge::FR_SEL + q];
  }
}

__global__ void __launch_bounds__(1024) rpn_merge_kernel(const float* __restrict__ kept, const int* __restrict__ kcount,
                                                         int post_k, float* __restrict__ props, int* __restrict__ n_prop) {
  const int f = blockIdx.x;
  int c[5], base[6];
  base[0] = 0;
#pragma unroll
  for (int l = 0; l < 5; ++l) {
    c[l] = kcount[f * 5 + l];
    base[l + 1] = base[l] + c[l];
  }
  const float* kf = kept + (size_t)f * 5 * vge::FR_MAXK * vge::FR_SEL;
  for (int g = threadIdx.x; g < base[5]; g += blockDim.x) {
    int l = 0;
    while (g >= base[l + 1]) ++l;
    const int j = g - base[l];
    const float* e = kf + ((size_t)l * vge::FR_MAXK + j) * vge::FR_SEL;
    const float s = e[4];
    int rank = j;
    for (int m = 0; m < 5; ++m) {
      if (m == l) continue;
      const float* lm = kf + (size_t)m * vge::FR_MAXK * vge::FR_SEL;
      int lo = 0, hi = c[m];  // first position whose score is below s (m < l: ties precede) / not above s (m > l)
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        const float v = lm[mid * vge::FR_SEL + 4];
        if (m < l ? (v >= s) : (v > s))
          lo = mid + 1;
        else
          hi = mid;
      }
      rank += lo;
    }
    if (rank < post_k) {
      float* o = props + ((size_t)f * post_k + rank) * 5;
#pragma unroll
      for (int q = 0; q < 5; ++q) o[q] = e[q];
    }
  }
  if (threadIdx.x == 0) n_prop[f] = base[5] < post_k ? base[5] : post_k;
}

// ------------------------------------------------------------------------------------------------ ROIAlignV2
__global__ void __launch_bounds__(256) roi_align_kernel(vge::RoiLevels L, const float* __restrict__ props,
                                                        const int* __restrict__ n_prop, int P, bf16* __restrict__ out) {
  const int f = blockIdx.x / P, r = blockIdx.x - f * P;
  bf16* o = out + (size_t)blockIdx.x * 49 * 256;
  const int g = threadIdx.x >> 5, c8 = (threadIdx.x & 31) * 8;
  if (r >= n_prop[f]) {
    bf16x8 z;
#pragma unroll
    for (int c = 0; c < 8; ++c) z[c] = (bf16)0.f;
    for (int b = g; b < 49; b += 8) *reinterpret_cast<bf16x8*>(o + b * 256 + c8) = z;
    return;
  }
  const float* pb = props + ((size_t)f * P + r) * 5;
  const float x1 = pb[0], y1 = pb[1], x2 = pb[2], y2 = pb[3];
  const float area = (x2 - x1) * (y2 - y1);
  float lvf = floorf(4.0f + log2f(sqrtf(area) / 224.0f + 1e-8f));
  lvf = fminf(fmaxf(lvf, 2.f), 5.f);
  const int l = (int)lvf - 2;
  const bf16* feat = static_cast<const bf16*>(l == 0 ? L.p[0] : l == 1 ? L.p[1] : l == 2 ? L.p[2] : L.p[3]);
  const int H = l == 0 ? L.h[0] : l == 1 ? L.h[1] : l == 2 ? L.h[2] : L.h[3];
  const int W = l == 0 ? L.w[0] : l == 1 ? L.w[1] : l == 2 ? L.w[2] : L.w[3];
  const float scale = l == 0 ? 0.25f : l == 1 ? 0.125f : l == 2 ? 0.0625f : 0.03125f;
  feat += (size_t)f * H * W * 256 + c8;
  const float sw = x1 * scale - 0.5f, sh = y1 * scale - 0.5f;
  const float ew = x2 * scale - 0.5f, eh = y2 * scale - 0.5f;
  const float rw = ew - sw, rh = eh - sh;
  const float bw = rw / 7.f, bh = rh / 7.f;
  const int gh = (int)ceilf(rh / 7.f), gw = (int)ceilf(rw / 7.f);
  const float cnt = (float)max(gh * gw, 1);
  for (int b = g; b < 49; b += 8) {
    const int ph = b / 7, pw = b - 7 * (b / 7);
    float acc[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) acc[c] = 0.f;
    for (int iy = 0; iy < gh; ++iy) {
      float y = (sh + (float)ph * bh) + (((float)iy + 0.5f) * bh) / (float)gh;
      for (int ix = 0; ix < gw; ++ix) {
        float x = (sw + (float)pw * bw) + (((float)ix + 0.5f) * bw) / (float)gw;
        if (y < -1.0f || y > (float)H || x < -1.0f || x > (float)W) continue;  // contributes 0
        float yy = y <= 0.f ? 0.f : y, xx = x <= 0.f ? 0.f : x;
        int yl = (int)yy, xl = (int)xx, yh, xh;
        if (yl >= H - 1) {
          yh = yl = H - 1;
          yy = (float)yl;
        } else {
          yh = yl + 1;
        }
        if (xl >= W - 1) {
          xh = xl = W - 1;
          xx = (float)xl;
        } else {
          xh = xl + 1;
        }
        const float ly = yy - (float)yl, lx = xx - (float)xl, hy = 1.f - ly, hx = 1.f - lx;
        const float w1 = hy * hx, w2 = hy * lx, w3 = ly * hx, w4 = ly * lx;
        const bf16x8 v1 = *reinterpret_cast<const bf16x8*>(feat + ((size_t)yl * W + xl) * 256);
        const bf16x8 v2 = *reinterpret_cast<const bf16x8*>(feat + ((size_t)yl * W + xh) * 256);
        const bf16x8 v3 = *reinterpret_cast<const bf16x8*>(feat + ((size_t)yh * W + xl) * 256);
        const bf16x8 v4 = *reinterpret_cast<const bf16x8*>(feat + ((size_t)yh * W + xh) * 256);
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          float t = w1 * (float)v1[c] + w2 * (float)v2[c];
          t = t + w3 * (float)v3[c];
          t = t + w4 * (float)v4[c];
          acc[c] = acc[c] + t;
        }
      }
    }
    bf16x8 q;
#pragma unroll
    for (int c = 0; c < 8; ++c) q[c] = (bf16)(acc[c] / cnt);
    *reinterpret_cast<bf16x8*>(o + b * 256 + c8) = q;
  }
}

// ROIAlignV2, separable form (the default).  A bin's sum over its gh x gw samples of the four bilinear taps is a sum
// over the cells of its support: sum_(cy, cx) Wy(cy) Wx(cx) f(cy, cx), with Wy(cy) = sum over the valid samples iy of
// the y-weight they give cell cy (hy to yl, ly to yh) and Wx likewise -- the sample grid is a product, a sample is
// valid iff its y and its x are, and the per-sample tap weights are products hy * hx.  The sample spacing is at most one
// cell, so a bin's support is gh + 1 cells along y (gh + 2 at most, float rounding), gw + 1 along x: (gh + 1)(gw + 1)
// cell terms instead of 4 gh gw sample taps (9 vs 16 at 2 x 2 samples, 16 vs 36 at 3 x 3), each one 16-B load and 8
// FMAs, and the per-sample coordinate / weight arithmetic leaves the channel loop.  Per ROI the
// 14 axis tables (7 bins x 2 axes) are built once in LDS; group g of 32 lanes (8 channels each) computes output row
// ph = g, loading a bin's cells in batches of 2 rows x 4 columns (8 loads in flight before their FMAs; the cells past
// the support read 0 through an empty buffer offset, with weight 0).  Bins wider than RA_MAXC - 3 samples (elongated boxes on a fine level) take the sample loop of
// roi_align_kernel.  The sums are reassociated relative to torchvision's sample order: rare 1-ulp bf16 differences.
constexpr int RA_MAXC = 16;
constexpr int RA_OOB = 0x7FFFFFF0;
// rows of cells per load batch (x 4 columns): 2 x 4 measured faster than 4 x 4, and skipping the FMAs of the cells
// outside the support (a uniform branch per column) no faster than weight 0 x a zero load (profiles/ab_r06ae_frcnn_roi_nms.json)
constexpr int RA_BR = 2;  // a buffer offset past any record range: the load returns 0

__device__ __forceinline__ void roi_axis_table(float s, float bs, int n, int p, int L, float* tab, int& c0, int& nc) {
#pragma unroll
  for (int j = 0; j < RA_MAXC + 4; ++j) tab[j] = 0.f;
  c0 = 0;
  nc = 0;
  bool first = true;
  for (int i = 0; i < n; ++i) {
    const float v = (s + (float)p * bs) + (((float)i + 0.5f) * bs) / (float)n;  // roi_align_kernel's y / x
    if (v < -1.0f || v > (float)L) continue;
    float vv = v <= 0.f ? 0.f : v;
    int lo = (int)vv, hi;
    if (lo >= L - 1) {
      hi = lo = L - 1;
      vv = (float)lo;
    } else {
      hi = lo + 1;
    }
    const float l = vv - (float)lo, h = 1.f - l;
    if (first) {
      c0 = lo;
      first = false;
    }
    if (hi - c0 >= RA_MAXC) break;  // not reached: the caller bounds n + 3 <= RA_MAXC
    tab[lo - c0] += h;
    tab[hi - c0] += l;
    nc = hi - c0 + 1;
  }
}

__global__ void __launch_bounds__(224) roi_align_sep_kernel(vge::RoiLevels L, const float* __restrict__ props,
                                                            const int* __restrict__ n_prop, int P,
                                                            bf16* __restrict__ out, int maxc) {
  __shared__ float wtab[14][RA_MAXC + 4];  // + 4: a batch's columns past the table read 0
  __shared__ int c0s[14], ncs[14];
  const int f = blockIdx.x / P, r = blockIdx.x - f * P;
  bf16* o = out + (size_t)blockIdx.x * 49 * 256;
  const int g = threadIdx.x >> 5, c8 = (threadIdx.x & 31) * 8;  // g = output row ph
  if (r >= n_prop[f]) {
    bf16x8 z;
#pragma unroll
    for (int c = 0; c < 8; ++c) z[c] = (bf16)0.f;
    for (int pw = 0; pw < 7; ++pw) *reinterpret_cast<bf16x8*>(o + (g * 7 + pw) * 256 + c8) = z;
    return;
  }
  const float* pb = props + ((size_t)f * P + r) * 5;
  const float x1 = pb[0], y1 = pb[1], x2 = pb[2], y2 = pb[3];
  const float area = (x2 - x1) * (y2 - y1);
  float lvf = floorf(4.0f + log2f(sqrtf(area) / 224.0f + 1e-8f));
  lvf = fminf(fmaxf(lvf, 2.f), 5.f);
  const int l = (int)lvf - 2;
  const bf16* feat = static_cast<const bf16*>(l == 0 ? L.p[0] : l == 1 ? L.p[1] : l == 2 ? L.p[2] : L.p[3]);
  const int H = l == 0 ? L.h[0] : l == 1 ? L.h[1] : l == 2 ? L.h[2] : L.h[3];
  const int W = l == 0 ? L.w[0] : l == 1 ? L.w[1] : l == 2 ? L.w[2] : L.w[3];
  const float scale = l == 0 ? 0.25f : l == 1 ? 0.125f : l == 2 ? 0.0625f : 0.03125f;
  const bf16* fbase = feat + (size_t)f * H * W * 256;  // uniform: the buffer resource's base
  feat = fbase + c8;
  const float sw = x1 * scale - 0.5f, sh = y1 * scale - 0.5f;
  const float ew = x2 * scale - 0.5f, eh = y2 * scale - 0.5f;
  const float rw = ew - sw, rh = eh - sh;
  const float bw = rw / 7.f, bh = rh / 7.f;
  const int gh = (int)ceilf(rh / 7.f), gw = (int)ceilf(rw / 7.f);
  const float cnt = (float)max(gh * gw, 1);
  if (gh + 3 > maxc || gw + 3 > maxc) {  // the sample loop (uniform per workgroup; maxc = RA_MAXC, 0 in a test)
    for (int pw = 0; pw < 7; ++pw) {
      const int ph = g;
      float acc[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) acc[c] = 0.f;
      for (int iy = 0; iy < gh; ++iy) {
        float y = (sh + (float)ph * bh) + (((float)iy + 0.5f) * bh) / (float)gh;
        for (int ix = 0; ix < gw; ++ix) {
          float x = (sw + (float)pw * bw) + (((float)ix + 0.5f) * bw) / (float)gw;
          if (y < -1.0f || y > (float)H || x < -1.0f || x > (float)W) continue;
          float yy = y <= 0.f ? 0.f : y, xx = x <= 0.f ? 0.f : x;
          int yl = (int)yy, xl = (int)xx, yh, xh;
          if (yl >= H - 1) {
            yh = yl = H - 1;
            yy = (float)yl;
          } else {
            yh = yl + 1;
          }
          if (xl >= W - 1) {
            xh = xl = W - 1;
            xx = (float)xl;
          } else {
            xh = xl + 1;
          }
          const float ly = yy - (float)yl, lx = xx - (float)xl, hy = 1.f - ly, hx = 1.f - lx;
          const float w1 = hy * hx, w2 = hy * lx, w3 = ly * hx, w4 = ly * lx;
          const bf16x8 v1 = *reinterpret_cast<const bf16x8*>(feat + ((size_t)yl * W + xl) * 256);
          const bf16x8 v2 = *reinterpret_cast<const bf16x8*>(feat + ((size_t)yl * W + xh) * 256);
          const bf16x8 v3 = *reinterpret_cast<const bf16x8*>(feat + ((size_t)yh * W + xl) * 256);
          const bf16x8 v4 = *reinterpret_cast<const bf16x8*>(feat + ((size_t)yh * W + xh) * 256);
#pragma unroll
          for (int c = 0; c < 8; ++c) {
            float t = w1 * (float)v1[c] + w2 * (float)v2[c];
            t = t + w3 * (float)v3[c];
            t = t + w4 * (float)v4[c];
            acc[c] = acc[c] + t;
          }
        }
      }
      bf16x8 q;
#pragma unroll
      for (int c = 0; c < 8; ++c) q[c] = (bf16)(acc[c] / cnt);
      *reinterpret_cast<bf16x8*>(o + (ph * 7 + pw) * 256 + c8) = q;
    }
    return;
  }
  if (threadIdx.x < 14) {  // tables: 0..6 the rows ph, 7..13 the columns pw
    const int t = threadIdx.x;
    const bool ya = t < 7;
    roi_axis_table(ya ? sh : sw, ya ? bh : bw, ya ? gh : gw, ya ? t : t - 7, ya ? H : W, wtab[t], c0s[t], ncs[t]);
  }
  __syncthreads();
  // cells in batches of 2 rows x 4 columns, the 8 loads issued before their FMAs; cells past the bin's support read
  // through an empty offset (buffer loads return 0 there) with weight 0 from the zero-filled tables
  const __amdgpu_buffer_rsrc_t fr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16*>(fbase), (short)0, H * W * 512, 0x00020000);
  const int ph = g, y0 = c0s[ph], ny = ncs[ph];
  for (int pw = 0; pw < 7; ++pw) {
    const int x0 = c0s[7 + pw], nx = ncs[7 + pw];
    float acc[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) acc[c] = 0.f;
    for (int j0 = 0; j0 < ny; j0 += RA_BR)
      for (int k0 = 0; k0 < nx; k0 += 4) {
        uintx4_t v[4 * RA_BR];
        float w[4 * RA_BR];
#pragma unroll
        for (int q = 0; q < 4 * RA_BR; ++q) {
          const int j = j0 + (q >> 2), k = k0 + (q & 3);
          const bool in = j < ny && k < nx;
          v[q] = __builtin_amdgcn_raw_buffer_load_b128(fr, in ? ((y0 + j) * W + x0 + k) * 512 + c8 * 2 : RA_OOB, 0, 0);
          w[q] = wtab[ph][j] * wtab[7 + pw][k];
        }
#pragma unroll
        for (int q = 0; q < 4 * RA_BR; ++q) {
          const bf16x8 x = __builtin_bit_cast(bf16x8, v[q]);
#pragma unroll
          for (int c = 0; c < 8; ++c) acc[c] = __builtin_fmaf(w[q], (float)x[c], acc[c]);
        }
      }
    bf16x8 q;
#pragma unroll
    for (int c = 0; c < 8; ++c) q[c] = (bf16)(acc[c] / cnt);
    *reinterpret_cast<bf16x8*>(o + (ph * 7 + pw) * 256 + c8) = q;
  }
}

// ------------------------------------------------------------------------------------- stem + max pool, fused
// ResNet BasicStem: conv1 7x7 / 2 (pad 3, 3 -> 64 channels, FrozenBN folded into the bias) + ReLU, then max_pool2d(3, 2,
// 1), without the stem's output going through HBM.  Persistent (one 512-thread workgroup per CU, the weights staged in
// LDS once); a tile is 7 x 16 pooled pixels, whose 15 x 33 stem pixels (the pool window's halo recomputed) are an
// implicit GEMM of 64 channels x 495 pixels x K = 400 (taps 0..49 x 8 input channels, the padded taps' weights 0) on
// v_mfma_f32_32x32x16_bf16 with the weights as the row operand: each wave owns 2 pixel tiles of 32 x both channel tiles,
// its pixel fragments read from the tile's input patch (35 x 71 pixels x 8 channels, zero outside the frame) in LDS, the
// weight fragments from LDS in fragment order (the patch rows stored as even then odd columns, so the 32 lanes'
// stride-2 pixels are consecutive 16-B chunks: no bank conflicts); a lane's accumulators then hold 4 consecutive channels of one pixel
// (8-B LDS stores of the ReLU'd bf16 values).  Each pooled pixel takes the max of its 3 x 3 window's stem pixels inside
// the frame (-inf padding: the values are >= 0 and the centre is inside, so the ones outside are left out).  Patch,
// stem values and weights have separate LDS regions, so a tile costs two barriers: [MFMAs(t)] | [stem values(t), the
// patch of t + G stored (its loads were issued a tile earlier), the loads of t + 2G issued] | [pool(t), MFMAs(t + G)].
// The stem conv kernel's arithmetic (16-k MFMA steps in tap order, bias then ReLU then bf16): bit-identical outputs.
constexpr int SP_TPH = 7, SP_TPW = 16;                          // pooled tile
constexpr int SP_SR = 2 * SP_TPH + 1, SP_SC = 2 * SP_TPW + 1;   // stem pixels of a tile: 15 x 33 = 495
constexpr int SP_PR = 2 * (SP_SR - 1) + 7, SP_PC = 2 * (SP_SC - 1) + 7;  // input patch: 35 x 71
constexpr int SP_NCH = SP_PR * SP_PC;                           // 16-B patch chunks (one pixel's 8 channels)
constexpr int SP_NLD = (SP_NCH + 511) / 512;                    // per thread: 5
constexpr int SP_STEPS = 25;                                    // K = 400 (taps 0..49)
constexpr int SP_SPITCH = 144;                                  // stem values: bytes per pixel (64 x 2 + 16: banks)
constexpr int SP_W_BYTES = SP_STEPS * 2 * 64 * 16;              // weights in fragment order: 51,200
constexpr int SP_PH = (SP_PC + 1) / 2;                          // patch row: even columns, then odd columns (36 each)
constexpr int SP_P_BYTES = SP_PR * 2 * SP_PH * 16;               // patch: 40,320
constexpr int SP_S_BYTES = SP_SR * SP_SC * SP_SPITCH;           // stem values: 71,280
constexpr int SP_LDS = SP_W_BYTES + SP_P_BYTES + SP_S_BYTES;    // 162,800
constexpr int SP_OOB = 0x7FFFFFF0;

__global__ void __launch_bounds__(512, 1) frcnn_stem_pool_kernel(const bf16* __restrict__ in, const bf16* __restrict__ w,
                                                                 int Kp, const float* __restrict__ bias,
                                                                 bf16* __restrict__ out, int n, int hp, int wp,
                                                                 int tiles_y, int tiles_x) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  char* wl = lds;
  char* pat = lds + SP_W_BYTES;
  char* stv = pat + SP_P_BYTES;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5;
  const int Hs = hp >> 1, Ws = wp >> 1, Hp = Hs >> 1, Wp = Ws >> 1;
  const int G = gridDim.x, tpi = tiles_y * tiles_x, ntiles = n * tpi;
  // weights [64][Kp] -> fragment order [step][u][lane] (16 B): channel 32u + (lane & 31), k = 16 step + 8 (lane >> 5)
  for (int c = tid; c < SP_STEPS * 2 * 64; c += 512) {
    const int l = c & 63, u = (c >> 6) & 1, st = c >> 7;
    const int col = 32 * u + (l & 31), k = 16 * st + 8 * (l >> 5);
    *reinterpret_cast<uintx4_t*>(wl + c * 16) = *reinterpret_cast<const uintx4_t*>(w + (size_t)col * Kp + k);
  }
  const int img_bytes = hp * wp * 16;
  auto load_patch = [&](int t, uintx4_t (&v)[SP_NLD]) {  // t >= ntiles: an empty record range (zeros, no traffic)
    const int img = t / tpi, r = t - img * tpi;
    const int ty = r / tiles_x, tx = r - ty * tiles_x;
    const int iy0 = 4 * SP_TPH * ty - 5, ix0 = 4 * SP_TPW * tx - 5;
    const __amdgpu_buffer_rsrc_t ir = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<bf16*>(in + (size_t)(t < ntiles ? img : 0) * hp * wp * 8), (short)0, t < ntiles ? img_bytes : 0,
        0x00020000);
#pragma unroll
    for (int q = 0; q < SP_NLD; ++q) {
      const int c = tid + 512 * q, pr = c / SP_PC, pc = c - pr * SP_PC;
      const int iy = iy0 + pr, ix = ix0 + pc;
      const bool ok = c < SP_NCH && (unsigned)iy < (unsigned)hp && (unsigned)ix < (unsigned)wp;
      v[q] = __builtin_amdgcn_raw_buffer_load_b128(ir, ok ? (iy * wp + ix) * 16 : SP_OOB, 0, 0);
    }
  };
  auto store_patch = [&](const uintx4_t (&v)[SP_NLD]) {
#pragma unroll
    for (int q = 0; q < SP_NLD; ++q) {
      const int c = tid + 512 * q, pr = c / SP_PC, pc = c - pr * SP_PC;
      if (c < SP_NCH) *reinterpret_cast<uintx4_t*>(pat + (pr * 2 * SP_PH + (pc & 1) * SP_PH + (pc >> 1)) * 16) = v[q];
    }
  };
  // this lane's pixel column: stem pixel 32 pt + (lane & 31) of pixel tiles pt = 2 wave, 2 wave + 1 (the last tile's
  // 17 pad columns are clamped to a real pixel and never stored)
  int pbase[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int sidx = min(32 * (2 * wave + i) + (lane & 31), SP_SR * SP_SC - 1);
    const int sr = sidx / SP_SC, sc = sidx - sr * SP_SC;
    pbase[i] = (2 * sr * 2 * SP_PH + sc) * 16;  // column 2 sc + kx: half kx & 1, index sc + kx / 2
  }
  // the bias of this lane's channels: 32u + 8g + 4h + j (accumulator register 4g + j)
  floatx4 bq[2][4];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int g = 0; g < 4; ++g) bq[u][g] = *reinterpret_cast<const floatx4*>(bias + 32 * u + 8 * g + 4 * h);

  uintx4_t pv[SP_NLD];
  int t = blockIdx.x;
  load_patch(t, pv);
  store_patch(pv);
  load_patch(t + G, pv);
  __syncthreads();  // weights and the first patch in LDS
  for (; t < ntiles; t += G) {
    floatx16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][u][r] = 0.f;
#pragma unroll
    for (int st = 0; st < SP_STEPS; ++st) {
      const int tap0 = 2 * st, tap1 = 2 * st + 1;  // this lane's tap: tap0 + h (tap 49 reads tap 48: weight 0)
      constexpr auto toffs = [](int tap) {
        const int ky = tap / 7, kx = tap % 7;
        return (ky * 2 * SP_PH + (kx & 1) * SP_PH + (kx >> 1)) * 16;
      };
      const int o0 = toffs(tap0), o1 = tap1 < 49 ? toffs(tap1) : o0;
      const int toff = h ? o1 : o0;
      bf16x8 px[2], wf[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) px[i] = *reinterpret_cast<const bf16x8*>(pat + pbase[i] + toff);
#pragma unroll
      for (int u = 0; u < 2; ++u) wf[u] = *reinterpret_cast<const bf16x8*>(wl + ((st * 2 + u) * 64 + lane) * 16);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int u = 0; u < 2; ++u) acc[i][u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[u], px[i], acc[i][u], 0, 0, 0);
    }
    __syncthreads();  // A: the patch is free, and every wave's pool of the previous tile is done
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int sidx = 32 * (2 * wave + i) + (lane & 31);
      if (sidx < SP_SR * SP_SC) {
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
            bf16x4_t o;
#pragma unroll
            for (int j = 0; j < 4; ++j) o[j] = (bf16)fmaxf(acc[i][u][4 * g + j] + bq[u][g][j], 0.f);
            *reinterpret_cast<bf16x4_t*>(stv + sidx * SP_SPITCH + (32 * u + 8 * g + 4 * h) * 2) = o;
          }
      }
    }
    store_patch(pv);        // the patch of t + G (zeros past the end)
    load_patch(t + 2 * G, pv);
    __syncthreads();  // B: stem values and the next patch in LDS
    const int img = t / tpi, r = t - img * tpi;
    const int ty = r / tiles_x, tx = r - ty * tiles_x;
    const int sy0 = 2 * SP_TPH * ty - 1, sx0 = 2 * SP_TPW * tx - 1;
    for (int task = tid; task < SP_TPH * SP_TPW * 8; task += 512) {  // 7 x 16 pooled pixels x 8 channel groups
      const int g = task & 7, pp = task >> 3, py = pp / SP_TPW, px = pp - py * SP_TPW;
      const int oy = SP_TPH * ty + py, ox = SP_TPW * tx + px;
      bf16x8 m;
#pragma unroll
      for (int c = 0; c < 8; ++c) m[c] = (bf16)0.f;
#pragma unroll
      for (int dy = 0; dy < 3; ++dy)
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) {  // a stem pixel outside the frame reads the centre instead (no branch)
          const int sr = 2 * py + dy, sc = 2 * px + dx;
          const bool in = (unsigned)(sy0 + sr) < (unsigned)Hs && (unsigned)(sx0 + sc) < (unsigned)Ws;
          const int cell = in ? sr * SP_SC + sc : (2 * py + 1) * SP_SC + 2 * px + 1;
          const bf16x8 v = *reinterpret_cast<const bf16x8*>(stv + cell * SP_SPITCH + g * 16);
#pragma unroll
          for (int c = 0; c < 8; ++c) m[c] = (float)v[c] > (float)m[c] ? v[c] : m[c];
        }
      if (oy < Hp && ox < Wp) *reinterpret_cast<bf16x8*>(out + (((size_t)img * Hp + oy) * Wp + ox) * 64 + g * 8) = m;
    }
  }
}

// ------------------------------------------------------------------------------------------------ box inference
// softmax of one head row over K + 1 <= 128 logits held two per lane (lane l: class l and 64 + l); returns the
// probabilities (0 outside the row)
__device__ __forceinline__ void row_probs(const float* row, int K1, int lane, float& p0, float& p1) {
  const float x0 = lane < K1 ? row[lane] : -INFINITY;
  const float x1 = 64 + lane < K1 ? row[64 + lane] : -INFINITY;
  const float m = wave_max(fmaxf(x0, x1));
  const float e0 = lane < K1 ? expf(x0 - m) : 0.f;
  const float e1 = 64 + lane < K1 ? expf(x1 - m) : 0.f;
  const float s = wave_sum(e0 + e1);
  p0 = e0 / s;
  p1 = e1 / s;
}

__global__ void __launch_bounds__(1024) det_post_kernel(vge::DetPostArgs a, int n) {
  const int f = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  __shared__ u64 keys[vge::FR_MAXCAND];
  __shared__ int rowc[vge::FR_MAXK];
  __shared__ int wsum[16];
  __shared__ float red[16];
  __shared__ int seg0[128], seg1[128];
  __shared__ int s_total;
  float* cand = a.scratch + (size_t)f * vge::FR_MAXCAND * 8;
  u64* mask = reinterpret_cast<u64*>(a.scratch + (size_t)n * vge::FR_MAXCAND * 8) + (size_t)f * vge::FR_MAXK * 16;
  const int R = a.n_prop[f], K = a.K, K1 = a.K + 1;
  const float* head = a.head + (size_t)f * a.P * a.ld;
  const float* props = a.props + (size_t)f * a.P * 5;

  // ---- pass 1: per proposal, the number of classes above the threshold (0 when the row is not finite)
  rowc[tid] = 0;
  __syncthreads();
  for (int r = wave; r < R; r += 16) {
    const float* row = head + (size_t)r * a.ld;
    float p0, p1;
    row_probs(row, K1, lane, p0, p1);
    const float* pb = props + r * 5;
    bool fin = isfinite(p0) && isfinite(p1);
    for (int h = 0; h < 2; ++h) {
      const int c = h * 64 + lane;
      if (c < K) {
        const float* d = row + K1 + 4 * c;
        float x1, y1, x2, y2;
        apply_delta(pb[0], pb[1], pb[2], pb[3], d[0], d[1], d[2], d[3], 10.f, 10.f, 5.f, 5.f, x1, y1, x2, y2);
        fin = fin && isfinite(x1) && isfinite(y1) && isfinite(x2) && isfinite(y2);
      }
    }
    const bool all_fin = __ballot(!fin) == 0ull;
    const int nc = __popcll(__ballot(lane < K && p0 > a.score_thresh)) +
                   __popcll(__ballot(64 + lane < K && p1 > a.score_thresh));
    if (lane == 0) rowc[r] = all_fin ? min(nc, 4) : 0;
  }
  __syncthreads();
  int total;
  const int rbase = block_excl_scan(rowc[tid], wsum, &total);
  __syncthreads();
  rowc[tid] = rbase;  // now the row's first candidate index
  __syncthreads();
  const int ncand = total;

  // ---- pass 2: the candidates in (proposal, class) order: decoded + clipped box, score, class
  for (int r = wave; r < R; r += 16) {
    const int b0 = rowc[r], b1 = r + 1 < vge::FR_MAXK ? rowc[r + 1] : ncand;
    if (b1 == b0) continue;
    const float* row = head + (size_t)r * a.ld;
    float p0, p1;
    row_probs(row, K1, lane, p0, p1);
    const float* pb = props + r * 5;
    const bool s0 = lane < K && p0 > a.score_thresh, s1 = 64 + lane < K && p1 > a.score_thresh;
    const u64 m0 = __ballot(s0), m1 = __ballot(s1);
    const int r0 = __popcll(m0 & ((1ull << lane) - 1ull)), r1 = __popcll(m0) + __popcll(m1 & ((1ull << lane) - 1ull));
    for (int h = 0; h < 2; ++h) {
      const bool s = h ? s1 : s0;
      const int rk = h ? r1 : r0;
      if (!s || b0 + rk >= b1) continue;  // (beyond the row's 4 slots: not reachable, see rowc)
      const int c = h * 64 + lane;
      const float* d = row + K1 + 4 * c;
      float x1, y1, x2, y2;
      apply_delta(pb[0], pb[1], pb[2], pb[3], d[0], d[1], d[2], d[3], 10.f, 10.f, 5.f, 5.f, x1, y1, x2, y2);
      float* e = cand + (size_t)(b0 + rk) * 8;
      *reinterpret_cast<floatx4*>(e) =
          floatx4{clampf(x1, a.img_w), clampf(y1, a.img_h), clampf(x2, a.img_w), clampf(y2, a.img_h)};
      *reinterpret_cast<floatx4*>(e + 4) = floatx4{h ? p1 : p0, (float)c, 0.f, 0.f};
    }
  }
  __syncthreads();

  // ---- the largest candidate coordinate (batched_nms offsets), per-class segments (class asc, score desc, index)
  float mx = -INFINITY;
  for (int i = tid; i < ncand; i += 1024) {
    const floatx4 b = *reinterpret_cast<const floatx4*>(cand + (size_t)i * 8);
    mx = fmaxf(mx, fmaxf(fmaxf(b.x, b.y), fmaxf(b.z, b.w)));
  }
  const float maxc = block_max(mx, red);
  for (int i = tid; i < vge::FR_MAXCAND; i += 1024) {
    u64 key = ~0ull;
    if (i < ncand) {
      const float sc = cand[(size_t)i * 8 + 4];
      const int c = (int)cand[(size_t)i * 8 + 5];
      key = ((u64)c << 44) | ((u64)(~__float_as_uint(sc)) << 12) | (u64)i;
    }
    keys[i] = key;
  }
  if (tid < 128) {
    seg0[tid] = 0;
    seg1[tid] = 0;
  }
  bitonic<vge::FR_MAXCAND, 1024, false>(keys);
  for (int p = tid; p < ncand; p += 1024) {
    const int c = (int)(keys[p] >> 44);
    if (p == 0 || (int)(keys[p - 1] >> 44) != c) seg0[c] = p;
    if (p == ncand - 1 || (int)(keys[p + 1] >> 44) != c) seg1[c] = p + 1;
  }
  __syncthreads();

  // ---- per-class greedy NMS (coordinate trick offsets: class x (max + 1))
  for (int c = 0; c < K; ++c) {
    const int s0 = seg0[c], nc = seg1[c] - s0;
    if (nc <= 0) continue;
    const float off = (float)c * (maxc + 1.0f);
    const int nw = (nc + 63) >> 6;
    for (int p = wave; p < nc * nw; p += 16) {
      const int i = p / nw, w = p - i * nw, j = 64 * w + lane;
      const floatx4 bi = *reinterpret_cast<const floatx4*>(cand + (keys[s0 + i] & 0xFFFull) * 8);
      const float4 oi = make_float4(bi.x + off, bi.y + off, bi.z + off, bi.w + off);
      bool sup = false;
      if (j > i && j < nc) {
        const floatx4 bj = *reinterpret_cast<const floatx4*>(cand + (keys[s0 + j] & 0xFFFull) * 8);
        const float4 oj = make_float4(bj.x + off, bj.y + off, bj.z + off, bj.w + off);
        sup = iou_gt(oi, (oi.z - oi.x) * (oi.w - oi.y), oj, (oj.z - oj.x) * (oj.w - oj.y), a.nms_thresh);
      }
      const u64 bits = __ballot(sup);
      if (lane == 0) mask[(size_t)i * 16 + w] = bits;
    }
    __syncthreads();
    if (wave == 0) {
      u64 remv = 0;
      for (int i = 0; i < nc; ++i) {
        const u64 word = readlane64(remv, i >> 6);
        if (((word >> (i & 63)) & 1ull) == 0ull) {
          if (lane < nw) remv |= mask[(size_t)i * 16 + lane];
          if (lane == 0) cand[(keys[s0 + i] & 0xFFFull) * 8 + 6] = 1.f;
        }
      }
    }
    __syncthreads();
  }

  // ---- kept candidates by (score desc, candidate order); the first det_per_img
  for (int i = tid; i < vge::FR_MAXCAND; i += 1024) {
    u64 key = ~0ull;
    if (i < ncand && cand[(size_t)i * 8 + 6] != 0.f)
      key = ((u64)(~__float_as_uint(cand[(size_t)i * 8 + 4])) << 12) | (u64)i;
    keys[i] = key;
  }
  bitonic<vge::FR_MAXCAND, 1024, false>(keys);
  if (tid == 0) {
    int nd = 0;
    while (nd < a.det_per_img && nd < ncand && keys[nd] != ~0ull) ++nd;
    s_total = nd;
  }
  __syncthreads();
  const int nd = s_total;
  if (a.pre_dets)
    for (int j = tid; j < nd; j += 1024) {
      const float* e = cand + (keys[j] & 0xFFFull) * 8;
      float* o = a.pre_dets + ((size_t)f * a.det_per_img + j) * 6;
#pragma unroll
      for (int q = 0; q < 6; ++q) o[q] = e[q];
    }
  if (tid == 0) {
    if (a.n_pre) a.n_pre[f] = nd;
    // detector_postprocess: scale to the frame, clip, drop empty boxes; the gate's person count
    int m = 0, np = 0, first = 0;
    float pers[2][5] = {{0.f, 0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f, 0.f}};
    for (int j = 0; j < nd; ++j) {
      const float* e = cand + (keys[j] & 0xFFFull) * 8;
      const float x1 = clampf(e[0] * a.sx, a.out_w), y1 = clampf(e[1] * a.sy, a.out_h);
      const float x2 = clampf(e[2] * a.sx, a.out_w), y2 = clampf(e[3] * a.sy, a.out_h);
      if (!((x2 - x1) > 0.f && (y2 - y1) > 0.f)) continue;
      const float sc = e[4], cl = e[5];
      if (a.dets) {
        float* o = a.dets + ((size_t)f * a.det_per_img + m) * 6;
        o[0] = x1;
        o[1] = y1;
        o[2] = x2;
        o[3] = y2;
        o[4] = sc;
        o[5] = cl;
      }
      ++m;
      if (cl == 0.f) {
        if (first < 2) {
          pers[first][0] = x1;
          pers[first][1] = y1;
          pers[first][2] = x2;
          pers[first][3] = y2;
          pers[first][4] = sc;
          ++first;
        }
        if (sc > a.gate_thresh) ++np;
      }
    }
    if (a.n_dets) a.n_dets[f] = m;
    a.n_person[f] = np;
    if (a.person)
      for (int q = 0; q < 10; ++q) a.person[(size_t)f * 10 + q] = pers[q / 5][q % 5];
  }
}

}  // namespace

namespace vge {

size_t det_post_scratch_bytes(int n) {
  return (size_t)n * FR_MAXCAND * 8 * sizeof(float) + (size_t)n * FR_MAXK * 16 * sizeof(u64);
}

hipError_t launch_frcnn_resize_h(const uint8_t* src, int n, int H, int W, int nw, const int* xb, const int* kk, int ks,
                                 uint8_t* dst, hipStream_t s) {
  const long tot = (long)n * H * nw;
  if (tot == 0) return hipSuccess;
  hipLaunchKernelGGL(frcnn_resize_h_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, src, n, H, W, nw, xb,
                     kk, ks, dst);
  return hipGetLastError();
}

hipError_t launch_frcnn_resize_v_norm(const uint8_t* tmp, int n, int H, int nw, int nh, int hp, int wp, const int* yb,
                                      const int* kk, int ks, uint8_t* resized, void* out, hipStream_t s) {
  const long tot = (long)n * hp * wp;
  if (tot == 0) return hipSuccess;
  hipLaunchKernelGGL(frcnn_resize_v_norm_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, tmp, n, H, nw,
                     nh, hp, wp, yb, kk, ks, resized, static_cast<bf16*>(out));
  return hipGetLastError();
}

hipError_t launch_frcnn_stem_pool(const void* in, const void* w, int Kp, const float* bias, void* out, int n, int hp,
                                  int wp, hipStream_t s) {
  if (n == 0) return hipSuccess;
  if (hp % 4 || wp % 4 || Kp < 2 * SP_STEPS * 8 || (long)hp * wp * 16 >= (1l << 31)) return hipErrorInvalidValue;
  const int Hp = hp / 4, Wp = wp / 4;
  const int ty = (Hp + SP_TPH - 1) / SP_TPH, tx = (Wp + SP_TPW - 1) / SP_TPW;
  const long ntiles = (long)n * ty * tx;
  if (ntiles >= (1l << 31)) return hipErrorInvalidValue;
  static LdsAttrOnce attr;
  if (const hipError_t e = attr(reinterpret_cast<const void*>(&frcnn_stem_pool_kernel), SP_LDS); e != hipSuccess) return e;
  int dev = 0, ncu = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return hipErrorUnknown;
  const int grid = (int)std::min<long>(ntiles, ncu);
  hipLaunchKernelGGL(frcnn_stem_pool_kernel, dim3(grid), dim3(512), SP_LDS, s, static_cast<const bf16*>(in),
                     static_cast<const bf16*>(w), Kp, bias, static_cast<bf16*>(out), n, hp, wp, ty, tx);
  return hipGetLastError();
}

hipError_t launch_frcnn_pool_s2(const void* x, void* y, int n, int H, int W, int C, int K, hipStream_t s) {
  const int Ho = (H + 2 * (K / 2) - K) / 2 + 1, Wo = (W + 2 * (K / 2) - K) / 2 + 1;
  const long tot = (long)n * Ho * Wo * (C / 8);
  if (tot == 0) return hipSuccess;
  if (C % 8) return hipErrorInvalidValue;
  const dim3 grid((unsigned)((tot + 255) / 256));
  if (K == 3)
    hipLaunchKernelGGL(frcnn_pool_s2_kernel<3>, grid, dim3(256), 0, s, static_cast<const bf16*>(x), static_cast<bf16*>(y),
                       n, H, W, C, Ho, Wo);
  else if (K == 1)
    hipLaunchKernelGGL(frcnn_pool_s2_kernel<1>, grid, dim3(256), 0, s, static_cast<const bf16*>(x), static_cast<bf16*>(y),
                       n, H, W, C, Ho, Wo);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_rpn_select(const RpnLevels& lv, int n, float img_h, float img_w, float* sel, float* sel_max,
                             hipStream_t s) {
  if (n == 0) return hipSuccess;
  for (int l = 0; l < 5; ++l)
    if (lv.l[l].k < 1 || lv.l[l].k > FR_MAXK) return hipErrorInvalidValue;
  hipLaunchKernelGGL(rpn_select_kernel, dim3(n, 5), dim3(1024), 0, s, lv, img_h, img_w, sel, sel_max);
  return hipGetLastError();
}

hipError_t launch_rpn_nms(const RpnLevels& lv, const float* sel, const float* sel_max, int n, float thr, float* kept,
                          int* kcount, hipStream_t s) {
  if (n == 0) return hipSuccess;
  static LdsAttrOnce attr;
  if (const hipError_t e = attr(reinterpret_cast<const void*>(&rpn_nms_kernel), NMS_LDS); e != hipSuccess) return e;
  hipLaunchKernelGGL(rpn_nms_kernel, dim3(n, 5), dim3(1024), NMS_LDS, s, lv, sel, sel_max, thr, kept, kcount);
  return hipGetLastError();
}

hipError_t launch_rpn_merge(const float* kept, const int* kcount, int n, int post_k, float* props, int* n_prop,
                            hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(rpn_merge_kernel, dim3(n), dim3(1024), 0, s, kept, kcount, post_k, props, n_prop);
  return hipGetLastError();
}

static int g_roi_direct = 0;  // vge_debug_set_roi_direct: 1 = the sample-order kernel, 2 = the separable kernel's
                             // sample-loop branch for every ROI (tests)

hipError_t launch_roi_align(const RoiLevels& lv, const float* props, const int* n_prop, int n, int P, void* out,
                            hipStream_t s) {
  if (n == 0 || P == 0) return hipSuccess;
  static const bool sep = [] {  // VGE_ROI_SEP=0: the sample-order kernel (A/B, tests)
    const char* e = getenv("VGE_ROI_SEP");
    return !(e && e[0] == '0');
  }();
  if (sep && g_roi_direct != 1)
    hipLaunchKernelGGL(roi_align_sep_kernel, dim3(n * P), dim3(224), 0, s, lv, props, n_prop, P, static_cast<bf16*>(out),
                       g_roi_direct == 2 ? 0 : RA_MAXC);
  else
    hipLaunchKernelGGL(roi_align_kernel, dim3(n * P), dim3(256), 0, s, lv, props, n_prop, P, static_cast<bf16*>(out));
  return hipGetLastError();
}

hipError_t launch_det_post(const DetPostArgs& a, int n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  if (a.K + 1 > 128 || a.P > FR_MAXK || a.det_per_img > FR_MAXK) return hipErrorInvalidValue;
  hipLaunchKernelGGL(det_post_kernel, dim3(n), dim3(1024), 0, s, a, n);
  return hipGetLastError();
}

}  // namespace vge

extern "C" int vge_debug_set_roi_direct(int mode) {  // tests / A/B: 1 = roi_align_kernel (torchvision's sample
  vge::g_roi_direct = mode;                           // order), 2 = roi_align_sep_kernel's sample loop for every ROI
  return 0;
}
