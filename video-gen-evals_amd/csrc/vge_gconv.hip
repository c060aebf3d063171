// Grouped 3x3 convolution of the gate detector's ResNeXt bottlenecks (detectron2 BottleneckBlock conv2:
// Conv2d(width, width, 3, stride, padding 1, groups=32, bias=False) + FrozenBatchNorm (folded into weight and bias) +
// ReLU; detectron2/modeling/backbone/resnet.py, the X101-32x8d-FPN config of /root/reference/modifications/
// mesh_generator.py:69-73), NHWC bf16 in and out, f32 accumulation.
//
// A grouped conv moves as many bytes as a dense one but does 1/32 of its arithmetic, so it is HBM-bound: one pass
// over the input (plus a halo) and one over the output.  One workgroup = a TH x TW tile of output pixels x one
// 64-channel slice (64 / group-width whole groups), for GC_NI images in turn (the next image's tile loads in flight
// during this one's MFMAs; the weights are read once for all of them):
//   * the input tile with its halo ((TH-1) S + 3) x ((TW-1) S + 3) pixels x 64 channels is read once into LDS (rows of
//     160 B per pixel and 192 B more per tile row at stride 1 (144 and 80 at stride 2): with those pads the 16-B B-fragment
//     reads of a pixel tile -- 16 pixels that may run across a row end -- hit distinct banks in every ds_read_b128 lane
//     group (2.4x conflicted at the round-5 144-B pitch on the 5 x 25 tiles; a bank model of every tile, tap and lane
//     group picked the pads);
//   * TH x TW is chosen per layer shape on the host (gc_pick_tile: up to 128 output pixels, the pixel tiles of 16 run
//     across the tile's rows), so that the tiles cover the output with little overhang: 5 x 25 at the detector's 200 /
//     100 / 50-wide stride-1 maps, where the fixed 4 x 32 tile ran 33 % idle pixel slots at 50 x 50 (res4);
//   * wave w owns output channels 16w..16w+15 of the slice; its weights (9 taps x the 16-channel K steps of its group,
//     v_mfma_f32_16x16x16_bf16 A fragments, 2 registers each) stay in registers for the whole tile;
//   * per 16-pixel tile, tap and K step one MFMA: A = weights [16 out ch x 16 in ch], B = input [16 in ch x 16 pixels]
//     (8 B per lane from LDS), so a lane ends with 4 consecutive output channels of one pixel: +bias, ReLU, one 8-B
//     store.
// K steps: a 16-channel output tile's inputs are its group's channels, max(group width, 16) of them (group width 8:
// the 16 x 16 weight block holds two groups' 8 x 8 blocks and zeros, as packed by vge_frcnn.cpp's gconv_bn).
#include "vge_common.h"
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <type_traits>

namespace {

typedef short short4v __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef unsigned uintx4_t __attribute__((ext_vector_type(4)));
typedef unsigned uintx2_t __attribute__((ext_vector_type(2)));
constexpr int GC_OOB = 0x7FFFFFF0;  // buffer offset past every record count: loads return 0, stores are dropped

// LDS bytes per input pixel (64 bf16 channels + pad) and extra bytes per input row (the header's bank model)
template <int S>
constexpr int gc_pitch() { return S == 1 ? 160 : 144; }
template <int S>
constexpr int gc_rowpad() { return S == 1 ? 192 : 80; }

struct GconvArgs {
  const __bf16* x;  long ldx;   // NHWC input, channel stride ldx (= width)
  const __bf16* w;  int Kp;     // packed [Npad][Kp = 9 * 64]: k = tap * 64 + (input channel - slice base)
  const float* bias;
  __bf16* out;      long ldo;
  int H, W, Ho, Wo, tiles_x, n_img;
  int th, tw, iw, npix;         // output tile th x tw (th * tw <= 16 gc_npt), input tile iw wide, npix pixels
  float inv_tw, inv_iw;         // 1 / tw, 1 / iw (gc_div)
  int ntiles, nslices, xcd;     // workgroup = (tile, 64-channel slice, image group), tile fastest; xcd: gc_xcd order
};

// Workgroup b of nblk -> its (tile, slice, image group) id.  Workgroups are dealt to the 8 XCDs round robin, so in
// launch order a tile's neighbours -- which read its halo rows -- run on other XCDs and fetch those rows into their own
// L2s; with xcd set each XCD takes a contiguous range of ids instead (bijective), the tiles of a slice and image group
// run side by side on one XCD and the halo rows hit its L2.
__device__ __forceinline__ int gc_xcd(int b, int nblk, int on) {
  if (!on) return b;
  const int q8 = nblk >> 3, r8 = nblk & 7, x8 = b & 7;
  return (x8 < r8 ? x8 * (q8 + 1) : r8 * (q8 + 1) + (x8 - r8) * q8) + (b >> 3);
}
#ifndef VGE_GC_NI
#define VGE_GC_NI 8  // (r06ad, same box: 8 images per workgroup -0.6 % on the detector vs 4)
#endif
#ifndef VGE_GC_PD
#define VGE_GC_PD 1  // images whose tile loads are in flight during an image's MFMAs: 2 measured no faster (r06ad)
#endif
constexpr int GC_NI = VGE_GC_NI;  // images per workgroup: its weights (up to 72 registers) are loaded once for all of them

// 16-pixel tiles per output tile at most: th * tw <= 128 at stride 1, 64 at stride 2 (its wider input tile per pixel)
template <int S>
constexpr int gc_npt() { return S == 1 ? 8 : 4; }
// input tile pixels at most (297 at stride 2: the 4 x 16 tile), and its LDS bytes with up to (16 - 1) S + 3 rows
template <int S>
constexpr int gc_npix_max() { return S == 1 ? 216 : 297; }
template <int S>
constexpr int gc_lds_bytes() { return gc_npix_max<S>() * gc_pitch<S>() + (15 * S + 3) * gc_rowpad<S>(); }

// n / d for 0 <= n < 2^12 and 1 <= d < 2^8 from inv = 1 / d: (n + 0.5) / d lies at least 1 / 512 from an integer, far
// more than the float product's error, so the truncation is exact
__device__ __forceinline__ int gc_div(int n, float inv) { return (int)(((float)n + 0.5f) * inv); }

// KS: 16-channel K steps per tap (max(group width, 16) / 16); S: stride; MF: 0 = v_mfma_f32_16x16x16_bf16 (one per
// 16-channel step), 1 = v_mfma_f32_16x16x32_bf16 (gfx950's full-rate bf16 form: the legacy 16x16x16 issues at half the
// rate, 16 cycles per 8 kFLOP, profiles/pmc_r05u_frcnn_sq.json): KS >= 2 -> two steps of a tap per MFMA, KS = 1 -> two
// taps per MFMA (lanes 0-31 carry tap 2p, lanes 32-63 tap 2p + 1; tap 9 is zero weights)
#ifndef VGE_GC_OCC
#define VGE_GC_OCC 1  // minimum waves per SIMD the register allocation must allow (= workgroups per CU)
#endif
#ifndef VGE_GC_OCC_SMALL
#define VGE_GC_OCC_SMALL 3  // the same for group widths <= 32 (res2-4): 3 fit without scratch (<= 163 VGPRs)
#endif
template <int KS, int S, int MF>
__global__ void __launch_bounds__(256, KS <= 2 ? VGE_GC_OCC_SMALL : VGE_GC_OCC) gconv3_kernel(GconvArgs a) {
  constexpr int NPIXM = gc_npix_max<S>();
  constexpr int PITCH = gc_pitch<S>(), ROWPAD = gc_rowpad<S>();
  __shared__ __attribute__((aligned(16))) char tile[gc_lds_bytes<S>()];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int bid = gc_xcd(blockIdx.x, gridDim.x, a.xcd), tile_id = bid % a.ntiles, rest = bid / a.ntiles;
  const int slice = rest % a.nslices, img0 = (rest / a.nslices) * GC_NI, nimg = min(GC_NI, a.n_img - img0);
  const int ty = tile_id / a.tiles_x, tx = tile_id - ty * a.tiles_x;
  const int TW = a.tw, IW = a.iw, NPIX = a.npix, NPX = a.th * TW, npt = (NPX + 15) >> 4;
  const int oy0 = ty * a.th, ox0 = tx * TW;
  const int iy0 = oy0 * S - 1, ix0 = ox0 * S - 1;

  // ---- the input tile of image img into registers: buffer loads through a per-image resource, a pixel outside the
  // image (the conv's zero padding) at an offset past the record count, so that every load issues unconditionally and
  // the next image's loads stay in flight across this image's MFMAs (a branch around each load made the compiler wait
  // for them right after issuing; stores count in the same vmcnt, so the epilogue stores are buffer stores too)
  constexpr int NLD = (NPIXM * 8 + 255) / 256;
  int gofs[NLD];  // byte offsets inside an image (the same for every image of the workgroup)
#pragma unroll
  for (int q = 0; q < NLD; ++q) {
    const int c = tid + 256 * q, p = c >> 3, j = c & 7;
    const int dy = gc_div(p, a.inv_iw), iy = iy0 + dy, ix = ix0 + p - dy * IW;
    gofs[q] = (p < NPIX && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W)
                  ? ((iy * a.W + ix) * (int)a.ldx + j * 8) * 2 : GC_OOB;
  }
  const int in_bytes = (a.H * a.W * (int)a.ldx - slice * 64) * 2;
  auto load_tile = [&](uintx4_t (&v)[NLD], int img, bool real) {  // real = false: the same loads, empty record range
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<__bf16*>(a.x + (size_t)img * a.H * a.W * a.ldx + slice * 64), (short)0, real ? in_bytes : 0,
        0x00020000);
#pragma unroll
    for (int q = 0; q < NLD; ++q) v[q] = __builtin_amdgcn_raw_buffer_load_b128(xr, gofs[q], 0, 0);
  };
  auto store_tile = [&](const uintx4_t (&v)[NLD]) {
#pragma unroll
    for (int q = 0; q < NLD; ++q) {
      const int c = tid + 256 * q, p = c >> 3, j = c & 7;
      if (p < NPIX) *reinterpret_cast<uintx4_t*>(tile + p * PITCH + gc_div(p, a.inv_iw) * ROWPAD + j * 16) = v[q];
    }
  };
  // ---- this wave's weights: 16 output channels x 9 taps x KS K steps (A fragments: lane = output channel l & 15,
  // input channels 4 (l >> 4) .. + 3 of the step)
  const int n0 = wave * 16;
  constexpr int G16 = KS * 16;
  const int cbase = (n0 / G16) * G16;
  // MF = 0: [tap][K step] short4v fragments (4 channels per lane); MF = 1, KS >= 2: [tap][KS / 2] bf16x8 (8 channels per
  // lane); MF = 1, KS = 1: [tap pair][0] bf16x8 (lane half h -> tap 2p + h)
  constexpr int NT = MF && KS == 1 ? 5 : 9;
  constexpr int NJ = MF ? (KS == 1 ? 1 : KS / 2) : KS;
  typedef typename std::conditional<MF != 0, bf16x8_t, short4v>::type Frag;
  Frag wa[NT][NJ];
  const int hh = lane >> 5;  // MF = 1, KS = 1: which tap of the pair
  const int cl = MF ? (KS == 1 ? 8 * ((lane >> 4) & 1) : 8 * (lane >> 4)) : 4 * (lane >> 4);
  const __bf16* wr = a.w + (size_t)(slice * 64 + n0 + (lane & 15)) * a.Kp + cbase + cl;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      if constexpr (MF && KS == 1) {  // (tap 9 loads tap 8 and zeroes it: no branch around a load)
        const int tap = 2 * t + hh;
        const Frag f = *reinterpret_cast<const Frag*>(wr + min(tap, 8) * 64);
        wa[t][j] = tap < 9 ? f : Frag{};
      } else {
        wa[t][j] = *reinterpret_cast<const Frag*>(wr + t * 64 + (MF ? 32 : 16) * j);
      }
    }
  const int px = lane & 15;
  const char* lb = tile + (cbase + cl) * 2;
  const int ch = slice * 64 + n0 + 4 * (lane >> 4);
  const floatx4 bv = *reinterpret_cast<const floatx4*>(a.bias + ch);

  // ---- one image from the LDS tile: MFMAs over pixel tiles pt = output pixels pt * 16 .. + 15 of the tile (row-major,
  // running across rows; lanes past the tile's last pixel recompute that pixel and store nothing), then bias + ReLU
  // and the 8 stores (all of them, out of range past npt or for real = false: a fixed store count)
  auto compute = [&](int img, bool real) {
    floatx4 acc[gc_npt<S>()];
#pragma unroll
    for (int pt = 0; pt < gc_npt<S>(); ++pt) acc[pt] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int pt = 0; pt < gc_npt<S>(); ++pt) {
      if (pt >= npt) break;
      const int op = min(pt * 16 + px, NPX - 1), orow = gc_div(op, a.inv_tw), ocol = op - orow * TW;
      const char* pb = lb + ((orow * S) * IW + ocol * S) * PITCH + orow * S * ROWPAD;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        if constexpr (MF && KS == 1) {
          const int ta = 2 * t, tb = 2 * t + 1 < 9 ? 2 * t + 1 : 8;  // (tap 9: zero weights on finite data)
          const int offa = ((ta / 3) * IW + (ta % 3)) * PITCH + (ta / 3) * ROWPAD;
          const int offb = ((tb / 3) * IW + (tb % 3)) * PITCH + (tb / 3) * ROWPAD;
          const bf16x8_t b = *reinterpret_cast<const bf16x8_t*>(pb + (hh ? offb : offa));
          acc[pt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[t][0], b, acc[pt], 0, 0, 0);
        } else {
          const int off = ((t / 3) * IW + (t % 3)) * PITCH + (t / 3) * ROWPAD;
#pragma unroll
          for (int j = 0; j < NJ; ++j) {
            if constexpr (MF) {
              const bf16x8_t b = *reinterpret_cast<const bf16x8_t*>(pb + off + 64 * j);
              acc[pt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[t][j], b, acc[pt], 0, 0, 0);
            } else {
              const short4v b = *reinterpret_cast<const short4v*>(pb + off + 32 * j);
              acc[pt] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(wa[t][j], b, acc[pt], 0, 0, 0);
            }
          }
        }
      }
    }
    // epilogue: lane = pixel l & 15 of the tile, output channels n0 + 4 (l >> 4) .. + 3
    const __amdgpu_buffer_rsrc_t orr = __builtin_amdgcn_make_buffer_rsrc(
        a.out + (size_t)img * a.Ho * a.Wo * a.ldo, (short)0, real ? a.Ho * a.Wo * (int)a.ldo * 2 : 0, 0x00020000);
#pragma unroll
    for (int pt = 0; pt < gc_npt<S>(); ++pt) {
      const int op = pt * 16 + px, r = gc_div(op, a.inv_tw), oy = oy0 + r, ox = ox0 + op - r * TW;
      const int oo = (op < NPX && oy < a.Ho && ox < a.Wo) ? ((oy * a.Wo + ox) * (int)a.ldo + ch) * 2 : GC_OOB;
      bf16x4_t o;
#pragma unroll
      for (int i = 0; i < 4; ++i) o[i] = (__bf16)fmaxf(acc[pt][i] + bv[i], 0.f);
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(uintx2_t, o), orr, oo, 0, 0);
    }
  };
  auto swap_tile = [&](const uintx4_t (&v)[NLD]) {
    __syncthreads();  // every wave is done reading the previous image's tile
    store_tile(v);
    __syncthreads();
  };
  // Every step issues the same loads and stores unconditionally (past the last image: an empty record range for the
  // loads, stores dropped), so the compiler's vmcnt wait for a tile register counts exactly the operations issued
  // after it instead of waiting for them too.  The weights and bias are loaded before the first tile: waiting for
  // the tile waits for them.
#if VGE_GC_PD == 2
  // two images' loads in flight: image k + 2's behind image k's MFMAs, in two alternating register sets
  uintx4_t va[NLD], vb[NLD];
  load_tile(va, img0, true);
  load_tile(vb, img0 + min(1, nimg - 1), 1 < nimg);
  store_tile(va);
  __syncthreads();
  for (int k = 0; k < nimg; k += 2) {
    load_tile(va, img0 + min(k + 2, nimg - 1), k + 2 < nimg);
    compute(img0 + k, true);
    swap_tile(vb);
    load_tile(vb, img0 + min(k + 3, nimg - 1), k + 3 < nimg);
    compute(img0 + min(k + 1, nimg - 1), k + 1 < nimg);
    if (k + 2 < nimg) swap_tile(va);
  }
#else
  uintx4_t v[NLD];
  load_tile(v, img0, true);
  store_tile(v);
  __syncthreads();
  for (int k = 0; k < nimg; ++k) {
    load_tile(v, img0 + min(k + 1, nimg - 1), k + 1 < nimg);  // in flight during this image's MFMAs
    compute(img0 + k, true);
    if (k + 1 < nimg) swap_tile(v);
  }
#endif
}

// Output tile of a grouped conv: th x tw pixels (th * tw <= 16 gc_npt, the input tile within gc_npix_max), by a
// cost per workgroup and image in LDS-byte units: 16-pixel slots x 9 taps x 64 B x 4 waves of B-fragment reads
// (idle slots of a partial tile cost the same), the input tile's global loads and LDS stores, and a fixed part
// (barriers, epilogue).  VGE_GC_TILE="THxTW" forces a tile (A/B), "legacy" the fixed 4 x 32 (stride 1) / 4 x 16.
void gc_pick_tile(int Ho, int Wo, int S, int& th, int& tw) {
  static int fth = -1, ftw = -1;
  if (fth < 0) {
    fth = ftw = 0;
    const char* e = getenv("VGE_GC_TILE");
    if (e && !strcmp(e, "legacy")) fth = ftw = -2;
    else if (e && sscanf(e, "%dx%d", &fth, &ftw) != 2) fth = ftw = 0;
  }
  const int npm = S == 1 ? gc_npix_max<1>() : gc_npix_max<2>(), npx = 16 * (S == 1 ? gc_npt<1>() : gc_npt<2>());
  auto fits = [&](int h, int w) {
    return h >= 1 && w >= 1 && h * w <= npx && ((h - 1) * S + 3) * ((w - 1) * S + 3) <= npm;
  };
  if (fth == -2) {
    th = 4;
    tw = S == 1 ? 32 : 16;
    return;
  }
  if (fth > 0 && fits(fth, ftw)) {
    th = fth;
    tw = ftw;
    return;
  }
  double best = 1e300;
  th = 4;
  tw = S == 1 ? 32 : 16;
  for (int w = 8; w <= 64; ++w)
    for (int h = 1; h <= 16; ++h) {
      if (!fits(h, w)) continue;
      const double tiles = (double)((Ho + h - 1) / h) * ((Wo + w - 1) / w);
      const int npix = ((h - 1) * S + 3) * ((w - 1) * S + 3);
      const double cost = tiles * (((h * w + 15) / 16) * 16.0 * 9 * 64 * 4 / 128 + npix * 5.0 + 600);
      if (cost < best) {
        best = cost;
        th = h;
        tw = w;
      }
    }
}

}  // namespace

namespace vge {

// x / out NHWC bf16 (channel strides ldx / ldo), C = groups x gw channels (a multiple of 64, gw | 64); w / bias as
// vge_frcnn.cpp's gconv_bn packs them; ReLU epilogue
hipError_t launch_gconv3(const void* x, long ldx, const void* w, int Kp, const float* bias, void* out, long ldo,
                         int n_img, int H, int W, int C, int gw, int stride, hipStream_t s) {
  if (C % 64 || gw < 1 || 64 % gw || (stride != 1 && stride != 2) || Kp != 9 * 64 || n_img < 1 || H < 1 || W < 1 ||
      ldx % 4 || ldo % 4 || (double)H * W * ldx * 2 >= 2147483632.0 ||
      (double)((H + 2 - 3) / stride + 1) * ((W + 2 - 3) / stride + 1) * ldo * 2 >= 2147483632.0)
    return hipErrorInvalidValue;  // per-image byte offsets and record counts are int, below GC_OOB
  GconvArgs a{reinterpret_cast<const __bf16*>(x), ldx, reinterpret_cast<const __bf16*>(w), Kp, bias,
              reinterpret_cast<__bf16*>(out), ldo, H, W, (H + 2 - 3) / stride + 1, (W + 2 - 3) / stride + 1, 0, n_img};
  int th, tw;
  gc_pick_tile(a.Ho, a.Wo, stride, th, tw);
  a.th = th;
  a.tw = tw;
  a.iw = (tw - 1) * stride + 3;
  a.npix = ((th - 1) * stride + 3) * a.iw;
  a.inv_tw = 1.f / tw;
  a.inv_iw = 1.f / a.iw;
  a.tiles_x = (a.Wo + tw - 1) / tw;
  a.ntiles = a.tiles_x * ((a.Ho + th - 1) / th);
  a.nslices = C / 64;
  static int xcd = -1;  // VGE_GC_XCD=0: launch order
  if (xcd < 0) {
    const char* e = getenv("VGE_GC_XCD");
    xcd = (e && e[0] == '0') ? 0 : 1;
  }
  a.xcd = xcd;
  const long nblk = (long)a.ntiles * a.nslices * ((n_img + GC_NI - 1) / GC_NI);
  if (nblk >= 2147483647L) return hipErrorInvalidValue;
  const dim3 grid((unsigned)nblk);
  const int ks = gw <= 16 ? 1 : gw / 16;
  static int mf = -1;  // VGE_GC_MF: 1 (default) = 16x16x32, 0 = 16x16x16
  if (mf < 0) {
    const char* e = getenv("VGE_GC_MF");
    mf = (e && e[0] == '0') ? 0 : 1;
  }
#define GC_LAUNCH(KS, S)                                                             \
  do {                                                                               \
    if (mf) hipLaunchKernelGGL((gconv3_kernel<KS, S, 1>), grid, dim3(256), 0, s, a); \
    else hipLaunchKernelGGL((gconv3_kernel<KS, S, 0>), grid, dim3(256), 0, s, a);    \
  } while (0)
  if (stride == 1) {
    if (ks == 1) GC_LAUNCH(1, 1);
    else if (ks == 2) GC_LAUNCH(2, 1);
    else GC_LAUNCH(4, 1);
  } else {
    if (ks == 1) GC_LAUNCH(1, 2);
    else if (ks == 2) GC_LAUNCH(2, 2);
    else GC_LAUNCH(4, 2);
  }
#undef GC_LAUNCH
  return hipGetLastError();
}

}  // namespace vge
