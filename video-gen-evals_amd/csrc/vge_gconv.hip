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
//     144 B: 64 channels + 8 pad, so 16 consecutive pixels' 8-B reads fall on distinct banks);
//   * wave w owns output channels 16w..16w+15 of the slice; its weights (9 taps x the 16-channel K steps of its group,
//     v_mfma_f32_16x16x16_bf16 A fragments, 2 registers each) stay in registers for the whole tile;
//   * per 16-pixel tile, tap and K step one MFMA: A = weights [16 out ch x 16 in ch], B = input [16 in ch x 16 pixels]
//     (8 B per lane from LDS), so a lane ends with 4 consecutive output channels of one pixel: +bias, ReLU, one 8-B
//     store.
// K steps: a 16-channel output tile's inputs are its group's channels, max(group width, 16) of them (group width 8:
// the 16 x 16 weight block holds two groups' 8 x 8 blocks and zeros, as packed by vge_frcnn.cpp's gconv_bn).
#include "vge_common.h"
#include <cstdlib>
#include <type_traits>

namespace {

typedef short short4v __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

constexpr int GC_PITCH = 144;  // LDS bytes per input pixel (64 bf16 channels + 8 pad)

struct GconvArgs {
  const __bf16* x;  long ldx;   // NHWC input, channel stride ldx (= width)
  const __bf16* w;  int Kp;     // packed [Npad][Kp = 9 * 64]: k = tap * 64 + (input channel - slice base)
  const float* bias;
  __bf16* out;      long ldo;
  int H, W, Ho, Wo, tiles_x, n_img;
};
#ifndef VGE_GC_NI
#define VGE_GC_NI 4
#endif
constexpr int GC_NI = VGE_GC_NI;  // images per workgroup: its weights (up to 72 registers) are loaded once for all of them

#ifndef VGE_GC_TH
#define VGE_GC_TH 4
#endif
template <int S>
constexpr int gc_th() { return S == 1 ? VGE_GC_TH : 4; }
template <int S>
constexpr int gc_tw() { return S == 1 ? 32 : 16; }
template <int S>
constexpr int gc_lds() { return ((gc_th<S>() - 1) * S + 3) * ((gc_tw<S>() - 1) * S + 3) * GC_PITCH; }

// KS: 16-channel K steps per tap (max(group width, 16) / 16); S: stride; MF: 0 = v_mfma_f32_16x16x16_bf16 (one per
// 16-channel step), 1 = v_mfma_f32_16x16x32_bf16 (gfx950's full-rate bf16 form: the legacy 16x16x16 issues at half the
// rate, 16 cycles per 8 kFLOP, profiles/pmc_r05u_frcnn_sq.json): KS >= 2 -> two steps of a tap per MFMA, KS = 1 -> two
// taps per MFMA (lanes 0-31 carry tap 2p, lanes 32-63 tap 2p + 1; tap 9 is zero weights)
#ifndef VGE_GC_OCC
#define VGE_GC_OCC 1  // minimum waves per SIMD the register allocation must allow (= workgroups per CU)
#endif
template <int KS, int S, int MF>
__global__ void __launch_bounds__(256, VGE_GC_OCC) gconv3_kernel(GconvArgs a) {
  constexpr int TH = gc_th<S>(), TW = gc_tw<S>(), NPT = TH * TW / 16;
  constexpr int IH = (TH - 1) * S + 3, IW = (TW - 1) * S + 3, NPIX = IH * IW;
  __shared__ __attribute__((aligned(16))) char tile[gc_lds<S>()];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int slice = blockIdx.y, img0 = blockIdx.z * GC_NI, nimg = min(GC_NI, a.n_img - img0);
  const int ty = blockIdx.x / a.tiles_x, tx = blockIdx.x - ty * a.tiles_x;
  const int oy0 = ty * TH, ox0 = tx * TW;
  const int iy0 = oy0 * S - 1, ix0 = ox0 * S - 1;

  // ---- the input tile of image img (zeros outside the image: the conv's padding) into registers
  constexpr int NLD = (NPIX * 8 + 255) / 256;
  uint4 v[NLD];
  auto load_tile = [&](int img) {
    const __bf16* xs = a.x + (size_t)img * a.H * a.W * a.ldx + slice * 64;
#pragma unroll
    for (int q = 0; q < NLD; ++q) {
      const int c = tid + 256 * q, p = c >> 3, j = c & 7;
      const int iy = iy0 + p / IW, ix = ix0 + p % IW;
      v[q] = make_uint4(0, 0, 0, 0);
      if (p < NPIX && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W)
        v[q] = *reinterpret_cast<const uint4*>(xs + ((long)iy * a.W + ix) * a.ldx + j * 8);
    }
  };
  load_tile(img0);
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
      if constexpr (MF && KS == 1) {
        const int tap = 2 * t + hh;
        wa[t][j] = tap < 9 ? *reinterpret_cast<const Frag*>(wr + tap * 64) : Frag{};
      } else {
        wa[t][j] = *reinterpret_cast<const Frag*>(wr + t * 64 + (MF ? 32 : 16) * j);
      }
    }
  const int px = lane & 15;
  const char* lb = tile + (cbase + cl) * 2;
  const int ch = slice * 64 + n0 + 4 * (lane >> 4);
  const floatx4 bv = *reinterpret_cast<const floatx4*>(a.bias + ch);
  for (int k = 0; k < nimg; ++k) {
    const int img = img0 + k;
    if (k > 0) __syncthreads();  // every wave is done reading the previous image's tile
#pragma unroll
    for (int q = 0; q < NLD; ++q) {
      const int c = tid + 256 * q, p = c >> 3, j = c & 7;
      if (p < NPIX) *reinterpret_cast<uint4*>(tile + p * GC_PITCH + j * 16) = v[q];
    }
    __syncthreads();
    if (k + 1 < nimg) load_tile(img + 1);  // the next image's loads in flight during this one's MFMAs

    // ---- MFMAs: pixel tile pt = output pixels pt * 16 .. + 15 of the tile (row-major, TW / 16 tiles per row)
    floatx4 acc[NPT];
#pragma unroll
    for (int pt = 0; pt < NPT; ++pt) acc[pt] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int pt = 0; pt < NPT; ++pt) {
      const int op = pt * 16 + px, orow = op / TW, ocol = op % TW;
      const char* pb = lb + ((orow * S) * IW + ocol * S) * GC_PITCH;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        if constexpr (MF && KS == 1) {
          const int ta = 2 * t, tb = 2 * t + 1 < 9 ? 2 * t + 1 : 8;  // (tap 9: zero weights on finite data)
          const int offa = ((ta / 3) * IW + (ta % 3)) * GC_PITCH, offb = ((tb / 3) * IW + (tb % 3)) * GC_PITCH;
          const bf16x8_t b = *reinterpret_cast<const bf16x8_t*>(pb + (hh ? offb : offa));
          acc[pt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[t][0], b, acc[pt], 0, 0, 0);
        } else {
          const int off = ((t / 3) * IW + (t % 3)) * GC_PITCH;
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
    // ---- epilogue: lane = pixel l & 15 of the tile, output channels n0 + 4 (l >> 4) .. + 3
#pragma unroll
    for (int pt = 0; pt < NPT; ++pt) {
      const int op = pt * 16 + px, oy = oy0 + op / TW, ox = ox0 + op % TW;
      if (oy < a.Ho && ox < a.Wo) {
        bf16x4_t o;
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = (__bf16)fmaxf(acc[pt][i] + bv[i], 0.f);
        *reinterpret_cast<bf16x4_t*>(a.out + (((size_t)img * a.Ho + oy) * a.Wo + ox) * a.ldo + ch) = o;
      }
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
      ldx % 4 || ldo % 4)
    return hipErrorInvalidValue;
  GconvArgs a{reinterpret_cast<const __bf16*>(x), ldx, reinterpret_cast<const __bf16*>(w), Kp, bias,
              reinterpret_cast<__bf16*>(out), ldo, H, W, (H + 2 - 3) / stride + 1, (W + 2 - 3) / stride + 1, 0, n_img};
  const int th = stride == 1 ? VGE_GC_TH : 4, tw = stride == 1 ? 32 : 16;
  a.tiles_x = (a.Wo + tw - 1) / tw;
  const dim3 grid(a.tiles_x * ((a.Ho + th - 1) / th), C / 64, (n_img + GC_NI - 1) / GC_NI);
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
