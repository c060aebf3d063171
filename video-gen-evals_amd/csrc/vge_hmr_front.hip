// TokenHMR front end (gfx950): the person crop of ViTDetDataset (4D-Humans hmr2/datasets/vitdet_dataset.py,
// driven by modifications/mesh_generator.py:119-145; third-party code absent from /root/reference, restated from
// its published algorithm -- parity unpinned):
//   box xyxy -> center = (p0 + p1) / 2, scale = 2.5 (p1 - p0) / 200, bbox = expand_to_aspect_ratio(scale * 200,
//   [192, 256]).max();  when bbox / 256 / 2 > 1.1 the frame is first blurred (skimage.filters.gaussian, sigma =
//   (bbox / 512 - 1) / 2, mode 'nearest', truncate 4);  cv2.warpAffine(INTER_LINEAR, BORDER_CONSTANT 0) of the
//   256 x 256 patch centred on the box (generate_image_patch_cv2, no flip / rotation).
// One thread per output pixel: the source point cx + (u - 128) k, cy + (v - 128) k (k = bbox / 256, the inverse of
// gen_trans_from_patch_cv), bilinear over the frame (the blurred frame's 4 taps are computed in place from the
// separable Gaussian), rounded to uint8 like warpAffine on a uint8 image.  Restated in float with contraction off,
// so the host oracle (oracle/hmr.py vitdet_crop) reproduces every byte of the unblurred path.
// Known deviations from ViTDetDataset, shared by the oracle (so its byte test cannot see them; parity unpinned):
//  * the blurred path rounds the patch to uint8 (the reference warps the float64 blurred frame and never
//    quantises it: <= 0.5 grey level per channel before the mean / std normalisation);
//  * bilinear weights are float, not cv2's 1/32-subpixel fixed-point INTER_LINEAR weights (<= 1 grey level).
// The Gaussian radius is scipy's int(4 sigma + 0.5) uncapped up to MAX_RADIUS (boxes up to ~8.6k px); a larger
// box is refused with hipErrorInvalidValue rather than blurred with a truncated kernel.
// HBM-bound: reads ~4 x 3 B of frame per output pixel (L2-resident rows), writes 196,608 B per crop.
#include "vge_common.h"

#include <cmath>
#include <vector>

namespace {

struct CropInst {
  int frame;
  float cx, cy, k;  // source centre, source pixels per output pixel
  int radius;       // Gaussian half width (0: no blur)
  float w[33];      // normalised Gaussian taps w[0..radius] (symmetric)
};

constexpr int CROP = 256;
constexpr int MAX_RADIUS = 32;

__global__ void __launch_bounds__(256) hmr_crop_kernel(const uint8_t* __restrict__ frames, int H, int W,
                                                       const CropInst* __restrict__ inst, int n,
                                                       uint8_t* __restrict__ out) {
#pragma clang fp contract(off)
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (long)n * CROP * CROP) return;
  const int u = (int)(gid % CROP), v = (int)((gid / CROP) % CROP);
  const int i = (int)(gid / ((long)CROP * CROP));
  const CropInst in = inst[i];
  const float sx = in.cx + ((float)u - 0.5f * (float)CROP) * in.k;
  const float sy = in.cy + ((float)v - 0.5f * (float)CROP) * in.k;
  const float x0f = floorf(sx), y0f = floorf(sy);
  const float fx = sx - x0f, fy = sy - y0f;
  const int x0 = (int)x0f, y0 = (int)y0f;
  const uint8_t* fr = frames + (long)in.frame * H * W * 3;
  uint8_t* o = out + gid * 3;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    auto px = [&](int yy, int xx) -> float {
      if ((unsigned)yy >= (unsigned)H || (unsigned)xx >= (unsigned)W) return 0.f;  // BORDER_CONSTANT 0
      if (in.radius == 0) return (float)fr[((long)yy * W + xx) * 3 + c];
      float s = 0.f;  // the blurred frame at (yy, xx): separable Gaussian, edges clamped ('nearest')
      for (int dy = -in.radius; dy <= in.radius; ++dy) {
        const int ry = min(max(yy + dy, 0), H - 1);
        float row = 0.f;
        for (int dx = -in.radius; dx <= in.radius; ++dx) {
          const int rx = min(max(xx + dx, 0), W - 1);
          row += in.w[dx < 0 ? -dx : dx] * (float)fr[((long)ry * W + rx) * 3 + c];
        }
        s += in.w[dy < 0 ? -dy : dy] * row;
      }
      return s;
    };
    const float top = (1.0f - fx) * px(y0, x0) + fx * px(y0, x0 + 1);
    const float bot = (1.0f - fx) * px(y0 + 1, x0) + fx * px(y0 + 1, x0 + 1);
    const float val = (1.0f - fy) * top + fy * bot;
    o[c] = (uint8_t)rintf(fminf(fmaxf(val, 0.f), 255.f));
  }
}

}  // namespace

namespace vge {

// host: ViTDetDataset's per-box geometry in float32 like its numpy code (boxes.astype(np.float32))
hipError_t launch_hmr_crop(const uint8_t* frames, int H, int W, const float* boxes, const int* frame_of, int n,
                           uint8_t* out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  std::vector<CropInst> ins((size_t)n);
  for (int i = 0; i < n; ++i) {
    const float* b = boxes + 4 * (size_t)i;
    CropInst& c = ins[(size_t)i];
    c = CropInst{};
    c.frame = frame_of ? frame_of[i] : i;
    c.cx = (b[2] + b[0]) / 2.0f;
    c.cy = (b[3] + b[1]) / 2.0f;
    const float sw = 2.5f * (b[2] - b[0]) / 200.0f, sh = 2.5f * (b[3] - b[1]) / 200.0f;
    // expand_to_aspect_ratio(scale * 200, [192, 256]).max()
    const double w = (double)(sw * 200.0f), h = (double)(sh * 200.0f);
    double wn = w, hn = h;
    if (h / w < 256.0 / 192.0) hn = std::max(w * 256.0 / 192.0, h);
    else wn = std::max(h * 192.0 / 256.0, w);
    const double bbox = std::max(wn, hn);
    c.k = (float)(bbox / CROP);
    const double df = bbox / CROP / 2.0;
    if (df > 1.1) {
      const double sigma = (df - 1.0) / 2.0;
      c.radius = (int)(4.0 * sigma + 0.5);
      if (c.radius > MAX_RADIUS) return hipErrorInvalidValue;
      double sum = 0.0, t[MAX_RADIUS + 1];
      for (int j = 0; j <= c.radius; ++j) {
        t[j] = std::exp(-0.5 * j * j / (sigma * sigma));
        sum += j == 0 ? t[j] : 2.0 * t[j];
      }
      for (int j = 0; j <= c.radius; ++j) c.w[j] = (float)(t[j] / sum);
    }
  }
  CropInst* d = nullptr;
  hipError_t e = hipMallocAsync(reinterpret_cast<void**>(&d), sizeof(CropInst) * (size_t)n, s);
  if (e != hipSuccess) return e;
  e = hipMemcpyAsync(d, ins.data(), sizeof(CropInst) * (size_t)n, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) {
    const long total = (long)n * CROP * CROP;
    hipLaunchKernelGGL(hmr_crop_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, frames, H, W, d, n,
                       out);
    e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(s);  // the host instance table is released on return
  }
  const hipError_t f = hipFreeAsync(d, s);
  return e != hipSuccess ? e : f;
}

}  // namespace vge
