// Featurisation and ModalityStats kernels (gfx950).
//
// Replaces WindowDataset._try_one (utils.py:383-516) and compute_stats_from_npz (utils.py:595-801).
// One 256-thread workgroup turns one 32-row tile of a video into 32 rows of the reference feats
// layout [raw 1370 | diff 1226] (keypoint_dir given), or of the keypoint-less layout [raw 1250 | diff 1106]
// (keypoint_dir None: the same columns without kp2d, the diff part 120 columns earlier, rows 2356 wide).  A tile is either a window (window mode: rows are the
// _slice_or_pad'ed frames start..start+31, first row self-diffs) or 32 consecutive frames of a
// full sequence (stats mode: diffs against the previous video frame, un-normalised output that
// the column reducer sums in float64).
//
// Numerics follow the reference op for op in float32 with FMA contraction off; the 2x2 SVD is a
// restatement of LAPACK sgesdd's 2x2 path (sgebrd Householder + sbdsqr threshold + slasv2 +
// sign fix/sort + sormbr), because utils.py:207-212 depends on LAPACK's singular-vector signs.
// Roofline: HBM-bound.  Algorithmic bytes per window tile: 32 rows x (1024+207+9+10+120) x 4 B
// read (175,360 B) + 32 x 2596 x 4 B written (332,288 B).
#include "vge_common.h"

#pragma clang fp contract(off)

#ifndef FEAT_VIT_PF
#define FEAT_VIT_PF 1  // vit rows in flight ahead of the one being finished (per wave)
#endif

namespace {

struct TileDesc {     // 8 x int32
  int video, mode, mesh_start, mesh_count, kp_start, kp_count, out_row, pad;
};

constexpr int C_VIT_RAW = 0, C_GORI_RAW = 1024, C_POSE_RAW = 1033, C_BETA_RAW = 1240, C_KP_RAW = 1250;
constexpr int C_VIT_DIFF = 1370, C_GORI_DIFF = 2394, C_POSE_DIFF = 2397, C_BETA_DIFF = 2466, C_KP_DIFF = 2476;

// ---------------------------------------------------------------- LAPACK 2x2 SVD (sgesdd path)
__device__ __forceinline__ float fsign(float a, float b) { return copysignf(fabsf(a), b); }

__device__ float slapy2(float x, float y) {
  float xa = fabsf(x), ya = fabsf(y);
  float w = fmaxf(xa, ya), z = fminf(xa, ya);
  if (z == 0.0f) return w;
  float q = z / w;
  return w * sqrtf(1.0f + q * q);
}

// slasv2(F, G, H): SVD of [[F, G], [0, H]]
__device__ void slasv2(float F, float G, float H, float& ssmin, float& ssmax, float& snr, float& csr,
                       float& snl, float& csl) {
  const float EPS = 5.9604644775390625e-08f;  // 2^-24
  float ft = F, fa = fabsf(F), ht = H, ha = fabsf(H);
  int pmax = 1;
  bool swap = ha > fa;
  if (swap) {
    pmax = 3;
    float t = ft; ft = ht; ht = t;
    t = fa; fa = ha; ha = t;
  }
  float gt = G, ga = fabsf(G);
  float clt, crt, slt, srt;
  if (ga == 0.0f) {
    ssmin = ha; ssmax = fa;
    clt = 1.0f; crt = 1.0f; slt = 0.0f; srt = 0.0f;
  } else {
    bool gasmal = true;
    if (ga > fa) {
      pmax = 2;
      if (fa / ga < EPS) {
        gasmal = false;
        ssmax = ga;
        if (ha > 1.0f) ssmin = fa / (ga / ha);
        else ssmin = (fa / ga) * ha;
        clt = 1.0f;
        slt = ht / gt;
        srt = 1.0f;
        crt = ft / gt;
      }
    }
    if (gasmal) {
      float d = fa - ha;
      float l = (d == fa) ? 1.0f : d / fa;
      float m = gt / ft;
      float t = 2.0f - l;
      float mm = m * m;
      float tt = t * t;
      float s = sqrtf(tt + mm);
      float r = (l == 0.0f) ? fabsf(m) : sqrtf(l * l + mm);
      float a = 0.5f * (s + r);
      ssmin = ha / a;
      ssmax = fa * a;
      if (mm == 0.0f) {
        if (l == 0.0f) t = fsign(2.0f, ft) * fsign(1.0f, gt);
        else t = gt / fsign(d, ft) + m / t;
      } else {
        t = (m / (s + t) + m / (r + l)) * (1.0f + a);
      }
      l = sqrtf(t * t + 4.0f);
      crt = 2.0f / l;
      srt = t / l;
      clt = (crt + srt * m) / a;
      slt = (ht / ft) * srt / a;
    }
  }
  if (swap) { csl = srt; snl = crt; csr = slt; snr = clt; }
  else { csl = clt; snl = slt; csr = crt; snr = srt; }
  float tsign;
  if (pmax == 1) tsign = fsign(1.0f, csr) * fsign(1.0f, csl) * fsign(1.0f, F);
  else if (pmax == 2) tsign = fsign(1.0f, snr) * fsign(1.0f, csl) * fsign(1.0f, G);
  else tsign = fsign(1.0f, snr) * fsign(1.0f, snl) * fsign(1.0f, H);
  ssmax = fsign(ssmax, tsign);
  ssmin = fsign(ssmin, tsign * fsign(1.0f, F) * fsign(1.0f, H));
}

// LAPACK-convention SVD of H = [[h00,h01],[h10,h11]]: returns U (col-major u[c*2+r]) and Vh (row-major)
__device__ void sgesdd_2x2(float h00, float h01, float h10, float h11, float U[2][2], float Vh[2][2]) {
  const float TOL = 5.9604644775390625e-07f;   // 10 * eps
  const float UNFL = 1.1754943508222875e-38f;  // 2^-126
  float a11 = h00, a21 = h10, a12 = h01, a22 = h11;
  // sgebrd: slarfg(2, a11, a21)
  bool refl = a21 != 0.0f;
  float tau = 0.0f, v2 = 0.0f, d1 = a11, e1 = a12, d2 = a22;
  if (refl) {
    float beta = -fsign(slapy2(a11, a21), a11);
    tau = (beta - a11) / beta;
    float scal = 1.0f / (a11 - beta);
    v2 = a21 * scal;
    d1 = beta;
    float w = a12 + a22 * v2;
    float tmp = -tau * w;
    e1 = a12 + tmp;
    d2 = a22 + v2 * tmp;
  }
  // sbdsqr relative-accuracy threshold
  float ad1 = fabsf(d1), ad2 = fabsf(d2), ae1 = fabsf(e1);
  float sminoa = 0.0f;
  if (ad1 != 0.0f) {
    float mu = ad2 * (ad1 / (ad1 + ae1));
    sminoa = fminf(ad1, mu);
  }
  sminoa = sminoa / 1.41421353816986083984375f;  // sqrt(real(2)) in float
  float thresh = fmaxf(TOL * sminoa, 24.0f * UNFL);
  float D1, D2, cr = 1.0f, sr = 0.0f, cl = 1.0f, sl = 0.0f;
  if (ae1 <= thresh) {
    D1 = d1; D2 = d2;
  } else {
    float smin, smax, snr, csr, snl, csl;
    slasv2(d1, e1, d2, smin, smax, snr, csr, snl, csl);
    D1 = smax; D2 = smin; cr = csr; sr = snr; cl = csl; sl = snl;
  }
  float VT[2][2] = {{cr, sr}, {-sr, cr}};
  float Ub[2][2] = {{cl, -sl}, {sl, cl}};  // Ub[r][c]
  if (D1 < 0.0f) { D1 = -D1; VT[0][0] = -VT[0][0]; VT[0][1] = -VT[0][1]; }
  if (D2 < 0.0f) { D2 = -D2; VT[1][0] = -VT[1][0]; VT[1][1] = -VT[1][1]; }
  if (D1 < D2) {
    float t;
    t = VT[0][0]; VT[0][0] = VT[1][0]; VT[1][0] = t;
    t = VT[0][1]; VT[0][1] = VT[1][1]; VT[1][1] = t;
    t = Ub[0][0]; Ub[0][0] = Ub[0][1]; Ub[0][1] = t;
    t = Ub[1][0]; Ub[1][0] = Ub[1][1]; Ub[1][1] = t;
  }
  // sormbr('Q','L','N'): U = H1 * Ub
  if (refl) {
    for (int j = 0; j < 2; ++j) {
      float wj = Ub[0][j] + Ub[1][j] * v2;
      float tj = -tau * wj;
      Ub[0][j] = Ub[0][j] + tj;
      Ub[1][j] = Ub[1][j] + v2 * tj;
    }
  }
  for (int r = 0; r < 2; ++r)
    for (int c = 0; c < 2; ++c) { U[r][c] = Ub[r][c]; Vh[r][c] = VT[r][c]; }
}

// ---------------------------------------------------------------- SO(3) log map (utils.py:130-140)
__device__ __forceinline__ void rot_delta(const float* __restrict__ Rp, const float* __restrict__ R, float w[3]) {
  float M[3][3];
  // Rrel = Rp^T R, k summed left to right
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
      M[i][j] = (Rp[0 * 3 + i] * R[0 * 3 + j] + Rp[1 * 3 + i] * R[1 * 3 + j]) + Rp[2 * 3 + i] * R[2 * 3 + j];
  float tr = (M[0][0] + M[1][1]) + M[2][2];
  tr = fminf(fmaxf(tr, -1.0f + 1e-6f), 3.0f - 1e-6f);
  float theta = acosf((tr - 1.0f) / 2.0f);
  float denom = fmaxf(2.0f * sinf(theta), 1e-6f);
  w[0] = theta * ((M[2][1] - M[1][2]) / denom);
  w[1] = theta * ((M[0][2] - M[2][0]) / denom);
  w[2] = theta * ((M[1][0] - M[0][1]) / denom);
}

__device__ __forceinline__ float znorm(float x, const float* __restrict__ mean, const float* __restrict__ stdv, int c) {
  if (mean == nullptr) return x;
  return (x - mean[c]) / (stdv[c] + 1e-6f);
}

struct RowSrc {
  int src, prv, first;
};

// mesh/kp frame of output row t (utils.py:366-381 in window mode; consecutive frames in stats mode)
__device__ __forceinline__ RowSrc row_src(int mode, int start, int L, int t) {
  RowSrc r;
  if (mode == 0) {
    auto f = [&](int tt) { return (start >= L) ? (L - 1) : min(start + tt, L - 1); };
    r.src = f(t);
    r.prv = (t == 0) ? r.src : f(t - 1);
    r.first = (t == 0);
  } else {
    r.src = start + t;
    r.prv = (r.src == 0) ? 0 : r.src - 1;
    r.first = (r.src == 0);
  }
  return r;
}

// ---- (a) vit raw + cosine delta (utils.py:142-147): 8 rows per wave, 16 floats per lane; the next row's
// loads are issued before the current row is finished, and each lane's z-norm divisors are inverted once
// (x - mean) * (1 / (std + 1e-6)) -- within an ulp of the division)
__device__ __forceinline__ void featurize_vit(const float* __restrict__ vit, int foff, int L, int mode, int mesh_start,
                                              int mcount, const float* __restrict__ mean,
                                              const float* __restrict__ stdv, float* __restrict__ out, int ld,
                                              int cvd, int wave, int lane) {
  float mr[16], ir[16], md[16], id[16];
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = k * 256 + lane * 4 + q;
      mr[k * 4 + q] = mean ? mean[C_VIT_RAW + c] : 0.f;
      ir[k * 4 + q] = mean ? 1.0f / (stdv[C_VIT_RAW + c] + 1e-6f) : 1.f;
      md[k * 4 + q] = mean ? mean[cvd + c] : 0.f;
      id[k * 4 + q] = mean ? 1.0f / (stdv[cvd + c] + 1e-6f) : 1.f;
    }
  auto issue = [&](int f, floatx4 (&x)[4]) {
    const floatx4* p = reinterpret_cast<const floatx4*>(vit + (size_t)(foff + f) * 1024);
#pragma unroll
    for (int k = 0; k < 4; ++k) x[k] = p[k * 64 + lane];
  };
  auto finish = [&](const floatx4 (&x)[4], float (&v)[16], float (&raw)[16]) {
    float ss = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        raw[k * 4 + q] = x[k][q];
        ss += x[k][q] * x[k][q];
      }
    // x / max(||x||, 1e-12) as x * (1 / max(...)): one division per row instead of 16 per lane (the division
    // sequences were a quarter of this part's VALU work); within an ulp of the quotient
    const float inv = 1.0f / fmaxf(sqrtf(wave_sum(ss)), 1e-12f);
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = raw[i] * inv;
  };
  const int t0 = wave * 8;
  if (t0 >= mcount) return;
  const int t1 = min(t0 + 8, mcount);
  float vprev[16], raw[16], vcur[16];
  floatx4 xa[4], xb[4];
#if FEAT_VIT_PF >= 2
  floatx4 xc[4];
#endif
  issue(row_src(mode, mesh_start, L, t0).prv, xa);
  issue(row_src(mode, mesh_start, L, t0).src, xb);
#if FEAT_VIT_PF >= 2
  if (t0 + 1 < t1) issue(row_src(mode, mesh_start, L, t0 + 1).src, xc);
#endif
  finish(xa, vprev, raw);
  for (int t = t0; t < t1; ++t) {
#pragma unroll
    for (int k = 0; k < 4; ++k) xa[k] = xb[k];
#if FEAT_VIT_PF >= 2
#pragma unroll
    for (int k = 0; k < 4; ++k) xb[k] = xc[k];
    if (t + 2 < t1) issue(row_src(mode, mesh_start, L, t + 2).src, xc);  // two rows in flight during this one
#else
    if (t + 1 < t1) issue(row_src(mode, mesh_start, L, t + 1).src, xb);  // in flight during this row
#endif
    finish(xa, vcur, raw);
    float* orow = out + (size_t)t * ld;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      floatx4 o, d4;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int i = k * 4 + q;
        o[q] = (raw[i] - mr[i]) * ir[i];
        d4[q] = ((vcur[i] - vprev[i]) - md[i]) * id[i];
      }
      const int c = k * 256 + lane * 4;
      *reinterpret_cast<floatx4*>(orow + C_VIT_RAW + c) = o;
      *reinterpret_cast<floatx2*>(orow + cvd + c) = (floatx2){d4[0], d4[1]};
      *reinterpret_cast<floatx2*>(orow + cvd + c + 2) = (floatx2){d4[2], d4[3]};
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) vprev[i] = vcur[i];
  }
}

// ---------------------------------------------------------------- the tile kernel
// The mesh / keypoint frames a tile reads, as 33 slots: slot 0 = the previous frame of row 0, slot t + 1 = the frame
// of row t (in both modes the previous frame of row t >= 1 is row t - 1's frame).  The rotation / beta and keypoint
// workgroups stage their slots in LDS with every load of the tile in flight at once (one memory round trip), then
// compute from LDS; issued row by row, a workgroup paid a round trip per row (latency-bound, ~1/3 of the kernel's
// bytes taking as long as the vit part).
constexpr int SLOTS = 33;
constexpr int ROT_W = 9 + 207 + 10;  // a slot's global_orient | body_pose | betas
__device__ __forceinline__ int slot_frame(int mode, int start, int L, int slot) {
  const RowSrc r = row_src(mode, start, L, slot == 0 ? 0 : slot - 1);
  return slot == 0 ? r.prv : r.src;
}

__global__ void __launch_bounds__(256) featurize_tiles_kernel(
    const float* __restrict__ pose, const float* __restrict__ gori, const float* __restrict__ betas,
    const float* __restrict__ vit, const float* __restrict__ kp, const int* __restrict__ videos,
    const TileDesc* __restrict__ tiles, const int* __restrict__ windows, const float* __restrict__ mean,
    const float* __restrict__ stdv, float* __restrict__ feats, int ld, int dsh) {
  // ld: feats row width (2596, or 2356 keypoint-less); dsh: how far the diff columns sit before the 2596 layout's
  // LDS for the keypoint workgroups only (16.4 KB: a featurise workgroup then fits beside a transformer workgroup's
  // 139 KB on a CU, so the side-stream featurise does not hold back the transformer's workgroups)
  __shared__ float pn[SLOTS][120];        // normalised keypoints of every slot
  __shared__ float kR[32][4];             // per row: H = X_{t-1}^T X_t, then the Procrustes rotation R (row-major)
  TileDesc td;
  if (windows != nullptr) {  // window mode straight from the {video, start} list
    const int v = windows[2 * blockIdx.x], st = windows[2 * blockIdx.x + 1];
    td = TileDesc{v, 0, st, 32, st, 32, (int)blockIdx.x * 32, 0};
  } else {
    td = tiles[blockIdx.x];
  }
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int* vd = videos + 4 * td.video;
  const int foff = vd[0], L = vd[1], koff = vd[2], Lk = vd[3];
  const int mode = td.mode;
  const int mcount = (mode == 0) ? 32 : td.mesh_count;
  const int kcount = (mode == 0) ? (Lk > 0 ? 32 : 0) : td.kp_count;
  float* out = feats + (size_t)td.out_row * ld;

  // three workgroups per tile: vit columns (3/4 of the bytes), rotations + betas, keypoints
  if (blockIdx.y == 0) {
#if !(defined(VGE_ABL) && (VGE_ABL & 2048))
    featurize_vit(vit, foff, L, mode, td.mesh_start, mcount, mean, stdv, out, ld, C_VIT_DIFF - dsh, wave, lane);
#endif
    return;
  }
#if defined(VGE_ABL) && (VGE_ABL & 1024)
  return;  // timing ablation: vit part only
#endif
  if (blockIdx.y == 1) {  // rotations + betas, straight from global memory: every load of a thread issued at once
    // ---- (b) rotations: raw flattened rotmats + SO(3) log-map deltas (utils.py:165-174); 32 rows x 24 joints = 3
    // items per thread, each R_t and R_{t-1} (the previous row's frame, or the window's previous frame for row 0)
    constexpr int RI = 32 * 24 / 256;
    float Rl[RI][9], Rpl[RI][9];
#pragma unroll
    for (int k = 0; k < RI; ++k) {
      const int it = tid + 256 * k, t = it / 24, j = it % 24;
      const bool ok = t < mcount;
      const size_t f = (size_t)(foff + slot_frame(mode, td.mesh_start, L, ok ? t + 1 : 0));
      const size_t fp = (size_t)(foff + slot_frame(mode, td.mesh_start, L, ok ? t : 0));
      const float* src = j == 0 ? gori + f * 9 : pose + f * 207 + (j - 1) * 9;
      const float* srcp = j == 0 ? gori + fp * 9 : pose + fp * 207 + (j - 1) * 9;
#pragma unroll
      for (int i = 0; i < 9; ++i) {
        Rl[k][i] = ok ? src[i] : 0.f;
        Rpl[k][i] = ok ? srcp[i] : 0.f;
      }
    }
#pragma unroll
    for (int k = 0; k < RI; ++k) {
      const int it = tid + 256 * k, t = it / 24, j = it % 24;
      if (t >= mcount) continue;
      float w[3];
      rot_delta(Rpl[k], Rl[k], w);
      float* orow = out + (size_t)t * ld;
      int craw = (j == 0) ? C_GORI_RAW : C_POSE_RAW + (j - 1) * 9;
      int cdif = ((j == 0) ? C_GORI_DIFF : C_POSE_DIFF + (j - 1) * 3) - dsh;
#pragma unroll
      for (int i = 0; i < 9; ++i) orow[craw + i] = znorm(Rl[k][i], mean, stdv, craw + i);
#pragma unroll
      for (int i = 0; i < 3; ++i) orow[cdif + i] = znorm(w[i], mean, stdv, cdif + i);
    }

    // ---- (c) betas raw + first difference (utils.py:161-163)
    for (int it = tid; it < 32 * 10; it += 256) {
      const int t = it / 10, i = it % 10;
      if (t >= mcount) continue;
      const float b = betas[(size_t)(foff + slot_frame(mode, td.mesh_start, L, t + 1)) * 10 + i];
      const float bp = betas[(size_t)(foff + slot_frame(mode, td.mesh_start, L, t)) * 10 + i];
      float* orow = out + (size_t)t * ld;
      orow[C_BETA_RAW + i] = znorm(b, mean, stdv, C_BETA_RAW + i);
      orow[C_BETA_DIFF - dsh + i] = znorm(b - bp, mean, stdv, C_BETA_DIFF - dsh + i);
    }
    return;
  }
  // (the keypoint-less layout launches no keypoint workgroups)
  if (kcount == 0) return;
  // ---- (d1) keypoints: centre + Frobenius-normalise every slot (utils.py:191-196), loaded straight into registers
  // (a wave's slots wave, wave + 4, ...; lane l holds point l), and the raw columns of the slot's row written from them.  A wave's slots (wave, wave + 4,
  // ...) are unrolled so their wave sums -- each a chain of six dependent lane shuffles -- run interleaved instead of
  // one after another (the keypoint workgroup was the kernel's long pole)
  {
    constexpr int KS = (SLOTS + 3) / 4;
    float x[KS], y[KS], cx[KS], cy[KS], mx[KS], my[KS], ss[KS];
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      const int slot = wave + 4 * k;
      const bool ok = slot <= kcount && lane < 60;
      const float* src = kp + (size_t)(koff + slot_frame(mode, td.kp_start, Lk, ok ? slot : 0)) * 120 + 2 * lane;
      x[k] = ok ? src[0] : 0.f;
      y[k] = ok ? src[1] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < KS; ++k) {  // slot s >= 1 is row s - 1's own frame: its raw keypoint columns
      const int slot = wave + 4 * k;
      if (slot >= 1 && slot <= kcount && lane < 60) {
        float* orow = out + (size_t)(slot - 1) * ld;
        orow[C_KP_RAW + 2 * lane] = znorm(x[k], mean, stdv, C_KP_RAW + 2 * lane);
        orow[C_KP_RAW + 2 * lane + 1] = znorm(y[k], mean, stdv, C_KP_RAW + 2 * lane + 1);
      }
    }
    // (wave_sum: the butterfly order the parity tests pinned; the Procrustes SVD is sensitive near rank 1)
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      mx[k] = wave_sum(x[k]) / 60.0f;
      my[k] = wave_sum(y[k]) / 60.0f;
    }
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      cx[k] = x[k] - mx[k];
      cy[k] = y[k] - my[k];
      ss[k] = wave_sum(lane < 60 ? (cx[k] * cx[k] + cy[k] * cy[k]) : 0.f);
    }
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      const int slot = wave + 4 * k;
      const float sc = fmaxf(sqrtf(ss[k]), 1e-6f);
      if (slot <= kcount && lane < 60) {
        pn[slot][2 * lane] = cx[k] / sc;
        pn[slot][2 * lane + 1] = cy[k] / sc;
      }
    }
  }
  __syncthreads();  // pn[] complete

  // ---- (d2) keypoints raw + Procrustes velocity (utils.py:177-217): H of every row by wave sums (a wave's 8 rows
  // unrolled, 32 independent sums), then the 2x2 SVDs of all rows in parallel on the lanes of wave 0 (one dependent
  // LAPACK chain instead of eight per wave), then the deltas
  {
    float h[8][4];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int t = wave + 4 * k;
      const bool use = t < kcount && !row_src(mode, td.kp_start, Lk, t).first;  // (wave-uniform)
      float x0 = 0.f, x1 = 0.f, y0 = 0.f, y1 = 0.f;
      if (use && lane < 60) {
        x0 = pn[t][2 * lane]; x1 = pn[t][2 * lane + 1];
        y0 = pn[t + 1][2 * lane]; y1 = pn[t + 1][2 * lane + 1];
      }
      h[k][0] = x0 * y0; h[k][1] = x0 * y1; h[k][2] = x1 * y0; h[k][3] = x1 * y1;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k)
#pragma unroll
      for (int q = 0; q < 4; ++q) h[k][q] = wave_sum(h[k][q]);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int t = wave + 4 * k;
      if (t < kcount) {
        if (lane == 0 && !row_src(mode, td.kp_start, Lk, t).first) {
          kR[t][0] = h[k][0]; kR[t][1] = h[k][1]; kR[t][2] = h[k][2]; kR[t][3] = h[k][3];
        }
      }
    }
  }
  __syncthreads();
  if (wave == 0 && lane < kcount && !row_src(mode, td.kp_start, Lk, lane).first) {
    const int t = lane;
    float U[2][2], Vh[2][2];
    sgesdd_2x2(kR[t][0], kR[t][1], kR[t][2], kR[t][3], U, Vh);
    // R = Vh @ U^T; det < 0: flip Vh's last column and recompute
    float R[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) R[i][j] = Vh[i][0] * U[j][0] + Vh[i][1] * U[j][1];
    const float det = R[0][0] * R[1][1] - R[0][1] * R[1][0];
    if (det < 0.0f) {
      Vh[0][1] = -Vh[0][1];
      Vh[1][1] = -Vh[1][1];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) R[i][j] = Vh[i][0] * U[j][0] + Vh[i][1] * U[j][1];
    }
    kR[t][0] = R[0][0]; kR[t][1] = R[0][1]; kR[t][2] = R[1][0]; kR[t][3] = R[1][1];
  }
  __syncthreads();
  for (int t = wave; t < kcount; t += 4) {
    const RowSrc rs = row_src(mode, td.kp_start, Lk, t);
    float* orow = out + (size_t)t * ld;
    float dx = 0.f, dy = 0.f;
    if (!rs.first && lane < 60) {
      const float x0 = pn[t][2 * lane], x1 = pn[t][2 * lane + 1];
      const float y0 = pn[t + 1][2 * lane], y1 = pn[t + 1][2 * lane + 1];
      dx = y0 - (x0 * kR[t][0] + x1 * kR[t][2]);
      dy = y1 - (x0 * kR[t][1] + x1 * kR[t][3]);
    }
    if (lane < 60) {
      orow[C_KP_DIFF + 2 * lane] = znorm(dx, mean, stdv, C_KP_DIFF + 2 * lane);
      orow[C_KP_DIFF + 2 * lane + 1] = znorm(dy, mean, stdv, C_KP_DIFF + 2 * lane + 1);
    }
  }
}

// ---------------------------------------------------------------- stats column reducer
// partial[chunk][2][2596] = (sum, sumsq) over the valid rows of tiles [chunk*G, chunk*G+G)
__global__ void __launch_bounds__(256) stats_colsum_kernel(const float* __restrict__ feats,
                                                           const TileDesc* __restrict__ tiles, int n_tiles,
                                                           int tiles_per_chunk, double* __restrict__ partial) {
  const int col = blockIdx.x * 256 + threadIdx.x;
  const int chunk = blockIdx.y;
  if (col >= VGE_FD) return;
  const bool is_kp = (col >= C_KP_RAW && col < C_VIT_DIFF) || col >= C_KP_DIFF;
  double s = 0.0, s2 = 0.0;
  const int t_end = min(n_tiles, (chunk + 1) * tiles_per_chunk);
  for (int ti = chunk * tiles_per_chunk; ti < t_end; ++ti) {
    const TileDesc td = tiles[ti];
    const int nrow = is_kp ? td.kp_count : td.mesh_count;
    const float* p = feats + (size_t)td.out_row * VGE_FD + col;
    // rows in order, their loads 8 at a time (one memory round trip per 8 rows, not per row)
    for (int r0 = 0; r0 < nrow; r0 += 8) {
      float xv[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) xv[k] = r0 + k < nrow ? p[(size_t)(r0 + k) * VGE_FD] : 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (r0 + k < nrow) {
          const double x = (double)xv[k];
          s += x;
          s2 += x * x;
        }
    }
  }
  partial[((size_t)chunk * 2 + 0) * VGE_FD + col] = s;
  partial[((size_t)chunk * 2 + 1) * VGE_FD + col] = s2;
}

__global__ void stats_reduce_kernel(const double* __restrict__ partial, int n_chunks, double* __restrict__ sums) {
  const int col = blockIdx.x * 256 + threadIdx.x;
  if (col >= VGE_FD) return;
  double s = 0.0, s2 = 0.0;
  for (int c = 0; c < n_chunks; ++c) {
    s += partial[((size_t)c * 2 + 0) * VGE_FD + col];
    s2 += partial[((size_t)c * 2 + 1) * VGE_FD + col];
  }
  sums[col] += s;
  sums[VGE_FD + col] += s2;
}

// mean / std in the feats column order of a layout of width ld: 2596, or 2356 keypoint-less (the kp2d columns
// dropped, the diff part 120 columns earlier; the sums are always in the 2596 order)
__global__ void stats_finalize_kernel(const double* __restrict__ sums, long long n_mesh, long long n_kp,
                                      float* __restrict__ mean, float* __restrict__ stdv, int ld) {
  const int oc = blockIdx.x * 256 + threadIdx.x;
  if (oc >= ld) return;
  const int col = (ld == VGE_FD || oc < C_KP_RAW) ? oc : oc + (C_VIT_DIFF - C_KP_RAW);
  const bool is_kp = (col >= C_KP_RAW && col < C_VIT_DIFF) || col >= C_KP_DIFF;
  double n = (double)max(1LL, is_kp ? n_kp : n_mesh);
  double m = sums[col] / n;
  double var = sums[VGE_FD + col] / n - m * m;
  double sd = sqrt(fmax(var, 0.0) + 1e-6);
  mean[oc] = (float)m;
  stdv[oc] = (float)sd;
}

}  // namespace

// ================================================================ host launchers (C ABI in vge_api.cpp)
namespace vge {

hipError_t launch_featurize_tiles(const float* pose, const float* gori, const float* betas, const float* vit,
                                  const float* kp, const int* videos, const void* tiles, const int* windows,
                                  int n_tiles, const float* mean, const float* stdv, float* feats, int with_kp,
                                  hipStream_t s) {
  if (n_tiles <= 0) return hipSuccess;
  hipLaunchKernelGGL(featurize_tiles_kernel, dim3(n_tiles, with_kp ? 3 : 2), dim3(256), 0, s, pose, gori, betas, vit,
                     kp, videos, reinterpret_cast<const TileDesc*>(tiles), windows, mean, stdv, feats,
                     with_kp ? VGE_FD : VGE_FD_NOKP, with_kp ? 0 : C_VIT_DIFF - C_KP_RAW);
  return hipGetLastError();
}

hipError_t launch_stats_colsum(const float* feats, const void* tiles, int n_tiles, int tiles_per_chunk,
                               int n_chunks, double* partial, double* sums, hipStream_t s) {
  if (n_tiles <= 0) return hipSuccess;
  hipLaunchKernelGGL(stats_colsum_kernel, dim3((VGE_FD + 255) / 256, n_chunks), dim3(256), 0, s, feats,
                     reinterpret_cast<const TileDesc*>(tiles), n_tiles, tiles_per_chunk, partial);
  hipLaunchKernelGGL(stats_reduce_kernel, dim3((VGE_FD + 255) / 256), dim3(256), 0, s, partial, n_chunks, sums);
  return hipGetLastError();
}

hipError_t launch_stats_finalize(const double* sums, long long n_mesh, long long n_kp, float* mean, float* stdv,
                                 int with_kp, hipStream_t s) {
  const int ld = with_kp ? VGE_FD : VGE_FD_NOKP;
  hipLaunchKernelGGL(stats_finalize_kernel, dim3((ld + 255) / 256), dim3(256), 0, s, sums, n_mesh, n_kp, mean, stdv,
                     ld);
  return hipGetLastError();
}

}  // namespace vge
