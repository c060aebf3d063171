// Staggered-halves probe (gfx950): the split conv kernel's phase structure with both MFMA shapes.  Waves 0-3
// (group A) and 4-7 (group B, one per SIMD beside A's) run the task sequence MFMA, MFMA, EPILOGUE with B one phase
// behind A and a workgroup barrier after every phase, so in two phases of three one wave per SIMD streams MFMAs while
// its partner runs epilogue-like VALU + LDS work.  MFMA tasks: the split stream loop of mfma_shape_probe.hip (A hi/lo
// from LDS, three products) on 32x32x16 (SHAPE 0) or 16x16x32 (SHAPE 1), same FLOPs.  Epilogue task: EPI rounds of
// exp2 / fma / fp16 split / LDS store + load per value.  Prints ms, TFLOP/s (MFMA work only) and the held clock.
// Build: hipcc --offload-arch=gfx950 -O3 -o stagger_probe stagger_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half2v __attribute__((ext_vector_type(2)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int ROWS = 128, XSB = 528, KSTEPS = 40;  // a conv's 80 chunks of 16 k = 40 steps of 32 k per MFMA task

template <int SHAPE>
__device__ __forceinline__ void mfma_task(const char* lds, floatx16 (&a0)[4], floatx4 (&a1)[8][2], const half8 (&bh)[2],
                                          const half8 (&bl)[2], int lane) {
  if constexpr (SHAPE == 0) {
    const int i = lane & 31, h = lane >> 5;
    for (int st = 0; st < KSTEPS; ++st) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int c = (2 * st + s) & 15;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const char* p = lds + (t * 32 + i) * XSB + c * 32 + h * 16;
          const half8 ah = *reinterpret_cast<const half8*>(p);
          const half8 al = *reinterpret_cast<const half8*>(p + ROWS * XSB);
          a0[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh[s], a0[t], 0, 0, 0);
          a0[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl[s], a0[t], 0, 0, 0);
          a0[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh[s], a0[t], 0, 0, 0);
        }
      }
    }
  } else {
    const int i = lane & 15, q = lane >> 4;
    for (int st = 0; st < KSTEPS; ++st) {
      const int c = st & 7;
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const char* p = lds + (t * 16 + i) * XSB + c * 64 + q * 16;
        const half8 ah = *reinterpret_cast<const half8*>(p);
        const half8 al = *reinterpret_cast<const half8*>(p + ROWS * XSB);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          a1[t][u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh[u], a1[t][u], 0, 0, 0);
          a1[t][u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl[u], a1[t][u], 0, 0, 0);
          a1[t][u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh[u], a1[t][u], 0, 0, 0);
        }
      }
    }
  }
}

// epilogue-like work on 64 values per lane: GELU-ish exp2 + fmas, the fp16 hi/lo split, an LDS store and a re-read
__device__ __forceinline__ float epi_task(char* scratch, float x, int lane, int rounds) {
  float acc = 0.f;
  for (int k = 0; k < rounds; ++k) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float y = x * (1.0f + 0.001f * j) + acc * 1e-7f;
      const float g = y * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-2.3f * y));
      const _Float16 hi = (_Float16)g;
      const _Float16 lo = (_Float16)(g - (float)hi);
      *reinterpret_cast<half2v*>(scratch + ((j * 64 + lane) * 4)) = half2v{hi, lo};
      acc += g;
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
    acc += (float)reinterpret_cast<const half2v*>(scratch + lane * 4)[0][0];
  }
  return acc;
}

template <int SHAPE>
__global__ void __launch_bounds__(512, 1) probe(const half8* __restrict__ src, float* __restrict__ out, int phases,
                                                int epi_rounds, long long* __restrict__ clk) {
  __shared__ __attribute__((aligned(16))) char lds[2 * ROWS * XSB + 8 * 2048];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, grp = wave >> 2;
  for (int k = tid; k < 2 * ROWS * XSB / 16; k += 512) reinterpret_cast<half8*>(lds)[k] = src[(blockIdx.x * 977 + k) % 65536];
  __syncthreads();
  char* scratch = lds + 2 * ROWS * XSB + wave * 2048;
  half8 bh[2], bl[2];
  for (int j = 0; j < 2; ++j) {
    bh[j] = src[(blockIdx.x * 131 + tid * 2 + j) % 65536];
    bl[j] = src[(blockIdx.x * 171 + tid * 2 + j + 7) % 65536] * (_Float16)0.0005f;
  }
  floatx16 a0[4] = {};
  floatx4 a1[8][2] = {};
  float e = 0.f, x = (float)bh[0][0];
  long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int p = 0; p < phases; ++p) {
    const int task = (p - grp + 3) % 3;  // 0, 1: MFMA (P1, P2), 2: epilogue; group B one phase behind
    if (p >= grp) {
      if (task < 2) mfma_task<SHAPE>(lds, a0, a1, bh, bl, lane);
      else e += epi_task(scratch, x + e * 1e-9f, lane, epi_rounds);
    }
    __syncthreads();
  }
  long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float res = e;
  for (int t = 0; t < 4; ++t)
    for (int r = 0; r < 16; ++r) res += a0[t][r];
  for (int t = 0; t < 8; ++t)
    for (int u = 0; u < 2; ++u)
      for (int r = 0; r < 4; ++r) res += a1[t][u][r];
  out[blockIdx.x * 512 + tid] = res;
  if (tid == 0) {
    clk[blockIdx.x * 2] = t1 - t0;
    clk[blockIdx.x * 2 + 1] = r1 - r0;
  }
}

int main(int argc, char** argv) {
  const int phases = argc > 1 ? atoi(argv[1]) : 3000, reps = argc > 2 ? atoi(argv[2]) : 4;
  hipDeviceProp_t pr;
  if (hipGetDeviceProperties(&pr, 0) != hipSuccess) return 1;
  const int G = pr.multiProcessorCount;
  std::vector<_Float16> h(65536 * 8);
  srand(1);
  for (auto& v : h) v = (_Float16)((rand() / (float)RAND_MAX) * 2.f - 1.f);
  half8* d_src; float* d_out; long long* d_clk;
  if (hipMalloc(&d_src, h.size() * 2) || hipMalloc(&d_out, (size_t)G * 512 * 4) || hipMalloc(&d_clk, (size_t)G * 16))
    return 1;
  if (hipMemcpy(d_src, h.data(), h.size() * 2, hipMemcpyHostToDevice)) return 1;
  std::vector<long long> clk(G * 2);
  for (int epi : {0, 24, 48, 72})
    for (int rep = 0; rep < reps; ++rep)
      for (int shape = 0; shape < 2; ++shape) {
        hipEvent_t e0, e1;
        if (hipEventCreate(&e0) || hipEventCreate(&e1) || hipEventRecord(e0)) return 1;
        if (shape == 0) hipLaunchKernelGGL(probe<0>, dim3(G), dim3(512), 0, 0, d_src, d_out, phases, epi, d_clk);
        else hipLaunchKernelGGL(probe<1>, dim3(G), dim3(512), 0, 0, d_src, d_out, phases, epi, d_clk);
        if (hipEventRecord(e1) || hipEventSynchronize(e1)) return 2;
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, e0, e1) || hipMemcpy(clk.data(), d_clk, G * 16, hipMemcpyDeviceToHost)) return 3;
        double ghz = 0, cyc = 0;
        for (int b = 0; b < G; ++b) {
          ghz += (double)clk[2 * b] / (clk[2 * b + 1] * 10.0);
          cyc += (double)clk[2 * b];
        }
        ghz /= G;
        cyc /= G;
        // MFMA tasks: 2 of every 3 phases per wave, KSTEPS x 32 k x 128 rows x 32 columns x 2 flop x 3 products
        const double flop = (double)G * 8 * (phases * 2.0 / 3.0) * KSTEPS * 32.0 * 128 * 32 * 2 * 3;
        printf("{\"shape\": \"%s\", \"epi_rounds\": %d, \"rep\": %d, \"ms\": %.3f, \"tflops\": %.1f, \"ghz\": %.3f, "
               "\"cycles_per_phase\": %.0f}\n",
               shape ? "16x16x32" : "32x32x16", epi, rep, ms, flop / ms / 1e9, ghz, cyc / phases);
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
      }
  return 0;
}
