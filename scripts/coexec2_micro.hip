// Do LDS stores / global loads of one wave slow down while another wave on the same SIMD runs f32 MFMAs?
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/coexec2_micro.hip -o scripts/coexec2_micro && ./scripts/coexec2_micro
// Waves 0-3: the probe (one per SIMD); waves 4-7: partner f32 16x16x4 MFMA chains (PARTNER = 1) or idle.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int PROBE, int PARTNER>   // PROBE 0: ds_write_b32 x 48, 1: global loads x 48 (L2-hot) + ds_write, 2: VALU
__global__ __launch_bounds__(512) void k(float* out, const float* __restrict__ src, int iters) {
  __shared__ float lds[4][64 * 52];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (w < 4) {
    float v[48];
#pragma unroll
    for (int i = 0; i < 48; ++i) v[i] = lane * 0.5f + i;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    float acc = 0.0f;
    for (int it = 0; it < iters; ++it) {
      if (PROBE == 1) {
        const float* s = src + (size_t)((it & 7) * 48) * 64 + lane;
#pragma unroll
        for (int i = 0; i < 48; ++i) v[i] = s[i * 64];
      }
      if (PROBE == 2) {
#pragma unroll
        for (int i = 0; i < 48; ++i) v[i] = fmaf(v[i], 1.0001f, 0.5f);
      } else {
#pragma unroll
        for (int i = 0; i < 48; ++i) lds[w][i * 64 + lane] = v[i];
      }
      __builtin_amdgcn_s_waitcnt(0);
      acc += v[0] + v[47];
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = acc + lds[w][lane];
    if (lane == 0) ((uint64_t*)(out + 1024))[blockIdx.x * 8 + w] = t1 - t0;
  } else if (PARTNER) {
    f32x4 x0 = {0, 0, 0, 0}, x1 = x0;
    const float a = lane * 1e-3f, b = 1.0001f;
    for (int i = 0; i < iters * 8; ++i) {
      x0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, x0, 0, 0, 0);
      x1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, x1, 0, 0, 0);
    }
    out[threadIdx.x] = x0[0] + x1[1];
  }
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <int PROBE, int PARTNER>
double run(float* out, const float* src, int iters) {
  hipLaunchKernelGGL((k<PROBE, PARTNER>), dim3(256), dim3(512), 0, 0, out, src, iters);
  hipDeviceSynchronize();
  hipLaunchKernelGGL((k<PROBE, PARTNER>), dim3(256), dim3(512), 0, 0, out, src, iters);
  hipDeviceSynchronize();
  static uint64_t h[256 * 8];
  hipMemcpy(h, out + 1024, sizeof(h), hipMemcpyDeviceToHost);
  double s = 0;
  for (int b = 0; b < 256; ++b) for (int w = 0; w < 4; ++w) s += h[b * 8 + w];
  return s / (256 * 4) / iters;
}

int main() {
  float *out, *src;
  CK(hipMalloc(&out, (1024 + 256 * 16) * 8));
  CK(hipMalloc(&src, 8 * 48 * 64 * 4 + 4096));
  CK(hipMemset(src, 0, 8 * 48 * 64 * 4 + 4096));
  const int it = 2000;
  printf("per-iteration cycles (s_memtime units) of the probe wave, alone / beside f32 MFMA chains:\n");
  printf("  48 ds_write_b32          : %.0f / %.0f\n", run<0, 0>(out, src, it), run<0, 1>(out, src, it));
  printf("  48 loads + 48 ds_write   : %.0f / %.0f\n", run<1, 0>(out, src, it), run<1, 1>(out, src, it));
  printf("  48 v_fma                 : %.0f / %.0f\n", run<2, 0>(out, src, it), run<2, 1>(out, src, it));
  return 0;
}
