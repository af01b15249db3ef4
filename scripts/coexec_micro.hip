// Does v_mfma_f32_16x16x4_f32 in one wave slow a VALU-bound wave on the same SIMD? (and bf16 MFMA for contrast)
//   hipcc --offload-arch=gfx950 -O3 scripts/coexec_micro.hip -o scripts/coexec_micro && ./scripts/coexec_micro
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));

template <int MODE>   // 0: VALU alone, 1: + f32 16x16x4 MFMA, 2: + bf16 MFMA, 3: f32 MFMA alone, 4: + f32 32x32x2
__global__ __launch_bounds__(512) void k(float* out, int iters) {
  const int w = threadIdx.x >> 6;
  float a = threadIdx.x * 1e-3f, b = 1.0001f, c0 = 0, c1 = 0, c2 = 0, c3 = 0, c4 = 0, c5 = 0, c6 = 0, c7 = 0;
  if (w < 4) {
    if (MODE == 3) return;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        c0 = fmaf(a, b, c0); c1 = fmaf(a, b, c1); c2 = fmaf(a, b, c2); c3 = fmaf(a, b, c3);
        c4 = fmaf(a, b, c4); c5 = fmaf(a, b, c5); c6 = fmaf(a, b, c6); c7 = fmaf(a, b, c7);
      }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7;
    if ((threadIdx.x & 63) == 0) ((uint64_t*)(out + 1024))[blockIdx.x * 8 + w] = t1 - t0;
  } else {
    if (MODE == 0) return;
    f32x4 x0 = {0, 0, 0, 0}, x1 = x0, x2 = x0, x3 = x0;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    typedef float f32x16 __attribute__((ext_vector_type(16)));
    if (MODE == 4) {
      f32x16 y0 = {}, y1 = {};
      for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          y0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, y0, 0, 0, 0);
          y1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, y1, 0, 0, 0);
        }
      }
      x0[0] = y0[0] + y1[1];
    } else if (MODE == 1 || MODE == 3) {
      for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          x0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, x0, 0, 0, 0);
          x1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, x1, 0, 0, 0);
          x2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, x2, 0, 0, 0);
          x3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, x3, 0, 0, 0);
        }
      }
    } else {
      bf16x8 av = {1, 2, 3, 4, 5, 6, 7, 8};
      for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          x0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, av, x0, 0, 0, 0);
          x1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, av, x1, 0, 0, 0);
          x2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, av, x2, 0, 0, 0);
          x3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, av, x3, 0, 0, 0);
        }
      }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = x0[0] + x1[1] + x2[2] + x3[3];
    if ((threadIdx.x & 63) == 0) ((uint64_t*)(out + 1024))[blockIdx.x * 8 + w] = t1 - t0;
  }
}

int main() {
  float* out; hipMalloc(&out, 1 << 20);
  const int iters = 200;
  const char* names[5] = {"VALU alone", "VALU + f32 MFMA", "VALU + bf16 MFMA", "f32 MFMA alone", "VALU + f32 32x32x2"};
  for (int mode = 0; mode < 5; ++mode) {
    for (int rep = 0; rep < 2; ++rep) {
      hipMemset(out, 0, 1 << 20);
      if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(256), dim3(512), 0, 0, out, iters);
      if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(256), dim3(512), 0, 0, out, iters);
      if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(256), dim3(512), 0, 0, out, iters);
      if (mode == 3) hipLaunchKernelGGL(k<3>, dim3(256), dim3(512), 0, 0, out, iters);
      if (mode == 4) hipLaunchKernelGGL(k<4>, dim3(256), dim3(512), 0, 0, out, iters);
      hipDeviceSynchronize();
    }
    uint64_t st[256 * 8];
    hipMemcpy(st, out + 1024, sizeof(st), hipMemcpyDeviceToHost);
    double v = 0, m = 0;
    for (int b = 0; b < 256; ++b) for (int w = 0; w < 8; ++w) (w < 4 ? v : m) += st[b * 8 + w];
    printf("%-18s VALU wave: %.1f cyc per 128 FMA-instr; MFMA wave: %.1f cyc per 16 MFMA\n", names[mode],
           v / 1024 / iters, m / 1024 / iters);
  }
  return 0;
}
