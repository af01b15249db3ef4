// v_mfma_f32_16x16x4_f32 cycles per instruction on one SIMD: NACC interleaved accumulator chains per wave,
// WPS waves per SIMD (4 * WPS waves per workgroup, one workgroup per CU). s_memtime around 480 MFMAs per wave.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
typedef float f32x4 __attribute__((ext_vector_type(4)));
template <int NACC>
__global__ void chain(float* out, unsigned long long* cyc, float a0, float b0) {
  f32x4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = f32x4{0, 0, 0, 0};
  float a = a0 + threadIdx.x * 1e-7f, b = b0;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < 480 / NACC; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
  }
  float s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 16 + (threadIdx.x >> 6)] = t1 - t0;
}
template <int NACC> void run(int wps) {
  const int blocks = 256, threads = 256 * wps;
  float* o; unsigned long long* c;
  hipMalloc(&o, blocks * threads * 4); hipMalloc(&c, blocks * 16 * 8);
  for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(chain<NACC>, dim3(blocks), dim3(threads), 0, 0, o, c, 1.0f, 0.5f);
  hipDeviceSynchronize();
  std::vector<unsigned long long> h(blocks * 16);
  hipMemcpy(h.data(), c, h.size() * 8, hipMemcpyDeviceToHost);
  std::vector<unsigned long long> v;
  for (int b = 0; b < blocks; ++b) for (int w = 0; w < 4 * wps; ++w) v.push_back(h[b * 16 + w]);
  std::sort(v.begin(), v.end());
  const double med = v[v.size() / 2];
  printf("NACC %d, %d wave(s)/SIMD: %.0f cycles per wave for 480 MFMAs -> %.1f cycles per MFMA per SIMD\n", NACC, wps,
         med, med / (480.0 * wps));
  hipFree(o); hipFree(c);
}
int main() {
  for (int wps : {1, 2, 3}) { run<1>(wps); run<2>(wps); run<4>(wps); }
  return 0;
}
