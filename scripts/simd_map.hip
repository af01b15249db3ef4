// Which SIMD does each wave of a workgroup land on? (HW_ID register: SIMD_ID bits 5:4, CU_ID 11:8, SE_ID 15:13)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <map>
__global__ void probe(unsigned* out) {
  const unsigned hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | ((32 - 1) << 11));
  // burn a little time so the workgroups overlap like real ones
  float x = threadIdx.x;
  for (int i = 0; i < 2000; ++i) x = x * 0.999f + 1.0f;
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * 16 + (threadIdx.x >> 6)] = hw | (x < 0 ? 1u : 0u);
}
int main() {
  for (int threads : {256, 512, 768, 1024}) {
    const int blocks = 512, nw = threads / 64;
    unsigned* d; hipMalloc(&d, blocks * 16 * 4); hipMemset(d, 0, blocks * 16 * 4);
    hipLaunchKernelGGL(probe, dim3(blocks), dim3(threads), 0, 0, d);
    hipDeviceSynchronize();
    std::vector<unsigned> h(blocks * 16);
    hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
    std::map<std::string, int> pat;
    for (int b = 0; b < blocks; ++b) {
      std::string s;
      for (int w = 0; w < nw; ++w) s += char('0' + ((h[b * 16 + w] >> 4) & 3));
      pat[s]++;
    }
    printf("%d threads: wave->SIMD patterns (wave 0 first), count over %d workgroups\n", threads, blocks);
    for (auto& kv : pat) printf("  %s  %d\n", kv.first.c_str(), kv.second);
    hipFree(d);
  }
  return 0;
}
