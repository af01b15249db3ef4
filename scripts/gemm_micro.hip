// GEMM core microbenchmark: dense C[z][M][N] = A[z][M][K] B[z][N][K]^T through gemm_f32_kernel, at the learner's
// small-GEMM shapes (hypernet: M = T*B, N = NH, K = S).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/gemm_micro.hip -o scripts/gemm_micro && ./scripts/gemm_micro
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#define MQ_GEMM_STAMPS
#include "../pymarl_amd/csrc/gemm_f32.hpp"
using namespace mq;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

template <int BN_, int MT_ = 1, bool VEC = false>
struct DenseProb {
  static constexpr int BN = BN_;
  static constexpr int MT = MT_;
  const float* A; const float* B; float* C;
  int M, N, K;
  using APat = KPat;
  using BPat = KPat;
  static constexpr bool kRowSum = false;
  struct Ctx { const float* arow; const float* brow[BN / 64]; };
  MQ_DEV Ctx make_ctx(int m0, int n0, int z, int tid) const {
    Ctx c;
    const int m = m0 + KPat::row(tid);
    c.arow = m < M ? A + ((int64_t)z * M + m) * K : nullptr;
#pragma unroll
    for (int p = 0; p < BN / 64; ++p) {
      const int nn = n0 + 64 * p + KPat::row(tid);
      c.brow[p] = nn < N ? B + ((int64_t)z * N + nn) * K : nullptr;
    }
    return c;
  }
  MQ_DEV void krange(int, int& kb, int& ke) const { kb = 0; ke = K; }
  MQ_DEV void load_a(const Ctx& c, int k0, int ke, float (&r)[4]) const {
    const int k = k0 + KPat::kq(threadIdx.x);
    if (VEC && c.arow && k + 3 < ke) {   // K % 4 == 0: 16-byte aligned rows
      const f32x4 v = *(const f32x4*)(c.arow + k);
      r[0] = v[0]; r[1] = v[1]; r[2] = v[2]; r[3] = v[3];
      return;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = (c.arow && k + i < ke) ? c.arow[k + i] : 0.0f;
  }
  MQ_DEV void load_b(const Ctx& c, int pass, int k0, int ke, float (&r)[4]) const {
    const int k = k0 + KPat::kq(threadIdx.x);
    if (VEC && c.brow[pass] && k + 3 < ke) {
      const f32x4 v = *(const f32x4*)(c.brow[pass] + k);
      r[0] = v[0]; r[1] = v[1]; r[2] = v[2]; r[3] = v[3];
      return;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = (c.brow[pass] && k + i < ke) ? c.brow[pass][k + i] : 0.0f;
  }
  MQ_DEV void epilogue(const Ctx&, const f32x16& acc, int mrow0, int ncol0, int z, int lane) const {
    const int j = ncol0 + (lane & 31);
    if (j >= N) return;
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int m = mrow0 + acc_row(reg, lane);
      if (m < M) C[((int64_t)z * M + m) * N + j] = acc[reg];
    }
  }
  MQ_DEV void rowsum_out(int, int, float) const {}
};

template <class F> float time_it(F f, int reps = 50) {
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  f(); CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) f();
  CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps * 1000.0f;
}

int main(int argc, char** argv) {
  uint64_t* stamp_buf;
  CK(hipMalloc(&stamp_buf, 8 << 20));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(mq_gemm_stamps), &stamp_buf, sizeof(stamp_buf)));
  struct Shape { const char* name; int M, N, K, Z; } shapes[] = {
      {"hyper 3840x352x168 z2", 3840, 352, 168, 2},
      {"fc1 30976x64x102 z2", 30976, 64, 102, 2},
      {"gi 30976x192x64 z2", 30976, 192, 64, 2},
      {"cfg3 fc1 625536x128x348", 625536, 128, 348, 1},
      {"cfg3 gi 625536x192x64 z2", 625536, 192, 64, 2},
      {"cfg3 dx1 625536x64x192", 625536, 64, 192, 1},
      {"big 4096x4096x4096", 4096, 4096, 4096, 1},
  };
  for (auto& s : shapes) {
    const size_t na = (size_t)s.Z * s.M * s.K, nb = (size_t)s.Z * s.N * s.K, nc = (size_t)s.Z * s.M * s.N;
    std::vector<float> h(std::max(na, nb));
    for (auto& x : h) x = (rand() / (float)RAND_MAX) - 0.5f;
    float *A, *B, *C;
    CK(hipMalloc(&A, na * 4)); CK(hipMalloc(&B, nb * 4)); CK(hipMalloc(&C, nc * 4));
    CK(hipMemcpy(A, h.data(), na * 4, hipMemcpyHostToDevice)); CK(hipMemcpy(B, h.data(), nb * 4, hipMemcpyHostToDevice));
    const double flop = 2.0 * s.M * s.N * (double)s.K * s.Z;
    DenseProb<64> p64{A, B, C, s.M, s.N, s.K};
    DenseProb<128> p128{A, B, C, s.M, s.N, s.K};
    DenseProb<192> p192{A, B, C, s.M, s.N, s.K};
    const int reps = s.K > 1000 ? 5 : 50;
    float t64 = time_it([&] { CK(launch_gemm(p64, s.M, s.N, s.Z, 0)); }, reps);
    float t128 = time_it([&] { CK(launch_gemm(p128, s.M, s.N, s.Z, 0)); }, reps);
    float t192 = time_it([&] { CK(launch_gemm(p192, s.M, s.N, s.Z, 0)); }, reps);
    printf("%-26s BN64 %8.1f us (%5.1f TF)  BN128 %8.1f us (%5.1f TF)  BN192 %8.1f us (%5.1f TF)\n", s.name, t64,
           flop / t64 * 1e-6, t128, flop / t128 * 1e-6, t192, flop / t192 * 1e-6);
    {
      DenseProb<64, 2> q64{A, B, C, s.M, s.N, s.K};
      DenseProb<128, 2> q128{A, B, C, s.M, s.N, s.K};
      DenseProb<192, 2> q192{A, B, C, s.M, s.N, s.K};
      float u64 = time_it([&] { CK(launch_gemm(q64, s.M, s.N, s.Z, 0)); }, reps);
      float u128 = time_it([&] { CK(launch_gemm(q128, s.M, s.N, s.Z, 0)); }, reps);
      float u192 = time_it([&] { CK(launch_gemm(q192, s.M, s.N, s.Z, 0)); }, reps);
      printf("%-26s MT2: BN64 %8.1f us (%5.1f TF)  BN128 %8.1f us (%5.1f TF)  BN192 %8.1f us (%5.1f TF)\n", "", u64,
             flop / u64 * 1e-6, u128, flop / u128 * 1e-6, u192, flop / u192 * 1e-6);
      // MT2 vs MT1 results (same k order per element: bitwise)
      std::vector<float> c1(nc), c2(nc);
      CK(launch_gemm(p128, s.M, s.N, s.Z, 0)); CK(hipDeviceSynchronize());
      CK(hipMemcpy(c1.data(), C, nc * 4, hipMemcpyDeviceToHost));
      CK(hipMemset(C, 0, nc * 4));
      CK(launch_gemm(q128, s.M, s.N, s.Z, 0)); CK(hipDeviceSynchronize());
      CK(hipMemcpy(c2.data(), C, nc * 4, hipMemcpyDeviceToHost));
      size_t nd = 0;
      for (size_t i = 0; i < nc; ++i) nd += c1[i] != c2[i];
      printf("   MT2 vs MT1 (BN128): %zu of %zu elements differ\n", nd, nc);
      if (s.K % 4 == 0) {
        DenseProb<128, 2, true> v128{A, B, C, s.M, s.N, s.K};
        DenseProb<64, 2, true> v64{A, B, C, s.M, s.N, s.K};
        DenseProb<128, 1, true> w128{A, B, C, s.M, s.N, s.K};
        const float x128 = time_it([&] { CK(launch_gemm(v128, s.M, s.N, s.Z, 0)); }, reps);
        const float x64 = time_it([&] { CK(launch_gemm(v64, s.M, s.N, s.Z, 0)); }, reps);
        const float y128 = time_it([&] { CK(launch_gemm(w128, s.M, s.N, s.Z, 0)); }, reps);
        printf("   b128 loads: MT2 BN128 %.1f us (%.1f TF) | MT2 BN64 %.1f us (%.1f TF) | MT1 BN128 %.1f us (%.1f TF)\n",
               x128, flop / x128 * 1e-6, x64, flop / x64 * 1e-6, y128, flop / y128 * 1e-6);
      }
    }
    {  // stamps of the BN64 run: per block (wave 0) cycles in stage stores (incl. load waits), barriers, MFMA
      const int nblk = ((s.M + 63) / 64) * ((s.N + 63) / 64) * s.Z;
      CK(launch_gemm(p64, s.M, s.N, s.Z, 0)); CK(hipDeviceSynchronize());
      std::vector<uint64_t> st(8 * nblk);
      CK(hipMemcpy(st.data(), stamp_buf, st.size() * 8, hipMemcpyDeviceToHost));
      double a[5] = {0, 0, 0, 0, 0};
      uint64_t t0 = ~0ull, t1 = 0;
      for (int b = 0; b < nblk; ++b) {
        for (int i = 0; i < 5; ++i) a[i] += st[8 * b + i];
        t0 = std::min(t0, st[8 * b + 5]); t1 = std::max(t1, st[8 * b + 5] + st[8 * b + 4]);
      }
      printf("   BN64 per block: store+wait %.0f, barrier %.0f, mfma %.0f, epilogue %.0f, total %.0f cycles; "
             "kernel span %.0f cycles, %d blocks\n", a[0] / nblk, a[1] / nblk, a[2] / nblk, a[3] / nblk, a[4] / nblk,
             (double)(t1 - t0), nblk);
    }
    CK(hipFree(A)); CK(hipFree(B)); CK(hipFree(C));
  }
  return 0;
}
