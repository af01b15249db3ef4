// fp32 MFMA GEMM core for the learner's row-parallel and weight-gradient contractions (gfx950).
//
//   C[m][n] = sum_k A(m, k) * B(k, n)
//
// One 256-thread workgroup (4 waves) owns a 64x64 C tile; each wave a 32x32 quadrant driven by
// v_mfma_f32_32x32x2_f32 (exact fp32 fma chain, 64 FLOP/clk/SIMD = the fp32 peak on CDNA4). A and B K-slices
// of depth 16 are staged through LDS, double-buffered so one barrier per K-step suffices, with the next slice's
// global loads issued before the current slice's MFMAs (register prefetch).
//
// The operands are "policies": each GEMM in the learner supplies how its A and B elements are fetched (gathered
// replay rows by episode id, one-hot virtual columns, transposed activations ...), which K range blockIdx.z owns
// (net index or split-K slice) and an epilogue. Two staging patterns cover every operand:
//   kpat: the thread's 4 elements are consecutive in K   (row-major operand, K contiguous)
//   mpat: the thread's 4 elements are consecutive in K but lanes walk M (column operand, M contiguous)
// Both write the LDS tile K-major ([k][m], pitch GLD) so the MFMA operand reads are bank-conflict free.
#pragma once
#include "common.hpp"

namespace mq {

constexpr int GBM = 64, GBN = 64, GBK = 16, GLD = 64 + 4;

struct KPat {   // thread -> (row = tid>>2, k = 4*(tid&3) + i)
  MQ_DEV static int row(int tid) { return tid >> 2; }
  MQ_DEV static int kq(int tid) { return (tid & 3) * 4; }
  MQ_DEV static void store(float* S, const float (&r)[4], int tid) {
    const int ml = row(tid), k = kq(tid);
#pragma unroll
    for (int i = 0; i < 4; ++i) S[(k + i) * GLD + ml] = r[i];
  }
};

struct MPat {   // thread -> (row = tid&63, k = 4*(tid>>6) + i)
  MQ_DEV static int row(int tid) { return tid & 63; }
  MQ_DEV static int kq(int tid) { return (tid >> 6) * 4; }
  MQ_DEV static void store(float* S, const float (&r)[4], int tid) {
    const int ml = row(tid), k = kq(tid);
#pragma unroll
    for (int i = 0; i < 4; ++i) S[(k + i) * GLD + ml] = r[i];
  }
};

// Row index (within the 64x64 tile) of accumulator register `reg` for `lane` (32x32 f32 MFMA C layout).
MQ_DEV int acc_row(int reg, int lane) { return (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5); }

template <class P>
__global__ __launch_bounds__(256) void gemm_f32_kernel(const P p) {
  __shared__ float As[2][GBK * GLD];
  __shared__ float Bs[2][GBK * GLD];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wm = w >> 1, wn = w & 1;
  const int m0 = blockIdx.x * GBM, n0 = blockIdx.y * GBN, z = blockIdx.z;
  typename P::Ctx ctx = p.make_ctx(m0, n0, z, tid);
  int kb, ke;
  p.krange(z, kb, ke);
  f32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.0f;
  float ra[4], rb[4], rsum = 0.0f;
  if (kb < ke) {
    p.load_a(ctx, kb, ke, ra);
    p.load_b(ctx, kb, ke, rb);
  }
  int buf = 0;
  for (int k0 = kb; k0 < ke; k0 += GBK) {
    P::APat::store(As[buf], ra, tid);
    P::BPat::store(Bs[buf], rb, tid);
    __syncthreads();
    if (k0 + GBK < ke) {
      p.load_a(ctx, k0 + GBK, ke, ra);
      p.load_b(ctx, k0 + GBK, ke, rb);
    }
    const float* a = As[buf] + (lane >> 5) * GLD + wm * 32 + (lane & 31);
    const float* b = Bs[buf] + (lane >> 5) * GLD + wn * 32 + (lane & 31);
#pragma unroll
    for (int kk = 0; kk < GBK; kk += 2)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[kk * GLD], b[kk * GLD], acc, 0, 0, 0);
    if (P::kRowSum) {
      if (blockIdx.y == 0 && tid < GBM) {
#pragma unroll
        for (int kk = 0; kk < GBK; ++kk) rsum += As[buf][kk * GLD + tid];
      }
    }
    buf ^= 1;
  }
  p.epilogue(ctx, acc, m0, n0, z, wm, wn, lane);
  if (P::kRowSum) {
    if (blockIdx.y == 0 && tid < GBM) p.rowsum_out(m0 + tid, z, rsum);
  }
}

template <class P>
inline hipError_t launch_gemm(const P& p, int M, int N, int Z, hipStream_t s) {
  dim3 grid((M + GBM - 1) / GBM, (N + GBN - 1) / GBN, Z);
  if (grid.x == 0 || grid.y == 0 || grid.z == 0) return hipSuccess;
  hipLaunchKernelGGL(gemm_f32_kernel<P>, grid, dim3(256), 0, s, p);
  return hipGetLastError();
}

}  // namespace mq
