// fp32 MFMA GEMM core for the learner's row-parallel and weight-gradient contractions (gfx950).
//
//   C[m][n] = sum_k A(m, k) * B(k, n)
//
// One 256-thread workgroup (4 waves, 2 x 2) owns a 64 x BN tile of C (BN = 64, 128 or 192); each wave a 32 x BN/2
// strip as BN/64 accumulators of v_mfma_f32_32x32x2_f32 (exact fp32 fma chain, 64 FLOP/clk/SIMD = the fp32 peak
// on CDNA4). K-slices of depth 16 are staged through LDS, double-buffered so one barrier per K-step suffices, with
// the next slice's global loads issued before the current slice's MFMAs (register prefetch).
//
// The operands are "policies": each GEMM in the learner supplies how its A and B elements are fetched (gathered
// replay rows by episode id, one-hot virtual columns, transposed activations ...), which K range blockIdx.z owns
// (net index or split-K slice) and an epilogue. Two staging patterns cover every operand:
//   KPat: the thread's 4 elements are consecutive in K   (row-major operand, K contiguous)
//   MPat: the thread's 4 elements are consecutive in K but lanes walk the rows (column operand, rows contiguous)
// B tiles wider than 64 rows are staged in BN/64 passes of the same pattern. Both write the LDS tile K-major
// ([k][row], padded pitch) so the MFMA operand reads are bank-conflict free.
#pragma once
#include "common.hpp"

namespace mq {

constexpr int GBM = 64, GBK = 16, GLDA = 64 + 4;

struct KPat {   // thread -> (row = 64*pass + (tid>>2), k = 4*(tid&3) + i)
  MQ_DEV static int row(int tid) { return tid >> 2; }
  MQ_DEV static int kq(int tid) { return (tid & 3) * 4; }
  template <int LD>
  MQ_DEV static void store(float* S, const float (&r)[4], int tid, int pass) {
    const int ml = 64 * pass + row(tid), k = kq(tid);
#pragma unroll
    for (int i = 0; i < 4; ++i) S[(k + i) * LD + ml] = r[i];
  }
};

struct MPat {   // thread -> (row = 64*pass + (tid&63), k = 4*(tid>>6) + i)
  MQ_DEV static int row(int tid) { return tid & 63; }
  MQ_DEV static int kq(int tid) { return (tid >> 6) * 4; }
  template <int LD>
  MQ_DEV static void store(float* S, const float (&r)[4], int tid, int pass) {
    const int ml = 64 * pass + row(tid), k = kq(tid);
#pragma unroll
    for (int i = 0; i < 4; ++i) S[(k + i) * LD + ml] = r[i];
  }
};

// Row index (within a 32x32 accumulator tile) of register `reg` for `lane` (32x32 f32 MFMA C layout).
MQ_DEV int acc_row(int reg, int lane) { return (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5); }

template <class P>
__global__ __launch_bounds__(256) void gemm_f32_kernel(const P p) {
  constexpr int BN = P::BN, NT = BN / 64, LDB = BN + 4;
  __shared__ float As[2][GBK * GLDA];
  __shared__ float Bs[2][GBK * LDB];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wm = w >> 1, wn = w & 1;
  const int m0 = blockIdx.x * GBM, n0 = blockIdx.y * BN, z = blockIdx.z;
  typename P::Ctx ctx = p.make_ctx(m0, n0, z, tid);
  int kb, ke;
  p.krange(z, kb, ke);
  f32x16 acc[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[nt][i] = 0.0f;
  // Two register sets: the loads for K-step i+2 are issued right after step i's tiles are published, so each load
  // has two K-steps of MFMAs to land (a 64-wide tile's single step is ~0.25 us of MFMA, below HBM latency).
  float ra[2][4], rb[2][NT][4], rsum = 0.0f;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    if (kb + s * GBK < ke) {
      p.load_a(ctx, kb + s * GBK, ke, ra[s]);
#pragma unroll
      for (int pp = 0; pp < NT; ++pp) p.load_b(ctx, pp, kb + s * GBK, ke, rb[s][pp]);
    }
  }
  for (int k00 = kb; k00 < ke; k00 += 2 * GBK) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int k0 = k00 + s * GBK;
      if (k0 >= ke) break;
      P::APat::template store<GLDA>(As[s], ra[s], tid, 0);
#pragma unroll
      for (int pp = 0; pp < NT; ++pp) P::BPat::template store<LDB>(Bs[s], rb[s][pp], tid, pp);
      lds_barrier();   // LDS only: the other register set's loads stay in flight
      if (k0 + 2 * GBK < ke) {
        p.load_a(ctx, k0 + 2 * GBK, ke, ra[s]);
#pragma unroll
        for (int pp = 0; pp < NT; ++pp) p.load_b(ctx, pp, k0 + 2 * GBK, ke, rb[s][pp]);
      }
      const float* a = As[s] + (lane >> 5) * GLDA + wm * 32 + (lane & 31);
      const float* b = Bs[s] + (lane >> 5) * LDB + wn * (BN / 2) + (lane & 31);
#pragma unroll
      for (int kk = 0; kk < GBK; kk += 2) {
        const float av = a[kk * GLDA];
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[nt] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, b[kk * LDB + nt * 32], acc[nt], 0, 0, 0);
      }
      if (P::kRowSum) {
        if (blockIdx.y == 0 && tid < GBM) {
#pragma unroll
          for (int kk = 0; kk < GBK; ++kk) rsum += As[s][kk * GLDA + tid];
        }
      }
    }
  }
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) p.epilogue(ctx, acc[nt], m0 + wm * 32, n0 + wn * (BN / 2) + nt * 32, z, lane);
  if (P::kRowSum) {
    if (blockIdx.y == 0 && tid < GBM) p.rowsum_out(m0 + tid, z, rsum);
  }
}

template <class P>
inline hipError_t launch_gemm(const P& p, int M, int N, int Z, hipStream_t s) {
  dim3 grid((M + GBM - 1) / GBM, (N + P::BN - 1) / P::BN, Z);
  if (grid.x == 0 || grid.y == 0 || grid.z == 0) return hipSuccess;
  hipLaunchKernelGGL(gemm_f32_kernel<P>, grid, dim3(256), 0, s, p);
  return hipGetLastError();
}

}  // namespace mq
