// fp32 MFMA GEMM core for the learner's row-parallel and weight-gradient contractions (gfx950).
//
//   C[m][n] = sum_k A(m, k) * B(k, n)
//
// One 256-thread workgroup (4 waves, 2 x 2) owns a 64 x BN tile of C (BN = 64, 128 or 192); each wave a 32 x BN/2
// strip as BN/64 accumulators of v_mfma_f32_32x32x2_f32 (exact fp32 fma chain, 64 FLOP/clk/SIMD = the fp32 peak
// on CDNA4). K advances in stages of 32, double-buffered in LDS (one barrier per stage), the next stage's global
// loads issued right after the barrier.
//
// LDS holds each operand row-major with K contiguous ([row][k], pitch 36): a stage is written with b128 stores and
// read as MFMA fragments with b128 loads. The MFMA K order is permuted for that: MFMA m of a stage takes k = m
// from lanes 0-31 and k = 16 + m from lanes 32-63, so each lane's 16 operands of a stage are 16 consecutive
// floats of its row (4 conflict-free ds_read_b128) instead of 16 strided b32 reads.
//
// The operands are "policies": each GEMM in the learner supplies how its A and B elements are fetched (gathered
// replay rows by episode id, one-hot virtual columns, transposed activations ...), which K range blockIdx.z owns
// (net index or split-K slice) and an epilogue. A policy's load returns 4 consecutive k of one row for a 16-deep
// half stage; two staging patterns cover every operand:
//   KPat: thread -> (row = tid >> 2, k = 4 (tid & 3) + i)   (row-major operand, K contiguous in memory)
//   MPat: thread -> (row = tid & 63, k = 4 (tid >> 6) + i)  (column operand, rows contiguous in memory)
// B tiles wider than 64 rows are staged in BN/64 passes of the same pattern.
#pragma once
#include <type_traits>
#include "common.hpp"

namespace mq {

constexpr int GBM = 64, GBK = 16, GSK = 32, GLD = GSK + 4;   // tile rows, half stage, stage depth, LDS pitch

struct KPat {
  MQ_DEV static int row(int tid) { return tid >> 2; }
  MQ_DEV static int kq(int tid) { return (tid & 3) * 4; }
};

struct MPat {
  MQ_DEV static int row(int tid) { return tid & 63; }
  MQ_DEV static int kq(int tid) { return (tid >> 6) * 4; }
};

// Row index (within a 32x32 accumulator tile) of register `reg` for `lane` (32x32 f32 MFMA C layout).
MQ_DEV int acc_row(int reg, int lane) { return (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5); }

template <class Pat>
MQ_DEV void stage_store(float* S, const float (&r)[4], int tid, int pass, int half) {
  *(f32x4*)&S[(64 * pass + Pat::row(tid)) * GLD + GBK * half + Pat::kq(tid)] = f32x4{r[0], r[1], r[2], r[3]};
}

#ifdef MQ_GEMM_STAMPS
__device__ uint64_t* mq_gemm_stamps;   // diagnostic build only (scripts/gemm_micro.hip)
#endif

// Row passes of a policy's A tile: P::MT when the policy declares it (1 or 2), else 1. With MT = 2 the workgroup
// owns a 128 x BN tile and each wave a 64 x BN/2 strip (2 x NT accumulators): twice the MFMAs per LDS fragment read
// and per staged B element, and half the B traffic per row of C.
template <class P, class = void>
struct gemm_mt {
  static constexpr int value = 1;
};
template <class P>
struct gemm_mt<P, std::void_t<decltype(P::MT)>> {
  static constexpr int value = P::MT;
};

template <class P>
__global__ __launch_bounds__(256) void gemm_f32_kernel(const P p) {
  constexpr int BN = P::BN, NT = BN / 64, MT = gemm_mt<P>::value, BM = GBM * MT;
  static_assert(MT == 1 || MT == 2, "MT");
  __shared__ float As[2][BM * GLD];
  __shared__ float Bs[2][BN * GLD];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wm = w >> 1, wn = w & 1, h = lane >> 5;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN, z = blockIdx.z;
  typename P::Ctx ctx[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) ctx[mt] = p.make_ctx(m0 + GBM * mt, n0, z, tid);
  int kb, ke;
  p.krange(z, kb, ke);
  f32x16 acc[MT][NT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[mt][nt][i] = 0.0f;
  float ra[2][MT][4], rb[2][NT][4], rsum = 0.0f;
  auto load = [&](int k0) {
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) p.load_a(ctx[mt], k0 + GBK * hf, ke, ra[hf][mt]);
#pragma unroll
      for (int pp = 0; pp < NT; ++pp) p.load_b(ctx[0], pp, k0 + GBK * hf, ke, rb[hf][pp]);
    }
  };
#ifdef MQ_GEMM_STAMPS
  uint64_t cs = 0, cb = 0, cm = 0, c0 = __builtin_amdgcn_s_memtime(), ca, cb0;
#endif
  if (kb < ke) load(kb);
  int buf = 0;
  for (int k0 = kb; k0 < ke; k0 += GSK) {
#ifdef MQ_GEMM_STAMPS
    ca = __builtin_amdgcn_s_memtime();
#endif
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) stage_store<typename P::APat>(As[buf], ra[hf][mt], tid, mt, hf);
#pragma unroll
      for (int pp = 0; pp < NT; ++pp) stage_store<typename P::BPat>(Bs[buf], rb[hf][pp], tid, pp, hf);
    }
#ifdef MQ_GEMM_STAMPS
    cb0 = __builtin_amdgcn_s_memtime(); cs += cb0 - ca;
#endif
    lds_barrier();   // LDS only: nothing global in flight yet
#ifdef MQ_GEMM_STAMPS
    ca = __builtin_amdgcn_s_memtime(); cb += ca - cb0;
#endif
    if (k0 + GSK < ke) load(k0 + GSK);
    if (MT == 1) {
      const float* a = As[buf] + (wm * 32 + (lane & 31)) * GLD + 16 * h;
      f32x4 av[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) av[i] = *(const f32x4*)&a[4 * i];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const float* bp = Bs[buf] + (wn * (BN / 2) + nt * 32 + (lane & 31)) * GLD + 16 * h;
        f32x4 bv[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) bv[i] = *(const f32x4*)&bp[4 * i];
#pragma unroll
        for (int m = 0; m < 16; ++m)
          acc[0][nt] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[m >> 2][m & 3], bv[m >> 2][m & 3], acc[0][nt], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const float* bp = Bs[buf] + (wn * (BN / 2) + nt * 32 + (lane & 31)) * GLD + 16 * h;
        f32x4 bv[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) bv[i] = *(const f32x4*)&bp[4 * i];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          const float* a = As[buf] + (wm * 32 * MT + mt * 32 + (lane & 31)) * GLD + 16 * h;
          f32x4 av[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) av[i] = *(const f32x4*)&a[4 * i];
#pragma unroll
          for (int m = 0; m < 16; ++m)
            acc[mt][nt] =
                __builtin_amdgcn_mfma_f32_32x32x2f32(av[m >> 2][m & 3], bv[m >> 2][m & 3], acc[mt][nt], 0, 0, 0);
        }
      }
    }
#ifdef MQ_GEMM_STAMPS
    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)
    { const uint64_t e = __builtin_amdgcn_s_memtime(); cm += e - ca; }
#endif
    if (P::kRowSum) {
      if (blockIdx.y == 0 && tid < BM) {
        const f32x4* rr = (const f32x4*)&As[buf][tid * GLD];
#pragma unroll
        for (int i = 0; i < GSK / 4; ++i) rsum += (rr[i][0] + rr[i][1]) + (rr[i][2] + rr[i][3]);
      }
    }
    buf ^= 1;
  }
#ifdef MQ_GEMM_STAMPS
  const uint64_t ce0 = __builtin_amdgcn_s_memtime();
#endif
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
      p.epilogue(ctx[mt], acc[mt][nt], m0 + wm * 32 * MT + mt * 32, n0 + wn * (BN / 2) + nt * 32, z, lane);
#ifdef MQ_GEMM_STAMPS
  if (tid == 0) {
    __builtin_amdgcn_s_waitcnt(0);
    const uint64_t ce1 = __builtin_amdgcn_s_memtime();
    uint64_t* st = mq_gemm_stamps + 8 * ((blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x);
    st[0] = cs; st[1] = cb; st[2] = cm; st[3] = ce1 - ce0; st[4] = ce1 - c0; st[5] = c0;
  }
#endif
  if (P::kRowSum) {
    if (blockIdx.y == 0 && tid < BM) p.rowsum_out(m0 + tid, z, rsum);
  }
}

template <class P>
inline hipError_t launch_gemm(const P& p, int M, int N, int Z, hipStream_t s) {
  constexpr int BM = GBM * gemm_mt<P>::value;
  dim3 grid((M + BM - 1) / BM, (N + P::BN - 1) / P::BN, Z);
  if (grid.x == 0 || grid.y == 0 || grid.z == 0) return hipSuccess;
  hipLaunchKernelGGL(gemm_f32_kernel<P>, grid, dim3(256), 0, s, p);
  return hipGetLastError();
}

}  // namespace mq
