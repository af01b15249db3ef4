// dW_hyper: the QMIX hypernet weight and bias gradients, summed over the M = T*B mixer rows
//   dW[j][s] = sum_m dHYP[m][j] S0[m][s],   db[j] = sum_m dHYP[m][j]
// (the backward of qmix.py:30-44's four state-fed Linear layers, in their concatenated order [hyper_w_1 |
// hyper_w_final | hyper_b_1 | V.0], see hyp_seg).
//
// Both operands are stored m-major (one contiguous row of NH / S floats per mixer row), so the MFMA operands come
// straight from global memory in v_mfma_f32_32x32x2_f32 layout with no LDS staging: lane l of a wave reads
// S0[m + (l >> 5)][s0 + (l & 31)] (A, rows = s) and dHYP[m + (l >> 5)][j0 + (l & 31)] (B, columns = j) — two
// 128-byte segments per operand per MFMA. The bias is a ones column appended to S0 (s == S), so db falls out of
// the same accumulator. A workgroup owns a 32 (s) x 32 (j) output tile and one of `nsplit` slices of m; its four
// waves take interleaved quarters of that slice and are summed through LDS, so each workgroup writes one partial
// tile (coalesced along s) into slab[z] in the parameter layout relative to hyper_w_1.weight. red_pass1 sums the
// nsplit partials. The m loop is branch-free: rows past the slice read a clamped row with a zero factor.
//
// Two hosts of dwh_body: dwh_red1_kernel (beside pass 1 of the slab reduction, the default) and the fused BPTT's
// appended workgroups (gru_bwd_fused.hpp, DWH = 1). Each wave walks the same m steps in the same order in both, so
// their results are bitwise equal. (A side-stream instance beside the BPTT lost its A/B in round 1 — its MFMA waves
// on the chain's SIMDs slowed the BPTT 14 %, profiles/r01m_ab_dwh/ — and was removed in round 4.)
#pragma once
#include "learner_gemms.hpp"
#include "optim_kernels.hpp"

namespace mq {

constexpr int DWH_T = 32;   // output tile edge

// grid = ceil(NH / 32) * ceil((S + 1) / 32) * nsplit (tiles_j = ceil(NH / 32)), 256 threads.
// U: MFMAs (2 m-rows each) per pipelined block.
// tid: the thread's index in its 256-thread group; red: that group's [4][DWH_T (DWH_T + 1)] floats of LDS (a
// 512-thread workgroup runs two tiles, one per half, with one workgroup barrier in common)
template <int U, int NB>
MQ_DEV void dwh_body(Dims d, Lay L, const float* __restrict__ dHYP, const float* __restrict__ S0,
                     float* __restrict__ slab, int64_t len, int nsplit, int tiles_j, int lin, int tid, float* red_) {
  float(*red)[DWH_T * (DWH_T + 1)] = (float(*)[DWH_T * (DWH_T + 1)])red_;
  const int lane = tid & 63, wv = tid >> 6;
  const int NH = d.NH, S = d.S, M = d.M;
  // 1-D grid, slice-minor: consecutive workgroups go to consecutive XCDs, so with nsplit a multiple of 8 every
  // workgroup of m-slice z runs on XCD z % 8 and the slice's dHYP / S0 rows are fetched into one L2 only
  const int z = lin % nsplit, tile = lin / nsplit;
  const int j0 = (tile % tiles_j) * DWH_T, s0 = (tile / tiles_j) * DWH_T;
  // m slice of this workgroup, in 2-row MFMA steps; wave wv takes steps wv, wv + 4, ..
  const int steps = (M + 1) >> 1;
  const int sb = (int)((int64_t)steps * z / nsplit), se = (int)((int64_t)steps * (z + 1) / nsplit);
  const int half = lane >> 5, c = lane & 31;
  const int jl = min(j0 + c, NH - 1);
  const int s = s0 + c, sl = min(s, S - 1);
  const float amul = s < S ? 1.0f : 0.0f, aadd = s == S ? 1.0f : 0.0f;

  f32x16 acc = {};
  // NB register buffers of U MFMA steps each (static indices only): block k + NB - 1 is fetched while block k's
  // MFMAs run, so NB - 1 blocks of loads are in flight. Each block costs ~one memory latency when NB = 2 (8 MFMAs
  // are ~0.2 us, a load round trip 1 - 2 us under the reduction's traffic): the m loop was latency-bound.
  float a[NB][U], b[NB][U];
  auto load = [&](float (&a)[U], float (&b)[U], int st0) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int stp = st0 + 4 * u;
      const int m = 2 * stp + half;
      const int mc = min(m, M - 1);
      const float live = (stp < se && m < M) ? 1.0f : 0.0f;
      a[u] = fmaf(S0[(int64_t)mc * S + sl], amul, aadd);
      b[u] = dHYP[(int64_t)mc * NH + jl] * live;
    }
  };
  auto mma = [&](const float (&a)[U], const float (&b)[U]) {
#pragma unroll
    for (int u = 0; u < U; ++u) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u], b[u], acc, 0, 0, 0);
  };
  constexpr int BLK = 4 * U;   // steps per block over the four waves
  const int st = sb + wv;
  const int nblk = (se - sb + BLK - 1) / BLK;
#pragma unroll
  for (int p = 0; p < NB - 1; ++p)
    if (p < nblk) load(a[p], b[p], st + p * BLK);
  for (int blk = 0; blk < nblk; blk += NB) {
#pragma unroll
    for (int q = 0; q < NB; ++q) {   // block blk + q sits in buffer q; block blk + q + NB - 1 goes to buffer q - 1
      if (blk + q >= nblk) break;
      if (blk + q + NB - 1 < nblk) load(a[(q + NB - 1) % NB], b[(q + NB - 1) % NB], st + (blk + q + NB - 1) * BLK);
      mma(a[q], b[q]);
    }
  }
  // D[i = s][j]: lane holds column j = c, rows i = 8 (r / 4) + 4 half + r % 4
#pragma unroll
  for (int r = 0; r < 16; ++r) red[wv][c * (DWH_T + 1) + 8 * (r >> 2) + 4 * half + (r & 3)] = acc[r];
  __syncthreads();
  float* out = slab + (int64_t)z * len;
  const int64_t base = L.o[MQ_P_HW1_W];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int e = tid + 256 * q, jj = j0 + (e >> 5), ss = s0 + (e & 31);
    const int o = (e >> 5) * (DWH_T + 1) + (e & 31);
    const float v = red[0][o] + red[1][o] + red[2][o] + red[3][o];
    if (jj < NH && ss <= S) {
      const HypSeg sg = hyp_seg(L, d.n * d.E, d.E, jj);
      if (ss < S) out[sg.w - base + (int64_t)sg.row * S + ss] = v;
      else out[sg.b - base + sg.row] = v;
    }
  }
}

// Horizontal fusion: dW_hyper (blocks [0, ndwh)) beside pass 1 of the slab reduction (blocks [ndwh_pad, ..)) in one
// launch. Neither reads the other's output (pass 1 covers the BPTT's and the mixer's slabs; dW_hyper's own slabs
// are summed in pass 2, which reads them directly), so the reduction's HBM reads overlap dW_hyper's MFMA chains
// instead of following them. ndwh_pad is a multiple of 16, so pass 1's block -> XCD mapping is unchanged.
template <int NB = 4>
__global__ __launch_bounds__(256) void dwh_red1_kernel(Dims d, Lay L, const float* __restrict__ dHYP,
                                                       const float* __restrict__ S0, float* __restrict__ slab,
                                                       int64_t len, int nsplit, int tiles_j, int ndwh, int ndwh_pad,
                                                       RedPlan pl) {
  const int b = blockIdx.x;
  if (b < ndwh_pad) {
    __shared__ float red[4 * DWH_T * (DWH_T + 1)];
    if (b < ndwh) dwh_body<8, NB>(d, L, dHYP, S0, slab, len, nsplit, tiles_j, b, threadIdx.x, red);
    return;
  }
  red_pass1_body(pl, b - ndwh_pad);
}

}  // namespace mq
