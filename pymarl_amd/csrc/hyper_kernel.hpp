// QMIX hypernet for both nets: HYP[z][m][NH] = state_{t+z}(m) W_z^T + b_z, m = t*B + b, NH = E (n + 3) outputs
// [hyper_w_1 | hyper_w_final | hyper_b_1 | V.0] (qmix.py:16-26, 30-44; q_learner.py:81-82 for both nets).
//
// A weight-streaming GEMM shaped for this problem (M = T*B ~ 4k rows, K = S ~ 170, N = NH ~ 350): a workgroup owns
// 32 gathered state rows of one net (in LDS for the whole kernel) and streams that net's weight matrix through LDS
// once, in 64-row chunks (coalesced loads; the next chunk is prefetched into registers under the current chunk's
// MFMAs). v_mfma_f32_16x16x4_f32 with the gru_fwd_fused.hpp operand maps: wave w owns N-tile w of a chunk for
// both 16-row M-tiles (one B fragment, two accumulators), lane group g a contiguous quarter of K (b128 reads).
// One workgroup per CU (see HyperGeom::lds_bytes). The z == 0 pass also writes the gathered rows to S0 (the
// dW_hyper GEMM's operand).
#pragma once
#include "learner_gemms.hpp"
#include "gru_fwd_fused.hpp"
#include <algorithm>

namespace mq {

constexpr int HYR = 32;   // state rows per workgroup
constexpr int HYW = 48;   // weight-chunk elements per thread: 64 rows * S / 256 threads, S <= 4 * HYW = 192

struct HyperGeom {   // dynamic LDS carve-up, shared by host (size) and device
  int Kq, SP, NCH;
  __host__ __device__ HyperGeom(int S, int NH) {
    Kq = (S + 15) / 16 * 4;   // k-blocks per lane group
    SP = HYW * 4 + 4;         // row pitch: every 64-column group of a row is stored (zeros past S)
    NCH = (NH + 63) / 64;     // 64-row weight chunks
  }
  __host__ __device__ size_t floats() const { return (size_t)HYR * SP + (size_t)64 * SP + 1024; }   // + biases
  // LDS request: at least 81 KB, so one workgroup per CU — ceil(M / 32) x 2 workgroups then spread over the
  // CUs instead of pairing up on half of them (each pays its full MFMA time either way)
  size_t lds_bytes() const { return std::max(floats() * sizeof(float), (size_t)81 * 1024); }
};

inline bool hyper_ok(int S, int NH) {
  return S <= 4 * HYW && NH <= 1024 && HyperGeom(S, NH).floats() * sizeof(float) <= 160 * 1024;
}

// grid = (ceil(M / 32), 2 nets), 256 threads. VAR (scripts/rec_micro.hip only): 1 stamp phases into S0[].
template <int VAR = 0>
__global__ __launch_bounds__(256) void hyper_kernel(Dims d, Rep rp, const float* __restrict__ P0,
                                                    const float* __restrict__ P1, Lay L, float* __restrict__ HYP,
                                                    float* __restrict__ S0) {
  uint64_t ts0 = (VAR & 1) ? __builtin_amdgcn_s_memtime() : 0, tstore = 0, tbar = 0, tmfma = 0, tfetch = 0, tg = 0;
  extern __shared__ float dyn[];
  const HyperGeom G(d.S, d.NH);
  float* st = dyn;                  // [32][SP] gathered states, zero-padded
  float* wst = st + HYR * G.SP;     // [64][SP] weight chunk
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, c16 = lane & 15;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: row-level address math stays scalar
  const int z = blockIdx.y, n = d.n, E = d.E, NH = d.NH, S = d.S, Kq = G.Kq, SP = G.SP;
  const int m0 = blockIdx.x * HYR;
  const float* __restrict__ P = z ? P1 : P0;

  // weight chunk c (rows 64c ..): wave wv loads rows 16 wv .. 16 wv + 15, lane l columns l, l + 64, l + 128
  // (coalesced; the row's parameter segment is wave-uniform, so the per-element address math is one add)
  constexpr int HCG = HYW / 16;   // column groups of 64: S <= 64 * HCG
  float wr[16][HCG];
  auto fetch = [&](int c) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int j = 64 * c + 16 * wv + i;
      const HypSeg sg = hyp_seg(L, n * E, E, min(j, NH - 1));
      const float* row = P + sg.w + (int64_t)sg.row * S;
      // unconditional loads from clamped addresses (a branch per load would force vmcnt(0) at every merge)
#pragma unroll
      for (int cg = 0; cg < HCG; ++cg) wr[i][cg] = row[min(lane + 64 * cg, S - 1)];
      if (j >= NH) {
#pragma unroll
        for (int cg = 0; cg < HCG; ++cg) wr[i][cg] = 0.0f;
      }
    }
  };
  fetch(0);
  if (VAR & 1) { __builtin_amdgcn_s_waitcnt(0); tg = __builtin_amdgcn_s_memtime(); }
  for (int e = tid; e < HYR * SP; e += 256) st[e] = 0.0f;
  for (int e = tid; e < 64 * SP; e += 256) wst[e] = 0.0f;
  __syncthreads();
  {
    // state rows: wave wv gathers rows 8 wv .. 8 wv + 7 (row base wave-uniform), lane l columns l, l + 64, ..
    constexpr int HCG2 = HYW / 16;
    float vs[HYR / 4][HCG2];
#pragma unroll
    for (int i = 0; i < HYR / 4; ++i) {
      const int m = m0 + (HYR / 4) * wv + i, mc = min(m, d.M - 1);
      const int t = (int)fdiv((uint32_t)mc, d.dB), b = mc - t * d.B;
      const float* row = rp.state + (rp.ep(b) * d.t_stride + t + z) * (int64_t)S;
#pragma unroll
      for (int cg = 0; cg < HCG2; ++cg) vs[i][cg] = row[min(lane + 64 * cg, S - 1)];
    }
#pragma unroll
    for (int i = 0; i < HYR / 4; ++i) {
      const int ii = (HYR / 4) * wv + i, m = m0 + ii;
#pragma unroll
      for (int cg = 0; cg < HCG2; ++cg) {
        const int col = lane + 64 * cg;
        const float v = (col < S && m < d.M) ? vs[i][cg] : 0.0f;
        st[ii * SP + col] = v;
        if (!(VAR & 1) && z == 0 && S0 && m < d.M && col < S) S0[(int64_t)m * S + col] = v;
      }
    }
  }
  float* out = HYP + (int64_t)z * d.M * NH;
  float* bias_s = wst + 64 * SP;   // [NH]
  for (int j = tid; j < NH; j += 256) {
    const HypSeg sg = hyp_seg(L, n * E, E, j);
    bias_s[j] = P[sg.b + sg.row];
  }
  uint64_t tl0 = (VAR & 1) ? __builtin_amdgcn_s_memtime() : 0;
  for (int c = 0; c < G.NCH; ++c) {
    uint64_t ta = (VAR & 1) ? __builtin_amdgcn_s_memtime() : 0;
    __syncthreads();   // previous chunk's operand reads of wst done (and, at c = 0, the state rows staged)
    if (VAR & 1) { const uint64_t tb = __builtin_amdgcn_s_memtime(); tbar += tb - ta; ta = tb; }
#pragma unroll
    for (int i = 0; i < 16; ++i)
#pragma unroll
      for (int cg = 0; cg < HCG; ++cg) {
        const int col = lane + 64 * cg;
        wst[(16 * wv + i) * SP + col] = col < S ? wr[i][cg] : 0.0f;
      }
    if (VAR & 1) { const uint64_t tb = __builtin_amdgcn_s_memtime(); tstore += tb - ta; ta = tb; }
    __syncthreads();
    if (VAR & 1) { const uint64_t tb = __builtin_amdgcn_s_memtime(); tbar += tb - ta; ta = tb; }
    if (c + 1 < G.NCH) fetch(c + 1);
    if (VAR & 1) { const uint64_t tb = __builtin_amdgcn_s_memtime(); tfetch += tb - ta; ta = tb; }
    f32x4 acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};   // M-tiles 0, 1 (rows c16 and 16 + c16)
    const float* a0 = st + c16 * SP + g * Kq;
    const float* a1 = a0 + 16 * SP;
    const float* bw = wst + (16 * wv + c16) * SP + g * Kq;
    for (int mm = 0; mm < Kq / 4; ++mm) {
      const f32x4 bv = *(const f32x4*)&bw[4 * mm];
      const f32x4 av0 = *(const f32x4*)&a0[4 * mm];
      const f32x4 av1 = *(const f32x4*)&a1[4 * mm];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        acc0 = mfma16x4(av0[e], bv[e], acc0);
        acc1 = mfma16x4(av1[e], bv[e], acc1);
      }
    }
    const int j = 64 * c + 16 * wv + c16;
    if (j < NH) {
      const float bj = bias_s[j];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + 4 * g + e;
        if (m < d.M) out[(int64_t)m * NH + j] = acc0[e] + bj;
        if (m + 16 < d.M) out[(int64_t)(m + 16) * NH + j] = acc1[e] + bj;
      }
    }
    if (VAR & 1) { __builtin_amdgcn_s_waitcnt(0xC07F); tmfma += __builtin_amdgcn_s_memtime() - ta; }
  }
  if ((VAR & 1) && tid == 0) {
    uint64_t* st8 = (uint64_t*)S0 + 8 * (blockIdx.y * gridDim.x + blockIdx.x);
    st8[0] = tg - ts0; st8[1] = tl0 - tg; st8[2] = tbar; st8[3] = tstore; st8[4] = tfetch; st8[5] = tmfma;
    st8[6] = __builtin_amdgcn_s_memtime() - ts0;
  }
}

}  // namespace mq
