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
#include "mix_kernels.hpp"
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
  // state rows | two weight-chunk buffers | biases
  __host__ __device__ size_t floats() const { return (size_t)HYR * SP + (size_t)128 * SP + 1024; }
  // LDS request: at least 81 KB, so one workgroup per CU — ceil(M / 32) x 2 workgroups then spread over the
  // CUs instead of pairing up on half of them (each pays its full MFMA time either way)
  size_t lds_bytes() const { return std::max(floats() * sizeof(float), (size_t)81 * 1024); }
};

inline bool hyper_ok(int S, int NH) {
  return S <= 4 * HYW && NH <= 1024 && HyperGeom(S, NH).floats() * sizeof(float) <= 160 * 1024;
}

// grid = (ceil(M / 32), 2 nets), 64 * NW threads (NW = 4 or 8 waves). VAR (the round-3 scripts/rec_micro.hip only): 1 stamp
// phases into S0[]. With 8 waves each wave owns one (16-row M-tile, 16-column N-tile) pair of a chunk; with 4 waves,
// one N-tile for both M-tiles.
template <int VAR = 0, int NW = 4>
__global__ __launch_bounds__(64 * NW) void hyper_kernel(Dims d, Rep rp, const float* __restrict__ P0,
                                                        const float* __restrict__ P1, Lay L, float* __restrict__ HYP,
                                                        float* __restrict__ S0) {
  constexpr int NT = 64 * NW, WR = 64 / NW, SR = HYR / NW;   // threads, weight rows / state rows per wave
  uint64_t ts0 = (VAR & 1) ? __builtin_amdgcn_s_memtime() : 0, tstore = 0, tbar = 0, tmfma = 0, tfetch = 0, tg = 0;
  extern __shared__ __attribute__((aligned(16))) float dyn[];
  const HyperGeom G(d.S, d.NH);
  float* st = dyn;                  // [32][SP] gathered states, zero-padded
  float* wst = st + HYR * G.SP;     // [2][64][SP] weight chunks (double-buffered)
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, c16 = lane & 15;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: row-level address math stays scalar
  const int z = blockIdx.y, n = d.n, E = d.E, NH = d.NH, S = d.S, Kq = G.Kq, SP = G.SP;
  const int m0 = blockIdx.x * HYR;
  const float* __restrict__ P = z ? P1 : P0;

  // weight chunk c (rows 64c ..): wave wv loads rows WR wv .. WR wv + WR - 1, lane l columns l, l + 64, l + 128
  // (coalesced; the row's parameter segment is wave-uniform, so the per-element address math is one add)
  constexpr int HCG = HYW / 16;   // column groups of 64: S <= 64 * HCG
  float wr[WR][HCG];
  auto fetch = [&](int c) {
#pragma unroll
    for (int i = 0; i < WR; ++i) {
      const int j = 64 * c + WR * wv + i;
      const HypSeg sg = hyp_seg(L, n * E, E, min(j, NH - 1));
      const float* row = P + sg.w + (int64_t)sg.row * S;
      // unconditional loads from clamped addresses (a branch per load would force vmcnt(0) at every merge); rows
      // past NH are zeroed at the LDS store
#pragma unroll
      for (int cg = 0; cg < HCG; ++cg) wr[i][cg] = row[min(lane + 64 * cg, S - 1)];
    }
  };
  fetch(0);
  if (VAR & 1) { __builtin_amdgcn_s_waitcnt(0); tg = __builtin_amdgcn_s_memtime(); }
  {
    // state rows: wave wv gathers rows SR wv .. SR wv + SR - 1 (row base wave-uniform), lane l columns l, l + 64, ..
    constexpr int HCG2 = HYW / 16;
    float vs[SR][HCG2];
#pragma unroll
    for (int i = 0; i < SR; ++i) {
      const int m = m0 + SR * wv + i, mc = min(m, d.M - 1);
      const int t = (int)fdiv((uint32_t)mc, d.dB), b = mc - t * d.B;
      const float* row = rp.state + (rp.ep(b) * d.t_stride + t + z) * (int64_t)S;
#pragma unroll
      for (int cg = 0; cg < HCG2; ++cg) vs[i][cg] = row[min(lane + 64 * cg, S - 1)];
    }
#pragma unroll
    for (int i = 0; i < SR; ++i) {
      const int ii = SR * wv + i, m = m0 + ii;
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
  float* bias_s = wst + 128 * SP;   // [NH]
  for (int j = tid; j < NH; j += NT) {
    const HypSeg sg = hyp_seg(L, n * E, E, j);
    bias_s[j] = P[sg.b + sg.row];
  }
  // every LDS element the MFMA loop reads is written (zeros past S / NH / M), so nothing is cleared first
  auto stage = [&](int c) {   // fetched chunk c -> buffer c & 1
    float* dst = wst + (c & 1) * 64 * SP;
#pragma unroll
    for (int i = 0; i < WR; ++i) {
      const float live = 64 * c + WR * wv + i < NH ? 1.0f : 0.0f;
#pragma unroll
      for (int cg = 0; cg < HCG; ++cg) {
        const int col = lane + 64 * cg;
        dst[(WR * wv + i) * SP + col] = col < S ? wr[i][cg] * live : 0.0f;
      }
    }
  };
  stage(0);
  if (G.NCH > 1) fetch(1);
  // this wave's N-tile within a chunk and its first M-tile (NW == 8: one M-tile per wave)
  const int ntile = NW == 8 ? (wv & 3) : wv, mt0 = NW == 8 ? (wv >> 2) : 0;
  uint64_t tl0 = (VAR & 1) ? __builtin_amdgcn_s_memtime() : 0;
  for (int c = 0; c < G.NCH; ++c) {
    uint64_t ta = (VAR & 1) ? __builtin_amdgcn_s_memtime() : 0;
    // buffer c & 1 staged; buffer (c + 1) & 1 no longer read (chunk c - 1's MFMAs); at c = 0 the state rows staged
    __syncthreads();
    if (VAR & 1) { const uint64_t tb = __builtin_amdgcn_s_memtime(); tbar += tb - ta; ta = tb; }
    if (c + 1 < G.NCH) stage(c + 1);   // fetched one chunk ago
    if (VAR & 1) { const uint64_t tb = __builtin_amdgcn_s_memtime(); tstore += tb - ta; ta = tb; }
    if (c + 2 < G.NCH) fetch(c + 2);
    if (VAR & 1) { const uint64_t tb = __builtin_amdgcn_s_memtime(); tfetch += tb - ta; ta = tb; }
    f32x4 acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};   // M-tiles mt0, mt0 + 1 (rows c16 and 16 + c16)
    const float* a0 = st + (16 * mt0 + c16) * SP + g * Kq;
    const float* a1 = a0 + 16 * SP;
    const float* bw = wst + (c & 1) * 64 * SP + (16 * ntile + c16) * SP + g * Kq;
    for (int mm = 0; mm < Kq / 4; ++mm) {
      const f32x4 bv = *(const f32x4*)&bw[4 * mm];
      const f32x4 av0 = *(const f32x4*)&a0[4 * mm];
      if (NW == 8) {
#pragma unroll
        for (int e = 0; e < 4; ++e) acc0 = mfma16x4(av0[e], bv[e], acc0);
      } else {
        const f32x4 av1 = *(const f32x4*)&a1[4 * mm];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          acc0 = mfma16x4(av0[e], bv[e], acc0);
          acc1 = mfma16x4(av1[e], bv[e], acc1);
        }
      }
    }
    const int j = 64 * c + 16 * ntile + c16;
    if (j < NH) {
      const float bj = bias_s[j];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + 16 * mt0 + 4 * g + e;
        if (m < d.M) out[(int64_t)m * NH + j] = acc0[e] + bj;
        if (NW == 4 && m + 16 < d.M) out[(int64_t)(m + 16) * NH + j] = acc1[e] + bj;
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

// Wave-specialised form: 4 loader waves (waves 0-3, dispatched first: their chunk-0 fetch is the critical path)
// and 8 MFMA waves (wave 4 + w: M-tile w >> 2, N-tile w & 3 of each 64-row chunk) in one 768-thread workgroup.
// The loaders stage chunk c + 1 into the idle LDS buffer and fetch chunk c + 2 while the MFMA waves consume chunk
// c: one barrier per chunk. gfx950 issues no VALU op while the SIMD's f32 MFMA pipe is busy
// (scripts/coexec2_micro.hip, in git at 2f3e4ef: 48 v_fma 56 -> 564 cycles beside MFMA chains), so the loader path carries no VALU
// and no branch: loader wave lw copies the 16 contiguous weight rows 16 (4c + lw) .. + 15 (one parameter segment
// when E % 16 == 0) as 48 x 64 floats (buffer loads: scalar row-group base, lane offset 4 lane + 256 q; past the
// group they read the following parameters, past the end zeros) into a 3072-float LDS slot (row pitch S, ds_write
// at immediate offsets). Fragment reads past column S of a row see finite neighbours, which meet the zero
// K-padding of the state rows; row groups past NH load a clamped real group whose outputs are never stored. The
// MFMA waves' K loop is a fixed 12 steps (immediate LDS offsets, no guards) and their outputs go out through a
// buffer descriptor (rows past M are dropped by its range check). Same operand maps and summation order as
// hyper_kernel: bitwise-identical HYP. grid = (ceil(M / 32), 2 nets), 768 threads, hyper_ws_lds_bytes().
constexpr int HYWS_THREADS = 768;
constexpr int HYWS_SPS = 4 * HYW + 4;   // state-row pitch
constexpr int HYWS_GS = 48 * 64;         // LDS slot of one 16-row weight group (16 S <= 3072 floats, S <= 192)
__host__ __device__ inline size_t hyper_ws_floats(int) {
  return (size_t)HYR * HYWS_SPS + 2 * 4 * HYWS_GS + 1024;   // states | 2 chunks of 4 groups | biases
}
inline size_t hyper_ws_lds_bytes(int S) { return hyper_ws_floats(S) * sizeof(float); }
inline bool hyper_ws_ok(int S, int E, int NH, int64_t M) {
  return S <= 4 * HYW && S % 4 == 0 && E % 16 == 0 && NH <= 1024 && hyper_ws_lds_bytes(S) <= 160 * 1024 &&
         M * NH * 4 < (1LL << 31);
}

template <int VAR = 0>
__global__ __launch_bounds__(HYWS_THREADS) void hyper_ws_kernel(Dims d, Rep rp, const float* __restrict__ P0,
                                                                const float* __restrict__ P1, Lay L,
                                                                float* __restrict__ HYP, float* __restrict__ S0) {
  constexpr int NLW = 4, SR = HYR / 8, SP = HYWS_SPS, HCG = HYW / 16;
  const uint64_t ts0 = (VAR & 1) ? __builtin_amdgcn_s_memtime() : 0;
  extern __shared__ __attribute__((aligned(16))) float dyn[];
  const int S = d.S, NH = d.NH, n = d.n, E = d.E;
  const int Kq = HYW, NCH = (NH + 63) / 64, WB = 4 * HYWS_GS;   // fixed K extent: 4 Kq = 192 >= S
  float* st = dyn;                  // [32][SP] gathered states, zero K-padding
  float* wst = st + HYR * SP;       // [2][4][HYWS_GS] weight chunks: 16-row groups, row pitch S
  float* bias_s = wst + 2 * WB;     // [NH]
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, c16 = lane & 15;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int z = blockIdx.y, m0 = blockIdx.x * HYR;
  const float* __restrict__ P = z ? P1 : P0;

  if (wv < NLW) {
    // ---- loader waves
    const int lw = wv;
    const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)P, (short)0, (int)(L.o[MQ_P_COUNT] * sizeof(float)), 0x00020000);
    const int voff = 4 * lane;
    uint64_t* stl = (uint64_t*)S0 + 32 * (blockIdx.y * gridDim.x + blockIdx.x) + 16;
    const bool stamp = (VAR & 1) && lw == 0 && lane == 0;
    if (stamp) stl[0] = __builtin_amdgcn_s_memtime();
    float wr[48];
    auto fetch = [&](int c) {
      const int j0 = min(16 * (4 * c + lw), NH - 16);
      const HypSeg sg = hyp_seg(L, n * E, E, j0);
      const int base = (int)(sg.w + (int64_t)sg.row * S) * 4;
#pragma unroll
      for (int q = 0; q < 48; ++q)
        wr[q] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(prs, voff, base + 256 * q, 0));
    };
    float* const dst0 = wst + lw * HYWS_GS + lane;
    auto stage = [&](int c) {
      float* dst = dst0 + (c & 1) * WB;
#pragma unroll
      for (int q = 0; q < 48; ++q) dst[64 * q] = wr[q];
    };
    fetch(0);
    for (int j = lw * 64 + lane; j < NH; j += NLW * 64) {
      const HypSeg sg = hyp_seg(L, n * E, E, j);
      bias_s[j] = P[sg.b + sg.row];
    }
    stage(0);
    if (NCH > 1) fetch(1);
    for (int c = 0; c < NCH; ++c) {
      if (stamp) stl[1 + min(c, 6)] = __builtin_amdgcn_s_memtime();
      __syncthreads();   // chunk c staged; buffer (c + 1) & 1 free
      if (c + 1 < NCH) stage(c + 1);
      if (c + 2 < NCH) fetch(c + 2);
    }
    if (stamp) stl[8] = __builtin_amdgcn_s_memtime();
    return;
  }
  // ---- MFMA waves: gather this wave's state rows (row base wave-uniform), then one (M-tile, N-tile) per chunk
  const int mw = wv - NLW;
  {
    float vs[SR][HCG];
#pragma unroll
    for (int i = 0; i < SR; ++i) {
      const int m = m0 + SR * mw + i, mc = min(m, d.M - 1);
      const int t = (int)fdiv((uint32_t)mc, d.dB), b = mc - t * d.B;
      const float* row = rp.state + (rp.ep(b) * d.t_stride + t + z) * (int64_t)S;
#pragma unroll
      for (int cg = 0; cg < HCG; ++cg) vs[i][cg] = row[min(lane + 64 * cg, S - 1)];
    }
#pragma unroll
    for (int i = 0; i < SR; ++i) {
      const int ii = SR * mw + i, m = m0 + ii;
#pragma unroll
      for (int cg = 0; cg < HCG; ++cg) {
        const int col = lane + 64 * cg;
        const float v = (col < S && m < d.M) ? vs[i][cg] : 0.0f;
        st[ii * SP + col] = v;
        if (!(VAR & 1) && z == 0 && S0 && m < d.M && col < S) S0[(int64_t)m * S + col] = v;
      }
    }
  }
  const int ntile = mw & 3, mt = mw >> 2;
  // outputs: rows m0 + 16 mt + 4 g + e, column 64 c + 16 ntile + c16; rows past M fall outside the descriptor
  const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(HYP + (int64_t)z * d.M * NH), (short)0, (int)((int64_t)d.M * NH * sizeof(float)), 0x00020000);
  const int obase = ((m0 + 16 * mt + 4 * g) * NH + 16 * ntile + c16) * 4;
  const float* a0 = st + (16 * mt + c16) * SP + g * Kq;
  uint64_t* stm = (uint64_t*)S0 + 32 * (blockIdx.y * gridDim.x + blockIdx.x);
  const bool stamp = (VAR & 1) && mw == 0 && lane == 0;
  if (stamp) { stm[0] = ts0; stm[1] = __builtin_amdgcn_s_memtime(); }
  for (int c = 0; c < NCH; ++c) {
    __syncthreads();
    if (stamp) stm[2 + min(c, 6)] = __builtin_amdgcn_s_memtime();
    f32x4 acc = {0, 0, 0, 0};
    const float* bw = wst + (c & 1) * WB + ntile * HYWS_GS + c16 * S + g * Kq;
#pragma unroll
    for (int mm = 0; mm < ((VAR & 4) ? 0 : HYW / 4); ++mm) {
      const f32x4 bv = *(const f32x4*)&bw[4 * mm];
      const f32x4 av = *(const f32x4*)&a0[4 * mm];
#pragma unroll
      for (int e = 0; e < 4; ++e) acc = mfma16x4(av[e], bv[e], acc);
    }
    if (64 * c + 16 * ntile < NH) {   // wave-uniform: NH % 16 == 0
      const float bj = bias_s[64 * c + 16 * ntile + c16];
#pragma unroll
      for (int e = 0; e < 4; ++e)
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, acc[e] + bj), ors, obase,
                                              (e * NH + 64 * c) * 4, 0);
    }
  }
  if (stamp) stm[9] = __builtin_amdgcn_s_memtime();
}

}  // namespace mq
