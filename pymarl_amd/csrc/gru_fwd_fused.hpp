// Fused agent forward for one-row workgroups: fc1 -> relu -> W_ih (MFMA) feeding the GRU recurrence (VALU), with
// fc2 (MFMA) behind it — rnn_agent.py:24-28 for every (t, row) of QLearner.train's unroll (q_learner.py:49-52,
// 60-62), online and target net in one grid (blockIdx.y).
//
// The recurrence is VALU-issue bound (W_hh in VGPRs, DPP quad reductions, one LDS barrier per step) and leaves the
// matrix cores idle, so the row-parallel contractions around it run on MFMA in the same workgroup, 16 steps at a
// time (the MFMA M dimension is time). 512 threads, two wave roles meeting at the one barrier per step:
//  * recurrence waves (0-3): the h chain as gru_fwd_body<1>, but with the step's input gates read from LDS (no
//    global loads at all: nothing for vmcnt to serialise on) and h kept as a 16-step history (fc2's operand);
//  * producer waves (4-7): per chunk c of the T loop (p = t & 15), for chunk c+1 and c-1
//      p = 0        fc2 of chunk c-1: Q[16][A] = H[16][64] W2^T + b2   (hidden-state history in LDS)
//      p = 1        issue chunk c+1's obs gather (registers; consumed 4 steps later)
//      p = 5, 6     stage chunk c+1's agent inputs in LDS: obs rows, last-action / agent-id one-hots
//      p = 7 .. 10  fc1 of chunk c+1: X1[16][64] = relu(XIN[16][I] W1^T + b1)
//      p = 11 .. 15 W_ih of chunk c+1: GI[16][192] = X1 W_ih^T + b_ih  -> LDS, read by chunk c+1's steps
//    unrolled over p so each phase is straight-line code (the gather's vmcnt wait is exact). At most 12
//    v_mfma_f32_16x16x4_f32 per producer wave and step: well inside one recurrence step.
// X1 / XIN (online net, for the backward pass) and Q leave as 16-row tiles; of the target net only Q is written.
//
// MFMA operand maps (v_mfma_f32_16x16x4_f32, lane l, g = l >> 4, c = l & 15): A[i = c][kk = g],
// B[kk = g][j = c], D[i = 4g + reg][j = c]. Lane group g owns a contiguous quarter of K (k = g * Kq + kb), so
// A and B fragments are row-contiguous LDS reads (W_ih's fragments stay in VGPRs).
#pragma once
#include <cstdlib>
#include "gru_kernels.hpp"
#include "learner_gemms.hpp"

namespace mq {

constexpr int FCH = 16;            // steps per chunk
constexpr int FKQ = 28;            // fc1 k-blocks per lane group: I <= 112
constexpr int FXP = 4 * FKQ + 4;   // xin / w1 pitch
constexpr int FGATHER = 8;         // obs gather slots per producer thread: 16 * O <= 2048

MQ_DEV f32x4 mfma16x4(float a, float b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }

// Hide a value's provenance from the optimiser so address math derived from it is recomputed where it is used
// instead of being hoisted out of the chunk loop (and spilled: the producer waves run at 128 VGPRs).
MQ_DEV int opaque(int x) {
  asm volatile("" : "+v"(x));
  return x;
}

// Host-side eligibility of the fused path.
inline bool fused_fwd_ok(int I, int O, int A, int n, int64_t RT) {
  return I <= 4 * FKQ && O <= 128 && A <= 16 && n * O < (1 << 16) && RT * I < (int64_t(1) << 31);
}

struct alignas(16) FusedLds {
  float h0[H];               // init_hidden: zeros (the h_{t-1} of step 0)
  float hs[2][FCH][H + 4];   // h of the last two chunks: the recurrence's h_{t-1} and fc2's operand
  float gi[2][FCH][G3];      // input gates of the current / next chunk
  float xin[FCH][FXP];       // agent inputs of the next chunk, zero-padded to 4 * Kq
  float x1[FCH][H + 4];
  float w1[H][FXP];          // fc1 weight [64][I], zero-padded
  float w2[16][H + 4];       // fc2 weight [A <= 16][64], zero-padded
  int aprev[FCH];
};

// ---- QMIX hypernet workgroups appended to the fused forward's grid (HYP = 1): hyper_ws_kernel's GEMM (same
// operand maps, K order and outputs: bitwise its HYP and S0) in a forward workgroup's shape — 512 threads, the
// forward's 128-VGPR budget, its static LDS (one weight-chunk buffer instead of two). Dispatched after every
// row-net of the forward, these workgroups take CU slots as row-nets finish: beside the second row-net of a CU at
// cfg2 (forward + hypernet LDS fit one CU), on the CUs a second wave of row-nets leaves idle at configs[3]'s shard;
// and the hypernet launch is gone. 4 loader waves stream 64-row chunks (the fetch of chunk c + 1 overlaps chunk c's
// MFMAs; staging waits for them), 4 MFMA waves own one N-tile of a chunk for both 16-row M-tiles.
constexpr int HYF_SP = 4 * 48 + 4;   // state-row pitch (hyper_kernel.hpp HYWS_SP)
constexpr int HYF_GS = 48 * 64;      // one 16-row weight group (HYWS_GS)
__host__ __device__ constexpr int hyf_floats() { return 32 * HYF_SP + 4 * HYF_GS + 1024; }
inline bool hyf_ok(int S, int E, int NH, int64_t M) {
  return S <= 192 && S % 4 == 0 && E % 16 == 0 && NH <= 1024 && M * NH * 4 < (1LL << 31);
}

MQ_DEV void hyper_fwd_body(const Dims& d, const Rep& rp, const float* __restrict__ P0, const float* __restrict__ P1,
                           const Lay& L, float* __restrict__ HYP, float* __restrict__ S0, float* lds, int hb) {
  constexpr int SR = 8, SP = HYF_SP, HCG = 3, Kq = 48;
  const int S = d.S, NH = d.NH, n = d.n, E = d.E, NCH = (NH + 63) / 64;
  const int z = hb & 1, m0 = (hb >> 1) * 32;
  const float* __restrict__ P = z ? P1 : P0;
  float* st = lds;                   // [32][SP] gathered states, zero K-padding
  float* wst = st + 32 * SP;         // [4][HYF_GS] one weight chunk
  float* bias_s = wst + 4 * HYF_GS;  // [NH]
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, c16 = lane & 15;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (wv < 4) {
    // ---- loader waves (hyper_ws_kernel's fetch / stage)
    const int lw = wv;
    const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)P, (short)0, (int)(L.o[MQ_P_COUNT] * sizeof(float)), 0x00020000);
    const int voff = 4 * lane;
    float wr[48];
    auto fetch = [&](int c) {
      const int j0 = min(16 * (4 * c + lw), NH - 16);
      const HypSeg sg = hyp_seg(L, n * E, E, j0);
      const int base = (int)(sg.w + (int64_t)sg.row * S) * 4;
#pragma unroll
      for (int q = 0; q < 48; ++q)
        wr[q] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(prs, voff, base + 256 * q, 0));
    };
    float* const dst = wst + lw * HYF_GS + lane;
    auto stage = [&]() {
#pragma unroll
      for (int q = 0; q < 48; ++q) dst[64 * q] = wr[q];
    };
    fetch(0);
    for (int j = lw * 64 + lane; j < NH; j += 4 * 64) {
      const HypSeg sg = hyp_seg(L, n * E, E, j);
      bias_s[j] = P[sg.b + sg.row];
    }
    stage();
    __syncthreads();   // B0: chunk 0, biases and states
    for (int c = 0; c < NCH; ++c) {
      if (c + 1 < NCH) fetch(c + 1);   // in flight under chunk c's MFMAs
      __syncthreads();                 // B1: chunk c consumed
      if (c + 1 < NCH) stage();
      __syncthreads();                 // B2: chunk c + 1 staged
    }
    return;
  }
  // ---- MFMA waves: gather this wave's 8 state rows, then N-tile mw of every chunk for both M-tiles
  const int mw = wv - 4;
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
        if (z == 0 && S0 && m < d.M && col < S) S0[(int64_t)m * S + col] = v;
      }
    }
  }
  const int ntile = mw;
  const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(HYP + (int64_t)z * d.M * NH), (short)0, (int)((int64_t)d.M * NH * sizeof(float)), 0x00020000);
  const float* a0 = st + c16 * SP + g * Kq;
  const float* a1 = st + (16 + c16) * SP + g * Kq;
  const float* bw = wst + ntile * HYF_GS + c16 * S + g * Kq;
  __syncthreads();   // B0
  for (int c = 0; c < NCH; ++c) {
    f32x4 acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
#pragma unroll
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
    __syncthreads();   // B1: the loaders may overwrite the chunk
    if (64 * c + 16 * ntile < NH) {   // wave-uniform: NH % 16 == 0
      const float bj = bias_s[64 * c + 16 * ntile + c16];
      const int ob0 = ((m0 + 4 * g) * NH + 16 * ntile + c16) * 4, ob1 = ob0 + 16 * NH * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, acc0[e] + bj), ors, ob0,
                                              (e * NH + 64 * c) * 4, 0);
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, acc1[e] + bj), ors, ob1,
                                              (e * NH + 64 * c) * 4, 0);
      }
    }
    __syncthreads();   // B2
  }
}

// Measured and removed in round 4 (records under profiles/r01*-r03*): the K4 mat-vec layout, chains without
// priority or with the target chain above the online one, gathers two chunks ahead, producer work spread over all 16
// phases; each was slower in the cfg2 pipeline.
// NG: obs gather slots per producer thread (16 * O <= 256 * NG); the host picks the smallest instantiation
// (launch_fwd_fused) because every slot holds two VGPRs across the whole T loop.
// HYP = 1: workgroups past the 2R row-nets run hyper_fwd_body (grid 2R + 2 ceil(M / 32), 1-D).
template <int NG = FGATHER, int HYP = 0>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4, 4))) void gru_fwd_fused_kernel(Dims d, Rep rp, const float* __restrict__ P0,
                                                               const float* __restrict__ P1, Lay L, Work w) {
  __shared__ FusedLds S;
  static_assert(sizeof(FusedLds) >= hyf_floats() * sizeof(float), "hypernet workgroups reuse the forward's LDS");
  // workgroup index: (row, net) of the (R, 2) grid, or (HYP) the 1-D grid's first 2R workgroups (online rows, then
  // target) followed by the hypernet's; the HYP = 0 instantiation keeps the 2-D indexing (its register allocation
  // is the production one)
  const int bid = blockIdx.y * gridDim.x + blockIdx.x;
  if constexpr (HYP != 0) {
    if (bid >= 2 * d.R) {
      hyper_fwd_body(d, rp, P0, P1, L, w.HYP, w.S0, (float*)&S, bid - 2 * d.R);
      return;
    }
  }
  const int z = HYP ? (bid >= d.R ? 1 : 0) : (int)blockIdx.y;
  const bool online = z == 0;
  const float* __restrict__ P = z ? P1 : P0;
  const int tid = threadIdx.x;
  const bool rec = tid < 256;
  const int R = d.R, Tp = d.Tp, I = d.I, O = d.O, A = d.A, n = d.n;
  const int cl = (Tp - 1) / FCH;   // last chunk
  const int r = HYP ? bid - z * R : (int)blockIdx.x;
  // Output addressing: a wave-uniform base (SGPR pointer) plus a 32-bit per-lane offset, so every global access is
  // one saddr load / store with no 64-bit VALU address math.
  const uint32_t RH = (uint32_t)R * H;

  // ---- producer addressing, and chunk 0's obs gather issued first: its HBM round trip overlaps the weight loads
  const int ptid = tid - 256;   // producer thread id (negative in the recurrence waves, which never use it)
  // replay addressing of this row (r = b * n + agent)
  const int b = (int)fdiv((uint32_t)r, d.dN), ag = r - b * n;
  const int64_t slot0 = rp.ep(b) * d.t_stride;
  const float* obs_row = rp.obs + (slot0 * n + ag) * (int64_t)O;   // + t * n * O
  float* X1o = w.X1;     // online X1 [RT][H]
  float* XINo = w.XIN;   // online XIN [RT][I]
  float* Qz = w.Q + (int64_t)z * d.RT() * A;
  const uint32_t RI = (uint32_t)R * I, RA = (uint32_t)R * A;

  // gather slot s: element e = ptid + 256 s of the chunk's [16][O] obs block -> (row i, column), packed once as
  // (i << 28) | (column << 20) | (i * n * O + column) (the last field: the element's offset from the chunk's first
  // obs row, < 2^20 since n * O < 2^16); -1 past the block
  int gsl[NG];
#pragma unroll
  for (int s = 0; s < NG; ++s) {
    const int e = ptid + 256 * s, i = (int)fdiv((uint32_t)e, d.dO), col = e - i * O;
    gsl[s] = e < FCH * O ? (i << 28) | (col << 20) | (i * n * O + col) : -1;
  }
  const int nO = n * O;
  float xr[NG];
  int f_ld = 0, a_ld = -1;   // low words of filled[t-1] / actions[t-1] (int64, little-endian, small values)
  auto issue_gather = [&](int cc) {
    const int t0 = FCH * cc;
    // unconditional loads from clamped addresses (no exec-masked branches); out-of-range slots are zeroed when
    // stored (store_gather)
    const float* base = obs_row + (int64_t)t0 * nO;
    const int lim = (Tp - 1 - t0) * nO + O - 1;   // last valid element offset of this chunk
#pragma unroll
    for (int s = 0; s < NG; ++s)
      xr[s] = ld_u32(base, (uint32_t)min(opaque(gsl[s]) & 0xFFFFF, lim));
    {
      const int t = min(max(t0 + (ptid & (FCH - 1)), 1), Tp - 1) - 1;
      f_ld = *(const int*)(rp.filled + slot0 + t);
      a_ld = *(const int*)(rp.actions + (slot0 + t) * n + ag);
    }
  };
  // ---- prologue: every global load of a role (shared LDS weights, its own register-resident weights, and for the
  // producers chunk 0's obs gather first) is in flight before the first LDS store: one HBM round trip. The shared
  // part runs inside each role's branch so the two roles' register weights never share a live range.
  constexpr int N1 = (H * FXP + 511) / 512, N2 = (16 * (H + 4) + 511) / 512;
  float v1[N1], v2[N2];
  auto shared_load = [&]() {
#pragma unroll
    for (int u = 0; u < N1; ++u) {
      const int e = tid + 512 * u, nn = e / FXP, k = e - nn * FXP;
      v1[u] = (e < H * FXP && k < I) ? P[L.o[MQ_P_FC1_W] + (int64_t)nn * I + k] : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < N2; ++u) {
      const int e = tid + 512 * u, a = e / (H + 4), k = e - a * (H + 4);
      v2[u] = (e < 16 * (H + 4) && a < A && k < H) ? P[L.o[MQ_P_FC2_W] + (int64_t)a * H + k] : 0.0f;
    }
  };
  auto shared_store = [&]() {   // fc1 / fc2 weights to LDS, zero padding, h0
#pragma unroll
    for (int u = 0; u < N1; ++u) {
      const int e = tid + 512 * u;
      if (e < H * FXP) (&S.w1[0][0])[e] = v1[u];
    }
#pragma unroll
    for (int u = 0; u < N2; ++u) {
      const int e = tid + 512 * u;
      if (e < 16 * (H + 4)) (&S.w2[0][0])[e] = v2[u];
    }
    for (int e = tid; e < FCH * FXP; e += 512) (&S.xin[0][0])[e] = 0.0f;
    if (tid < H) S.h0[tid] = 0.0f;   // init_hidden: h0 = 0
  };

  if (rec) {
    // ================================================================ recurrence waves
    const int j = tid >> 2, q = tid & 3;
    f32x2 wr[8], wz[8], wn[8];   // W_hh[gate * 64 + j][16 q .. 16 q + 15] as pairs for v_pk_fma_f32
    shared_load();
    {
      const float* Whh = P + L.o[MQ_P_RNN_W_HH];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        wr[k] = f32x2{Whh[(0 * H + j) * H + 16 * q + 2 * k], Whh[(0 * H + j) * H + 16 * q + 2 * k + 1]};
        wz[k] = f32x2{Whh[(1 * H + j) * H + 16 * q + 2 * k], Whh[(1 * H + j) * H + 16 * q + 2 * k + 1]};
        wn[k] = f32x2{Whh[(2 * H + j) * H + 16 * q + 2 * k], Whh[(2 * H + j) * H + 16 * q + 2 * k + 1]};
      }
    }
    const float bhr = P[L.o[MQ_P_RNN_B_HH] + j], bhz = P[L.o[MQ_P_RNN_B_HH] + H + j],
                bhn = P[L.o[MQ_P_RNN_B_HH] + 2 * H + j];
    shared_store();
    drain_vmem();
    for (int i = 0; i < 5; ++i) lds_barrier();   // the producers' chunk-0 prologue (5 barriers)
    float* Hz = w.Hs;   // online only: the backward pass reads h_{t-1}
    const int gcol = min(q, 2) * H + j;
    // lane-split selectors as 0/1 factors: select by multiply-add, so no lane-dependent branch enters the chain
    const float m0 = q == 0 ? 1.0f : 0.0f, m1 = q == 1 ? 1.0f : 0.0f, m2 = q == 2 ? 1.0f : 0.0f;
    const float m3 = q == 3 ? 1.0f : 0.0f;
    const float bsel = m0 * bhr + m1 * bhz;
    float hprev = 0.0f;   // h_{t-1}[j]: every lane of the quad computes unit j's h, so it never re-reads LDS
    const uint32_t hlo = q == 0 ? ((uint32_t)r * H + j) * 4 : kDrop, glo = ((uint32_t)r * (4 * H) + q * H + j) * 4;
    auto step = [&](int t) {
      const int p = t & (FCH - 1), c = t / FCH;
      const float* hb = t == 0 ? S.h0 : S.hs[((t - 1) / FCH) & 1][(t - 1) & (FCH - 1)];
      const float own = S.gi[c & 1][p][gcol];   // issued with the h reads below (same LDS latency window)
      float sr, sz, sn;
      {
        const f32x4* hv4 = (const f32x4*)(&hb[16 * q]);
        f32x2 ar = {0.0f, 0.0f}, az = {0.0f, 0.0f}, an = {0.0f, 0.0f};
#pragma unroll
        for (int k4 = 0; k4 < 4; ++k4) {
          const f32x4 hv = hv4[k4];
          const f32x2 h01 = {hv[0], hv[1]}, h23 = {hv[2], hv[3]};
          ar = pk_fma(wr[2 * k4], h01, ar); ar = pk_fma(wr[2 * k4 + 1], h23, ar);
          az = pk_fma(wz[2 * k4], h01, az); az = pk_fma(wz[2 * k4 + 1], h23, az);
          an = pk_fma(wn[2 * k4], h01, an); an = pk_fma(wn[2 * k4 + 1], h23, an);
        }
        sr = quad_sum(ar.x + ar.y);
        sz = quad_sum(az.x + az.y);
        sn = quad_sum(an.x + an.y);
      }
      // lane-split gate math (as gru_fwd_body<1>): lane 0 r, lane 1 z, lane 2 n; lane q stores component q
      const float gh = fmaf(m0, sr, fmaf(m1, sz, bsel));
      const float sg = sigm_fast(gh + own);
      const float rg = quad_bcast<0>(sg), zg = quad_bcast<1>(sg);
      const float ghn = sn + bhn;
      const float ng = quad_bcast<2>(tanh_fast(own + ghn * rg));
      const float h1 = (hprev - ng) * zg + ng;   // ATen gru_cell: (hx - n) * z + n
      hprev = h1;
      if (q == 0) S.hs[c & 1][p][j] = h1;
      if (online) {
        buf_st(buf_rsrc(Hz + (int64_t)t * RH), hlo, h1);   // wave-uniform bases; lanes q != 0 drop the h store
        buf_st(buf_rsrc(w.Gates + (int64_t)t * (4 * RH)), glo, fmaf(m0, rg, fmaf(m1, zg, fmaf(m2, ng, m3 * ghn))));
      }
      lds_barrier();
    };
    // the chains of both nets issue ahead of every producer wave on the CU (the online workgroups are older and
    // would otherwise win arbitration against the target chain too)
    __builtin_amdgcn_s_setprio(2);
    for (int t = 0; t < Tp; ++t) step(t);
    __builtin_amdgcn_s_setprio(0);
    return;
  }

  // ================================================================== producer waves
  const int wv = ptid >> 6, lane = ptid & 63, g = lane >> 4, c16 = lane & 15;
  const int Kq = (I + 15) / 16 * 4;   // k-blocks per lane group (multiple of 4: b128 operand reads)
  issue_gather(0);
  shared_load();
  float wih[3][16], bih[3];
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    const int nn = 16 * (3 * wv + s) + c16;
    const float* Wi = P + L.o[MQ_P_RNN_W_IH] + (int64_t)nn * H + 16 * g;
#pragma unroll
    for (int kb = 0; kb < 16; ++kb) wih[s][kb] = Wi[kb];
    bih[s] = P[L.o[MQ_P_RNN_B_IH] + nn];
  }
  const float b1 = P[L.o[MQ_P_FC1_B] + 16 * wv + c16];
  const float b2 = c16 < A ? P[L.o[MQ_P_FC2_B] + c16] : 0.0f;
  shared_store();

  auto store_gather = [&](int cc, int s0 = 0, int s1 = NG) {
    const int t0 = FCH * cc;
    const auto xr_rsrc = buf_rsrc(XINo + ((int64_t)t0 * R + r) * I);   // wave-uniform
#pragma unroll
    for (int s = 0; s < NG; ++s) {
      if (s < s0 || s >= s1) continue;
      const int gs = opaque(gsl[s]);
      const int i = (int)((uint32_t)gs >> 28), col = (gs >> 20) & 0xFF;
      const bool live = gs != -1, ok = live && t0 + i < Tp;   // (i >= 8 sets the sign bit: compare with -1)
      // a slot past the block writes the never-read pad column xin[0][FXP - 1] and drops its global store
      (&S.xin[0][0])[live ? i * FXP + col : FXP - 1] = ok ? xr[s] : 0.0f;
      if (online) buf_st(xr_rsrc, ok ? ((uint32_t)i * RI + col) * 4 : kDrop, xr[s]);
    }
    // actions_onehot[t-1] is zero unless slot t-1 was filled (runner contract)
    if (s1 == NG && ptid < FCH) {
      const int t = t0 + ptid;
      S.aprev[ptid] = (d.last_action && t > 0 && t < Tp && f_ld) ? a_ld : -1;
    }
  };
  auto onehots = [&](int cc) {
    const int t0 = FCH * cc, wd = I - O, i = ptid >> 4, t = t0 + i;
    const auto xo = buf_rsrc(XINo + ((int64_t)t0 * R + r) * I + O);   // wave-uniform
    const uint32_t ro = (uint32_t)i * RI;
    for (int col = ptid & 15; col < wd; col += 16) {
      float v;
      if (d.last_action && col < A) v = col == S.aprev[i] ? 1.0f : 0.0f;
      else v = (col - (d.last_action ? A : 0)) == ag ? 1.0f : 0.0f;
      S.xin[i][O + col] = v;
      if (online) buf_st(xo, t < Tp ? (ro + col) * 4 : kDrop, v);   // rows past Tp drop
    }
  };
  f32x4 acc1 = {0, 0, 0, 0}, acc1b = {0, 0, 0, 0}, accg[3] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
  auto fc1_part = [&](int m0, int m1) {   // b128 groups [m0, m1) of this lane group's Kq k-blocks
#pragma unroll
    for (int m = m0; m < m1; ++m) {
      if (4 * m >= Kq) break;
      const f32x4 av = *(const f32x4*)&S.xin[c16][g * Kq + 4 * m];
      const f32x4 bv = *(const f32x4*)&S.w1[16 * wv + c16][g * Kq + 4 * m];
      acc1 = mfma16x4(av[0], bv[0], acc1);
      acc1b = mfma16x4(av[1], bv[1], acc1b);
      acc1 = mfma16x4(av[2], bv[2], acc1);
      acc1b = mfma16x4(av[3], bv[3], acc1b);
    }
  };
  auto fc1_epi = [&](int cc) {
    const int t0 = FCH * cc;
    const auto xb = buf_rsrc(X1o + ((int64_t)t0 * R + r) * H);   // wave-uniform
    const uint32_t lo = (uint32_t)(4 * g) * RH + 16 * wv + c16;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int i = 4 * g + e, t = t0 + i;
      const float x = fmaxf((acc1[e] + acc1b[e]) + b1, 0.0f);
      S.x1[i][16 * wv + c16] = x;
      if (online) buf_st(xb, t < Tp ? (lo + e * RH) * 4 : kDrop, x);
    }
    acc1 = f32x4{0, 0, 0, 0};
    acc1b = f32x4{0, 0, 0, 0};
  };
  auto gi_part = [&](int k0, int k1) {    // k-blocks [k0, k1) of this lane group's 16
#pragma unroll
    for (int kb = k0; kb < k1; ++kb) {
      const float av = S.x1[c16][16 * g + kb];
#pragma unroll
      for (int s = 0; s < 3; ++s) accg[s] = mfma16x4(av, wih[s][kb], accg[s]);
    }
  };
  auto gi_epi = [&](int cc) {
#pragma unroll
    for (int s = 0; s < 3; ++s) {
#pragma unroll
      for (int e = 0; e < 4; ++e) S.gi[cc & 1][4 * g + e][16 * (3 * wv + s) + c16] = accg[s][e] + bih[s];
      accg[s] = f32x4{0, 0, 0, 0};
    }
  };
  // fc2 of a chunk in two steps: every producer wave multiplies its 16-wide K quarter (4 MFMAs) into a partial
  // tile in LDS (aliasing x1, idle at p = 0, 1); wave 0 sums the four partials and stores Q.
  float(*qpart)[FCH][16] = (float(*)[FCH][16])&S.x1[0][0];   // [4 waves][16 steps][16 actions]
  auto fc2_partial = [&](int cc) {
    f32x4 acc2 = {0, 0, 0, 0};
    const f32x4 av = *(const f32x4*)&S.hs[cc & 1][c16][16 * wv + 4 * g];
    const f32x4 bv = *(const f32x4*)&S.w2[c16][16 * wv + 4 * g];
#pragma unroll
    for (int e = 0; e < 4; ++e) acc2 = mfma16x4(av[e], bv[e], acc2);
#pragma unroll
    for (int e = 0; e < 4; ++e) qpart[wv][4 * g + e][c16] = acc2[e];
  };
  auto fc2_store = [&](int cc) {
    if (wv != 0) return;
    const int t0 = FCH * cc;
    const auto qb = buf_rsrc(Qz + ((int64_t)t0 * R + r) * A);   // wave-uniform
    const uint32_t lo = (uint32_t)(4 * g) * RA + c16;
    float v[4];   // every LDS read first, then the stores
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int i = 4 * g + e;
      v[e] = ((qpart[0][i][c16] + qpart[1][i][c16]) + (qpart[2][i][c16] + qpart[3][i][c16])) + b2;
    }
#pragma unroll
    for (int e = 0; e < 4; ++e)
      buf_st(qb, (t0 + 4 * g + e < Tp && c16 < A) ? (lo + e * RA) * 4 : kDrop, v[e]);
  };

  // chunk 0 synchronously (5 barriers, matched by the recurrence waves)
  drain_vmem();   // chunk 0's gather (issued before the weight loads)
  lds_barrier();   // 1: weights, padding staged
  store_gather(0);
  lds_barrier();   // 2
  onehots(0);
  lds_barrier();   // 3
  fc1_part(0, FKQ / 4);
  fc1_epi(0);
  lds_barrier();   // 4
  gi_part(0, 16);
  gi_epi(0);
  lds_barrier();   // 5

  for (int c = 0; c <= cl; ++c) {
    const int t0 = FCH * c;
    const bool next = c + 1 <= cl;
#pragma unroll
    for (int p = 0; p < FCH; ++p) {
      if (t0 + p >= Tp) continue;   // last chunk: no work past Tp (no work for chunk c+1 either)
      if (p == 0) {
        if (c >= 1) fc2_partial(c - 1);
        if (next) issue_gather(c + 1);
      }
      if (p == 1 && c >= 1) fc2_store(c - 1);
      if (next) {
        if (p == 5) store_gather(c + 1);
        if (p == 6) onehots(c + 1);
        if (p == 7) fc1_part(0, 2);
        if (p == 8) fc1_part(2, 4);
        if (p == 9) fc1_part(4, 6);
        if (p == 10) { fc1_part(6, 8); fc1_epi(c + 1); }
        if (p == 11) gi_part(0, 4);
        if (p == 12) gi_part(4, 7);
        if (p == 13) gi_part(7, 10);
        if (p == 14) gi_part(10, 13);
        if (p == 15) { gi_part(13, 16); gi_epi(c + 1); }
      }
      lds_barrier();
    }
  }
  // the last chunk (and the previous one's store when the last chunk is a single step) after the final barrier,
  // in wave 0 alone
  if (cl >= 1 && Tp - FCH * cl < 2) fc2_store(cl - 1);
  if (wv == 0) {
    f32x4 q0 = {0, 0, 0, 0}, q1 = {0, 0, 0, 0};
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const f32x4 av = *(const f32x4*)&S.hs[cl & 1][c16][16 * g + 4 * m];
      const f32x4 bv = *(const f32x4*)&S.w2[c16][16 * g + 4 * m];
      q0 = mfma16x4(av[0], bv[0], q0);
      q1 = mfma16x4(av[1], bv[1], q1);
      q0 = mfma16x4(av[2], bv[2], q0);
      q1 = mfma16x4(av[3], bv[3], q1);
    }
    const int t0 = FCH * cl;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int t = t0 + 4 * g + e;
      if (t < Tp && c16 < A) Qz[((int64_t)t * R + r) * A + c16] = (q0[e] + q1[e]) + b2;
    }
  }
}

// Host: the fused forward with the smallest gather-slot instantiation that covers O.
inline void launch_fwd_fused(dim3 grid, hipStream_t s, const Dims& d, const Rep& rp, const float* P0, const float* P1,
                             const Lay& L, const Work& w) {
  if (FCH * d.O <= 256 * 5)
    hipLaunchKernelGGL((gru_fwd_fused_kernel<5>), grid, dim3(512), 0, s, d, rp, P0, P1, L, w);
  else
    hipLaunchKernelGGL((gru_fwd_fused_kernel<FGATHER>), grid, dim3(512), 0, s, d, rp, P0, P1, L, w);
}
// The production forward with the QMIX hypernet's workgroups appended (HYP = 1; the caller checked hyf_ok).
inline void launch_fwd_fused_hyp(hipStream_t s, const Dims& d, const Rep& rp, const float* P0, const float* P1,
                                 const Lay& L, const Work& w) {
  const dim3 grid(2 * d.R + 2 * ((d.M + 31) / 32));
  if (FCH * d.O <= 256 * 5)
    hipLaunchKernelGGL((gru_fwd_fused_kernel<5, 1>), grid, dim3(512), 0, s, d, rp, P0, P1, L, w);
  else
    hipLaunchKernelGGL((gru_fwd_fused_kernel<FGATHER, 1>), grid, dim3(512), 0, s, d, rp, P0, P1, L, w);
}

}  // namespace mq
