// Row-tile agent forward and BPTT for large batches (BASELINE configs[2]: B = 128 episodes x n = 27 agents =
// 3,456 rows, T + 1 = 181 steps, I = 348 agent inputs, A = 36 actions): the throughput regime, where the learner
// is MFMA-bound rather than latency-bound, so the recurrence itself goes on the matrix cores and every activation
// that the row-parallel GEMM path round-trips through HBM (GI, dGI, dX1, XIN) stays on chip.
//
// rnn_agent.py:27-36 (fc1 -> relu -> GRUCell -> fc2) and its backward (q_learner.py:100-101), per workgroup of rows:
//
// Forward, gru_fwd_tile_kernel: one workgroup = 32 rows (two 16-row MFMA M-tiles) of one net, 512 threads in two
// roles (recurrence waves 0-3, projection waves 4-7). Waves w and w + 4 own hidden units 16 (w & 3) .. + 15: the
// N-tile of fc1 and fc2 and the gate columns {w, 4 + w, 8 + w} (r, z, n of its units) of the two 192-wide products,
// so the GRU gate math is lane-local. Per step t, one LDS barrier, and the step's work is software-pipelined across
// steps:
//   GH_t  = h_{t-1} W_hh^T              [32 x 64] x [64 x 192]   (the serial part)
//   gates -> h_t (LDS, + Hs / Gates for the BPTT when online; the tile path's Gates record is [RT][H][4] =
//   (r, z, n, W_hn h + b_hn) per unit, one 16-byte store / load per (row, unit))
//   GI_{t+1} = X1_{t+1} W_ih^T + b_ih    [32 x 64] x [64 x 192]   (registers until step t + 1)
//   X1_{t+2} = relu(obs_{t+2} W1_obs^T + W1[:, O + a_{t+1}] + W1[:, O + A + agent] + b1)   [32 x O] x [O x 64]
//   Q_{t-1} = h_{t-1} W2^T + b2           [32 x 64] x [64 x A]
// with the obs rows of step t + 4 loaded from the replay (wave-uniform row bases) while step t computes. The weight
// B-fragments (W_hh, W_ih, W1's obs part, W2) stay in VGPRs for the whole T loop; the one-hot columns of W1 are
// gathered from LDS. v_mfma_f32_16x16x4_f32 throughout (fp32 in, fp32 accumulate: the reference's arithmetic).
//
// Backward, gru_bwd_split_kernel (online net): one workgroup = 16 rows, 512 threads in two roles (chain and
// weight-gradient waves); waves w and w + 4 own units 16 (w & 3) .. + 15. Per step t (descending), two LDS barriers:
//   dh = carry + dchosen W2[a_t];  dgi, dgh from the stored gates (lane-local, as the forward's gate math)
//   carry_{t-1} = dh z + dgh W_hh         [16 x 192] x [192 x 64]
//   dX1 = (dgi W_ih) o [X1 > 0]           [16 x 192] x [192 x 64]
//   dW_hh += dgh^T h_{t-1}, dW_ih += dgi^T X1      [192 x 16] x [16 x 64]
//   dW1 += dX1^T xin_t  (xin rebuilt from the replay rows: obs | onehot(a_{t-1}) | onehot(agent))   [64 x 16] x [16 x I]
//   dW2 += onehot(a_t)^T (dchosen h_t)    [A x 16] x [16 x 64]
// The weight gradients accumulate in MFMA C registers for the whole T loop and leave as one slab per workgroup
// (slab_rnn / slab_fc1 in parameter layout), summed in fixed order by the learner's two-pass reduction: the step is
// deterministic.
//
// MFMA operand maps (v_mfma_f32_16x16x4_f32, lane l, g = l >> 4, c = l & 15): A[i = c][kk = g], B[kk = g][j = c],
// D[i = 4g + e][j = c]. Where K is a feature dimension, lane group g owns a contiguous quarter of it (k = Kq g + s),
// so A and B fragments are b128 reads; where K is the 16 rows of a tile, lane group g takes rows 4 g .. 4 g + 3
// (k = 4 g + s: with the tiles' row pitches = 4 mod 64 banks, the 64 lanes' scalar operand reads hit 64 banks).
#pragma once
#include "gru_kernels.hpp"
#include "gru_fwd_fused.hpp"

namespace mq {

constexpr int TR_F = 32;   // rows per forward workgroup (two M-tiles)
constexpr int TR_B = 16;   // rows per backward workgroup
constexpr int T_HP = H + 4;   // LDS row pitch of 64-wide tiles

// Shape limits of the row-tile path: O <= 4 * KQ1 <= 320 (KQ1 = k-steps per lane group of fc1's obs part),
// A <= 48 (three 16-wide action tiles), I <= 384 (dW1's 24 column tiles), one-hot columns <= 128.
constexpr int T_KQ1_MAX = 80;
constexpr int T_NI = 24;
inline int tile_kq1(int O) {
  const int k = (O + 15) / 16 * 4;
  return k <= 8 ? 8 : k <= 20 ? 20 : k <= 40 ? 40 : k <= 72 ? 72 : k <= 80 ? 80 : -1;
}
constexpr int T_TMAX = 512;   // steps (t_len) the forward's per-step one-hot table holds
constexpr int T_NOH = 80;     // one-hot columns (last action + agent id) of W1 staged in LDS
inline bool tiles_ok(int I, int O, int A, int n, int Tp, int64_t RT) {
  // RT * H * 4 bytes: the Hs stores go through one buffer descriptor (num_records 0x7FFFFFF0) with byte offsets up
  // to RT * H * 4, so a larger batch would have its stores past 2 GiB dropped by the range check
  return tile_kq1(O) > 0 && A <= 48 && I <= 16 * T_NI && I - O <= T_NOH && Tp <= T_TMAX && n * O < (1 << 24) &&
         RT * G3 < (int64_t(1) << 31) && RT * H * 4 < int64_t(0x7FFFFFF0);
}

template <int KQ1>
struct alignas(16) FwdTileLds {
  float xo[2][TR_F][4 * KQ1 + 4];   // obs rows of steps t + 2 / t + 3 (zero past O)
  float hb[2][TR_F][T_HP];          // h_{t-1} / h_t
  float x1[2][TR_F][T_HP];          // X1 of steps t + 1 / t + 2
  float w1oh[T_NOH][H];             // W1's one-hot columns, [column - O][unit]
  int8_t ap[T_TMAX][TR_F];          // a_{t-1} of every step and row (-1: zero one-hot), built in the prologue
  int agent[TR_F];                  // agent index of each row (the agent-id one-hot)
};

// grid = 16 ceil(ceil(R / 32) / 8) (row tiles x 2 nets, XCD-paired), 512 threads: two waves per SIMD with split
// roles. Waves 0-3 run the recurrence (GH, the gate math, GI; W_hh and W_ih in registers), waves 4-7 the projections
// (fc1 with the obs staging, fc2; W1's obs part and W2 in registers). Wave w and wave w + 4 share a SIMD and own the
// same 16 units, so each SIMD interleaves a recurrence stream (192 MFMAs a step) with a projection stream (176): one
// wave's LDS and MFMA latencies are covered by the other's issue, and neither wave has to hold the other's 88-96
// weight registers. Each role is its own T loop; both pass the same barriers (one per step).
template <int KQ1>
__global__ __launch_bounds__(512, 1) void gru_fwd_tile_kernel(Dims d, Rep rp, const float* __restrict__ P0,
                                                              const float* __restrict__ P1, Lay L, Work w) {
  __shared__ FwdTileLds<KQ1> S;
  constexpr int NS = (4 * KQ1 + 63) / 64;   // obs gather slots per lane and row
  // 1-D grid in groups of 16: block 16 k + 8 n + i is row tile 8 k + i of net n, so the two nets' workgroups of a
  // row tile are blocks b and b + 8, which the dispatcher deals to the same XCD: the second net's obs gather hits the
  // L2 lines the first net's brought in
  const int nx = (d.R + TR_F - 1) / TR_F;
  const int xt = 8 * (blockIdx.x >> 4) + (blockIdx.x & 7);
  if (xt >= nx) return;
  const int z = (blockIdx.x >> 3) & 1;
  const bool online = z == 0;
  const float* __restrict__ P = z ? P1 : P0;
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, c = lane & 15;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ub = wv & 3;   // this wave's unit block
  const int R = d.R, Tp = d.Tp, O = d.O, A = d.A, n = d.n, I = d.I;
  const int r0 = xt * TR_F;
  const int j = 16 * ub + c;   // this lane's hidden unit in the D layout
  const uint32_t RH = (uint32_t)R * H;

  const int noh = I - O;   // one-hot columns (last action, agent id)
  for (int e = tid; e < noh * H; e += 512) {
    const int col = e / H, u = e - col * H;
    S.w1oh[col][u] = P[L.o[MQ_P_FC1_W] + (int64_t)u * I + O + col];
  }
  for (int e = tid; e < TR_F * T_HP; e += 512) (&S.hb[1][0][0])[e] = 0.0f;   // h_{-1} = 0 (init_hidden)
  if (tid < TR_F) {
    const int r = min(r0 + tid, R - 1);
    S.agent[tid] = r - (int)fdiv((uint32_t)r, d.dN) * n;
  }
  // the last-action one-hot of every (step, row): a_{t-1} when t > 0 and slot t - 1 was filled (runner contract),
  // so the T loop issues no small dependent loads
  for (int e = tid; e < Tp * TR_F; e += 512) {
    const int t = e / TR_F, i = e - t * TR_F;
    const int r = min(r0 + i, R - 1);
    const int b = (int)fdiv((uint32_t)r, d.dN), ag = r - b * n;
    const int64_t slot = rp.ep(b) * d.t_stride + max(t - 1, 0);
    int a = -1;
    if (d.last_action && t > 0 && *(const int*)(rp.filled + slot)) a = *(const int*)(rp.actions + slot * n + ag);
    S.ap[t][i] = (int8_t)a;
  }

  if (wv < 4) {
    // ================================================================ recurrence waves
    f32x4 whh[3][4], wih[3][4];   // [gate][b128 group]: W[gate * 64 + j][16 g + 4 q + e]
    {
      const float* Wh = P + L.o[MQ_P_RNN_W_HH];
      const float* Wi = P + L.o[MQ_P_RNN_W_IH];
#pragma unroll
      for (int gt = 0; gt < 3; ++gt)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          whh[gt][q] = *(const f32x4*)(Wh + (int64_t)(gt * H + j) * H + 16 * g + 4 * q);
          wih[gt][q] = *(const f32x4*)(Wi + (int64_t)(gt * H + j) * H + 16 * g + 4 * q);
        }
    }
    const float bi[3] = {P[L.o[MQ_P_RNN_B_IH] + j], P[L.o[MQ_P_RNN_B_IH] + H + j], P[L.o[MQ_P_RNN_B_IH] + 2 * H + j]};
    const float bh[3] = {P[L.o[MQ_P_RNN_B_HH] + j], P[L.o[MQ_P_RNN_B_HH] + H + j], P[L.o[MQ_P_RNN_B_HH] + 2 * H + j]};
    // the 192-wide product of a 32 x 64 LDS tile with a register-resident weight (A fragments read up front); the
    // accumulators start at the bias (this lane's unit column), as addmm's beta * bias + x W^T does
    auto prod3 = [&](const float (*tile)[T_HP], const f32x4 (&wt)[3][4], const float (&bias)[3],
                     f32x4 (&out)[2][3]) {
      f32x4 av[2][4];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int q = 0; q < 4; ++q) av[mt][q] = *(const f32x4*)(&tile[16 * mt + c][16 * g + 4 * q]);
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
#pragma unroll
        for (int gt = 0; gt < 3; ++gt) out[mt][gt] = f32x4{bias[gt], bias[gt], bias[gt], bias[gt]};
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int gt = 0; gt < 3; ++gt) out[mt][gt] = mfma16x4(av[mt][q][e], wt[gt][q][e], out[mt][gt]);
      }
    };
    lds_barrier();   // #1: tables, h_{-1}; X1 tiles being built by the projection waves
    lds_barrier();   // #2: X1 of steps 0 and 1
    f32x4 gi[2][3];
    prod3(S.x1[0], wih, bi, gi);   // GI_0 = X1_0 W_ih^T + b_ih
    lds_barrier();   // #3
    float hprev[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
    const auto hsb = buf_rsrc(w.Hs);
    // one step: the input gates of step t in gi_t (registers), those of step t + 1 into gi_n. The loop runs two steps
    // per iteration with the two sets swapping roles, so no register copy carries GI across the back edge.
    auto step = [&](int t, const f32x4 (&gi_t)[2][3], f32x4 (&gi_n)[2][3]) {
      // GH_t = h_{t-1} W_hh^T + b_hh
      f32x4 gh[2][3];
      prod3(S.hb[(t + 1) & 1], whh, bh, gh);
      // gates -> h_t (ATen gru_cell order: r, z from (W_h h + b_h) + gi; n = tanh(gi_n + r (W_hn h + b_hn));
      // h = (h_{t-1} - n) z + n)
      const auto gb = buf_rsrc(w.Gates + (int64_t)t * (4 * RH));
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int i = 16 * mt + 4 * g + e, r = r0 + i;
          const float rg = sigm_fast(gh[mt][0][e] + gi_t[mt][0][e]);
          const float zg = sigm_fast(gh[mt][1][e] + gi_t[mt][1][e]);
          const float ghn = gh[mt][2][e];
          const float ng = tanh_fast(gi_t[mt][2][e] + ghn * rg);
          const float h1 = (hprev[mt][e] - ng) * zg + ng;
          hprev[mt][e] = h1;
          S.hb[t & 1][i][j] = h1;
          const bool st = online && r < R;
          buf_st(hsb, st ? (((uint32_t)t * R + r) * H + j) * 4 : kDrop, h1);
          buf_st4(gb, st ? ((uint32_t)r * H + j) * 16 : kDrop, f32x4{rg, zg, ng, ghn});
        }
      // GI of step t + 1 = X1_{t+1} W_ih^T + b_ih (X1_{t+1}: built by the projection waves in step t - 1)
      prod3(S.x1[(t + 1) & 1], wih, bi, gi_n);
      lds_barrier();
    };
    f32x4 gi2[2][3];
    int t = 0;
    for (; t + 1 < Tp; t += 2) {
      step(t, gi, gi2);
      step(t + 1, gi2, gi);
    }
    if (t < Tp) step(t, gi, gi2);
  } else {
    // ================================================================ projection waves
    float w1[KQ1];   // W1[j][KQ1 g + s] (obs part; zero past O)
    {
      const float* W1 = P + L.o[MQ_P_FC1_W] + (int64_t)j * I;
#pragma unroll
      for (int s = 0; s < KQ1; ++s) {
        const int k = KQ1 * g + s;
        w1[s] = W1[min(k, O - 1)];
        if (k >= O) w1[s] = 0.0f;
      }
    }
    f32x4 w2[4];   // W2[16 ub + c][16 g + 4 q + e] (zero past A)
    {
      const int a = min(j, A - 1);
      const float* W2 = P + L.o[MQ_P_FC2_W] + (int64_t)a * H;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x4 v = *(const f32x4*)(W2 + 16 * g + 4 * q);
        w2[q] = j < A ? v : f32x4{0, 0, 0, 0};
      }
    }
    const float b1 = P[L.o[MQ_P_FC1_B] + j];
    const float b2 = j < A ? P[L.o[MQ_P_FC2_B] + j] : 0.0f;
    const int nO = n * O;
    // ---- obs gather: wave ub stages rows 8 ub .. 8 ub + 7 (wave-uniform row bases), lane l columns l + 64 s
    const float* rowb[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r = min(r0 + 8 * ub + i, R - 1);
      const int b = (int)fdiv((uint32_t)r, d.dN), ag = r - b * n;
      const uint64_t pa = (uint64_t)(uintptr_t)(rp.obs + (rp.ep(b) * d.t_stride * n + ag) * (int64_t)O);
      const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)pa), hi = __builtin_amdgcn_readfirstlane((uint32_t)(pa >> 32));
      rowb[i] = (const float*)(uintptr_t)(((uint64_t)hi << 32) | lo);   // wave-uniform: a descriptor base below
    }
    // the obs rows go through one buffer descriptor per row and step (SGPR base, O floats long): columns past O
    // read 0 from the range check, so neither a clamp nor a select per element is needed
    float xr[8][NS];
    auto issue_obs = [&](int t) {
      t = __builtin_amdgcn_readfirstlane(t);   // uniform already; said so, or hipcc keeps t in a VGPR here
      const int tc = min(t, Tp - 1);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const auto ors = __builtin_amdgcn_make_buffer_rsrc((void*)(rowb[i] + (int64_t)tc * nO), (short)0, O * 4,
                                                           0x00020000);
#pragma unroll
        for (int s = 0; s < NS; ++s)
          xr[i][s] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ors, (lane + 64 * s) * 4, 0, 0));
      }
    };
    auto stage_obs = [&](int t) {
      const int buf = t & 1;
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          const int col = lane + 64 * s;
          if (col < 4 * KQ1) S.xo[buf][8 * ub + i][col] = xr[i][s];
        }
    };
    // the agent-id one-hot term of this lane's 8 (row, unit) pairs (constant over t; read once the table is up)
    float agt[2][4];
    // fc1 of step tt (obs in xo[tt & 1]) -> X1 (LDS x1[tt & 1]; HBM when online)
    auto fc1 = [&](int tt) {
      const int buf = tt & 1;
      const int tcl = min(tt, Tp - 1);
      // a_{tt-1} of rows 16 mt + 4 g .. + 3 (four int8 in one word) and their W1 one-hot columns, read ahead
      uint32_t apw[2];
      float oh[2][4];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        apw[mt] = *(const uint32_t*)&S.ap[tcl][16 * mt + 4 * g];
#pragma unroll
        for (int e = 0; e < 4; ++e) oh[mt][e] = S.w1oh[max((int)(int8_t)(apw[mt] >> (8 * e)), 0)][j];
      }
      // both M-tiles together, the A fragments read in blocks of QB b128 per tile ahead of their MFMAs
      constexpr int NQ = KQ1 / 4;
      constexpr int QB = NQ % 6 == 0 ? 6 : NQ % 5 == 0 ? 5 : 2;
      f32x4 acc[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}}, acc2[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
#pragma unroll
      for (int qb = 0; qb < NQ; qb += QB) {
        f32x4 av[2][QB];
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
          for (int u = 0; u < QB; ++u) av[mt][u] = *(const f32x4*)(&S.xo[buf][16 * mt + c][KQ1 * g + 4 * (qb + u)]);
#pragma unroll
        for (int u = 0; u < QB; ++u)
#pragma unroll
          for (int mt = 0; mt < 2; ++mt) {
            const int q = qb + u;
            acc[mt] = mfma16x4(av[mt][u][0], w1[4 * q], acc[mt]);
            acc2[mt] = mfma16x4(av[mt][u][1], w1[4 * q + 1], acc2[mt]);
            acc[mt] = mfma16x4(av[mt][u][2], w1[4 * q + 2], acc[mt]);
            acc2[mt] = mfma16x4(av[mt][u][3], w1[4 * q + 3], acc2[mt]);
          }
      }
      const auto xb = buf_rsrc(w.X1 + (int64_t)tt * RH);
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int i = 16 * mt + 4 * g + e, r = r0 + i;
          float v = acc[mt][e] + acc2[mt][e];
          if ((int8_t)(apw[mt] >> (8 * e)) >= 0) v += oh[mt][e];
          if (d.agent_id) v += agt[mt][e];
          const float x = fmaxf(v + b1, 0.0f);
          S.x1[buf][i][j] = x;
          buf_st(xb, (online && r < R && tt < Tp) ? ((uint32_t)r * H + j) * 4 : kDrop, x);
        }
      }
    };
    // Q of step tt (h_tt in hb[tt & 1])
    const uint32_t RA = (uint32_t)R * A;
    float* Qz = w.Q + (int64_t)z * d.RT() * A;
    auto fc2 = [&](int tt) {
      const int buf = tt & 1;
      const auto qb = buf_rsrc(Qz + (int64_t)max(tt, 0) * RA);
      f32x4 av[2][4];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int q = 0; q < 4; ++q) av[mt][q] = *(const f32x4*)(&S.hb[buf][16 * mt + c][16 * g + 4 * q]);
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        f32x4 acc = {0, 0, 0, 0};
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int e = 0; e < 4; ++e) acc = mfma16x4(av[mt][q][e], w2[q][e], acc);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r = r0 + 16 * mt + 4 * g + e;
          buf_st(qb, (tt >= 0 && r < R && j < A) ? ((uint32_t)r * A + j) * 4 : kDrop, acc[e] + b2);
        }
      }
    };

    // ---- prologue: X1 of steps 0 and 1, obs of step 2 staged and step 3's in flight
    issue_obs(0);
    drain_vmem();
    stage_obs(0);
    issue_obs(1);
    drain_vmem();
    stage_obs(1);
    lds_barrier();   // #1
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        agt[mt][e] = d.agent_id ? S.w1oh[(d.last_action ? A : 0) + S.agent[16 * mt + 4 * g + e]][j] : 0.0f;
    fc1(0);
    fc1(1);
    issue_obs(2);
    drain_vmem();
    lds_barrier();   // #2
    stage_obs(2);    // xo[0]: fc1(0) has read it
    issue_obs(3);
    lds_barrier();   // #3
    // the projection waves (the younger half) at priority 1: they otherwise lose every issue arbitration to the
    // recurrence waves, and the step waits on their fc1 (r04r: forward 1.33 -> 1.28 ms; the BPTT's weight-gradient
    // waves measured slower with it)
    __builtin_amdgcn_s_setprio(1);
    for (int t = 0; t < Tp; ++t) {
      // obs of step t + 3 into xo[(t + 3) & 1] (fc1(t + 1) read it in step t - 1), then step t + 4's loads
      stage_obs(t + 3);
      issue_obs(t + 4);
      fc2(t - 1);      // h_{t-1}: hb[(t + 1) & 1], read alongside the recurrence's GH
      fc1(t + 2);      // X1_{t+2} -> x1[t & 1] (its GI is step t + 1's)
      lds_barrier();
    }
    fc2(Tp - 1);
  }
}

// ------------------------------------------------------------------------------------------------ backward
template <int KQ1>
struct alignas(16) BwdTileLds {
  float dgh[TR_B][G3 + 4];        // the step's dgh = [da_r | da_z | da_n r]
  float dgi[TR_B][G3 + 4];        // the step's dgi = [da_r | da_z | da_n]
  float hb[3][TR_B][T_HP];        // h_tau in hb[tau % 3]: h_{t-1} (dW_hh) and h_t (dW2) of step t
  float x1[TR_B][T_HP];           // X1_t (dW_ih)
  float dx1[TR_B][T_HP];          // dX1_t (dW1)
  float xin[2][TR_B][16 * T_NI + 4];   // agent inputs of step t: obs | onehot(a_{t-1}) | onehot(agent), zero past I
  float w2[48][H];                // W2 (dh's dchosen term)
  // per-row streams of step t in ring slot t & 3, stored one step ahead: a_{t-1} (-1: zero one-hot), dchosen
  // (0 at t = T and past R), a_t
  int ap[4][TR_B];
  float dchs[4][TR_B];
  int acts[4][TR_B];
  int agent[TR_B];
};

// grid = ceil(R / 16), 512 threads. slab_len / slab1_len: per-workgroup slab strides (len_rnn, H * I + H).
// Two waves per SIMD with split roles, both on units 16 ub .. 16 ub + 15 (ub = wave & 3), two barriers a step:
//   chain waves 0-3:   stage, dh and the gate derivatives | B1 | carry              | B2 | dW1 column tiles [0, 12)
//   weight waves 4-7:                                      | B1 | dX1, dW_hh, dW_ih | B2 | dW1 tiles [12, NI), dW2
// (96 / 196 MFMAs a step at cfg3's shape). The serial chain's LDS and MFMA latencies are filled by the weight
// waves' work on the same SIMD, and each role holds only its own weights, accumulators and prefetches (the chain:
// W_hh and the next step's gate / h / X1 / obs loads; the weight waves: W_ih and 100 accumulators), which is what
// fits two roles in 2 x 256 registers (one role per wave needed 480 registers in one wave per SIMD: 1.99 ms
// against 1.27 ms at cfg3; that variant was removed in round 5).
constexpr int T_NIC = 12;               // dW1 column tiles of the chain waves
constexpr int T_NIW = T_NI - T_NIC;     // of the weight waves
template <int KQ1>
__global__ __launch_bounds__(512, 1) void gru_bwd_split_kernel(Dims d, Rep rp, const float* __restrict__ P, Lay L,
                                                               Work w, int64_t slab_len, int64_t slab1_len) {
  __shared__ BwdTileLds<KQ1> S;
  constexpr int NS = (4 * KQ1 + 63) / 64;
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, c = lane & 15;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ub = wv & 3;
  const int R = d.R, Tp = d.Tp, T = d.T, O = d.O, A = d.A, n = d.n, I = d.I;
  const int NI = (I + 15) / 16;
  const int r0 = blockIdx.x * TR_B;
  const int j = 16 * ub + c;
  const uint32_t RH = (uint32_t)R * H;
  auto row_of = [&](int i) { return min(r0 + i, R - 1); };

  for (int e = tid; e < 48 * H; e += 512) (&S.w2[0][0])[e] = e < A * H ? P[L.o[MQ_P_FC2_W] + e] : 0.0f;
  for (int e = tid; e < 3 * TR_B * T_HP; e += 512) (&S.hb[0][0][0])[e] = 0.0f;
  for (int e = tid; e < 2 * TR_B * (16 * T_NI + 4); e += 512) (&S.xin[0][0][0])[e] = 0.0f;
  if (tid < TR_B) {
    const int r = row_of(tid);
    S.agent[tid] = r - (int)fdiv((uint32_t)r, d.dN) * n;
  }

  const int64_t base = L.o[MQ_P_RNN_W_IH];
  float* slab = w.slab_rnn + (int64_t)blockIdx.x * slab_len;
  float* slab1 = w.slab_fc1 + (int64_t)blockIdx.x * slab1_len;
  const int64_t o_hh = L.o[MQ_P_RNN_W_HH] - base, o_bi = L.o[MQ_P_RNN_B_IH] - base,
                o_bh = L.o[MQ_P_RNN_B_HH] - base, o_w2 = L.o[MQ_P_FC2_W] - base, o_b2 = L.o[MQ_P_FC2_B] - base;
  // bias gradients: a lane's partials cover rows 4 g .. 4 g + 3 (db2 too); sum the four lane groups
  auto gsum = [](float v) {
    v += __shfl_xor(v, 16, 64);
    return v + __shfl_xor(v, 32, 64);
  };
  // dW1 += dX1^T xin_t over column tiles q0 + [0, NQ) below q1, in pairs (a pair starting past NI is skipped; a
  // pair's second tile past NI is computed and never written out) (K = the 16 rows, k = 4 g + s)
  auto dw1_tiles = [&](int t, auto& acc, int q0, int q1) {
    constexpr int NQ = sizeof(acc) / sizeof(acc[0]);
    const float(*xi)[16 * T_NI + 4] = S.xin[t & 1];
    float av[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) av[s] = S.dx1[4 * g + s][j];
#pragma unroll
    for (int qp = 0; qp < NQ; qp += 2) {
      if (q0 + qp < q1) {
        float bv[4][2];
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int u = 0; u < 2; ++u) bv[s][u] = xi[4 * g + s][16 * (q0 + qp + u) + c];
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int u = 0; u < 2; ++u) acc[qp + u] = mfma16x4(av[s], bv[s][u], acc[qp + u]);
      }
    }
  };
  auto dw1_out = [&](const auto& acc, int q0, int q1) {
    constexpr int NQ = sizeof(acc) / sizeof(acc[0]);
#pragma unroll
    for (int q = 0; q < NQ; ++q)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int u = 16 * ub + 4 * g + e, col = 16 * (q0 + q) + c;
        if (q0 + q < q1 && col < I) slab1[(int64_t)u * I + col] = acc[q][e];
      }
  };

  if (wv < 4) {
    // ================================================================ chain waves
    // ---- W_hh as B fragments: W[48 g + s][j] (K = the 192 gate columns, contiguous quarter per lane group)
    float whh[48];
    {
      const float* Wh = P + L.o[MQ_P_RNN_W_HH];
#pragma unroll
      for (int s = 0; s < 48; ++s) whh[s] = Wh[(int64_t)(48 * g + s) * H + j];
    }
    // obs rows 4 ub + i (wave-uniform row bases, made provably uniform: they become buffer descriptors below)
    const int nO = n * O;
    const float* rowb[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = row_of(4 * ub + i);
      const int b = (int)fdiv((uint32_t)r, d.dN), ag = r - b * n;
      const uint64_t pa = (uint64_t)(uintptr_t)(rp.obs + (rp.ep(b) * d.t_stride * n + ag) * (int64_t)O);
      const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)pa), hi = __builtin_amdgcn_readfirstlane((uint32_t)(pa >> 32));
      rowb[i] = (const float*)(uintptr_t)(((uint64_t)hi << 32) | lo);
    }
    // lane tid < 16: row tid's action, filled and dchosen streams (staged into LDS per step)
    const int rl = row_of(tid & 15);
    const bool rl_live = r0 + (tid & 15) < R;
    const int bl = (int)fdiv((uint32_t)rl, d.dN);
    const int64_t* act_l = rp.actions + rp.ep(bl) * d.t_stride * n + (rl - bl * n);
    const int64_t* fil_l = rp.filled + rp.ep(bl) * d.t_stride;

    // ---- the prefetched inputs of one step: own (row, unit) pairs
    struct In {
      float gr[4], gz[4], gn[4], ghn[4];   // gates r, z, n and W_hn h + b_hn
      float hp[4], x1[4];                  // h_{t-1}, X1_t
      float ob[4][NS];                     // obs rows 4 ub + i, columns lane + 64 s
    };
    // tid < 16: the raw dchosen, a_t, filled[t-1] and a_{t-1} words of row tid for the step two ahead (the selects
    // wait for store_row, so no load result is consumed in the step that issues it)
    float dch_n = 0.0f;
    int act_n = 0, fil_n = 0, apv_n = 0, t_n = 0;
    // the loads go through buffer descriptors with a per-step SGPR base and per-lane byte offsets fixed for the
    // whole loop (no 64-bit address arithmetic on the chain waves' VALU, which f32 MFMA blocks)
    uint32_t off_rj[4], off_ob[NS];
#pragma unroll
    for (int e = 0; e < 4; ++e) off_rj[e] = ((uint32_t)row_of(4 * g + e) * H + j) * 4;
#pragma unroll
    for (int s = 0; s < NS; ++s) off_ob[s] = (uint32_t)min(lane + 64 * s, O - 1) * 4;
    auto fetch = [&](int t, In& x) {
      t = __builtin_amdgcn_readfirstlane(t);   // uniform already; said so, or hipcc keeps t in a VGPR here and
                                               // waterfall-loops every descriptor built from it
      const int tc = max(t, 0), tm = max(t - 1, 0);
      const auto grs = buf_rsrc(w.Gates + (int64_t)tc * (4 * RH));   // the tile path's [RT][H][4] gate record
      const auto hrs = buf_rsrc(w.Hs + (int64_t)tm * RH);
      const auto xrs = buf_rsrc(w.X1 + (int64_t)tc * RH);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const f32x4 gv = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(grs, 4 * off_rj[e], 0, 0));
        x.gr[e] = gv[0];
        x.gz[e] = gv[1];
        x.gn[e] = gv[2];
        x.ghn[e] = gv[3];
        x.hp[e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(hrs, off_rj[e], 0, 0));
        x.x1[e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xrs, off_rj[e], 0, 0));
      }
      // obs rows of step tc (registers until stage: an LDS-DMA here would make the compiler wait for it at every
      // later LDS read of the step)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const auto ors = buf_rsrc(rowb[i] + (int64_t)tc * nO);
#pragma unroll
        for (int s = 0; s < NS; ++s)
          x.ob[i][s] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ors, off_ob[s], 0, 0));
      }
    };
    // row tid's dchosen and a_t of step t, and a_{t-1} (when t > 0 and slot t - 1 was filled: the last-action
    // one-hot). Rows past R (a partial last tile) get dchosen = 0: their dh, gate derivatives and every gradient
    // contribution are then exactly 0; step T has no dchosen (q_learner.py:55 uses mac_out[:, :-1]).
    auto fetch_row = [&](int t) {
      const int tc = min(max(t, 0), Tp - 1), tp = max(tc - 1, 0);
      dch_n = ld_u32(w.dch + (int64_t)min(tc, T - 1) * R, (uint32_t)rl);
      act_n = *(const int*)(act_l + (int64_t)tc * n);
      fil_n = *(const int*)(fil_l + tp);
      apv_n = *(const int*)(act_l + (int64_t)tp * n);
      t_n = t;
    };
    auto store_row = [&](int t) {   // into the ring slot of step t (read during step t: two barriers later)
      const bool live = t_n >= 0 && t_n < Tp;
      S.dchs[t & 3][tid] = (rl_live && live && t_n < T) ? dch_n : 0.0f;
      S.acts[t & 3][tid] = act_n;
      S.ap[t & 3][tid] = (d.last_action && live && t_n > 0 && fil_n) ? apv_n : -1;
    };
    // stage step t's tiles: h_{t-1} -> hb[(t - 1) % 3], X1_t -> x1, the obs and one-hot columns of xin[t & 1]
    auto stage = [&](int t, const In& x) {
      drain_vmem();   // this wave's loads have landed
      const int hbuf = (t + 2) % 3;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int i = 4 * g + e;
        S.hb[hbuf][i][j] = t > 0 ? x.hp[e] : 0.0f;
        S.x1[i][j] = x.x1[e];
      }
      float(*xi)[16 * T_NI + 4] = S.xin[t & 1];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int s = 0; s < NS; ++s)
          if (lane + 64 * s < O) xi[4 * ub + i][lane + 64 * s] = x.ob[i][s];
      // the last-action one-hot of rows 4 ub .. 4 ub + 3: clear the one this buffer held two steps ago (a_{t+1}, still
      // in ring slot t + 2), set a_{t-1}'s (the agent-id ones were set in the prologue, the rest stays zero)
      if (d.last_action && lane < 4) {
        const int i = 4 * ub + lane;
        const int old = S.ap[(t + 2) & 3][i], now = S.ap[t & 3][i];
        if (old >= 0) xi[i][O + old] = 0.0f;
        if (now >= 0) xi[i][O + now] = 1.0f;
      }
    };

    f32x4 acc_w1[T_NIC];
#pragma unroll
    for (int q = 0; q < T_NIC; ++q) acc_w1[q] = f32x4{0, 0, 0, 0};
    float dbi[3] = {0, 0, 0}, dbh[3] = {0, 0, 0};
    float carry[4] = {0, 0, 0, 0};

    // ---- prologue: a_{t-1} of the two top steps into the ring, step Tp - 1's inputs in registers
    In cur;
    if (wv == 0) (&S.ap[0][0])[lane] = -1;   // the ring's a_{t-1} slots start empty (stage clears slot t + 2's)
    if (tid < TR_B) {
      fetch_row(Tp - 1);
      store_row(Tp - 1);
    }
    lds_barrier();   // the zeroed xin / hb and the ring before any stage writes
    if (d.agent_id && lane < 8) {   // the agent-id one-hots of this wave's rows, both buffers, for the whole loop
      const int i = 4 * ub + (lane & 3);
      S.xin[lane >> 2][i][O + (d.last_action ? A : 0) + S.agent[i]] = 1.0f;
    }
    if (tid < TR_B) fetch_row(Tp - 2);   // stored by the first iteration
    fetch(Tp - 1, cur);

    for (int t = Tp - 1; t >= 0; --t) {
      // P0: stage step t (its loads were issued during step t + 1)
      stage(t, cur);
      if (tid < TR_B) store_row(t - 1);   // fetched during step t + 1
      // P1: dh and the gate derivatives of this lane's own (row, unit) pairs
      float dh[4], zz[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int i = 4 * g + e;
        const float dchv = S.dchs[t & 3][i];
        const int a = min(max(S.acts[t & 3][i], 0), A - 1);
        dh[e] = carry[e] + dchv * S.w2[a][j];
        const float gr = cur.gr[e], gz = cur.gz[e], gn = cur.gn[e], ghn = cur.ghn[e];
        const float hp = t > 0 ? cur.hp[e] : 0.0f;
        const float dn = dh[e] * (1.0f - gz);
        const float dz = dh[e] * (hp - gn);
        const float dan = dn * (1.0f - gn * gn);
        const float dar = (dan * ghn) * (gr * (1.0f - gr));
        const float daz = dz * (gz * (1.0f - gz));
        S.dgi[i][j] = dar; S.dgi[i][H + j] = daz; S.dgi[i][2 * H + j] = dan;
        S.dgh[i][j] = dar; S.dgh[i][H + j] = daz; S.dgh[i][2 * H + j] = dan * gr;
        dbi[0] += dar; dbi[1] += daz; dbi[2] += dan;
        dbh[0] += dar; dbh[1] += daz; dbh[2] += dan * gr;
        zz[e] = gz;
      }
      lds_barrier();   // B1: dgi / dgh, h_{t-1}, X1, xin of step t
      // P2: the next step's loads, in flight under this step's MFMAs
      if (t > 0) fetch(t - 1, cur);
      if (tid < TR_B) fetch_row(t - 2);
      // P3: carry_{t-1} = dh z + dgh W_hh  (A fragments read in blocks ahead of their MFMAs)
      {
        const float* ah = &S.dgh[c][48 * g];
        f32x4 ca = {0, 0, 0, 0}, cb = {0, 0, 0, 0};
#pragma unroll
        for (int qb = 0; qb < 12; qb += 3) {
          f32x4 vh[3];
#pragma unroll
          for (int u = 0; u < 3; ++u) vh[u] = *(const f32x4*)(ah + 4 * (qb + u));
#pragma unroll
          for (int u = 0; u < 3; ++u) {
            const int q = qb + u;
            ca = mfma16x4(vh[u][0], whh[4 * q], ca);
            cb = mfma16x4(vh[u][1], whh[4 * q + 1], cb);
            ca = mfma16x4(vh[u][2], whh[4 * q + 2], ca);
            cb = mfma16x4(vh[u][3], whh[4 * q + 3], cb);
          }
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) carry[e] = dh[e] * zz[e] + (ca[e] + cb[e]);
      }
      lds_barrier();   // B2: dX1 of step t (weight waves)
      // P4: dW1 column tiles [0, T_NIC)
      dw1_tiles(t, acc_w1, 0, NI);
    }
    dw1_out(acc_w1, 0, NI);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const float si = gsum(dbi[k]), sh = gsum(dbh[k]);
      if (g == 0) { slab[o_bi + k * H + j] = si; slab[o_bh + k * H + j] = sh; }
    }
  } else {
    // ================================================================ weight-gradient waves
    f32x4 acc_hh[3][4], acc_ih[3][4], acc_w1[T_NIW], acc_w2[3];
#pragma unroll
    for (int m = 0; m < 3; ++m)
#pragma unroll
      for (int q = 0; q < 4; ++q) { acc_hh[m][q] = f32x4{0, 0, 0, 0}; acc_ih[m][q] = f32x4{0, 0, 0, 0}; }
#pragma unroll
    for (int q = 0; q < T_NIW; ++q) acc_w1[q] = f32x4{0, 0, 0, 0};
#pragma unroll
    for (int m = 0; m < 3; ++m) acc_w2[m] = f32x4{0, 0, 0, 0};
    float db2[3] = {0, 0, 0}, db1 = 0.0f;
    float wih[48];   // W_ih as B fragments, W[48 g + s][j]
    {
      const float* Wi = P + L.o[MQ_P_RNN_W_IH];
#pragma unroll
      for (int s = 0; s < 48; ++s) wih[s] = Wi[(int64_t)(48 * g + s) * H + j];
    }
    lds_barrier();   // the chain waves' prologue barrier
    for (int t = Tp - 1; t >= 0; --t) {
      lds_barrier();   // B1
      // dX1 = (dgi W_ih) o [X1 > 0]
      {
        const float* ai = &S.dgi[c][48 * g];
        f32x4 xa = {0, 0, 0, 0}, xb = {0, 0, 0, 0};
#pragma unroll
        for (int qb = 0; qb < 12; qb += 3) {
          f32x4 vi[3];
#pragma unroll
          for (int u = 0; u < 3; ++u) vi[u] = *(const f32x4*)(ai + 4 * (qb + u));
#pragma unroll
          for (int u = 0; u < 3; ++u) {
            const int q = qb + u;
            xa = mfma16x4(vi[u][0], wih[4 * q], xa);
            xb = mfma16x4(vi[u][1], wih[4 * q + 1], xb);
            xa = mfma16x4(vi[u][2], wih[4 * q + 2], xa);
            xb = mfma16x4(vi[u][3], wih[4 * q + 3], xb);
          }
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float v = S.x1[4 * g + e][j] > 0.0f ? xa[e] + xb[e] : 0.0f;   // relu'(X1_t)
          S.dx1[4 * g + e][j] = v;
          db1 += v;
        }
      }
      // dW_hh += dgh^T h_{t-1}, dW_ih += dgi^T X1 (K = the 16 rows, k = 4 g + s)
      {
        const int hbuf = (t + 2) % 3;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int row = 4 * g + s;
          float a_h[3], a_i[3], b_h[4], b_x[4];
#pragma unroll
          for (int m = 0; m < 3; ++m) {
            a_h[m] = S.dgh[row][16 * (4 * m + ub) + c];
            a_i[m] = S.dgi[row][16 * (4 * m + ub) + c];
          }
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            b_h[q] = S.hb[hbuf][row][16 * q + c];
            b_x[q] = S.x1[row][16 * q + c];
          }
#pragma unroll
          for (int m = 0; m < 3; ++m)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              acc_hh[m][q] = mfma16x4(a_h[m], b_h[q], acc_hh[m][q]);
              acc_ih[m][q] = mfma16x4(a_i[m], b_x[q], acc_ih[m][q]);
            }
        }
      }
      lds_barrier();   // B2
      // dW1 column tiles [T_NIC, NI);  dW2 += onehot(a_t)^T (dchosen h_t);  db2
      dw1_tiles(t, acc_w1, T_NIC, NI);
      {
        const int hbuf = t % 3;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int row = 4 * g + s;
          const float dchv = S.dchs[t & 3][row];
          const int aw = S.acts[t & 3][row];
          const float bv = S.hb[hbuf][row][j];
#pragma unroll
          for (int m = 0; m < 3; ++m) {
            const float av = aw == 16 * m + c ? dchv : 0.0f;
            acc_w2[m] = mfma16x4(av, bv, acc_w2[m]);
            if (ub == 0) db2[m] += av;   // rows 4 g + s of this lane group; the groups are summed at the end
          }
        }
      }
    }
    // ---- slabs: [w_ih | w_hh | b_ih | b_hh | fc2.w | fc2.b] and [fc1.w | fc1.b], parameter layout
#pragma unroll
    for (int m = 0; m < 3; ++m)
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int gc = 16 * (4 * m + ub) + 4 * g + e, u = 16 * q + c;
          slab[gc * H + u] = acc_ih[m][q][e];
          slab[o_hh + gc * H + u] = acc_hh[m][q][e];
        }
    dw1_out(acc_w1, T_NIC, NI);
    const float s1 = gsum(db1);
    if (g == 0) slab1[(int64_t)H * I + j] = s1;
#pragma unroll
    for (int m = 0; m < 3; ++m)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int a = 16 * m + 4 * g + e;
        if (a < A) slab[o_w2 + a * H + j] = acc_w2[m][e];
      }
    if (ub == 0) {
#pragma unroll
      for (int m = 0; m < 3; ++m) {
        const float s2 = gsum(db2[m]);
        if (g == 0 && 16 * m + c < A) slab[o_b2 + 16 * m + c] = s2;
      }
    }
  }
}

}  // namespace mq
