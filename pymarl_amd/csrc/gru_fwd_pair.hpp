// Row-pair fused agent forward: one workgroup per row r runs BOTH nets' unrolls (online z = 0, target z = 1) of
// QLearner.train (q_learner.py:49-52, 60-62; rnn_agent.py:24-28), sharing the row's agent inputs.
//
// Why a pair. At cfg2 the per-row forward (gru_fwd_fused.hpp, one row-net per workgroup, two per CU) is bound by the
// SIMDs' issue slots, not by latency: each SIMD hosts two recurrence waves (the CU's two row-nets) whose per-step
// overhead — DPP sums, the lane-split gate math, selects, stores — is paid by all four K-quarter lanes of every
// unit, plus two producer waves. Here the recurrence of a net runs on TWO waves (lane pair per unit, a K half each):
// the same W_hh FMAs per SIMD, a third of the DPP / gate instructions, one recurrence wave per SIMD. The producers
// stage the row's inputs once for both nets (the target net reads the same obs and one-hots).
//
// 512 threads, one workgroup per CU (waves w and w + 4 share a SIMD):
//  * waves 0-3, recurrences: net z = wave >> 1; lane l of the net's 128 lanes owns unit j = l >> 1 and K half
//    hk = l & 1 (W_hh[gate][j][32 hk .. 32 hk + 31] as 48 register pairs for v_pk_fma_f32); the pair meets in one
//    DPP add per gate; lane hk = 0 evaluates the r gate, lane 1 the z gate, both the n gate;
//  * waves 4-7, producers for both nets, per 16-step chunk c (MFMA M dimension = time), for chunk c + 1:
//      p0        stage the inputs (obs gathered a chunk ahead, one-hots) and issue chunk c + 2's gather;
//                fc2 partials of chunk c - 1 (both nets)
//      p1        Q stores of chunk c - 1
//      p1-p6     fc1 of both nets: X1 = relu(XIN W1^T + b1)
//      p5-p14    W_ih of both nets: GI = X1 W_ih^T + b_ih -> LDS, read by chunk c + 1's steps
//    about ten v_mfma_f32_16x16x4_f32 per producer wave and step.
// Outputs as gru_fwd_fused_kernel: Q of both nets; X1, XIN, Hs and the gate records of the online net.
#pragma once
#include "gru_fwd_fused.hpp"

namespace mq {

struct alignas(16) PairLds {
  float h0[H];                    // init_hidden: zeros
  float hs[2][2][FCH][H + 4];     // [net][chunk & 1][step][unit]: h_{t-1} of the recurrence, fc2's operand
  float gi[2][2][FCH][G3];        // [net][chunk & 1][step][gate column]
  float xin[FCH][FXP];            // agent inputs of the next chunk (both nets)
  float x1[2][FCH][H + 4];        // [net] X1 of the next chunk; fc2's partial tiles at p0 / p1
  float w1[2][H][FXP];            // fc1 weights, zero-padded
  float w2[2][16][H + 4];         // fc2 weights (A <= 16), zero-padded
};

inline bool pair_fwd_ok(int I, int O, int A, int n, int64_t RT) { return fused_fwd_ok(I, O, A, n, RT); }

// SPLIT: the two roles on disjoint SIMDs (waves w and w + 4 share one): recurrences on waves 0, 1, 4, 5 (two SIMDs,
// one wave of each net per SIMD), producers on waves 2, 3, 6, 7, so no f32 MFMA ever holds a recurrence wave's SIMD.
// Otherwise waves 0-3 / 4-7 (each SIMD one recurrence and one producer wave).
// STAMP (diagnostic, MQ_PAIR_STAMP): lane 0 of recurrence wave 0 and of producer wave 0 of the first 8 workgroups
// write s_memtime at each step's barrier arrival and (recurrence) release into w.slab_rnn as uint32
// [block][3][Tp]: 0 release, 1 recurrence arrival, 2 producer arrival.
template <int NG, bool SPLIT, bool STAMP = false>
__global__ __launch_bounds__(512, 1) void gru_fwd_pair_kernel(Dims d, Rep rp, const float* __restrict__ P0,
                                                              const float* __restrict__ P1, Lay L, Work w) {
  __shared__ PairLds S;
  const int tid = threadIdx.x;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int R = d.R, Tp = d.Tp, I = d.I, O = d.O, A = d.A, n = d.n;
  const int cl = (Tp - 1) / FCH;   // last chunk
  const int r = blockIdx.x;
  const uint32_t RH = (uint32_t)R * H;

  // ---- both nets' fc1 / fc2 weights to LDS (all 512 threads), zero padding, h0
  constexpr int N1 = (H * FXP + 511) / 512, N2 = (16 * (H + 4) + 511) / 512;
  float v1[2][N1], v2[2][N2];
  auto shared_load = [&]() {
#pragma unroll
    for (int z = 0; z < 2; ++z) {
      const float* __restrict__ P = z ? P1 : P0;
#pragma unroll
      for (int u = 0; u < N1; ++u) {
        const int e = tid + 512 * u, nn = e / FXP, k = e - nn * FXP;
        v1[z][u] = (e < H * FXP && k < I) ? P[L.o[MQ_P_FC1_W] + (int64_t)nn * I + k] : 0.0f;
      }
#pragma unroll
      for (int u = 0; u < N2; ++u) {
        const int e = tid + 512 * u, a = e / (H + 4), k = e - a * (H + 4);
        v2[z][u] = (e < 16 * (H + 4) && a < A && k < H) ? P[L.o[MQ_P_FC2_W] + (int64_t)a * H + k] : 0.0f;
      }
    }
  };
  auto shared_store = [&]() {
#pragma unroll
    for (int z = 0; z < 2; ++z) {
#pragma unroll
      for (int u = 0; u < N1; ++u) {
        const int e = tid + 512 * u;
        if (e < H * FXP) (&S.w1[z][0][0])[e] = v1[z][u];
      }
#pragma unroll
      for (int u = 0; u < N2; ++u) {
        const int e = tid + 512 * u;
        if (e < 16 * (H + 4)) (&S.w2[z][0][0])[e] = v2[z][u];
      }
    }
    if (tid < H) S.h0[tid] = 0.0f;
  };
  constexpr int kPrologueBarriers = 3;
  uint32_t* const stp = (uint32_t*)w.slab_rnn + (size_t)blockIdx.x * 3 * Tp;
  auto stamp = [&](int k, int t) {
    if ((tid & 63) == 0 && blockIdx.x < 8 && (wv == 0 || wv == (SPLIT ? 2 : 4)))
      stp[k * Tp + t] = (uint32_t)__builtin_amdgcn_s_memtime();
  };

  const bool rec = SPLIT ? (wv & 2) == 0 : wv < 4;
  const int ridx = SPLIT ? (wv & 1) | ((wv >> 2) << 1) : (wv & 3);   // index of this wave within its role
  if (rec) {
    // ================================================================ recurrence waves
    const int z = ridx >> 1;
    const float* __restrict__ P = z ? P1 : P0;
    const int lr = ((ridx & 1) << 6) | (tid & 63), j = lr >> 1, hk = lr & 1;
    f32x2 wr[16], wz[16], wn[16];   // W_hh[gate * 64 + j][32 hk + 2 k, + 1]
    shared_load();
    {
      const float* Whh = P + L.o[MQ_P_RNN_W_HH] + 32 * hk;
#pragma unroll
      for (int k4 = 0; k4 < 8; ++k4) {
        const f32x4 a = *(const f32x4*)(Whh + (int64_t)(0 * H + j) * H + 4 * k4);
        const f32x4 b = *(const f32x4*)(Whh + (int64_t)(1 * H + j) * H + 4 * k4);
        const f32x4 c = *(const f32x4*)(Whh + (int64_t)(2 * H + j) * H + 4 * k4);
        wr[2 * k4] = f32x2{a[0], a[1]}; wr[2 * k4 + 1] = f32x2{a[2], a[3]};
        wz[2 * k4] = f32x2{b[0], b[1]}; wz[2 * k4 + 1] = f32x2{b[2], b[3]};
        wn[2 * k4] = f32x2{c[0], c[1]}; wn[2 * k4 + 1] = f32x2{c[2], c[3]};
      }
    }
    const float bhr = P[L.o[MQ_P_RNN_B_HH] + j], bhz = P[L.o[MQ_P_RNN_B_HH] + H + j],
                bhn = P[L.o[MQ_P_RNN_B_HH] + 2 * H + j];
    shared_store();
    drain_vmem();
    for (int i = 0; i < kPrologueBarriers; ++i) lds_barrier();
    const bool online = z == 0;
    const float bsel = hk ? bhz : bhr;
    const int gcol = hk ? H + j : j;
    float hprev = 0.0f;
    // online stores: lane hk = 0 the h value and the (r, z) record components, lane 1 (n, W_hn h + b_hn)
    const uint32_t hlo = hk == 0 ? ((uint32_t)r * H + j) * 4 : kDrop;
    const uint32_t glo = ((uint32_t)r * (4 * H) + (hk ? 2 * H : 0) + j) * 4;
    auto step = [&](int t) {
      const int p = t & (FCH - 1), c = t / FCH;
      const float* hb = t == 0 ? S.h0 : S.hs[z][((t - 1) / FCH) & 1][(t - 1) & (FCH - 1)];
      const float own = S.gi[z][c & 1][p][gcol];
      const float own_n = S.gi[z][c & 1][p][2 * H + j];
      const f32x4* hv4 = (const f32x4*)(&hb[32 * hk]);
      f32x2 ar = {0.0f, 0.0f}, az = {0.0f, 0.0f}, an = {0.0f, 0.0f};
#pragma unroll
      for (int k4 = 0; k4 < 8; ++k4) {
        const f32x4 hv = hv4[k4];
        const f32x2 h01 = {hv[0], hv[1]}, h23 = {hv[2], hv[3]};
        ar = pk_fma(wr[2 * k4], h01, ar); az = pk_fma(wz[2 * k4], h01, az); an = pk_fma(wn[2 * k4], h01, an);
        ar = pk_fma(wr[2 * k4 + 1], h23, ar); az = pk_fma(wz[2 * k4 + 1], h23, az);
        an = pk_fma(wn[2 * k4 + 1], h23, an);
      }
      float sr = ar.x + ar.y, sz = az.x + az.y, sn = an.x + an.y;
      sr += quad_xor1(sr);   // the pair's two K halves (the same total on both lanes)
      sz += quad_xor1(sz);
      sn += quad_xor1(sn);
      // ATen gru_cell: r, z = sigmoid((W_h h + b_h) + gi); n = tanh(gi_n + r (W_hn h + b_hn)); h = (h - n) z + n
      const float sg = sigm_fast(((hk ? sz : sr) + bsel) + own);   // lane 0: r, lane 1: z
      const float so = quad_xor1(sg);
      const float rg = hk ? so : sg, zg = hk ? sg : so;
      const float ghn = sn + bhn;
      const float ng = tanh_fast(own_n + ghn * rg);
      const float h1 = (hprev - ng) * zg + ng;
      hprev = h1;
      S.hs[z][c & 1][p][j] = h1;   // both lanes of the pair store the same value
      if (online) {
        buf_st(buf_rsrc(w.Hs + (int64_t)t * RH), hlo, h1);
        const auto gb = buf_rsrc(w.Gates + (int64_t)t * (4 * RH));
        buf_st(gb, glo, hk ? ng : rg);
        buf_st(gb, glo + 4 * H, hk ? ghn : zg);
      }
      if constexpr (STAMP) stamp(1, t);
      lds_barrier();
      if constexpr (STAMP) stamp(0, t);
    };
    __builtin_amdgcn_s_setprio(2);
    for (int t = 0; t < Tp; ++t) step(t);
    __builtin_amdgcn_s_setprio(0);
    return;
  }

  // ================================================================== producer waves
  const int pw = ridx, lane = tid & 63, g = lane >> 4, c16 = lane & 15;
  const int ptid = pw * 64 + lane;
  const int Kq = (I + 15) / 16 * 4;   // fc1 k-blocks per lane group (multiple of 4: b128 operand reads)
  const int b = (int)fdiv((uint32_t)r, d.dN), ag = r - b * n;
  const int64_t slot0 = rp.ep(b) * d.t_stride;
  const float* obs_row = rp.obs + (slot0 * n + ag) * (int64_t)O;   // + t * n * O
  const uint32_t RI = (uint32_t)R * I, RA = (uint32_t)R * A;
  const int nO = n * O;
  // gather slot s: element e = ptid + 256 s of the chunk's [16][O] obs block, packed as in gru_fwd_fused_kernel
  int gsl[NG];
#pragma unroll
  for (int s = 0; s < NG; ++s) {
    const int e = ptid + 256 * s, i = (int)fdiv((uint32_t)e, d.dO), col = e - i * O;
    gsl[s] = e < FCH * O ? (i << 28) | (col << 20) | (i * n * O + col) : -1;
  }
  float xr[NG];
  // this thread's one-hot row (step i = ptid >> 4 of a chunk): filled[t-1] / actions[t-1] low words
  const int oi = ptid >> 4;
  int f_ld = 0, a_ld = -1;
  auto issue_gather = [&](int cc) {
    const int t0 = FCH * cc;
    const float* base = obs_row + (int64_t)t0 * nO;
    const int lim = (Tp - 1 - t0) * nO + O - 1;
#pragma unroll
    for (int s = 0; s < NG; ++s) xr[s] = ld_u32(base, (uint32_t)min(opaque(gsl[s]) & 0xFFFFF, lim));
    const int t = min(max(t0 + oi, 1), Tp - 1) - 1;
    f_ld = *(const int*)(rp.filled + slot0 + t);
    a_ld = *(const int*)(rp.actions + (slot0 + t) * n + ag);
  };
  issue_gather(0);
  shared_load();
  float wih[2][3][16], bih[2][3], b1[2], b2[2];
#pragma unroll
  for (int z = 0; z < 2; ++z) {
    const float* __restrict__ P = z ? P1 : P0;
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      const int nn = 16 * (3 * pw + s) + c16;
      const float* Wi = P + L.o[MQ_P_RNN_W_IH] + (int64_t)nn * H + 16 * g;
#pragma unroll
      for (int kb = 0; kb < 16; ++kb) wih[z][s][kb] = Wi[kb];
      bih[z][s] = P[L.o[MQ_P_RNN_B_IH] + nn];
    }
    b1[z] = P[L.o[MQ_P_FC1_B] + 16 * pw + c16];
    b2[z] = c16 < A ? P[L.o[MQ_P_FC2_B] + c16] : 0.0f;
  }
  shared_store();

  float* X1o = w.X1;
  float* XINo = w.XIN;
  const int wd = I - O;
  auto store_gather = [&](int cc) {
    const int t0 = FCH * cc;
    const auto xr_rsrc = buf_rsrc(XINo + ((int64_t)t0 * R + r) * I);   // wave-uniform
#pragma unroll
    for (int s = 0; s < NG; ++s) {
      const int gs = opaque(gsl[s]);
      const int i = (int)((uint32_t)gs >> 28), col = (gs >> 20) & 0xFF;
      const bool live = gs != -1, ok = live && t0 + i < Tp;
      (&S.xin[0][0])[live ? i * FXP + col : FXP - 1] = ok ? xr[s] : 0.0f;
      buf_st(xr_rsrc, ok ? ((uint32_t)i * RI + col) * 4 : kDrop, xr[s]);
    }
    // one-hot columns of step oi: last action (zero unless slot t-1 was filled, runner contract), agent id
    const int t = t0 + oi;
    const int ap = (d.last_action && t > 0 && t < Tp && f_ld) ? a_ld : -1;
    const auto xo = buf_rsrc(XINo + ((int64_t)t0 * R + r) * I + O);
    const uint32_t ro = (uint32_t)oi * RI;
    for (int col = ptid & 15; col < wd; col += 16) {
      float v;
      if (d.last_action && col < A) v = col == ap ? 1.0f : 0.0f;
      else v = (col - (d.last_action ? A : 0)) == ag ? 1.0f : 0.0f;
      S.xin[oi][O + col] = v;
      buf_st(xo, t < Tp ? (ro + col) * 4 : kDrop, v);
    }
  };
  f32x4 acc1 = {0, 0, 0, 0}, acc1b = {0, 0, 0, 0};
  f32x4 accg[2][3] = {{{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}}, {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}}};
  auto fc1_part = [&](int z, int m0, int m1) {   // b128 groups [m0, m1) of this lane group's Kq k-blocks
#pragma unroll
    for (int m = m0; m < m1; ++m) {
      if (4 * m >= Kq) break;
      const f32x4 av = *(const f32x4*)&S.xin[c16][g * Kq + 4 * m];
      const f32x4 bv = *(const f32x4*)&S.w1[z][16 * pw + c16][g * Kq + 4 * m];
      acc1 = mfma16x4(av[0], bv[0], acc1);
      acc1b = mfma16x4(av[1], bv[1], acc1b);
      acc1 = mfma16x4(av[2], bv[2], acc1);
      acc1b = mfma16x4(av[3], bv[3], acc1b);
    }
  };
  auto fc1_epi = [&](int z, int cc) {
    const int t0 = FCH * cc;
    const auto xb = buf_rsrc(X1o + ((int64_t)t0 * R + r) * H);   // wave-uniform
    const uint32_t lo = (uint32_t)(4 * g) * RH + 16 * pw + c16;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int i = 4 * g + e, t = t0 + i;
      const float x = fmaxf((acc1[e] + acc1b[e]) + b1[z], 0.0f);
      S.x1[z][i][16 * pw + c16] = x;
      if (z == 0) buf_st(xb, t < Tp ? (lo + e * RH) * 4 : kDrop, x);
    }
    acc1 = f32x4{0, 0, 0, 0};
    acc1b = f32x4{0, 0, 0, 0};
  };
  auto gi_part = [&](int z, int k0, int k1) {   // k-blocks [k0, k1) of this lane group's 16
#pragma unroll
    for (int kb = k0; kb < k1; ++kb) {
      const float av = S.x1[z][c16][16 * g + kb];
#pragma unroll
      for (int s = 0; s < 3; ++s) accg[z][s] = mfma16x4(av, wih[z][s][kb], accg[z][s]);
    }
  };
  auto gi_epi = [&](int z, int cc) {
#pragma unroll
    for (int s = 0; s < 3; ++s) {
#pragma unroll
      for (int e = 0; e < 4; ++e) S.gi[z][cc & 1][4 * g + e][16 * (3 * pw + s) + c16] = accg[z][s][e] + bih[z][s];
      accg[z][s] = f32x4{0, 0, 0, 0};
    }
  };
  // fc2 of a chunk in two steps: every producer wave multiplies its 16-wide K quarter into a partial tile in LDS
  // (aliasing the net's x1, idle at p0 / p1); wave 0 sums the four partials and stores Q
  auto fc2_partial = [&](int z, int cc) {
    float(*qpart)[FCH][16] = (float(*)[FCH][16])&S.x1[z][0][0];   // [4 waves][16 steps][16 actions]
    f32x4 acc2 = {0, 0, 0, 0};
    const f32x4 av = *(const f32x4*)&S.hs[z][cc & 1][c16][16 * pw + 4 * g];
    const f32x4 bv = *(const f32x4*)&S.w2[z][c16][16 * pw + 4 * g];
#pragma unroll
    for (int e = 0; e < 4; ++e) acc2 = mfma16x4(av[e], bv[e], acc2);
#pragma unroll
    for (int e = 0; e < 4; ++e) qpart[pw][4 * g + e][c16] = acc2[e];
  };
  auto fc2_store = [&](int z, int cc) {
    if (pw != 0) return;
    float(*qpart)[FCH][16] = (float(*)[FCH][16])&S.x1[z][0][0];
    const int t0 = FCH * cc;
    const auto qb = buf_rsrc(w.Q + (int64_t)z * d.RT() * A + ((int64_t)t0 * R + r) * A);   // wave-uniform
    const uint32_t lo = (uint32_t)(4 * g) * RA + c16;
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int i = 4 * g + e;
      v[e] = ((qpart[0][i][c16] + qpart[1][i][c16]) + (qpart[2][i][c16] + qpart[3][i][c16])) + b2[z];
    }
#pragma unroll
    for (int e = 0; e < 4; ++e)
      buf_st(qb, (t0 + 4 * g + e < Tp && c16 < A) ? (lo + e * RA) * 4 : kDrop, v[e]);
  };

  // ---- prologue (3 barriers, matched by the recurrence waves): chunk 0's inputs, X1 and GI of both nets
  drain_vmem();
  store_gather(0);
  lds_barrier();   // 1: weights, h0, chunk 0's inputs
  if (cl >= 1) issue_gather(1);
#pragma unroll
  for (int z = 0; z < 2; ++z) {
    fc1_part(z, 0, FKQ / 4);
    fc1_epi(z, 0);
  }
  lds_barrier();   // 2
#pragma unroll
  for (int z = 0; z < 2; ++z) {
    gi_part(z, 0, 16);
    gi_epi(z, 0);
  }
  lds_barrier();   // 3

  for (int c = 0; c <= cl; ++c) {
    const int t0 = FCH * c;
    const bool next = c + 1 <= cl;
#pragma unroll
    for (int p = 0; p < FCH; ++p) {
      if (t0 + p >= Tp) continue;   // last chunk: no work past Tp (and none for a next chunk)
      if (p == 0) {
        if (next) {
          store_gather(c + 1);
          if (c + 2 <= cl) issue_gather(c + 2);
        }
        if (c >= 1) { fc2_partial(0, c - 1); fc2_partial(1, c - 1); }
      }
      if (p == 1 && c >= 1) { fc2_store(0, c - 1); fc2_store(1, c - 1); }
      if (next) {
        // about ten MFMAs a phase: fc1 (7 b128 groups per net) then W_ih (16 k-blocks per net)
        if (p == 1) fc1_part(0, 0, 3);
        if (p == 2) fc1_part(0, 3, 5);
        if (p == 3) { fc1_part(0, 5, 7); fc1_epi(0, c + 1); }
        if (p == 4) fc1_part(1, 0, 3);
        if (p == 5) { fc1_part(1, 3, 5); gi_part(0, 0, 1); }
        if (p == 6) { fc1_part(1, 5, 7); fc1_epi(1, c + 1); gi_part(0, 1, 2); }
        if (p == 7) gi_part(0, 2, 6);
        if (p == 8) gi_part(0, 6, 10);
        if (p == 9) gi_part(0, 10, 13);
        if (p == 10) { gi_part(0, 13, 16); gi_epi(0, c + 1); gi_part(1, 0, 1); }
        if (p == 11) gi_part(1, 1, 5);
        if (p == 12) gi_part(1, 5, 9);
        if (p == 13) gi_part(1, 9, 13);
        if (p == 14) { gi_part(1, 13, 16); gi_epi(1, c + 1); }
      }
      if constexpr (STAMP) stamp(2, t0 + p);
      lds_barrier();
    }
  }
  // the last chunk (and the previous one's Q stores when the last chunk is a single step) after the final barrier:
  // producer wave z does net z
  if (cl >= 1 && Tp - FCH * cl < 2) { fc2_store(0, cl - 1); fc2_store(1, cl - 1); }
  if (pw < 2) {
    const int z = pw;
    f32x4 q0 = {0, 0, 0, 0}, q1 = {0, 0, 0, 0};
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const f32x4 av = *(const f32x4*)&S.hs[z][cl & 1][c16][16 * g + 4 * m];
      const f32x4 bv = *(const f32x4*)&S.w2[z][c16][16 * g + 4 * m];
      q0 = mfma16x4(av[0], bv[0], q0);
      q1 = mfma16x4(av[1], bv[1], q1);
      q0 = mfma16x4(av[2], bv[2], q0);
      q1 = mfma16x4(av[3], bv[3], q1);
    }
    const int t0 = FCH * cl;
    float* Qz = w.Q + (int64_t)z * d.RT() * A;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int t = t0 + 4 * g + e;
      if (t < Tp && c16 < A) Qz[((int64_t)t * R + r) * A + c16] = (q0[e] + q1[e]) + b2[z];
    }
  }
}

// Host: the row-pair forward, grid R, with the smallest gather-slot instantiation that covers O.
inline void launch_fwd_pair(hipStream_t s, const Dims& d, const Rep& rp, const float* P0, const float* P1,
                            const Lay& L, const Work& w, bool split, bool stamp = false) {
  const bool g5 = FCH * d.O <= 256 * 5;
  if (stamp) {
    if (split) hipLaunchKernelGGL((gru_fwd_pair_kernel<5, true, true>), dim3(d.R), dim3(512), 0, s, d, rp, P0, P1, L, w);
    else hipLaunchKernelGGL((gru_fwd_pair_kernel<5, false, true>), dim3(d.R), dim3(512), 0, s, d, rp, P0, P1, L, w);
  } else if (split) {
    if (g5) hipLaunchKernelGGL((gru_fwd_pair_kernel<5, true>), dim3(d.R), dim3(512), 0, s, d, rp, P0, P1, L, w);
    else hipLaunchKernelGGL((gru_fwd_pair_kernel<FGATHER, true>), dim3(d.R), dim3(512), 0, s, d, rp, P0, P1, L, w);
  } else {
    if (g5) hipLaunchKernelGGL((gru_fwd_pair_kernel<5, false>), dim3(d.R), dim3(512), 0, s, d, rp, P0, P1, L, w);
    else hipLaunchKernelGGL((gru_fwd_pair_kernel<FGATHER, false>), dim3(d.R), dim3(512), 0, s, d, rp, P0, P1, L, w);
  }
}

}  // namespace mq
