// Persistent per-row GRU recurrences (the serial T loop of QLearner.train, q_learner.py:49-52 / 60-62 / 101).
//
// Only the h -> h dependency is serial: the input side (fc1, W_ih) was hoisted into the row-parallel GEMMs, so
// each step here is the 64x192 W_hh mat-vec plus gate math (forward) or its transpose plus the gate
// derivatives (backward). A workgroup owns RW rows for the whole T loop; W_hh stays in VGPRs and the hidden /
// gate-gradient vectors round-trip through double-buffered LDS, one LDS-only barrier per step.
//
// Thread map (256 threads): unit j = tid >> 2 (0..63), quarter q = tid & 3. The four lanes of a quad hold the
// four K-quarters of one hidden unit and meet in a DPP quad reduction (no LDS). Gate math for row i runs on the
// lane with q == i % 4.
//
// Latency structure of one step (what the code is arranged around):
//  * the step's global inputs are prefetched one step ahead into one of two register sets; the T loop is
//    unrolled by two so the sets swap roles without register moves at the loop latch (a move would force a
//    vmcnt wait that, counters being in-order on gfx950, also waits for the step's output stores);
//  * forward: the loop is VALU-issue bound (two waves per SIMD), so everything not on the h chain is out of
//    it: fc2 runs afterwards as a row-parallel GEMM over the stored hidden states of both nets;
//  * backward: W2 is staged in LDS so the dchosen -> dh term is an LDS gather, and the per-row replay
//    addressing (episode id -> action row) is resolved once before the loop.
#pragma once
#include "learner_types.hpp"

namespace mq {

// Pick row i's value out of a per-row array held by every lane, with compile-time indices only.
template <int RW>
MQ_DEV float pick_row(const float (&v)[RW], int ii, int q) {
  float out = 0.0f;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int i = 4 * ii + s;
    if (i < RW && s == q) out = v[i];
  }
  return out;
}

// tanh(x) = 1 - 2 / (1 + e^{2x}): one v_exp + one v_rcp; absolute error ~1e-7 (relative error grows only where
// |tanh| < 1e-3, where the absolute error is what enters h).
MQ_DEV float tanh_fast(float x) {
  return 1.0f - 2.0f * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(2.8853900817779268f * x));
}

MQ_DEV float sigm_fast(float x) {   // 1 / (1 + e^-x) with v_exp_f32 / v_rcp_f32
  return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.4426950408889634f * x));
}

// ------------------------------------------------------------------------------------------------ forward
// VAR: ablation bits for the round-3 scripts/rec_micro.hip only (production = 0): 1 skip Hs/Gates stores,
// 2 stamp the T loop (cycles, 100 MHz ticks) into w.slab_mix.
template <int RW, bool ONLINE, int VAR>
MQ_DEV void gru_fwd_body(const Dims& d, const float* __restrict__ P, const Lay& L, const Work& w, int z) {
  constexpr int RL = (RW + 3) / 4;
  const int tid = threadIdx.x, j = tid >> 2, q = tid & 3;
  const int R = d.R, Tp = d.Tp;
  const int64_t RT = d.RT();
  __shared__ float hbuf[2][RW][H];

  float wr[16], wz[16], wn[16];
  {
    const float* Whh = P + L.o[MQ_P_RNN_W_HH];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      wr[k] = Whh[(0 * H + j) * H + 16 * q + k];
      wz[k] = Whh[(1 * H + j) * H + 16 * q + k];
      wn[k] = Whh[(2 * H + j) * H + 16 * q + k];
    }
  }
  const float bhr = P[L.o[MQ_P_RNN_B_HH] + j], bhz = P[L.o[MQ_P_RNN_B_HH] + H + j],
              bhn = P[L.o[MQ_P_RNN_B_HH] + 2 * H + j];

  const int r0 = blockIdx.x * RW;
  int rr[RL];
  bool rv[RL];
#pragma unroll
  for (int ii = 0; ii < RL; ++ii) {
    const int i = RW == 1 ? 0 : 4 * ii + q, r = r0 + i;   // RW == 1: all four lanes of a quad share the row
    rv[ii] = (RW == 1 || i < RW) && r < R;
    rr[ii] = min(r, R - 1);
  }
  for (int i = tid; i < RW * H; i += 256) hbuf[0][i / H][i % H] = 0.0f;   // init_hidden: h0 = 0

  const float* GI = w.GI + (int64_t)z * RT * G3;
  float* Hz = w.Hs + (int64_t)z * RT * H;
  auto load = [&](int t, float (&g)[RL][3]) {
    const int tc = min(t, Tp - 1);
    if constexpr (RW == 1) {   // lane-split gates: lane q of the quad owns gate component min(q, 2)
      g[0][0] = GI[((int64_t)tc * R + rr[0]) * G3 + min(q, 2) * H + j];
    } else {
#pragma unroll
      for (int ii = 0; ii < RL; ++ii) {
        const float* p = GI + ((int64_t)tc * R + rr[ii]) * G3;
        g[ii][0] = p[j]; g[ii][1] = p[H + j]; g[ii][2] = p[2 * H + j];
      }
    }
  };
  auto step = [&](int t, const float (&cur)[RL][3], float (&nxt)[RL][3]) {
    load(t + 1, nxt);   // next step's input gates, in flight under this step
    const float (*hb)[H] = hbuf[t & 1];
    float (*hn)[H] = hbuf[(t + 1) & 1];
    float sr[RW], sz[RW], sn[RW];
#pragma unroll
    for (int i = 0; i < RW; ++i) {
      const f32x4* hv4 = (const f32x4*)(&hb[i][16 * q]);
      float ar = 0.0f, az = 0.0f, an = 0.0f, ar2 = 0.0f, az2 = 0.0f, an2 = 0.0f;
#pragma unroll
      for (int k4 = 0; k4 < 4; ++k4) {
        const f32x4 hv = hv4[k4];
#pragma unroll
        for (int e = 0; e < 4; e += 2) {
          const int k = 4 * k4 + e;
          ar = fmaf(wr[k], hv[e], ar); ar2 = fmaf(wr[k + 1], hv[e + 1], ar2);
          az = fmaf(wz[k], hv[e], az); az2 = fmaf(wz[k + 1], hv[e + 1], az2);
          an = fmaf(wn[k], hv[e], an); an2 = fmaf(wn[k + 1], hv[e + 1], an2);
        }
      }
      sr[i] = quad_sum(ar + ar2);
      sz[i] = quad_sum(az + az2);
      sn[i] = quad_sum(an + an2);
    }
    if constexpr (RW == 1) {
      // One row, four lanes per unit: lane 0 computes r, lane 1 z (one sigmoid sequence for both), lane 2 n,
      // broadcast inside the quad by DPP; lane q stores gate component q. 1/4 of the gate VALU of the
      // one-lane form, and one GI load / one Gates store per lane.
      const float own = cur[0][0];
      const float gh = q == 0 ? sr[0] + bhr : (q == 1 ? sz[0] + bhz : 0.0f);
      const float sg = sigm_fast(gh + own);
      const float rg = quad_bcast<0>(sg), zg = quad_bcast<1>(sg);
      const float ghn = sn[0] + bhn;
      const float ng = quad_bcast<2>(tanh_fast(own + ghn * rg));
      const float hp = hb[0][j];
      const float h1 = (hp - ng) * zg + ng;   // ATen gru_cell: (hx - n) * z + n
      if (q == 0) hn[0][j] = h1;
      if (!(VAR & 1) && rv[0]) {
        const int64_t tr = (int64_t)t * R + rr[0];
        if (q == 0) Hz[tr * H + j] = h1;   // both nets: fc2 runs afterwards as a row-parallel GEMM over H
        if (ONLINE) w.Gates[tr * (4 * H) + q * H + j] = q == 0 ? rg : (q == 1 ? zg : (q == 2 ? ng : ghn));
      }
      lds_barrier();
      return;
    }
#pragma unroll
    for (int ii = 0; ii < RL; ++ii) {
      const int i = 4 * ii + q;
      const float ghr = pick_row<RW>(sr, ii, q) + bhr;
      const float ghz = pick_row<RW>(sz, ii, q) + bhz;
      const float ghn = pick_row<RW>(sn, ii, q) + bhn;
      if (i < RW) {
        const float hp = hb[i][j];
        const float rg = sigm_fast(ghr + cur[ii][0]);
        const float zg = sigm_fast(ghz + cur[ii][1]);
        const float ng = tanh_fast(cur[ii][2] + ghn * rg);
        const float h1 = (hp - ng) * zg + ng;   // ATen gru_cell: (hx - n) * z + n
        hn[i][j] = h1;
        if (!(VAR & 1) && rv[ii]) {
          const int64_t tr = (int64_t)t * R + rr[ii];
          Hz[tr * H + j] = h1;   // both nets: fc2 runs afterwards as a row-parallel GEMM over H
          if (ONLINE) {
            float* g = w.Gates + tr * (4 * H);
            g[j] = rg; g[H + j] = zg; g[2 * H + j] = ng; g[3 * H + j] = ghn;
          }
        }
      }
    }
    lds_barrier();
  };

  float ga[RL][3], gb[RL][3];
  load(0, ga);
  drain_vmem();
  lds_barrier();
  uint64_t c0 = 0, r0t = 0;
  if (VAR & 2) { c0 = __builtin_amdgcn_s_memtime(); r0t = __builtin_amdgcn_s_memrealtime(); }
  int t = 0;
  for (; t + 1 < Tp; t += 2) {
    step(t, ga, gb);
    step(t + 1, gb, ga);
  }
  if (t < Tp) step(t, ga, gb);
  if ((VAR & 2) && tid == 0) {   // diagnostic only: shader cycles and 100 MHz ticks of the whole T loop
    const uint64_t c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    ((uint64_t*)w.slab_mix)[2 * (blockIdx.y * gridDim.x + blockIdx.x)] = c1 - c0;
    ((uint64_t*)w.slab_mix)[2 * (blockIdx.y * gridDim.x + blockIdx.x) + 1] = r1 - r0t;
  }
}

// grid = (ceil(R / RW), 2 nets). Writes Hs for both nets and Gates for the online net.
template <int RW, int VAR = 0>
__global__ __launch_bounds__(256) void gru_fwd_kernel(Dims d, const float* __restrict__ P0,
                                                      const float* __restrict__ P1, Lay L, Work w) {
  if (blockIdx.y == 0) gru_fwd_body<RW, true, VAR>(d, P0, L, w, 0);
  else gru_fwd_body<RW, false, VAR>(d, P1, L, w, 1);
}

// ------------------------------------------------------------------------------------------------ backward
// BPTT over the online net (q_learner.py:100-101). grid = ceil(R / RW), 512 threads = two wave roles:
//  * chain waves (0-3, s_setprio 2): the serial part — gate derivatives from dh, the W_hh^T mat-vec, the carry;
//  * accumulator waves (4-7): dW_hh += dgh h_{t-1}^T, dW_ih += dgi x1^T and the fc2 grads for the same step,
//    read from the same LDS buffers after the step barrier. Half the per-step FMAs leave the chain; on each SIMD the
//    accumulator wave fills the chain wave's LDS / barrier / transcendental bubbles.
// Writes dGI for the dX1 GEMM and a per-workgroup slab [w_ih | w_hh | b_ih | b_hh | fc2.w | fc2.b].
struct BwdIn {
  float gr, gz, gn, ghn, hp, x1, dch;
  int act;
};

// DY (COMA actor, coma_learner.py:70-81): the output-layer gradient enters as a dense per-row vector
// w.dHo[t][row][64] = dLogits W2 for every step t < Tp, instead of dchosen * W2[a_t] for t < T; the fc2 grads are
// then a separate GEMM (Dw2Prob) and the slab's fc2 part stays zero.
template <int RW, int VAR = 0, bool DY = false>
__global__ __launch_bounds__(512) void gru_bwd_kernel(Dims d, Rep rp, const float* __restrict__ P, Lay L,
                                                      Work w, int64_t slab_len) {
  constexpr int RL = (RW + 3) / 4;
  const int tid = threadIdx.x;
  const bool chain = tid < 256;
  const int lt = tid & 255, k = lt >> 2, q = lt & 3;
  const int R = d.R, A = d.A, T = d.T;
  // Per row and step: gh_s = [dgh (3H) | h_{t-1} (H)], gi_s = [dgi (3H) | x1 (H)]; one 4H record each, so the
  // lane-split RW == 1 path writes component q of both with one unconditional LDS store per lane.
  __shared__ float gh_s[2][RW][4 * H];
  __shared__ float gi_s[2][RW][4 * H];
  __shared__ float dch_s[2][RW];   // per row: dLoss/dchosen (0 at t = T) and its action, for the fc2 grads
  __shared__ int act_s[2][RW];
  extern __shared__ float dyn[];   // W2 [A][H] | dW2 partial [A][H] | db2 [A]
  float* w2_s = dyn;
  float* dw2_s = dyn + A * H;
  float* db2_s = dyn + 2 * A * H;

  // Role-shared registers (the roles are disjoint per thread, so one allocation serves both):
  //   chain waves: wT = W_hh[48q..48q+47][k] (accI unused); accumulator waves: wT = dW_hh, accI = dW_ih slices.
  float wT[48], accI[48];
  const float* Whh = P + L.o[MQ_P_RNN_W_HH];
#pragma unroll
  for (int c = 0; c < 48; ++c) {
    wT[c] = chain ? Whh[(48 * q + c) * H + k] : 0.0f;
    accI[c] = 0.0f;
  }
  float (&accH)[48] = wT;
  for (int i = tid; i < A * H; i += 512) { w2_s[i] = P[L.o[MQ_P_FC2_W] + i]; dw2_s[i] = 0.0f; }
  for (int i = tid; i < A; i += 512) db2_s[i] = 0.0f;

  const int r0 = blockIdx.x * RW;
  int rr[RL];
  bool rv[RL];
  const int64_t* arow[RL];   // &actions[ep(b)][0][agent], stride n per step
#pragma unroll
  for (int ii = 0; ii < RL; ++ii) {
    const int i = RW == 1 ? 0 : 4 * ii + q, r = r0 + i;   // RW == 1: all four lanes of a quad share the row
    rv[ii] = (RW == 1 || i < RW) && r < R;
    rr[ii] = min(r, R - 1);
    const int b = (int)fdiv((uint32_t)rr[ii], d.dN), ag = rr[ii] - b * d.n;
    arow[ii] = rp.actions + rp.ep(b) * d.t_stride * d.n + ag;
  }
  auto load = [&](int t, BwdIn (&s)[RL]) {
    const int tc = (VAR & 4) ? d.Tp - 1 : max(t, 0);   // VAR bit 4 (microbenchmark): cache-resident inputs
    const int td = min(tc, T - 1);
    if constexpr (RW == 1) {
      // lane-split: lane q loads gate component q and one of (h_{t-1}, x1, dch, action) — two loads per lane, no
      // branches (divergent loads would blur the vmcnt bookkeeping the prefetch relies on). The action is read as
      // the low word of the int64 (little-endian, 0 <= a < A).
      const int64_t tr = (int64_t)tc * R + rr[0];
      const float* src = q == 0   ? w.Hs + (tc > 0 ? tr - R : tr) * H + k
                         : q == 1 ? w.X1 + tr * H + k
                         : q == 2 ? (DY ? w.dHo + tr * H + k : w.dch + (int64_t)td * R + rr[0])
                                  : (const float*)(arow[0] + (int64_t)tc * d.n);
      s[0].gr = w.Gates[tr * (4 * H) + q * H + k];
      s[0].hp = *src;
      return;
    }
#pragma unroll
    for (int ii = 0; ii < RL; ++ii) {
      const int64_t tr = (int64_t)tc * R + rr[ii];
      const float* g = w.Gates + tr * (4 * H);
      s[ii].gr = g[k]; s[ii].gz = g[H + k]; s[ii].gn = g[2 * H + k]; s[ii].ghn = g[3 * H + k];
      s[ii].hp = w.Hs[(tc > 0 ? tr - R : tr) * H + k];
      s[ii].x1 = w.X1[tr * H + k];
      s[ii].dch = DY ? w.dHo[tr * H + k] : w.dch[(int64_t)td * R + rr[ii]];
      s[ii].act = (int)arow[ii][(int64_t)tc * d.n];
    }
  };

  float carry[RL];
  float dbi0 = 0, dbi1 = 0, dbi2 = 0, dbh2 = 0;   // RW == 1: dbi0 / dbh2 hold this lane's component q of b_ih / b_hh
#pragma unroll
  for (int ii = 0; ii < RL; ++ii) carry[ii] = 0.0f;

  auto chain_pre = [&](int t, const BwdIn (&cur)[RL], BwdIn (&nxt)[RL], float (&cz)[RL]) {
    load(t - 1, nxt);   // previous (earlier) step's inputs, in flight under this step
    const int pb = t & 1;
    if constexpr (RW == 1) {
      // lane-split: every lane of the quad gets the unit's inputs by DPP broadcast and computes the (cheap) gate
      // derivatives redundantly; lane q then owns component q of every store.
      const bool live = rv[0];
      const float g = cur[0].gr, aux = cur[0].hp;
      const float gr = quad_bcast<0>(g), gz = quad_bcast<1>(g), gn = quad_bcast<2>(g), ghn = quad_bcast<3>(g);
      const float hp = t > 0 ? quad_bcast<0>(aux) : 0.0f, x1 = quad_bcast<1>(aux);
      const float dchv = (live && (DY || t < T)) ? quad_bcast<2>(aux) : 0.0f;
      const int a = __builtin_bit_cast(int, quad_bcast<3>(aux));
      const float dh = carry[0] + (DY ? dchv : dchv * w2_s[a * H + k]);
      if (k == 0 && q == 0) { dch_s[pb][0] = dchv; act_s[pb][0] = a; }
      const float dn = dh * (1.0f - gz);
      const float dz = dh * (hp - gn);
      const float dan = dn * (1.0f - gn * gn);
      const float dar = (dan * ghn) * (gr * (1.0f - gr));
      const float daz = dz * (gz * (1.0f - gz));
      const float mine_i = q == 0 ? dar : (q == 1 ? daz : dan);   // dgi component q
      const float mine_h = q == 2 ? dan * gr : mine_i;             // dgh component q
      gi_s[pb][0][q * H + k] = q < 3 ? mine_i : x1;
      gh_s[pb][0][q * H + k] = q < 3 ? mine_h : hp;
      if (live && q < 3) w.dGI[((int64_t)t * R + rr[0]) * G3 + q * H + k] = mine_i;
      dbi0 += q < 3 ? mine_i : 0.0f;
      dbh2 += q < 3 ? mine_h : 0.0f;
      cz[0] = dh * gz;
      return;
    }
#pragma unroll
    for (int ii = 0; ii < RL; ++ii) {
      const int i = 4 * ii + q;
      cz[ii] = 0.0f;
      if (i >= RW) continue;
      const bool live = rv[ii];
      const float gr = live ? cur[ii].gr : 0.0f, gz = live ? cur[ii].gz : 0.0f;
      const float gn = live ? cur[ii].gn : 0.0f, ghn = live ? cur[ii].ghn : 0.0f;
      const float hp = (live && t > 0) ? cur[ii].hp : 0.0f, x1 = live ? cur[ii].x1 : 0.0f;
      float dh = carry[ii];
      const float dchv = (live && (DY || t < T)) ? cur[ii].dch : 0.0f;
      const int a = cur[ii].act;
      dh += DY ? dchv : dchv * w2_s[a * H + k];
      if (k == 0) { dch_s[pb][i] = dchv; act_s[pb][i] = a; }
      const float dn = dh * (1.0f - gz);
      const float dz = dh * (hp - gn);
      const float dan = dn * (1.0f - gn * gn);
      const float dar = (dan * ghn) * (gr * (1.0f - gr));
      const float daz = dz * (gz * (1.0f - gz));
      if (live) {
        float* o = w.dGI + ((int64_t)t * R + rr[ii]) * G3;
        o[k] = dar; o[H + k] = daz; o[2 * H + k] = dan;
      }
      gi_s[pb][i][k] = dar; gi_s[pb][i][H + k] = daz; gi_s[pb][i][2 * H + k] = dan;
      gh_s[pb][i][k] = dar; gh_s[pb][i][H + k] = daz; gh_s[pb][i][2 * H + k] = dan * gr;
      gh_s[pb][i][G3 + k] = hp;
      gi_s[pb][i][G3 + k] = x1;
      dbi0 += dar; dbi1 += daz; dbi2 += dan; dbh2 += dan * gr;
      cz[ii] = dh * gz;
    }
  };
  auto chain_post = [&](int t, const float (&cz)[RL]) {
    const int pb = t & 1;
    float s[RW];
#pragma unroll
    for (int i = 0; i < RW; ++i) {
      const f32x4* dg4 = (const f32x4*)(&gh_s[pb][i][48 * q]);
      float a0 = 0.0f, a1 = 0.0f, a2 = 0.0f, a3 = 0.0f;
#pragma unroll
      for (int c4 = 0; c4 < 12; ++c4) {
        const f32x4 dg = dg4[c4];
        const int c = 4 * c4;
        a0 = fmaf(wT[c], dg[0], a0); a1 = fmaf(wT[c + 1], dg[1], a1);
        a2 = fmaf(wT[c + 2], dg[2], a2); a3 = fmaf(wT[c + 3], dg[3], a3);
      }
      s[i] = quad_sum((a0 + a1) + (a2 + a3));
    }
    if constexpr (RW == 1) {
      carry[0] = cz[0] + s[0];   // every lane of the quad keeps the unit's carry
    } else {
#pragma unroll
      for (int ii = 0; ii < RL; ++ii) carry[ii] = cz[ii] + pick_row<RW>(s, ii, q);
    }
  };
  float h_next[RW];   // accumulator waves: h_t[k] of each row, read at step t+1
#pragma unroll
  for (int i = 0; i < RW; ++i) h_next[i] = 0.0f;
  auto accumulate = [&](int t) {
    const int pb = t & 1;
    // fc2 grads: dW2[a][k] += dchosen * h_t[k]; (a, k) is owned by lane (k, q = a % 4), so no two lanes ever
    // update the same word. h_t was the h_{t-1} record of step t+1, kept in a register since accumulate(t+1).
    if (!DY && t < T) {
#pragma unroll
      for (int i = 0; i < RW; ++i) {
        const int a = act_s[pb][i];
        if ((a & 3) == q) {
          const float dchv = dch_s[pb][i];
          dw2_s[a * H + k] += dchv * h_next[i];
          if (k == 0) db2_s[a] += dchv;
        }
      }
    }
#pragma unroll
    for (int i = 0; i < RW; ++i) {
      const f32x4* dg4 = (const f32x4*)(&gh_s[pb][i][48 * q]);
      const f32x4* di4 = (const f32x4*)(&gi_s[pb][i][48 * q]);
      const float hpk = gh_s[pb][i][G3 + k], x1k = gi_s[pb][i][G3 + k];
      h_next[i] = hpk;
#pragma unroll
      for (int c4 = 0; c4 < 12; ++c4) {
        const f32x4 dg = dg4[c4], di = di4[c4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          accH[4 * c4 + e] = fmaf(dg[e], hpk, accH[4 * c4 + e]);
          accI[4 * c4 + e] = fmaf(di[e], x1k, accI[4 * c4 + e]);
        }
      }
    }
  };
  // The two roles run separate loops that meet at one barrier per step: chain_pre(t) writes record buffer t & 1,
  // the barrier publishes it, then chain_post(t) and accumulate(t) both read it while chain_pre(t-1) fills the
  // other buffer (rewritten only after the next barrier, which accumulate(t) reaches first).
  uint64_t cyc_pre = 0, cyc_bar = 0, cyc_post = 0;   // VAR bit 2 (microbenchmark): chain section cycle stamps
  if (chain) {
    __builtin_amdgcn_s_setprio(2);
    BwdIn sa[RL], sb[RL];
    load(d.Tp - 1, sa);
    drain_vmem();
    lds_barrier();
    auto step = [&](int t, const BwdIn (&cur)[RL], BwdIn (&nxt)[RL]) {
      float cz[RL];
      uint64_t c0 = 0, c1 = 0, c2 = 0;
      if (VAR & 2) c0 = __builtin_amdgcn_s_memtime();
      chain_pre(t, cur, nxt, cz);
      if (VAR & 2) c1 = __builtin_amdgcn_s_memtime();
      lds_barrier();
      if (VAR & 2) c2 = __builtin_amdgcn_s_memtime();
      chain_post(t, cz);
      if (VAR & 2) {
        __builtin_amdgcn_s_waitcnt(0);   // keep the mat-vec inside the stamp
        const uint64_t c3 = __builtin_amdgcn_s_memtime();
        cyc_pre += c1 - c0; cyc_bar += c2 - c1; cyc_post += c3 - c2;
      }
    };
    int t = d.Tp - 1;
    for (; t - 1 >= 0; t -= 2) {
      step(t, sa, sb);
      step(t - 1, sb, sa);
    }
    if (t >= 0) step(t, sa, sb);
    __builtin_amdgcn_s_setprio(0);
  } else {
    lds_barrier();
    for (int t = d.Tp - 1; t >= 0; --t) {
      lds_barrier();
      if (!(VAR & 8)) accumulate(t);   // VAR bit 8 (microbenchmark): chain alone
    }
  }
  if ((VAR & 2) && tid == 0) {
    uint64_t* st = (uint64_t*)w.slab_mix + 4 * blockIdx.x;
    st[0] = cyc_pre; st[1] = cyc_bar; st[2] = cyc_post; st[3] = (uint64_t)__builtin_bit_cast(uint32_t, carry[0]);
  }

  // per-workgroup partial slab
  float* slab = w.slab_rnn + (int64_t)blockIdx.x * slab_len;
  const int64_t base = L.o[MQ_P_RNN_W_IH];
  const int64_t o_ih = 0, o_hh = L.o[MQ_P_RNN_W_HH] - base, o_bi = L.o[MQ_P_RNN_B_IH] - base,
                o_bh = L.o[MQ_P_RNN_B_HH] - base, o_w2 = L.o[MQ_P_FC2_W] - base, o_b2 = L.o[MQ_P_FC2_B] - base;
  if (!chain) {
#pragma unroll
    for (int c = 0; c < 48; ++c) {
      slab[o_ih + (48 * q + c) * H + k] = accI[c];
      slab[o_hh + (48 * q + c) * H + k] = accH[c];
    }
  } else {
    if constexpr (RW == 1) {
      if (q < 3) { slab[o_bi + q * H + k] = dbi0; slab[o_bh + q * H + k] = dbh2; }
    } else {
      dbi0 = quad_sum(dbi0); dbi1 = quad_sum(dbi1); dbi2 = quad_sum(dbi2); dbh2 = quad_sum(dbh2);
      if (q == 0) {
        slab[o_bi + k] = dbi0; slab[o_bi + H + k] = dbi1; slab[o_bi + 2 * H + k] = dbi2;
        slab[o_bh + k] = dbi0; slab[o_bh + H + k] = dbi1; slab[o_bh + 2 * H + k] = dbh2;
      }
    }
  }
  lds_barrier();
  for (int i = tid; i < A * H; i += 512) slab[o_w2 + i] = dw2_s[i];
  for (int i = tid; i < A; i += 512) slab[o_b2 + i] = db2_s[i];
}

}  // namespace mq
