// Fused backward for one-row workgroups: BPTT of the online agent (q_learner.py:100-101 through rnn_agent.py:24-28)
// with every weight-gradient contraction and the fc1 input gradient on MFMA beside the VALU chain.
//
// 512 threads, two wave roles meeting at one barrier per step (T loop runs backwards):
//  * chain waves (0-3): the serial part, as gru_bwd_kernel<1>: gate derivatives from dh (lane-split), the
//    W_hh^T mat-vec, the carry. Each step's [dgh | h_{t-1}] and dgi land in a 16-step LDS history instead of
//    HBM (no dGI round trip);
//  * producer waves (4-7): the fc2 grads of the step (VALU, as before) and, for the last complete 16-step chunk
//    C while the chain walks chunk C-1 (u = 16(C-1) + 15 - t):
//      u = 0         issue C's X1 / XIN row loads (written by the forward)
//      u = 1 .. 4    dW_hh += dGH^T H_prev   [192 x 64, K = 16 steps]      12 MFMA / step
//      u = 4         stage X1 / XIN in LDS
//      u = 5 .. 8    dW_ih += dGI^T X1       [192 x 64, K = 16]            12 MFMA / step
//      u = 9 .. 12   dX1 = (dGI W_ih) o relu'(X1)   [16 x 64, K = 192]     12 MFMA / step (W_ih in LDS)
//      u = 13 .. 15  dW1 += dX1^T XIN        [64 x I, K = 16]              7 / 7 / 14 MFMA
//    and chunk 0 after the chain finishes. dW_hh / dW_ih / dW1 accumulate in the MFMA C layout for the whole T
//    loop (48 + 48 + 28 VGPRs), so the Dx1 / Dw1 GEMMs and the dGI / dX1 buffers of the unfused path disappear.
// Writes the per-workgroup slabs [w_ih | w_hh | b_ih | b_hh | fc2.w | fc2.b] (row pitch slab_len, a multiple of 4; the
// two matrices in the accumulators' C-tile order, see the tail) and [fc1.w | fc1.b].
//
// MFMA maps as gru_fwd_fused.hpp (v_mfma_f32_16x16x4_f32: A[i = c][kk = g], B[kk = g][j = c], D[4g + r][c]).
#pragma once
#include <cstdlib>
#include "gru_fwd_fused.hpp"
#include "dwh_kernel.hpp"

namespace mq {

constexpr int BRP = 4 * H + 4;   // history row pitch: [dgh | h_{t-1}] and [dgi | -], padded against bank conflicts

struct alignas(16) BwdFusedLds {
  float gh[2][FCH][BRP];     // per step: dgh (3H) | h_{t-1} (H), chunk-double-buffered
  float gi[2][FCH][BRP];     // per step: dgi (3H) | unused
  float x1[FCH][H + 4];      // X1 of the chunk being reduced
  float xin[FCH][FXP];       // XIN of the chunk being reduced (zero-padded to 4 * Kq)
  float dx1[FCH][H + 4];     // dX1 of the chunk being reduced
  float db1[4][H];           // fc1 bias-grad partials of the four lane groups
  float wih[G3][H + 1];      // W_ih (dX1's B operand); odd pitch: the four lane groups read rows 48 apart
};

inline bool fused_bwd_ok(int I, int O, int A, int n, int64_t RT) { return fused_fwd_ok(I, O, A, n, RT); }

// The chain step is linearised: every gate derivative of a step is dh times a coefficient of that step's inputs:
// dn = dh (1 - z), dz = dh (h_{t-1} - n), d(a_n) = dh (1 - z)(1 - n^2), d(a_r) = d(a_n) ghn r (1 - r),
// d(a_z) = dh (h_{t-1} - n) z (1 - z). So each lane's record value is dh * c (+ h_{t-1} in the h slot) and the
// carry's own term is dh * z, with c computed from the gate record before dh is known: during the previous step,
// beside its mat-vec. What stays on the dh chain is dh = carry + dchosen W2[a], two products, the record stores and
// the mat-vec. Inputs are loaded three steps ahead (four slots). (Round 3: -3.5 us a BPTT against the
// non-linearised step; profiles/r03_ab_lin_k12.json.)
//
// K12 layout of the W_hh^T mat-vec: lane c of 16-lane DPP row r16 sums the 12 terms k in [12c, 12c + 12) for the
// row's four units 4 r16 .. +3 (48 FMAs, as 24 v_pk_fma_f32 with dgh[k] in both halves) and reads only those 12
// values from LDS (12 KB a step for the four chain waves, against 48 KB for a per-unit layout). The four partial
// sums per lane are reduce-scattered over the row with no selects: the W pairs are ordered per lane (bit 3 of c
// picks which unit pair stays in A, bit 2 which unit leads each pair), so one row_ror:8 add (pairs c, c ^ 8), one
// row_half_mirror add (pairs c, 7 - c: bit 2 differs) and the quad sum leave unit 4 r16 + 2 b3 + b2 = the lane's own
// quad index in all four lanes of the quad: the lane-split gate-math layout.
//
// Measured and removed in round 4 (records under profiles/r01*-r03*): decoupled roles meeting through LDS flags,
// SIMD-split roles, the non-linearised step, four accumulator pairs, the next step's W2 lookup a step early, plain
// vs non-temporal slab stores, per-weight dword prologue loads; all were slower than this kernel.
//
// DWH = 1: workgroups past the R rows compute dW_hyper tiles (dwh_body, two 256-thread tiles per workgroup, tile
// geometry in w.dwh_*): dispatched after every row, they take the CUs a second wave of rows leaves idle
// (configs[3]'s shard, R = 320 > 256 CUs) instead of running in the reduction's launch. Same tiles, same m order:
// bitwise dwh_red1_kernel's slabs.
// STAMP (diagnostic, MQ_DIAG bwd_stamp=<file>; Tp <= BSTN - BSTH): s_memtime stamps of the first 8 workgroups, written to
// w.GI (unused on this path) as uint32 [block][BSTN]: [0] entry, [1] chain wave 0 past the prologue barrier, [2] its
// loop end, [3] producer wave 4's tail (chunk 0) done, [4] the slabs written (after the last barrier), [5] the fc2 /
// bias slabs written; producer wave 4 in the tail: [6] dW_hh of chunk 0 done, [7] its slab stores issued, [8] past the
// tail's first barrier, [9] dW_ih done, [10] its slab issued, [11] dX1 done; [16 + u] chain wave 0's step t = Tp - 1 - u
// done.
constexpr int BSTH = 16, BSTN = BSTH + 152;
template <int DWH = 0, bool STAMP = false>
__global__ __launch_bounds__(512) void gru_bwd_fused_kernel(Dims d, Rep rp, const float* __restrict__ P, Lay L,
                                                            Work w, int64_t slab_len, int64_t slab1_len) {
  __shared__ BwdFusedLds S;
  extern __shared__ float dyn[];   // W2 [A][H] | dW2 partial [A][H] | db2 [A]
  __shared__ uint32_t bst[STAMP ? BSTN : 1];
  auto bstamp = [&](int slot) {
    if constexpr (STAMP) {
      uint64_t tt;
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(tt)::"memory");
      __builtin_amdgcn_sched_barrier(0);
      if ((threadIdx.x & 63) == 0) bst[slot] = (uint32_t)tt;
    }
  };
  if (threadIdx.x == 0) bstamp(0);
  if constexpr (DWH != 0) {
    static_assert(sizeof(BwdFusedLds) >= 2 * 4 * DWH_T * (DWH_T + 1) * sizeof(float), "dW_hyper tiles reuse the LDS");
    if ((int)blockIdx.x >= d.R) {
      const int half = (int)threadIdx.x >> 8;
      const int lin = min(2 * ((int)blockIdx.x - d.R) + half, w.dwh_n - 1);   // an odd count repeats the last tile
      dwh_body<8, 4>(d, L, w.dHYP, w.S0, w.slab_mix, w.dwh_len, w.dwh_ns, w.dwh_tj, lin, (int)threadIdx.x & 255,
                        (float*)&S + half * 4 * DWH_T * (DWH_T + 1));
      return;
    }
  }
  const int tid = threadIdx.x;
  const bool chain = tid < 256;
  // role-local thread id 0..255 (wave-uniform role; lanes of a quad stay in one wave)
  const int lt = tid & 255, k = lt >> 2, q = lt & 3;
  const int R = d.R, A = d.A, T = d.T, Tp = d.Tp, I = d.I;
  const int cl = (Tp - 1) / FCH;
  const int r = blockIdx.x;
  float* w2_s = dyn;
  float* dw2_s = dyn + A * H;
  float* db2_s = dyn + 2 * A * H;

  // the workgroup's LDS set-up (every thread, after its role's own first loads are in flight, so the kernel start
  // pays one memory latency, not two): W2 staged and dW2 / db2 zeroed, the history rows past Tp of the top (partial)
  // chunk and the XIN padding zeroed, W_ih staged (dX1's B operand)
  auto stage_common = [&]() {
    constexpr int NW2 = 16 * H / 512;   // A <= 16: all W2 loads in flight before the stores
    constexpr int NW = G3 * H / 512;
    float v2[NW2], v[NW];
#pragma unroll
    for (int u = 0; u < NW2; ++u) v2[u] = tid + 512 * u < A * H ? P[L.o[MQ_P_FC2_W] + tid + 512 * u] : 0.0f;
#pragma unroll
    for (int u = 0; u < NW; ++u) v[u] = P[L.o[MQ_P_RNN_W_IH] + tid + 512 * u];
    for (int i = tid; i < A; i += 512) db2_s[i] = 0.0f;
    for (int e = tid; e < 2 * FCH * BRP; e += 512) { (&S.gh[0][0][0])[e] = 0.0f; (&S.gi[0][0][0])[e] = 0.0f; }
    for (int e = tid; e < FCH * FXP; e += 512) (&S.xin[0][0])[e] = 0.0f;
#pragma unroll
    for (int u = 0; u < NW2; ++u)
      if (tid + 512 * u < A * H) { w2_s[tid + 512 * u] = v2[u]; dw2_s[tid + 512 * u] = 0.0f; }
#pragma unroll
    for (int u = 0; u < NW; ++u) {
      const int e = tid + 512 * u, m = e / H;
      S.wih[m][e - m * H] = v[u];
    }
  };

  const int b = (int)fdiv((uint32_t)r, d.dN), ag = r - b * d.n;
  const int64_t* arow = rp.actions + rp.ep(b) * d.t_stride * d.n + ag;   // &actions[ep(b)][0][agent]
  const int64_t base = L.o[MQ_P_RNN_W_IH];
  float* slab = w.slab_rnn + (int64_t)blockIdx.x * slab_len;
  const int64_t o_hh = L.o[MQ_P_RNN_W_HH] - base, o_bi = L.o[MQ_P_RNN_B_IH] - base,
                o_bh = L.o[MQ_P_RNN_B_HH] - base, o_w2 = L.o[MQ_P_FC2_W] - base, o_b2 = L.o[MQ_P_FC2_B] - base;

  if (chain) {
    // ================================================================ chain waves
    f32x2 wT[24];   // W_hh^T slice as pairs for v_pk_fma_f32 (K12 layout, see above)
    const int c16 = lt & 15;   // lane within the 16-lane DPP row
    const int b3 = (c16 >> 3) & 1, b2 = (c16 >> 2) & 1, u0 = 4 * (lt >> 4);
    f32x4 xr[12];   // W_hh rows 12 c16 .. + 11, units u0 .. u0 + 3 (loaded first, picked apart after the set-up)
    {
      const float* Whh = P + L.o[MQ_P_RNN_W_HH];
#pragma unroll
      for (int kk = 0; kk < 12; ++kk) xr[kk] = *(const f32x4*)(Whh + (12 * c16 + kk) * H + u0);
    }
    // K12 mat-vec on the 12 dgh values of this lane, reduced to the lane's unit (all four lanes of its quad)
    auto k12_sum = [&](const f32x4 (&dv)[3]) {
      f32x2 aA = {0.0f, 0.0f}, aB = {0.0f, 0.0f};
#pragma unroll
      for (int m = 0; m < 3; ++m)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const f32x2 dd = {dv[m][e], dv[m][e]};
          aA = pk_fma(wT[2 * (4 * m + e)], dd, aA);
          aB = pk_fma(wT[2 * (4 * m + e) + 1], dd, aB);
        }
      const float x = aA.x + row_ror8(aB.x), y = aA.y + row_ror8(aB.y);
      return quad_sum(x + row_half_mirror(y));
    };
    // lane-split inputs of a step: lane q loads gate component q and one of (h_{t-1}, dch, dch, action) at
    // base + idx * stride with per-lane constants, so no lane-dependent branch enters the chain. idx = t except
    // at the edges, clamped with per-lane 0/1 flags: h row 0 stands in for row -1 at t = 0 (hp is zeroed there),
    // dch row T-1 for row T at t = T (dchv is zeroed there). The action is read as the low word of the int64
    // (little-endian, 0 <= a < A). w2 = W2[a_t][k] is looked up one step ahead, off the dh chain.
    struct In { float g, aux, w2, wd, ci, ch, hq, gz; };   // wd .. gz: the step's coefficients
    const float* aux_base;
    int64_t aux_stride;
    if (q == 0) { aux_base = w.Hs + (int64_t)r * H + k - (int64_t)R * H; aux_stride = (int64_t)R * H; }
    else if (q == 3) { aux_base = (const float*)arow; aux_stride = 2 * (int64_t)d.n; }
    else { aux_base = w.dch + r; aux_stride = R; }
    const float* g_base = w.Gates + (int64_t)r * (4 * H) + q * H + k;
    const int e0 = q == 0 ? 1 : 0, e12 = (q == 1 || q == 2) ? 1 : 0;
    auto load = [&](int t, In& s) {
      const int tc = max(t, 0);
      const int idx = tc + (e0 & (tc == 0 ? 1 : 0)) - (e12 & (tc >= T ? 1 : 0));
      s.g = g_base[(int64_t)tc * R * (4 * H)];
      s.aux = aux_base[idx * aux_stride];
    };
    auto lookup_w2 = [&](In& s) { s.w2 = w2_s[__builtin_bit_cast(int, quad_bcast<3>(s.aux)) * H + k]; };
    // lane-split selectors as 0/1 factors (multiply-add selects, no branches)
    const float m0 = q == 0 ? 1.0f : 0.0f, m1 = q == 1 ? 1.0f : 0.0f, m2 = q == 2 ? 1.0f : 0.0f;
    const float m3 = q == 3 ? 1.0f : 0.0f;
    float carry = 0.0f, db_i = 0.0f, db_h = 0.0f;   // bias grads: this lane's component q of b_ih / b_hh
    // the step's coefficients (see the note above), computed one step ahead
    auto coeffs = [&](int t, In& s) {
      const float gr = quad_bcast<0>(s.g), gz = quad_bcast<1>(s.g), gn = quad_bcast<2>(s.g), ghn = quad_bcast<3>(s.g);
      const float hp = t > 0 ? quad_bcast<0>(s.aux) : 0.0f;
      const float dchv = t < T ? quad_bcast<2>(s.aux) : 0.0f;
      const float an = (1.0f - gz) * (1.0f - gn * gn);
      const float ar = (an * ghn) * (gr * (1.0f - gr));
      const float az = (hp - gn) * (gz * (1.0f - gz));
      const float rzc = fmaf(m0, ar, m1 * az);
      s.ci = fmaf(m2 + m3, an, rzc);       // dgi component q (q = 3: the unused slot)
      s.ch = fmaf(m2, an * gr, rzc);       // dgh component q (q = 3: 0, the slot holds h_{t-1})
      s.hq = m3 * hp;
      s.wd = dchv * s.w2;
      s.gz = gz;
    };
    auto lstep = [&](int t, const In& cur, In& nxt, In& ahead) {
      load(t - 3, ahead);
      const int p = t & (FCH - 1), cb = (t / FCH) & 1;
      const float dh = carry + cur.wd;
      const float mine_i = dh * cur.ci;
      const float mine_h = fmaf(dh, cur.ch, cur.hq);
      S.gh[cb][p][q * H + k] = mine_h;
      S.gi[cb][p][q * H + k] = mine_i;
      db_i = fmaf(1.0f - m3, mine_i, db_i);
      db_h = fmaf(1.0f - m3, mine_h, db_h);
      lds_barrier();
      // dh_{t-1} = dh * z + W_hh^T dgh
      const f32x4* d12 = (const f32x4*)(&S.gh[cb][p][12 * c16]);
      const f32x4 dv[3] = {d12[0], d12[1], d12[2]};
      lookup_w2(nxt);   // the next step's W2[a][k] and coefficients, beside this step's LDS reads and FMAs
      coeffs(t - 1, nxt);
      carry = fmaf(dh, cur.gz, k12_sum(dv));
      if constexpr (STAMP) { if (tid < 64 && Tp - 1 - t < BSTN - BSTH) bstamp(BSTH + Tp - 1 - t); }
    };
    In sa, sb, sc, sd;
    load(Tp - 1, sa);
    load(Tp - 2, sb);
    load(Tp - 3, sc);
    stage_common();
    {
      const int a0 = u0 + 2 * b3 + b2, a1 = u0 + 2 * b3 + 1 - b2;               // pair A: the units kept
      const int v0 = u0 + 2 * (1 - b3) + b2, v1 = u0 + 2 * (1 - b3) + 1 - b2;   // pair B: the partner's
      // units a0, a1, v0, v1 are u0 .. u0 + 3 in a lane-dependent order: one 16-byte load per row (the compiler
      // cannot merge the four lane-permuted dword loads itself), then selects
      auto pick = [](const f32x4& x, int i) { return i == 0 ? x[0] : i == 1 ? x[1] : i == 2 ? x[2] : x[3]; };
      const int i0 = a0 - u0, i1 = a1 - u0, i2 = v0 - u0, i3 = v1 - u0;
#pragma unroll
      for (int kk = 0; kk < 12; ++kk) {
        wT[2 * kk] = f32x2{pick(xr[kk], i0), pick(xr[kk], i1)};
        wT[2 * kk + 1] = f32x2{pick(xr[kk], i2), pick(xr[kk], i3)};
      }
    }
    drain_vmem();
    lds_barrier();
    if (tid == 0) bstamp(1);
    lookup_w2(sa);
    coeffs(Tp - 1, sa);
    int t = Tp - 1;
    for (; t - 3 >= 0; t -= 4) {
      lstep(t, sa, sb, sd);
      lstep(t - 1, sb, sc, sa);
      lstep(t - 2, sc, sd, sb);
      lstep(t - 3, sd, sa, sc);
    }
    if (t >= 0) lstep(t, sa, sb, sd);
    if (t - 1 >= 0) lstep(t - 1, sb, sc, sa);
    if (t - 2 >= 0) lstep(t - 2, sc, sd, sb);
    if (tid == 0) bstamp(2);
    lds_barrier();   // producer tail: chunk 0 (2 barriers)
    lds_barrier();
    if (q < 3) { slab[o_bi + q * H + k] = db_i; slab[o_bh + q * H + k] = db_h; }
  } else {
    // ================================================================== producer waves
    const int ptid = tid - 256, wv = ptid >> 6, lane = ptid & 63, g = lane >> 4, c16 = lane & 15;
    const int Kq = (I + 15) / 16 * 4;
    f32x4 acc_hh[3][4], acc_ih[3][4], acc_w1[7];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) { acc_hh[i][jj] = f32x4{0, 0, 0, 0}; acc_ih[i][jj] = f32x4{0, 0, 0, 0}; }
#pragma unroll
    for (int i = 0; i < 7; ++i) acc_w1[i] = f32x4{0, 0, 0, 0};
    f32x4 dxa = {0, 0, 0, 0}, dxb = {0, 0, 0, 0};
    float db1p = 0.0f;

    // X1 / XIN rows of a chunk: slot s of this thread covers element ptid + 256 s of [16][H] and of [16][I]
    constexpr int NX1 = FCH * H / 256, NXI = (FCH * 4 * FKQ + 255) / 256;
    float rx1[NX1], rxi[NXI];
    auto issue_rows = [&](int C) {
      const int t0 = FCH * C;
#pragma unroll
      for (int s = 0; s < NX1; ++s) {
        const int e = ptid + 256 * s, i = e / H, col = e - i * H, t = min(t0 + i, Tp - 1);
        rx1[s] = w.X1[((int64_t)t * R + r) * H + col];
      }
#pragma unroll
      for (int s = 0; s < NXI; ++s) {
        const int e = opaque(ptid + 256 * s), i = (int)fdiv((uint32_t)e, d.dI), col = e - i * I;
        const int t = min(t0 + i, Tp - 1);
        rxi[s] = e < FCH * I ? w.XIN[((int64_t)t * R + r) * I + col] : 0.0f;
      }
    };
    auto store_rows = [&](int C) {
      const int t0 = FCH * C;
#pragma unroll
      for (int s = 0; s < NX1; ++s) {
        const int e = ptid + 256 * s, i = e / H, col = e - i * H;
        S.x1[i][col] = t0 + i < Tp ? rx1[s] : 0.0f;
      }
#pragma unroll
      for (int s = 0; s < NXI; ++s) {
        const int e = opaque(ptid + 256 * s), i = (int)fdiv((uint32_t)e, d.dI), col = e - i * I;
        if (e < FCH * I) S.xin[i][col] = t0 + i < Tp ? rxi[s] : 0.0f;
      }
    };
    // dW_hh / dW_ih: wave wv owns M-tiles 3wv .. 3wv+2 (gate rows) x all 4 N-tiles; K = 16 steps, kk = 4 kb + g
    auto dw_rec = [&](int C, int kb0, int kb1, bool ih) {
      const int cb = C & 1;
#pragma unroll
      for (int kb = kb0; kb < kb1; ++kb) {
        const int row = 4 * kb + g;
        float av[3], bv[4];
#pragma unroll
        for (int i = 0; i < 3; ++i) av[i] = (ih ? S.gi : S.gh)[cb][row][16 * (3 * wv + i) + c16];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) bv[jj] = ih ? S.x1[row][16 * jj + c16] : S.gh[cb][row][3 * H + 16 * jj + c16];
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) {
            if (ih) acc_ih[i][jj] = mfma16x4(av[i], bv[jj], acc_ih[i][jj]);
            else acc_hh[i][jj] = mfma16x4(av[i], bv[jj], acc_hh[i][jj]);
          }
      }
    };
    // dX1[16][64] = dGI[16][192] W_ih[192][64]: wave wv owns N-tile wv; lane group g owns k in [48 g, 48 g + 48)
    auto dx1_part = [&](int C, int m0, int m1) {   // b128 groups [m0, m1) of 12
      const int cb = C & 1;
#pragma unroll
      for (int m = m0; m < m1; ++m) {
        const f32x4 av = *(const f32x4*)&S.gi[cb][c16][48 * g + 4 * m];
        const float* wb = &S.wih[48 * g + 4 * m][16 * wv + c16];
        dxa = mfma16x4(av[0], wb[0], dxa);
        dxb = mfma16x4(av[1], wb[H + 1], dxb);
        dxa = mfma16x4(av[2], wb[2 * (H + 1)], dxa);
        dxb = mfma16x4(av[3], wb[3 * (H + 1)], dxb);
      }
    };
    auto dx1_epi = [&]() {   // relu'(X1) mask, fc1 bias-grad partial
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int i = 4 * g + e, col = 16 * wv + c16;
        const float v = S.x1[i][col] > 0.0f ? dxa[e] + dxb[e] : 0.0f;
        S.dx1[i][col] = v;
        db1p += v;
      }
      dxa = f32x4{0, 0, 0, 0};
      dxb = f32x4{0, 0, 0, 0};
    };
    // dW1[64][I] += dX1^T XIN: wave wv owns M-tile wv (fc1 unit rows) x 7 N-tiles (inputs); kk = 4 kb + g
    auto dw1_part = [&](int kb0, int kb1) {
#pragma unroll
      for (int kb = kb0; kb < kb1; ++kb) {
        const int row = 4 * kb + g;
        const float av = S.dx1[row][16 * wv + c16];
#pragma unroll
        for (int nt = 0; nt < 7; ++nt) {
          if (16 * nt >= 4 * Kq) break;
          acc_w1[nt] = mfma16x4(av, S.xin[row][16 * nt + c16], acc_w1[nt]);
        }
      }
    };
    // fc2 grads of step t: dW2[a][k] += dchosen * h_t[k]; (a, k) owned by lane (k, q = a % 4); h_t was the
    // h_{t-1} record of step t+1. dchosen_t and a_t are wave-uniform loads issued one step ahead.
    float h_next = 0.0f, dch_n = 0.0f;
    int act_n = 0;
    auto fc2_fetch = [&](int t) {
      const int tc = max(t, 0);
      dch_n = w.dch[(int64_t)min(tc, T - 1) * R + r];
      act_n = *(const int*)(arow + (int64_t)tc * d.n);
    };
    auto fc2_grads = [&](int t) {
      const int p = t & (FCH - 1), cb = (t / FCH) & 1;
      const float dchv = t < T ? dch_n : 0.0f;
      const int a = act_n;
      fc2_fetch(t - 1);
      if (t < T && (a & 3) == q) {
        dw2_s[a * H + k] += dchv * h_next;
        if (k == 0) db2_s[a] += dchv;
      }
      h_next = S.gh[cb][p][3 * H + k];
    };
    fc2_fetch(Tp - 1);
    issue_rows(cl);   // the X1 / XIN rows one chunk ahead (the top chunk's up front)
    stage_common();

    lds_barrier();
    for (int c = cl; c >= 0; --c) {
      const int C = c + 1;
      const bool work = C <= cl;
#pragma unroll
      for (int u = 0; u < FCH; ++u) {
        const int t = FCH * c + FCH - 1 - u;
        if (t >= Tp) continue;
        lds_barrier();   // step t's records published
        fc2_grads(t);
        if (work) {
          if (u >= 1 && u <= 4) dw_rec(C, u - 1, u, false);
          if (u == 4) store_rows(C);
          if (u >= 5 && u <= 8) dw_rec(C, u - 5, u - 4, true);
          if (u >= 9 && u <= 12) dx1_part(C, 3 * (u - 9), 3 * (u - 8));
          if (u == 12) dx1_epi();
          if (u == 13) dw1_part(0, 1);
          if (u == 14) dw1_part(1, 2);
          if (u == 15) dw1_part(2, 4);
        }
        if (u == 5 && c < cl) issue_rows(c);   // stored at u = 4 of the next chunk
      }
    }
    // tail: chunk 0 (2 barriers, matched by the chain waves). Each accumulator's slab is written as soon as it is
    // final, so the slab stores (133 KB a workgroup, every workgroup at once: HBM-bound) overlap the remaining MFMAs
    // instead of all following them. [W_ih | W_hh] go out as the accumulators sit in the registers, one 16-byte
    // store per lane and tile (a wave writes 1 KB contiguous per instruction; element (16 mt + 4 g + e, 16 jj + c16)
    // at ((mt * 4 + jj) * 64 + lane) * 4 + e, which the reduction maps back: optim_kernels.hpp red_dst) instead of
    // 48 dword stores of 4 x 64-byte runs, which the CU's memory pipeline issued at ~46 cycles each (stamps).
    auto write_rec = [&](const f32x4 (&acc)[3][4], int64_t o) {
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
          *(f32x4*)&slab[o + (((3 * wv + i) * 4 + jj) * 64 + lane) * 4] = acc[i][jj];
    };
    dw_rec(0, 0, 4, false);
    if (ptid == 0) bstamp(6);
    store_rows(0);   // (the compiler waits for these rows' loads only, not for the slab stores below)
    write_rec(acc_hh, o_hh);
    if (ptid == 0) bstamp(7);
    lds_barrier();
    if (ptid == 0) bstamp(8);
    dw_rec(0, 0, 4, true);
    if (ptid == 0) bstamp(9);
    write_rec(acc_ih, 0);
    if (ptid == 0) bstamp(10);
    dx1_part(0, 0, 12);
    dx1_epi();
    if (ptid == 0) bstamp(11);
    lds_barrier();
    dw1_part(0, 4);
    if (ptid == 0) bstamp(3);

    float* slab1 = w.slab_fc1 + (int64_t)blockIdx.x * slab1_len;
#pragma unroll
    for (int nt = 0; nt < 7; ++nt)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = 16 * wv + 4 * g + e, nn = 16 * nt + c16;
        if (nn < I) slab1[m * I + nn] = acc_w1[nt][e];
      }
    S.db1[g][16 * wv + c16] = db1p;
  }
  lds_barrier();
  if (tid == 0) bstamp(4);
  for (int i = tid; i < A * H; i += 512) slab[o_w2 + i] = dw2_s[i];
  for (int i = tid; i < A; i += 512) slab[o_b2 + i] = db2_s[i];
  if (tid < H)
    w.slab_fc1[(int64_t)blockIdx.x * slab1_len + H * I + tid] =
        (S.db1[0][tid] + S.db1[1][tid]) + (S.db1[2][tid] + S.db1[3][tid]);
  if constexpr (STAMP) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) bstamp(5);
    __syncthreads();
    if (blockIdx.x < 8)
      for (int i = tid; i < BSTN; i += 512) ((uint32_t*)w.GI)[(size_t)blockIdx.x * BSTN + i] = bst[i];
  }
}

// Host: the fused BPTT, with dW_hyper's tiles appended (DWH = 1; w.dwh_* set by the caller) or without.
inline void launch_bwd_fused_dwh(size_t dyn, hipStream_t s, const Dims& d, const Rep& rp, const float* P,
                                 const Lay& L, const Work& w, int64_t slab_len, int64_t slab1_len) {
  const dim3 grid(d.R + (w.dwh_n + 1) / 2);
  hipLaunchKernelGGL((gru_bwd_fused_kernel<1>), grid, dim3(512), dyn, s, d, rp, P, L, w, slab_len, slab1_len);
}
inline void launch_bwd_fused(dim3 grid, size_t dyn, hipStream_t s, const Dims& d, const Rep& rp, const float* P,
                             const Lay& L, const Work& w, int64_t slab_len, int64_t slab1_len, bool stamp = false) {
  if (stamp)
    hipLaunchKernelGGL((gru_bwd_fused_kernel<0, true>), grid, dim3(512), dyn, s, d, rp, P, L, w, slab_len, slab1_len);
  else
    hipLaunchKernelGGL((gru_bwd_fused_kernel<0>), grid, dim3(512), dyn, s, d, rp, P, L, w, slab_len, slab1_len);
}

}  // namespace mq
