// Row-pair fused agent forward: one workgroup per row r runs BOTH nets' unrolls (online z = 0, target z = 1) of
// QLearner.train (q_learner.py:49-52, 60-62; rnn_agent.py:24-28), with ONE recurrence wave per net and no barrier
// inside a 16-step chunk.
//
// Why. In the one-row-net kernel (gru_fwd_fused.hpp) the 64 hidden units of a step are spread over four waves, which
// meet at an LDS barrier every step to exchange h. Stamps of that arrangement (scripts/pair_stamps.py, round 5) put a
// step at ~1,260 cycles: ~940 of recurrence work, whose per-unit overhead (DPP sums, lane-split gate math, selects)
// is paid by every K-split lane of a unit, and ~300 of barrier. Here lane j of a net's recurrence wave owns unit j
// whole (K = 64, no cross-lane sum, no gate broadcast) and reads h_{t-1} back from LDS itself (two broadcast reads of
// 32 floats), so the h chain never leaves the wave; its three W_hh rows live in 192 VGPRs.
// The matrix-core work (fc1, W_ih, fc2) runs on the two other SIMDs, decoupled by a two-chunk pipeline, and the roles
// meet once per chunk.
//
// 512 threads, one workgroup per CU; waves w and w + 4 share a SIMD:
//  * wave 0 / wave 1: the recurrence of net 0 / net 1 (SIMDs s0, s1); waves 4 and 5 (the same SIMDs) only stage
//    weights and pass the chunk barriers, so no MFMA ever holds a recurrence wave's SIMD;
//  * waves 2, 3, 6, 7: producers p = 0..3 (SIMDs s2, s3), during chunk c, for both nets:
//      fc2 of chunk c - 1 (producer p < 2 does net p: Q[16][A] = H W2^T + b2, K = 64 in one wave)
//      GI of chunk c + 1 = X1 W_ih^T + b_ih (N-tiles 3p .. 3p + 2) -> LDS, read by chunk c + 1's steps
//      fc1 of chunk c + 2: X1 = relu(XIN W1^T + b1) (N-tile p, W1 in registers)
//      the inputs of chunk c + 3 staged (obs gathered a chunk earlier, one-hots); chunk c + 4's gather issued.
// Outputs as gru_fwd_fused_kernel: Q of both nets; X1, XIN, Hs and the gate records of the online net. X1 and GI are
// bitwise the one-row-net kernel's (same MFMA operand maps and order); h and Q differ by summation order.
#pragma once
#include "gru_fwd_fused.hpp"

namespace mq {

struct alignas(16) PairLds {
  float h0[H];                    // init_hidden: zeros
  float hs[2][2][FCH][H + 4];     // [net][chunk & 1][step][unit]: h_t (the recurrence's h_{t-1}, fc2's operand)
  float gi[2][2][FCH][G3];        // [net][chunk & 1][step][gate column]
  float xin[2][FCH][FXP];         // [chunk & 1] agent inputs (both nets)
  float x1[2][2][FCH][H + 4];     // [net][chunk & 1] X1
};

inline bool pair_fwd_ok(int I, int O, int A, int n, int64_t RT) { return fused_fwd_ok(I, O, A, n, RT); }

// STAMP (diagnostic, MQ_PAIR_STAMP): lane 0 of recurrence wave 0 and of producer 0 in the first 8 workgroups write
// s_memtime into w.slab_rnn as uint32 [block][3][Tp]: 0 the end of each step (recurrence), 1 the recurrence's
// chunk-barrier arrival, 2 the producers' chunk-barrier arrival (both at the chunk's last step).
template <int NG, bool STAMP>
MQ_DEV void pair_body(const Dims& d, const Rep& rp, const float* __restrict__ P0, const float* __restrict__ P1,
                      const Lay& L, const Work& w, PairLds& S) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int R = d.R, Tp = d.Tp, I = d.I, O = d.O, A = d.A, n = d.n;
  const int cl = (Tp - 1) / FCH;   // last chunk
  const int r = blockIdx.x;
  const uint32_t RH = (uint32_t)R * H;
  uint32_t* const stp = (uint32_t*)w.slab_rnn + (size_t)blockIdx.x * 3 * Tp;
  auto stamp = [&](int k, int t) {
    if (STAMP && lane == 0 && blockIdx.x < 8) stp[k * Tp + t] = (uint32_t)__builtin_amdgcn_s_memtime();
  };

  if (tid < H) S.h0[tid] = 0.0f;
  constexpr int kPrologueBarriers = 3;
  const bool producer = (wv & 2) != 0;

  if (!producer) {
    if (wv >= 2) {   // waves 4, 5: the recurrence SIMDs' second slots stay free of work; they pass the barriers
      for (int i = 0; i < kPrologueBarriers + cl + 1; ++i) lds_barrier();
      return;
    }
    // ================================================================ recurrence wave of net z (wave z)
    const int z = wv, j = lane;
    const float* __restrict__ P = z ? P1 : P0;
    f32x2 wr[32], wz[32], wn[32];   // W_hh[gate * 64 + j][2 k, 2 k + 1]
    {
      const float* Whh = P + L.o[MQ_P_RNN_W_HH];
#pragma unroll
      for (int k4 = 0; k4 < 16; ++k4) {
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
    drain_vmem();
    for (int i = 0; i < kPrologueBarriers; ++i) lds_barrier();
    const bool online = z == 0;
    float hprev = 0.0f;
    const uint32_t hlo = ((uint32_t)r * H + j) * 4, glo = ((uint32_t)r * (4 * H) + j) * 4;
    __builtin_amdgcn_s_setprio(2);
    for (int c = 0; c <= cl; ++c) {
      const int pend = min(FCH, Tp - FCH * c);
      for (int p = 0; p < pend; ++p) {
        const int t = FCH * c + p;
        const float* hb = t == 0 ? S.h0 : S.hs[z][((t - 1) / FCH) & 1][(t - 1) & (FCH - 1)];
        const float gr = S.gi[z][c & 1][p][j], gz = S.gi[z][c & 1][p][H + j], gn = S.gi[z][c & 1][p][2 * H + j];
        f32x2 ar = {0.0f, 0.0f}, az = {0.0f, 0.0f}, an = {0.0f, 0.0f};
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {   // two halves of h: 8 broadcast b128 reads in flight, then 24 FMAs
          f32x4 hv[8];
#pragma unroll
          for (int q = 0; q < 8; ++q) hv[q] = *(const f32x4*)&hb[32 * hh + 4 * q];
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const int k4 = 8 * hh + q;
            const f32x2 h01 = {hv[q][0], hv[q][1]}, h23 = {hv[q][2], hv[q][3]};
            ar = pk_fma(wr[2 * k4], h01, ar); az = pk_fma(wz[2 * k4], h01, az); an = pk_fma(wn[2 * k4], h01, an);
            ar = pk_fma(wr[2 * k4 + 1], h23, ar); az = pk_fma(wz[2 * k4 + 1], h23, az);
            an = pk_fma(wn[2 * k4 + 1], h23, an);
          }
        }
        const float sr = ar.x + ar.y, sz = az.x + az.y, sn = an.x + an.y;
        // ATen gru_cell: r, z = sigmoid((W_h h + b_h) + gi); n = tanh(gi_n + r (W_hn h + b_hn)); h = (h - n) z + n
        const float rg = sigm_fast((sr + bhr) + gr), zg = sigm_fast((sz + bhz) + gz);
        const float ghn = sn + bhn;
        const float ng = tanh_fast(gn + ghn * rg);
        const float h1 = (hprev - ng) * zg + ng;
        hprev = h1;
        S.hs[z][c & 1][p][j] = h1;   // read back by this wave's next step (in-order LDS, no barrier)
        if (online) {
          buf_st(buf_rsrc(w.Hs + (int64_t)t * RH), hlo, h1);
          const auto gb = buf_rsrc(w.Gates + (int64_t)t * (4 * RH));
          buf_st(gb, glo, rg);
          buf_st(gb, glo + 4 * H, zg);
          buf_st(gb, glo + 8 * H, ng);
          buf_st(gb, glo + 12 * H, ghn);
        }
        if (z == 0) stamp(0, t);
      }
      if (z == 0) stamp(1, FCH * c + pend - 1);
      lds_barrier();   // chunk c's h history complete; chunk c + 1's GI staged
    }
    __builtin_amdgcn_s_setprio(0);
    return;
  }

  // ================================================================== producer waves 2, 3, 6, 7
  const int pw = (wv & 1) | ((wv >> 2) << 1);
  const int g = lane >> 4, c16 = lane & 15;
  const int ptid = pw * 64 + lane;
  const int Kq = (I + 15) / 16 * 4;   // fc1 k-blocks per lane group (multiple of 4)
  const int b = (int)fdiv((uint32_t)r, d.dN), ag = r - b * n;
  const int64_t slot0 = rp.ep(b) * d.t_stride;
  const float* obs_row = rp.obs + (slot0 * n + ag) * (int64_t)O;   // + t * n * O
  const uint32_t RI = (uint32_t)R * I, RA = (uint32_t)R * A;
  const int nO = n * O;
  int gsl[NG];   // gather slot s: element ptid + 256 s of a chunk's [16][O] obs block (gru_fwd_fused_kernel's packing)
#pragma unroll
  for (int s = 0; s < NG; ++s) {
    const int e = ptid + 256 * s, i = (int)fdiv((uint32_t)e, d.dO), col = e - i * O;
    gsl[s] = e < FCH * O ? (i << 28) | (col << 20) | (i * n * O + col) : -1;
  }
  float xr[NG];
  const int oi = ptid >> 4;   // this thread's one-hot row (step oi of a chunk)
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
  // register-resident weights of both nets: W1 (fc1 B fragments of N-tile pw), W_ih (3 N-tiles), W2 (K = 64)
  float w1r[2][FKQ], wih[2][3][16], w2r[16], bih[2][3], b1[2], b2;
#pragma unroll
  for (int z = 0; z < 2; ++z) {
    const float* __restrict__ P = z ? P1 : P0;
    const float* W1 = P + L.o[MQ_P_FC1_W] + (int64_t)(16 * pw + c16) * I;
#pragma unroll
    for (int k = 0; k < FKQ; ++k) {
      const int kk = g * Kq + k;
      w1r[z][k] = (k < Kq && kk < I) ? W1[min(kk, I - 1)] : 0.0f;
    }
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      const int nn = 16 * (3 * pw + s) + c16;
      const float* Wi = P + L.o[MQ_P_RNN_W_IH] + (int64_t)nn * H + 16 * g;
#pragma unroll
      for (int kb = 0; kb < 16; ++kb) wih[z][s][kb] = Wi[kb];
      bih[z][s] = P[L.o[MQ_P_RNN_B_IH] + nn];
    }
    b1[z] = P[L.o[MQ_P_FC1_B] + 16 * pw + c16];
  }
  {
    const int zf = pw & 1;   // fc2: producer 0 does net 0, producer 1 net 1
    const float* __restrict__ P = zf ? P1 : P0;
    const float* W2 = P + L.o[MQ_P_FC2_W] + (int64_t)min(c16, A - 1) * H + 16 * g;
#pragma unroll
    for (int kb = 0; kb < 16; ++kb) w2r[kb] = c16 < A ? W2[kb] : 0.0f;
    b2 = c16 < A ? P[L.o[MQ_P_FC2_B] + c16] : 0.0f;
  }

  float* X1o = w.X1;
  float* XINo = w.XIN;
  const int wd = I - O, npad = 4 * Kq - I;
  auto store_gather = [&](int cc) {   // the obs gathered by issue_gather(cc) and the one-hots -> xin[cc & 1]
    const int t0 = FCH * cc;
    float* xb = &S.xin[cc & 1][0][0];
    const auto xr_rsrc = buf_rsrc(XINo + ((int64_t)t0 * R + r) * I);   // wave-uniform
#pragma unroll
    for (int s = 0; s < NG; ++s) {
      const int gs = opaque(gsl[s]);
      const int i = (int)((uint32_t)gs >> 28), col = (gs >> 20) & 0xFF;
      const bool live = gs != -1, ok = live && t0 + i < Tp;
      xb[live ? i * FXP + col : FXP - 1] = ok ? xr[s] : 0.0f;   // a dead slot writes the never-read pad column
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
      xb[oi * FXP + O + col] = v;
      buf_st(xo, t < Tp ? (ro + col) * 4 : kDrop, v);
    }
    // zero K padding (columns I .. 4 Kq), which neither the gather nor the one-hots write
    for (int e = ptid; e < FCH * npad; e += 256) {
      const int i = e / npad;
      xb[i * FXP + I + (e - i * npad)] = 0.0f;
    }
  };
  auto fc1 = [&](int z, int cc) {   // X1 of chunk cc (inputs in xin[cc & 1]), N-tile pw -> x1[z][cc & 1]
    f32x4 acc = {0, 0, 0, 0}, acc2 = {0, 0, 0, 0};
    const float* xa = &S.xin[cc & 1][c16][g * Kq];
#pragma unroll
    for (int m = 0; m < FKQ / 4; ++m) {
      if (4 * m >= Kq) break;
      const f32x4 av = *(const f32x4*)&xa[4 * m];
      acc = mfma16x4(av[0], w1r[z][4 * m], acc);
      acc2 = mfma16x4(av[1], w1r[z][4 * m + 1], acc2);
      acc = mfma16x4(av[2], w1r[z][4 * m + 2], acc);
      acc2 = mfma16x4(av[3], w1r[z][4 * m + 3], acc2);
    }
    const int t0 = FCH * cc;
    const auto xb = buf_rsrc(X1o + ((int64_t)t0 * R + r) * H);   // wave-uniform
    const uint32_t lo = (uint32_t)(4 * g) * RH + 16 * pw + c16;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int i = 4 * g + e, t = t0 + i;
      const float x = fmaxf((acc[e] + acc2[e]) + b1[z], 0.0f);
      S.x1[z][cc & 1][i][16 * pw + c16] = x;
      if (z == 0) buf_st(xb, t < Tp ? (lo + e * RH) * 4 : kDrop, x);
    }
  };
  auto gi = [&](int z, int cc) {   // GI of chunk cc from x1[z][cc & 1], N-tiles 3 pw .. 3 pw + 2 -> gi[z][cc & 1]
    f32x4 accg[3] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
#pragma unroll
    for (int kq = 0; kq < 4; ++kq) {
      const f32x4 av = *(const f32x4*)&S.x1[z][cc & 1][c16][16 * g + 4 * kq];
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int s = 0; s < 3; ++s) accg[s] = mfma16x4(av[e], wih[z][s][4 * kq + e], accg[s]);
    }
#pragma unroll
    for (int s = 0; s < 3; ++s)
#pragma unroll
      for (int e = 0; e < 4; ++e) S.gi[z][cc & 1][4 * g + e][16 * (3 * pw + s) + c16] = accg[s][e] + bih[z][s];
  };
  auto fc2 = [&](int cc) {   // Q of chunk cc for net pw (pw < 2), K = 64 in this wave
    const int z = pw;
    f32x4 q0 = {0, 0, 0, 0}, q1 = {0, 0, 0, 0};
#pragma unroll
    for (int kq = 0; kq < 4; ++kq) {
      const f32x4 av = *(const f32x4*)&S.hs[z][cc & 1][c16][16 * g + 4 * kq];
      q0 = mfma16x4(av[0], w2r[4 * kq], q0);
      q1 = mfma16x4(av[1], w2r[4 * kq + 1], q1);
      q0 = mfma16x4(av[2], w2r[4 * kq + 2], q0);
      q1 = mfma16x4(av[3], w2r[4 * kq + 3], q1);
    }
    const int t0 = FCH * cc;
    const auto qb = buf_rsrc(w.Q + (int64_t)z * d.RT() * A + ((int64_t)t0 * R + r) * A);   // wave-uniform
    const uint32_t lo = (uint32_t)(4 * g) * RA + c16;
#pragma unroll
    for (int e = 0; e < 4; ++e)
      buf_st(qb, (t0 + 4 * g + e < Tp && c16 < A) ? (lo + e * RA) * 4 : kDrop, (q0[e] + q1[e]) + b2);
  };

  // ---- prologue (3 barriers, matched by the other waves): xin(0), xin(1) -> X1(0), X1(1) -> GI(0); xin(2) staged
  drain_vmem();
  store_gather(0);
  if (cl >= 1) { issue_gather(1); drain_vmem(); store_gather(1); }
  if (cl >= 2) issue_gather(2);
  lds_barrier();   // 1: xin(0), xin(1), h0
#pragma unroll
  for (int z = 0; z < 2; ++z) {
    fc1(z, 0);
    if (cl >= 1) fc1(z, 1);
  }
  lds_barrier();   // 2: X1(0), X1(1); xin(0) free
  if (cl >= 2) { store_gather(2); if (cl >= 3) issue_gather(3); }
#pragma unroll
  for (int z = 0; z < 2; ++z) gi(z, 0);
  lds_barrier();   // 3: GI(0), xin(2)

  for (int c = 0; c <= cl; ++c) {
    // chunk c: the recurrences run steps 16 c .. 16 c + 15 meanwhile
    if (c >= 1 && pw < 2) fc2(c - 1);
    if (c + 1 <= cl) { gi(0, c + 1); gi(1, c + 1); }
    if (c + 2 <= cl) { fc1(0, c + 2); fc1(1, c + 2); }
    if (c + 3 <= cl) { store_gather(c + 3); if (c + 4 <= cl) issue_gather(c + 4); }
    if (pw == 0) stamp(2, min(FCH * c + FCH - 1, Tp - 1));
    lds_barrier();
  }
  if (pw < 2) fc2(cl);   // the last chunk's h history is complete after the final barrier
}

// HYP = 1: the QMIX hypernet as the forward's epilogue. Once a workgroup's row is done, its whole CU (all eight
// waves, the LDS) runs hyper_fwd_body for hypernet block r, r + R, .. (32 state rows of one net each): the fp32 MFMA
// work of hyper_ws_kernel (bitwise its HYP and S0) without its launch, and on CUs whose matrix cores the recurrence
// SIMDs left idle.
template <int NG, bool STAMP = false, int HYP = 0>
__global__ __launch_bounds__(512, 1) void gru_fwd_pair_kernel(Dims d, Rep rp, const float* __restrict__ P0,
                                                              const float* __restrict__ P1, Lay L, Work w) {
  __shared__ PairLds S;
  static_assert(sizeof(PairLds) >= hyf_floats() * sizeof(float), "the hypernet epilogue reuses the forward's LDS");
  pair_body<NG, STAMP>(d, rp, P0, P1, L, w, S);
  if constexpr (HYP != 0) {
    const int nhb = 2 * ((d.M + 31) / 32);
    for (int hb = blockIdx.x; hb < nhb; hb += gridDim.x) {
      __syncthreads();   // the row's (or the previous block's) last LDS reads are done
      hyper_fwd_body(d, rp, P0, P1, L, w.HYP, w.S0, (float*)&S, hb);
    }
  }
}

// Host: the row-pair forward, grid R, with the smallest gather-slot instantiation that covers O.
inline void launch_fwd_pair(hipStream_t s, const Dims& d, const Rep& rp, const float* P0, const float* P1,
                            const Lay& L, const Work& w, bool hyp, bool stamp = false) {
  const dim3 g(d.R), b(512);
  const bool g5 = FCH * d.O <= 256 * 5;
  if (stamp) {
    if (hyp) hipLaunchKernelGGL((gru_fwd_pair_kernel<5, true, 1>), g, b, 0, s, d, rp, P0, P1, L, w);
    else hipLaunchKernelGGL((gru_fwd_pair_kernel<5, true, 0>), g, b, 0, s, d, rp, P0, P1, L, w);
  } else if (hyp) {
    if (g5) hipLaunchKernelGGL((gru_fwd_pair_kernel<5, false, 1>), g, b, 0, s, d, rp, P0, P1, L, w);
    else hipLaunchKernelGGL((gru_fwd_pair_kernel<FGATHER, false, 1>), g, b, 0, s, d, rp, P0, P1, L, w);
  } else {
    if (g5) hipLaunchKernelGGL((gru_fwd_pair_kernel<5, false, 0>), g, b, 0, s, d, rp, P0, P1, L, w);
    else hipLaunchKernelGGL((gru_fwd_pair_kernel<FGATHER, false, 0>), g, b, 0, s, d, rp, P0, P1, L, w);
  }
}

}  // namespace mq
