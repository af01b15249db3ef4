// One-chain-wave BPTT: the fused backward of the online agent (q_learner.py:100-101 through rnn_agent.py:24-28) with
// ONE chain wave per row and no barrier inside a 16-step chunk, the weight-gradient contractions on the other two
// SIMDs. NR rows per workgroup (NR = 2 when the rows exceed the CUs: configs[3]'s shard, R = 320, runs as 160
// workgroups, one wave of them, instead of 256 + 64).
//
// Why. gru_bwd_fused_kernel spreads a step's W_hh^T mat-vec over four chain waves (K12 layout: a quad of lanes per
// unit, DPP reduce-scatter) that meet at a workgroup barrier every step, and its producer waves share those SIMDs.
// Here lane k of the chain wave owns unit k whole: the column W_hh[:, k] lives in 96 packed VGPR pairs, the step's
// 192 gate-derivative values go to LDS and come back as 48 broadcast reads (the same wave: in-order LDS, no
// barrier), 96 v_pk_fma_f32 on two accumulators. Everything that does not depend on dh is computed a step ahead
// (the linearised step, gru_bwd_fused.hpp), so the chain is: dh = carry + dchosen W2[a], six products, seven LDS
// stores, the reads and the FMAs.
//
// 512 threads; waves w and w + 4 share SIMD w mod 4:
//  * waves 0 .. NR-1 (SIMDs s0, s1): the chain of row NR b + z, writing per step [dgh | h_{t-1}] and dgi into a
//    chunk-double-buffered LDS history;
//  * waves 2, 3, 6, 7 (SIMDs s2, s3): producers p = 0..3. While the chains walk chunk c - 1 they reduce chunk c of
//    every row of the workgroup into MFMA accumulators held for the whole T loop:
//      dW_hh += dGH^T H_prev [192 x 64]  M-tiles 3p .. 3p+2 x 4 N-tiles, K = 16 steps (gh history in LDS)
//      dW_ih += dGI^T X1      [192 x 64]  same tiles (gi history; X1 fragments from HBM)
//      dX1 = (dGI W_ih) o relu'(X1)  [16 x 64]  N-tile p, K = 192 (W_ih fragments in registers)
//      dW1 += dX1^T XIN       [64 x I]   M-tile p x 7 N-tiles, K = 16 (its own dX1 tile through a wave-private
//                                         LDS transpose; XIN fragments from HBM)
//    so no producer waits for another: the only hand-off is the chain's chunk barrier. Producer 0 also takes the
//    fc2 gradients (dW2[a_t] += dchosen_t h_t, VALU, per step of the chunk).
//  * waves 4, 5 (and 1 when NR = 1): pass the barriers.
// Outputs: per-workgroup slabs in gru_bwd_fused_kernel's layout ([w_ih | w_hh | b_ih | b_hh | fc2.w | fc2.b] and
// [fc1.w | fc1.b]), the workgroup's rows summed; the reduction takes ceil(R / NR) slabs.
// DWH = 1: workgroups past the rows compute dW_hyper tiles (dwh_body), as gru_bwd_fused_kernel<1>.
#pragma once
#include <type_traits>
#include "gru_bwd_fused.hpp"

namespace mq {

constexpr int BGP = G3 + 4;   // dgi history pitch

template <int NR>
struct alignas(16) BwdPairLds {
  float gh[NR][2][FCH][BRP];   // [row][chunk & 1][step]: dgh (3H) | h_{t-1} (H)
  float gi[NR][2][FCH][BGP];   // [row][chunk & 1][step]: dgi (3H) | dchosen_t, a_t (bits)
  float dxp[4][FCH][17];       // producer p's dX1 tile, transposed for dW1's A operand (wave-private)
  float db1[4][H];             // fc1 bias-grad partials of the four lane groups
  float dbr[NR][2][G3];        // the chains' b_ih / b_hh gradients
  float wih[G3][H + 1];        // W_ih, dX1's B operand (odd pitch: the lane groups read rows 48 apart)
  f32x4 cg[NR][2][FCH][H];     // [row][chunk & 1][step][unit]: the chain's gate record (r, z, n, W_hn h + b_hn)
  float chp[NR][2][FCH][H];    //   h_{t-1}
  float cdch[NR][2][FCH];      //   dchosen_t (0 for t >= T)
  int cact[NR][2][FCH];        //   a_t
};

inline size_t bwd_pair_dyn(int A) { return ((size_t)2 * A * H + A) * sizeof(float); }
inline bool bwd_pair_ok(int I, int O, int A, int n, int64_t RT) {
  return fused_bwd_ok(I, O, A, n, RT) && sizeof(BwdPairLds<1>) + bwd_pair_dyn(A) <= 160 * 1024;
}

// 256 threads, one workgroup per CU, so each wave has a SIMD to itself and 512 registers (VGPRs + AGPRs): the chain
// holds its whole W_hh column, the producers their accumulators.
template <int NR, int DWH = 0>
__global__ __launch_bounds__(256, 1) __attribute__((amdgpu_waves_per_eu(1, 1))) void gru_bwd_pair_kernel(Dims d, Rep rp, const float* __restrict__ P, Lay L,
                                                              Work w, int64_t slab_len, int64_t slab1_len) {
  constexpr int NP = 4 - NR;   // producer waves
  __shared__ BwdPairLds<NR> S;
  extern __shared__ float dyn[];   // W2 [A][H] | dW2 partial [A][H] | db2 [A]
  const int nrow_wg = (d.R + NR - 1) / NR;
  if constexpr (DWH != 0) {
    static_assert(sizeof(BwdPairLds<NR>) >= 4 * DWH_T * (DWH_T + 1) * sizeof(float), "dW_hyper tiles reuse LDS");
    if ((int)blockIdx.x >= nrow_wg) {
      dwh_body<8, 4>(d, L, w.dHYP, w.S0, w.slab_mix, w.dwh_len, w.dwh_ns, w.dwh_tj, (int)blockIdx.x - nrow_wg,
                        (int)threadIdx.x, (float*)&S);
      return;
    }
  }
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int R = d.R, A = d.A, T = d.T, Tp = d.Tp, I = d.I;
  const int cl = (Tp - 1) / FCH;
  float* w2_s = dyn;
  float* dw2_s = dyn + A * H;
  float* db2_s = dyn + 2 * A * H;
  const int64_t base = L.o[MQ_P_RNN_W_IH];
  const int64_t o_hh = L.o[MQ_P_RNN_W_HH] - base, o_bi = L.o[MQ_P_RNN_B_IH] - base,
                o_bh = L.o[MQ_P_RNN_B_HH] - base, o_w2 = L.o[MQ_P_FC2_W] - base, o_b2 = L.o[MQ_P_FC2_B] - base;
  float* slab = w.slab_rnn + (int64_t)blockIdx.x * slab_len;

  // ---- prologue: W2 in LDS, dW2 / db2 zeroed, both record buffers zeroed (the top chunk's rows past Tp stay 0)
  for (int i = tid; i < A * H; i += 256) { w2_s[i] = P[L.o[MQ_P_FC2_W] + i]; dw2_s[i] = 0.0f; }
  for (int i = tid; i < A; i += 256) db2_s[i] = 0.0f;
  for (int e = tid; e < NR * 2 * FCH * BRP; e += 256) (&S.gh[0][0][0][0])[e] = 0.0f;
  for (int e = tid; e < NR * 2 * FCH * BGP; e += 256) (&S.gi[0][0][0][0])[e] = 0.0f;

  // the chains' inputs of chunk cc (row z) into LDS buffer cc & 1: gate records, h_{t-1}, dchosen, actions
  // (coalesced 16-byte loads; staged a chunk ahead by the producers, the top chunk in the prologue)
  auto stage_inputs = [&](int cc, int z, int th, int nth) {   // nth >= 192: at most six elements a thread
    constexpr int SL = (FCH * H + 191) / 192;
    const int rr = min(NR * (int)blockIdx.x + z, R - 1), cb = cc & 1, t0 = FCH * cc;
    f32x4 gv[SL];
    float hv[SL];
#pragma unroll
    for (int q = 0; q < SL; ++q) {   // every load first: one round trip, not six
      const int e = min(th + nth * q, FCH * H - 1), i = e >> 6, u = e & 63, t = min(t0 + i, Tp - 1);
      const float* gp = w.Gates + ((int64_t)t * R + rr) * (4 * H) + u;
      gv[q] = f32x4{gp[0], gp[H], gp[2 * H], gp[3 * H]};
      hv[q] = w.Hs[((int64_t)max(t - 1, 0) * R + rr) * H + u];
    }
#pragma unroll
    for (int q = 0; q < SL; ++q) {
      const int e = th + nth * q, i = e >> 6, u = e & 63;
      if (e < FCH * H) {
        S.cg[z][cb][i][u] = gv[q];
        S.chp[z][cb][i][u] = t0 + i > 0 ? hv[q] : 0.0f;
      }
    }
    if (th < FCH) {
      const int t = t0 + th, b = (int)fdiv((uint32_t)rr, d.dN), ag = rr - b * d.n;
      S.cdch[z][cb][th] = t < T ? w.dch[(int64_t)t * R + rr] : 0.0f;
      const int a = t < Tp ? *(const int*)(rp.actions + (rp.ep(b) * d.t_stride + t) * d.n + ag) : 0;
      S.cact[z][cb][th] = min(max(a, 0), A - 1);
    }
  };
  for (int z = 0; z < NR; ++z) stage_inputs(cl, z, tid, 256);

  if (wv < NR) {
    // ================================================================ chain wave of row rr (wave z)
    const int z = wv, k = lane, rr = NR * (int)blockIdx.x + z;
    const bool live = rr < R;
    f32x2 wt[96];   // W_hh[2 m][k], W_hh[2 m + 1][k]: lane k's column, coalesced row loads
    {
      const float* Whh = P + L.o[MQ_P_RNN_W_HH] + k;
#pragma unroll
      for (int m = 0; m < 96; ++m) wt[m] = f32x2{Whh[(2 * m) * H], Whh[(2 * m + 1) * H]};
    }
    float carry = 0.0f;
    float dbi0 = 0.0f, dbi1 = 0.0f, dbi2 = 0.0f, dbh2 = 0.0f;   // b_hh's r / z gradients equal b_ih's
    drain_vmem();
    lds_barrier();   // prologue: W2 and the top chunk's inputs staged, records zeroed
    __builtin_amdgcn_s_setprio(2);
    for (int c = cl; c >= 0; --c) {
      const int cb = c & 1, pend = min(FCH, Tp - FCH * c);
      // step pend - 1's inputs; each step then reads the next one's (in this chunk) beside its mat-vec
      f32x4 gx = S.cg[z][cb][pend - 1][k];
      float hx = S.chp[z][cb][pend - 1][k];
      float dx = S.cdch[z][cb][pend - 1];
      int ax = S.cact[z][cb][pend - 1];
      for (int p = pend - 1; p >= 0; --p) {
        // the step's coefficients (gru_bwd_fused.hpp's linearised step); hp = 0 at t = 0 (staged)
        const float gr = gx[0], gz = gx[1], gn = gx[2], ghn = gx[3], hp = hx;
        const float an = (1.0f - gz) * (1.0f - gn * gn);
        const float ar = (an * ghn) * (gr * (1.0f - gr));
        const float az = (hp - gn) * (gz * (1.0f - gz));
        const float wd = dx * w2_s[ax * H + k];
        const float dh = carry + wd;
        const float gr_ = dh * ar, gz_ = dh * az, gn_ = dh * an, hn_ = gn_ * gr;
        float* gh = S.gh[z][cb][p];
        float* gi = S.gi[z][cb][p];
        gh[k] = gr_; gh[H + k] = gz_; gh[2 * H + k] = hn_; gh[3 * H + k] = hp;
        gi[k] = gr_; gi[H + k] = gz_; gi[2 * H + k] = gn_;
        if (k == 0) { gi[G3] = dx; gi[G3 + 1] = __int_as_float(ax); }   // for the producers' fc2 gradients
        dbi0 += gr_; dbi1 += gz_; dbi2 += gn_; dbh2 += hn_;
        asm volatile("" ::: "memory");   // the mat-vec reads other lanes' stores: not above them
        if (p > 0) {   // the next step's inputs, in flight under the mat-vec
          gx = S.cg[z][cb][p - 1][k];
          hx = S.chp[z][cb][p - 1][k];
          dx = S.cdch[z][cb][p - 1];
          ax = S.cact[z][cb][p - 1];
        }
        // dh_{t-1} = dh z + W_hh^T dgh: the 192 values just stored, read back by this wave (in-order LDS)
        f32x2 a0 = {0.0f, 0.0f}, a1 = {0.0f, 0.0f};
#pragma unroll
        for (int hh = 0; hh < 4; ++hh) {   // quarters: 12 broadcast b128 reads in flight, then 24 FMAs
          f32x4 dv[12];
#pragma unroll
          for (int q = 0; q < 12; ++q) dv[q] = *(const f32x4*)&gh[48 * hh + 4 * q];
#pragma unroll
          for (int q = 0; q < 12; ++q) {
            const int m = 24 * hh + 2 * q;
            a0 = pk_fma(wt[m], f32x2{dv[q][0], dv[q][1]}, a0);
            a1 = pk_fma(wt[m + 1], f32x2{dv[q][2], dv[q][3]}, a1);
          }
        }
        carry = fmaf(dh, gz, (a0.x + a0.y) + (a1.x + a1.y));
      }
      lds_barrier();   // chunk c's records complete; chunk c - 1's inputs staged
    }
    __builtin_amdgcn_s_setprio(0);
    if (!live) { dbi0 = dbi1 = dbi2 = dbh2 = 0.0f; }
    S.dbr[z][0][k] = dbi0; S.dbr[z][0][H + k] = dbi1; S.dbr[z][0][2 * H + k] = dbi2;
    S.dbr[z][1][k] = dbi0; S.dbr[z][1][H + k] = dbi1; S.dbr[z][1][2 * H + k] = dbh2;
    lds_barrier();   // final
  } else {
    // ================================================================== producer waves pw = 0 .. NP-1
    // tiles round-robin over the producers: dW_hh / dW_ih M-tiles (12), dX1 N-tiles and dW1 M-tiles (4)
    // NP = 3 (NR = 1): producer 0 owns dX1 / dW1 tiles 0 and 3 (152 MFMAs a chunk) and so only dW M-tiles 0, 1;
    // producers 1 and 2 own one dX1 / dW1 tile and five dW M-tiles each (216 / 236 / 236 MFMAs a chunk, against
    // 280 / 204 / 204 round-robin); producer 0 also takes the fc2 gradients
    static_assert(NR == 1 && NP == 3, "the producers' tile split and chunk-ahead prefetch assume one row per workgroup");
    // each producer's code is specialised on its index (tile ownership known at compile time: no branch around each
    // MFMA group, which also kept hipcc from scheduling LDS operand reads across groups, ISA round 5)
    auto producer = [&](auto pw_c) {
    constexpr int PW = decltype(pw_c)::value;
    constexpr int MT = 5, XT = PW == 0 ? 2 : 1;
    const int pw = PW;
    constexpr int mt0 = PW == 0 ? 0 : 2 + 5 * (PW - 1), mtn = PW == 0 ? 2 : 5;
    auto mtile = [&](int i) { return mt0 + i; };   // this wave's i-th dW M-tile
    auto mvalid = [&](int i) { return i < mtn; };
    constexpr int pfc2 = 0;   // the fc2 gradients go to the producer with the fewest MFMAs
    const int g = lane >> 4, c16 = lane & 15;
    const int Kq = (I + 15) / 16 * 4;
    const int nt1 = min(7, Kq / 4);   // dW1 N-tiles
    f32x4 acc_hh[MT][4], acc_ih[MT][4], acc_w1[XT][7];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) { acc_hh[i][jj] = f32x4{0, 0, 0, 0}; acc_ih[i][jj] = f32x4{0, 0, 0, 0}; }
#pragma unroll
    for (int x = 0; x < XT; ++x)
#pragma unroll
      for (int i = 0; i < 7; ++i) acc_w1[x][i] = f32x4{0, 0, 0, 0};
    float db1p[XT];
#pragma unroll
    for (int x = 0; x < XT; ++x) db1p[x] = 0.0f;
    {   // W_ih into LDS (the producers' threads, coalesced)
      const float* Wi = P + L.o[MQ_P_RNN_W_IH];
      for (int e = pw * 64 + lane; e < G3 * H; e += 64 * NP) S.wih[e / H][e % H] = Wi[e];
    }
    drain_vmem();
    lds_barrier();   // prologue (the matching barrier of the chains)
    if (cl >= 1) stage_inputs(cl - 1, 0, pw * 64 + lane, 64 * NP);
    const int rr = (int)blockIdx.x;
    // HBM fragments of a chunk, prefetched one chunk ahead (in flight across the barrier): X1 (dW_ih's B), the relu
    // mask of this wave's dX1 tiles, XIN (dW1's B), and (producer 0) h_t of the chunk's steps for the fc2 grads
    float x1b[4][4], x1m[XT][4], xib[4][7], hst[FCH];
    auto fetch = [&](int cc) {
      const int t0 = FCH * cc;
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        const int t = min(t0 + 4 * kb + g, Tp - 1);
        const float* xr = w.X1 + ((int64_t)t * R + rr) * H + c16;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) x1b[kb][jj] = t0 + 4 * kb + g < Tp ? xr[16 * jj] : 0.0f;
        const float* ir = w.XIN + ((int64_t)t * R + rr) * I;
#pragma unroll
        for (int nt = 0; nt < 7; ++nt) {
          const int col = 16 * nt + c16;
          xib[kb][nt] = (nt < nt1 && col < I) ? ir[col] : 0.0f;
        }
      }
#pragma unroll
      for (int x = 0; x < XT; ++x)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int t = min(t0 + 4 * g + e, Tp - 1);
          x1m[x][e] = w.X1[((int64_t)t * R + rr) * H + 16 * min(pw + NP * x, 3) + c16];
        }
      if constexpr (PW == pfc2) {
#pragma unroll
        for (int i = 0; i < FCH; ++i) hst[i] = w.Hs[((int64_t)min(t0 + i, Tp - 1) * R + rr) * H + lane];
      }
    };
    fetch(cl);
    for (int c = cl; c >= 0; --c) {
      lds_barrier();   // chunk c's records complete (the chains go on with chunk c - 1, whose inputs are staged)
      const int cb = c & 1, t0 = FCH * c;
      if (c >= 2)   // chunk c - 2's inputs into buffer c & 1, which the chains left at this barrier
        stage_inputs(c - 2, 0, pw * 64 + lane, 64 * NP);
      const int z = 0;
      // dW_hh += dGH^T H_prev (M-tiles pw, pw + NP, ..)
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        const float* ghr = S.gh[z][cb][4 * kb + g];
        float bv[4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) bv[jj] = ghr[3 * H + 16 * jj + c16];
#pragma unroll
        for (int i = 0; i < MT; ++i) {
          const int mt = mtile(i);
          if (mvalid(i)) {
            const float av = ghr[16 * mt + c16];
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) acc_hh[i][jj] = mfma16x4(av, bv[jj], acc_hh[i][jj]);
          }
        }
      }
      // dW_ih += dGI^T X1
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        const float* gir = S.gi[z][cb][4 * kb + g];
#pragma unroll
        for (int i = 0; i < MT; ++i) {
          const int mt = mtile(i);
          if (mvalid(i)) {
            const float av = gir[16 * mt + c16];
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) acc_ih[i][jj] = mfma16x4(av, x1b[kb][jj], acc_ih[i][jj]);
          }
        }
      }
#pragma unroll
      for (int x = 0; x < XT; ++x) {
        const int nt = pw + NP * x;   // dX1 N-tile = dW1 M-tile (fc1 units 16 nt ..)
        if (nt >= 4) break;
        // dX1 tile nt = dGI W_ih (two accumulators, K = 192)
        f32x4 dxa = {0, 0, 0, 0}, dxb = {0, 0, 0, 0};
#pragma unroll
        for (int m = 0; m < 12; ++m) {
          const f32x4 av = *(const f32x4*)&S.gi[z][cb][c16][48 * g + 4 * m];
          const float* wb = &S.wih[48 * g + 4 * m][16 * nt + c16];
          dxa = mfma16x4(av[0], wb[0], dxa);
          dxb = mfma16x4(av[1], wb[H + 1], dxb);
          dxa = mfma16x4(av[2], wb[2 * (H + 1)], dxa);
          dxb = mfma16x4(av[3], wb[3 * (H + 1)], dxb);
        }
        // relu'(X1), the fc1 bias gradient, and the tile transposed through this wave's LDS corner
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int i = 4 * g + e;
          const float v = (t0 + i < Tp && x1m[x][e] > 0.0f) ? dxa[e] + dxb[e] : 0.0f;
          db1p[x] += v;
          S.dxp[pw][i][c16] = v;
        }
        // other lanes' values come back below: keep hipcc from moving those reads above these writes (it may,
        // per-thread, where a lane's own addresses differ); the wave's LDS operations then run in order
        asm volatile("" ::: "memory");
        // dW1 += dX1^T XIN: A[i = unit c16][kk = step g]
#pragma unroll
        for (int kb = 0; kb < 4; ++kb) {
          const float av = S.dxp[pw][4 * kb + g][c16];
#pragma unroll
          for (int j = 0; j < 7; ++j)
            acc_w1[x][j] = mfma16x4(av, xib[kb][j], acc_w1[x][j]);   // zero B past I
        }
      }
      // fc2 gradients of the chunk's steps (producer pfc2): dW2[a_t][k] += dchosen_t h_t[k], t descending; dchosen
      // and a_t from the chain's records, h_t prefetched
      if constexpr (PW == pfc2) {
        const int hi = min(t0 + FCH, T) - 1;
#pragma unroll
        for (int i = FCH - 1; i >= 0; --i) {
          if (t0 + i > hi) continue;
          const float dchv = S.gi[z][cb][i][G3];
          const int a = __float_as_int(S.gi[z][cb][i][G3 + 1]);
          dw2_s[a * H + lane] += dchv * hst[i];
          if (lane == 0) db2_s[a] += dchv;
        }
      }
      if (c >= 1) fetch(c - 1);   // in flight across the next barrier
    }
    // slabs in the MFMA C layout: element (16 tile + 4 g + e, 16 tile' + c16)
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const int mt = mtile(i);
      if (!mvalid(i)) break;
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int m = 16 * mt + 4 * g + e, nn = 16 * jj + c16;
          slab[m * H + nn] = acc_ih[i][jj][e];
          slab[o_hh + m * H + nn] = acc_hh[i][jj][e];
        }
    }
    float* slab1 = w.slab_fc1 + (int64_t)blockIdx.x * slab1_len;
#pragma unroll
    for (int x = 0; x < XT; ++x) {
      const int nt = pw + NP * x;
      if (nt >= 4) break;
#pragma unroll
      for (int j = 0; j < 7; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int m = 16 * nt + 4 * g + e, nn = 16 * j + c16;
          if (j < nt1 && nn < I) slab1[m * I + nn] = acc_w1[x][j][e];
        }
      S.db1[g][16 * nt + c16] = db1p[x];
    }
    };
    const int pwr = wv - NR;
    if (pwr == 0) producer(std::integral_constant<int, 0>{});
    else if (pwr == 1) producer(std::integral_constant<int, 1>{});
    else producer(std::integral_constant<int, 2>{});
    lds_barrier();   // final
  }
  // after the final barrier: dW2 / db2, the chains' bias gradients (rows summed), the fc1 bias
  for (int i = tid; i < A * H; i += 256) slab[o_w2 + i] = dw2_s[i];
  for (int i = tid; i < A; i += 256) slab[o_b2 + i] = db2_s[i];
  for (int i = tid; i < 2 * G3; i += 256) {
    float v = 0.0f;
#pragma unroll
    for (int z = 0; z < NR; ++z) v += S.dbr[z][i / G3][i % G3];
    slab[(i < G3 ? o_bi : o_bh - G3) + i] = v;
  }
  if (tid < H)
    w.slab_fc1[(int64_t)blockIdx.x * slab1_len + H * I + tid] =
        (S.db1[0][tid] + S.db1[1][tid]) + (S.db1[2][tid] + S.db1[3][tid]);
}

// Host: ceil(R / NR) row workgroups (+ dW_hyper tiles when w.dwh_n > 0 and DWH = 1).
template <int NR>
inline void launch_bwd_pair(bool dwh, hipStream_t s, const Dims& d, const Rep& rp, const float* P, const Lay& L,
                            const Work& w, int64_t slab_len, int64_t slab1_len) {
  const int rows = (d.R + NR - 1) / NR;
  const size_t dyn = bwd_pair_dyn(d.A);
  if (dwh)
    hipLaunchKernelGGL((gru_bwd_pair_kernel<NR, 1>), dim3(rows + w.dwh_n), dim3(256), dyn, s, d, rp, P, L, w,
                       slab_len, slab1_len);
  else
    hipLaunchKernelGGL((gru_bwd_pair_kernel<NR, 0>), dim3(rows), dim3(256), dyn, s, d, rp, P, L, w, slab_len,
                       slab1_len);
}

}  // namespace mq
