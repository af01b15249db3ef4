// EXPERIMENT, not part of the library (scripts/chain_micro.hip only). Measured at cfg2 on MI355X
// (profiles/r03_chain_micro.txt): slabs equal to the production kernel's to 3.7e-8 relative, but 169.7 us against
// 88.9 us; a stripped one-wave chain alone (no producers) takes 120-130 us. One wave cannot issue the 96 pk_fma +
// 48 LDS broadcasts + gate math of a step faster than four waves sharing it plus their barrier: refuted.
//
// Fused BPTT with a ONE-WAVE dh chain (q_learner.py:100-101 through rnn_agent.py:24-28): the same arithmetic and
// slabs as gru_bwd_fused.hpp, re-partitioned so the serial chain never waits on another wave within a step.
//
// gru_bwd_fused.hpp spreads the chain over four waves (lane = unit x quarter of K): every step ends in an s_barrier
// of all eight waves, because the four chain waves exchange dgh through LDS, and the producer waves' f32 MFMAs run
// on the chain's SIMDs. Measured at cfg2 (scripts/chain_micro.hip): 1,420 cycles a step, of which 333 waiting at the
// barrier and 478 in the dgh reads; alone (producers idle) 1,050.
//
// Here (512 threads, waves w and w + 4 share a SIMD):
//  * wave 0, the chain: lane j owns hidden unit j for the whole T loop: W_hh column j in 96 VGPR pairs, the gate
//    derivatives of unit j, the step's records to LDS, and the W_hh^T mat-vec over all 192 dgh values, read back as
//    48 LDS broadcasts. One wave publishes and consumes its own records, and a wave's LDS operations complete in
//    order: no barrier, no flag, no DPP inside a step;
//  * wave 4 (the chain's SIMD): no work, so nothing shares the chain's issue slots;
//  * waves 1, 2, 3, 5, 6, 7 (SIMDs 1 - 3, two each): the producers. They work on whole 16-step chunks, one chunk
//    behind the chain, and meet it at ONE s_barrier per chunk: at the end of the chain's chunk c, the producers have
//    finished chunk c + 1 (its record buffer is free for chunk c - 1) and take chunk c.
//      producer p = 0 .. 3:  dW_hh and dW_ih for gate-row tile p, dX1 for hidden-unit tile p (K = 192, W_ih slice
//                            in VGPRs), relu', db1, dW1 for unit tile p, fc2's grads for units 16 p .. 16 p + 15
//      producer p = 4, 5:    dW_hh and dW_ih for gate-row tiles 4 .. 7 / 8 .. 11
//    (108 / 128 v_mfma_f32_16x16x4_f32 per chunk and wave), and they stage the next chunk's X1 / XIN rows.
// Per-step record (LDS): [dr | dz | dn | dn * r | h_{t-1}], dr = d(a_r), dz = d(a_z), dn = d(a_n): dGI = the first
// three, dGH = (dr, dz, dn * r).
//
// Accumulation orders: every MFMA accumulator takes its chunks in the default kernel's order; the chain's mat-vec
// sums the 192 terms in four interleaved partial sums (the default: 4-way K split + DPP quad sum), so dh differs
// from gru_bwd_fused_kernel's by rounding only.
#pragma once
#include "../pymarl_amd/csrc/gru_bwd_fused.hpp"

namespace mq {

constexpr int W1RP = 5 * H + 4;   // record row pitch

struct BwdW1Lds {
  float rec[2][FCH][W1RP];    // per step [dr | dz | dn | dn r | h_{t-1}], chunk-double-buffered
  float x1[2][FCH][H + 4];    // X1 rows of a chunk (double-buffered: staged one chunk ahead)
  float xin[2][FCH][FXP];     // XIN rows of a chunk, zero-padded to 4 * Kq
  float dx1[FCH][H + 4];      // dX1 of the chunk (each producer 0..3 its own 16 columns)
  float db1[4][H];            // fc1 bias-grad partials of the four lane groups
  float hnext[H];             // h of the first step of the chunk processed last (fc2's operand)
  float wih[G3][H + 1];       // W_ih (dX1's B operand); odd pitch: the four lane groups read rows 48 apart
  f32x2 whn[H / 2][H];        // the chain's W_hh n-gate rows: [k / 2][unit j] = W_hh[128 + k .. + 1][j]
};

// The chain's mat-vec is written with inline asm (LDS reads, waits, packed FMAs): as plain C++ the compiler issues
// every LDS read of the step up front (256 VGPRs of results beside the W_hh column) and spills the column. Volatile
// asm keeps program order, so the reads are software-pipelined one group ahead with exact lgkmcnt waits (LDS
// operations of a wave complete in order; no scalar-memory load is issued inside the region).
MQ_DEV uint32_t lds_off(const void* p) { return (uint32_t)(uintptr_t)p; }
MQ_DEV f32x2 ds_b64(uint32_t a) {
  f32x2 v;
  asm volatile("ds_read_b64 %0, %1" : "=v"(v) : "v"(a) : "memory");
  return v;
}
template <int N>
MQ_DEV void lgkm_wait() { asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory"); }
MQ_DEV void pk_fma_asm(f32x2& acc, const f32x2& a, const f32x2& b) {
  asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
}

// gate-row tile m (16 rows of the 192 W_hh / W_ih rows) -> its dGH column in the record ([dr | dz | dn r] live at
// columns 0..127 and 192..255)
MQ_DEV int w1_ghcol(int m) { return m < 8 ? 16 * m : 16 * m + 64; }

template <int VAR = 0>
__global__ __launch_bounds__(512) void gru_bwd_w1_kernel(Dims d, Rep rp, const float* __restrict__ P, Lay L, Work w,
                                                         int64_t slab_len, int64_t slab1_len) {
  __shared__ BwdW1Lds S;
  extern __shared__ float dyn[];   // W2 [A][H] | dW2 partial [A][H] | db2 [A]
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int R = d.R, A = d.A, T = d.T, Tp = d.Tp, I = d.I;
  const int cl = (Tp - 1) / FCH;
  const int r = blockIdx.x;
  float* w2_s = dyn;
  float* dw2_s = dyn + A * H;
  float* db2_s = dyn + 2 * A * H;
  {
    constexpr int NW2 = 16 * H / 512;
    float v[NW2];
#pragma unroll
    for (int u = 0; u < NW2; ++u) v[u] = tid + 512 * u < A * H ? P[L.o[MQ_P_FC2_W] + tid + 512 * u] : 0.0f;
#pragma unroll
    for (int u = 0; u < NW2; ++u)
      if (tid + 512 * u < A * H) { w2_s[tid + 512 * u] = v[u]; dw2_s[tid + 512 * u] = 0.0f; }
  }
  for (int i = tid; i < A; i += 512) db2_s[i] = 0.0f;
  // the top (partial) chunk's rows past Tp are read by the producers: zero records and the XIN padding
  for (int e = tid; e < 2 * FCH * W1RP; e += 512) (&S.rec[0][0][0])[e] = 0.0f;
  for (int e = tid; e < 2 * FCH * FXP; e += 512) (&S.xin[0][0][0])[e] = 0.0f;
  {
    constexpr int NW = G3 * H / 512;   // W_ih to LDS, all loads in flight first
    float v[NW];
#pragma unroll
    for (int u = 0; u < NW; ++u) v[u] = P[L.o[MQ_P_RNN_W_IH] + tid + 512 * u];
#pragma unroll
    for (int u = 0; u < NW; ++u) {
      const int e = tid + 512 * u, m = e / H;
      S.wih[m][e - m * H] = v[u];
    }
  }

  for (int e = tid; e < H * H; e += 512) {   // W_hh n-gate rows, column-paired for the chain's per-lane reads
    const int k = e / H, jj = e - k * H;
    ((float*)&S.whn[k >> 1][jj])[k & 1] = P[L.o[MQ_P_RNN_W_HH] + (int64_t)(2 * H + k) * H + jj];
  }

  const int b = (int)fdiv((uint32_t)r, d.dN), ag = r - b * d.n;
  const int64_t* arow = rp.actions + rp.ep(b) * d.t_stride * d.n + ag;   // &actions[ep(b)][0][agent]
  const int64_t base = L.o[MQ_P_RNN_W_IH];
  float* slab = w.slab_rnn + (int64_t)blockIdx.x * slab_len;
  const int64_t o_hh = L.o[MQ_P_RNN_W_HH] - base, o_bi = L.o[MQ_P_RNN_B_IH] - base,
                o_bh = L.o[MQ_P_RNN_B_HH] - base, o_w2 = L.o[MQ_P_FC2_W] - base, o_b2 = L.o[MQ_P_FC2_B] - base;

  if ((VAR & 1) ? wave != 0 : (VAR & 2) ? wave == 0 : false) {
    // diagnostic builds (spill isolation): this role only meets the barriers
    lds_barrier();
    for (int c = cl; c >= 0; --c) lds_barrier();
  } else if (wave == 0) {
    // ================================================================ the chain: lane j = hidden unit j
    const int j = lane;
    // {W_hh[k][j], W_hh[k + 1][j]}, k = 0, 2, .., 126 (the r and z rows) in VGPRs; the n rows come from LDS
    // (S.whn) each step: 192 VGPRs of W_hh would leave too few for the rest of the step
    f32x2 wp[64];
    {
      const float* Whh = P + L.o[MQ_P_RNN_W_HH];
#pragma unroll
      for (int i = 0; i < 64; ++i) wp[i] = f32x2{Whh[(2 * i) * H + j], Whh[(2 * i + 1) * H + j]};
    }
    struct In { float gr, gz, gn, ghn, hp, dch; int a; };
    // per-lane records through wave-uniform buffer descriptors + 32-bit lane offsets; dchosen and the action are
    // wave-uniform (one row): read into SGPRs, so a slot costs five VGPRs next to the 192 of W_hh's column
    const uint32_t R4H = (uint32_t)R * 4 * H, RH = (uint32_t)R * H;
    const auto grs = buf_rsrc(w.Gates + (int64_t)r * (4 * H));
    const auto hrs = buf_rsrc(w.Hs + (int64_t)r * H);
    auto load = [&](int t, In& s) {   // step t's inputs (t clamped: edges are masked where used)
      const uint32_t tc = (uint32_t)max(t, 0);
      const uint32_t go = (tc * R4H + (uint32_t)j) * 4;
      s.gr = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(grs, go, 0, 0));
      s.gz = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(grs, go + 4 * H, 0, 0));
      s.gn = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(grs, go + 8 * H, 0, 0));
      s.ghn = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(grs, go + 12 * H, 0, 0));
      s.hp = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                           hrs, ((tc > 0 ? tc - 1 : 0) * RH + (uint32_t)j) * 4, 0, 0));
      s.dch = __builtin_bit_cast(
          float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, w.dch[(int64_t)min((int)tc, T - 1) * R + r])));
      s.a = __builtin_amdgcn_readfirstlane(*(const int*)(arow + (int64_t)tc * d.n));
    };
    float carry = 0.0f, db_r = 0.0f, db_z = 0.0f, db_in = 0.0f, db_hn = 0.0f;
    auto step = [&](int t, const In& cur, In& ahead, int dist) {
      load(t - dist, ahead);
      const int p = t & (FCH - 1), cb = (t / FCH) & 1;
      const float w2 = w2_s[cur.a * H + j];
      const float hp = t > 0 ? cur.hp : 0.0f;
      const float dchv = t < T ? cur.dch : 0.0f;
      const float dh = carry + dchv * w2;
      const float dn = dh * (1.0f - cur.gz);
      const float dz = dh * (hp - cur.gn);
      const float dan = dn * (1.0f - cur.gn * cur.gn);
      const float dar = (dan * cur.ghn) * (cur.gr * (1.0f - cur.gr));
      const float daz = dz * (cur.gz * (1.0f - cur.gz));
      const float dhn = dan * cur.gr;
      float* rw = &S.rec[cb][p][0];
      rw[j] = dar; rw[H + j] = daz; rw[2 * H + j] = dan; rw[3 * H + j] = dhn; rw[4 * H + j] = hp;
      db_r += dar; db_z += daz; db_in += dan; db_hn += dhn;
      // dh_{t-1} = dh z + W_hh^T dgh: the 192 dGH values of this step (this wave's own stores, in LDS order)
      const f32x4* g4 = (const f32x4*)rw;
      // groups of eight LDS reads: 0..7 the r / z dGH pairs (W from VGPRs), 8..15 four n dGH pairs + their four
      // W_hh pairs from S.whn; group g + 1 in flight while group g's FMAs run
      f32x2 a0 = {0.0f, 0.0f}, a1 = {0.0f, 0.0f}, a2 = {0.0f, 0.0f}, a3 = {0.0f, 0.0f};
      const uint32_t rb = lds_off(rw), wb = lds_off(&S.whn[0][j]);
      f32x2 buf[2][8];
      auto issue = [&](int gi, f32x2 (&dst)[8]) {
        if (gi < 8) {
#pragma unroll
          for (int q = 0; q < 8; ++q) dst[q] = ds_b64(rb + 8 * (8 * gi + q));
        } else {
          const int h = gi - 8;
#pragma unroll
          for (int q = 0; q < 4; ++q) dst[q] = ds_b64(rb + 4 * 192 + 8 * (4 * h + q));
#pragma unroll
          for (int q = 0; q < 4; ++q) dst[4 + q] = ds_b64(wb + 8 * H * (4 * h + q));
        }
      };
      auto fmas = [&](int gi, const f32x2 (&v)[8]) {
        if (gi < 8) {
#pragma unroll
          for (int q = 0; q < 8; q += 4) {
            pk_fma_asm(a0, wp[8 * gi + q], v[q]);
            pk_fma_asm(a1, wp[8 * gi + q + 1], v[q + 1]);
            pk_fma_asm(a2, wp[8 * gi + q + 2], v[q + 2]);
            pk_fma_asm(a3, wp[8 * gi + q + 3], v[q + 3]);
          }
        } else {
          pk_fma_asm(a0, v[4], v[0]);
          pk_fma_asm(a1, v[5], v[1]);
          pk_fma_asm(a2, v[6], v[2]);
          pk_fma_asm(a3, v[7], v[3]);
        }
      };
      issue(0, buf[0]);
#pragma unroll
      for (int gi = 0; gi < 16; ++gi) {
        if (gi + 1 < 16) {
          issue(gi + 1, buf[(gi + 1) & 1]);
          lgkm_wait<8>();
        } else {
          lgkm_wait<0>();
        }
        fmas(gi, buf[gi & 1]);
      }
      carry = dh * cur.gz + (((a0.x + a0.y) + (a1.x + a1.y)) + ((a2.x + a2.y) + (a3.x + a3.y)));
      if (p == 0) lds_barrier();   // end of chunk t / 16: the producers take it
    };
    In sa, sb;   // two slots: step t's inputs are loaded during step t + 1
    load(Tp - 1, sa);
    drain_vmem();
    lds_barrier();   // prologue: LDS initialised
    int t = Tp - 1;
    for (; t - 1 >= 0; t -= 2) {
      step(t, sa, sb, 1);
      step(t - 1, sb, sa, 1);
    }
    if (t >= 0) step(t, sa, sb, 1);
    slab[o_bi + j] = db_r; slab[o_bi + H + j] = db_z; slab[o_bi + 2 * H + j] = db_in;
    slab[o_bh + j] = db_r; slab[o_bh + H + j] = db_z; slab[o_bh + 2 * H + j] = db_hn;
  } else if (wave == 4) {
    // ================================================================ the chain's SIMD partner: barriers only
    lds_barrier();
    for (int c = cl; c >= 0; --c) lds_barrier();
  } else {
    // ================================================================ producers pw = 0 .. 5
    const int pw = wave < 4 ? wave - 1 : wave - 2;
    const int pt = 64 * pw + lane;   // producer thread 0 .. 383
    const int g = lane >> 4, c16 = lane & 15;
    const int Kq = (I + 15) / 16 * 4;
    // X1 / XIN rows of a chunk: slot s covers element pt + 384 s of [16][H] and of [16][I]
    constexpr int NX1 = (FCH * H + 383) / 384, NXI = (FCH * 4 * FKQ + 383) / 384;
    float rx1[NX1], rxi[NXI];
    auto issue_rows = [&](int C) {
      const int t0 = FCH * C;
#pragma unroll
      for (int s = 0; s < NX1; ++s) {
        const int e = pt + 384 * s, i = e / H, col = e - i * H, t = min(t0 + i, Tp - 1);
        rx1[s] = e < FCH * H ? w.X1[((int64_t)t * R + r) * H + col] : 0.0f;
      }
#pragma unroll
      for (int s = 0; s < NXI; ++s) {
        const int e = opaque(pt + 384 * s), i = (int)fdiv((uint32_t)e, d.dI), col = e - i * I;
        const int t = min(t0 + i, Tp - 1);
        rxi[s] = e < FCH * I ? w.XIN[((int64_t)t * R + r) * I + col] : 0.0f;
      }
    };
    auto store_rows = [&](int C) {
      const int t0 = FCH * C, cb = C & 1;
#pragma unroll
      for (int s = 0; s < NX1; ++s) {
        const int e = pt + 384 * s, i = e / H, col = e - i * H;
        if (e < FCH * H) S.x1[cb][i][col] = t0 + i < Tp ? rx1[s] : 0.0f;
      }
#pragma unroll
      for (int s = 0; s < NXI; ++s) {
        const int e = opaque(pt + 384 * s), i = (int)fdiv((uint32_t)e, d.dI), col = e - i * I;
        if (e < FCH * I) S.xin[cb][i][col] = t0 + i < Tp ? rxi[s] : 0.0f;
      }
    };
    // dW_hh / dW_ih for NM gate-row tiles m0 .. m0 + NM - 1 x all 4 hidden tiles; K = the chunk's 16 steps,
    // kk = 4 kb + g
    auto dw_rec = [&](int C, bool ih, int m0, auto& acc) {
      constexpr int NM = sizeof(acc) / sizeof(acc[0]);
      const int cb = C & 1;
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        const int row = 4 * kb + g;
        const float* rr = &S.rec[cb][row][0];
        float bv[4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) bv[jj] = ih ? S.x1[cb][row][16 * jj + c16] : rr[4 * H + 16 * jj + c16];
#pragma unroll
        for (int i = 0; i < NM; ++i) {
          const int m = m0 + i;
          const float av = rr[(ih ? 16 * m : w1_ghcol(m)) + c16];
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) acc[i][jj] = mfma16x4(av, bv[jj], acc[i][jj]);
        }
      }
    };
    auto write_tiles = [&](int m0, auto& acc_ih, auto& acc_hh) {   // MFMA C layout: (16 tile + 4 g + e, 16 jj + c16)
      constexpr int NM = sizeof(acc_ih) / sizeof(acc_ih[0]);
#pragma unroll
      for (int i = 0; i < NM; ++i)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int m = 16 * (m0 + i) + 4 * g + e, nn = 16 * jj + c16;
            slab[m * H + nn] = acc_ih[i][jj][e];
            slab[o_hh + m * H + nn] = acc_hh[i][jj][e];
          }
    };
    issue_rows(cl);
    drain_vmem();
    lds_barrier();   // prologue: LDS initialised
    store_rows(cl);  // published to every producer by the first chunk barrier
    if (pw < 4) {
      // ---- dX1 / dW1 / fc2 owner of hidden-unit tile pw, + dW_hh / dW_ih gate-row tile pw
      f32x4 acc_hh[1][4], acc_ih[1][4], acc_w1[7];
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) { acc_hh[0][jj] = f32x4{0, 0, 0, 0}; acc_ih[0][jj] = f32x4{0, 0, 0, 0}; }
#pragma unroll
      for (int i = 0; i < 7; ++i) acc_w1[i] = f32x4{0, 0, 0, 0};
      float db1p = 0.0f;
      // fc2 grads of chunk C's steps, t descending: dW2[a][k] += dchosen_t h_t[k], h_t = the h_{t-1} record of
      // step t + 1; lane (k = 16 pw + (lane >> 2), q = lane & 3) owns the actions a = q (mod 4) of unit k
      const int kf = 16 * pw + (lane >> 2), qf = lane & 3;
      auto fc2_chunk = [&](int C) {
        const int cb = C & 1, t0 = FCH * C;
#pragma unroll
        for (int p = FCH - 1; p >= 0; --p) {
          const int t = t0 + p;
          if (t >= T) continue;
          const float hn = p < FCH - 1 ? S.rec[cb][p + 1][4 * H + kf] : S.hnext[kf];
          const float dchv = w.dch[(int64_t)t * R + r];
          const int a = *(const int*)(arow + (int64_t)t * d.n);
          if ((a & 3) == qf) {
            dw2_s[a * H + kf] += dchv * hn;
            if (kf == 0) db2_s[a] += dchv;
          }
        }
        if (qf == 0) S.hnext[kf] = S.rec[cb][0][4 * H + kf];   // h_{16 C - 1}: read by chunk C - 1's last step
      };
      auto dx_chunk = [&](int C) {   // dX1 tile pw = (dGI W_ih)[16][16 pw ..] o relu'(X1), db1, dW1 tile pw
        const int cb = C & 1;
        f32x4 dxa = {0, 0, 0, 0}, dxb = {0, 0, 0, 0};
#pragma unroll
        for (int m = 0; m < 12; ++m) {
          const f32x4 av = *(const f32x4*)&S.rec[cb][c16][48 * g + 4 * m];
          const float* wb = &S.wih[48 * g + 4 * m][16 * pw + c16];
          dxa = mfma16x4(av[0], wb[0], dxa);
          dxb = mfma16x4(av[1], wb[H + 1], dxb);
          dxa = mfma16x4(av[2], wb[2 * (H + 1)], dxa);
          dxb = mfma16x4(av[3], wb[3 * (H + 1)], dxb);
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int i = 4 * g + e, col = 16 * pw + c16;
          const float v = S.x1[cb][i][col] > 0.0f ? dxa[e] + dxb[e] : 0.0f;
          S.dx1[i][col] = v;   // this wave's own columns: read back below by this wave only
          db1p += v;
        }
#pragma unroll
        for (int kb = 0; kb < 4; ++kb) {
          const int row = 4 * kb + g;
          const float av = S.dx1[row][16 * pw + c16];
#pragma unroll
          for (int nt = 0; nt < 7; ++nt) {
            if (16 * nt >= 4 * Kq) break;
            acc_w1[nt] = mfma16x4(av, S.xin[cb][row][16 * nt + c16], acc_w1[nt]);
          }
        }
      };
      for (int c = cl; c >= 0; --c) {
        lds_barrier();   // the chain has published chunk c; every producer has finished chunk c + 1
        if (c > 0) issue_rows(c - 1);
        dw_rec(c, false, pw, acc_hh);
        dw_rec(c, true, pw, acc_ih);
        dx_chunk(c);
        fc2_chunk(c);
        if (c > 0) store_rows(c - 1);   // buffer (c - 1) & 1: chunk c + 1's, finished before this chunk's barrier
      }
      write_tiles(pw, acc_ih, acc_hh);
      float* slab1 = w.slab_fc1 + (int64_t)blockIdx.x * slab1_len;
#pragma unroll
      for (int nt = 0; nt < 7; ++nt)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int m = 16 * pw + 4 * g + e, nn = 16 * nt + c16;
          if (nn < I) slab1[m * I + nn] = acc_w1[nt][e];
        }
      S.db1[g][16 * pw + c16] = db1p;
    } else {
      // ---- dW_hh / dW_ih gate-row tiles 4 .. 7 (pw 4) or 8 .. 11 (pw 5)
      const int m0 = 4 * (pw - 3);
      f32x4 acc_hh[4][4], acc_ih[4][4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) { acc_hh[i][jj] = f32x4{0, 0, 0, 0}; acc_ih[i][jj] = f32x4{0, 0, 0, 0}; }
      for (int c = cl; c >= 0; --c) {
        lds_barrier();
        if (c > 0) issue_rows(c - 1);
        dw_rec(c, false, m0, acc_hh);
        dw_rec(c, true, m0, acc_ih);
        if (c > 0) store_rows(c - 1);
      }
      write_tiles(m0, acc_ih, acc_hh);
    }
  }
  lds_barrier();
  for (int i = tid; i < A * H; i += 512) slab[o_w2 + i] = dw2_s[i];
  for (int i = tid; i < A; i += 512) slab[o_b2 + i] = db2_s[i];
  if (tid < H)
    w.slab_fc1[(int64_t)blockIdx.x * slab1_len + H * I + tid] =
        (S.db1[0][tid] + S.db1[1][tid]) + (S.db1[2][tid] + S.db1[3][tid]);
}

inline void launch_bwd_w1(dim3 grid, size_t dyn, hipStream_t s, const Dims& d, const Rep& rp, const float* P,
                          const Lay& L, const Work& w, int64_t slab_len, int64_t slab1_len) {
  hipLaunchKernelGGL(gru_bwd_w1_kernel<0>, grid, dim3(512), dyn, s, d, rp, P, L, w, slab_len, slab1_len);
}

}  // namespace mq
