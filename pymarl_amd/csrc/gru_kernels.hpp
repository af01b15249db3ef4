// Persistent per-row GRU recurrences (the serial T loop of QLearner.train, q_learner.py:49-52 / 60-62 / 101).
//
// Only the h -> h dependency is serial: the input side (fc1, W_ih) was hoisted into the row-parallel GEMMs, so
// each step here is the 64x192 W_hh mat-vec plus gate math (forward) or its transpose plus the gate
// derivatives (backward). A workgroup owns RW rows for the whole T loop; W_hh stays in VGPRs and the hidden /
// gate-gradient vectors round-trip through double-buffered LDS, one barrier per step.
//
// Thread map (256 threads): unit j = tid >> 2 (0..63), quarter q = tid & 3. The four lanes of a quad hold the
// four K-quarters of one hidden unit and meet in a DPP quad reduction (no LDS). Gate math for row i runs on the
// lane with q == i % 4, so RW = 4 keeps every lane busy.
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

// ------------------------------------------------------------------------------------------------ forward
// grid = (ceil(R / RW), 2 nets). Writes Q for both nets; Hs and Gates for the online net only.
// VAR: ablation bits for scripts/rec_micro.hip only (production = 0): 1 skip Hs/Gates stores, 2 skip fc2,
// 4 skip the GI prefetch (load at use).
template <int RW, int VAR = 0>
__global__ __launch_bounds__(256) void gru_fwd_kernel(Dims d, const float* __restrict__ P0,
                                                      const float* __restrict__ P1, Lay L, Work w) {
  constexpr int RL = (RW + 3) / 4;   // rows per lane in the gate phase
  const int z = blockIdx.y;
  const float* __restrict__ P = z ? P1 : P0;
  const int tid = threadIdx.x, j = tid >> 2, q = tid & 3;
  const int R = d.R, A = d.A;
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
  // fc2 role: action a = j (< A), same quarter split of K.
  const bool has_a = j < A;
  float w2[16];
  float b2 = 0.0f;
#pragma unroll
  for (int k = 0; k < 16; ++k) w2[k] = has_a ? P[L.o[MQ_P_FC2_W] + j * H + 16 * q + k] : 0.0f;
  if (has_a) b2 = P[L.o[MQ_P_FC2_B] + j];

  const int r0 = blockIdx.x * RW;
  for (int i = tid; i < RW * H; i += 256) hbuf[0][i / H][i % H] = 0.0f;   // init_hidden: h0 = 0

  const float* GI = w.GI + (int64_t)z * RT * G3;
  float* Q = w.Q + (int64_t)z * RT * A;
  float gi_r[RL], gi_z[RL], gi_n[RL];
  auto load_gi = [&](int t) {
#pragma unroll
    for (int ii = 0; ii < RL; ++ii) {
      const int i = 4 * ii + q, r = r0 + i;
      if (i < RW && r < R && t < d.Tp) {
        const float* g = GI + ((int64_t)t * R + r) * G3;
        gi_r[ii] = g[j]; gi_z[ii] = g[H + j]; gi_n[ii] = g[2 * H + j];
      } else {
        gi_r[ii] = gi_z[ii] = gi_n[ii] = 0.0f;
      }
    }
  };
  load_gi(0);
  drain_vmem();
  lds_barrier();

  for (int t = 0; t < d.Tp; ++t) {
    float cr[RL], cz[RL], cn[RL];
#pragma unroll
    for (int ii = 0; ii < RL; ++ii) { cr[ii] = gi_r[ii]; cz[ii] = gi_z[ii]; cn[ii] = gi_n[ii]; }
    if (!(VAR & 4)) load_gi(t + 1);   // prefetch the next step's input gates under this step's mat-vec

    float (*hb)[H] = hbuf[t & 1];
    float (*hn)[H] = hbuf[(t + 1) & 1];
    float sr[RW], sz[RW], sn[RW];
#pragma unroll
    for (int i = 0; i < RW; ++i) {
      const f32x4* hv4 = (const f32x4*)(&hb[i][16 * q]);
      float ar = 0.0f, az = 0.0f, an = 0.0f, ar2 = 0.0f, az2 = 0.0f, an2 = 0.0f;
#pragma unroll
      for (int k4 = 0; k4 < 4; ++k4) {
        const f32x4 hv = hv4[k4];
        ar = fmaf(wr[4 * k4 + 0], hv[0], ar); ar2 = fmaf(wr[4 * k4 + 1], hv[1], ar2);
        az = fmaf(wz[4 * k4 + 0], hv[0], az); az2 = fmaf(wz[4 * k4 + 1], hv[1], az2);
        an = fmaf(wn[4 * k4 + 0], hv[0], an); an2 = fmaf(wn[4 * k4 + 1], hv[1], an2);
        ar = fmaf(wr[4 * k4 + 2], hv[2], ar); ar2 = fmaf(wr[4 * k4 + 3], hv[3], ar2);
        az = fmaf(wz[4 * k4 + 2], hv[2], az); az2 = fmaf(wz[4 * k4 + 3], hv[3], az2);
        an = fmaf(wn[4 * k4 + 2], hv[2], an); an2 = fmaf(wn[4 * k4 + 3], hv[3], an2);
      }
      sr[i] = quad_sum(ar + ar2);
      sz[i] = quad_sum(az + az2);
      sn[i] = quad_sum(an + an2);
    }
#pragma unroll
    for (int ii = 0; ii < RL; ++ii) {
      const int i = 4 * ii + q, r = r0 + i;
      const float ghr = pick_row<RW>(sr, ii, q) + bhr;
      const float ghz = pick_row<RW>(sz, ii, q) + bhz;
      const float ghn = pick_row<RW>(sn, ii, q) + bhn;
      if (i < RW) {
        const float hp = hb[i][j];
        const float rg = sigmoidf_(ghr + cr[ii]);
        const float zg = sigmoidf_(ghz + cz[ii]);
        const float ng = tanhf_(cn[ii] + ghn * rg);
        const float h1 = (hp - ng) * zg + ng;   // ATen gru_cell: (hx - n) * z + n
        hn[i][j] = h1;
        if (!(VAR & 1) && z == 0 && r < R) {
          const int64_t tr = (int64_t)t * R + r;
          w.Hs[tr * H + j] = h1;
          float* g = w.Gates + tr * (4 * H);
          g[j] = rg; g[H + j] = zg; g[2 * H + j] = ng; g[3 * H + j] = ghn;
        }
      }
    }
    lds_barrier();
    if (VAR & 4) load_gi(t + 1);
    // fc2 on the new hidden state: q = W2 h + b2 (rnn_agent.py:35)
#pragma unroll
    for (int i = 0; i < (VAR & 2 ? 0 : RW); ++i) {
      const f32x4* hv4 = (const f32x4*)(&hn[i][16 * q]);
      float s = 0.0f, s2 = 0.0f;
#pragma unroll
      for (int k4 = 0; k4 < 4; ++k4) {
        const f32x4 hv = hv4[k4];
        s = fmaf(w2[4 * k4 + 0], hv[0], s); s2 = fmaf(w2[4 * k4 + 1], hv[1], s2);
        s = fmaf(w2[4 * k4 + 2], hv[2], s); s2 = fmaf(w2[4 * k4 + 3], hv[3], s2);
      }
      s = quad_sum(s + s2);
      const int r = r0 + i;
      if (has_a && q == 0 && r < R) Q[((int64_t)t * R + r) * A + j] = s + b2;
    }
  }
}

// ------------------------------------------------------------------------------------------------ backward
// BPTT over the online net (q_learner.py:100-101). grid = ceil(R / RW). Writes dGI for the dX1 GEMM and a
// per-workgroup partial slab [w_ih | w_hh | b_ih | b_hh | fc2.w | fc2.b] of the gradient.
template <int RW>
__global__ __launch_bounds__(256) void gru_bwd_kernel(Dims d, Rep rp, const float* __restrict__ P, Lay L,
                                                      Work w, int64_t slab_len) {
  constexpr int RL = (RW + 3) / 4;
  const int tid = threadIdx.x, k = tid >> 2, q = tid & 3;
  const int R = d.R, A = d.A;
  __shared__ float dgh_s[2][RW][G3];
  __shared__ float dgi_s[2][RW][G3];
  __shared__ float hp_s[2][RW][H];
  __shared__ float x1_s[2][RW][H];
  extern __shared__ float dyn[];   // dW2 partial [A][H] then db2 [A]
  float* dw2_s = dyn;
  float* db2_s = dyn + A * H;

  const float* Whh = P + L.o[MQ_P_RNN_W_HH];
  const float* W2 = P + L.o[MQ_P_FC2_W];
  float wT[48], accH[48], accI[48];
#pragma unroll
  for (int c = 0; c < 48; ++c) {
    wT[c] = Whh[(48 * q + c) * H + k];
    accH[c] = 0.0f;
    accI[c] = 0.0f;
  }
  for (int i = tid; i < A * H + A; i += 256) dyn[i] = 0.0f;

  const int r0 = blockIdx.x * RW;
  float carry[RL], cz[RL], ht[RL];
  float dbi0 = 0, dbi1 = 0, dbi2 = 0, dbh2 = 0;
#pragma unroll
  for (int ii = 0; ii < RL; ++ii) { carry[ii] = 0.0f; cz[ii] = 0.0f; ht[ii] = 0.0f; }
  drain_vmem();
  lds_barrier();

  for (int t = d.Tp - 1; t >= 0; --t) {
    const int pb = t & 1;
    int pa[RL];
    float pv[RL], pd[RL];
#pragma unroll
    for (int ii = 0; ii < RL; ++ii) {
      const int i = 4 * ii + q, r = r0 + i;
      pa[ii] = -1;
      pv[ii] = pd[ii] = 0.0f;
      if (i >= RW) continue;
      float dh = carry[ii], gr = 0, gz = 0, gn = 0, ghn = 0, hp = 0, x1 = 0;
      if (r < R) {
        const int64_t tr = (int64_t)t * R + r;
        if (t < d.T) {
          const int b = (int)fdiv((uint32_t)r, d.dN), ag = r - b * d.n;
          const float dchv = w.dch[(int64_t)t * R + r];
          const int a = (int)rp.actions[(rp.ep(b) * d.t_stride + t) * d.n + ag];
          dh += dchv * W2[a * H + k];
          pa[ii] = a;
          pv[ii] = dchv * ht[ii];   // dW2[a][k] += dchosen * h_t[k]
          pd[ii] = dchv;
        }
        const float* g = w.Gates + tr * (4 * H);
        gr = g[k]; gz = g[H + k]; gn = g[2 * H + k]; ghn = g[3 * H + k];
        hp = t > 0 ? w.Hs[(tr - R) * H + k] : 0.0f;
        x1 = w.X1[tr * H + k];
      }
      const float dn = dh * (1.0f - gz);
      const float dz = dh * (hp - gn);
      const float dan = dn * (1.0f - gn * gn);
      const float dar = (dan * ghn) * (gr * (1.0f - gr));
      const float daz = dz * (gz * (1.0f - gz));
      if (r < R) {
        float* o = w.dGI + ((int64_t)t * R + r) * G3;
        o[k] = dar; o[H + k] = daz; o[2 * H + k] = dan;
      }
      dgi_s[pb][i][k] = dar; dgi_s[pb][i][H + k] = daz; dgi_s[pb][i][2 * H + k] = dan;
      dgh_s[pb][i][k] = dar; dgh_s[pb][i][H + k] = daz; dgh_s[pb][i][2 * H + k] = dan * gr;
      hp_s[pb][i][k] = hp;
      x1_s[pb][i][k] = x1;
      dbi0 += dar; dbi1 += daz; dbi2 += dan; dbh2 += dan * gr;
      cz[ii] = dh * gz;
      ht[ii] = hp;   // h_{t-1} is the next (earlier) step's h_t
    }
    // fc2 gradient into LDS; the four lanes of a quad share unit k and may share an action, so they take
    // turns (separate instructions) instead of racing on the same word.
#pragma unroll
    for (int ii = 0; ii < RL; ++ii) {
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2) {
        if (q == s2 && pa[ii] >= 0) {
          dw2_s[pa[ii] * H + k] += pv[ii];
          if (k == 0) db2_s[pa[ii]] += pd[ii];
        }
        __builtin_amdgcn_wave_barrier();
      }
    }
    lds_barrier();
    float s[RW];
#pragma unroll
    for (int i = 0; i < RW; ++i) {
      const f32x4* dg4 = (const f32x4*)(&dgh_s[pb][i][48 * q]);
      const f32x4* di4 = (const f32x4*)(&dgi_s[pb][i][48 * q]);
      const float hpk = hp_s[pb][i][k], x1k = x1_s[pb][i][k];
      float a0 = 0.0f, a1 = 0.0f;
#pragma unroll
      for (int c4 = 0; c4 < 12; ++c4) {
        const f32x4 dg = dg4[c4], di = di4[c4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int c = 4 * c4 + e;
          if (e & 1) a1 = fmaf(wT[c], dg[e], a1); else a0 = fmaf(wT[c], dg[e], a0);
          accH[c] = fmaf(dg[e], hpk, accH[c]);
          accI[c] = fmaf(di[e], x1k, accI[c]);
        }
      }
      s[i] = quad_sum(a0 + a1);
    }
#pragma unroll
    for (int ii = 0; ii < RL; ++ii) carry[ii] = cz[ii] + pick_row<RW>(s, ii, q);
  }

  // per-workgroup partial slab
  float* slab = w.slab_rnn + (int64_t)blockIdx.x * slab_len;
  const int64_t base = L.o[MQ_P_RNN_W_IH];
  const int64_t o_ih = 0, o_hh = L.o[MQ_P_RNN_W_HH] - base, o_bi = L.o[MQ_P_RNN_B_IH] - base,
                o_bh = L.o[MQ_P_RNN_B_HH] - base, o_w2 = L.o[MQ_P_FC2_W] - base, o_b2 = L.o[MQ_P_FC2_B] - base;
#pragma unroll
  for (int c = 0; c < 48; ++c) {
    slab[o_ih + (48 * q + c) * H + k] = accI[c];
    slab[o_hh + (48 * q + c) * H + k] = accH[c];
  }
  dbi0 = quad_sum(dbi0); dbi1 = quad_sum(dbi1); dbi2 = quad_sum(dbi2); dbh2 = quad_sum(dbh2);
  if (q == 0) {
    slab[o_bi + k] = dbi0; slab[o_bi + H + k] = dbi1; slab[o_bi + 2 * H + k] = dbi2;
    slab[o_bh + k] = dbi0; slab[o_bh + H + k] = dbi1; slab[o_bh + 2 * H + k] = dbh2;
  }
  lds_barrier();
  for (int i = tid; i < A * H; i += 256) slab[o_w2 + i] = dw2_s[i];
  for (int i = tid; i < A; i += 256) slab[o_b2 + i] = db2_s[i];
}

}  // namespace mq
