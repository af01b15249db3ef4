// The learner's row-parallel and weight-gradient contractions as policies of gemm_f32_kernel.
//
// Forward (grid.z = net: 0 online, 1 target; both nets read the same replay rows):
//   Fc1Prob : X1 = relu(xin W1^T + b1), xin = [obs_t | onehot(a_{t-1}) | onehot(agent)] built on the fly from the
//             replay rows gathered by episode id (BasicMAC._build_inputs, basic_controller.py:100-135; fc1 + relu,
//             rnn_agent.py:32); the online pass also writes xin densely (XIN) for the dW1 contraction
//   GiProb  : GI = X1 W_ih^T + b_ih                 (GRUCell input gates)
//   Fc2Prob : Q = Hs W2^T + b2                      (fc2 over the recurrence's stored hidden states)
//   HypProb : HYP = state_row W_hyper^T + b_hyper   (QMixer hyper_w_1 | hyper_w_final | hyper_b_1 | V.0,
//             qmix.py:30-39; online on state[:, :-1], target on state[:, 1:]); the online pass writes the
//             gathered states densely (S0) for the dW_hyper contraction
// Backward:
//   Dx1Prob : dP1 = (dGI W_ih) * [X1 > 0]
//   Dw1Prob : [dW1 | db1] = dP1^T XIN                  split-K over (t, row)
// (dW_hyper has its own kernel: dwh_kernel.hpp)
#pragma once
#include "gemm_f32.hpp"
#include "learner_types.hpp"

namespace mq {

MQ_DEV void krange_split(int K, int nsplit, int z, int& kb, int& ke) {
  int chunk = (K + nsplit - 1) / nsplit;
  chunk = (chunk + GBK - 1) / GBK * GBK;
  kb = z * chunk;
  ke = min(K, kb + chunk);
}

MQ_DEV void ld4(const float* p, float (&r)[4]) {   // 16-B aligned row segment, or zeros
  f32x4 v = p ? *(const f32x4*)p : f32x4{0, 0, 0, 0};
  r[0] = v[0]; r[1] = v[1]; r[2] = v[2]; r[3] = v[3];
}

MQ_DEV void ld4u(const float* p, float (&r)[4]) {   // 4-byte aligned row segment: one global_load_dwordx4
  f32x4 v;
  __builtin_memcpy(&v, p, sizeof(v));
  r[0] = v[0]; r[1] = v[1]; r[2] = v[2]; r[3] = v[3];
}

// C tile store helper: rows mrow0 + acc_row(reg), column ncol0 + lane%32.
template <class F>
MQ_DEV void for_tile(const f32x16& acc, int mrow0, int ncol0, int lane, F&& f) {
  const int j = ncol0 + (lane & 31);
#pragma unroll
  for (int reg = 0; reg < 16; ++reg) f(mrow0 + acc_row(reg, lane), j, acc[reg]);
}

// ---------------------------------------------------------------------------------------------- forward
// Both nets in one pass: the B tile's 128 columns are [online W1 rows | target W1 rows] (BN = 128, grid.z = 1), so
// each agent-input row is gathered and built once and feeds both nets' fc1.
struct Fc1Prob {
  static constexpr int BN = 2 * H;
  Dims d;
  Rep rp;
  const float* P0;
  const float* P1;
  int64_t o_w, o_b;
  float* X1;   // [2][M][H]
  float* XIN;  // [M][I], written once
  int64_t M;
  using APat = KPat;
  using BPat = KPat;
  static constexpr bool kRowSum = false;
  struct Ctx {
    const float* arow;
    const float* brow[2];
    int m, aprev, ag;
  };
  MQ_DEV Ctx make_ctx(int m0, int, int, int tid) const {
    Ctx c;
    c.m = m0 + KPat::row(tid);
    c.arow = nullptr;
    c.aprev = -1;
    c.ag = -1;
    if (c.m < M) {
      int t, r, b, ag;
      split_tr(d, (uint32_t)c.m, t, r, b, ag);
      const int64_t slot = rp.ep(b) * d.t_stride + t;
      c.arow = rp.obs + (slot * d.n + ag) * (int64_t)d.O;
      c.ag = ag;
      // actions_onehot[t-1] is zero unless slot t-1 was filled (runner contract, synthetic.py)
      if (d.last_action && t > 0 && rp.filled[slot - 1]) c.aprev = (int)rp.actions[(slot - 1) * d.n + ag];
    }
    const int nn = KPat::row(tid);   // < H: pass p covers net p's 64 output units
    c.brow[0] = P0 + o_w + (int64_t)nn * d.I;
    c.brow[1] = P1 + o_w + (int64_t)nn * d.I;
    return c;
  }
  MQ_DEV void krange(int, int& kb, int& ke) const { kb = 0; ke = d.I; }
  MQ_DEV void load_a(const Ctx& c, int k0, int ke, float (&r)[4]) const {
    const int k = k0 + KPat::kq(threadIdx.x);
    if (c.arow && k + 3 < d.O) {   // the common case: four obs features, one dword-aligned 16-byte load
      ld4u(c.arow + k, r);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int kk = k + i;
        float v = 0.0f;
        if (c.arow && kk < ke) {
          if (kk < d.O) {
            v = c.arow[kk];
          } else {
            int f = kk - d.O;
            if (d.last_action) {
              if (f < d.A) v = f == c.aprev ? 1.0f : 0.0f;
              f -= d.A;
            }
            if (f >= 0 && f == c.ag) v = 1.0f;
          }
        }
        r[i] = v;
      }
    }
    if (XIN && c.arow) {
      float* dst = XIN + (int64_t)c.m * d.I + k;
      if ((d.I & 3) == 0 && k + 3 < ke) {   // one 16-byte store (I % 4 == 0: rows and k-quads 16-B aligned)
        *(f32x4*)dst = f32x4{r[0], r[1], r[2], r[3]};
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (k + i < ke) dst[i] = r[i];
      }
    }
  }
  MQ_DEV void load_b(const Ctx& c, int pass, int k0, int ke, float (&r)[4]) const {
    const int k = k0 + KPat::kq(threadIdx.x);
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = k + i < ke ? c.brow[pass][k + i] : 0.0f;
  }
  MQ_DEV void epilogue(const Ctx&, const f32x16& acc, int mrow0, int ncol0, int, int lane) const {
    const int z = ncol0 >= H ? 1 : 0;
    const int c0 = ncol0 - z * H;
    const float bj = (z ? P1 : P0)[o_b + c0 + (lane & 31)];
    float* out = X1 + (int64_t)z * M * H;
    for_tile(acc, mrow0, c0, lane, [&](int m, int jj, float v) {
      if (m < M) out[(int64_t)m * H + jj] = fmaxf(v + bj, 0.0f);
    });
  }
  MQ_DEV void rowsum_out(int, int, float) const {}
};

struct GiProb {
  static constexpr int BN = 192;
  const float* X1;   // [2][M][H]
  const float* P0;
  const float* P1;
  int64_t o_w, o_b;
  float* GI;         // [2][M][3H]
  int64_t M;
  using APat = KPat;
  using BPat = KPat;
  static constexpr bool kRowSum = false;
  struct Ctx {
    const float* arow;
    const float* brow[3];
  };
  MQ_DEV Ctx make_ctx(int m0, int, int z, int tid) const {
    Ctx c;
    const int m = m0 + KPat::row(tid);
    c.arow = (m < M) ? X1 + ((int64_t)z * M + m) * H : nullptr;
    const float* W = (z ? P1 : P0) + o_w;
#pragma unroll
    for (int p = 0; p < 3; ++p) c.brow[p] = W + (int64_t)(64 * p + KPat::row(tid)) * H;
    return c;
  }
  MQ_DEV void krange(int, int& kb, int& ke) const { kb = 0; ke = H; }
  MQ_DEV void load_a(const Ctx& c, int k0, int, float (&r)[4]) const {
    ld4(c.arow ? c.arow + k0 + KPat::kq(threadIdx.x) : nullptr, r);
  }
  MQ_DEV void load_b(const Ctx& c, int pass, int k0, int, float (&r)[4]) const {
    ld4(c.brow[pass] + k0 + KPat::kq(threadIdx.x), r);
  }
  MQ_DEV void epilogue(const Ctx&, const f32x16& acc, int mrow0, int ncol0, int z, int lane) const {
    const int j = ncol0 + (lane & 31);
    const float bj = (z ? P1 : P0)[o_b + j];
    float* out = GI + (int64_t)z * M * G3;
    for_tile(acc, mrow0, ncol0, lane, [&](int m, int jj, float v) {
      if (m < M) out[(int64_t)m * G3 + jj] = v + bj;
    });
  }
  MQ_DEV void rowsum_out(int, int, float) const {}
};

// Q = Hs W2^T + b2 for both nets (fc2 of rnn_agent.py:35, out of the recurrence).
struct Fc2Prob {
  static constexpr int BN = 64;   // MT = 2 measured slower at configs[2] (0.17 -> 0.21 ms, r03)
  const float* Hs;   // [2][M][H]
  const float* P0;
  const float* P1;
  int64_t o_w, o_b;
  float* Q;          // [2][M][A]
  int64_t M;
  int A;
  using APat = KPat;
  using BPat = KPat;
  static constexpr bool kRowSum = false;
  struct Ctx {
    const float* arow;
    const float* brow;
  };
  MQ_DEV Ctx make_ctx(int m0, int n0, int z, int tid) const {
    Ctx c;
    const int m = m0 + KPat::row(tid);
    c.arow = (m < M) ? Hs + ((int64_t)z * M + m) * H : nullptr;
    const int nn = n0 + KPat::row(tid);
    c.brow = (nn < A) ? (z ? P1 : P0) + o_w + (int64_t)nn * H : nullptr;
    return c;
  }
  MQ_DEV void krange(int, int& kb, int& ke) const { kb = 0; ke = H; }
  MQ_DEV void load_a(const Ctx& c, int k0, int, float (&r)[4]) const {
    ld4(c.arow ? c.arow + k0 + KPat::kq(threadIdx.x) : nullptr, r);
  }
  MQ_DEV void load_b(const Ctx& c, int, int k0, int, float (&r)[4]) const {
    ld4(c.brow ? c.brow + k0 + KPat::kq(threadIdx.x) : nullptr, r);
  }
  MQ_DEV void epilogue(const Ctx&, const f32x16& acc, int mrow0, int ncol0, int z, int lane) const {
    const int j = ncol0 + (lane & 31);
    if (j >= A) return;
    const float bj = (z ? P1 : P0)[o_b + j];
    float* out = Q + (int64_t)z * M * A;
    for_tile(acc, mrow0, ncol0, lane, [&](int m, int jj, float v) {
      if (m < M) out[(int64_t)m * A + jj] = v + bj;
    });
  }
  MQ_DEV void rowsum_out(int, int, float) const {}
};

// Hypernet row j of the concatenation [hyper_w_1 (nE) | hyper_w_final (E) | hyper_b_1 (E) | V.0 (E)].
struct HypSeg {
  int64_t w, b;
  int row;
};
MQ_DEV HypSeg hyp_seg(const Lay& L, int nE, int E, int j) {
  HypSeg s;
  if (j < nE) { s.w = L.o[MQ_P_HW1_W]; s.b = L.o[MQ_P_HW1_B]; s.row = j; }
  else if (j < nE + E) { s.w = L.o[MQ_P_HWF_W]; s.b = L.o[MQ_P_HWF_B]; s.row = j - nE; }
  else if (j < nE + 2 * E) { s.w = L.o[MQ_P_HB1_W]; s.b = L.o[MQ_P_HB1_B]; s.row = j - nE - E; }
  else { s.w = L.o[MQ_P_V0_W]; s.b = L.o[MQ_P_V0_B]; s.row = j - nE - 2 * E; }
  return s;
}

struct HypProb {
  static constexpr int BN = 64;   // M = T*B is small: more n-tiles keep more workgroups (and loads) in flight
  Dims d;
  Rep rp;
  Lay L;
  const float* P0;
  const float* P1;
  float* HYP;   // [2][M][NH]
  float* S0;    // [M][S] gathered state[:, :-1] rows, written by the z == 0 pass
  using APat = KPat;
  using BPat = KPat;
  static constexpr bool kRowSum = false;
  struct Ctx {
    const float* arow;
    const float* brow[BN / 64];
    int m;
  };
  MQ_DEV Ctx make_ctx(int m0, int n0, int z, int tid) const {
    Ctx c;
    c.m = m0 + KPat::row(tid);
    c.arow = nullptr;
    if (c.m < d.M) {
      const int t = (int)fdiv((uint32_t)c.m, d.dB), b = c.m - t * d.B;
      c.arow = rp.state + (rp.ep(b) * d.t_stride + t + z) * (int64_t)d.S;
    }
#pragma unroll
    for (int p = 0; p < BN / 64; ++p) {
      const int nn = n0 + 64 * p + KPat::row(tid);
      c.brow[p] = nullptr;
      if (nn < d.NH) {
        HypSeg s = hyp_seg(L, d.n * d.E, d.E, nn);
        c.brow[p] = (z ? P1 : P0) + s.w + (int64_t)s.row * d.S;
      }
    }
    return c;
  }
  MQ_DEV void krange(int, int& kb, int& ke) const { kb = 0; ke = d.S; }
  MQ_DEV void load_a(const Ctx& c, int k0, int ke, float (&r)[4]) const {
    const int k = k0 + KPat::kq(threadIdx.x);
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = (c.arow && k + i < ke) ? c.arow[k + i] : 0.0f;
    if (S0 && c.arow && blockIdx.z == 0 && blockIdx.y == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (k + i < ke) S0[(int64_t)c.m * d.S + k + i] = r[i];
    }
  }
  MQ_DEV void load_b(const Ctx& c, int pass, int k0, int ke, float (&r)[4]) const {
    const int k = k0 + KPat::kq(threadIdx.x);
    const float* p = c.brow[pass];
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = (p && k + i < ke) ? p[k + i] : 0.0f;
  }
  MQ_DEV void epilogue(const Ctx&, const f32x16& acc, int mrow0, int ncol0, int z, int lane) const {
    const int j = ncol0 + (lane & 31);
    if (j >= d.NH) return;
    HypSeg s = hyp_seg(L, d.n * d.E, d.E, j);
    const float bj = (z ? P1 : P0)[s.b + s.row];
    float* out = HYP + (int64_t)z * d.M * d.NH;
    for_tile(acc, mrow0, ncol0, lane, [&](int m, int jj, float v) {
      if (m < d.M) out[(int64_t)m * d.NH + jj] = v + bj;
    });
  }
  MQ_DEV void rowsum_out(int, int, float) const {}
};

// ---------------------------------------------------------------------------------------------- backward
struct Dx1Prob {
  static constexpr int BN = 64;   // MT = 2 measured slower in the configs[2] pipeline (0.22 -> 0.31 ms, r03)
  const float* dGI;   // [M][3H]
  const float* Wih;   // online w_ih [3H][H]
  const float* X1o;   // online X1 [M][H]
  float* dP1;         // [M][H]
  int64_t M;
  using APat = KPat;
  using BPat = MPat;
  static constexpr bool kRowSum = false;
  struct Ctx {
    const float* arow;
  };
  MQ_DEV Ctx make_ctx(int m0, int, int, int tid) const {
    Ctx c;
    const int m = m0 + KPat::row(tid);
    c.arow = (m < M) ? dGI + (int64_t)m * G3 : nullptr;
    return c;
  }
  MQ_DEV void krange(int, int& kb, int& ke) const { kb = 0; ke = G3; }
  MQ_DEV void load_a(const Ctx& c, int k0, int, float (&r)[4]) const {
    ld4(c.arow ? c.arow + k0 + KPat::kq(threadIdx.x) : nullptr, r);
  }
  MQ_DEV void load_b(const Ctx&, int, int k0, int, float (&r)[4]) const {
    const int nn = MPat::row(threadIdx.x), k = k0 + MPat::kq(threadIdx.x);
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = Wih[(int64_t)(k + i) * H + nn];
  }
  MQ_DEV void epilogue(const Ctx&, const f32x16& acc, int mrow0, int ncol0, int, int lane) const {
    for_tile(acc, mrow0, ncol0, lane, [&](int m, int j, float v) {
      if (m < M) {
        const int64_t o = (int64_t)m * H + j;
        dP1[o] = X1o[o] > 0.0f ? v : 0.0f;
      }
    });
  }
  MQ_DEV void rowsum_out(int, int, float) const {}
};

// [dW1 | db1] slab: out row j (hidden unit), out col f (agent input feature), reduction over rows tr.
struct Dw1Prob {
  static constexpr int BN = 128;
  int I;
  const float* dP1;   // [RT][H]
  const float* XIN;   // [RT][I]
  float* slab;        // [nsplit][H*I + H]
  int64_t K;          // RT
  int nsplit;
  using APat = MPat;
  using BPat = MPat;
  static constexpr bool kRowSum = true;
  struct Ctx {
    int f0;
  };
  MQ_DEV Ctx make_ctx(int, int n0, int, int tid) const { return Ctx{n0 + MPat::row(tid)}; }
  MQ_DEV void krange(int z, int& kb, int& ke) const { krange_split((int)K, nsplit, z, kb, ke); }
  MQ_DEV void load_a(const Ctx&, int k0, int ke, float (&r)[4]) const {
    const int j = MPat::row(threadIdx.x), k = k0 + MPat::kq(threadIdx.x);
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = (k + i < ke) ? dP1[(int64_t)(k + i) * H + j] : 0.0f;
  }
  MQ_DEV void load_b(const Ctx& c, int pass, int k0, int ke, float (&r)[4]) const {
    const int f = c.f0 + 64 * pass, k = k0 + MPat::kq(threadIdx.x);
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = (f < I && k + i < ke) ? XIN[(int64_t)(k + i) * I + f] : 0.0f;
  }
  MQ_DEV void epilogue(const Ctx&, const f32x16& acc, int mrow0, int ncol0, int z, int lane) const {
    const int f = ncol0 + (lane & 31);
    if (f >= I) return;
    float* out = slab + (int64_t)z * (H * I + H);
    for_tile(acc, mrow0, ncol0, lane, [&](int j, int ff, float v) {
      if (j < H) out[(int64_t)j * I + ff] = v;
    });
  }
  MQ_DEV void rowsum_out(int j, int z, float v) const {
    if (j < H) slab[(int64_t)z * (H * I + H) + H * I + j] = v;
  }
};

}  // namespace mq
