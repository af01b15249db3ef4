// The learner's row-parallel and weight-gradient contractions as policies of gemm_f32_kernel.
//
// Forward (grid.z = net: 0 online, 1 target; both nets read the same replay rows):
//   Fc1Prob : X1 = relu(obs_row . W1[:, :O]^T + W1[:, O + a_{t-1}] + W1[:, O + A + agent] + b1)
//             (BasicMAC._build_inputs one-hot columns folded into the epilogue as column gathers,
//              basic_controller.py:100-135; fc1 + relu of rnn_agent.py:32)
//   GiProb  : GI = X1 W_ih^T + b_ih                 (GRUCell input gates)
//   Fc2Prob : Q = Hs W2^T + b2                      (fc2 over the recurrence's stored hidden states)
//   HypProb : HYP = state_row W_hyper^T + b_hyper   (QMixer hyper_w_1 | hyper_w_final | hyper_b_1 | V.0,
//             qmix.py:30-39; online on state[:, :-1], target on state[:, 1:])
// Backward:
//   Dx1Prob : dP1 = (dGI W_ih) * [X1 > 0]
//   Dw1Prob : [dW1 | db1] = dP1^T [xin]   split-K over (t, row); one-hot columns generated on the fly
//   DwhProb : [dW_hyper | db_hyper] = dHYP^T [state]   split-K over (t, episode)
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

// ---------------------------------------------------------------------------------------------- forward
struct Fc1Prob {
  Dims d;
  Rep rp;
  const float* P0;
  const float* P1;
  int64_t o_w, o_b;
  float* X1;
  int64_t M;
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
    c.arow = nullptr;
    if (m < M) {
      int t, r, b, ag;
      split_tr(d, (uint32_t)m, t, r, b, ag);
      c.arow = rp.obs + ((rp.ep(b) * d.t_stride + t) * d.n + ag) * (int64_t)d.O;
    }
    const int nn = n0 + KPat::row(tid);
    c.brow = (nn < H) ? (z ? P1 : P0) + o_w + (int64_t)nn * d.I : nullptr;
    return c;
  }
  MQ_DEV void krange(int, int& kb, int& ke) const { kb = 0; ke = d.O; }
  MQ_DEV void load_a(const Ctx& c, int k0, int ke, float (&r)[4]) const {
    const int k = k0 + KPat::kq(threadIdx.x);
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = (c.arow && k + i < ke) ? c.arow[k + i] : 0.0f;
  }
  MQ_DEV void load_b(const Ctx& c, int k0, int ke, float (&r)[4]) const {
    const int k = k0 + KPat::kq(threadIdx.x);
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = (c.brow && k + i < ke) ? c.brow[k + i] : 0.0f;
  }
  MQ_DEV void epilogue(const Ctx&, const f32x16& acc, int m0, int n0, int z, int wm, int wn, int lane) const {
    const float* P = z ? P1 : P0;
    const float* W = P + o_w;
    const int j = n0 + wn * 32 + (lane & 31);
    if (j >= H) return;
    const float bj = P[o_b + j];
    const int a_off = d.O, id_off = d.O + (d.last_action ? d.A : 0);
    float* out = X1 + (int64_t)z * M * H;
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int m = m0 + wm * 32 + acc_row(reg, lane);
      if (m >= M) continue;
      int t, r, b, ag;
      split_tr(d, (uint32_t)m, t, r, b, ag);
      float v = acc[reg] + bj;
      if (d.last_action && t > 0) {
        const int64_t e = rp.ep(b);
        const int64_t slot = e * d.t_stride + (t - 1);
        if (rp.filled[slot]) v += W[(int64_t)j * d.I + a_off + (int)rp.actions[slot * d.n + ag]];
      }
      if (d.agent_id) v += W[(int64_t)j * d.I + id_off + ag];
      out[(int64_t)m * H + j] = fmaxf(v, 0.0f);
    }
  }
  MQ_DEV void rowsum_out(int, int, float) const {}
};

struct GiProb {
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
    const float* brow;
  };
  MQ_DEV Ctx make_ctx(int m0, int n0, int z, int tid) const {
    Ctx c;
    const int m = m0 + KPat::row(tid);
    c.arow = (m < M) ? X1 + ((int64_t)z * M + m) * H : nullptr;
    const int nn = n0 + KPat::row(tid);
    c.brow = (nn < G3) ? (z ? P1 : P0) + o_w + (int64_t)nn * H : nullptr;
    return c;
  }
  MQ_DEV void krange(int, int& kb, int& ke) const { kb = 0; ke = H; }
  MQ_DEV void load_a(const Ctx& c, int k0, int, float (&r)[4]) const {
    const int k = k0 + KPat::kq(threadIdx.x);
    f32x4 v = c.arow ? *(const f32x4*)(c.arow + k) : f32x4{0, 0, 0, 0};
    r[0] = v[0]; r[1] = v[1]; r[2] = v[2]; r[3] = v[3];
  }
  MQ_DEV void load_b(const Ctx& c, int k0, int, float (&r)[4]) const {
    const int k = k0 + KPat::kq(threadIdx.x);
    f32x4 v = c.brow ? *(const f32x4*)(c.brow + k) : f32x4{0, 0, 0, 0};
    r[0] = v[0]; r[1] = v[1]; r[2] = v[2]; r[3] = v[3];
  }
  MQ_DEV void epilogue(const Ctx&, const f32x16& acc, int m0, int n0, int z, int wm, int wn, int lane) const {
    const int j = n0 + wn * 32 + (lane & 31);
    if (j >= G3) return;
    const float bj = (z ? P1 : P0)[o_b + j];
    float* out = GI + (int64_t)z * M * G3;
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int m = m0 + wm * 32 + acc_row(reg, lane);
      if (m < M) out[(int64_t)m * G3 + j] = acc[reg] + bj;
    }
  }
  MQ_DEV void rowsum_out(int, int, float) const {}
};

// Q = Hs W2^T + b2 for both nets (fc2 of rnn_agent.py:35, out of the recurrence).
struct Fc2Prob {
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
    const int k = k0 + KPat::kq(threadIdx.x);
    f32x4 v = c.arow ? *(const f32x4*)(c.arow + k) : f32x4{0, 0, 0, 0};
    r[0] = v[0]; r[1] = v[1]; r[2] = v[2]; r[3] = v[3];
  }
  MQ_DEV void load_b(const Ctx& c, int k0, int, float (&r)[4]) const {
    const int k = k0 + KPat::kq(threadIdx.x);
    f32x4 v = c.brow ? *(const f32x4*)(c.brow + k) : f32x4{0, 0, 0, 0};
    r[0] = v[0]; r[1] = v[1]; r[2] = v[2]; r[3] = v[3];
  }
  MQ_DEV void epilogue(const Ctx&, const f32x16& acc, int m0, int n0, int z, int wm, int wn, int lane) const {
    const int j = n0 + wn * 32 + (lane & 31);
    if (j >= A) return;
    const float bj = (z ? P1 : P0)[o_b + j];
    float* out = Q + (int64_t)z * M * A;
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int m = m0 + wm * 32 + acc_row(reg, lane);
      if (m < M) out[(int64_t)m * A + j] = acc[reg] + bj;
    }
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
  Dims d;
  Rep rp;
  Lay L;
  const float* P0;
  const float* P1;
  float* HYP;   // [2][M][NH]
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
    c.arow = nullptr;
    if (m < d.M) {
      const int t = (int)fdiv((uint32_t)m, d.dB), b = m - t * d.B;
      c.arow = rp.state + (rp.ep(b) * d.t_stride + t + z) * (int64_t)d.S;
    }
    const int nn = n0 + KPat::row(tid);
    c.brow = nullptr;
    if (nn < d.NH) {
      HypSeg s = hyp_seg(L, d.n * d.E, d.E, nn);
      c.brow = (z ? P1 : P0) + s.w + (int64_t)s.row * d.S;
    }
    return c;
  }
  MQ_DEV void krange(int, int& kb, int& ke) const { kb = 0; ke = d.S; }
  MQ_DEV void load_a(const Ctx& c, int k0, int ke, float (&r)[4]) const {
    const int k = k0 + KPat::kq(threadIdx.x);
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = (c.arow && k + i < ke) ? c.arow[k + i] : 0.0f;
  }
  MQ_DEV void load_b(const Ctx& c, int k0, int ke, float (&r)[4]) const {
    const int k = k0 + KPat::kq(threadIdx.x);
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = (c.brow && k + i < ke) ? c.brow[k + i] : 0.0f;
  }
  MQ_DEV void epilogue(const Ctx&, const f32x16& acc, int m0, int n0, int z, int wm, int wn, int lane) const {
    const int j = n0 + wn * 32 + (lane & 31);
    if (j >= d.NH) return;
    HypSeg s = hyp_seg(L, d.n * d.E, d.E, j);
    const float bj = (z ? P1 : P0)[s.b + s.row];
    float* out = HYP + (int64_t)z * d.M * d.NH;
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int m = m0 + wm * 32 + acc_row(reg, lane);
      if (m < d.M) out[(int64_t)m * d.NH + j] = acc[reg] + bj;
    }
  }
  MQ_DEV void rowsum_out(int, int, float) const {}
};

// ---------------------------------------------------------------------------------------------- backward
struct Dx1Prob {
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
    const int k = k0 + KPat::kq(threadIdx.x);
    f32x4 v = c.arow ? *(const f32x4*)(c.arow + k) : f32x4{0, 0, 0, 0};
    r[0] = v[0]; r[1] = v[1]; r[2] = v[2]; r[3] = v[3];
  }
  MQ_DEV void load_b(const Ctx&, int k0, int, float (&r)[4]) const {
    const int nn = MPat::row(threadIdx.x), k = k0 + MPat::kq(threadIdx.x);
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = Wih[(int64_t)(k + i) * H + nn];
  }
  MQ_DEV void epilogue(const Ctx&, const f32x16& acc, int m0, int n0, int, int wm, int wn, int lane) const {
    const int j = n0 + wn * 32 + (lane & 31);
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int m = m0 + wm * 32 + acc_row(reg, lane);
      if (m < M) {
        const int64_t o = (int64_t)m * H + j;
        dP1[o] = X1o[o] > 0.0f ? acc[reg] : 0.0f;
      }
    }
  }
  MQ_DEV void rowsum_out(int, int, float) const {}
};

// [dW1 | db1] slab: out row j (hidden unit), out col f (agent input feature), reduction over rows tr.
struct Dw1Prob {
  Dims d;
  Rep rp;
  const float* dP1;   // [RT][H]
  float* slab;        // [nsplit][H*I + H]
  int64_t K;          // RT
  int nsplit;
  using APat = MPat;
  using BPat = MPat;
  static constexpr bool kRowSum = true;
  struct Ctx {
    int f;
  };
  MQ_DEV Ctx make_ctx(int, int n0, int, int tid) const { return Ctx{n0 + MPat::row(tid)}; }
  MQ_DEV void krange(int z, int& kb, int& ke) const { krange_split((int)K, nsplit, z, kb, ke); }
  MQ_DEV void load_a(const Ctx&, int k0, int ke, float (&r)[4]) const {
    const int j = blockIdx.x * GBM + MPat::row(threadIdx.x), k = k0 + MPat::kq(threadIdx.x);
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = (k + i < ke) ? dP1[(int64_t)(k + i) * H + j] : 0.0f;
  }
  MQ_DEV float xin(uint32_t tr, int f) const {
    int t, r, b, ag;
    split_tr(d, tr, t, r, b, ag);
    const int64_t slot = rp.ep(b) * d.t_stride + t;
    if (f < d.O) return rp.obs[(slot * d.n + ag) * d.O + f];
    f -= d.O;
    if (d.last_action) {
      if (f < d.A) {
        if (t == 0 || !rp.filled[slot - 1]) return 0.0f;
        return (int)rp.actions[(slot - 1) * d.n + ag] == f ? 1.0f : 0.0f;
      }
      f -= d.A;
    }
    return (d.agent_id && f == ag) ? 1.0f : 0.0f;
  }
  MQ_DEV void load_b(const Ctx& c, int k0, int ke, float (&r)[4]) const {
    const int k = k0 + MPat::kq(threadIdx.x);
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = (c.f < d.I && k + i < ke) ? xin((uint32_t)(k + i), c.f) : 0.0f;
  }
  MQ_DEV void epilogue(const Ctx&, const f32x16& acc, int m0, int n0, int z, int wm, int wn, int lane) const {
    const int f = n0 + wn * 32 + (lane & 31);
    if (f >= d.I) return;
    float* out = slab + (int64_t)z * (H * d.I + H);
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int j = m0 + wm * 32 + acc_row(reg, lane);
      if (j < H) out[(int64_t)j * d.I + f] = acc[reg];
    }
  }
  MQ_DEV void rowsum_out(int j, int z, float v) const {
    if (j < H) slab[(int64_t)z * (H * d.I + H) + H * d.I + j] = v;
  }
};

// [dW_hyper | db_hyper] slab over the contiguous QMixer region hyper_w_1.weight .. V.0.bias.
struct DwhProb {
  Dims d;
  Rep rp;
  Lay L;
  const float* dHYP;   // [M][NH]
  float* slab;         // [nsplit][len]
  int64_t len;
  int nsplit;
  using APat = MPat;
  using BPat = MPat;
  static constexpr bool kRowSum = true;
  struct Ctx {
    int s;
  };
  MQ_DEV Ctx make_ctx(int, int n0, int, int tid) const { return Ctx{n0 + MPat::row(tid)}; }
  MQ_DEV void krange(int z, int& kb, int& ke) const { krange_split(d.M, nsplit, z, kb, ke); }
  MQ_DEV void load_a(const Ctx&, int k0, int ke, float (&r)[4]) const {
    const int j = blockIdx.x * GBM + MPat::row(threadIdx.x), k = k0 + MPat::kq(threadIdx.x);
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = (j < d.NH && k + i < ke) ? dHYP[(int64_t)(k + i) * d.NH + j] : 0.0f;
  }
  MQ_DEV void load_b(const Ctx& c, int k0, int ke, float (&r)[4]) const {
    const int k = k0 + MPat::kq(threadIdx.x);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float v = 0.0f;
      if (c.s < d.S && k + i < ke) {
        const int m = k + i, t = (int)fdiv((uint32_t)m, d.dB), b = m - t * d.B;
        v = rp.state[(rp.ep(b) * d.t_stride + t) * (int64_t)d.S + c.s];
      }
      r[i] = v;
    }
  }
  MQ_DEV void epilogue(const Ctx&, const f32x16& acc, int m0, int n0, int z, int wm, int wn, int lane) const {
    const int s = n0 + wn * 32 + (lane & 31);
    if (s >= d.S) return;
    float* out = slab + (int64_t)z * len;
    const int64_t base = L.o[MQ_P_HW1_W];
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int j = m0 + wm * 32 + acc_row(reg, lane);
      if (j < d.NH) {
        HypSeg sg = hyp_seg(L, d.n * d.E, d.E, j);
        out[sg.w - base + (int64_t)sg.row * d.S + s] = acc[reg];
      }
    }
  }
  MQ_DEV void rowsum_out(int j, int z, float v) const {
    if (j < d.NH) {
      HypSeg sg = hyp_seg(L, d.n * d.E, d.E, j);
      slab[(int64_t)z * len + sg.b - L.o[MQ_P_HW1_W] + sg.row] = v;
    }
  }
};

}  // namespace mq
