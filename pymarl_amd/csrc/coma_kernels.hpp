// COMA learner kernels: the centralised critic's T sequential RMSprop steps and the
// counterfactual policy-gradient step of COMALearner.train (coma_learner.py:32-148), gfx950, fp32 throughout.
//
// Critic (coma.py:22-58, fc 868 -> 128 -> 128 -> A at MMM2). Each train() takes one optimiser step per t in
// reversed order, every step on B*n rows only, so the critic is a chain of T tiny dependent steps. One step is three
// launches, split where the data dependence forces a grid-wide exchange:
//   l1     partial H1 pre-activations X_t W1^T over K slices     grid (K slices) x (8 unit tiles of 16) x (row tiles)
//   head   sum of the partials + b1, relu, H2, Q, TD error, loss sums, dQ, dH2, dH1   (1024 threads)
//   wgrad  dW1 = dH1^T X_t, dW2 = dH2^T H1, dW3, biases, per-workgroup sums of squares (each gradient element has
//          exactly one writer: no slabs, no atomics)
// The RMSprop update of step t+1 (clip coefficient from wgrad's sums of squares) is applied inside step t's l1 while
// it stages the weights, so applying costs no launch: every W1 slice is owned by exactly one l1 block (K-split),
// which updates it in registers, writes the new version back and multiplies with it; the first K slice's blocks
// update fc1.bias / fc2 / fc3 in slices, which head then reads. Versions ping-pong between the caller's buffers and
// a shadow (live step L reads version L-1 from buffer (L-1)&1, writes version L to L&1), so no block reads what
// another block of the same launch writes. The last step's update is one more launch after the loop.
// Steps whose mask is empty are skipped on the device (coma_learner.py:121-122) and leave the pending update for the
// next live step.
//
// MFMA: v_mfma_f32_16x16x4_f32 (exact fp32 FMA chain). Lane l, g = l >> 4, c = l & 15: A[i = c][kk = g],
// B[kk = g][j = c], D[i = 4g + reg][j = c].
#pragma once
#include "learner_gemms.hpp"
#include "optim_kernels.hpp"

namespace mq {

constexpr int CH = 128;   // critic hidden width (coma.py:17-19)

MQ_DEV f32x4 mfma_f32_16x4(float a, float b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }

MQ_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

struct CDims {
  int n, A, O, S, Kc, Kp, R, B, Tp, T, t_stride;
  float lg, og;      // f32(td_lambda * gamma), f32((1 - td_lambda) * gamma): rounded on the host in double, as the
                     // reference's Python-float scalar products are
  FastDiv dR, dN;
};

// reference mask (coma_learner.py:39-41): filled[t] * (1 - terminated[t-1])
MQ_DEV float coma_mask(const Rep& rp, int64_t slot, int t) {
  float m = (float)rp.filled[slot];
  if (t > 0) m *= 1.0f - (float)rp.term[slot - 1];
  return m;
}

// ------------------------------------------------------------------------------------------- critic inputs
// X[t][r][k] for every stored step of the batch (COMACritic._build_inputs, coma.py:30-58):
// state | obs | actions_onehot[t] of every agent with the row's own block zeroed | actions_onehot[t-1] (0 at t = 0)
// | onehot(agent) | zero padding to Kp. actions_onehot is the reference's OneHot transform of the stored action,
// zero on unfilled slots (the runner never writes them).
// t0: first stored step (the standalone COMACritic.forward(batch, t) builds one step's rows, coma.py:40-45).
__global__ __launch_bounds__(256) void coma_xin_kernel(CDims d, Rep rp, float* __restrict__ X, int t0 = 0) {
  const int tr = blockIdx.x;
  const int tl = (int)fdiv((uint32_t)tr, d.dR), r = tr - tl * d.R, t = t0 + tl;
  const int b = (int)fdiv((uint32_t)r, d.dN), ag = r - b * d.n;
  const int64_t slot = rp.ep(b) * d.t_stride + t;
  const float* st = rp.state + slot * d.S;
  const float* ob = rp.obs + (slot * d.n + ag) * d.O;
  const int nA = d.n * d.A, k1 = d.S + d.O, k2 = k1 + nA, k3 = k2 + nA;
  const bool fill_t = rp.filled[slot] != 0, fill_p = t > 0 && rp.filled[slot - 1] != 0;
  float* out = X + (int64_t)tr * d.Kp;
  for (int k = threadIdx.x; k < d.Kp; k += 256) {
    float v = 0.0f;
    if (k < d.S) {
      v = st[k];
    } else if (k < k1) {
      v = ob[k - d.S];
    } else if (k < k2) {
      const int j = (k - k1) / d.A, a = (k - k1) - j * d.A;
      v = (j != ag && fill_t && rp.actions[slot * d.n + j] == a) ? 1.0f : 0.0f;
    } else if (k < k3) {
      const int j = (k - k2) / d.A, a = (k - k2) - j * d.A;
      v = (fill_p && rp.actions[(slot - 1) * d.n + j] == a) ? 1.0f : 0.0f;
    } else if (k < d.Kc) {
      v = (k - k3) == ag ? 1.0f : 0.0f;
    }
    out[k] = v;
  }
}

// Sum of the critic mask of step t over (episode, agent) (mask_t.sum(), coma_learner.py:120-122), t < T.
__global__ __launch_bounds__(256) void coma_mask_kernel(CDims d, Rep rp, float* __restrict__ msum) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= d.T) return;
  float s = 0.0f;
  for (int b = 0; b < d.B; ++b) s += coma_mask(rp, rp.ep(b) * d.t_stride + t, t);
  msum[t] = s * (float)d.n;
}

// Dense linear layer for the target critic's all-steps forward: out[m][j] = act(X[m][:K] . W[j][:K] + bias[j]).
// BN_ = 64 for the wide-K layer: twice the workgroups (two per CU at cfg5) for latency hiding
template <int BN_ = 128>
struct CLinProbT {
  static constexpr int BN = BN_;
  const float* X;   // [M][ldx]
  int ldx;
  const float* W;   // [N][K] row-major (the reference layout)
  const float* bias;
  float* out;       // [M][N]
  int64_t M;
  int N, K, relu;
  bool vec_a = false, vec_b = false;   // set by with_vec(): 16-B aligned rows
  CLinProbT with_vec() const {
    CLinProbT q = *this;
    q.vec_a = ldx % 4 == 0 && ((uintptr_t)X & 15) == 0;
    q.vec_b = K % 4 == 0 && ((uintptr_t)W & 15) == 0;
    return q;
  }
  using APat = KPat;
  using BPat = KPat;
  static constexpr bool kRowSum = false;
  struct Ctx {
    const float* arow;
    const float* brow[2];
  };
  MQ_DEV Ctx make_ctx(int m0, int n0, int, int tid) const {
    Ctx c;
    const int64_t m = m0 + KPat::row(tid);
    c.arow = m < M ? X + m * ldx : nullptr;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int nn = n0 + 64 * p + KPat::row(tid);
      c.brow[p] = nn < N ? W + (int64_t)nn * K : nullptr;
    }
    return c;
  }
  MQ_DEV void krange(int, int& kb, int& ke) const { kb = 0; ke = K; }
  // 16-B loads where the 4-run is inside K (rows are 16-B aligned: ldx and K are multiples of 4 wherever the
  // vector path is taken, checked by vec_ok), element loads at the K tail
  MQ_DEV void load_a(const Ctx& c, int k0, int ke, float (&r)[4]) const {
    const int k = k0 + KPat::kq(threadIdx.x);
    if (c.arow && vec_a && k + 3 < ke) {
      const f32x4 v = *(const f32x4*)&c.arow[k];
      r[0] = v[0]; r[1] = v[1]; r[2] = v[2]; r[3] = v[3];
      return;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = (c.arow && k + i < ke) ? c.arow[k + i] : 0.0f;
  }
  MQ_DEV void load_b(const Ctx& c, int pass, int k0, int ke, float (&r)[4]) const {
    const int k = k0 + KPat::kq(threadIdx.x);
    const float* p = c.brow[pass];
    if (p && vec_b && k + 3 < ke) {
      const f32x4 v = *(const f32x4*)&p[k];
      r[0] = v[0]; r[1] = v[1]; r[2] = v[2]; r[3] = v[3];
      return;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = (p && k + i < ke) ? p[k + i] : 0.0f;
  }
  MQ_DEV void epilogue(const Ctx&, const f32x16& acc, int mrow0, int ncol0, int, int lane) const {
    const int j = ncol0 + (lane & 31);
    if (j >= N) return;
    const float bj = bias[j];
    for_tile(acc, mrow0, ncol0, lane, [&](int m, int jj, float v) {
      if (m < M) {
        const float y = v + bj;
        out[(int64_t)m * N + jj] = relu ? fmaxf(y, 0.0f) : y;
      }
    });
  }
  MQ_DEV void rowsum_out(int, int, float) const {}
};
using CLinProb = CLinProbT<128>;

// build_td_lambda_targets (rl_utils.py:4-14), one workgroup per episode: the recursion's inputs (the target critic's
// Q at the taken action for every (t, agent), reward, terminated, mask) are gathered into LDS by all threads, then
// one thread per agent runs the backward recursion out of LDS
//   ret_T = Q'_T(a_T) (1 - sum_t term_t),
//   ret_t = lambda gamma ret_{t+1} + mask_t (r_t + (1 - lambda) gamma Q'_{t+1}(a_{t+1}) (1 - term_t)),
// in torch's evaluation order without FMA contraction. Writes targets [T][R]. LDS: Tp * (n + 3) floats.
__global__ __launch_bounds__(256) void coma_td_kernel(CDims d, Rep rp, const float* __restrict__ Qt,
                                                      float* __restrict__ tgt) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int b = blockIdx.x, n = d.n, Tp = d.Tp;
  float* tq = sm;              // [Tp][n]
  float* rw = tq + Tp * n;     // [Tp]
  float* om = rw + Tp;         // [Tp] 1 - terminated
  float* mk = om + Tp;         // [Tp] mask
  const int64_t e0 = rp.ep(b) * d.t_stride;
  for (int e = threadIdx.x; e < Tp * n; e += 256) {
    const int t = e / n, ag = e - t * n;
    const int r = b * n + ag;
    tq[e] = Qt[((int64_t)t * d.R + r) * d.A + (int)rp.actions[(e0 + t) * n + ag]];
  }
  for (int t = threadIdx.x; t < Tp; t += 256) {
    rw[t] = rp.reward[e0 + t];
    om[t] = 1.0f - (float)rp.term[e0 + t];
    mk[t] = coma_mask(rp, e0 + t, t);
  }
  __syncthreads();
  const int ag = threadIdx.x;
  if (ag >= n) return;
  float tsum = 0.0f;
  for (int t = 0; t < d.T; ++t) tsum += 1.0f - om[t];
  float ret = tq[(Tp - 1) * n + ag] * (1.0f - tsum);
  float* out = tgt + b * n + ag;
  for (int t = Tp - 2; t >= 0; --t) {
    const float inner = __fadd_rn(rw[t], __fmul_rn(__fmul_rn(d.og, tq[(t + 1) * n + ag]), om[t]));
    ret = __fadd_rn(__fmul_rn(d.lg, ret), __fmul_rn(mk[t], inner));
    out[(int64_t)t * d.R] = ret;
  }
}

// ------------------------------------------------------------------------------------------ critic steps
struct CritArgs {
  CDims d;
  Rep rp;
  float* P[2];       // critic params (reference layout): [0] the caller's buffer, [1] a shadow. Live step L reads
  float* SQ[2];      // version L-1 from [(L-1) & 1] and writes version L to [L & 1] (no block ever reads what
                     // another block of the same launch writes); the last update lands in [0]
  float* G;          // raw critic grads of the pending (last live) step [Pc] + tail: [0] = its mask sum
  int64_t o_w1, o_b1, o_w2, o_b2, o_w3, o_b3, Pc;
  const float* X;    // [Tp][R][Kp]
  const float* tgt;  // [T][R]
  const float* msum; // [T]
  float* H1p;        // [KS][R][CH] l1's partial pre-activations, one per K slice
  int KS;            // K slices of W1 (l1 grid.x)
  float* H1c;        // [R][CH] this step's activations / gradients
  float* H2c;
  float* dH1c;
  float* dH2c;
  float* dqc;        // [R]
  int* actc;         // [R]
  float* qvals;      // [T][R][A]
  float* cpart;      // [head blocks][8]
  float* cnorm;      // [wgrad blocks]
  int nhead, nwgrad;
  float* crec;       // [T][8]: sum (td m)^2, sum m, sum |td m|, sum q m, sum y m, grad norm, live
  int* cstate;       // [0] live steps so far, [1] t of the last live step
  OptHP hp;
};

// Clip coefficient of the pending critic update (clip_grad_norm_ over the critic, coma_learner.py:133): every block
// re-derives it from the same partials in the same order, so all blocks agree bitwise.
MQ_DEV void crit_coef(const CritArgs& a, float* sh) {
  if (threadIdx.x < 64) {
    float s = 0.0f;
    for (int i = threadIdx.x; i < a.nwgrad; i += 64) s += a.cnorm[i];
    s = wave_sum(s);
    if (threadIdx.x == 0) {
      const float inv = 1.0f / a.G[a.Pc];
      const float norm = sqrtf(s) * inv;
      sh[0] = inv;
      sh[1] = fminf(a.hp.clip / (norm + 1e-6f), 1.0f);
      sh[2] = norm;
    }
  }
}

// RMSprop on one element of the pending update (torch: v = a v + (1-a) g^2; p += -lr g / (sqrt(v) + eps)), from
// buffer src into buffer dst (write = the designated block).
MQ_DEV float crit_rms(const CritArgs& a, int64_t i, float inv, float coef, int src, int dst, bool write) {
  const float g = (a.G[i] * inv) * coef;
  const float v = a.SQ[src][i] * a.hp.alpha + (1.0f - a.hp.alpha) * (g * g);
  const float p = a.P[src][i] + (-a.hp.lr) * (g / (sqrtf(v) + a.hp.eps));
  if (write) { a.SQ[dst][i] = v; a.P[dst][i] = p; }
  return p;
}

// Stage elements [0, N) of a parameter region into LDS (dst_lds(e) <- parameter o + idx(e)), applying the pending
// update on the way. All loads of a batch of kStageB elements per thread are issued before any use: the loop is
// latency-bound (G / square_avg / params come from L2 or HBM), not issue-bound.
constexpr int kStageB = 16;
template <class Idx, class Put>
MQ_DEV void crit_stage(const CritArgs& a, int N, bool pend, float inv, float coef, int src, int dst, bool owner,
                       Idx idx, Put put) {
  const int nt = blockDim.x;
  for (int e0 = threadIdx.x; e0 < N; e0 += nt * kStageB) {
    float gv[kStageB], sv[kStageB], pv[kStageB];
#pragma unroll
    for (int u = 0; u < kStageB; ++u) {
      const int e = e0 + nt * u;
      const int64_t i = idx(e < N ? e : N - 1);
      pv[u] = a.P[src][i];
      if (pend) { gv[u] = a.G[i]; sv[u] = a.SQ[src][i]; }
    }
#pragma unroll
    for (int u = 0; u < kStageB; ++u) {
      const int e = e0 + nt * u;
      if (e >= N) break;
      float p = pv[u];
      if (pend) {
        const float g = (gv[u] * inv) * coef;
        const float v = sv[u] * a.hp.alpha + (1.0f - a.hp.alpha) * (g * g);
        p = p + (-a.hp.lr) * (g / (sqrtf(v) + a.hp.eps));
        if (owner) {
          const int64_t i = idx(e);
          a.SQ[dst][i] = v;
          a.P[dst][i] = p;
        }
      }
      put(e, p);
    }
  }
}

// Two-phase form of crit_stage for the largest region of a launch: the loads are issued before the clip coefficient
// is known (it needs its own round trip to the norm partials), so both round trips overlap.
template <int NE>
struct StageRegs {
  float p[NE], g[NE], s[NE];
};

template <int NE, class Idx>
MQ_DEV void stage_load(const CritArgs& a, int N, bool pend, int src, Idx idx, StageRegs<NE>& r) {
#pragma unroll
  for (int u = 0; u < NE; ++u) {
    const int e = threadIdx.x + blockDim.x * u;
    const int64_t i = idx(e < N ? e : N - 1);
    r.p[u] = a.P[src][i];
    if (pend) { r.g[u] = a.G[i]; r.s[u] = a.SQ[src][i]; }
  }
}

template <int NE, class Idx, class Put>
MQ_DEV void stage_apply(const CritArgs& a, int N, bool pend, float inv, float coef, int dst, bool owner,
                        const StageRegs<NE>& r, Idx idx, Put put) {
#pragma unroll
  for (int u = 0; u < NE; ++u) {
    const int e = threadIdx.x + blockDim.x * u;
    if (e >= N) break;
    float p = r.p[u];
    if (pend) {
      const float g = (r.g[u] * inv) * coef;
      const float v = r.s[u] * a.hp.alpha + (1.0f - a.hp.alpha) * (g * g);
      p = p + (-a.hp.lr) * (g / (sqrtf(v) + a.hp.eps));
      if (owner) {
        const int64_t i = idx(e);
        a.SQ[dst][i] = v;
        a.P[dst][i] = p;
      }
    }
    put(e, p);
  }
}

constexpr int kHeadThreads = 1024;
constexpr int KW = 176;        // W1 columns per l1 block: 44 MFMA k-steps
constexpr int kL1Rows = 128;   // rows of X_t one l1 block stages (grid.z covers more)

__host__ __device__ inline int l1_slices(int Kp) { return (Kp + KW - 1) / KW; }

// l1: partial H1 pre-activations over one K slice: block (ks, ut, rc) owns W1[16 ut .. +16][KW ks .. +KW] — it is
// the only block that stages, updates and writes back those weights — and multiplies them with rows
// [128 rc, +128) of X_t. The head sums the KS partials in slice order and adds b1.
// Lexp = T-1-t, the live-step count when no step was skipped: the parameter version to read is assumed from it so
// the weight loads do not wait for cstate / msum; a skipped step (rare) re-issues them from the right buffer.
__global__ __launch_bounds__(256) void coma_l1_kernel(CritArgs a, int t, int Lexp) {
  const float mt = a.msum[t];
  const int L = a.cstate[0];
  extern __shared__ __attribute__((aligned(16))) float sm[];
  constexpr int WP = KW + 1;
  const int Kp = a.d.Kp, Kc = a.d.Kc, R = a.d.R;
  const int ks = blockIdx.x, u0 = blockIdx.y * 16, rbase = blockIdx.z * kL1Rows;
  const int k0 = ks * KW, kw = min(KW, Kp - k0), kwc = max(0, min(KW, Kc - k0));   // staged / real columns
  const int nr = min(kL1Rows, R - rbase);
  float* Ws = sm;               // [16][WP]
  float* Xs = Ws + 16 * WP;     // [kL1Rows][WP]
  __shared__ float sh[4];
  const int tid = threadIdx.x;
  const int owner = blockIdx.z == 0;
  // W1 slice: 16 rows of kwc elements; all loads (params, grads, square_avg) in flight with X_t's
  constexpr int NE = (16 * KW + 255) / 256;
  auto widx = [&](int e) { const int u = e / KW, k = e - u * KW; return a.o_w1 + (int64_t)(u0 + u) * Kc + k0 + k; };
  StageRegs<NE> wr;
  auto load_w = [&](int from) {
#pragma unroll
    for (int q = 0; q < NE; ++q) {
      const int e = tid + 256 * q, u = e / KW, k = e - u * KW;
      const bool ok = e < 16 * KW && k < kwc;
      const int64_t i = ok ? widx(e) : a.o_w1;
      wr.p[q] = a.P[from][i];
      wr.g[q] = a.G[i];
      wr.s[q] = a.SQ[from][i];
    }
  };
  const int src_spec = Lexp > 0 ? (Lexp - 1) & 1 : 0;
  load_w(src_spec);
  const int nv = kw / 4;   // b128 per row
  constexpr int XB = (kL1Rows * KW / 4 + 255) / 256;
  f32x4 xv[XB];
#pragma unroll
  for (int q = 0; q < XB; ++q) {
    const int e = tid + 256 * q, rr = e / nv, kv = e - rr * nv;
    xv[q] = (rr < nr) ? *(const f32x4*)&a.X[((int64_t)t * R + rbase + rr) * Kp + k0 + 4 * kv] : f32x4{0, 0, 0, 0};
  }
  if (!(mt > 0.0f)) return;   // step skipped (coma_learner.py:121-122)
  const bool pend = L > 0;
  const int src = pend ? (L - 1) & 1 : 0, dst = L & 1;
  if (src != src_spec) load_w(src);
  if (pend) crit_coef(a, sh);
  __syncthreads();
  const float inv = pend ? sh[0] : 0.0f, coef = pend ? sh[1] : 0.0f;
  if (pend && owner && ks == 0 && blockIdx.y == 0 && tid == 0) a.crec[a.cstate[1] * 8 + 5] = sh[2];
#pragma unroll
  for (int q = 0; q < NE; ++q) {
    const int e = tid + 256 * q, u = e / KW, k = e - u * KW;
    if (e >= 16 * KW) break;
    float p = 0.0f;
    if (k < kwc) {
      p = wr.p[q];
      if (pend) {
        const float g = (wr.g[q] * inv) * coef;
        const float v = wr.s[q] * a.hp.alpha + (1.0f - a.hp.alpha) * (g * g);
        p = p + (-a.hp.lr) * (g / (sqrtf(v) + a.hp.eps));
        if (owner) {
          const int64_t i = widx(e);
          a.SQ[dst][i] = v;
          a.P[dst][i] = p;
        }
      }
    }
    Ws[u * WP + k] = p;
  }
#pragma unroll
  for (int q = 0; q < XB; ++q) {
    const int e = tid + 256 * q, rr = e / nv, kv = e - rr * nv;
    if (rr >= kL1Rows) break;
    float* d = &Xs[rr * WP + 4 * kv];
    d[0] = xv[q][0]; d[1] = xv[q][1]; d[2] = xv[q][2]; d[3] = xv[q][3];
  }
  if (pend && ks == 0 && owner) {   // fc1.bias and fc2 / fc3: one slice per (ut) block of the first K slice
    const int nb = gridDim.y, lb = blockIdx.y;
    const int64_t beg0 = a.o_b1, NT = a.Pc - a.o_b1;   // fc1.bias, fc2.*, fc3.* are contiguous from o_b1
    const int64_t chunk = (NT + nb - 1) / nb, beg = beg0 + lb * chunk;
    const int cnt = (int)max<int64_t>(0, min<int64_t>(chunk, a.Pc - beg));
    crit_stage(a, cnt, true, inv, coef, src, dst, true, [&](int e) { return beg + e; }, [&](int, float) {});
  }
  __syncthreads();
  const int w = tid >> 6, lane = tid & 63, g = lane >> 4, c = lane & 15;
  for (int rt = w; rt * 16 < nr; rt += 4) {   // row tiles of 16 over the waves, the whole K slice each
    f32x4 acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
    const float* xr = Xs + (16 * rt + c) * WP + g;
    const float* wrow = Ws + c * WP + g;
    int k = 0;
    for (; k + 8 <= kw; k += 8) {
      acc0 = mfma_f32_16x4(xr[k], wrow[k], acc0);
      acc1 = mfma_f32_16x4(xr[k + 4], wrow[k + 4], acc1);
    }
    if (k < kw) acc0 = mfma_f32_16x4(xr[k], wrow[k], acc0);
    float* out = a.H1p + ((int64_t)ks * R + rbase + 16 * rt) * CH + u0 + c;
#pragma unroll
    for (int reg = 0; reg < 4; ++reg)
      if (16 * rt + 4 * g + reg < nr) out[(int64_t)(4 * g + reg) * CH] = acc0[reg] + acc1[reg];
  }
}

// head: for a 16-row tile, H2 = relu(H1 W2^T + b2), Q = H2 W3^T + b3, the TD error against the TD(lambda) target,
// the loss sums, dQ (unnormalised: d sum (td m)^2 / dq_taken = 2 td m m), dH2 = dQ W3 o [H2 > 0], dH1 = dH2 W2 o
// [H1 > 0]. Stages (and applies the pending update to) W2 / b2 / W3 / b3; block 0 writes them back.
__global__ __launch_bounds__(kHeadThreads) void coma_head_kernel(CritArgs a, int t, int Lexp) {
  const float mt = a.msum[t];
  const int L = a.cstate[0];
  extern __shared__ __attribute__((aligned(16))) float sm[];
  constexpr int CP = CH + 1;
  const int A = a.d.A, A16 = (A + 15) / 16 * 16, R = a.d.R, n = a.d.n;
  float* W2s = sm;                 // [CH][CP]
  float* W3s = W2s + CH * CP;      // [A16][CP]
  float* H1s = W3s + A16 * CP;     // [16][CP]
  float* H2s = H1s + 16 * CP;      // [16][CP]
  float* dHs = H2s + 16 * CP;      // [16][CP]
  float* Qs = dHs + 16 * CP;       // [16][A16 + 1]
  float* b2s = Qs + 16 * (A16 + 1);   // [CH]
  float* b3s = b2s + CH;              // [A16]
  __shared__ float dqs[16];
  __shared__ int acts[16];
  __shared__ float part[16][5];
  const int tid = threadIdx.x, r0 = blockIdx.x * 16;
  // fc2 / fc3 at this step's version (l1 applied the pending update into P[L & 1]), assumed from Lexp
  const float* Pv = a.P[Lexp & 1];
  auto load_fc = [&]() {
    constexpr int NB = 16;
    const int N2 = CH * CH / 4, N3 = A * CH / 4;   // b128 units (CH = 128: rows never straddle a unit)
    for (int e0 = tid; e0 < N2 + N3; e0 += kHeadThreads * NB) {
      f32x4 v[NB];
#pragma unroll
      for (int u = 0; u < NB; ++u) {
        const int e = min(e0 + kHeadThreads * u, N2 + N3 - 1);
        v[u] = e < N2 ? *(const f32x4*)&Pv[a.o_w2 + 4 * e] : *(const f32x4*)&Pv[a.o_w3 + 4 * (e - N2)];
      }
#pragma unroll
      for (int u = 0; u < NB; ++u) {
        const int e = e0 + kHeadThreads * u;
        if (e >= N2 + N3) break;
        float* d = e < N2 ? &W2s[((4 * e) >> 7) * CP + ((4 * e) & 127)]
                          : &W3s[((4 * (e - N2)) >> 7) * CP + ((4 * (e - N2)) & 127)];
        d[0] = v[u][0]; d[1] = v[u][1]; d[2] = v[u][2]; d[3] = v[u][3];
      }
    }
  };
  load_fc();
  if (!(mt > 0.0f)) return;
  if ((L & 1) != (Lexp & 1)) {   // a skipped step shifted the version parity
    Pv = a.P[L & 1];
    load_fc();
  }
  for (int e = A * CH + tid; e < A16 * CH; e += kHeadThreads) W3s[(e >> 7) * CP + (e & 127)] = 0.0f;
  if (tid < CH) b2s[tid] = Pv[a.o_b2 + tid];
  if (tid < A) b3s[tid] = Pv[a.o_b3 + tid];
  if (tid >= A && tid < A16) b3s[tid] = 0.0f;
  if (tid < 512) {   // H1 = relu(sum of the K-slice partials in slice order + b1): 16 x 128 = 512 b128
    const int i = tid >> 5, kv = tid & 31;
    f32x4 hv = {0, 0, 0, 0};
    if (r0 + i < R) {
      for (int ks = 0; ks < a.KS; ++ks) hv += *(const f32x4*)&a.H1p[((int64_t)ks * R + r0 + i) * CH + 4 * kv];
      const f32x4 bb = *(const f32x4*)&Pv[a.o_b1 + 4 * kv];
      hv += bb;
      hv[0] = fmaxf(hv[0], 0.0f); hv[1] = fmaxf(hv[1], 0.0f); hv[2] = fmaxf(hv[2], 0.0f); hv[3] = fmaxf(hv[3], 0.0f);
      *(f32x4*)&a.H1c[(int64_t)(r0 + i) * CH + 4 * kv] = hv;
    }
    float* d = &H1s[i * CP + 4 * kv];
    d[0] = hv[0]; d[1] = hv[1]; d[2] = hv[2]; d[3] = hv[3];
  }
  __syncthreads();
  const int w = tid >> 6, lane = tid & 63, g = lane >> 4, c = lane & 15;
  // H2 = relu(H1 W2^T + b2): wave w < 8 owns unit tile w
  if (w < 8) {
    const int jt = w;
    f32x4 acc = {0, 0, 0, 0};
    for (int k = 0; k < CH; k += 4) acc = mfma_f32_16x4(H1s[c * CP + k + g], W2s[(16 * jt + c) * CP + k + g], acc);
#pragma unroll
    for (int reg = 0; reg < 4; ++reg)
      H2s[(4 * g + reg) * CP + 16 * jt + c] = fmaxf(acc[reg] + b2s[16 * jt + c], 0.0f);
  }
  __syncthreads();
  // Q = H2 W3^T + b3
  for (int qt = w; qt < A16 / 16; qt += kHeadThreads / 64) {
    f32x4 acc = {0, 0, 0, 0};
    for (int k = 0; k < CH; k += 4) acc = mfma_f32_16x4(H2s[c * CP + k + g], W3s[(16 * qt + c) * CP + k + g], acc);
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) Qs[(4 * g + reg) * (A16 + 1) + 16 * qt + c] = acc[reg] + b3s[16 * qt + c];
  }
  __syncthreads();
  // TD error, loss sums, dQ at the taken action (coma_learner.py:124-131)
  if (tid < 16) {
    const int rr = r0 + tid;
    float m = 0.0f, q = 0.0f, y = 0.0f, dq = 0.0f;
    int at = 0;
    if (rr < R) {
      const int b = (int)fdiv((uint32_t)rr, a.d.dN), ag = rr - b * n;
      const int64_t slot = a.rp.ep(b) * a.d.t_stride + t;
      at = (int)a.rp.actions[slot * n + ag];
      m = coma_mask(a.rp, slot, t);
      q = Qs[tid * (A16 + 1) + at];
      y = a.tgt[(int64_t)t * R + rr];
      const float mtd = (q - y) * m;
      dq = (2.0f * mtd) * m;
      part[tid][0] = mtd * mtd; part[tid][1] = m; part[tid][2] = fabsf(mtd); part[tid][3] = q * m;
      part[tid][4] = y * m;
      a.dqc[rr] = dq;
      a.actc[rr] = at;
    } else {
      part[tid][0] = part[tid][1] = part[tid][2] = part[tid][3] = part[tid][4] = 0.0f;
    }
    dqs[tid] = dq;
    acts[tid] = at;
  }
  for (int e = tid; e < 16 * A; e += kHeadThreads) {   // the Q values the actor's baseline uses (coma_learner.py:126)
    const int i = e / A, aa = e - i * A;
    if (r0 + i < R) a.qvals[((int64_t)t * R + r0 + i) * A + aa] = Qs[i * (A16 + 1) + aa];
  }
  __syncthreads();
  if (tid < 5) {
    float s = 0.0f;
    for (int i = 0; i < 16; ++i) s += part[i][tid];
    a.cpart[blockIdx.x * 8 + tid] = s;
  }
  // dH2 = dQ W3 o [H2 > 0] (dQ is one-hot at the taken action)
  for (int e = tid; e < 16 * CH; e += kHeadThreads) {
    const int i = e >> 7, u = e & 127;
    const float h2 = H2s[i * CP + u];
    const float v = h2 > 0.0f ? dqs[i] * W3s[acts[i] * CP + u] : 0.0f;
    dHs[i * CP + u] = v;
    if (r0 + i < R) {
      a.dH2c[(int64_t)(r0 + i) * CH + u] = v;
      a.H2c[(int64_t)(r0 + i) * CH + u] = h2;
    }
  }
  __syncthreads();
  // dH1 = dH2 W2 o [H1 > 0]: B[kk][j] = W2[kk][j]
  if (w < 8) {
    const int jt = w;
    f32x4 acc = {0, 0, 0, 0};
    for (int k = 0; k < CH; k += 4) acc = mfma_f32_16x4(dHs[c * CP + k + g], W2s[(k + g) * CP + 16 * jt + c], acc);
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      const int i = 4 * g + reg, j = 16 * jt + c;
      if (r0 + i < R) a.dH1c[(int64_t)(r0 + i) * CH + j] = H1s[i * CP + j] > 0.0f ? acc[reg] : 0.0f;
    }
  }
}

// wgrad: every critic gradient element of step t on MFMA, one writer each, per-block sums of squares for the norm.
// A block owns 16 output rows (units, or actions for fc3) x 64 columns; wave w 16 of those columns; K = the R rows
// of the step. The bias gradient is the column one past the weight's last (its B operand is the constant 1), so
// every reduction over rows runs in the same MFMA order and no block loops over rows on its own.
//   blocks [0, 8 N1)              dW1 | db1   (B = X_t, N1 = ceil((Kc + 1) / 64) column tiles)
//   blocks [8 N1, 8 N1 + 24)      dW2 | db2   (B = H1)
//   blocks [.., + 3 A16 / 16)     dW3 | db3   (A = dQ, one-hot at the taken action; B = H2)
//   last block                    the step's bookkeeping
__host__ __device__ inline int wgrad_blocks(const CDims& d) {
  const int N1 = (d.Kc + 1 + 63) / 64, A16 = (d.A + 15) / 16 * 16;
  return 8 * N1 + 24 + 3 * (A16 / 16) + 1;
}

__global__ __launch_bounds__(256) void coma_wgrad_kernel(CritArgs a, int t) {
  const float mt = a.msum[t];   // checked once the first operands are in flight
  const int R = a.d.R, Kp = a.d.Kp, Kc = a.d.Kc, A = a.d.A;
  const int N1 = (Kc + 1 + 63) / 64, A16 = (A + 15) / 16 * 16;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, g = lane >> 4, c = lane & 15;
  const int bid = blockIdx.x;
  __shared__ float redsq[4];
  float sq = 0.0f;
  const int nb1 = 8 * N1, nb2 = nb1 + 24, nb3 = nb2 + 3 * (A16 / 16);
  if (bid < nb3) {
    int kind, u0, j0;
    if (bid < nb1) { kind = 1; u0 = 16 * (bid / N1); j0 = 64 * (bid % N1); }
    else if (bid < nb2) { kind = 2; u0 = 16 * ((bid - nb1) / 3); j0 = 64 * ((bid - nb1) % 3); }
    else { kind = 3; u0 = 16 * ((bid - nb2) / 3); j0 = 64 * ((bid - nb2) % 3); }
    const float* Bop = kind == 1 ? a.X + (int64_t)t * R * Kp : (kind == 2 ? a.H1c : a.H2c);
    const int ldb = kind == 1 ? Kp : CH, ncol = kind == 1 ? Kc : CH;
    const int nrow = kind == 3 ? A : CH;
    const int64_t o_w = kind == 1 ? a.o_w1 : (kind == 2 ? a.o_w2 : a.o_w3);
    const int64_t o_b = kind == 1 ? a.o_b1 : (kind == 2 ? a.o_b2 : a.o_b3);
    const float* dH = kind == 1 ? a.dH1c : a.dH2c;
    const int jc = j0 + 16 * w + c, u = u0 + c;
    f32x4 acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
    auto opA = [&](int rr) -> float {
      if (rr >= R) return 0.0f;
      if (kind == 3) return a.actc[rr] == u ? a.dqc[rr] : 0.0f;
      return dH[(int64_t)rr * CH + u];
    };
    auto opB = [&](int rr) -> float {
      if (rr >= R) return 0.0f;
      return jc < ncol ? Bop[(int64_t)rr * ldb + jc] : (jc == ncol ? 1.0f : 0.0f);
    };
    constexpr int RC = 32;   // k-steps of 4 rows whose operands are loaded in one round trip
    for (int r0 = 0; r0 < R; r0 += 4 * RC) {
      float av[RC], bv[RC];
#pragma unroll
      for (int q = 0; q < RC; ++q) { av[q] = opA(r0 + 4 * q + g); bv[q] = opB(r0 + 4 * q + g); }
      if (r0 == 0 && !(mt > 0.0f)) return;
#pragma unroll
      for (int q = 0; q < RC; q += 2) {
        acc0 = mfma_f32_16x4(av[q], bv[q], acc0);
        acc1 = mfma_f32_16x4(av[q + 1], bv[q + 1], acc1);
      }
    }
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      const int row = u0 + 4 * g + reg;
      const float v = acc0[reg] + acc1[reg];
      if (row < nrow && jc <= ncol) {
        if (jc < ncol) a.G[o_w + (int64_t)row * ncol + jc] = v;
        else a.G[o_b + row] = v;
        sq = fmaf(v, v, sq);
      }
    }
  } else if (!(mt > 0.0f)) {
    return;
  } else if (tid == 0) {
    float* rec = a.crec + t * 8;
    for (int k = 0; k < 5; ++k) {
      if (k == 1) continue;
      float s = 0.0f;
      for (int i = 0; i < a.nhead; ++i) s += a.cpart[i * 8 + k];
      rec[k] = s;
    }
    rec[1] = a.msum[t];   // = the sum of the head partials [1] (integer-valued); the global one when data-parallel
    rec[6] = 1.0f;
    a.G[a.Pc] = a.msum[t];   // normaliser of the pending update
    a.cstate[0] += 1;
    a.cstate[1] = t;
  }
  sq = wave_sum(sq);
  if (lane == 0) redsq[w] = sq;
  __syncthreads();
  if (tid == 0) a.cnorm[bid] = (redsq[0] + redsq[1]) + (redsq[2] + redsq[3]);
}

// The last live step's update over every critic parameter (after the reversed-t loop), into the caller's buffers
// (in place when the last version already lives there: each element is read and written by one thread). The
// clipped gradient stays in G, as .grad holds the last critic step's after the reference's train().
__global__ __launch_bounds__(256) void coma_capply_kernel(CritArgs a) {
  const int L = a.cstate[0];
  if (L <= 0) return;
  __shared__ float sh[4];
  crit_coef(a, sh);
  __syncthreads();
  const float inv = sh[0], coef = sh[1];
  const int src = (L - 1) & 1;
  if (blockIdx.x == 0 && threadIdx.x == 0) a.crec[a.cstate[1] * 8 + 5] = sh[2];
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < a.Pc; i += (int64_t)gridDim.x * 256) {
    const float g = (a.G[i] * inv) * coef;
    const float v = a.SQ[src][i] * a.hp.alpha + (1.0f - a.hp.alpha) * (g * g);
    a.P[0][i] = a.P[src][i] + (-a.hp.lr) * (g / (sqrtf(v) + a.hp.eps));
    a.SQ[0][i] = v;
    a.G[i] = g;
  }
}

// ----------------------------------------------------------------------------------------------- actor
// One wave per (t, row), lanes = actions: BasicMAC.forward's pi_logits branch (basic_controller.py:53-73) and the
// learner's renormalised masked policy, counterfactual baseline, advantage and log-pi term (coma_learner.py:59-77),
// and the backward of sum(adv log pi m) down to the logits (unnormalised: the apply divides by sum m).
// Writes dL [RT][Ap] (pad columns zero), pi [RT][A], per-block sums:
// [0] -sum adv log pi m, [1] sum m, [2] sum adv m, [3] sum max(pi) m.
// qvals [T][qv_R][A]: the critic's Q values, this launch's rows starting at row qv_r0 (an actor shard of a
// replicated critic; else qv_R = d.R, qv_r0 = 0).
__global__ __launch_bounds__(256) void coma_policy_kernel(Dims d, Rep rp, const float* __restrict__ logits,
                                                          const float* __restrict__ qvals, int qv_R, int qv_r0,
                                                          float eps, float omeps,
                                                          int mbs,
                                                          int Ap, float* __restrict__ dL, float* __restrict__ pi_out,
                                                          float* __restrict__ part) {
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t tr = (int64_t)blockIdx.x * 4 + wv;
  const int A = d.A, n = d.n;
  const int64_t RT = d.RT();
  __shared__ float red[4][4];
  float s_loss = 0.0f, s_m = 0.0f, s_adv = 0.0f, s_pmax = 0.0f;
  if (tr < RT) {
    const int t = (int)fdiv((uint32_t)tr, d.dR), r = (int)(tr - (int64_t)t * d.R);
    const int b = (int)fdiv((uint32_t)r, d.dN), ag = r - b * n;
    const int64_t slot = rp.ep(b) * d.t_stride + t;
    const bool on = lane < A;
    const int av = on ? rp.avail[(slot * n + ag) * A + lane] : 0;
    float l = on ? logits[tr * A + lane] : -INFINITY;
    if (mbs && on && !av) l = -1e10f;
    const float mx = wave_max(l);
    const float ex = on ? expf(l - mx) : 0.0f;
    const float sm = ex / wave_sum(ex);
    const float nact = mbs ? wave_sum(av ? 1.0f : 0.0f) : (float)A;
    float out = on ? omeps * sm + eps / nact : 0.0f;
    if (!av) out = 0.0f;                                   // mac_out[avail == 0] = 0
    const float s = wave_sum(out);
    const float p = (av && s > 0.0f) ? out / s : 0.0f;     // renormalise; 0/0 rows -> 0 (coma_learner.py:60-62)
    const float qv = on ? qvals[((int64_t)t * qv_R + qv_r0 + r) * A + lane] : 0.0f;
    const float baseline = wave_sum(p * qv);
    const int at = (int)rp.actions[slot * n + ag];
    const float q_taken = __shfl(qv, at, 64);
    const float m = coma_mask(rp, slot, t);
    const float pt = m == 0.0f ? 1.0f : __shfl(p, at, 64);
    const float adv = q_taken - baseline;
    const float lp = logf(pt);
    const float pmax = wave_max(on ? p : -INFINITY);
    s_loss = -(adv * lp) * m; s_m = m; s_adv = adv * m; s_pmax = pmax * m;
    // backward of -sum adv log pi m (unnormalised) down to the logits
    const float dpt = m == 0.0f ? 0.0f : (-(adv * m)) / pt;
    const float dp = (av && lane == at) ? dpt : 0.0f;
    const float dout = (av && s > 0.0f) ? (dp - dpt * pt) / s : 0.0f;
    const float dsm = omeps * dout;
    float dl = sm * (dsm - wave_sum(sm * dsm));
    if (mbs && !av) dl = 0.0f;
    if (lane < Ap) dL[tr * Ap + lane] = on ? dl : 0.0f;
    if (on) pi_out[tr * A + lane] = p;
  }
  if (lane == 0) { red[wv][0] = s_loss; red[wv][1] = s_m; red[wv][2] = s_adv; red[wv][3] = s_pmax; }
  __syncthreads();
  if (threadIdx.x < 8) {
    const int k = threadIdx.x;
    part[(int64_t)blockIdx.x * 8 + k] = k < 4 ? ((red[0][k] + red[1][k]) + (red[2][k] + red[3][k])) : 0.0f;
  }
}

// dHo = dL W2: the output-layer gradient entering the BPTT chain, [RT][64] (K = n_actions).
struct DhoProb {
  static constexpr int BN = 64;
  const float* dL;   // [M][Ap]
  int Ap, A;
  const float* W2;   // [A][H]
  float* dHo;        // [M][H]
  int64_t M;
  using APat = KPat;
  using BPat = MPat;
  static constexpr bool kRowSum = false;
  struct Ctx {
    const float* arow;
  };
  MQ_DEV Ctx make_ctx(int m0, int, int, int tid) const {
    const int64_t m = m0 + KPat::row(tid);
    return Ctx{m < M ? dL + m * Ap : nullptr};
  }
  MQ_DEV void krange(int, int& kb, int& ke) const { kb = 0; ke = A; }
  MQ_DEV void load_a(const Ctx& c, int k0, int, float (&r)[4]) const {
    const int k = k0 + KPat::kq(threadIdx.x);
    ld4((c.arow && k < Ap) ? c.arow + k : nullptr, r);
  }
  MQ_DEV void load_b(const Ctx&, int, int k0, int ke, float (&r)[4]) const {
    const int nn = MPat::row(threadIdx.x), k = k0 + MPat::kq(threadIdx.x);
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = k + i < ke ? W2[(int64_t)(k + i) * H + nn] : 0.0f;
  }
  MQ_DEV void epilogue(const Ctx&, const f32x16& acc, int mrow0, int ncol0, int, int lane) const {
    for_tile(acc, mrow0, ncol0, lane, [&](int m, int j, float v) {
      if (m < M) dHo[(int64_t)m * H + j] = v;
    });
  }
  MQ_DEV void rowsum_out(int, int, float) const {}
};

// [dW2 | db2] slab = dL^T Hs over rows tr (split-K), fc2 of rnn_agent.py:35.
struct Dw2Prob {
  static constexpr int BN = 64;
  const float* dL;   // [K][Ap]
  int Ap, A;
  const float* Hs;   // [K][H] online hidden states
  float* slab;       // [nsplit][A*H + A]
  int64_t K;
  int nsplit;
  using APat = MPat;
  using BPat = MPat;
  static constexpr bool kRowSum = true;
  struct Ctx {
    int dummy;
  };
  MQ_DEV Ctx make_ctx(int, int, int, int) const { return Ctx{0}; }
  MQ_DEV void krange(int z, int& kb, int& ke) const { krange_split((int)K, nsplit, z, kb, ke); }
  MQ_DEV void load_a(const Ctx&, int k0, int ke, float (&r)[4]) const {
    const int aa = MPat::row(threadIdx.x), k = k0 + MPat::kq(threadIdx.x);
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = (aa < A && k + i < ke) ? dL[(int64_t)(k + i) * Ap + aa] : 0.0f;
  }
  MQ_DEV void load_b(const Ctx&, int, int k0, int ke, float (&r)[4]) const {
    const int j = MPat::row(threadIdx.x), k = k0 + MPat::kq(threadIdx.x);
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = (k + i < ke) ? Hs[(int64_t)(k + i) * H + j] : 0.0f;
  }
  MQ_DEV void epilogue(const Ctx&, const f32x16& acc, int mrow0, int ncol0, int z, int lane) const {
    float* out = slab + (int64_t)z * (A * H + A);
    for_tile(acc, mrow0, ncol0, lane, [&](int aa, int j, float v) {
      if (aa < A) out[(int64_t)aa * H + j] = v;
    });
  }
  MQ_DEV void rowsum_out(int aa, int z, float v) const {
    if (aa < A) slab[(int64_t)z * (A * H + A) + A * H + aa] = v;
  }
};

// Data-parallel ranks other than 0 zero the replicated fields of the per-step record (mask sum, grad norm, live flag)
// before it is summed over the ranks, so the sum carries rank 0's values exactly.
__global__ __launch_bounds__(256) void coma_dp_crec_kernel(float* __restrict__ crec, int T) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t < T) { crec[t * 8 + 1] = 0.0f; crec[t * 8 + 5] = 0.0f; crec[t * 8 + 6] = 0.0f; }
}

// Final stats (coma_learner.py:85-96): means of the per-step critic stats over the live steps in the order the
// reference logs them (reversed t), then the actor's stats from the agent apply (stats[8..11] scratch on entry).
__global__ void coma_stats_kernel(const float* __restrict__ crec, int T, const int* __restrict__ cstate,
                                  float* __restrict__ stats) {
  // one wave: lane l takes steps l, l + 64, .. (all loads in flight), then a fixed butterfly over the lanes
  // (a single thread walking T records was ~61 us at T = 180: one dependent load chain)
  if (blockIdx.x != 0) return;
  const int lane = threadIdx.x;
  double s[5] = {0, 0, 0, 0, 0};
  double cntd = 0.0;
  for (int t0 = 0; t0 < T; t0 += 256) {
    float r[4][8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int t = t0 + lane + 64 * j;
#pragma unroll
      for (int k = 0; k < 8; ++k) r[j][k] = t < T ? crec[t * 8 + k] : 0.0f;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (r[j][6] == 0.0f) continue;
      const double msum = r[j][1];
      s[0] += (double)(r[j][0] / r[j][1]);
      s[1] += (double)r[j][5];
      s[2] += (double)r[j][2] / msum;
      s[3] += (double)r[j][3] / msum;
      s[4] += (double)r[j][4] / msum;
      cntd += 1.0;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
#pragma unroll
    for (int k = 0; k < 5; ++k) s[k] += __shfl_xor(s[k], o, 64);
    cntd += __shfl_xor(cntd, o, 64);
  }
  if (lane != 0) return;
  const int cnt = (int)cntd;
  // the agent apply_kernel wrote [loss, norm, sums[2]/msum, sums[3]/msum, sums[4]/msum, msum, coef, 0] at stats + 8
  const float a_loss = stats[8], a_norm = stats[9], a_adv = stats[10], a_pmax = stats[11], a_msum = stats[13];
  for (int k = 0; k < 5; ++k) stats[k] = cnt ? (float)(s[k] / cnt) : 0.0f;
  if (cstate[3] != 0)   // the persistent critic chain's error word (a grid barrier timed out): loud, not silent
    for (int k = 0; k < 5; ++k) stats[k] = __builtin_nanf("");
  stats[5] = a_adv;
  stats[6] = a_loss;
  stats[7] = a_norm;
  stats[8] = a_pmax;
  stats[9] = cstate[3] != 0 ? -1.0f : (float)cstate[0];   // -1: the critic chain failed (the learner raises)
  stats[10] = a_msum;
}

// BasicMAC.forward's pi_logits post-processing on the rollout side (basic_controller.py:53-73), in place.
__global__ __launch_bounds__(256) void mc_policy_kernel(float* __restrict__ x, const int32_t* __restrict__ avail,
                                                        int rows, int A, float eps, int mbs, int test_mode) {
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + wv;
  if (row >= rows) return;
  const bool on = lane < A;
  const int av = on ? avail[(int64_t)row * A + lane] : 0;
  float l = on ? x[(int64_t)row * A + lane] : -INFINITY;
  if (mbs && on && !av) l = -1e10f;
  const float mx = wave_max(l);
  const float ex = on ? expf(l - mx) : 0.0f;
  float p = ex / wave_sum(ex);
  if (!test_mode) {
    const float nact = mbs ? wave_sum(av ? 1.0f : 0.0f) : (float)A;
    p = (1.0f - eps) * p + (1.0f * eps) / nact;
    if (mbs && !av) p = 0.0f;
  }
  if (on) x[(int64_t)row * A + lane] = p;
}

}  // namespace mq
