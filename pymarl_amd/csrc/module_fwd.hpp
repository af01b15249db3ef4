// Standalone module forwards outside train(): QMixer.forward (qmix.py:28-47) and COMACritic.forward
// (coma.py:22-58), for callers that evaluate a mixer or a critic directly (evaluation / analysis scripts).
// Inside the learners both run fused into the train step; these kernels serve the module API.
#pragma once
#include "coma_kernels.hpp"

namespace mq {

constexpr int QMF_ROWS = 4;   // (batch, t) rows per workgroup: the hypernet weights are read once per 4 rows

// Mixer parameter block (QMixer.parameters() order, qmix.py:17-26), offsets relative to hyper_w_1.weight.
struct QmixOff {
  int64_t w1w, w1b, wfw, wfb, b1w, b1b, v0w, v0b, v2w, v2b;
  MQ_DEV QmixOff(int n, int S, int E) {
    w1w = 0; w1b = (int64_t)E * n * S; wfw = w1b + (int64_t)E * n; wfb = wfw + (int64_t)E * S; b1w = wfb + E;
    b1b = b1w + (int64_t)E * S; v0w = b1b + E; v0b = v0w + (int64_t)E * S; v2w = v0b + E; v2b = v2w + E;
  }
};

inline size_t qmix_forward_lds(int n, int S, int E) {
  return (size_t)QMF_ROWS * (S + (size_t)E * (n + 3)) * sizeof(float);
}

// One workgroup per QMF_ROWS rows. Phase 1: the hypernet outputs of the rows (thread o computes output o of
// [hyper_w_1 | hyper_w_final | hyper_b_1 | V.0] for all rows, states broadcast from LDS). Phase 2: wave w mixes row
// w: lane e < E forms hidden_e = elu(sum_i q_i |w1[i][e]| + b1_e), the wave sums hidden_e |wf_e| and
// relu(V.0(s))_e V.2_e, and adds V.2's bias.
__global__ __launch_bounds__(256) void qmix_forward_kernel(const float* __restrict__ W, int n, int S, int E,
                                                           const float* __restrict__ qs, const float* __restrict__ st,
                                                           float* __restrict__ out, int rows) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int NH = E * (n + 3);
  float* s_st = lds;                       // [QMF_ROWS][S]
  float* s_h = lds + QMF_ROWS * S;         // [QMF_ROWS][NH]
  const int m0 = blockIdx.x * QMF_ROWS;
  const QmixOff o(n, S, E);
  for (int e = threadIdx.x; e < QMF_ROWS * S; e += 256) {
    const int i = e / S, k = e - i * S;
    s_st[e] = m0 + i < rows ? st[(int64_t)(m0 + i) * S + k] : 0.0f;
  }
  __syncthreads();
  for (int oo = threadIdx.x; oo < NH; oo += 256) {
    const float* wrow;
    float bias;
    if (oo < E * n) { wrow = W + o.w1w + (int64_t)oo * S; bias = W[o.w1b + oo]; }
    else if (oo < E * n + E) { const int j = oo - E * n; wrow = W + o.wfw + (int64_t)j * S; bias = W[o.wfb + j]; }
    else if (oo < E * n + 2 * E) { const int j = oo - E * n - E; wrow = W + o.b1w + (int64_t)j * S; bias = W[o.b1b + j]; }
    else { const int j = oo - E * n - 2 * E; wrow = W + o.v0w + (int64_t)j * S; bias = W[o.v0b + j]; }
    float acc[QMF_ROWS];
#pragma unroll
    for (int i = 0; i < QMF_ROWS; ++i) acc[i] = 0.0f;
    for (int k = 0; k < S; ++k) {
      const float wk = wrow[k];
#pragma unroll
      for (int i = 0; i < QMF_ROWS; ++i) acc[i] = fmaf(wk, s_st[i * S + k], acc[i]);
    }
#pragma unroll
    for (int i = 0; i < QMF_ROWS; ++i) s_h[i * NH + oo] = acc[i] + bias;
  }
  __syncthreads();
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63, m = m0 + wv;
  if (wv >= QMF_ROWS || m >= rows) return;
  const float* h = s_h + wv * NH;
  float part = 0.0f, vpart = 0.0f;
  if (lane < E) {
    float pre = 0.0f;
    for (int i = 0; i < n; ++i) pre = fmaf(qs[(int64_t)m * n + i], fabsf(h[i * E + lane]), pre);
    pre += h[E * n + E + lane];                                   // + b1
    const float hid = pre > 0.0f ? pre : expm1f(pre);              // F.elu
    part = hid * fabsf(h[E * n + lane]);                           // bmm(hidden, |w_final|)
    vpart = fmaxf(h[E * n + 2 * E + lane], 0.0f) * W[o.v2w + lane];   // V.2(relu(V.0 s))
  }
#pragma unroll
  for (int sh = 32; sh > 0; sh >>= 1) {
    part += __shfl_xor(part, sh, 64);
    vpart += __shfl_xor(vpart, sh, 64);
  }
  if (lane == 0) out[m] = part + (vpart + W[o.v2b]);
}

// COMACritic output layout: the GEMM writes Q[t][b * n + agent][A]; the module returns [b][t][agent][A].
__global__ __launch_bounds__(256) void coma_q_layout_kernel(const float* __restrict__ q, float* __restrict__ out,
                                                            int Tq, int B, int n, int A) {
  const int64_t total = (int64_t)Tq * B * n * A;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int a = (int)(e % A);
    int64_t rest = e / A;
    const int ag = (int)(rest % n);
    rest /= n;
    const int t = (int)(rest % Tq);
    const int b = (int)(rest / Tq);
    out[e] = q[(((int64_t)t * B + b) * n + ag) * A + a];
  }
}

}  // namespace mq
