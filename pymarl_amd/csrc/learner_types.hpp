// Shapes, replay view and workspace of one learner train step (shared by every kernel of the step).
#pragma once
#include "common.hpp"
#include "../../include/mq_learner.h"

namespace mq {

constexpr int H = 64;        // rnn_hidden_dim (reference default, rnn_agent.py:19-21)
constexpr int G3 = 3 * H;    // GRU gate width (r, z, n)

struct Dims {
  int n, A, O, S, E, I, NH;  // agents, actions, obs, state, mixer embed, agent input width, hypernet outputs
  int B, Tp, T, R, M;        // episodes, unrolled steps (max_t_filled), transitions, rows B*n, mixer rows T*B
  int t_stride;              // storage max_seq_length
  int last_action, agent_id, mixer, double_q;
  float gamma;
  float huber;                      // TD loss: 0 = masked L2 (the reference), > 0 = Huber delta (opt-in)
  FastDiv dR, dN, dB, dO, dI, dS;   // fast division by R, n, B, obs / agent-input / state widths
  MQ_DEV int64_t RT() const { return (int64_t)Tp * R; }
};

// The masked TD loss term of one transition and its derivative d/dQ_tot (before the 1 / mask_sum scale).
// delta == 0: L2, (td m)^2 (q_learner.py:96-97, the reference's loss and the default). delta > 0: Huber, an opt-in
// the reference lacks (north_star names it): 0.5 x^2 for |x| <= delta, delta (|x| - delta / 2) beyond, x = td m.
MQ_DEV float td_loss(float mtd, float delta) {
  if (delta > 0.0f) {
    const float ax = fabsf(mtd);
    return ax <= delta ? 0.5f * mtd * mtd : delta * (ax - 0.5f * delta);
  }
  return mtd * mtd;
}
MQ_DEV float td_dy(float mtd, float mask, float delta) {
  return delta > 0.0f ? fminf(fmaxf(mtd, -delta), delta) * mask : (2.0f * mtd) * mask;
}

// Borrowed replay storage (reference scheme dtypes), episode-major, plus the sampled episode ids.
struct Rep {
  const float* obs;
  const float* state;
  const int64_t* actions;
  const int32_t* avail;
  const float* reward;
  const uint8_t* term;
  const int64_t* filled;
  const int64_t* ep_ids;
  const uint64_t* avail_bits = nullptr;   // optional bitmask view of avail (mq_replay.avail_bits); NULL: avail
  int32_t nids;                    // > 0: the ids live in `ids` (kernel arguments), ep_ids unused
  int32_t ids[MQ_INLINE_IDS];
  MQ_DEV int64_t ep(int b) const { return nids ? (int64_t)ids[b] : (ep_ids ? ep_ids[b] : (int64_t)b); }
};

struct Lay {
  int64_t o[MQ_P_COUNT + 1];
};

// Activation workspace, time-major: row index tr = t*R + r with r = b*n + agent.
struct Work {
  float* X1;      // [2][RT][H]   relu(fc1) per net
  float* GI;      // [2][RT][3H]  W_ih x1 + b_ih per net
  float* Hs;      // [2][RT][H]   hidden after step t per net
  float* Gates;   // [RT][4H]     online r, z, n, W_hn h + b_hn
  float* Q;       // [2][RT][A]   mac_out / target_mac_out
  float* HYP;     // [2][M][NH]   QMIX hypernet outputs per net (state t for online, t+1 for target)
  float* dHYP;    // [M][NH]
  float* dch;     // [T*R]        dLoss_num/dchosen
  float* dGI;     // [RT][3H]
  float* dP1;     // [RT][H]
  float* slab_fc1;   // [nsplit][H*I + H]
  float* slab_rnn;   // [blocks][len_rnn]   w_ih, w_hh, b_ih, b_hh, fc2.w, fc2.b
  float* slab_mix;   // [nsplit][len_mix]   hyper_w_1 .. V.0 (weights+biases)
  float* slab_v2;    // [mix blocks][E+1]   V.2 weight, bias
  float* loss_part;  // [mix blocks][8]
  float* norm_part;  // [norm blocks]
  int32_t* curmax;   // [T*R]
  float* red_tmp;    // two-pass slab reduction partials
  float* XIN;        // [RT][I]  dense agent inputs (written by the fc1 pass, read by dW1)
  float* S0;         // [M][S]   gathered state[:, :-1] rows (written by the hypernet pass, read by dW_hyper)
  float* dHo;        // [RT][H]  COMA actor only: dLogits W2 per (t, row), read by gru_bwd_kernel<.., DY = true>
  // dW_hyper tiles appended to the fused BPTT's grid (gru_bwd_fused.hpp, DWH = 1): slab length, m-slices, j-tiles,
  // tile count
  int64_t dwh_len = 0;
  int dwh_ns = 0, dwh_tj = 0, dwh_n = 0;
};

MQ_DEV void split_tr(const Dims& d, uint32_t tr, int& t, int& r, int& b, int& ag) {
  t = (int)fdiv(tr, d.dR);
  r = (int)tr - t * d.R;
  b = (int)fdiv((uint32_t)r, d.dN);
  ag = r - b * d.n;
}

}  // namespace mq
