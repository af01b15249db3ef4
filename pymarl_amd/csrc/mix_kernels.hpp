// Per-(episode, t) tail of QLearner.train: chosen-action gather, double-Q target selection, QMIX / VDN mixing
// (forward for both nets), 1-step TD target, masked L2 terms, the learner stats sums, and the mixer backward
// down to dLoss/dchosen (q_learner.py:39-97; qmix.py:28-47; vdn.py:9-10).
//
// One wave per (t, b) pair m = t*B + b; 4 pairs per 256-thread workgroup. Lanes play agents for the
// selection (argmax over available actions, first index on ties as torch max) and embedding units for the
// mixer; the few cross-lane sums are wave reductions. Loss sums stay UNNORMALISED (sum (td*m)^2 etc.) so a
// data-parallel all-reduce of them reproduces the reference's global / sum(mask) exactly.
#pragma once
#include "learner_types.hpp"

namespace mq {

MQ_DEV float sgnf(float x) { return (float)((x > 0.0f) - (x < 0.0f)); }
MQ_DEV float eluf(float x) { return x > 0.0f ? x : expm1f(x); }

struct MixOut {
  float y, pre, hid, wf_raw, hv;   // lane-e intermediates of the online mixer (QMIX)
};

// QMIX forward for one (t, b): lanes e < E. Returns y (same on every lane).
MQ_DEV float qmix_fwd_lane(const float* hyp, const float* qs_lds, const float* V2w, float V2b, int n, int E,
                           int lane, MixOut* keep) {
  const int nE = n * E;
  float prod = 0.0f, vt = 0.0f, pre = 0.0f, hid = 0.0f, wfr = 0.0f, hv = 0.0f;
  if (lane < E) {
    float acc = 0.0f;
    for (int a0 = 0; a0 < n; a0 += 8) {   // bmm(q, |w1|), 8 independent loads per round trip
      float hv8[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) hv8[u] = hyp[min(a0 + u, n - 1) * E + lane];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (a0 + u < n) acc = fmaf(qs_lds[a0 + u], fabsf(hv8[u]), acc);
    }
    pre = acc + hyp[nE + E + lane];                                                          // + b1
    hid = eluf(pre);
    wfr = hyp[nE + lane];
    prod = hid * fabsf(wfr);                                                                 // bmm(hid, |wf|)
    hv = hyp[nE + 2 * E + lane];
    vt = fmaxf(hv, 0.0f) * V2w[lane];                                                        // V(s)
  }
  const float y = wave_sum(prod) + (wave_sum(vt) + V2b);
  if (keep) { keep->y = y; keep->pre = pre; keep->hid = hid; keep->wf_raw = wfr; keep->hv = hv; }
  return y;
}

// STREAM (mix_stream_ok: n * A <= MIXS_MAX): the selection's operands — the four items' Q rows at t+1 (one
// contiguous run of 4 n A floats when B % 4 == 0) and their avail rows — are staged by the whole workgroup with
// coalesced loads, every load in flight at once, masked on the way into LDS; each agent lane then scans its row
// from LDS. The generic form has every agent lane walk its own row in global memory (A-strided 4-byte loads,
// ceil(A / 12) dependent rounds), which held configs[2]'s mixer (n = 27, A = 36) at 2 TB/s. Same comparisons in the
// same order: identical outputs.
constexpr int MIXS_MAX = 1024;   // n * A staged per item
constexpr int MIXS_NPT = MIXS_MAX / 256;
inline bool mix_stream_ok(int n, int A) { return n * A <= MIXS_MAX; }

template <bool STREAM>
__global__ __launch_bounds__(256) void mix_kernel(Dims d, Rep rp, const float* __restrict__ P0,
                                                  const float* __restrict__ P1, Lay L, Work w, int32_t* curmax_out) {
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int m = blockIdx.x * 4 + wv;
  const int n = d.n, A = d.A, E = d.E, R = d.R, NH = d.NH;
  __shared__ float chs[4][64], tms[4][64], dps[4][64];
  __shared__ float red[4][8];
  __shared__ float v2red[4][65];
  float l2 = 0.0f, msk = 0.0f, abs_ = 0.0f, qs = 0.0f, tg = 0.0f;   // lane-0 partials of this wave
  float dv2 = 0.0f, dv2b = 0.0f;
  const bool valid = m < d.M;
  int t = 0, b = 0;
  int64_t ep = 0;
  if (valid) {
    t = (int)fdiv((uint32_t)m, d.dB);
    b = m - t * d.B;
    ep = rp.ep(b);
  }
  const float* Qon = w.Q;
  const float* Qtg = w.Q + d.RT() * A;
  float chosen = 0.0f, tmax = 0.0f;
  // the transition's mask / reward / terminated words, independent of the selection: in flight with it
  float mask = 0.0f, rew = 0.0f, term = 0.0f;
  if (valid) {
    const int64_t slot = ep * d.t_stride + t;
    mask = (float)rp.filled[slot];
    if (t > 0) mask *= 1.0f - (float)rp.term[slot - 1];   // q_learner.py:42-43
    rew = rp.reward[slot];
    term = (float)rp.term[slot];
  }
  if constexpr (STREAM) {
    __shared__ float qm[4 * MIXS_MAX];      // the four items' masked selection rows [item][agent][action]
    __shared__ uint8_t avs[4 * MIXS_MAX];   // their avail bits
    const int nA = n * A;
    const float* qsel_base = d.double_q ? Qon : Qtg;
    float qv[4][MIXS_NPT];
    int32_t avv[4][MIXS_NPT];
    // the agent lane's action first (its chosen value is one more round trip), then every staging load of the block
    // (avail as int32 here: per-element bit extraction from mq_replay.avail_bits measured slower, 74 vs 70 us)
    const int at = (valid && lane < n) ? (int)rp.actions[(ep * d.t_stride + t) * n + lane] : 0;
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int mi = min((int)blockIdx.x * 4 + it, d.M - 1);
      const int ti = (int)fdiv((uint32_t)mi, d.dB), bi = mi - ti * d.B;
      const float* qrow = qsel_base + ((int64_t)(ti + 1) * R + (int64_t)bi * n) * A;
      const int32_t* arow = rp.avail + ((rp.ep(bi) * d.t_stride + ti + 1) * n) * (int64_t)A;
#pragma unroll
      for (int k = 0; k < MIXS_NPT; ++k) {
        const int e = min((int)threadIdx.x + 256 * k, nA - 1);
        qv[it][k] = qrow[e];
        avv[it][k] = arow[e];
      }
    }
    if (valid && lane < n) chosen = Qon[((int64_t)t * R + b * n + lane) * A + at];
#pragma unroll
    for (int it = 0; it < 4; ++it)
#pragma unroll
      for (int k = 0; k < MIXS_NPT; ++k) {
        const int e = threadIdx.x + 256 * k;
        if (e < nA) {
          qm[it * nA + e] = avv[it][k] ? qv[it][k] : kNegMask;
          avs[it * nA + e] = avv[it][k] ? 1 : 0;
        }
      }
    __syncthreads();
    if (valid && lane < n) {
      const int r = b * n + lane;
      const float* row = qm + wv * nA + lane * A;
      float best = 0.0f;
      int cur = 0;
      for (int a = 0; a < A; ++a) {
        const float v = row[a];
        if (a == 0 || v > best) { best = v; cur = a; }
      }
      if (d.double_q) tmax = avs[wv * nA + lane * A + cur] ? Qtg[((int64_t)(t + 1) * R + r) * A + cur] : kNegMask;
      else tmax = best;
      if (curmax_out) curmax_out[(int64_t)t * R + r] = cur;
    }
  } else
  // ---- chosen action values and double-Q target selection (q_learner.py:55, 68-78); lane = agent
  if (valid && lane < n) {
    const int r = b * n + lane;
    const int64_t slot = ep * d.t_stride + t;
    const int at = (int)rp.actions[slot * n + lane];
    chosen = Qon[((int64_t)t * R + r) * A + at];
    const float* qn = Qon + ((int64_t)(t + 1) * R + r) * A;
    const float* qt = Qtg + ((int64_t)(t + 1) * R + r) * A;
    const int32_t* av = rp.avail + ((slot + 1) * n + lane) * (int64_t)A;
    const uint64_t abits = rp.avail_bits ? rp.avail_bits[(slot + 1) * n + lane] : 0;
    auto avail_at = [&](int a) { return rp.avail_bits ? (int32_t)((abits >> a) & 1u) : av[a]; };
    // argmax over available actions, first index on ties (torch max): the row is fetched in blocks of kMB
    // independent loads so a wave waits on ceil(A / kMB) round trips instead of A
    const float* qsel = d.double_q ? qn : qt;
    constexpr int kMB = 12;
    float best = 0.0f;
    int cur = 0;
    for (int a0 = 0; a0 < A; a0 += kMB) {
      float qv[kMB];
      int32_t avv[kMB];
#pragma unroll
      for (int u = 0; u < kMB; ++u) {
        const int a = min(a0 + u, A - 1);
        qv[u] = qsel[a];
        avv[u] = avail_at(a);
      }
#pragma unroll
      for (int u = 0; u < kMB; ++u) {
        const int a = a0 + u;
        const float v = avv[u] ? qv[u] : kNegMask;
        if (a < A && (a == 0 || v > best)) { best = v; cur = a; }
      }
    }
    if (d.double_q) tmax = avail_at(cur) ? qt[cur] : kNegMask;
    else tmax = best;
    if (curmax_out) curmax_out[(int64_t)t * R + r] = cur;
  }
  chs[wv][lane] = chosen;
  tms[wv][lane] = tmax;
  __syncthreads();

  const float gamma = d.gamma;
  if (d.mixer == MQ_MIXER_QMIX) {
    const float* hon = w.HYP + (int64_t)m * NH;
    const float* htg = w.HYP + ((int64_t)d.M + m) * NH;
    const float* V2w0 = P0 + L.o[MQ_P_V2_W];
    const float* V2w1 = P1 + L.o[MQ_P_V2_W];
    MixOut k;
    float y = 0.0f, yt = 0.0f;
    if (valid) {
      y = qmix_fwd_lane(hon, chs[wv], V2w0, P0[L.o[MQ_P_V2_B]], n, E, lane, &k);
      yt = qmix_fwd_lane(htg, tms[wv], V2w1, P1[L.o[MQ_P_V2_B]], n, E, lane, nullptr);
    } else {
      k.y = k.pre = k.hid = k.wf_raw = k.hv = 0.0f;
    }
    const float target = rew + gamma * (1.0f - term) * yt;   // q_learner.py:86
    const float td = y - target;
    const float mtd = td * mask;
    l2 = td_loss(mtd, d.huber); msk = mask; abs_ = fabsf(mtd); qs = y * mask; tg = target * mask;
    const float dy = td_dy(mtd, mask, d.huber);   // d sum loss(td*m) / d Q_tot
    // ---- QMIX backward (lanes e < E)
    float dpre = 0.0f;
    if (valid && lane < E) {
      const float wf = fabsf(k.wf_raw);
      const float dhid = dy * wf;
      float* dh = w.dHYP + (int64_t)m * NH;
      dh[n * E + lane] = dy * k.hid * sgnf(k.wf_raw);                         // hyper_w_final
      dpre = dhid * (k.pre > 0.0f ? 1.0f : expf(k.pre));                      // elu'
      dh[n * E + E + lane] = dpre;                                            // hyper_b_1
      dh[n * E + 2 * E + lane] = dy * V2w0[lane] * (k.hv > 0.0f ? 1.0f : 0.0f);   // V.0 (through relu)
      dv2 = dy * fmaxf(k.hv, 0.0f);                                           // V.2 weight
      for (int a0 = 0; a0 < n; a0 += 8) {                                     // hyper_w_1 (through |.|)
        float hv8[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) hv8[u] = hon[min(a0 + u, n - 1) * E + lane];
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (a0 + u < n) dh[(a0 + u) * E + lane] = (chs[wv][a0 + u] * dpre) * sgnf(hv8[u]);
      }
    }
    dv2b = dy;
    dps[wv][lane] = dpre;
    __syncthreads();
    if (valid && lane < n) {
      float acc = 0.0f;
      for (int e0 = 0; e0 < E; e0 += 8) {
        float hv8[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) hv8[u] = hon[lane * E + min(e0 + u, E - 1)];
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (e0 + u < E) acc = fmaf(fabsf(hv8[u]), dps[wv][e0 + u], acc);
      }
      w.dch[(int64_t)t * R + b * n + lane] = acc;
    }
  } else {
    float y, yt;
    if (d.mixer == MQ_MIXER_VDN) {
      y = wave_sum(lane < n ? chosen : 0.0f);
      yt = wave_sum(lane < n ? tmax : 0.0f);
    } else {   // no mixer: per-agent TD (q_learner.py:81 skipped; mask expanded over agents)
      y = chosen;
      yt = tmax;
    }
    const float target = rew + gamma * (1.0f - term) * yt;
    const float td = y - target;
    const float mtd = td * mask;
    const float dy = td_dy(mtd, mask, d.huber);
    if (d.mixer == MQ_MIXER_VDN) {
      l2 = td_loss(mtd, d.huber); msk = mask; abs_ = fabsf(mtd); qs = y * mask; tg = target * mask;
    } else {
      const bool on = lane < n;
      l2 = wave_sum(on ? td_loss(mtd, d.huber) : 0.0f);
      msk = wave_sum(on ? mask : 0.0f);
      abs_ = wave_sum(on ? fabsf(mtd) : 0.0f);
      qs = wave_sum(on ? y * mask : 0.0f);
      tg = wave_sum(on ? target * mask : 0.0f);
    }
    if (valid && lane < n) w.dch[(int64_t)t * R + b * n + lane] = dy;
    __syncthreads();   // match the QMIX branch's barrier count
  }
  if (!valid) { l2 = msk = abs_ = qs = tg = 0.0f; dv2 = dv2b = 0.0f; }
  // ---- deterministic per-workgroup partials
  if (lane == 0) {
    red[wv][0] = l2; red[wv][1] = msk; red[wv][2] = abs_; red[wv][3] = qs; red[wv][4] = tg;
    v2red[wv][64] = dv2b;
  }
  v2red[wv][lane] = dv2;
  __syncthreads();
  if (threadIdx.x < 8) {
    const int c = threadIdx.x;
    float* out = w.loss_part + (int64_t)blockIdx.x * 8;
    out[c] = c < 5 ? ((red[0][c] + red[1][c]) + (red[2][c] + red[3][c])) : 0.0f;
  }
  if (d.mixer == MQ_MIXER_QMIX && threadIdx.x <= E) {
    const int e = threadIdx.x == E ? 64 : threadIdx.x;
    w.slab_v2[(int64_t)blockIdx.x * (E + 1) + threadIdx.x] =
        (v2red[0][e] + v2red[1][e]) + (v2red[2][e] + v2red[3][e]);
  }
}

}  // namespace mq

namespace mq {

// mix_kernel with every independent load of a wave issued up front (A <= MA actions, n <= MN agents, E <= 64):
// the agent's Q rows at t+1 (both nets), its avail row and action, the QMIX hypernet outputs of both nets, V.2 and
// the mask / reward / terminated words, all in one round trip; only the chosen-action value waits on the action.
// The generic kernel fetches them in dependent stages (action -> chosen, argmax blocks -> target value, then the
// hypernet rows after a barrier). Same arithmetic in the same order: bitwise-identical outputs.
//
// mix_fast_row is one wave's (t, b) row m: hon / htg point at its hypernet outputs (HYP rows in global memory),
// `sc` is the wave's LDS scratch, and the row's loss / V.2 partials
// land in red_slot[0..4] / v2_slot[0..64] for the caller's fixed-order block sums. Two workgroup barriers inside:
// every wave of the workgroup must call it the same number of times.
template <int MN>
struct alignas(16) MixScratch {
  float chs[64], tms[64], dps[64];
  float w1s[MN][65];   // |hyper_w_1| rows of the online mixer, for dLoss/dchosen
};

template <int MA, int MN>
MQ_DEV void mix_fast_row(const Dims& d, const Rep& rp, const float* __restrict__ P0, const float* __restrict__ P1,
                         const Lay& L, const Work& w, int32_t* curmax_out, int m, int lane, const float* hon,
                         const float* htg, MixScratch<MN>& sc, float* red_slot, float* v2_slot) {
  const int n = d.n, A = d.A, E = d.E, R = d.R, NH = d.NH;
  const bool qmix = d.mixer == MQ_MIXER_QMIX;
  float l2 = 0.0f, msk = 0.0f, abs_ = 0.0f, qs = 0.0f, tg = 0.0f;
  float dv2 = 0.0f, dv2b = 0.0f;
  const bool valid = m < d.M;
  int t = 0, b = 0;
  int64_t ep = 0;
  if (valid) {
    t = (int)fdiv((uint32_t)m, d.dB);
    b = m - t * d.B;
    ep = rp.ep(b);
  }
  const int64_t slot = ep * d.t_stride + t;
  const float* Qon = w.Q;
  const float* Qtg = w.Q + d.RT() * A;
  // ---- every independent load of the wave
  const bool agent_lane = valid && lane < n;
  const int r = b * n + min(lane, n - 1);
  int at = 0;
  float qsel[MA], qtr[MA];
  int32_t avr[MA];
  if (agent_lane) {
    at = (int)rp.actions[slot * n + lane];
    const float* qn = Qon + ((int64_t)(t + 1) * R + r) * A;
    const float* qt = Qtg + ((int64_t)(t + 1) * R + r) * A;
    const float* qs_row = d.double_q ? qn : qt;
    const int32_t* av = rp.avail + ((slot + 1) * n + lane) * (int64_t)A;
    const uint64_t abits = rp.avail_bits ? rp.avail_bits[(slot + 1) * n + lane] : 0;
#pragma unroll
    for (int u = 0; u < MA; ++u) {
      const int a = min(u, A - 1);
      qsel[u] = qs_row[a];
      qtr[u] = qt[a];
      avr[u] = rp.avail_bits ? (int32_t)((abits >> a) & 1u) : av[a];
    }
  }
  const bool e_lane = qmix && valid && lane < E;
  float won[MN], wtg[MN], xon[3], xtg[3], v2w0 = 0.0f, v2w1 = 0.0f;
  if (e_lane) {
#pragma unroll
    for (int ag = 0; ag < MN; ++ag) {
      won[ag] = hon[min(ag, n - 1) * E + lane];
      wtg[ag] = htg[min(ag, n - 1) * E + lane];
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {   // hyper_w_final, hyper_b_1, V.0 outputs
      xon[k] = hon[n * E + k * E + lane];
      xtg[k] = htg[n * E + k * E + lane];
    }
    v2w0 = P0[L.o[MQ_P_V2_W] + lane];
    v2w1 = P1[L.o[MQ_P_V2_W] + lane];
  }
  float mask = 0.0f, rew = 0.0f, term = 0.0f;
  if (valid) {
    mask = (float)rp.filled[slot];
    if (t > 0) mask *= 1.0f - (float)rp.term[slot - 1];   // q_learner.py:42-43
    rew = rp.reward[slot];
    term = (float)rp.term[slot];
  }
  const float v2b0 = qmix ? P0[L.o[MQ_P_V2_B]] : 0.0f, v2b1 = qmix ? P1[L.o[MQ_P_V2_B]] : 0.0f;
  // ---- chosen value and double-Q selection (q_learner.py:55, 68-78), first index on ties
  float chosen = 0.0f, tmax = 0.0f;
  if (agent_lane) {
    chosen = Qon[((int64_t)t * R + r) * A + at];
    float best = 0.0f;
    int cur = 0;
#pragma unroll
    for (int u = 0; u < MA; ++u) {
      const float v = avr[u] ? qsel[u] : kNegMask;
      if (u < A && (u == 0 || v > best)) { best = v; cur = u; }
    }
    if (d.double_q) {
      float qc = 0.0f;
      int ac = 0;
#pragma unroll
      for (int u = 0; u < MA; ++u)
        if (u == cur) { qc = qtr[u]; ac = avr[u]; }
      tmax = ac ? qc : kNegMask;
    } else {
      tmax = best;
    }
    if (curmax_out) curmax_out[(int64_t)t * R + r] = cur;
  }
  sc.chs[lane] = chosen;
  sc.tms[lane] = tmax;
  if (e_lane) {
#pragma unroll
    for (int ag = 0; ag < MN; ++ag) sc.w1s[ag][lane] = fabsf(won[ag]);
  }
  __syncthreads();
  const float gamma = d.gamma;
  if (qmix) {
    // QMIX forward of both nets (qmix_fwd_lane's arithmetic, operands from registers)
    float y = 0.0f, yt = 0.0f, pre = 0.0f, hid = 0.0f;
    {
      float prod = 0.0f, vt = 0.0f, prod_t = 0.0f, vt_t = 0.0f;
      if (e_lane) {
        float acc = 0.0f, acc_t = 0.0f;
#pragma unroll
        for (int ag = 0; ag < MN; ++ag) {
          if (ag < n) {
            acc = fmaf(sc.chs[ag], fabsf(won[ag]), acc);
            acc_t = fmaf(sc.tms[ag], fabsf(wtg[ag]), acc_t);
          }
        }
        pre = acc + xon[1];
        hid = eluf(pre);
        prod = hid * fabsf(xon[0]);
        vt = fmaxf(xon[2], 0.0f) * v2w0;
        const float pre_t = acc_t + xtg[1];
        prod_t = eluf(pre_t) * fabsf(xtg[0]);
        vt_t = fmaxf(xtg[2], 0.0f) * v2w1;
      }
      y = wave_sum(prod) + (wave_sum(vt) + v2b0);
      yt = wave_sum(prod_t) + (wave_sum(vt_t) + v2b1);
    }
    if (!valid) y = yt = 0.0f;
    const float target = rew + gamma * (1.0f - term) * yt;   // q_learner.py:86
    const float td = y - target;
    const float mtd = td * mask;
    l2 = td_loss(mtd, d.huber); msk = mask; abs_ = fabsf(mtd); qs = y * mask; tg = target * mask;
    const float dy = td_dy(mtd, mask, d.huber);
    float dpre = 0.0f;
    if (e_lane) {
      const float wf = fabsf(xon[0]);
      const float dhid = dy * wf;
      float* dh = w.dHYP + (int64_t)m * NH;
      dh[n * E + lane] = dy * hid * sgnf(xon[0]);                             // hyper_w_final
      dpre = dhid * (pre > 0.0f ? 1.0f : expf(pre));                          // elu'
      dh[n * E + E + lane] = dpre;                                            // hyper_b_1
      dh[n * E + 2 * E + lane] = dy * v2w0 * (xon[2] > 0.0f ? 1.0f : 0.0f);   // V.0 (through relu)
      dv2 = dy * fmaxf(xon[2], 0.0f);                                         // V.2 weight
#pragma unroll
      for (int ag = 0; ag < MN; ++ag)                                         // hyper_w_1 (through |.|)
        if (ag < n) dh[ag * E + lane] = (sc.chs[ag] * dpre) * sgnf(won[ag]);
    }
    dv2b = dy;
    sc.dps[lane] = dpre;
    __syncthreads();
    if (agent_lane) {
      float acc = 0.0f;
      for (int e = 0; e < E; ++e) acc = fmaf(sc.w1s[lane][e], sc.dps[e], acc);
      w.dch[(int64_t)t * R + b * n + lane] = acc;
    }
  } else {
    float y, yt;
    if (d.mixer == MQ_MIXER_VDN) {
      y = wave_sum(lane < n ? chosen : 0.0f);
      yt = wave_sum(lane < n ? tmax : 0.0f);
    } else {
      y = chosen;
      yt = tmax;
    }
    const float target = rew + gamma * (1.0f - term) * yt;
    const float td = y - target;
    const float mtd = td * mask;
    const float dy = td_dy(mtd, mask, d.huber);
    if (d.mixer == MQ_MIXER_VDN) {
      l2 = td_loss(mtd, d.huber); msk = mask; abs_ = fabsf(mtd); qs = y * mask; tg = target * mask;
    } else {
      const bool on = lane < n;
      l2 = wave_sum(on ? td_loss(mtd, d.huber) : 0.0f);
      msk = wave_sum(on ? mask : 0.0f);
      abs_ = wave_sum(on ? fabsf(mtd) : 0.0f);
      qs = wave_sum(on ? y * mask : 0.0f);
      tg = wave_sum(on ? target * mask : 0.0f);
    }
    if (agent_lane) w.dch[(int64_t)t * R + b * n + lane] = dy;
    __syncthreads();
  }
  if (!valid) { l2 = msk = abs_ = qs = tg = 0.0f; dv2 = dv2b = 0.0f; }
  if (lane == 0) {
    red_slot[0] = l2; red_slot[1] = msk; red_slot[2] = abs_; red_slot[3] = qs; red_slot[4] = tg;
    v2_slot[64] = dv2b;
  }
  v2_slot[lane] = dv2;
}

template <int MA, int MN>
__global__ __launch_bounds__(256) void mix_fast_kernel(Dims d, Rep rp, const float* __restrict__ P0,
                                                       const float* __restrict__ P1, Lay L, Work w,
                                                       int32_t* curmax_out) {
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int m = blockIdx.x * 4 + wv;
  const int E = d.E, NH = d.NH;
  const bool qmix = d.mixer == MQ_MIXER_QMIX;
  __shared__ MixScratch<MN> sc[4];
  __shared__ float red[4][8];
  __shared__ float v2red[4][65];
  const float* hon = w.HYP + (int64_t)m * NH;
  const float* htg = w.HYP + ((int64_t)d.M + m) * NH;
  mix_fast_row<MA, MN>(d, rp, P0, P1, L, w, curmax_out, m, lane, hon, htg, sc[wv], red[wv], v2red[wv]);
  __syncthreads();
  if (threadIdx.x < 8) {
    const int c = threadIdx.x;
    float* out = w.loss_part + (int64_t)blockIdx.x * 8;
    out[c] = c < 5 ? ((red[0][c] + red[1][c]) + (red[2][c] + red[3][c])) : 0.0f;
  }
  if (qmix && threadIdx.x <= E) {
    const int e = threadIdx.x == E ? 64 : threadIdx.x;
    w.slab_v2[(int64_t)blockIdx.x * (E + 1) + threadIdx.x] =
        (v2red[0][e] + v2red[1][e]) + (v2red[2][e] + v2red[3][e]);
  }
}

}  // namespace mq
