// Host side of the COMA learner step (include/mc_coma.h), included at the end of mq_learner.hip so it shares the
// QMIX learner's error handling, replay plumbing and agent kernels. The agent (RNNAgent) forward / BPTT reuses an
// internal mq_handle (no mixer) for its workspace; the critic has its own.
#include "../../include/mc_coma.h"
#include "coma_chain.hpp"

struct mc_handle {
  mc_config cfg;
  mq_handle* ah = nullptr;   // agent workspace + kernels
  int I, Kc, Kp, Ap;
  int64_t aoff[MQ_P_COUNT + 1];
  int64_t coff[MC_P_COUNT + 1];
  int64_t Pa, Pc;
  float *agent = nullptr, *agrad = nullptr, *asq = nullptr, *critic = nullptr, *tcritic = nullptr,
        *cgrad = nullptr, *csq = nullptr, *stats = nullptr;
  void* ws = nullptr;
  // critic workspace
  float *X, *H1t, *H2t, *Qt, *tgt, *msum, *H1p, *H1c, *H2c, *dH1c, *dH2c, *dqc, *qvals, *cpart, *cnorm, *crec;
  float *Pshadow, *SQshadow;
  float* Pbak;   // [2][Pc] critic params / square_avg before the chain: restored if a hand-off times out
  int* actc;
  int* cstate;
  // actor workspace
  float *dL, *dHo, *pi, *ppart, *slab_fc2, *red_tmp, *norm_part;
  int last_T = 0, last_R = 0, last_Rc = 0;
  bool timing = false;
  // persistent critic chain (coma_chain.hpp): off with MQ_PLAN coma_chain=0, or where cc_ok rejects the shape
  bool chain_env = true;
  int num_cu = 0;
  bool chain_attr = false;
  int last_path = -1;
  unsigned long long* chain_trace = nullptr;   // MQ_DIAG coma_trace: phase timestamps printed after each train
  // data parallel (mc_set_data_parallel)
  mc_allreduce_fn dp_fn = nullptr;
  void* dp_ctx = nullptr;
  int dp_rank = 0;
  float* dp_scratch = nullptr;
  int64_t dp_scratch_n = 0;
  std::vector<float> dp_msum;
  ncclComm_t comm = nullptr;   // mc_comm_attach: native RCCL exchange steps
  float* comm_scratch = nullptr;
  bool comm_owned = false;   // mc_comm_attach created it; mc_comm_use borrows the caller's
  // mc_set_actor_shard: replicated-critic data parallelism (every rank runs the critic on the whole batch, the actor
  // on episodes [shard_lo, shard_hi) with one all-reduce of the agent gradient); off while shard_hi <= shard_lo
  int shard_lo = 0, shard_hi = 0;
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
};

namespace {

// One exchange step of the data-parallel mode: sum `n` floats at `buf` (caller-owned) over the ranks.
int mc_allreduce(mc_handle* h, float* buf, int64_t n, hipStream_t s) {
  if (h->dp_fn(buf, n, (void*)s, h->dp_ctx) != 0) return set_err(MQ_ERR_STATE, "data-parallel all-reduce callback failed");
  return MQ_OK;
}

// Library-owned arrays travel through the caller's scratch buffer.
int mc_allreduce_ws(mc_handle* h, float* ws_buf, int64_t n, hipStream_t s) {
  MQ_HIP(hipMemcpyAsync(h->dp_scratch, ws_buf, n * sizeof(float), hipMemcpyDeviceToDevice, s));
  int rc = mc_allreduce(h, h->dp_scratch, n, s);
  if (rc) return rc;
  MQ_HIP(hipMemcpyAsync(ws_buf, h->dp_scratch, n * sizeof(float), hipMemcpyDeviceToDevice, s));
  return MQ_OK;
}

// Episodes [lo, hi) of a batch as a batch of their own: the id slice, or for a dense batch (no ids) every field
// pointer advanced by lo episodes.
mq_replay shard_replay(const mc_config& c, const mq_replay& b, int lo, int hi) {
  mq_replay s = b;
  s.batch_size = hi - lo;
  if (b.ep_ids_host) s.ep_ids_host = b.ep_ids_host + lo;
  if (b.ep_ids) s.ep_ids = b.ep_ids + lo;
  if (!b.ep_ids && !(b.ep_ids_host && b.batch_size <= MQ_INLINE_IDS)) {
    const int64_t e = (int64_t)lo * b.t_stride, n = c.n_agents;
    if (s.obs) s.obs += e * n * c.obs_dim;
    if (s.state) s.state += e * c.state_dim;
    if (s.actions) s.actions += e * n;
    if (s.avail_actions) s.avail_actions += e * n * c.n_actions;
    if (s.reward) s.reward += e;
    if (s.terminated) s.terminated += e;
    if (s.filled) s.filled += e;
    s.n_episodes = b.n_episodes - lo;
  }
  return s;
}

int mc_agent_config(const mc_config& c, mq_config* a) {
  std::memset(a, 0, sizeof(*a));
  a->n_agents = c.n_agents; a->n_actions = c.n_actions; a->obs_dim = c.obs_dim; a->state_dim = c.state_dim;
  a->rnn_hidden_dim = c.rnn_hidden_dim; a->mixing_embed_dim = 0; a->mixer = MQ_MIXER_NONE; a->double_q = 0;
  a->obs_last_action = c.obs_last_action; a->obs_agent_id = c.obs_agent_id; a->gamma = c.gamma; a->lr = c.lr;
  a->optim_alpha = c.optim_alpha; a->optim_eps = c.optim_eps; a->grad_norm_clip = c.grad_norm_clip;
  a->max_batch = c.max_batch; a->max_seq = c.max_seq;
  return MQ_OK;
}

}  // namespace

extern "C" {

int64_t mc_critic_forward_workspace(const mc_config* cfg, int32_t batch_size, int32_t t_count) {
  if (!cfg || batch_size < 1 || t_count < 1) return -1;
  const int n = cfg->n_agents, A = cfg->n_actions;
  const int64_t Kp = ((int64_t)cfg->state_dim + cfg->obs_dim + 2 * n * A + n + 3) & ~int64_t(3);
  const int64_t M = (int64_t)t_count * batch_size * n;
  return align_up(M * Kp) + 2 * align_up(M * CH) + align_up(M * A);
}

int mc_critic_forward(const float* critic, const mc_config* cfg, const mq_replay* batch, int32_t t, float* q_out,
                      float* workspace, void* stream) {
  if (!critic || !cfg || !batch || !q_out || !workspace) return set_err(MQ_ERR_ARG, "mc_critic_forward: NULL pointer");
  if (!batch->obs || !batch->state || !batch->actions || !batch->filled)
    return set_err(MQ_ERR_ARG, "mc_critic_forward: batch needs obs, state, actions and filled");
  if (batch->batch_size < 1 || batch->t_len < 1 || batch->t_len > batch->t_stride)
    return set_err(MQ_ERR_ARG, "mc_critic_forward: bad batch dimensions");
  if (t >= batch->t_len) return set_err(MQ_ERR_ARG, "mc_critic_forward: t outside the batch");
  if (batch->ep_ids_host && batch->batch_size > MQ_INLINE_IDS && !batch->ep_ids)
    return set_err(MQ_ERR_ARG, "mc_critic_forward: more than MQ_INLINE_IDS episodes need device ids");
  hipStream_t s = (hipStream_t)stream;
  const int n = cfg->n_agents, A = cfg->n_actions, B = batch->batch_size, R = B * n;
  const int Tq = t < 0 ? batch->t_len : 1, t0 = t < 0 ? 0 : t;
  CDims cd{};
  cd.n = n; cd.A = A; cd.O = cfg->obs_dim; cd.S = cfg->state_dim;
  cd.Kc = cfg->state_dim + cfg->obs_dim + 2 * n * A + n;
  cd.Kp = (cd.Kc + 3) & ~3;
  cd.R = R; cd.B = B; cd.Tp = batch->t_len; cd.T = batch->t_len - 1; cd.t_stride = batch->t_stride;
  cd.dR = make_fastdiv((uint32_t)R);
  cd.dN = make_fastdiv((uint32_t)n);
  const Rep rp = make_rep(batch);
  const int64_t M = (int64_t)Tq * R;
  float* X = workspace;
  float* H1 = X + align_up(M * cd.Kp);
  float* H2 = H1 + align_up(M * CH);
  float* Q = H2 + align_up(M * CH);
  // offsets of fc1.weight .. fc3.bias (MC_P_* order)
  const int64_t o_w1 = 0, o_b1 = (int64_t)CH * cd.Kc, o_w2 = o_b1 + CH, o_b2 = o_w2 + (int64_t)CH * CH,
                o_w3 = o_b2 + CH, o_b3 = o_w3 + (int64_t)A * CH;
  hipLaunchKernelGGL(coma_xin_kernel, dim3((unsigned)M), dim3(256), 0, s, cd, rp, X, t0);
  MQ_HIP(hipGetLastError());
  const CLinProbT<64> l1 = CLinProbT<64>{X, cd.Kp, critic + o_w1, critic + o_b1, H1, M, CH, cd.Kc, 1}.with_vec();
  MQ_HIP(launch_gemm(l1, (int)M, CH, 1, s));
  const CLinProbT<64> l2 = CLinProbT<64>{H1, CH, critic + o_w2, critic + o_b2, H2, M, CH, CH, 1}.with_vec();
  MQ_HIP(launch_gemm(l2, (int)M, CH, 1, s));
  const CLinProbT<64> l3 = CLinProbT<64>{H2, CH, critic + o_w3, critic + o_b3, Q, M, A, CH, 0}.with_vec();
  MQ_HIP(launch_gemm(l3, (int)M, A, 1, s));
  const int64_t tot = M * A;
  hipLaunchKernelGGL(coma_q_layout_kernel, dim3((unsigned)std::min<int64_t>((tot + 255) / 256, 4096)), dim3(256), 0, s,
                     (const float*)Q, q_out, Tq, B, n, A);
  MQ_HIP(hipGetLastError());
  return MQ_OK;
}

int mc_create(const mc_config* cfg, mc_handle** out) {
  if (!cfg || !out) return set_err(MQ_ERR_ARG, "NULL argument");
  const mc_config& c = *cfg;
  if (c.n_actions < 1 || c.n_actions > 64) return set_err(MQ_ERR_ARG, "n_actions must be in [1, 64]");
  if (c.max_batch * c.n_agents > MQ_INLINE_IDS * 64) return set_err(MQ_ERR_ARG, "max_batch * n_agents too large");
  mq_config ac;
  mc_agent_config(c, &ac);
  mq_handle* ah = nullptr;
  int rc = mq_create(&ac, &ah);
  if (rc) return rc;
  mc_handle* h = new mc_handle();
  h->cfg = c;
  h->ah = ah;
  h->I = ah->I;
  for (int i = 0; i <= MQ_P_COUNT; ++i) h->aoff[i] = ah->off[i];
  h->Pa = ah->P;
  const int n = c.n_agents, A = c.n_actions;
  h->Kc = c.state_dim + c.obs_dim + 2 * n * A + n;   // coma.py:61-70
  h->Kp = (h->Kc + 3) & ~3;
  h->Ap = (A + 3) & ~3;
  const int64_t sz[MC_P_COUNT] = {(int64_t)CH * h->Kc, CH, (int64_t)CH * CH, CH, (int64_t)A * CH, A};
  int64_t o = 0;
  for (int i = 0; i < MC_P_COUNT; ++i) { h->coff[i] = o; o += sz[i]; }
  h->coff[MC_P_COUNT] = o;
  h->Pc = o;

  const int64_t Tp = c.max_seq, R = (int64_t)c.max_batch * n, T = Tp - 1;
  const int64_t RTa = T * R;   // actor rows (T steps)
  const int64_t nwg = 8 * ((h->Kc + 1 + 63) / 64) + 24 + 3 * ((A + 15) / 16) + 1, nhead = (R + 15) / 16;
  const int64_t ns2 = kNsplitMax;
  const int64_t red_tmp = kRedZ * ((int64_t)mq::H * h->I + mq::H) + kRedZ * h->ah->len_rnn +
                          kRedZ * (A * mq::H + A) + kRedZ * 8;
  int64_t sizes[] = {
      Tp * R * h->Kp,              // X
      Tp * R * CH, Tp * R * CH,    // H1t, H2t
      Tp * R * A,                  // Qt
      T * R, T,                    // tgt, msum
      (int64_t)std::max(l1_slices(h->Kp), cc_nk(h->Kc)) * R * CH,   // H1p (three-launch l1 or chain phase A)
      R * CH, R * CH, R * CH, R * CH,   // H1c H2c dH1c dH2c
      R, R,                        // dqc, actc
      T * R * A,                   // qvals
      nhead * 8, std::max<int64_t>(nwg, 1024), T * 8,   // cpart, cnorm (chain: 256 8-B granules + flags), crec
      h->Pc, h->Pc,                // shadow params / square_avg (the chain's gradient exchange: Pshadow)
      8,                           // cstate (+ the critic chain's sync words)
      RTa * h->Ap, RTa * mq::H, RTa * A,   // dL, dHo, pi
      ((RTa + 3) / 4) * 8,         // ppart
      ns2 * (A * mq::H + A),       // slab_fc2
      red_tmp,                     // red_tmp
      4096,                        // norm_part
      2 * h->Pc,                   // Pbak
  };
  const int NS = (int)(sizeof(sizes) / sizeof(sizes[0]));
  int64_t total = 0, offs[32];
  for (int i = 0; i < NS; ++i) { offs[i] = total; total += align_up(std::max<int64_t>(sizes[i], 1)); }
  hipError_t e = hipMalloc(&h->ws, total * sizeof(float));
  if (e != hipSuccess) {
    mq_destroy(ah);
    delete h;
    return set_err(MQ_ERR_HIP, std::string("COMA workspace hipMalloc: ") + hipGetErrorString(e));
  }
  float* b = (float*)h->ws;
  int k = 0;
  h->X = b + offs[k++]; h->H1t = b + offs[k++]; h->H2t = b + offs[k++]; h->Qt = b + offs[k++];
  h->tgt = b + offs[k++]; h->msum = b + offs[k++]; h->H1p = b + offs[k++];
  h->H1c = b + offs[k++]; h->H2c = b + offs[k++]; h->dH1c = b + offs[k++]; h->dH2c = b + offs[k++];
  h->dqc = b + offs[k++]; h->actc = (int*)(b + offs[k++]);
  h->qvals = b + offs[k++]; h->cpart = b + offs[k++]; h->cnorm = b + offs[k++]; h->crec = b + offs[k++];
  h->Pshadow = b + offs[k++]; h->SQshadow = b + offs[k++];
  h->cstate = (int*)(b + offs[k++]);
  h->dL = b + offs[k++]; h->dHo = b + offs[k++]; h->pi = b + offs[k++]; h->ppart = b + offs[k++];
  h->slab_fc2 = b + offs[k++]; h->red_tmp = b + offs[k++]; h->norm_part = b + offs[k++];
  h->Pbak = b + offs[k++];
  h->chain_env = plan_int("coma_chain", 1) != 0;   // MQ_PLAN coma_chain=0: three launches per critic step
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&h->num_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    h->num_cu = 0;
  *out = h;
  return MQ_OK;
}

int mc_destroy(mc_handle* h) {
  if (!h) return MQ_OK;
  if (h->ws) (void)hipFree(h->ws);
  if (h->chain_trace) (void)hipFree(h->chain_trace);
  if (h->comm && h->comm_owned) (void)ncclCommDestroy(h->comm);
  if (h->comm_scratch) (void)hipFree(h->comm_scratch);
  for (auto& e : h->ev)
    if (e) (void)hipEventDestroy(e);
  mq_destroy(h->ah);
  delete h;
  return MQ_OK;
}

int mc_param_offsets(const mc_handle* h, int64_t* agent_offsets, int64_t* critic_offsets) {
  if (!h) return set_err(MQ_ERR_ARG, "NULL handle");
  if (agent_offsets)
    for (int i = 0; i <= MQ_P_COUNT; ++i) agent_offsets[i] = h->aoff[i];
  if (critic_offsets)
    for (int i = 0; i <= MC_P_COUNT; ++i) critic_offsets[i] = h->coff[i];
  return MQ_OK;
}

int mc_bind(mc_handle* h, float* agent, float* agent_grad, float* agent_sq, float* critic, float* target_critic,
            float* critic_grad, float* critic_sq, float* stats) {
  if (!h || !agent || !agent_grad || !agent_sq || !critic || !target_critic || !critic_grad || !critic_sq || !stats)
    return set_err(MQ_ERR_ARG, "mc_bind: NULL pointer");
  h->agent = agent; h->agrad = agent_grad; h->asq = agent_sq; h->critic = critic; h->tcritic = target_critic;
  h->cgrad = critic_grad; h->csq = critic_sq; h->stats = stats;
  // the agent handle: online = target = the agent params (the actor has no target net); stats land at stats + 8
  return mq_bind(h->ah, agent, agent, agent_grad, agent_sq, stats + 8, nullptr);
}

int mc_train_step(mc_handle* h, const mq_replay* batch, float epsilon, void* stream) {
  if (!h || !h->agent) return set_err(MQ_ERR_STATE, "mc_train_step before mc_bind");
  mq_handle* ah = h->ah;
  int rc = check_batch(ah, batch);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  const mc_config& c = h->cfg;
  const int n = c.n_agents, A = c.n_actions;
  const int Tp = batch->t_len, T = Tp - 1, R = batch->batch_size * n;
  const Rep rp = make_rep(batch);

  CDims cd;
  cd.n = n; cd.A = A; cd.O = c.obs_dim; cd.S = c.state_dim; cd.Kc = h->Kc; cd.Kp = h->Kp; cd.R = R;
  cd.B = batch->batch_size; cd.Tp = Tp; cd.T = T; cd.t_stride = batch->t_stride;
  cd.lg = (float)((double)c.td_lambda * (double)c.gamma);
  cd.og = (float)((1.0 - (double)c.td_lambda) * (double)c.gamma);
  cd.dR = make_fastdiv((uint32_t)R);
  cd.dN = make_fastdiv((uint32_t)n);

  const bool repl = h->shard_hi > h->shard_lo;
  if (repl && (h->shard_lo < 0 || h->shard_hi > batch->batch_size))
    return set_err(MQ_ERR_ARG, "actor shard [" + std::to_string(h->shard_lo) + ", " + std::to_string(h->shard_hi) +
                                   ") outside the batch of " + std::to_string(batch->batch_size) + " episodes");
  if (repl && !h->dp_fn)
    return set_err(MQ_ERR_STATE, "a replicated critic needs an all-reduce for the actor (mc_set_data_parallel / "
                                 "mc_comm_attach)");
  if (h->timing) MQ_HIP(hipEventRecord(h->ev[0], s));
  MQ_HIP(hipMemsetAsync(h->crec, 0, (size_t)T * 8 * sizeof(float), s));
  MQ_HIP(hipMemsetAsync(h->cstate, 0, 8 * sizeof(int), s));
  hipLaunchKernelGGL(coma_mask_kernel, dim3((T + 255) / 256), dim3(256), 0, s, cd, rp, h->msum);
  MQ_HIP(hipGetLastError());
  const bool dp = h->dp_fn != nullptr && !repl;   // exchange mode: the critic steps are summed over the ranks
  if (dp) {   // global per-step mask sums: every rank normalises by them and skips the same steps
    if (h->dp_scratch_n < 8LL * T) return set_err(MQ_ERR_ARG, "data-parallel scratch smaller than 8 * t_len");
    rc = mc_allreduce_ws(h, h->msum, T, s);
    if (rc) return rc;
  }
  hipLaunchKernelGGL(coma_xin_kernel, dim3(Tp * R), dim3(256), 0, s, cd, rp, h->X);
  MQ_HIP(hipGetLastError());
  // target critic over every stored step (coma_learner.py:102), then TD(lambda) (rl_utils.py:4-14)
  {
    const int64_t M = (int64_t)Tp * R;
    const float* tc = h->tcritic;
    const CLinProbT<64> l1 =
        CLinProbT<64>{h->X, h->Kp, tc + h->coff[MC_P_FC1_W], tc + h->coff[MC_P_FC1_B], h->H1t, M, CH, h->Kc, 1}
            .with_vec();
    MQ_HIP(launch_gemm(l1, (int)M, CH, 1, s));
    const CLinProbT<64> l2 =
        CLinProbT<64>{h->H1t, CH, tc + h->coff[MC_P_FC2_W], tc + h->coff[MC_P_FC2_B], h->H2t, M, CH, CH, 1}.with_vec();
    MQ_HIP(launch_gemm(l2, (int)M, CH, 1, s));
    const CLinProbT<64> l3 =
        CLinProbT<64>{h->H2t, CH, tc + h->coff[MC_P_FC3_W], tc + h->coff[MC_P_FC3_B], h->Qt, M, A, CH, 0}.with_vec();
    MQ_HIP(launch_gemm(l3, (int)M, A, 1, s));
  }
  const size_t lds_td = (size_t)Tp * (n + 3) * sizeof(float);
  if (lds_td > 160 * 1024 || n > 256) return set_err(MQ_ERR_ARG, "episode too long for the LDS TD(lambda) pass");
  hipLaunchKernelGGL(coma_td_kernel, dim3(batch->batch_size), dim3(256), lds_td, s, cd, rp, h->Qt, h->tgt);
  MQ_HIP(hipGetLastError());

  // the critic's T sequential steps (coma_learner.py:118-139)
  CritArgs ca;
  ca.d = cd; ca.rp = rp;
  ca.P[0] = h->critic; ca.P[1] = h->Pshadow; ca.SQ[0] = h->csq; ca.SQ[1] = h->SQshadow; ca.G = h->cgrad;
  ca.o_w1 = h->coff[MC_P_FC1_W]; ca.o_b1 = h->coff[MC_P_FC1_B]; ca.o_w2 = h->coff[MC_P_FC2_W];
  ca.o_b2 = h->coff[MC_P_FC2_B]; ca.o_w3 = h->coff[MC_P_FC3_W]; ca.o_b3 = h->coff[MC_P_FC3_B]; ca.Pc = h->Pc;
  ca.X = h->X; ca.tgt = h->tgt; ca.msum = h->msum; ca.H1p = h->H1p; ca.KS = l1_slices(h->Kp); ca.H1c = h->H1c; ca.H2c = h->H2c; ca.dH1c = h->dH1c;
  ca.dH2c = h->dH2c; ca.dqc = h->dqc; ca.actc = h->actc; ca.qvals = h->qvals; ca.cpart = h->cpart;
  ca.cnorm = h->cnorm; ca.crec = h->crec; ca.cstate = h->cstate;
  ca.nhead = (R + 15) / 16;
  ca.nwgrad = wgrad_blocks(cd);
  ca.hp = OptHP{c.critic_lr, c.optim_alpha, c.optim_eps, c.grad_norm_clip, 1};
  const int A16 = (A + 15) / 16 * 16;
  const size_t lds_l1 = (size_t)(16 + kL1Rows) * (KW + 1) * sizeof(float);
  const size_t lds_head = ((size_t)(CH + A16 + 48) * (CH + 1) + 16 * (A16 + 1) + CH + A16) * sizeof(float);
  if (lds_l1 > 160 * 1024 || lds_head > 160 * 1024)
    return set_err(MQ_ERR_ARG, "critic input width or n_actions too large for the LDS-staged critic step");
  MQ_HIP(hipMemsetAsync(h->qvals, 0, (size_t)T * R * A * sizeof(float), s));   // skipped steps keep q_vals = 0
  if (dp) {   // the host needs the live steps to place the per-step exchanges (one synchronisation per train)
    h->dp_msum.resize(T);
    MQ_HIP(hipMemcpyAsync(h->dp_msum.data(), h->msum, (size_t)T * sizeof(float), hipMemcpyDeviceToHost, s));
    MQ_HIP(hipStreamSynchronize(s));
  }
  // ---- the actor's agent unroll over t < T (coma_learner.py:52-57), online net only. It reads nothing the critic
  // writes, so beside the persistent chain it runs on the side stream in the CUs the chain leaves idle.
  // replicated critic: the actor trains this rank's episodes only (the critic above saw the whole batch)
  mq_replay av = repl ? shard_replay(c, *batch, h->shard_lo, h->shard_hi) : *batch;
  av.t_len = T;
  const Rep rpa = repl ? make_rep(&av) : rp;
  const int qv_r0 = repl ? h->shard_lo * n : 0;   // this rank's first row in the critic's [T][B n][A] Q values
  Dims d = make_dims(ah, &av);
  const Lay L = make_lay(ah);
  Work w = ah->w;
  w.dHo = h->dHo;
  const int64_t RT = (int64_t)T * d.R;   // the actor's rows (its shard under a replicated critic)
  const float* Pa = h->agent;
  auto agent_forward = [&](hipStream_t st) -> int {
    const int rw_fwd = pick_rw(d.R, 512);
    if (rw_fwd == 1 && fused_fwd_ok(d.I, d.O, d.A, d.n, RT)) {
      launch_fwd_fused(dim3(d.R, 1), st, d, rpa, Pa, Pa, L, w);
      MQ_HIP(hipGetLastError());
    } else {
      Fc1Prob p1{d, rpa, Pa, Pa, ah->off[MQ_P_FC1_W], ah->off[MQ_P_FC1_B], w.X1, w.XIN, RT};
      MQ_HIP(launch_gemm(p1, (int)RT, 2 * mq::H, 1, st));
      GiProb p2{w.X1, Pa, Pa, ah->off[MQ_P_RNN_W_IH], ah->off[MQ_P_RNN_B_IH], w.GI, RT};
      MQ_HIP(launch_gemm(p2, (int)RT, mq::G3, 1, st));
      const dim3 grid((d.R + rw_fwd - 1) / rw_fwd, 1);
      if (rw_fwd == 1) hipLaunchKernelGGL((gru_fwd_kernel<1, 0>), grid, dim3(256), 0, st, d, Pa, Pa, L, w);
      else if (rw_fwd == 2) hipLaunchKernelGGL((gru_fwd_kernel<2, 0>), grid, dim3(256), 0, st, d, Pa, Pa, L, w);
      else if (rw_fwd == 4) hipLaunchKernelGGL((gru_fwd_kernel<4, 0>), grid, dim3(256), 0, st, d, Pa, Pa, L, w);
      else hipLaunchKernelGGL((gru_fwd_kernel<8, 0>), grid, dim3(256), 0, st, d, Pa, Pa, L, w);
      MQ_HIP(hipGetLastError());
      Fc2Prob p3{w.Hs, Pa, Pa, ah->off[MQ_P_FC2_W], ah->off[MQ_P_FC2_B], w.Q, RT, d.A};
      MQ_HIP(launch_gemm(p3, (int)RT, d.A, 1, st));
    }
    return MQ_OK;
  };
  // MQ_PLAN coma_overlap=0: the actor's agent unroll stays on the caller's stream
  const bool try_overlap = !dp && !h->timing && plan_int("coma_overlap", 1) != 0 && h->chain_env &&
                           cc_ok(R, A, h->Kc, h->num_cu);
  if (try_overlap) {
    MQ_HIP(ensure_side(ah));
    MQ_HIP(hipEventRecord(ah->ev_fork, s));   // before the chain: the side stream does not wait for it
  }
  bool actor_side = false;
  if (h->timing) MQ_HIP(hipEventRecord(h->ev[1], s));
  bool chained = false;
  if (!dp && h->chain_env && cc_ok(R, A, h->Kc, h->num_cu)) {   // every critic step in one persistent launch
    CChain cc;
    cc.d = cd; cc.rp = rp; cc.P = h->critic; cc.SQ = h->csq; cc.G = h->cgrad;
    cc.o_w1 = ca.o_w1; cc.o_b1 = ca.o_b1; cc.o_w2 = ca.o_w2; cc.o_b2 = ca.o_b2; cc.o_w3 = ca.o_w3; cc.o_b3 = ca.o_b3;
    cc.Pc = h->Pc; cc.X = h->X; cc.tgt = h->tgt; cc.msum = h->msum; cc.H1p = h->H1p;
    cc.H1x = h->H1c; cc.H2x = h->H2c; cc.dH2x = h->dH2c; cc.dH1x = h->dH1c; cc.dqx = h->dqc; cc.actx = h->actc;
    cc.part = h->cpart; cc.normg = (unsigned long long*)h->cnorm; cc.GW = h->Pshadow; cc.qvals = h->qvals;
    cc.crec = h->crec; cc.cstate = h->cstate; cc.sync = (unsigned*)(h->cstate + 2);   // zeroed above
    cc.NK = cc_nk(h->Kc); cc.NG = 8 * cc.NK; cc.NHEAD = (R + 15) / 16;
    cc.hp = ca.hp;
    if (env_item("MQ_DIAG", "coma_trace") && !h->chain_trace)
      MQ_HIP(hipMalloc(&h->chain_trace, 16 * 8 * sizeof(unsigned long long)));
    cc.trace = h->chain_trace;
    cc.fault_wg = env_int("MQ_DIAG", "coma_fault", -1);   // test hook: a workgroup that stops flagging
    // cnorm: [0, 2 G) the norm granules, [512, 512 + G) flagA, [768, 768 + NHEAD) flagB; no stale step tags
    cc.flagA = (unsigned*)(h->cnorm + 512);
    cc.flagB = (unsigned*)(h->cnorm + 768);
    MQ_HIP(hipMemsetAsync(h->cnorm, 0, 1024 * sizeof(float), s));
    const size_t lds = cc_lds_bytes(A);
    MQ_LDS(coma_chain_kernel, lds);
    if (!h->chain_attr) {
      MQ_HIP(hipFuncSetAttribute((const void*)coma_chain_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      h->chain_attr = true;
    }
    // the chain updates the critic in place: keep the pre-train version, restored below if a hand-off times out
    MQ_HIP(hipMemcpyAsync(h->Pbak, h->critic, (size_t)h->Pc * sizeof(float), hipMemcpyDeviceToDevice, s));
    MQ_HIP(hipMemcpyAsync(h->Pbak + h->Pc, h->csq, (size_t)h->Pc * sizeof(float), hipMemcpyDeviceToDevice, s));
    // A plain launch: the grid (cc_ok: at most one 512-thread workgroup per CU, NG <= the CU count) is resident
    // by its size alone, which is all a cooperative launch would add a check for (MI355X_MICROARCH.md "Residency
    // and cooperative launch": plain and cooperative launches give the same residency). Nothing else on the device
    // waits on the chain, so a workgroup that starts late only delays it; every spin is bounded. The cooperative
    // launch also cost 15-19 us of host time per train and, under rocprofv3, its dedicated HIP queue crashed the
    // runtime's exit-time teardown (round 4: profiles/r04a_cfg5_rocprof_exit_crash.txt)
    hipLaunchKernelGGL(coma_chain_kernel, dim3(cc.NG), dim3(CC_THREADS), lds, s, cc);
    const hipError_t e = hipGetLastError();
    if (e == hipSuccess) {
      chained = true;
      // failure semantics: after a timed-out hand-off the critic (params, square_avg) is put back to its pre-train
      // version before the actor's apply (coma_chain_restore_kernel below) and the actor's apply is skipped (its
      // halt word), so the learner state is this train()'s starting state and COMALearner.train raises
      if (h->chain_trace) {   // debug: per-phase spans of workgroup 0 (100 MHz clock), averaged over <= 16 steps
        unsigned long long hb[16 * 8];
        MQ_HIP(hipMemcpyAsync(hb, h->chain_trace, sizeof(hb), hipMemcpyDeviceToHost, s));
        MQ_HIP(hipStreamSynchronize(s));
        double acc[8] = {0};
        for (int i = 1; i < 15; ++i)
          for (int k = 0; k < 8; ++k) acc[k] += 10.0 * (double)((k < 7 ? hb[i * 8 + k + 1] : hb[(i + 1) * 8]) - hb[i * 8 + k]);
        std::fprintf(stderr, "coma_chain ns/step: A %.0f bar1 %.0f B %.0f bar2 %.0f C %.0f bar3 %.0f D %.0f next %.0f\n",
                     acc[0] / 14, acc[1] / 14, acc[2] / 14, acc[3] / 14, acc[4] / 14, acc[5] / 14, acc[6] / 14, acc[7] / 14);
      }
    } else {   // the launch was refused: the three-launch path, from now on
      h->chain_env = false;
    }
    // Launched after the chain on a low-priority stream, so the chain's workgroups are normally dispatched first.
    // That order is a heuristic across hardware queues, not a guarantee: if actor workgroups take CUs first, the
    // chain's late workgroups start when they finish (the actor never waits on the chain), well inside the chain's
    // spin bound (CC_SPIN_LIMIT polls, orders of magnitude longer than the actor unroll); a timeout would still be
    // loud and leave the learner state unchanged (restore above)
    if (chained && try_overlap) {
      MQ_HIP(hipStreamWaitEvent(ah->side, ah->ev_fork, 0));
      if ((rc = agent_forward(ah->side)) != MQ_OK) return rc;
      MQ_HIP(hipEventRecord(ah->ev_join, ah->side));
      actor_side = true;
    }
  }
  int live = 0;
  for (int t = T - 1; t >= 0 && !chained; --t) {
    // live steps before t: exact in data-parallel mode, else assumed none was skipped (the kernels correct it)
    const int Lexp = dp ? live : T - 1 - t;
    hipLaunchKernelGGL(coma_l1_kernel, dim3(ca.KS, CH / 16, (R + kL1Rows - 1) / kL1Rows), dim3(256), lds_l1, s, ca, t,
                       Lexp);
    hipLaunchKernelGGL(coma_head_kernel, dim3(ca.nhead), dim3(kHeadThreads), lds_head, s, ca, t, Lexp);
    hipLaunchKernelGGL(coma_wgrad_kernel, dim3(ca.nwgrad), dim3(256), 0, s, ca, t);
    if (dp && h->dp_msum[t] > 0.0f) {   // sum the step's unnormalised gradient, then its norm from the sum
      ++live;
      MQ_HIP(hipGetLastError());
      rc = mc_allreduce(h, h->cgrad, h->Pc, s);
      if (rc) return rc;
      hipLaunchKernelGGL(sumsq_kernel, dim3(ca.nwgrad), dim3(256), 0, s, (const float*)h->cgrad, h->Pc, h->cnorm);
    }
  }
  MQ_HIP(hipGetLastError());
  if (!chained)
    hipLaunchKernelGGL(coma_capply_kernel, dim3((int)std::min<int64_t>((h->Pc + 255) / 256, 512)), dim3(256), 0, s,
                       ca);
  MQ_HIP(hipGetLastError());
  if (dp) {   // per-step critic stat sums; the replicated fields (mask sum, norm, live flag) come from rank 0
    if (h->dp_rank != 0) hipLaunchKernelGGL(coma_dp_crec_kernel, dim3((T + 255) / 256), dim3(256), 0, s, h->crec, T);
    MQ_HIP(hipGetLastError());
    rc = mc_allreduce_ws(h, h->crec, 8LL * T, s);
    if (rc) return rc;
  }

  if (h->timing) MQ_HIP(hipEventRecord(h->ev[2], s));
  // ---- actor: the agent unroll over t < T (coma_learner.py:52-57), online net only (launched above)
  if (actor_side) MQ_HIP(hipStreamWaitEvent(s, ah->ev_join, 0));
  else if ((rc = agent_forward(s)) != MQ_OK) return rc;
  // policy, baseline, advantage, loss sums and dLogits (coma_learner.py:59-77, basic_controller.py:53-73)
  const int npol = (int)((RT + 3) / 4);
  const float eps = epsilon, omeps = (float)(1.0 - (double)epsilon);
  hipLaunchKernelGGL(coma_policy_kernel, dim3(npol), dim3(256), 0, s, d, rpa, (const float*)w.Q,
                     (const float*)h->qvals, R, qv_r0, eps, omeps, (int)(c.mask_before_softmax != 0), h->Ap, h->dL,
                     h->pi, h->ppart);
  MQ_HIP(hipGetLastError());
  // BPTT with the dense output gradient
  {
    DhoProb p{h->dL, h->Ap, A, Pa + ah->off[MQ_P_FC2_W], h->dHo, RT};
    MQ_HIP(launch_gemm(p, (int)RT, mq::H, 1, s));
  }
  const int rw_bwd = std::min(2, pick_rw(d.R, 256));
  int nblk_bwd = (d.R + rw_bwd - 1) / rw_bwd;
  const size_t dyn = ((size_t)2 * d.A * mq::H + d.A) * sizeof(float);
  if (rw_bwd == 1)
    hipLaunchKernelGGL((gru_bwd_kernel<1, 0, true>), dim3(nblk_bwd), dim3(512), dyn, s, d, rpa, Pa, L, w, ah->len_rnn);
  else
    hipLaunchKernelGGL((gru_bwd_kernel<2, 0, true>), dim3(nblk_bwd), dim3(512), dyn, s, d, rpa, Pa, L, w, ah->len_rnn);
  MQ_HIP(hipGetLastError());
  {
    Dx1Prob p{w.dGI, Pa + ah->off[MQ_P_RNN_W_IH], w.X1, w.dP1, RT};
    MQ_HIP(launch_gemm(p, (int)RT, mq::H, 1, s));
  }
  int ns1;
  {
    const int tiles = (d.I + Dw1Prob::BN - 1) / Dw1Prob::BN;
    int ns = (int)std::min<int64_t>(kNsplitMax, std::max<int64_t>(1, RT / 256));
    ns = std::max(1, std::min(ns, (512 + tiles - 1) / tiles));
    int64_t chunk = ((RT + ns - 1) / ns + GBK - 1) / GBK * GBK;
    ns = (int)((RT + chunk - 1) / chunk);
    ns1 = ns;
    Dw1Prob p{d.I, w.dP1, w.XIN, w.slab_fc1, RT, ns};
    MQ_HIP(launch_gemm(p, mq::H, d.I, ns, s));
  }
  int ns2;
  {
    int ns = (int)std::min<int64_t>(kNsplitMax, std::max<int64_t>(1, RT / 256));
    int64_t chunk = ((RT + ns - 1) / ns + GBK - 1) / GBK * GBK;
    ns = (int)((RT + chunk - 1) / chunk);
    ns2 = ns;
    Dw2Prob p{h->dL, h->Ap, A, w.Hs, h->slab_fc2, RT, ns};
    MQ_HIP(launch_gemm(p, A, mq::H, ns, s));
  }
  int nnorm;
  {
    RedBuilder rb(h->red_tmp);
    rb.add(w.slab_fc1, ns1, (int64_t)mq::H * d.I + mq::H, h->agrad + ah->off[MQ_P_FC1_W], true);
    // W_ih .. b_hh: the prefix of each BPTT slab (its fc2 part is unused in the dense-dy mode)
    rb.add(w.slab_rnn, nblk_bwd, ah->off[MQ_P_FC2_W] - ah->off[MQ_P_RNN_W_IH], h->agrad + ah->off[MQ_P_RNN_W_IH],
           true, ah->len_rnn);
    rb.add(h->slab_fc2, ns2, (int64_t)A * mq::H + A, h->agrad + ah->off[MQ_P_FC2_W], true);
    rb.add(h->ppart, npol, MQ_NSUMS, h->agrad + h->Pa, false);
    hipLaunchKernelGGL(red_pass1_kernel, dim3(rb.b1), dim3(256), 0, s, rb.pl);
    MQ_HIP(hipGetLastError());
    if (rb.b2 > 4096) return set_err(MQ_ERR_ARG, "agent too large for the norm partial buffer");
    hipLaunchKernelGGL(red_pass2_kernel, dim3(rb.b2), dim3(256), 0, s, rb.pl, h->norm_part);
    MQ_HIP(hipGetLastError());
    nnorm = rb.b2;
  }
  if (repl && chained) {   // the chain's error word rides in the agent sums' spare slot 7 (0 on success)
    hipLaunchKernelGGL(coma_halt_to_sum_kernel, dim3(1), dim3(64), 0, s, (const int*)(h->cstate + 3),
                       h->agrad + h->Pa + 7);
    MQ_HIP(hipGetLastError());
  }
  if (dp || repl) {   // the agent gradient + loss / mask sums, then the norm partials of the summed gradient
    rc = mc_allreduce(h, h->agrad, h->Pa + MQ_NSUMS, s);
    if (rc) return rc;
    if (repl && chained) {   // any rank's chain failure halts every rank: all roll back, skip the apply and raise
      hipLaunchKernelGGL(coma_sum_to_halt_kernel, dim3(1), dim3(64), 0, s, (const float*)(h->agrad + h->Pa + 7),
                         h->cstate + 3);
      MQ_HIP(hipGetLastError());
    }
    nnorm = 256;
    hipLaunchKernelGGL(sumsq_kernel, dim3(nnorm), dim3(256), 0, s, (const float*)h->agrad, h->Pa, h->norm_part);
    MQ_HIP(hipGetLastError());
  }
  if (chained) {   // a timed-out chain (on any rank, when replicated): the critic back to its pre-train version
    hipLaunchKernelGGL(coma_chain_restore_kernel, dim3(64), dim3(256), 0, s, (const int*)h->cstate,
                       (const float*)h->Pbak, h->critic, h->csq, h->Pc);
    MQ_HIP(hipGetLastError());
  }
  {
    OptHP hp{c.lr, c.optim_alpha, c.optim_eps, c.grad_norm_clip, 1};
    const int blocks = (int)std::min<int64_t>((h->Pa + 255) / 256, 1024);
    hipLaunchKernelGGL(apply_kernel, dim3(blocks), dim3(256), 0, s, h->agent, h->agrad, h->asq, h->Pa,
                       (const float*)h->norm_part, nnorm, hp, h->stats + 8,
                       chained ? (const int*)(h->cstate + 3) : (const int*)nullptr);   // no actor step after a failure
    MQ_HIP(hipGetLastError());
  }
  hipLaunchKernelGGL(coma_stats_kernel, dim3(1), dim3(64), 0, s, (const float*)h->crec, T,
                     (const int*)h->cstate, h->stats);
  MQ_HIP(hipGetLastError());
  if (h->timing) MQ_HIP(hipEventRecord(h->ev[3], s));
  h->last_path = chained ? 1 : 0;
  h->last_T = T;
  h->last_R = d.R;   // the rows of pi (the actor's); qvals / targets keep the critic's R rows
  h->last_Rc = R;
  return MQ_OK;
}

int mc_set_data_parallel(mc_handle* h, mc_allreduce_fn allreduce, void* ctx, int32_t rank, float* scratch,
                         int64_t scratch_count) {
  if (!h) return set_err(MQ_ERR_ARG, "NULL handle");
  if (allreduce && (!scratch || scratch_count < 8LL * h->cfg.max_seq))
    return set_err(MQ_ERR_ARG, "mc_set_data_parallel: scratch must hold 8 * max_seq floats");
  h->dp_fn = allreduce;
  h->dp_ctx = ctx;
  h->dp_rank = rank;
  h->dp_scratch = scratch;
  h->dp_scratch_n = scratch_count;
  return MQ_OK;
}

// mc_allreduce_fn over the handle's RCCL communicator (ctx = the mc_handle)
static int mc_rccl_allreduce(float* buf, int64_t count, void* stream, void* ctx) {
  mc_handle* h = (mc_handle*)ctx;
  return ncclAllReduce(buf, buf, (size_t)count, ncclFloat, ncclSum, h->comm, (hipStream_t)stream) == ncclSuccess ? 0 : 1;
}

int mc_set_actor_shard(mc_handle* h, int32_t lo, int32_t hi) {
  if (!h) return set_err(MQ_ERR_ARG, "NULL handle");
  if (hi > lo && (lo < 0 || hi > h->cfg.max_batch)) return set_err(MQ_ERR_ARG, "mc_set_actor_shard: bad episode range");
  h->shard_lo = hi > lo ? lo : 0;
  h->shard_hi = hi > lo ? hi : 0;
  return MQ_OK;
}

int mc_comm_attach(mc_handle* h, const uint8_t* id, int32_t rank, int32_t world) {
  if (!h) return set_err(MQ_ERR_ARG, "NULL handle");
  if (h->comm) return set_err(MQ_ERR_STATE, "a communicator is already attached");
  const int64_t n = 8LL * h->cfg.max_seq;
  if (!h->comm_scratch) MQ_HIP(hipMalloc(&h->comm_scratch, n * sizeof(float)));
  const int rc = comm_init(&h->comm, id, rank, world);
  if (rc) return rc;
  h->comm_owned = true;
  return mc_set_data_parallel(h, mc_rccl_allreduce, h, rank, h->comm_scratch, n);
}

int mc_comm_use(mc_handle* h, void* comm) {
  if (!h || !comm) return set_err(MQ_ERR_ARG, "NULL handle or communicator");
  if (h->comm) return set_err(MQ_ERR_STATE, "a communicator is already attached");
  int rank = 0;
  const ncclResult_t r = ncclCommUserRank((ncclComm_t)comm, &rank);
  if (r != ncclSuccess) return set_err(MQ_ERR_ARG, std::string("ncclCommUserRank: ") + ncclGetErrorString(r));
  const int64_t n = 8LL * h->cfg.max_seq;
  if (!h->comm_scratch) MQ_HIP(hipMalloc(&h->comm_scratch, n * sizeof(float)));
  h->comm = (ncclComm_t)comm;
  h->comm_owned = false;
  return mc_set_data_parallel(h, mc_rccl_allreduce, h, rank, h->comm_scratch, n);
}

int mc_comm_detach(mc_handle* h) {
  if (!h) return set_err(MQ_ERR_ARG, "NULL handle");
  if (h->comm && h->comm_owned) (void)ncclCommDestroy(h->comm);
  const bool was_rccl = h->dp_fn == mc_rccl_allreduce;
  h->comm = nullptr;
  h->comm_owned = false;
  return was_rccl ? mc_set_data_parallel(h, nullptr, nullptr, 0, nullptr, 0) : MQ_OK;
}

int mc_set_timing(mc_handle* h, int32_t on) {
  if (!h) return set_err(MQ_ERR_ARG, "NULL handle");
  for (auto& e : h->ev)
    if (!e) MQ_HIP(hipEventCreate(&e));
  h->timing = on != 0;
  return MQ_OK;
}

int mc_phase_times(mc_handle* h, float* ms) {
  if (!h || !ms) return set_err(MQ_ERR_ARG, "NULL argument");
  if (!h->ev[3]) return set_err(MQ_ERR_STATE, "timing was never enabled");
  MQ_HIP(hipEventSynchronize(h->ev[3]));
  for (int i = 0; i < 3; ++i) MQ_HIP(hipEventElapsedTime(&ms[i], h->ev[i], h->ev[i + 1]));
  return MQ_OK;
}

int32_t mc_last_critic_path(const mc_handle* h) { return h ? h->last_path : -1; }

int mc_update_targets(mc_handle* h, void* stream) {
  if (!h || !h->critic) return set_err(MQ_ERR_STATE, "mc_update_targets before mc_bind");
  MQ_HIP(hipMemcpyAsync(h->tcritic, h->critic, h->Pc * sizeof(float), hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return MQ_OK;
}

int mc_policy(float* logits, const int32_t* avail, int32_t rows, int32_t n_actions, float epsilon,
              int32_t mask_before_softmax, int32_t test_mode, void* stream) {
  if (!logits || !avail || rows < 0 || n_actions < 1 || n_actions > 64) return set_err(MQ_ERR_ARG, "bad mc_policy args");
  if (rows == 0) return MQ_OK;
  hipLaunchKernelGGL(mc_policy_kernel, dim3((rows + 3) / 4), dim3(256), 0, (hipStream_t)stream, logits, avail,
                     (int)rows, (int)n_actions, epsilon, (int)mask_before_softmax, (int)test_mode);
  MQ_HIP(hipGetLastError());
  return MQ_OK;
}

int mc_copy_intermediate(mc_handle* h, int which, float* dst, int64_t* count, void* stream) {
  if (!h || h->last_T <= 0) return set_err(MQ_ERR_STATE, "no COMA train step has run");
  const int64_t TR = (int64_t)h->last_T * h->last_R, TRc = (int64_t)h->last_T * h->last_Rc;
  const float* src;
  int64_t cnt;
  switch (which) {
    case 0: src = h->qvals; cnt = TRc * h->cfg.n_actions; break;
    case 1: src = h->tgt; cnt = TRc; break;
    case 2: src = h->pi; cnt = TR * h->cfg.n_actions; break;
    default: return set_err(MQ_ERR_ARG, "unknown COMA intermediate id");
  }
  if (count) *count = cnt;
  if (dst) MQ_HIP(hipMemcpyAsync(dst, src, cnt * sizeof(float), hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return MQ_OK;
}

}  // extern "C"
