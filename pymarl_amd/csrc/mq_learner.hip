// libmq_learner: MI355X-native QMIX/VDN learner step behind the C ABI of include/mq_learner.h.
//
// One train step (QLearner.train, q_learner.py:37-116) is this stream-ordered launch sequence:
//   fc1      gemm  X1 = relu(W1 [obs | a_{t-1} | id] + b1)               both nets, rows gathered by episode id
//   gi       gemm  GI = W_ih X1 + b_ih                                    both nets
//   gru_fwd  recur h_t = GRU(GI_t, h_{t-1})                              both nets, serial over T
//   fc2      gemm  Q = W2 H + b2                                          both nets
//   hyper    gemm  QMIX hypernet outputs of state[:, :-1] / state[:, 1:] both nets (QMIX only)
//   mix      per (t, episode): chosen gather, double-Q select, mixer fwd, TD, masked L2 sums, mixer bwd
//   gru_bwd  recur BPTT; dW_hh, dW_ih, dW2 and biases accumulated in-kernel, dGI written out
//   dx1      gemm  dP1 = (dGI W_ih) * [X1 > 0]
//   dw1      gemm  [dW1 | db1] = dP1^T xin                                split-K
//   dwh      gemm  [dW_hyper | db_hyper] = dHYP^T state                   split-K (QMIX only)
//   reduce   deterministic two-pass slab sums -> flat gradient buffer (+ loss sums), per-block sums of squares
//   --- (data-parallel all-reduce of the gradient buffer happens here, in the caller)
//   apply    / sum(mask), clip_grad_norm_, RMSprop
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include <rccl/rccl.h>
#include "learner_gemms.hpp"
#include "gru_kernels.hpp"
#include "gru_fwd_fused.hpp"
#include "gru_fwd_pair.hpp"
#include "gru_bwd_fused.hpp"
#include "gru_tiles.hpp"
#include "mix_kernels.hpp"
#include "hyper_kernel.hpp"
#include "dwh_kernel.hpp"
#include "optim_kernels.hpp"
#include "module_fwd.hpp"
#include "switches.hpp"

using namespace mq;

namespace {

std::mutex g_err_mu;
std::string g_err;

int set_err(int code, const std::string& msg) {
  std::lock_guard<std::mutex> lk(g_err_mu);
  g_err = msg;
  return code;
}

// A kernel's static LDS plus a launch's dynamic LDS against the CU's LDS (160 KB on gfx950), checked before the
// launch (the static size is looked up once per kernel). A dispatch past it aborts the whole queue
// (HSA_STATUS_ERROR_INVALID_ALLOCATION), which HIP then reports at the next runtime call as "an illegal memory access
// was encountered", far from its cause: the round-5 fault of a stamped BPTT build was exactly that.
int lds_fits(const void* fn, size_t dyn, const char* what) {
  static std::mutex mu;
  static std::vector<std::pair<const void*, size_t>> known;
  static int limit = 0;
  size_t st = 0;
  bool found = false;
  {
    std::lock_guard<std::mutex> lk(mu);
    for (const auto& k : known)
      if (k.first == fn) { st = k.second; found = true; break; }
  }
  if (!found) {
    hipFuncAttributes fa;
    if (hipFuncGetAttributes(&fa, fn) != hipSuccess) return set_err(MQ_ERR_HIP, std::string(what) + ": hipFuncGetAttributes");
    st = fa.sharedSizeBytes;
    std::lock_guard<std::mutex> lk(mu);
    known.emplace_back(fn, st);
    if (limit == 0) {
      int dev = 0, v = 0;
      limit = (hipGetDevice(&dev) == hipSuccess &&
               hipDeviceGetAttribute(&v, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev) == hipSuccess && v > 0)
                  ? v : 160 * 1024;
    }
  }
  if (st + dyn > (size_t)limit)
    return set_err(MQ_ERR_ARG, std::string(what) + " needs " + std::to_string(st) + " B of static + " +
                                   std::to_string(dyn) + " B of dynamic LDS, past the " + std::to_string(limit) +
                                   " B a workgroup can have");
  return MQ_OK;
}
#define MQ_LDS(fn, dyn)                                                        \
  do {                                                                         \
    const int _rc = lds_fits((const void*)(fn), (size_t)(dyn), #fn);          \
    if (_rc) return _rc;                                                       \
  } while (0)

#define MQ_HIP(expr)                                                                        \
  do {                                                                                      \
    hipError_t _e = (expr);                                                                 \
    if (_e != hipSuccess)                                                                   \
      return set_err(MQ_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));        \
  } while (0)

constexpr int kNsplitMax = 128;
enum Phase { PH_FC1, PH_GI, PH_GRUF, PH_FC2, PH_HYP, PH_MIX, PH_GRUB, PH_DX1, PH_DW1, PH_DWH, PH_RED, PH_APPLY,
             PH_N };
const char* kPhaseNames = "fc1;gi;gru_fwd;fc2;hyper;mix;gru_bwd;dx1;dw1;dwh;reduce;apply";

int pick_rw(int R, int max_blocks) {
  const int rws[4] = {1, 2, 4, 8};
  for (int i = 0; i < 4; ++i)
    if ((R + rws[i] - 1) / rws[i] <= max_blocks) return rws[i];
  return 8;
}

}  // namespace

struct mq_handle {
  mq_config cfg;
  int I, E, NH;
  int64_t off[MQ_P_COUNT + 1];
  int64_t P;
  int64_t len_rnn, len_mix;
  int64_t pitch_rnn;   // the fused BPTT's slab pitch: len_rnn rounded up to 4 floats (16-byte slab rows)
  // bound (caller-owned)
  float *on = nullptr, *tg = nullptr, *grad = nullptr, *sq = nullptr, *stats = nullptr;
  int32_t* curmax_user = nullptr;
  // workspace (handle-owned)
  void* ws = nullptr;
  Work w;
  int32_t* curmax_ws = nullptr;
  // last step bookkeeping
  bool have_fb = false;
  Dims last;
  mq_plan plan{};
  int nsplit_fc1 = 1, nsplit_mix = 1, nblk_bwd = 1, nblk_mix = 1, n_norm_part = 0;
  // plan overrides (switches.hpp MQ_PLAN; A/B runs and tests, read once here)
  bool force_unfused = plan_flag("unfused_fwd");       // the unfused forward (GEMMs around gru_fwd<RW>)
  bool force_unfused_bwd = plan_flag("unfused_bwd");   // the unfused BPTT (gru_bwd<RW> + dX1 / dW1 GEMMs)
  // rows up to which the fused BPTT (one row per workgroup, one workgroup per CU) is used: past the CU count the
  // rows run as a second wave of workgroups, which still beats gru_bwd<2> + dX1 + dW1 at configs[3]'s shard
  // (R = 320; round 3)
  static constexpr int fused_bwd_rmax = 512;
  // m-slices of the dW_hyper pass (A/B at cfg2, DESIGN §3: 4 / 8 / 16 / 32 -> 238.5 / 235.1 / 236.3 / 237.4 us)
  int dwh_split = plan_int("dwh_split", 8);
  // the row-tile MFMA forward / BPTT (gru_tiles.hpp) for batches past the one-row fused kernels (R > 512 rows);
  // row_tiles=1 forces it on any batch it can take (tests), =0 turns it off (A/B: the unfused GEMM path)
  int row_tiles = plan_int("row_tiles", -1);
  bool dp = false;   // gradient buffer is summed across ranks between mq_forward_backward and mq_apply
  ncclComm_t comm = nullptr;   // mq_comm_attach / mq_comm_use: the library all-reduces the grad buffer itself
  int comm_world = 0;
  bool comm_owned = false;     // mq_comm_attach created it (freed on detach); mq_comm_use borrows the caller's
  hipStream_t side = nullptr;   // COMA: the actor's side stream (coma_host.hpp)
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  // QMIX hypernet workgroups appended to the fused forward's grid (gru_fwd_fused.hpp hyper_fwd_body) when the
  // forward's 2R row-nets exceed two per CU: its second wave leaves CUs idle, and the hypernet fills them
  // (configs[3]'s shard, R = 320: 0.364 -> 0.346 ms a step). hyp_in_fwd=0 never appends (and launches hyper_ws_kernel
  // after the row-pair forward instead of running the hypernet inside it), =1 always (HYP bitwise the same either way)
  int hyp_in_fwd = plan_int("hyp_in_fwd", -1);
  // dW_hyper's tiles appended to the fused BPTT's grid (gru_bwd_fused.hpp, DWH = 1) when its rows exceed the CUs
  // (a second wave of rows leaves CUs idle); dwh_in_bwd=0 never, =1 always (bitwise either way)
  int dwh_in_bwd = plan_int("dwh_in_bwd", -1);
  // the row-pair forward (gru_fwd_pair.hpp: both nets of a row in one workgroup, one per CU) when the rows fit one
  // wave of workgroups; fwd_pair=0 keeps the one-row-net kernel, =1 forces the pair
  int fwd_pair = plan_int("fwd_pair", -1);
  bool pair_hyp_epi = plan_flag("pair_hyp_epi");   // the pair forward's hypernet as its epilogue, not on waves 4 / 5
  // mix_kernel<false> where mix_kernel<true> (staged selection rows) would run
  bool mix_generic = plan_flag("mix_generic");
  int num_cu = 0;
  // timing: a ring of `slots` steps x PH_N (start, stop) event pairs; phases outside `mask` are not recorded
  int slots = 0;
  uint32_t mask = 0;
  int64_t tstep = 0;
  std::vector<hipEvent_t> ev0, ev1;
  std::vector<uint8_t> ev_used;
};

namespace {

void compute_layout(mq_handle* h) {
  const mq_config& c = h->cfg;
  const int Hd = mq::H, n = c.n_agents, A = c.n_actions, S = c.state_dim, E = h->E, I = h->I;
  int64_t sz[MQ_P_COUNT] = {};
  sz[MQ_P_FC1_W] = (int64_t)Hd * I; sz[MQ_P_FC1_B] = Hd;
  sz[MQ_P_RNN_W_IH] = 3LL * Hd * Hd; sz[MQ_P_RNN_W_HH] = 3LL * Hd * Hd;
  sz[MQ_P_RNN_B_IH] = 3 * Hd; sz[MQ_P_RNN_B_HH] = 3 * Hd;
  sz[MQ_P_FC2_W] = (int64_t)A * Hd; sz[MQ_P_FC2_B] = A;
  if (c.mixer == MQ_MIXER_QMIX) {
    sz[MQ_P_HW1_W] = (int64_t)E * n * S; sz[MQ_P_HW1_B] = (int64_t)E * n;
    sz[MQ_P_HWF_W] = (int64_t)E * S; sz[MQ_P_HWF_B] = E;
    sz[MQ_P_HB1_W] = (int64_t)E * S; sz[MQ_P_HB1_B] = E;
    sz[MQ_P_V0_W] = (int64_t)E * S; sz[MQ_P_V0_B] = E;
    sz[MQ_P_V2_W] = E; sz[MQ_P_V2_B] = 1;
  }
  int64_t o = 0;
  for (int i = 0; i < MQ_P_COUNT; ++i) { h->off[i] = o; o += sz[i]; }
  h->off[MQ_P_COUNT] = o;
  h->P = o;
  h->len_rnn = h->off[MQ_P_FC2_B] + A - h->off[MQ_P_RNN_W_IH];
  h->pitch_rnn = (h->len_rnn + 3) & ~int64_t(3);
  h->len_mix = h->off[MQ_P_V2_W] - h->off[MQ_P_HW1_W];
}

int64_t align_up(int64_t x) { return (x + 63) & ~int64_t(63); }

Dims make_dims(const mq_handle* h, const mq_replay* b) {
  const mq_config& c = h->cfg;
  Dims d;
  d.n = c.n_agents; d.A = c.n_actions; d.O = c.obs_dim; d.S = c.state_dim; d.E = h->E; d.I = h->I; d.NH = h->NH;
  d.B = b->batch_size; d.Tp = b->t_len; d.T = b->t_len - 1; d.R = d.B * d.n; d.M = d.T * d.B;
  d.t_stride = b->t_stride;
  d.last_action = c.obs_last_action; d.agent_id = c.obs_agent_id; d.mixer = c.mixer; d.double_q = c.double_q;
  d.gamma = c.gamma;
  d.huber = c.huber_delta;
  d.dR = make_fastdiv((uint32_t)d.R);
  d.dN = make_fastdiv((uint32_t)d.n);
  d.dB = make_fastdiv((uint32_t)d.B);
  d.dO = make_fastdiv((uint32_t)d.O);
  d.dI = make_fastdiv((uint32_t)d.I);
  d.dS = make_fastdiv((uint32_t)std::max(d.S, 1));
  return d;
}

Rep make_rep(const mq_replay* b) {
  Rep r;
  r.obs = b->obs; r.state = b->state; r.actions = b->actions; r.avail = b->avail_actions; r.reward = b->reward;
  r.term = b->terminated; r.filled = b->filled; r.ep_ids = b->ep_ids; r.avail_bits = b->avail_bits;
  r.nids = 0;
  if (b->ep_ids_host && b->batch_size <= MQ_INLINE_IDS) {   // ids in the kernel arguments (check_batch validated)
    r.nids = b->batch_size;
    for (int i = 0; i < b->batch_size; ++i) r.ids[i] = (int32_t)b->ep_ids_host[i];
  }
  return r;
}

Lay make_lay(const mq_handle* h) {
  Lay L;
  for (int i = 0; i <= MQ_P_COUNT; ++i) L.o[i] = h->off[i];
  return L;
}

int check_batch(const mq_handle* h, const mq_replay* b) {
  if (!b) return set_err(MQ_ERR_ARG, "batch is NULL");
  if (!b->obs || !b->actions || !b->avail_actions || !b->reward || !b->terminated || !b->filled)
    return set_err(MQ_ERR_ARG, "batch is missing a required field pointer");
  if (h->cfg.mixer == MQ_MIXER_QMIX && !b->state) return set_err(MQ_ERR_ARG, "QMIX needs batch.state");
  if (b->batch_size < 1 || b->batch_size > h->cfg.max_batch)
    return set_err(MQ_ERR_ARG, "batch_size " + std::to_string(b->batch_size) + " outside [1, max_batch=" +
                                   std::to_string(h->cfg.max_batch) + "]");
  if (b->t_len < 2 || b->t_len > h->cfg.max_seq || b->t_len > b->t_stride)
    return set_err(MQ_ERR_ARG, "t_len " + std::to_string(b->t_len) + " must be in [2, min(max_seq, t_stride)]");
  if ((int64_t)b->t_len * b->batch_size * h->cfg.n_agents >= (1LL << 31))
    return set_err(MQ_ERR_ARG, "batch too large for 32-bit row indices");
  if (b->ep_ids_host && b->batch_size <= MQ_INLINE_IDS) {
    for (int i = 0; i < b->batch_size; ++i)
      if (b->ep_ids_host[i] < 0 || b->ep_ids_host[i] >= b->n_episodes)
        return set_err(MQ_ERR_ARG, "episode id " + std::to_string(b->ep_ids_host[i]) + " outside [0, n_episodes)");
  } else if (!b->ep_ids && b->batch_size > b->n_episodes) {
    return set_err(MQ_ERR_ARG, "batch_size exceeds n_episodes with no episode ids");
  }
  return MQ_OK;
}

struct PhaseTimer {
  mq_handle* h;
  hipStream_t s;
  int cur = -1;
  int idx(int p) const { return (int)(h->tstep % h->slots) * PH_N + p; }
  void begin(int p) {
    end();
    if (h->slots <= 0 || !((h->mask >> p) & 1u)) return;
    (void)hipEventRecord(h->ev0[idx(p)], s);
    h->ev_used[idx(p)] = 1;
    cur = p;
  }
  void end() {
    if (cur < 0) return;
    (void)hipEventRecord(h->ev1[idx(cur)], s);
    cur = -1;
  }
};

template <int RW>
hipError_t launch_gru_fwd(const Dims& d, const mq_handle* h, const Lay& L, const Work& w, hipStream_t s) {
  dim3 grid((d.R + RW - 1) / RW, 2);
  hipLaunchKernelGGL(gru_fwd_kernel<RW>, grid, dim3(256), 0, s, d, (const float*)h->on, (const float*)h->tg, L, w);
  return hipGetLastError();
}

template <int RW>
hipError_t launch_gru_bwd(const Dims& d, const Rep& rp, const mq_handle* h, const Lay& L, const Work& w,
                          hipStream_t s, int* nblk) {
  *nblk = (d.R + RW - 1) / RW;
  const size_t dyn = ((size_t)2 * d.A * mq::H + d.A) * sizeof(float);
  hipLaunchKernelGGL(gru_bwd_kernel<RW>, dim3(*nblk), dim3(512), dyn, s, d, rp, (const float*)h->on, L, w,
                     h->len_rnn);
  return hipGetLastError();
}

// Plan the slab reductions of one step: regions in gradient order, then the loss sums (not part of the norm).
struct RedBuilder {
  RedPlan pl{};
  int b1 = 0, b2 = 0;
  float* tmp;
  explicit RedBuilder(float* t) : tmp(t) {}
  // returns true when the region is summed by pass 2 straight from its slabs (no pass-1 blocks read them)
  bool add(const float* src, int nslab, int64_t len, float* dst, bool sq, int64_t pitch = 0, bool direct_ok = false,
           int perm = 0) {
    if (len <= 0 || nslab <= 0) return false;
    RedRegion& R = pl.r[pl.nr++];
    R.src = src; R.dst = dst; R.len = len; R.pitch = pitch > 0 ? pitch : len; R.nslab = nslab; R.sq = sq ? 1 : 0;
    R.perm = perm;
    if (direct_ok && nslab <= kRedZ) {   // pass 2 sums the slabs themselves: no pass-1 blocks, no tmp
      R.zc = 1; R.ng = nslab; R.tmp = (float*)src; R.tpitch = R.pitch; R.vec = 0; R.xcd = 0;
      R.blk1 = b1;
      R.blk2 = b2; b2 += (int)((len + 255) / 256);
      return true;
    }
    R.tpitch = len;
    // at most kRedZ groups, so pass 2 sums <= 16 partials per element with all loads in flight
    R.zc = (nslab + kRedZ - 1) / kRedZ;
    R.ng = (nslab + R.zc - 1) / R.zc;
    R.tmp = tmp;
    tmp += R.ng * len;
    R.vec = (len % 4 == 0 && R.pitch % 4 == 0 && ((uintptr_t)src & 15) == 0 && ((uintptr_t)R.tmp & 15) == 0) ? 1 : 0;
    R.xcd = (nslab % 128 == 0 && R.ng == kRedZ && b1 % 16 == 0) ? 1 : 0;
    const int nb = (int)((len + 255) / 256), nb1 = R.vec ? (int)((len + 1023) / 1024) : nb;
    R.blk1 = b1; b1 += nb1 * R.ng;
    R.blk2 = b2; b2 += nb;
    return false;
  }
};

// Side stream and fork / join events (COMA's actor overlap), created on first use. Lowest stream priority: the
// work on the caller's stream keeps the arbiter's preference.
hipError_t ensure_side(mq_handle* h) {
  if (h->side) return hipSuccess;
  int least = 0, greatest = 0;
  hipError_t e = hipDeviceGetStreamPriorityRange(&least, &greatest);
  if (e == hipSuccess) e = hipStreamCreateWithPriority(&h->side, hipStreamNonBlocking, least);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&h->ev_fork, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&h->ev_join, hipEventDisableTiming);
  return e;
}

int device_cus(mq_handle* h) {
  if (h->num_cu == 0) {
    int dev = 0, ncu = 0;
    h->num_cu = (hipGetDevice(&dev) == hipSuccess &&
                 hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess) ? ncu : -1;
  }
  return h->num_cu;
}

}  // namespace

extern "C" {

const char* mq_last_error(void) {
  std::lock_guard<std::mutex> lk(g_err_mu);
  return g_err.c_str();
}

const char* mq_phase_names(void) { return kPhaseNames; }

int mq_create(const mq_config* cfg, mq_handle** out) {
  if (!cfg || !out) return set_err(MQ_ERR_ARG, "NULL argument");
  const mq_config& c = *cfg;
  if (c.mixer != MQ_MIXER_NONE && c.mixer != MQ_MIXER_VDN && c.mixer != MQ_MIXER_QMIX)
    return set_err(MQ_ERR_ARG, "Mixer " + std::to_string(c.mixer) + " not recognised.");
  if (c.rnn_hidden_dim != mq::H) return set_err(MQ_ERR_ARG, "rnn_hidden_dim must be 64");
  if (c.n_agents < 1 || c.n_agents > 64) return set_err(MQ_ERR_ARG, "n_agents must be in [1, 64]");
  if (c.n_actions < 1 || c.n_actions > 64) return set_err(MQ_ERR_ARG, "n_actions must be in [1, 64]");
  if (c.obs_dim < 1 || c.state_dim < 1) return set_err(MQ_ERR_ARG, "obs_dim / state_dim must be positive");
  if (c.mixer == MQ_MIXER_QMIX && (c.mixing_embed_dim < 1 || c.mixing_embed_dim > 64))
    return set_err(MQ_ERR_ARG, "mixing_embed_dim must be in [1, 64]");
  if (c.max_batch < 1 || c.max_seq < 2) return set_err(MQ_ERR_ARG, "max_batch >= 1 and max_seq >= 2 required");
  if (!(c.huber_delta >= 0.0f)) return set_err(MQ_ERR_ARG, "huber_delta must be >= 0 (0: the reference's L2 loss)");

  mq_handle* h = new mq_handle();
  h->cfg = c;
  h->E = c.mixer == MQ_MIXER_QMIX ? c.mixing_embed_dim : 0;
  h->I = c.obs_dim + (c.obs_last_action ? c.n_actions : 0) + (c.obs_agent_id ? c.n_agents : 0);
  h->NH = h->E * (c.n_agents + 3);
  compute_layout(h);

  const int64_t n = c.n_agents, A = c.n_actions, Hd = mq::H;
  const int64_t RT = (int64_t)c.max_seq * c.max_batch * n;
  const int64_t Mm = (int64_t)(c.max_seq - 1) * c.max_batch;
  const int64_t Rm = (int64_t)c.max_batch * n;
  const int64_t nmix = (Mm + 3) / 4;
  const int64_t NH = h->NH;
  auto ng = [](int64_t ns) { return std::min<int64_t>(ns, kRedZ); };
  const int64_t nfc1 = std::max<int64_t>(kNsplitMax, Rm);   // fc1 slabs: split-K GEMM, or one per fused-BPTT row
  const int64_t red_tmp = ng(Rm) * h->len_rnn + ng(nfc1) * (Hd * h->I + Hd) + ng(kNsplitMax) * h->len_mix +
                          ng(nmix) * (h->E + 1) + ng(nmix) * 8;
  const int64_t norm_parts = (Hd * h->I + Hd + 255) / 256 + (h->len_rnn + 255) / 256 + (h->len_mix + 255) / 256 +
                             (h->E + 1 + 255) / 256 + 1 + 8;
  int64_t sizes[20] = {
      2 * RT * Hd,                                   // X1
      2 * RT * 3 * Hd,                               // GI
      2 * RT * Hd,                                   // Hs (both nets)
      RT * 4 * Hd,                                   // Gates
      2 * RT * A,                                    // Q
      2 * Mm * NH,                                   // HYP
      Mm * NH,                                       // dHYP
      Mm * n,                                        // dch
      RT * 3 * Hd,                                   // dGI
      RT * Hd,                                       // dP1
      nfc1 * (Hd * h->I + Hd),                       // slab_fc1
      Rm * h->pitch_rnn,                             // slab_rnn (RW = 1 worst case)
      (int64_t)kNsplitMax * h->len_mix,              // slab_mix
      nmix * (h->E + 1),                             // slab_v2
      nmix * 8,                                      // loss_part
      std::max<int64_t>(norm_parts, 256),            // norm_part
      Mm * n,                                        // curmax (int32)
      red_tmp,                                       // two-pass reduction partials
      RT * h->I,                                     // XIN (dense agent inputs)
      Mm * c.state_dim,                              // S0 (gathered state[:, :-1] rows)
  };
  int64_t total = 0, offs[20];
  for (int i = 0; i < 20; ++i) { offs[i] = total; total += align_up(std::max<int64_t>(sizes[i], 1)); }
  hipError_t e = hipMalloc(&h->ws, total * sizeof(float));
  if (e != hipSuccess) {
    delete h;
    return set_err(MQ_ERR_HIP, std::string("workspace hipMalloc(") + std::to_string(total * 4) + " B): " +
                                   hipGetErrorString(e));
  }
  float* base = (float*)h->ws;
  Work& w = h->w;
  w.X1 = base + offs[0]; w.GI = base + offs[1]; w.Hs = base + offs[2]; w.Gates = base + offs[3];
  w.Q = base + offs[4]; w.HYP = base + offs[5]; w.dHYP = base + offs[6]; w.dch = base + offs[7];
  w.dGI = base + offs[8]; w.dP1 = base + offs[9]; w.slab_fc1 = base + offs[10]; w.slab_rnn = base + offs[11];
  w.slab_mix = base + offs[12]; w.slab_v2 = base + offs[13]; w.loss_part = base + offs[14];
  w.norm_part = base + offs[15];
  h->curmax_ws = (int32_t*)(base + offs[16]);
  w.red_tmp = base + offs[17];
  w.XIN = base + offs[18];
  w.S0 = base + offs[19];
  w.curmax = h->curmax_ws;
  *out = h;
  return MQ_OK;
}

int mq_destroy(mq_handle* h) {
  if (!h) return MQ_OK;
  for (auto e : h->ev0) (void)hipEventDestroy(e);
  for (auto e : h->ev1) (void)hipEventDestroy(e);
  if (h->ev_fork) (void)hipEventDestroy(h->ev_fork);
  if (h->ev_join) (void)hipEventDestroy(h->ev_join);
  if (h->side) (void)hipStreamDestroy(h->side);
  if (h->ws) (void)hipFree(h->ws);
  if (h->comm && h->comm_owned) (void)ncclCommDestroy(h->comm);
  delete h;
  return MQ_OK;
}

int mq_param_offsets(const mq_handle* h, int64_t* offsets) {
  if (!h || !offsets) return set_err(MQ_ERR_ARG, "NULL argument");
  for (int i = 0; i <= MQ_P_COUNT; ++i) offsets[i] = h->off[i];
  return MQ_OK;
}

int mq_bind(mq_handle* h, float* online, float* target, float* grad, float* sq_avg, float* stats,
            int32_t* cur_max) {
  // target/grad/sq_avg/stats may be NULL for an inference-only handle (mq_mac_forward / mq_agent_forward)
  if (!h || !online) return set_err(MQ_ERR_ARG, "NULL handle or online parameters in mq_bind");
  h->on = online; h->tg = target; h->grad = grad; h->sq = sq_avg; h->stats = stats; h->curmax_user = cur_max;
  return MQ_OK;
}

static int fb_impl(mq_handle* h, const mq_replay* batch, hipStream_t s);

int mq_forward_backward(mq_handle* h, const mq_replay* batch, void* stream) {
  return fb_impl(h, batch, (hipStream_t)stream);
}

int mq_train_step(mq_handle* h, const mq_replay* batch, void* stream) {
  if (!h) return set_err(MQ_ERR_ARG, "NULL handle");
  const int rc = fb_impl(h, batch, (hipStream_t)stream);
  if (rc) return rc;
  return mq_apply(h, stream);
}

static int fb_impl(mq_handle* h, const mq_replay* batch, hipStream_t s) {
  if (!h) return set_err(MQ_ERR_ARG, "NULL handle");
  if (!h->on || !h->tg || !h->grad || !h->sq || !h->stats)
    return set_err(MQ_ERR_STATE, "training needs online, target, grad, sq_avg and stats bound (mq_bind)");
  int rc = check_batch(h, batch);
  if (rc) return rc;
  const Dims d = make_dims(h, batch);
  const Rep rp = make_rep(batch);
  const Lay L = make_lay(h);
  Work w = h->w;
  int32_t* curmax = h->curmax_user ? h->curmax_user : h->curmax_ws;
  const int64_t RT = (int64_t)d.Tp * d.R;
  PhaseTimer pt{h, s};
  const mq_config& c = h->cfg;

  mq_plan plan{};
  plan.rows = d.R;
  plan.inline_ids = rp.nids > 0 ? 1 : 0;
  const int rw_bwd = std::min(2, pick_rw(d.R, 256));
  const int kq1 = tile_kq1(d.O);
  const bool tiles = tiles_ok(d.I, d.O, d.A, d.n, d.Tp, RT) && !h->force_unfused && !h->force_unfused_bwd &&
                     (h->row_tiles == 1 || (h->row_tiles < 0 && d.R > 512));
  const bool fused_bwd = !tiles && d.R <= h->fused_bwd_rmax && fused_bwd_ok(d.I, d.O, d.A, d.n, RT) &&
                         !h->force_unfused_bwd;
  const int rw_fwd = pick_rw(d.R, 512);
  bool hyp_in_fwd = false;
  plan.tiles = tiles ? 1 : 0;
  if (tiles) {
    // row tiles of 32 (two M-tiles) per workgroup, both nets: the recurrence and fc1 / W_ih / fc2 on MFMA
    pt.begin(PH_GRUF);
    const dim3 grid(16 * (((d.R + TR_F - 1) / TR_F + 7) / 8));   // row tiles x 2 nets, XCD-paired (gru_tiles.hpp)
    const float *P0 = h->on, *P1 = h->tg;
    if (kq1 == 8) hipLaunchKernelGGL(gru_fwd_tile_kernel<8>, grid, dim3(512), 0, s, d, rp, P0, P1, L, w);
    else if (kq1 == 20) hipLaunchKernelGGL(gru_fwd_tile_kernel<20>, grid, dim3(512), 0, s, d, rp, P0, P1, L, w);
    else if (kq1 == 40) hipLaunchKernelGGL(gru_fwd_tile_kernel<40>, grid, dim3(512), 0, s, d, rp, P0, P1, L, w);
    else if (kq1 == 72) hipLaunchKernelGGL(gru_fwd_tile_kernel<72>, grid, dim3(512), 0, s, d, rp, P0, P1, L, w);
    else hipLaunchKernelGGL(gru_fwd_tile_kernel<80>, grid, dim3(512), 0, s, d, rp, P0, P1, L, w);
    MQ_HIP(hipGetLastError());
  } else if (rw_fwd == 1 && fused_fwd_ok(d.I, d.O, d.A, d.n, RT) && !h->force_unfused) {
    plan.fused_fwd = 1;
    // one row per workgroup: fc1 / W_ih / fc2 ride on the recurrence's idle matrix cores (gru_fwd_fused.hpp)
    pt.begin(PH_GRUF);
    const bool two_waves = device_cus(h) > 0 && d.R > h->num_cu;   // 2R row-nets at two per CU
    // the row-pair forward when the rows fit one wave of workgroups (MQ_PLAN fwd_pair=1 forces it, =0 keeps the one-row-net
    // kernel); hyp_in_fwd=1 asks for the one-row-net kernel with the hypernet appended to its grid
    const bool pair = h->hyp_in_fwd != 1 && pair_fwd_ok(d.I, d.O, d.A, d.n, RT) &&
                      (h->fwd_pair == 1 || (h->fwd_pair < 0 && !two_waves && device_cus(h) > 0));
    hyp_in_fwd = !pair && (h->hyp_in_fwd == 1 || (h->hyp_in_fwd < 0 && two_waves)) && c.mixer == MQ_MIXER_QMIX &&
                 hyper_ws_ok(d.S, d.E, d.NH, d.M) && hyf_ok(d.S, d.E, d.NH, d.M);
    if (hyp_in_fwd) {
      plan.hyper = MQ_HYP_WS;
      launch_fwd_fused_hyp(s, d, rp, (const float*)h->on, (const float*)h->tg, L, w);
    } else if (pair) {
      plan.fused_fwd = 2;
      // the QMIX hypernet as the pair kernel's epilogue (hyp_in_fwd=0 keeps hyper_ws_kernel after it)
      hyp_in_fwd = h->hyp_in_fwd != 0 && c.mixer == MQ_MIXER_QMIX && hyper_ws_ok(d.S, d.E, d.NH, d.M) &&
                   hyf_ok(d.S, d.E, d.NH, d.M);
      if (hyp_in_fwd) plan.hyper = MQ_HYP_WS;
      std::string stamp_path;   // diagnostic (MQ_DIAG pair_stamp=<file>): step stamps of the first 8 workgroups
      const bool want_stamp = env_item("MQ_DIAG", "pair_stamp", &stamp_path) && !stamp_path.empty();
      const int hsched = env_int("MQ_DIAG", "hyp_sched", kHypSched, 16);   // tuning: the in-loop tile schedule
      // on waves 4 / 5 inside the kernel when every hypernet block has a workgroup, else as its epilogue
      // (pair_hyp_epi forces the epilogue)
      const int pair_hyp = !hyp_in_fwd ? 0 : (2 * ((d.M + 31) / 32) <= d.R && !h->pair_hyp_epi) ? 2 : 1;
      // the stamp build has the 5-slot gather only: shapes past it run unstamped (never a partial gather)
      const bool stamp = want_stamp && d.Tp <= 512 && FCH * d.O <= 256 * 5;
      launch_fwd_pair(s, d, rp, (const float*)h->on, (const float*)h->tg, L, w, pair_hyp, stamp, hsched);
      if (stamp) {
        std::vector<uint32_t> st((size_t)8 * PST);
        MQ_HIP(hipMemcpyAsync(st.data(), w.slab_rnn, st.size() * 4, hipMemcpyDeviceToHost, s));
        MQ_HIP(hipStreamSynchronize(s));
        if (FILE* f = fopen(stamp_path.c_str(), "ab")) { fwrite(st.data(), 4, st.size(), f); fclose(f); }
      }
    } else {
      launch_fwd_fused(dim3(d.R, 2), s, d, rp, (const float*)h->on, (const float*)h->tg, L, w);
    }
    MQ_HIP(hipGetLastError());
  } else {
    plan.rw_fwd = rw_fwd;
    pt.begin(PH_FC1);
    {
      // the dense agent-input copy (XIN) is dW1's operand, fused or not
      Fc1Prob p{d, rp, h->on, h->tg, h->off[MQ_P_FC1_W], h->off[MQ_P_FC1_B], w.X1, w.XIN, RT};
      MQ_HIP(launch_gemm(p, (int)RT, 2 * mq::H, 1, s));
    }
    pt.begin(PH_GI);
    {
      GiProb p{w.X1, h->on, h->tg, h->off[MQ_P_RNN_W_IH], h->off[MQ_P_RNN_B_IH], w.GI, RT};
      MQ_HIP(launch_gemm(p, (int)RT, mq::G3, 2, s));
    }
    pt.begin(PH_GRUF);
    {
      hipError_t e = rw_fwd == 1 ? launch_gru_fwd<1>(d, h, L, w, s)
                   : rw_fwd == 2 ? launch_gru_fwd<2>(d, h, L, w, s)
                   : rw_fwd == 4 ? launch_gru_fwd<4>(d, h, L, w, s)
                                 : launch_gru_fwd<8>(d, h, L, w, s);
      MQ_HIP(e);
    }
    pt.begin(PH_FC2);
    {
      Fc2Prob p{w.Hs, h->on, h->tg, h->off[MQ_P_FC2_W], h->off[MQ_P_FC2_B], w.Q, RT, d.A};
      MQ_HIP(launch_gemm(p, (int)RT, d.A, 2, s));
    }
  }
  h->nblk_mix = (d.M + 3) / 4;
  if (c.mixer == MQ_MIXER_QMIX && !hyp_in_fwd) {
    pt.begin(PH_HYP);
    if (hyper_ws_ok(d.S, d.E, d.NH, d.M)) {
      plan.hyper = MQ_HYP_WS;
      // wave-specialised weight streaming (hyper_kernel.hpp)
      MQ_LDS(hyper_ws_kernel<0>, hyper_ws_lds_bytes(d.S));
      hipLaunchKernelGGL(hyper_ws_kernel<0>, dim3((d.M + HYR - 1) / HYR, 2), dim3(HYWS_THREADS),
                         hyper_ws_lds_bytes(d.S), s, d, rp, (const float*)h->on, (const float*)h->tg, L, w.HYP,
                         w.S0);
      MQ_HIP(hipGetLastError());
    } else if (hyper_ok(d.S, d.NH)) {
      plan.hyper = MQ_HYP_LDS;
      const size_t dyn = HyperGeom(d.S, d.NH).lds_bytes();
      MQ_LDS(hyper_kernel<0>, dyn);
      hipLaunchKernelGGL(hyper_kernel<0>, dim3((d.M + HYR - 1) / HYR, 2), dim3(256), dyn, s, d, rp,
                         (const float*)h->on, (const float*)h->tg, L, w.HYP, w.S0);
      MQ_HIP(hipGetLastError());
    } else {
      plan.hyper = MQ_HYP_GEMM;
      HypProb p{d, rp, L, h->on, h->tg, w.HYP, w.S0};
      MQ_HIP(launch_gemm(p, d.M, d.NH, 2, s));
    }
  }
  pt.begin(PH_MIX);
  {
    const bool fast = d.n <= 16 && d.E <= 64;   // mix_kernel serves the rest (n > 16 or A > 32)
    const bool stream = mix_stream_ok(d.n, d.A) && !h->mix_generic;
    plan.mix = fast && d.A <= 16 ? MQ_MIX_FAST16 : fast && d.A <= 32 ? MQ_MIX_FAST32 : stream ? MQ_MIX_STREAM
                                                                                             : MQ_MIX_GENERIC;
    if (fast && d.A <= 16)
      hipLaunchKernelGGL((mix_fast_kernel<16, 16>), dim3(h->nblk_mix), dim3(256), 0, s, d, rp, (const float*)h->on,
                         (const float*)h->tg, L, w, curmax);
    else if (fast && d.A <= 32)
      hipLaunchKernelGGL((mix_fast_kernel<32, 16>), dim3(h->nblk_mix), dim3(256), 0, s, d, rp, (const float*)h->on,
                         (const float*)h->tg, L, w, curmax);
    else if (stream)
      hipLaunchKernelGGL(mix_kernel<true>, dim3(h->nblk_mix), dim3(256), 0, s, d, rp, (const float*)h->on,
                         (const float*)h->tg, L, w, curmax);
    else
      hipLaunchKernelGGL(mix_kernel<false>, dim3(h->nblk_mix), dim3(256), 0, s, d, rp, (const float*)h->on,
                         (const float*)h->tg, L, w, curmax);
    MQ_HIP(hipGetLastError());
  }
  pt.begin(PH_GRUB);
  bool dwh_in_bwd = false;
  int dwh_mode = 0;   // where dW_hyper runs (mq_plan.dwh)
  // dW_hyper's m-slices (A/B at cfg2: 4 / 8 / 16 / 32 -> 238.5 / 235.1 / 236.3 / 237.4 us, round 1)
  const int dwh_ns = std::max(1, std::min({h->dwh_split, kRedZ, (d.M + 1) / 2}));
  plan.fused_bwd = fused_bwd ? 1 : 0;
  plan.rw_bwd = fused_bwd || tiles ? 0 : rw_bwd;
  if (tiles) {
    const int nblk = (d.R + TR_B - 1) / TR_B;
    h->nblk_bwd = nblk;
    h->nsplit_fc1 = nblk;
    const int64_t l1 = (int64_t)mq::H * d.I + mq::H;
    const float* P0 = h->on;
    // the two-role (chain / weight-gradient waves) BPTT, 512 threads
#define MQ_BWD_TILE(K) \
  hipLaunchKernelGGL(gru_bwd_split_kernel<K>, dim3(nblk), dim3(512), 0, s, d, rp, P0, L, w, h->len_rnn, l1);
    if (kq1 == 8) { MQ_BWD_TILE(8) }
    else if (kq1 == 20) { MQ_BWD_TILE(20) }
    else if (kq1 == 40) { MQ_BWD_TILE(40) }
    else if (kq1 == 72) { MQ_BWD_TILE(72) }
    else { MQ_BWD_TILE(80) }
#undef MQ_BWD_TILE
    MQ_HIP(hipGetLastError());
  } else if (fused_bwd) {
    // one row per workgroup: dW_hh / dW_ih / dX1 / dW1 on the chain's idle matrix cores (gru_bwd_fused.hpp)
    const bool many = device_cus(h) > 0 && d.R > h->num_cu;   // a second wave of rows leaves CUs idle
    h->nblk_bwd = d.R;
    h->nsplit_fc1 = h->nblk_bwd;
    const size_t dyn = ((size_t)2 * d.A * mq::H + d.A) * sizeof(float);
    // dW_hyper: appended to the BPTT's grid when its rows exceed the CUs (mode 1: the second wave of rows leaves
    // CUs idle), else beside pass 1 of the reduction (mode 0); MQ_PLAN dwh_in_bwd=0|1 forces one. (Round 6: its
    // tiles on the BPTT's chain waves in the kernel's tail, idle while the producers reduce the last chunk, made the
    // BPTT 14 us longer against the 8.6 us they took out of the reduction's launch: four waves per CU leave each
    // tile's load round trips exposed. Removed.)
    if (c.mixer == MQ_MIXER_QMIX) {
      const int tj = (d.NH + DWH_T - 1) / DWH_T, ts = (d.S + 1 + DWH_T - 1) / DWH_T;
      dwh_mode = h->dwh_in_bwd >= 0 ? (h->dwh_in_bwd ? 1 : 0) : many ? 1 : 0;
      if (dwh_mode != 0) {   // the reduction's dW_hyper blocks, same geometry (see dwh_fused below)
        w.dwh_tj = tj;
        w.dwh_ns = dwh_ns;
        w.dwh_n = tj * ts * dwh_ns;
        w.dwh_len = h->len_mix;
        h->nsplit_mix = dwh_ns;
      }
    }
    dwh_in_bwd = dwh_mode != 0;
    plan.dwh = dwh_mode;
    const float* P0 = (const float*)h->on;
    const int64_t l1 = (int64_t)mq::H * d.I + mq::H;
    // diagnostic (MQ_DIAG bwd_stamp=<file>): step stamps of the first 8 workgroups
    std::string bstamp_path;
    const bool bstamp = dwh_mode != 1 && env_item("MQ_DIAG", "bwd_stamp", &bstamp_path) && !bstamp_path.empty() &&
                        d.Tp <= BSTN - BSTH;
    if (dwh_mode == 1) MQ_LDS(gru_bwd_fused_kernel<1>, dyn);
    else MQ_LDS((gru_bwd_fused_kernel<0, true>), dyn);   // the larger of the two builds
    if (dwh_mode == 1) launch_bwd_fused_dwh(dyn, s, d, rp, P0, L, w, h->pitch_rnn, l1);
    else launch_bwd_fused(dim3(d.R), dyn, s, d, rp, P0, L, w, h->pitch_rnn, l1, bstamp);
    if (bstamp) {
      std::vector<uint32_t> st((size_t)8 * BSTN);
      MQ_HIP(hipMemcpyAsync(st.data(), w.GI, st.size() * 4, hipMemcpyDeviceToHost, s));
      MQ_HIP(hipStreamSynchronize(s));
      if (FILE* f = fopen(bstamp_path.c_str(), "ab")) { fwrite(st.data(), 4, st.size(), f); fclose(f); }
    }
    MQ_HIP(hipGetLastError());
  } else {
    {
      // RW >= 4 spills the 96 role registers + per-row prefetch sets at 512 threads; cap at 2
      const size_t dyn = ((size_t)2 * d.A * mq::H + d.A) * sizeof(float);
      if (rw_bwd == 1) MQ_LDS(gru_bwd_kernel<1>, dyn);
      else if (rw_bwd == 2) MQ_LDS(gru_bwd_kernel<2>, dyn);
      else MQ_LDS(gru_bwd_kernel<4>, dyn);
      hipError_t e = rw_bwd == 1 ? launch_gru_bwd<1>(d, rp, h, L, w, s, &h->nblk_bwd)
                   : rw_bwd == 2 ? launch_gru_bwd<2>(d, rp, h, L, w, s, &h->nblk_bwd)
                                 : launch_gru_bwd<4>(d, rp, h, L, w, s, &h->nblk_bwd);
      MQ_HIP(e);
    }
    pt.begin(PH_DX1);
    {
      Dx1Prob p{w.dGI, h->on + h->off[MQ_P_RNN_W_IH], w.X1, w.dP1, RT};
      MQ_HIP(launch_gemm(p, (int)RT, mq::H, 1, s));
    }
    pt.begin(PH_DW1);
    {
      const int tiles = (d.I + Dw1Prob::BN - 1) / Dw1Prob::BN;
      int ns = (int)std::min<int64_t>(kNsplitMax, std::max<int64_t>(1, RT / 256));
      ns = std::max(1, std::min(ns, (512 + tiles - 1) / tiles));
      // keep every split non-empty under krange_split's GBK rounding
      int64_t chunk = ((RT + ns - 1) / ns + GBK - 1) / GBK * GBK;
      ns = (int)((RT + chunk - 1) / chunk);
      h->nsplit_fc1 = ns;
      Dw1Prob p{d.I, w.dP1, w.XIN, w.slab_fc1, RT, ns};
      MQ_HIP(launch_gemm(p, mq::H, d.I, ns, s));
    }
  }
  // dW_hyper runs fused with pass 1 of the reduction (dwh_red1_kernel), unless its tiles rode in the BPTT's grid
  const bool dwh_fused = c.mixer == MQ_MIXER_QMIX && !dwh_in_bwd;
  {
    int tj = 0, ts = 0, ns = 0, ndwh = 0;
    if (dwh_fused) {
      tj = (d.NH + DWH_T - 1) / DWH_T;
      ts = (d.S + 1 + DWH_T - 1) / DWH_T;
      // pass 1 shares this launch with dW_hyper, so dW_hyper's slabs must go straight to pass 2: at most kRedZ
      ns = dwh_ns;
      h->nsplit_mix = ns;
      ndwh = tj * ts * ns;
    }
    RedBuilder rb(w.red_tmp);
    rb.add(w.slab_fc1, h->nsplit_fc1, (int64_t)mq::H * d.I + mq::H, h->grad + h->off[MQ_P_FC1_W], true);
    if (fused_bwd) {   // [W_ih | W_hh] in the BPTT's C-tile order (red_dst), then the biases and fc2
      const int64_t lm = 2LL * mq::G3 * mq::H;
      rb.add(w.slab_rnn, h->nblk_bwd, lm, h->grad + h->off[MQ_P_RNN_W_IH], true, h->pitch_rnn, false, 1);
      rb.add(w.slab_rnn + lm, h->nblk_bwd, h->len_rnn - lm, h->grad + h->off[MQ_P_RNN_W_IH] + lm, true, h->pitch_rnn);
    } else {
      rb.add(w.slab_rnn, h->nblk_bwd, h->len_rnn, h->grad + h->off[MQ_P_RNN_W_IH], true);
    }
    if (c.mixer == MQ_MIXER_QMIX) {
      // dW_hyper's few m-slice slabs go straight to pass 2 (they are written in the same launch as pass 1)
      const bool direct = rb.add(w.slab_mix, h->nsplit_mix, h->len_mix, h->grad + h->off[MQ_P_HW1_W], true, 0, true);
      if (dwh_fused && !direct)   // pass-1 blocks would read slabs the dW_hyper blocks of the same grid still write
        return set_err(MQ_ERR_STATE, "dW_hyper fused with reduction pass 1 needs a direct slab region");
      rb.add(w.slab_v2, h->nblk_mix, d.E + 1, h->grad + h->off[MQ_P_V2_W], true);
    }
    rb.add(w.loss_part, h->nblk_mix, MQ_NSUMS, h->grad + h->P, false);
    if (dwh_fused) {
      pt.begin(PH_DWH);
      const int ndwh_pad = (ndwh + 15) / 16 * 16;
      hipLaunchKernelGGL(dwh_red1_kernel<4>, dim3(ndwh_pad + rb.b1), dim3(256), 0, s, d, L, (const float*)w.dHYP,
                         (const float*)w.S0, w.slab_mix, h->len_mix, ns, tj, ndwh, ndwh_pad, rb.pl);
      MQ_HIP(hipGetLastError());
      pt.begin(PH_RED);
    } else {
      pt.begin(PH_RED);
      if (rb.b1 > 0) {
        hipLaunchKernelGGL(red_pass1_kernel, dim3(rb.b1), dim3(256), 0, s, rb.pl);
        MQ_HIP(hipGetLastError());
      }
    }
    hipLaunchKernelGGL(red_pass2_kernel, dim3(rb.b2), dim3(256), 0, s, rb.pl, w.norm_part);
    MQ_HIP(hipGetLastError());
    h->n_norm_part = rb.b2;
  }
  pt.end();
  if (h->comm) {   // native data parallelism: the whole [grads | sums] buffer, summed over the ranks in stream order
    const ncclResult_t r = ncclAllReduce(h->grad, h->grad, (size_t)(h->P + MQ_NSUMS), ncclFloat, ncclSum, h->comm, s);
    if (r != ncclSuccess) return set_err(MQ_ERR_HIP, std::string("ncclAllReduce: ") + ncclGetErrorString(r));
  }
  h->last = d;
  h->plan = plan;
  h->have_fb = true;
  return MQ_OK;
}

int mq_apply(mq_handle* h, void* stream) {
  if (!h || !h->on) return set_err(MQ_ERR_STATE, "mq_apply before mq_bind");
  if (!h->have_fb) return set_err(MQ_ERR_STATE, "mq_apply before mq_forward_backward");
  hipStream_t s = (hipStream_t)stream;
  PhaseTimer pt{h, s};
  pt.begin(PH_APPLY);
  if (h->dp || h->comm) {   // the gradient was all-reduced after the reduce pass: its norm partials are stale
    h->n_norm_part = 256;
    hipLaunchKernelGGL(sumsq_kernel, dim3(h->n_norm_part), dim3(256), 0, s, (const float*)h->grad, h->P,
                       h->w.norm_part);
    MQ_HIP(hipGetLastError());
  }
  OptHP hp{h->cfg.lr, h->cfg.optim_alpha, h->cfg.optim_eps, h->cfg.grad_norm_clip, h->cfg.n_agents};
  int blocks = (int)std::min<int64_t>((h->P + 255) / 256, 1024);
  hipLaunchKernelGGL(apply_kernel, dim3(blocks), dim3(256), 0, s, h->on, h->grad, h->sq, h->P,
                     (const float*)h->w.norm_part, h->n_norm_part, hp, h->stats, (const int*)nullptr);
  MQ_HIP(hipGetLastError());
  pt.end();
  ++h->tstep;
  return MQ_OK;
}

int mq_last_plan(const mq_handle* h, mq_plan* out) {
  if (!h || !out) return set_err(MQ_ERR_ARG, "NULL argument");
  if (!h->have_fb) return set_err(MQ_ERR_STATE, "no forward/backward has run");
  *out = h->plan;
  return MQ_OK;
}

int mq_set_data_parallel(mq_handle* h, int32_t on) {
  if (!h) return set_err(MQ_ERR_ARG, "NULL handle");
  h->dp = on != 0;
  return MQ_OK;
}

int mq_comm_unique_id(uint8_t* id) {
  if (!id) return set_err(MQ_ERR_ARG, "NULL id");
  ncclUniqueId u;
  const ncclResult_t r = ncclGetUniqueId(&u);
  if (r != ncclSuccess) return set_err(MQ_ERR_HIP, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
  static_assert(sizeof(u) == MQ_COMM_ID_BYTES, "ncclUniqueId size");
  std::memcpy(id, &u, sizeof(u));
  return MQ_OK;
}

// One RCCL communicator over `world` ranks (the calling process's current HIP device).
static int comm_init(ncclComm_t* out, const uint8_t* id, int32_t rank, int32_t world) {
  if (!id || world < 1 || rank < 0 || rank >= world) return set_err(MQ_ERR_ARG, "mq_comm_attach: bad id, rank or world");
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  const ncclResult_t r = ncclCommInitRank(out, world, u, rank);
  if (r != ncclSuccess) return set_err(MQ_ERR_HIP, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
  return MQ_OK;
}

int mq_comm_attach(mq_handle* h, const uint8_t* id, int32_t rank, int32_t world) {
  if (!h) return set_err(MQ_ERR_ARG, "NULL handle");
  if (h->comm) return set_err(MQ_ERR_STATE, "a communicator is already attached (mq_comm_detach first)");
  const int rc = comm_init(&h->comm, id, rank, world);
  if (rc) return rc;
  h->comm_world = world;
  h->comm_owned = true;
  return MQ_OK;
}

int mq_comm_create(const uint8_t* id, int32_t rank, int32_t world, void** comm) {
  if (!comm) return set_err(MQ_ERR_ARG, "NULL comm");
  ncclComm_t c = nullptr;
  const int rc = comm_init(&c, id, rank, world);
  if (rc) return rc;
  *comm = (void*)c;
  return MQ_OK;
}

int mq_comm_free(void* comm) {
  if (comm) (void)ncclCommDestroy((ncclComm_t)comm);
  return MQ_OK;
}

int mq_comm_use(mq_handle* h, void* comm) {
  if (!h || !comm) return set_err(MQ_ERR_ARG, "NULL handle or communicator");
  if (h->comm) return set_err(MQ_ERR_STATE, "a communicator is already attached (mq_comm_detach first)");
  int world = 0;
  const ncclResult_t r = ncclCommCount((ncclComm_t)comm, &world);
  if (r != ncclSuccess) return set_err(MQ_ERR_ARG, std::string("ncclCommCount: ") + ncclGetErrorString(r));
  h->comm = (ncclComm_t)comm;
  h->comm_world = world;
  h->comm_owned = false;
  return MQ_OK;
}

int32_t mq_comm_world(const mq_handle* h) { return h ? h->comm_world : 0; }

int mq_comm_detach(mq_handle* h) {
  if (!h) return set_err(MQ_ERR_ARG, "NULL handle");
  if (h->comm && h->comm_owned) (void)ncclCommDestroy(h->comm);
  h->comm = nullptr;
  h->comm_world = 0;
  h->comm_owned = false;
  return MQ_OK;
}

int mq_update_targets(mq_handle* h, void* stream) {
  if (!h || !h->on || !h->tg) return set_err(MQ_ERR_STATE, "mq_update_targets needs online and target bound");
  MQ_HIP(hipMemcpyAsync(h->tg, h->on, h->P * sizeof(float), hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return MQ_OK;
}

int mq_copy_intermediate(mq_handle* h, int which, float* dst, int64_t* count, void* stream) {
  if (!h || !h->have_fb) return set_err(MQ_ERR_STATE, "no forward/backward has run");
  const Dims& d = h->last;
  const int64_t RT = (int64_t)d.Tp * d.R;
  const float* src;
  int64_t cnt;
  switch (which) {
    case 0: src = h->w.Q; cnt = RT * d.A; break;
    case 1: src = h->w.Q + RT * d.A; cnt = RT * d.A; break;
    case 2: src = h->w.dch; cnt = (int64_t)d.T * d.R; break;
    case 3: src = h->w.X1; cnt = RT * mq::H; break;
    default: return set_err(MQ_ERR_ARG, "unknown intermediate id");
  }
  if (count) *count = cnt;
  if (dst) MQ_HIP(hipMemcpyAsync(dst, src, cnt * sizeof(float), hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return MQ_OK;
}

int mq_mac_forward(mq_handle* h, const mq_replay* batch, int32_t t, const float* h_in, float* h_out, float* q_out,
                   int32_t which, void* stream) {
  if (!h || !h->on) return set_err(MQ_ERR_STATE, "mq_mac_forward before mq_bind");
  if (which && !h->tg) return set_err(MQ_ERR_STATE, "target parameters not bound");
  if (!batch || !batch->obs || !batch->actions || !batch->filled || !h_in || !h_out || !q_out)
    return set_err(MQ_ERR_ARG, "NULL pointer in mq_mac_forward");
  if (t < 0 || t >= batch->t_stride) return set_err(MQ_ERR_ARG, "t outside the stored episode");
  if (batch->batch_size < 1) return set_err(MQ_ERR_ARG, "empty batch");
  mq_replay b = *batch;
  b.t_len = std::max(2, std::min(b.t_stride, 2));
  const Dims d = make_dims(h, &b);
  const Rep rp = make_rep(batch);
  const Lay L = make_lay(h);
  const size_t smem = (size_t)(((d.I + 3) & ~3) + mq::H * 3 + mq::G3 * 2) * sizeof(float);
  hipLaunchKernelGGL(mac_step_kernel, dim3(d.R), dim3(256), smem, (hipStream_t)stream, d, rp,
                     (const float*)(which ? h->tg : h->on), L, (int)t, (const float*)nullptr, h_in, h_out, q_out);
  MQ_HIP(hipGetLastError());
  return MQ_OK;
}

int mq_agent_forward(mq_handle* h, const float* inputs, int32_t rows, const float* h_in, float* h_out, float* q_out,
                     int32_t which, void* stream) {
  if (!h || !h->on) return set_err(MQ_ERR_STATE, "mq_agent_forward before mq_bind");
  if (which && !h->tg) return set_err(MQ_ERR_STATE, "target parameters not bound");
  if (!inputs || !h_in || !h_out || !q_out || rows < 0) return set_err(MQ_ERR_ARG, "bad mq_agent_forward args");
  if (rows == 0) return MQ_OK;
  mq_replay b;
  std::memset(&b, 0, sizeof(b));
  b.batch_size = 1; b.t_len = 2; b.t_stride = 2;
  Dims d = make_dims(h, &b);
  d.n = 1;   // rows are independent here: block -> row, agent id unused
  const Rep rp = make_rep(&b);
  const Lay L = make_lay(h);
  const size_t smem = (size_t)(((d.I + 3) & ~3) + mq::H * 3 + mq::G3 * 2) * sizeof(float);
  hipLaunchKernelGGL(mac_step_kernel, dim3(rows), dim3(256), smem, (hipStream_t)stream, d, rp,
                     (const float*)(which ? h->tg : h->on), L, 0, inputs, h_in, h_out, q_out);
  MQ_HIP(hipGetLastError());
  return MQ_OK;
}

int mq_greedy_actions(const float* q, const int32_t* avail, int64_t* out, int32_t rows, int32_t n_actions,
                      void* stream) {
  if (!q || !avail || !out || rows < 0 || n_actions < 1) return set_err(MQ_ERR_ARG, "bad mq_greedy_actions args");
  if (rows == 0) return MQ_OK;
  hipLaunchKernelGGL(greedy_kernel, dim3((rows + 255) / 256), dim3(256), 0, (hipStream_t)stream, q, avail, out,
                     (int)rows, (int)n_actions);
  MQ_HIP(hipGetLastError());
  return MQ_OK;
}

int mq_qmix_forward(const float* mixer, int32_t n_agents, int32_t state_dim, int32_t embed_dim,
                    const float* agent_qs, const float* states, float* q_tot, int32_t rows, void* stream) {
  if (!mixer || !agent_qs || !states || !q_tot || rows < 0) return set_err(MQ_ERR_ARG, "bad mq_qmix_forward args");
  if (n_agents < 1 || n_agents > 64 || embed_dim < 1 || embed_dim > 64 || state_dim < 1)
    return set_err(MQ_ERR_ARG, "mq_qmix_forward: n_agents / embed_dim in [1, 64], state_dim >= 1");
  if (rows == 0) return MQ_OK;
  const size_t lds = qmix_forward_lds(n_agents, state_dim, embed_dim);
  if (lds > 160 * 1024) return set_err(MQ_ERR_ARG, "mq_qmix_forward: state_dim too large for the LDS staging");
  hipLaunchKernelGGL(qmix_forward_kernel, dim3((rows + QMF_ROWS - 1) / QMF_ROWS), dim3(256), lds,
                     (hipStream_t)stream, mixer, (int)n_agents, (int)state_dim, (int)embed_dim, agent_qs, states,
                     q_tot, (int)rows);
  MQ_HIP(hipGetLastError());
  return MQ_OK;
}

int mq_set_timing(mq_handle* h, int32_t slots, uint32_t phase_mask) {
  if (!h || slots < 0 || slots > 4096) return set_err(MQ_ERR_ARG, "bad mq_set_timing args");
  for (auto e : h->ev0) (void)hipEventDestroy(e);
  for (auto e : h->ev1) (void)hipEventDestroy(e);
  h->ev0.clear(); h->ev1.clear(); h->ev_used.clear();
  h->slots = slots;
  h->mask = phase_mask;
  h->tstep = 0;
  const size_t n = (size_t)slots * PH_N;
  h->ev0.resize(n); h->ev1.resize(n); h->ev_used.assign(n, 0);
  for (size_t i = 0; i < n; ++i) {
    MQ_HIP(hipEventCreate(&h->ev0[i]));
    MQ_HIP(hipEventCreate(&h->ev1[i]));
  }
  return MQ_OK;
}

int mq_phase_times(mq_handle* h, float* ms, int32_t cap, int32_t* n) {
  if (!h || !ms) return set_err(MQ_ERR_ARG, "NULL argument");
  if (n) *n = PH_N;
  for (int p = 0; p < PH_N && p < cap; ++p) {
    double sum = 0.0;
    int cnt = 0;
    for (int sl = 0; sl < h->slots; ++sl) {
      const size_t i = (size_t)sl * PH_N + p;
      if (!h->ev_used[i]) continue;
      float t = 0.0f;
      MQ_HIP(hipEventSynchronize(h->ev1[i]));
      MQ_HIP(hipEventElapsedTime(&t, h->ev0[i], h->ev1[i]));
      sum += t;
      ++cnt;
    }
    ms[p] = cnt ? (float)(sum / cnt) : 0.0f;
  }
  return MQ_OK;
}

}  // extern "C"
#include "coma_host.hpp"
