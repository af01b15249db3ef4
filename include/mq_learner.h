/* C ABI of the MI355X-native QMIX/VDN learner hot path (libmq_learner.so, gfx950).
 *
 * This is the drop-in boundary behind pymarl's learner plugin API: the host shim
 * pymarl_amd/learners/q_learner.py (registered as learners.REGISTRY["q_learner"]) binds these symbols with
 * ctypes. Every pointer passed in is a DEVICE pointer owned by the caller (borrowed for the call or, for
 * mq_bind, until the next mq_bind / mq_destroy); the handle owns only its activation workspace. All calls
 * are asynchronous on the given HIP stream (passed as void*; NULL = the null stream) unless stated otherwise.
 * Every function returns MQ_OK (0) or an error code; mq_last_error() gives the text. No C++ exception crosses
 * this boundary.
 *
 * Reference interfaces replaced (nicholasburden/pymarl, /root/reference):
 *   mq_train_step        QLearner.train(batch, t_env, episode_num)      src/learners/q_learner.py:37-116
 *   mq_forward_backward  q_learner.py:39-101 (loss + backward, before clip/step)
 *   mq_apply             q_learner.py:102-103 (clip_grad_norm_ + RMSprop.step) and the stats of :109-116
 *   mq_update_targets    QLearner._update_targets                       src/learners/q_learner.py:118-122
 *   mq_mac_forward       BasicMAC.forward(ep_batch, t)                   src/controllers/basic_controller.py:40-75
 *   mq_agent_forward     RNNAgent.forward(inputs, hidden_state)          src/modules/agents/rnn_agent.py:27-36
 *   mq_greedy_actions    EpsilonGreedyActionSelector greedy branch      src/components/action_selectors.py:44-62
 *   mq_qmix_forward      QMixer.forward(agent_qs, states)                src/modules/mixers/qmix.py:28-47
 *   mq_replay.ep_ids     ReplayBuffer.sample -> EpisodeBatch.__getitem__ gather, episode_buffer.py:165-217,291-298
 *                        (ids drawn on the host exactly as the reference does; the gather is fused into kernels)
 */
#ifndef MQ_LEARNER_H
#define MQ_LEARNER_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { MQ_MIXER_NONE = 0, MQ_MIXER_VDN = 1, MQ_MIXER_QMIX = 2 };
enum { MQ_OK = 0, MQ_ERR_ARG = 1, MQ_ERR_HIP = 2, MQ_ERR_STATE = 3 };
enum { MQ_NSUMS = 8 };   /* tail of the gradient buffer: sum (td*m)^2 (Huber: sum huber(td*m)), sum m, sum |td*m|, sum Q_tot*m, sum y*m */
enum { MQ_NSTATS = 8 };  /* loss, grad_norm, td_error_abs, q_taken_mean, target_mean, mask_sum, clip coefficient,
                           0 (reserved) */

/* Parameter tensors, in the reference's parameters()/state_dict order: RNNAgent (rnn_agent.py:19-21) then
 * QMixer (qmix.py:14-23). mq_param_offsets fills offsets[MQ_P_COUNT + 1] (last = total). */
enum {
  MQ_P_FC1_W, MQ_P_FC1_B, MQ_P_RNN_W_IH, MQ_P_RNN_W_HH, MQ_P_RNN_B_IH, MQ_P_RNN_B_HH, MQ_P_FC2_W, MQ_P_FC2_B,
  MQ_P_HW1_W, MQ_P_HW1_B, MQ_P_HWF_W, MQ_P_HWF_B, MQ_P_HB1_W, MQ_P_HB1_B, MQ_P_V0_W, MQ_P_V0_B, MQ_P_V2_W,
  MQ_P_V2_B, MQ_P_COUNT
};

typedef struct mq_config {
  int32_t n_agents, n_actions, obs_dim, state_dim;
  int32_t rnn_hidden_dim;    /* 64 (the reference default; the kernels are built for it) */
  int32_t mixing_embed_dim;  /* QMIX embed dim, <= 64 */
  int32_t mixer;             /* MQ_MIXER_*; unknown -> MQ_ERR_ARG (reference: ValueError, q_learner.py:26) */
  int32_t double_q, obs_last_action, obs_agent_id;
  float gamma, lr, optim_alpha, optim_eps, grad_norm_clip;
  int32_t max_batch;         /* most episodes one call may train on (workspace bound) */
  int32_t max_seq;           /* most stored steps per episode (episode_limit + 1) */
  float huber_delta;         /* TD loss: 0 = masked L2 (q_learner.py:96-97, default); > 0 = masked Huber with this
                                delta, an opt-in the reference lacks (not pinned by its goldens) */
} mq_config;

/* A batch of episodes as the learner reads it: the replay storage (reference scheme dtypes, episode-major
 * [episode][t][...], run.py:122-135) plus the sampled episode ids. t_len = max_t_filled() of the batch
 * (run.py:211-212), t_stride = the storage's max_seq_length. */
typedef struct mq_replay {
  const float* obs;            /* [N][t_stride][n_agents][obs_dim] */
  const float* state;          /* [N][t_stride][state_dim] */
  const int64_t* actions;      /* [N][t_stride][n_agents][1] */
  const int32_t* avail_actions;/* [N][t_stride][n_agents][n_actions] */
  const float* reward;         /* [N][t_stride][1] */
  const uint8_t* terminated;   /* [N][t_stride][1] */
  const int64_t* filled;       /* [N][t_stride][1] */
  const int64_t* ep_ids;       /* [batch_size] episode ids (device); NULL = 0..batch_size-1 */
  int64_t n_episodes;
  int32_t batch_size, t_len, t_stride;
  /* Optional HOST copy of the ids, read during the call: when set and batch_size <= MQ_INLINE_IDS the ids travel
   * in the kernel arguments and ep_ids is not read (no host-to-device copy per step). */
  const int64_t* ep_ids_host;
  /* Optional [N][t_stride][n_agents] bitmask view of avail_actions (bit a set iff avail_actions[..][a] != 0), kept
   * by the replay buffer as episodes are inserted. When set, the mixer's double-Q selection reads these 8 bytes per
   * agent row instead of 4 n_actions (configs[2], 27m: 82 of the mixer's 262 MB); NULL reads avail_actions. */
  const uint64_t* avail_bits;
} mq_replay;

#define MQ_INLINE_IDS 256

typedef struct mq_handle mq_handle;

const char* mq_last_error(void);
int mq_create(const mq_config* cfg, mq_handle** out);
int mq_destroy(mq_handle* h);
int mq_param_offsets(const mq_handle* h, int64_t* offsets /* [MQ_P_COUNT + 1] */);

/* online/target/sq_avg: [P] floats (only `online` is required for an inference-only handle); grad: [P + MQ_NSUMS] floats (clipped grads land here after mq_apply,
 * as .grad does after clip_grad_norm_); stats: [MQ_NSTATS] floats; cur_max: optional [max_seq*max_batch*n]
 * int32 double-Q greedy actions of the last step ([t][b][agent], t < t_len-1), may be NULL. */
int mq_bind(mq_handle* h, float* online, float* target, float* grad, float* sq_avg, float* stats,
            int32_t* cur_max);

/* Loss + backward of QLearner.train on `batch`: writes UNNORMALISED gradients d(sum (td*m)^2)/dtheta and the
 * MQ_NSUMS partial sums into grad. Data-parallel callers all-reduce grad (whole buffer) between the two calls. */
int mq_forward_backward(mq_handle* h, const mq_replay* batch, void* stream);
/* Normalise by sum(m), clip_grad_norm_(grad_norm_clip), RMSprop(lr, alpha, eps) step, write stats. */
int mq_apply(mq_handle* h, void* stream);
/* mq_forward_backward + mq_apply in one call (with a communicator attached, the all-reduce between them too). */
int mq_train_step(mq_handle* h, const mq_replay* batch, void* stream);
/* Declare that the caller sums the gradient buffer across ranks between mq_forward_backward and mq_apply
 * (mq_apply then recomputes the global gradient norm from the reduced buffer). */
int mq_set_data_parallel(mq_handle* h, int32_t on);
/* Native RCCL data parallelism (SURVEY.md §8b's mq_allreduce_attach): rank 0 calls mq_comm_unique_id and ships
 * the MQ_COMM_ID_BYTES bytes to every rank over any channel; every rank (one process per GPU) then calls
 * mq_comm_attach(h, id, rank, world) once. From then on mq_forward_backward ends with one RCCL all-reduce (sum) of
 * the whole grad buffer [P + MQ_NSUMS] on `stream`, and mq_apply recomputes the norm from the sum: one call of
 * mq_train_step is a full data-parallel QLearner.train step, with no host collective in between. world = 1 is
 * allowed (the all-reduce is the identity). mq_comm_world reports the attached world size (0: none);
 * mq_comm_detach frees the communicator (mq_destroy does too). */
enum { MQ_COMM_ID_BYTES = 128 };
int mq_comm_unique_id(uint8_t* id /* [MQ_COMM_ID_BYTES] */);
int mq_comm_attach(mq_handle* h, const uint8_t* id, int32_t rank, int32_t world);
int32_t mq_comm_world(const mq_handle* h);
int mq_comm_detach(mq_handle* h);
/* SURVEY.md §8b's mq_allreduce_attach(handle, ncclComm_t): attach a communicator the CALLER owns (an ncclComm_t,
 * passed as void* so this header needs no RCCL include). The handle borrows it: detach / destroy leave it alive,
 * and one communicator may serve several handles (QMIX and COMA learners of one process). mq_comm_create /
 * mq_comm_free make and release one from a unique id for hosts without their own RCCL setup. */
int mq_comm_use(mq_handle* h, void* nccl_comm);
int mq_comm_create(const uint8_t* id, int32_t rank, int32_t world, void** nccl_comm);
int mq_comm_free(void* nccl_comm);
int mq_update_targets(mq_handle* h, void* stream);

/* Copy an intermediate of the last mq_forward_backward into dst (device): 0 = online mac_out [t][b*n+a][A],
 * 1 = target mac_out (same layout), 2 = dQ/dchosen [t][b*n+a] (unnormalised), 3 = online relu(fc1) activations
 * [t][b*n+a][64]. Returns element count in *count. */
int mq_copy_intermediate(mq_handle* h, int which, float* dst, int64_t* count, void* stream);

/* BasicMAC.forward(ep_batch, t) for every episode of `batch`: h_in/h_out [batch*n][64] (h_in may equal
 * h_out), q_out [batch*n][n_actions]; which = 0 online params, 1 target params. */
int mq_mac_forward(mq_handle* h, const mq_replay* batch, int32_t t, const float* h_in, float* h_out,
                   float* q_out, int32_t which, void* stream);
/* RNNAgent.forward(inputs, hidden) (rnn_agent.py:27-36) on given inputs [rows][input_dim]. */
int mq_agent_forward(mq_handle* h, const float* inputs, int32_t rows, const float* h_in, float* h_out,
                     float* q_out, int32_t which, void* stream);
/* argmax over available actions (unavailable = -inf, first index on ties) of q [rows][n_actions]. */
int mq_greedy_actions(const float* q, const int32_t* avail, int64_t* out, int32_t rows, int32_t n_actions,
                      void* stream);

/* QMixer.forward(agent_qs, states) outside train(): mixer = the mixer's parameters in QMixer.parameters() order
 * (hyper_w_1.weight .. V.2.bias, the MQ_P_HW1_W .. MQ_P_V2_B block), agent_qs [rows][n_agents], states
 * [rows][state_dim], q_tot [rows]. */
int mq_qmix_forward(const float* mixer, int32_t n_agents, int32_t state_dim, int32_t embed_dim,
                    const float* agent_qs, const float* states, float* q_tot, int32_t rows, void* stream);

/* Which kernel variants the last mq_forward_backward launched (test / profiling introspection; no device sync).
 * rw_fwd / rw_bwd: rows per workgroup of the unfused recurrences (0 when the fused kernel ran). */
enum { MQ_HYP_NONE = 0, MQ_HYP_WS = 1, MQ_HYP_LDS = 2, MQ_HYP_GEMM = 3 };
enum { MQ_MIX_FAST16 = 0, MQ_MIX_FAST32 = 1, MQ_MIX_GENERIC = 2, MQ_MIX_STREAM = 3 };
typedef struct mq_plan {
  int32_t rows;          /* R = batch_size * n_agents */
  int32_t fused_fwd;     /* gru_fwd_fused_kernel (1), gru_fwd_pair_kernel (2) or fc1 / gi / gru_fwd<rw_fwd> / fc2 (0) */
  int32_t rw_fwd;
  int32_t fused_bwd;     /* gru_bwd_fused_kernel (1) or gru_bwd<rw_bwd> / dx1 / dw1 (0) */
  int32_t rw_bwd;
  int32_t inline_ids;    /* episode ids in the kernel arguments (1) or read from mq_replay.ep_ids (0) */
  int32_t hyper;         /* MQ_HYP_* */
  int32_t mix;           /* MQ_MIX_* */
  int32_t tiles;         /* 1: the row-tile MFMA forward / BPTT of large batches (gru_fwd_tile / gru_bwd_tile);
                            fused_fwd / fused_bwd / rw_* are then 0 */
  int32_t dwh;           /* QMIX dW_hyper: beside reduction pass 1 (0) or appended to the fused BPTT's grid (1) */
} mq_plan;
int mq_last_plan(const mq_handle* h, mq_plan* out);

/* Optional per-kernel HIP-event timing of train steps (bench / profiling): events bracket every phase whose bit
 * is set in phase_mask (bit i = phase i of mq_phase_names), in a ring of `slots` steps; slots = 0 turns it off. */
int mq_set_timing(mq_handle* h, int32_t slots, uint32_t phase_mask);
/* Mean ms per phase over the recorded steps (synchronises on the events); *n = number of phases. */
int mq_phase_times(mq_handle* h, float* ms, int32_t cap, int32_t* n);
const char* mq_phase_names(void);

#ifdef __cplusplus
}
#endif
#endif /* MQ_LEARNER_H */
