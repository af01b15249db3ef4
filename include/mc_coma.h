/* C ABI of the MI355X-native COMA learner step (libmq_learner.so, gfx950) — SURVEY.md §8f row f1.
 *
 * The drop-in boundary behind pymarl's learners.REGISTRY["coma_learner"]: the host shim
 * pymarl_amd/learners/coma_learner.py binds these symbols with ctypes. Conventions as include/mq_learner.h:
 * DEVICE pointers owned by the caller, asynchronous on the given HIP stream, int status + mq_last_error().
 *
 * Reference interfaces replaced (nicholasburden/pymarl, /root/reference):
 *   mc_train_step      COMALearner.train(batch, t_env, episode_num) minus the target-update decision
 *                      src/learners/coma_learner.py:32-98, with _train_critic :100-148, COMACritic
 *                      src/modules/critics/coma.py:22-58, build_td_lambda_targets src/utils/rl_utils.py:4-14 and
 *                      BasicMAC.forward's pi_logits branch src/controllers/basic_controller.py:53-73
 *   mc_update_targets  COMALearner._update_targets                       src/learners/coma_learner.py:150-152
 *   mc_policy          BasicMAC.forward pi_logits post-processing        src/controllers/basic_controller.py:53-73
 *   mc_critic_forward  COMACritic.forward(batch, t=None)                 src/modules/critics/coma.py:22-58
 *   mc_copy_intermediate  (test hook) the critic's per-step Q values, the TD(lambda) targets, the policy
 *   mc_set_data_parallel  no reference counterpart: data-parallel COMA ("COMA caveat")
 */
#ifndef MC_COMA_H
#define MC_COMA_H

#include "mq_learner.h"

#ifdef __cplusplus
extern "C" {
#endif

enum { MC_CRITIC_HIDDEN = 128 };   /* coma.py:17-19 */
/* Critic parameter tensors in COMACritic.parameters() order (coma.py:17-19). */
enum { MC_P_FC1_W, MC_P_FC1_B, MC_P_FC2_W, MC_P_FC2_B, MC_P_FC3_W, MC_P_FC3_B, MC_P_COUNT };
enum { MC_NTAIL = 8 };    /* tail of the critic gradient buffer (sum of the mask of the pending step ...) */
/* stats[MC_NSTATS]: critic_loss, critic_grad_norm, td_error_abs, q_taken_mean, target_mean (means over the
 * logged critic steps, coma_learner.py:85-88), advantage_mean, coma_loss, agent_grad_norm, pi_max (:90-93),
 * critic training steps taken, agent mask sum; [11..15] scratch. */
enum { MC_NSTATS = 16 };

typedef struct mc_config {
  int32_t n_agents, n_actions, obs_dim, state_dim;
  int32_t rnn_hidden_dim;          /* 64 */
  int32_t obs_last_action, obs_agent_id;
  int32_t mask_before_softmax;     /* basic_controller.py:56 (getattr default True; coma_smac.yaml: False) */
  float gamma, td_lambda, lr, critic_lr, optim_alpha, optim_eps, grad_norm_clip;
  int32_t max_batch, max_seq;
} mc_config;

typedef struct mc_handle mc_handle;

int mc_create(const mc_config* cfg, mc_handle** out);
int mc_destroy(mc_handle* h);
/* agent_offsets[MQ_P_COUNT + 1] (RNNAgent layout, mixer entries empty), critic_offsets[MC_P_COUNT + 1]. */
int mc_param_offsets(const mc_handle* h, int64_t* agent_offsets, int64_t* critic_offsets);
/* agent / agent_sq: [Pa]; agent_grad: [Pa + MQ_NSUMS]; critic / target_critic / critic_sq: [Pc];
 * critic_grad: [Pc + MC_NTAIL]; stats: [MC_NSTATS]. Clipped gradients of the agent step and of the last critic
 * step are left in the grad buffers, as .grad holds them after the reference's train(). */
int mc_bind(mc_handle* h, float* agent, float* agent_grad, float* agent_sq, float* critic, float* target_critic,
            float* critic_grad, float* critic_sq, float* stats);
/* One COMALearner.train on `batch` (t_len = max_t_filled): T = t_len - 1 critic RMSprop steps in reversed t, the
 * policy-gradient agent step, stats. epsilon = the MAC's action_selector.epsilon (the reference reads it through
 * BasicMAC.forward, basic_controller.py:64-67). The caller reads stats[9] (critic steps) for the target update. */
int mc_train_step(mc_handle* h, const mq_replay* batch, float epsilon, void* stream);
int mc_update_targets(mc_handle* h, void* stream);
/* BasicMAC.forward's pi_logits branch on logits [rows][n_actions] in place: optional -1e10 mask, softmax, and
 * unless test_mode the epsilon floor (+ zeroing when mask_before_softmax). avail [rows][n_actions] int32. */
int mc_policy(float* logits, const int32_t* avail, int32_t rows, int32_t n_actions, float epsilon,
              int32_t mask_before_softmax, int32_t test_mode, void* stream);
/* COMACritic.forward(batch, t) outside train(): critic = fc1.weight .. fc3.bias (MC_P_* order); t < 0 means
 * every stored step of the batch (t=None), else the single step t. q_out [batch_size][Tq][n_agents][n_actions],
 * Tq = t_len or 1; workspace: mc_critic_forward_workspace(cfg, batch_size, Tq) floats of device memory. */
int64_t mc_critic_forward_workspace(const mc_config* cfg, int32_t batch_size, int32_t t_count);
int mc_critic_forward(const float* critic, const mc_config* cfg, const mq_replay* batch, int32_t t, float* q_out,
                      float* workspace, void* stream);
/* Optional HIP-event timing of train steps (bench / profiling): on != 0 records events around the critic's
 * target pass + TD(lambda), the T-step critic chain, and the actor part of every following mc_train_step;
 * mc_phase_times writes the last step's [prologue, critic chain, actor] ms (synchronises on the events). */
int mc_set_timing(mc_handle* h, int32_t on);
int mc_phase_times(mc_handle* h, float* ms /* [3] */);
/* How the last mc_train_step ran the critic's T steps: 1 = the persistent critic chain (one launch; the
 * default where the shape fits: B * n_agents <= 80, n_actions <= 32, not data-parallel; MQ_COMA_CHAIN=0 at
 * mc_create turns it off), 0 = three launches per step, -1 = no train step yet. */
int32_t mc_last_critic_path(const mc_handle* h);
/* Data-parallel COMA: each rank passes its contiguous shard of the same global sample to
 * mc_train_step; the library calls `allreduce` at every exchange step, in stream order on `stream`:
 *   once       the per-step mask sums (T floats, through `scratch`), so every rank skips the same steps
 *              (coma_learner.py:121-122) and normalises by the global sum(mask);
 *   per live critic step  the unnormalised critic gradient [Pc] (then its norm is recomputed from the sum);
 *   once       the per-step critic stat sums (8*T floats, through `scratch`; rank != 0 contributes zeros for the
 *              replicated fields);
 *   once       the agent gradient + sums [Pa + MQ_NSUMS] (then its norm is recomputed).
 * `allreduce(buf, count, stream, ctx)` sums `count` floats at the device pointer `buf` over the ranks in place and
 * returns 0 on success; `buf` is always critic_grad, agent_grad or `scratch` (all caller-owned). In this mode the
 * host reads the global mask sums back once per train (one synchronisation) to know the live steps.
 * `scratch` holds >= 8 * max_seq floats. allreduce = NULL switches data parallelism off. */
typedef int (*mc_allreduce_fn)(float* buf, int64_t count, void* stream, void* ctx);
/* The same exchange steps over a native RCCL communicator (id from mq_comm_unique_id, one process per GPU): no
 * host callback per critic step. Replaces any mc_set_data_parallel callback; scratch is library-owned. */
int mc_comm_attach(mc_handle* h, const uint8_t* id, int32_t rank, int32_t world);
/* The same over a communicator the caller owns (see mq_comm_use): borrowed, never freed by the handle. */
int mc_comm_use(mc_handle* h, void* nccl_comm);
/* Drop the attached communicator (freed only if mc_comm_attach created it) and, if it carried the exchange steps,
 * switch data parallelism off. A host that frees a communicator it lent with mc_comm_use detaches first. */
int mc_comm_detach(mc_handle* h);
int mc_set_data_parallel(mc_handle* h, mc_allreduce_fn allreduce, void* ctx, int32_t rank, float* scratch,
                         int64_t scratch_count);
/* Replicated-critic data parallelism, for batches whose critic fits the persistent chain (B * n_agents <= 80, as
 * coma_smac's B = 8 at MMM2's 10 agents): every rank passes the WHOLE sampled batch to mc_train_step and runs the
 * critic's T steps on it (identical on every rank: no per-step exchange, coma_learner.py:118-139 unchanged), and
 * the actor (coma_learner.py:52-83) on episodes [lo, hi) only; the agent gradient + sums are then summed with ONE
 * all-reduce (the mc_set_data_parallel callback or mc_comm_attach communicator, which must be set). hi <= lo turns
 * it off (then an all-reduce set means the exchange mode above, on per-rank shards). */
int mc_set_actor_shard(mc_handle* h, int32_t lo, int32_t hi);
/* 0 = critic Q values the actor used [T][B*n][A]; 1 = TD(lambda) targets [T][B*n]; 2 = policy pi [T][rows][A]
 * (rows = the actor's: its shard under mc_set_actor_shard). */
int mc_copy_intermediate(mc_handle* h, int which, float* dst, int64_t* count, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MC_COMA_H */
