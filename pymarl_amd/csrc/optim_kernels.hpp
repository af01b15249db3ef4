// Gradient slab reduction, clip_grad_norm_ and RMSprop over the flat parameter vector (q_learner.py:100-103),
// plus the single-step agent forward and greedy selection used on the rollout side
// (basic_controller.py:40-75, action_selectors.py:44-62).
#pragma once
#include "learner_types.hpp"

namespace mq {

// Deterministic two-pass reduction of every gradient slab of a train step in two launches (a launch costs
// ~4.5 us on this path whatever its size, so one launch per region was the bigger cost):
//   pass 1: block (region, z-group, chunk) sums zc consecutive slabs of its 256 elements -> tmp[group][len]
//           (zc chosen so there are at most 16 groups)
//   pass 2: block (region, chunk) sums the groups in order -> dst, and writes its partial sum of squares of the
//           gradient elements (regions with sq = 1) for clip_grad_norm_ -> norm_part[block]
// Fixed summation order throughout: bitwise reproducible. A region of at most 16 slabs is "direct": it has no
// pass-1 blocks and pass 2 sums its slabs in slab order (what pass 1 would have copied, group by group).
constexpr int kRedZ = 16;
constexpr int kRedMaxRegions = 6;
struct RedRegion {
  const float* src;
  float* dst;
  float* tmp;
  int64_t len;
  int64_t pitch;    // slab stride in src (>= len: a region may cover a prefix of each slab)
  int64_t tpitch;   // group stride in tmp (len; pitch for a direct region, whose pass 2 reads the slabs themselves)
  int nslab, zc, ng, sq;
  int vec;          // pass 1 in float4 (len, pitch multiples of 4; src and tmp 16-byte aligned)
  int xcd;          // pass 1 groups slabs by XCD (ng = 16, nslab % 128 == 0, blk1 % 16 == 0): group g holds slabs
                    // r == g (mod 8), summed by blocks with blockIdx == g (mod 8), i.e. on the XCD whose L2 holds
                    // them when slab r was written by workgroup r (the per-row BPTT slabs)
  int blk1, blk2;   // first block of this region in pass 1 / pass 2
  int perm;         // 1: the slabs hold [W_ih | W_hh] ([2][G3][H]) in the fused BPTT's MFMA C-tile order (red_dst)
};
struct RedPlan {
  RedRegion r[kRedMaxRegions];
  int nr;
};

MQ_DEV int red_region(const RedPlan& pl, int b, bool pass2) {
  int k = 0;
#pragma unroll
  for (int j = 1; j < kRedMaxRegions; ++j)
    if (j < pl.nr && b >= (pass2 ? pl.r[j].blk2 : pl.r[j].blk1)) k = j;
  return k;
}

MQ_DEV void red_pass1_body(const RedPlan& pl, int blk) {
  const int k = red_region(pl, blk, false);
  const RedRegion& R = pl.r[k];
  if (R.vec) {   // 1024 elements per block, one float4 per thread and slab
    const int nb = (int)((R.len + 1023) / 1024), lb = blk - R.blk1;
    const int g = R.xcd ? lb % R.ng : lb / nb, chunk = R.xcd ? lb / R.ng : lb - g * nb;
    const int64_t i = (int64_t)chunk * 1024 + 4 * threadIdx.x;
    if (i >= R.len) return;
    const int z0 = g * R.zc, z1 = min(R.nslab, z0 + R.zc);
    // slab of group member z: z itself, or (XCD grouping) the (z - z0)-th slab r == g (mod 8) of sub-group g / 8
    auto slab = [&](int z) { return R.xcd ? 8 * ((g >> 3) * R.zc + (z - z0)) + (g & 7) : z; };
    f32x4 v[kRedZ];
    f32x4 s = {0.0f, 0.0f, 0.0f, 0.0f};
    for (int zb = z0; zb < z1; zb += kRedZ) {
#pragma unroll
      for (int u = 0; u < kRedZ; ++u)
        v[u] = (zb + u < z1) ? *(const f32x4*)(R.src + (int64_t)slab(zb + u) * R.pitch + i)
                             : f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int u = 0; u < kRedZ; ++u) s += v[u];   // per component: the scalar path's order
    }
    *(f32x4*)(R.tmp + (int64_t)g * R.len + i) = s;
    return;
  }
  const int nb = (int)((R.len + 255) / 256), lb = blk - R.blk1;
  const int g = R.xcd ? lb % R.ng : lb / nb, chunk = R.xcd ? lb / R.ng : lb - g * nb;
  const int64_t i = (int64_t)chunk * 256 + threadIdx.x;
  if (i >= R.len) return;
  const int z0 = g * R.zc, z1 = min(R.nslab, z0 + R.zc);
  auto slab = [&](int z) { return R.xcd ? 8 * ((g >> 3) * R.zc + (z - z0)) + (g & 7) : z; };
  float v[kRedZ];
  float s = 0.0f;
  for (int zb = z0; zb < z1; zb += kRedZ) {
#pragma unroll
    for (int u = 0; u < kRedZ; ++u) v[u] = (zb + u < z1) ? R.src[(int64_t)slab(zb + u) * R.pitch + i] : 0.0f;
#pragma unroll
    for (int u = 0; u < kRedZ; ++u) s += v[u];
  }
  R.tmp[(int64_t)g * R.len + i] = s;
}

__global__ __launch_bounds__(256) void red_pass1_kernel(RedPlan pl) { red_pass1_body(pl, blockIdx.x); }

// Destination of region element i. perm = 1 (the fused BPTT's [W_ih | W_hh] slabs, gru_bwd_fused.hpp): the slab stores
// each wave's accumulators as they sit in its registers, one 16-byte store per lane and tile, so element
// p = ((mt * 4 + jj) * 64 + lane) * 4 + e of matrix z holds W[16 mt + 4 (lane >> 4) + e][16 jj + (lane & 15)].
MQ_DEV int64_t red_dst(const RedRegion& R, int64_t i) {
  if (!R.perm) return i;
  const int z = (int)(i / (G3 * H)), p = (int)(i - (int64_t)z * (G3 * H));
  const int e = p & 3, lane = (p >> 2) & 63, rest = p >> 8, jj = rest & 3, mt = rest >> 2;
  return (int64_t)z * (G3 * H) + (16 * mt + 4 * (lane >> 4) + e) * H + 16 * jj + (lane & 15);
}

__global__ __launch_bounds__(256) void red_pass2_kernel(RedPlan pl, float* __restrict__ norm_part) {
  const int k = red_region(pl, blockIdx.x, true);
  const RedRegion& R = pl.r[k];
  const int64_t i = (int64_t)(blockIdx.x - R.blk2) * 256 + threadIdx.x;
  float sq = 0.0f;
  if (i < R.len) {
    float u[kRedZ];
#pragma unroll
    for (int g = 0; g < kRedZ; ++g) u[g] = g < R.ng ? R.tmp[(int64_t)g * R.tpitch + i] : 0.0f;
    float v = 0.0f;
#pragma unroll
    for (int g = 0; g < kRedZ; ++g) v += u[g];
    R.dst[red_dst(R, i)] = v;
    if (R.sq) sq = v * v;
  }
  __shared__ float red[4];
  sq = wave_sum(sq);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sq;
  __syncthreads();
  if (threadIdx.x == 0) norm_part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// Per-block partial sum of squares of the (unnormalised) gradient.
__global__ __launch_bounds__(256) void sumsq_kernel(const float* __restrict__ g, int64_t n, float* __restrict__ part) {
  __shared__ float red[4];
  float s = 0.0f;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) s = fmaf(g[i], g[i], s);
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

struct OptHP {
  float lr, alpha, eps, clip;
  int n_agents;
};

// Normalise by sum(mask), clip by the global norm (torch clip_grad_norm_: coef = clip / (norm + 1e-6),
// clamped to 1), RMSprop (torch: v = a v + (1-a) g^2; p += -lr * g / (sqrt(v) + eps)). Every block re-derives
// the norm from the same partials in the same order, so all blocks agree bitwise.
__global__ __launch_bounds__(256) void apply_kernel(float* __restrict__ p, float* __restrict__ g, float* __restrict__ sq,
                                                    int64_t n, const float* __restrict__ part, int npart,
                                                    OptHP hp, float* __restrict__ stats,
                                                    const int* __restrict__ halt) {
  // halt (may be NULL): a non-zero word means an earlier kernel of the step failed (the COMA critic chain's error
  // word); the parameters, gradient and square_avg are then left untouched
  if (halt && *halt != 0) return;
  __shared__ float sh[2];
  // the first element's operands and the mask sum do not depend on the norm: their loads go out before it
  const int64_t i0 = (int64_t)blockIdx.x * 256 + threadIdx.x, stride = (int64_t)gridDim.x * 256;
  const bool have0 = i0 < n;
  const float g0 = have0 ? g[i0] : 0.0f, v0 = have0 ? sq[i0] : 0.0f, p0 = have0 ? p[i0] : 0.0f;
  const float* sums = g + n;   // MQ_NSUMS tail
  const float msum = sums[1];
  if (threadIdx.x < 64) {
    float s = 0.0f;
    for (int i = threadIdx.x; i < npart; i += 64) s += part[i];
    s = wave_sum(s);
    if (threadIdx.x == 0) sh[0] = s;
  }
  __syncthreads();
  const float inv = 1.0f / msum;
  const float norm = sqrtf(sh[0]) * inv;
  const float coef = fminf(hp.clip / (norm + 1e-6f), 1.0f);
  auto upd = [&](int64_t i, float gv, float sv, float pv) {
    const float gi = (gv * inv) * coef;
    g[i] = gi;
    const float v = sv * hp.alpha + (1.0f - hp.alpha) * (gi * gi);
    sq[i] = v;
    p[i] = pv + (-hp.lr) * (gi / (sqrtf(v) + hp.eps));
  };
  if (have0) upd(i0, g0, v0, p0);
  for (int64_t i = i0 + stride; i < n; i += stride) upd(i, g[i], sq[i], p[i]);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    stats[0] = sums[0] / msum;                         // loss
    stats[1] = norm;                                   // grad_norm
    stats[2] = sums[2] / msum;                         // td_error_abs
    stats[3] = sums[3] / (msum * (float)hp.n_agents);  // q_taken_mean (q_learner.py:114 divisor)
    stats[4] = sums[4] / (msum * (float)hp.n_agents);  // target_mean
    stats[5] = msum;
    stats[6] = coef;
    stats[7] = 0.0f;
  }
}

// One BasicMAC.forward step for every (episode, agent) row: inputs [obs_t | onehot(a_{t-1}) | onehot(agent)],
// fc1 -> relu -> GRUCell -> fc2. One 256-thread workgroup per row (rollout batches are small).
// xin_dense != NULL: the inputs are given ([rows][I], RNNAgent.forward); otherwise they are built from the replay.
__global__ __launch_bounds__(256) void mac_step_kernel(Dims d, Rep rp, const float* __restrict__ P, Lay L, int t,
                                                       const float* __restrict__ xin_dense,
                                                       const float* __restrict__ h_in, float* __restrict__ h_out,
                                                       float* __restrict__ q_out) {
  extern __shared__ __attribute__((aligned(16))) float sm[];   // xin [I] | x1 [H] | h [H] | gi [3H] | gh [3H] | h1 [H]
  float* xin = sm;
  float* x1 = xin + ((d.I + 3) & ~3);
  float* hh = x1 + H;
  float* gi = hh + H;
  float* gh = gi + G3;
  float* h1 = gh + G3;
  const int row = blockIdx.x, b = row / d.n, ag = row - b * d.n, tid = threadIdx.x;
  const int64_t slot = xin_dense ? 0 : rp.ep(b) * d.t_stride + t;
  for (int f = tid; f < d.I; f += 256) {
    float v;
    if (xin_dense) {
      v = xin_dense[(int64_t)row * d.I + f];
    } else if (f < d.O) {
      v = rp.obs[(slot * d.n + ag) * d.O + f];
    } else {
      int g = f - d.O;
      v = 0.0f;
      bool done = false;
      if (d.last_action) {
        if (g < d.A) {
          if (t > 0 && rp.filled[slot - 1]) v = (int)rp.actions[(slot - 1) * d.n + ag] == g ? 1.0f : 0.0f;
          done = true;
        }
        g -= d.A;
      }
      if (!done) v = (d.agent_id && g == ag) ? 1.0f : 0.0f;
    }
    xin[f] = v;
  }
  if (tid < H) hh[tid] = h_in[(int64_t)row * H + tid];
  __syncthreads();
  if (tid < H) {
    const float* w = P + L.o[MQ_P_FC1_W] + (int64_t)tid * d.I;
    float s = 0.0f;
    for (int k = 0; k < d.I; ++k) s = fmaf(w[k], xin[k], s);
    x1[tid] = fmaxf(s + P[L.o[MQ_P_FC1_B] + tid], 0.0f);
  }
  __syncthreads();
  if (tid < G3) {
    const float* wi = P + L.o[MQ_P_RNN_W_IH] + tid * H;
    const float* wh = P + L.o[MQ_P_RNN_W_HH] + tid * H;
    float si = 0.0f, shh = 0.0f;
    for (int k = 0; k < H; ++k) { si = fmaf(wi[k], x1[k], si); shh = fmaf(wh[k], hh[k], shh); }
    gi[tid] = si + P[L.o[MQ_P_RNN_B_IH] + tid];
    gh[tid] = shh + P[L.o[MQ_P_RNN_B_HH] + tid];
  }
  __syncthreads();
  if (tid < H) {
    const float r = sigmoidf_(gh[tid] + gi[tid]);
    const float zg = sigmoidf_(gh[H + tid] + gi[H + tid]);
    const float ng = tanhf_(gi[2 * H + tid] + gh[2 * H + tid] * r);
    const float v = (hh[tid] - ng) * zg + ng;
    h1[tid] = v;
  }
  __syncthreads();
  if (tid < H) h_out[(int64_t)row * H + tid] = h1[tid];
  if (tid < d.A) {
    const float* w = P + L.o[MQ_P_FC2_W] + tid * H;
    float s = 0.0f;
    for (int k = 0; k < H; ++k) s = fmaf(w[k], h1[k], s);
    q_out[(int64_t)row * d.A + tid] = s + P[L.o[MQ_P_FC2_B] + tid];
  }
}

// Masked greedy argmax (unavailable = -inf, first max index), one lane per row.
__global__ __launch_bounds__(256) void greedy_kernel(const float* __restrict__ q, const int32_t* __restrict__ avail,
                                                     int64_t* __restrict__ out, int rows, int A) {
  const int row = blockIdx.x * 256 + threadIdx.x;
  if (row >= rows) return;
  float best = 0.0f;
  int arg = 0;
  bool any = false;
  for (int a = 0; a < A; ++a) {
    const float v = avail[(int64_t)row * A + a] ? q[(int64_t)row * A + a] : -INFINITY;
    if (!any || v > best) { best = v; arg = a; any = true; }
  }
  out[row] = arg;
}

}  // namespace mq
