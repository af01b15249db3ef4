// Persistent COMA critic chain: every live critic step of one COMALearner.train (coma_learner.py:118-139) in ONE
// persistent launch, instead of three launches per step (coma_l1 / coma_head / coma_wgrad).
//
// G = 8 * NK workgroups of 512 threads, all resident (G <= the CU count, one per CU). Workgroup (ut, ks) owns the W1
// tile [16 units ut][CC_KW columns ks] for the whole train: the tile stays in LDS and its RMSprop square_avg and
// gradient in registers, so W1 (the critic's 111k-element bulk at MMM2) never leaves the CU between steps. The first
// NHEAD = ceil(R / 16) workgroups (grouped on as few XCDs as possible) also run the head of one 16-row tile. fc1.bias / fc2 / fc3 live in P (the caller's
// buffer): the lane that computes an element's gradient in phase C applies its update in place in phase D, and the
// heads reload the new version into LDS at the start of the next step. One live step t is four phases:
//   A  (all)   H1p[ks][r][16 ut ..] = X_t[r][K slice] W1_tile^T                         (MFMA; X_t prefetched)
//   B  (heads) reload b1 / W2 / b2 / W3 / b3, H1 = relu(sum_ks H1p + b1), H2 = relu(H1 W2^T + b2), Q = H2 W3^T + b3,
//              TD error vs the TD(lambda) target, loss sums, dQ, dH2 = dQ W3 o [H2 > 0], dH1 = dH2 W2 o [H1 > 0]
//   C  (all)   dW1 tile = dH1[:, units]^T X_t[:, K slice] (registers), db1 (ks = 0), the 64 dW2 16x16 tiles and
//              the dW3 tiles round-robin over the workgroups, per-workgroup sum of squares
//   D  (all)   the global gradient norm from the G partials (fixed order), clip coefficient, RMSprop on the owned
//              W1 tile and on the fc1.bias .. fc3.bias elements whose gradients the workgroup computed in C (still in
//              registers: no gradient exchange); the last workgroup records the stats
// The hand-offs are flags, not grid barriers: A -> B every workgroup flags, only the heads wait; B -> C the heads
// flag, every workgroup waits; C -> D each workgroup publishes its sum of squares as one 8-B {value, step tag}
// granule after draining its stores, and every workgroup's wave 0 polls all G granules. Buffers reused by the next
// step are safe because each write of step t + 1 sits behind a wait on flags posted after the step-t reads.
// Hand-offs between workgroups: every exchanged word is stored write-through (sc1) and loaded sc1 by the consumer
// (4-B, or 16-B where the layout allows), behind step-tagged flags (every wave drains its stores, workgroup barrier,
// one lane stores the flag write-through; the consumer polls sc1 with s_sleep) — MI355X_MICROARCH.md § visibility,
// Valid forms, row 1; no cache fences. Spins are bounded: a timeout sets the error word, every workgroup leaves, and the
// stats come out NaN. Skipped steps (empty mask, coma_learner.py:121-122) are skipped by every workgroup alike.
// The products are the three-launch path's; the bias gradients (db1 in row order, db2 / db3 as per-lane partials
// combined over the four lane groups), the norm partials and the H2 / Q / dH1 k-chains (two interleaved
// accumulators) are summed in other fixed orders, so the two paths agree to float rounding, not bitwise. The RMSprop
// update is applied at the end of its own step instead of inside the next step's staging. Both paths are checked
// against the oracle and against each other (tests/test_gpu_coma.py).
// Measured at cfg5 (MMM2 shape, R = 80, Kc = 868, G = 64; MQ_DIAG coma_trace prints workgroup 0's phase spans):
// DESIGN.md §3b.
#pragma once
#include "coma_kernels.hpp"

namespace mq {

constexpr int CC_THREADS = 512;   // 8 waves: 2 per SIMD, so a wave may hold 256 VGPRs (no spills)
constexpr int CC_KW = 112;      // W1 columns per owner workgroup: 7 MFMA N-tiles, 28 k-steps
constexpr int CC_KP = CC_KW + 1;
constexpr int CC_MAXR = 80;     // rows (B * n) of one critic step the LDS budget allows
constexpr int CC_CP = CH + 4;   // head-array row pitch: 16-B rows for the b128 operand reads of phase B
constexpr unsigned CC_SPIN_LIMIT = 1u << 20;
constexpr int CC_XV = CC_KW / 4;                                     // 16-B units per X row slice
constexpr int CC_XPT = (CC_MAXR * CC_XV + CC_THREADS - 1) / CC_THREADS;  // of them per thread

typedef __attribute__((address_space(1))) unsigned cc_gu32;
typedef __attribute__((address_space(1))) unsigned long long cc_gu64;

MQ_DEV void st_wt(float* p, float v) {
  __hip_atomic_store((cc_gu32*)p, __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
MQ_DEV void st_wt_i(int* p, int v) {
  __hip_atomic_store((cc_gu32*)p, (unsigned)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
MQ_DEV float ld_wt(const float* p) {
  return __uint_as_float(__hip_atomic_load((cc_gu32*)(float*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
MQ_DEV int ld_wt_i(const int* p) {
  return (int)__hip_atomic_load((cc_gu32*)(int*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// 16-B write-through-coherent load (global_load_dwordx4 sc1), for bulk hand-offs: the value is NOT ready until
// cc_vm_wait(); cc_vm_wait() then cc_ready(v) on every such value before its first use (the empty asm ties the use
// behind the wait, which the compiler cannot see through)
MQ_DEV f32x4 ld_wt4(const float* p) {
  f32x4 v;
  asm volatile("global_load_dwordx4 %0, %1, off sc1" : "=v"(v) : "v"(p) : "memory");
  return v;
}
// 16-B write-through store (global_store_dwordx4 sc1); drained by cc_post's vmcnt(0) like every store
MQ_DEV void st_wt4(float* p, f32x4 v) { asm volatile("global_store_dwordx4 %0, %1, off sc1" : : "v"(p), "v"(v) : "memory"); }
constexpr int kCpolSc1 = 16;   // buffer-instruction cache policy: sc1 (write-through store / L2-coherent load)
MQ_DEV void cc_vm_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
MQ_DEV void cc_ready(f32x4& v) { asm volatile("" : "+v"(v)); }

struct CChain {
  CDims d;
  Rep rp;
  float* P;           // critic params (caller's buffer), MC_P layout: read at the start, final version at the end
  float* SQ;          // critic square_avg (caller's)
  float* G;           // critic grads (caller's): the last live step's clipped gradient at the end
  int64_t o_w1, o_b1, o_w2, o_b2, o_w3, o_b3, Pc;
  const float* X;     // [Tp][R][Kp]
  const float* tgt;   // [T][R]
  const float* msum;  // [T]
  float* H1p;         // [NK][R][CH]
  float* H1x;         // [R][CH]
  float* H2x;
  float* dH2x;
  float* dH1x;
  float* dqx;         // [R]
  int* actx;          // [R]
  float* part;        // [NHEAD][8]
  unsigned long long* normg;   // [G] {sum of squares, step tag} granules (zeroed before the launch)
  float* GW;          // [Pc] gradient exchange (b1, W2, b2, W3, b3 regions)
  float* qvals;       // [T][R][A]
  float* crec;        // [T][8]
  int* cstate;        // [0] live steps, [1] t of the last live step
  unsigned* sync;     // [1] error word (zeroed before the launch)
  unsigned* flagA;    // [G] phase-A-done step tags (zeroed before the launch)
  unsigned* flagB;    // [NHEAD] phase-B-done step tags of the heads
  int NK, NG, NHEAD;
  OptHP hp;
  unsigned long long* trace;   // optional (MQ_DIAG coma_trace): workgroup 0's phase timestamps, [16 steps][8]
  int fault_wg;                // test hook (MQ_DIAG coma_fault): this workgroup never flags its phase A of the
                               // second live step, so the heads time out (-1: none)
};

// LDS carve (floats)
struct CCLds {
  int w1, xs, du, w2, w3, b1, b2, b3, h1, h2, dh2, q, misc, total;
  __host__ __device__ CCLds(int A16) {
    w1 = 0;                           // [16][CC_KP]
    xs = w1 + 16 * CC_KP;             // [CC_MAXR][CC_KP]
    du = xs + CC_MAXR * CC_KP;        // [CC_MAXR][17]  dH1 of the owned units (phase C)
    w2 = du + CC_MAXR * 17;           // [CH][CC_CP]    heads
    w3 = w2 + CH * CC_CP;             // [A16][CC_CP]
    b1 = w3 + A16 * CC_CP;            // [CH]
    b2 = b1 + CH;                     // [CH]
    b3 = b2 + CH;                     // [A16]
    h1 = b3 + A16;                    // [16][CC_CP]
    h2 = h1 + 16 * CC_CP;             // [16][CC_CP]
    dh2 = h2 + 16 * CC_CP;            // [16][CC_CP]
    q = dh2 + 16 * CC_CP;             // (unused: Q is consumed where it is summed)
    misc = q;                         // 176 floats of scalars / partials (CC_MISC)
    total = misc + 176;
  }
};

// LDS index of element e of the contiguous fc1.bias | fc2.weight | fc2.bias | fc3.weight | fc3.bias block (MC_P order)
MQ_DEV int head_lds_index(const CCLds& Lo, int e, int A) {
  if (e < CH) return Lo.b1 + e;
  e -= CH;
  if (e < CH * CH) return Lo.w2 + (e >> 7) * CC_CP + (e & 127);
  e -= CH * CH;
  if (e < CH) return Lo.b2 + e;
  e -= CH;
  if (e < A * CH) return Lo.w3 + (e >> 7) * CC_CP + (e & 127);
  return Lo.b3 + (e - A * CH);
}

inline size_t cc_lds_bytes(int A) { return (size_t)CCLds((A + 15) / 16 * 16).total * sizeof(float); }
inline int cc_nk(int Kc) { return (Kc + CC_KW - 1) / CC_KW; }
inline bool cc_ok(int R, int A, int Kc, int num_cu) {
  return R >= 1 && R <= CC_MAXR && A <= 32 && 8 * cc_nk(Kc) <= 256 && cc_lds_bytes(A) <= 160 * 1024 && 8 * cc_nk(Kc) <= num_cu &&
         8 * cc_nk(Kc) >= (R + 15) / 16 && 8 * cc_nk(Kc) <= 256;
}

// Hand-off flags (MI355X_MICROARCH.md Valid forms row 1): the publisher drains every wave's write-through stores,
// joins a workgroup barrier, and one lane stores the step tag to its flag word write-through; a consumer's wave 0
// polls the `count` flags it depends on (lane i: flags i, i + 64, ..) until each reaches the tag, and the other
// waves join behind a workgroup barrier. Tags grow by one per live step and the words are zeroed per launch.
// Returns false (error word set) on a timeout or a peer's error.
MQ_DEV void cc_post(unsigned* flag, unsigned tag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store((cc_gu32*)flag, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

MQ_DEV bool cc_wait(const CChain& a, const unsigned* flags, int count, unsigned tag, float* misc) {
  if (threadIdx.x < 64) {
    int fail = 0;
    for (int i = threadIdx.x; i < count && !fail; i += 64) {
      unsigned spins = 0;
      while (__hip_atomic_load((cc_gu32*)(unsigned*)(flags + i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < tag) {
        if (++spins > CC_SPIN_LIMIT ||
            __hip_atomic_load((cc_gu32*)(a.sync + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) {
          fail = 1;
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
    }
    const bool any = __ballot(fail) != 0ull;
    if (threadIdx.x == 0) {
      if (any) __hip_atomic_store((cc_gu32*)(a.sync + 1), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      misc[63] = any ? 0.0f : 1.0f;
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // keeps the exchanged-data loads below the poll
  return misc[63] != 0.0f;
}

__global__ __launch_bounds__(CC_THREADS) void coma_chain_kernel(CChain a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int A = a.d.A, A16 = (A + 15) / 16 * 16, R = a.d.R, n = a.d.n, Kc = a.d.Kc, Kp = a.d.Kp, T = a.d.T;
  const CCLds Lo(A16);
  float* W1t = lds + Lo.w1;
  float* Xs = lds + Lo.xs;
  float* Du = lds + Lo.du;
  float* W2s = lds + Lo.w2;
  float* W3s = lds + Lo.w3;
  float* b1s = lds + Lo.b1;
  float* b2s = lds + Lo.b2;
  float* b3s = lds + Lo.b3;
  float* H1s = lds + Lo.h1;
  float* H2s = lds + Lo.h2;
  float* dH2s = lds + Lo.dh2;
  float* misc = lds + Lo.misc;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, g = lane >> 4, c = lane & 15;
  const int wg = blockIdx.x, ut = wg & 7, ks = wg >> 3;
  const int u0 = 16 * ut, k0 = ks * CC_KW;
  const int kwc = max(0, min(CC_KW, Kc - k0));       // real W1 columns of this tile
  // head slot hs of this workgroup: slot-major within an XCD (blocks b and b + 8 share one, MI355X_MICROARCH.md
  // § dispatch), so the heads (hs < NHEAD) sit on as few XCDs as the grid allows and their per-step reload of
  // fc1.bias .. fc3.bias, 76 KB each, is served by one L2 after the first miss (placement only: correctness does
  // not depend on it)
  const int hs = (wg & 7) * a.NK + (wg >> 3);
  const bool head = hs < a.NHEAD;
  const int r0 = 16 * hs, nr = head ? min(16, R - r0) : 0;
  const int npart = (int)(a.Pc - a.o_b1);            // b1 .. b3, contiguous
  const float alpha = a.hp.alpha, lr = a.hp.lr, eps = a.hp.eps;

  // ---- prologue: the owned W1 tile (LDS) with its square_avg in the dW1 accumulator layout (registers)
  for (int e = tid; e < 16 * CC_KP; e += CC_THREADS) {
    const int u = e / CC_KP, k = e - u * CC_KP;
    W1t[e] = k < kwc ? a.P[a.o_w1 + (int64_t)(u0 + u) * Kc + k0 + k] : 0.0f;
  }
  // dW1 layout: wave w < 7 owns N-tile w (columns 16 w .. +15 of the slice); lane element e: unit 4 g + e, column c
  float sq1[4] = {0, 0, 0, 0}, gl1[4] = {0, 0, 0, 0};
  if (w < 7) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int u = 4 * g + e, k = 16 * w + c;
      sq1[e] = k < kwc ? a.SQ[a.o_w1 + (int64_t)(u0 + u) * Kc + k0 + k] : 0.0f;
    }
  }
  if (head) {   // fc3's padding rows / bias lanes stay zero (phase B reloads rows < A only)
    for (int e = A * CH + tid; e < A16 * CH; e += CC_THREADS) W3s[(e >> 7) * CC_CP + (e & 127)] = 0.0f;
    if (tid >= A && tid < A16) b3s[tid] = 0.0f;
  }
  // fc1.bias .. fc3.bias: every element's gradient is computed in phase C by exactly one lane (the first dW2 / dW3
  // tile of each workgroup, wave 7 / 6, with the tile's bias column; db1 by wave 5 of the ks = 0 workgroups), and that
  // lane also applies its RMSprop update in phase D with the gradient still in registers (own slots 0..3: the tile
  // elements, 4: the bias element; -1: none), so no gradient crosses a workgroup. Tiles past a workgroup's first
  // (grids of fewer than 64 workgroups) go through the GW exchange instead.
  // own_index(oi): this lane's owned elements (called where needed, so nothing stays live across the phases)
  auto own_index = [&](int (&oi)[5], int w, int g, int c, int lane) {
#pragma unroll
    for (int s = 0; s < 5; ++s) oi[s] = -1;
    const int nat = A16 / 16;
    if (w == 7 && wg < 64) {
      const int qu = wg >> 3, qj = wg & 7;
#pragma unroll
      for (int e = 0; e < 4; ++e) oi[e] = (int)a.o_w2 + (16 * qu + 4 * g + e) * CH + 16 * qj + c;
      if (qj == 0 && lane < 16) oi[4] = (int)a.o_b2 + 16 * qu + lane;
    } else if (w == 6 && wg < 8 * nat) {
      const int qa = wg >> 3, qj = wg & 7;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int arow = 16 * qa + 4 * g + e;
        if (arow < A) oi[e] = (int)a.o_w3 + arow * CH + 16 * qj + c;
      }
      if (qj == 0 && lane < 16 && 16 * qa + c < A) oi[4] = (int)a.o_b3 + 16 * qa + c;
    } else if (w == 5 && ks == 0 && lane < 16) {
      oi[4] = (int)a.o_b1 + u0 + lane;
    }
  };
  __syncthreads();

  // X_t of the next live step, prefetched into registers (plain loads: X is written before the launch)
  f32x4 xv[CC_XPT];
  auto load_x = [&](int tt, int tidv) {
#pragma unroll
    for (int q = 0; q < CC_XPT; ++q) {
      const int e = tidv + CC_THREADS * q, rr = e / CC_XV, k = 4 * (e - rr * CC_XV);
      const float* src = a.X + ((int64_t)tt * R + rr) * Kp + k0 + k;
      xv[q] = f32x4{0, 0, 0, 0};
      if (tt >= 0 && rr < R) {
        if (k0 + k + 3 < Kp) {   // columns Kc .. Kp are the X builder's zero padding
          xv[q] = *(const f32x4*)src;
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i) xv[q][i] = k0 + k + i < Kp ? src[i] : 0.0f;
        }
      }
    }
  };
  // X_t of the coming step from the prefetch registers into Xs (LDS). Called where Xs is free (after phase C's dW1
  // reads, before phase D) and the prefetch is known complete (behind phase C's drain), so no wait here and no
  // phase-D store ever sits in front of it in the wave's memory counter.
  auto stage_x = [&](int tidv) {
#pragma unroll
    for (int q = 0; q < CC_XPT; ++q) {
      const int e = tidv + CC_THREADS * q, rr = e / CC_XV, k = 4 * (e - rr * CC_XV);
      if (rr < R) {
        float* d = &Xs[rr * CC_KP + k];
        d[0] = xv[q][0]; d[1] = xv[q][1]; d[2] = xv[q][2]; d[3] = xv[q][3];
      }
    }
  };
  // the first live step below `t0` (-1 if none): 64 mask sums per round trip, the highest live one wins
  auto next_live = [&](int t0) {
    for (int base = t0 - 1; base >= 0; base -= 64) {
      const int tt = base - (int)(threadIdx.x & 63);
      const unsigned long long bal = __ballot(tt >= 0 && a.msum[tt] > 0.0f);
      if (bal) return base - (int)__builtin_ctzll(bal);
    }
    return -1;
  };
  // the loop walks the live steps only: the next one (and its mask sum) is found during phase B, so no load opens a
  // step (a load there would wait behind the previous step's phase-D stores: one vmcnt for loads and stores)
  int t = next_live(T);
  float mt = t >= 0 ? a.msum[t] : 0.0f;
  load_x(t, tid);
  stage_x(tid);
  for (int e = R * CC_KP + tid; e < CC_MAXR * CC_KP; e += CC_THREADS) Xs[e] = 0.0f;   // rows R ..: zero for good
  int live = 0, last_t = -1;
  // misc: [0, 16) dQ of the head's rows, [16, 32) their actions (as float), [32, 40) phase C's per-wave partials,
  // [48, 51) phase D's scalars, [63] the poll result, [64, 80) / [80, 96) the rows' masks / TD targets, [96, 176) the
  // rows' five loss terms
  float* dqs = misc;
  float* acts = misc + 16;
  auto stamp = [&](int k) {
    if (a.trace && wg == 0 && tid == 0 && live < 16) a.trace[live * 8 + k] = __builtin_amdgcn_s_memrealtime();
  };
  // a diagnostic build (-DMQ_COMA_BTRACE, scripts/gpu_ab_coma.sh btrace) moves stamps 3 .. 7 into phase B: H1 (the
  // fan-in) | H2 | Q + TD | dH2 | dH1, printed under the labels B | bar2 | C | bar3 | D; "next" is then the rest
#ifdef MQ_COMA_BTRACE
  auto stamp_b = [&](int k) { stamp(k); };
  auto stamp_n = [&](int) {};
#else
  auto stamp_b = [&](int) {};
  auto stamp_n = [&](int k) { stamp(k); };
#endif
  bool ok = true;
  while (t >= 0 && ok) {   // uniform: every workgroup walks the same live steps
    stamp(0);
    // per-thread indices recomputed every step: the laundered copy keeps the compiler from hoisting every address
    // derived from them out of the loop (that hoisting spilled ~350 B per thread)
    int tid_l = tid;
    asm volatile("" : "+v"(tid_l));
    const int tid = tid_l, w = __builtin_amdgcn_readfirstlane(tid_l >> 6), lane = tid_l & 63, g = lane >> 4,
              c = lane & 15;
    // ================================================================ A: H1 partial pre-activations
    {   // X_t is in Xs already (staged before the previous step's phase D, or in the prologue)
      if (head && tid < 16) {   // the TD inputs of the head's rows, loaded now so phase B does not wait on them
        const int i = tid, rr = r0 + i;
        int at = 0;
        float m = 0.0f, y = 0.0f;
        if (i < nr) {
          const int b = (int)fdiv((uint32_t)rr, a.d.dN), ag = rr - b * n;
          const int64_t slot = a.rp.ep(b) * a.d.t_stride + t;
          at = (int)a.rp.actions[slot * n + ag];
          m = coma_mask(a.rp, slot, t);
          y = a.tgt[(int64_t)t * R + rr];
        }
        acts[i] = (float)at;
        misc[64 + i] = m;
        misc[80 + i] = y;
      }
      __syncthreads();
      const int nrt = (R + 15) / 16;
      if (w < nrt) {   // wave w: rows 16 w .. +15, the whole K slice
        f32x4 acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
        const float* xr = Xs + (16 * w + c) * CC_KP + g;
        const float* wr = W1t + c * CC_KP + g;
        for (int k = 0; k < CC_KW; k += 8) {
          acc0 = mfma_f32_16x4(xr[k], wr[k], acc0);
          acc1 = mfma_f32_16x4(xr[k + 4], wr[k + 4], acc1);
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int rr = 16 * w + 4 * g + e;
          if (rr < R) st_wt(&a.H1p[((int64_t)ks * R + rr) * CH + u0 + c], acc0[e] + acc1[e]);
        }
      }
    }
    stamp(1);
    // A -> B: every workgroup flags its H1 partials (and the phase-D stores before them); only the heads wait
    if (!(wg == a.fault_wg && live == 1)) cc_post(a.flagA + wg, (unsigned)(live + 1));
    if (head && !(ok = cc_wait(a, a.flagA, a.NG, (unsigned)(live + 1), misc))) break;
    stamp(2);
    const int t_next = next_live(t);
    const float mt_next = t_next >= 0 ? a.msum[t_next] : 0.0f;
    load_x(t_next, tid);   // lands while the heads run phase B
    // ================================================================ B: the head of rows r0 .. r0 + 15
    if (head) {
      {   // H1 = relu(sum of the NK slice partials in slice order + b1). Thread = one row x 4 columns (16 x 128 =
          // 512 units of 16 B); the partials' 16-B loads go first, then fc1.bias .. fc3.bias at this step's version
          // (updated in place in P by their owners in the previous step's phase D) are reloaded into LDS while the
          // partials land
        static_assert(16 * CH / 4 == CC_THREADS, "one 16-B unit of the head's H1 tile per thread");
        const int i = tid >> 5, col = 4 * (tid & 31);
        f32x4 hv = {0, 0, 0, 0};
        for (int s0 = 0; s0 < a.NK; s0 += 8) {
          f32x4 pv[8];
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            pv[q] = f32x4{0, 0, 0, 0};
            if (i < nr && s0 + q < a.NK) pv[q] = ld_wt4(a.H1p + ((int64_t)(s0 + q) * R + r0 + i) * CH + col);
          }
          if (s0 == 0) {
            // fc1.bias .. fc3.bias: 16-B units (o_b1 = CH * Kc is a multiple of 4; a 4-unit never crosses an array
            // boundary since CH % 4 == 0; the tail below npart % 4 goes element by element)
            constexpr int NB = (CH + CH * CH + CH + 32 * CH + 32 + 4 * CC_THREADS - 1) / (4 * CC_THREADS);
            const int nvec = npart >> 2;
            f32x4 rv[NB];
#pragma unroll
            for (int q = 0; q < NB; ++q) {
              const int e = 4 * (tid + CC_THREADS * q);
              rv[q] = f32x4{0, 0, 0, 0};
              if ((e >> 2) < nvec) rv[q] = ld_wt4(a.P + a.o_b1 + e);
            }
            float rt = 0.0f;
            const int et = 4 * nvec + tid;
            if (et < npart) rt = ld_wt(&a.P[a.o_b1 + et]);
            cc_vm_wait();
#pragma unroll
            for (int q = 0; q < NB; ++q) {
              cc_ready(rv[q]);
              const int e = 4 * (tid + CC_THREADS * q);
              if ((e >> 2) < nvec) {
                const int li = head_lds_index(Lo, e, A);   // 4 consecutive LDS words: one array row segment
                lds[li] = rv[q][0]; lds[li + 1] = rv[q][1]; lds[li + 2] = rv[q][2]; lds[li + 3] = rv[q][3];
              }
            }
            if (et < npart) lds[head_lds_index(Lo, et, A)] = rt;
            __syncthreads();   // b1s complete before the sums below use it
          }
          cc_vm_wait();
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            cc_ready(pv[q]);
            if (s0 + q < a.NK) hv += pv[q];   // slice order, per element
          }
        }
        f32x4 h = {0, 0, 0, 0};
        if (i < nr) {
#pragma unroll
          for (int e = 0; e < 4; ++e) h[e] = fmaxf(hv[e] + b1s[col + e], 0.0f);
          st_wt4(a.H1x + (int64_t)(r0 + i) * CH + col, h);
        }
        float* d = &H1s[i * CC_CP + col];
        d[0] = h[0]; d[1] = h[1]; d[2] = h[2]; d[3] = h[3];
      }
      __syncthreads();
      stamp_b(3);
      // The head's three products take K in lane-group blocks: MFMA step m of lane group g contracts k = 32 g + m
      // (H2, dH1) or kq kw + (kw / 4) g + m (Q), so each lane reads its A / B operands as 16-B runs of a row.
      if (w < 8) {   // H2 = relu(H1 W2^T + b2): wave w owns unit tile w
        f32x4 acc = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};   // two interleaved chains (even / odd k-steps)
        const float* ar = H1s + c * CC_CP + 32 * g;
        const float* br = W2s + (16 * w + c) * CC_CP + 32 * g;
#pragma unroll
        for (int mm = 0; mm < 8; ++mm) {
          const f32x4 av = *(const f32x4*)&ar[4 * mm], bv = *(const f32x4*)&br[4 * mm];
          acc = mfma_f32_16x4(av[0], bv[0], acc);
          acc1 = mfma_f32_16x4(av[1], bv[1], acc1);
          acc = mfma_f32_16x4(av[2], bv[2], acc);
          acc1 = mfma_f32_16x4(av[3], bv[3], acc1);
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int i = 4 * g + e, j = 16 * w + c;
          const float h2 = fmaxf((acc[e] + acc1[e]) + b2s[j], 0.0f);
          H2s[i * CC_CP + j] = h2;
          if (i < nr) st_wt(&a.H2x[(int64_t)(r0 + i) * CH + j], h2);
        }
      }
      __syncthreads();
      stamp_b(4);
      {   // Q = H2 W3^T + b3 on all 8 waves: (action tile qn, K part kq); the K parts' partials meet in dH2s (free
          // until dH2 below) and are summed in kq order
        const int nat = A16 / 16, ksp = 8 / nat, kw = CH / ksp;   // nat in {1, 2}: 8 or 4 K parts of 16 or 32
        const int qn = w % nat, kq = w / nat;
        f32x4 acc = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
        const int kg = kw / 4;   // 4 or 8 k per lane group
        const float* ar = H2s + c * CC_CP + kq * kw + kg * g;
        const float* br = W3s + (16 * qn + c) * CC_CP + kq * kw + kg * g;
        for (int mm = 0; mm < kg; mm += 4) {
          const f32x4 av = *(const f32x4*)&ar[mm], bv = *(const f32x4*)&br[mm];
          acc = mfma_f32_16x4(av[0], bv[0], acc);
          acc1 = mfma_f32_16x4(av[1], bv[1], acc1);
          acc = mfma_f32_16x4(av[2], bv[2], acc);
          acc1 = mfma_f32_16x4(av[3], bv[3], acc1);
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) dH2s[(kq * 16 + 4 * g + e) * A16 + 16 * qn + c] = acc[e] + acc1[e];
        __syncthreads();
        // thread (row i, action j) sums Q[i][j] in kq order; it stores the Q value the actor's baseline uses
        // (coma_learner.py:126), and the thread of the taken action computes the TD error, dQ and the row's loss
        // terms (coma_learner.py:124-131)
        if (tid < 16 * A16) {
          const int i = tid / A16, j = tid - i * A16, rr = r0 + i;
          float q = 0.0f;
          for (int p = 0; p < ksp; ++p) q += dH2s[(p * 16 + i) * A16 + j];
          q = q + b3s[j];
          if (i < nr && j < A) a.qvals[((int64_t)t * R + rr) * A + j] = q;
          const int at = (int)acts[i];
          if (j == at) {
            const float m = misc[64 + i], y = misc[80 + i];
            float qa = 0.0f, dq = 0.0f, mtd = 0.0f;
            if (i < nr) {
              qa = q;
              mtd = (q - y) * m;
              dq = (2.0f * mtd) * m;
              st_wt(&a.dqx[rr], dq);
              st_wt_i(&a.actx[rr], at);
            }
            dqs[i] = dq;
            misc[96 + i] = mtd * mtd;
            misc[112 + i] = m;
            misc[128 + i] = fabsf(mtd);
            misc[144 + i] = qa * m;
            misc[160 + i] = y * m;
          }
        }
      }
      __syncthreads();
      stamp_b(5);
      for (int e = tid; e < 16 * CH; e += CC_THREADS) {   // dH2 = dQ W3[a] o [H2 > 0]
        const int i = e >> 7, u = e & 127;
        const float h2 = H2s[i * CC_CP + u];
        const float v = h2 > 0.0f ? dqs[i] * W3s[(int)acts[i] * CC_CP + u] : 0.0f;
        dH2s[i * CC_CP + u] = v;
        if (i < nr) st_wt(&a.dH2x[(int64_t)(r0 + i) * CH + u], v);
      }
      __syncthreads();
      stamp_b(6);
      if (w < 8) {   // dH1 = dH2 W2 o [H1 > 0]: B[kk][j] = W2[kk][j]
        f32x4 acc = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
        const float* ar = dH2s + c * CC_CP + 32 * g;
        const float* br = W2s + (32 * g) * CC_CP + 16 * w + c;
#pragma unroll
        for (int mm = 0; mm < 8; ++mm) {
          const f32x4 av = *(const f32x4*)&ar[4 * mm];
          acc = mfma_f32_16x4(av[0], br[(4 * mm) * CC_CP], acc);
          acc1 = mfma_f32_16x4(av[1], br[(4 * mm + 1) * CC_CP], acc1);
          acc = mfma_f32_16x4(av[2], br[(4 * mm + 2) * CC_CP], acc);
          acc1 = mfma_f32_16x4(av[3], br[(4 * mm + 3) * CC_CP], acc1);
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int i = 4 * g + e, j = 16 * w + c;
          if (i < nr) st_wt(&a.dH1x[(int64_t)(r0 + i) * CH + j], H1s[i * CC_CP + j] > 0.0f ? acc[e] + acc1[e] : 0.0f);
        }
      }
      if (w == 0 && lane < 5) {   // the five loss sums over the tile's rows, in row order (the three-launch head's)
        float rv[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) rv[j] = misc[96 + 16 * lane + j];
        float sum = 0.0f;
#pragma unroll
        for (int j = 0; j < 16; ++j) sum += rv[j];
        st_wt(&a.part[hs * 8 + lane], sum);
      }
#ifdef MQ_COMA_BTRACE
      __syncthreads();
#endif
      stamp_b(7);
    }
    stamp_n(3);
    // B -> C: the heads flag H1 / H2 / dH2 / dH1 / dQ / actions / loss partials; every workgroup waits for them
    if (head) cc_post(a.flagB + hs, (unsigned)(live + 1));
    if (!(ok = cc_wait(a, a.flagB, a.NHEAD, (unsigned)(live + 1), misc))) break;
    stamp_n(4);
    // ================================================================ C: gradients, per-workgroup sum of squares
    float sq = 0.0f;
    float og[5] = {0, 0, 0, 0, 0};   // the owned elements' raw gradients (own_index order)
    {
      // operands of the dW2 (wave 7) and dW3 (wave 6) tiles: all CC_MAXR / 4 k-steps of one tile per round trip, in
      // flight while the other waves load dH1 and run the dW1 tile
      const int nat = A16 / 16;
      float pA[CC_MAXR / 4], pB[CC_MAXR / 4];
      int pI[CC_MAXR / 4];
      auto load_w2 = [&](int qt) {   // A = dH2[rows][units of qu], B = H1[rows][columns of qj]
        const int qu = qt >> 3, qj = qt & 7;
        const float* pa = a.dH2x + (int64_t)g * CH + 16 * qu + c;
        const float* pb = a.H1x + (int64_t)g * CH + 16 * qj + c;
#pragma unroll
        for (int q = 0; q < CC_MAXR / 4; ++q) {
          const bool in = 4 * q + g < R;
          pA[q] = in ? ld_wt(pa + q * 4 * CH) : 0.0f;
          pB[q] = in ? ld_wt(pb + q * 4 * CH) : 0.0f;
        }
      };
      auto load_w3 = [&](int qt) {   // A = one-hot dQ (action, dq per row), B = H2[rows][columns of qj]
        const int qj = qt & 7;
        const float* pb = a.H2x + (int64_t)g * CH + 16 * qj + c;
#pragma unroll
        for (int q = 0; q < CC_MAXR / 4; ++q) {
          const int row = 4 * q + g;
          const bool in = row < R;
          pI[q] = in ? ld_wt_i(&a.actx[row]) : -1;
          pA[q] = in ? ld_wt(&a.dqx[row]) : 0.0f;
          pB[q] = in ? ld_wt(pb + q * 4 * CH) : 0.0f;
        }
      };
      if (w == 7 && wg < 64) load_w2(wg);
      if (w == 6 && wg < 8 * nat) load_w3(wg);
      {   // dH1 of the owned units (rows R .. CC_MAXR zero): thread = one row x 4 units, one 16-B load
        static_assert(CC_MAXR * 4 <= CC_THREADS, "one 16-B unit of dH1 per thread");
        const int rr = tid >> 2, u = 4 * (tid & 3);
        f32x4 dv = {0, 0, 0, 0};
        if (rr < R) dv = ld_wt4(a.dH1x + (int64_t)rr * CH + u0 + u);
        // only the waves holding rows (16 w < R) wait: the dW2 / dW3 waves (6, 7; rows >= 96) reach the barrier
        // at once, and their own operand loads are waited for where their MFMAs use them
        if (16 * w < R) cc_vm_wait();
        cc_ready(dv);
        if (rr < CC_MAXR) {
          float* d = &Du[rr * 17 + u];
          d[0] = dv[0]; d[1] = dv[1]; d[2] = dv[2]; d[3] = dv[3];
        }
      }
      __syncthreads();
      // waves 0 .. 6: the dW1 tile's 7 N-tiles; wave 5 then db1 (ks = 0), wave 6 then its dW3 tiles; wave 7: dW2
      if (w < 7) {   // dW1 tile, N-tile w: A[i = unit][kk = row] = dH1, B[kk = row][j = column] = X_t
        f32x4 acc = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};   // two interleaved k-chains (even / odd 4-row steps)
#pragma unroll
        for (int q = 0; q < CC_MAXR / 4; ++q) {
          const int row = 4 * q + g;   // rows R .. CC_MAXR are zero in both operands
          const float av = Du[row * 17 + c];
          const float bv = Xs[row * CC_KP + 16 * w + c];
          if (q & 1) acc1 = mfma_f32_16x4(av, bv, acc1);
          else acc = mfma_f32_16x4(av, bv, acc);
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bool valid = 16 * w + c < kwc;
          gl1[e] = valid ? acc[e] + acc1[e] : 0.0f;   // raw (unnormalised) gradient until phase D
          sq = fmaf(gl1[e], gl1[e], sq);
        }
      }
      if (w == 5 && ks == 0) {   // db1 of the owned units: column sums of dH1, in row order
        if (lane < 16) {   // all CC_MAXR rows (rows R .. are zero), read 16 at a time ahead of the serial sum
          float s = 0.0f;
#pragma unroll
          for (int r16 = 0; r16 < CC_MAXR; r16 += 16) {
            float v[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) v[j] = Du[(r16 + j) * 17 + lane];
#pragma unroll
            for (int j = 0; j < 16; ++j) s += v[j];
          }
          og[4] = s;
          sq = fmaf(s, s, sq);
        }
      } else if (w == 7) {   // dW2 tiles (16 units x 16 columns, K = rows), round-robin over the workgroups
        for (int qt = wg; qt < 64; qt += a.NG) {
          const int qu = qt >> 3, qj = qt & 7;
          const bool first = qt == wg;
          if (!first) load_w2(qt);
          f32x4 acc = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
          float bs = 0.0f;
#pragma unroll
          for (int q = 0; q < CC_MAXR / 4; ++q) {
            if (q & 1) acc1 = mfma_f32_16x4(pA[q], pB[q], acc1);
            else acc = mfma_f32_16x4(pA[q], pB[q], acc);
            bs += pA[q];
          }
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float gv = acc[e] + acc1[e];
            if (first) og[e] = gv;
            else st_wt(&a.GW[a.o_w2 + (int64_t)(16 * qu + 4 * g + e) * CH + 16 * qj + c], gv);
            sq = fmaf(gv, gv, sq);
          }
          if (qj == 0) {   // db2 of the tile's units: lane groups g hold rows g, g + 4, ..: combine the four
            bs += __shfl_xor(bs, 16, 64);
            bs += __shfl_xor(bs, 32, 64);
            if (lane < 16) {
              if (first) og[4] = bs;
              else st_wt(&a.GW[a.o_b2 + 16 * qu + lane], bs);
              sq = fmaf(bs, bs, sq);
            }
          }
        }
      }
      if (w == 6) {   // dW3 tiles (16 actions x 16 columns; A = one-hot dQ, B = H2)
        for (int qt = wg; qt < 8 * nat; qt += a.NG) {
          const int qa = qt >> 3, qj = qt & 7;
          const int aa = 16 * qa + c;
          const bool first = qt == wg;
          if (!first) load_w3(qt);
          f32x4 acc = {0, 0, 0, 0};
          float bs = 0.0f;
          f32x4 acc1 = {0, 0, 0, 0};
#pragma unroll
          for (int q = 0; q < CC_MAXR / 4; ++q) {
            const float av = pI[q] == aa ? pA[q] : 0.0f;
            if (q & 1) acc1 = mfma_f32_16x4(av, pB[q], acc1);
            else acc = mfma_f32_16x4(av, pB[q], acc);
            bs += av;
          }
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int arow = 16 * qa + 4 * g + e;
            if (arow < A) {
              const float gv = acc[e] + acc1[e];
              if (first) og[e] = gv;
              else st_wt(&a.GW[a.o_w3 + (int64_t)arow * CH + 16 * qj + c], gv);
              sq = fmaf(gv, gv, sq);
            }
          }
          if (qj == 0) {   // db3
            bs += __shfl_xor(bs, 16, 64);
            bs += __shfl_xor(bs, 32, 64);
            if (lane < 16 && aa < A) {
              if (first) og[4] = bs;
              else st_wt(&a.GW[a.o_b3 + aa], bs);
              sq = fmaf(bs, bs, sq);
            }
          }
        }
      }
      sq = wave_sum(sq);
      if (lane == 0) misc[32 + w] = sq;   // misc[32 .. 39]: per-wave partials
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave's write-through stores of C drained ...
#pragma unroll
      for (int q = 0; q < CC_XPT; ++q) cc_ready(xv[q]);   // (the next step's X prefetch landed with them)
      __syncthreads();
      if (tid == 0) {   // ... before this workgroup's {sum of squares, step tag} granule: its flag for phase D
        float s = 0.0f;
        for (int i = 0; i < CC_THREADS / 64; ++i) s += misc[32 + i];
        const unsigned long long gv = ((unsigned long long)(unsigned)(live + 1) << 32) | __float_as_uint(s);
        __hip_atomic_store((cc_gu64*)(a.normg + wg), gv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      stage_x(tid);   // Xs is free (the dW1 reads are behind the barrier); phase A reads it after its own barrier
    }
    // the owned elements' parameter and square_avg (written by this lane only), loaded while wave 0 polls the
    // granules. Branch-free: buffer accesses whose offset kDrop (no owned element) lies past the range, so every slot
    // is one instruction on every path and the compiler's wait counts stay exact (with the slots under branches it
    // waited for each slot's write-through stores before the next slot's math)
    int oi[5];
    own_index(oi, w, g, c, lane);
    const auto prs = buf_rsrc(a.P), srs = buf_rsrc(a.SQ), grs = buf_rsrc(a.G);
    uint32_t ooff[5];
    float op[5], os[5];
#pragma unroll
    for (int s = 0; s < 5; ++s) {
      ooff[s] = oi[s] >= 0 ? (uint32_t)oi[s] * 4u : kDrop;
      op[s] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(prs, ooff[s], 0, kCpolSc1));
      os[s] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(srs, ooff[s], 0, kCpolSc1));
    }
    stamp_n(5);
    // no counter barrier here: wave 0 polls the G granules (one 8-B write-through store each, MI355X_MICROARCH.md
    // Valid forms: R2 granules / row 1 flags), and the other waves join behind the workgroup barrier below
    stamp_n(6);
    // ================================================================ D: clip + RMSprop (coma_learner.py:132-134)
    if (w == 0) {   // the squared norm: each lane sums its partials (lane, lane + 64, ..), then a fixed butterfly
      float pv[4];
      const unsigned tag = (unsigned)(live + 1);
      int fail = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        pv[j] = 0.0f;
        const int i = lane + 64 * j;
        if (i < a.NG) {
          unsigned spins = 0;
          unsigned long long gv;
          while (((gv = __hip_atomic_load((cc_gu64*)(a.normg + i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) >> 32) !=
                 tag) {
            if (++spins > CC_SPIN_LIMIT ||
                __hip_atomic_load((cc_gu32*)(a.sync + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) {
              fail = 1;
              break;
            }
            __builtin_amdgcn_s_sleep(2);
          }
          pv[j] = __uint_as_float((unsigned)gv);
        }
      }
      const float s = wave_sum((pv[0] + pv[1]) + (pv[2] + pv[3]));
      if (__ballot(fail) != 0ull) {
        if (lane == 0) __hip_atomic_store((cc_gu32*)(a.sync + 1), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (lane == 0) misc[63] = __ballot(fail) != 0ull ? 0.0f : 1.0f;
      if (lane == 0) {
        const float inv = 1.0f / mt;
        const float norm = sqrtf(s) * inv;
        misc[48] = inv;
        misc[49] = fminf(a.hp.clip / (norm + 1e-6f), 1.0f);
        misc[50] = norm;
      }
    } else if (w == 1 && wg == a.NG - 1 && lane < 8) {   // the step's critic stats (coma_learner.py:136-139), off
      // workgroup 0's path (a head): lane k sums loss partial k over the heads in head order (written in phase B,
      // ordered by the B -> C flags)
      const int k = lane;
      float s = 0.0f;
      for (int h = 0; h < a.NHEAD; ++h) s += ld_wt(&a.part[h * 8 + k]);
      float* rec = a.crec + t * 8;
      if (k == 0 || k == 2 || k == 3 || k == 4) rec[k] = s;
      else if (k == 1) rec[1] = mt;
      else if (k == 6) rec[6] = 1.0f;
    }
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // keeps the exchanged-data loads below the poll
    if (misc[63] == 0.0f) { ok = false; break; }
    const float inv = misc[48], coef = misc[49];
    if (w < 7) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int u = 4 * g + e, k = 16 * w + c;
        if (k < kwc) {
          const float gg = (gl1[e] * inv) * coef;
          const float v = sq1[e] * alpha + (1.0f - alpha) * (gg * gg);
          W1t[u * CC_KP + k] = W1t[u * CC_KP + k] + (-lr) * (gg / (sqrtf(v) + eps));
          sq1[e] = v;
          gl1[e] = gg;
        }
      }
    }
    // the owned elements of fc1.bias .. fc3.bias, from registers; P write-through (the heads reload it in phase B),
    // G the last live step's clipped gradient
#pragma unroll
    for (int s = 0; s < 5; ++s) {
      const float gg = (og[s] * inv) * coef;
      const float v = os[s] * alpha + (1.0f - alpha) * (gg * gg);
      const float pn = op[s] + (-lr) * (gg / (sqrtf(v) + eps));
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, pn), prs, ooff[s], 0, kCpolSc1);
      buf_st(srs, ooff[s], v);
      buf_st(grs, ooff[s], gg);
    }
    if (w >= 6 && wg + a.NG < 64) {   // tiles past the first (grids of fewer than 64 workgroups): via GW
      auto upd = [&](int64_t i) {
        const float gg = (ld_wt(&a.GW[i]) * inv) * coef;
        const float v = a.SQ[i] * alpha + (1.0f - alpha) * (gg * gg);
        st_wt(&a.P[i], ld_wt(&a.P[i]) + (-lr) * (gg / (sqrtf(v) + eps)));
        a.SQ[i] = v;
        a.G[i] = gg;
      };
      const int nat = A16 / 16;
      for (int qt = wg + a.NG; qt < (w == 7 ? 64 : 8 * nat); qt += a.NG) {
        const int qr = qt >> 3, qj = qt & 7;
        const int64_t ow = w == 7 ? a.o_w2 : a.o_w3, ob = w == 7 ? a.o_b2 : a.o_b3;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (w == 7 || 16 * qr + 4 * g + e < A) upd(ow + (int64_t)(16 * qr + 4 * g + e) * CH + 16 * qj + c);
        if (qj == 0 && lane < 16 && (w == 7 || 16 * qr + c < A)) upd(ob + 16 * qr + lane);
      }
    }
    if (wg == a.NG - 1 && tid == 0) a.crec[t * 8 + 5] = misc[50];   // the step's gradient norm
    stamp_n(7);
    ++live;
    last_t = t;
    t = t_next;
    mt = mt_next;
    lds_barrier();   // W1t / misc reuse; the phase-D stores drain behind the next step's work (cc_post waits for them)
  }
  if (!ok || live == 0) {
    if (wg == 0 && tid == 0) { a.cstate[0] = ok ? 0 : -1; a.cstate[1] = 0; }
    return;
  }
  // ---- the final version into the caller's buffers; the last live step's clipped gradient into G
  if (w < 7) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int u = 4 * g + e, k = 16 * w + c;
      if (k < kwc) {
        const int64_t i = a.o_w1 + (int64_t)(u0 + u) * Kc + k0 + k;
        a.P[i] = W1t[u * CC_KP + k];
        a.SQ[i] = sq1[e];
        a.G[i] = gl1[e];
      }
    }
  }

  if (wg == 0 && tid == 0) {   // fc1.bias .. fc3.bias are final in P / SQ / G already
    a.G[a.Pc] = a.msum[last_t];
    a.cstate[0] = live;
    a.cstate[1] = last_t;
  }
}

// After the chain: if its error word (cstate[3]) is set, put the critic params and square_avg back to the copy
// taken before the launch (a timed-out chain leaves workgroups at different steps, with W1 tiles never written back).
__global__ __launch_bounds__(256) void coma_chain_restore_kernel(const int* __restrict__ cstate,
                                                                 const float* __restrict__ bak, float* __restrict__ P,
                                                                 float* __restrict__ SQ, int64_t Pc) {
  if (cstate[3] == 0) return;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < Pc; i += (int64_t)gridDim.x * 256) {
    P[i] = bak[i];
    SQ[i] = bak[Pc + i];
  }
}

// Replicated data-parallel critic: the chain's error word travels to every rank in the agent gradient's all-reduce
// (the spare sum slot 7, 0 on success), and every rank then halts on the sum, so all ranks roll back together.
__global__ void coma_halt_to_sum_kernel(const int* __restrict__ halt, float* __restrict__ slot) {
  if (threadIdx.x == 0) *slot = *halt != 0 ? 1.0f : 0.0f;
}
__global__ void coma_sum_to_halt_kernel(const float* __restrict__ slot, int* __restrict__ halt) {
  if (threadIdx.x == 0) *halt = *slot > 0.5f ? 1 : 0;
}

}  // namespace mq
