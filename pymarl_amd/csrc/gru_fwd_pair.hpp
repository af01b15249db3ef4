// Row-pair fused agent forward: one workgroup per row r runs BOTH nets' unrolls (online z = 0, target z = 1) of
// QLearner.train (q_learner.py:49-52, 60-62; rnn_agent.py:24-28), with ONE recurrence wave per net and no barrier
// inside a 16-step chunk.
//
// Why. In the one-row-net kernel (gru_fwd_fused.hpp) the 64 hidden units of a step are spread over four waves, which
// meet at an LDS barrier every step to exchange h. Stamps of that arrangement (scripts/pair_stamps.py, round 5) put a
// step at ~1,260 cycles: ~940 of recurrence work, whose per-unit overhead (DPP sums, lane-split gate math, selects)
// is paid by every K-split lane of a unit, and ~300 of barrier. Here lane j of a net's recurrence wave owns unit j
// whole (K = 64, no cross-lane sum, no gate broadcast) and reads h_{t-1} back from LDS itself (two broadcast reads of
// 32 floats), so the h chain never leaves the wave; its three W_hh rows live in 192 VGPRs.
// The matrix-core work (fc1, W_ih, fc2) runs on the two other SIMDs, decoupled by a two-chunk pipeline, and the roles
// meet once per chunk.
//
// 512 threads, one workgroup per CU; waves w and w + 4 share a SIMD:
//  * wave 0 / wave 1: the recurrence of net 0 / net 1 (SIMDs s0, s1); waves 4 and 5 (the same SIMDs) only stage
//    weights and pass the chunk barriers, so no MFMA ever holds a recurrence wave's SIMD;
//  * waves 2, 3, 6, 7: producers p = 0..3 (SIMDs s2, s3), during chunk c, for both nets:
//      fc2 of chunk c - 1 (producer p < 2 does net p: Q[16][A] = H W2^T + b2, K = 64 in one wave)
//      GI of chunk c + 1 = X1 W_ih^T + b_ih (N-tiles 3p .. 3p + 2) -> LDS, read by chunk c + 1's steps
//      fc1 of chunk c + 2: X1 = relu(XIN W1^T + b1) (N-tile p, W1 in registers)
//      the inputs of chunk c + 3 staged (obs gathered a chunk earlier, one-hots); chunk c + 4's gather issued.
// Outputs as gru_fwd_fused_kernel: Q of both nets; X1, XIN, Hs and the gate records of the online net. fc1 and GI
// take their K in the order that makes the producers' direct weight loads coalesced (below); X1, h and Q therefore
// differ from the one-row-net kernel's by summation order only.
//
// Prologue (round 6). The recurrences need W_hh and GI(0); GI(0) needs X1(0) and W_ih; X1(0) needs the gathered inputs
// and W1. Round 5 staged W_hh and then W_ih through LDS one after the other and read W1 lane by lane (64 cache lines a
// load instruction through L1), so the recurrences started ~58k cycles in (stamps). Now the producers load W1, W_ih
// and W2 straight into their fragment registers at kernel entry, with K maps chosen so the four lane groups of a load
// instruction read one contiguous 32 / 64-byte run of a weight row (16 lines an instruction), while the other four
// waves stage W_hh through LDS (coalesced 16-byte loads, 16-byte groups XOR-swizzled by row, so the recurrence lanes'
// pick-up reads are conflict-free at pitch 64). Three barriers: S1 (W_hh staged, xin(0)), S2 (X1(0), xin(1), W_hh
// picked up), S3 (GI(0), X1(1), xin(2)); then the T loop.
#pragma once
#include "gru_fwd_fused.hpp"

namespace mq {

struct alignas(16) PairLds {
  float h0[H];                    // init_hidden: zeros
  int psync[4];                   // LDS counters: [0] the producers' chunk-0 rendezvous (X1(1), xin(2) complete),
                                  // [1] the hypernet waves' (their staged states)
  float xin[2][FCH][FXP];         // [chunk & 1] agent inputs (both nets)
  float x1[2][2][FCH][H + 4];     // [net][chunk & 1] X1 (written by fc1(0) while W_hh is still staged)
  // from here on, the prologue's W_hh staging area ([net][192 rows][64], XOR-swizzled) overlays the T loop's buffers
  float hs[2][2][FCH][H + 4];     // [net][chunk & 1][step][unit]: h_t (the recurrence's h_{t-1}, fc2's operand)
  float gi[2][2][FCH][G3];        // [net][chunk & 1][step][gate column]
  f32x4 grec[2][FCH][H];          // [chunk & 1][step][unit] online gate record (r, z, n, W_hn h + b_hn)
};
static_assert(sizeof(PairLds) - offsetof(PairLds, hs) >= 2 * G3 * H * sizeof(float), "W_hh staging fits");
constexpr int kPairPrologueBarriers = 3;   // S1, S2, S3

inline bool pair_fwd_ok(int I, int O, int A, int n, int64_t RT) { return fused_fwd_ok(I, O, A, n, RT); }

// STAMP (diagnostic, MQ_DIAG pair_stamp=<file>; Tp <= 512): s_memtime stamps of the first 8 workgroups
// (cdna_hip_programming.md §7 form: s_memtime + lgkmcnt(0) in one asm statement), kept in LDS and written to
// w.slab_rnn as uint32 [block][PSH + 2 * 512] at the end: [0] kernel entry, [1] recurrence loop start, [2] its end,
// [4] the kernel's end, W_hh staging: wave 0's first loads issued [10], all stored [5]; the hypernet waves' states
// staged [3]; [8] producer 0 at S3 (GI(0), X1(1), xin(2) done), [9] the recurrence's W_hh picked up,
// [11 .. 13] the hypernet waves' S1 / S2 / chunk-0 intervals done, [15] their exit; producer 0: [16] its entry loads
// issued, [17] xin(0) stored, [18] after S1, [19] X1(0) and xin(1) done, [20] after S2; [PSH + t] the recurrence's
// step t end; [PSH + 512 + t] the producers' arrival at the barrier closing the chunk of step t (chunk ends only).
constexpr int PSH = 32;   // header slots
constexpr int PST = PSH + 2 * 512;
MQ_DEV uint32_t stamp_now() {
  uint64_t t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return (uint32_t)t;
}
// ---- HYP = 2: the QMIX hypernet (qmix.py:30-44) for block hb = r (32 state rows of net hb & 1) on waves 4 and 5,
// which otherwise only stage W_hh and pass barriers. Those waves share SIMDs s0 / s1 with the recurrences, whose
// matrix cores are idle; in the prologue the recurrences themselves wait for the producers' first chunk, so the
// hypernet's MFMAs fill dead time there, and the rest is spread thinly over the T loop's chunks. Wave hw owns
// N-tiles hw, hw + 2, .. of NH / 16, both 16-row M-tiles each; the A operand (states, zero K padding) is staged once
// in LDS, the B fragments come straight from the parameters (one tile ahead, in registers). Operand maps, K order and
// bias add are hyper_ws_kernel's: HYP and S0 are bitwise its outputs.
constexpr int HT_SP = 4 * 48 + 4;   // row pitch of the staged states (K padded to 192, zeros)
// Tiles a wave has finished by the end of the interval that barrier i (0 = S1, 1 = S2, 2 = S3, which opens chunk 0;
// 3 + c closes chunk c) opens, from the schedule `hs`: nibbles 0..2 the cumulative counts after the S1, S2 and
// chunk-0 intervals, nibble 4 the tiles left for the interval after the last chunk barrier (beside the producers'
// last fc2 and records); the rest spread evenly over chunks 1 .. cl, where every MFMA delays the recurrence wave
// sharing the SIMD by about its own issue time (stamps, round 5).
MQ_DEV int hyp_tiles_by(int i, int cnt, int nbar, int hs) {
  if (i >= nbar - 1) return cnt;
  if (i < 3) return min(cnt, (hs >> (4 * i)) & 15);
  const int c2 = min(cnt, (hs >> 8) & 15), rem = max(cnt - c2 - ((hs >> 16) & 15), 0);
  const int nl = nbar - 4;   // chunks 1 .. cl (i = 3 .. nbar - 2)
  return min(cnt, c2 + (rem * (i - 2) + nl - 1) / nl);
}
constexpr int kHypSched = 0x10421;
template <bool STAMP>
MQ_DEV void hyper_waves(const Dims& d, const Rep& rp, const float* __restrict__ P0, const float* __restrict__ P1,
                        const Lay& L, const Work& w, float* hst, uint32_t* stl, int nbar, int hsched, int* hsync) {
  const int lane = threadIdx.x & 63, g = lane >> 4, c16 = lane & 15;
  const int hw = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) - 4;
  const int hb = blockIdx.x, S = d.S, NH = d.NH, E = d.E, nE = d.n * d.E;
  const bool act = hb < 2 * ((d.M + 31) / 32);   // the host launches HYP = 2 only when every block has a row
  const int z = hb & 1, m0 = (hb >> 1) * 32;
  const float* __restrict__ P = z ? P1 : P0;
  const int NT = NH / 16, cnt = act ? (NT - hw + 1) / 2 : 0;
  // states: wave hw gathers rows 16 hw .. 16 hw + 15 (lanes: columns l, l + 64, l + 128) and stages them. The
  // gather (replay rows scattered over HBM, ~10k cycles at the kernel's start) stays in flight across S1, and the two
  // waves meet on an LDS counter after their stores, so it delays neither S1 nor any other wave.
  if constexpr (STAMP) { const uint32_t v = stamp_now(); if (hw == 0 && lane == 0) stl[25] = v; }
  float vs[16][3];
  if (act) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int m = min(m0 + 16 * hw + i, d.M - 1), t = (int)fdiv((uint32_t)m, d.dB), b = m - t * d.B;
      const float* row = rp.state + (rp.ep(b) * d.t_stride + t + z) * (int64_t)S;
#pragma unroll
      for (int cg = 0; cg < 3; ++cg) vs[i][cg] = row[min(lane + 64 * cg, S - 1)];
    }
  }
  if constexpr (STAMP) { const uint32_t v = stamp_now(); if (hw == 0 && lane == 0) stl[26] = v; }
  lds_barrier();   // S1
  if (act) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int ii = 16 * hw + i, m = m0 + ii;
#pragma unroll
      for (int cg = 0; cg < 3; ++cg) {
        const int col = lane + 64 * cg;
        const float v = (col < S && m < d.M) ? vs[i][cg] : 0.0f;
        hst[ii * HT_SP + col] = v;
        if (z == 0 && w.S0 && m < d.M && col < S) w.S0[(int64_t)m * S + col] = v;
      }
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's state rows are in LDS
  if (lane == 0) __hip_atomic_fetch_add(hsync, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  while (__hip_atomic_load(hsync, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < 2) __builtin_amdgcn_s_sleep(1);
  if constexpr (STAMP) { const uint32_t v = stamp_now(); if (hw == 0 && lane == 0) stl[3] = v; }
  const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)P, (short)0, (int)(L.o[MQ_P_COUNT] * sizeof(float)), 0x00020000);
  const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(w.HYP + (int64_t)z * d.M * NH), (short)0, (int)((int64_t)d.M * NH * sizeof(float)), 0x00020000);
  f32x4 ba[12], bb[12];
  float bja = 0.0f, bjb = 0.0f;
  auto fetch = [&](int k, f32x4 (&bf)[12], float& bj) {   // B fragments of local tile k: row j0 + c16, columns 48 g ..
    const HypSeg sg = hyp_seg(L, nE, E, 16 * (hw + 2 * k));   // wave-uniform: a 16-row tile never straddles segments
    const int row = sg.row + c16;
    const int base = (int)(sg.w + (int64_t)row * S) * 4 + 192 * g;
#pragma unroll
    for (int mm = 0; mm < 12; ++mm)
      bf[mm] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(prs, base + 16 * mm, 0, 0));
    bj = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(prs, (int)(sg.b + row) * 4, 0, 0));
    __builtin_amdgcn_sched_barrier(0);   // the loads stay ahead of the MFMAs that follow
  };
  const float* a0 = hst + c16 * HT_SP + 48 * g;   // A fragments: states rows c16 and 16 + c16, columns 48 g ..
  const float* a1 = a0 + 16 * HT_SP;
  auto tile = [&](int k, const f32x4 (&bf)[12], float bj) {
    f32x4 acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
#pragma unroll
    for (int mm = 0; mm < 12; ++mm) {
      const f32x4 av0 = *(const f32x4*)&a0[4 * mm];
      const f32x4 av1 = *(const f32x4*)&a1[4 * mm];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        acc0 = mfma16x4(av0[e], bf[mm][e], acc0);
        acc1 = mfma16x4(av1[e], bf[mm][e], acc1);
      }
    }
    const int ob0 = ((m0 + 4 * g) * NH + 16 * (hw + 2 * k) + c16) * 4, ob1 = ob0 + 16 * NH * 4;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, acc0[e] + bj), ors, ob0, e * NH * 4, 0);
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, acc1[e] + bj), ors, ob1, e * NH * 4, 0);
    }
  };
  if (cnt > 0) fetch(0, ba, bja);
  int done = 0;
  for (int i = 0; i < nbar; ++i) {
    if (i > 0) lds_barrier();   // barrier i (S1 was passed above, .. the last chunk's)
    // tiles go in pairs (set a holds the next tile at the top of the loop, set b its successor) so both register
    // sets keep fixed roles, and every prefetch is unconditional (past the last tile a harmless repeat): with a set
    // chosen at run time, or a prefetch behind a branch, the compiler joined the sets with copies and waited for the
    // loads just issued (ISA, round 5); an odd count refills set a itself after its tile
    const int upto = hyp_tiles_by(i, cnt, nbar, hsched);
    while (done + 1 < upto) {   // wave-uniform
      fetch(min(done + 1, cnt - 1), bb, bjb);
      tile(done, ba, bja);
      fetch(min(done + 2, cnt - 1), ba, bja);
      tile(done + 1, bb, bjb);
      done += 2;
    }
    if (done < upto) {   // an odd tile: set a is free again once its MFMAs have read it
      tile(done, ba, bja);
      fetch(min(done + 1, cnt - 1), ba, bja);
      ++done;
    }
    if constexpr (STAMP) {
      if (hw == 0 && i < 3) { const uint32_t v = stamp_now(); if (lane == 0) stl[11 + i] = v; }
    }
  }
  if constexpr (STAMP) { const uint32_t v = stamp_now(); if (hw == 0 && lane == 0) stl[15] = v; }
}

template <int NG, bool STAMP, int HYP = 0>
MQ_DEV void pair_body(const Dims& d, const Rep& rp, const float* __restrict__ P0, const float* __restrict__ P1,
                      const Lay& L, const Work& w, PairLds& S, uint32_t* stl, float* hst = nullptr,
                      int hsched = kHypSched) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int R = d.R, Tp = d.Tp, I = d.I, O = d.O, A = d.A, n = d.n;
  const int cl = (Tp - 1) / FCH;   // last chunk
  const int r = blockIdx.x;
  const uint32_t RH = (uint32_t)R * H;
  auto stamp = [&](int slot) {
    if constexpr (STAMP) {
      const uint32_t v = stamp_now();
      if (lane == 0) stl[slot] = v;
    }
  };

  if (tid < H) S.h0[tid] = 0.0f;
  if (tid < 2) S.psync[tid] = 0;
  const bool producer = (wv & 2) != 0;
  // W_hh of both nets reaches the recurrence waves' registers through LDS: lane j needs rows j, 64 + j, 128 + j whole,
  // and loading that layout directly hits 64 cache lines per instruction (~15k cycles through L1, round 5). Waves
  // 0, 1, 4 and 5 read it with coalesced 16-byte loads (a wave covers 1 KB per instruction) into [net][row][64] over
  // the T loop's buffers, the 16-byte group c4 of row q at position c4 ^ (q & 15), so the pick-up (lane j reads group
  // k4 of its rows) touches 16 distinct 4-bank groups per 16 lanes. Each workgroup starts at a different sixteenth of
  // the rows, so the 256 CUs do not request the same L2 lines at the same time.
  float* const stg = &S.hs[0][0][0][0];
  const int srot = (int)(blockIdx.x & 15);
  auto stage_whh = [&](int st) {   // st: this thread's index among the 128 staging threads (waves 0, 1)
    constexpr int NV = 2 * G3 * H / 4, NQ = 24, NR = NV / 128 / NQ;   // two rounds of 24 loads in flight
    const int o_param = (int)L.o[MQ_P_RNN_W_HH];
#pragma unroll
    for (int rnd = 0; rnd < NR; ++rnd) {
      f32x4 v[NQ];
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int e = st + 128 * ((NQ * rnd + q + srot) % (NQ * NR)), z = e >= NV / 2, rem = 4 * (e - z * (NV / 2));
        v[q] = *(const f32x4*)((z ? P1 : P0) + o_param + rem);
      }
      if (wv == 0 && rnd == 0) stamp(10);
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int e = st + 128 * ((NQ * rnd + q + srot) % (NQ * NR)), z = e >= NV / 2, rem = 4 * (e - z * (NV / 2));
        const int row = rem >> 6, c4 = (rem >> 2) & 15;
        *(f32x4*)&stg[((z * G3 + row) * 16 + (c4 ^ (row & 15))) * 4] = v[q];
      }
    }
    if (wv == 0) stamp(5);
  };
  const int nbar = kPairPrologueBarriers + cl + 1;

  if (!producer) {
    if (wv >= 4) {   // waves 4, 5 (the recurrence SIMDs' second slots)
      if constexpr (HYP == 2) {
        hyper_waves<STAMP>(d, rp, P0, P1, L, w, hst, stl, nbar, hsched, &S.psync[1]);
        return;
      }
      for (int i = 0; i < nbar; ++i) lds_barrier();
      return;
    }
    // ================================================================ recurrence wave of net z (wave z)
    const int z = wv, j = lane;
    const float* __restrict__ P = z ? P1 : P0;
    if (z == 0) stamp(24);
    const float bhr = P[L.o[MQ_P_RNN_B_HH] + j], bhz = P[L.o[MQ_P_RNN_B_HH] + H + j],
                bhn = P[L.o[MQ_P_RNN_B_HH] + 2 * H + j];
    stage_whh(wv * 64 + lane);
    lds_barrier();   // S1: W_hh staged (xin(0) too)
    f32x2 wr[32], wz[32], wn[32];   // W_hh[gate * 64 + j][2 k, 2 k + 1], from the staged rows
    {
      const float* Whh = stg + (z * G3 + j) * 64;
#pragma unroll
      for (int k4 = 0; k4 < 16; ++k4) {
        const int o = 4 * (k4 ^ (j & 15));
        const f32x4 a = *(const f32x4*)(Whh + (0 * H) * 64 + o);
        const f32x4 b = *(const f32x4*)(Whh + (1 * H) * 64 + o);
        const f32x4 c = *(const f32x4*)(Whh + (2 * H) * 64 + o);
        wr[2 * k4] = f32x2{a[0], a[1]}; wr[2 * k4 + 1] = f32x2{a[2], a[3]};
        wz[2 * k4] = f32x2{b[0], b[1]}; wz[2 * k4 + 1] = f32x2{b[2], b[3]};
        wn[2 * k4] = f32x2{c[0], c[1]}; wn[2 * k4 + 1] = f32x2{c[2], c[3]};
      }
    }
    if (z == 0) stamp(9);
    lds_barrier();   // S2: W_hh picked up (the staging area is free)
    lds_barrier();   // S3: GI(0)
    const bool online = z == 0;
    float hprev = 0.0f;
    if (z == 0) stamp(1);
    __builtin_amdgcn_s_setprio(2);
    for (int c = 0; c <= cl; ++c) {
      const int pend = min(FCH, Tp - FCH * c);
      for (int p = 0; p < pend; ++p) {
        const int t = FCH * c + p;
        const float* hb = t == 0 ? S.h0 : S.hs[z][((t - 1) / FCH) & 1][(t - 1) & (FCH - 1)];
        const float gr = S.gi[z][c & 1][p][j], gz = S.gi[z][c & 1][p][H + j], gn = S.gi[z][c & 1][p][2 * H + j];
        f32x2 ar = {0.0f, 0.0f}, az = {0.0f, 0.0f}, an = {0.0f, 0.0f};
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {   // two halves of h: 8 broadcast b128 reads in flight, then 24 FMAs
          f32x4 hv[8];
#pragma unroll
          for (int q = 0; q < 8; ++q) hv[q] = *(const f32x4*)&hb[32 * hh + 4 * q];
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const int k4 = 8 * hh + q;
            const f32x2 h01 = {hv[q][0], hv[q][1]}, h23 = {hv[q][2], hv[q][3]};
            ar = pk_fma(wr[2 * k4], h01, ar); az = pk_fma(wz[2 * k4], h01, az); an = pk_fma(wn[2 * k4], h01, an);
            ar = pk_fma(wr[2 * k4 + 1], h23, ar); az = pk_fma(wz[2 * k4 + 1], h23, az);
            an = pk_fma(wn[2 * k4 + 1], h23, an);
          }
        }
        const float sr = ar.x + ar.y, sz = az.x + az.y, sn = an.x + an.y;
        // ATen gru_cell: r, z = sigmoid((W_h h + b_h) + gi); n = tanh(gi_n + r (W_hn h + b_hn)); h = (h - n) z + n
        const float rg = sigm_fast((sr + bhr) + gr), zg = sigm_fast((sz + bhz) + gz);
        const float ghn = sn + bhn;
        const float ng = tanh_fast(gn + ghn * rg);
        const float h1 = (hprev - ng) * zg + ng;
        hprev = h1;
        S.hs[z][c & 1][p][j] = h1;   // read back by this wave's next step (in-order LDS, no barrier)
        // the online record goes to HBM through the producers (one chunk later), not from this wave
        if (online) S.grec[c & 1][p][j] = f32x4{rg, zg, ng, ghn};
        if (z == 0) stamp(PSH + t);
      }
      lds_barrier();   // chunk c's h history complete; chunk c + 1's GI staged
    }
    __builtin_amdgcn_s_setprio(0);
    if (z == 0) stamp(2);
    return;
  }

  // ================================================================== producer waves 2, 3, 6, 7
  const int pw = (wv & 1) | ((wv >> 2) << 1);
  const int g = lane >> 4, c16 = lane & 15;
  const int ptid = pw * 64 + lane;
  const int Kq = (I + 15) / 16 * 4;   // fc1 k-blocks per lane group (multiple of 4)
  const int b = (int)fdiv((uint32_t)r, d.dN), ag = r - b * n;
  const int64_t slot0 = rp.ep(b) * d.t_stride;
  const float* obs_row = rp.obs + (slot0 * n + ag) * (int64_t)O;   // + t * n * O
  const uint32_t RI = (uint32_t)R * I, RA = (uint32_t)R * A;
  const int nO = n * O;
  int gsl[NG];   // gather slot s: element ptid + 256 s of a chunk's [16][O] obs block (gru_fwd_fused_kernel's packing)
#pragma unroll
  for (int s = 0; s < NG; ++s) {
    const int e = ptid + 256 * s, i = (int)fdiv((uint32_t)e, d.dO), col = e - i * O;
    gsl[s] = e < FCH * O ? (i << 28) | (col << 20) | (i * n * O + col) : -1;
  }
  float xr[NG];
  const int oi = ptid >> 4;   // this thread's one-hot row (step oi of a chunk)
  int f_ld = 0, a_ld = -1;
  auto issue_gather = [&](int cc) {
    const int t0 = FCH * cc;
    const float* base = obs_row + (int64_t)t0 * nO;
    const int lim = (Tp - 1 - t0) * nO + O - 1;
#pragma unroll
    for (int s = 0; s < NG; ++s) xr[s] = ld_u32(base, (uint32_t)min(opaque(gsl[s]) & 0xFFFFF, lim));
    const int t = min(max(t0 + oi, 1), Tp - 1) - 1;
    f_ld = *(const int*)(rp.filled + slot0 + t);
    a_ld = *(const int*)(rp.actions + (slot0 + t) * n + ag);
  };
  if (pw == 0) stamp(21);
  issue_gather(0);
  if (pw == 0) stamp(22);
  // register-resident weights of both nets, loaded straight from the parameters with every load of the prologue in
  // flight at once: W1 (fc1 B fragments of N-tile pw), W_ih (GI's, N-tiles 3 pw .. 3 pw + 2), W2 (fc2's, K = 64).
  // K orders (A and B agree; both differ from gru_fwd_fused_kernel's only in summation order): fc1's slot q of lane
  // group g is K = 8 (q / 2) + 2 g + q % 2, GI's slot 4 kq + e is K = 16 kq + 4 g + e, so the four lane groups of
  // one load instruction read one contiguous 32- / 64-byte run of each of 16 weight rows (16 cache lines, not 64)
  float w1r[2][FKQ], wih[2][3][16], w2r[16], bih[2][3], b1[2], b2;
#pragma unroll
  for (int z = 0; z < 2; ++z) {
    const float* __restrict__ P = z ? P1 : P0;
    // (addresses clamped into the row, out-of-range slots zeroed after the load: no exec-masked load branches)
    const float* W1 = P + L.o[MQ_P_FC1_W] + (int64_t)(16 * pw + c16) * I;
    if ((I & 1) == 0) {   // rows 8-byte aligned; 8 jj + 2 g < I covers the pair
#pragma unroll
      for (int jj = 0; jj < FKQ / 2; ++jj) {
        const int k = 8 * jj + 2 * g;
        const f32x2 v = *(const f32x2*)(W1 + min(k, I - 2));
        const bool ok = 2 * jj < Kq && k < I;
        w1r[z][2 * jj] = ok ? v[0] : 0.0f;
        w1r[z][2 * jj + 1] = ok ? v[1] : 0.0f;
      }
    } else {
#pragma unroll
      for (int q = 0; q < FKQ; ++q) {
        const int k = 8 * (q >> 1) + 2 * g + (q & 1);
        const float v = W1[min(k, I - 1)];
        w1r[z][q] = (q < Kq && k < I) ? v : 0.0f;
      }
    }
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      const float* Wi = P + L.o[MQ_P_RNN_W_IH] + (int64_t)(16 * (3 * pw + s) + c16) * H + 4 * g;
#pragma unroll
      for (int kq = 0; kq < 4; ++kq) {
        const f32x4 v = *(const f32x4*)(Wi + 16 * kq);
#pragma unroll
        for (int e = 0; e < 4; ++e) wih[z][s][4 * kq + e] = v[e];
      }
    }
    if (pw == 0 && z == 0) stamp(23);
#pragma unroll
    for (int s = 0; s < 3; ++s) bih[z][s] = P[L.o[MQ_P_RNN_B_IH] + 16 * (3 * pw + s) + c16];
    b1[z] = P[L.o[MQ_P_FC1_B] + 16 * pw + c16];
  }
  {
    const int zf = pw & 1;   // fc2: producer 0 does net 0, producer 1 net 1
    const float* __restrict__ P = zf ? P1 : P0;
    const float* W2 = P + L.o[MQ_P_FC2_W] + (int64_t)min(c16, A - 1) * H + 16 * g;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4 v = *(const f32x4*)(W2 + 4 * q);
#pragma unroll
      for (int e = 0; e < 4; ++e) w2r[4 * q + e] = c16 < A ? v[e] : 0.0f;
    }
    b2 = c16 < A ? P[L.o[MQ_P_FC2_B] + c16] : 0.0f;
  }

  float* X1o = w.X1;
  float* XINo = w.XIN;
  const int wd = I - O, npad = 4 * Kq - I;
  auto store_gather = [&](int cc) {   // the obs gathered by issue_gather(cc) and the one-hots -> xin[cc & 1]
    const int t0 = FCH * cc;
    float* xb = &S.xin[cc & 1][0][0];
    const auto xr_rsrc = buf_rsrc(XINo + ((int64_t)t0 * R + r) * I);   // wave-uniform
#pragma unroll
    for (int s = 0; s < NG; ++s) {
      const int gs = opaque(gsl[s]);
      const int i = (int)((uint32_t)gs >> 28), col = (gs >> 20) & 0xFF;
      const bool live = gs != -1, ok = live && t0 + i < Tp;
      xb[live ? i * FXP + col : FXP - 1] = ok ? xr[s] : 0.0f;   // a dead slot writes the never-read pad column
      buf_st(xr_rsrc, ok ? ((uint32_t)i * RI + col) * 4 : kDrop, xr[s]);
    }
    // one-hot columns of step oi: last action (zero unless slot t-1 was filled, runner contract), agent id
    const int t = t0 + oi;
    const int ap = (d.last_action && t > 0 && t < Tp && f_ld) ? a_ld : -1;
    const auto xo = buf_rsrc(XINo + ((int64_t)t0 * R + r) * I + O);
    const uint32_t ro = (uint32_t)oi * RI;
    for (int col = ptid & 15; col < wd; col += 16) {
      float v;
      if (d.last_action && col < A) v = col == ap ? 1.0f : 0.0f;
      else v = (col - (d.last_action ? A : 0)) == ag ? 1.0f : 0.0f;
      xb[oi * FXP + O + col] = v;
      buf_st(xo, t < Tp ? (ro + col) * 4 : kDrop, v);
    }
    // zero K padding (columns I .. 4 Kq), which neither the gather nor the one-hots write
    for (int e = ptid; e < FCH * npad; e += 256) {
      const int i = e / npad;
      xb[i * FXP + I + (e - i * npad)] = 0.0f;
    }
  };
  auto fc1 = [&](int z, int cc) {   // X1 of chunk cc (inputs in xin[cc & 1]), N-tile pw -> x1[z][cc & 1]
    f32x4 acc = {0, 0, 0, 0}, acc2 = {0, 0, 0, 0};
    const float* xa = &S.xin[cc & 1][c16][2 * g];
#pragma unroll
    for (int jj = 0; jj < FKQ / 2; ++jj) {
      if (2 * jj >= Kq) break;
      const f32x2 av = *(const f32x2*)&xa[8 * jj];
      acc = mfma16x4(av[0], w1r[z][2 * jj], acc);
      acc2 = mfma16x4(av[1], w1r[z][2 * jj + 1], acc2);
    }
    const int t0 = FCH * cc;
    const auto xb = buf_rsrc(X1o + ((int64_t)t0 * R + r) * H);   // wave-uniform
    const uint32_t lo = (uint32_t)(4 * g) * RH + 16 * pw + c16;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int i = 4 * g + e, t = t0 + i;
      const float x = fmaxf((acc[e] + acc2[e]) + b1[z], 0.0f);
      S.x1[z][cc & 1][i][16 * pw + c16] = x;
      if (z == 0) buf_st(xb, t < Tp ? (lo + e * RH) * 4 : kDrop, x);
    }
  };
  auto gi = [&](int z, int cc) {   // GI of chunk cc from x1[z][cc & 1], N-tiles 3 pw .. 3 pw + 2 -> gi[z][cc & 1]
    f32x4 accg[3] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
#pragma unroll
    for (int kq = 0; kq < 4; ++kq) {
      const f32x4 av = *(const f32x4*)&S.x1[z][cc & 1][c16][16 * kq + 4 * g];
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int s = 0; s < 3; ++s) accg[s] = mfma16x4(av[e], wih[z][s][4 * kq + e], accg[s]);
    }
#pragma unroll
    for (int s = 0; s < 3; ++s)
#pragma unroll
      for (int e = 0; e < 4; ++e) S.gi[z][cc & 1][4 * g + e][16 * (3 * pw + s) + c16] = accg[s][e] + bih[z][s];
  };
  auto fc2 = [&](int cc) {   // Q of chunk cc for net pw (pw < 2), K = 64 in this wave
    const int z = pw;
    f32x4 q0 = {0, 0, 0, 0}, q1 = {0, 0, 0, 0};
#pragma unroll
    for (int kq = 0; kq < 4; ++kq) {
      const f32x4 av = *(const f32x4*)&S.hs[z][cc & 1][c16][16 * g + 4 * kq];
      q0 = mfma16x4(av[0], w2r[4 * kq], q0);
      q1 = mfma16x4(av[1], w2r[4 * kq + 1], q1);
      q0 = mfma16x4(av[2], w2r[4 * kq + 2], q0);
      q1 = mfma16x4(av[3], w2r[4 * kq + 3], q1);
    }
    const int t0 = FCH * cc;
    const auto qb = buf_rsrc(w.Q + (int64_t)z * d.RT() * A + ((int64_t)t0 * R + r) * A);   // wave-uniform
    const uint32_t lo = (uint32_t)(4 * g) * RA + c16;
#pragma unroll
    for (int e = 0; e < 4; ++e)
      buf_st(qb, (t0 + 4 * g + e < Tp && c16 < A) ? (lo + e * RA) * 4 : kDrop, (q0[e] + q1[e]) + b2);
  };

  // the online net's h and gate records of chunk cc (LDS hs[0] / grec, written by the recurrence) -> Hs / Gates:
  // 16 steps x 64 units; thread (step 4 k + (ptid >> 6), unit ptid & 63), coalesced along the units
  auto store_records = [&](int cc) {
    const int t0 = FCH * cc, j = ptid & 63;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int i = 4 * k + (ptid >> 6), t = t0 + i;
      const f32x4 gv = S.grec[cc & 1][i][j];
      const float hv = S.hs[0][cc & 1][i][j];
      const bool ok = t < Tp;
      buf_st(buf_rsrc(w.Hs + (int64_t)min(t, Tp - 1) * RH), ok ? ((uint32_t)r * H + j) * 4 : kDrop, hv);
      const auto gb = buf_rsrc(w.Gates + (int64_t)min(t, Tp - 1) * (4 * RH));
      const uint32_t go = ((uint32_t)r * (4 * H) + j) * 4;
#pragma unroll
      for (int q = 0; q < 4; ++q) buf_st(gb, ok ? go + q * 4 * H : kDrop, gv[q]);
    }
  };

  // ---- prologue (S1 .. S3, matched by the other waves): xin(0); X1(0), xin(1); GI(0). The recurrences start once
  // GI(0) is in LDS; X1(1) and xin(2), which only chunk 0's producer work needs, are built inside chunk 0 behind a
  // producers-only rendezvous (an LDS counter), so they are off the loop's start.
  if (pw == 0) stamp(16);
  store_gather(0);   // waits for the gather only: the weight loads issued after it stay in flight
  if (cl >= 1) issue_gather(1);
  if (pw == 0) stamp(17);
  lds_barrier();   // S1: xin(0) (and W_hh staged for the recurrences)
  if (pw == 0) stamp(18);
  fc1(0, 0);
  fc1(1, 0);
  if (cl >= 1) { store_gather(1); if (cl >= 2) issue_gather(2); }
  if (pw == 0) stamp(19);
  lds_barrier();   // S2: X1(0), xin(1); the recurrences have W_hh (the staging area under gi is free)
  if (pw == 0) stamp(20);
  gi(0, 0);
  gi(1, 0);
  if (pw == 0) stamp(8);
  lds_barrier();   // S3: GI(0)

  // chunk 0 (the recurrences run steps 0 .. 15 meanwhile): X1(1) and xin(2) first, then the steady-state work
  if (cl >= 1) {
    fc1(0, 1);
    fc1(1, 1);
    if (cl >= 2) { store_gather(2); if (cl >= 3) issue_gather(3); }
    // every producer's X1(1) N-tile and xin(2) rows are in LDS before any producer reads them: each wave's LDS
    // writes complete before its count, and the reads follow the wait (the recurrence waves are not involved)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's LDS stores done
    if (lane == 0) __hip_atomic_fetch_add(&S.psync[0], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    while (__hip_atomic_load(&S.psync[0], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < 4)
      __builtin_amdgcn_s_sleep(1);
    gi(0, 1);
    gi(1, 1);
  }
  if (cl >= 2) { fc1(0, 2); fc1(1, 2); }
  if (cl >= 3) { store_gather(3); if (cl >= 4) issue_gather(4); }
  if (pw == 0) stamp(PSH + 512 + min(FCH - 1, Tp - 1));
  lds_barrier();
  for (int c = 1; c <= cl; ++c) {
    // chunk c: the recurrences run steps 16 c .. 16 c + 15 meanwhile
    if (pw < 2) fc2(c - 1);
    store_records(c - 1);
    if (c + 1 <= cl) { gi(0, c + 1); gi(1, c + 1); }
    if (c + 2 <= cl) { fc1(0, c + 2); fc1(1, c + 2); }
    if (c + 3 <= cl) { store_gather(c + 3); if (c + 4 <= cl) issue_gather(c + 4); }
    if (pw == 0) stamp(PSH + 512 + min(FCH * c + FCH - 1, Tp - 1));
    lds_barrier();
  }
  if (pw < 2) fc2(cl);   // the last chunk's h history is complete after the final barrier
  store_records(cl);
}

// HYP = 1: the QMIX hypernet as the forward's epilogue: once a workgroup's row is done, its CU runs hyper_fwd_body
// (gru_fwd_fused.hpp) for hypernet blocks r, r + R, .. — for grids with more blocks than rows. HYP = 2: blocks on
// waves 4 / 5 during the prologue and T loop (hyper_waves above), one block per workgroup.
template <int NG, bool STAMP = false, int HYP = 0>
__global__ __launch_bounds__(512, 1) void gru_fwd_pair_kernel(Dims d, Rep rp, const float* __restrict__ P0,
                                                              const float* __restrict__ P1, Lay L, Work w,
                                                              int hsched) {
  __shared__ PairLds S;
  static_assert(sizeof(PairLds) >= hyf_floats() * sizeof(float), "the hypernet epilogue reuses the forward's LDS");
  __shared__ uint32_t stl[STAMP ? PST : 1];
  __shared__ float hst[HYP == 2 ? 32 * HT_SP : 1];
  if constexpr (STAMP) {
    const uint32_t t0 = stamp_now();
    if (threadIdx.x == 0) stl[0] = t0;
  }
  pair_body<NG, STAMP, HYP>(d, rp, P0, P1, L, w, S, stl, hst, hsched);
  if constexpr (HYP == 1) {
    const int nhb = 2 * ((d.M + 31) / 32);
    for (int hb = blockIdx.x; hb < nhb; hb += gridDim.x) {
      __syncthreads();   // the row's (or the previous block's) last LDS reads are done
      hyper_fwd_body(d, rp, P0, P1, L, w.HYP, w.S0, (float*)&S, hb);
    }
  }
  if constexpr (STAMP) {
    __syncthreads();
    const uint32_t te = stamp_now();
    if (threadIdx.x == 0) stl[4] = te;
    __syncthreads();
    if (blockIdx.x < 8)
      for (int i = threadIdx.x; i < PST; i += 512) ((uint32_t*)w.slab_rnn)[(size_t)blockIdx.x * PST + i] = stl[i];
  }
}

// Host: the row-pair forward, grid R, with the smallest gather-slot instantiation that covers O.
inline void launch_fwd_pair(hipStream_t s, const Dims& d, const Rep& rp, const float* P0, const float* P1,
                            const Lay& L, const Work& w, int hyp, bool stamp = false,
                            int hsched = kHypSched) {
  const dim3 g(d.R), b(512);
  const bool g5 = FCH * d.O <= 256 * 5;
#define MQ_PAIR_LAUNCH(NG, ST, HY) hipLaunchKernelGGL((gru_fwd_pair_kernel<NG, ST, HY>), g, b, 0, s, d, rp, P0, P1, L, w, hsched)
  if (stamp) {
    if (hyp == 2) MQ_PAIR_LAUNCH(5, true, 2);
    else if (hyp == 1) MQ_PAIR_LAUNCH(5, true, 1);
    else MQ_PAIR_LAUNCH(5, true, 0);
  } else if (g5) {
    if (hyp == 2) MQ_PAIR_LAUNCH(5, false, 2);
    else if (hyp == 1) MQ_PAIR_LAUNCH(5, false, 1);
    else MQ_PAIR_LAUNCH(5, false, 0);
  } else {
    if (hyp == 2) MQ_PAIR_LAUNCH(FGATHER, false, 2);
    else if (hyp == 1) MQ_PAIR_LAUNCH(FGATHER, false, 1);
    else MQ_PAIR_LAUNCH(FGATHER, false, 0);
  }
#undef MQ_PAIR_LAUNCH
}

}  // namespace mq
