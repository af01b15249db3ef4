// Per-step cycle budget of the two fused recurrences at the cfg2 shape (B = 32, n = 8, T = 120), cache-hot, random
// data: kernel time of production vs producers idle, and s_memtime phase stamps of the chain step (VAR 2048 in the
// forward, 8192 in the BPTT; each the production schedule with the chain's LDS reads completed before its FMAs).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/chain_micro.hip -o scripts/chain_micro && scripts/chain_micro
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "gru_bwd_w1.hpp"
using namespace mq;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

template <class F> float time_med(F f, int reps = 20, int rounds = 7) {
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  f(); CK(hipDeviceSynchronize());
  std::vector<float> v;
  for (int r = 0; r < rounds; ++r) {
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) f();
    CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    v.push_back(ms / reps * 1000.0f);
  }
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

float* dev_rand(size_t n, float scale) {
  std::vector<float> h(n);
  for (auto& x : h) x = scale * ((rand() / (float)RAND_MAX) * 2.0f - 1.0f);
  float* d; CK(hipMalloc(&d, n * 4)); CK(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice));
  return d;
}

// Prototype: the whole BPTT dh chain of one row in ONE wave (lane j = unit j): W_hh columns in VGPRs (96 pairs), the
// 192 dgh values of a step broadcast from LDS (48 ds_read_b128, all lanes one address), no cross-wave sync at all.
// Writes the same [dgh | h_{t-1}] / dgi history rows as the production chain (into a chunk ring in LDS) so the LDS
// traffic is representative; NACC independent accumulator pairs in the mat-vec.
template <int NACC>
__global__ __launch_bounds__(512) void w1_chain_proto(Dims d, const float* __restrict__ P, Lay L, Work w,
                                                      const int64_t* __restrict__ acts, float* __restrict__ out) {
  __shared__ float gh[2][FCH][BRP], gi[2][FCH][BRP];
  __shared__ float w2s[16 * H];
  const int tid = threadIdx.x, r = blockIdx.x, R = d.R, T = d.T, Tp = d.Tp;
  for (int i = tid; i < d.A * H; i += 512) w2s[i] = P[L.o[MQ_P_FC2_W] + i];
  __syncthreads();
  if (tid >= 64) return;
  const int j = tid;
  f32x2 wp[96];
  const float* Whh = P + L.o[MQ_P_RNN_W_HH];
#pragma unroll
  for (int i = 0; i < 96; ++i) wp[i] = f32x2{Whh[(2 * i) * H + j], Whh[(2 * i + 1) * H + j]};
  struct In { float gr, gz, gn, ghn, hp, dch; int a; };
  auto load = [&](int t, In& s) {
    const int tc = max(t, 0);
    const float* g = w.Gates + ((int64_t)tc * R + r) * (4 * H) + j;
    s.gr = g[0]; s.gz = g[H]; s.gn = g[2 * H]; s.ghn = g[3 * H];
    s.hp = w.Hs[((int64_t)max(tc - 1, 0) * R + r) * H + j];
    s.dch = w.dch[(int64_t)min(tc, T - 1) * R + r];
    s.a = (int)acts[(int64_t)tc * R + r];
  };
  In sa, sb, sc;
  load(Tp - 1, sa); load(Tp - 2, sb);
  float carry = 0.0f, dbs = 0.0f;
  auto step = [&](int t, const In& cur, In& ahead) {
    load(t - 2, ahead);
    const int p = t & (FCH - 1), cb = (t / FCH) & 1;
    const float hp = t > 0 ? cur.hp : 0.0f, dchv = t < T ? cur.dch : 0.0f;
    const float dh = carry + dchv * w2s[cur.a * H + j];
    const float dn = dh * (1.0f - cur.gz), dz = dh * (hp - cur.gn);
    const float dan = dn * (1.0f - cur.gn * cur.gn);
    const float dar = (dan * cur.ghn) * (cur.gr * (1.0f - cur.gr));
    const float daz = dz * (cur.gz * (1.0f - cur.gz));
    gh[cb][p][j] = dar; gh[cb][p][H + j] = daz; gh[cb][p][2 * H + j] = dan * cur.gr; gh[cb][p][3 * H + j] = hp;
    gi[cb][p][j] = dar; gi[cb][p][H + j] = daz; gi[cb][p][2 * H + j] = dan;
    dbs += dar + daz + dan;
    const f32x4* dg4 = (const f32x4*)&gh[cb][p][0];
    f32x2 acc[NACC];
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = f32x2{0.0f, 0.0f};
#pragma unroll
    for (int c4 = 0; c4 < 48; ++c4) {
      const f32x4 v = dg4[c4];
      acc[(2 * c4) % NACC] = pk_fma(wp[2 * c4], f32x2{v[0], v[1]}, acc[(2 * c4) % NACC]);
      acc[(2 * c4 + 1) % NACC] = pk_fma(wp[2 * c4 + 1], f32x2{v[2], v[3]}, acc[(2 * c4 + 1) % NACC]);
    }
    float sum = 0.0f;
#pragma unroll
    for (int i = 0; i < NACC; ++i) sum += acc[i].x + acc[i].y;
    carry = dh * cur.gz + sum;
  };
  int t = Tp - 1;
  for (; t - 2 >= 0; t -= 3) { step(t, sa, sc); step(t - 1, sb, sa); step(t - 2, sc, sb); }
  if (t >= 0) step(t, sa, sc);
  if (t - 1 >= 0) step(t - 1, sb, sa);
  out[(int64_t)r * H + j] = carry + dbs;
}

int main(int argc, char** argv) {
  int B = argc > 1 ? atoi(argv[1]) : 32, n = argc > 2 ? atoi(argv[2]) : 8, T = argc > 3 ? atoi(argv[3]) : 120;
  const int A = 14, O = 80;
  Dims d{};
  d.n = n; d.A = A; d.O = O; d.S = 168; d.E = 32; d.I = O + A + n; d.NH = 32 * (n + 3);
  d.B = B; d.Tp = T + 1; d.T = T; d.R = B * n; d.M = T * B; d.t_stride = T + 1;
  d.last_action = 1; d.agent_id = 1; d.mixer = 2; d.double_q = 1; d.gamma = 0.99f;
  d.dR = make_fastdiv(d.R); d.dN = make_fastdiv(n); d.dB = make_fastdiv(B);
  d.dO = make_fastdiv(O); d.dI = make_fastdiv(d.I);
  const int64_t RT = (int64_t)d.Tp * d.R;
  Lay L{};
  int64_t o = 0, sz[MQ_P_COUNT] = {};
  sz[MQ_P_FC1_W] = 64 * d.I; sz[MQ_P_FC1_B] = 64; sz[MQ_P_RNN_W_IH] = 192 * 64; sz[MQ_P_RNN_W_HH] = 192 * 64;
  sz[MQ_P_RNN_B_IH] = 192; sz[MQ_P_RNN_B_HH] = 192; sz[MQ_P_FC2_W] = A * 64; sz[MQ_P_FC2_B] = A;
  for (int i = 0; i < MQ_P_COUNT; ++i) { L.o[i] = o; o += sz[i]; }
  L.o[MQ_P_COUNT] = o;
  float* P0 = dev_rand(o, 0.12f);
  float* P1 = dev_rand(o, 0.12f);
  Work w{};
  CK(hipMalloc(&w.Hs, 2 * RT * 64 * 4)); CK(hipMalloc(&w.Gates, RT * 256 * 4)); CK(hipMalloc(&w.Q, 2 * RT * A * 4));
  CK(hipMalloc(&w.X1, 2 * RT * 64 * 4)); CK(hipMemset(w.X1, 0, 2 * RT * 64 * 4));
  CK(hipMalloc(&w.XIN, RT * d.I * 4)); CK(hipMemset(w.XIN, 0, RT * d.I * 4));
  w.dch = dev_rand(RT, 0.1f);
  CK(hipMalloc(&w.slab_mix, 32 * 8 * 2 * (int64_t)d.R));
  const int64_t len_rnn = L.o[MQ_P_FC2_B] + A - L.o[MQ_P_RNN_W_IH], len1 = 64 * d.I + 64;
  CK(hipMalloc(&w.slab_rnn, (int64_t)d.R * len_rnn * 4));
  CK(hipMalloc(&w.slab_fc1, (int64_t)d.R * len1 * 4));
  std::vector<int64_t> acts((int64_t)B * (T + 1) * n);
  for (auto& a : acts) a = rand() % A;
  int64_t* dacts; CK(hipMalloc(&dacts, acts.size() * 8)); CK(hipMemcpy(dacts, acts.data(), acts.size() * 8, hipMemcpyHostToDevice));
  std::vector<int64_t> fl((int64_t)B * (T + 1), 1);
  int64_t* dfl; CK(hipMalloc(&dfl, fl.size() * 8)); CK(hipMemcpy(dfl, fl.data(), fl.size() * 8, hipMemcpyHostToDevice));
  Rep rp{};
  rp.actions = dacts; rp.filled = dfl; rp.obs = dev_rand((int64_t)B * (T + 1) * n * O, 1.0f);
  printf("B=%d n=%d T=%d rows=%d\n", B, n, T, d.R);

  auto runf = [&](auto kern) {
    return time_med([&] { hipLaunchKernelGGL(kern, dim3(d.R, 2), dim3(512), 0, 0, d, rp, (const float*)P0, (const float*)P1, L, w); });
  };
  auto fwd_budget = [&](const char* name) {
    std::vector<uint64_t> sb(16 * 2 * (size_t)d.R);
    CK(hipMemcpy(sb.data(), w.slab_mix, sb.size() * 8, hipMemcpyDeviceToHost));
    const char* ph[5] = {"lds reads", "fmas", "quad sums", "gates+st", "barrier"};
    printf("fwd %s cycles/step:", name);
    double tot = 0;
    for (int k = 0; k < 5; ++k) {
      double c = 0;
      for (int i = 0; i < 2 * d.R; ++i) c += sb[16 * i + 8 + k];
      c /= 2.0 * d.R * d.Tp;
      tot += c;
      printf(" %s %.0f |", ph[k], c);
    }
    printf(" total %.0f\n", tot);
  };
  printf("fused fwd production %.1f us | producers idle %.1f us\n", runf(gru_fwd_fused_kernel<0, 5>),
         runf(gru_fwd_fused_kernel<4, 5>));
  printf("fused fwd stamped %.1f us | stamped, producers idle %.1f us\n", runf(gru_fwd_fused_kernel<2048, 5>),
         runf(gru_fwd_fused_kernel<2052, 5>));
  hipLaunchKernelGGL((gru_fwd_fused_kernel<2048, 5>), dim3(d.R, 2), dim3(512), 0, 0, d, rp, (const float*)P0, (const float*)P1, L, w);
  CK(hipDeviceSynchronize());
  fwd_budget("production");
  hipLaunchKernelGGL((gru_fwd_fused_kernel<2052, 5>), dim3(d.R, 2), dim3(512), 0, 0, d, rp, (const float*)P0, (const float*)P1, L, w);
  CK(hipDeviceSynchronize());
  fwd_budget("producers idle");
  {  // K4 mat-vec layout: time, budget, and its outputs against production's
    const int64_t nq = 2 * RT * A, nh = RT * 64;
    std::vector<float> q0(nq), q1(nq), h0(nh), h1(nh);
    hipLaunchKernelGGL((gru_fwd_fused_kernel<0, 5>), dim3(d.R, 2), dim3(512), 0, 0, d, rp, (const float*)P0, (const float*)P1, L, w);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(q0.data(), w.Q, nq * 4, hipMemcpyDeviceToHost)); CK(hipMemcpy(h0.data(), w.Hs, nh * 4, hipMemcpyDeviceToHost));
    hipLaunchKernelGGL((gru_fwd_fused_kernel<4096, 5>), dim3(d.R, 2), dim3(512), 0, 0, d, rp, (const float*)P0, (const float*)P1, L, w);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(q1.data(), w.Q, nq * 4, hipMemcpyDeviceToHost)); CK(hipMemcpy(h1.data(), w.Hs, nh * 4, hipMemcpyDeviceToHost));
    double mq = 0, dq = 0, dh = 0;
    for (int64_t i = 0; i < nq; ++i) { mq = std::max(mq, (double)fabsf(q0[i])); dq = std::max(dq, (double)fabsf(q0[i] - q1[i])); }
    for (int64_t i = 0; i < nh; ++i) dh = std::max(dh, (double)fabsf(h0[i] - h1[i]));
    printf("K4 vs production: max |dQ| %.3e (of max |Q| %.3e), max |dh| %.3e\n", dq, mq, dh);
    printf("fused fwd K4 %.1f us | production %.1f us | K4 producers idle %.1f us\n", runf(gru_fwd_fused_kernel<4096, 5>),
           runf(gru_fwd_fused_kernel<0, 5>), runf(gru_fwd_fused_kernel<4100, 5>));
    hipLaunchKernelGGL((gru_fwd_fused_kernel<4096 + 2048, 5>), dim3(d.R, 2), dim3(512), 0, 0, d, rp, (const float*)P0, (const float*)P1, L, w);
    CK(hipDeviceSynchronize());
    fwd_budget("K4 (lds | - | fmas+reduction | gates | barrier)");
  }

  const size_t dyn = (2 * A * 64 + A) * 4;
  auto runb = [&](auto kern) {
    return time_med([&] { hipLaunchKernelGGL(kern, dim3(d.R), dim3(512), dyn, 0, d, rp, (const float*)P0, L, w, len_rnn, len1); });
  };
  auto bwd_budget = [&](const char* name) {
    std::vector<uint64_t> sb(32 * (size_t)d.R);
    CK(hipMemcpy(sb.data(), w.slab_mix, sb.size() * 8, hipMemcpyDeviceToHost));
    const char* ph[5] = {"gates+st", "barrier", "lds reads", "fmas", "quad sum+w2"};
    printf("bwd %s cycles/step:", name);
    double tot = 0;
    for (int k = 0; k < 5; ++k) {
      double c = 0;
      for (int i = 0; i < d.R; ++i) c += sb[32 * i + 17 + k];
      c /= (double)d.R * d.Tp;
      tot += c;
      printf(" %s %.0f |", ph[k], c);
    }
    printf(" total %.0f\n", tot);
  };
  printf("fused bwd production(768) %.1f us | producers idle(772) %.1f us\n", runb(gru_bwd_fused_kernel<768>),
         runb(gru_bwd_fused_kernel<772>));
  printf("fused bwd stamped %.1f us | stamped, producers idle %.1f us\n", runb(gru_bwd_fused_kernel<768 + 8192>),
         runb(gru_bwd_fused_kernel<772 + 8192>));
  hipLaunchKernelGGL(gru_bwd_fused_kernel<768 + 8192>, dim3(d.R), dim3(512), dyn, 0, d, rp, (const float*)P0, L, w, len_rnn, len1);
  CK(hipDeviceSynchronize());
  bwd_budget("production");
  {  // linearised step (VAR 65536): slabs vs production (rounding) and time
    auto slabs = [&]() {
      std::vector<float> a((size_t)d.R * len_rnn), b((size_t)d.R * len1);
      CK(hipMemcpy(a.data(), w.slab_rnn, a.size() * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(b.data(), w.slab_fc1, b.size() * 4, hipMemcpyDeviceToHost));
      a.insert(a.end(), b.begin(), b.end());
      return a;
    };
    hipLaunchKernelGGL(gru_bwd_fused_kernel<768>, dim3(d.R), dim3(512), dyn, 0, d, rp, (const float*)P0, L, w, len_rnn, len1);
    CK(hipDeviceSynchronize());
    const std::vector<float> ref = slabs();
    for (int v : {65536, 65536 + 16384}) {
      if (v == 65536)
        hipLaunchKernelGGL(gru_bwd_fused_kernel<768 + 65536>, dim3(d.R), dim3(512), dyn, 0, d, rp, (const float*)P0, L, w, len_rnn, len1);
      else
        hipLaunchKernelGGL(gru_bwd_fused_kernel<768 + 65536 + 16384>, dim3(d.R), dim3(512), dyn, 0, d, rp, (const float*)P0, L, w, len_rnn, len1);
      CK(hipDeviceSynchronize());
      const std::vector<float> got = slabs();
      double mx = 0, md = 0;
      for (size_t i = 0; i < ref.size(); ++i) { mx = std::max(mx, (double)fabsf(ref[i])); md = std::max(md, (double)fabsf(ref[i] - got[i])); }
      printf("linearised%s vs production slabs: max |diff| %.3e of max |ref| %.3e (rel %.2e)\n", v == 65536 ? "" : "+K12", md, mx, md / mx);
    }
    printf("fused bwd linearised %.1f us | linearised+K12 %.1f us | production %.1f us\n",
           runb(gru_bwd_fused_kernel<768 + 65536>), runb(gru_bwd_fused_kernel<768 + 65536 + 16384>),
           runb(gru_bwd_fused_kernel<768>));
    printf("fused bwd producers idle: linearised %.1f us | linearised+K12 %.1f us | production %.1f us\n",
           runb(gru_bwd_fused_kernel<772 + 65536>), runb(gru_bwd_fused_kernel<772 + 65536 + 16384>),
           runb(gru_bwd_fused_kernel<772>));
  }
  // diagnostic: the chain's global loads all hit one cache-resident step (results meaningless)
  printf("fused bwd fixed-address loads: linearised+K12 %.1f us | idle %.1f us | production %.1f us | idle %.1f us\n",
         runb(gru_bwd_fused_kernel<768 + 65536 + 16384 + 131072>), runb(gru_bwd_fused_kernel<772 + 65536 + 16384 + 131072>),
         runb(gru_bwd_fused_kernel<768 + 131072>), runb(gru_bwd_fused_kernel<772 + 131072>));
  if (argc > 4 && atoi(argv[4]) == 0) return 0;   // only the production and linearised sections
  // K12 mat-vec layout: time, phase budget, and its slabs against production's (same inputs; rounding only)
  {
    auto slabs = [&]() {
      std::vector<float> a((size_t)d.R * len_rnn), b((size_t)d.R * len1);
      CK(hipMemcpy(a.data(), w.slab_rnn, a.size() * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(b.data(), w.slab_fc1, b.size() * 4, hipMemcpyDeviceToHost));
      a.insert(a.end(), b.begin(), b.end());
      return a;
    };
    hipLaunchKernelGGL(gru_bwd_fused_kernel<768>, dim3(d.R), dim3(512), dyn, 0, d, rp, (const float*)P0, L, w, len_rnn, len1);
    CK(hipDeviceSynchronize());
    const std::vector<float> ref = slabs();
    hipLaunchKernelGGL(gru_bwd_fused_kernel<768 + 16384>, dim3(d.R), dim3(512), dyn, 0, d, rp, (const float*)P0, L, w, len_rnn, len1);
    CK(hipDeviceSynchronize());
    const std::vector<float> got = slabs();
    double mx = 0, md = 0;
    for (size_t i = 0; i < ref.size(); ++i) { mx = std::max(mx, (double)fabsf(ref[i])); md = std::max(md, (double)fabsf(ref[i] - got[i])); }
    printf("K12 vs production slabs: max |diff| %.3e of max |ref| %.3e (rel %.2e)\n", md, mx, md / mx);
    printf("fused bwd K12 %.1f us | production %.1f us | K12 stamped %.1f us\n",
           runb(gru_bwd_fused_kernel<768 + 16384>), runb(gru_bwd_fused_kernel<768>),
           runb(gru_bwd_fused_kernel<768 + 16384 + 8192>));
    hipLaunchKernelGGL(gru_bwd_fused_kernel<768 + 16384 + 8192>, dim3(d.R), dim3(512), dyn, 0, d, rp, (const float*)P0, L, w, len_rnn, len1);
    CK(hipDeviceSynchronize());
    bwd_budget("K12 (fmas+reduction in the last bin)");
    printf("fused bwd K12 producers idle %.1f us\n", runb(gru_bwd_fused_kernel<772 + 16384>));
    // decoupled roles: bitwise production, and its time
    hipLaunchKernelGGL(gru_bwd_fused_kernel<768 + 32768>, dim3(d.R), dim3(512), dyn, 0, d, rp, (const float*)P0, L, w, len_rnn, len1);
    CK(hipDeviceSynchronize());
    const std::vector<float> dec = slabs();
    size_t ndiff = 0;
    for (size_t i = 0; i < ref.size(); ++i) ndiff += ref[i] != dec[i];
    printf("decoupled vs production slabs: %zu of %zu differ\n", ndiff, ref.size());
    printf("fused bwd decoupled %.1f us | decoupled+K12 %.1f us | production %.1f us\n",
           runb(gru_bwd_fused_kernel<768 + 32768>), runb(gru_bwd_fused_kernel<768 + 32768 + 16384>),
           runb(gru_bwd_fused_kernel<768>));
    hipLaunchKernelGGL(gru_bwd_fused_kernel<768 + 32768 + 8192>, dim3(d.R), dim3(512), dyn, 0, d, rp, (const float*)P0, L, w, len_rnn, len1);
    CK(hipDeviceSynchronize());
    bwd_budget("decoupled (barrier bin = chain group sync)");
    // SIMD-split roles (chain waves 0, 1, 4, 5 on SIMDs 0 / 1; producers on 2 / 3) with decoupled syncs
    hipLaunchKernelGGL(gru_bwd_fused_kernel<768 + 32768 + 1024>, dim3(d.R), dim3(512), dyn, 0, d, rp, (const float*)P0, L, w, len_rnn, len1);
    CK(hipDeviceSynchronize());
    const std::vector<float> spl = slabs();
    ndiff = 0;
    for (size_t i = 0; i < ref.size(); ++i) ndiff += ref[i] != spl[i];
    printf("split+decoupled vs production slabs: %zu of %zu differ\n", ndiff, ref.size());
    printf("fused bwd split+decoupled %.1f us | split+decoupled+K12 %.1f us | decoupled+prio %.1f us | split+dec idle %.1f us\n",
           runb(gru_bwd_fused_kernel<768 + 32768 + 1024>), runb(gru_bwd_fused_kernel<768 + 32768 + 1024 + 16384>),
           runb(gru_bwd_fused_kernel<768 + 32768 + 128>), runb(gru_bwd_fused_kernel<772 + 32768 + 1024>));
    hipLaunchKernelGGL(gru_bwd_fused_kernel<768 + 32768 + 1024 + 8192>, dim3(d.R), dim3(512), dyn, 0, d, rp, (const float*)P0, L, w, len_rnn, len1);
    CK(hipDeviceSynchronize());
    bwd_budget("split+decoupled");
    hipLaunchKernelGGL(gru_bwd_fused_kernel<768 + 32768 + 1024 + 8192 + 16384>, dim3(d.R), dim3(512), dyn, 0, d, rp, (const float*)P0, L, w, len_rnn, len1);
    CK(hipDeviceSynchronize());
    bwd_budget("split+decoupled+K12");
  }
  {  // the one-wave-chain BPTT kernel: slabs vs production (rounding) and time
    const size_t dyn = (2 * A * 64 + A) * 4;
    auto slabs = [&]() {
      std::vector<float> a((size_t)d.R * len_rnn), b((size_t)d.R * len1);
      CK(hipMemcpy(a.data(), w.slab_rnn, a.size() * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(b.data(), w.slab_fc1, b.size() * 4, hipMemcpyDeviceToHost));
      a.insert(a.end(), b.begin(), b.end());
      return a;
    };
    hipLaunchKernelGGL(gru_bwd_fused_kernel<768>, dim3(d.R), dim3(512), dyn, 0, d, rp, (const float*)P0, L, w, len_rnn, len1);
    CK(hipDeviceSynchronize());
    const std::vector<float> ref = slabs();
    hipLaunchKernelGGL(gru_bwd_w1_kernel<0>, dim3(d.R), dim3(512), dyn, 0, d, rp, (const float*)P0, L, w, len_rnn, len1);
    CK(hipDeviceSynchronize());
    const std::vector<float> got = slabs();
    // per region: w_ih, w_hh, b_ih, b_hh, fc2.w, fc2.b of every row slab, then fc1 slabs
    double mx = 0, md = 0;
    size_t worst = 0;
    for (size_t i = 0; i < ref.size(); ++i) {
      mx = std::max(mx, (double)fabsf(ref[i]));
      const double dd = fabs((double)ref[i] - got[i]);
      if (dd > md) { md = dd; worst = i; }
    }
    printf("W1 vs production slabs: max |diff| %.3e of max |ref| %.3e (rel %.2e) at %zu (ref %.6e got %.6e)\n", md, mx,
           md / mx, worst, ref[worst], got[worst]);
    printf("fused bwd W1 %.1f us | production %.1f us\n",
           runb(gru_bwd_w1_kernel<0>), runb(gru_bwd_fused_kernel<768>));
  }
  {  // one-wave chain prototype (timing only)
    std::vector<int64_t> ta((int64_t)(T + 1) * d.R);
    for (auto& a : ta) a = rand() % A;
    int64_t* dta; CK(hipMalloc(&dta, ta.size() * 8)); CK(hipMemcpy(dta, ta.data(), ta.size() * 8, hipMemcpyHostToDevice));
    float* o1; CK(hipMalloc(&o1, (int64_t)d.R * 64 * 4));
    auto runp = [&](auto kern) {
      return time_med([&] { hipLaunchKernelGGL(kern, dim3(d.R), dim3(512), 0, 0, d, (const float*)P0, L, w, (const int64_t*)dta, o1); });
    };
    printf("one-wave chain prototype: NACC 2 %.1f us | 4 %.1f us | 8 %.1f us\n", runp(w1_chain_proto<2>),
           runp(w1_chain_proto<4>), runp(w1_chain_proto<8>));
  }
  hipLaunchKernelGGL(gru_bwd_fused_kernel<772 + 8192>, dim3(d.R), dim3(512), dyn, 0, d, rp, (const float*)P0, L, w, len_rnn, len1);
  CK(hipDeviceSynchronize());
  bwd_budget("producers idle");
  return 0;
}
