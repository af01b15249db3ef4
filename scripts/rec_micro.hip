// Microbenchmark of the persistent GRU recurrence kernels at a given (B, n, T) with random data.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/rec_micro.hip -o /tmp/rec_micro && /tmp/rec_micro 32 8 120
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../pymarl_amd/csrc/gru_bwd_fused.hpp"
#include "../pymarl_amd/csrc/hyper_kernel.hpp"
#include "../pymarl_amd/csrc/dwh_kernel.hpp"
using namespace mq;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

template <class F> float time_it(F f, int reps = 20) {
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  f(); CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) f();
  CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps * 1000.0f;   // us
}

float* dev_rand(size_t n, float scale) {
  std::vector<float> h(n);
  for (auto& x : h) x = scale * ((rand() / (float)RAND_MAX) * 2.0f - 1.0f);
  float* d; CK(hipMalloc(&d, n * 4)); CK(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice));
  return d;
}

__global__ void empty_kernel(float* p) {
  if (p && threadIdx.x == 0 && blockIdx.x == 0) p[0] = 1.0f;
}

int main(int argc, char** argv) {
  int B = argc > 1 ? atoi(argv[1]) : 32, n = argc > 2 ? atoi(argv[2]) : 8, T = argc > 3 ? atoi(argv[3]) : 120;
  int A = 14, O = 80;
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
  {  // QMIX mixer params (for the hypernet kernel)
    const int E = 32, S = d.S;
    sz[MQ_P_HW1_W] = (int64_t)E * n * S; sz[MQ_P_HW1_B] = E * n; sz[MQ_P_HWF_W] = (int64_t)E * S; sz[MQ_P_HWF_B] = E;
    sz[MQ_P_HB1_W] = (int64_t)E * S; sz[MQ_P_HB1_B] = E; sz[MQ_P_V0_W] = (int64_t)E * S; sz[MQ_P_V0_B] = E;
    sz[MQ_P_V2_W] = E; sz[MQ_P_V2_B] = 1;
  }
  for (int i = 0; i < MQ_P_COUNT; ++i) { L.o[i] = o; o += sz[i]; }
  L.o[MQ_P_COUNT] = o;
  float* P0 = dev_rand(o, 0.12f);
  float* P1 = dev_rand(o, 0.12f);
  Work w{};
  w.GI = dev_rand(2 * RT * 192, 1.0f);
  CK(hipMalloc(&w.Hs, 2 * RT * 64 * 4)); CK(hipMalloc(&w.Gates, RT * 256 * 4)); CK(hipMalloc(&w.Q, 2 * RT * A * 4));
  auto run = [&](auto kern, int rw) {
    dim3 grid((d.R + rw - 1) / rw, 2);
    return time_it([&] { hipLaunchKernelGGL(kern, grid, dim3(256), 0, 0, d, (const float*)P0, (const float*)P1, L, w); });
  };
  printf("B=%d n=%d T=%d rows=%d\n", B, n, T, d.R);
  printf("fwd RW1 %.1f us\n", run(gru_fwd_kernel<1, 0>, 1));
  printf("fwd RW1 V1(no Hs/Gates st) %.1f us\n", run(gru_fwd_kernel<1, 1>, 1));
  {
    CK(hipMalloc(&w.slab_mix, 2 * 8 * 2 * d.R));
    run(gru_fwd_kernel<1, 2>, 1);
    std::vector<uint64_t> st(2 * 2 * d.R);
    CK(hipMemcpy(st.data(), w.slab_mix, st.size() * 8, hipMemcpyDeviceToHost));
    double cyc = 0, tick = 0;
    for (int i = 0; i < 2 * d.R; ++i) { cyc += st[2 * i]; tick += st[2 * i + 1]; }
    cyc /= 2 * d.R; tick /= 2 * d.R;
    printf("fwd RW1 stamped: %.0f cycles/step, %.3f us/step, clock %.2f GHz\n", cyc / d.Tp, tick / 100.0 / d.Tp,
           cyc / (tick * 10.0));
  }
  printf("fwd RW2 %.1f us\n", run(gru_fwd_kernel<2, 0>, 2));
  printf("fwd RW4 %.1f us\n", run(gru_fwd_kernel<4, 0>, 4));
  printf("fwd RW8 %.1f us\n", run(gru_fwd_kernel<8, 0>, 8));
  // backward
  CK(hipMalloc(&w.X1, RT * 64 * 4)); CK(hipMemset(w.X1, 0, RT * 64 * 4));
  w.dch = dev_rand(RT, 0.1f);
  CK(hipMalloc(&w.dGI, RT * 192 * 4));
  int64_t len_rnn = L.o[MQ_P_FC2_B] + A - L.o[MQ_P_RNN_W_IH];
  CK(hipMalloc(&w.slab_rnn, (int64_t)d.R * len_rnn * 4));
  std::vector<int64_t> acts((int64_t)B * (T + 1) * n);
  for (auto& a : acts) a = rand() % A;
  int64_t* dacts; CK(hipMalloc(&dacts, acts.size() * 8)); CK(hipMemcpy(dacts, acts.data(), acts.size() * 8, hipMemcpyHostToDevice));
  Rep rp{}; rp.actions = dacts;
  auto runb = [&](auto kern, int rw) {
    size_t dyn = (2 * A * 64 + A) * 4;
    return time_it([&] { hipLaunchKernelGGL(kern, dim3((d.R + rw - 1) / rw), dim3(512), dyn, 0, d, rp, (const float*)P0, L, w, len_rnn); });
  };
  {  // fused agent forward (fc1 / W_ih / fc2 on MFMA inside the recurrence)
    float* obs = dev_rand((int64_t)B * (T + 1) * n * O, 1.0f);
    std::vector<int64_t> fl((int64_t)B * (T + 1), 1);
    int64_t* dfl; CK(hipMalloc(&dfl, fl.size() * 8)); CK(hipMemcpy(dfl, fl.data(), fl.size() * 8, hipMemcpyHostToDevice));
    Rep rf = rp; rf.obs = obs; rf.filled = dfl;
    CK(hipMalloc(&w.XIN, RT * d.I * 4));
    auto runf = [&](auto kern) {
      return time_it([&] { hipLaunchKernelGGL(kern, dim3(d.R, 2), dim3(512), 0, 0, d, rf, (const float*)P0, (const float*)P1, L, w); });
    };
    printf("fused fwd %.1f us\n", runf(gru_fwd_fused_kernel<0, 5>));
    {
      auto run1 = [&]() {
        return time_it([&] { hipLaunchKernelGGL((gru_fwd_fused_kernel<0, 5>), dim3(d.R, 1), dim3(512), 0, 0, d, rf, (const float*)P0, (const float*)P1, L, w); });
      };
      std::vector<float> a, b;
      for (int round = 0; round < 7; ++round) { a.push_back(runf(gru_fwd_fused_kernel<0, 5>)); b.push_back(run1()); }
      std::sort(a.begin(), a.end()); std::sort(b.begin(), b.end());
      printf("fused fwd both nets median %.1f us | online net only (grid R x 1) median %.1f us\n", a[3], b[3]);
    }
    {  // interleaved rounds (one process): median / min per variant
      const char* names[] = {"V0 (prio)", "V128 no prio", "V512 rebal", "V640 rebal no prio", "V1536 tprio+rebal"};
      std::vector<std::vector<float>> ts(5);
      for (int round = 0; round < 9; ++round) {
        ts[0].push_back(runf(gru_fwd_fused_kernel<0, 5>));
        ts[1].push_back(runf(gru_fwd_fused_kernel<128, 5>));
        ts[2].push_back(runf(gru_fwd_fused_kernel<512, 5>));
        ts[3].push_back(runf(gru_fwd_fused_kernel<640, 5>));
        ts[4].push_back(runf(gru_fwd_fused_kernel<1536, 5>));
      }
      for (int v = 0; v < 5; ++v) {
        std::sort(ts[v].begin(), ts[v].end());
        printf("fused fwd %-20s median %.1f us min %.1f us\n", names[v], ts[v][ts[v].size() / 2], ts[v][0]);
      }
    }
    printf("fused fwd V1(no Hs/Gates st) %.1f us\n", runf(gru_fwd_fused_kernel<1, 5>));
    printf("fused fwd V4(no chunk pipeline) %.1f us\n", runf(gru_fwd_fused_kernel<4, 5>));
    printf("fused fwd V5 %.1f us\n", runf(gru_fwd_fused_kernel<5, 5>));
    printf("fused fwd V128(no chain prio) %.1f us\n", runf(gru_fwd_fused_kernel<128, 5>));
    printf("fused fwd V256(early gather) %.1f us\n", runf(gru_fwd_fused_kernel<256, 5>));
    printf("fused fwd V384(early gather, no prio) %.1f us\n", runf(gru_fwd_fused_kernel<384, 5>));
    printf("fused fwd V640(rebalanced, no prio) %.1f us\n", runf(gru_fwd_fused_kernel<640, 5>));
    printf("fused fwd V512(rebalanced) %.1f us\n", runf(gru_fwd_fused_kernel<512, 5>));
    printf("fused fwd V1536(target prio+rebalanced) %.1f us\n", runf(gru_fwd_fused_kernel<1536, 5>));
    printf("fused fwd V1280(target prio+early) %.1f us\n", runf(gru_fwd_fused_kernel<1280, 5>));
    for (int var : {130, 258, 642, 1538}) {
      if (var == 130) runf(gru_fwd_fused_kernel<130, 5>);
      else if (var == 258) runf(gru_fwd_fused_kernel<258, 5>);
      else if (var == 642) runf(gru_fwd_fused_kernel<642, 5>);
      else runf(gru_fwd_fused_kernel<1538, 5>);
      std::vector<uint64_t> sv(2 * 2 * d.R);
      CK(hipMemcpy(sv.data(), w.slab_mix, sv.size() * 8, hipMemcpyDeviceToHost));
      for (int net = 0; net < 2; ++net) {
        double cn = 0;
        for (int i = net * d.R; i < (net + 1) * d.R; ++i) cn += sv[2 * i];
        printf("  V%d net %d loop: %.0f cycles/step\n", var, net, cn / d.R / d.Tp);
      }
    }
    runf(gru_fwd_fused_kernel<2, 5>);
    std::vector<uint64_t> st(2 * 2 * d.R);
    CK(hipMemcpy(st.data(), w.slab_mix, st.size() * 8, hipMemcpyDeviceToHost));
    double cyc = 0, tick = 0;
    for (int i = 0; i < 2 * d.R; ++i) { cyc += st[2 * i]; tick += st[2 * i + 1]; }
    cyc /= 2 * d.R; tick /= 2 * d.R;
    printf("fused fwd stamped: %.0f cycles/step, %.3f us/step\n", cyc / d.Tp, tick / 100.0 / d.Tp);
    for (int net = 0; net < 2; ++net) {
      double cn = 0, tn = 0;
      for (int i = net * d.R; i < (net + 1) * d.R; ++i) { cn += st[2 * i]; tn += st[2 * i + 1]; }
      printf("  net %d loop: %.0f cycles/step, %.3f us/step\n", net, cn / d.R / d.Tp, tn / d.R / 100.0 / d.Tp);
    }
    runf(gru_fwd_fused_kernel<6, 5>);
    CK(hipMemcpy(st.data(), w.slab_mix, st.size() * 8, hipMemcpyDeviceToHost));
    cyc = 0; for (int i = 0; i < 2 * d.R; ++i) cyc += st[2 * i];
    printf("fused fwd V4 stamped: %.0f cycles/step\n", cyc / (2 * d.R) / d.Tp);
    {
      CK(hipFree(w.slab_mix)); CK(hipMalloc(&w.slab_mix, 16 * 8 * 2 * d.R));
      runf(gru_fwd_fused_kernel<64, 5>);
      std::vector<uint64_t> sb(16 * 2 * d.R);
      CK(hipMemcpy(sb.data(), w.slab_mix, sb.size() * 8, hipMemcpyDeviceToHost));
      uint64_t t0 = ~0ull;
      for (int i = 0; i < 2 * d.R; ++i) t0 = std::min(t0, sb[16 * i]);
      for (int net = 0; net < 2; ++net) {
        printf("fused prologue milestones net %d (us after the earliest WG start, mean / max over WGs):", net);
        for (int k = 0; k <= 8; ++k) {
          double m = 0, mx = 0;
          for (int i = net * d.R; i < (net + 1) * d.R; ++i) {
            double v = (sb[16 * i + k] - t0) / 100.0; m += v; mx = std::max(mx, v);
          }
          printf(" [%d] %.2f/%.2f", k, m / d.R, mx);
        }
        printf("\n");
      }
    }
    for (int var : {8, 12, 136, 264, 648, 1544}) {
      CK(hipFree(w.slab_mix)); CK(hipMalloc(&w.slab_mix, 16 * 8 * 2 * d.R));
      if (var == 8) runf(gru_fwd_fused_kernel<8, 5>);
      else if (var == 12) runf(gru_fwd_fused_kernel<12, 5>);
      else if (var == 136) runf(gru_fwd_fused_kernel<136, 5>);
      else if (var == 264) runf(gru_fwd_fused_kernel<264, 5>);
      else if (var == 648) runf(gru_fwd_fused_kernel<648, 5>);
      else runf(gru_fwd_fused_kernel<1544, 5>);

      std::vector<uint64_t> sb(16 * 2 * d.R);
      CK(hipMemcpy(sb.data(), w.slab_mix, sb.size() * 8, hipMemcpyDeviceToHost));
      printf("fused V%d cycles per step by phase p:", var);
      const int nch = (d.Tp + 15) / 16;
      for (int p = 0; p < 16; ++p) {
        double c = 0; for (int i = 0; i < 2 * d.R; ++i) c += sb[16 * i + p];
        const int cnt = nch - (p >= d.Tp - 16 * (nch - 1) ? 1 : 0);
        printf(" %.0f", c / (2 * d.R) / cnt);
      }
      printf("\n");
    }
  }
  {  // fused BPTT
    int64_t len1 = 64 * d.I + 64;
    CK(hipMalloc(&w.slab_fc1, (int64_t)d.R * len1 * 4));
    float* obs = dev_rand((int64_t)B * (T + 1) * n * O, 1.0f);
    Rep rf = rp; rf.obs = obs;
    if (!w.XIN) CK(hipMalloc(&w.XIN, RT * d.I * 4));
    CK(hipMemset(w.XIN, 0, RT * d.I * 4));
    auto runbf = [&](auto kern) {
      size_t dyn = (2 * A * 64 + A) * 4;
      return time_it([&] { hipLaunchKernelGGL(kern, dim3(d.R), dim3(512), dyn, 0, d, rf, (const float*)P0, L, w, len_rnn, len1); });
    };
    printf("fused bwd %.1f us\n", runbf(gru_bwd_fused_kernel<0>));
    printf("fused bwd V4(no producer MFMA) %.1f us\n", runbf(gru_bwd_fused_kernel<4>));
    printf("fused bwd V128(chain prio) %.1f us\n", runbf(gru_bwd_fused_kernel<128>));
    {
      std::vector<float> a, b;
      for (int round = 0; round < 9; ++round) {
        a.push_back(runbf(gru_bwd_fused_kernel<0>));
        b.push_back(runbf(gru_bwd_fused_kernel<128>));
      }
      std::sort(a.begin(), a.end()); std::sort(b.begin(), b.end());
      printf("fused bwd V0 median %.1f min %.1f | V128 median %.1f min %.1f\n", a[4], a[0], b[4], b[0]);
    }
    printf("fused bwd V768 %.1f us | V772 (producers idle) %.1f | V1792 (SIMD split) %.1f | V1796 %.1f\n",
           runbf(gru_bwd_fused_kernel<768>), runbf(gru_bwd_fused_kernel<772>), runbf(gru_bwd_fused_kernel<1792>),
           runbf(gru_bwd_fused_kernel<1796>));
    CK(hipFree(w.slab_mix)); CK(hipMalloc(&w.slab_mix, 32 * 8 * d.R));
    for (int var : {776, 780, 1800, 1804}) {
      if (var == 776) runbf(gru_bwd_fused_kernel<776>);
      else if (var == 780) runbf(gru_bwd_fused_kernel<780>);
      else if (var == 1800) runbf(gru_bwd_fused_kernel<1800>);
      else runbf(gru_bwd_fused_kernel<1804>);
      std::vector<uint64_t> sb(32 * d.R);
      CK(hipMemcpy(sb.data(), w.slab_mix, sb.size() * 8, hipMemcpyDeviceToHost));
      double tot = 0; for (int i = 0; i < d.R; ++i) tot += sb[32 * i + 16];
      printf("fused bwd V%d loop %.0f cycles/step; by phase u:", var, tot / d.R / d.Tp);
      const int nch = (d.Tp + 15) / 16;
      for (int u = 0; u < 16; ++u) {
        double c = 0; for (int i = 0; i < d.R; ++i) c += sb[32 * i + u];
        printf(" %.0f", c / d.R / nch);
      }
      printf("\n");
    }
  }
  {  // hypernet
    d.dS = make_fastdiv(d.S);
    float* state = dev_rand((int64_t)B * (T + 1) * d.S, 1.0f);
    Rep rh = rp; rh.state = state;
    float *HYPb, *S0b;
    CK(hipMalloc(&HYPb, (int64_t)2 * d.M * d.NH * 4)); CK(hipMalloc(&S0b, (int64_t)d.M * d.S * 4 + (1 << 20)));
    const size_t dynh = HyperGeom(d.S, d.NH).lds_bytes();
    dim3 gh((d.M + HYR - 1) / HYR, 2);
    printf("hyper %.1f us\n", time_it([&] { hipLaunchKernelGGL((hyper_kernel<0, 4>), gh, dim3(256), dynh, 0, d, rh, (const float*)P0, (const float*)P1, L, HYPb, S0b); }));
    {
      const size_t nh = (size_t)2 * d.M * d.NH;
      std::vector<float> h4(nh), h8(nh);
      hipLaunchKernelGGL((hyper_kernel<0, 4>), gh, dim3(256), dynh, 0, d, rh, (const float*)P0, (const float*)P1, L, HYPb, S0b);
      CK(hipMemcpy(h4.data(), HYPb, nh * 4, hipMemcpyDeviceToHost));
      CK(hipMemset(HYPb, 0, nh * 4));
      hipLaunchKernelGGL((hyper_kernel<0, 8>), gh, dim3(512), dynh, 0, d, rh, (const float*)P0, (const float*)P1, L, HYPb, S0b);
      CK(hipMemcpy(h8.data(), HYPb, nh * 4, hipMemcpyDeviceToHost));
      size_t bad = 0;
      for (size_t i = 0; i < nh; ++i) bad += h4[i] != h8[i];
      printf("hyper 4 vs 8 waves: %zu of %zu outputs differ\n", bad, nh);
      CK(hipMemset(HYPb, 0, nh * 4));
      hipLaunchKernelGGL(hyper_ws_kernel<0>, gh, dim3(HYWS_THREADS), hyper_ws_lds_bytes(d.S), 0, d, rh, (const float*)P0, (const float*)P1, L, HYPb, S0b);
      CK(hipMemcpy(h8.data(), HYPb, nh * 4, hipMemcpyDeviceToHost));
      bad = 0;
      double md = 0.0;
      for (size_t i = 0; i < nh; ++i) {
        bad += h4[i] != h8[i];
        md = std::max(md, (double)fabsf(h4[i] - h8[i]) / (1e-3 + fabsf(h4[i])));
      }
      printf("hyper 4 waves vs wave-specialised: %zu of %zu outputs differ, max rel diff %.2e\n", bad, nh, md);
    }
    printf("hyper 8 waves %.1f us\n", time_it([&] { hipLaunchKernelGGL((hyper_kernel<0, 8>), gh, dim3(512), dynh, 0, d, rh, (const float*)P0, (const float*)P1, L, HYPb, S0b); }));
    printf("hyper wave-specialised %.1f us\n", time_it([&] { hipLaunchKernelGGL(hyper_ws_kernel<0>, gh, dim3(HYWS_THREADS), hyper_ws_lds_bytes(d.S), 0, d, rh, (const float*)P0, (const float*)P1, L, HYPb, S0b); }));
    printf("hyper wave-specialised V2(chunk-0 weights only) %.1f us\n", time_it([&] { hipLaunchKernelGGL(hyper_ws_kernel<2>, gh, dim3(HYWS_THREADS), hyper_ws_lds_bytes(d.S), 0, d, rh, (const float*)P0, (const float*)P1, L, HYPb, S0b); }));
    printf("hyper wave-specialised V4(no MFMA) %.1f us, V8(no staging) %.1f us, V12 %.1f us\n",
      time_it([&] { hipLaunchKernelGGL(hyper_ws_kernel<4>, gh, dim3(HYWS_THREADS), hyper_ws_lds_bytes(d.S), 0, d, rh, (const float*)P0, (const float*)P1, L, HYPb, S0b); }),
      time_it([&] { hipLaunchKernelGGL(hyper_ws_kernel<8>, gh, dim3(HYWS_THREADS), hyper_ws_lds_bytes(d.S), 0, d, rh, (const float*)P0, (const float*)P1, L, HYPb, S0b); }),
      time_it([&] { hipLaunchKernelGGL(hyper_ws_kernel<12>, gh, dim3(HYWS_THREADS), hyper_ws_lds_bytes(d.S), 0, d, rh, (const float*)P0, (const float*)P1, L, HYPb, S0b); }));
    hipLaunchKernelGGL(hyper_ws_kernel<1>, gh, dim3(HYWS_THREADS), hyper_ws_lds_bytes(d.S), 0, d, rh, (const float*)P0, (const float*)P1, L, HYPb, S0b);
    CK(hipDeviceSynchronize());
    const int nb = gh.x * gh.y;
    std::vector<uint64_t> hs(32 * nb);
    CK(hipMemcpy(hs.data(), S0b, hs.size() * 8, hipMemcpyDeviceToHost));
    double mm[10] = {}, ll[9] = {};
    for (int i = 0; i < nb; ++i) {
      const uint64_t* r = &hs[32 * i];
      for (int k = 0; k < 10; ++k) mm[k] += (double)(int64_t)(r[k] - r[0]);
      for (int k = 0; k < 9; ++k) ll[k] += (double)(int64_t)(r[16 + k] - r[0]);
    }
    printf("hyper_ws stamps (cycles after the MFMA wave's start, mean over %d WGs)\n  MFMA wave: prologue done %.0f, after barrier c:", nb, mm[1] / nb);
    for (int k = 2; k < 8; ++k) printf(" %.0f", mm[k] / nb);
    printf(", end %.0f\n  loader   : start %.0f, at barrier c:", mm[9] / nb, ll[0] / nb);
    for (int k = 1; k < 7; ++k) printf(" %.0f", ll[k] / nb);
    printf(", end %.0f\n", ll[8] / nb);
  }
  {  // dW_hyper
    float* dH = dev_rand((int64_t)d.M * d.NH, 1.0f);
    float* S0d = dev_rand((int64_t)d.M * d.S, 1.0f);
    const int64_t len = L.o[MQ_P_V2_W] - L.o[MQ_P_HW1_W];
    float* slab; CK(hipMalloc(&slab, 128 * len * 4));
    const int tj = (d.NH + DWH_T - 1) / DWH_T, ts = (d.S + 1 + DWH_T - 1) / DWH_T;
    for (int nb : {1, 256, 528, 2048})
      printf("empty kernel, %d WGs: %.1f us\n", nb, time_it([&] { hipLaunchKernelGGL(empty_kernel, dim3(nb), dim3(256), 0, 0, slab); }));
    for (int ns : {8, 16, 32}) {
      auto go = [&](auto k) { return time_it([&] { hipLaunchKernelGGL(k, dim3(tj * ts * ns), dim3(256), 0, 0, d, L, (const float*)dH, (const float*)S0d, slab, len, ns, tj); }); };
      printf("dwh ns=%d: %.1f us, V1(no MFMA) %.1f, V2(no loads) %.1f, V3 %.1f\n", ns, go(dwh_kernel<0>), go(dwh_kernel<1>),
             go(dwh_kernel<2>), go(dwh_kernel<3>));
    }
  }
  printf("bwd RW1 %.1f us\n", runb(gru_bwd_kernel<1, 0>, 1));
  printf("bwd RW1 V4(cached inputs) %.1f us\n", runb(gru_bwd_kernel<1, 4>, 1));
  printf("bwd RW1 V8(no accumulate) %.1f us\n", runb(gru_bwd_kernel<1, 8>, 1));
  printf("bwd RW1 V12 %.1f us\n", runb(gru_bwd_kernel<1, 12>, 1));
  for (int var : {2, 14}) {
    if (var == 2) runb(gru_bwd_kernel<1, 2>, 1); else runb(gru_bwd_kernel<1, 14>, 1);
    std::vector<uint64_t> st(4 * d.R);
    CK(hipMemcpy(st.data(), w.slab_mix, st.size() * 8, hipMemcpyDeviceToHost));
    double c[3] = {0, 0, 0};
    for (int i = 0; i < d.R; ++i) for (int j = 0; j < 3; ++j) c[j] += st[4 * i + j];
    printf("bwd RW1 V%d stamped cycles/step: pre %.0f barrier %.0f post %.0f\n", var, c[0] / d.R / d.Tp,
           c[1] / d.R / d.Tp, c[2] / d.R / d.Tp);
  }
  printf("bwd RW2 %.1f us\n", runb(gru_bwd_kernel<2, 0>, 2));

  return 0;
}
