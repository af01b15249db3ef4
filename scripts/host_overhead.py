"""Host-side cost of one QLearner.train() at cfg2 versus the GPU step: wall time per step for K steps without a
sync inside the loop (the bench's timed region), and the host time spent inside train() alone (GPU queue kept
full), to see whether the host keeps ahead of the GPU. Usage: python scripts/host_overhead.py [cfg2]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch as th

import bench


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg2"
    args, buf, learner, data = bench.build_workload(cfg, th.device("cuda:0"))
    B = bench.CONFIGS[cfg][6]
    np.random.seed(2)

    def step(k, host_times=None):
        gb = buf.sample(B)
        batch = gb[:, :gb.max_t_filled()]
        t0 = time.perf_counter()
        learner.train(batch, t_env=1000 * k, episode_num=8 * k)
        if host_times is not None:
            host_times.append(time.perf_counter() - t0)

    for k in range(10):
        step(k)
    th.cuda.synchronize()
    for K in (20, 50, 200):
        th.cuda.synchronize()
        t0 = time.perf_counter()
        ht = []
        for k in range(K):
            step(k, ht)
        t1 = time.perf_counter()
        th.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"K={K}: wall {1e3 * (t2 - t0) / K:.4f} ms/step, host loop {1e3 * (t1 - t0) / K:.4f} ms/step, "
              f"train() median {1e3 * np.median(ht):.4f} ms, max {1e3 * max(ht):.3f} ms", flush=True)
    if os.environ.get("HOST_PROFILE"):
        import cProfile
        import pstats
        pr = cProfile.Profile()
        pr.enable()
        for k in range(200):
            step(k)
        pr.disable()
        th.cuda.synchronize()
        pstats.Stats(pr).sort_stats("tottime").print_stats(22)
    # with a sync after every step: GPU step + launch latency
    ts = []
    for k in range(50):
        th.cuda.synchronize()
        t0 = time.perf_counter()
        step(k)
        th.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    print(f"synced per step: median {1e3 * np.median(ts):.4f} ms", flush=True)


if __name__ == "__main__":
    main()
