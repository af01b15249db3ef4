"""Experiment (round 6): the row-pair forward's stamps with a replay buffer of only `n` episodes (all of it hot in
L2 / MALL, few pages) against the bench's 5000-episode buffer, to tell the replay gathers' start-up latency (TLB /
HBM) apart from the rest of the prologue. Usage: MQ_DIAG=pair_stamp=<file> python scripts/exp_hot_replay.py n"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch as th

import bench

n = int(sys.argv[1])
dev = th.device("cuda:0")
args, buf, learner, data = bench.build_workload("cfg2", dev, n_episodes=n, unique=min(n, 512))
np.random.seed(2)
for k in range(6):
    gb = buf.sample(32)
    learner.train(gb[:, :gb.max_t_filled()], t_env=1000 * k, episode_num=8 * k)
th.cuda.synchronize()
print("done", n)
