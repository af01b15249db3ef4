"""Quick COMA train() timing at the cfg5 (MMM2) shape on one GPU (development helper; bench.py --config cfg5 is
the reported measurement)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch as th  # noqa: E402

from bench import build_coma_workload  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
args, buf, learner, data, mac = build_coma_workload("cfg5", th.device("cuda", 0))
np.random.seed(2)
B = args.batch_size
for k in range(3):
    b = buf.sample(B)
    learner.train(b[:, :b.max_t_filled()], 1000 * k, 8 * k)
th.cuda.synchronize()
t0 = time.perf_counter()
for k in range(steps):
    b = buf.sample(B)
    learner.train(b[:, :b.max_t_filled()], 1000 * k, 8 * k)
th.cuda.synchronize()
dt = (time.perf_counter() - t0) / steps
print("coma cfg5: {:.3f} ms/train, {:.3e} samples/s".format(dt * 1e3, B * 180 * 10 / dt), learner.last_stats())
