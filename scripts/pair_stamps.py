"""Decode the row-pair forward's stamps (MQ_DIAG=pair_stamp=<file>, gru_fwd_pair.hpp STAMP) of the last train(), cycles
(s_memtime ticks) from kernel entry: prologue, recurrence loop, epilogue; per-step cost inside a chunk and across a
chunk boundary; producers' slack at each chunk barrier. Usage: python scripts/pair_stamps.py <file> <Tp>"""
import sys
import numpy as np

PSH = 32
PST = PSH + 2 * 512
path, Tp = sys.argv[1], int(sys.argv[2])
a = np.fromfile(path, dtype=np.uint32)[-8 * PST:].reshape(8, PST).astype(np.int64)
rel = (a - a[:, :1]) % (1 << 32)
entry, lstart, lend, pro, kend = (rel[:, i] for i in range(5))
steps = rel[:, PSH:PSH + Tp]
print("per block (mean of 8): recurrence loop starts at %.0f, loop ends at %.0f, kernel ends at %.0f cycles" %
      (lstart.mean(), lend.mean(), kend.mean()))
per = np.diff(steps, axis=1)
t = np.arange(1, Tp)
ins = (t % 16) != 0
print("W_hh staging: wave 0 first loads issued %.0f, all stored %.0f; hypernet states staged %.0f; recurrence W_hh "
      "picked up %.0f" % tuple(rel[:, i].mean() for i in (10, 5, 3, 9)))
print("producer 0's prologue: entry loads issued %.0f, xin(0) %.0f, S1 %.0f, X1(0) + xin(1) %.0f, S2 %.0f, "
      "GI(0) + X1(1) + xin(2) %.0f" % tuple(rel[:, i].mean() for i in (16, 17, 18, 19, 20, 8)))
print("role entries: producer 0 %.0f (gather issued %.0f, net-0 W1 / W_ih issued %.0f), recurrence 0 %.0f, hypernet 0 "
      "%.0f (state loads issued %.0f)" % tuple(rel[:, i].mean() for i in (21, 22, 23, 24, 25, 26)))
print("hypernet waves (HYP=2): tiles done in the S1 / S2 / chunk-0 intervals %s, exit %.0f" %
      ([round(rel[:, 11 + i].mean()) for i in range(3)], rel[:, 15].mean()))
print("step cycles inside a chunk: mean %.0f, median %.0f; first step of a chunk: mean %.0f; step 0 ends %.0f after "
      "the loop start" % (per[:, ins].mean(), np.median(per[:, ins]), per[:, ~ins].mean(),
                          (steps[:, 0] - lstart).mean()))
last = np.arange(15, Tp, 16)
arr = rel[:, PSH + 512 + last]
print("producers' chunk-barrier arrival - recurrence's chunk end (cycles, + = producers late):",
      np.round((arr - steps[:, last]).mean(0)).astype(int).tolist())
