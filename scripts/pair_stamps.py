"""Decode the row-pair forward's stamps (MQ_PAIR_STAMP=<file>, gru_fwd_pair.hpp STAMP) of the last train(): the
recurrence's cycles per step inside a chunk, across a chunk boundary, and how early or late the producers reach each
chunk barrier relative to the recurrence. Usage: python scripts/pair_stamps.py <file> <Tp>"""
import sys
import numpy as np

path, Tp = sys.argv[1], int(sys.argv[2])
a = np.fromfile(path, dtype=np.uint32)
a = a[-8 * 3 * Tp:].reshape(8, 3, Tp).astype(np.int64)   # [block][step end, rec chunk arrival, prod chunk arrival][t]
end, arr_r, arr_p = a[:, 0], a[:, 1], a[:, 2]
per = np.diff(end, axis=1)                                # cycles of step t (t >= 1)
t = np.arange(1, Tp)
inside, first = per[:, (t % 16) != 0], per[:, (t % 16) == 0]
last = np.arange(15, Tp, 16)
print("steps inside a chunk: mean %.0f, median %.0f cycles; first step of a chunk: mean %.0f" %
      (inside.mean(), np.median(inside), first.mean()))
print("whole T loop %.0f cycles (%d steps)" % ((end[:, -1] - end[:, 0]).mean(), Tp))
print("producer arrival - recurrence arrival at each chunk barrier (cycles, + = producers late):")
print(" ", np.round((arr_p[:, last] - arr_r[:, last]).mean(0)).astype(int).tolist())
