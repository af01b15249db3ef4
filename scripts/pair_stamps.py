"""Decode the row-pair forward's step stamps (MQ_PAIR_STAMP=<file>, gru_fwd_pair.hpp STAMP): per chunk phase p, the
mean cycles from the previous barrier release to the recurrence wave's / producer wave's arrival, and the step period.
Usage: python scripts/pair_stamps.py <file> <Tp>"""
import sys
import numpy as np

path, Tp = sys.argv[1], int(sys.argv[2])
a = np.fromfile(path, dtype=np.uint32)
rec = 8 * 3 * Tp
a = a[-rec:].reshape(8, 3, Tp).astype(np.int64)   # last train(): [block][release, rec arrival, prod arrival][t]
rel, arr_r, arr_p = a[:, 0], a[:, 1], a[:, 2]
per = np.diff(rel, axis=1)                        # step t period (t >= 1)
rb = arr_r[:, 1:] - rel[:, :-1]                   # recurrence work of step t
pb = arr_p[:, 1:] - rel[:, :-1]                   # producer work of step t
print("mean step period %.0f cycles (median %.0f), first release -> last %.0f cycles" %
      (per.mean(), np.median(per), (rel[:, -1] - rel[:, 0]).mean()))
print(" p  period  rec_busy  prod_busy")
t = np.arange(1, Tp)
for p in range(16):
    sel = (t % 16) == p
    print("%2d  %6.0f  %8.0f  %9.0f" % (p, per[:, sel].mean(), rb[:, sel].mean(), pb[:, sel].mean()))
