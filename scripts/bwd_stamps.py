"""Decode the fused BPTT's stamps (MQ_DIAG=bwd_stamp=<file>, gru_bwd_fused.hpp STAMP) of the last train(): cycles
(s_memtime ticks) from kernel entry of the prologue, the chain's T loop, the producers' tail and the slab writes,
and the chain's per-step cost. Usage: python scripts/bwd_stamps.py <file> <Tp>"""
import sys
import numpy as np

BSTH = 16
BSTN = BSTH + 152
path, Tp = sys.argv[1], int(sys.argv[2])
a = np.fromfile(path, dtype=np.uint32)[-8 * BSTN:].reshape(8, BSTN).astype(np.int64)
rel = (a - a[:, :1]) % (1 << 32)
print("per block (mean of 8): chain past the prologue %.0f, chain loop end %.0f, producers' tail done %.0f, slabs "
      "written %.0f, kernel end %.0f cycles" % tuple(rel[:, i].mean() for i in (1, 2, 3, 4, 5)))
print("producer tail: dW_hh(0) %.0f, its slab issued %.0f, barrier %.0f, dW_ih(0) %.0f, its slab issued %.0f, dX1(0) "
      "%.0f" % tuple(rel[:, i].mean() for i in (6, 7, 8, 9, 10, 11)))
steps = rel[:, BSTH:BSTH + Tp]
per = np.diff(steps, axis=1)
print("chain step cycles: mean %.0f, median %.0f, first %.0f; by chunk (16 steps from the top):" %
      (per.mean(), np.median(per), (steps[:, 0] - rel[:, 1]).mean()),
      [int(per[:, i:i + 16].mean()) for i in range(0, per.shape[1], 16)])
