import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from tests.golden_utils import Case
from tests.gpu_helpers import build, rel
c = Case("tiny_qmix_full")
args, buf, mac, learner, logger = build(c)
np.random.seed(c.sampler_seed)
b = buf.sample(c.B); b = b[:, :b.max_t_filled()]
learner.train(b, 0, 0)
mo = learner.last_intermediate(0).cpu().numpy()
ref = c.z["step0_mac_out"]
print("rel", rel(mo, ref))
err = np.abs(mo - ref).max(axis=(0, 2, 3))
print("per-t max err", np.round(err, 5))
print(mo[0, 1, 0, :5], ref[0, 1, 0, :5])
