"""Per-step drift of the HIP learner vs the golden reference trajectory and vs the numpy oracle in lockstep."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from tests.golden_utils import Case
from tests.gpu_helpers import build, flat_params, flat_grads, rel
from oracle.qlearner_np import OracleQLearner

name = sys.argv[1] if len(sys.argv) > 1 else "cfg2_qmix"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
c = Case(name)
args, buf, mac, learner, logger = build(c)
o = OracleQLearner(c.agent_params, c.mixer_params, c.cfg())
np.random.seed(c.sampler_seed)
for k in range(min(steps, c.steps)):
    batch = buf.sample(c.B)
    mt = batch.max_t_filled()
    batch = batch[:, :mt]
    nb, _ = c.batch(k)
    fw = o.forward(nb)
    st_o = o.train(nb, 1000 * k, c.episodes[k])
    p_before = flat_params(learner)
    learner.train(batch, 1000 * k, c.episodes[k])
    st = learner.last_stats()
    mo = learner.last_intermediate(0).cpu().numpy()
    cm = learner.last_cur_max_actions().cpu().numpy()
    g_gpu = flat_grads(learner)
    g_or = np.concatenate([v.ravel() for v in o.last["grads"].values()])
    print(f"step {k}: loss gpu {st['loss']:.7f} oracle {st_o['loss']:.7f} ref {c.z['stat_loss'][k]:.7f} | "
          f"rel(gpu,ref) {abs(st['loss']-c.z['stat_loss'][k])/c.z['stat_loss'][k]:.2e} "
          f"gn {st['grad_norm']:.5f}/{st_o['grad_norm']:.5f} macout-rel {rel(mo, fw['mac_out']):.2e} "
          f"curmax-mismatch {(cm != fw['cur_max_actions']).sum()} grad-rel {rel(g_gpu, g_or):.2e} "
          f"param-rel {rel(flat_params(learner), o.flat()):.2e}")
    # worst param blocks
    offs = np.cumsum([0] + [v.size for v in list(o.p.values()) + list(o.mp.values())])
    names = list(o.p.keys()) + list(o.mp.keys())
    errs = [(rel(g_gpu[offs[i]:offs[i+1]], g_or[offs[i]:offs[i+1]]), names[i]) for i in range(len(names))]
    print("   grad rel per tensor:", " ".join(f"{n}:{e:.1e}" for e, n in errs))
