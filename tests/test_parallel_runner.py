"""ParallelRunner (batch_size_run worker processes over pipes, reference src/runners/parallel_runner.py:11-256) on the
synthetic FakeEnv writes exactly the batches the reference ParallelRunner writes (tests/golden/runner_parallel_fake.npz,
made by tests/golden/make_golden_runner.py with the same env arguments and the same seeded stub MAC): every field of
every run bit for bit (envs ending at different steps included), t_env after each run, and the logged stats. CPU."""
import os
from types import SimpleNamespace as SN

import numpy as np
import torch as th

from pymarl_amd.components.transforms import OneHot
from pymarl_amd.runners import REGISTRY as runner_REGISTRY
from tests.test_runner import FIELDS, N_ACTIONS, N_AGENTS, OBS, STATE, LIMIT, Logger, StubMAC, scheme

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "runner_parallel_fake.npz")
PAR_ENVS, PAR_RUNS, END_THRESHOLD = 4, 6, -0.9


class StubBatchMAC(StubMAC):
    def select_actions(self, ep_batch, t_ep, t_env, bs=slice(None), test_mode=False):
        avail = ep_batch["avail_actions"][bs, t_ep].cpu().numpy()
        keys = self.rng.random(avail.shape)
        keys[avail == 0] = -1.0
        return th.as_tensor(keys.argmax(-1), dtype=th.long)


def test_parallel_runner_matches_reference():
    z = np.load(GOLDEN, allow_pickle=False)
    args = SN(batch_size_run=PAR_ENVS, env="fake",
              env_args=dict(n_agents=N_AGENTS, n_actions=N_ACTIONS, obs_dim=OBS, state_dim=STATE,
                            episode_limit=LIMIT, seed=3, end_threshold=END_THRESHOLD),
              device="cpu", buffer_cpu_only=True, test_nepisode=4, runner_log_interval=25)
    logger = Logger()
    runner = runner_REGISTRY["parallel"](args, logger)
    try:
        assert runner.get_env_info()["episode_limit"] == LIMIT
        runner.setup(scheme(), {"agents": N_AGENTS}, {"actions": ("actions_onehot", [OneHot(out_dim=N_ACTIONS)])},
                     StubBatchMAC())
        lengths = set()
        for e in range(PAR_RUNS):
            b = runner.run(test_mode=(e == PAR_RUNS - 1))
            for k in FIELDS:
                got = b[k].numpy()
                ref = z["run{}_{}".format(e, k)]
                assert got.shape == ref.shape and got.dtype == ref.dtype, (e, k, got.shape, ref.shape)
                assert np.array_equal(got, ref), (e, k)
            assert runner.t_env == int(z["run{}_t_env".format(e)])
            lengths |= set(b["filled"].numpy().sum((1, 2)).tolist())
        assert len(lengths) > 1   # the envs of one run ended at different steps
    finally:
        runner.close_env()
    names = list(z["stat_names"])
    ref_stats = sorted((names[int(i)], int(t), v) for i, v, t in z["stats"])
    got_stats = sorted((k, t, v) for k, v, t in logger.stats)
    # the order of the per-key "_mean" stats follows a Python set (hash-seed dependent in the reference too)
    assert [(k, t) for k, t, _ in got_stats] == [(k, t) for k, t, _ in ref_stats]
    for (k, _, v), (_, _, rv) in zip(got_stats, ref_stats):
        assert abs(v - rv) <= 1e-6 * max(1.0, abs(rv)), (k, v, rv)
