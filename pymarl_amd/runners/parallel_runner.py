"""ParallelRunner: batch_size_run environments, one per worker process on the host cores
(reference: src/runners/parallel_runner.py:11-214, env_worker :217-256).

The envs step concurrently in their workers while the parent runs one batched HIP MAC step per time step for all
running envs (BasicMAC.select_actions on the device-resident EpisodeBatch); only the chosen actions and the envs'
replies cross the process / host-device boundary. Loop, replay layout and stats: rollout.BatchRollout.
"""
from functools import partial

from ..components.episode_buffer import EpisodeBatch
from ..envs import REGISTRY as env_REGISTRY
from .env_pool import WorkerEnvs
from .rollout import BatchRollout


class ParallelRunner(BatchRollout):
    def __init__(self, args, logger):
        env_fn = partial(env_REGISTRY[args.env], **args.env_args)
        self._init_rollout(args, logger, WorkerEnvs(env_fn, args.batch_size_run,
                                                    getattr(args, "worker_start_method", "spawn")))

    def setup(self, scheme, groups, preprocess, mac):
        device = "cpu" if getattr(self.args, "buffer_cpu_only", False) else self.args.device
        self.new_batch = partial(EpisodeBatch, scheme, groups, self.batch_size, self.episode_limit + 1,
                                 preprocess=preprocess, device=device)
        self.mac = mac
        self.scheme, self.groups, self.preprocess = scheme, groups, preprocess

    def save_replay(self):
        pass
