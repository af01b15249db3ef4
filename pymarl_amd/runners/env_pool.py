"""Environment groups behind the batched rollout loop (pymarl_amd/runners/rollout.py).

Both groups expose the same four calls, so one loop drives either:
  reset()              -> per env: (state, avail_actions, obs)
  step(idx, actions)   -> per stepped env: (reward, terminated, info, state, avail_actions, obs)
  env_info() / stats() / close()

`InProcessEnvs` wraps one env object in the learner's process (EpisodeRunner, reference
src/runners/episode_runner.py). `WorkerEnvs` runs one env per worker process and talks to it over a Pipe
(ParallelRunner, reference src/runners/parallel_runner.py:11-26, env_worker :217-256): the host cores step the
environments while the parent runs the batched HIP MAC step on the GPU. Workers are started with the "spawn"
method: a fresh interpreter per worker, so no worker ever inherits the parent's HIP context.
"""
from __future__ import annotations

import multiprocessing as mp
import pickle

import numpy as np

# worker opcodes
_RESET, _STEP, _INFO, _STATS, _CLOSE = range(5)


def _dumps(fn):
    try:
        import cloudpickle   # env constructors may be lambdas / partials of local functions
        return cloudpickle.dumps(fn)
    except ImportError:  # pragma: no cover
        return pickle.dumps(fn)


def _observe(env):
    return env.get_state(), env.get_avail_actions(), env.get_obs()


def _serve(conn, blob):
    """Worker loop: build the env from the pickled constructor, answer opcodes until _CLOSE."""
    env = pickle.loads(blob)()
    try:
        while True:
            op, arg = conn.recv()
            if op == _STEP:
                reward, terminated, info = env.step(arg)
                conn.send((reward, terminated, info) + _observe(env))
            elif op == _RESET:
                env.reset()
                conn.send(_observe(env))
            elif op == _INFO:
                conn.send(env.get_env_info())
            elif op == _STATS:
                conn.send(env.get_stats() if hasattr(env, "get_stats") else {})
            elif op == _CLOSE:
                env.close()
                break
            else:
                raise ValueError("unknown env-worker opcode {}".format(op))
    finally:
        conn.close()


class InProcessEnvs:
    """A single environment stepped in the calling process."""

    def __init__(self, env):
        self.env = env
        self.n = 1

    def env_info(self):
        return self.env.get_env_info()

    def reset(self):
        self.env.reset()
        return [_observe(self.env)]

    def step(self, idx, actions):
        assert list(idx) == [0]
        reward, terminated, info = self.env.step(actions[0])
        return [(reward, terminated, info) + _observe(self.env)]

    def stats(self):
        return [self.env.get_stats()] if hasattr(self.env, "get_stats") else [{}]

    def close(self):
        self.env.close()


class WorkerEnvs:
    """n environments, one per worker process; requests fan out to every addressed worker before any reply is
    read, so the envs step concurrently on the host cores."""

    def __init__(self, env_fn, n, start_method="spawn"):
        ctx = mp.get_context(start_method)
        self.n = int(n)
        pipes = [ctx.Pipe() for _ in range(self.n)]
        self.conns = [p[0] for p in pipes]
        blob = _dumps(env_fn)
        self.procs = [ctx.Process(target=_serve, args=(p[1], blob), daemon=True) for p in pipes]
        for p in self.procs:
            p.start()
        for p in pipes:
            p[1].close()   # the parent keeps only its end
        self._closed = False

    def _ask(self, idx, op, args=None):
        for j, i in enumerate(idx):
            self.conns[i].send((op, None if args is None else args[j]))
        return [self.conns[i].recv() for i in idx]

    def env_info(self):
        return self._ask([0], _INFO)[0]

    def reset(self):
        return self._ask(range(self.n), _RESET)

    def step(self, idx, actions):
        return self._ask(idx, _STEP, actions)

    def stats(self):
        return self._ask(range(self.n), _STATS)

    def close(self):
        if self._closed:
            return
        self._closed = True
        for c in self.conns:
            try:
                c.send((_CLOSE, None))
            except (BrokenPipeError, OSError):
                pass
        for p in self.procs:
            p.join(timeout=10)
            if p.is_alive():
                p.terminate()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def stack_pre(obs_list):
    """[(state, avail, obs)] -> the pre-transition update dict, one host array per field (one H2D copy each)."""
    return {"state": np.asarray([o[0] for o in obs_list]),
            "avail_actions": np.asarray([o[1] for o in obs_list]),
            "obs": np.asarray([o[2] for o in obs_list])}
