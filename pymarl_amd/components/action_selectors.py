"""Action selectors (reference: src/components/action_selectors.py:8-65).

The greedy branch of EpsilonGreedyActionSelector (masked argmax, first index on ties) runs as the HIP
`mq_greedy_actions` kernel; the epsilon-random branch stays on torch's RNG as in the reference (:57-59), since
parity is defined on greedy actions only (SURVEY.md §7 "Host RNG").
"""
import torch as th
from torch.distributions import Categorical

from .. import _lib
from .epsilon_schedules import DecayThenFlatSchedule

REGISTRY = {}


def greedy_actions(q, avail):
    """argmax_a q[..., a] over avail[..., a] != 0 (unavailable = -inf) on the GPU kernel. q (..., A)."""
    _lib.require_gpu(q)
    lib = _lib.load()
    A = q.shape[-1]
    qf = q.detach().contiguous().float()
    av = avail.to(dtype=th.int32).contiguous()
    out = th.empty(qf.shape[:-1], dtype=th.int64, device=q.device)
    rows = out.numel()
    _lib.check(lib.mq_greedy_actions(_lib.ptr(qf), _lib.ptr(av), _lib.ptr(out), rows, A, _lib.stream_ptr()))
    return out


class MultinomialActionSelector:
    def __init__(self, args):
        self.args = args
        self.schedule = DecayThenFlatSchedule(args.epsilon_start, args.epsilon_finish, args.epsilon_anneal_time,
                                              decay="linear")
        self.epsilon = self.schedule.eval(0)
        self.test_greedy = getattr(args, "test_greedy", True)

    def select_action(self, agent_inputs, avail_actions, t_env, test_mode=False):
        masked = agent_inputs.clone()
        masked[avail_actions == 0.0] = 0.0
        self.epsilon = self.schedule.eval(t_env)
        if test_mode and self.test_greedy:
            return masked.max(dim=2)[1]
        return Categorical(masked).sample().long()


REGISTRY["multinomial"] = MultinomialActionSelector


class EpsilonGreedyActionSelector:
    def __init__(self, args):
        self.args = args
        self.schedule = DecayThenFlatSchedule(args.epsilon_start, args.epsilon_finish, args.epsilon_anneal_time,
                                              decay="linear")
        self.epsilon = self.schedule.eval(0)

    def select_action(self, agent_inputs, avail_actions, t_env, test_mode=False):
        self.epsilon = self.schedule.eval(t_env)
        if test_mode:
            self.epsilon = 0.0
        greedy = greedy_actions(agent_inputs, avail_actions)
        # both draws happen in test mode too (epsilon 0), as in the reference (:57-59): the torch RNG stream then
        # stays the reference's across interleaved test episodes
        random_numbers = th.rand_like(agent_inputs[:, :, 0])
        pick_random = (random_numbers < self.epsilon).long()
        random_actions = Categorical(avail_actions.float()).sample().long()
        return pick_random * random_actions + (1 - pick_random) * greedy


REGISTRY["epsilon_greedy"] = EpsilonGreedyActionSelector
