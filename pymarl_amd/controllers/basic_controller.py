"""BasicMAC: parameter-shared multi-agent controller (reference: src/controllers/basic_controller.py:10-154).

`forward(ep_batch, t)` is one fused HIP step (`mq_mac_forward`): it builds [obs_t | onehot(a_{t-1}) | onehot(id)]
from the replay rows in-kernel (basic_controller.py:100-135) and runs fc1 -> GRUCell -> fc2 for every
(episode, agent) row. For agent_output_type "pi_logits" (COMA) a second HIP kernel (`mc_policy`) applies the
reference's -1e10 mask, softmax and epsilon floor in place (basic_controller.py:53-73).

A host-resident batch (the reference ParallelRunner's batch under buffer_cpu_only, parallel_runner.py:45) is read
the reference's way: the step's rows go to the device first (basic_controller.py:105-115, `.to(self.args.device)`),
and `forward` returns its output on the batch's device (:75); `select_actions` keeps it on the device (:30-38).
"""
from types import SimpleNamespace as SN

import torch as th

from .. import _lib
from ..components.action_selectors import REGISTRY as action_REGISTRY
from ..modules.agents import REGISTRY as agent_REGISTRY


def _on_device(ep_batch):
    return th.device(ep_batch.device).type == "cuda"


class BasicMAC:
    def __init__(self, scheme, groups, args):
        self.n_agents = args.n_agents
        self.args = args
        input_shape = self._get_input_shape(scheme)
        self._build_agents(input_shape)
        self.agent_output_type = args.agent_output_type
        self.action_selector = action_REGISTRY[args.action_selector](args)
        self.hidden_states = None

    def select_actions(self, ep_batch, t_ep, t_env, bs=slice(None), test_mode=False):
        agent_outputs = self._forward(ep_batch, t_ep, test_mode=test_mode)
        avail_actions = ep_batch["avail_actions"][:, t_ep].to(agent_outputs.device)
        return self.action_selector.select_action(agent_outputs[bs], avail_actions[bs], t_env, test_mode=test_mode)

    def forward(self, ep_batch, t, test_mode=False):
        out = self._forward(ep_batch, t, test_mode)
        return out if _on_device(ep_batch) else out.to(ep_batch.device)   # basic_controller.py:75

    @staticmethod
    def _device_step(ep_batch, t, device):
        """The slots one MAC step reads (obs at t; actions / filled at t - 1 for the last-action one-hot) of a
        host-resident batch, copied to `device` as a two-slot dense batch; returns (batch, t within it)."""
        from ..components.episode_buffer import EpisodeBatch
        t0 = max(0, t - 1)
        data = {k: ep_batch[k][:, t0:t0 + 2].contiguous().to(device) for k in ("obs", "actions", "filled")}
        Tw = data["obs"].shape[1]
        return EpisodeBatch(ep_batch.scheme, ep_batch.groups, ep_batch.batch_size, Tw,
                            data=SN(transition_data=data, episode_data={}), device=device), t - t0

    def _forward(self, ep_batch, t, test_mode=False):
        if self.agent_output_type not in ("q", "pi_logits"):
            raise NotImplementedError("agent_output_type {!r}".format(self.agent_output_type))
        from ..learners.q_learner import replay_view
        dev = self.agent.fc1.weight.device
        _lib.require_gpu(self.agent.fc1.weight)
        t_run = t
        if not _on_device(ep_batch):   # host-resident (buffer_cpu_only): the step's rows to the device
            ep_view, t_run = self._device_step(ep_batch, t, dev)
        else:
            ep_view = ep_batch
        rep, keep = replay_view(ep_view)
        bs = ep_batch.batch_size
        H = self.args.rnn_hidden_dim
        h_in = self.hidden_states.reshape(bs * self.n_agents, H).float().contiguous()
        _lib.require_gpu(h_in)
        h_out = th.empty_like(h_in)
        q = th.empty(bs * self.n_agents, self.args.n_actions, dtype=th.float32, device=h_in.device)
        hd = self.agent.handle()
        _lib.check(hd.lib.mq_mac_forward(hd.h, rep, int(t_run), _lib.ptr(h_in), _lib.ptr(h_out), _lib.ptr(q), 0,
                                         _lib.stream_ptr()))
        del keep
        self.hidden_states = h_out.view(bs, self.n_agents, H)
        if self.agent_output_type == "pi_logits":
            avail = ep_batch["avail_actions"][:, t].to(device=dev, dtype=th.int32).contiguous()
            eps = float(self.action_selector.epsilon)
            _lib.check(hd.lib.mc_policy(_lib.ptr(q), _lib.ptr(avail), q.shape[0], q.shape[1], eps,
                                        int(bool(getattr(self.args, "mask_before_softmax", True))),
                                        int(bool(test_mode)), _lib.stream_ptr()))
        return q.view(bs, self.n_agents, -1)

    def init_hidden(self, batch_size):
        self.hidden_states = self.agent.init_hidden().unsqueeze(0).expand(batch_size, self.n_agents, -1)

    def parameters(self):
        return self.agent.parameters()

    def load_state(self, other_mac):
        self.agent.load_state_dict(other_mac.agent.state_dict())

    def cuda(self):
        self.agent.cuda()

    def save_models(self, path):
        th.save(self.agent.state_dict(), "{}/agent.th".format(path))

    def load_models(self, path):
        self.agent.load_state_dict(th.load("{}/agent.th".format(path), map_location=lambda s, loc: s,
                                           weights_only=True))

    def _build_agents(self, input_shape):
        self.agent = agent_REGISTRY[self.args.agent](input_shape, self.args)

    def _get_input_shape(self, scheme):
        """basic_controller.py:137-154, without mutating `scheme` (the reference's in-place int->tuple rewrite of
        scheme["obs"]["vshape"] is what breaks COMACritic)."""
        vs = scheme["obs"]["vshape"]
        obs = vs if isinstance(vs, int) else int(vs[0])
        width = obs
        if self.args.obs_last_action:
            oh = scheme["actions_onehot"]["vshape"]
            width += oh if isinstance(oh, int) else int(oh[0])
        if self.args.obs_agent_id:
            width += self.n_agents
        return (width,)
