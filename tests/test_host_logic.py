"""Host-side mirror of the reference interfaces (CPU): EpisodeBatch / ReplayBuffer semantics, SampledBatch
zero-copy views, parameter packing and checkpoint compatibility, and the no-CPU-fallback rule."""
import logging
import os
from types import SimpleNamespace as SN

import numpy as np
import pytest
import torch as th

from pymarl_amd import _lib
from pymarl_amd.components.episode_buffer import EpisodeBatch, ReplayBuffer, SampledBatch
from pymarl_amd.components.transforms import OneHot
from pymarl_amd.controllers import REGISTRY as mac_REGISTRY
from pymarl_amd.learners import REGISTRY as le_REGISTRY
from pymarl_amd.utils.logging import Logger
from pymarl_amd.utils.synthetic import agent_param_shapes, qmix_param_shapes


def scheme(O=3, A=5, S=4):
    return {
        "state": {"vshape": S},
        "obs": {"vshape": O, "group": "agents"},
        "actions": {"vshape": (1,), "group": "agents", "dtype": th.long},
        "avail_actions": {"vshape": (A,), "group": "agents", "dtype": th.int},
        "reward": {"vshape": (1,)},
        "terminated": {"vshape": (1,), "dtype": th.uint8},
    }


def args(mixer="qmix", n=2, A=5, O=3, S=4):
    return SN(n_agents=n, n_actions=A, state_shape=S, obs_shape=O, rnn_hidden_dim=64, mixing_embed_dim=32,
              mixer=mixer, lr=5e-4, optim_alpha=0.99, optim_eps=1e-5, grad_norm_clip=10.0, gamma=0.99,
              double_q=True, target_update_interval=200, learner_log_interval=0, obs_last_action=True,
              obs_agent_id=True, agent="rnn", mac="basic_mac", agent_output_type="q",
              action_selector="epsilon_greedy", epsilon_start=1.0, epsilon_finish=0.05, epsilon_anneal_time=50000,
              batch_size=3, device="cpu")


def test_episode_batch_update_and_onehot_preprocess():
    pre = {"actions": ("actions_onehot", [OneHot(out_dim=5)])}
    eb = EpisodeBatch(scheme(), {"agents": 2}, 4, 3, preprocess=pre)
    eb.update({"actions": th.ones(2, 1).long(), "obs": th.ones(2, 3), "state": th.ones(4)}, 0, 0)
    assert eb["filled"][0, 0, 0] == 1 and eb["filled"][1, 0, 0] == 0
    assert th.equal(eb["actions_onehot"][0, 0], th.tensor([[0, 1., 0, 0, 0]] * 2))
    with pytest.raises(KeyError):
        eb.update({"nope": th.ones(1)}, 0, 0)
    with pytest.raises(ValueError):
        eb["nope"]
    sub = eb[1:3, :2]
    assert sub.batch_size == 2 and sub.max_seq_length == 2 and sub["obs"].shape == (2, 2, 2, 3)


def test_replay_buffer_wraparound_and_lengths():
    pre = {"actions": ("actions_onehot", [OneHot(out_dim=5)])}
    rb = ReplayBuffer(scheme(), {"agents": 2}, 5, 3, preprocess=pre)
    eb = EpisodeBatch(scheme(), {"agents": 2}, 4, 3, preprocess=pre)
    for t in range(2):
        eb.update({"obs": th.full((4, 2, 3), float(t))}, ts=t)
    rb.insert_episode_batch(eb)
    rb.insert_episode_batch(eb)   # 4 + 4 > 5: wraps (episode_buffer.py:283-286)
    assert rb.episodes_in_buffer == 5 and rb.buffer_index == 3
    assert list(rb.episode_lengths) == [2, 2, 2, 2, 2]


def _packed(av):
    out = np.zeros(av.shape[:-1], np.uint64)
    for a in range(av.shape[-1]):
        out |= (av[..., a] != 0).astype(np.uint64) << np.uint64(a)
    return out.view(np.int64)


@pytest.mark.parametrize("A", [5, 64])
def test_replay_buffer_avail_bits_follow_every_write(A):
    """ReplayBuffer.avail_bits (the mixer's bitmask view of avail_actions, mq_replay.avail_bits) equals the packed
    storage after insert_episode_batch (wraparound included), update() and load_arrays(); bit 63 at A = 64."""
    rng = np.random.default_rng(0)
    rb = ReplayBuffer(scheme(A=A), {"agents": 2}, 5, 3)
    eb = EpisodeBatch(scheme(A=A), {"agents": 2}, 4, 3)
    for t in range(3):
        eb.update({"avail_actions": th.from_numpy(rng.integers(0, 3, (4, 2, A)).astype(np.int32))}, ts=t)
    rb.insert_episode_batch(eb)
    rb.insert_episode_batch(eb)   # wraps
    assert np.array_equal(rb.avail_bits.numpy(), _packed(rb["avail_actions"].numpy()))
    rb.update({"avail_actions": th.ones(2, A, dtype=th.int32)}, bs=1, ts=2)
    assert np.array_equal(rb.avail_bits.numpy(), _packed(rb["avail_actions"].numpy()))
    arr = rng.integers(0, 2, (5, 3, 2, A)).astype(np.int32)
    rb.load_arrays({"avail_actions": arr, "filled": np.ones((5, 3, 1), np.int64)})
    assert np.array_equal(rb.avail_bits.numpy(), _packed(arr))


def test_sample_matches_reference_rng_and_gather():
    rb = ReplayBuffer(scheme(), {"agents": 2}, 10, 4)
    rb.load_arrays({"obs": np.arange(10 * 4 * 2 * 3, dtype=np.float32).reshape(10, 4, 2, 3),
                    "filled": np.ones((10, 4, 1), dtype=np.int64)})
    np.random.seed(5)
    s = rb.sample(3)
    np.random.seed(5)
    ids = np.random.choice(10, 3, replace=False)      # episode_buffer.py:297
    assert isinstance(s, SampledBatch) and np.array_equal(s.ep_ids_np, ids)
    assert th.equal(s["obs"], rb["obs"][th.as_tensor(ids)])
    s2 = s[:, :2]
    assert s2.t_len == 2 and s2["obs"].shape == (3, 2, 2, 3) and s2.max_t_filled() == 2
    assert th.equal(s2.materialize()["obs"], rb["obs"][th.as_tensor(ids)][:, :2])
    sh = s.shard(1, 2)
    assert np.array_equal(sh.ep_ids_np, ids[1:3])
    full = ReplayBuffer(scheme(), {"agents": 2}, 3, 4)
    full.load_arrays({"filled": np.ones((3, 4, 1), dtype=np.int64)})
    st = np.random.get_state()
    assert np.array_equal(full.sample(3).ep_ids_np, np.arange(3))   # no RNG draw (episode_buffer.py:293-294)
    assert np.random.get_state()[2] == st[2]


def build_cpu(mixer="qmix"):
    a = args(mixer)
    sch = scheme()
    rb = ReplayBuffer(sch, {"agents": 2}, 4, 3, preprocess={"actions": ("actions_onehot", [OneHot(5)])})
    mac = mac_REGISTRY["basic_mac"](rb.scheme, {"agents": 2}, a)
    learner = le_REGISTRY["q_learner"](mac, rb.scheme, Logger(logging.getLogger("t")), a)
    return a, rb, mac, learner


def test_parameter_names_order_and_flat_layout():
    a, rb, mac, learner = build_cpu()
    I = 3 + 5 + 2
    want = list(agent_param_shapes(I, 64, 5).items())
    got = [(k, tuple(v.shape)) for k, v in mac.agent.state_dict().items()]
    assert got == [(k, tuple(s)) for k, s in want]
    mix = [(k, tuple(v.shape)) for k, v in learner.mixer.state_dict().items()]
    assert mix == [(k, tuple(s)) for k, s in qmix_param_shapes(4, 2, 32).items()]
    # every parameter is a view into the one flat buffer, in MQ_P_* order
    o = 0
    for p in learner.params:
        assert p.data_ptr() == learner._online.data_ptr() + 4 * o
        o += p.numel()
    assert o == learner.n_params
    assert learner.target_mac.agent.fc1.weight.data_ptr() == learner._target.data_ptr()
    with th.no_grad():
        learner.mixer.hyper_b_1.bias.fill_(3.0)
    assert learner._online[learner.n_params - 1 - 1 - 32 - 32 * 4 - 32: learner.n_params].max() == 3.0


def test_unknown_mixer_raises_value_error():
    a = args("foo")
    rb = ReplayBuffer(scheme(), {"agents": 2}, 4, 3, preprocess={"actions": ("actions_onehot", [OneHot(5)])})
    mac = mac_REGISTRY["basic_mac"](rb.scheme, {"agents": 2}, a)
    with pytest.raises(ValueError, match="Mixer foo not recognised"):
        le_REGISTRY["q_learner"](mac, rb.scheme, Logger(logging.getLogger("t")), a)


def test_checkpoint_roundtrip(tmp_path):
    a, rb, mac, learner = build_cpu()
    with th.no_grad():
        learner._online.normal_()
        learner._sq.uniform_()
    learner.save_models(str(tmp_path))
    assert sorted(os.listdir(tmp_path)) == ["agent.th", "mixer.th", "opt.th"]
    sd = th.load(tmp_path / "opt.th", weights_only=True)
    assert len(sd["state"]) == len(learner.params) and "square_avg" in sd["state"][0]
    a2, rb2, mac2, learner2 = build_cpu()
    learner2.load_models(str(tmp_path))
    assert th.equal(learner2._online, learner._online)
    assert th.equal(learner2._sq, learner._sq)
    Pa = sum(p.numel() for p in learner.mac.agent.parameters())
    # target agent reloads from the online agent.th; the target mixer is not reloaded (q_learner.py:137-143)
    assert th.equal(learner2._target[:Pa], learner._online[:Pa])
    assert learner2.mac.agent.fc1.weight.data_ptr() == learner2._online.data_ptr()


@pytest.mark.parametrize("name", ["tiny_qmix", "tiny_vdn"])
def test_load_reference_checkpoint(golden_cases, name):
    """agent.th / mixer.th / opt.th written by the REFERENCE's QLearner.save_models (q_learner.py:131-135) after
    golden step 2 load with weights_only=True into the flat buffers: parameters bit-equal to the reference's, the
    RMSprop square_avg and step count from opt.th."""
    from tests.golden_utils import GOLDEN
    from tests.gpu_helpers import CKPT, build
    case = golden_cases[name]
    args_, buf, mac, learner, logger = build(case, device="cpu")
    path = os.path.join(GOLDEN, CKPT[name])
    learner.load_models(path)
    assert np.array_equal(learner._online[:learner.n_params].numpy(), case.z["step_params"][2])
    sd = th.load(os.path.join(path, "opt.th"), weights_only=True)
    sq = th.cat([sd["state"][i]["square_avg"].reshape(-1) for i in range(len(learner.params))])
    assert th.equal(learner._sq, sq)
    assert learner._opt_steps == 3 and float(learner.optimiser.state[learner.params[0]]["step"]) == 3
    Pa = sum(p.numel() for p in mac.agent.parameters())
    assert th.equal(learner._target[:Pa], learner._online[:Pa])   # target agent reloads agent.th (:138-140)


def test_no_cpu_fallback():
    a, rb, mac, learner = build_cpu("vdn")
    rb.load_arrays({"filled": np.ones((4, 3, 1), dtype=np.int64)})
    with pytest.raises(_lib.MQError, match="no CPU"):
        learner.train(rb.sample(3), 0, 0)


def test_logger_interface():
    """utils/logging.py keeps the reference's Logger contract: history, sacred sink, recent-stats printing."""
    lines = []
    console = SN(info=lines.append)
    lg = Logger(console)
    assert not lg.use_tb and not lg.use_sacred
    run = SN(info={})
    lg.setup_sacred(run)
    for t in range(7):
        lg.log_stat("loss", float(t), t)
        lg.log_stat("epsilon", 1.0 - 0.1 * t, t)
    lg.log_stat("episode", 12, 6)
    lg.log_stat("hidden", 1.0, 6, to_sacred=False)
    assert lg.use_sacred and run.info["loss"] == [float(t) for t in range(7)] and run.info["loss_T"] == list(range(7))
    assert "hidden" not in run.info
    assert lg.stats["loss"][-1] == (6, 6.0)
    assert lg.recent("loss") == np.mean([2, 3, 4, 5, 6]) and abs(lg.recent("epsilon") - 0.4) < 1e-12
    lg.print_recent_stats()
    assert lines[-1].startswith("Recent Stats | t_env:          6 | Episode:       12\n")
    assert "loss:" in lines[-1] and "4.0000" in lines[-1]


def test_test_stat_threshold_matches_reference_runners():
    """When the runners log test stats: the reference ParallelRunner rounds test_nepisode to whole runs of
    batch_size_run (parallel_runner.py:194-195), EpisodeRunner compares with test_nepisode exactly (episode_runner.py:105)."""
    from types import SimpleNamespace as SN
    from pymarl_amd.runners.episode_runner import EpisodeRunner
    from pymarl_amd.runners.parallel_runner import ParallelRunner
    for cls, bs, n, want in [(ParallelRunner, 4, 6, 4), (ParallelRunner, 4, 2, 4), (ParallelRunner, 8, 16, 16),
                             (EpisodeRunner, 1, 3, 3), (EpisodeRunner, 1, 0, 0)]:
        r = cls.__new__(cls)
        r.args, r.batch_size = SN(test_nepisode=n), bs
        assert r.n_test_episodes() == want, (cls.__name__, bs, n)


@pytest.mark.parametrize("how", ["index", "view", "replace", "update_after"])
def test_avail_bits_never_stale_after_direct_writes(how):
    """The avail bitmask is a derived cache: a write to transition_data["avail_actions"] that bypasses update()
    (what bench.py and make_golden do, as user code may) must never leave the mixer reading stale bits.
    ReplayBuffer.avail_bits_current() (what replay_view hands the kernels) notices the storage's write counter moved
    and rebuilds; a later partial update() after such a write rebuilds everything, not only its own rows."""
    A = 7
    rng = np.random.default_rng(1)
    rb = ReplayBuffer(scheme(A=A), {"agents": 2}, 6, 4)
    rb.load_arrays({"avail_actions": rng.integers(0, 2, (6, 4, 2, A)).astype(np.int32),
                    "filled": np.ones((6, 4, 1), np.int64)})
    assert np.array_equal(rb.avail_bits_current().numpy(), _packed(rb["avail_actions"].numpy()))
    new = th.from_numpy(rng.integers(0, 2, (6, 4, 2, A)).astype(np.int32))
    td = rb.data.transition_data
    if how == "index":
        td["avail_actions"][2] = new[2]
    elif how == "view":
        td["avail_actions"].view(-1, A)[5] = 1 - td["avail_actions"].view(-1, A)[5]
    elif how == "replace":
        td["avail_actions"] = new.clone()
    else:   # a direct write, then a partial update() of OTHER rows
        td["avail_actions"][0] = new[0]
        rb.update({"avail_actions": th.ones(2, A, dtype=th.int32)}, bs=4, ts=1)
        assert np.array_equal(rb.avail_bits.numpy(), _packed(rb["avail_actions"].numpy()))
    s = rb.sample(3)
    bits = s.source.avail_bits_current()
    assert np.array_equal(bits.numpy(), _packed(rb["avail_actions"].numpy()))
    assert rb.avail_bits_current() is bits   # current now: no second rebuild
