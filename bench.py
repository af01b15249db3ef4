"""Learner throughput bench: QLearner.train on synthetic replay, MI355X, 1..8 GPUs (one process per GPU).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config cfg2|cfg3|cfg4|cfg5] [--no-cpu-baseline]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 --master-port P bench.py --gpus N

`--gpus N` means N ranks: launched without torch.distributed.run (WORLD_SIZE unset) and N > 1, the parent starts
`torch.distributed.run --nproc-per-node N` as a child process before it touches the GPU and exits with its code;
under torch.distributed.run a WORLD_SIZE different from --gpus is an error (exit 2).

Metric (BASELINE.json): learner samples/s = B*T*n_agents per train() / wall seconds, whole job (all ranks).
Default workload = BASELINE configs[1]: QMIX synthetic replay n_agents=8, T=120, obs=80, state=168, batch=32 per
GPU (weak scaling: every rank passes the same global sample of 32·N episodes to QLearner.train, as the reference's
run loop does, the learner trains its own 32-episode shard and the ranks all-reduce the gradient once per step over
RCCL). The replay (5000 episodes, SURVEY.md §8d recipe) lives in HBM; a step is the
full train(): id sampling on the host, fused gather, both unrolls, double-Q, mixer, loss, BPTT, clip, RMSprop,
the episode-counted target update — nothing skipped.

The JSON line also carries:
* roofline: the dominant kernel (longest mean duration in an untimed 4-step phase survey) priced by its
  ALGORITHMIC fp32 flops per launch (DESIGN.md "Roofline") against the gfx950 fp32 peak; its average launch
  duration comes from HIP events on the learner's stream over a second timed region of the same K steps (the
  first timed region, which gives `value`, carries no events); `traffic` = PMC-measured HBM bytes per launch of
  that kernel, read from profiles/ if a pmc summary for this config is committed there (null otherwise).
  The PMC summary is stamped with a hash of the kernel sources it measured (pymarl_amd/csrc); a summary whose hash
  differs from the sources this bench runs is stale and is not used (traffic null, `traffic_source` says why).
* cpu_baseline: the numpy oracle's train() (oracle/qlearner_np.py, a restatement of the reference's QLearner.train
  pinned to golden vectors of the reference itself) timed on this host, rank 0 at N=1 only, on a bounded sample.
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import sys
import time
from types import SimpleNamespace as SN

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "learner samples/sec (B×T×n_agents), synthetic replay, 1/2/4/8 MI355X"
FP32_PEAK_TFLOPS = 157.3      # MI355X_MICROARCH.md: fp32 vector = fp32 matrix peak
HBM_PEAK_GBS = 8000.0

CONFIGS = {
    # name: (mixer, n, A, O, S, T, B, description)
    "cfg2": ("qmix", 8, 14, 80, 168, 120, 32, "QMIX synthetic replay n_agents=8 T=120 obs=80 state=168 batch=32"),
    "cfg3": ("vdn", 27, 36, 285, 1170, 180, 128, "VDN synthetic 27m_vs_30m shape n_agents=27 T=180 batch=128"),
    "cfg4": ("qmix", 5, 11, 80, 120, 120, 64, "QMIX 2s3z shape, 64 episodes per GPU (512 over 8 GPUs)"),
    # COMALearner; coma_smac.yaml batch_size 8
    "cfg5": ("coma", 10, 18, 176, 322, 180, 8, "COMA critic counterfactual baseline, MMM2 shape n_agents=10 "
                                               "n_actions=18 T=180 batch=8"),
}


def algorithmic_flops(phase, n, A, O, S, T, B, E=32, H=64, mixer="qmix", fused_fwd=False, fused_bwd=False,
                      hyp_in_fwd=False):
    """fp32 flops one launch of `phase` must do (matmul terms, 2 flop per MAC; elementwise ignored).

    fused_fwd / fused_bwd: the one-row-per-workgroup kernels also carry fc1 / W_ih / fc2 (forward) and
    dW_hh / dW_ih / dX1 / dW1 (backward) — DESIGN.md "Roofline". hyp_in_fwd: the forward launch also runs the QMIX
    hypernet (the row-pair kernel's waves 4 / 5, or workgroups appended to the one-row-net grid).
    """
    Tp = T + 1
    R = B * n
    RT = Tp * R
    I = O + A + n
    NH = E * (n + 3)
    M = T * B
    f = {
        "fc1": 2 * 2 * RT * H * O,                          # both nets, obs part (one-hot columns are gathers)
        "gi": 2 * 2 * RT * 3 * H * H,                       # both nets
        "gru_fwd": 2 * 2 * RT * 3 * H * H,                  # W_hh mat-vec, both nets
        "fc2": 2 * 2 * RT * H * A,
        "hyper": 2 * 2 * M * NH * S if mixer == "qmix" else 0,
        "gru_bwd": 2 * RT * (3 * H * H) * 3,                # W_hh^T mat-vec + dW_hh + dW_ih accumulations
        "dx1": 2 * RT * 3 * H * H,
        "dw1": 2 * RT * H * I,
        "dwh": 2 * M * NH * S if mixer == "qmix" else 0,
    }
    if fused_fwd:
        f["gru_fwd"] = f["fc1"] + f["gi"] + f["gru_fwd"] + f["fc2"]
    if fused_bwd:
        f["gru_bwd"] = f["gru_bwd"] + f["dx1"] + f["dw1"]
    if hyp_in_fwd:
        f["gru_fwd"] = f["gru_fwd"] + f["hyper"]
    return f.get(phase)


def build_workload(cfg_name, device, n_episodes=5000, unique=512, seed=0):
    import torch as th
    from pymarl_amd.components.episode_buffer import ReplayBuffer
    from pymarl_amd.components.transforms import OneHot
    from pymarl_amd.controllers import REGISTRY as mac_REGISTRY
    from pymarl_amd.learners import REGISTRY as le_REGISTRY
    from pymarl_amd.utils.logging import Logger
    from pymarl_amd.utils.synthetic import make_replay

    mixer, n, A, O, S, T, B, _ = CONFIGS[cfg_name]
    args = SN(n_agents=n, n_actions=A, state_shape=S, obs_shape=O, rnn_hidden_dim=64, mixing_embed_dim=32,
              mixer=mixer, lr=5e-4, optim_alpha=0.99, optim_eps=1e-5, grad_norm_clip=10.0, gamma=0.99,
              double_q=True, target_update_interval=200, learner_log_interval=10 ** 12, obs_last_action=True,
              obs_agent_id=True, agent="rnn", mac="basic_mac", agent_output_type="q",
              action_selector="epsilon_greedy", epsilon_start=1.0, epsilon_finish=0.05, epsilon_anneal_time=50000,
              batch_size=B, learner="q_learner", learner_dp=True, device=str(device), use_cuda=True)
    scheme = {
        "state": {"vshape": S},
        "obs": {"vshape": O, "group": "agents"},
        "actions": {"vshape": (1,), "group": "agents", "dtype": th.long},
        "avail_actions": {"vshape": (A,), "group": "agents", "dtype": th.int},
        "reward": {"vshape": (1,)},
        "terminated": {"vshape": (1,), "dtype": th.uint8},
    }
    groups = {"agents": n}
    buf = ReplayBuffer(scheme, groups, n_episodes, T + 1, preprocess={"actions": ("actions_onehot", [OneHot(A)])},
                       device=device)
    data = make_replay(unique, T, n, A, O, S, seed=seed)
    for start in range(0, n_episodes, unique):   # tile the unique episodes across the HBM-resident buffer
        m = min(unique, n_episodes - start)
        for k, v in data.items():
            buf.data.transition_data[k][start:start + m] = th.as_tensor(v[:m], device=device)
    buf.episode_lengths[:] = buf.data.transition_data["filled"].sum(1).reshape(-1).cpu().numpy()
    buf.refresh_avail_bits()   # direct storage writes: rebuild the buffer's avail bitmask (what inserts maintain)
    buf.episodes_in_buffer = n_episodes
    th.manual_seed(seed)   # identical random-init weights on every rank (data-parallel replicas start equal)
    mac = mac_REGISTRY["basic_mac"](buf.scheme, groups, args)
    learner = le_REGISTRY["q_learner"](mac, buf.scheme, Logger(logging.getLogger("bench")), args)
    learner.cuda()
    return args, buf, learner, data


def build_coma_workload(cfg_name, device, n_episodes=1000, unique=128, seed=0, dp=False):
    """COMALearner on an HBM-resident synthetic replay (coma_smac.yaml hyper-parameters)."""
    import torch as th
    from pymarl_amd.components.episode_buffer import ReplayBuffer
    from pymarl_amd.components.transforms import OneHot
    from pymarl_amd.controllers import REGISTRY as mac_REGISTRY
    from pymarl_amd.learners import REGISTRY as le_REGISTRY
    from pymarl_amd.utils.logging import Logger
    from pymarl_amd.utils.synthetic import make_replay

    _, n, A, O, S, T, B, _ = CONFIGS[cfg_name]
    args = SN(n_agents=n, n_actions=A, state_shape=S, obs_shape=O, rnn_hidden_dim=64, lr=5e-4, critic_lr=5e-4,
              optim_alpha=0.99, optim_eps=1e-5, grad_norm_clip=10.0, gamma=0.99, td_lambda=0.8,
              target_update_interval=200, learner_log_interval=10 ** 12, obs_last_action=True, obs_agent_id=True,
              agent="rnn", mac="basic_mac", agent_output_type="pi_logits", action_selector="multinomial",
              epsilon_start=0.5, epsilon_finish=0.01, epsilon_anneal_time=100000, mask_before_softmax=False,
              batch_size=B, learner="coma_learner", learner_dp=dp, device=str(device), use_cuda=True)
    scheme = {
        "state": {"vshape": S},
        "obs": {"vshape": O, "group": "agents"},
        "actions": {"vshape": (1,), "group": "agents", "dtype": th.long},
        "avail_actions": {"vshape": (A,), "group": "agents", "dtype": th.int},
        "reward": {"vshape": (1,)},
        "terminated": {"vshape": (1,), "dtype": th.uint8},
    }
    groups = {"agents": n}
    buf = ReplayBuffer(scheme, groups, n_episodes, T + 1, preprocess={"actions": ("actions_onehot", [OneHot(A)])},
                       device=device)
    data = make_replay(unique, T, n, A, O, S, seed=seed)
    for start in range(0, n_episodes, unique):
        m = min(unique, n_episodes - start)
        for k, v in data.items():
            buf.data.transition_data[k][start:start + m] = th.as_tensor(v[:m], device=device)
    buf.episode_lengths[:] = buf.data.transition_data["filled"].sum(1).reshape(-1).cpu().numpy()
    buf.refresh_avail_bits()   # direct storage writes: rebuild the buffer's avail bitmask (what inserts maintain)
    buf.episodes_in_buffer = n_episodes
    th.manual_seed(seed)   # identical random-init weights on every rank (data-parallel replicas start equal)
    mac = mac_REGISTRY["basic_mac"](buf.scheme, groups, args)
    learner = le_REGISTRY["coma_learner"](mac, buf.scheme, Logger(logging.getLogger("bench")), args)
    learner.cuda()
    return args, buf, learner, data, mac


def rollout_baseline(cfg_name, device, budget_s=6.0, workers=8):
    """The rollout side (north_star: ParallelRunner stays on the host cores), timed on this host: ParallelRunner with
    `workers` env processes (batch_size_run = 8, qmix_smac.yaml) on the seeded FakeEnv at the config's shape
    (SC2 / SMAC cannot run offline), the batched HIP MAC step choosing actions for every running env, each run's
    batch written straight into an HBM replay."""
    import torch as th
    from pymarl_amd.components.episode_buffer import ReplayBuffer
    from pymarl_amd.components.transforms import OneHot
    from pymarl_amd.controllers import REGISTRY as mac_REGISTRY
    from pymarl_amd.runners import REGISTRY as r_REGISTRY
    from pymarl_amd.utils.logging import Logger
    _, n, A, O, S, T, B, _ = CONFIGS[cfg_name]
    args = SN(n_agents=n, n_actions=A, state_shape=S, obs_shape=O, rnn_hidden_dim=64, obs_last_action=True,
              obs_agent_id=True, agent="rnn", mac="basic_mac", agent_output_type="q",
              action_selector="epsilon_greedy", epsilon_start=1.0, epsilon_finish=0.05, epsilon_anneal_time=50000,
              batch_size_run=workers, env="fake", env_args=dict(n_agents=n, n_actions=A, obs_dim=O, state_dim=S,
                                                                 episode_limit=T, seed=5),
              device=str(device), use_cuda=True, test_nepisode=workers, runner_log_interval=10 ** 9)
    logger = Logger(logging.getLogger("bench-rollout"))
    runner = r_REGISTRY["parallel"](args, logger)
    try:
        scheme = {"state": {"vshape": S}, "obs": {"vshape": O, "group": "agents"},
                  "actions": {"vshape": (1,), "group": "agents", "dtype": th.long},
                  "avail_actions": {"vshape": (A,), "group": "agents", "dtype": th.int},
                  "reward": {"vshape": (1,)}, "terminated": {"vshape": (1,), "dtype": th.uint8}}
        groups = {"agents": n}
        preprocess = {"actions": ("actions_onehot", [OneHot(out_dim=A)])}
        buf = ReplayBuffer(scheme, groups, 256, T + 1, preprocess=preprocess, device=device)
        mac = mac_REGISTRY["basic_mac"](buf.scheme, groups, args)
        mac.cuda()
        runner.setup(scheme=scheme, groups=groups, preprocess=preprocess, mac=mac)
        buf.insert_episode_batch(runner.run(test_mode=False))   # warm-up run
        th.cuda.synchronize()
        steps, eps, t0 = 0, 0, time.perf_counter()
        while time.perf_counter() - t0 < budget_s:
            b = runner.run(test_mode=False)
            buf.insert_episode_batch(b)
            steps += int(b["filled"].sum().item()) - workers
            eps += workers
        th.cuda.synchronize()
        dt = time.perf_counter() - t0
    finally:
        runner.close_env()
    return {"value": steps / dt, "unit": "env steps/s", "cores": workers, "kind": "port",
            "sample": f"{eps} episodes ({steps} env steps) of ParallelRunner, {workers} env worker processes, on "
                      f"FakeEnv at {cfg_name}'s shape (n={n}, A={A}, obs={O}, state={S}, limit={T}); SC2 unavailable "
                      f"offline; batched HIP MAC step, HBM replay inserts; {dt / (eps / workers) * 1e3:.1f} ms per "
                      f"{workers}-episode run"}


def cpu_baseline(cfg_name, data, budget_s=12.0):
    """Time the numpy oracle's train() on this host's cores (bounded sample)."""
    from oracle.qlearner_np import OracleQLearner
    from pymarl_amd.utils.synthetic import agent_param_shapes, init_params, qmix_param_shapes
    try:
        from threadpoolctl import threadpool_limits
    except Exception:  # pragma: no cover
        threadpool_limits = None
    mixer, n, A, O, S, T, B, _ = CONFIGS[cfg_name]
    cores = len(os.sched_getaffinity(0))
    cores = min(cores, int(os.environ.get("OMP_NUM_THREADS", cores)))
    cfg = dict(n_agents=n, n_actions=A, mixer=mixer, gamma=0.99, lr=5e-4, optim_alpha=0.99, optim_eps=1e-5,
               grad_norm_clip=10.0, double_q=True, target_update_interval=200, learner_log_interval=0)
    ap = init_params(agent_param_shapes(O + A + n, 64, A), 1)
    mp = init_params(qmix_param_shapes(S, n, 32), 101) if mixer == "qmix" else {}
    o = OracleQLearner(ap, mp, cfg)
    rng = np.random.RandomState(7)
    ctx = threadpool_limits(limits=cores) if threadpool_limits else None
    times = []
    t_start = time.perf_counter()
    try:
        while True:
            ids = rng.choice(len(data["obs"]), B, replace=False)
            batch = {k: v[ids] for k, v in data.items()}
            t0 = time.perf_counter()
            o.train(batch, 0, len(times))
            times.append(time.perf_counter() - t0)
            if time.perf_counter() - t_start > budget_s and len(times) >= 2:
                break
    finally:
        if ctx is not None:
            ctx.unregister() if hasattr(ctx, "unregister") else None
    s = float(np.median(times))
    return {"value": B * T * n / s, "unit": "samples/s", "cores": cores, "kind": "port",
            "sample": f"{len(times)} numpy-oracle train() steps of {cfg_name} (B={B}, T={T}, n={n}), "
                      f"median {s * 1e3:.1f} ms/step, {cores} BLAS threads"}


def coma_cpu_baseline(cfg_name, data, budget_s=12.0):
    """Time the numpy COMA oracle's train() (oracle/coma_np.py) on this host's cores (bounded sample)."""
    from oracle.coma_np import OracleCOMALearner, critic_input_dim, critic_param_shapes
    from pymarl_amd.utils.synthetic import agent_param_shapes, init_params
    try:
        from threadpoolctl import threadpool_limits
    except Exception:  # pragma: no cover
        threadpool_limits = None
    _, n, A, O, S, T, B, _ = CONFIGS[cfg_name]
    cores = len(os.sched_getaffinity(0))
    cores = min(cores, int(os.environ.get("OMP_NUM_THREADS", cores)))
    cfg = dict(n_agents=n, n_actions=A, gamma=0.99, td_lambda=0.8, lr=5e-4, critic_lr=5e-4, optim_alpha=0.99,
               optim_eps=1e-5, grad_norm_clip=10.0, target_update_interval=200, mask_before_softmax=False)
    o = OracleCOMALearner(init_params(agent_param_shapes(O + A + n, 64, A), 1),
                          init_params(critic_param_shapes(critic_input_dim(n, A, O, S), A), 201), cfg)
    rng = np.random.RandomState(7)
    ctx = threadpool_limits(limits=cores) if threadpool_limits else None
    times = []
    t_start = time.perf_counter()
    while True:
        ids = rng.choice(len(data["obs"]), B, replace=False)
        batch = {k: v[ids] for k, v in data.items()}
        t0 = time.perf_counter()
        o.train(batch, 0, len(times), 0.3)
        times.append(time.perf_counter() - t0)
        if time.perf_counter() - t_start > budget_s and len(times) >= 2:
            break
    del ctx
    s = float(np.median(times))
    return {"value": B * T * n / s, "unit": "samples/s", "cores": cores, "kind": "port",
            "sample": f"{len(times)} numpy-oracle COMA train() steps of {cfg_name} (B={B}, T={T}, n={n}), "
                      f"median {s * 1e3:.1f} ms/step, {cores} BLAS threads"}


def kernel_source_hash():
    """sha256 of the kernel sources (pymarl_amd/csrc): stamps PMC summaries so a stale one is never reported."""
    import hashlib
    hsh = hashlib.sha256()
    csrc = os.path.join(ROOT, "pymarl_amd", "csrc")
    for name in sorted(os.listdir(csrc)):
        if name.endswith((".hpp", ".hip", ".h")) or name == "Makefile":
            hsh.update(name.encode())
            with open(os.path.join(csrc, name), "rb") as f:
                hsh.update(f.read())
    for name in sorted(os.listdir(os.path.join(ROOT, "include"))):
        with open(os.path.join(ROOT, "include", name), "rb") as f:
            hsh.update(f.read())
    return hsh.hexdigest()


def launch_ranks(a):
    """--gpus N > 1 without torch.distributed.run: run it as a child (the parent never initialises the GPU)."""
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def init_distributed(expect_world=None):
    """One process per GPU (torch.distributed.run env); returns (world, rank, device)."""
    import torch as th
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # MQ_BENCH_BACKEND=gloo + more ranks than GPUs: rehearsal of the N>1 control flow on a 1-GPU box (ranks share
    # devices round-robin; RCCL refuses two ranks on one GPU). The driver's N>1 runs use the default, RCCL.
    backend = os.environ.get("MQ_BENCH_BACKEND", "nccl")
    dev_index = local_rank % max(1, th.cuda.device_count())
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        th.cuda.set_device(dev_index)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=th.device("cuda", dev_index))
        else:
            dist.init_process_group(backend)
        assert dist.get_world_size() == world, (dist.get_world_size(), world)
    if expect_world is not None and world != expect_world:
        raise SystemExit(f"bench.py: --gpus {expect_world} but the process group has {world} ranks")
    device = th.device("cuda", dev_index)
    th.cuda.set_device(device)
    return world, rank, device


def dist_info(world, learner=None, what="all_reduce(sum) of the fused [grads | sums] buffer"):
    import torch.distributed as dist
    if world > 1 and dist.is_initialized():
        how = learner.collective() if learner is not None else None
        where = ("in stream order inside libmq_learner (the library's RCCL communicator, id broadcast once)"
                 if how == "rccl-native" else "torch.distributed on a communication stream")
        return {"world_size": dist.get_world_size(), "backend": str(dist.get_backend()),
                "collective": "{}, {}".format(what, where), "path": how}
    return {"world_size": 1, "backend": None, "collective": None}


def release_handles(*objs):
    """Destroy the library handles these objects own (mc_destroy / mq_destroy: side streams, events, communicators)
    now, with the HIP runtime and any profiler's interception layer still up, instead of in interpreter-exit
    teardown (a cfg5 run under rocprofv3 crashed there after writing its results)."""
    import gc
    import torch as th
    th.cuda.synchronize()
    for o in objs:
        for attr in ("_handle", "_mac_handle", "_policy_handle"):
            if getattr(o, attr, None) is not None:
                setattr(o, attr, None)
    gc.collect()
    th.cuda.synchronize()


def coma_bench(a):
    """cfg5: COMALearner.train on coma_smac's batch of B = 8 episodes (MMM2 shape: 80 critic rows). N > 1 is strong
    scaling of that batch: every rank passes the same global sample, runs the critic's T dependent optimiser steps
    on all of it through the persistent chain (replicated: no per-step exchange), the actor on its B / N episodes,
    and ONE all-reduce sums the agent gradient (COMALearner "replicated" mode, include/mc_coma.h
    mc_set_actor_shard). The exchange mode (T + 3 all-reduces, SURVEY.md §8e "COMA caveat") is the fallback for
    batches the chain does not take."""
    import torch as th
    import torch.distributed as dist
    world, rank, device = init_distributed(a.gpus)
    args, buf, learner, data, mac = build_coma_workload(a.config, device, dp=world > 1)
    _, n, A, O, S, T, B, desc = CONFIGS[a.config]
    np.random.seed(2)

    def barrier():
        if world > 1:
            dist.barrier()

    def step(k):
        gb = buf.sample(B)   # the global sample: the learner trains this rank's share of it
        mac.action_selector.epsilon = mac.action_selector.schedule.eval(1000 * k)
        learner.train(gb[:, :gb.max_t_filled()], 1000 * k, 8 * k)

    for k in range(max(1, a.warmup)):
        step(k)
    th.cuda.synchronize()
    barrier()
    th.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(a.steps):
        step(k)
    th.cuda.synchronize()
    barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = th.tensor([dt], dtype=th.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    learner.set_timing(True)
    chains = []
    for k in range(min(a.steps, 20)):
        step(k)
        chains.append(learner.phase_times())
    learner.set_timing(False)
    chain_ms = float(np.mean([c["critic_chain"] for c in chains]))
    Kc = S + O + 2 * n * A + n
    R = B * n
    step_flops = 2 * R * (2 * Kc * 128 + 3 * 128 * 128 + 2 * 128 * A)   # one critic step, fwd + bwd
    achieved = step_flops / (chain_ms * 1e-3 / T) / 1e12
    value = B * T * n * a.steps / dt
    if rank != 0:
        from pymarl_amd.learners.dp import SharedComm
        release_handles(learner, mac)
        SharedComm.free()
        dist.destroy_process_group()
        return
    cpu = None if (a.no_cpu_baseline or world > 1) else coma_cpu_baseline(a.config, data)
    # PMC bytes of the whole persistent chain launch, per critic step like `achieved` and `launch_ms`
    traffic, traffic_src = (pmc_traffic(a.config, "coma_chain") if learner.critic_path() == "chain"
                            else (None, "PMC covers the persistent chain only"))
    if traffic is not None:
        traffic, traffic_src = traffic / T, traffic_src + f"; the chain launch's bytes / T = {T} critic steps"
    line = {
        "metric": METRIC, "value": value, "unit": "samples/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": dt / a.steps * 1e3, "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
        "dtype": "fp32", "data": "synthetic (SURVEY.md §8d replay recipe, random-init weights)",
        "config": {"workload": desc, "learner": "coma_learner", "n_agents": n, "n_actions": A, "obs_dim": O,
                   "state_dim": S, "episode_limit": T, "batch_per_gpu": B / world, "global_batch": B,
                   "replay_episodes": buf.buffer_size, "parallelism": f"dp{world}",
                   "coma_dp_mode": learner.dp_mode(B)},
        "dist": dist_info(world, learner, "critic replicated on the whole batch, actor sharded: all_reduce(sum) of "
                                          "the agent [grads | sums] buffer once per train"),
        "roofline": {"bound": "mfma", "kernel": ("coma_chain_kernel (one persistent launch, T critic steps)"
                                                 if learner.critic_path() == "chain"
                                                 else "critic step chain (l1 + head + wgrad, x T)"),
                     "critic_path": learner.critic_path(),
                     "achieved": achieved, "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved / FP32_PEAK_TFLOPS, "traffic": traffic, "traffic_source": traffic_src,
                     "launch_ms": chain_ms / T,
                     "flops_per_launch": step_flops,
                     "phases_ms": {k: float(np.mean([c[k] for c in chains])) for k in chains[0]}},
        "cpu_baseline": cpu,
    }
    print(json.dumps(line), flush=True)
    release_handles(learner, mac)
    if world > 1:
        from pymarl_amd.learners.dp import SharedComm
        SharedComm.free()
        dist.destroy_process_group()


def pmc_traffic(cfg_name, phase):
    """(HBM bytes per launch of `phase`, provenance) from the newest committed PMC summary (profiles/*pmc*.json)
    whose kernel-source hash matches the sources this run uses; (None, reason) otherwise."""
    import glob
    want = kernel_source_hash()
    stale = []
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json")), reverse=True):
        try:
            with open(path) as f:
                d = json.load(f)
        except Exception:
            continue
        v = d.get(cfg_name, {}).get(phase, {}).get("hbm_bytes_per_launch")
        if not v:
            continue
        rel = os.path.relpath(path, ROOT)
        if d.get("source_sha256") != want:
            stale.append(rel)
            continue
        return float(v), f"{rel} (PMC FETCH_SIZE/WRITE_SIZE passes of these kernel sources, sha256 {want[:12]})"
    return None, ("no PMC summary of these kernel sources" +
                  (f"; stale (other sources): {', '.join(stale[:3])}" if stale else ""))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="cfg2", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--phases", action="store_true", help="print every phase's mean ms to stderr")
    a = ap.parse_args()
    if a.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and a.gpus > 1:
        sys.exit(launch_ranks(a))
    if int(env_world or 1) != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={env_world}", file=sys.stderr)
        sys.exit(2)
    if a.config == "cfg5":
        return coma_bench(a)

    import torch as th
    import torch.distributed as dist

    world, rank, device = init_distributed(a.gpus)
    args, buf, learner, data = build_workload(a.config, device)
    mixer, n, A, O, S, T, B, desc = CONFIGS[a.config]

    def barrier():
        if world > 1:
            dist.barrier()

    np.random.seed(2)
    episode = 0

    def step(k):
        nonlocal episode
        # run.py:207-219 unchanged: the global sample, truncated to its max filled length, on every rank; the
        # data-parallel learner trains its own B-episode shard of it (QLearner.train, learners/dp.py)
        gb = buf.sample(B * world)
        learner.train(gb[:, :gb.max_t_filled()], t_env=1000 * k, episode_num=episode)
        episode += 8   # batch_size_run episodes per outer-loop iteration (run.py:247, qmix_smac.yaml:10)

    for k in range(max(1, a.warmup)):
        step(k)
    th.cuda.synchronize()
    # phase survey (untimed): which kernel dominates
    names = learner.phase_names()
    learner.set_timing(slots=4)
    for k in range(4):
        step(k)
    th.cuda.synchronize()
    survey = learner.phase_times()
    dominant = max(survey, key=survey.get)
    plan = learner.last_plan()   # the kernel variants the timed steps run (row tiles, fused kernels, hypernet, mixer)
    fused_fwd = survey.get("fc1", 0.0) == 0.0     # the fused agent forward carries fc1 / W_ih / fc2
    fused_bwd = survey.get("dx1", 0.0) == 0.0     # the fused BPTT carries dX1 / dW1
    # no hypernet launch of its own under QMIX: the forward carries it
    hyp_in_fwd = mixer == "qmix" and survey.get("hyper", 0.0) == 0.0

    def timed():
        barrier()
        th.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(a.steps):
            step(k)
        th.cuda.synchronize()
        barrier()
        return time.perf_counter() - t0

    # timed region 1 -> value: no events in the stream
    learner.set_timing(slots=0)
    dt = timed()
    # timed region 2 -> roofline: the same K steps with HIP events (learner stream) around the dominant kernel
    learner.set_timing(slots=min(a.steps, 4096), phases=[dominant])
    timed()
    dom_ms = learner.phase_times()[dominant]
    learner.set_timing(slots=0)
    if world > 1:
        t = th.tensor([dt], dtype=th.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    samples = B * T * n * world * a.steps
    value = samples / dt
    if rank == 0:
        if a.phases:
            print(json.dumps({"phase_ms": survey}), file=sys.stderr)
        fl = algorithmic_flops(dominant, n, A, O, S, T, B, mixer=mixer, fused_fwd=fused_fwd, fused_bwd=fused_bwd,
                               hyp_in_fwd=hyp_in_fwd)
        achieved = (fl / (dom_ms * 1e-3) / 1e12) if (fl and dom_ms > 0) else None
        traffic, traffic_src = pmc_traffic(a.config, dominant)
        roof = {"bound": "mfma", "kernel": dominant, "achieved": achieved, "peak": FP32_PEAK_TFLOPS,
                "unit": "TFLOP/s", "frac": (achieved / FP32_PEAK_TFLOPS) if achieved else None,
                "traffic": traffic, "traffic_source": traffic_src, "launch_ms": dom_ms, "flops_per_launch": fl,
                "fused": {"fwd": fused_fwd, "bwd": fused_bwd, "hyp_in_fwd": hyp_in_fwd}, "plan": plan}
        cpu = rollout = None
        if world == 1 and not a.no_cpu_baseline:
            cpu = cpu_baseline(a.config, data)
            rollout = rollout_baseline(a.config, device)
        bytes_per_sample = (O * 4 + (S * 4) / n + 8 + A * 4 + (4 + 1 + 8) / n)   # read-once replay bytes
        line = {
            "metric": METRIC, "value": value, "unit": "samples/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": dt / a.steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "fp32", "data": "synthetic (SURVEY.md §8d replay recipe, random-init weights)",
            "config": {"workload": desc, "mixer": mixer, "n_agents": n, "n_actions": A, "obs_dim": O,
                       "state_dim": S, "episode_limit": T, "batch_per_gpu": B, "global_batch": B * world,
                       "replay_episodes": buf.buffer_size, "parallelism": f"dp{world}"},
            "dist": dist_info(world, learner),
            "roofline": roof,
            "hbm_roofline_whole_step": {"achieved_GBs": value * bytes_per_sample / 1e9, "peak_GBs": HBM_PEAK_GBS,
                                        "frac": value * bytes_per_sample / 1e9 / HBM_PEAK_GBS},
            "cpu_baseline": cpu,
            "rollout_baseline": rollout,
        }
        print(json.dumps(line))
    if world > 1:
        from pymarl_amd.learners.dp import SharedComm
        release_handles(learner)
        SharedComm.free()
        dist.destroy_process_group()


if __name__ == "__main__":
    if os.environ.get("MQ_DUMP_MAPS"):
        # diagnostics: the process's mappings as Python exits (before the C-level exit handlers run), so the frames
        # of a crash in exit-time teardown can be resolved to library + offset
        import atexit
        import shutil
        atexit.register(lambda: shutil.copyfile("/proc/self/maps", os.environ["MQ_DUMP_MAPS"]))
    main()
    # release the learners' library handles (cycles included) while the HIP runtime — and a profiler's interception
    # layer, when one is loaded — is still up, not from interpreter-exit finalisers (a cfg5 run under rocprofv3
    # crashed in exit-time teardown after writing its results)
    import gc
    gc.collect()
    if "torch" in sys.modules:
        import torch as _th
        if _th.cuda.is_initialized():
            _th.cuda.synchronize()
