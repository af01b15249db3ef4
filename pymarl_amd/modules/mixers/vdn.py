"""VDNMixer: Q_tot = sum over agents (reference: src/modules/mixers/vdn.py:5-10).

Inside QLearner.train the sum is fused into mix_kernel; this standalone forward is the same reduction.
"""
import torch as th
import torch.nn as nn


class VDNMixer(nn.Module):
    def forward(self, agent_qs, batch):
        return th.sum(agent_qs, dim=2, keepdim=True)
