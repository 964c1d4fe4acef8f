"""BaseFlow (mirrors enflow/flow/base.py:5-17).

The reference casts the whole model to float64 (base.py:12).  The HIP kernels
compute in float32, so the modules stay float32; data of any floating dtype
is accepted and results are returned in the input dtype.
"""
import torch


class BaseFlow(torch.nn.Module):
    def __init__(self, networks, dequant_network, dt):
        super().__init__()
        self.networks = torch.nn.ModuleList(networks)
        self.dequantize = dequant_network
        self.dt = dt
        self.dt_2 = 0.5 * dt

    def forward(self, data):
        pass

    def reverse(self, data):
        pass
