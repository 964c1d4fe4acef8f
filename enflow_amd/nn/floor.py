"""Floor dequantiser (mirrors enflow/nn/floor.py:5-13).

Inside LFIntegrator the uniform dequantisation and the final floor are fused
into the flow kernel (ENFLOW_DEQUANT_FLOOR); these element-wise methods serve
direct callers.
"""
import torch


class Floor(torch.nn.Module):
    def __init__(self, dequant_scale=1):
        super().__init__()
        self.dequant_scale = dequant_scale

    def forward(self, z):
        return z + self.dequant_scale * torch.rand_like(z).detach(), 0

    def reverse(self, z):
        return torch.floor(z)
