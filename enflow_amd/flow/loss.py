"""Alchemical negative log-likelihood (mirrors enflow/flow/loss.py:5-24).

__call__(out, ldj) -> 0-d tensor, computed by enflow_alchemical_nll_f32: one
workgroup per molecule sums the softened LJ energy over i < j pairs (zero
distances dropped, loss.py:14-18), sum vel^2, h^2, g^2; a fixed-order double
reduction forms the reference's scalar.
"""
import torch

from .. import _lib
from ..utils.helpers import batch_meta


class Alchemical_NLL:
    def __init__(self, kBT, partition_func=10, softening=0):
        self.kBT = kBT
        self.z_lj = partition_func
        self.softening = softening

    def __call__(self, out, ldj):
        _lib.require_gpu(out.pos)
        L = _lib.lib()
        dev = out.pos.device
        f = lambda t: t.detach().to(device=dev, dtype=torch.float32).contiguous()  # noqa: E731
        h, g, pos, vel = f(out.h), f(out.g), f(out.pos), f(out.vel)
        ptr, max_n = batch_meta(out, dev)
        M = ptr.numel() - 1
        ldj_t = torch.as_tensor(ldj, device=dev).to(torch.float32).reshape(1).contiguous()
        nll_mol = torch.empty((max(M, 1), 4), dtype=torch.float32, device=dev)
        loss = torch.empty(1, dtype=torch.float32, device=dev)
        _lib.check(L.enflow_alchemical_nll_f32(M, h.shape[0], max_n, h.shape[1], _lib.ptr(ptr),
                                               _lib.ptr(h), _lib.ptr(g), _lib.ptr(pos), _lib.ptr(vel),
                                               _lib.ptr(ldj_t), float(self.kBT), float(self.softening),
                                               float(self.z_lj), _lib.ptr(nll_mol), _lib.ptr(loss),
                                               _lib.stream_ptr(dev)), "enflow_alchemical_nll_f32")
        return loss.reshape(()).to(out.h.dtype)
